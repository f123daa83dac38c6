"""Drop-in surface on the GPU: ReplayBuffer / MADDPGAgentTrainer / U.* / train.py,
used exactly as the reference's own code uses them."""
import argparse
import hashlib
import os
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no ROCm GPU", allow_module_level=True)

from maddpg_amd.common import tf_util as U  # noqa: E402
from maddpg_amd.envs import Discrete  # noqa: E402
from maddpg_amd.trainer.maddpg import MADDPGAgentTrainer  # noqa: E402
from maddpg_amd.trainer.replay_buffer import ReplayBuffer  # noqa: E402
from oracle import mpe  # noqa: E402
from oracle.pyrandom import MT19937  # noqa: E402
from tests.helpers import golden_case  # noqa: E402


def _digest(arrays):
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


@pytest.mark.parametrize("name", ["small_s0", "wrap_s1", "spread_s12345"])
def test_replay_buffer_facade_matches_reference(golden, name):
    """replay_buffer.py used as the reference uses it: add, random.seed, make_index
    per agent, sample_index of every agent's buffer (maddpg.py:167-178)."""
    c = golden_case(golden, name)
    data = c["data"]()
    bufs = []
    for (o, a, r, on, d) in data:
        rb = ReplayBuffer(c["cap"])
        for k in range(c["n_added"]):
            rb.add(o[k], a[k], float(r[k]), on[k], float(d[k]))
        bufs.append(rb)
    assert len(bufs[0]) == min(c["cap"], c["n_added"])
    random.seed(c["seed"])
    n = len(c["dims"])
    for i in range(n):
        ix = bufs[i].make_index(c["B"])
        assert ix == c["idx"][i].tolist()
        arrs = []
        for j in range(n):
            o, a, _r, on, _d = bufs[j].sample_index(ix)
            assert o.dtype == np.float64 and a.dtype == np.float32
            arrs += [o, a, on]
        own = bufs[i].sample_index(ix)
        arrs += [own[2], own[4]]
        assert _digest(arrs) == c["sha"][i]
    np.testing.assert_array_equal(np.array(random.getstate()[1], np.uint32), c["state"])


def test_trainer_facade_in_reference_loop(tmp_path):
    """experiments/train.py:110-161 written against the drop-in classes, MPE on the host."""
    args = argparse.Namespace(lr=1e-2, gamma=0.95, batch_size=64, num_units=64, max_episode_len=5)
    sc = mpe.make("simple_spread")
    rng = np.random.default_rng(0)
    with U.single_threaded_session():
        trainers = [MADDPGAgentTrainer(f"agent_{i}", None, [(18,)] * 3, [Discrete(5)] * 3, i, args)
                    for i in range(3)]
        U.initialize()
        random.seed(5)
        ref_rng = MT19937(5)
        st = sc.reset(rng, 1)
        obs_n = [o[0] for o in sc.observation(st)]
        episode_step = train_step = 0
        trained = 0
        for _ in range(520):
            action_n = [a.action(o) for a, o in zip(trainers, obs_n)]
            for a in action_n:
                assert a.shape == (5,) and a.dtype == np.float32 and abs(float(a.sum()) - 1) < 1e-5
            st, new_obs_n, rew = sc.step(st, np.array(action_n)[None])
            episode_step += 1
            terminal = episode_step >= args.max_episode_len
            for i, ag in enumerate(trainers):
                ag.experience(obs_n[i], action_n[i], rew[0, i], new_obs_n[i][0], False, terminal)
            obs_n = [o[0] for o in new_obs_n]
            if terminal:
                st = sc.reset(rng, 1)
                obs_n = [o[0] for o in sc.observation(st)]
                episode_step = 0
            train_step += 1
            for ag in trainers:
                ag.preupdate()
            for ag in trainers:
                loss = ag.update(trainers, train_step)
                gate = len(ag.replay_buffer) >= 320 and train_step % 100 == 0
                if not gate:
                    assert loss is None
                    continue
                trained += 1
                want = ref_rng.make_index(len(ag.replay_buffer), 64)
                np.testing.assert_array_equal(ag.replay_sample_index.cpu().numpy(), want)
                # the reference's return value (maddpg.py:196): a list; q_loss, p_loss
                # and mean(target_q_next) fp32 (TF1 fetches / an fp32 array's mean),
                # mean / std of the fp64 TD target and mean(rew) float64
                assert type(loss) is list and len(loss) == 6 and all(np.isfinite(loss))
                assert [type(x) for x in loss] == [np.float32, np.float32, np.float64, np.float64,
                                                   np.float32, np.float64]
                dev = U.get_session().engine().stats(ag.agent_index)      # the fp64 device stats
                assert [float(x) for x in loss] == [float(t(v)) for t, v in zip(map(type, loss), dev)]
        assert trained == 3 * 2            # gate opens at 320 rows: t = 400, 500
        assert random.getstate()[1] == ref_rng.state()
        # p_debug / q_debug surfaces
        ob = np.stack([obs_n[0]] * 7)
        assert trainers[0].p_debug["target_act"](ob).shape == (7, 5)
        assert trainers[0].p_debug["p_values"](ob).shape == (7, 5)
        act = np.full((7, 5), 0.2, np.float32)
        q = trainers[1].q_debug["target_q_values"](ob, ob, ob, act, act, act)
        assert q.shape == (7,) and np.all(np.isfinite(q))
        # save / restore round trip (tf_util.save_state / load_state)
        eng = U.get_session().engine()
        before = eng.get_params(2, "tgt_critic")["W2"].copy()
        path = U.save_state(str(tmp_path) + "/")
        eng.set_params(2, "tgt_critic", {k: v * 0 for k, v in eng.get_params(2, "tgt_critic").items()})
        U.load_state(str(tmp_path) + "/")
        np.testing.assert_array_equal(eng.get_params(2, "tgt_critic")["W2"], before)
        assert os.path.exists(path)
        # the same through a TF1 checkpoint (tf.train.Saver's files, the reference's names)
        sd0 = eng.state_dict()
        prefix = str(tmp_path) + "/tf1/"
        U.save_state(prefix, fmt="tf1")
        assert os.path.exists(prefix + ".index") and os.path.exists(prefix + ".data-00000-of-00001")
        for w in eng.SETS:
            eng.set_params(1, w, {k: v * 0 for k, v in eng.get_params(1, w).items()})
        eng.set_beta_powers(1, 0, np.zeros(2, np.float32))
        U.load_state(prefix)
        sd1 = eng.state_dict()
        assert sd0.keys() == sd1.keys()
        for k in sd0:
            np.testing.assert_array_equal(sd1[k], sd0[k], err_msg=k)
        # an npz save at the same prefix replaces the TF1 bundle: a later restore
        # must not pick up the stale bundle (and the reverse)
        eng.set_params(0, "actor", {k: v + 1 for k, v in eng.get_params(0, "actor").items()})
        sd2 = eng.state_dict()
        U.save_state(prefix)
        assert not os.path.exists(prefix + ".index")
        eng.set_params(0, "actor", {k: v * 0 for k, v in eng.get_params(0, "actor").items()})
        U.load_state(prefix)
        np.testing.assert_array_equal(eng.state_dict()["agent_0/actor/W1"], sd2["agent_0/actor/W1"])
        U.save_state(prefix, fmt="tf1")
        assert not os.path.exists(eng.checkpoint_path(prefix))


@pytest.mark.parametrize("scenario,extra", [
    ("simple_spread", []),
    ("simple_adversary", ["--num-adversaries", "1", "--adv-policy", "ddpg"]),
    ("simple_tag", ["--num-adversaries", "3"]),
    ("simple", []),
    ("simple_spread", ["--save-format", "tf1"]),     # the reference's checkpoint files, restored below
    # the reference's constants as flags, and the debug NaN check on every training step
    ("simple_spread", ["--tau", "0.05", "--grad-clip", "0.2", "--actor-reg", "0.01", "--buffer-size", "50000",
                       "--check-nan"]),
])
def test_train_cli_runs(tmp_path, capsys, scenario, extra):
    from experiments.train import parse_args, train
    a = parse_args(["--scenario", scenario, "--num-envs", "64", "--num-episodes", "300", "--save-rate", "100",
                    "--batch-size", "64", "--max-episode-len", "5", "--save-dir", str(tmp_path) + "/",
                    "--plots-dir", str(tmp_path) + "/", "--exp-name", "t"] + extra)
    runner = train(a)
    out = capsys.readouterr().out
    assert "Starting iterations..." in out and "...Finished total of" in out
    assert out.count("mean episode reward") >= 2
    # SURVEY 5's throughput counters, after the reference's last line
    assert out.rstrip().splitlines()[-1].startswith("throughput: ") and "env-steps/s" in out
    assert runner.throughput["env_steps_per_sec"] > 0 and runner.throughput["trainer_updates_per_sec"] > 0
    assert os.path.exists(str(tmp_path) + "/t_rewards.pkl")
    assert runner.rounds > 0
    # restore the saved model into a fresh run
    a2 = parse_args(["--scenario", scenario, "--num-envs", "64", "--num-episodes", "10", "--restore",
                     "--batch-size", "64", "--max-episode-len", "5", "--save-dir", str(tmp_path) + "/",
                     "--plots-dir", str(tmp_path) + "/", "--exp-name", "t2"] + extra)
    if "tf1" in extra:
        assert os.path.exists(str(tmp_path) + "/.index") and os.path.exists(str(tmp_path) + "/checkpoint")
        assert not os.path.exists(str(tmp_path) + "/maddpg_amd_state.npz")
    train(a2)
    assert "Loading previous state..." in capsys.readouterr().out


@pytest.mark.parametrize("scenario,extra", [
    ("simple_spread", []),
    ("simple_tag", ["--num-adversaries", "3"]),
    ("simple_adversary", ["--num-adversaries", "1"]),
])
def test_train_cli_benchmark_mode(tmp_path, capsys, scenario, extra):
    """--benchmark (train.py:139-148): loads the saved policies, records
    benchmark_data every step, pickles agent_info[:-1], trains nothing."""
    import pickle
    from experiments.train import parse_args, train
    common = ["--scenario", scenario, "--batch-size", "64", "--max-episode-len", "5",
              "--save-dir", str(tmp_path) + "/", "--plots-dir", str(tmp_path) + "/"] + extra
    train(parse_args(common + ["--num-envs", "64", "--num-episodes", "100", "--save-rate", "50",
                               "--exp-name", "t"]))
    capsys.readouterr()
    r = train(parse_args(common + ["--num-envs", "1", "--benchmark", "--benchmark-iters", "12",
                                   "--benchmark-dir", str(tmp_path) + "/bench/", "--exp-name", "b"]))
    out = capsys.readouterr().out
    assert "Loading previous state..." in out and "Finished benchmarking, now saving..." in out
    assert r.rounds == 0
    info = pickle.load(open(str(tmp_path) + "/bench/b.pkl", "rb"))
    # E=1, 5-step episodes, stop at the first terminal with train_step > 12 (t=15):
    # entries = episodes 1..3 closed; first holds 4 steps, then 5 each
    assert [len(ep[0]) for ep in info] == [4, 5, 5]
    assert all(len(ep) == 1 for ep in info)
    assert all(len(step) == r.n for ep in info for step in ep[0])


def test_train_cli_curve_cadence_many_envs(tmp_path, capsys):
    """--num-envs > --save-rate: every save_rate multiple crossed by one vector
    step is one print and one curve point (train.py:164-178), up to the length
    the reference stops at; the curve equals LearningCurve over the episode log."""
    import pickle
    from experiments.train import parse_args, train
    a = parse_args(["--scenario", "simple_spread", "--num-envs", "256", "--num-episodes", "1000",
                    "--save-rate", "100", "--batch-size", "64", "--max-episode-len", "5",
                    "--save-dir", str(tmp_path) + "/", "--plots-dir", str(tmp_path) + "/", "--exp-name", "c"])
    runner = train(a)
    out = capsys.readouterr().out
    curve = pickle.load(open(str(tmp_path) + "/c_rewards.pkl", "rb"))
    # the reference stops at len(episode_rewards) = 1001: points at 100, 200, ..., 1000
    assert len(curve) == 10 and out.count("mean episode reward") == 10
    assert len(pickle.load(open(str(tmp_path) + "/c_agrewards.pkl", "rb"))) == 10 * 3
    log = runner.episode_rewards(0, 999)
    want = [float(np.sum(log[m - 100:m - 1, 0], dtype=np.float64) / 100) for m in range(100, 1001, 100)]
    np.testing.assert_allclose(curve, want, rtol=1e-6)


def test_train_cli_display_headless(tmp_path, capsys):
    """--display (train.py:150-154): loads the saved policies, steps without
    training, renders env copy 0 to PNG frames."""
    from experiments.train import parse_args, train
    common = ["--scenario", "simple_adversary", "--num-adversaries", "1", "--batch-size", "64",
              "--max-episode-len", "5", "--save-dir", str(tmp_path) + "/", "--plots-dir", str(tmp_path) + "/"]
    train(parse_args(common + ["--num-envs", "64", "--num-episodes", "100", "--save-rate", "50", "--exp-name", "t"]))
    capsys.readouterr()
    r = train(parse_args(common + ["--display", "--display-frames", "7", "--exp-name", "v"]))
    out = capsys.readouterr().out
    assert "Loading previous state..." in out and "Rendered 7 frames" in out
    assert r.rounds == 0
    d = os.path.join(str(tmp_path), "v_display")
    assert sorted(os.listdir(d))[:2] == ["frame_00000.png", "frame_00001.png"]
    pos = np.load(os.path.join(d, "positions.npz"))["pos"]
    assert pos.shape == (7, 5, 2) and np.all(np.isfinite(pos))


def test_train_cli_num_gpus_two_ranks(tmp_path):
    """`python experiments/train.py --num-gpus 2` starts two rank processes itself
    (maddpg_amd.launch, as bench.py --gpus does); on this one-GPU box both share
    cuda:0 (MDP_SHARED_GPU=1, gloo group, the real xGMI exchange).  Rank 0 alone
    prints the reference's lines and writes the curve; throughput counts both
    ranks' env copies."""
    import pickle
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MDP_SHARED_GPU="1", MDP_DP_XGMI="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(root, "experiments", "train.py"), "--num-gpus", "2",
                        "--scenario", "simple_spread", "--num-envs", "64", "--num-episodes", "300",
                        "--save-rate", "100", "--batch-size", "64", "--max-episode-len", "5",
                        "--save-dir", str(tmp_path) + "/", "--plots-dir", str(tmp_path) + "/", "--exp-name", "m"],
                       cwd=root, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    out = r.stdout
    assert out.count("Starting iterations...") == 1 and out.count("...Finished total of") == 1, out[-2000:]
    assert out.count("mean episode reward") == 3
    assert out.rstrip().splitlines()[-1].startswith("throughput: ")
    assert len(pickle.load(open(str(tmp_path) + "/m_rewards.pkl", "rb"))) == 3
