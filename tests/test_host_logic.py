"""CPU tests of the host side: C-ABI exports, CLI surface, cadence, scenario tables."""
import ctypes

import pytest

from maddpg_amd import _lib
from maddpg_amd.envs import spec
from maddpg_amd.runner import rounds_due


def test_library_exports_every_header_symbol():
    lib = _lib.load()
    syms = _lib.header_symbols()
    assert len(syms) >= 40
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    assert set(_lib.SIGNATURES) <= set(syms)
    assert lib.mdp_abi_version() == _lib.ABI_VERSION == 5


def _cfg(**kw):
    c = _lib.MdpConfig()
    c.n_agents = 3
    for i in range(3):
        c.obs_dim[i] = 18
    c.act_dim, c.num_units, c.batch_size, c.max_episode_len = 5, 64, 1024, 25
    c.capacity, c.num_envs, c.scenario = 1000000, 1024, 2
    c.lr, c.tau, c.grad_clip, c.actor_reg = 1e-2, 1e-2, 0.5, 1e-3
    c.adam_b1, c.adam_b2, c.adam_eps, c.gamma = 0.9, 0.999, 1e-8, 0.95
    for k, v in kw.items():
        setattr(c, k, v)
    return c


def test_arena_size_and_config_validation():
    lib = _lib.load()
    pt = ctypes.c_int64()
    nb = lib.mdp_arena_bytes(ctypes.byref(_cfg()), ctypes.byref(pt))
    # params: 3 x (actor 5701 + critic 8705) floats, each tensor padded to 4 floats
    assert pt.value >= 3 * (5701 + 8705) and pt.value < 3 * (5701 + 8705) + 3 * 12 * 4
    # replay 1e6 rows x 132 floats dominates
    assert nb > 4 * 1_000_000 * 132
    # any --num-units the reference takes (train.py:24) up to 256: the device
    # nets are padded to the kernel width 64 / 128 / 256
    for u, dev in [(1, 64), (32, 64), (64, 64), (96, 128), (128, 128), (200, 256), (256, 256)]:
        pu = ctypes.c_int64()
        assert lib.mdp_arena_bytes(ctypes.byref(_cfg(num_units=u)), ctypes.byref(pu)) > 0
        per_agent = (18 * dev + dev + dev * dev + dev + dev * 5 + 8) + (69 * dev + dev + dev * dev + dev + dev + 4)
        assert pu.value == 3 * per_agent, (u, pu.value)
    assert lib.mdp_arena_bytes(ctypes.byref(_cfg(num_units=0)), None) < 0
    assert lib.mdp_arena_bytes(ctypes.byref(_cfg(num_units=257)), None) < 0
    assert lib.mdp_arena_bytes(ctypes.byref(_cfg(act_dim=4)), None) < 0
    bad = _cfg()
    bad.obs_dim[1] = 17                                                          # not simple_spread
    assert lib.mdp_arena_bytes(ctypes.byref(bad), None) < 0
    assert lib.mdp_arena_bytes(ctypes.byref(_cfg(scenario=0, num_envs=0)), None) > 0


def _envelope_cfg(dims, units):
    c = _cfg(scenario=0, num_envs=0, n_agents=len(dims), num_units=units)
    for i, d in enumerate(dims):
        c.obs_dim[i] = d
    return c


# the largest per-agent obs dim that fits the kernels' LDS envelope (measured
# with mdp_arena_bytes): (agents, units) -> obs dim
LDS_EDGE = {(8, 64): 66, (3, 256): 95, (8, 256): 33, (1, 256): 256}


@pytest.mark.parametrize("n,units", sorted(LDS_EDGE))
def test_lds_envelope_refused_at_create(n, units):
    """A configuration whose 16-row tile does not fit a CU's LDS is refused by
    mdp_arena_bytes / mdp_create with the reason, not by its first update; the
    edge itself is accepted (tests/test_gpu_parity.py trains it)."""
    lib = _lib.load()
    edge = LDS_EDGE[(n, units)]
    assert lib.mdp_arena_bytes(ctypes.byref(_envelope_cfg([edge] * n, units)), None) > 0
    if edge == 256:                       # obs_dim's own range ends first
        return
    over = _envelope_cfg([edge + 1] * n, units)
    assert lib.mdp_arena_bytes(ctypes.byref(over), None) < 0
    h = ctypes.c_void_p()
    assert lib.mdp_create(ctypes.byref(over), None, 0, None, ctypes.byref(h)) < 0
    msg = lib.mdp_last_error(h).decode()
    lib.mdp_destroy(h)
    assert "LDS envelope" in msg and f"sum of obs dims {(edge + 1) * n}" in msg, msg


def test_cli_flags_mirror_reference_defaults():
    from experiments.train import parse_args
    a = parse_args([])
    # experiments/train.py:14-36 of the reference
    assert (a.scenario, a.max_episode_len, a.num_episodes, a.num_adversaries) == ("simple", 25, 60000, 0)
    assert (a.good_policy, a.adv_policy, a.lr, a.gamma) == ("maddpg", "maddpg", 1e-2, 0.95)
    assert (a.batch_size, a.num_units, a.exp_name, a.save_dir) == (1024, 64, None, "/tmp/policy/")
    assert (a.save_rate, a.load_dir, a.restore, a.display, a.benchmark) == (1000, "", False, False, False)
    assert (a.benchmark_iters, a.benchmark_dir, a.plots_dir) == (100000, "./benchmark_files/", "./learning_curves/")
    assert a.num_envs == 1          # default = the reference's single env
    # its hard-coded constants, exposed with its values (maddpg.py:21,56,130,142,147)
    assert (a.tau, a.grad_clip, a.actor_reg, a.buffer_size) == (1e-2, 0.5, 1e-3, 1000000)
    assert a.check_nan is False


@pytest.mark.parametrize("t0,t1,want", [(0, 1, 0), (99, 100, 1), (100, 101, 0), (0, 1024, 10),
                                        (1024, 2048, 10), (2010, 3100, 11), (0, 100, 1)])
def test_update_cadence(t0, t1, want):
    assert rounds_due(t0, t1) == want


def test_cadence_e1_matches_reference_modulo():
    # E=1: a round exactly at the steps where train_step % 100 == 0
    hits = [t for t in range(1, 1001) if rounds_due(t - 1, t)]
    assert hits == [t for t in range(1, 1001) if t % 100 == 0]


def test_scenario_tables():
    assert spec("simple").obs_dims == [4]
    assert spec("simple_spread").obs_dims == [18, 18, 18]
    assert spec("simple_adversary").obs_dims == [8, 10, 10]
    assert spec("simple_tag").obs_dims == [16, 16, 16, 14]
    assert spec("simple_tag", 6, 4).obs_dims == [22, 22, 22, 22, 20, 20]
    with pytest.raises(ValueError):
        spec("simple_crypto")


def test_product_path_refuses_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from maddpg_amd.engine import Engine
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        Engine([4], batch_size=8, capacity=16)


class _StubEngine:
    """CPU stand-in for Engine.env_step_bench (host logic only): the oracle's
    spread records of a random state each step."""

    def __init__(self, E, n):
        import numpy as np
        from oracle import mpe
        self.rng = np.random.default_rng(0)
        self.sc = mpe.SimpleSpread(n)
        self.E, self.n = E, n

    def env_step_bench(self):
        import numpy as np
        import torch
        st = self.sc.reset(self.rng, self.E)
        recs = self.sc.benchmark_data(st)
        out = np.zeros((self.E, self.n, 8), np.float32)
        for i in range(self.n):
            out[:, i, :recs[i].shape[1]] = recs[i]
        return torch.from_numpy(out)


def test_benchmark_mode_pickle_structure(tmp_path):
    """train.py:139-148 agent_info bookkeeping with E env copies (stub engine)."""
    import pickle
    import types
    from experiments.train import benchmark, parse_args
    from maddpg_amd.envs import spec
    for E, iters, want in [(1, 12, [4, 5, 5]), (2, 12, [4, 4, 5, 5]), (1, 0, [4])]:
        a = parse_args(["--scenario", "simple_spread", "--max-episode-len", "5", "--num-envs", str(E),
                        "--benchmark-iters", str(iters), "--benchmark-dir", str(tmp_path) + "/"])
        runner = types.SimpleNamespace(eng=_StubEngine(E, 3), spec=spec("simple_spread"), n=3,
                                       synchronize=lambda: None)
        benchmark(a, runner, "x", 0)
        info = pickle.load(open(str(tmp_path) + "/x.pkl", "rb"))
        assert [len(ep[0]) for ep in info] == want
        rec = info[0][0][0][0]
        assert isinstance(rec, tuple) and len(rec) == 4 and isinstance(rec[1], int) and rec[1] >= 1
        assert abs(rec[0] - (-rec[2] - rec[1])) < 1e-4


def test_oracle_benchmark_records():
    import numpy as np
    from maddpg_amd.envs import bench_record, spec
    from oracle import mpe
    rng = np.random.default_rng(1)
    for name, sc, sp in [("simple_spread", mpe.SimpleSpread(3), spec("simple_spread")),
                         ("simple_adversary", mpe.SimpleAdversary(), spec("simple_adversary")),
                         ("simple_tag", mpe.SimpleTag(), spec("simple_tag"))]:
        st = sc.reset(rng, 50)
        recs = sc.benchmark_data(st)
        assert len(recs) == sc.n_agents
        for i, r in enumerate(recs):
            row = np.zeros(8, np.float32)
            row[:r.shape[1]] = r[0]
            a, b = bench_record(sp, row, i), sc.record(r[0], i)
            assert type(a) is type(b)
            if isinstance(a, tuple):
                np.testing.assert_allclose(a, b, rtol=1e-6, atol=1e-6)
            else:
                assert abs(a - b) < 1e-5
    try:
        mpe.Simple().benchmark_data(mpe.Simple().reset(rng, 1))
        raise AssertionError("simple has no benchmark_data")
    except AttributeError:
        pass


def _reference_curve(rewards, save_rate, num_episodes):
    """experiments/train.py:123-189 with episodes ending one at a time: the
    episode_rewards list, the save_rate check after each reset, the stop."""
    import numpy as np
    ep = [0.0]
    curve = []
    for r in rewards:
        ep[-1] += r
        ep.append(0.0)                                   # reset (:127-133)
        if len(ep) % save_rate == 0:                     # :164
            curve.append(float(np.mean(ep[-save_rate:])))
        if len(ep) > num_episodes:                       # :181
            break
    return curve, len(ep)


@pytest.mark.parametrize("E,save_rate,num_episodes", [(1, 1000, 5000), (64, 100, 300), (4096, 1000, 20000),
                                                      (5, 3, 40), (7, 1, 20), (1024, 1000, 3000)])
def test_learning_curve_cadence_matches_reference(E, save_rate, num_episodes):
    """E env copies terminating together give the reference's curve: one point
    per save_rate multiple crossed (several per step when E > save_rate), each
    the mean over the last save_rate entries incl. the fresh 0, up to the
    length the reference stops at."""
    import numpy as np
    from experiments.train import LearningCurve
    rng = np.random.default_rng(E + save_rate)
    total = num_episodes + 2 * E
    rewards = rng.normal(-30, 5, size=total).astype(np.float32)
    want, final_len = _reference_curve(rewards.astype(np.float64), save_rate, num_episodes)
    lc = LearningCurve(save_rate, num_episodes, 1)
    log = np.stack([rewards, rewards], 1)
    got = []
    while not lc.done:
        pts = lc.finish(E, lambda first, count: log[first:first + count])
        got += [p[1] for p in pts]
    assert len(got) == len(want) == final_len // save_rate - 1 // save_rate
    np.testing.assert_allclose(got, want, rtol=1e-6)
    assert lc.final_ep_rewards == got and len(lc.final_ep_ag_rewards) == len(got)


def test_model_must_be_mlp_model():
    import types
    from maddpg_amd.trainer.maddpg import check_model, mlp_model

    def mlp_model_ref(input, num_outputs, scope, reuse=False, num_units=64, rnn_cell=None):
        pass
    mlp_model_ref.__name__ = "mlp_model"          # the reference's own function (train.py:39)
    for m in (None, mlp_model, mlp_model_ref):
        check_model(m, 64)
    with pytest.raises(NotImplementedError, match="mlp_model"):
        check_model(lambda x, n, s: x, 64)
    with pytest.raises(NotImplementedError):
        check_model(types.SimpleNamespace(), 64)
    with pytest.raises(ValueError):
        check_model(mlp_model, 300)


def test_optimizer_coresidency_plan():
    """mdp_ra_plan: the fused optimizer launch (chunk workgroups spin on each
    other's norm partials / the xGMI peers) is used only when its whole grid is
    co-resident; otherwise that net falls back to k_reduce + k_apply.  MI355X:
    256 CUs x 1 workgroup of 1024 threads (k_reduce_apply's occupancy)."""
    lib = _lib.load()
    out = (ctypes.c_int32 * 16)()
    # S2 at H=64, chunks of 256 per tensor: critic W1 18 + b1 1 + W2 16 + b2 1 +
    # W3 1 + b3 1 + stats 1 + a slot for an index-draw workgroup = 40; actor 5 +
    # 1 + 16 + 1 + 2 + 1 = 26, + 13 Polyak workgroups of the critic (1,024-
    # parameter chunks) + stats + draw slot = 41 (3 agents)
    assert lib.mdp_ra_plan(ctypes.byref(_cfg()), 256, 1, out) == 0
    assert list(out[:6]) == [41, 40] * 3
    # the same launch on a device holding 40 workgroups: the actor steps fall back
    assert lib.mdp_ra_plan(ctypes.byref(_cfg()), 40, 1, out) == 3
    assert list(out[:6]) == [-41, 40] * 3
    # H=256: the 256x256 W2 alone is 256 chunks -> every critic step (331
    # workgroups) and actor step exceed 256 slots
    n = lib.mdp_ra_plan(ctypes.byref(_cfg(num_units=256)), 256, 1, out)
    assert n == 6 and all(v < 0 for v in out[:6]) and -out[1] > 256
    # configs[4] topology (tag N=6, H=128): every net fits on one MI355X
    tag = _cfg(n_agents=6, num_units=128, scenario=4, num_adversaries=4)
    for i, d in enumerate([22, 22, 22, 22, 20, 20]):
        tag.obs_dim[i] = d
    assert lib.mdp_ra_plan(ctypes.byref(tag), 256, 1, out) == 0
    assert max(out[:12]) <= 256
    assert lib.mdp_ra_plan(ctypes.byref(_cfg(num_units=0)), 256, 1, out) < 0


def test_headless_display_frames(tmp_path):
    """--display's renderer (train.py:150-154, MPE env.render without a window):
    PNG frames that decode to the right size with the entities drawn."""
    import struct
    import zlib

    import numpy as np
    from maddpg_amd.render import FrameWriter, entity_table, rasterize
    for name, n, na in [("simple", None, None), ("simple_spread", None, None), ("simple_adversary", None, None),
                        ("simple_tag", 6, 4)]:
        sp = spec(name, n, na)
        tab = entity_table(sp)
        assert len(tab) == sp.n_agents + {"simple": 1, "simple_spread": sp.n_agents,
                                          "simple_adversary": sp.n_agents - 1, "simple_tag": 2}[name]
    sp = spec("simple_spread")
    pos = np.array([[0.0, 0.0], [0.5, 0.5], [-0.5, -0.5], [0.9, -0.9], [-0.9, 0.9], [0.0, 0.6]], np.float32)
    img = rasterize(pos, entity_table(sp), px=200)
    assert img.shape == (200, 200, 3)
    assert tuple(img[100, 100]) == (89, 89, 217)          # agent 0 at the centre, MPE agent colour
    assert tuple(img[0, 0]) == (255, 255, 255)
    w = FrameWriter(str(tmp_path / "d"), sp)
    for k in range(3):
        w.add(pos + 0.01 * k)
    assert w.close() == 3
    raw = open(tmp_path / "d" / "frame_00002.png", "rb").read()
    assert raw[:8] == b"\x89PNG\r\n\x1a\n"
    wdt, hgt = struct.unpack(">II", raw[16:24])
    assert (wdt, hgt) == (256, 256)
    idat = raw[raw.index(b"IDAT") + 4: raw.index(b"IEND") - 8]
    assert len(zlib.decompress(idat)) == hgt * (1 + 3 * wdt)
    assert np.load(tmp_path / "d" / "positions.npz")["pos"].shape == (3, 6, 2)


def test_bench_algorithmic_model_matches_survey():
    """bench.py's roofline model against SURVEY 8d's per-unit figures: S2 critic
    step 95.4 MFLOP / 0.863 MB, actor step 0.500 MB (58.6 MFLOP by the kernels'
    MAC count), S5 critic step 2,009 MFLOP / 6.40 MB; and the roofline fields
    the line carries (frac from the committed rocprof duration, live beside it)."""
    import types
    import bench

    s2 = types.SimpleNamespace(num_units=64, batch_size=1024, obs_dims=[18, 18, 18], n=3,
                               local_q=[False] * 3)
    assert abs(bench.flops_critic_grad(s2, 0) / 1e6 - 95.4) < 0.1
    assert abs(bench.bytes_critic_grad(s2, 0) - 863068) <= 4
    assert abs(bench.bytes_actor_grad(s2, 0) / 1e6 - 0.500) < 0.005
    assert abs(bench.flops_actor_grad(s2, 0) / 1e6 - 58.6) < 0.1
    s5 = types.SimpleNamespace(num_units=128, batch_size=4096, obs_dims=[22, 22, 22, 22, 20, 20], n=6,
                               local_q=[False] * 6)
    assert abs(bench.flops_critic_grad(s5, 0) / 1e6 - 2009) < 2
    assert abs(bench.bytes_critic_grad(s5, 0) / 1e6 - 6.40) < 0.01
    assert bench.MARKER_KINDS == ("allreduce", "gather")


def test_update_stats_reference_dtypes():
    """update()'s return value (maddpg.py:196) from the fp64 device stats: a
    list; q_loss, p_loss (TF1 fp32 fetches, :91 / :54-56) and mean(Q') (the mean
    of an fp32 array, :185) fp32; mean / std of the fp64 TD target and the mean
    reward (:186) float64 -- each the device value rounded once."""
    import numpy as np
    from maddpg_amd.engine import update_stats
    dev = [0.1234567891234, -1.5e-3, 3.000000001, -0.25, 7.123456789, 0.0625]
    got = update_stats(dev)
    assert type(got) is list
    assert [type(x) for x in got] == [np.float32, np.float32, np.float64, np.float64, np.float32, np.float64]
    assert [float(x) for x in got] == [float(np.float32(dev[0])), float(np.float32(dev[1])), dev[2], dev[3],
                                       float(np.float32(dev[4])), dev[5]]
