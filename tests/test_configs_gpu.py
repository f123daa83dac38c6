"""BASELINE configs[2], [3] and [4] at their per-GPU sizes, 4096 env copies per
GPU (experiments/train.py:110-161 vectorised; maddpg.py:161-196 per rank):
  * configs[2]: simple_spread N=3, batch 1024, 64 units;
  * configs[3]: simple_adversary (1 adversary trained with DDPG, 2 good agents
    with MADDPG: train.py:63-75's policy split), batch 1024, 64 units;
  * configs[4]: simple_tag N=6 (4 adversaries + 2 good), 128 units, batch 4096
    (the general gradient kernels).

The multi-GPU runs shard env copies (each rank owns its 4096 copies, replay
shard and index stream) and exchange gradients; what one rank computes is
exactly this workload.  Checked through the C ABI on the device path:
  * the rollout of a training step (policy actions + MPE physics + replay
    append) for a sample of the 4096 env copies against oracle/mpe.py from
    the same pre-step state (fp64 oracle, fp32 device: 2e-5);
  * 40-41 strict update rounds per vector step (one per 100 transitions):
    stats and every parameter finite, no device fault, the Adam step counters
    advanced once per round;
  * the finished-episode log in env order (deterministic), each row equal to
    that env's rewards summed from its replay rows.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no ROCm GPU", allow_module_level=True)

from maddpg_amd.runner import VecRunner  # noqa: E402
from oracle import mpe  # noqa: E402
from tests.helpers import row_layout  # noqa: E402

ACT = 5
E = 4096


def _oracle(r):
    sp = r.spec
    if sp.name == "simple_tag":
        return mpe.SimpleTag(n_adv=sp.num_adversaries, n_good=sp.n_agents - sp.num_adversaries)
    if sp.name == "simple_adversary":
        return mpe.SimpleAdversary(n_good=sp.n_agents - sp.num_adversaries, n_adv=sp.num_adversaries)
    return mpe.SimpleSpread(sp.n_agents)


def _check_rollout_rows(r, before, rows, sample):
    sc = _oracle(r)
    n, dims = r.n, r.spec.obs_dims
    lay, _ = row_layout(dims)
    ost = {"pos": before["pos"][sample].astype(np.float64), "vel": before["vel"][sample].astype(np.float64),
           "goal": before["goal"][sample]}
    obs0 = sc.observation(ost)
    rs = rows[sample]
    act = np.stack([rs[:, lay[j]["act"]:lay[j]["act"] + ACT] for j in range(n)], 1)
    assert np.allclose(act.sum(-1), 1.0, atol=1e-5) and np.all(act >= 0)
    _, obs1, rew = sc.step(ost, act.astype(np.float64))
    for j in range(n):
        lj, o = lay[j], dims[j]
        np.testing.assert_allclose(rs[:, lj["obs"]:lj["obs"] + o], obs0[j], atol=2e-5)
        np.testing.assert_allclose(rs[:, lj["nobs"]:lj["nobs"] + o], obs1[j], atol=2e-5)
        np.testing.assert_allclose(rs[:, lj["rew"]], rew[:, j], rtol=1e-5, atol=5e-5)
        assert np.all(rs[:, lj["done"]] == 0)


def _run_config(r, steps=3):
    r.prefill()                                   # to the gate B * 25 rows
    assert r.eng.buffer_len() >= r.gate
    rng = np.random.default_rng(0)
    sample = np.sort(rng.choice(E, 384, replace=False))
    sample[0], sample[-1] = 0, E - 1
    total_rounds = 0
    for step in range(steps):
        before = r.eng.env_state()
        head = r.eng.buffer_len()                 # ring not yet wrapped: rows append at len
        k = r.step()
        total_rounds += k
        assert k in (40, 41)                      # 4096 transitions per step, one round per 100
        rows = r.eng.replay_rows(head, E).cpu().numpy()
        _check_rollout_rows(r, before, rows, sample)
    r.synchronize()                               # raises on a recorded device fault
    assert r.rounds == total_rounds
    for i in range(r.n):
        st = r.stats(i)
        assert len(st) == 6 and all(np.isfinite(st))
        for w in ("actor", "critic", "tgt_actor", "tgt_critic", "m_actor", "v_critic"):
            for k_, v in r.eng.get_params(i, w).items():
                assert np.all(np.isfinite(v)), (i, w, k_)
        for net in (0, 1):
            b1p, b2p = r.eng.get_beta_powers(i, net)
            assert np.isclose(b1p, 0.9 ** (total_rounds + 1), rtol=1e-4)   # one Adam step per round
    return total_rounds


def test_configs2_per_gpu_rollout_and_rounds():
    r = VecRunner("simple_spread", E, batch_size=1024, seed=11, max_episode_len=25)
    _run_config(r)
    assert r.eng.buffer_len() == 10 * E           # 7 prefill steps (28,672 >= 25,600 rows) + 3


def test_configs3_adversary_per_gpu_rollout_and_rounds():
    """configs[3]: 1 DDPG adversary (critic input 13) + 2 MADDPG good agents."""
    r = VecRunner("simple_adversary", E, num_adversaries=1, adv_policy="ddpg", good_policy="maddpg",
                  batch_size=1024, seed=13, max_episode_len=25)
    assert list(r.eng.local_q) == [True, False, False]
    _run_config(r)


def test_configs4_tag6_per_gpu_rollout_and_rounds():
    """configs[4]: simple_tag N=6 (4 adversaries, 2 good), 128-unit MLPs,
    batch 4096 (gate 102,400 rows: 25 prefill steps, the last one terminal),
    on the general gradient kernels."""
    r = VecRunner("simple_tag", E, n_agents=6, scenario_adversaries=4, batch_size=4096, num_units=128,
                  seed=14, max_episode_len=25)
    assert r.eng.lib.mdp_grad_variant(r.eng.h, 0) == 0   # general kernels (H = 128, 6 target actors)
    _run_config(r, steps=2)


def test_configs2_episode_log_env_order():
    """one 25-step episode of all 4096 copies: log row e is env e's episode"""
    L = 5
    r = VecRunner("simple_spread", E, batch_size=1024, seed=12, max_episode_len=L)
    for _ in range(L):
        r.rollout()
    assert r.episodes() == E
    log = r.episode_rewards(0, E)
    rows = r.eng.replay_rows(0, L * E).cpu().numpy().reshape(L, E, -1)
    lay, _ = row_layout(r.spec.obs_dims)
    per_agent = np.stack([rows[:, :, lay[j]["rew"]].astype(np.float64).sum(0) for j in range(3)], 1)
    np.testing.assert_allclose(log[:, 1:], per_agent, rtol=1e-5, atol=1e-4)
    np.testing.assert_allclose(log[:, 0], per_agent.sum(1), rtol=1e-5, atol=1e-3)
    # a second identical run logs the identical rows (no arrival-order dependence)
    r2 = VecRunner("simple_spread", E, batch_size=1024, seed=12, max_episode_len=L)
    for _ in range(L):
        r2.rollout()
    np.testing.assert_array_equal(r2.episode_rewards(0, E), log)
