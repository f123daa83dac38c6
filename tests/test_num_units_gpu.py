"""--num-units generality (experiments/train.py:24 takes any int; mlp_model,
train.py:39-46, builds two hidden layers of that width).

The library pads the hidden width to the kernel width (64 / 128 / 256) with
zero weights; these tests check, through the C ABI, that the padded device
nets give the unpadded reference math: full update() parity against the
oracle at S2 topology (spread N=3, B=1024) for widths served by each kernel
family -- 32 (fast H=64 kernels), 96 (general H=128), 256 (general H=256) --
that the pad entries of every parameter set stay exactly zero through the
update, and the policy / critic evaluation and the device env rollout at a
padded width.
"""
import copy

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no ROCm GPU", allow_module_level=True)

from maddpg_amd.engine import Engine  # noqa: E402
from oracle import nets, trainer  # noqa: E402
from tests.helpers import joint_rows, synthetic_trainer_case  # noqa: E402

SETS = ("actor", "critic", "tgt_actor", "tgt_critic", "m_actor", "v_actor", "m_critic", "v_critic")
REGION_OF = {"actor": "theta", "critic": "theta", "tgt_actor": "target", "tgt_critic": "target",
             "m_actor": "adam_m", "v_actor": "adam_v", "m_critic": "adam_m", "v_critic": "adam_v"}


def _pad_entries_zero(eng):
    """every arena entry outside the logical [rows, cols] block of each tensor is 0"""
    bad = 0
    for which in SETS:
        reg = eng.region(REGION_OF[which]).cpu().numpy()
        net = 1 if "critic" in which else 0
        for i in range(eng.n):
            for (off, r, c, dr, dc) in eng.net_tensors(i, net):
                blk = reg[off:off + dr * dc].reshape(dr, dc)
                mask = np.ones((dr, dc), bool)
                mask[:r, :c] = False
                bad += int(np.count_nonzero(blk[mask]))
    return bad


@pytest.mark.parametrize("H,variant", [(32, 1), (96, 0), (256, 0)])
def test_update_parity_num_units(H, variant):
    dims, B, L = [18, 18, 18], 1024, 4000
    c = synthetic_trainer_case(dims, B, L, seed=31 + H, H=H)
    n = len(dims)
    eng = Engine(dims, num_units=H, batch_size=B, capacity=L + 7)
    assert eng.lib.mdp_grad_variant(eng.h, 0) == variant
    shapes = eng._flat_shapes(0, "critic")
    assert shapes == [(69, H), (1, H), (H, H), (1, H), (H, 1), (1, 1)]
    eng.add_rows(torch.from_numpy(joint_rows(c["data"], dims)))
    for i, p in enumerate(c["params"]):
        for w in ("actor", "critic", "tgt_actor", "tgt_critic"):
            eng.set_params(i, w, p[w])
    # round trip of the logical values through the padded layout
    got = eng.get_params(1, "tgt_critic")
    for k, v in c["params"][1]["tgt_critic"].items():
        np.testing.assert_array_equal(got[k], np.asarray(v, np.float32).reshape(got[k].shape))
    agents = [trainer.AgentParams(**copy.deepcopy(p), local_q=False) for p in c["params"]]
    worst = 0.0
    for i in range(n):
        eng.update(i, idx=torch.from_numpy(c["idx"][i]), u_tgt=torch.from_numpy(c["u_tgt"][i]),
                   u_act=torch.from_numpy(c["u_act"][i]))
        got = eng.stats(i)
        want, _ = trainer.update(agents, i, c["data"], c["idx"][i], c["u_tgt"][i], c["u_act"][i])
        assert abs(got[0] - want[0]) <= 1e-5 * abs(want[0]) + 1e-7, (H, i, got[0], want[0])
        np.testing.assert_allclose(got[1:], want[1:], rtol=2e-5, atol=2e-6)
        for w, ref in (("actor", agents[i].actor), ("critic", agents[i].critic),
                       ("tgt_actor", agents[i].tgt_actor), ("tgt_critic", agents[i].tgt_critic)):
            dev = eng.get_params(i, w)
            for k in ref:
                err = float(np.abs(dev[k] - ref[k].reshape(dev[k].shape)).max())
                worst = max(worst, err)
                assert err < 1e-4, (H, i, w, k, err)
    print(f"num_units={H}: worst param |diff| = {worst:.3e}")
    assert _pad_entries_zero(eng) == 0


@pytest.mark.parametrize("H", [32, 256])
def test_act_q_and_rollout_num_units(H):
    dims = [18, 18, 18]
    c = synthetic_trainer_case(dims, B=100, L=100, seed=5, H=H)
    eng = Engine(dims, num_units=H, batch_size=100, capacity=2048, num_envs=100, scenario="simple_spread")
    for i, p in enumerate(c["params"]):
        for w in ("actor", "critic", "tgt_actor", "tgt_critic"):
            eng.set_params(i, w, p[w])
    obs = c["data"][0][0][:100].astype(np.float32)
    u = c["u_act"][0][:100]
    ag = trainer.AgentParams(**c["params"][0])
    got = eng.act(0, torch.from_numpy(obs), u=torch.from_numpy(u)).cpu().numpy()
    np.testing.assert_allclose(got, trainer.act(ag, obs, u), atol=2e-6)
    x = np.random.default_rng(0).normal(size=(50, 69)).astype(np.float32)
    q = eng.q_values(0, torch.from_numpy(x)).cpu().numpy()
    np.testing.assert_allclose(q, nets.mlp_fwd(ag.critic, x)[0][:, 0], rtol=1e-5, atol=2e-5)
    # the device rollout's policy actions at this width equal the oracle actor on the same obs
    eng.env_reset()
    obs_dev = eng.env_obs().cpu().numpy()
    uu = np.random.default_rng(1).uniform(1e-6, 1.0, size=(100, 3, 5)).astype(np.float32)
    eng.env_step(u=torch.from_numpy(uu))
    eng.synchronize()
    rows = eng.replay_rows(0, 100).cpu().numpy()
    lay = eng.row_layout
    for j in range(3):
        aj = trainer.AgentParams(**c["params"][j])
        o = obs_dev[:, 18 * j:18 * (j + 1)]
        np.testing.assert_allclose(rows[:, lay[j][1]:lay[j][1] + 5], trainer.act(aj, o, uu[:, j]), atol=2e-6)
