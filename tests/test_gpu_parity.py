"""GPU parity: the HIP path (through the C ABI) against the reference's golden
fixtures and the CPU oracle, on identical seeded inputs.

Tolerances (north_star): replay index selection and gathers bit-exact; critic
loss within 1e-5 (relative, fp32); parameters after a full update within the
fp32 accumulation-order noise stated per test.
"""
import copy
import hashlib
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no ROCm GPU", allow_module_level=True)

from maddpg_amd.engine import UPDATE_STAT_DTYPES, Engine  # noqa: E402
from oracle import mpe, nets, trainer  # noqa: E402
from tests.helpers import (case_names, golden_case, joint_rows, relu_margin_clean_idx, row_layout,  # noqa: E402
                           synthetic_trainer_case)

ACT = 5


def _digest(arrays):
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def _engine_with_case(c, **kw):
    eng = Engine(c["dims"], batch_size=c["B"], capacity=c["cap"], **kw)
    rows = joint_rows(c["data"](), c["dims"])
    eng.add_rows(torch.from_numpy(rows))
    assert eng.buffer_len() == min(c["cap"], c["n_added"])
    return eng


# ------------------------------------------------------------- replay index
@pytest.mark.parametrize("name", ["spread_s0", "spread_s1", "spread_s12345", "simple_s0", "wrap_s1",
                                  "tag6_s0", "tag6_s12345", "small_s1"])
def test_make_index_bit_exact_vs_reference(golden, name):
    c = golden_case(golden, name)
    eng = _engine_with_case(c)
    eng.seed_py_random(c["seed"])
    n, B = len(c["dims"]), c["B"]
    idx = eng.make_index(n * B).cpu().numpy().reshape(n, B)
    np.testing.assert_array_equal(idx, c["idx"])
    np.testing.assert_array_equal(eng.get_rng_state(), c["state"])
    # per-agent draws (maddpg.py:167 called agent by agent) give the same stream
    eng.seed_py_random(c["seed"])
    for i in range(n):
        np.testing.assert_array_equal(eng.make_index(B).cpu().numpy(), c["idx"][i])
    np.testing.assert_array_equal(eng.get_rng_state(), c["state"])


@pytest.mark.parametrize("name", ["spread_s0", "wrap_s12345", "tag6_s1", "small_s0", "simple_s12345"])
def test_fused_gather_bit_exact_vs_reference(golden, name):
    c = golden_case(golden, name)
    eng = _engine_with_case(c)
    lay, stride = row_layout(c["dims"])
    n = len(c["dims"])
    for i in range(n):
        rows = eng.sample_rows(torch.from_numpy(c["idx"][i])).cpu().numpy()
        arrs = []
        for j in range(n):
            lj, o = lay[j], c["dims"][j]
            arrs += [rows[:, lj["obs"]:lj["obs"] + o].astype(np.float64),
                     rows[:, lj["act"]:lj["act"] + ACT].astype(np.float32),
                     rows[:, lj["nobs"]:lj["nobs"] + o].astype(np.float64)]
        arrs += [rows[:, lay[i]["rew"]].astype(np.float64), rows[:, lay[i]["done"]].astype(np.float64)]
        assert _digest(arrs) == c["sha"][i], f"agent {i}"


@pytest.mark.parametrize("dims,rows", [([18, 18, 18], 300_000), ([22, 22, 22, 22, 20, 20], 131_071), ([4], 1)])
def test_gather_large_batches_bit_exact(dims, rows):
    """k_gather_rows beyond the golden fixtures' sizes: enough rows that every
    thread of the capped grid runs the 4-element unrolled loop AND the tail
    (S2: 300K rows x 33 float4 > 4096 x 256 x 3), an odd count, a single row.
    A row copy, so bit-exact against indexing the ring on the device."""
    cap = 1 << 18
    eng = Engine(dims, batch_size=8, capacity=cap)
    eng.add_rows(torch.rand(cap, eng.row_stride))
    idx = torch.randint(0, cap, (rows,), dtype=torch.int32)
    idx[0], idx[-1] = 0, cap - 1
    got = eng.sample_rows(idx)
    ring = eng.region("replay")[:cap * eng.row_stride].view(cap, eng.row_stride)
    want = ring[idx.to(ring.device).long()]
    assert torch.equal(got, want)


def test_make_index_continues_python_global_state():
    random.seed(99)
    for _ in range(37):
        random.random()
    eng = Engine([4], batch_size=8, capacity=5000)
    eng.add_rows(torch.zeros((3333, eng.row_stride)))
    eng.set_rng_state(np.array(random.getstate()[1], dtype=np.uint64))
    got = eng.make_index(2000).cpu().numpy()
    want = [random.randint(0, 3332) for _ in range(2000)]
    np.testing.assert_array_equal(got, want)
    np.testing.assert_array_equal(eng.get_rng_state(), np.array(random.getstate()[1], np.uint32))


def test_make_index_edge_lengths():
    eng = Engine([4], batch_size=8, capacity=70000)
    for L in (1, 2, 3, 624, 625, 65536, 65537):
        eng.set_ring(L, L % 70000)
        g = random.Random(L)
        eng.set_rng_state(np.array(g.getstate()[1], dtype=np.uint64))
        got = eng.make_index(1500).cpu().numpy()
        np.testing.assert_array_equal(got, [g.randint(0, L - 1) for _ in range(1500)])


# ----------------------------------------------------------- policy / critic
def test_act_and_q_values_match_oracle():
    dims = [18, 18, 18]
    c = synthetic_trainer_case(dims, B=100, L=100, seed=11)
    eng = Engine(dims, batch_size=100, capacity=200)
    for i, p in enumerate(c["params"]):
        for w in ("actor", "critic", "tgt_actor", "tgt_critic"):
            eng.set_params(i, w, p[w])
    obs = c["data"][1][0][:100].astype(np.float32)
    u = c["u_act"][1][:100]
    got = eng.act(1, torch.from_numpy(obs), u=torch.from_numpy(u)).cpu().numpy()
    ag = trainer.AgentParams(**c["params"][1])
    np.testing.assert_allclose(got, trainer.act(ag, obs, u), atol=2e-6)
    got_t = eng.act(1, torch.from_numpy(obs), target=True, u=torch.from_numpy(u)).cpu().numpy()
    np.testing.assert_allclose(got_t, trainer.target_act(ag, obs, u), atol=2e-6)
    lg = eng.actor_logits(1, torch.from_numpy(obs)).cpu().numpy()
    np.testing.assert_allclose(lg, nets.mlp_fwd(ag.actor, obs)[0], atol=2e-5)
    x = np.random.default_rng(0).normal(size=(77, 69)).astype(np.float32)
    q = eng.q_values(1, torch.from_numpy(x), target=True).cpu().numpy()
    np.testing.assert_allclose(q, nets.mlp_fwd(ag.tgt_critic, x)[0][:, 0], rtol=1e-5, atol=2e-5)


@pytest.mark.parametrize("H", [64, 128])
def test_device_gumbel_noise_is_the_pinned_philox(H):
    """The device's own Gumbel noise (mdp_act without injected uniforms) is
    Philox4x32-10 with the 23-bit float: every sampled action equals the
    oracle's gumbel_softmax on oracle/philox.py's uniforms for the same
    (seed, stream, counter, row) -- and that generator is pinned to the
    Random123 known-answer vectors (tests/test_oracle.py).  The seed uses both
    key words; 100 rows = 6 full tiles + a ragged one; the counter advances per
    call (stream 0x40000 | agent << 1 | target, mdp_api.cpp mdp_act)."""
    from oracle import philox
    dims = [18, 18, 18]
    seed = 0x9E3779B97F4A7C15
    c = synthetic_trainer_case(dims, B=100, L=100, seed=13, H=H)
    eng = Engine(dims, num_units=H, batch_size=100, capacity=200, seed=seed)
    for i, p in enumerate(c["params"]):
        for w in ("actor", "critic", "tgt_actor", "tgt_critic"):
            eng.set_params(i, w, p[w])
    obs = c["data"][0][0][:100].astype(np.float32)
    for k, (agent, target) in enumerate([(1, False), (1, True), (2, False), (0, True), (1, False)]):
        got = eng.act(agent, torch.from_numpy(obs), target=target).cpu().numpy()
        u = philox.uniforms5(seed, 0x40000 | (agent << 1) | int(target), k, np.arange(100))
        ag = trainer.AgentParams(**c["params"][agent])
        want = (trainer.target_act if target else trainer.act)(ag, obs, u)
        np.testing.assert_allclose(got, want, atol=2e-6, err_msg=f"call {k}: agent {agent} target {target}")


# ------------------------------------------------------------------ update
def _device_grads(eng, agent, net):
    """the batch-reduced gradient the optimizer step of (agent, net) consumed
    (GRAD region, written by k_reduce_apply / k_reduce), per tensor"""
    g = eng.region("grad").cpu().numpy()
    out = {}
    for k, (off, r, c_, dr, dc) in zip(("W1", "b1", "W2", "b2", "W3", "b3"), eng.net_tensors(agent, net)):
        a = g[off:off + dr * dc].reshape(dr, dc)[:r, :c_]
        out[k] = a[0].copy() if k.startswith("b") else a.copy()
    return out


def _clip_mode_distance(eng, c, i, dgs):
    """SURVEY App. A / tf_util.py:178-180: which clip_by_norm arithmetic the
    device implements.  Agent i's first Adam step (from the case's pre-update
    weights) re-run on the DEVICE's batch-reduced gradient with the tensor
    norm taken in fp64 (the device's choice) and in fp32 (TF1's reduce_sum):
    the worst |theta_device - theta_mode| per net and mode, and the worst
    relative gap between the two norms over the net's tensors."""
    out = {}
    for net, w in ((1, "critic"), (0, "actor")):
        dev = eng.get_params(i, w)
        g = {k: np.asarray(v, np.float32).reshape(dev[k].shape) for k, v in dgs[net].items()}
        n64 = {k: float(nets.tensor_norm(v, "fp64")) for k, v in g.items()}
        n32 = {k: float(nets.tensor_norm(v, "fp32")) for k, v in g.items()}
        out[(w, "norm_rel_gap")] = max(abs(n32[k] - n64[k]) / max(n64[k], 1e-30) for k in g)
        for mode in ("fp64", "fp32"):
            p = {k: np.asarray(v, np.float32).reshape(dev[k].shape).copy() for k, v in c["params"][i][w].items()}
            nets.Adam(p).apply(p, {k: nets.clip_by_norm(v, 0.5, mode) for k, v in g.items()})
            out[(w, mode)] = max(float(np.abs(dev[k] - p[k]).max()) for k in p)
    return out


def _philox_case_noise(c, n, B, key):
    """the uniforms the device draws itself in agent i's strict update (counter
    upd_ctr = i on a fresh engine): target actor j on stream (i << 8) | (j + 1),
    the actor-loss sample on (i << 8) | 0x80, row = batch row (mdp_grads*.hip)"""
    from oracle import philox
    rows = np.arange(B)
    c["u_tgt"] = [np.stack([philox.uniforms5(key, (i << 8) | (j + 1), i, rows) for j in range(n)]) for i in range(n)]
    c["u_act"] = [philox.uniforms5(key, (i << 8) | 0x80, i, rows) for i in range(n)]


def _update_parity(dims, B, L, seed, local_q=None, H=64, check_round=True, device_noise_key=None):
    c = synthetic_trainer_case(dims, B, L, seed, local_q, H)
    n = len(dims)
    kw = {} if device_noise_key is None else {"seed": device_noise_key}
    if device_noise_key is not None:
        _philox_case_noise(c, n, B, device_noise_key)
    eng = Engine(dims, c["local_q"], num_units=H, batch_size=B, capacity=L + 7, **kw)
    eng.add_rows(torch.from_numpy(joint_rows(c["data"], dims)))
    for i, p in enumerate(c["params"]):
        for w in ("actor", "critic", "tgt_actor", "tgt_critic"):
            eng.set_params(i, w, p[w])
    agents = [trainer.AgentParams(**copy.deepcopy(p), local_q=c["local_q"][i]) for i, p in enumerate(c["params"])]
    report, greport, wreport, creport = [], [], [], []
    for i in range(n if check_round else 1):
        if device_noise_key is None:
            eng.update(i, idx=torch.from_numpy(c["idx"][i]), u_tgt=torch.from_numpy(c["u_tgt"][i]),
                       u_act=torch.from_numpy(c["u_act"][i]))
        else:                                     # the device's own Philox noise
            eng.update(i, idx=torch.from_numpy(c["idx"][i]))
        got = eng.stats(i)
        want, og = trainer.update(agents, i, c["data"], c["idx"][i], c["u_tgt"][i], c["u_act"][i])
        conditioned = {}
        dgs = {net: _device_grads(eng, i, net) for net in (0, 1)}
        cm = _clip_mode_distance(eng, c, i, dgs)
        creport.append(cm)
        for w in ("critic", "actor"):
            # the device's step IS the fp64-norm clip applied to its own gradient
            assert cm[(w, "fp64")] < 1e-6, (i, w, cm)
        for net, name in ((1, "grad_critic"), (0, "grad_actor")):
            dg = dgs[net]
            for k, ref in og[name].items():
                ref = np.asarray(ref, np.float64).reshape(dg[k].shape)
                scale = float(np.abs(ref).max()) or 1.0
                gerr = float(np.abs(dg[k] - ref).max()) / scale
                greport.append((i, net, k, gerr))
                # the batch-reduced gradient itself: fp32 summation order only
                # (observed <= 2.0e-6 of the tensor's largest entry)
                assert gerr < 1e-5, (i, name, k, gerr)
                conditioned[(net, k)] = np.abs(ref) > 1e-3 * scale
        # critic loss (pre-update) within 1e-5 relative; other stats fp64 reductions of fp32 values
        assert abs(got[0] - want[0]) <= 1e-5 * abs(want[0]) + 1e-7, (got[0], want[0])
        np.testing.assert_allclose(got[1:], want[1:], rtol=2e-5, atol=2e-6)
        for w, ref in (("actor", agents[i].actor), ("critic", agents[i].critic),
                       ("tgt_actor", agents[i].tgt_actor), ("tgt_critic", agents[i].tgt_critic)):
            dev = eng.get_params(i, w)
            for k in ref:
                err = np.abs(dev[k] - ref[k].reshape(dev[k].shape))
                report.append((i, w, k, float(err.max())))
                if w in ("actor", "critic"):
                    # where the gradient is not a near-cancelling sum (|g| > 1e-3 max|g|)
                    # Adam is well-conditioned: observed <= 2.5e-7
                    m = conditioned[(1 if w == "critic" else 0, k)].reshape(err.shape)
                    werr = float(err[m].max()) if m.any() else 0.0
                    wreport.append((i, w, k, werr))
                    assert werr < 1e-6, (i, w, k, werr)
                # every weight: Adam's first step is ~lr g / (|g| + 3e-7), so an
                # entry whose gradient is a near-cancelling sum (|g| ~ 1e-7) moves
                # by up to ~lr * (its relative rounding): observed <= 1.9e-5
                assert err.max() < 2e-4, (i, w, k, float(err.max()))
        for net in (0, 1):
            bp = eng.get_beta_powers(i, net)
            opt = agents[i].opt_actor if net == 0 else agents[i].opt_critic
            assert bp[0] == opt.b1p and bp[1] == opt.b2p
    worst = max(r[3] for r in report)
    print(f"update parity dims={dims} B={B} H={H} local_q={c['local_q']}: worst param |diff| = {worst:.3e}")
    print(f"   worst grad |diff|/max|g| = {max(r[3] for r in greport):.3e} (critic "
          f"{max(r[3] for r in greport if r[1] == 1):.3e}); worst conditioned param |diff| = "
          f"{max(r[3] for r in wreport):.3e}")
    for w in ("critic", "actor"):
        print(f"   clip_by_norm on the device gradient, {w}: theta vs fp64-norm step "
              f"{max(r[(w, 'fp64')] for r in creport):.3e}, vs fp32-norm (TF1 reduce_sum) step "
              f"{max(r[(w, 'fp32')] for r in creport):.3e}; |norm32 - norm64| / norm64 <= "
              f"{max(r[(w, 'norm_rel_gap')] for r in creport):.3e}")
    return worst


def test_update_parity_spread_b1024():
    _update_parity([18, 18, 18], B=1024, L=4000, seed=21)


@pytest.mark.parametrize("seed", [0, 1, 12345])
def test_update_parity_spread_survey_seeds(seed):
    # SURVEY 8d's synthetic-input seeds at BASELINE configs[1]'s update shape:
    # simple_spread N=3, B=1024, the replay filled to the gate (L = B * 25)
    _update_parity([18, 18, 18], B=1024, L=25600, seed=seed)


def test_update_parity_simple():
    _update_parity([4], B=1024, L=2000, seed=22)


def test_update_parity_adversary_mixed_ddpg():
    _update_parity([8, 10, 10], B=512, L=3000, seed=23, local_q=[True, False, False])


def test_update_parity_ragged_batch():
    _update_parity([18, 18, 18], B=200, L=900, seed=24)


def test_update_parity_tag6_h128():
    _update_parity([22, 22, 22, 22, 20, 20], B=256, L=1500, seed=25, H=128)


def test_update_parity_tag6_full_size():
    # BASELINE configs[4] at its full size: simple_tag N=6 (4 adversaries: obs 22,
    # 2 good: obs 20; critic input 158), H=128, B=4096 -> 256 gradient workgroups
    worst = _update_parity([22, 22, 22, 22, 20, 20], B=4096, L=102400, seed=28, H=128)
    assert worst < 2e-4


def test_update_parity_adversary_full_size():
    # BASELINE configs[3]: 1 DDPG adversary (critic input 13) + 2 MADDPG good agents, B=1024
    _update_parity([8, 10, 10], B=1024, L=25600, seed=29, local_q=[True, False, False])


def test_update_parity_tag4_h64_general_kernels():
    # 4 target actors: outside the register-resident kernels' envelope -> general kernels
    _update_parity([16, 16, 16, 14], B=512, L=2000, seed=26)


@pytest.mark.parametrize("local_q", [None, [True, False, False]])
def test_update_parity_general_kernels_forced(monkeypatch, local_q):
    # the general kernels (mdp_grads.hip) on a configuration the fast ones also serve
    monkeypatch.setenv("MDP_GENERAL_GRADS", "1")
    _update_parity([18, 18, 18], B=256, L=1200, seed=27, local_q=local_q)


def test_update_parity_general_ragged_batch(monkeypatch):
    # the general kernels' last 16-row tile only partly filled (B = 200: 12 tiles + 8 rows)
    monkeypatch.setenv("MDP_GENERAL_GRADS", "1")
    _update_parity([18, 18, 18], B=200, L=900, seed=31)


def test_update_parity_tag6_h128_ragged():
    # tag N=6 at H=128, B = 1000: the work-queue layer phase over 62 row tiles + 8 rows
    _update_parity([22, 22, 22, 22, 20, 20], B=1000, L=6000, seed=32, H=128)


@pytest.mark.parametrize("dims,H,B,local_q,general", [
    ([18, 18, 18], 64, 1024, None, False),                           # S2 shape, register-resident kernels
    ([8, 10, 10], 64, 512, [True, False, False], False),             # a DDPG critic: its own target actor only
    ([18, 18, 18], 64, 200, None, True),                             # general kernels, ragged
    ([22, 22, 22, 22, 20, 20], 128, 256, None, False),               # tag N=6, H=128
])
def test_update_parity_device_noise_is_pinned_philox(monkeypatch, dims, H, B, local_q, general):
    """mdp_update drawing its own Gumbel noise (no injected uniforms) is the
    oracle update on the KAT-pinned Philox uniforms of each agent's streams at
    counter i (agent i's update on a fresh engine), both key words in use"""
    if general:
        monkeypatch.setenv("MDP_GENERAL_GRADS", "1")
    _update_parity(dims, B=B, L=4 * B, seed=40 + B, local_q=local_q, H=H, device_noise_key=0xC0FFEE0123456789)


@pytest.mark.parametrize("dims,H,B,local_q", [
    ([66] * 8, 64, 100, None),                       # 8 agents, critic input 568
    ([95] * 3, 256, 80, [False, True, False]),       # H = 256, critic input 300, one DDPG critic
    ([33] * 8, 256, 48, None),                       # 8 agents at H = 256
])
def test_update_parity_lds_envelope_edge(dims, H, B, local_q):
    """the largest configurations the kernels' LDS envelope admits
    (tests/test_host_logic.py LDS_EDGE: one more obs unit is refused at create)
    train in parity with the oracle: the gradient tiles at ~160 KB of LDS and
    the optimizer on nets of up to 150K parameters"""
    _update_parity(dims, B=B, L=5 * B, seed=33 + H, local_q=local_q, H=H)


@pytest.mark.parametrize("dims,local_q,B,H", [([18, 18, 18], None, 1024, 64),
                                              ([8, 10, 10], [True, False, False], 256, 64),
                                              ([22, 22, 20], None, 256, 128)])
def test_update_parity_consecutive_rounds(dims, local_q, B, H):
    """Four consecutive strict-mode rounds (maddpg.py:161-196 per agent, agent
    order of train.py:160-161), each with fresh injected indices and Gumbel
    uniforms, vs the oracle carried along the same path.  Covers what one round
    cannot: Adam moments and beta powers at t = 2..4, targets drifting from
    Polyak on top of Polyak, later agents' critics reading earlier agents'
    stepped target actors of the same round.  Tolerances: critic loss 1e-5
    relative per round; after the last round every parameter within 1e-4
    absolute (fp32 summation-order noise over four Adam steps; observed on
    MI355X: 8.9e-7 spread, 8.0e-7 adversary, 7.3e-6 H=128)."""
    rounds, L = 4, 3000
    c = synthetic_trainer_case(dims, B, L, seed=71, local_q=local_q, H=H)
    n = len(dims)
    eng = Engine(dims, c["local_q"], num_units=H, batch_size=B, capacity=L + 7)
    eng.add_rows(torch.from_numpy(joint_rows(c["data"], dims)))
    for i, p in enumerate(c["params"]):
        for w in ("actor", "critic", "tgt_actor", "tgt_critic"):
            eng.set_params(i, w, p[w])
    agents = [trainer.AgentParams(**copy.deepcopy(p), local_q=c["local_q"][i]) for i, p in enumerate(c["params"])]
    rng = np.random.default_rng(72)
    for r in range(rounds):
        idx = rng.integers(0, L, size=(n, B)).astype(np.int32)
        u_tgt = rng.uniform(1e-6, 1.0, size=(n, n, B, 5)).astype(np.float32)
        u_act = rng.uniform(1e-6, 1.0, size=(n, B, 5)).astype(np.float32)
        for i in range(n):
            eng.update(i, idx=torch.from_numpy(idx[i]), u_tgt=torch.from_numpy(u_tgt[i]),
                       u_act=torch.from_numpy(u_act[i]))
            got = eng.stats(i)
            want, _ = trainer.update(agents, i, c["data"], idx[i], u_tgt[i], u_act[i])
            assert abs(got[0] - want[0]) <= 1e-5 * abs(want[0]) + 1e-7, (r, i, got[0], want[0])
            np.testing.assert_allclose(got[1:], want[1:], rtol=1e-4, atol=1e-5)
    worst = 0.0
    for i in range(n):
        for w, ref in (("actor", agents[i].actor), ("critic", agents[i].critic),
                       ("tgt_actor", agents[i].tgt_actor), ("tgt_critic", agents[i].tgt_critic)):
            dev = eng.get_params(i, w)
            for k in ref:
                err = float(np.abs(dev[k] - ref[k].reshape(dev[k].shape)).max())
                worst = max(worst, err)
                assert err < 1e-4, (i, w, k, err)
        for net in (0, 1):
            bp = eng.get_beta_powers(i, net)
            opt = agents[i].opt_actor if net == 0 else agents[i].opt_critic
            assert bp[0] == opt.b1p and bp[1] == opt.b2p
    print(f"{rounds} rounds dims={dims} B={B} H={H}: worst param |diff| = {worst:.3e}")


@pytest.mark.parametrize("dims,local_q,B,H,general", [
    ([18, 18, 18], None, 1024, 64, False), ([4], None, 512, 64, False),
    ([8, 10, 10], [True, False, False], 256, 64, False),
    # the general kernels: one gradient launch per agent and step kind
    ([22, 22, 22, 22, 20, 20], None, 256, 128, False), ([16, 16, 16, 14], None, 256, 64, False),
    ([8, 10, 10], [True, False, False], 256, 64, True),
    # BASELINE configs[4] at full size (the gradient-pair launch: 2 x 256 workgroups,
    # the per-agent optimizer pair, k_polyak) and a ragged batch of the same topology
    ([22, 22, 22, 22, 20, 20], None, 4096, 128, False), ([22, 22, 22, 22, 20, 20], None, 1000, 128, False)])
def test_throughput_mode_round_parity(monkeypatch, dims, local_q, B, H, general):
    """Throughput mode (opt-in): one round = every agent's critic and
    actor gradients from the round-start parameters, then every clip + Adam +
    Polyak (mdp_update_all) vs oracle.trainer.update_round_throughput on the
    same injected indices and uniforms: critic loss within 1e-5 relative,
    parameters within the fp32 tolerance of the strict-mode parity test."""
    _throughput_round_parity(monkeypatch, dims, local_q, B, H, general)


@pytest.mark.parametrize("dims,local_q,B,H,general", [
    ([18, 18, 18], None, 1024, 64, False), ([8, 10, 10], [True, False, False], 256, 64, True),
    ([22, 22, 22, 22, 20, 20], None, 1000, 128, False)])
def test_throughput_mode_device_noise_is_pinned_philox(monkeypatch, dims, local_q, B, H, general):
    """the same round drawing its own noise: agent i at counter upd_ctr + i
    (mdp_grads*.hip), i.e. the KAT-pinned Philox streams of strict mode's
    agent i on a fresh engine"""
    _throughput_round_parity(monkeypatch, dims, local_q, B, H, general, device_noise_key=0x5EED5EED00C0FFEE)


def _throughput_round_parity(monkeypatch, dims, local_q, B, H, general, device_noise_key=None):
    if general:
        monkeypatch.setenv("MDP_GENERAL_GRADS", "1")
    L = 3000
    c = synthetic_trainer_case(dims, B, L, seed=61, local_q=local_q, H=H)
    if device_noise_key is not None:
        _philox_case_noise(c, len(dims), B, device_noise_key)
        c["u_tgt"], c["u_act"] = np.stack(c["u_tgt"]), np.stack(c["u_act"])
    # no batch row with a ReLU input within 1e-5 of its layer's scale of zero: there two
    # correct fp32 evaluations may mask differently (see relu_margin_clean_idx; at B = 4096
    # the unconditioned batch flips one mask of agent 2's actor step, 7e-4 of max|g|)
    relu_margin_clean_idx(c)
    n = len(dims)
    kw = {} if device_noise_key is None else {"seed": device_noise_key}
    eng = Engine(dims, c["local_q"], num_units=H, batch_size=B, capacity=L + 7, **kw)
    eng.add_rows(torch.from_numpy(joint_rows(c["data"], dims)))
    for i, p in enumerate(c["params"]):
        for w in ("actor", "critic", "tgt_actor", "tgt_critic"):
            eng.set_params(i, w, p[w])
    eng.set_update_mode("throughput")
    agents = [trainer.AgentParams(**copy.deepcopy(p), local_q=c["local_q"][i]) for i, p in enumerate(c["params"])]
    # the round-start gradients of every agent (what update_round_throughput steps with)
    def round_grads():
        out = []
        for i in range(n):
            batch_n = [tuple(x[c["idx"][i]] for x in c["data"][j]) for j in range(n)]
            out.append({1: trainer.critic_grads(agents, i, batch_n, c["u_tgt"][i])[0],
                        0: trainer.actor_grads(agents, i, batch_n, c["u_act"][i])[0]})
        return out

    og = round_grads()
    old32 = (nets.F32, trainer.F32)
    nets.F32 = trainer.F32 = np.float64  # the same restatement in fp64: the fp32 rounding of the reference itself
    try:
        og64 = round_grads()
    finally:
        nets.F32, trainer.F32 = old32
    if device_noise_key is None:
        eng.update_all(idx=torch.from_numpy(c["idx"]), u_tgt=torch.from_numpy(c["u_tgt"]),
                       u_act=torch.from_numpy(c["u_act"]))
    else:                                         # the device's own Philox noise
        eng.update_all(idx=torch.from_numpy(c["idx"]))
    want = trainer.update_round_throughput(agents, c["data"], c["idx"], c["u_tgt"], c["u_act"])
    tworst, gworst, cworst = 0.0, 0.0, 0.0
    for i in range(n):
        got = eng.stats(i)
        assert abs(got[0] - want[i][0]) <= 1e-5 * abs(want[i][0]) + 1e-7, (i, got[0], want[i][0])
        np.testing.assert_allclose(got[1:], want[i][1:], rtol=2e-5, atol=2e-6)
        conditioned = {}
        for net in (0, 1):
            dg = _device_grads(eng, i, net)
            for k, ref in og[i][net].items():
                ref = np.asarray(ref, np.float64).reshape(dg[k].shape)
                r64 = np.asarray(og64[i][net][k], np.float64).reshape(dg[k].shape)
                scale = float(np.abs(r64).max()) or 1.0
                gerr = float(np.abs(dg[k] - r64).max()) / scale
                own = float(np.abs(ref - r64).max()) / scale   # the fp32 oracle's own rounding
                gworst = max(gworst, gerr)
                # the batch-reduced gradient against the fp64 restatement: fp32 summation
                # order only, within 1e-5 of the tensor's largest entry (the fp32 restatement's
                # own distance `own` is of the same order)
                assert gerr < 1e-5, (i, net, k, gerr, own)
                conditioned[(net, k)] = np.abs(r64) > 1e-3 * scale
        for w, ref in (("actor", agents[i].actor), ("critic", agents[i].critic),
                       ("tgt_actor", agents[i].tgt_actor), ("tgt_critic", agents[i].tgt_critic)):
            dev = eng.get_params(i, w)
            for k in ref:
                e = np.abs(dev[k] - ref[k].reshape(dev[k].shape))
                err = float(e.max())
                tworst = max(tworst, err)
                if w in ("actor", "critic"):
                    m = conditioned[(1 if w == "critic" else 0, k)].reshape(e.shape)
                    if m.any():
                        cworst = max(cworst, float(e[m].max()))
                        assert float(e[m].max()) < 1e-6, (i, w, k)   # Adam well-conditioned
                # every weight: Adam's first step is ~lr g / (|g| + eps), so an entry whose
                # gradient is a near-cancelling sum moves by up to ~lr x its relative rounding
                assert err < 2e-4, (i, w, k, err)
        for net in (0, 1):
            bp = eng.get_beta_powers(i, net)
            opt = agents[i].opt_actor if net == 0 else agents[i].opt_critic
            assert bp[0] == opt.b1p and bp[1] == opt.b2p
    print(f"throughput round dims={dims} B={B} H={H} general={general}: worst param |diff| = {tworst:.3e}, "
          f"worst grad |diff|/max|g| = {gworst:.3e}, worst conditioned param |diff| = {cworst:.3e}")
    assert _ctl_u32(eng, CTL_UPD_CTR_OFFSET) == n           # every agent used upd_ctr + agent
    assert _ctl_u32(eng, CTL_FAULT_OFFSET) == 0
    # strict mode again on the same handle: mode switches are clean
    eng.set_update_mode("strict")
    eng.update_round()
    eng.synchronize()
    assert all(np.all(np.isfinite(eng.stats(i))) for i in range(n))


def test_throughput_grad_pair_bit_identical(monkeypatch):
    """Throughput mode on the general kernels: agent i's critic and actor gradient
    steps as ONE launch (k_grad_pair, the default) and as two launches
    (MDP_GRAD_PAIR=0) give the same bits -- two rounds, tag N=6 at H=128."""
    dims, B, L = [22, 22, 22, 22, 20, 20], 512, 3000
    c = synthetic_trainer_case(dims, B, L, seed=66, H=128)
    n = len(dims)
    rng = np.random.default_rng(7)

    def run(pair):
        monkeypatch.setenv("MDP_GRAD_PAIR", pair)
        eng = Engine(dims, num_units=128, batch_size=B, capacity=L + 7)
        eng.add_rows(torch.from_numpy(joint_rows(c["data"], dims)))
        for i, p in enumerate(c["params"]):
            for w in ("actor", "critic", "tgt_actor", "tgt_critic"):
                eng.set_params(i, w, p[w])
        eng.set_update_mode("throughput")
        return eng

    a, b = run("1"), run("0")
    for r in range(2):
        idx = torch.from_numpy(rng.integers(0, L, size=(n, B)).astype(np.int32))
        for e in (a, b):
            e.update_all(idx=idx)
    a.synchronize()
    b.synchronize()
    for i in range(n):
        for w in ("actor", "critic", "tgt_actor", "tgt_critic", "m_actor", "v_critic"):
            pa, pb = a.get_params(i, w), b.get_params(i, w)
            for k in pa:
                np.testing.assert_array_equal(pa[k], pb[k])
        np.testing.assert_array_equal(a.stats(i), b.stats(i))


def test_torch_distributed_throughput_round_parity():
    """The torch.distributed fallback's throughput round (parallel.throughput_round
    over EngineOps: per-agent phase launches, ONE all-reduce over
    EngineOps.round_grad_view, steps x 1/G) against
    oracle.trainer.update_round_throughput.  The all-reduce stand-in doubles the
    span in place and G = 2, so a net outside the span would come out halved."""
    from maddpg_amd.parallel import EngineOps, throughput_round
    dims, B, L = [18, 18, 18], 512, 3000
    c = synthetic_trainer_case(dims, B, L, seed=63)
    n = len(dims)
    eng = Engine(dims, batch_size=B, capacity=L + 7)
    eng.add_rows(torch.from_numpy(joint_rows(c["data"], dims)))
    for i, p in enumerate(c["params"]):
        for w in ("actor", "critic", "tgt_actor", "tgt_critic"):
            eng.set_params(i, w, p[w])
    eng.set_update_mode("throughput")
    dev = torch.device("cuda")
    idx = torch.from_numpy(c["idx"]).to(dev)
    u_tgt = torch.from_numpy(c["u_tgt"]).to(dev)
    u_act = torch.from_numpy(c["u_act"]).to(dev)

    class Injected(EngineOps):  # the test's indices and uniforms instead of the device streams
        def draw_indices(self):
            pass

        def critic_grad(self, i):
            self.eng.critic_grad(i, idx[i], u_tgt[i])

        def actor_grad(self, i):
            self.eng.actor_grad(i, idx[i], u_act[i])

    span = []

    def allreduce(t):
        span.append(t.numel())
        t.mul_(2.0)

    throughput_round(Injected(eng), n, 2, allreduce)
    eng.synchronize()
    assert span == [int(eng.grad_view(n - 1, 1).data_ptr() - eng.grad_view(0, 0).data_ptr()) // 4
                    + eng.grad_view(n - 1, 1).numel()]
    agents = [trainer.AgentParams(**copy.deepcopy(p)) for p in c["params"]]
    trainer.update_round_throughput(agents, c["data"], c["idx"], c["u_tgt"], c["u_act"])
    for i in range(n):
        for w, ref in (("actor", agents[i].actor), ("critic", agents[i].critic),
                       ("tgt_actor", agents[i].tgt_actor), ("tgt_critic", agents[i].tgt_critic)):
            got = eng.get_params(i, w)
            for k in ref:
                assert np.max(np.abs(got[k] - ref[k].reshape(got[k].shape))) < 2e-4, (i, w, k)


@pytest.mark.parametrize("cfg", ["spread", "tag6_h128", "tag_ddpg_h64"])
def test_throughput_mode_train_step_graph_equals_eager(cfg):
    """mdp_train_step in throughput mode (rollout + k rounds as one graph) is the
    same work as env_step + k x update_round in throughput mode (tag6_h128: the
    general kernels, one gradient launch per agent and step kind; tag_ddpg_h64:
    DDPG adversaries pass the register kernels' limits, the MADDPG good agent
    (critic input 82) does not -- agent 0 alone would allow the critic-launch
    prefetch, so every round after a step's first must still draw fresh
    indices, in the optimizer pair launches)."""
    from maddpg_amd.runner import VecRunner
    kw = {"tag6_h128": dict(n_agents=6, scenario_adversaries=4, num_units=128),
          "tag_ddpg_h64": dict(num_adversaries=3, adv_policy="ddpg")}.get(cfg, {})
    scen = "simple_spread" if cfg == "spread" else "simple_tag"

    def make():
        r = VecRunner(scen, 64, batch_size=128, capacity=20000, seed=3, train_every=16, **kw)
        r.eng.set_update_mode("throughput")
        r.prefill()
        return r

    a, b = make(), make()
    for _ in range(3):
        t0 = a.train_step
        k = a.step()
        b.rollout()
        assert b.due_rounds(t0, b.train_step) == k
        for _ in range(k):
            b.train_round()
    a.eng.synchronize()
    b.eng.synchronize()
    assert a.rounds > 0
    for i in range(a.n):
        for w in ("actor", "critic", "tgt_actor", "tgt_critic", "m_critic", "v_actor"):
            pa, pb = a.eng.get_params(i, w), b.eng.get_params(i, w)
            for key in pa:
                np.testing.assert_array_equal(pa[key], pb[key])
        np.testing.assert_array_equal(a.eng.stats(i), b.eng.stats(i))


def _ctl_u32(eng, off):
    ctl = eng.region("ctl", torch.uint8).cpu().numpy()
    return int(ctl[off:off + 4].view(np.uint32)[0])


CTL_UPD_CTR_OFFSET = 2568  # Ctl.upd_ctr (mdp_topo.h)
CTL_FAULT_OFFSET = 2572    # Ctl.fault


def test_update_round_uses_device_index_stream():
    """mdp_update_round draws agent 0's B indices first, then agent 1's ...
    (maddpg.py:167 per agent, train.py:160-161 agent order) from the MT stream."""
    dims = [18, 18, 18]
    B, L = 256, 3000
    c = synthetic_trainer_case(dims, B, L, seed=31)
    eng = Engine(dims, batch_size=B, capacity=L)
    eng.add_rows(torch.from_numpy(joint_rows(c["data"], dims)))
    eng.init_params(5)
    eng.seed_py_random(1234)
    eng.update_round()
    eng.synchronize()
    g = random.Random(1234)
    want = np.array([[g.randint(0, L - 1) for _ in range(B)] for _ in range(3)])
    got = eng.region("index", torch.int32)[:3 * B].cpu().numpy().reshape(3, B)
    np.testing.assert_array_equal(got, want)
    for i in range(3):
        assert all(np.isfinite(eng.stats(i)))


def _rounds_engine(dims, B, L, c, rounds):
    eng = Engine(dims, batch_size=B, capacity=L)
    eng.add_rows(torch.from_numpy(joint_rows(c["data"], dims)))
    eng.init_params(7)
    eng.seed_py_random(99)
    for _ in range(rounds):
        eng.update_round()
    eng.synchronize()
    return eng



def test_fused_reduce_apply_matches_two_kernel_path(monkeypatch):
    """k_reduce_apply (one launch: batch reduction, cross-workgroup clip norm,
    Adam, Polyak, beta advance) vs k_reduce + k_apply: same index/noise streams,
    so one round agrees to fp32 summation order; 12 rounds: no spin timed out,
    identical optimizer step counts."""
    dims = [18, 18, 18]
    B, L = 1024, 5000
    c = synthetic_trainer_case(dims, B, L, seed=41)
    fused1 = _rounds_engine(dims, B, L, c, 1)
    fused12 = _rounds_engine(dims, B, L, c, 12)
    monkeypatch.setenv("MDP_UNFUSED_APPLY", "1")
    ref1 = _rounds_engine(dims, B, L, c, 1)
    ref12 = _rounds_engine(dims, B, L, c, 12)
    ctl = fused12.region("ctl", torch.uint8).cpu().numpy()
    assert int(ctl[CTL_FAULT_OFFSET:CTL_FAULT_OFFSET + 4].view(np.uint32)[0]) == 0
    for i in range(3):
        for net in (0, 1):
            np.testing.assert_array_equal(fused12.get_beta_powers(i, net), ref12.get_beta_powers(i, net))
        for w in ("actor", "critic", "tgt_actor", "tgt_critic", "m_actor", "v_critic"):
            a, b = fused1.get_params(i, w), ref1.get_params(i, w)
            for k in a:
                np.testing.assert_allclose(a[k], b[k], rtol=0, atol=2e-4, err_msg=f"{i} {w} {k}")
                assert np.all(np.isfinite(fused12.get_params(i, w)[k]))
        np.testing.assert_allclose(fused1.stats(i), ref1.stats(i), rtol=1e-4, atol=1e-6)


# --------------------------------------------------------------------- env
# ("simple_spread", 8, 0): the maximum sizes -- 8 agents (MDP_MAX_AGENTS) and 16
# entities (MDP_MAX_ENT), every thread of the rollout tile in the per-(env,
# entity) physics and 128 of them in the per-(env, agent) observations
SCENARIOS = [("simple", 1, 0), ("simple_spread", 3, 0), ("simple_adversary", 3, 1),
             ("simple_tag", 4, 3), ("simple_tag", 6, 4), ("simple_spread", 8, 0)]


def _oracle_scn(name, n, na):
    if name == "simple_tag":
        return mpe.SimpleTag(n_adv=na, n_good=n - na)
    if name == "simple_adversary":
        return mpe.SimpleAdversary(n_good=n - na, n_adv=na)
    if name == "simple_spread":
        return mpe.SimpleSpread(n)
    return mpe.Simple()


@pytest.mark.parametrize("name,n,na", SCENARIOS)
def test_env_step_parity(name, n, na):
    from maddpg_amd.envs import spec
    sp = spec(name, n, na if na else None)
    E = 37   # ragged: not a multiple of the 16-env tile
    eng = Engine(sp.obs_dims, batch_size=16, capacity=1000, num_envs=E, scenario=name,
                 num_adversaries=sp.num_adversaries, max_episode_len=25, seed=3)
    eng.env_reset()
    st = eng.env_state()
    assert np.all(np.abs(st["pos"]) <= 1.0) and np.all(st["vel"] == 0)
    sc = _oracle_scn(name, n, na)
    rng = np.random.default_rng(4)
    # move away from the reset state so velocities are non-zero
    for step in range(3):
        z = rng.normal(size=(E, n, ACT))
        act = (np.exp(z) / np.exp(z).sum(-1, keepdims=True)).astype(np.float32)
        st = eng.env_state()
        ost = {"pos": st["pos"].astype(np.float64), "vel": st["vel"].astype(np.float64), "goal": st["goal"]}
        obs0 = sc.observation(ost)
        nst, obs1, rew = sc.step(ost, act.astype(np.float64))
        eng.env_step(act_in=torch.from_numpy(act))
        got = eng.env_state()
        np.testing.assert_allclose(got["pos"], nst["pos"], atol=2e-5)
        np.testing.assert_allclose(got["vel"], nst["vel"], atol=2e-5)
        rows = eng.replay_rows(step * E, E).cpu().numpy()
        lay, _ = row_layout(sp.obs_dims)
        for j in range(n):
            lj, o = lay[j], sp.obs_dims[j]
            np.testing.assert_allclose(rows[:, lj["obs"]:lj["obs"] + o], obs0[j], atol=2e-5)
            np.testing.assert_array_equal(rows[:, lj["act"]:lj["act"] + ACT], act[:, j])
            np.testing.assert_allclose(rows[:, lj["nobs"]:lj["nobs"] + o], obs1[j], atol=2e-5)
            np.testing.assert_allclose(rows[:, lj["rew"]], rew[:, j], rtol=1e-5, atol=5e-5)
            assert np.all(rows[:, lj["done"]] == 0)
    assert eng.buffer_len() == 3 * E


@pytest.mark.parametrize("name,n,na", SCENARIOS + [("simple_adversary", 8, 1)])
def test_env_reset_is_the_scenario_reset_on_pinned_philox(name, n, na):
    """mdp_env_reset = the scenario's reset_world (oracle/mpe.py) drawing the
    device's Philox uniforms (oracle/philox.py, KAT-pinned): every position to
    fp32 rounding, velocities zero, the adversary goal exact.  The 8-agent
    spread (16 entities, 32 uniform slots) and the 8-agent adversary (15
    entities + the goal: 31 slots) need more than the 20 uniforms an earlier
    revision of env_reset_one kept, which it then read past; two resets
    advance the counter."""
    from oracle import philox
    from maddpg_amd.envs import spec
    sp = spec(name, n, na if na else None)
    E, seed = 37, 0x0123456789ABCDEF
    eng = Engine(sp.obs_dims, batch_size=16, capacity=1000, num_envs=E, scenario=name,
                 num_adversaries=sp.num_adversaries, max_episode_len=25, seed=seed)
    sc = _oracle_scn(name, n, na)
    ne = sc.n_entities
    for k in range(2):
        eng.env_reset()
        st = eng.env_state()
        u = philox.slot_uniforms(seed, 0x30000, k, np.arange(E), 2 * ne + 1)
        want = sc.reset(philox.ResetStream(u, ne), E)
        np.testing.assert_allclose(st["pos"], want["pos"], rtol=0, atol=1e-6, err_msg=f"reset {k}")
        assert np.all(st["vel"] == 0) and np.all(st["ep_step"] == 0)
        if name == "simple_adversary":
            np.testing.assert_array_equal(st["goal"], want["goal"])
            assert len(set(st["goal"].tolist())) > 1


def test_env_episode_reset_and_log():
    from maddpg_amd.envs import spec
    sp = spec("simple_spread")
    E = 20
    eng = Engine(sp.obs_dims, batch_size=16, capacity=1000, num_envs=E, scenario="simple_spread",
                 max_episode_len=3, seed=8)
    eng.env_reset()
    eng.init_params(0)
    for _ in range(3):
        eng.env_step()
    st = eng.env_state()
    assert np.all(st["ep_step"] == 0)
    assert eng.episode_count() == E
    log = eng.episode_log(0, E)
    rows = eng.replay_rows(0, 3 * E).cpu().numpy()
    lay, _ = row_layout(sp.obs_dims)
    per_env = sum(rows[k * E:(k + 1) * E, lay[j]["rew"]] for k in range(3) for j in range(3))
    # lockstep envs log in env order (slot = episodes + env index)
    np.testing.assert_allclose(log[:, 0], per_env, rtol=1e-5, atol=1e-4)
    np.testing.assert_allclose(log[:, 0], log[:, 1:].sum(1), rtol=1e-5, atol=1e-4)


def test_rollout_policy_actions_match_oracle():
    from maddpg_amd.envs import spec
    sp = spec("simple_spread")
    E = 40
    eng = Engine(sp.obs_dims, batch_size=16, capacity=1000, num_envs=E, scenario="simple_spread", seed=9)
    eng.init_params(3)
    eng.env_reset()
    obs = eng.env_obs().cpu().numpy()
    u = np.random.default_rng(2).uniform(1e-6, 1, size=(E, 3, ACT)).astype(np.float32)
    eng.env_step(u=torch.from_numpy(u))
    rows = eng.replay_rows(0, E).cpu().numpy()
    lay, _ = row_layout(sp.obs_dims)
    for j in range(3):
        p = eng.get_params(j, "actor")
        logits = nets.mlp_fwd(p, obs[:, lay[j]["obs"]:lay[j]["obs"] + 18])[0]
        want = nets.gumbel_softmax(logits, u[:, j])
        np.testing.assert_allclose(rows[:, lay[j]["act"]:lay[j]["act"] + ACT], want, atol=2e-6)


@pytest.mark.parametrize("name,n,na,H", [("simple_spread", 3, 0, 64), ("simple_tag", 6, 4, 128),
                                         ("simple_adversary", 8, 1, 64)])
def test_rollout_own_noise_and_episode_reset_are_pinned_philox(name, n, na, H):
    """k_rollout without injected uniforms: every stored action is the oracle's
    gumbel-softmax of the device actor on the stored obs with the KAT-pinned
    Philox uniforms of (seed, stream 0x10000 | agent, counter = vector step,
    row = env), and the episode end's env.reset() (train.py:127-133) is the
    scenario's reset_world on stream 0x20000 at the terminal step's counter."""
    from oracle import philox
    from maddpg_amd.envs import spec
    sp = spec(name, n, na if na else None)
    E, seed, T = 37, 0xDEADBEEF12345678, 3
    eng = Engine(sp.obs_dims, num_units=H, batch_size=16, capacity=1000, num_envs=E, scenario=name,
                 num_adversaries=sp.num_adversaries, max_episode_len=T, seed=seed)
    eng.init_params(4)
    eng.env_reset()
    lay, _ = row_layout(sp.obs_dims)
    actors = [eng.get_params(j, "actor") for j in range(n)]
    for k in range(T):
        eng.env_step()
        eng.synchronize()       # no injected tensors: the step did not order torch's stream after it
        rows = eng.replay_rows(k * E, E).cpu().numpy()
        for j in range(n):
            o = sp.obs_dims[j]
            logits = nets.mlp_fwd(actors[j], rows[:, lay[j]["obs"]:lay[j]["obs"] + o])[0]
            u = philox.uniforms5(seed, 0x10000 | j, k, np.arange(E))
            np.testing.assert_allclose(rows[:, lay[j]["act"]:lay[j]["act"] + ACT], nets.gumbel_softmax(logits, u),
                                       atol=2e-6, err_msg=f"step {k} agent {j}")
    st = eng.env_state()
    assert np.all(st["ep_step"] == 0) and eng.episode_count() == E
    sc = _oracle_scn(name, n, na)
    ne = sc.n_entities
    want = sc.reset(philox.ResetStream(philox.slot_uniforms(seed, 0x20000, T - 1, np.arange(E), 2 * ne + 1), ne), E)
    np.testing.assert_allclose(st["pos"], want["pos"], rtol=0, atol=1e-6)
    assert np.all(st["vel"] == 0)
    if name == "simple_adversary":
        np.testing.assert_array_equal(st["goal"], want["goal"])


@pytest.mark.parametrize("scenario,adv_policy,cap,general", [
    ("simple_spread", "maddpg", 20000, False),
    ("simple_spread", "maddpg", 3300, False),
    ("simple_spread", "maddpg", 20000, True),
    ("simple", "maddpg", 20000, False),             # one agent: no critic split carried onto itself
    ("simple_adversary", "ddpg", 20000, False),     # agent 0 a DDPG critic: the carry into it is skipped
])
def test_train_step_graph_equals_step_then_rounds(monkeypatch, scenario, adv_policy, cap, general):
    """mdp_train_step(k) (rollout + k rounds replayed as one graph; the first
    round's agent-0 indices drawn by an extra rollout workgroup, every later
    agent's B indices one agent ahead -- by the previous agent's fast critic
    kernel or, on the general kernels, in two pieces by its optimizer
    launches; the critic split carried from a round's last actor
    launch into the next round's agent 0) is the same work as env_step + k x
    update_round (eager rounds, no carry): bit-identical state and RNG stream
    after 4 steps.  cap=3300: the ring fills during the steps (draws against
    the capped length)."""
    from maddpg_amd.runner import VecRunner
    if general:
        monkeypatch.setenv("MDP_GENERAL_GRADS", "1")

    def make():
        r = VecRunner(scenario, 64, batch_size=128, capacity=cap, seed=3, train_every=16,
                      num_adversaries=1 if scenario == "simple_adversary" else 0, adv_policy=adv_policy)
        r.prefill()
        return r

    a, b = make(), make()
    for _ in range(4):
        t0 = a.train_step
        k = a.step()                      # world 1: mdp_train_step
        assert k == 4
        b.rollout()
        assert b.due_rounds(t0, b.train_step) == k
        for _ in range(k):
            b.train_round()
    a.eng.synchronize()
    b.eng.synchronize()
    for i in range(a.n):
        for w in ("actor", "critic", "tgt_actor", "tgt_critic"):
            pa, pb = a.eng.get_params(i, w), b.eng.get_params(i, w)
            for key in pa:
                np.testing.assert_array_equal(pa[key], pb[key])
    np.testing.assert_array_equal(a.eng.replay_rows(0, 2000).cpu().numpy(), b.eng.replay_rows(0, 2000).cpu().numpy())
    assert a.eng.buffer_len() == b.eng.buffer_len()
    np.testing.assert_array_equal(a.eng.get_rng_state(), b.eng.get_rng_state())


@pytest.mark.parametrize("general", [False, True])
def test_draw_ahead_equals_per_round_draw(monkeypatch, general):
    """The index draw one agent ahead (MDP_DRAW_AHEAD, default on: the rollout
    draws agent 0's B, every agent's launches the next agent's) is the same MT19937
    stream as one n*B draw per round (MDP_DRAW_AHEAD=0): bit-identical
    parameters, replay ring and RNG state after 4 training steps of 4 rounds,
    on the fast kernels and on the general ones (draw pieces in the optimizer
    launches)."""
    from maddpg_amd.runner import VecRunner
    if general:
        monkeypatch.setenv("MDP_GENERAL_GRADS", "1")

    def run(ahead):
        monkeypatch.setenv("MDP_DRAW_AHEAD", ahead)
        r = VecRunner("simple_spread", 64, batch_size=128, capacity=20000, seed=5, train_every=16)
        r.prefill()
        for _ in range(4):
            assert r.step() == 4
        r.eng.synchronize()
        return r

    a, b = run("1"), run("0")
    for i in range(a.n):
        for w in ("actor", "critic", "tgt_actor", "tgt_critic", "m_critic", "v_actor"):
            pa, pb = a.eng.get_params(i, w), b.eng.get_params(i, w)
            for key in pa:
                np.testing.assert_array_equal(pa[key], pb[key])
    np.testing.assert_array_equal(a.eng.replay_rows(0, 2000).cpu().numpy(), b.eng.replay_rows(0, 2000).cpu().numpy())
    np.testing.assert_array_equal(a.eng.get_rng_state(), b.eng.get_rng_state())


@pytest.mark.parametrize("general", [False, True])
def test_train_steps_group_graph_equals_step_graphs(monkeypatch, general):
    """mdp_train_steps (several consecutive steps captured as ONE graph, captured
    ahead of time with launch=0, then replayed) is the same work as the
    steps one by one (one graph per step): bit-identical parameters, Adam
    moments, replay ring, RNG stream and finished-episode count after two
    groups (5 + 3 steps; the ring fills and wraps on the way, cap=3300)."""
    from maddpg_amd.runner import VecRunner
    if general:
        monkeypatch.setenv("MDP_GENERAL_GRADS", "1")

    def make():
        r = VecRunner("simple_spread", 64, batch_size=128, capacity=3300, seed=7, train_every=16)
        r.prefill()
        r.step()                          # the one eager training step
        return r

    a, b = make(), make()
    sizes = a.prepare_steps(8, 5)
    assert sizes == [5, 3]
    ra = sum(a.steps(g) for g in sizes)
    rb = sum(b.step() for _ in range(8))
    assert ra == rb == 32 and a.train_step == b.train_step
    a.eng.synchronize()
    b.eng.synchronize()
    for i in range(a.n):
        for w in ("actor", "critic", "tgt_actor", "tgt_critic", "m_actor", "v_critic"):
            pa, pb = a.eng.get_params(i, w), b.eng.get_params(i, w)
            for key in pa:
                np.testing.assert_array_equal(pa[key], pb[key])
        for net in (0, 1):
            np.testing.assert_array_equal(a.eng.get_beta_powers(i, net), b.eng.get_beta_powers(i, net))
    np.testing.assert_array_equal(a.eng.replay_rows(0, 3300).cpu().numpy(), b.eng.replay_rows(0, 3300).cpu().numpy())
    assert a.eng.buffer_len() == b.eng.buffer_len()
    np.testing.assert_array_equal(a.eng.get_rng_state(), b.eng.get_rng_state())
    assert a.episodes() == b.episodes()


@pytest.mark.parametrize("scenario,E,every,gate_open,n,group", [
    ("simple_spread", 64, 100, True, 12, 6), ("simple_spread", 1, 100, True, 120, 60),
    ("simple_spread", 64, 100, False, 12, 6), ("simple_adversary", 16, 400, True, 60, 30),
    ("simple_tag", 8, 200, True, 60, 30)])
def test_train_steps_group_with_rollout_only_steps(scenario, E, every, gate_open, n, group):
    """Groups whose steps do not all train (64 transitions per step and a round
    per 100: rounds 1, 0, 1, 1, 0, ...; E = 1, the reference's own structure:
    one round in 100 steps; a group that starts below the replay gate): the
    group graph == the steps one by one, bit for bit, and the episode log.
    With E <= 16 a stretch of steps without a round is ONE k_rollout launch of
    that many steps (env state, returns and goals carried in LDS: the adversary's
    goal landmark and tag's collisions across episode ends included)."""
    from maddpg_amd.runner import VecRunner

    def make():
        r = VecRunner(scenario, E, batch_size=64, capacity=2000, seed=11, train_every=every)
        if gate_open:
            r.prefill()
            while r.step() == 0:              # the one eager training step
                pass
        return r

    a, b = make(), make()
    pa_ = a.plan(n)                           # E = 1: the next round is 100 steps after the eager one
    assert 0 in pa_ and (not gate_open or any(pa_)), pa_
    if gate_open:
        sizes = a.prepare_steps(n, group)
    else:                                     # below the gate: no eager step yet, groups fall back to one by one
        sizes = [group] * (n // group)
    ra = sum(a.steps(g) for g in sizes)
    rb = sum(b.step() for _ in range(n))
    assert ra == rb and a.train_step == b.train_step and a.rounds == b.rounds
    a.eng.synchronize()
    b.eng.synchronize()
    for i in range(a.n):
        for w in ("actor", "critic", "tgt_actor", "tgt_critic", "m_actor", "v_critic"):
            pa, pb = a.eng.get_params(i, w), b.eng.get_params(i, w)
            for key in pa:
                np.testing.assert_array_equal(pa[key], pb[key])
    np.testing.assert_array_equal(a.eng.replay_rows(0, 2000).cpu().numpy(), b.eng.replay_rows(0, 2000).cpu().numpy())
    assert a.eng.buffer_len() == b.eng.buffer_len()
    np.testing.assert_array_equal(a.eng.get_rng_state(), b.eng.get_rng_state())
    assert a.episodes() == b.episodes()
    np.testing.assert_array_equal(a.episode_rewards(0, a.episodes()), b.episode_rewards(0, b.episodes()))


# ---------------------------------------------------- size-independent checks
def test_full_size_index_stream_properties():
    """BASELINE S3-sized draw (1e6-row ring, 6 x 4096 indices): bit-exact vs
    CPython and the stream position continues correctly across calls."""
    eng = Engine([18, 18, 18], batch_size=4096, capacity=1_000_000)
    eng.set_ring(1_000_000, 0)
    eng.seed_py_random(2024)
    g = random.Random(2024)
    for _ in range(3):
        got = eng.make_index(6 * 4096).cpu().numpy()
        want = [g.randint(0, 999_999) for _ in range(6 * 4096)]
        np.testing.assert_array_equal(got, want)
    np.testing.assert_array_equal(eng.get_rng_state(), np.array(g.getstate()[1], np.uint32))


# ------------------------------------------------------- --benchmark records
@pytest.mark.parametrize("name,n,na", [s for s in SCENARIOS if s[0] != "simple"])
def test_env_benchmark_data_parity(name, n, na):
    """mdp_env_step_bench: every agent's benchmark_data() record of the
    post-physics state equals the oracle's on that same (device) state."""
    from maddpg_amd.envs import bench_record, spec
    sp = spec(name, n, na if na else None)
    E = 37
    eng = Engine(sp.obs_dims, batch_size=16, capacity=1000, num_envs=E, scenario=name,
                 num_adversaries=sp.num_adversaries, max_episode_len=25, seed=5)
    eng.init_params(2)
    eng.env_reset()
    sc = _oracle_scn(name, n, na)
    for _ in range(4):
        info = eng.env_step_bench().cpu().numpy()
        st = eng.env_state()                       # not terminal: the post-physics state
        ost = {"pos": st["pos"].astype(np.float64), "vel": st["vel"].astype(np.float64), "goal": st["goal"]}
        want = sc.benchmark_data(ost)
        for i in range(n):
            w = want[i]
            np.testing.assert_allclose(info[:, i, :w.shape[1]], w, rtol=1e-5, atol=2e-5)
            assert np.all(info[:, i, w.shape[1]:] == 0)
            for e in range(0, E, 7):
                got_rec, want_rec = bench_record(sp, info[e, i], i), sc.record(w[e], i)
                assert type(got_rec) is type(want_rec)
    # simple has no benchmark_data (the reference's make_env raises)
    s1 = Engine([4], batch_size=16, capacity=100, num_envs=4, scenario="simple")
    with pytest.raises(Exception, match="benchmark_data"):
        s1.env_step_bench()


@pytest.mark.parametrize("dims,local_q", [([18, 18, 18], None), ([8, 10, 10], [True, False, False]), ([4], None)])
def test_split_steps_bit_identical(monkeypatch, dims, local_q):
    """The actor step's forward computed in the critic launch (actor_pre) and
    the critic step split around the previous agent's update (critic_pre ->
    critic_post within a round) are scheduling choices: the same MFMA chains in
    the same order.  Three rounds with both on (update_round), with both off
    (MDP_ACTOR_PRE=0 MDP_CRITIC_PRE=0), and agent by agent through mdp_update
    (no cross-agent split) must agree bit for bit.  The split carried ACROSS
    rounds (mdp_train_step) is covered by
    test_train_step_graph_equals_step_then_rounds, incl. one agent and a DDPG
    agent 0."""
    B, L = 256, 3000
    c = synthetic_trainer_case(dims, B, L, seed=91, local_q=local_q)
    n = len(dims)

    def run(mode):
        eng = Engine(dims, c["local_q"], batch_size=B, capacity=L)
        eng.add_rows(torch.from_numpy(joint_rows(c["data"], dims)))
        eng.init_params(4)
        eng.seed_py_random(17)
        for _ in range(3):
            if mode == "agents":
                for i in range(n):
                    eng.update(i)
            else:
                eng.update_round()
        eng.synchronize()
        return eng

    on, agents = run("round"), run("agents")
    monkeypatch.setenv("MDP_ACTOR_PRE", "0")
    monkeypatch.setenv("MDP_CRITIC_PRE", "0")
    off = run("round")
    for i in range(n):
        for w in ("actor", "critic", "tgt_actor", "tgt_critic", "m_actor", "v_critic"):
            a, b, d = on.get_params(i, w), off.get_params(i, w), agents.get_params(i, w)
            for k in a:
                np.testing.assert_array_equal(a[k], b[k], err_msg=f"{i} {w} {k} split vs unsplit")
                np.testing.assert_array_equal(a[k], d[k], err_msg=f"{i} {w} {k} round vs per-agent")
        np.testing.assert_array_equal(on.stats(i), off.stats(i))


def test_agent_update_literal_abi_vs_oracle():
    """mdp_agent_update (SURVEY 8b's one-call update: gates at t, update, 6 stats)
    against mdp_update + mdp_get_stats and the oracle: below the replay gate
    and off the t % 100 cadence it returns None without drawing (the device MT
    state is unchanged); on the cadence it trains with the injected indices and
    uniforms and returns the oracle's stats."""
    dims, B = [18, 18, 18], 256
    L = B * 25 + 100                      # past the gate: len >= B * max_episode_len
    c = synthetic_trainer_case(dims, B, L, seed=71)
    rows = joint_rows(c["data"], dims)
    engines = []
    for n_rows in (B * 25 - 1, L):
        e = Engine(dims, batch_size=B, capacity=L + 7)
        e.add_rows(torch.from_numpy(rows[:n_rows]))
        for i, p in enumerate(c["params"]):
            for w in ("actor", "critic", "tgt_actor", "tgt_critic"):
                e.set_params(i, w, p[w])
        engines.append(e)
    eng, eng2 = engines
    st0, st1 = eng.get_rng_state(), eng2.get_rng_state()
    assert eng.agent_update(0, 100) is None                     # len < B * 25: maddpg.py:162-163
    assert eng2.agent_update(0, 101) is None                    # t % 100 != 0: maddpg.py:164-165
    assert np.array_equal(eng.get_rng_state(), st0) and np.array_equal(eng2.get_rng_state(), st1)
    agents = [trainer.AgentParams(**copy.deepcopy(p)) for p in c["params"]]
    for i in range(3):
        u = np.concatenate([c["u_tgt"][i].ravel(), c["u_act"][i].ravel()])
        got = eng2.agent_update(i, 200, idx=torch.from_numpy(c["idx"][i]), u=torch.from_numpy(u))
        want, _ = trainer.update(agents, i, c["data"], c["idx"][i], c["u_tgt"][i], c["u_act"][i])
        assert type(got) is list and len(got) == 6
        # the reference's dtypes (maddpg.py:91,54-56,185,196), the oracle's too
        assert [type(x) for x in got] == [type(x) for x in want] == list(UPDATE_STAT_DTYPES)
        assert [float(x) for x in got] == [float(t(v)) for t, v in zip(UPDATE_STAT_DTYPES, eng2.stats(i))]
        assert abs(got[0] - want[0]) <= 1e-5 * abs(want[0]) + 1e-7, (got, want)
        np.testing.assert_allclose(np.array(got[1:], np.float64), np.array(want[1:], np.float64),
                                   rtol=2e-5, atol=2e-6)


def test_check_finite_counts_nan_and_inf():
    """mdp_check_finite (the reference's opt-in check_nan, tf_util.py:322,366-368):
    0 on a trained engine; a NaN weight and an Inf Adam slot are counted; the
    facade raises the reference's "Nan detected" from update() when the session
    asks for the check."""
    dims, B, L = [18, 18, 18], 256, 1200
    c = synthetic_trainer_case(dims, B, L, seed=51)
    eng = Engine(dims, batch_size=B, capacity=L)
    eng.add_rows(torch.from_numpy(joint_rows(c["data"], dims)))
    eng.init_params(3)
    eng.update(0, idx=torch.from_numpy(c["idx"][0]))
    eng.synchronize()
    assert eng.check_finite() == 0
    w = eng.get_params(1, "critic")
    w["W2"][3, 5] = np.nan
    eng.set_params(1, "critic", w)
    assert eng.check_finite() == 1
    v = eng.get_params(2, "v_actor")
    v["b1"][0] = np.inf
    eng.set_params(2, "v_actor", v)
    assert eng.check_finite() == 2


def test_facade_check_nan_raises_like_the_reference():
    import argparse

    from maddpg_amd.common import tf_util as U
    from maddpg_amd.envs import Discrete
    from maddpg_amd.trainer.maddpg import MADDPGAgentTrainer
    args = argparse.Namespace(lr=1e-2, gamma=0.95, batch_size=32, num_units=64, max_episode_len=2)
    rng = np.random.default_rng(0)
    with U.single_threaded_session(check_nan=True):
        trainers = [MADDPGAgentTrainer(f"agent_{i}", None, [(18,)] * 3, [Discrete(5)] * 3, i, args)
                    for i in range(3)]
        U.initialize()
        for _ in range(100):
            obs = [rng.uniform(-1, 1, 18).astype(np.float32) for _ in range(3)]
            act = [np.full(5, 0.2, np.float32) for _ in range(3)]
            for i, ag in enumerate(trainers):
                ag.experience(obs[i], act[i], -1.0, obs[i], False, False)
        assert trainers[0].update(trainers, 100) is not None       # finite: trains, no raise
        eng = U.get_session().engine()
        w = eng.get_params(0, "actor")
        w["W1"][0, 0] = np.nan
        eng.set_params(0, "actor", w)
        with pytest.raises(RuntimeError, match="Nan detected"):
            trainers[1].update(trainers, 200)


def test_update_parity_non_default_constants():
    """The reference's hard-coded constants as train.py flags (--tau, --grad-clip,
    --actor-reg): one update per agent with tau 0.05, clip 0.2, actor
    regulariser 1e-2 against the oracle run with the same constants."""
    dims, B, L = [18, 18, 18], 512, 3000
    c = synthetic_trainer_case(dims, B, L, seed=61)
    tau, clip, reg = 0.05, 0.2, 1e-2
    eng = Engine(dims, batch_size=B, capacity=L + 7, tau=tau, grad_clip=clip, actor_reg=reg)
    eng.add_rows(torch.from_numpy(joint_rows(c["data"], dims)))
    for i, p in enumerate(c["params"]):
        for w in ("actor", "critic", "tgt_actor", "tgt_critic"):
            eng.set_params(i, w, p[w])
    agents = [trainer.AgentParams(**copy.deepcopy(p)) for p in c["params"]]
    for i in range(3):
        eng.update(i, idx=torch.from_numpy(c["idx"][i]), u_tgt=torch.from_numpy(c["u_tgt"][i]),
                   u_act=torch.from_numpy(c["u_act"][i]))
        got = eng.stats(i)
        want, _ = trainer.update(agents, i, c["data"], c["idx"][i], c["u_tgt"][i], c["u_act"][i],
                                 grad_clip=clip, tau=tau, actor_reg=reg)
        assert abs(got[0] - want[0]) <= 1e-5 * abs(want[0]) + 1e-7, (i, got[0], want[0])
        assert abs(got[1] - want[1]) <= 2e-5 * abs(want[1]) + 2e-6, (i, got[1], want[1])   # p_loss uses reg
        for w, ref in (("actor", agents[i].actor), ("tgt_actor", agents[i].tgt_actor),
                       ("critic", agents[i].critic), ("tgt_critic", agents[i].tgt_critic)):
            dev = eng.get_params(i, w)
            for k in ref:
                assert np.max(np.abs(dev[k] - ref[k].reshape(dev[k].shape))) < 2e-4, (i, w, k)
