"""Second, independent derivation of the trainer oracle's gradients.

oracle/trainer.py differentiates the reference's losses by hand (the
backward of mlp_model, of the critic-input slice a_i, of the Gumbel-softmax
and of the 1e-3 regulariser).  Here the same losses are written forward-only
in torch and differentiated by torch.autograd in float64:

  critic  maddpg.py:85-91    L_q = mean((Q_i(concat(obs_n, act_n)) - y)^2),
                             y = r + gamma (1 - d) Q'_i(concat(obs'_n, a~_n)),
                             a~_j = softmax(mu'_j(obs'_j) - log(-log u_j))
  actor   maddpg.py:37-58    L_p = -mean(Q_i(obs_n, act_n with a_i := softmax(
                             mu_i(obs_i) - log(-log u)))) + 1e-3 mean(mu_i(obs_i)^2),
                             gradients w.r.t. the actor's variables only

The oracle is run in float64 too (its dtype is a module constant), so the two
derivations must agree to rounding (1e-10 relative), on S2 (spread N=3), S4
(adversary with a DDPG agent, critic input [o_i, a_i]) and S5 (tag N=6 at
H=128) shapes.  A misreading shared by the hand-written backward and the HIP
kernels (slice offset of a_i in the critic input, the regulariser's scale,
the softmax backward) would fail here.  This does not pin TF1 itself (absent).
"""
import contextlib

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from oracle import nets, trainer  # noqa: E402
from tests.helpers import synthetic_trainer_case  # noqa: E402

F64 = torch.float64


@contextlib.contextmanager
def fp64_oracle():
    old = (nets.F32, trainer.F32)
    nets.F32 = trainer.F32 = np.float64
    try:
        yield
    finally:
        nets.F32, trainer.F32 = old


def _t(p, grad=False):
    return {k: torch.tensor(np.asarray(v, np.float64), dtype=F64, requires_grad=grad) for k, v in p.items()}


def _mlp(p, x):
    h1 = torch.relu(x @ p["W1"] + p["b1"])
    h2 = torch.relu(h1 @ p["W2"] + p["b2"])
    return h2 @ p["W3"] + p["b3"]


def _gsm(logits, u):
    return torch.softmax(logits - torch.log(-torch.log(u)), dim=-1)


def _cin(obs_n, act_n, i, local_q):
    return torch.cat([obs_n[i], act_n[i]], 1) if local_q else torch.cat(list(obs_n) + list(act_n), 1)


def _case(dims, B, H, local_q, seed):
    c = synthetic_trainer_case(dims, B, L=4 * B, seed=seed, local_q=local_q, H=H)
    n = len(dims)
    idx = c["idx"][0]
    batch_n = [tuple(np.asarray(x[idx], np.float64) for x in c["data"][j]) for j in range(n)]
    params = [{w: {k: np.asarray(v, np.float64) for k, v in p[w].items()} for w in p} for p in c["params"]]
    return c, n, batch_n, params


CASES = [([18, 18, 18], 64, 64, None), ([8, 10, 10], 48, 64, [True, False, False]),
         ([22, 22, 22, 22, 20, 20], 32, 128, None)]


@pytest.mark.parametrize("dims,B,H,local_q", CASES)
def test_critic_grads_match_autograd(dims, B, H, local_q):
    gamma = 0.95
    c, n, batch_n, params = _case(dims, B, H, local_q, seed=101)
    lq = c["local_q"]
    for i in range(n):
        u_tgt = np.asarray(c["u_tgt"][i], np.float64)
        with fp64_oracle():
            agents = [trainer.AgentParams(**{w: dict(p[w]) for w in p}, local_q=lq[j]) for j, p in enumerate(params)]
            g, st = trainer.critic_grads(agents, i, batch_n, u_tgt, gamma)
        obs_n = [torch.tensor(b[0], dtype=F64) for b in batch_n]
        act_n = [torch.tensor(b[1], dtype=F64) for b in batch_n]
        obs2_n = [torch.tensor(b[3], dtype=F64) for b in batch_n]
        rew, done = torch.tensor(batch_n[i][2], dtype=F64), torch.tensor(batch_n[i][4], dtype=F64)
        with torch.no_grad():
            tgt_act = [_gsm(_mlp(_t(params[j]["tgt_actor"]), obs2_n[j]), torch.tensor(u_tgt[j], dtype=F64))
                       for j in range(n)]
            q_next = _mlp(_t(params[i]["tgt_critic"]), _cin(obs2_n, tgt_act, i, lq[i]))[:, 0]
            y = rew + gamma * (1.0 - done) * q_next                           # maddpg.py:186
        cp = _t(params[i]["critic"], grad=True)
        q = _mlp(cp, _cin(obs_n, act_n, i, lq[i]))[:, 0]
        loss = torch.mean((q - y) ** 2)                                       # maddpg.py:91
        gt = dict(zip(cp, torch.autograd.grad(loss, list(cp.values()))))
        assert abs(st["q_loss"] - loss.item()) <= 1e-12 * abs(loss.item())
        np.testing.assert_allclose(st["target_q"], y.numpy(), rtol=1e-12, atol=1e-12)
        for k in nets.NAMES:
            want = gt[k].numpy().reshape(np.shape(g[k]))
            np.testing.assert_allclose(g[k], want, rtol=1e-10, atol=1e-14 * max(1.0, np.abs(want).max()),
                                       err_msg=f"agent {i} critic {k}")


@pytest.mark.parametrize("dims,B,H,local_q", CASES)
def test_actor_grads_match_autograd(dims, B, H, local_q):
    reg = 1e-3
    c, n, batch_n, params = _case(dims, B, H, local_q, seed=202)
    lq = c["local_q"]
    for i in range(n):
        u_act = np.asarray(c["u_act"][i], np.float64)
        with fp64_oracle():
            agents = [trainer.AgentParams(**{w: dict(p[w]) for w in p}, local_q=lq[j]) for j, p in enumerate(params)]
            g, p_loss = trainer.actor_grads(agents, i, batch_n, u_act, actor_reg=reg)
        obs_n = [torch.tensor(b[0], dtype=F64) for b in batch_n]
        act_n = [torch.tensor(b[1], dtype=F64) for b in batch_n]
        ap = _t(params[i]["actor"], grad=True)
        logits = _mlp(ap, obs_n[i])                                           # maddpg.py:39
        act_in = list(act_n)
        act_in[i] = _gsm(logits, torch.tensor(u_act, dtype=F64))             # :45-49
        q = _mlp(_t(params[i]["critic"]), _cin(obs_n, act_in, i, lq[i]))[:, 0]   # :50-53
        loss = -torch.mean(q) + reg * torch.mean(logits ** 2)                # :46,54-56
        gt = dict(zip(ap, torch.autograd.grad(loss, list(ap.values()))))
        assert abs(p_loss - loss.item()) <= 1e-12 * abs(loss.item())
        for k in nets.NAMES:
            want = gt[k].numpy().reshape(np.shape(g[k]))
            np.testing.assert_allclose(g[k], want, rtol=1e-10, atol=1e-14 * max(1.0, np.abs(want).max()),
                                       err_msg=f"agent {i} actor {k}")


def test_fp64_switch_restores_fp32():
    with fp64_oracle():
        assert nets.F32 is np.float64
    assert nets.F32 is np.float32 and trainer.F32 is np.float32
    y, _ = nets.mlp_fwd(nets.xavier_init(np.random.default_rng(0), 3, 2, 8), np.ones((2, 3)))
    assert y.dtype == np.float32
