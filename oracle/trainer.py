"""Restatement of ``MADDPGAgentTrainer`` (``maddpg/trainer/maddpg.py:28-196``) in numpy.

All randomness is injected so the HIP path can be checked on identical inputs:
``idx`` (replay indices, normally from ``oracle.pyrandom``), ``u_tgt``
(uniforms for every agent's target-actor Gumbel sample, ``maddpg.py:70,184``)
and ``u_act`` (uniforms for the actor-loss Gumbel sample, ``maddpg.py:49``).

Semantics reproduced deliberately:
* target nets initialised independently (caller supplies them);
* TD target ``rew + gamma*(1-done)*Q'`` in float64 (``maddpg.py:186``), fed
  to the fp32 placeholder (``:83``);
* critic loss returned pre-update (``tf_util.py:364``); actor uses the
  post-update critic (``maddpg.py:188,191``);
* per-tensor clip 0.5 (``:130,142``), own Adam per net, Polyak actor then
  critic (``:193-194``); agents update sequentially and later agents see the
  earlier agents' Polyak-updated target actors (``experiments/train.py:160-161``).
"""
import numpy as np

from . import nets

F32 = np.float32


class AgentParams:
    def __init__(self, actor, critic, tgt_actor, tgt_critic, local_q=False, lr=1e-2):
        self.actor, self.critic = actor, critic
        self.tgt_actor, self.tgt_critic = tgt_actor, tgt_critic
        self.local_q = local_q
        self.opt_actor = nets.Adam(actor, lr=lr)
        self.opt_critic = nets.Adam(critic, lr=lr)


def critic_input(obs_n, act_n, i, local_q):
    if local_q:                                      # maddpg.py:86-87
        return np.concatenate([obs_n[i], act_n[i]], 1).astype(F32)
    return np.concatenate(list(obs_n) + list(act_n), 1).astype(F32)   # :85


def target_act(ag, obs, u):
    """p_debug['target_act'] (maddpg.py:66-71)."""
    logits, _ = nets.mlp_fwd(ag.tgt_actor, obs)
    return nets.gumbel_softmax(logits, u)


def act(ag, obs, u):
    """MADDPGAgentTrainer.action / p_train's act (maddpg.py:45,62,151-152)."""
    logits, _ = nets.mlp_fwd(ag.actor, obs)
    return nets.gumbel_softmax(logits, u)


def update(agents, i, buffers, idx, u_tgt, u_act, gamma=0.95, grad_clip=0.5):
    """One ``agents[i].update(agents, t)`` past the gates (maddpg.py:167-196).

    buffers[j] = (obs[L,o_j], act[L,A], rew[L], obs_next[L,o_j], done[L]) of
    agent j.  Returns the 6 stats and mutates agents[i] params in place.
    """
    n = len(agents)
    ag = agents[i]
    obs_n, act_n, obs_next_n = [], [], []
    for j in range(n):                              # :173-177
        o, a, _r, on, _d = buffers[j]
        obs_n.append(o[idx].astype(F32))
        act_n.append(a[idx].astype(F32))
        obs_next_n.append(on[idx].astype(F32))
    rew = buffers[i][2][idx].astype(np.float64)      # :178
    done = buffers[i][4][idx].astype(np.float64)
    B = len(idx)

    # ---- train q network (:180-188)
    tgt_act_n = [target_act(agents[j], obs_next_n[j], u_tgt[j]) for j in range(n)]
    xq_t = critic_input(obs_next_n, tgt_act_n, i, ag.local_q)
    target_q_next = nets.mlp_fwd(ag.tgt_critic, xq_t)[0][:, 0]
    target_q = rew + gamma * (1.0 - done) * target_q_next.astype(np.float64)
    y = target_q.astype(F32)

    xq = critic_input(obs_n, act_n, i, ag.local_q)
    q, cache = nets.mlp_fwd(ag.critic, xq)
    q = q[:, 0]
    q_loss = np.mean((q.astype(np.float64) - y.astype(np.float64)) ** 2)
    dq = ((F32(2) * (q - y)) * F32(1.0 / B)).astype(F32)[:, None]
    gq = nets.mlp_bwd(ag.critic, cache, dq)
    gq = {k: nets.clip_by_norm(v, grad_clip) for k, v in gq.items()}
    ag.opt_critic.apply(ag.critic, gq)

    # ---- train p network (:190-191; loss :46-56)
    logits, pcache = nets.mlp_fwd(ag.actor, obs_n[i])
    a_i = nets.gumbel_softmax(logits, u_act)
    act_in = list(act_n)
    act_in[i] = a_i
    xp = critic_input(obs_n, act_in, i, ag.local_q)
    qp, qcache = nets.mlp_fwd(ag.critic, xp)
    qp = qp[:, 0]
    A = logits.shape[1]
    p_reg = np.mean(logits.astype(np.float64) ** 2)
    p_loss = -np.mean(qp.astype(np.float64)) + 1e-3 * p_reg
    dqp = np.full((B, 1), -1.0 / B, F32)
    dx = nets.input_grad(ag.critic, qcache, dqp)
    off = (obs_n[i].shape[1] if ag.local_q else sum(o.shape[1] for o in obs_n)) + \
        (0 if ag.local_q else A * i)
    da = dx[:, off:off + A]
    dz = nets.softmax_bwd(a_i, da)
    dlogits = (dz + logits * F32(2e-3 / (B * A))).astype(F32)
    gp = nets.mlp_bwd(ag.actor, pcache, dlogits)
    gp = {k: nets.clip_by_norm(v, grad_clip) for k, v in gp.items()}
    ag.opt_actor.apply(ag.actor, gp)

    # ---- target updates (:193-194)
    nets.polyak(ag.tgt_actor, ag.actor)
    nets.polyak(ag.tgt_critic, ag.critic)

    return [float(q_loss), float(p_loss), float(np.mean(target_q)), float(np.mean(rew)),
            float(np.mean(target_q_next.astype(np.float64))), float(np.std(target_q))], \
        {"grad_critic": gq, "grad_actor": gp, "y": y, "q": q}
