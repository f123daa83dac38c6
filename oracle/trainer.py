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


def update(agents, i, buffers, idx, u_tgt, u_act, gamma=0.95, grad_clip=0.5, tau=1e-2, actor_reg=1e-3):
    """One ``agents[i].update(agents, t)`` past the gates (maddpg.py:167-196).

    buffers[j] = (obs[L,o_j], act[L,A], rew[L], obs_next[L,o_j], done[L]) of
    agent j.  Returns the 6 stats and mutates agents[i] params in place.
    """
    n = len(agents)
    batch_n = [tuple(x[idx] for x in buffers[j]) for j in range(n)]   # :173-178
    return update_batch(agents, i, batch_n, u_tgt, u_act, gamma, grad_clip, tau, actor_reg)


def critic_grads(agents, i, batch_n, u_tgt, gamma=0.95):
    """maddpg.py:180-188 up to the raw (unclipped) critic gradients."""
    n = len(agents)
    ag = agents[i]
    obs_n = [b[0].astype(F32) for b in batch_n]
    act_n = [b[1].astype(F32) for b in batch_n]
    obs_next_n = [b[3].astype(F32) for b in batch_n]
    rew = np.asarray(batch_n[i][2], np.float64)
    done = np.asarray(batch_n[i][4], np.float64)
    B = len(rew)
    tgt_act_n = [target_act(agents[j], obs_next_n[j], u_tgt[j]) for j in range(n)]
    xq_t = critic_input(obs_next_n, tgt_act_n, i, ag.local_q)
    target_q_next = nets.mlp_fwd(ag.tgt_critic, xq_t)[0][:, 0]
    target_q = rew + gamma * (1.0 - done) * target_q_next.astype(np.float64)   # :186 (fp64)
    y = target_q.astype(F32)                                                     # :83 fp32 placeholder
    xq = critic_input(obs_n, act_n, i, ag.local_q)
    q, cache = nets.mlp_fwd(ag.critic, xq)
    q = q[:, 0]
    q_loss = np.mean((q.astype(np.float64) - y.astype(np.float64)) ** 2)     # :91
    dq = ((F32(2) * (q - y)) * F32(1.0 / B)).astype(F32)[:, None]
    g = nets.mlp_bwd(ag.critic, cache, dq)
    stats = {"q_loss": float(q_loss), "target_q": target_q, "rew": rew, "target_q_next": target_q_next}
    return g, stats


def actor_grads(agents, i, batch_n, u_act, actor_reg=1e-3):
    """maddpg.py:37-58 raw actor gradients (critic = its current, post-step weights)."""
    ag = agents[i]
    obs_n = [b[0].astype(F32) for b in batch_n]
    act_n = [b[1].astype(F32) for b in batch_n]
    B = obs_n[0].shape[0]
    logits, pcache = nets.mlp_fwd(ag.actor, obs_n[i])
    a_i = nets.gumbel_softmax(logits, u_act)                      # :49 fresh sample
    act_in = list(act_n)
    act_in[i] = a_i
    xp = critic_input(obs_n, act_in, i, ag.local_q)
    qp, qcache = nets.mlp_fwd(ag.critic, xp)
    qp = qp[:, 0]
    A = logits.shape[1]
    p_reg = np.mean(logits.astype(np.float64) ** 2)               # :46
    p_loss = -np.mean(qp.astype(np.float64)) + actor_reg * p_reg   # :54-56
    dqp = np.full((B, 1), -1.0 / B, F32)
    dx = nets.input_grad(ag.critic, qcache, dqp)
    off = (obs_n[i].shape[1] if ag.local_q else sum(o.shape[1] for o in obs_n)) + \
        (0 if ag.local_q else A * i)
    dz = nets.softmax_bwd(a_i, dx[:, off:off + A])
    dlogits = (dz + logits * F32(2 * actor_reg / (B * A))).astype(F32)
    return nets.mlp_bwd(ag.actor, pcache, dlogits), float(p_loss)


def apply_grads(opt, params, g, grad_clip=0.5):
    """minimize_and_clip (tf_util.py:177-182): per-tensor clip, then Adam."""
    opt.apply(params, {k: nets.clip_by_norm(v, grad_clip) for k, v in g.items()})


def reference_stats(st, p_loss):
    """``update()``'s return value (maddpg.py:196) with the reference's dtypes:
    ``q_loss`` / ``p_loss`` are the fp32 scalars ``U.function`` fetches from
    TF1 (``:91``, ``:54-56``; TF's fp32 ``reduce_mean`` accumulation order is
    unpinned -- restated as the fp64 mean rounded once to fp32);
    ``np.mean(target_q_next)`` is numpy's mean of the fp32 Q' array (fp32,
    ``:185``); ``np.mean(target_q)``, ``np.mean(rew)`` and ``np.std(target_q)``
    are float64 (the TD target is fp64, ``:186``; rewards come from the float64
    replay arrays)."""
    tq = st["target_q"]
    return [np.float32(st["q_loss"]), np.float32(p_loss), np.float64(np.mean(tq)), np.float64(np.mean(st["rew"])),
            np.mean(st["target_q_next"].astype(F32)), np.float64(np.std(tq))]


def update_batch(agents, i, batch_n, u_tgt, u_act, gamma=0.95, grad_clip=0.5, tau=1e-2, actor_reg=1e-3):
    """``update`` on already-gathered batches batch_n[j] = sample_index(idx) of agent j."""
    ag = agents[i]
    gq, st = critic_grads(agents, i, batch_n, u_tgt, gamma)
    apply_grads(ag.opt_critic, ag.critic, gq, grad_clip)          # :188
    gp, p_loss = actor_grads(agents, i, batch_n, u_act, actor_reg)  # :191 (post-step critic)
    apply_grads(ag.opt_actor, ag.actor, gp, grad_clip)
    nets.polyak(ag.tgt_actor, ag.actor, tau)                       # :193
    nets.polyak(ag.tgt_critic, ag.critic, tau)                     # :194
    return reference_stats(st, p_loss), {"grad_critic": gq, "grad_actor": gp}


def update_round_throughput(agents, buffers, idx_n, u_tgt_n, u_act_n, gamma=0.95, grad_clip=0.5):
    """Throughput mode -- NOT the reference's order: every
    agent's critic gradients (targets from the round-start target actors) and
    actor gradients (against the round-start critic) first, then every clip +
    Adam + Polyak.  idx_n[i], u_tgt_n[i] (= agent i's u_tgt), u_act_n[i].
    Returns the per-agent stats lists."""
    n = len(agents)
    grads, stats = [], []
    for i in range(n):
        batch_n = [tuple(x[idx_n[i]] for x in buffers[j]) for j in range(n)]
        gq, st = critic_grads(agents, i, batch_n, u_tgt_n[i], gamma)
        gp, p_loss = actor_grads(agents, i, batch_n, u_act_n[i])
        grads.append((gq, gp))
        stats.append(reference_stats(st, p_loss))
    for i, ag in enumerate(agents):
        gq, gp = grads[i]
        apply_grads(ag.opt_critic, ag.critic, gq, grad_clip)
        apply_grads(ag.opt_actor, ag.actor, gp, grad_clip)
        nets.polyak(ag.tgt_actor, ag.actor)
        nets.polyak(ag.tgt_critic, ag.critic)
    return stats
