"""CPU baseline: the reference's training loop restated on the oracle (TEST/BASELINE ONLY).

Follows ``experiments/train.py:110-161`` call for call: per env step, N
batch-1 ``action()`` calls (``maddpg.py:151-152``), one MPE step, N
``experience()`` appends to Python-list replay buffers
(``replay_buffer.py:25-32``), episode bookkeeping with reset at
``max_episode_len``, ``train_step += 1``, then ``preupdate()`` and
``update(trainers, train_step)`` for every agent in order, each gated on
``len(buffer) >= batch*max_episode_len`` and ``train_step % 100 == 0``
(``maddpg.py:162-165``) and gathering N+1 times through ``sample_index``
(``maddpg.py:173-178``).  Math is numpy fp32 (fp64 MPE, fp64 TD target) on one
thread, standing in for TF1's ``single_threaded_session`` (``tf_util.py:202-204``).

bench.py times a bounded sample of it on the GPU box's host (``cpu_baseline``
with ``kind: "port"``); the reference itself cannot run there (TF1 absent,
the reference never travels).

    OMP_NUM_THREADS=1 python -m oracle.train_loop --seconds 15
"""
import argparse
import json
import os
import time

import numpy as np

from . import mpe, nets, trainer
from .pyrandom import MT19937
from .replay import ReplayBuffer


def make_scenario(name, n_agents=None, n_adv=None):
    if name == "simple_tag" and n_agents:
        return mpe.SimpleTag(n_adv=n_adv or 3, n_good=n_agents - (n_adv or 3))
    return mpe.make(name)


def run(scenario="simple_spread", seconds=15.0, batch_size=1024, num_units=64, max_episode_len=25,
        seed=0, prefill=None, gamma=0.95, max_steps=None, local_q=None):
    sc = make_scenario(scenario)
    n = sc.n_agents
    dims = sc.obs_dims()
    rng = np.random.default_rng(seed)
    S = sum(dims)
    agents = []
    local_q = [False] * n if local_q is None else list(local_q)     # train.py:67-74 (ddpg: local critic)
    for i in range(n):
        cin = dims[i] + 5 if local_q[i] else S + 5 * n
        agents.append(trainer.AgentParams(
            nets.xavier_init(rng, dims[i], 5, num_units), nets.xavier_init(rng, cin, 1, num_units),
            nets.xavier_init(rng, dims[i], 5, num_units), nets.xavier_init(rng, cin, 1, num_units),
            local_q=local_q[i]))
    bufs = [ReplayBuffer(1e6) for _ in range(n)]
    g = MT19937(seed)
    gate = batch_size * max_episode_len
    prefill = gate if prefill is None else prefill
    # untimed prefill with synthetic transitions so the sample exercises training
    for _ in range(prefill):
        for i in range(n):
            o = rng.uniform(-1, 1, dims[i])
            z = rng.normal(size=5)
            a = (np.exp(z) / np.exp(z).sum()).astype(np.float32)
            bufs[i].add(o, a, float(rng.normal(-3, 1)), rng.uniform(-1, 1, dims[i]), 0.0)

    st = sc.reset(rng, 1)
    obs_n = sc.observation(st)
    episode_step = 0
    train_step = prefill
    env_steps = updates = 0
    ep_rew, episode_rewards = np.zeros(n), []                      # train.py:121-124 (per agent)
    t0 = time.perf_counter()
    while True:
        action_n = []
        for i in range(n):                                         # train.py:112
            u = rng.random((1, 5), dtype=np.float32)                   # [0, 1) like tf.random_uniform
            action_n.append(trainer.act(agents[i], obs_n[i][0:1], u)[0])
        st, new_obs_n, rew = sc.step(st, np.array(action_n)[None])  # :114
        episode_step += 1
        terminal = episode_step >= max_episode_len
        for i in range(n):                                         # :119-120
            bufs[i].add(obs_n[i][0], action_n[i], float(rew[0, i]), new_obs_n[i][0], 0.0)
        obs_n = new_obs_n
        ep_rew += rew[0]
        if terminal:                                               # :127-128
            episode_rewards.append([float(ep_rew.sum())] + [float(v) for v in ep_rew])
            ep_rew = np.zeros(n)
            st = sc.reset(rng, 1)
            obs_n = sc.observation(st)
            episode_step = 0
        train_step += 1                                            # :136
        env_steps += 1
        for i in range(n):                                         # :158-161
            if len(bufs[i]) < gate or train_step % 100 != 0:
                continue
            idx = bufs[i].make_index(batch_size, g)
            batch_n = [bufs[j].sample_index(idx) for j in range(n)]
            own = bufs[i].sample_index(idx)
            batch_n[i] = own
            # fp32 draws in [0, 1): a float64 draw cast to fp32 rounds to 1.0 about
            # once in 3e7 draws, and u = 1 makes -log(-log u) infinite (NaN actions)
            u_tgt = rng.random((n, batch_size, 5), dtype=np.float32)
            u_act = rng.random((batch_size, 5), dtype=np.float32)
            trainer.update_batch(agents, i, batch_n, u_tgt, u_act, gamma)
            updates += 1
        el = time.perf_counter() - t0
        if (el >= seconds and train_step % 100 == 0) or (max_steps and env_steps >= max_steps):
            break
    el = time.perf_counter() - t0
    return {"env_steps_per_sec": env_steps / el, "trainer_updates_per_sec": updates / el,
            "env_steps": env_steps, "updates": updates, "seconds": el, "scenario": scenario,
            "batch_size": batch_size, "num_units": num_units, "prefill": prefill, "n_agents": n,
            "episode_rewards": episode_rewards}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scenario", default="simple_spread")
    ap.add_argument("--seconds", type=float, default=15.0)
    ap.add_argument("--batch-size", type=int, default=1024)
    ap.add_argument("--num-units", type=int, default=64)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--pin-core", type=int, default=0)
    a = ap.parse_args()
    if a.pin_core >= 0 and hasattr(os, "sched_setaffinity"):
        try:
            os.sched_setaffinity(0, {a.pin_core})
        except OSError:
            pass
    out = run(a.scenario, a.seconds, a.batch_size, a.num_units, seed=a.seed)
    out["threads"] = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
