"""Vectorised, device-resident version of ``experiments/train.py``'s loop.

One ``step()`` = one vector env step of E env copies on this rank (actors +
Gumbel + MPE physics + replay append + episode resets, ``k_rollout``) followed
by the update rounds the reference cadence makes due: the reference trains
when ``train_step % 100 == 0`` with ``train_step`` counting single-env steps
(``maddpg.py:164``, ``train.py:136``); with E copies ``train_step`` advances
by E per vector step, so a round runs for every multiple of 100 crossed
(E=1 is exactly the reference).  The replay-size gate (``maddpg.py:162``)
applies unchanged.  Index draws, gathers, both optimiser steps and Polyak
updates run on the device in the reference's agent order.
"""
import os
from . import envs
from .engine import Engine
from .parallel import EngineOps, make_allreduce, strict_round, throughput_round


def rounds_due(t_before, t_after, every=100):
    """update rounds for train_step going t_before -> t_after: one per multiple of
    `every` crossed (maddpg.py:164 ``t % 100 == 0`` checked at every t)."""
    return t_after // every - t_before // every


def select_exchange(eng, world_size, rank, environ=None):
    """Which gradient exchange a data-parallel rank runs over, decided the
    same on every rank: the direct xGMI exchange when every rank opened,
    connected and probed it (parallel.xgmi_handshake; a peer that never
    answers the probe fails it after the probe's bounded wait), else the
    library's own RCCL communicator, else torch.distributed (strict_round).
    Returns (native_dp, kind)."""
    env = os.environ if environ is None else environ
    if world_size <= 1:
        return False, None
    if env.get("MDP_NATIVE_DP", "1") == "1":
        if env.get("MDP_DP_XGMI", "1") == "1" and eng.dp_xgmi_init_from_dist(world_size, rank):
            return True, "native-xgmi"
        if eng.dp_init_from_dist(world_size, rank):
            return True, "native-rccl"
    return False, "torch.distributed"


class VecRunner:
    def __init__(self, scenario="simple_spread", num_envs=1024, *, n_agents=None, scenario_adversaries=None,
                 num_adversaries=0, good_policy="maddpg", adv_policy="maddpg", batch_size=1024,
                 num_units=64, lr=1e-2, gamma=0.95, max_episode_len=25, capacity=int(1e6), seed=0,
                 train_every=100, world_size=1, rank=0, device=None, episode_log_rows=0, tau=1e-2,
                 grad_clip=0.5, actor_reg=1e-3):
        sp = envs.spec(scenario, n_agents, scenario_adversaries)
        self.spec = sp
        n = sp.n_agents
        n_adv_pol = min(n, num_adversaries)                  # train.py:84
        local_q = [(adv_policy == "ddpg") if i < n_adv_pol else (good_policy == "ddpg") for i in range(n)]
        self.eng = Engine(sp.obs_dims, local_q, num_units=num_units, batch_size=batch_size,
                          max_episode_len=max_episode_len, capacity=capacity, num_envs=num_envs,
                          scenario=scenario, num_adversaries=sp.num_adversaries, lr=lr, gamma=gamma,
                          tau=tau, grad_clip=grad_clip, actor_reg=actor_reg,
                          seed=seed * 1000003 + 17, world_size=world_size, rank=rank, device=device,
                          episode_log_rows=episode_log_rows)
        self.eng.init_params(seed)                           # identical replicas on every rank
        self.eng.seed_py_random(seed + rank)                 # per-rank index stream
        self.eng.env_reset()
        self.n = n
        self.num_envs = num_envs
        self.batch_size = batch_size
        self.gate = batch_size * max_episode_len
        self.train_every = train_every
        self.world_size = world_size
        self.train_step = 0
        self.rounds = 0
        self._ops = EngineOps(self.eng) if world_size > 1 else None
        self._allreduce = make_allreduce(self.eng.stream) if world_size > 1 else None
        # native data parallelism: the library's own RCCL communicator, so a whole
        # vector step (rollout + due rounds with their all-reduces) is one C call;
        # MDP_NATIVE_DP=0 keeps the torch.distributed path (strict_round).  The
        # exchange is the direct xGMI one inside the optimizer kernel when every
        # rank can map every peer (MDP_DP_XGMI=0: RCCL all-reduces instead)
        self.native_dp, self.dp_kind = select_exchange(self.eng, world_size, rank)

    def rollout(self):
        self.eng.env_step()
        self.train_step += self.num_envs

    def due_rounds(self, t_before, t_after):
        if self.eng.buffer_len() < self.gate:
            return 0
        return rounds_due(t_before, t_after, self.train_every)

    def train_round(self):
        if self.world_size == 1:
            self.eng.update_round()
        elif getattr(self.eng, "update_mode", "strict") == "throughput":
            throughput_round(self._ops, self.n, self.world_size, self._allreduce)
        else:
            strict_round(self._ops, self.n, self.world_size, self._allreduce)
        self.rounds += 1

    def step(self):
        t0 = self.train_step
        if self.world_size == 1 or self.native_dp:
            # rollout + the due rounds as one graph replay (mdp_train_step); the
            # cadence is decided on the host from the ring mirror after this step
            t1 = t0 + self.num_envs
            len_after = min(self.eng.capacity, self.eng.buffer_len() + self.num_envs)
            k = 0 if len_after < self.gate else rounds_due(t0, t1, self.train_every)
            self.eng.train_step(k)
            self.train_step = t1
            self.rounds += k
            return k
        self.rollout()
        k = self.due_rounds(t0, self.train_step)
        for _ in range(k):
            self.train_round()
        return k

    def plan(self, n, skip=0):
        """the update rounds of vector steps skip .. skip + n - 1 from now (the
        cadence of step(); 0 for a step that does not train: replay below the
        gate, or no multiple of train_every crossed)"""
        ks, t, ln = [], self.train_step, self.eng.buffer_len()
        for i in range(skip + n):
            ln = min(self.eng.capacity, ln + self.num_envs)
            k = 0 if ln < self.gate else rounds_due(t, t + self.num_envs, self.train_every)
            t += self.num_envs
            if i >= skip:
                ks.append(k)
        return ks

    def steps(self, n):
        """n (<= 64) vector steps as one graph replay (mdp_train_steps: the steps
        that do not train are their rollout launch alone) on a single GPU or
        the native exchanges; otherwise step() n times.  Returns the update
        rounds run."""
        ks = self.plan(n) if (self.world_size == 1 or self.native_dp) else None
        if ks is None:
            return sum(self.step() for _ in range(n))
        self.eng.train_steps(ks)
        self.train_step += n * self.num_envs
        self.rounds += sum(ks)
        return sum(ks)

    def prepare_steps(self, n, group):
        """capture ahead of time the graphs steps(group) will replay over the next
        n vector steps (nothing runs); returns the group sizes to call steps() with"""
        sizes = [min(group, n - i) for i in range(0, n, group)]
        if self.world_size == 1 or self.native_dp:
            done = 0
            for g in sizes:
                ks = self.plan(g, skip=done)
                if ks is not None:
                    self.eng.train_steps(ks, launch=False)
                done += g
        return sizes

    def prefill(self):
        """vector steps without training until the replay gate opens (train.py warm-up)."""
        while self.eng.buffer_len() < self.gate:
            self.rollout()

    def episodes(self):
        return self.eng.episode_count()

    def episode_rewards(self, first, count):
        """[count, 1 + n]: total reward (sum over agents) then per-agent rewards."""
        return self.eng.episode_log(first, count)

    def stats(self, agent):
        return self.eng.stats(agent)

    def synchronize(self):
        self.eng.synchronize()
