"""Data parallelism for the MADDPG update (one process per GPU, RCCL over xGMI).

Sharding: every rank owns an independent shard of env copies,
its own replay shard and its own CPython-compatible index stream
(``seed + rank``); actor/critic parameters and Adam state are replicated and
stay bit-identical because every rank applies the same all-reduced gradient
with the same deterministic clip + Adam kernel.

Exchange step (strict reference semantics, ``maddpg.py:188-194`` order): per
agent, the critic gradient is reduced on device into one flat fp32 buffer,
summed across ranks with ONE all-reduce, scaled by 1/G inside the apply
kernel, clipped per tensor and applied; then the same for the actor (whose
loss uses the updated critic).  That is 2 all-reduces per agent per round --
the order the reference's sequential update implies.  Messages are 23-150 KB:
latency-bound on xGMI, so each is a single flat buffer (no per-tensor calls).

The orchestration below is backend-agnostic: ``ops`` is the Engine on a GPU
and an oracle-backed stand-in in the CPU (gloo) tests.
"""
import os

import torch
import torch.distributed as dist


def init_process_group_from_env(backend=None):
    """torchrun-style init (RANK/WORLD_SIZE/MASTER_ADDR/MASTER_PORT).

    MDP_SHARED_GPU=1 is a rehearsal of the multi-rank path on a 1-GPU box:
    every rank on cuda:0 and a gloo process group (RCCL refuses two ranks on
    one device); the data path (xGMI exchange or torch.distributed fallback)
    is unchanged."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        return 1, 0, 0
    rank = int(os.environ["RANK"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    if os.environ.get("MDP_SHARED_GPU", "0") == "1":
        local, backend = 0, "gloo"
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(local)
    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(backend=backend)
    return world, rank, local


def make_allreduce(stream=None):
    """sum all-reduce of a flat fp32 tensor, ordered on `stream` (the engine's)."""
    def allreduce(t):
        if stream is None:
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
        else:
            with torch.cuda.stream(stream):
                dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return allreduce


def strict_round(ops, n_agents, world_size, allreduce):
    """One update round in the reference's order with 2 all-reduces per agent.

    ops: draw_indices(), critic_grad(i), actor_grad(i), reduce_grad(i, net),
         grad_view(i, net) -> flat tensor, apply_grad(i, net, scale)
    net 1 = critic (Adam only), net 0 = actor (Adam + Polyak of both nets).
    """
    ops.draw_indices()                       # maddpg.py:167 for every agent, agent 0 first
    scale = 1.0 / float(world_size)
    for i in range(n_agents):                # train.py:160-161
        ops.critic_grad(i)                   # maddpg.py:180-188 (grads)
        ops.reduce_grad(i, 1)
        allreduce(ops.grad_view(i, 1))
        ops.apply_grad(i, 1, scale)          # clip + Adam (tf_util.py:177-182)
        ops.actor_grad(i)                    # maddpg.py:191 with the updated critic
        ops.reduce_grad(i, 0)
        allreduce(ops.grad_view(i, 0))
        ops.apply_grad(i, 0, scale)          # clip + Adam + Polyak (maddpg.py:193-194)


def throughput_round(ops, n_agents, world_size, allreduce):
    """One round of the opt-in throughput mode (NOT the reference's
    order) with ONE all-reduce: every agent's critic gradients (targets from the
    round-start target actors) and actor gradients (against the round-start
    critic), the whole gradient region summed over the ranks at once, then every
    clip + Adam (x 1/G) and Polyak -- oracle.trainer.update_round_throughput on
    the global batch.  The torch.distributed counterpart of the library's native
    throughput DP round (reduce pass -> ncclAllReduce -> step pass).

    ops: as strict_round, plus round_grad_view() -> one flat tensor spanning
    every net's gradient (written by reduce_grad)."""
    ops.draw_indices()
    scale = 1.0 / float(world_size)
    for i in range(n_agents):
        ops.critic_grad(i)                   # partials of this net, reduced before the next launch
        ops.reduce_grad(i, 1)
        ops.actor_grad(i)                    # round-start critic: nothing stepped yet
        ops.reduce_grad(i, 0)
    allreduce(ops.round_grad_view())
    for i in range(n_agents):
        ops.apply_grad(i, 1, scale)
        ops.apply_grad(i, 0, scale)          # + Polyak of both nets


class EngineOps:
    """strict_round ops on a maddpg_amd Engine (device indices for this rank)."""

    def __init__(self, eng):
        self.eng = eng
        self.idx = eng.region("index", torch.int32)

    def draw_indices(self):
        e = self.eng
        e.make_index(e.n * e.batch_size, out=self.idx[: e.n * e.batch_size])

    def _slot(self, i):
        B = self.eng.batch_size
        return self.idx[i * B:(i + 1) * B]

    def critic_grad(self, i):
        self.eng.critic_grad(i, self._slot(i))

    def actor_grad(self, i):
        self.eng.actor_grad(i, self._slot(i))

    def reduce_grad(self, i, net):
        self.eng.reduce_grad(i, net)

    def grad_view(self, i, net):
        return self.eng.grad_view(i, net)

    def apply_grad(self, i, net, scale):
        self.eng.apply_grad(i, net, scale)

    def round_grad_view(self):
        """every agent's actor + critic gradient: one contiguous span of the GRAD region"""
        e = self.eng
        g = e.region("grad")
        a = e.grad_view(0, 0)
        z = e.grad_view(e.n - 1, 1)
        start = (a.data_ptr() - g.data_ptr()) // 4
        end = (z.data_ptr() - g.data_ptr()) // 4 + z.numel()
        return g[start:end]


def xgmi_handshake(ops, world, rank):
    """Set-up of the direct xGMI gradient exchange (mdp_dp_xgmi_*), every rank
    in step over torch.distributed.  ops: open(world, rank) -> 64-byte handle,
    connect(handles in rank order), probe(), enable(), close() -- the Engine on
    a GPU, a stand-in in the CPU (gloo) tests.  Enables only when every rank
    succeeded at every stage; otherwise closes it on every rank and returns
    (False, error of this rank or None) so all ranks fall back together."""
    dev = getattr(ops, "device", None)

    def agree(ok):
        t = torch.tensor([1 if ok else 0], dtype=torch.int32,
                         device=dev if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return bool(t.item())

    err = None
    try:
        handle = ops.open(world, rank)
    except Exception as e:  # noqa: BLE001 -- every rank falls back together
        handle, err = None, e
    handles = [None] * world
    dist.all_gather_object(handles, handle)
    ok = all(x is not None for x in handles)
    if ok:
        try:
            ops.connect(handles)
        except Exception as e:  # noqa: BLE001
            ok, err = False, e
    ok = agree(ok)
    if ok:
        try:
            ops.probe()
        except Exception as e:  # noqa: BLE001
            ok, err = False, e
        ok = agree(ok)
    if ok:
        ops.enable()
    else:
        ops.close()
    return ok, err
