"""Data-parallel update path on CPU: world_size 2 over gloo.

``maddpg_amd.parallel.strict_round`` is the orchestration the GPU ranks run
(reduce -> all_reduce -> apply(scale 1/G) per optimizer phase, agents in the
reference order).  Here its ops are backed by the oracle: each rank computes
gradients on its half of the batch; after the round the replicas must be
identical and equal to the single-process update on the whole batch.
"""
import copy
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from maddpg_amd.parallel import make_allreduce, strict_round, throughput_round
from oracle import nets, trainer
from tests.helpers import synthetic_trainer_case

NAMES = ("W1", "b1", "W2", "b2", "W3", "b3")


class OracleOps:
    """strict_round ops on oracle math (the GPU path uses parallel.EngineOps)."""

    def __init__(self, agents, batches, u_tgt, u_act):
        self.agents, self.batches, self.u_tgt, self.u_act = agents, batches, u_tgt, u_act
        self.g, self.flat = {}, {}

    def draw_indices(self):
        pass

    def critic_grad(self, i):
        self.g[(i, 1)] = trainer.critic_grads(self.agents, i, self.batches[i], self.u_tgt[i])[0]

    def actor_grad(self, i):
        self.g[(i, 0)] = trainer.actor_grads(self.agents, i, self.batches[i], self.u_act[i])[0]

    def reduce_grad(self, i, net):
        g = self.g[(i, net)]
        self.flat[(i, net)] = torch.from_numpy(np.concatenate([g[k].ravel() for k in NAMES]).astype(np.float32))

    def grad_view(self, i, net):
        return self.flat[(i, net)]

    def round_grad_view(self):
        """every net's flat gradient as views of ONE tensor (the one all-reduce of a
        throughput round sums them all in place)"""
        keys = sorted(self.flat)
        whole = torch.cat([self.flat[k] for k in keys])
        s = 0
        for k in keys:
            n = self.flat[k].numel()
            self.flat[k] = whole[s:s + n]
            s += n
        return whole

    def apply_grad(self, i, net, scale):
        ag = self.agents[i]
        params = ag.critic if net else ag.actor
        flat = self.flat[(i, net)].numpy()
        g, s = {}, 0
        for k in NAMES:
            n = params[k].size
            g[k] = (flat[s:s + n].reshape(params[k].shape) * np.float32(scale)).astype(np.float32)
            s += n
        trainer.apply_grads(ag.opt_critic if net else ag.opt_actor, params, g)
        if net == 0:
            nets.polyak(ag.tgt_actor, ag.actor)
            nets.polyak(ag.tgt_critic, ag.critic)


def _case():
    dims = [6, 8, 7]
    c = synthetic_trainer_case(dims, B=64, L=200, seed=42, H=16)
    return dims, c


def _batches(c, rows):
    n = len(c["params"])
    out = []
    for i in range(n):
        idx = c["idx"][i][rows]
        out.append([tuple(x[idx] for x in c["data"][j]) for j in range(n)])
    return out


def _worker(rank, world, port, q, mode="strict"):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dims, c = _case()
    B = 64
    rows = slice(rank * B // world, (rank + 1) * B // world)
    agents = [trainer.AgentParams(**copy.deepcopy(p)) for p in c["params"]]
    ops = OracleOps(agents, _batches(c, rows), c["u_tgt"][:, :, rows], c["u_act"][:, rows])
    rnd = strict_round if mode == "strict" else throughput_round
    rnd(ops, len(dims), world, make_allreduce(None))
    flat = np.concatenate([np.concatenate([a.actor[k].ravel() for k in NAMES] +
                                          [a.critic[k].ravel() for k in NAMES] +
                                          [a.tgt_actor[k].ravel() for k in NAMES] +
                                          [a.tgt_critic[k].ravel() for k in NAMES]) for a in agents])
    q.put((rank, flat))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_ranks(world, mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, mode)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    # replicas bit-identical
    for r in range(1, world):
        np.testing.assert_array_equal(res[0], res[r])
    return res


@pytest.mark.parametrize("world", [2, 4, 8])
def test_strict_round_ranks_match_full_batch(world):
    res = _run_ranks(world, "strict")
    # equal to the single-process update on the whole batch (reference order)
    dims, c = _case()
    agents = [trainer.AgentParams(**copy.deepcopy(p)) for p in c["params"]]
    batches = _batches(c, slice(0, 64))
    for i in range(len(dims)):
        trainer.update_batch(agents, i, batches[i], c["u_tgt"][i], c["u_act"][i])
    want = np.concatenate([np.concatenate([a.actor[k].ravel() for k in NAMES] +
                                          [a.critic[k].ravel() for k in NAMES] +
                                          [a.tgt_actor[k].ravel() for k in NAMES] +
                                          [a.tgt_critic[k].ravel() for k in NAMES]) for a in agents])
    np.testing.assert_allclose(res[0], want, atol=2e-5)


def test_strict_round_single_rank_is_update_batch():
    dims, c = _case()
    a1 = [trainer.AgentParams(**copy.deepcopy(p)) for p in c["params"]]
    a2 = [trainer.AgentParams(**copy.deepcopy(p)) for p in c["params"]]
    batches = _batches(c, slice(0, 64))
    strict_round(OracleOps(a1, batches, c["u_tgt"], c["u_act"]), len(dims), 1, lambda t: None)
    for i in range(len(dims)):
        trainer.update_batch(a2, i, batches[i], c["u_tgt"][i], c["u_act"][i])
    for x, y in zip(a1, a2):
        for k in NAMES:
            np.testing.assert_array_equal(x.actor[k], y.actor[k])
            np.testing.assert_array_equal(x.tgt_critic[k], y.tgt_critic[k])


@pytest.mark.parametrize("world", [2, 4, 8])
def test_throughput_round_ranks_match_full_batch(world):
    """throughput mode: ONE all-reduce of every net's gradient per
    round; the replicas equal oracle.trainer.update_round_throughput on the
    whole batch"""
    res = _run_ranks(world, "throughput")
    dims, c = _case()
    agents = [trainer.AgentParams(**copy.deepcopy(p)) for p in c["params"]]
    n = len(dims)
    idx_n = [c["idx"][i][:64] for i in range(n)]
    trainer.update_round_throughput(agents, c["data"], idx_n, [c["u_tgt"][i] for i in range(n)],
                                    [c["u_act"][i] for i in range(n)])
    want = np.concatenate([np.concatenate([a.actor[k].ravel() for k in NAMES] +
                                          [a.critic[k].ravel() for k in NAMES] +
                                          [a.tgt_actor[k].ravel() for k in NAMES] +
                                          [a.tgt_critic[k].ravel() for k in NAMES]) for a in agents])
    np.testing.assert_allclose(res[0], want, atol=2e-5)


def test_throughput_round_single_rank_is_oracle_round():
    dims, c = _case()
    n = len(dims)
    a1 = [trainer.AgentParams(**copy.deepcopy(p)) for p in c["params"]]
    a2 = [trainer.AgentParams(**copy.deepcopy(p)) for p in c["params"]]
    throughput_round(OracleOps(a1, _batches(c, slice(0, 64)), c["u_tgt"], c["u_act"]), n, 1, lambda t: None)
    trainer.update_round_throughput(a2, c["data"], [c["idx"][i][:64] for i in range(n)],
                                    [c["u_tgt"][i] for i in range(n)], [c["u_act"][i] for i in range(n)])
    for x, y in zip(a1, a2):
        for k in NAMES:
            np.testing.assert_array_equal(x.actor[k], y.actor[k])
            np.testing.assert_array_equal(x.critic[k], y.critic[k])
            np.testing.assert_array_equal(x.tgt_critic[k], y.tgt_critic[k])


def _env_init_worker(rank, world, port, shared, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if shared:
        os.environ["MDP_SHARED_GPU"] = "1"
    from maddpg_amd.parallel import init_process_group_from_env
    w, r, local = init_process_group_from_env()
    t = torch.tensor([float(r + 1)])
    dist.all_reduce(t)
    q.put((r, w, local, dist.get_backend(), float(t.item())))
    dist.destroy_process_group()


@pytest.mark.parametrize("shared", [False, True])
def test_init_process_group_from_env(shared):
    """torchrun-style init as bench.py uses it; MDP_SHARED_GPU=1 (the 1-GPU
    rehearsal of the multi-rank command) puts every rank on device 0 with gloo."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_env_init_worker, args=(r, 2, port, shared, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [g[0] for g in got] == [0, 1] and all(g[1] == 2 for g in got)
    assert all(g[3] == "gloo" and g[4] == 3.0 for g in got)
    assert [g[2] for g in got] == ([0, 0] if shared else [0, 1])
