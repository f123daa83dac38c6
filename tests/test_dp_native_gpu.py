"""Native data parallelism (mdp_dp_init: the library's own RCCL communicator).

On a 1-GPU box the communicator has one rank, so the data-parallel update
(critic grads -> reduce -> ncclAllReduce -> clip+Adam x 1/G, then the actor)
must reproduce the two-kernel single-GPU path (k_reduce + k_apply) bit for
bit -- eagerly and with the collectives captured in the step graph.  The
2-rank test needs 2 visible GPUs (skipped otherwise).
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

pytestmark = pytest.mark.gpu

NETS = ("actor", "critic", "tgt_actor", "tgt_critic", "m_actor", "v_critic")


def _runner(dp):
    from maddpg_amd.runner import VecRunner
    r = VecRunner("simple_spread", 64, batch_size=128, capacity=20000, seed=3, train_every=16)
    if dp:
        r.eng.dp_init(1, 0)
        r.native_dp = True
    r.prefill()
    return r


@pytest.mark.parametrize("graphs", ["0", "1"])
def test_native_dp_single_rank_matches_two_kernel_path(monkeypatch, graphs):
    monkeypatch.setenv("MDP_UNFUSED_APPLY", "1")
    monkeypatch.setenv("MDP_DP_GRAPHS", graphs)
    a, b = _runner(True), _runner(False)
    for _ in range(3):
        assert a.step() == b.step() == 4
    a.eng.synchronize()
    b.eng.synchronize()
    for i in range(3):
        for w in NETS:
            pa, pb = a.eng.get_params(i, w), b.eng.get_params(i, w)
            for k in pa:
                np.testing.assert_array_equal(pa[k], pb[k], err_msg=f"{i} {w} {k}")
        for net in (0, 1):
            np.testing.assert_array_equal(a.eng.get_beta_powers(i, net), b.eng.get_beta_powers(i, net))


@pytest.mark.parametrize("graphs", ["0", "1"])
def test_native_dp_throughput_mode_single_rank_matches_single_gpu(monkeypatch, graphs):
    """Throughput mode with the native communicator: gradients, reduce pass, ONE
    all-reduce of the whole gradient region, step pass (x 1/1) == the single-GPU
    throughput round (fused reduce + step) bit for bit."""
    monkeypatch.setenv("MDP_DP_GRAPHS", graphs)
    a, b = _runner(True), _runner(False)
    a.eng.set_update_mode("throughput")
    b.eng.set_update_mode("throughput")
    for _ in range(3):
        assert a.step() == b.step() == 4
    a.eng.synchronize()
    b.eng.synchronize()
    for i in range(3):
        for w in NETS:
            pa, pb = a.eng.get_params(i, w), b.eng.get_params(i, w)
            for k in pa:
                np.testing.assert_array_equal(pa[k], pb[k], err_msg=f"{i} {w} {k}")
        for net in (0, 1):
            np.testing.assert_array_equal(a.eng.get_beta_powers(i, net), b.eng.get_beta_powers(i, net))
        np.testing.assert_array_equal(a.eng.stats(i), b.eng.stats(i))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, q, mode="strict"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist
    from maddpg_amd.runner import VecRunner
    torch.cuda.set_device(rank)
    dist.init_process_group("nccl")
    r = VecRunner("simple_spread", 64, batch_size=128, capacity=20000, seed=3, train_every=16,
                  world_size=world, rank=rank)
    assert r.native_dp
    if mode != "strict":
        r.eng.set_update_mode(mode)
    r.prefill()
    for _ in range(3):
        r.step()
    r.eng.synchronize()
    flat = np.concatenate([v.ravel() for i in range(3) for w in NETS for v in r.eng.get_params(i, w).values()])
    q.put((rank, flat))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs 2 GPUs")
@pytest.mark.parametrize("mode", ["strict", "throughput"])
def test_native_dp_two_ranks_replicas_identical(mode):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank_main, args=(r, 2, port, q, mode)) for r in range(2)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    np.testing.assert_array_equal(got[0], got[1])
    assert np.all(np.isfinite(got[0]))
