"""Direct xGMI gradient exchange (mdp_dp_xgmi_*: the exchange inside the fused
optimizer kernel).

Runs two rank processes on ONE visible GPU (the IPC mapping, the LL protocol
and the rank-order sum are the same code as across GPUs; only the link
differs), with a gloo process group for the handle exchange:

* the connection probe passes;
* both ranks fed IDENTICAL data: the world sum is 2g and the step scales it by
  1/2 (both exact), so every parameter, Adam moment, beta power and stat must
  equal an undistributed single-GPU run bit for bit -- strict and throughput
  mode, eager and graph-replayed;
* ranks with their own env copies and index streams (the real sharding): the
  replicas stay bit-identical and finite;
* four ranks (three peers per exchange).
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
STEPS = 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _state(r):
    r.eng.synchronize()
    out = []
    for i in range(r.n):
        for w in NETS:
            out += [v.ravel() for v in r.eng.get_params(i, w).values()]
        for net in (0, 1):
            out.append(np.asarray(r.eng.get_beta_powers(i, net), np.float32).ravel())
    return np.concatenate(out)


def _stats(r):
    return np.concatenate([np.asarray(r.eng.stats(i), np.float64) for i in range(r.n)])


# "tag6": BASELINE configs[4]'s topology (simple_tag, 4 adversaries + 2 good,
# H=128) -> the general gradient kernels with the exchange in the same fused
# optimizer launch
CONFIGS = {"spread": dict(scenario="simple_spread"),
           "tag6": dict(scenario="simple_tag", n_agents=6, scenario_adversaries=4, num_units=128)}


def _make(identical, rank, cfg="spread", **kw):
    from maddpg_amd.runner import VecRunner
    # identical: both processes are "rank 0" of the data (same env copies, same
    # index stream); the exchange is still joined as ranks 0 and 1
    c = dict(CONFIGS[cfg])
    return VecRunner(c.pop("scenario"), 64, batch_size=128, capacity=20000, seed=3, train_every=16,
                     world_size=1, rank=0 if identical else rank, **c, **kw)


def _rank_main(rank, world, port, q, mode, identical, graphs, cfg):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import torch.distributed as dist
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        r = _make(identical, rank, cfg)
        r.eng.set_graphs(graphs)
        ok = r.eng.dp_xgmi_init_from_dist(world, rank)
        assert ok, "xGMI exchange could not be set up"
        r.native_dp = True
        if mode != "strict":
            r.eng.set_update_mode(mode)
        r.prefill()
        ks = [r.step() for _ in range(STEPS)]
        st, stats = _state(r), _stats(r)
        ref = ref_stats = None
        if identical and rank == 0:   # the undistributed run of the same data
            b = _make(True, 0, cfg)
            b.eng.set_graphs(graphs)
            if mode != "strict":
                b.eng.set_update_mode(mode)
            b.prefill()
            kb = [b.step() for _ in range(STEPS)]
            assert kb == ks
            ref, ref_stats = _state(b), _stats(b)
        q.put((rank, ks, st, stats, ref, ref_stats, None))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001 -- surfaced by the parent
        import traceback
        q.put((rank, None, None, None, None, None, traceback.format_exc()[-3000:]))
        raise


def _run(mode, identical, graphs=True, world=2, cfg="spread"):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank_main, args=(r, world, port, q, mode, identical, graphs, cfg)) for r in range(world)]
    for p in ps:
        p.start()
    got = {}
    for _ in ps:
        item = q.get(timeout=240)
        assert item[-1] is None, item[-1]
        got[item[0]] = item
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    return got


@pytest.mark.parametrize("mode,graphs", [("strict", True), ("strict", False), ("throughput", True)])
def test_xgmi_identical_ranks_equal_single_gpu(mode, graphs):
    got = _run(mode, True, graphs)
    _, ks, st0, stats0, ref, ref_stats, _ = got[0]
    assert sum(ks) > 0
    np.testing.assert_array_equal(got[1][2], st0)
    np.testing.assert_array_equal(st0, ref)
    np.testing.assert_array_equal(stats0, ref_stats)


@pytest.mark.parametrize("mode", ["strict", "throughput"])
def test_xgmi_sharded_replicas_identical(mode):
    got = _run(mode, False)
    np.testing.assert_array_equal(got[0][2], got[1][2])
    assert np.all(np.isfinite(got[0][2]))
    # the shards really differ: each rank's own batch statistics
    assert not np.array_equal(got[0][3], got[1][3])


def test_xgmi_four_ranks():
    """world 4 (rank-order sum over 3 peers), identical data: the four replicas
    are bit-identical, and match the single-GPU run up to the rounding of the
    partial sum 3g (((g + g) + g) + g) / 4 need not be exactly g)."""
    got = _run("strict", True, True, world=4)
    for r in range(1, 4):
        np.testing.assert_array_equal(got[r][2], got[0][2])
    np.testing.assert_allclose(got[0][2], got[0][4], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("mode,identical", [("strict", True), ("strict", False), ("throughput", True)])
def test_xgmi_tag6_h128_general_kernels(mode, identical):
    """configs[4]'s topology (tag N=6, H=128: general gradient kernels; strict:
    12 optimizer launches per round each carrying its exchange, throughput: one
    batched launch): identical data reproduces the single-GPU run bit for bit;
    sharded data keeps the replicas bit-identical."""
    got = _run(mode, identical, True, cfg="tag6")
    np.testing.assert_array_equal(got[0][2], got[1][2])
    assert np.all(np.isfinite(got[0][2]))
    if identical:
        assert sum(got[0][1]) > 0
        np.testing.assert_array_equal(got[0][2], got[0][4])
        np.testing.assert_array_equal(got[0][3], got[0][5])
    else:
        assert not np.array_equal(got[0][3], got[1][3])
