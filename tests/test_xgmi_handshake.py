"""Host logic of the direct xGMI exchange set-up (parallel.xgmi_handshake) on
CPU: world_size 2 over gloo with stand-in ops.  Every rank must end in the
same state -- all enabled, or all closed (so they fall back to RCCL
together) -- whichever rank fails at whichever stage."""
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from maddpg_amd.parallel import xgmi_handshake


class FakeOps:
    def __init__(self, rank, fail_at):
        self.rank, self.fail_at, self.log = rank, fail_at, []

    def _step(self, name):
        self.log.append(name)
        if self.fail_at == name:
            raise RuntimeError(f"{name} failed on rank {self.rank}")

    def open(self, world, rank):
        self._step("open")
        return bytes([rank]) * 64

    def connect(self, handles):
        self._step("connect")
        self.handles = handles

    def probe(self):
        self._step("probe")

    def enable(self):
        self.log.append("enable")

    def close(self):
        self.log.append("close")


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, fail_rank, fail_at, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ops = FakeOps(rank, fail_at if rank == fail_rank else None)
    ok, err = xgmi_handshake(ops, world, rank)
    q.put((rank, ok, err is not None, ops.log, getattr(ops, "handles", None)))
    dist.barrier()
    dist.destroy_process_group()


def _run(fail_rank, fail_at, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, fail_rank, fail_at, q)) for r in range(world)]
    for p in ps:
        p.start()
    got = dict((item[0], item[1:]) for item in (q.get(timeout=120) for _ in ps))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    return got


@pytest.mark.parametrize("world", [2, 8])
def test_all_ranks_enable_with_handles_in_rank_order(world):
    got = _run(None, None, world)
    for r in range(world):
        ok, has_err, log, handles = got[r]
        assert ok and not has_err
        assert log == ["open", "connect", "probe", "enable"]
        assert handles == [bytes([q]) * 64 for q in range(world)]


@pytest.mark.parametrize("fail_rank,fail_at,world", [(1, "open", 2), (0, "connect", 2), (1, "probe", 2),
                                                     (5, "open", 8), (7, "probe", 8)])
def test_any_failure_closes_every_rank(fail_rank, fail_at, world):
    got = _run(fail_rank, fail_at, world)
    for r in range(world):
        ok, has_err, log, _ = got[r]
        assert not ok
        assert log[-1] == "close" and "enable" not in log
        assert has_err == (r == fail_rank)
        if fail_at == "open":   # nobody connects when a handle is missing
            assert "connect" not in log
        if fail_at == "probe":  # every rank ran the probe (its peers wait on it)
            assert "probe" in log


# --------------------------------------------- probe timeout -> RCCL fallback
PROBE_WAIT_S = 3.0   # stands in for the device probe's bounded wait (30 s on the GPU)


class FakeEngine:
    """The Engine surface runner.select_exchange drives, on CPU: the xGMI
    handshake calls of Engine.dp_xgmi_init_from_dist (its real code runs) and
    an RCCL join that broadcasts the id over torch.distributed like
    Engine.dp_init_from_dist.  On `stall_rank` the probe never sees its peer's
    words: it returns only when its bounded wait expires, with an error."""
    device = "cpu"

    def __init__(self, rank, stall_rank):
        self.rank, self.stall_rank, self.log = rank, stall_rank, []

    def dp_xgmi_open(self, world, rank):
        self.log.append("open")
        return bytes([rank]) * 64

    def dp_xgmi_connect(self, handles):
        self.log.append("connect")

    def dp_xgmi_probe(self):
        self.log.append("probe")
        if self.rank == self.stall_rank:
            import time
            time.sleep(PROBE_WAIT_S)
            raise RuntimeError("mdp_dp_xgmi_probe: a peer's words did not arrive within the bounded wait")
        return 0

    def _c(self, name, *args):
        self.log.append({"mdp_dp_xgmi_enable": "enable", "mdp_dp_xgmi_close": "close"}.get(name, name))

    def dp_init_from_dist(self, world, rank):
        obj = [b"rccl-id" if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        self.log.append("rccl")
        return obj[0] is not None


def _select_worker(rank, world, port, stall_rank, q):
    import time

    from maddpg_amd.engine import Engine
    from maddpg_amd.runner import select_exchange
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    eng = FakeEngine(rank, stall_rank)
    eng.dp_xgmi_init_from_dist = lambda w, r: Engine.dp_xgmi_init_from_dist(eng, w, r)
    t0 = time.monotonic()
    got = select_exchange(eng, world, rank, environ={})
    q.put((rank, got, time.monotonic() - t0, eng.log))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("stall_rank,world", [(0, 2), (1, 2), (6, 8)])
def test_probe_timeout_falls_back_to_rccl_on_every_rank(stall_rank, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_select_worker, args=(r, world, port, stall_rank, q)) for r in range(world)]
    for p in ps:
        p.start()
    got = dict((item[0], item[1:]) for item in (q.get(timeout=120) for _ in ps))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        (native, kind), elapsed, log = got[r]
        assert (native, kind) == (True, "native-rccl")
        assert log == ["open", "connect", "probe", "close", "rccl"], log
        # every rank decides within the probe's bounded wait (plus set-up), not later
        assert elapsed < PROBE_WAIT_S + 20.0, elapsed
        if r != stall_rank:   # the healthy rank waited for the stalled one's verdict
            assert elapsed >= PROBE_WAIT_S * 0.9, elapsed
