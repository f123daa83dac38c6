"""Rehearsal of the data-parallel exchange on a 1-GPU box: two rank processes
share cuda:0 (gloo process group for the handshake).  Times the same strict
workload as bench.py (simple_spread, E envs per rank, B=1024) three ways:

  solo   -- one process alone (no DP)
  pair   -- two independent processes at once (no exchange: GPU sharing cost)
  xgmi   -- two ranks with the direct exchange inside the optimizer kernel
  rccl1  -- one process, 1-rank RCCL communicator (launch/collective cost)

xgmi - pair isolates what the exchange adds per step on top of sharing the GPU.

    python tools/xgmi_pair_bench.py [--envs 1024] [--steps 30] [--ranks 2]
"""
import argparse
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _time(r, steps, warm):
    for _ in range(warm):
        r.step()
    r.eng.synchronize()
    t = time.perf_counter()
    k = 0
    for _ in range(steps):
        k += r.step()
    r.eng.synchronize()
    return time.perf_counter() - t, k


def _worker(rank, world, port, q, kind, a):
    import torch
    import torch.distributed as dist
    from maddpg_amd.runner import VecRunner
    torch.cuda.set_device(0)
    if world > 1:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
    r = VecRunner("simple_spread", a.envs, batch_size=1024, seed=0, world_size=1, rank=rank)
    if kind == "xgmi":
        assert r.eng.dp_xgmi_init_from_dist(world, rank)
        r.native_dp = True
    elif kind == "rccl1":
        r.eng.dp_init(1, 0)
        r.native_dp = True
    r.prefill()
    if world > 1:
        dist.barrier()
    dt, k = _time(r, a.steps, a.warmup)
    q.put((rank, dt, k))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--ranks", type=int, default=2, help="rank processes of the pair/xgmi runs (<= 8)")
    ap.add_argument("--only-shared", action="store_true", help="skip the solo and rccl1 runs")
    a = ap.parse_args()
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    res = {}
    runs = [("pair", a.ranks), ("xgmi", a.ranks)]
    if not a.only_shared:
        runs = [("solo", 1), ("rccl1", 1)] + runs
    for kind, world in runs:
        q = ctx.Queue()
        port = _port()
        # "pair": `ranks` world-1 processes at once (no process group)
        ps = [ctx.Process(target=_worker, args=(r, 1 if kind == "pair" else world, port, q, kind, a))
              for r in range(world)]
        for p in ps:
            p.start()
        got = [q.get(timeout=300) for _ in ps]
        for p in ps:
            p.join(timeout=60)
        dt = max(g[1] for g in got)
        k = got[0][2]
        res[kind] = {"env_steps_per_sec": round(a.envs * a.steps * world / dt, 1),
                     "ms_per_step": round(dt / a.steps * 1e3, 4), "rounds": k,
                     "us_per_round": round(dt / max(k, 1) * 1e6, 2)}
        print(kind, res[kind], flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
