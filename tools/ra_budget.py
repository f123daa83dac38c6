"""Latency budget of the fused optimizer launch (k_reduce_apply) at S2, per phase.

    make -C maddpg_amd/csrc stamps
    MDP_LIB=maddpg_amd/libmaddpg_hip_stamps.so python tools/ra_budget.py [--json out.json]

The stamps build records, for every workgroup of the last critic-step and the
last actor-step optimizer launch of a graph-replayed round, s_memrealtime
(100 MHz, 10 ns) at (mdp_apply_fused.hip, MDP_RA_PH):
  0 start | 1 partial slabs loaded + group sums in LDS | 2 wave 0: tree sum +
  sum of squares | 3 norm published + reduced gradient stored | 4 norm
  handshake done (every chunk of the tensor seen) | 5 Adam (+ Polyak) stores
  issued (chunk workgroups end) ; stats workgroup: 5 stats written | 6 every
  chunk workgroup arrived | 7 beta powers / epochs advanced (its end).
Durations per launch from HIP events on the launch's own dispatch packet (the
interval rocprof reports) in an eager pass of the same rounds are printed
beside the in-kernel span: the difference is the dispatch + completion
overhead outside any workgroup.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from maddpg_amd import _lib  # noqa: E402
from maddpg_amd.engine import Engine  # noqa: E402

US = 0.01  # one s_memrealtime tick in us


def launch_budget(ph, rblk_end):
    """ph [1024][8] stamps of one launch; chunk workgroups [0, rblk_end), then
    Polyak workgroups (actor step), the stats workgroup last"""
    used = np.nonzero(ph[:, 0])[0]
    n = int(used.max()) + 1
    ph = ph[:n].astype(np.int64)
    t0 = ph[:, 0].min()
    rel = (ph - t0) * US
    ch = np.arange(min(rblk_end, n))
    st = n - 1                          # the stats workgroup (grid = chunks [+ Polyak] + stats)
    ends = np.where(np.arange(n) == st, rel[:, 7], rel[:, 5])
    last = int(np.argmax(ends))
    d = lambda a, b, rows=ch: rel[rows, b] - rel[rows, a]  # noqa: E731
    q = lambda x: {"median": round(float(np.median(x)), 3), "max": round(float(np.max(x)), 3)}  # noqa: E731
    return {
        "workgroups": n, "chunk_workgroups": int(len(ch)),
        "dispatch_ramp_us": round(float(rel[:, 0].max()), 3),
        "phases_us": {
            "partial_slab_loads_and_group_sums": q(d(0, 1)),
            "tree_sum_and_sum_of_squares": q(d(1, 2)),
            "norm_publish_and_grad_store": q(d(2, 3)),
            "norm_handshake_wait": q(d(3, 4)),
            "adam_polyak_stores": q(d(4, 5)),
        },
        "stats_workgroup_us": {"start": round(float(rel[st, 0]), 3), "stats_done": round(float(rel[st, 5]), 3),
                               "all_chunks_arrived": round(float(rel[st, 6]), 3),
                               "beta_tail_end": round(float(rel[st, 7]), 3)},
        "in_kernel_span_us": round(float(ends.max()), 3),
        "last_workgroup": {"wg": last, "is_stats": last == st,
                           "stamps_us": [round(float(x), 3) if ph[last, k] else None for k, x in enumerate(rel[last])]},
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json")
    ap.add_argument("--rounds", type=int, default=6)
    args = ap.parse_args()
    assert "stamps" in _lib.LIB_PATH, "run with MDP_LIB=maddpg_amd/libmaddpg_hip_stamps.so"
    eng = Engine([18, 18, 18], batch_size=1024, capacity=30000)
    eng.add_rows(torch.rand(eng.capacity, eng.row_stride))
    eng.init_params(0)
    eng.seed_py_random(0)
    lib = _lib.load()
    lib.mdp_debug_ra_phases.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
    for _ in range(args.rounds):     # the first round eager, then graph replays
        eng.update_round()
    eng.synchronize()
    lib.mdp_debug_ra_phases_reset()
    eng.update_round()               # one graph-replayed round: its last critic / actor launch stamped
    eng.synchronize()
    buf = (ctypes.c_ulonglong * (2 * 1024 * 8))()
    lib.mdp_debug_ra_phases(buf)
    ph = np.array(buf[:], dtype=np.uint64).reshape(2, 1024, 8)
    # chunk workgroups = 256-parameter chunks of the net's 6 tensors (mdp_ra_grid)
    def chunks(agent, which):
        return sum((int(np.prod(v.shape)) + 255) // 256 for v in eng.get_params(agent, which).values())
    out = {"config": "S2 simple_spread N=3, B=1024, H=64 (agent 2's launches of a graph-replayed round)",
           "critic_step": launch_budget(ph[0], chunks(2, "critic")),
           "actor_step": launch_budget(ph[1], chunks(2, "actor"))}
    # the same launches' durations on their dispatch packets (eager pass)
    eng.prof_enable("reduce_apply", True)   # (profiling runs the rounds eagerly)
    for _ in range(args.rounds):
        eng.update_round()
    eng.synchronize()
    ms, n = eng.prof_read("reduce_apply")
    eng.prof_enable("reduce_apply", False)
    out["packet_event_avg_us"] = round(ms / n * 1e3, 3) if n else None
    out["packet_event_launches"] = n
    print(json.dumps(out, indent=1))
    if args.json:
        json.dump(out, open(args.json, "w"), indent=1)


if __name__ == "__main__":
    main()
