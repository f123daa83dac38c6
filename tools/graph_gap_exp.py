"""Where does the step-boundary gap come from?  S2 training steps (bench.py's
main line: simple_spread N=3, 1024 envs, batch 1024, 64 units) timed with the
per-step graph replay and with eager launches, plus the host's own issue time
(the loop without the final synchronize), to tell a GPU-side graph-boundary
cost from a host that falls behind.

    python tools/graph_gap_exp.py [graphs|eager|both] [steps]
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from maddpg_amd.runner import VecRunner


def run(graphs, steps=30, warmup=5):
    r = VecRunner("simple_spread", 1024, n_agents=3, batch_size=1024, num_units=64, seed=0, train_every=100)
    r.eng.set_graphs(graphs)
    r.prefill()
    for _ in range(warmup):
        r.step()
    r.synchronize()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rounds = 0
    for _ in range(steps):
        rounds += r.step()
    t_issue = time.perf_counter() - t0
    r.synchronize()
    dt = time.perf_counter() - t0
    r.close() if hasattr(r, "close") else None
    return {"graphs": graphs, "env_steps_per_sec": round(1024 * steps / dt), "ms_per_step": round(dt / steps * 1e3, 4),
            "host_issue_ms_per_step": round(t_issue / steps * 1e3, 4), "rounds": rounds}


if __name__ == "__main__":
    mode = sys.argv[1] if len(sys.argv) > 1 else "both"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    modes = {"graphs": [True], "eager": [False], "both": [True, False, True, False]}[mode]
    for g in modes:
        print(json.dumps(run(g, steps)), flush=True)
