"""Diagnostic: the S5 critic step's layer work queue, unit by unit (workgroup 0).

    make -C maddpg_amd/csrc stamps
    MDP_LIB=maddpg_amd/libmaddpg_hip_stamps.so python tools/queue_trace.py
Every 64-column unit of fwd_phase_l12 (layer 1 / layer 2 of the target actors,
the critic and the target critic's obs' part) with the wave that took it and
its take / done times (s_memrealtime, 100 MHz), from one critic launch of
BASELINE configs[4] (simple_tag 4+2 agents, H=128, B=4096)."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from maddpg_amd import _lib  # noqa: E402
from maddpg_amd.engine import Engine  # noqa: E402

assert "stamps" in _lib.LIB_PATH
eng = Engine([22, 22, 22, 22, 20, 20], num_units=128, batch_size=4096, capacity=120000)
eng.add_rows(torch.rand(eng.capacity, eng.row_stride))
eng.init_params(0)
eng.seed_py_random(0)
lib = _lib.load()
fn = lib.mdp_debug_q_trace
fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
for it in range(3):
    eng.update_round()
eng.synchronize()
runs = []
for rep in range(4):
    fn(None, 1)
    eng.update(rep % 6)
    eng.synchronize()
    buf = (ctypes.c_ulonglong * (160 * 5))()
    fn(buf, 0)
    t = np.array(buf[:], dtype=np.int64).reshape(160, 5)
    t = t[t[:, 3] > 0]
    runs.append(t)
n_act = 6
for rep, t in enumerate(runs):
    t0 = t[:, 3].min()
    end = (t[:, 4].max() - t0) * 10 / 1000
    print(f"launch {rep} (agent {rep % 6}): {len(t)} units, queue span {end:.2f} us")
    order = np.argsort(t[:, 3])
    for i in order:
        w, ln, g, a, b = t[i]
        layer, net = ln >> 8, ln & 255
        name = ("actor%d" % net) if net < n_act else ("critic" if net == n_act else "tgtQ-obs'")
        print(f"  wave {w:2d}  L{layer + 1} {name:9s} g{g}  take {(a - t0) * 0.01:6.2f}  done {(b - t0) * 0.01:6.2f}"
              f"  ({(b - a) * 0.01:5.2f} us)")
    # per-wave busy end
    ends = {}
    for w, ln, g, a, b in t:
        ends[w] = max(ends.get(w, 0), b)
    print("  per-wave last unit done:", " ".join(f"{(ends[w] - t0) * 0.01:5.2f}" for w in sorted(ends)))
