"""Diagnostic: which workgroup ends a k_reduce_apply launch (the last one of a
round) at S5 (tag N=6, H=128, B=4096) or S2 (MDP_STAMP_CFG=s2):
    make -C maddpg_amd/csrc stamps
    MDP_LIB=maddpg_amd/libmaddpg_hip_stamps.so python tools/ra_wg_times.py
Workgroup starts / ends in us after the launch's first start (s_memrealtime,
100 MHz).  The last workgroup of the grid is the index-draw piece, the one
before it the stats workgroup, the chunk workgroups come first."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from maddpg_amd import _lib  # noqa: E402
from maddpg_amd.engine import Engine  # noqa: E402

assert "stamps" in _lib.LIB_PATH
if os.environ.get("MDP_STAMP_CFG") == "s2":
    eng = Engine([18, 18, 18], batch_size=1024, capacity=30000)
else:
    eng = Engine([22, 22, 22, 22, 20, 20], num_units=128, batch_size=4096, capacity=120000)
eng.add_rows(torch.rand(eng.capacity, eng.row_stride))
eng.init_params(0)
eng.seed_py_random(0)
lib = _lib.load()
fn = lib.mdp_debug_ra_wg
fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
for _ in range(4):
    eng.update_round()
    eng.synchronize()
t0 = (ctypes.c_ulonglong * 1024)()
t1 = (ctypes.c_ulonglong * 1024)()
fn(t0, t1, 1024)
a0 = np.array(t0[:], dtype=np.int64)
a1 = np.array(t1[:], dtype=np.int64)
# slots keep the LAST launch that had that many workgroups: the round's last
# launch is the set that started within 15 us of the latest start
last = a0.max()
sel = [i for i in range(1024) if a0[i] > 0 and a0[i] >= last - 1500]
n = max(sel) + 1
assert sel == list(range(n)), "slots of the last launch are not contiguous"
base = a0[:n].min()
s = (a0[:n] - base) * 10 / 1000
e = (a1[:n] - base) * 10 / 1000
print(f"grid {n}: starts {s.min():.2f}..{s.max():.2f} us, ends {e.min():.2f}..{e.max():.2f} us")
print(f"  draw piece (wg {n - 1}): start {s[n - 1]:.2f} end {e[n - 1]:.2f}; stats (wg {n - 2}): start {s[n - 2]:.2f} "
      f"end {e[n - 2]:.2f}")
ch = np.arange(n - 2)
print(f"  other wgs: end median {np.median(e[ch]):.2f}, p90 {np.percentile(e[ch], 90):.2f}, max {e[ch].max():.2f} "
      f"(wg {int(ch[np.argmax(e[ch])])}); duration median {np.median(e[ch] - s[ch]):.2f}")
order = np.argsort(-e)[:8]
print("  latest ends:", ", ".join(f"wg {i}: {s[i]:.2f}->{e[i]:.2f}" for i in order))
hist = np.histogram(e[ch], bins=8)
print("  end-time histogram of the other wgs:", list(zip(np.round(hist[1][:-1], 2).tolist(), hist[0].tolist())))
