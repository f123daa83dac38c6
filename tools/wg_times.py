"""Diagnostic: which workgroup role ends each fast gradient launch (S2).

    make -C maddpg_amd/csrc stamps
    MDP_LIB=maddpg_amd/libmaddpg_hip_stamps.so python tools/wg_times.py
Per role of the last k_critic_grad_r / k_actor_grad_r launch of a round:
the earliest start, the latest start and the latest end, in us after the
launch's first workgroup started (s_memrealtime, 100 MHz), and each wave's
end after its own workgroup's start."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from maddpg_amd import _lib  # noqa: E402
from maddpg_amd.engine import Engine  # noqa: E402

assert "stamps" in _lib.LIB_PATH
eng = Engine([18, 18, 18], batch_size=1024, capacity=30000)
eng.add_rows(torch.rand(eng.capacity, eng.row_stride))
eng.init_params(0)
eng.seed_py_random(0)
lib = _lib.load()
fn = lib.mdp_debug_wg_times
fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.POINTER(ctypes.c_ulonglong)]
for it in range(5):
    eng.update_round()
    eng.synchronize()
t0 = (ctypes.c_ulonglong * (2 * 512))()
t1 = (ctypes.c_ulonglong * (2 * 512 * 8))()
assert fn(t0, t1) == 0
t0 = np.array(t0[:], dtype=np.int64).reshape(2, 512)
t1 = np.array(t1[:], dtype=np.int64).reshape(2, 512, 8)
nwg = 64
for k, name, roles in ((0, "critic launch", [("critic step", 0, nwg), ("actor_pre", nwg, 2 * nwg), ("draw", 2 * nwg, 2 * nwg + 1)]),
                       (1, "actor launch", [("actor step", 0, nwg), ("critic_pre", nwg, 2 * nwg)])):
    used = t0[k] > 0
    base = t0[k][used].min()
    print(name)
    for rn, lo, hi in roles:
        s = t0[k][lo:hi]
        if not (s > 0).any():
            continue
        e = t1[k][lo:hi].max(axis=1)
        print(f"  {rn:>12s}: start {(s.min() - base) / 100:5.2f}..{(s.max() - base) / 100:5.2f} us, "
              f"end median {(np.median(e) - base) / 100:5.2f}, max {(e.max() - base) / 100:5.2f} us")
        # per wave: end after its own workgroup's start (median over the role's workgroups)
        ok = s > 0
        w = t1[k][lo:hi][ok]
        rel = np.where(w > 0, w - s[ok][:, None], -1)
        print(" " * 16 + "per-wave end after own start (us): " +
              " ".join(f"w{q}:{np.median(rel[:, q]) / 100:.2f}" if (rel[:, q] >= 0).any() else f"w{q}:-"
                       for q in range(8)))

# critic_pre's per-wave phase points (us after the workgroup's first point,
# median over its row tiles): 1 rows ready, 2 at B2, 3 after B2, 4 stores issued (waves 4..7), 5 end
f2 = lib.mdp_debug_cpre_times
f2.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
ct = (ctypes.c_ulonglong * (64 * 8 * 6))()
assert f2(ct) == 0
ct = np.array(ct[:], dtype=np.int64).reshape(64, 8, 6)
base = ct[:, :, 0].min(axis=1)
print("critic_pre phase points (us after the tile's start; waves 0..2 target actors, 3 critic, 4..7 gather + target-critic tiles)")
for q in range(8):
    row = []
    for i in range(1, 6):
        v = ct[:, q, i]
        ok = v > 0
        row.append(f"{np.median(v[ok] - base[ok]) / 100:5.2f}" if ok.any() else "    -")
    print(f"  w{q}: rows {row[0]}  B2 {row[1]} -> {row[2]}  stores {row[3]}  end {row[4]}")

# the critic step after B5 (weight-gradient tiles, column sums), per wave: us
# after the workgroup's earliest B5 exit, median over its row tiles
f3 = lib.mdp_debug_crit_times
f3.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
ct = (ctypes.c_ulonglong * (64 * 8 * 6))()
assert f3(ct) == 0
ct = np.array(ct[:], dtype=np.int64).reshape(64, 8, 6)
base = ct[:, :, 0].min(axis=1)
print("critic step after B5 (us after the tile's first B5 exit)")
for q in range(8):
    row = [f"{np.median(ct[:, q, i] - base) / 100:5.2f}" for i in range(5)]
    print(f"  w{q}: B5 exit {row[0]}  dW2 {row[1]}  dW1 obs {row[2]}  dW1 act {row[3]}  colsums {row[4]}")
