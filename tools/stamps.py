"""Diagnostic: phase timings of k_critic_grad workgroup 0 from the -DMDP_STAMPS build.

    make -C maddpg_amd/csrc stamps
    MDP_LIB=maddpg_amd/libmaddpg_hip_stamps.so python tools/stamps.py
Stamps come from s_memrealtime (100 MHz); read the SHARES, not the total
(the stamp build serialises phases the real kernel may overlap)."""
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
eng.add_rows(torch.rand(30000, eng.row_stride))
eng.init_params(0)
eng.seed_py_random(0)
lib = _lib.load()
lib.mdp_debug_stamps.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
names = {0: "start", 1: "gather+copies", 2: "tgt actors+critic fwd", 3: "tgt critic", 4: "TD,stats,dW3,d2",
         5: "dh1,dW2,dW1"}
for it in range(5):
    eng.update_round()
    eng.synchronize()
buf = (ctypes.c_ulonglong * 64)()
lib.mdp_debug_stamps(buf, 64)
st = np.array(buf[:6], dtype=np.int64)
prev = st[0]
for i in range(1, 6):
    if st[i] == 0:
        continue
    print(f"{names.get(i, i):>14s}: {(st[i] - prev) * 10 / 1000:7.2f} us")
    prev = st[i]
print(f"{'total':>14s}: {(st[5] - st[0]) * 10 / 1000:7.2f} us")
