"""Diagnostic: phase timings of the pair critic kernel (k_critic_pair), pair 0,
from the -DMDP_STAMPS build.

    make -C maddpg_amd/csrc stamps
    MDP_LIB=maddpg_amd/libmaddpg_hip_stamps.so python tools/pair_stamps.py
BASELINE configs[4] shapes (simple_tag 4+2 agents, H=128, B=4096).  Stamps
are s_memrealtime (100 MHz) of thread 0; both workgroups share one clock."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from maddpg_amd import _lib  # noqa: E402
from maddpg_amd.engine import Engine  # noqa: E402

assert "stamps" in _lib.LIB_PATH
B = int(os.environ.get("MDP_STAMP_B", "4096"))
eng = Engine([22, 22, 22, 22, 20, 20], num_units=128, batch_size=B, capacity=120000)
eng.add_rows(torch.rand(eng.capacity, eng.row_stride))
eng.init_params(0)
eng.seed_py_random(0)
lib = _lib.load()
fn = lib.mdp_debug_stamps_pair
fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
for it in range(5):
    eng.update_round()
    eng.synchronize()
buf = (ctypes.c_ulonglong * 64)()
fn(buf, 64)
st = np.array(buf[:], dtype=np.int64)
t0 = min(st[0], st[32])


def us(x):
    return (x - t0) * 10 / 1000


print("A (target actors), t in us from the first workgroup start:")
for i, nm in [(0, "start"), (1, "gather obs'"), (2, "group0 L1"), (3, "group0 L2"), (4, "group0 heads"),
              (5, "group0 Gumbel+stores"), (6, "group1 L1"), (7, "group1 L2"), (8, "group1 heads"),
              (9, "group1 Gumbel+stores"), (15, "published")]:
    if st[i]:
        print(f"  {nm:>24s}: t={us(st[i]):6.2f}")
print("B (critic), t in us:")
for i, nm in [(0, "start"), (1, "gather rows"), (2, "critic L1 + tc obs'"), (3, "critic L2"), (4, "q head + wait"),
              (5, "a~ loads"), (6, "tc L1 a~ part"), (7, "tc L2"), (8, "tc head"), (9, "TD"), (10, "dW3, d2"),
              (11, "dh1 + dW2"), (12, "dW1 (end)")]:
    if st[32 + i]:
        print(f"  {nm:>24s}: t={us(st[32 + i]):6.2f}")
