"""Diagnostic: the index-draw workgroup of k_rollout (the step's first draw)
against env workgroup 0 of the same launch, on the s_memrealtime clock, from
the -DMDP_STAMPS build, S2 or (arg tag6) S5:
    make -C maddpg_amd/csrc stamps
    MDP_LIB=maddpg_amd/libmaddpg_hip_stamps.so python tools/draw_stamps.py [tag6]"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from maddpg_amd import _lib  # noqa: E402
from maddpg_amd.engine import Engine  # noqa: E402

assert "stamps" in _lib.LIB_PATH
if sys.argv[1:] == ["tag6"]:
    eng = Engine([22, 22, 22, 22, 20, 20], num_units=128, batch_size=4096, capacity=60000, num_envs=4096,
                 scenario="simple_tag", num_adversaries=4)
else:
    eng = Engine([18, 18, 18], batch_size=1024, capacity=60000, num_envs=1024, scenario="simple_spread")
eng.init_params(0)
eng.env_reset()
for _ in range(4):
    eng.env_step()
lib = _lib.load()
fn = lib.mdp_debug_stamps_k
fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
buf = (ctypes.c_ulonglong * 64)()
for _ in range(3):
    eng.train_step(1)
    eng.synchronize()
    fn(buf, 64)
    st = np.array(buf[:], dtype=np.int64)
    t0 = min(st[40], st[48])
    us = lambda i: (st[i] - t0) * 10 / 1000  # noqa: E731
    print(f"draw workgroup {us(48):6.2f} .. {us(49):6.2f} us ({us(49) - us(48):6.2f});"
          f"  env workgroup 0 {us(40):6.2f} .. {us(47):6.2f} us ({us(47) - us(40):6.2f})")
