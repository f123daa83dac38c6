"""Diagnostic: phase timings of k_rollout workgroup 0 (S2, E=1024) from the
-DMDP_STAMPS build:
    make -C maddpg_amd/csrc stamps
    MDP_LIB=maddpg_amd/libmaddpg_hip_stamps.so python tools/rollout_stamps.py [tag6]
(tag6: simple_tag N=6, H=128, E=4096 -- the S5 rollout)"""
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
for _ in range(8):
    eng.env_step()
eng.synchronize()
lib = _lib.load()
fn = lib.mdp_debug_stamps_k
fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
buf = (ctypes.c_ulonglong * 64)()
fn(buf, 64)
st = np.array(buf[:], dtype=np.int64)
names = [(41, "state load + obs"), (42, "agent 0 forward + sample"), (43, "agent 1"), (44, "agent 2"), (45, "agent 3"),
         (46, "physics, reward, obs', episode"), (47, "replay append + state store")]
prev = st[40]
for i, nm in names:
    if st[i] == 0:
        continue
    print(f"{nm:>32s}: {(st[i] - prev) * 10 / 1000:6.2f} us  (t={(st[i] - st[40]) * 10 / 1000:6.2f})")
    prev = st[i]
