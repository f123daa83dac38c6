"""Diagnostic: sha256 of every parameter region after three update rounds on
fixed data (S2 at B=1024, tag N=6 at H=128, B=1000, and H=256), to check that a
scheduling change is bit-identical against another build:
    python tools/param_hash.py; MDP_LIB=maddpg_amd/libmaddpg_hip_ref.so python tools/param_hash.py"""
import hashlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from maddpg_amd.engine import Engine  # noqa: E402

for dims, H, B in (([18, 18, 18], 64, 1024), ([22, 22, 22, 22, 20, 20], 128, 1000), ([16, 16], 256, 512)):
    g = torch.Generator().manual_seed(5)
    eng = Engine(dims, num_units=H, batch_size=B, capacity=30000)
    eng.add_rows(torch.rand(eng.capacity, eng.row_stride, generator=g))
    eng.init_params(3)
    eng.seed_py_random(11)
    for _ in range(3):
        eng.update_round()
    eng.synchronize()
    h = hashlib.sha256()
    for reg in ("theta", "target", "adam_m", "adam_v"):
        h.update(eng.region(reg).cpu().numpy().tobytes())
    print(f"dims={dims} H={H} B={B}: {h.hexdigest()[:16]}")

# the device rollout: replay rows and env state after a few vector env steps
for dims, H, scn, na in (([18, 18, 18], 64, "simple_spread", 0), ([22, 22, 22, 22, 20, 20], 128, "simple_tag", 4),
                         ([18, 18, 18], 256, "simple_spread", 0)):
    eng = Engine(dims, num_units=H, batch_size=256, capacity=8192, num_envs=1000, scenario=scn, num_adversaries=na)
    eng.init_params(3)
    eng.env_reset()
    for _ in range(6):
        eng.env_step()
    eng.synchronize()
    h = hashlib.sha256()
    h.update(eng.region("replay").cpu().numpy().tobytes())
    print(f"rollout {scn} H={H}: {h.hexdigest()[:16]}")
