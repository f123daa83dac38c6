"""Diagnostic: what the boundary between two graph-replayed training steps
costs on the GPU clock (S2).  rocprof shows the rollout of every step starting
~8 us after the previous step's last optimizer launch ended, while every
boundary inside a step shows ~2 us; eager launches show the same gap, and the
host issues a step in ~0.05 ms of the ~0.93 ms it runs (tools/graph_gap_exp.py),
so the host is not behind.

    make -C maddpg_amd/csrc timeline
    MDP_LIB=maddpg_amd/libmaddpg_hip_tl.so [MDP_SB_EAGER=1] [MDP_TL_CFG=tag6] python tools/step_boundary.py

Per boundary: last optimizer end -> rollout first workgroup start, the
rollout's body (first start -> last end), and rollout end -> first critic
launch start, from s_memrealtime (100 MHz, one clock for the GPU)."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from maddpg_amd import _lib  # noqa: E402
from maddpg_amd.runner import VecRunner  # noqa: E402

assert "_tl" in _lib.LIB_PATH, "run with MDP_LIB=maddpg_amd/libmaddpg_hip_tl.so"
NS, NW = 1024, 512
lib = _lib.load()
fns = {}
for name in ("mdp_debug_tl_r", "mdp_debug_tl_ra", "mdp_debug_tl_roll"):
    f = getattr(lib, name)
    f.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    fns[name] = f


def read(name, shape):
    buf = np.zeros(int(np.prod(shape)), dtype=np.uint64)
    assert fns[name](buf.ctypes.data_as(ctypes.POINTER(ctypes.c_ulonglong)), 0) == 0
    return buf.reshape(shape)


if os.environ.get("MDP_TL_CFG") == "tag6":  # S5: only the rollout's own workgroups
    r = VecRunner("simple_tag", 4096, n_agents=6, scenario_adversaries=4, batch_size=4096, num_units=128, seed=0)
else:
    r = VecRunner("simple_spread", 1024, batch_size=1024, seed=0)
if os.environ.get("MDP_SB_EAGER") == "1":  # eager launches instead of the step graph
    r.eng.set_graphs(False)
r.prefill()
for _ in range(3):
    r.step()
r.synchronize()
pre, roll, post, rbody, wg0, envmax, envmed, envst = [], [], [], [], [], [], [], []
for rep in range(12 if os.environ.get("MDP_TL_CFG") != "tag6" else 4):
    for f in fns.values():
        assert f(None, 1) == 0
    k1 = r.step()
    k2 = r.step()
    r.synchronize()
    if k1 == 0 or k2 == 0:
        continue
    ro = read("mdp_debug_tl_roll", (NW, 2))
    ok = ro[:, 1] > 0
    rs, re_ = int(ro[ok, 0].min()), int(ro[ok, 1].max())
    ends, starts = [], []
    for name in ("mdp_debug_tl_r", "mdp_debug_tl_ra"):
        a = read(name, (NS, NW, 2))
        e = a[:, :, 1]
        s = a[:, :, 0]
        ends.append(e[e > 0])
        starts.append(s[s > 0])
    ends = np.concatenate(ends).astype(np.int64)
    starts = np.concatenate(starts).astype(np.int64)
    before = ends[ends < rs]
    after = starts[starts > re_]
    rbody.append((re_ - rs) / 100.0)
    # workgroup 0 draws the first round's indices; the others step the env copies
    wg0.append((int(ro[0, 1]) - rs) / 100.0)
    envmax.append((int(ro[1:][ok[1:], 1].max()) - rs) / 100.0)
    envmed.append((float(np.median(ro[1:][ok[1:], 1].astype(np.int64))) - rs) / 100.0)
    envst.append((int(ro[1:][ok[1:], 0].max()) - rs) / 100.0)
    if len(before) and len(after):  # instrumented launches on both sides (S2)
        pre.append((rs - before.max()) / 100.0)
        post.append((after.min() - re_) / 100.0)
for nm, v in (("last optimizer end -> rollout start", pre), ("rollout body", rbody),
              ("rollout end -> critic launch start", post), ("draw workgroup (0) end", wg0),
              ("env workgroups: last start", envst), ("env workgroups: median end", envmed),
              ("env workgroups: last end", envmax)):
    v = np.array(v)
    if len(v) == 0:
        continue
    print(f"{nm:>36s}: n={len(v):2d} median {np.median(v):6.2f} us (min {v.min():.2f}, max {v.max():.2f})")
