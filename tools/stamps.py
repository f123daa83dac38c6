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
# MDP_STAMP_CFG=tag6: BASELINE configs[4] (simple_tag 4+2 agents, H=128, B=4096; general kernels)
if os.environ.get("MDP_STAMP_CFG") == "tag6":
    eng = Engine([22, 22, 22, 22, 20, 20], num_units=128, batch_size=4096, capacity=120000)
else:
    eng = Engine([18, 18, 18], batch_size=1024, capacity=30000)
eng.add_rows(torch.rand(eng.capacity, eng.row_stride))
eng.init_params(0)
eng.seed_py_random(0)
lib = _lib.load()
fast = eng.lib.mdp_grad_variant(eng.h, 0) == 1
fn = lib.mdp_debug_stamps_r if fast else lib.mdp_debug_stamps
fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
for it in range(5):
    eng.update_round()
    eng.synchronize()
buf = (ctypes.c_ulonglong * 64)()
fn(buf, 64)
st = np.array(buf[:], dtype=np.int64)
if not fast:
    names = {0: "start", 1: "gather+copies", 6: "L1 phase (group 0)", 7: "L2 phase", 8: "heads",
             2: "Gumbel (+ later groups)", 3: "tgt critic", 4: "TD,stats,dW3,d2", 5: "dh1,dW2,dW1"}
    prev = st[0]
    for i in (1, 6, 7, 8, 2, 3, 4, 5):
        print(f"{names[i]:>32s}: {(st[i] - prev) * 10 / 1000:7.2f} us  (t={(st[i] - st[0]) * 10 / 1000:6.2f})")
        prev = st[i]
    print("per-wave layer-phase ends (us after the gather; L1 waves 0..15 | L2 waves 0..15):")
    print("  L1:", " ".join(f"{(st[16 + w] - st[1]) * 10 / 1000:5.2f}" for w in range(16)))
    print("  L2:", " ".join(f"{(st[40 + w] - st[6]) * 10 / 1000:5.2f}" for w in range(16)))
    if st[32]:
        anames = [(33, "gather"), (34, "actor L1"), (35, "actor L2"), (36, "head + Gumbel"), (37, "critic L1"),
                  (38, "critic L2"), (39, "q, d2c"), (56, "dh1c"), (57, "da, softmax bwd"), (58, "dW3a, d2a"),
                  (59, "dh1a, dW2a"), (60, "dW1a")]
        print("general actor step (wave 0):")
        prev = st[32]
        for i, nm in anames:
            print(f"{nm:>32s}: {(st[i] - prev) * 10 / 1000:7.2f} us  (t={(st[i] - st[32]) * 10 / 1000:6.2f})")
            prev = st[i]
    seq = []
else:
    names = {0: "start", 1: "B1 gather+weights (w0)", 2: "tgt actor fwd+gumbel (w0)", 3: "critic L1+L2 (w3)",
             4: "B2 (w4)", 5: "tgt L1 a~ part | B3 (w4)", 6: "tgt L2 tile | B4 (w4)", 7: "head, TD, d2 (w4)",
             8: "B5 (w4)", 9: "dh1 tile, dW2 | B6 (w4)", 10: "dW1 end (w0)",
             16: "start", 17: "B1 gather+weights (w0)", 18: "actor fwd+gumbel (w0)", 19: "B2 (w1)",
             20: "critic fwd, d2c (w1)", 21: "B3 (w4)", 22: "dh1c tile | B4 (w4)", 23: "after B4 (w0)",
             24: "da, softmax bwd, d2a (w0)", 25: "B5 (w4)", 26: "dh1a tile, dW2a | B6 (w4)", 27: "dW1a end (w0)"}
    names.update({11: "role entry (w0)", 12: "kernarg chain (w0)", 13: "weights issued (w0)",
                  14: "weights landed (w0)", 15: "gather landed (w4, from t=0)"})
    seq = [(0, 11), (0, 1), (16, 28)]
    print("actor fwd detail (w0): L1 %.2f  L2 %.2f  head %.2f  gumbel %.2f us" % tuple(
        (st[b] - st[a]) * 10 / 1000 for a, b in ((1, 41), (41, 42), (42, 43), (43, 2))))
    wall = (st[2] - st[1]) * 10e-9
    print("in-kernel clock over the actor forward: %.3f GHz" % ((st[44] - st[40]) / wall / 1e9))
    prev = st[0]
    for i in (11, 12, 13, 14, 15, 1):
        print(f"{names[i]:>32s}: {(st[i] - prev) * 10 / 1000:7.2f} us")
        prev = st[i]
    print()
for lo, hi in seq:
    prev = st[lo]
    for i in range(lo + 1, hi):
        if st[i] == 0:
            continue
        print(f"{names.get(i, i):>32s}: {(st[i] - prev) * 10 / 1000:7.2f} us  (t={(st[i] - st[lo]) * 10 / 1000:6.2f})")
        prev = st[i]
    print()
if fast and st[48]:
    # critic_post (the last critic launch of the round: agent n-1, split around agent n-2)
    print("critic_post from start: w0 loads issued %.2f, rows %.2f, L1 tile %.2f, L2 tiles all %.2f, head+gumbel %.2f, "
          "B2 %.2f | w3 cpre loaded %.2f, w3 L2 tile %.2f us" % tuple(
              (st[i] - st[0]) * 10 / 1000 for i in (48, 49, 50, 51, 52, 53, 54, 55)))
if fast and st[60]:
    print("critic TD phase (w4): B4 -> dq %.2f, d2/dW3 loop %.2f, stats sums + stores %.2f us" % (
        (st[60] - st[6]) * 10 / 1000, (st[61] - st[60]) * 10 / 1000, (st[7] - st[61]) * 10 / 1000))
if fast and st[56]:
    print("actor step from start: w1 rows ready %.2f, w1 L1 third done %.2f, w3 L1 third done %.2f us" % tuple(
        (st[i] - st[16]) * 10 / 1000 for i in (56, 57, 58)))
lib_ra = getattr(lib, "mdp_debug_stamps_ra", None)
if lib_ra is not None:
    lib_ra.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    rb = (ctypes.c_ulonglong * 64)()
    lib_ra(rb, 64)
    ra = np.array(rb[:], dtype=np.int64)
    if ra[30]:
        print("k_reduce_apply wg 0 (last launch): partial loads + combine %.2f us, norm handshake %.2f us, "
              "clip/Adam/stores %.2f us" % ((ra[31] - ra[30]) * 10 / 1000, (ra[32] - ra[31]) * 10 / 1000,
                                            (ra[33] - ra[32]) * 10 / 1000))
    if ra[34]:
        us = lambda a_, b_: (ra[b_] - ra[a_]) * 10 / 1000
        print("  detail: barrier -> 16-group combine %.2f, sum of squares %.2f, grad stores %.2f, publish %.2f, "
              "poll %.2f, Adam + stores %.2f us" % (us(31, 34), us(34, 35), us(35, 36), us(36, 32), us(32, 37),
                                                    us(37, 33)))
