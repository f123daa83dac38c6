"""Diagnostic: the graph-replayed training step's launch bodies and the gaps
between them (S2 by default; MDP_TL_CFG=tag6 for S5).

    make -C maddpg_amd/csrc timeline
    MDP_LIB=maddpg_amd/libmaddpg_hip_tl.so python tools/timeline.py

Each instrumented launch records its first workgroup start and its last wave
end per role (s_memrealtime, 100 MHz, one clock for the whole GPU), keyed by
the update counter (one agent update = critic launch, its optimizer launch,
actor launch, its optimizer launch).  Printed: medians over the step's agent
updates of every launch's body (first start -> last end), of each role's end
relative to the launch's start, and of the gap from one launch's last end to
the next launch's first start -- what a kernel boundary costs in this graph."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from maddpg_amd import _lib  # noqa: E402
from maddpg_amd.runner import VecRunner  # noqa: E402

assert "_tl" in _lib.LIB_PATH, "run with MDP_LIB=maddpg_amd/libmaddpg_hip_tl.so"
if os.environ.get("MDP_TL_CFG") == "tag6":
    r = VecRunner("simple_tag", 4096, n_agents=6, scenario_adversaries=4, batch_size=4096, num_units=128, seed=0)
else:
    r = VecRunner("simple_spread", 1024, batch_size=1024, seed=0)
r.prefill()
for _ in range(3):
    r.step()
r.synchronize()
lib = _lib.load()
fns = []
for name in ("mdp_debug_tl_r", "mdp_debug_tl_ra"):
    f = getattr(lib, name)
    f.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    fns.append(f)
for f in fns:
    assert f(None, 1) == 0
rounds = r.step()
r.synchronize()
NS, NW = 1024, 512
st_all = np.full((NS, NW), np.iinfo(np.uint64).max, dtype=np.uint64)
en_all = np.zeros((NS, NW), dtype=np.uint64)
for f in fns:
    buf = np.zeros(NS * NW * 2, dtype=np.uint64)
    assert f(buf.ctypes.data_as(ctypes.POINTER(ctypes.c_ulonglong)), 0) == 0
    a = buf.reshape(NS, NW, 2)
    st_all = np.where(a[:, :, 0] > 0, np.minimum(st_all, a[:, :, 0]), st_all)
    en_all = np.maximum(en_all, a[:, :, 1])
tl = np.zeros((NS, 2), dtype=np.uint64)
tl[:, 0] = st_all.min(axis=1)
tl[:, 1] = en_all.max(axis=1)
wg_end = en_all.reshape(64, 4, 4, NW)  # per-workgroup ends
wg_st = st_all.reshape(64, 4, 4, NW)
tl = tl.reshape(64, 4, 4, 2)  # ctr, kind, role, (start, end)
used = np.where(tl[:, :, :, 1].max(axis=(1, 2)) > 0)[0]
KIND = ["critic launch", "critic optimizer", "actor launch", "actor optimizer"]
ROLE = [["critic step", "actor_pre", "index draw", "-"], ["chunks/stats", "-", "-", "draw piece"],
        ["actor step", "critic_pre", "-", "-"], ["chunks/Polyak/stats", "-", "-", "draw piece"]]
# launches in time order: (ctr, kind) -> (start, end) over the roles that ran
seq = []
for c in used:
    for k in range(4):
        st = tl[c, k, :, 0]
        en = tl[c, k, :, 1]
        ok = en > 0
        if ok.any():
            seq.append((int(st[ok].min()), int(en[ok].max()), int(c), k))
seq.sort()
print(f"{rounds} rounds, {len(seq)} instrumented launches (ctr {used.min()}..{used.max()})")
body = {k: [] for k in range(4)}
role_end = {(k, q): [] for k in range(4) for q in range(4)}
gap = {}
for i, (s0, e0, c, k) in enumerate(seq):
    body[k].append((e0 - s0) / 100.0)
    for q in range(4):
        if tl[c, k, q, 1] > 0:
            role_end[(k, q)].append((int(tl[c, k, q, 1]) - s0) / 100.0)
    if i + 1 < len(seq):
        s1, _, _, k1 = seq[i + 1]
        gap.setdefault((k, k1), []).append((s1 - e0) / 100.0)
span = (seq[-1][1] - seq[0][0]) / 100.0
print(f"first start -> last end: {span:.1f} us ({span / max(rounds, 1):.2f} us per round)")
tot_body = sum(sum(v) for v in body.values())
tot_gap = sum(sum(v) for v in gap.values())
print(f"sum of launch bodies {tot_body:.1f} us, sum of gaps {tot_gap:.1f} us")
for k in range(4):
    if body[k]:
        v = np.array(body[k])
        print(f"{KIND[k]:>17s}: n={len(v):3d} body median {np.median(v):6.2f} us (min {v.min():.2f}, max {v.max():.2f})")
        for q in range(4):
            e = role_end[(k, q)]
            if e:
                print(f"{'':>19s}{ROLE[k][q]:<20s} ends at median {np.median(e):6.2f} us")
for (k0, k1), v in sorted(gap.items()):
    v = np.array(v)
    print(f"gap {KIND[k0]:>17s} -> {KIND[k1]:<17s} n={len(v):3d} median {np.median(v):5.2f} us (min {v.min():.2f})")

# per-workgroup start / end of the optimizer launches (median over updates):
# which workgroups set the launch's length
for k in (1, 3):
    rel_s, rel_e = [], []
    for c in used:
        st = wg_st[c, k]
        en = wg_end[c, k]
        ok = en.max(axis=0) > 0
        if not ok.any():
            continue
        s0 = st.min()
        rel_s.append(np.where(ok, (st.min(axis=0).astype(np.float64) - s0) / 100.0, np.nan))
        rel_e.append(np.where(ok, (en.max(axis=0).astype(np.float64) - s0) / 100.0, np.nan))
    if not rel_e:
        continue
    ms = np.nanmedian(np.array(rel_s), axis=0)
    me = np.nanmedian(np.array(rel_e), axis=0)
    n = int(np.sum(~np.isnan(me)))
    print(f"{KIND[k]} per workgroup (median over updates), start / end us:")
    print("  " + "  ".join(f"{w}:{ms[w]:.2f}/{me[w]:.2f}" for w in range(n)))
for k in (0, 2):
    rel_s = []
    for c in used:
        st = wg_st[c, k]
        en = wg_end[c, k]
        ok = en.max(axis=0) > 0
        if not ok.any():
            continue
        s0 = st.min()
        rel_s.append(np.where(ok, (st.min(axis=0).astype(np.float64) - s0) / 100.0, np.nan))
    ms = np.nanmedian(np.array(rel_s), axis=0)
    print(f"{KIND[k]} dispatch: last workgroup starts at median {np.nanmax(ms):.2f} us")
