"""Phase budget of the S2 gradient launches (k_critic_grad_r, k_actor_grad_r).

    make -C maddpg_amd/csrc budget
    rocprofv3 --kernel-trace --stats -d <dir> -o run --output-format csv -- \
        env MDP_LIB=... python3 tools/grad_budget.py --out <json>     (see tools/_cmd_r06d.sh)

The budget build (-DMDP_BUDGET, mdp_grads_r.hip) has every workgroup of agent
1's critic-step and actor-step launches store s_memrealtime (100 MHz, one clock
for the whole GPU) at its phase points, without adding any wait.  After a few
graph-replayed S2 training steps (BASELINE configs[1], the bench's workload)
this reads the last such launch of each kind and prints, per role, the
workgroup start spread (the dispatch ramp) and every phase point as the median
over the role's workgroups and for the workgroup that ends the launch; the
critical workgroup's phases sum exactly to the launch's in-kernel span (first
workgroup start -> last wave end).  What rocprof adds beyond that span (the
dispatch packet's begin -> first start, last end -> end of packet) is the
rocprof average of the same run minus the span: `--rocprof-csv` reads it.
"""
import argparse
import csv
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# phase points (mdp_grads_r.hip MDP_STAMP / MDP_STAMPW / CRIT_T / CPRE_T under MDP_BUDGET)
CRITIC_STEP = [  # (point, wave, what the interval ending here holds)
    (0, "all", "kernel-argument and LDS set-up, B0 entry"),
    (54, "w3", "cpre block and critic-head weight loads issued"),
    (48, "w0", "target actor pprev: weight loads issued (16-B, register-resident), Gumbel noise"),
    (49, "w0", "replay rows landed in LDS (gather by waves 4..7: index load -> row loads)"),
    (50, "w0", "target actor pprev: L1 + L2 column tile (MFMA chain)"),
    (55, "w3", "wave 3's L2 tile done"),
    (51, "w0", "all four L2 tiles handed over (LDS counter)"),
    (52, "w0", "target actor head + Gumbel-softmax sample a~"),
    (53, "w0", "B2 (a~ of every target actor in LDS)"),
    (4, "w4", "B2 exit (target-critic waves)"),
    (5, "w4", "target critic L1: the a~ k-steps (resumed from cpre) | B3"),
    (6, "w4", "target critic L2 tile | B4"),
    (60, "w4", "target-critic head q', fp64 TD target, dL/dq"),
    (61, "w4", "d2 = dq W3 o [h2 > 0], dW3 / db3 column loop"),
    (7, "w4", "dW3 / db3 partial-slab stores issued"),
    (8, "w4", "B5 (d2, dh1 ready)"),
    (28, "last", "B5 exit, every wave"),
    (29, "last", "dW2 tiles (partial-slab stores issued)"),
    (30, "last", "dW1 tiles over the obs part"),
    (31, "last", "dW1 tiles over the act part"),
    (32, "last", "db2 / db1 column sums"),
    (9, "w4", "wave 4 after its weight-gradient tiles"),
    (10, "last", "stats partials"),
    (63, "last", "last wave's end"),
]
ACTOR_STEP = [
    (16, "all", "kernel-argument and LDS set-up, B0 entry"),
    (18, "w0", "apre block (actor forward from the critic launch) + backward weights issued"),
    (56, "w1", "replay rows landed (apre rows; waves 2..7)"),
    (57, "w1", "critic L1, wave 1's third of the replay-part contraction"),
    (58, "w3", "critic L1, wave 3's third"),
    (19, "w1", "B2 exit (the thirds in LDS)"),
    (20, "w1", "critic L1 sum + a_i part | B2b, critic L2 tile + q partials"),
    (21, "w4", "B3 exit"),
    (22, "w4", "dh1c tile | B4"),
    (23, "w0", "B4 exit (wave 0)"),
    (24, "w0", "da, softmax backward + reg, d2a rows | B4b"),
    (25, "w4", "B5 exit"),
    (26, "w4", "dh1a tile, dW2a tiles | B6"),
    (27, "last", "dW1a tiles, db1a, stats partials"),
    (63, "last", "last wave's end"),
]
CRITIC_PRE = [(33, "last", "start"), (34, "last", "rows landed"), (35, "last", "forward chains to B2"),
              (36, "last", "B2 exit"), (37, "last", "hand-off stores issued"), (38, "last", "tile end"),
              (63, "last", "last wave's end")]
US = 0.01  # one s_memrealtime tick = 10 ns
# slots: 62 / 63 the workgroup's start / end on the shader clock (s_memtime, the
# clock of every other point), 64 / 65 the same on s_memrealtime


def role_table(b, wgs, points, t_launch):
    wgs = np.asarray([w for w in wgs if b[w, 64] > 0 and b[w, 65] > b[w, 64]])
    start = b[wgs, 62].astype(np.int64)          # shader clock
    rstart = b[wgs, 64].astype(np.int64)         # GPU-wide clock
    rend = b[wgs, 65].astype(np.int64)
    # us per shader tick of each workgroup (its start -> end on both clocks)
    k = (rend - rstart) * US / np.maximum(b[wgs, 63].astype(np.int64) - start, 1)
    rows = []
    for pt, wave, what in points:
        if pt == 63:
            rel = (rend - rstart) * US
            good = np.ones(len(wgs), bool)
        else:
            v = b[wgs, pt].astype(np.int64)
            good = v >= start
            if not good.any():
                continue
            rel = (v[good] - start[good]) * k[good]
        rows.append({"point": pt, "wave": wave, "what": what, "median_us": round(float(np.median(rel)), 3),
                     "max_us": round(float(rel.max()), 3)})
    crit = int(np.argmax(rend))
    cw = int(wgs[crit])
    # the critical workgroup's points in time order: consecutive deltas sum to its span
    pts = sorted((int(b[cw, pt]), pt, wave, what) for pt, wave, what in points if int(b[cw, pt]) >= start[crit])
    path, prev = [], int(start[crit])
    for v, pt, wave, what in pts:
        path.append({"point": pt, "wave": wave, "what": what, "at_us": round((v - start[crit]) * k[crit], 3),
                     "delta_us": round((v - prev) * k[crit], 3)})
        prev = v
    return {"workgroups": int(len(wgs)),
            "shader_clock_ghz_median": round(float(np.median(1e-3 / k)), 3),
            "start_spread_us": [round((rstart.min() - t_launch) * US, 3), round((rstart.max() - t_launch) * US, 3)],
            "end_median_us": round(float(np.median(rend - t_launch)) * US, 3),
            "end_max_us": round(float((rend.max() - t_launch) * US), 3),
            "span_median_us": round(float(np.median(rend - rstart)) * US, 3),
            "points": rows,
            "critical_wg": {"wg": cw, "start_us": round((rstart[crit] - t_launch) * US, 3),
                            "end_us": round((rend[crit] - t_launch) * US, 3), "path": path}}


def launch_summary(b, roles):
    used = b[:, 64] > 0
    t0 = int(b[used, 64].min())
    t1 = int(b[used, 65].max())
    out = {"in_kernel_span_us": round((t1 - t0) * US, 3), "roles": {}}
    for name, wgs, pts in roles:
        wgs = [w for w in wgs if b[w, 64] > 0]
        if wgs:
            out["roles"][name] = role_table(b, wgs, pts, t0)
    return out


def rocprof_avgs(path):
    avg = {}
    for r in csv.DictReader(open(path)):
        n = r["Name"].split("(")[0].replace("void ", "").split("<")[0]
        avg[n] = float(r["AverageNs"]) / 1000
    return avg


def agent_durations(trace_csv, n=3):
    """per-dispatch durations (us) of the gradient kernels by agent, from a
    rocprofv3 kernel trace: the launches after each k_rollout come as rounds of
    n agents, so the j-th critic (actor) launch after a rollout is agent j mod n"""
    rows = sorted(csv.DictReader(open(trace_csv)), key=lambda r: int(r["Start_Timestamp"]))
    out = {"k_critic_grad_r": [[] for _ in range(n)], "k_actor_grad_r": [[] for _ in range(n)]}
    cnt = {k: 0 for k in out}
    for r in rows:
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0]
        if name == "k_rollout":
            cnt = {k: 0 for k in out}
        elif name in out:
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
            out[name][cnt[name] % n].append(dur)
            cnt[name] += 1
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out")
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--rocprof-csv", help="summarise: kernel_stats.csv of the run that made --in")
    ap.add_argument("--product-csv", help="kernel_stats.csv of the shipped library (instrumentation overhead)")
    ap.add_argument("--in", dest="inp")
    ap.add_argument("--trace-csv", help="kernel_trace.csv of the run that made --in")
    ap.add_argument("--product-trace-csv", help="kernel_trace.csv of the shipped library's bench")
    a = ap.parse_args()
    if a.inp:   # offline: combine the recorded points with rocprof averages
        d = json.load(open(a.inp))
        avg = rocprof_avgs(a.rocprof_csv)
        prod = rocprof_avgs(a.product_csv) if a.product_csv else {}
        for kind, kern in (("critic", "k_critic_grad_r"), ("actor", "k_actor_grad_r")):
            L = d[kind]
            L["rocprof_avg_us_budget_build"] = round(avg[kern], 3)
            L["outside_workgroups_us"] = round(avg[kern] - L["in_kernel_span_us"], 3)
            if kern in prod:
                L["rocprof_avg_us_product"] = round(prod[kern], 3)
                L["instrumentation_overhead_us"] = round(avg[kern] - prod[kern], 3)
        if a.trace_csv:
            bud = agent_durations(a.trace_csv)
            prd = agent_durations(a.product_trace_csv) if a.product_trace_csv else None
            for kind, kern in (("critic", "k_critic_grad_r"), ("actor", "k_actor_grad_r")):
                L = d[kind]
                own = bud[kern][1]
                # the recorded launch is agent 1's last one: its own packet duration
                L["rocprof_this_launch_us"] = round(own[-1], 3)
                L["outside_workgroups_this_launch_us"] = round(own[-1] - L["in_kernel_span_us"], 3)
                L["rocprof_agent1_avg_us_budget_build"] = round(float(np.mean(own)), 3)
                L["rocprof_by_agent_us_budget_build"] = [round(float(np.mean(x)), 3) for x in bud[kern]]
                if prd:
                    L["rocprof_agent1_avg_us_product"] = round(float(np.mean(prd[kern][1])), 3)
                    L["rocprof_by_agent_us_product"] = [round(float(np.mean(x)), 3) for x in prd[kern]]
        json.dump(d, open(a.out, "w"), indent=1)
        print(json.dumps({k: {x: v for x, v in d[k].items() if x != "roles"} for k in ("critic", "actor")}, indent=1))
        return
    from maddpg_amd import _lib
    from maddpg_amd.runner import VecRunner
    assert "budget" in _lib.LIB_PATH, "run with MDP_LIB=maddpg_amd/libmaddpg_hip_budget{,2}.so"
    lib = _lib.load()
    fn = lib.mdp_debug_budget
    fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    r = VecRunner("simple_spread", 1024, batch_size=1024, seed=0)   # BASELINE configs[1]
    r.prefill()
    for _ in range(a.steps):
        r.step()
    r.synchronize()
    buf = (ctypes.c_ulonglong * (2 * 160 * 72))()
    assert fn(buf, 0) == 0
    b = np.array(buf[:], dtype=np.uint64).reshape(2, 160, 72)
    nwg = 64
    res = {"config": "S2: simple_spread N=3, E=1024, B=1024, H=64; agent 1's launches of the last graph-replayed step",
           "rounds": r.rounds,
           "critic": launch_summary(b[0], [("critic_step", range(nwg), CRITIC_STEP),
                                            ("actor_pre", range(nwg, 2 * nwg), [(63, "last", "end")]),
                                            ("draw", [2 * nwg], [(63, "last", "end")])]),
           "actor": launch_summary(b[1], [("actor_step", range(nwg), ACTOR_STEP),
                                           ("critic_pre", range(nwg, 2 * nwg), CRITIC_PRE)])}
    s = json.dumps(res, indent=1)
    if a.out:
        open(a.out, "w").write(s)
    print(s)


if __name__ == "__main__":
    main()
