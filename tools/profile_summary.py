"""Summarise rocprofv3 runs of bench.py into profiles/.

    python tools/profile_summary.py --tag r01 --trace gpurun_out/prof_trace \
        --fetch gpurun_out/pmc_fetch --write gpurun_out/pmc_write --bench gpurun_out/prof_bench.json

Writes profiles/<tag>_kernel_stats.csv (the --kernel-trace --stats summary),
profiles/<tag>_lib.json (the sha256 of the library every bench line of the run
loaded -- they must agree),
profiles/<tag>_pmc.csv (per-kernel average FETCH_SIZE / WRITE_SIZE per launch)
and updates profiles/pmc_traffic.json, which bench.py reads for the
roofline's `traffic` field.  HBM bytes per launch follow
MI355X_MICROARCH.md §HBM for gfx950: FETCH_SIZE (KiB) reports half of the
bytes of wide coalesced reads -> x2; WRITE_SIZE (KiB) is exact for 16-B stores:
    hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024
(other access widths are uncalibrated; the value is an estimate).
"""
import argparse
import collections
import csv
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    n = name.split("(")[0]
    for pre in ("void ",):
        if n.startswith(pre):
            n = n[len(pre):]
    return n.split("<")[0]


def counters(d, cname):
    agg = collections.defaultdict(list)
    for f in os.listdir(d):
        if f.endswith("counter_collection.csv"):
            for r in csv.DictReader(open(os.path.join(d, f))):
                if r["Counter_Name"] == cname:
                    agg[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("--trace", required=True)
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--bench")
    ap.add_argument("--mfma", help="rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE pass")
    ap.add_argument("--sq", help="rocprofv3 --pmc pass of the SQ wave-state counters (profile_run.sh pass 6)")
    ap.add_argument("--clock-ghz", type=float, default=2.3, help="shader clock for the MFMA busy fraction")
    ap.add_argument("--config-key", default=None)
    a = ap.parse_args()
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = [f for f in os.listdir(a.trace) if f.endswith("kernel_stats.csv")][0]
    shutil.copy(os.path.join(a.trace, stats), os.path.join(prof, f"{a.tag}_kernel_stats.csv"))
    rows = list(csv.DictReader(open(os.path.join(a.trace, stats))))
    avg_ns = {short(r["Name"]): float(r["AverageNs"]) for r in rows}
    key = a.config_key
    bench = None
    lib = None
    if a.bench and os.path.exists(a.bench):
        bench = json.loads(open(a.bench).read().strip().splitlines()[-1])
        lib = bench.get("lib_sha256")
        if key is None:
            cfg = bench["config"]
            key = f"{cfg['scenario']}_E{cfg['num_envs_per_gpu']}_B{cfg['global_batch'] // bench['n_gpus']}_H64"
        shutil.copy(a.bench, os.path.join(prof, f"{a.tag}_bench.json"))
    # every bench line of the run (trace, PMC passes, plain bench) must come from ONE
    # library build: its sha256 goes with the summary, and bench.py uses the committed
    # durations only for that build
    seen = {}
    run_dir = os.path.dirname(os.path.normpath(a.trace))
    for f in sorted(os.listdir(run_dir)):
        if f.endswith(".json"):
            try:
                line = json.loads(open(os.path.join(run_dir, f)).read().strip().splitlines()[-1])
            except (ValueError, IndexError):
                continue
            if isinstance(line, dict) and line.get("lib_sha256"):
                seen[f] = line["lib_sha256"]
    if len(set(seen.values())) > 1:
        raise SystemExit(f"bench lines of {run_dir} come from different library builds: {seen}")
    lib = lib or next(iter(seen.values()), None)
    json.dump({"tag": a.tag, "lib_sha256": lib, "bench_lines": seen, "config_key": key},
              open(os.path.join(prof, f"{a.tag}_lib.json"), "w"), indent=1, sort_keys=True)
    out = {}
    if a.fetch and a.write:
        fe, wr = counters(a.fetch, "FETCH_SIZE"), counters(a.write, "WRITE_SIZE")
        with open(os.path.join(prof, f"{a.tag}_pmc.csv"), "w") as fp:
            fp.write("kernel,avg_ns,FETCH_SIZE_KiB,WRITE_SIZE_KiB,hbm_bytes_per_launch\n")
            for k in sorted(set(fe) | set(wr)):
                hb = (2 * fe.get(k, 0.0) + wr.get(k, 0.0)) * 1024
                out[k] = {"fetch_kib": fe.get(k), "write_kib": wr.get(k), "hbm_bytes_per_launch": hb,
                          "avg_ns": avg_ns.get(k)}
                fp.write(f"{k},{avg_ns.get(k, '')},{fe.get(k, '')},{wr.get(k, '')},{hb:.0f}\n")
        path = os.path.join(prof, "pmc_traffic.json")
        allj = json.load(open(path)) if os.path.exists(path) else {}
        allj[key] = dict(out, _source=f"{a.tag}_pmc.csv", _lib_sha256=lib)
        json.dump(allj, open(path, "w"), indent=1, sort_keys=True)
    mf = {}
    if a.mfma:
        busy, gui = counters(a.mfma, "SQ_VALU_MFMA_BUSY_CYCLES"), counters(a.mfma, "GRBM_GUI_ACTIVE")
        with open(os.path.join(prof, f"{a.tag}_mfma.csv"), "w") as fp:
            # busy fraction of the chip's 1024 SIMDs over the kernel's average duration
            fp.write("kernel,avg_ns,SQ_VALU_MFMA_BUSY_CYCLES,GRBM_GUI_ACTIVE,mfma_busy_frac_of_1024_simds\n")
            for k in sorted(busy):
                ns = avg_ns.get(k)
                frac = busy[k] / (ns * 1e-9 * a.clock_ghz * 1e9 * 1024) if ns else None
                mf[k] = {"mfma_busy_cycles": busy[k], "grbm_gui_active": gui.get(k), "mfma_busy_frac": frac}
                fp.write(f"{k},{ns or ''},{busy[k]:.0f},{gui.get(k, '')},{'' if frac is None else f'{frac:.5f}'}\n")
        if key:
            path = os.path.join(prof, "pmc_traffic.json")
            allj = json.load(open(path)) if os.path.exists(path) else {}
            for k, v in mf.items():
                allj.setdefault(key, {}).setdefault(k, {}).update(v)
            json.dump(allj, open(path, "w"), indent=1, sort_keys=True)
    sq = {}
    if a.sq:
        names = ["SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_ANY",
                 "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_LDS_BANK_CONFLICT"]
        got = {n: counters(a.sq, n) for n in names}
        kern = sorted(set().union(*[set(g) for g in got.values()]))
        with open(os.path.join(prof, f"{a.tag}_sq.csv"), "w") as fp:
            # per launch; wave-state counters in quad-cycles summed over every wave of the launch;
            # the shares are of SQ_WAVE_CYCLES (WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES)
            fp.write("kernel,avg_ns," + ",".join(names) +
                     ",wait_any_share,wait_inst_any_share,wait_inst_lds_share,active_share\n")
            for k in kern:
                v = {n: got[n].get(k) for n in names}
                wc = v["SQ_WAVE_CYCLES"] or 0.0
                sh = [(v[n] or 0.0) / wc if wc else 0.0 for n in
                      ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_ANY")]
                sq[k] = dict(v, shares=sh)
                fp.write(f"{k},{avg_ns.get(k, '')}," + ",".join("" if v[n] is None else f"{v[n]:.0f}" for n in names)
                         + "," + ",".join(f"{x:.4f}" for x in sh) + "\n")
    print(json.dumps({"tag": a.tag, "config_key": key, "lib_sha256": lib, "avg_ns": avg_ns, "pmc": out, "mfma": mf, "sq": sq}, indent=1))


if __name__ == "__main__":
    main()
