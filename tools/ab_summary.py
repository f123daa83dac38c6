"""Summarise tools/ab_s2.sh output: value and per-kernel event times, base vs variant."""
import glob
import json
import sys

d = sys.argv[1]
for kind in ("base", "var"):
    rows = [json.load(open(f)) for f in sorted(glob.glob(f"{d}/{kind}*.json"))]
    ks = rows[0]["kernel_pass"]["per_kind_ms_per_launch"].keys()
    avg = {k: sum(r["kernel_pass"]["per_kind_ms_per_launch"][k] for r in rows) / len(rows) * 1e3 for k in ks}
    print(kind, [round(r["value"]) for r in rows], {k: round(v, 2) for k, v in avg.items()})
