"""Summarise A/B output (tools/ab_s2.sh, ab_lib.sh, ab_var.sh): value and
per-kernel event times, base vs variant, per file prefix:
    python3 tools/ab_summary.py <dir> [prefix ...]   (prefixes e.g. s5_ s2_; default none)"""
import glob
import json
import sys

d = sys.argv[1]
for pre in (sys.argv[2:] or [""]):
    for kind in ("base", "var", "ref"):
        files = sorted(glob.glob(f"{d}/{pre}{kind}*.json"))
        rows = []
        for f in files:
            try:
                rows.append(json.load(open(f)))
            except ValueError:
                print(f, "unreadable")
        if not rows:
            continue
        ks = rows[0]["kernel_pass"]["per_kind_ms_per_launch"].keys()
        avg = {k: sum(r["kernel_pass"]["per_kind_ms_per_launch"][k] for r in rows) / len(rows) * 1e3 for k in ks}
        print(pre + kind, [round(r["value"]) for r in rows], {k: round(v, 2) for k, v in avg.items()})
