"""Summarise S5 A/B runs of several variants: python3 tools/s5_variants.py <dir> [prefix]"""
import glob
import json
import re
import sys

d = sys.argv[1]
pre = sys.argv[2] if len(sys.argv) > 2 else "s5_"
rows = {}
for f in sorted(glob.glob(f"{d}/{pre}*.json")):
    kind = re.sub(r"\d+$", "", f.split("/")[-1][len(pre):-5])
    try:
        b = json.load(open(f))
    except ValueError:
        print(f, "unreadable")
        continue
    rows.setdefault(kind, []).append(b)
for kind, bs in rows.items():
    ks = bs[0]["kernel_pass"]["per_kind_ms_per_launch"]
    avg = {k: round(sum(b["kernel_pass"]["per_kind_ms_per_launch"][k] for b in bs) / len(bs) * 1e3, 2) for k in ks}
    print(f"{kind:10s}", [round(b["value"]) for b in bs], avg)
