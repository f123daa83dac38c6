"""Median idle gap between consecutive kernels (rocprofv3 --kernel-trace csv).

    python tools/gaps.py gpurun_out/<dir>/run_kernel_trace.csv
"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
gaps = collections.defaultdict(list)
dur = collections.defaultdict(list)
for r in rows:
    dur[r["Kernel_Name"].split("(")[0].replace("void ", "")].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for a, b in zip(rows, rows[1:]):
    g = int(b["Start_Timestamp"]) - int(a["End_Timestamp"])
    ka = a["Kernel_Name"].split("(")[0].replace("void ", "")
    kb = b["Kernel_Name"].split("(")[0].replace("void ", "")
    if g < 50000:
        gaps[(ka, kb)].append(g)
for k, v in sorted(gaps.items(), key=lambda x: -len(x[1])):
    v.sort()
    print(f"{k[0]:>22s} -> {k[1]:<22s} n={len(v):5d} median gap {v[len(v) // 2] / 1000:6.2f} us")
for k, v in sorted(dur.items()):
    v.sort()
    print(f"{k:>24s} n={len(v):5d} median {v[len(v) // 2] / 1000:7.2f} us")
