"""Per-kernel average of rocprofv3 PMC counters (counter_collection.csv files under a dir)."""
import collections
import csv
import os
import sys

agg = collections.defaultdict(list)
for root, _, files in os.walk(sys.argv[1]):
    for f in files:
        if f.endswith("counter_collection.csv"):
            for r in csv.DictReader(open(os.path.join(root, f))):
                k = r["Kernel_Name"].split("(")[0].replace("void ", "")
                agg[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
kern = sorted({k for k, _ in agg})
cnts = sorted({c for _, c in agg})
for k in kern:
    if k.startswith("__amd"):
        continue
    print(k)
    for c in cnts:
        v = agg.get((k, c))
        if v:
            print(f"   {c:28s} {sum(v) / len(v):14.1f}")
