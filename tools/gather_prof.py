"""The gather stage at one size, for a rocprofv3 --kernel-trace --stats cross-check
of bench.py's event-timed k_gather_rows duration:

    rocprofv3 --kernel-trace --stats -d gpurun_out/gprof -o run --output-format csv -- \
        python3 tools/gather_prof.py --rows 4194304
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=1 << 22)
ap.add_argument("--iters", type=int, default=20)
a = ap.parse_args()
print(json.dumps(bench.gather_stage([18, 18, 18], sizes=(a.rows,), iters=a.iters)))
