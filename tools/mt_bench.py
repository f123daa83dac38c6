"""Time k_make_index (CPython MT19937 + randint) for the S2 and S5 draw counts."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from maddpg_amd.engine import Engine  # noqa: E402

eng = Engine([18, 18, 18], batch_size=1024, capacity=200000)
eng.add_rows(torch.rand(110000, eng.row_stride))
eng.seed_py_random(0)
for count in (3072, 24576):
    out = torch.empty(count, dtype=torch.int32, device=eng.device)
    for _ in range(3):
        eng.make_index(count, out)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 50
    a.record()
    for _ in range(n):
        eng.make_index(count, out)
    b.record()
    torch.cuda.synchronize()
    print(f"count {count}: {a.elapsed_time(b) / n * 1000:.2f} us per draw launch", flush=True)
