import os, sys, time, json
sys.path.insert(0, os.getcwd())
import torch
from maddpg_amd.runner import VecRunner
res = {}
for dp in (0, 1):
    r = VecRunner("simple_spread", 1024, batch_size=1024, seed=0)
    if dp:
        r.eng.dp_init(1, 0); r.native_dp = True
    r.prefill()
    for _ in range(5): r.step()
    r.eng.synchronize(); t = time.perf_counter()
    for _ in range(30): r.step()
    r.eng.synchronize(); dt = time.perf_counter() - t
    res[f"dp{dp}_graphs{os.environ.get('MDP_DP_GRAPHS','0')}"] = 1024 * 30 / dt
print(json.dumps(res))
