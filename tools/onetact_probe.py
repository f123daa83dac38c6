"""Timing bound of hoisting target actors out of the S5 critic launch.

    MDP_LIB=maddpg_amd/libmaddpg_hip_onetact.so python tools/onetact_probe.py   # -DMDP_EXP_ONE_TACT build
    python tools/onetact_probe.py                                                # the shipped library

S5 topology (tag N=6, H=128, B=4096); every update starts from the same
finite parameters (restored before each one), so the timing-only build --
which runs ONE target actor in the critic launch and fills the other five
actors' a~ columns with a constant -- never trains itself into non-finite
values.  Prints the packet-event average of the critic-step launch."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from maddpg_amd import _lib  # noqa: E402
from maddpg_amd.engine import Engine  # noqa: E402

dims = [22, 22, 22, 22, 20, 20]
eng = Engine(dims, num_units=128, batch_size=4096, capacity=120000)
eng.add_rows(torch.rand(eng.capacity, eng.row_stride) * 2 - 1)
eng.init_params(0)
eng.seed_py_random(0)
saved = [{w: eng.get_params(i, w) for w in ("actor", "critic", "tgt_actor", "tgt_critic")} for i in range(eng.n)]
g = torch.Generator().manual_seed(0)
idx = torch.randint(0, eng.capacity, (4096,), dtype=torch.int32, generator=g)
for it in range(8):
    if it == 3:
        eng.prof_enable("critic_grad", True)
    for i, p in enumerate(saved):
        for w, v in p.items():
            eng.set_params(i, w, v)
    eng.update(1, idx=idx)
eng.synchronize()
ms, n = eng.prof_read("critic_grad")
st = eng.stats(1)
print(json.dumps({"lib": os.path.basename(_lib.LIB_PATH), "critic_launch_us": round(ms / n * 1e3, 3), "launches": n,
                  "stats_finite": bool(all(abs(x) < 1e30 for x in st))}))
