"""Diagnostic: throughput-mode gradients vs the fp64 restatement, per agent / net / tensor.

    python tools/tp_grad_check.py [B] [general(0/1)]       (MDP_GRAD_PAIR=0/1 in the env)
"""
import copy
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from maddpg_amd.engine import Engine  # noqa: E402
from oracle import nets, trainer  # noqa: E402
from tests.helpers import joint_rows, synthetic_trainer_case  # noqa: E402
from tests.test_gpu_parity import _device_grads  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
mode = sys.argv[2] if len(sys.argv) > 2 else "throughput"
dims, H, L = [22, 22, 22, 22, 20, 20], 128, 3000
c = synthetic_trainer_case(dims, B, L, seed=61, H=H)
n = len(dims)
eng = Engine(dims, c["local_q"], num_units=H, batch_size=B, capacity=L + 7)
eng.add_rows(torch.from_numpy(joint_rows(c["data"], dims)))
for i, p in enumerate(c["params"]):
    for w in ("actor", "critic", "tgt_actor", "tgt_critic"):
        eng.set_params(i, w, p[w])
agents = [trainer.AgentParams(**copy.deepcopy(p), local_q=c["local_q"][i]) for i, p in enumerate(c["params"])]
nets.F32 = trainer.F32 = np.float64
og = []
for i in range(n):
    batch_n = [tuple(x[c["idx"][i]] for x in c["data"][j]) for j in range(n)]
    og.append({1: trainer.critic_grads(agents, i, batch_n, c["u_tgt"][i])[0],
               0: trainer.actor_grads(agents, i, batch_n, c["u_act"][i])[0]})
if mode == "throughput":
    eng.set_update_mode("throughput")
    eng.update_all(idx=torch.from_numpy(c["idx"]), u_tgt=torch.from_numpy(c["u_tgt"]),
                   u_act=torch.from_numpy(c["u_act"]))
    eng.synchronize()
    grads = {(i, net): _device_grads(eng, i, net) for i in range(n) for net in (0, 1)}
else:   # per agent, strict launches but on the round-start parameters: critic_grad + reduce per net
    grads = {}
    for i in range(n):
        idx = torch.from_numpy(c["idx"][i])
        eng.critic_grad(i, idx, torch.from_numpy(c["u_tgt"][i]))
        eng.reduce_grad(i, 1)
        eng.actor_grad(i, idx, torch.from_numpy(c["u_act"][i]))
        eng.reduce_grad(i, 0)
        eng.synchronize()
        grads[(i, 0)] = _device_grads(eng, i, 0)
        grads[(i, 1)] = _device_grads(eng, i, 1)
for i in range(n):
    for net in (1, 0):
        dg = grads[(i, net)]
        errs = []
        for k, ref in og[i][net].items():
            ref = np.asarray(ref, np.float64).reshape(dg[k].shape)
            scale = float(np.abs(ref).max()) or 1.0
            errs.append(f"{k} {float(np.abs(dg[k] - ref).max()) / scale:.1e}")
        print(f"agent {i} {'critic' if net else 'actor '}: " + "  ".join(errs))
