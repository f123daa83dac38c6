"""Child process of tests/test_dp_standin_gpu.py (not collected by pytest).

Runs the library's NATIVE data-parallel path (mdp_dp_init + the RCCL calls
issued from C++) with a world of G = 2 (MDP_STANDIN_G: any power of two, e.g. 8) on one GPU: MDP_RCCL_LIB points the
library's dlopen at tests/rccl_standin/libnccl_standin.so, whose
ncclAllReduce multiplies in place by the communicator size -- the sum over two
replicas holding this rank's data -- and logs every call.  The RCCL library is
chosen once per process, hence a child of its own.  Prints one JSON line.

    MDP_RCCL_LIB=.../libnccl_standin.so python tests/standin_child.py strict|throughput|graph
"""
import copy
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from maddpg_amd.engine import Engine  # noqa: E402
from oracle import trainer  # noqa: E402
from tests.helpers import joint_rows, synthetic_trainer_case  # noqa: E402

G = int(os.environ.get("MDP_STANDIN_G", "2"))   # communicator size (a power of two: x G is exact)
SETS = ("actor", "critic", "tgt_actor", "tgt_critic", "m_actor", "v_actor", "m_critic", "v_critic")


def calls(reset=True):
    lib = ctypes.CDLL(os.environ["MDP_RCCL_LIB"])   # the instance the engine dlopened (same path)
    lib.mdp_standin_calls.restype = ctypes.c_int64
    buf = (ctypes.c_int64 * (7 * 4096))()
    n = lib.mdp_standin_calls(buf, 4096, 1 if reset else 0)
    rows = np.frombuffer(buf, np.int64)[:7 * min(n, 4096)].reshape(-1, 7)
    return [dict(count=int(r[0]), recv=int(r[1]), send=int(r[2]), op=int(r[3]), dtype=int(r[4]),
                 nranks=int(r[5]), captured=int(r[6])) for r in rows]


def engine(dims, B, L, c, dp):
    eng = Engine(dims, batch_size=B, capacity=L + 7)
    eng.add_rows(torch.from_numpy(joint_rows(c["data"], dims)))
    for i, p in enumerate(c["params"]):
        for w in ("actor", "critic", "tgt_actor", "tgt_critic"):
            eng.set_params(i, w, p[w])
    if dp:
        eng.dp_init(G, 0)
    return eng


def spans(eng):
    """(offset in floats from the GRAD region's start, length) of every net's gradient"""
    base = eng.region("grad").data_ptr()
    return {(i, net): ((eng.grad_view(i, net).data_ptr() - base) // 4, eng.grad_view(i, net).numel())
            for i in range(eng.n) for net in (0, 1)}


def max_param_diff(a, b):
    return max(float(np.max(np.abs(a.get_params(i, w)[k] - b.get_params(i, w)[k])))
               for i in range(a.n) for w in SETS for k in a.get_params(i, w))


def oracle_err(eng, agents, want):
    loss = max(float(abs(eng.stats(i)[0] - want[i][0]) / (abs(want[i][0]) + 1e-12)) for i in range(eng.n))
    par = 0.0
    for i in range(eng.n):
        for w, ref in (("actor", agents[i].actor), ("critic", agents[i].critic),
                       ("tgt_actor", agents[i].tgt_actor), ("tgt_critic", agents[i].tgt_critic)):
            dev = eng.get_params(i, w)
            for k in ref:
                par = max(par, float(np.max(np.abs(dev[k] - ref[k].reshape(dev[k].shape)))))
    return loss, par


def strict(rounds=2):
    """the reference's order (maddpg.py:188-194) per agent: critic grads -> k_reduce ->
    ncclAllReduce(critic span) -> clip + Adam x 1/G, then the same for the actor"""
    dims, B, L = [18, 18, 18], 256, 1200
    c = synthetic_trainer_case(dims, B, L, seed=41)
    a, b = engine(dims, B, L, c, True), engine(dims, B, L, c, False)
    agents = [trainer.AgentParams(**copy.deepcopy(p)) for p in c["params"]]
    rng = np.random.default_rng(5)
    sp = spans(a)
    grad0 = a.region("grad").data_ptr()
    calls()
    out = {"rounds": [], "G": G}
    for r in range(rounds):
        idx = c["idx"] if r == 0 else rng.integers(0, L, size=(3, B)).astype(np.int32)
        ut = c["u_tgt"] if r == 0 else rng.uniform(1e-6, 1, c["u_tgt"].shape).astype(np.float32)
        ua = c["u_act"] if r == 0 else rng.uniform(1e-6, 1, c["u_act"].shape).astype(np.float32)
        want = []
        for i in range(3):
            kw = dict(idx=torch.from_numpy(idx[i]), u_tgt=torch.from_numpy(ut[i]), u_act=torch.from_numpy(ua[i]))
            a.update(i, **kw)
            b.update(i, **kw)
            want.append(trainer.update(agents, i, c["data"], idx[i], ut[i], ua[i])[0])
        a.synchronize()
        b.synchronize()
        log = calls()
        loss, par = oracle_err(a, agents, want)
        exp = [sp[(i, net)] for i in range(3) for net in (1, 0)]   # critic then actor, agent by agent
        got = [((x["recv"] - grad0) // 4, x["count"]) for x in log]
        out["rounds"].append(dict(
            allreduces=len(log), spans_match=got == exp, in_place=all(x["recv"] == x["send"] for x in log),
            nranks=sorted({x["nranks"] for x in log}), sum_fp32=all(x["op"] == 0 and x["dtype"] == 7 for x in log),
            dp_vs_single_max_diff=max_param_diff(a, b), loss_rel_err=loss, param_abs_err=par,
            stats_equal=all(np.array_equal(a.stats(i), b.stats(i)) for i in range(3))))
    out["dp_info"] = a.dp_info()
    return out


def throughput():
    """one all-reduce of the whole gradient region per round (SURVEY 8e's throughput mode)"""
    dims, B, L = [18, 18, 18], 256, 1200
    c = synthetic_trainer_case(dims, B, L, seed=43)
    a, b = engine(dims, B, L, c, True), engine(dims, B, L, c, False)
    a.set_update_mode("throughput")
    b.set_update_mode("throughput")
    agents = [trainer.AgentParams(**copy.deepcopy(p)) for p in c["params"]]
    grad = a.region("grad")
    calls()
    kw = dict(idx=torch.from_numpy(c["idx"]), u_tgt=torch.from_numpy(c["u_tgt"]), u_act=torch.from_numpy(c["u_act"]))
    a.update_all(**kw)
    b.update_all(**kw)
    want = trainer.update_round_throughput(agents, c["data"], c["idx"], c["u_tgt"], c["u_act"])
    a.synchronize()
    b.synchronize()
    log = calls()
    loss, par = oracle_err(a, agents, want)
    sp = spans(a)
    last = max(o + n for o, n in sp.values())
    out = dict(allreduces=len(log), recv_is_grad_base=all(x["recv"] == grad.data_ptr() for x in log),
               count=[x["count"] for x in log], covers_every_net=bool(log) and log[0]["count"] >= last,
               nranks=sorted({x["nranks"] for x in log}), dp_vs_single_max_diff=max_param_diff(a, b),
               loss_rel_err=loss, param_abs_err=par)
    # two more rounds, the device noise and index stream this time: the update
    # counter (Ctl.upd_ctr, the Philox counter of the actor-loss samples) must
    # advance by n per round on the data-parallel path as on one GPU -- the
    # general kernels' pair lists bump it once, in the step pass
    for _ in range(2):
        a.update_all()
        b.update_all()
    a.synchronize()
    b.synchronize()
    calls()
    out.update(rounds=3, n=a.n, upd_ctr=[upd_ctr(a), upd_ctr(b)], dp_vs_single_after=max_param_diff(a, b))
    return out


CTL_UPD_CTR_OFFSET = 2568  # Ctl.upd_ctr (mdp_topo.h; tests/test_gpu_parity.py)


def upd_ctr(eng):
    ctl = eng.region("ctl", torch.uint8).cpu().numpy()
    return int(ctl[CTL_UPD_CTR_OFFSET:CTL_UPD_CTR_OFFSET + 4].view(np.uint32)[0])


def graph():
    """the training loop (rollout + due rounds, mdp_train_step) over the stand-in world:
    eager collectives and collectives captured in the step graph (MDP_DP_GRAPHS=1)
    both equal the single-GPU two-kernel path bit for bit"""
    from maddpg_amd.runner import VecRunner

    def runner(dp):
        r = VecRunner("simple_spread", 64, batch_size=128, capacity=20000, seed=3, train_every=16)
        if dp:
            r.eng.dp_init(G, 0)
            r.native_dp = True
        r.prefill()
        return r

    a, b = runner(True), runner(False)
    calls()
    rounds = 0
    for _ in range(3):
        k = a.step()
        assert k == b.step()
        rounds += k
    a.eng.synchronize()
    b.eng.synchronize()
    log = calls()
    return dict(rounds=rounds, allreduces=len(log), captured=sum(x["captured"] for x in log),
                dp_vs_single_max_diff=max_param_diff(a.eng, b.eng),
                beta_equal=all(np.array_equal(a.eng.get_beta_powers(i, n), b.eng.get_beta_powers(i, n))
                               for i in range(3) for n in (0, 1)))


if __name__ == "__main__":
    assert torch.cuda.is_available()
    mode = sys.argv[1]
    res = {"strict": strict, "throughput": throughput, "graph": graph}[mode]()
    print(json.dumps(res))
