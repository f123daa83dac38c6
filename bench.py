"""Benchmark: MADDPG training loop on MI355X (BASELINE.json metric).

metric: env-steps/sec (+ trainer-updates/sec), simple_spread N=3, batch 1024.
A "step" is one vector env step of E env copies per rank (actors + Gumbel +
MPE physics + replay append, all on the device) plus the update rounds the
reference cadence makes due (one round = every agent's update, per 100
transitions per rank, maddpg.py:164).  The replay is prefilled to the
reference's gate (batch*max_episode_len rows) before warm-up, so every timed
step trains.  `value` = env transitions of all ranks / wall time (max over
ranks) with everything resident in HBM.

    python bench.py                        # N=1, E=1024 (BASELINE configs[1])
    torchrun --nproc-per-node N bench.py --gpus N
    python bench.py --gpus N               # launches the N ranks itself (torchrun as a child)
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from maddpg_amd import _lib  # noqa: E402
from maddpg_amd.parallel import init_process_group_from_env  # noqa: E402
from maddpg_amd.runner import VecRunner  # noqa: E402

MARKER_KINDS = ("allreduce", "gather")   # timed by marker events around the call (mdp_api.cpp ProfScope)
FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: F32 matrix/vector dense peak
HBM_PEAK_GBS = 8000.0           # MI355X_MICROARCH.md: HBM3E 8 TB/s spec


def flops_critic_grad(eng, agent):
    """algorithmic flops of one k_critic_grad launch (batch B, agent's critic step)."""
    H, B = eng.num_units, eng.batch_size
    dims = eng.obs_dims
    lq = eng.local_q[agent]
    cin = dims[agent] + 5 if lq else sum(dims) + 5 * eng.n
    actors = [agent] if lq else range(eng.n)
    mac = sum(dims[j] * H + H * H + 5 * H for j in actors)       # target actors
    mac += 2 * (cin * H + H * H + H)                              # target critic + critic fwd
    mac += 2 * H * H + cin * H + 2 * H                            # critic backward (dW3,dh2,dW2,dh1,dW1)
    return 2.0 * B * mac


def flops_actor_grad(eng, agent):
    H, B = eng.num_units, eng.batch_size
    o = eng.obs_dims[agent]
    cin = o + 5 if eng.local_q[agent] else sum(eng.obs_dims) + 5 * eng.n
    mac = 2 * o * H + 5 * H * H + cin * H + 22 * H
    return 2.0 * B * mac


def bytes_critic_grad(eng, agent):
    """algorithmic bytes of one agent's critic step: the B fused replay
    rows (every agent's obs, act, obs', rew, done) + the indices + 8 touches of the
    critic (theta, target, Adam m/v read and written, grad) + every target actor read"""
    B, o, n = eng.batch_size, eng.obs_dims, eng.n
    row = 4 * (2 * sum(o) + 5 * n + 2)
    actors = [agent] if eng.local_q[agent] else range(n)
    return B * row + 4 * B + 4 * (8 * param_count(eng, agent, "critic") +
                                  sum(param_count(eng, j, "actor") for j in actors))


def bytes_actor_grad(eng, agent):
    """algorithmic bytes of one agent's actor step: the critic-input rows, the
    indices, the critic read once, 8 touches of the actor (theta, target, Adam)"""
    B, o, n = eng.batch_size, eng.obs_dims, eng.n
    cin = o[agent] + 5 if eng.local_q[agent] else sum(o) + 5 * n
    return 4 * B * cin + 4 * B + 4 * (param_count(eng, agent, "critic") + 8 * param_count(eng, agent, "actor"))


def param_count(eng, agent, net):
    """logical parameter count of one net (maddpg.py:113-149, mlp_model train.py:39-46)"""
    H, o, n = eng.num_units, eng.obs_dims, eng.n
    if net == "actor":
        return o[agent] * H + H + H * H + H + 5 * H + 5
    cin = o[agent] + 5 if eng.local_q[agent] else sum(o) + 5 * n
    return cin * H + H + H * H + H + H + 1


def bytes_rollout(eng):
    ne = eng.n_entities
    per_env = 4 * eng.row_stride + 2 * 2 * (4 * 2 * ne) + 16 + 4 * eng.n
    return per_env * eng.num_envs


def roofline_for(kind, eng, ms_avg):
    tp = getattr(eng, "update_mode", "strict") == "throughput"   # one launch serves every agent
    suffix = "_r" if eng.lib.mdp_grad_variant(eng.h, 0) == 1 else ""
    if kind == "grads":
        # the critic-step and actor-step launches of one agent's update, together:
        # each launch also runs part of the OTHER step (the actor step's forward
        # rides in the critic launch, the next critic step's independent part in
        # the actor launch), so the algorithmic flops are attributed to the pair
        fl = sum(flops_critic_grad(eng, i) + flops_actor_grad(eng, i) for i in range(eng.n)) / (1 if tp else eng.n)
        by = sum(bytes_critic_grad(eng, i) + bytes_actor_grad(eng, i) for i in range(eng.n)) / (1 if tp else eng.n)
        ach = fl / (ms_avg * 1e-3) / 1e12
        return {"bound": "mfma", "achieved": round(ach, 4), "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(ach / FP32_MFMA_PEAK_TFLOPS, 6), "traffic": None,
                "kernel": f"k_critic_grad{suffix}+k_actor_grad{suffix}", "kernels": [f"k_critic_grad{suffix}",
                                                                               f"k_actor_grad{suffix}"],
                "algorithmic_per_launch": fl, "algorithmic_bytes_per_launch": by, "avg_launch_ms": ms_avg,
                "launch_unit": "one critic-step launch + one actor-step launch (one agent's update)"}
    if kind in ("critic_grad", "actor_grad"):
        f = flops_critic_grad if kind == "critic_grad" else flops_actor_grad
        fl = sum(f(eng, i) for i in range(eng.n)) / (1 if tp else eng.n)
        ach = fl / (ms_avg * 1e-3) / 1e12
        return {"bound": "mfma", "achieved": round(ach, 4), "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(ach / FP32_MFMA_PEAK_TFLOPS, 6), "traffic": None,
                "kernel": f"k_{kind}{suffix}", "algorithmic_per_launch": fl, "avg_launch_ms": ms_avg}
    if kind == "rollout":
        by = bytes_rollout(eng)
    elif kind == "reduce_apply":
        # per launch (critic and actor launches alternate): the nwg partial
        # gradients + m, v, theta (read + write) + grad write + target (actor)
        H, o = eng.num_units, eng.obs_dims
        pa = sum(d * H + H + H * H + H + 5 * H + 5 for d in o) / eng.n
        cin = sum(o) + 5 * eng.n
        pc = cin * H + H + H * H + H + H + 1
        nwg = (eng.batch_size + 15) // 16
        by = 4 * ((pc + pa) / 2) * (nwg + 7) + 4 * pa
        if tp:   # one launch steps every net (2n), each with its own Polyak
            by = 4 * eng.n * (pc + pa) * (nwg + 8)
    else:
        return None
    ach = by / (ms_avg * 1e-3) / 1e9
    return {"bound": "hbm", "achieved": round(ach, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 6), "traffic": None, "kernel": f"k_{kind}",
            "algorithmic_per_launch": by, "avg_launch_ms": ms_avg}


MALL_BYTES = 256 << 20          # MI355X_MICROARCH.md: 256 MB Infinity Cache (MALL) in front of HBM
HBM_ACHIEVABLE_GBS = 6290.0     # MI355X_MICROARCH.md: measured achievable HBM read+write rate


def gather_stage(obs_dims, sizes=(1024, 1 << 16, 1 << 20, 1 << 22), iters=12, capacity=1 << 22):
    """SURVEY 8d's gather-only stage (replay_buffer.py:34-44 sample_index /
    _encode_sample, the HBM-roofline part of the north_star's fused
    sample+gather): k_gather_rows through mdp_sample_rows on uniform indices
    over a full 2^22-row ring (2.2 GB at S2's 528-B rows, 8.7x the 256 MB
    Infinity Cache), at the training batch and at bandwidth-bound row counts.
    Every timed launch draws FRESH indices (its own index tensor, all drawn
    before the timed launches), so no launch re-reads rows an earlier launch
    left in the MALL; the written rows rotate over two output buffers.
    Algorithmic bytes per launch = B*row (read) + 4B (indices) + B*row (the
    gathered rows written out; inside the gradient kernels they go to LDS
    instead).  Duration: a HIP event pair around every launch on the engine
    stream (mdp_prof_*, the empty pair's cost subtracted), so host issue gaps
    between small launches do not count.  `bound` per size: "hbm" when the
    ring the indices range over is larger than the MALL (a random row hits it
    with probability ~MALL/ring), "latency" for the training batch (a few
    microseconds per launch: the dispatch and one row round trip bound it)."""
    from maddpg_amd.engine import Engine
    eng = Engine(obs_dims, batch_size=1024, capacity=capacity)
    eng.set_ring(capacity, 0)
    row_b = eng.row_stride * 4
    ring_b = capacity * row_b
    ev = event_overhead_ms(eng.stream)
    res = []
    for B in sizes:
        gen = torch.Generator(device=eng.device)
        gen.manual_seed(B)
        # one index set per launch: iters timed + 2 warm-up
        idxs = [torch.randint(0, capacity, (B,), dtype=torch.int32, device=eng.device, generator=gen)
                for _ in range(iters + 2)]
        outs = [torch.empty((B, eng.row_stride), dtype=torch.float32, device=eng.device) for _ in range(2)]
        torch.cuda.synchronize()
        for k in range(2):
            eng.sample_rows(idxs[k], outs[k & 1])
        eng.synchronize()
        eng.prof_enable("gather", True)
        for k in range(iters):
            eng.sample_rows(idxs[2 + k], outs[k & 1])
        eng.synchronize()
        ms_tot, n = eng.prof_read("gather")
        eng.prof_enable("gather", False)
        ms = max(ms_tot / n - ev, 1e-6)
        by = 2 * B * row_b + 4 * B
        gbs = by / (ms * 1e-3) / 1e9
        bound = "latency" if B * row_b < (8 << 20) else ("hbm" if ring_b > 4 * MALL_BYTES else "cache")
        res.append({"rows": B, "bytes_per_launch": by, "avg_launch_ms": round(ms, 5), "achieved": round(gbs, 1),
                    "frac": round(gbs / HBM_PEAK_GBS, 4), "frac_of_achievable": round(gbs / HBM_ACHIEVABLE_GBS, 4),
                    "bound": bound, "fresh_indices_per_launch": True})
        del idxs, outs
    eng.close()
    return {"kernel": "k_gather_rows", "unit": "GB/s", "peak": HBM_PEAK_GBS, "achievable": HBM_ACHIEVABLE_GBS,
            "row_bytes": row_b, "ring_rows": capacity, "ring_bytes": ring_b, "mall_bytes": MALL_BYTES,
            "expected_mall_hit_share": round(min(1.0, MALL_BYTES / ring_b), 4), "sizes": res}


def event_overhead_ms(stream, pairs=64):
    """elapsed time of an EMPTY start/stop event pair on `stream` (what a bracketing
    pair adds to every measured launch), median of `pairs` samples."""
    evs = []
    for _ in range(pairs):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        b.record(stream)
        evs.append((a, b))
    stream.synchronize()
    ts = sorted(a.elapsed_time(b) for a, b in evs)
    return ts[len(ts) // 2]


def lib_sha256():
    """first 16 hex digits of the sha256 of the library this process loads: ties a
    committed rocprof summary (profiles/pmc_traffic.json `_lib_sha256`) to the
    build it measured"""
    import hashlib
    with open(_lib.LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def load_pmc(kernel, config_key):
    """the committed rocprofv3 PMC summary of `kernel` (profiles/pmc_traffic.json, written by
    tools/profile_summary.py): per-launch HBM bytes and the MFMA busy fraction."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return {}
    try:
        cfg = json.load(open(path)).get(config_key, {})
        out = dict(cfg.get(kernel) or {})
        if out and cfg.get("_source"):
            out["_source"] = "profiles/" + cfg["_source"]
        if out:
            out["_lib_sha256"] = cfg.get("_lib_sha256")
        return out
    except Exception:
        return {}


def cpu_baseline(args, threads=1, seconds=None, scenario=None):
    """the oracle's reference-structured loop on the host: 1 pinned core (the
    reference's single_threaded_session), or `threads` BLAS threads unpinned"""
    seconds = args.cpu_seconds if seconds is None else seconds
    scenario = scenario or args.scenario
    env = dict(os.environ)
    for k in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS"):
        env[k] = str(threads)
    cmd = [sys.executable, "-m", "oracle.train_loop", "--scenario", scenario,
           "--seconds", str(seconds), "--batch-size", str(args.batch_size),
           "--num-units", str(args.num_units), "--pin-core", "0" if threads == 1 else "-1"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=seconds * 6 + 120)
    if r.returncode != 0:
        return {"error": r.stderr[-500:]}
    out = json.loads(r.stdout.strip().splitlines()[-1])
    if threads != 1:
        return {"value": round(out["env_steps_per_sec"], 3), "unit": "env-steps/s", "cores": threads,
                "trainer_updates_per_sec": round(out["trainer_updates_per_sec"], 3),
                "sample": f"the same loop with {threads} BLAS threads, unpinned, {out['seconds']:.1f} s"}
    return {"value": round(out["env_steps_per_sec"], 3), "unit": "env-steps/s", "cores": 1, "kind": "port",
            "trainer_updates_per_sec": round(out["trainer_updates_per_sec"], 3),
            "sample": (f"oracle/train_loop.py: {scenario} N={out.get('n_agents', '?')}, 1 env, batch {args.batch_size}, "
                       f"{args.num_units}-unit MLPs, reference call structure (batch-1 action per agent, "
                       f"Python-list replay, sequential per-agent updates every 100 steps), numpy fp32 on "
                       f"1 pinned core, replay prefilled to the gate; {out['env_steps']} env steps + "
                       f"{out['updates']} updates in {out['seconds']:.1f} s")}


def configs2_per_gpu(args, steps=12, warmup=3):
    """BASELINE configs[2]'s per-GPU share on this GPU: simple_spread N=3 with
    4096 env copies, batch 1024, the same cadence (41 update rounds per vector
    step); the multi-GPU runs use this E per rank"""
    E = 4096
    # pinned to BASELINE configs[2] (simple_spread N=3, maddpg policies,
    # 64 units), whatever --scenario the main line ran
    r = VecRunner("simple_spread", E, n_agents=3, batch_size=args.batch_size, num_units=64, seed=args.seed + 1,
                  train_every=args.train_every)
    r.prefill()
    for _ in range(warmup):
        r.step()
    r.synchronize()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rounds = 0
    for _ in range(steps):
        rounds += r.step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    r.synchronize()
    finite = all(bool(np.isfinite(v).all()) for i in range(r.n) for v in r.eng.get_params(i, "critic").values())
    out = {"env_steps_per_sec": round(E * steps / dt, 3), "trainer_updates_per_sec": round(rounds * r.n / dt, 3),
           "rounds_per_sec": round(rounds / dt, 3), "ms_per_step": round(dt / steps * 1e3, 4), "steps": steps,
           "num_envs": E, "params_finite": finite,
           "note": "configs[2] per-GPU workload (4096 simple_spread copies per GPU) on 1 GPU; "
                   "the N>1 bench lines run exactly this per rank"}
    r.eng.close()
    return out


# What an N-GPU line of BASELINE configs[2] (simple_spread N=3, E = 4096 env
# copies per rank, B = 1024, H = 64) should show before any 8-GPU node ran it
# (DESIGN §5 "Expected 1 -> 8 GPU curve").  Each rank runs the single-GPU step
# (measured on one MI355X, profiles/r05u_configs/s3_spread_e4096.json: 3.5602 ms
# per step strict, 1.4274 ms throughput mode, 40.96 rounds per step, the
# rollout 26 us) plus, per round, the gradient exchanges inside the optimizer
# launches: 2N = 6 (strict) or 1 (throughput) at `exchange_us` each (every
# chunk's store to the 7 peers and the wait for theirs: peer skew + the fabric).
SCALE_MODEL = {"rollout_us": 26.0, "rounds_per_step": 40.96, "envs_per_rank": 4096, "n_agents": 3,
               "step_us": {"strict": 3560.2, "throughput": 1427.4},
               "exchanges_per_round": {"strict": 6, "throughput": 1},
               # per-exchange cost: the one-GPU 2-rank rehearsal's 1.48 us (no fabric) as the
               # floor, 3 us the central guess (+ an xGMI hop and peer skew), 5 us pessimistic
               "exchange_us": {"low": 1.5, "mid": 3.0, "high": 5.0}}


def predict_scaling(world, mode="strict", exchange_us=None):
    """predicted env-steps/s, updates/s and weak-scaling efficiency of a
    `world`-rank configs[2] line (SCALE_MODEL); exchange_us: None = the central
    guess, or a measured per-exchange cost (the line's exchange_per_rank)"""
    m = SCALE_MODEL
    c = m["exchange_us"]["mid"] if exchange_us is None else float(exchange_us)
    r1 = (m["step_us"][mode] - m["rollout_us"]) / m["rounds_per_step"]       # one round on one GPU
    rn = r1 + (m["exchanges_per_round"][mode] * c if world > 1 else 0.0)
    step = m["rollout_us"] + m["rounds_per_step"] * rn
    env = world * m["envs_per_rank"] / step * 1e6
    return {"env_steps_per_sec": round(env, 1),
            "trainer_updates_per_sec": round(m["rounds_per_step"] * m["n_agents"] / step * 1e6, 1),
            "round_us": round(rn, 2), "weak_scaling_efficiency": round(r1 / rn if world > 1 else 1.0, 4),
            "exchange_us": c if world > 1 else 0.0}


def exchange_limit_us(mode="strict", efficiency=0.8):
    """the per-exchange cost above which the exchange, not the kernels, holds
    the weak-scaling efficiency below `efficiency`"""
    m = SCALE_MODEL
    r1 = (m["step_us"][mode] - m["rollout_us"]) / m["rounds_per_step"]
    return round(r1 * (1.0 / efficiency - 1.0) / m["exchanges_per_round"][mode], 2)


def rank_launch_plan(gpus, environ, argv, port=None):
    """How `bench.py --gpus N` becomes N ranks (maddpg_amd.launch: WORLD_SIZE set
    must equal N; unset with N > 1: a torchrun child of N fresh rank processes;
    otherwise None, this process is the single rank)."""
    from maddpg_amd.launch import rank_launch_plan as plan
    return plan(gpus, environ, os.path.join(ROOT, "bench.py"), argv, port, who="bench.py")


def run_ranks(plan):
    from maddpg_amd.launch import run_ranks as run
    return run(plan, cwd=ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--scenario", default="simple_spread")
    ap.add_argument("--num-envs", type=int, default=None,
                    help="env copies per GPU (default: 1024 = configs[1] at N=1, 4096 = configs[2] at N>1)")
    ap.add_argument("--batch-size", type=int, default=1024)
    ap.add_argument("--num-units", type=int, default=64)
    ap.add_argument("--train-every", type=int, default=100)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--rollout-only", action="store_true", help="time env steps without training")
    # BASELINE configs[3]/[4]: simple_adversary with mixed maddpg/ddpg policies, simple_tag N=6
    ap.add_argument("--num-agents", type=int, default=None, help="scenario agent count override")
    ap.add_argument("--scenario-adversaries", type=int, default=None, help="adversaries in the scenario world")
    ap.add_argument("--num-adversaries", type=int, default=0, help="agents trained with --adv-policy")
    ap.add_argument("--good-policy", default="maddpg")
    ap.add_argument("--adv-policy", default="maddpg")
    ap.add_argument("--update-mode", choices=["strict", "throughput"], default="strict",
                    help="throughput: SURVEY 8e's round-parallel mode (not the reference's update order)")
    ap.add_argument("--no-throughput-figure", action="store_true",
                    help="skip the secondary throughput-mode measurement of a strict run")
    ap.add_argument("--no-configs2", action="store_true",
                    help="skip the 4096-envs-per-GPU figure (BASELINE configs[2]) of an N=1 run")
    ap.add_argument("--allow-torch-dist", action="store_true",
                    help="N>1: accept the torch.distributed fallback exchange (~14x slower per round) when "
                         "neither the direct xGMI exchange nor the library's RCCL communicator came up")
    ap.add_argument("--step-group", type=int, default=1,
                    help="timed steps replayed as graphs of this many consecutive steps (mdp_train_steps; "
                         "1: one graph per step)")
    ap.add_argument("--no-gather-stage", action="store_true",
                    help="skip the gather-only stage figure (SURVEY 8d, rank 0 at N=1)")
    ap.add_argument("--launch-check", action="store_true",
                    help="print this rank's (rank, world, local rank) as JSON and exit before any GPU call "
                         "(tests the --gpus N launch on a CPU host)")
    args = ap.parse_args()

    # --gpus N is a contract: N ranks or no line at all.  Without torchrun's
    # environment the bench launches the N rank processes itself (fresh
    # children, before this process touches the GPU) and exits with their
    # status; a WORLD_SIZE that disagrees with --gpus is an error.
    plan = rank_launch_plan(args.gpus, os.environ, sys.argv[1:])
    if plan is not None:
        sys.exit(run_ranks(plan))
    if args.launch_check:
        print(json.dumps({"rank": int(os.environ.get("RANK", "0")), "world": int(os.environ.get("WORLD_SIZE", "1")),
                          "local_rank": int(os.environ.get("LOCAL_RANK", "0")), "gpus": args.gpus}))
        return
    world, rank, local = init_process_group_from_env()
    if args.num_envs is None:   # BASELINE configs[1] on one GPU, configs[2] across GPUs
        args.num_envs = 1024 if world == 1 else 4096
    torch.cuda.set_device(local)
    r = VecRunner(args.scenario, args.num_envs, n_agents=args.num_agents,
                  scenario_adversaries=args.scenario_adversaries, num_adversaries=args.num_adversaries,
                  good_policy=args.good_policy, adv_policy=args.adv_policy, batch_size=args.batch_size,
                  num_units=args.num_units, seed=args.seed, train_every=args.train_every, world_size=world,
                  rank=rank)
    eng = r.eng
    if (world > 1 and not r.native_dp and os.environ.get("MDP_NATIVE_DP", "1") == "1"
            and not args.allow_torch_dist):
        # the native exchanges (direct xGMI, then RCCL from C++) both failed to set up:
        # a line measured on the host-driven fallback would misreport the path
        print(f"rank {rank}: data-parallel exchange fell back to {r.dp_kind} (native xGMI and RCCL "
              f"set-up failed); refusing to report it -- pass --allow-torch-dist to measure it anyway",
              file=sys.stderr)
        sys.exit(3)
    if args.update_mode != "strict":
        eng.set_update_mode(args.update_mode)
    r.prefill()
    kinds = [k for k in _lib.KERNEL]

    def one_step():
        if args.rollout_only:
            r.rollout()
            return 0
        return r.step()

    for _ in range(args.warmup):
        one_step()
    r.synchronize()

    xgmi = world > 1 and getattr(r, "dp_kind", None) == "native-xgmi"
    # the timed steps as graphs of step_group consecutive steps, captured here
    # ahead of the timed region (the same launches as step-by-step graphs; one
    # graph-launch boundary per group instead of per step)
    groups = r.prepare_steps(args.steps, args.step_group) if (args.step_group > 1 and not args.rollout_only) \
        else None
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rounds = 0
    if groups:
        for g in groups:
            rounds += r.steps(g)
    else:
        for _ in range(args.steps):
            rounds += one_step()
    torch.cuda.synchronize()
    dt_local = time.perf_counter() - t0     # this rank's own finish, before the closing barrier
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    # the run validates itself: every rank's ms/step, the communicator the
    # exchange ran over, and bit-identical replicas (strict data parallelism
    # keeps every rank's weights, targets, Adam moments and beta powers equal).
    # At N=1 the same fields describe the single replica (no communicator).
    r.synchronize()
    info = {"ms_per_step": round(dt_local / args.steps * 1e3, 4), "checksum": eng.param_checksum(),
            "rounds": rounds}
    if world > 1:
        info["dp"] = eng.dp_info() if getattr(r, "native_dp", False) else {"kind": r.dp_kind, "ranks": world}
        allinfo = [None] * world
        dist.all_gather_object(allinfo, info)
    else:
        info["dp"] = {"kind": "none", "ranks": 1, "rank": 0, "peers": 0}
        allinfo = [info]
    dp_check = {"replicas_identical": all(x["checksum"] == allinfo[0]["checksum"] for x in allinfo),
                "per_rank_ms_per_step": [x["ms_per_step"] for x in allinfo],
                "communicator": allinfo[0]["dp"],
                "peers_per_rank": [x["dp"].get("peers") for x in allinfo]}
    # second figure: rollout only (actors + Gumbel + MPE physics + replay
    # append) over the same env copies, no training
    ro_steps = max(10, args.steps)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(ro_steps):
        r.rollout()
    torch.cuda.synchronize()
    ro_dt = time.perf_counter() - t1
    if world > 1:
        t = torch.tensor([ro_dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ro_dt = float(t.item())
    rollout_only = args.num_envs * ro_steps * world / ro_dt
    ro_ms_local = ro_dt / ro_steps * 1e3
    # Kernel timing pass: the same workload again with a HIP event pair around
    # every launch of every kernel kind on the engine stream (this forces the
    # eager launch path; the timed region above replays the captured round graph).
    for k in kinds:
        eng.prof_enable(k, True)
    if xgmi:   # the exchange waits are stamped in this pass only (off in the timed graphs)
        eng.dp_exchange_stats_enable(True)
        eng.dp_exchange_stats(reset=True)
    prof_steps = max(3, args.steps // 3)
    for _ in range(prof_steps):
        one_step()
    r.synchronize()
    if xgmi:
        info["xgmi_wait"] = eng.dp_exchange_stats(reset=True)
        eng.dp_exchange_stats_enable(False)
    per_kind = {k: eng.prof_read(k) for k in kinds}
    for k in kinds:
        eng.prof_enable(k, False)
    if world > 1:
        # the first multi-GPU run diagnoses itself: per rank, what one gradient
        # exchange costs and the share of an update round spent in exchanges
        # (strict: 2N per round, one per optimizer step; throughput: one)
        ex_per_round = 1 if args.update_mode == "throughput" else 2 * r.n
        rps = info["rounds"] / args.steps if args.steps else 0.0
        round_us = ((info["ms_per_step"] - ro_ms_local) * 1e3 / rps) if rps else None
        ex = {"kind": r.dp_kind, "exchanges_per_round": ex_per_round,
              "round_us": round(round_us, 3) if round_us else None}
        if xgmi:
            w = info["xgmi_wait"]
            ex.update(source="in-kernel s_memrealtime in the eager kernel pass: chunk stores -> every "
                             "peer's chunk arrived",
                      per_exchange_us=round(w["mean_us"], 3), longest_wait_us=round(w["max_us"], 3),
                      chunk_exchanges=w["chunk_exchanges"])
        elif per_kind.get("allreduce", (0, 0))[1]:
            ms_ar, n_ar = per_kind["allreduce"]
            ex.update(source="HIP events around each ncclAllReduce (kernel pass, eager)",
                      per_exchange_us=round((ms_ar / n_ar - event_overhead_ms(eng.stream)) * 1e3, 3),
                      allreduces_timed=n_ar)
        if ex.get("per_exchange_us") is not None and round_us:
            ex["wait_us_per_round"] = round(ex["per_exchange_us"] * ex_per_round, 3)
            ex["wait_fraction_of_round"] = round(ex["wait_us_per_round"] / round_us, 4)
        exall = [None] * world
        dist.all_gather_object(exall, ex)
        dp_check["exchange_per_rank"] = exall
    prediction = None
    if (world > 1 and args.scenario == "simple_spread" and r.n == 3 and args.num_envs == 4096
            and args.batch_size == 1024 and args.num_units == 64 and args.train_every == 100
            and not args.rollout_only):
        # the curve stated before the first 8-GPU run, and the same model
        # with this run's own measured exchange cost plugged in
        meas = [e.get("per_exchange_us") for e in dp_check.get("exchange_per_rank", []) if e]
        meas = [x for x in meas if x is not None]
        prediction = {"model": "per rank: the one-GPU configs[2] step + exchanges per round x per-exchange "
                               "cost (bench.SCALE_MODEL, DESIGN §5)",
                      "central": predict_scaling(world, args.update_mode),
                      "range": [predict_scaling(world, args.update_mode, SCALE_MODEL["exchange_us"][k])
                                ["env_steps_per_sec"] for k in ("high", "low")],
                      "exchange_limits_scaling_above_us": exchange_limit_us(args.update_mode),
                      "with_measured_exchange": (predict_scaling(world, args.update_mode, max(meas))
                                                 if meas else None)}
    # the dominant kernel among those with a roofline model (the gradient launch
    # pair: MFMA; rollout, optimizer step: HBM)
    if per_kind["critic_grad"][1] and per_kind["critic_grad"][1] == per_kind["actor_grad"][1]:
        per_kind["grads"] = (per_kind["critic_grad"][0] + per_kind["actor_grad"][0], per_kind["critic_grad"][1])
    modelled = [k for k in ("grads", "rollout", "reduce_apply") if per_kind.get(k, (0, 0))[1]]
    # every kernel kind is timed on its own dispatch packet (hipExtLaunchKernel
    # start/stop events: the packet's begin -> end, what rocprofv3 reports), so
    # no marker overhead is subtracted; only the RCCL call and the multi-launch
    # gather are bracketed by marker events (MARKER_KINDS)
    dominant = max(modelled, key=lambda k: per_kind[k][0]) if modelled else None
    ms_tot, launches = per_kind[dominant] if dominant else (0.0, 0)

    # secondary figure: the same workload in throughput mode (every
    # agent's gradients from the round-start parameters, one all-reduce per
    # round) -- NOT the reference's update order, never `value`
    tp_fig = None
    if (args.update_mode == "strict" and not args.rollout_only and not args.no_throughput_figure
            and (world == 1 or getattr(r, "native_dp", False))):
        try:
            eng.set_update_mode("throughput")
        except Exception as e:  # outside the fast kernels' envelope
            tp_fig = {"skipped": str(e)[:200]}
        if tp_fig is None:
            for _ in range(args.warmup):
                one_step()
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            tp_rounds = 0
            for _ in range(args.steps):
                tp_rounds += one_step()
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            tp_dt = time.perf_counter() - t2
            if world > 1:
                t = torch.tensor([tp_dt], dtype=torch.float64, device="cuda")
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                tp_dt = float(t.item())
            eng.set_update_mode("strict")
            tp_fig = {"env_steps_per_sec": round(args.num_envs * args.steps * world / tp_dt, 3),
                      "trainer_updates_per_sec": round(tp_rounds * r.n / tp_dt, 3),
                      "rounds_per_sec": round(tp_rounds / tp_dt, 3),
                      "ms_per_step": round(tp_dt / args.steps * 1e3, 4),
                      "note": "throughput update mode (SURVEY 8e): every agent's gradients from the round-start "
                              "parameters, one optimizer launch (and one all-reduce) per round -- not the "
                              "reference's update order"}

    env_steps = args.num_envs * args.steps * world
    updates = rounds * r.n           # optimiser updates (each on world*B samples)
    value = env_steps / dt
    ev_ms = event_overhead_ms(eng.stream)
    roof = None
    if launches:
        roof = roofline_for(dominant, eng, ms_tot / launches)
        roof["dominant_of_all_kinds"] = max((k for k in per_kind if per_kind[k][1] and k != "grads"),
                                            key=lambda k: per_kind[k][0])
        roof["timing"] = ("HIP start/stop events carried on each launch's own dispatch packet "
                          "(hipExtLaunchKernel) in an eager pass of the same workload; the pair's two "
                          "launch durations summed")
        roof["launches_timed"] = launches
    lib_hash = lib_sha256()
    cfg_key = f"{args.scenario}_E{args.num_envs}_B{args.batch_size}_H{args.num_units}"
    if args.num_agents is not None:
        cfg_key += f"_N{args.num_agents}"
    if roof is not None and "kernels" in roof:
        # the pair: HBM bytes and MFMA busy cycles of both kernels, durations summed
        parts = [load_pmc(k, cfg_key) for k in roof["kernels"]]
        pmc = {}
        if all(p.get("hbm_bytes_per_launch") is not None for p in parts):
            pmc["hbm_bytes_per_launch"] = sum(p["hbm_bytes_per_launch"] for p in parts)
        if all(p.get("avg_ns") for p in parts):
            pmc["avg_ns"] = sum(p["avg_ns"] for p in parts)
            pmc["_source"] = parts[0].get("_source")
            pmc["_lib_sha256"] = parts[0].get("_lib_sha256")
            if all(p.get("mfma_busy_frac") is not None for p in parts):
                pmc["mfma_busy_frac"] = sum(p["mfma_busy_frac"] * p["avg_ns"] for p in parts) / pmc["avg_ns"]
    elif roof is not None:
        pmc = load_pmc(roof["kernel"], cfg_key)
    if roof is not None:
        roof["traffic"] = pmc.get("hbm_bytes_per_launch")
        if pmc.get("mfma_busy_frac") is not None:
            # SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x kernel cycles), profiles/<tag>_mfma.csv
            roof["mfma_busy_frac_rocprof"] = round(pmc["mfma_busy_frac"], 5)
        if pmc.get("avg_ns"):
            # the committed rocprofv3 --kernel-trace --stats average of the same kernel and
            # workload (profiles/, mostly graph-replayed launches) is the headline duration ONLY
            # when that profile measured this very library (same sha256); otherwise the live
            # packet-event figure (eager launches of the kernel pass) is the headline and the
            # stale profile is reported beside it
            live_ms = roof["avg_launch_ms"]
            prof_ms = pmc["avg_ns"] * 1e-6
            roof["rocprof_avg_launch_ms"] = round(prof_ms, 6)
            roof["rocprof_lib_sha256"] = pmc.get("_lib_sha256")
            roof["live_avg_launch_ms"] = live_ms
            roof["live_achieved"] = roof["achieved"]
            roof["live_frac"] = roof["frac"]
            roof["live_vs_rocprof_duration"] = round(live_ms / prof_ms, 4)
            if pmc.get("_lib_sha256") and pmc.get("_lib_sha256") == lib_hash:
                scale = live_ms / prof_ms
                roof["avg_launch_ms"] = prof_ms
                roof["achieved"] = round(roof["achieved"] * scale, 4)
                roof["frac"] = round(roof["frac"] * scale, 6)
                roof["duration_source"] = (f"rocprofv3 --kernel-trace --stats average ({pmc.get('_source', 'profiles')}, "
                                           f"library sha256 {lib_hash}, the one this run loaded)")
            else:
                roof["duration_source"] = (f"live packet events (the committed rocprof summary measured library "
                                           f"{pmc.get('_lib_sha256')}, this run loaded {lib_hash})")
        else:
            roof["duration_source"] = "live packet events (no committed rocprof summary for this workload)"
        if roof.get("traffic") and roof.get("algorithmic_bytes_per_launch"):
            # counted HBM bytes (2*FETCH + WRITE) over the algorithmic bytes: the re-read /
            # write-back excess of the launch (partial-gradient slabs, hand-off blocks, weights per XCD)
            roof["traffic_ratio"] = round(roof["traffic"] / roof["algorithmic_bytes_per_launch"], 3)
        if pmc.get("_source") or pmc:
            roof["pmc_source"] = "profiles/pmc_traffic.json"
    if rank == 0:
        out = {
            "lib_sha256": lib_hash,
            "metric": (f"env-steps/sec (end-to-end at the reference update cadence), {args.scenario} N={r.n}, "
                       f"batch {args.batch_size}"),
            "value": round(value, 3),
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic (random-init weights, device MPE env rollouts)",
            "config": {"workload": f"{args.scenario} N={r.n}, {args.num_envs} env copies per GPU, batch "
                                   f"{args.batch_size}, {args.num_units}-unit MLPs, 1 update round per "
                                   f"{args.train_every} transitions per rank"
                                   + (f", policies {['ddpg' if q else 'maddpg' for q in eng.local_q]}"
                                      if any(eng.local_q) else ""),
                       "scenario": args.scenario, "num_envs_per_gpu": args.num_envs,
                       "global_batch": args.batch_size * world, "parallelism": f"dp{world}",
                       "mode": "rollout-only" if args.rollout_only else args.update_mode,
                       "step_graph_group": args.step_group if groups else 1},
            "trainer_updates_per_sec": round(updates / dt, 3),
            "rounds_per_sec": round(rounds / dt, 3),
            "rollout_only_env_steps_per_sec": round(rollout_only, 3),
            "update_rounds": rounds,
            "dp": r.dp_kind if world > 1 else None,
            "dp_check": dp_check,
            "kernel_pass": {"steps": prof_steps, "marker_pair_overhead_ms": round(ev_ms, 5),
                            "timing": "dispatch-packet events per launch; marker pairs (their overhead "
                                      "subtracted) only for " + ", ".join(MARKER_KINDS),
                            "per_kind_ms_per_launch": {k: round(v[0] / v[1] - (ev_ms if k in MARKER_KINDS else 0.0),
                                                                5) for k, v in per_kind.items()
                                                       if v[1] and k != "grads"},
                            "per_kind_launches": {k: v[1] for k, v in per_kind.items() if k != "grads"}},
            "roofline": roof,
            "throughput_mode": tp_fig,
        }
        if prediction is not None:
            out["predicted_value"] = prediction["central"]["env_steps_per_sec"]
            out["prediction"] = prediction
        if (world == 1 and not args.no_configs2 and
                not (args.scenario == "simple_spread" and r.n == 3 and args.num_envs == 4096)):
            out["configs2_per_gpu"] = configs2_per_gpu(args)
        if world == 1 and not args.no_gather_stage:
            out["gather_stage"] = gather_stage(r.spec.obs_dims)
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args)
            # also the host's cores (the box's CPU share, at most 16)
            out["cpu_baseline"]["all_cores"] = cpu_baseline(args, threads=min(16, os.cpu_count() or 1),
                                                            seconds=max(5.0, args.cpu_seconds / 2))
            # BASELINE configs[0], the designated CPU config: scenario simple (1 agent), 1 env,
            # batch 1024, 64-unit MLPs -- 1 pinned core and the host's cores
            simple = cpu_baseline(args, seconds=max(5.0, args.cpu_seconds / 2), scenario="simple")
            simple["all_cores"] = cpu_baseline(args, threads=min(16, os.cpu_count() or 1),
                                               seconds=max(5.0, args.cpu_seconds / 3), scenario="simple")
            out["cpu_baseline"]["configs0_simple"] = simple
        print(json.dumps(out))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
