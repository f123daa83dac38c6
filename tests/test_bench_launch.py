"""`bench.py --gpus N` is N ranks or no line (CPU tests of the launch contract).

The driver runs the multi-GPU series as `torchrun --nproc-per-node N bench.py
--gpus N`; a bare `python bench.py --gpus N` (no WORLD_SIZE) must not measure
and report a one-GPU world under n_gpus = N.  bench.rank_launch_plan decides:
torchrun's environment present -> it must agree with --gpus; absent with N > 1
-> start the N rank processes as a child torchrun (fresh processes, before any
GPU call in this one).  `--launch-check` makes every rank report its
(rank, world) and exit before touching the GPU, so the real launch runs here.
"""
import json
import os
import subprocess
import sys

import pytest

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_plan_single_gpu_runs_in_process():
    assert bench.rank_launch_plan(1, {}, []) is None


@pytest.mark.parametrize("n", [2, 4, 8])
def test_plan_without_world_size_launches_n_ranks(n):
    plan = bench.rank_launch_plan(n, {}, ["--gpus", str(n), "--steps", "7"])
    assert plan[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert f"--nproc-per-node={n}" in plan and "--nnodes=1" in plan
    # torchrun's rendezvous store picks its own port (no probe-then-bind race)
    assert "--rdzv-backend=c10d" in plan and "--rdzv-endpoint=127.0.0.1:0" in plan
    assert plan[plan.index("--local-addr") + 1] == "127.0.0.1"
    assert "--rdzv-endpoint=127.0.0.1:29555" in bench.rank_launch_plan(n, {}, [], port=29555)
    assert plan[-4:] == ["--gpus", str(n), "--steps", "7"]
    assert os.path.basename(plan[-5]) == "bench.py"


def test_plan_under_torchrun_runs_in_process():
    assert bench.rank_launch_plan(8, {"WORLD_SIZE": "8", "RANK": "3"}, []) is None


@pytest.mark.parametrize("gpus,ws", [(8, "1"), (8, "4"), (2, "8"), (1, "2")])
def test_plan_world_size_mismatch_exits_nonzero(gpus, ws):
    with pytest.raises(SystemExit) as e:
        bench.rank_launch_plan(gpus, {"WORLD_SIZE": ws}, [])
    assert e.value.code not in (0, None)


def _run(args, **env):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    e.update(env)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT, env=e,
                          capture_output=True, text=True, timeout=240)


def test_bare_gpus_2_starts_two_ranks():
    """the real launch path on the CPU: python bench.py --gpus 2 -> torchrun child -> 2 ranks"""
    r = _run(["--gpus", "2", "--launch-check"])
    assert r.returncode == 0, r.stderr[-2000:]
    got = sorted((d["rank"], d["world"], d["local_rank"], d["gpus"])
                 for d in (json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")))
    assert got == [(0, 2, 0, 2), (1, 2, 1, 2)]


def test_world_size_disagreeing_with_gpus_fails():
    r = _run(["--gpus", "8", "--launch-check"], WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    assert r.returncode == 2
    assert "refusing" in r.stderr and not r.stdout.strip()


def test_scaling_prediction_model():
    """DESIGN §5's expected 1 -> 8 GPU curve (bench.predict_scaling): N = 1
    reproduces the measured one-GPU configs[2] figure, every N > 1 rank pays its
    exchanges per round, more exchange cost never predicts more, and the stated
    limit is where the efficiency crosses 80 %."""
    for mode, one in (("strict", 1150497.68), ("throughput", 2869503.58)):   # profiles/r05u_configs/s3
        p1 = bench.predict_scaling(1, mode)
        assert abs(p1["env_steps_per_sec"] / one - 1) < 1e-3 and p1["weak_scaling_efficiency"] == 1.0
        prev = None
        for n in (2, 4, 8):
            lo, mid, hi = (bench.predict_scaling(n, mode, bench.SCALE_MODEL["exchange_us"][k])
                           for k in ("low", "mid", "high"))
            assert lo["env_steps_per_sec"] > mid["env_steps_per_sec"] > hi["env_steps_per_sec"]
            assert mid["env_steps_per_sec"] < n * p1["env_steps_per_sec"]
            if prev:
                assert abs(mid["env_steps_per_sec"] / prev - n / (n // 2)) < 1e-6   # weak scaling past N = 2
            prev = mid["env_steps_per_sec"]
        lim = bench.exchange_limit_us(mode)
        assert abs(bench.predict_scaling(8, mode, lim)["weak_scaling_efficiency"] - 0.8) < 1e-3


# experiments/train.py --num-gpus N: the same launcher (maddpg_amd.launch)
def _train(args, **env):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    e.update(env)
    return subprocess.run([sys.executable, os.path.join(ROOT, "experiments", "train.py")] + args, cwd=ROOT,
                          env=e, capture_output=True, text=True, timeout=120)


def test_train_num_gpus_plan():
    from maddpg_amd.launch import rank_launch_plan
    script = os.path.join(ROOT, "experiments", "train.py")
    plan = rank_launch_plan(4, {}, script, ["--num-gpus", "4", "--num-envs", "64"], who="train.py")
    assert plan[:3] == [sys.executable, "-m", "torch.distributed.run"] and "--nproc-per-node=4" in plan
    assert plan[-5:] == [script, "--num-gpus", "4", "--num-envs", "64"]
    assert rank_launch_plan(4, {"WORLD_SIZE": "4"}, script, []) is None
    assert rank_launch_plan(1, {}, script, []) is None
    with pytest.raises(SystemExit):
        rank_launch_plan(0, {}, script, [])


def test_train_num_gpus_disagreeing_with_torchrun_fails():
    """under torchrun, --num-gpus must equal WORLD_SIZE: exit 2 before any import of torch"""
    r = _train(["--num-gpus", "8"], WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    assert r.returncode == 2 and "refusing" in r.stderr and "train.py" in r.stderr
    assert not r.stdout.strip()
