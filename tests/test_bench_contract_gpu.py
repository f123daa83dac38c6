"""The bench.py output contract the driver reads (one JSON line on rank 0), and
__graft_entry__.smoke(), on a short run."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

pytestmark = pytest.mark.gpu


def test_bench_json_line():
    r = subprocess.run([sys.executable, "bench.py", "--steps", "3", "--warmup", "1", "--cpu-seconds", "1",
                        "--no-throughput-figure"], cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["warmup"] == 1
    assert d["value"] > 0 and d["higher_is_better"] is True and d["scaling"] == "weak"
    assert "workload" in d["config"]
    roof = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in roof, k
    assert roof["bound"] in ("hbm", "mfma") and 0 < roof["frac"] < 1
    assert abs(roof["frac"] - roof["achieved"] / roof["peak"]) < 1e-3
    cb = d["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in cb, k
    assert cb["kind"] == "port" and cb["cores"] == 1 and cb["value"] > 0


def test_smoke():
    import __graft_entry__
    __graft_entry__.smoke()


def test_bench_two_ranks_driver_command_shape():
    """The driver's N>1 command (torchrun, one rank per GPU, `--gpus N`) on this
    one-GPU box: both ranks on cuda:0 (MDP_SHARED_GPU=1, a gloo group -- RCCL
    refuses two ranks on one device), the real xGMI exchange between them.  One
    JSON line from rank 0 with the whole-job value, and replicas bit-identical."""
    import random
    env = dict(os.environ, MDP_SHARED_GPU="1", MDP_DP_XGMI="1")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(29400 + random.randrange(400)),
           "bench.py", "--gpus", "2", "--steps", "3", "--warmup", "1", "--no-throughput-figure"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "weak" and d["value"] > 0
    dp = d["dp_check"]
    assert dp["replicas_identical"] is True
    assert dp["peers_per_rank"] == [1, 1]
    # the default N > 1 workload (configs[2]: 4,096 env copies per rank) carries the
    # expected curve of DESIGN §5 and the model with this run's exchange cost
    assert d["config"]["num_envs_per_gpu"] == 4096
    assert d["predicted_value"] == d["prediction"]["central"]["env_steps_per_sec"] > 0
    lo, hi = sorted(d["prediction"]["range"])
    assert lo < d["predicted_value"] < hi
    assert d["prediction"]["exchange_limits_scaling_above_us"] > 0
    assert d["prediction"]["with_measured_exchange"] is not None
