"""Native data parallelism at world size 2 and 8 on one GPU (the exchange
order of maddpg.py:188-194 / train.py:160-161).

The library's native path opens RCCL itself (mdp_dp_init) and issues the
all-reduces from C++.  RCCL refuses two ranks on one device, so here the
library loads an in-tree stand-in communicator instead (MDP_RCCL_LIB ->
tests/rccl_standin/libnccl_standin.so): a world of G = 2 whose peers hold this
rank's data, i.e. ncclAllReduce(sum) = an in-place x2, each call logged.  Every
case runs in a child process (tests/standin_child.py), because the library
binds its RCCL once per process.  Checked:
  * strict mode: exactly 2N all-reduces per round, each over exactly that
    phase's gradient span (critic, then actor, agent by agent), in place, sum
    over fp32 on the 2-rank communicator; the 1/G scale makes the step equal
    the single-GPU two-kernel step bit for bit; critic loss and parameters
    against the CPU oracle (oracle/trainer.py) within the update-parity
    tolerances, over two rounds;
  * throughput mode: ONE all-reduce per round over the whole gradient region,
    vs oracle.trainer.update_round_throughput and the single-GPU round;
  * the training loop (mdp_train_step) with the collectives issued eagerly and
    captured in the step graph (MDP_DP_GRAPHS=1): bit-identical to one GPU.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STANDIN = os.path.join(ROOT, "tests", "rccl_standin", "libnccl_standin.so")

pytestmark = pytest.mark.gpu


def _child(mode, **env):
    if not os.path.exists(STANDIN):
        pytest.fail(f"{STANDIN} missing: build it with make -C maddpg_amd/csrc")
    e = dict(os.environ, MDP_RCCL_LIB=STANDIN, **env)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "standin_child.py"), mode], env=e, cwd=ROOT,
                       capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    print(mode, env, json.dumps(out))
    return out


@pytest.mark.parametrize("G", [2, 8])
def test_standin_strict_two_allreduces_per_agent_vs_oracle(G):
    out = _child("strict", MDP_UNFUSED_APPLY="1", MDP_STANDIN_G=str(G))
    assert out["dp_info"] == {"kind": "rccl", "ranks": G, "rank": 0, "peers": G - 1}
    for r in out["rounds"]:
        assert r["allreduces"] == 2 * 3                 # 2N per round
        assert r["spans_match"] and r["in_place"] and r["sum_fp32"]
        assert r["nranks"] == [G]
        assert r["dp_vs_single_max_diff"] == 0.0        # (G g) x 1/G == g exactly (G a power of two)
        assert r["stats_equal"]
        assert r["loss_rel_err"] <= 1e-5
        assert r["param_abs_err"] < 2e-4


@pytest.mark.parametrize("G,general", [(2, "0"), (8, "0"), (2, "1")])
def test_standin_throughput_one_allreduce_per_round_vs_oracle(G, general):
    # general = "1": the general kernels' round (per-agent gradient pairs and
    # reduce-only optimizer pairs, then the one all-reduce and the step pass)
    # against the single-GPU general round (optimizer pairs + k_polyak)
    out = _child("throughput", MDP_STANDIN_G=str(G), MDP_GENERAL_GRADS=general)
    assert out["allreduces"] == 1
    assert out["recv_is_grad_base"] and out["covers_every_net"]
    assert out["nranks"] == [G]
    assert out["dp_vs_single_max_diff"] == 0.0
    assert out["loss_rel_err"] <= 1e-5
    assert out["param_abs_err"] < 2e-4
    # k rounds advance the update counter by n k on both paths (the
    # general kernels' pair lists bump it once per round, in the step pass)
    assert out["upd_ctr"] == [out["n"] * out["rounds"]] * 2
    assert out["dp_vs_single_after"] == 0.0


@pytest.mark.parametrize("graphs,G", [("0", 2), ("1", 2), ("1", 8)])
def test_standin_train_step_matches_single_gpu(graphs, G):
    out = _child("graph", MDP_UNFUSED_APPLY="1", MDP_DP_GRAPHS=graphs, MDP_STANDIN_G=str(G))
    assert out["rounds"] == 12
    assert out["dp_vs_single_max_diff"] == 0.0 and out["beta_equal"]
    if graphs == "0":
        assert out["allreduces"] == 2 * 3 * out["rounds"] and out["captured"] == 0
    else:   # captured once per round count, replayed afterwards
        assert 0 < out["allreduces"] <= 2 * 3 * out["rounds"] and out["captured"] > 0
