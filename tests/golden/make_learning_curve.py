"""Learning-curve fixture of the reference's call structure (TEST ONLY).

Runs oracle/train_loop.py -- experiments/train.py:110-161 restated call for
call on one env copy (batch-1 action() per agent, Python-list replay, one
update round per 100 transitions, numpy fp32 trainer, fp64 MPE) -- from an
empty replay (no synthetic prefill, so training starts when the gate
B * 25 opens after 1,024 real episodes, as on the device) and writes the mean
total episode reward of every 1,024 consecutive episodes:

    OMP_NUM_THREADS=4 python tests/golden/make_learning_curve.py simple 5 0
    OMP_NUM_THREADS=4 python tests/golden/make_learning_curve.py simple_spread 12 0
    OMP_NUM_THREADS=4 python tests/golden/make_learning_curve.py simple_adversary 16 0 ddpg

-> tests/golden/learning_<scenario>[_<adv policy>]_s<seed>.json (an adversary
policy argument trains the scenario's adversaries with it: train.py's
--num-adversaries = the scenario's, --adv-policy ddpg).  tests/test_learning_gpu.py
compares the device loop's curve (1,024 env copies in lockstep, the same
transitions per update round) with it batch by batch.  Different RNG streams
(numpy here, Philox on the device), so the comparison is statistical.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import train_loop  # noqa: E402


def main():
    scenario, batches, seed = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    adv_policy = sys.argv[4] if len(sys.argv) > 4 else None
    sc = train_loop.make_scenario(scenario)
    n_adv = sum(getattr(sc, "adversary", [])) if adv_policy else 0
    local_q = [adv_policy == "ddpg" and i < n_adv for i in range(sc.n_agents)]
    per = 1024
    t0 = time.time()
    r = train_loop.run(scenario, seconds=1e12, prefill=0, max_steps=25 * per * batches, seed=seed,
                       local_q=local_q)
    e = r["episode_rewards"]                      # [episodes][1 + n]: total, then per agent
    pts = [[sum(x[k] for x in e[i:i + per]) / per for k in range(1 + sc.n_agents)]
           for i in range(0, len(e) - per + 1, per)]
    curve = [p[0] for p in pts]
    out = {"generator": "tests/golden/make_learning_curve.py (oracle/train_loop.py, one env copy)",
           "scenario": scenario, "adv_policy": adv_policy, "local_q": local_q, "seed": seed,
           "episodes_per_point": per, "points": len(curve),
           "update_rounds": r["updates"] // r["n_agents"], "seconds": round(time.time() - t0, 1),
           "mean_episode_reward": [round(v, 3) for v in curve],
           "mean_agent_reward": [[round(v, 3) for v in p[1:]] for p in pts]}
    tag = f"{scenario}_{adv_policy}" if adv_policy else scenario
    path = os.path.join(ROOT, "tests", "golden", f"learning_{tag}_s{seed}.json")
    with open(path, "w") as f:
        json.dump(out, f)
        f.write("\n")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
