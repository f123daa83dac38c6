"""Learning curve of the device training loop (GPU box):

    python tools/learning_curve.py --scenario simple --num-envs 1024 --episodes 60

Runs VecRunner (the train.py loop: rollout + the reference's update cadence,
strict order) and prints one JSON line: the mean total episode reward of
every batch of E lockstep episodes (train.py:141's episode_rewards, averaged
over the E env copies), so a curve that rises from the random policy's level
shows the path learns, not just that it matches the oracle step by step.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def curve(scenario, num_envs, episodes, seed=0, num_agents=None, scenario_adversaries=None,
          num_adversaries=0, max_episode_len=25, batch_size=1024, num_units=64, update_mode="strict",
          adv_policy="maddpg"):
    from maddpg_amd.runner import VecRunner
    r = VecRunner(scenario, num_envs, n_agents=num_agents, scenario_adversaries=scenario_adversaries,
                  num_adversaries=num_adversaries, adv_policy=adv_policy, batch_size=batch_size, num_units=num_units, seed=seed,
                  max_episode_len=max_episode_len, episode_log_rows=4 * num_envs)
    if update_mode != "strict":
        r.eng.set_update_mode(update_mode)
    out, agents, rounds, t0 = [], [], 0, time.time()
    for _ in range(episodes):
        for _ in range(max_episode_len):
            rounds += r.step()
        r.synchronize()
        n = r.episodes()
        rew = r.episode_rewards(n - num_envs, num_envs)
        out.append(float(rew[:, 0].mean()))
        agents.append([round(float(v), 3) for v in rew[:, 1:].mean(0)])
        print(f"{len(out)} {out[-1]:.3f} rounds {rounds}", file=sys.stderr, flush=True)
    return {"scenario": scenario, "update_mode": update_mode, "seed": seed, "num_envs": num_envs, "episodes_per_point": num_envs,
            "points": len(out), "transitions": episodes * max_episode_len * num_envs, "update_rounds": rounds,
            "seconds": round(time.time() - t0, 2), "mean_episode_reward": [round(v, 3) for v in out],
            "mean_agent_reward": agents}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scenario", default="simple")
    ap.add_argument("--num-envs", type=int, default=1024)
    ap.add_argument("--episodes", type=int, default=60, help="lockstep episode batches (each num_envs episodes)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--num-agents", type=int, default=None)
    ap.add_argument("--scenario-adversaries", type=int, default=None)
    ap.add_argument("--num-adversaries", type=int, default=0)
    ap.add_argument("--adv-policy", default="maddpg")
    ap.add_argument("--num-units", type=int, default=64)
    ap.add_argument("--batch-size", type=int, default=1024)
    ap.add_argument("--update-mode", choices=["strict", "throughput"], default="strict")
    a = ap.parse_args()
    print(json.dumps(curve(a.scenario, a.num_envs, a.episodes, a.seed, a.num_agents, a.scenario_adversaries,
                           a.num_adversaries, batch_size=a.batch_size, num_units=a.num_units,
                           update_mode=a.update_mode, adv_policy=a.adv_policy)), flush=True)


if __name__ == "__main__":
    main()
