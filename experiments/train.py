"""MADDPG training on MI355X -- drop-in for the reference's ``experiments/train.py``.

Same flags, defaults and console lines as ``experiments/train.py:11-189``.
The loop runs on the device (``maddpg_amd.runner.VecRunner``): E copies of the
MPE scenario step per launch, experience goes straight into the device
replay, and every agent's ``update()`` runs in the reference's order at the
reference cadence (one round per 100 transitions; with E=1 -- the default --
this is exactly the reference loop).  Extra flags: ``--num-envs``, ``--seed``,
``--num-agents``/``--scenario-adversaries`` (scenario size), ``--train-every``.

Episode accounting follows the reference exactly: ``len(episode_rewards)`` is
the number of finished episodes + 1 (a new 0 entry is appended at every reset,
``train.py:127-133``), the progress line is printed when that length is a
multiple of ``--save-rate`` and averages the last ``--save-rate`` entries
(including the fresh 0), and training stops once it exceeds
``--num-episodes``.  Every env copy terminates at ``--max-episode-len`` steps
(MPE scenarios have no done callback), so the episode count is known on the
host without a device sync.

    python experiments/train.py --scenario simple_spread --num-envs 1024 --exp-name spread
    python experiments/train.py --scenario simple_spread --num-envs 4096 --num-gpus 8
    torchrun --nproc-per-node 8 experiments/train.py --scenario simple_spread --num-envs 4096
"""
import argparse
import os
import pickle
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def parse_args(argv=None):
    parser = argparse.ArgumentParser("Reinforcement Learning experiments for multiagent environments")
    # Environment
    parser.add_argument("--scenario", type=str, default="simple", help="name of the scenario script")
    parser.add_argument("--max-episode-len", type=int, default=25, help="maximum episode length")
    parser.add_argument("--num-episodes", type=int, default=60000, help="number of episodes")
    parser.add_argument("--num-adversaries", type=int, default=0, help="number of adversaries")
    parser.add_argument("--good-policy", type=str, default="maddpg", help="policy for good agents")
    parser.add_argument("--adv-policy", type=str, default="maddpg", help="policy of adversaries")
    # Core training parameters
    parser.add_argument("--lr", type=float, default=1e-2, help="learning rate for Adam optimizer")
    parser.add_argument("--gamma", type=float, default=0.95, help="discount factor")
    parser.add_argument("--batch-size", type=int, default=1024, help="number of episodes to optimize at the same time")
    parser.add_argument("--num-units", type=int, default=64, help="number of units in the mlp")
    # Checkpointing
    parser.add_argument("--exp-name", type=str, default=None, help="name of the experiment")
    parser.add_argument("--save-dir", type=str, default="/tmp/policy/", help="directory in which training state and model should be saved")
    parser.add_argument("--save-rate", type=int, default=1000, help="save model once every time this many episodes are completed")
    parser.add_argument("--load-dir", type=str, default="", help="directory in which training state and model are loaded")
    # Evaluation
    parser.add_argument("--restore", action="store_true", default=False)
    parser.add_argument("--display", action="store_true", default=False)
    parser.add_argument("--benchmark", action="store_true", default=False)
    parser.add_argument("--benchmark-iters", type=int, default=100000, help="number of iterations run for benchmarking")
    parser.add_argument("--benchmark-dir", type=str, default="./benchmark_files/", help="directory where benchmark data is saved")
    parser.add_argument("--plots-dir", type=str, default="./learning_curves/", help="directory where plot data is saved")
    # MI355X build extensions
    parser.add_argument("--num-envs", type=int, default=1, help="env copies stepped together per GPU")
    parser.add_argument("--seed", type=int, default=0, help="seed of weights, index stream and device RNG")
    parser.add_argument("--num-agents", type=int, default=None, help="scenario agent count override")
    parser.add_argument("--scenario-adversaries", type=int, default=None, help="adversaries in the scenario world")
    parser.add_argument("--train-every", type=int, default=100, help="transitions per update round (maddpg.py:164)")
    parser.add_argument("--display-frames", type=int, default=100,
                        help="--display: steps rendered to PNG frames (no window on a GPU box)")
    parser.add_argument("--save-format", choices=["npz", "tf1"], default="npz",
                        help="checkpoint format: npz, or tf1 (a tf.train.Saver checkpoint with the reference's "
                             "variable names; --load-dir reads either)")
    # the reference's hard-coded constants, as flags with its values
    parser.add_argument("--tau", type=float, default=1e-2, help="Polyak rate of the target nets (maddpg.py:21)")
    parser.add_argument("--grad-clip", type=float, default=0.5, help="per-tensor clip_by_norm (maddpg.py:130,142)")
    parser.add_argument("--actor-reg", type=float, default=1e-3, help="actor logits regulariser (maddpg.py:56)")
    parser.add_argument("--buffer-size", type=int, default=int(1e6), help="replay capacity (maddpg.py:147)")
    parser.add_argument("--check-nan", action="store_true", default=False,
                        help="debug: after every training step check every parameter, Adam slot and update stat "
                             "for NaN / Inf and stop with 'Nan detected' (the reference's _Function(check_nan), "
                             "tf_util.py:322,366-368)")
    parser.add_argument("--num-gpus", type=int, default=None,
                        help="start one rank per GPU from this command (torchrun child, 127.0.0.1 rendezvous); "
                             "under torchrun it must equal WORLD_SIZE (default: torchrun's world, else 1)")
    parser.add_argument("--update-mode", choices=["strict", "throughput"], default="strict",
                        help="strict: the reference's update order; throughput: every agent's gradients from "
                             "the round-start parameters, then every optimizer step (SURVEY 8e, single GPU)")
    return parser.parse_args(argv)


class LearningCurve:
    """The reference's episode bookkeeping (train.py:123-133, 164-189) for E env
    copies that terminate together.

    ``len(episode_rewards)`` is finished episodes + 1 (a fresh 0 entry is
    appended at every reset).  The reference, whose episodes end one at a
    time, checks ``len % save_rate == 0`` after each reset and stops once the
    length exceeds ``num_episodes``; E simultaneous terminations step the
    length by E, so every multiple of ``save_rate`` crossed -- up to the
    length the reference stops at, num_episodes + 1 -- gives one print and one
    curve point, each the mean of the last ``save_rate`` entries at that length
    (save_rate - 1 finished episodes, in env order, plus the fresh 0).
    ``read(first, count)`` returns finished episodes [first, first + count) as
    [count, 1 + n] rows (total, per agent).
    """

    def __init__(self, save_rate, num_episodes, n):
        self.save_rate, self.num_episodes, self.n = save_rate, num_episodes, n
        self.finished = 0
        self.final_ep_rewards, self.final_ep_ag_rewards = [], []

    @property
    def length(self):
        return self.finished + 1

    @property
    def done(self):
        return self.length > self.num_episodes

    def finish(self, count, read):
        """`count` episodes ended; returns [(length, mean reward, per-agent means)]
        for every save_rate multiple crossed (read=None: count only, no points)."""
        before = self.length
        self.finished += count
        last = min(self.length, self.num_episodes + 1)
        sr = self.save_rate
        marks = list(range((before // sr + 1) * sr, last + 1, sr))
        if not marks or read is None:
            return []
        lo = marks[0] - sr                       # first finished episode any window needs
        span = marks[-1] - 1 - lo
        log = read(lo, span) if span > 0 else np.zeros((0, 1 + self.n), np.float32)
        out = []
        for mk in marks:
            w = log[mk - sr - lo: mk - 1 - lo]   # episodes [mk - sr, mk - 1) + the fresh 0
            mean_ep = float(np.sum(w[:, 0], dtype=np.float64) / sr)
            mean_ag = [float(np.sum(w[:, 1 + j], dtype=np.float64) / sr) for j in range(self.n)]
            self.final_ep_rewards.append(mean_ep)
            self.final_ep_ag_rewards.extend(mean_ag)
            out.append((mk, mean_ep, mean_ag))
        return out


def benchmark(arglist, runner, exp_name, rank):
    """--benchmark (train.py:139-148): run the loaded policies, record every
    agent's scenario benchmark_data() each step, no training.  The reference
    keeps ``agent_info`` = one entry per episode, each ``[[info_n['n'] per
    step]]``; a reset appends the new entry BEFORE the step's info is stored,
    so an episode's terminal-step record opens the next entry, and the dump
    (once train_step > --benchmark-iters at a terminal step) drops the last
    entry.  With E env copies every copy keeps its own episode stream; the
    pickle lists episodes in (episode, env copy) order.  E=1 is the reference
    structure exactly."""
    from maddpg_amd.envs import bench_record
    eng, sp, n = runner.eng, runner.spec, runner.n
    E, L = arglist.num_envs, arglist.max_episode_len
    if sp.name == "simple":
        raise AttributeError("'Scenario' object has no attribute 'benchmark_data' (scenario simple)")
    open_eps = [[[]] for _ in range(E)]
    closed = []
    train_step = 0
    vec_steps = 0
    while True:
        info = eng.env_step_bench().cpu().numpy()        # [E, n, BENCH_W]
        vec_steps += 1
        train_step += E
        terminal = vec_steps % L == 0
        if terminal:
            closed.extend(open_eps)
            open_eps = [[[]] for _ in range(E)]
        for e in range(E):
            open_eps[e][0].append([bench_record(sp, info[e, i], i) for i in range(n)])
        if train_step > arglist.benchmark_iters and terminal:
            if rank == 0:
                file_name = arglist.benchmark_dir + exp_name + '.pkl'
                print('Finished benchmarking, now saving...', flush=True)
                os.makedirs(os.path.dirname(file_name) or ".", exist_ok=True)
                with open(file_name, 'wb') as fp:
                    pickle.dump(closed, fp)
            break
    runner.synchronize()
    return runner


def display(arglist, runner, exp_name, rank):
    """--display (train.py:150-154): the loaded policies act, nothing trains,
    every step is rendered.  Headless: env copy 0 is rasterised to
    <plots-dir><exp-name>_display/frame_NNNNN.png (+ positions.npz) for
    --display-frames steps (the reference loops until interrupted)."""
    from maddpg_amd.render import FrameWriter
    out = FrameWriter(os.path.join(arglist.plots_dir, exp_name + "_display"), runner.spec)
    for _ in range(arglist.display_frames):
        runner.rollout()                                   # action_n, env.step, reset at terminal
        if rank == 0:
            st = runner.eng.env_state()
            out.add(st["pos"][0], st["goal"][0])
    if rank == 0:
        print(f"Rendered {out.close()} frames to {out.dir}", flush=True)
    runner.synchronize()
    return runner


def train(arglist):
    import torch

    from maddpg_amd.parallel import init_process_group_from_env
    from maddpg_amd.runner import VecRunner

    exp_name = arglist.exp_name if arglist.exp_name is not None else arglist.scenario
    world, rank, local = init_process_group_from_env()
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
    runner = VecRunner(arglist.scenario, arglist.num_envs, n_agents=arglist.num_agents,
                       scenario_adversaries=arglist.scenario_adversaries,
                       num_adversaries=arglist.num_adversaries, good_policy=arglist.good_policy,
                       adv_policy=arglist.adv_policy, batch_size=arglist.batch_size,
                       num_units=arglist.num_units, lr=arglist.lr, gamma=arglist.gamma,
                       max_episode_len=arglist.max_episode_len, seed=arglist.seed,
                       train_every=arglist.train_every, world_size=world, rank=rank,
                       tau=arglist.tau, grad_clip=arglist.grad_clip, actor_reg=arglist.actor_reg,
                       capacity=arglist.buffer_size,
                       # the learning-curve windows of one terminal step span <= save_rate + E episodes
                       episode_log_rows=max(4096, 4 * arglist.num_envs, arglist.save_rate + 2 * arglist.num_envs))
    if arglist.update_mode != "strict":
        runner.eng.set_update_mode(arglist.update_mode)
    n = runner.n
    num_adversaries = min(n, arglist.num_adversaries)
    say = (lambda *a: print(*a, flush=True)) if rank == 0 else (lambda *a: None)
    say('Using good policy {} and adv policy {}'.format(arglist.good_policy, arglist.adv_policy))

    if arglist.load_dir == "":
        arglist.load_dir = arglist.save_dir
    if arglist.restore or arglist.benchmark or arglist.display:   # train.py:92-96
        say('Loading previous state...')
        runner.eng.load_state(arglist.load_dir)
    if arglist.benchmark:
        return benchmark(arglist, runner, exp_name, rank)
    if arglist.display:
        return display(arglist, runner, exp_name, rank)

    E, L = arglist.num_envs, arglist.max_episode_len
    curve = LearningCurve(arglist.save_rate, arglist.num_episodes, n)
    t_start = time.time()
    t_run = time.perf_counter()
    vec_steps = 0
    say('Starting iterations...')
    from maddpg_amd.common.tf_util import check_nan
    # one episode of every env copy (L vector steps, the steps without a round
    # included) as one graph replay; --check-nan looks after every step
    group = L if (L <= 64 and not arglist.check_nan) else 1
    while True:
        if group > 1:
            runner.steps(group)
            vec_steps += group
        else:
            if runner.step() and arglist.check_nan:
                check_nan(runner.eng)
            vec_steps += 1
            if vec_steps % L:
                continue
        # every env copy just terminated (train.py:116,127): E new episodes
        steps = vec_steps * E
        points = curve.finish(E, runner.episode_rewards if rank == 0 else None)
        if points and rank == 0:
            runner.eng.save_state(arglist.save_dir, arglist.save_format)
        for length, mean_ep, mean_ag in points:
            if rank != 0:
                break
            if num_adversaries == 0:
                print("steps: {}, episodes: {}, mean episode reward: {}, time: {}".format(
                    steps, length, mean_ep, round(time.time() - t_start, 3)), flush=True)
            else:
                print("steps: {}, episodes: {}, mean episode reward: {}, agent episode reward: {}, time: {}".format(
                    steps, length, mean_ep, mean_ag, round(time.time() - t_start, 3)), flush=True)
            t_start = time.time()
        if curve.done:
            if rank == 0:
                os.makedirs(arglist.plots_dir, exist_ok=True)
                with open(arglist.plots_dir + exp_name + '_rewards.pkl', 'wb') as fp:
                    pickle.dump(curve.final_ep_rewards, fp)
                with open(arglist.plots_dir + exp_name + '_agrewards.pkl', 'wb') as fp:
                    pickle.dump(curve.final_ep_ag_rewards, fp)
            say('...Finished total of {} episodes.'.format(curve.length))
            break
    runner.synchronize()
    # SURVEY 5's counters beside the reference's prints: env-steps/s (transitions
    # of every env copy on every rank) and trainer-updates/s over the whole run
    el = time.perf_counter() - t_run
    runner.throughput = {"env_steps_per_sec": vec_steps * E * world / el,
                         "trainer_updates_per_sec": runner.rounds * n / el, "seconds": el}
    say('throughput: {:.1f} env-steps/s, {:.1f} trainer-updates/s over {:.2f} s'.format(
        runner.throughput["env_steps_per_sec"], runner.throughput["trainer_updates_per_sec"], el))
    return runner


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    arglist = parse_args(argv)
    if arglist.num_gpus is not None:
        from maddpg_amd.launch import rank_launch_plan, run_ranks
        plan = rank_launch_plan(arglist.num_gpus, os.environ, os.path.abspath(__file__), argv,
                                who="train.py")
        if plan is not None:          # N > 1 without torchrun: N rank processes, this one only waits
            return run_ranks(plan)
    train(arglist)
    return 0


if __name__ == '__main__':
    sys.exit(main())
