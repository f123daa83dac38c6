"""One process per GPU from a single command (no torch import: this runs before
anything touches the GPU).

`bench.py --gpus N` and `experiments/train.py --num-gpus N` started without
torchrun's environment start their N rank processes themselves: a torchrun
child in its own process group, launched before this process makes any GPU
call, whose exit status the launcher returns.  Under torchrun (WORLD_SIZE set)
the count must agree with the environment.
"""
import os
import signal
import subprocess
import sys


def rank_launch_plan(gpus, environ, script, argv, port=None, who=None):
    """How `<script> --gpus/--num-gpus N` becomes N ranks (pure host logic).

    * WORLD_SIZE set (torchrun / a driver's launch): it must equal N, else
      SystemExit(2) -- a run on another world size would be reported under
      the wrong N;
    * WORLD_SIZE unset and N > 1: the torchrun command that starts N fresh rank
      processes of `script` (one per GPU), to run as a child process before
      this one makes any GPU call; the rendezvous store binds its own port
      (endpoint port 0: no probe-then-bind race on a shared box) and every
      address is 127.0.0.1;
    * otherwise None: run here as the single rank."""
    who = who or os.path.basename(script)
    if gpus < 1:
        raise SystemExit(f"{who}: {gpus} GPUs requested: need at least one")
    ws = environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != gpus:
            print(f"{who}: {gpus} GPUs requested but WORLD_SIZE={ws}; refusing to report a {ws}-rank run as "
                  f"n_gpus={gpus}", file=sys.stderr)
            raise SystemExit(2)
        return None
    if gpus == 1:
        return None
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--rdzv-backend=c10d", f"--rdzv-endpoint=127.0.0.1:{int(port or 0)}", "--local-addr", "127.0.0.1",
            script] + list(argv)


def run_ranks(plan, cwd=None):
    """run the torchrun child in its own process group; a SIGTERM / SIGINT to
    this launcher (a time limit) is passed on to the whole group, so no rank
    outlives it"""
    child = subprocess.Popen(plan, cwd=cwd, start_new_session=True)

    def forward(sig, _frame):
        try:
            os.killpg(child.pid, sig)
        except ProcessLookupError:
            pass
    for s in (signal.SIGTERM, signal.SIGINT):
        signal.signal(s, forward)
    return child.wait()
