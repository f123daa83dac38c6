#!/bin/bash
# Round-end validation of the tree on one GPU box (through gpurun from the repo root):
#   gpurun --timeout 1150 -- 'bash tools/final_validation.sh r06bn'
# GPU tests, smoke, S2 and S5 rocprof + PMC passes with their bench lines,
# every BASELINE config, the reference's default training command (simple_spread
# on 1,024 env copies) and its one-env structure (simple).  Stops at the first failure.
set -e
TAG=${1:-final}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
bash tools/profile_run.sh ${TAG}_p
bash tools/profile_s5.sh $TAG
bash tools/bench_configs.sh $TAG
timeout -k 10 300 python experiments/train.py --scenario simple_spread --num-envs 1024 --num-episodes 60000 \
    --exp-name spread --save-dir /tmp/policy_s/ --plots-dir $O/cli/ > $O/train_spread.log 2>&1
timeout -k 10 300 python experiments/train.py --scenario simple --num-episodes 4000 --exp-name simple1 \
    --save-dir /tmp/policy_1/ --plots-dir $O/cli/ > $O/train_simple_e1.log 2>&1
echo "final validation $TAG done"
