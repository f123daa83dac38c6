#!/bin/bash
# One-GPU bench lines for every BASELINE.json config (run on a GPU box via gpurun):
#   gpurun --timeout 900 -- 'bash tools/bench_configs.sh r01e'
# configs[0] simple N=1 with one env (the reference's own CPU case, on the GPU), configs[1] spread E=1024 (the default bench), configs[2]'s per-GPU size (E=4096),
# configs[3] adversary 1 adv (ddpg) + 2 good (maddpg), E=4096, configs[4] tag N=6
# (4 adv + 2 good), H=128, B=4096.  Stops at the first failure.
set -e
TAG=${1:-cfg}
O=gpurun_out/$TAG/configs
mkdir -p $O
B="python3 bench.py --no-cpu-baseline --no-gather-stage --no-configs2 --steps 20 --warmup 3"
# configs[0]: one env copy, an episode (25 steps, 24 of them without a round) per graph replay, as train.py runs it
timeout -k 10 240 $B --steps 1000 --step-group 25 --scenario simple --num-agents 1 --num-envs 1 > $O/s1_simple_e1.json 2> $O/s1.err
timeout -k 10 240 $B > $O/s2_spread_e1024.json 2> $O/s2.err
timeout -k 10 240 $B --num-envs 4096 > $O/s3_spread_e4096.json 2> $O/s3.err
timeout -k 10 240 $B --scenario simple_adversary --num-envs 4096 --num-adversaries 1 --adv-policy ddpg \
    > $O/s4_adversary_e4096.json 2> $O/s4.err
timeout -k 10 300 $B --scenario simple_tag --num-agents 6 --scenario-adversaries 4 --num-adversaries 4 \
    --num-units 128 --batch-size 4096 --num-envs 4096 > $O/s5_tag6_h128_b4096.json 2> $O/s5.err
echo "configs $TAG done"
