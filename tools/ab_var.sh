#!/bin/bash
# A/B of the current library against a variant build (tools/build_variant.sh)
# on S5 (tag6 H=128 B=4096) and S2, alternating, N runs each:
#   bash tools/ab_var.sh <tag> <variant-name> [N]
set -e
O=gpurun_out/$1; mkdir -p $O
L=maddpg_amd/libmaddpg_hip_$2.so
N=${3:-3}
B="python3 bench.py --no-cpu-baseline --no-throughput-figure --no-gather-stage --no-configs2"
S5="--scenario simple_tag --num-agents 6 --scenario-adversaries 4 --num-adversaries 4 --num-units 128 --batch-size 4096 --num-envs 4096 --steps 10 --warmup 2"
for i in $(seq 1 $N); do
  timeout -k 10 200 $B $S5 > $O/s5_base$i.json 2> $O/s5_base$i.err
  MDP_LIB=$L timeout -k 10 200 $B $S5 > $O/s5_var$i.json 2> $O/s5_var$i.err
done
for i in $(seq 1 $N); do
  timeout -k 10 150 $B --steps 30 --warmup 5 > $O/s2_base$i.json 2> $O/s2_base$i.err
  MDP_LIB=$L timeout -k 10 150 $B --steps 30 --warmup 5 > $O/s2_var$i.json 2> $O/s2_var$i.err
done
echo "ab_var done"
