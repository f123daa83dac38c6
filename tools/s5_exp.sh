#!/bin/bash
# S5 (simple_tag N=6, H=128, B=4096) check of a general-kernel change: GPU tests,
# the stamped critic timeline, two bench lines.  Stops at the first failure.
set -e
O=gpurun_out/${1:-s5exp}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/test.log 2>&1
MDP_STAMP_CFG=tag6 MDP_LIB=maddpg_amd/libmaddpg_hip_stamps.so timeout -k 10 120 python3 tools/stamps.py > $O/stamps.txt 2>&1
B="python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 --no-throughput-figure --scenario simple_tag --num-agents 6 --scenario-adversaries 4 --num-adversaries 4 --num-units 128 --batch-size 4096 --num-envs 4096"
for i in 1 2; do timeout -k 10 200 $B > $O/tag6_$i.json 2> $O/tag6_$i.err; done
echo "s5 exp done"
