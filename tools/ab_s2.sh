#!/bin/bash
# A/B of two library builds on the default S2 bench (alternating, 3 runs each):
#   bash tools/ab_s2.sh <tag> maddpg_amd/libmaddpg_hip_<variant>.so
set -e
O=gpurun_out/${1:-ab}; mkdir -p $O
V=${2:?variant library}
B="python3 bench.py --no-cpu-baseline --no-throughput-figure --steps 30 --warmup 5"
for i in 1 2 3; do
  timeout -k 10 150 $B > $O/base$i.json 2> $O/base$i.err
  MDP_LIB=$V timeout -k 10 150 $B > $O/var$i.json 2> $O/var$i.err
done
echo "ab done"
