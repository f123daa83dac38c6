#!/bin/bash
# A/B of one environment switch on the default S2 bench (alternating, N runs each):
#   bash tools/ab_env.sh <tag> "MDP_ACTOR_PRE=0" [N] [extra bench args]
set -e
O=gpurun_out/${1:-ab}; mkdir -p $O
V=${2:?variant env assignment}
N=${3:-3}
B="python3 bench.py --no-cpu-baseline --no-throughput-figure --no-gather-stage --no-configs2 --steps 30 --warmup 5 ${4:-}"
for i in $(seq 1 $N); do
  timeout -k 10 150 $B > $O/base$i.json 2> $O/base$i.err
  env $V timeout -k 10 150 $B > $O/var$i.json 2> $O/var$i.err
done
echo "ab done"
