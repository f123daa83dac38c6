#!/bin/bash
# A/B of the current library against another build of it (e.g. the previous
# commit, built by tools/build_ref_lib.sh into maddpg_amd/libmaddpg_hip_ref.so),
# alternating on the default S2 bench, N runs each:
#   bash tools/ab_lib.sh <tag> [N] [lib] [extra bench args]
set -e
O=gpurun_out/${1:-ablib}; mkdir -p $O
N=${2:-3}
L=${3:-maddpg_amd/libmaddpg_hip_ref.so}
B="python3 bench.py --no-cpu-baseline --no-throughput-figure --no-gather-stage --no-configs2 --steps 30 --warmup 5 ${4:-}"
for i in $(seq 1 $N); do
  timeout -k 10 150 $B > $O/base$i.json 2> $O/base$i.err
  MDP_LIB=$L timeout -k 10 150 $B > $O/ref$i.json 2> $O/ref$i.err
done
echo "ab_lib done"
