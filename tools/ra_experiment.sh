#!/bin/bash
# timing experiment: reduce_apply variants (MDP_RA_DBG) + stamps timeline
set -e
O=gpurun_out/ra_exp; mkdir -p $O
for d in 0 1 2 3 8; do
  MDP_RA_DBG=$d timeout -k 10 120 python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 > $O/ra_$d.json 2> $O/ra_$d.err
done
MDP_LIB=maddpg_amd/libmaddpg_hip_stamps.so timeout -k 10 120 python3 tools/stamps.py > $O/stamps.txt 2>&1
echo done
