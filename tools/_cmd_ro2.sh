#!/bin/bash
set -e
O=gpurun_out/${1:-ro2}; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "env or rollout or train_step or configs or facade or benchmark or graph" > $O/tests.log 2>&1
MDP_LIB=maddpg_amd/libmaddpg_hip_stamps.so timeout -k 10 200 python3 tools/rollout_stamps.py > $O/rollout_stamps.txt 2>&1
bash tools/ab_var.sh $(basename $O)/ab ref 3 > /dev/null
echo "ro2 done"
