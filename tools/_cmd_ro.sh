#!/bin/bash
set -e
O=gpurun_out/${1:-ro1}; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "env or rollout or train_step or configs or facade or benchmark" > $O/tests.log 2>&1
bash tools/ab_var.sh $(basename $O)/ab ref 3 > /dev/null
echo "ro done"
