#!/bin/bash
# S5 grad-kernel time vs batch (workgroups = B/16): per-CU-bound phases keep their
# time as the grid shrinks, aggregate-bound (L2 / fabric) ones shrink with it.
set -e
O=gpurun_out/${1:-s5sweep}; mkdir -p $O
B="python3 bench.py --no-cpu-baseline --steps 4 --warmup 1 --no-throughput-figure --scenario simple_tag --num-agents 6 --scenario-adversaries 4 --num-adversaries 4 --num-units 128 --num-envs 4096"
for b in 4096 2048 1024 512; do timeout -k 10 200 $B --batch-size $b > $O/b$b.json 2> $O/b$b.err; done
echo sweep done
