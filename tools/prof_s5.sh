#!/bin/bash
# rocprofv3 kernel stats of the S5 bench (tag N=6, H=128, B=4096): bash tools/prof_s5.sh <tag> [env assignment]
set -e
export TMPDIR=/tmp
O=gpurun_out/$1; rm -rf $O; mkdir -p $O
S5="--scenario simple_tag --num-agents 6 --scenario-adversaries 4 --num-adversaries 4 --num-units 128 --batch-size 4096 --num-envs 4096 --steps 4 --warmup 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --no-throughput-figure --no-gather-stage --no-configs2 $S5 > $O/bench.json 2> $O/bench.err
find $O/trace -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
echo "prof done"
