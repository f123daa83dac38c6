#!/bin/bash
# rocprofv3 passes of the configs[4] bench (simple_tag N=6, H=128, B=4096, 4096
# env copies; the general gradient kernels), each in its own run:
#   gpurun --timeout 900 -- 'bash tools/profile_s5.sh r03a'
# 1) --kernel-trace --stats, 2)/3) FETCH_SIZE and WRITE_SIZE, 4) MFMA busy cycles,
# 5) the plain bench line.  Then: python tools/profile_summary.py --tag <tag>_s5 \
#   --trace gpurun_out/<tag>_s5/trace --fetch ... --write ... --mfma ... \
#   --bench gpurun_out/<tag>_s5/bench.json --config-key simple_tag_E4096_B4096_H128_N6
set -e
TAG=${1:-prof}
export TMPDIR=/tmp
O=gpurun_out/${TAG}_s5
rm -rf $O; mkdir -p $O
S5="--scenario simple_tag --num-agents 6 --scenario-adversaries 4 --num-adversaries 4 --num-units 128 --batch-size 4096 --num-envs 4096"
Q="--no-cpu-baseline --no-throughput-figure --no-gather-stage --no-configs2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
    python3 bench.py $Q $S5 --steps 8 --warmup 2 > $O/prof_bench.json 2> $O/prof_bench.err
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- \
    python3 bench.py $Q $S5 --steps 2 --warmup 1 > $O/fetch.json 2> $O/fetch.err
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- \
    python3 bench.py $Q $S5 --steps 2 --warmup 1 > $O/write.json 2> $O/write.err
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/mfma -o run --output-format csv -- \
    python3 bench.py $Q $S5 --steps 2 --warmup 1 > $O/mfma.json 2> $O/mfma.err
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY \
    SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT -d $O/sq -o run --output-format csv -- \
    python3 bench.py $Q $S5 --steps 2 --warmup 1 > $O/sq.json 2> $O/sq.err
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-gather-stage --no-configs2 $S5 --steps 20 --warmup 3 \
    > $O/bench.json 2> $O/bench.err
echo "profile ${TAG}_s5 done"
