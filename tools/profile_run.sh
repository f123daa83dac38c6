#!/bin/bash
# Profile the bench on a GPU box (run through gpurun from the repo root):
#   gpurun --timeout 1100 -- 'bash tools/profile_run.sh r01b'
# 1) rocprofv3 --kernel-trace --stats, 2)/3) FETCH_SIZE and WRITE_SIZE in their
# own passes, 4) the plain bench with the CPU baseline, 5) MFMA busy cycles.  Stops at the first failure.
set -e
TAG=${1:-prof}
export TMPDIR=/tmp
O=gpurun_out/$TAG
rm -rf $O; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-throughput-figure --no-gather-stage --no-configs2 > $O/prof_bench.json 2> $O/prof_bench.err
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-throughput-figure --no-gather-stage --no-configs2 > $O/fetch.json 2> $O/fetch.err
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-throughput-figure --no-gather-stage --no-configs2 > $O/write.json 2> $O/write.err
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/mfma -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-throughput-figure --no-gather-stage --no-configs2 > $O/mfma.json 2> $O/mfma.err
# 6) wave-state counters of every kernel (quad-cycles): parked at s_waitcnt / barrier, issue-stalled,
#    LDS-issue-stalled, active; VALU / LDS activity and bank conflicts (tools/profile_summary.py --sq)
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY \
    SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT -d $O/sq -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-throughput-figure --no-gather-stage --no-configs2 > $O/sq.json 2> $O/sq.err
echo "profile $TAG done"
