#!/bin/bash
# One PMC pass (stall breakdown) over the tag6 config: wave-cycle buckets, MFMA busy, LDS conflicts, L2 hits.
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-pmc_s5}
mkdir -p $O
B="python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 --no-throughput-figure --scenario simple_tag --num-agents 6 --scenario-adversaries 4 --num-adversaries 4 --num-units 128 --batch-size 4096 --num-envs 4096"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES -d $O/sq -o run --output-format csv -- $B > $O/sq.json 2> $O/sq.err
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $O/tcc -o run --output-format csv -- $B > $O/tcc.json 2> $O/tcc.err
echo done
