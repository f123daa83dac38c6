#!/bin/bash
# Bound of the batch-reduction work in the S2 gradient launches (round 6):
# shipped library vs timing-only SLAB_NONE and SLAB_NONE + DW_NONE builds
# (tools/build_variant.sh), alternating on the default S2 bench, then one
# rocprofv3 --kernel-trace --stats pass of the shipped and the DW_NONE build.
#   gpurun -- 'bash tools/ab_dw.sh r06bf'
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-abdw}; mkdir -p $O
B="python3 bench.py --no-cpu-baseline --no-throughput-figure --no-gather-stage --no-configs2 --steps 30 --warmup 5"
for i in 1 2 3; do
  timeout -k 10 150 $B > $O/base$i.json 2> $O/base$i.err
  MDP_LIB=maddpg_amd/libmaddpg_hip_slabnone.so timeout -k 10 150 $B > $O/slabnone$i.json 2> $O/slabnone$i.err
  MDP_LIB=maddpg_amd/libmaddpg_hip_dwnone.so timeout -k 10 150 $B > $O/dwnone$i.json 2> $O/dwnone$i.err
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/trace_base -o run --output-format csv -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-throughput-figure --no-gather-stage --no-configs2 > $O/tb.json 2> $O/tb.err
MDP_LIB=maddpg_amd/libmaddpg_hip_dwnone.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/trace_dw -o run --output-format csv -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-throughput-figure --no-gather-stage --no-configs2 > $O/td.json 2> $O/td.err
echo "ab_dw done"
