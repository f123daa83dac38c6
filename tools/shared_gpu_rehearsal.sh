#!/bin/bash
# Rehearsal of bench.py's multi-rank path on a 1-GPU box (run through gpurun
# from the repo root):  gpurun --timeout 600 -- 'bash tools/shared_gpu_rehearsal.sh r01k'
# Every rank on cuda:0 with a gloo process group (MDP_SHARED_GPU=1); the exchange
# is the real one: direct xGMI inside the optimizer kernel, or with
# MDP_NATIVE_DP=0 the torch.distributed all-reduce path.  Ranks share one GPU, so
# the rates say nothing about scaling; this checks that the N>1 code path of the
# driver's command runs to its JSON line.  Stops at the first failure.
set -e
TAG=${1:-rehearsal}
O=gpurun_out/$TAG/shared_gpu
mkdir -p $O
export MDP_SHARED_GPU=1
run() {  # name nproc env-assignment [bench args...]
  local name=$1 np=$2 ev=$3; shift 3
  env $ev timeout -k 10 240 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $np \
      --master-addr 127.0.0.1 --master-port $((29600 + RANDOM % 200)) \
      bench.py --gpus $np --steps 10 --warmup 2 "$@" > $O/$name.json 2> $O/$name.err
  echo "$name: $(tail -c 400 $O/$name.json)"
}
run xgmi2 2 MDP_DP_XGMI=1
run xgmi4 4 MDP_DP_XGMI=1 --no-throughput-figure
run torchdist2 2 MDP_NATIVE_DP=0
# 8 ranks (7 peers per exchange, MDP_XCH_MAXW filled) launched by bench.py itself
# (--gpus 8 without torchrun's environment), small E per rank
env MDP_DP_XGMI=1 timeout -k 10 300 python3 bench.py --gpus 8 --num-envs 512 --steps 5 --warmup 2 \
    --no-throughput-figure > $O/xgmi8.json 2> $O/xgmi8.err
echo "xgmi8: $(tail -c 400 $O/xgmi8.json)"
# configs[4]'s topology (general H=128 kernels), 2 ranks over xGMI
run tag6_xgmi2 2 MDP_DP_XGMI=1 --scenario simple_tag --num-agents 6 --scenario-adversaries 4 \
    --num-adversaries 4 --num-units 128 --batch-size 4096 --num-envs 4096 --steps 5 --no-throughput-figure
echo "rehearsal $TAG done"
