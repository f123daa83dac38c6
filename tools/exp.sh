set -e
O=gpurun_out/cg; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/test.log 2>&1
for i in 1 2; do timeout -k 10 120 python3 bench.py --no-cpu-baseline --steps 20 --warmup 3 > $O/b_$i.json 2> $O/b.err; done
MDP_LIB=maddpg_amd/libmaddpg_hip_stamps.so timeout -k 10 120 python3 tools/stamps.py > $O/stamps.txt 2>&1
