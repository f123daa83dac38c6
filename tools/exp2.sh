set -e
O=gpurun_out/gen2; mkdir -p $O
MDP_STAMP_CFG=tag6 MDP_LIB=maddpg_amd/libmaddpg_hip_stamps.so timeout -k 10 120 python3 tools/stamps.py > $O/stamps.txt 2>&1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/test.log 2>&1
timeout -k 10 200 python3 bench.py --scenario simple_tag --num-agents 6 --scenario-adversaries 4 --num-adversaries 4 --num-units 128 --batch-size 4096 --num-envs 4096 --no-cpu-baseline --steps 10 --warmup 2 > $O/tag6.json 2> $O/tag6.err
timeout -k 10 120 python3 bench.py --no-cpu-baseline --steps 20 --warmup 3 > $O/s2.json 2> $O/s2.err
