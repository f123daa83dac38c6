set -e
O=gpurun_out/xg; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_dp_xgmi_gpu.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 300 python3 tools/xgmi_pair_bench.py --ranks 4 --only-shared > $O/new4.log 2>&1
MDP_LIB=maddpg_amd/libmaddpg_hip_oldx.so timeout -k 10 300 python3 tools/xgmi_pair_bench.py --ranks 4 --only-shared > $O/old4.log 2>&1
timeout -k 10 300 python3 tools/xgmi_pair_bench.py --ranks 4 --only-shared > $O/new4b.log 2>&1
MDP_LIB=maddpg_amd/libmaddpg_hip_oldx.so timeout -k 10 300 python3 tools/xgmi_pair_bench.py --ranks 4 --only-shared > $O/old4b.log 2>&1
echo xg done
