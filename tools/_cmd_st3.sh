set -e
mkdir -p gpurun_out/r03b
MDP_LIB=maddpg_amd/libmaddpg_hip_stamps.so timeout -k 10 120 python3 tools/stamps.py > gpurun_out/r03b/stamps_s2.txt 2>&1
MDP_LIB=maddpg_amd/libmaddpg_hip_stamps.so MDP_STAMP_CFG=tag6 timeout -k 10 180 python3 tools/stamps.py > gpurun_out/r03b/stamps_s5.txt 2>&1
echo done
