B="python3 bench.py --no-cpu-baseline --no-throughput-figure --steps 30"
for v in "X=1" "HIP_FORCE_DEV_KERNARG=1" "HIP_FORCE_DEV_KERNARG=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1" "ROC_ACTIVE_WAIT_TIMEOUT=0" "HIP_LAUNCH_BLOCKING=0 AMD_SERIALIZE_KERNEL=0"; do
  env $v timeout -k 10 120 $B > gpurun_out/env.json 2>/dev/null && python3 -c "
import json;d=json.load(open('gpurun_out/env.json'));print('$v', d['value'], d['ms_per_step'])" >> gpurun_out/envexp.log
done
