#!/bin/bash
# full GPU test suite + smoke + profile passes + per-config bench lines; stops at the first failure
set -e
T=${1:-r02f}
mkdir -p gpurun_out/$T-t
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$T-t/gpu_tests.log 2>&1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$T-t/smoke.log 2>&1
bash tools/profile_run.sh $T
bash tools/bench_configs.sh $T
echo "full $T done"
