set -e
mkdir -p gpurun_out/r03c
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r03c/gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03c/smoke.log 2>&1
timeout -k 10 900 bash tools/shared_gpu_rehearsal.sh r03c
