set -e
O=gpurun_out/tp2; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/test.log 2>&1
timeout -k 10 120 python3 bench.py --no-cpu-baseline --steps 20 --warmup 3 --update-mode throughput > $O/tp.json 2> $O/tp.err
