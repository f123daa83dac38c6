B="python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 --no-throughput-figure"
timeout -k 10 240 $B --scenario simple_tag --num-agents 6 --scenario-adversaries 4 --num-adversaries 4 --num-units 128 --batch-size 4096 --num-envs 4096
