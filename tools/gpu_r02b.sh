#!/bin/bash
# Round 2: the pipelined fold kernel -- parity, graph replay, timing, stamps.
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=8
step fold_tests 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "fold or config3 or config5 or golden or delta"
step c3 240 python3 bench.py --config 3 --no-cpu-baseline --steps 10 --warmup 2 --force-graph
step c5 240 python3 bench.py --config 5 --no-cpu-baseline --steps 10 --warmup 2 --force-graph
step prof_c3 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof2_c3 -o run -- python3 bench.py --config 3 --no-cpu-baseline --steps 10 --warmup 2 --no-graph
step prof_c5 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof2_c5 -o run -- python3 bench.py --config 5 --no-cpu-baseline --steps 10 --warmup 2 --no-graph
step probe_c3 120 tools/fold_probe 3
step probe_c5 120 tools/fold_probe 5
