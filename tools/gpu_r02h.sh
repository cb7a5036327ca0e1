#!/bin/bash
# Round 2: pipelined tile kernel + RCCL ABI -- parity, config-4 timing, kernel trace.
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=12
step comm_tests 300 python -u -m pytest tests/test_gpu_comm.py -x -v --timeout 120 --timeout-method thread
step tile_tests 900 python -u -m pytest tests/test_gpu_tiles.py -x -q --timeout 600 --timeout-method thread
TAILN=3
step c4 300 python3 bench.py --config 4 --no-cpu-baseline --steps 10 --warmup 2 --repeats 2
step prof_c4 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4b -o run -- python3 bench.py --config 4 --no-cpu-baseline --steps 10 --warmup 2 --repeats 1
