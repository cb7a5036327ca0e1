#!/bin/bash
# Round 3: full GPU suite after the fold shapes / counting sort and the C++
# mirror's interner rewrite; fold stamps + timing; boundary at 16 threads.
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=4
step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
grep -q " failed\| error" gpurun_out/gpu_tests.log && exit 1
TAILN=14
step probe_c3 120 tools/fold_probe 3
step probe_c5 120 tools/fold_probe 5
TAILN=1
step bench_c3 300 python3 bench.py --config 3 --legs 5 --no-cpu-baseline --no-boundary --no-box-probe --steps 20 --warmup 5
step boundary16 300 go-crdt-playground_amd/host/build/boundary_bench 65536
step boundary16b 300 go-crdt-playground_amd/host/build/boundary_bench 262144
