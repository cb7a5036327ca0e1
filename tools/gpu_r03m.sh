#!/bin/bash
# Round 3: AWSet fold at 5 waves per SIMD; map node reuse in the C++ mirror's
# apply: fold parity, host tests, boundary, config 5/3 timing.
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=4
step fold_tests 600 python -u -m pytest tests/test_gpu_parity.py tests/test_scenarios_gpu.py tests/test_host_cpp.py -x -q --timeout 300 --timeout-method thread
grep -q " failed\| error" gpurun_out/fold_tests.log && exit 1
TAILN=1
step boundary16 300 go-crdt-playground_amd/host/build/boundary_bench 65536
step boundary16b 300 go-crdt-playground_amd/host/build/boundary_bench 65536
step bench_c5 300 python3 bench.py --config 5 --legs 3 --no-cpu-baseline --no-boundary --no-sort --no-box-probe --steps 20 --warmup 5
