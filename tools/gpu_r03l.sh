#!/bin/bash
# Round 3: mbcnt lane ranks + trimmed meta vectors: fold parity; AWSet fold at
# 4 vs 5 waves per SIMD (timing builds, config 5); pipelined C++ ExchangeBatch.
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=4
step fold_tests 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_apply.py tests/test_gpu_sort.py tests/test_host_cpp.py -x -q --timeout 300 --timeout-method thread
grep -q " failed\| error" gpurun_out/fold_tests.log && exit 1
TAILN=3
step t5_w4 120 tools/fold_time_w4 5
step t5_w5 120 tools/fold_time_w5 5
TAILN=1
step boundary16 300 go-crdt-playground_amd/host/build/boundary_bench 65536
step boundary16c 300 env CRDT_HOST_CHUNK_DOCS=16384 go-crdt-playground_amd/host/build/boundary_bench 65536
step boundary16n 300 env CRDT_HOST_CHUNK_DOCS=65536 go-crdt-playground_amd/host/build/boundary_bench 65536
step boundary2 300 go-crdt-playground_amd/host/build/boundary_bench 262144
