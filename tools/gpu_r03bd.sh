#!/bin/bash
# Round 3: boundary staging read by a kernel from page-locked memory (CRDT_ZERO_COPY=1)
# vs runtime copies; then the C++ mirror's GPU tests with it on.
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=1
for r in 1 2; do
for z in 0 1; do
step bnd_z${z}_$r 120 env CRDT_TRACE_STAGE=1 CRDT_ZERO_COPY=$z go-crdt-playground_amd/host/build/boundary_bench 65536
grep "exchange_batch" gpurun_out/bnd_z${z}_$r.log | tail -5
done
done
TAILN=3
step mirror_z1 600 env CRDT_ZERO_COPY=1 python -u -m pytest tests/test_host_cpp.py -x -q --timeout 300 --timeout-method thread
