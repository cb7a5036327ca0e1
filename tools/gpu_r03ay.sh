#!/bin/bash
# Round 3: where the boundary's device call (ExchangeBatch, 65,536 docs) spends its time:
# per-stage host timing and a HIP API + memory-copy + kernel trace of the same binary.
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=12
step bnd_stage 120 env CRDT_TRACE_STAGE=1 go-crdt-playground_amd/host/build/boundary_bench 65536
step bnd_trace 180 rocprofv3 --hip-runtime-trace --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/prof_bnd -o run -- go-crdt-playground_amd/host/build/boundary_bench 65536
