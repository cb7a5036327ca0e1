#!/bin/bash
# Round 3: boundary device call, host time per phase (CRDT_TRACE_STAGE), untraced.
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=3
step bnd_phase 120 env CRDT_TRACE_STAGE=1 go-crdt-playground_amd/host/build/boundary_bench 65536
grep "exchange_batch" gpurun_out/bnd_phase.log | head -12
