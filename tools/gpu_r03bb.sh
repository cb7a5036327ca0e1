#!/bin/bash
# Round 3: boundary device call with copies as blit kernels (HSA_ENABLE_SDMA=0) vs SDMA.
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=1
for r in 1 2; do
step bnd_sdma$r 120 env CRDT_TRACE_STAGE=1 go-crdt-playground_amd/host/build/boundary_bench 65536
grep "exchange_batch" gpurun_out/bnd_sdma$r.log | tail -5
step bnd_blit$r 120 env CRDT_TRACE_STAGE=1 HSA_ENABLE_SDMA=0 go-crdt-playground_amd/host/build/boundary_bench 65536
grep "exchange_batch" gpurun_out/bnd_blit$r.log | tail -5
done
step h2d_blit 60 env HSA_ENABLE_SDMA=0 tools/h2d_probe 0
