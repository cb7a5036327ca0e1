#!/bin/bash
# Round 3: boundary device phase with the device kept busy through the host packing
# (crdt_ctx_touch before the pack; CRDT_TOUCH_US) vs idle.
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=1
for r in 1 2; do
for t in none 20000 40000; do
if [ $t = none ]; then
step bnd_t${t}_$r 120 env CRDT_TRACE_STAGE=1 go-crdt-playground_amd/host/build/boundary_bench 65536
else
step bnd_t${t}_$r 120 env CRDT_TRACE_STAGE=1 CRDT_TOUCH_US=$t go-crdt-playground_amd/host/build/boundary_bench 65536
fi
grep "exchange_batch" gpurun_out/bnd_t${t}_$r.log | tail -5
done
done
