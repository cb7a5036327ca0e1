#!/bin/bash
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=60
step bnd_trace 120 env CRDT_TRACE_STAGE=1 go-crdt-playground_amd/host/build/boundary_bench 65536
