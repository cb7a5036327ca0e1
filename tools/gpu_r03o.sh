#!/bin/bash
# Round 3: where the boundary's device call goes (kernel + copy trace).
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
TAILN=2
step prof_boundary 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/prof_bnd -o run -- go-crdt-playground_amd/host/build/boundary_bench 65536
find gpurun_out/prof_bnd -name "*stats*" | head
