#!/bin/bash
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=18
step probe_c3 120 tools/fold_probe 3
step probe_c5 120 tools/fold_probe 5
