#!/bin/bash
# Round 3: boundary staging -- page-locked H2D copy rate per hipMemcpyAsync and in total.
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=8
step h2d_0 60 tools/h2d_probe 0
step h2d_1 60 tools/h2d_probe 1
step h2d_2 60 tools/h2d_probe 2
