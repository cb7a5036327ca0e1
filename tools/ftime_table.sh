#!/bin/bash
# Summarise a tools/gpu_run.sh ftime run (gpurun stdout file): ms per launch by
# variant and config, rounds side by side, plus each variant's output checksums.
f=${1:?usage: tools/ftime_table.sh GPURUN_STDOUT}
grep -A1 "^\[ftime" "$f" | grep -v "^--" | paste - - |
  sed -E 's/^\[ftime_(.*)_c([35])_([0-9])\].*docs, ([0-9.]+) ms.*/\1 c\2 \4/' |
  awk '{k=$1" "$2; v[k]=v[k]" "$3} END {for (k in v) print k":"v[k]}' | sort
for l in gpurun_out/ftime_*_1.log; do printf '%s %s\n' "$(basename "$l" .log)" "$(grep -o 'checksum [0-9a-f]*' "$l")"; done
