#!/bin/bash
# Round 3 closing evidence at HEAD: full GPU suite, smoke, default bench line under a kernel
# trace of the same run, line-vs-trace check (kernels unchanged since r03aw: its PMC passes stand).
set -u
cd "$(dirname "$0")/.."
source tools/gpu_step.sh
TAILN=3
step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
grep -q " failed\| error" gpurun_out/gpu_tests.log && exit 1
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
TAILN=1
step bench_traced 700 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r03bf -o run -- python3 bench.py
T=$(find gpurun_out/prof_r03bf -name "run_kernel_trace.csv" | head -1)
grep '^{"metric"' gpurun_out/bench_traced.log > gpurun_out/r03bf_bench.json
python3 tools/trace_check.py gpurun_out/r03bf_bench.json "$T" > gpurun_out/r03bf_trace_check.json
cat gpurun_out/r03bf_trace_check.json | python3 -c "import json,sys; d=json.load(sys.stdin); [print(k, round(v['trace_mean_ms'],4), round(v['ratio_line_over_trace'],3), round(v['frac_from_trace'],3)) for k,v in d.items()]"
