#!/usr/bin/env python3
"""Check a bench line against the rocprofv3 kernel trace of the SAME run.

For the headline and every leg, the dominant kernel's launches are picked out
of run_kernel_trace.csv by name and grid size (the headline's exchange and
config 4's small-document wave launches share a kernel name; every launch of
the group counts, eager checks and warmup included), and the mean duration is
compared with the line's roofline.launch_ms; frac is
recomputed from the trace mean and the line's algorithmic bytes.

  python3 tools/trace_check.py LINE.json TRACE.csv > profiles/rNN_trace_check.json
"""

import csv
import json
import sys
from collections import defaultdict

PEAK = 8000.0

# config -> kernel name prefix of its dominant launch
KERNELS = {
    "config2": "void crdt::join_wave_kernel<4, 8, 2, true, true>",
    "config3": "void crdt::fold_pipe_kernel<8, true, true, false>",
    "config4": "void crdt::join_tile_pipe_kernel<512, 2, true, true, true>",
    "config5": "void crdt::fold_pipe_kernel<32, false, true, false>",
}


def main():
    line = json.load(open(sys.argv[1]))
    by = defaultdict(list)
    for r in csv.DictReader(open(sys.argv[2])):
        by[(r["Kernel_Name"], int(r["Grid_Size_X"]))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    legs = {"config2" if line["config"]["workload"].startswith("config2") else "head": line}
    legs.update(line.get("legs", {}))
    out = {}
    for name, leg in legs.items():
        if name not in KERNELS:
            continue
        prefix = KERNELS[name]
        cands = [(k, v) for k, v in by.items() if k[0].startswith(prefix)]
        if not cands:
            continue
        # the leg's launches: the (name, grid) group with the most launches
        (kname, grid), durs = max(cands, key=lambda kv: len(kv[1]))
        mean = sum(durs) / len(durs)
        roof = leg["roofline"]
        b = roof["algorithmic_bytes_per_launch"]
        out[name] = {
            "kernel": kname, "grid_x": grid, "launches_in_trace": len(durs),
            "trace_mean_ms": mean, "trace_min_ms": min(durs), "trace_max_ms": max(durs),
            "line_launch_ms": roof["launch_ms"], "ratio_line_over_trace": roof["launch_ms"] / mean,
            "frac_line": roof["frac"], "frac_from_trace": b / (mean / 1e3) / 1e9 / PEAK,
            "note": {"config4": "config4's line times the whole exchange call (wave + plan + tile kernels); the trace "
                                "mean is join_tile_pipe_kernel alone",
                     "config3": "the line times the whole fold call (lean pass + the general pass over the "
                                "deferred documents); the trace mean is the lean pass alone",
                     "config5": "the line times the whole fold call (lean pass + the general pass over the "
                                "deferred documents); the trace mean is the lean pass alone"}.get(name, ""),
        }
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
