#!/usr/bin/env python3
"""Timeline of the boundary bench's HIP calls next to what the GPU was doing
(tools/gpu_run.sh btrace: rocprofv3 --hip-trace --memory-copy-trace
--kernel-trace of go-crdt-playground_amd/host/build/boundary_bench).

For every HIP API call of the main thread that took longer than a threshold,
prints when it started and ended (ms from the first call of the process) and
which copies / kernels were running on the GPU during it, so a call that
blocks can be matched with the device work it waited for.

  python3 tools/btrace_timeline.py gpurun_out/btrace_TAG [min_ms]
"""
import csv
import glob
import os
import sys


def rows(d, pat):
    out = []
    for fn in glob.glob(os.path.join(d, "**", pat), recursive=True):
        with open(fn) as f:
            out.extend(csv.DictReader(f))
    return out


def main():
    d = sys.argv[1]
    thr = float(sys.argv[2]) if len(sys.argv) > 2 else 0.3
    api = rows(d, "*hip_api_trace.csv")
    cp = rows(d, "*memory_copy_trace.csv")
    kt = rows(d, "*kernel_trace.csv")
    if not api:
        print("no hip_api_trace.csv under", d)
        return
    t0 = min(int(r["Start_Timestamp"]) for r in api)
    ms = lambda t: (int(t) - t0) / 1e6  # noqa: E731
    gpu = [(ms(r["Start_Timestamp"]), ms(r["End_Timestamp"]), "copy %s %s B" % (r.get("Direction", "?"),
                                                                                  r.get("Size", "?"))) for r in cp]
    gpu += [(ms(r["Start_Timestamp"]), ms(r["End_Timestamp"]), "kernel " + r["Kernel_Name"].split("(")[0][:48])
            for r in kt]
    gpu.sort()
    own = {}  # correlation id -> the GPU op the call submitted
    for r in cp + kt:
        own[r["Correlation_Id"]] = (ms(r["Start_Timestamp"]), ms(r["End_Timestamp"]))
    calls = sorted(api, key=lambda r: int(r["Start_Timestamp"]))
    main_tid = max(set(r["Thread_Id"] for r in calls), key=lambda t: sum(1 for r in calls if r["Thread_Id"] == t))
    busy_total = 0.0
    for r in calls:
        if r["Thread_Id"] != main_tid:
            continue
        a, b = ms(r["Start_Timestamp"]), ms(r["End_Timestamp"])
        if b - a < thr:
            continue
        during = [(s, e, w) for s, e, w in gpu if e > a and s < b]
        busy = sum(min(e, b) - max(s, a) for s, e, _ in during)
        busy_total += b - a
        mine = own.get(r["Correlation_Id"])
        print("%10.3f %8.3f ms  %-22s gpu busy %5.1f%% of it;%s %s" % (
            a, b - a, r["Function"][:22], 100.0 * busy / (b - a) if b > a else 0.0,
            (" its own op starts %+.3f ms after the call returns;" % (mine[0] - b)) if mine else "",
            "; ".join("%s [%.3f-%.3f]" % (w, s, e) for s, e, w in during[:3])))
    print("calls >= %.2f ms on the main thread: %.1f ms in total" % (thr, busy_total))


if __name__ == "__main__":
    main()
