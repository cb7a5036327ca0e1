#!/usr/bin/env python3
"""GPU timeline of the boundary bench's timed device call (the last
crdt_awset_exchange_batch of tests/cpp/boundary_bench.cpp), from a
`tools/gpu_run.sh btrace` run (rocprofv3 --memory-copy-trace --kernel-trace).

The call's device work is its staging copies (host -> device), the order
check, the merge kernels and the packed-output scan and gather (which writes
the page-locked outputs over PCIe).  Prints the span from the call's first
copy to its last kernel, the time the GPU was busy in it (union of the copy
and kernel intervals), and the per-kind sums, to compare with the line's
`device_s` (the host's wall clock around the same call).

  python3 tools/boundary_gpu_timeline.py gpurun_out/btrace_TAG
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
    ev = []
    for r in rows(d, "*kernel_trace.csv"):
        ev.append(("kernel", r["Kernel_Name"].split("(")[0][:60], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    for r in rows(d, "*memory_copy_trace.csv"):
        ev.append(("copy " + r.get("Direction", "?"), "%s B" % r.get("Size", "?"), int(r["Start_Timestamp"]),
                   int(r["End_Timestamp"])))
    ev.sort(key=lambda e: e[2])
    # batch calls: from a host -> device copy to the next pack_out_kernel; the
    # bench's first is untimed (it sizes the staging), the second is the timed
    # one (the single-merge checks after it stage nothing through copies)
    calls, i = [], 0
    while i < len(ev):
        if ev[i][0].startswith("copy") and "HOST_TO_DEVICE" in ev[i][0]:
            j = i
            while j < len(ev) and not (ev[j][0] == "kernel" and "pack_out_kernel" in ev[j][1]):
                j += 1
            if j == len(ev):
                break
            calls.append(ev[i:j + 1])
            i = j + 1
        else:
            i += 1
    if len(calls) < 2:
        sys.exit("fewer than two batch calls in the trace")
    call = calls[1]
    t0, t1 = call[0][2], max(e[3] for e in call)
    busy, cur_s, cur_e = 0, None, None
    for _, _, s, e in sorted(call, key=lambda x: x[2]):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    sums = {}
    for k, _, s, e in call:
        sums[k] = sums.get(k, 0) + (e - s)
    print("timed call: %d GPU operations, first copy -> last kernel %.3f ms, GPU busy %.3f ms" % (
        len(call), (t1 - t0) / 1e6, busy / 1e6))
    for k, v in sorted(sums.items()):
        print("  %-24s %.3f ms" % (k, v / 1e6))
    for k, name, s, e in call:
        print("  %8.3f %8.3f  %-14s %s" % ((s - t0) / 1e6, (e - s) / 1e6, k, name))


if __name__ == "__main__":
    main()
