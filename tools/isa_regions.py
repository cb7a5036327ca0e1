#!/usr/bin/env python3
"""Static instruction mix of a kernel's ISA between consecutive s_memtime
stamps (the CRDT_STAMPS build of tools/fold_probe.hip): a quick map of which
phase of the fold carries the VALU / SALU / LDS / VMEM instructions.

  hipcc --offload-arch=gfx950 -O3 -std=c++17 -DCRDT_STAMPS -S --cuda-device-only \\
      tools/fold_probe.hip -o /tmp/probe.s
  python3 tools/isa_regions.py /tmp/probe.s fold_pipe_kernelILi32ELb0E
"""
import sys


def main():
    path, sym = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    body, on = [], False
    for ln in lines:
        if not on and ln.startswith("_Z") and sym in ln and ln.split(";")[0].rstrip().endswith(":"):
            on = True
            continue
        if on:
            body.append(ln)
            if ln.strip().startswith("s_endpgm"):
                break
    regions, cur, start = [], None, 0

    def fresh():
        return {"valu": 0, "salu": 0, "lds": 0, "vmem": 0, "all": 0}

    cur = fresh()
    for i, ln in enumerate(body):
        t = ln.strip()
        if not t or t.startswith((";", ".")) or t.endswith(":"):
            continue
        op = t.split()[0]
        if op == "s_memtime":
            regions.append((start, i, cur))
            cur, start = fresh(), i
            continue
        cur["all"] += 1
        if op.startswith("v_"):
            cur["valu"] += 1
        elif op.startswith("s_"):
            cur["salu"] += 1
        elif op.startswith("ds_"):
            cur["lds"] += 1
        elif op.startswith(("buffer_", "global_", "flat_")):
            cur["vmem"] += 1
    regions.append((start, len(body), cur))
    for s, e, c in regions:
        print("%6d-%6d  %s" % (s, e, "  ".join("%s=%d" % kv for kv in c.items())))


if __name__ == "__main__":
    main()
