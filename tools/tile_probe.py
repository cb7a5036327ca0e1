#!/usr/bin/env python3
"""Diagnostic (GPU box only): where join_tile_kernel's cycles go on the config-4
exchange.  Loads the stamped build of the library (make -C
go-crdt-playground_amd/csrc stamps -> tools/libcrdtgpu_stamps.so), runs the
exchange, and prints the per-phase share of wave cycles (s_memtime stamps; the
stamped build is slower than the product kernel: read the shares)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["CRDTGPU_LIB"] = os.path.join(ROOT, "tools", "libcrdtgpu_stamps.so")
sys.path[:0] = [ROOT, os.path.join(ROOT, "go-crdt-playground_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import crdtgpu  # noqa: E402
from crdtgpu.batch import OutBuffers  # noqa: E402
from crdtgpu.engine import zipf_sizes  # noqa: E402

PHASES = ["wait data + stage", "merge walk / rank decide", "survivor scan + stage idx", "look-back + dispense",
          "next geo + issue", "stores", "(wave 0) publish + look-back", "(wave 0) dispense atomic"]


def main():
    n = 16384
    shape = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    dev = torch.device("cuda:0")
    eng = crdtgpu.Engine(0)
    eng.set_option("join_tile_shape", shape)
    lib = ctypes.CDLL(os.environ["CRDTGPU_LIB"])
    lib.crdt_probe_tile_stamps.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    sizes = zipf_sizes(0x5EED, n)
    offs = np.zeros(n + 1, dtype=np.uint32)
    np.cumsum(sizes, out=offs[1:])
    total = int(offs[-1])
    d_offs = torch.from_numpy(offs.view(np.int32).copy()).to(dev)
    A, B = OutBuffers(n, 2, total, device=dev), OutBuffers(n, 2, total, device=dev)
    eng.gen_zipf_async(0x5EED, n, d_offs, A, B)
    o1, o2 = OutBuffers(n, 2, 2 * total, device=dev), OutBuffers(n, 2, 2 * total, device=dev)
    a, b = A.as_batch(), B.as_batch()
    eng.exchange_async(a, b, o1, o2)
    eng.sync()
    buf = (ctypes.c_ulonglong * 16)()
    lib.crdt_probe_tile_stamps(buf, 1)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    reps = 5
    for _ in range(reps):
        eng.exchange_async(a, b, o1, o2)
    ev[1].record()
    eng.sync()
    lib.crdt_probe_tile_stamps(buf, 0)
    tot = sum(buf[i] for i in range(len(PHASES)))  # wave 0's split of phase 3 counts once: 3 = waves 1..3 + wave 0 rest
    print("shape %d: %.3f ms per stamped exchange call" % (shape, ev[0].elapsed_time(ev[1]) / reps))
    for i, name in enumerate(PHASES):
        print("  %-28s %5.1f%%" % (name, 100.0 * buf[i] / max(tot, 1)))
    tiles = None
    print("  look-back polls per launch: %d summing, %d finding a predecessor unpublished" %
          (buf[8] // reps, buf[9] // reps))
    eng.close()


if __name__ == "__main__":
    main()
