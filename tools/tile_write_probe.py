#!/usr/bin/env python3
"""Config-4 exchange under one tile-store variant, for the write counters
(the tile kernel's WRITE_SIZE is 1.35x its survivors' bytes).
Prints the survivors' bytes of the two outputs, so a `rocprofv3 --pmc
WRITE_SIZE ...` run of this script compares them with what the counters saw.
GPU box only; diagnostic.

  python3 tools/tile_write_probe.py SHAPE NT_STORES SHARED_KEYS [CALLS]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "go-crdt-playground_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import crdtgpu  # noqa: E402
from crdtgpu.batch import OutBuffers  # noqa: E402
from crdtgpu.engine import zipf_sizes  # noqa: E402


def main():
    shape, nts, shared = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    calls = int(sys.argv[4]) if len(sys.argv) > 4 else 2
    n = 16384
    dev = torch.device("cuda:0")
    eng = crdtgpu.Engine(0)
    sizes = zipf_sizes(0x5EED, n)
    offs = np.zeros(n + 1, dtype=np.uint32)
    np.cumsum(sizes, out=offs[1:])
    total = int(offs[-1])
    d_offs = torch.from_numpy(offs.view(np.int32).copy()).to(dev)
    A, B = OutBuffers(n, 2, total, device=dev), OutBuffers(n, 2, total, device=dev)
    eng.gen_zipf_async(0x5EED, n, d_offs, A, B)
    o1 = OutBuffers(n, 2, 2 * total, device=dev)
    o2 = OutBuffers(n, 2, 2 * total, device=dev, shared_keys=o1 if shared else None)
    eng.set_option("join_tile_shape", shape)
    eng.set_option("join_tile_nt_stores", nts)
    eng.set_max_doc_entries()
    for _ in range(calls):
        eng.exchange_async(A.as_batch(), B.as_batch(), o1, o2)
    eng.sync()
    c1 = int(o1.counts.to(torch.int64).sum())
    c2 = int(o2.counts.to(torch.int64).sum())
    small = int((torch.from_numpy(sizes.astype(np.int64)) <= 64).sum())
    la, lb = int(A.counts.to(torch.int64).sum()), int(B.counts.to(torch.int64).sum())
    w = c1 * 20 + c2 * (12 if shared else 20)
    print("shape %d nt_stores %d shared_keys %d: survivors %d + %d, survivor bytes per call %d (%.3f GB); "
          "live input entries %d + %d (%.3f GB read) in %d slots a side; docs of <= 64 slots %d" % (
              shape, nts, shared, c1, c2, w, w / 1e9, la, lb, 20 * (la + lb) / 1e9, total, small), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
