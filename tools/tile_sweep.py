#!/usr/bin/env python3
"""Sweep the large-document tile kernel's shape (crdt_ctx_set_option
"join_tile_shape") on the config-4 exchange: HIP-event time per call.
GPU box only."""
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
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    dev = torch.device("cuda:0")
    eng = crdtgpu.Engine(0)
    sizes = zipf_sizes(0x5EED, n)
    offs = np.zeros(n + 1, dtype=np.uint32)
    np.cumsum(sizes, out=offs[1:])
    total = int(offs[-1])
    d_offs = torch.from_numpy(offs.view(np.int32).copy()).to(dev)
    A, B = OutBuffers(n, 2, total, device=dev), OutBuffers(n, 2, total, device=dev)
    eng.gen_zipf_async(0x5EED, n, d_offs, A, B)
    o1, o2 = OutBuffers(n, 2, 2 * total, device=dev), OutBuffers(n, 2, 2 * total, device=dev)
    a, b = A.as_batch(), B.as_batch()
    ref = None
    eng.set_option("join_tile_capacity", 1 << 22)  # room for the smaller tile shapes (2.07 M tiles of 512)
    # shape:nt_stores[:split workgroups per CU[:dispenser words]]
    dflt = (9, 1, 4, 8)
    shapes = [tuple([int(v) for v in a.split(":")] + list(dflt[len(a.split(":")):])) for a in sys.argv[2:]] or \
        [(9, 1, 4, 8), (9, 1, 4, 1)]
    for shape, nts, sbpc, shards in shapes:
        eng.set_option("join_tile_shape", shape)
        eng.set_option("join_tile_nt_stores", nts)
        eng.set_option("join_tile_split_blocks_per_cu", sbpc)
        eng.set_option("join_tile_dispensers", shards)
        eng.exchange_async(a, b, o1, o2)
        eng.sync()
        got = (o1.counts.clone(), o1.keys.clone(), o1.actors.clone(), o1.counters.clone(), o2.counts.clone(),
               o2.keys.clone(), o2.actors.clone(), o2.counters.clone(), o1.vv.clone(), o2.vv.clone())
        if ref is None:
            ref = got
        same = all(torch.equal(x, y) for x, y in zip(ref, got))
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        for _ in range(5):
            eng.exchange_async(a, b, o1, o2)
        ev[1].record()
        eng.sync()
        print("shape %d nt %d split_bpc %d dispensers %d: %.3f ms per exchange call (same output: %s)" % (
            shape, nts, sbpc, shards, ev[0].elapsed_time(ev[1]) / 5, same), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
