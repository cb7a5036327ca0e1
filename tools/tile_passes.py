#!/usr/bin/env python3
"""Config-4 exchange with the tile workspace below the call's tiles
(crdt_ctx_set_option "join_tile_capacity"): passes of `cap` tiles (tile.hip,
launch_join_tiles) against one pass, interleaved rounds, HIP-event time per
call and the outputs compared with the one-pass call's bitwise.
GPU box only:  python3 tools/tile_passes.py [docs] [cap ...]"""
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
    caps = [int(c) for c in sys.argv[2:]] or [1 << 22, 400_000, 300_000]
    dev = torch.device("cuda:0")
    eng = crdtgpu.Engine(0)
    sizes = zipf_sizes(0x5EED, n)
    offs = np.zeros(n + 1, dtype=np.uint32)
    np.cumsum(sizes, out=offs[1:])
    total = int(offs[-1])
    d_offs = torch.from_numpy(offs.view(np.int32).copy()).to(dev)
    A, B = OutBuffers(n, 2, total, device=dev), OutBuffers(n, 2, total, device=dev)
    eng.gen_zipf_async(0x5EED, n, d_offs, A, B)
    eng.sync()
    nd = A.counts.to(torch.int64).cpu().numpy()
    ns = B.counts.to(torch.int64).cpu().numpy()
    big = (nd > 64) | (ns > 64)
    tiles = int(((nd + ns + 1023) // 1024)[big].sum())
    print("config 4: %d docs, %d tiles of 1024 merged positions" % (n, tiles), flush=True)
    o1, o2 = OutBuffers(n, 2, 2 * total, device=dev), OutBuffers(n, 2, 2 * total, device=dev)
    a, b = A.as_batch(), B.as_batch()
    ref = None
    res = {c: [] for c in caps}
    for rnd in range(3):
        for cap in caps:
            eng.set_option("join_tile_capacity", cap)
            for t in (o1.keys, o1.actors, o1.counters, o2.keys, o2.actors, o2.counters):
                t.fill_(-1)
            eng.exchange_async(a, b, o1, o2)
            eng.sync()
            got = [o1.counts.clone(), o2.counts.clone(), o1.vv.clone(), o2.vv.clone()]
            live = torch.zeros(2 * total, dtype=torch.bool, device=dev)
            starts = o1.offsets[:-1].to(torch.int64)
            cnt = o1.counts.to(torch.int64)
            idx = torch.repeat_interleave(starts, cnt) + (torch.arange(int(cnt.sum()), device=dev)
                                                           - torch.repeat_interleave(torch.cumsum(cnt, 0) - cnt, cnt))
            live[idx] = True
            for o in (o1, o2):
                got += [o.keys[live].clone(), o.actors[live].clone(), o.counters[live].clone()]
            if ref is None:
                ref = got
            same = all(torch.equal(x, y) for x, y in zip(ref, got))
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            for _ in range(5):
                eng.exchange_async(a, b, o1, o2)
            ev[1].record()
            eng.sync()
            ms = ev[0].elapsed_time(ev[1]) / 5
            res[cap].append(ms)
            print("round %d cap %8d (%d passes needed): %.3f ms per exchange call, same output as the first: %s" % (
                rnd, cap, (tiles + cap - 1) // cap, ms, same), flush=True)
    base = min(res[caps[0]])
    for cap in caps:
        print("cap %8d: best %.3f ms, %.3fx the cap-%d call" % (cap, min(res[cap]), min(res[cap]) / base, caps[0]))
    eng.set_option("join_tile_capacity", 1 << 22)
    eng.close()


if __name__ == "__main__":
    main()
