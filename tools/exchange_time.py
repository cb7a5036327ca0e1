#!/usr/bin/env python3
"""Time the config-2 exchange (1,048,576 docs x 2 replicas x 64 entries) with
whatever libcrdtgpu.so CRDTGPU_LIB names: median of 6 rounds of 20 launches,
plus a checksum of the outputs so that library variants can be compared.
GPU box only (A/B of build variants)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "go-crdt-playground_amd"))
import torch  # noqa: E402

import crdtgpu  # noqa: E402
from crdtgpu.batch import OutBuffers  # noqa: E402

n = 1 << 20
dev = torch.device("cuda:0")
eng = crdtgpu.Engine(0)
eng.set_max_doc_entries(64)
A, B = OutBuffers(n, 2, n * 64, device=dev), OutBuffers(n, 2, n * 64, device=dev)
eng.gen_pair_async(0x5EED, n, A, B)
o1 = OutBuffers(n, 2, 2 * n * 64, device=dev)
# the bench's form: one key column shared by the two outputs (OWN_KEYS=1: one each)
o2 = OutBuffers(n, 2, 2 * n * 64, device=dev, shared_keys=None if os.environ.get("OWN_KEYS") == "1" else o1)
a, b = A.as_batch(), B.as_batch()
s = torch.cuda.current_stream()
eng.exchange_async(a, b, o1, o2, stream=s)
eng.sync()
# checksum of the live entries only (slack slots are unspecified: variants may write them)
live = (torch.arange(128, device=dev).view(1, 128) < o1.counts.to(torch.int64).view(n, 1)).view(-1)
chk = (int(o1.keys[live].sum()) ^ int(o2.counters[live].sum()) ^ int(o1.actors[live].to(torch.int64).sum() << 20)
       ^ int(o2.actors[live].to(torch.int64).sum() << 40) ^ int(o1.counters[live].sum()) ^ int(o1.vv.sum())
       ^ int(o1.counts.to(torch.int64).sum()))
assert bool((o1.offsets[:n].to(torch.int64) == torch.arange(n, device=dev) * 128).all())
ts = []
for _ in range(6):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(20):
        eng.exchange_async(a, b, o1, o2, stream=s)
    e1.record(s)
    e1.synchronize()
    ts.append(e0.elapsed_time(e1) / 20)
ts.sort()
print("%s: median %.4f ms min %.4f ms checksum %x" % (os.path.basename(os.environ.get("CRDTGPU_LIB", "libcrdtgpu.so")),
                                                      ts[3], ts[0], chk & 0xFFFFFFFFFFFF))
