#!/usr/bin/env python3
"""Is the A<-B / B<-A asymmetry the direction or the output buffer?  (GPU box.)"""
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
A = OutBuffers(n, 2, n * 64, device=dev)
B = OutBuffers(n, 2, n * 64, device=dev)
eng.gen_pair_async(0x5EED, n, A, B)
o1 = OutBuffers(n, 2, 2 * n * 64, device=dev)
o2 = OutBuffers(n, 2, 2 * n * 64, device=dev)
eng.sync()
a, b = A.as_batch(), B.as_batch()
cases = {"A<-B>o1": (a, b, o1), "B<-A>o2": (b, a, o2), "A<-B>o2": (a, b, o2), "B<-A>o1": (b, a, o1),
         "A<-A>o1": (a, a, o1), "B<-B>o1": (b, b, o1)}
res = {k: [] for k in cases}
s = torch.cuda.current_stream()
for rnd in range(5):
    for k, (x, y, o) in cases.items():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        eng.join_async(x, y, o, stream=s)
        e0.record(s)
        for _ in range(6):
            eng.join_async(x, y, o, stream=s)
        e1.record(s)
        e1.synchronize()
        res[k].append(e0.elapsed_time(e1) / 6)
for k, v in res.items():
    v = sorted(v)
    print("%-10s median %.4f ms min %.4f" % (k, v[len(v) // 2], v[0]))
print("ptrs A.keys %x B.keys %x o1.keys %x o2.keys %x" % (A.keys.data_ptr(), B.keys.data_ptr(), o1.keys.data_ptr(),
                                                          o2.keys.data_ptr()))
