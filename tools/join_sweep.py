#!/usr/bin/env python3
"""A/B the join wave kernel's tuning knobs in ONE process, interleaved rounds
(cdna_hip_programming.md 5.4 rule 24).  GPU box only."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "go-crdt-playground_amd"))
import torch  # noqa: E402

import crdtgpu  # noqa: E402
from crdtgpu.batch import OutBuffers  # noqa: E402

n = int(os.environ.get("DOCS", 1 << 20))
dev = torch.device("cuda:0")
eng = crdtgpu.Engine(0)
eng.set_max_doc_entries(64)
A = OutBuffers(n, 2, n * 64, device=dev)
B = OutBuffers(n, 2, n * 64, device=dev)
eng.gen_pair_async(0x5EED, n, A, B)
o = OutBuffers(n, 2, 2 * n * 64, device=dev)
eng.sync()
a, b = A.as_batch(), B.as_batch()
Ks = [(int(k), int(nt)) for k in os.environ.get("KS", "1,2,4,8,16").split(",") for nt in os.environ.get("NT", "0,1").split(",")]
res = {k: [] for k in Ks}
s = torch.cuda.current_stream()
for rnd in range(int(os.environ.get("ROUNDS", 6))):
    for k in Ks:
        eng.set_option("join_docs_per_wave", k[0])
        eng.set_option("join_nt_stores", k[1])
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        eng.join_async(a, b, o, stream=s)
        e0.record(s)
        for _ in range(10):
            eng.join_async(a, b, o, stream=s)
        e1.record(s)
        e1.synchronize()
        res[k].append(e0.elapsed_time(e1) / 10)
eng.sync()
nout = int(o.counts.to(torch.int64).sum())
byt = 20 * (128 * n + nout) + 60 * n
for k in Ks:
    v = sorted(res[k])
    print("K=%-3d nt=%d median %.4f ms  min %.4f ms  -> %.0f GB/s (median)" % (k[0], k[1], v[len(v) // 2], v[0],
                                                                          byt / (v[len(v) // 2] / 1e3) / 1e9))
