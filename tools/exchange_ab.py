#!/usr/bin/env python3
"""A/B of the config-2 exchange's forms in ONE process, interleaved rounds:
LDS-staged contiguous stores vs lane-scattered stores ("join_stage_stores"),
one shared key column for the two outputs or one each, and the block order
("join_slab_blocks_per_cu": 0 = in order; FORMS env: "stage,shared,slab;...").  Prints the median launch time, the HBM bytes each form
writes, and whether every form's outputs equal the first form's (live entries,
counts, VVs).  Also the box's copy and 3:4 mix probes.  GPU box only."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "go-crdt-playground_amd"))
import torch  # noqa: E402

import crdtgpu  # noqa: E402
from crdtgpu import abi  # noqa: E402
from crdtgpu.batch import OutBuffers  # noqa: E402

n = int(os.environ.get("DOCS", 1 << 20))
rounds = int(os.environ.get("ROUNDS", 8))
dev = torch.device("cuda:0")
eng = crdtgpu.Engine(0)
eng.set_max_doc_entries(64)
A, B = OutBuffers(n, 2, n * 64, device=dev), OutBuffers(n, 2, n * 64, device=dev)
eng.gen_pair_async(0x5EED, n, A, B)
a, b = A.as_batch(), B.as_batch()
o1 = OutBuffers(n, 2, 2 * n * 64, device=dev)
o2 = OutBuffers(n, 2, 2 * n * 64, device=dev)
o2s = OutBuffers(n, 2, 2 * n * 64, device=dev, shared_keys=o1)
s = torch.cuda.current_stream()
_DEF = (1, 1, 0, 8, 1)
forms = [tuple([int(x) for x in f.split(",")] + list(_DEF[len(f.split(",")):]))
         for f in os.environ.get("FORMS", "1,1,0;1,1,7;1,1,14;1,1,4;1,0,0;1,0,7").split(";")]


def run(form, reps):
    eng.set_option("join_stage_stores", form[0])
    eng.set_option("join_slab_blocks_per_cu", form[2])
    eng.set_option("join_docs_per_wave", form[3])
    eng.set_option("join_nt_stores", form[4])
    eng.exchange_async(a, b, o1, o2s if form[1] else o2, stream=s)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        eng.exchange_async(a, b, o1, o2s if form[1] else o2, stream=s)
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / max(reps, 1)


def snapshot(form):
    for t in (o1.keys, o1.actors, o1.counters, o2.keys, o2.actors, o2.counters, o2s.actors, o2s.counters):
        t.fill_(-1)
    run(form, 0)
    eng.sync()
    q = o2s if form[1] else o2
    cnt = o1.counts.to(torch.int64)
    live = torch.zeros(2 * n * 64, dtype=torch.bool, device=dev)
    offs = o1.offsets[:n].to(torch.int64)
    idx = torch.arange(128, device=dev).view(1, 128)
    m = idx < cnt.view(n, 1)
    live[(offs.view(n, 1) + idx)[m]] = True
    return [o1.counts.clone(), o1.vv.clone(), q.counts.clone(), q.vv.clone(), o1.keys[live].clone(),
            o1.actors[live].clone(), o1.counters[live].clone(), q.keys[live].clone(), q.actors[live].clone(),
            q.counters[live].clone()], int(cnt.sum())


ref, n_out = snapshot(forms[0])
same = {}
for f in forms:
    got, _ = snapshot(f)
    same[f] = all(bool(torch.equal(x, y)) for x, y in zip(ref, got))
    del got
res = {f: [] for f in forms}
for _ in range(rounds):
    for f in forms:
        res[f].append(run(f, 20))
eng.sync()
n_in = int(A.counts.to(torch.int64).sum()) + int(B.counts.to(torch.int64).sum())
for f in forms:
    v = sorted(res[f])
    med = v[len(v) // 2]
    # bytes: inputs 20 B/entry, out1 20 B/entry, out2 20 (own keys) or 12 B/entry, VVs/offsets/counts
    byt = 20 * n_in + (20 + (12 if f[1] else 20)) * n_out + n * (2 * 2 * 8 + 2 * 2 * 8 + 2 * 8 + 2 * 8)
    print("stage=%d shared_keys=%d slab=%-2d K=%-2d nt=%d median %.4f ms  min %.4f ms  %.0f GB/s algorithmic (%.3f GB)  "
          "same=%s" % (f[0], f[1], f[2], f[3], f[4], med, v[0], byt / med / 1e6, byt / 1e9, same[f]))
eng.set_option("join_stage_stores", 1)
eng.set_option("join_slab_blocks_per_cu", 0)
eng.set_option("join_docs_per_wave", 8)
eng.set_option("join_nt_stores", 1)
del o1, o2, o2s, A, B
torch.cuda.empty_cache()
x = torch.empty(2 << 30, dtype=torch.uint8, device=dev)
y = torch.empty(2 << 30, dtype=torch.uint8, device=dev)
x.fill_(0x5A)
for bpc in (8, 16, 32):
    eng.set_option("probe_blocks_per_cu", bpc)
    print("probe bpc=%d copy_nt %.0f mix_nt %.0f mix_plain %.0f write_nt %.0f read %.0f GB/s" % (
        bpc, eng.bw_probe(abi.CRDT_PROBE_COPY, x, y, 2 << 30, 10), eng.bw_probe(abi.CRDT_PROBE_MIX, x, y, 2 << 30, 10),
        eng.bw_probe(abi.CRDT_PROBE_MIX_PLAIN, x, y, 2 << 30, 10), eng.bw_probe(abi.CRDT_PROBE_WRITE, None, y, 2 << 30, 10),
        eng.bw_probe(abi.CRDT_PROBE_READ, x, y, 2 << 30, 10)))
