"""Shared generator for batched local-op cases (tests of crdt_awset_apply_*):
random replica states and op scripts, replayed through the map-based
restatement of the reference (oracle/awset_ref.py: AWSet.Add awset.go:89-94,
AWSet.Del :96-101, AWSetDelta.Del awset-delta_test.go:14-33) for the expected
result, and encoded as the engine's op batch."""

from __future__ import annotations

import random

import numpy as np

from crdtgpu import CRDT_OP_ADD, CRDT_OP_DEL, CRDT_OP_DELTA_DEL, CRDT_OP_DELTA_DEL_KEY
from crdtgpu.batch import AWSetBatch, OpBatch, TombBatch
from oracle import awset_ref as ref


def random_doc(rng: random.Random, R: int, n_state: int, n_tomb: int, universe: int, max_c: int):
    keys = sorted(rng.sample(range(universe), min(n_state, universe)))
    ents = [(k, rng.randrange(R), rng.randint(1, max_c)) for k in keys]
    tkeys = sorted(rng.sample(range(universe), min(n_tomb, universe)))
    tombs = [(k, rng.randrange(R), rng.randint(1, max_c)) for k in tkeys]
    vv = [rng.randint(0, max_c) for _ in range(R)]
    return ents, tombs, vv


def random_calls(rng: random.Random, n_ops: int, universe: int, keys_hint, p_ddel=0.3):
    """A call script of about n_ops ops: [('add'|'del'|'ddel', [keys])]."""
    calls, n = [], 0
    pool = list(keys_hint) or [0]
    while n < n_ops:
        kind = rng.choices(["add", "del", "ddel"], [0.45, 0.25, p_ddel])[0]
        m = rng.randint(0 if kind == "ddel" else 1, 4)
        ks = [rng.choice(pool) if rng.random() < 0.6 else rng.randrange(universe) for _ in range(m)]
        cost = m + (1 if kind == "ddel" else 0)
        if n + cost > n_ops:
            break
        calls.append((kind, ks))
        n += cost
        pool.extend(ks)
    return calls


def encode(calls):
    ops = []
    for kind, ks in calls:
        if kind == "add":
            ops += [(CRDT_OP_ADD, k) for k in ks]
        elif kind == "del":
            ops += [(CRDT_OP_DEL, k) for k in ks]
        else:
            ops.append((CRDT_OP_DELTA_DEL, 0))
            ops += [(CRDT_OP_DELTA_DEL_KEY, k) for k in ks]
    return ops


def replay(actor, R, ents, tombs, vv, calls):
    """Expected (entries, tombstones, vv) or the GoPanic the reference raises."""
    s = ref.AWSetDelta(actor, ref.VersionVector(list(vv)), {k: ref.Dot(a, c) for k, a, c in ents},
                       {k: ref.Dot(a, c) for k, a, c in tombs} if tombs else None)
    for kind, ks in calls:
        if kind == "add":
            s.Add(*ks)
        elif kind == "del":
            ref.AWSet.Del(s, *ks)
        else:
            s.Del(*ks)
    e = sorted((k, d.actor, d.counter) for k, d in s.Entries.items())
    t = sorted((k, d.actor, d.counter) for k, d in (s.Deleted or {}).items())
    return e, t, list(s.VersionVector)


def make_case(rng, n_docs, R, state_size, ops_size, universe=300, max_c=40, tomb_size=None, panic_rate=0.0):
    """(state batch, tomb batch, op batch, expected per doc: (entries, tombs, vv) or None on panic)."""
    docs, tombs, per_ops, actors, want = [], [], [], [], []
    for _ in range(n_docs):
        ents, tb, vv = random_doc(rng, R, state_size(), tomb_size() if tomb_size else rng.randint(0, 3), universe,
                                  max_c)
        actor = R if rng.random() < panic_rate else rng.randrange(R)
        calls = random_calls(rng, ops_size(), universe, [k for k, _, _ in ents])
        try:
            w = replay(actor, R, ents, tb, vv, calls)
        except ref.GoPanic:
            w = None
        docs.append((ents, vv))
        tombs.append(tb)
        per_ops.append(encode(calls))
        actors.append(actor)
        want.append(w)
    return AWSetBatch.from_docs(R, docs), TombBatch.from_lists(tombs), OpBatch.from_lists(per_ops, actors), want


def doc_of(out, tout, d, R):
    o, n = int(out.offsets[d]), int(out.counts[d])
    e = list(zip(out.keys[o:o + n].tolist(), out.actors[o:o + n].tolist(), out.counters[o:o + n].tolist()))
    t = tout.doc(d) if tout is not None else []
    return e, t, [int(x) for x in out.vv[d * R:(d + 1) * R]]


def outputs_equal(a, b):
    """Bit-exact comparison of two apply outputs ((out, tout) pairs) over all docs and arrays."""
    (oa, ta), (ob, tb) = a, b
    for f in ("offsets", "counts", "vv"):
        if not (np.asarray(getattr(oa, f)) == np.asarray(getattr(ob, f))).all():
            return f
    for f in ("offsets", "counts"):
        if not (np.asarray(getattr(ta, f)) == np.asarray(getattr(tb, f))).all():
            return "tomb " + f
    return None
