"""GPU: the opt-in tombstone GC (crdt_tombstone_gc_async; the reference's
gcDeleted is an empty stub, awset-delta_test.go:67-77) and the elementwise
u64 min that computes a causally stable clock (crdt_vv_min_async), against the
C oracle (oracle_tomb_gc) and numpy.  The rule has no reference output to pin
it: parity here is with the restated rule (keep (k, x) unless
stable.HasDot(x), actor >= R kept)."""

import random

import numpy as np
import pytest

import crdtgpu
from crdtgpu.batch import TombBatch, TombBuffers
from oracle import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t

    assert t.cuda.is_available(), "GPU tests need a HIP device"
    return t


@pytest.fixture(scope="module")
def eng(torch):
    e = crdtgpu.Engine(0)
    yield e
    e.close()


def _i64(a, torch, dev):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).to(dev)


def test_vv_min(eng, torch):
    rng = np.random.default_rng(1)
    a = rng.integers(0, 2**64 - 1, 100_003, dtype=np.uint64)
    b = rng.integers(0, 2**64 - 1, 100_003, dtype=np.uint64)
    a[5], b[5] = np.uint64(2**63), np.uint64(2**63 - 1)  # unsigned order, not signed
    dev = torch.device("cuda:0")
    da, db = _i64(a, torch, dev), _i64(b, torch, dev)
    eng.vv_min_async(da, db, a.size)
    eng.sync()
    assert (da.cpu().numpy().view(np.uint64) == np.minimum(a, b)).all()


@pytest.mark.parametrize("R", [2, 8, 64])
def test_tombstone_gc_matches_oracle(eng, torch, R):
    rng = random.Random(R)
    per_doc, n = [], 4000
    for _ in range(n):
        keys = sorted(rng.sample(range(10 ** 6), rng.choice([0, 1, 3, 63, 64, 65, 300])))
        per_doc.append([(k, rng.randrange(R + 2), rng.randint(1, 50)) for k in keys])  # actors >= R kept
    tb = TombBatch.from_lists(per_doc)
    stable = np.array([rng.randint(0, 50) for _ in range(n * R)], dtype=np.uint64)
    rc, want = oracle.tomb_gc(tb, R, stable)
    assert rc == 0
    dev = torch.device("cuda:0")
    out = TombBuffers(n, int(tb.offsets[-1]), device=dev)
    eng.tombstone_gc_async(tb.to(dev), R, _i64(stable, torch, dev), out)
    eng.sync()
    got = TombBatch(*(t.cpu().numpy().view(np.uint32 if t.dtype == torch.int32 else np.uint64)
                      for t in (out.offsets, out.keys, out.actors, out.counters)),
                    counts=out.counts.cpu().numpy().view(np.uint32))
    assert (got.offsets == want.offsets).all()
    for d in range(n):
        assert got.doc(d) == want.doc(d), d
    # the rule itself, restated in numpy for a few docs
    for d in range(0, n, 397):
        keep = [(k, a, c) for k, a, c in per_doc[d] if not (a < R and stable[d * R + a] >= c)]
        assert want.doc(d) == keep
