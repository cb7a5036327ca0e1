"""GPU: the ingest sort (crdt_awset_sort_*, csrc/sort.hip) -- a producer that
packs Go maps (random iteration order, awset.go:55-59) hands each document's
entries over unsorted; the device orders them by key for the merge kernels.
Checked against numpy per document (empty, ragged, slack slots, 1 to 100,000
entries), the repeated-key error, and a sort -> join round trip against the C
oracle join of the pre-sorted batch."""

import random

import numpy as np
import pytest

import crdtgpu
from crdtgpu.batch import AWSetBatch, OutBuffers
from helpers import batch_of, random_state
from oracle import oracle
from test_gpu_parity import assert_same, host_out

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


def shuffled(b: AWSetBatch, rng) -> AWSetBatch:
    """The same batch with each doc's live entries in a random order (slack kept)."""
    keys, acts, cnts = b.keys.copy(), b.actors.copy(), b.counters.copy()
    for d in range(b.n_docs):
        o, n = int(b.offsets[d]), b.live(d)
        p = rng.permutation(n) + o
        keys[o:o + n], acts[o:o + n], cnts[o:o + n] = keys[p], acts[p], cnts[p]
    return AWSetBatch(b.R, b.offsets, keys, acts, cnts, b.vv, b.counts)


@pytest.mark.parametrize("slack", [0, 3])
def test_sort_random_docs(eng, slack):
    rng = random.Random(slack)
    nrng = np.random.default_rng(slack)
    R = 3
    docs = [random_state(rng, R, rng.choice([0, 1, 2, 63, 64, 65, 300, 5000]), 10 ** 9, 50) for _ in range(800)]
    b = batch_of(R, docs, slack=slack)
    got = eng.sort(shuffled(b, nrng))
    for d in range(b.n_docs):
        o, n = int(got.offsets[d]), int(got.counts[d])
        assert n == b.live(d)
        e = list(zip(got.keys[o:o + n].tolist(), got.actors[o:o + n].tolist(), got.counters[o:o + n].tolist()))
        assert e == b.doc(d)[0], d
        assert got.vv[d * R:(d + 1) * R].tolist() == b.doc(d)[1]


@pytest.mark.parametrize("universe", [600, 30_000, 10 ** 15, 2 ** 64])
def test_sort_key_widths_and_run_edges(eng, universe):
    """Every compare width of the in-register sort (keys spanning < 2^15 ids:
    32-bit packed; < 2^47: 64-bit packed; wider, up to the full u64 range:
    80-bit) and the run edges of both paths (64/128/256 in registers, 257+
    through the merge-path passes, 1 to 4 passes)."""
    rng = random.Random(universe % 1000 + 7)
    nrng = np.random.default_rng(universe % 1000 + 7)
    R = 2
    sizes = [0, 1, 63, 64, 65, 127, 128, 129, 255, 256, 257, 511, 512, 513, 1024, 1025, 2049, 4100]
    def state(n):
        if universe < 2 ** 62:
            return random_state(rng, R, min(n, universe), universe, 50)
        ks = {0, 2 ** 64 - 1} if n >= 2 else set()  # both ends of the key range
        while len(ks) < n:
            ks.add(rng.getrandbits(64))
        return [(k, rng.randint(0, R - 1), rng.randint(1, 50)) for k in sorted(ks)], [rng.randint(0, 50)] * R

    docs = [state(n) for n in sizes for _ in range(3)]
    b = batch_of(R, docs, slack=1)
    got = eng.sort(shuffled(b, nrng))
    for d in range(b.n_docs):
        o, n = int(got.offsets[d]), int(got.counts[d])
        assert n == b.live(d)
        e = list(zip(got.keys[o:o + n].tolist(), got.actors[o:o + n].tolist(), got.counters[o:o + n].tolist()))
        assert e == b.doc(d)[0], (d, n)


@pytest.mark.parametrize("n", [40, 200, 3000])
def test_sort_duplicate_in_each_path(eng, n):
    """A repeated key is found by the register path and the merge-path passes."""
    nrng = np.random.default_rng(n)
    keys = nrng.choice(np.arange(10 ** 6, dtype=np.uint64), n, replace=False)
    keys[n // 2] = keys[n // 3]
    b = AWSetBatch(2, np.array([0, n], np.uint32), keys, np.zeros(n, np.uint32), np.ones(n, np.uint64),
                   np.zeros(2, np.uint64))
    with pytest.raises(crdtgpu.CrdtError) as ei:
        eng.sort(b)
    assert ei.value.code == crdtgpu.CRDT_E_DUP_KEY


def test_sort_large_doc_and_duplicates(eng):
    nrng = np.random.default_rng(2)
    n = 100_000
    keys = np.sort(nrng.choice(np.arange(10 ** 7, dtype=np.uint64), n, replace=False))
    b = AWSetBatch(2, np.array([0, n], np.uint32), keys, nrng.integers(0, 2, n).astype(np.uint32),
                   nrng.integers(1, 99, n).astype(np.uint64), np.array([5, 7], np.uint64))
    got = eng.sort(shuffled(b, nrng))
    assert (got.keys[:n] == keys).all() and (got.actors[:n] == b.actors).all() and (got.counters[:n] == b.counters).all()
    dup = AWSetBatch(2, np.array([0, 3], np.uint32), np.array([4, 9, 4], np.uint64), np.zeros(3, np.uint32),
                     np.ones(3, np.uint64), np.zeros(2, np.uint64))
    with pytest.raises(crdtgpu.CrdtError) as ei:
        eng.sort(dup)
    assert ei.value.code == crdtgpu.CRDT_E_DUP_KEY


def test_sort_then_join_device(eng, torch):
    """Unsorted device-resident states -> ingest sort -> join: equals the oracle
    join of the sorted states."""
    rng = random.Random(3)
    nrng = np.random.default_rng(3)
    R = 2
    dst = batch_of(R, [random_state(rng, R, rng.randint(0, 90), 400, 9) for _ in range(2000)])
    src = batch_of(R, [random_state(rng, R, rng.randint(0, 90), 400, 9) for _ in range(2000)])
    rc, want = oracle.join(dst, src)
    assert rc == 0
    dev = torch.device("cuda:0")
    sd, ss = OutBuffers(dst.n_docs, R, int(dst.offsets[-1]), device=dev), OutBuffers(src.n_docs, R,
                                                                                     int(src.offsets[-1]), device=dev)
    eng.sort_async(shuffled(dst, nrng).to(dev), int(dst.offsets[-1]), sd)
    eng.sort_async(shuffled(src, nrng).to(dev), int(src.offsets[-1]), ss)
    out = OutBuffers(dst.n_docs, R, int(dst.offsets[-1]) + int(src.offsets[-1]), device=dev)
    eng.join_async(sd.as_batch(), ss.as_batch(), out)
    eng.sync()
    assert_same(host_out(out, torch), want, dst.n_docs, R)
