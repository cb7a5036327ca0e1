"""GPU parity of the large-document join path (csrc/tile.hip): merge-path tiles
of 2048 merged positions spread one document over many workgroups, with a
decoupled look-back placing each tile's survivors (awset.go:103-161 applied to
documents of up to 2^20 entries per side).

Bit-exact vs the C oracle (oracle/awset_oracle.c) on: tile boundaries that
split a common key's (dst, src) pair, documents of 1 to 2^20 entries, the
exchange (both directions from one read), tile workspaces smaller than the
call's tiles (passes of `join_tile_capacity` tiles, a document straddling
them), the fallback to the per-document block kernel past the last pass, and
all 16,384 documents of BASELINE config 4 in both directions, in one pass and
in three.
"""

import random

import numpy as np
import pytest

from crdtgpu.batch import AWSetBatch, OutBuffers
from helpers import batch_of, random_state
from oracle import oracle
from test_gpu_parity import assert_same, assert_same_all, gen_zipf, host_out

pytestmark = pytest.mark.gpu

TILE = 2048


@pytest.fixture(scope="module")
def torch():
    import torch as t

    assert t.cuda.is_available(), "GPU tests need a HIP device"
    return t


@pytest.fixture(scope="module")
def eng(torch):
    import crdtgpu

    e = crdtgpu.Engine(0)
    yield e
    e.close()


# every tile shape (threads x positions; look-back per tile or deferred by one)
# must give the same bits
SHAPES = [9, 0, 1, 2, 3, 4, 5, 6, 7, 8]


@pytest.fixture(params=SHAPES, ids=lambda s: "shape%d" % s)
def shaped(eng, request):
    eng.set_option("join_tile_shape", request.param)
    yield eng
    eng.set_option("join_tile_shape", DEFAULT_SHAPE)


DEFAULT_SHAPE = 9


def interleaved(rng, n, R, share):
    """Two states over one key range: a fraction `share` of dst's keys also in
    src, so common pairs fall on every tile boundary sooner or later."""
    base = sorted(rng.sample(range(0, n * 6), n))
    dk = base
    sk = sorted(set(k for k in base if rng.random() < share) |
                set(rng.sample(range(n * 6, n * 6 + n * 4), max(0, n - int(n * share)))))[:n]

    def ent(keys):
        return [(k, rng.randrange(R), rng.randint(1, 40)) for k in keys]

    vv = lambda: [rng.randint(0, 40) for _ in range(R)]  # noqa: E731
    return (ent(dk), vv()), (ent(sk), vv())


def check_join_and_exchange(eng, dst, src, R):
    rc, want = oracle.join(dst, src)
    assert rc == 0
    assert_same(eng.join(dst, src), want, dst.n_docs, R)
    rc2, want2 = oracle.join(src, dst)
    assert rc2 == 0
    o1, o2 = eng.exchange(dst, src)
    assert_same(o1, want, dst.n_docs, R)
    assert_same(o2, want2, dst.n_docs, R)


@pytest.mark.parametrize("n", [TILE // 2 - 1, TILE // 2, TILE // 2 + 1, TILE - 1, TILE, TILE + 1, 3 * TILE + 7])
def test_tile_boundaries_split_common_pairs(shaped, n):
    """Sizes around multiples of the tile; common keys everywhere; both HasDot
    sides live (dots above and below the other side's clock)."""
    rng = random.Random(n)
    R = 3
    docs_d, docs_s = [], []
    for _ in range(6):
        d, s = interleaved(rng, n, R, rng.choice([0.3, 0.9, 1.0]))
        docs_d.append(d)
        docs_s.append(s)
    dst, src = batch_of(R, docs_d), batch_of(R, docs_s)
    check_join_and_exchange(shaped, dst, src, R)


def test_tile_equal_key_sets(shaped):
    """Identical key sets: every dst element is followed by its src twin, so the
    merge path cuts between twins at every odd tile boundary."""
    rng = random.Random(5)
    R = 2
    docs_d, docs_s = [], []
    for n in (TILE // 2 + 1, 5 * TILE + 3, 40000):
        keys = sorted(rng.sample(range(10 ** 9), n))
        docs_d.append(([(k, rng.randrange(2), rng.randint(1, 9)) for k in keys], [5, 5]))
        docs_s.append(([(k, rng.randrange(2), rng.randint(1, 9)) for k in keys], [4, 6]))
    check_join_and_exchange(shaped, batch_of(R, docs_d), batch_of(R, docs_s), R)


def test_tile_disjoint_key_ranges(shaped):
    """Every dst key below every src key, and the reverse: the merge path runs
    along one run and then the other, so each tile's split is as far as it gets
    from the proportional guess the plan's galloping search starts from
    (tile.hip, merge_path_gallop)."""
    rng = random.Random(11)
    R = 2
    docs_d, docs_s = [], []
    for nd, ns in ((3 * TILE + 5, 9000), (9000, 3 * TILE + 5), (TILE + 1, 40000), (70, 5 * TILE)):
        lo = sorted(rng.sample(range(0, 10 ** 6), nd))
        hi = sorted(rng.sample(range(2 * 10 ** 6, 3 * 10 ** 6), ns))
        ent = lambda keys: [(k, rng.randrange(R), rng.randint(1, 9)) for k in keys]  # noqa: E731
        flip = len(docs_d) % 2 == 1
        docs_d.append((ent(hi if flip else lo), [5, 5]))
        docs_s.append((ent(lo if flip else hi), [4, 6]))
    check_join_and_exchange(shaped, batch_of(R, docs_d), batch_of(R, docs_s), R)


def test_tile_mixed_with_small_docs_and_slack(shaped, torch):
    """Small (wave path) and large (tile path) documents in one batch, counts <
    slots on both inputs, device-resident through the async ABI."""
    rng = random.Random(7)
    R = 4
    sz = lambda: rng.choice([0, 3, 64, 65, 2047, 2048, 2049, 9000])  # noqa: E731
    dsts = [random_state(rng, R, sz(), 30000, 25) for _ in range(300)]
    srcs = [random_state(rng, R, sz(), 30000, 25) for _ in range(300)]
    dst, src = batch_of(R, dsts, slack=5), batch_of(R, srcs, slack=2)
    rc, want = oracle.join(dst, src)
    assert rc == 0
    dev = torch.device("cuda:0")
    out = OutBuffers(dst.n_docs, R, int(dst.offsets[-1]) + int(src.offsets[-1]), device=dev)
    shaped.join_async(dst.to(dev), src.to(dev), out)
    shaped.sync()
    assert_same(host_out(out, torch), want, dst.n_docs, R)


def test_tile_one_document_of_a_million(shaped):
    """One 2^20 + 2^20 document (1,024 tiles in one look-back chain)."""
    rng = np.random.default_rng(9)
    R = 2
    n = 1 << 20
    univ = rng.choice(np.arange(3 * n, dtype=np.uint64), size=int(1.5 * n), replace=False)
    univ.sort()
    pick = lambda: np.sort(rng.choice(univ, size=n, replace=False))  # noqa: E731

    def side(keys):
        return AWSetBatch(R, np.array([0, n], dtype=np.uint32), keys.astype(np.uint64),
                          rng.integers(0, 2, n).astype(np.uint32), rng.integers(1, 1000, n).astype(np.uint64),
                          rng.integers(0, 1000, R).astype(np.uint64))

    a, b = side(pick()), side(pick())
    check_join_and_exchange(shaped, a, b, R)


def host_tiles(a, b, tile=TILE // 2):
    """Tiles a join of host batches a <- b has (tile.hip: ceil((nd + ns) / T) per
    document with more than 64 live entries on a side; T = 1024 for the default
    shape)."""
    nd = np.array([a.live(d) for d in range(a.n_docs)], dtype=np.int64)
    ns = np.array([b.live(d) for d in range(b.n_docs)], dtype=np.int64)
    big = (nd > 64) | (ns > 64)
    return int(((nd + ns + tile - 1) // tile)[big].sum())


def test_tile_fallback_and_switch(eng):
    """More tiles than tile_max_passes x join_tile_capacity -> the per-document
    block kernel; join_tiles=0 -> block kernel always.  Same results either way."""
    rng = random.Random(8)
    R = 2
    dsts = [random_state(rng, R, rng.choice([100, 5000, 9000]), 20000, 20) for _ in range(40)]
    srcs = [random_state(rng, R, rng.choice([100, 5000, 9000]), 20000, 20) for _ in range(40)]
    dst, src = batch_of(R, dsts), batch_of(R, srcs)
    assert host_tiles(dst, src) > 3
    rc, want = oracle.join(dst, src)
    assert rc == 0
    try:
        eng.set_option("join_tile_capacity", 3)
        eng.set_option("join_tile_max_passes", 1)
        assert_same(eng.join(dst, src), want, dst.n_docs, R)
        rc, want2 = oracle.join(src, dst)
        assert rc == 0
        o1, o2 = eng.exchange(dst, src)  # both block-kernel passes (their own dequeue heads)
        assert_same(o1, want, dst.n_docs, R)
        assert_same(o2, want2, dst.n_docs, R)
        eng.set_option("join_tile_capacity", 1 << 22)
        eng.set_option("join_tile_max_passes", 256)
        eng.set_option("join_tiles", 0)
        assert_same(eng.join(dst, src), want, dst.n_docs, R)
    finally:
        eng.set_option("join_tiles", 1)
        eng.set_option("join_tile_capacity", 1 << 22)
        eng.set_option("join_tile_max_passes", 256)
    assert_same(eng.join(dst, src), want, dst.n_docs, R)


@pytest.mark.parametrize("cap", [1, 3, 7, 64])
def test_tile_passes_small_capacity(eng, cap):
    """A workspace of `cap` tiles: the tile path runs ceil(tiles / cap) passes
    (tile.hip, launch_join_tiles), and a pass ends inside a document whenever
    one straddles it -- cap 1 makes every tile its own pass, so every later
    tile of a document takes its placed count from the carry word instead of a
    look-back.  Join and exchange, host path (exact tile count), bit-exact."""
    rng = random.Random(100 + cap)
    R = 3
    sz = lambda: rng.choice([0, 5, 64, 65, 1023, 1024, 2049, 7000])  # noqa: E731
    dsts = [random_state(rng, R, sz(), 40000, 20) for _ in range(60)]
    srcs = [random_state(rng, R, sz(), 40000, 20) for _ in range(60)]
    dst, src = batch_of(R, dsts), batch_of(R, srcs)
    tiles = host_tiles(dst, src)
    assert tiles >= 2 * cap
    try:
        eng.set_option("join_tile_capacity", cap)
        eng.set_option("join_tile_max_passes", 4096)
        check_join_and_exchange(eng, dst, src, R)
    finally:
        eng.set_option("join_tile_capacity", 1 << 22)
        eng.set_option("join_tile_max_passes", 256)


def test_tile_passes_one_document_many_passes(eng, torch):
    """One 2^17 + 2^17 document (256 tiles) in passes of 37 tiles, device-resident
    through the async ABI (passes bounded from the batch size, most of them past
    the call's tiles and returning at once): the carry crosses six pass
    boundaries inside the document."""
    rng = np.random.default_rng(12)
    R = 2
    n = 1 << 17
    univ = np.sort(rng.choice(np.arange(3 * n, dtype=np.uint64), size=int(1.5 * n), replace=False))
    pick = lambda: np.sort(rng.choice(univ, size=n, replace=False))  # noqa: E731

    def side(keys):
        return AWSetBatch(R, np.array([0, n], dtype=np.uint32), keys.astype(np.uint64),
                          rng.integers(0, 2, n).astype(np.uint32), rng.integers(1, 1000, n).astype(np.uint64),
                          rng.integers(0, 1000, R).astype(np.uint64))

    a, b = side(pick()), side(pick())
    rc, want = oracle.join(a, b)
    assert rc == 0
    rc, want2 = oracle.join(b, a)
    assert rc == 0
    dev = torch.device("cuda:0")
    try:
        eng.set_option("join_tile_capacity", 37)
        eng.set_option("join_tile_max_passes", 65536)
        eng.set_max_doc_entries(n)  # (the async bound then counts passes from the promise)
        da, db = a.to(dev), b.to(dev)
        o1 = OutBuffers(1, R, 2 * n, device=dev)
        o2 = OutBuffers(1, R, 2 * n, device=dev)
        eng.exchange_async(da, db, o1, o2)
        eng.sync()
    finally:
        eng.set_option("join_tile_capacity", 1 << 22)
        eng.set_option("join_tile_max_passes", 256)
        eng.set_max_doc_entries()
    assert_same(host_out(o1, torch), want, 1, R)
    assert_same(host_out(o2, torch), want2, 1, R)


@pytest.mark.parametrize("dispensers", [1, 8])
def test_tile_dispensers(eng, dispensers):
    """The tile dispenser as one word or sharded over eight (tile.hip,
    tile_take): the same bits, on documents of many tiles next to small ones."""
    rng = random.Random(9)
    R = 3
    sz = lambda: rng.choice([5, 64, 300, 2047, 2049, 9000, 40000])  # noqa: E731
    dsts = [random_state(rng, R, sz(), 90000, 30) for _ in range(48)]
    srcs = [random_state(rng, R, sz(), 90000, 30) for _ in range(48)]
    dst, src = batch_of(R, dsts), batch_of(R, srcs)
    try:
        eng.set_option("join_tile_dispensers", dispensers)
        check_join_and_exchange(eng, dst, src, R)
    finally:
        eng.set_option("join_tile_dispensers", 8)


def _sub(h, d0, d1, R):
    """Host sub-batch of docs [d0, d1), offsets rebased."""
    o = np.asarray(h.offsets).astype(np.int64)
    lo, hi = int(o[d0]), int(o[d1])
    return AWSetBatch(R, (o[d0:d1 + 1] - lo).astype(np.uint32), h.keys[lo:hi], h.actors[lo:hi], h.counters[lo:hi],
                      h.vv[d0 * R:d1 * R], None if h.counts is None else h.counts[d0:d1])


@pytest.mark.parametrize("cap", [1 << 22, 300_000], ids=["one_pass", "three_passes"])
def test_config4_full_size_exchange(eng, torch, cap):
    """BASELINE config 4 at its stated size: 16,384 docs, Zipf(1.1) sizes up to
    2^20, 50% concurrent add/remove conflicts, R = 2.  The exchange writes
    A<-B and B<-A; every document of both is compared with the oracle (in
    chunks of documents, so the host copy stays bounded).  Also with a tile
    workspace of 300,000 tiles, below the call's 780,811: three passes."""
    n = 16384
    R = 2
    A, B, total = gen_zipf(eng, torch, n)
    dev = torch.device("cuda:0")
    oab = OutBuffers(n, R, 2 * total, device=dev)
    oba = OutBuffers(n, R, 2 * total, device=dev)
    try:
        eng.set_option("join_tile_capacity", cap)
        eng.exchange_async(A.as_batch(), B.as_batch(), oab, oba)
        eng.sync()
    finally:
        eng.set_option("join_tile_capacity", 1 << 22)
    ha, hb = host_out(A, torch).as_batch(), host_out(B, torch).as_batch()
    del A, B
    if cap < (1 << 22):
        assert host_tiles(ha, hb) > 2 * cap  # at least three passes
    for o, (x, y) in ((oab, (ha, hb)), (oba, (hb, ha))):
        ho = host_out(o, torch)
        oo = np.asarray(ho.offsets).astype(np.int64)
        bounds = list(range(0, n, 2048)) + [n]
        for d0, d1 in zip(bounds[:-1], bounds[1:]):
            rc, want = oracle.join(_sub(x, d0, d1, R), _sub(y, d0, d1, R))
            assert rc == 0
            lo, hi = int(oo[d0]), int(oo[d1])
            got = OutBuffers(d1 - d0, R, 0)
            got.offsets = (oo[d0:d1 + 1] - lo).astype(np.uint32)
            got.counts = ho.counts[d0:d1]
            got.keys, got.actors, got.counters = ho.keys[lo:hi], ho.actors[lo:hi], ho.counters[lo:hi]
            got.vv = ho.vv[d0 * R:d1 * R]
            assert_same_all(got, want, d1 - d0, R)
        del ho
