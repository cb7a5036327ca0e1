"""GPU parity: the HIP kernels, called through the C ABI, against the C oracle.

Bit-exact on every document: entries (keys, dot actors, dot counters), live
counts, slot bounds and version vectors.  Covers the wave path (<= 64 entries
per side), the block path (larger documents), empty and ragged documents, the
64/65 boundary, the actor == len(vv) panic, ordered AWSet folds, AWSetDelta
folds (first contact, pruning, no-op, tombstones, re-adds, LDS overflow
hand-off), the device-side workload generator, and the config-2 size with
size-independent properties.
"""

import json
import random

import numpy as np
import pytest

import crdtgpu
from crdtgpu import CRDT_FOLD_AWSET, CRDT_FOLD_DELTA, workloads
from crdtgpu.batch import AWSetBatch, OutBuffers, SrcBatch, SrcBuffers
from helpers import GOLDEN, batch_of, out_doc, outs_equal, random_state, snap_entries, src_batch_of
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


def host_out(out, torch):
    torch.cuda.synchronize()
    h = OutBuffers(out.n_docs, out.R, 0)
    for f in ("offsets", "counts", "keys", "actors", "counters", "vv"):
        a = getattr(out, f).cpu().numpy()
        setattr(h, f, a.view(np.uint32 if a.dtype == np.int32 else np.uint64))
    return h


def assert_same(got, want, n_docs, R):
    bad = outs_equal(got, want, n_docs, R)
    if bad is not None:
        raise AssertionError("doc %s differs:\n gpu    %s\n oracle %s" % (
            bad, out_doc(got, bad, R) if bad >= 0 else got.offsets[:8],
            out_doc(want, bad, R) if bad >= 0 else want.offsets[:8]))


def assert_same_all(got, want, n_docs, R):
    """Vectorised bit-exact comparison of two outputs over every document."""
    assert (np.asarray(got.offsets[: n_docs + 1]) == np.asarray(want.offsets[: n_docs + 1])).all(), "offsets"
    assert (np.asarray(got.counts[:n_docs]) == np.asarray(want.counts[:n_docs])).all(), "counts"
    assert (np.asarray(got.vv[: n_docs * R]) == np.asarray(want.vv[: n_docs * R])).all(), "vv"
    cnt = np.asarray(want.counts[:n_docs]).astype(np.int64)
    starts = np.asarray(want.offsets[:n_docs]).astype(np.int64)
    idx = np.repeat(starts, cnt) + (np.arange(cnt.sum()) - np.repeat(np.cumsum(cnt) - cnt, cnt))
    for f in ("keys", "actors", "counters"):
        g, w = np.asarray(getattr(got, f))[idx], np.asarray(getattr(want, f))[idx]
        if not (g == w).all():
            bad = int(np.nonzero(g != w)[0][0])
            doc = int(np.searchsorted(np.cumsum(cnt), bad, side="right"))
            raise AssertionError("%s differ first at doc %d" % (f, doc))


def join_case(rng, n_docs, R, size_fn, universe, max_c, actor_hi=None):
    dsts, srcs = [], []
    for _ in range(n_docs):
        dsts.append(random_state(rng, R, size_fn(), universe, max_c, actor_hi))
        srcs.append(random_state(rng, R, size_fn(), universe, max_c, actor_hi))
    return batch_of(R, dsts), batch_of(R, srcs)


# ---------------------------------------------------------------- golden

def test_golden_merges_on_gpu(eng):
    g = json.load(open(GOLDEN))
    n = 0
    for sc in g["scenarios"]:
        for m in sc["merges"]:
            keys = sorted({e[0] for s in (m["dst"], m["src"], m["out"]) for e in s["entries"] + s.get("deleted", [])})
            ids = {k: i for i, k in enumerate(keys)}
            R = len(m["dst"]["vv"])
            dst = batch_of(R, [(snap_entries(m["dst"], ids), m["dst"]["vv"])])
            if sc["kind"] == "awset":
                out = eng.join(dst, batch_of(R, [(snap_entries(m["src"], ids), m["src"]["vv"])]))
            else:
                s = m["src"]
                dele = sorted((ids[k], a, c) for k, a, c in s["deleted"])
                out = eng.fold(CRDT_FOLD_DELTA, dst, src_batch_of(R, [[(s["actor"], s["vv"], snap_entries(s, ids),
                                                                        dele)]]))
            e, vv = out_doc(out, 0, R)
            assert e == snap_entries(m["out"], ids), (sc["name"], m["dst_name"], m["src_name"])
            assert vv == m["out"]["vv"]
            n += 1
    assert n == 23


# ---------------------------------------------------------------- join

@pytest.mark.parametrize("R,maxn,universe", [(2, 64, 100), (3, 64, 70), (16, 40, 200), (64, 64, 128)])
def test_join_wave_path_random(eng, R, maxn, universe):
    rng = random.Random(R * 1000 + maxn)
    dst, src = join_case(rng, 3000, R, lambda: rng.randint(0, maxn), universe, 9)
    rc, want = oracle.join(dst, src)
    assert rc == 0
    assert_same(eng.join(dst, src), want, dst.n_docs, R)


def test_join_boundary_sizes(eng):
    rng = random.Random(11)
    R = 2
    sizes = [(0, 0), (0, 64), (64, 0), (64, 64), (63, 64), (64, 65), (65, 64), (65, 65), (1, 200), (200, 1),
             (128, 0), (0, 129), (1000, 1000), (4097, 10), (3, 5000)]
    dsts = [random_state(rng, R, a, 12000, 20) for a, _ in sizes]
    srcs = [random_state(rng, R, b, 12000, 20) for _, b in sizes]
    dst, src = batch_of(R, dsts), batch_of(R, srcs)
    rc, want = oracle.join(dst, src)
    assert rc == 0
    assert_same(eng.join(dst, src), want, dst.n_docs, R)


def test_join_block_path_large_random(eng):
    rng = random.Random(12)
    R = 4
    dst, src = join_case(rng, 64, R, lambda: rng.choice([65, 300, 1023, 1024, 1025, 2500, 7000]), 20000, 30)
    rc, want = oracle.join(dst, src)
    assert rc == 0
    assert_same(eng.join(dst, src), want, dst.n_docs, R)


def test_join_mixed_sizes_device_async(eng, torch):
    """Device-resident inputs with counts < slots (slack), through the async ABI."""
    rng = random.Random(13)
    R = 2
    sz = lambda: rng.choice([0, 1, 7, 33, 64, 64, 65, 150])  # noqa: E731
    dsts = [random_state(rng, R, sz(), 400, 12) for _ in range(2000)]
    srcs = [random_state(rng, R, sz(), 400, 12) for _ in range(2000)]
    dst, src = batch_of(R, dsts, slack=3), batch_of(R, srcs, slack=1)
    rc, want = oracle.join(dst, src)
    assert rc == 0
    dev = torch.device("cuda:0")
    dd, ds = dst.to(dev), src.to(dev)
    out = OutBuffers(dst.n_docs, R, int(dst.offsets[-1]) + int(src.offsets[-1]), device=dev)
    s = torch.cuda.current_stream()
    eng.join_async(dd, ds, out, stream=s)
    eng.sync(s)
    assert_same(host_out(out, torch), want, dst.n_docs, R)


def test_join_actor_range_error(eng):
    R = 2
    dst = batch_of(R, [([(1, 0, 1)], [1, 0]), ([(1, 2, 1)], [1, 1])])
    src = batch_of(R, [([], [0, 0]), ([], [1, 1])])
    with pytest.raises(crdtgpu.CrdtError) as ei:
        eng.join(dst, src)
    assert ei.value.code == crdtgpu.CRDT_E_ACTOR_RANGE
    # the status is cleared afterwards, and actor > R is legal ("never seen")
    rc, want = oracle.join(batch_of(R, [([(1, 5, 1)], [1, 1])]), batch_of(R, [([], [1, 1])]))
    got = eng.join(batch_of(R, [([(1, 5, 1)], [1, 1])]), batch_of(R, [([], [1, 1])]))
    assert rc == 0
    assert_same(got, want, 1, R)


def test_join_actor_range_error_block_path(eng):
    R = 2
    big = [(k, 0, 1) for k in range(100)] + [(1000, 2, 1)]
    with pytest.raises(crdtgpu.CrdtError) as ei:
        eng.join(batch_of(R, [(big, [1, 0])]), batch_of(R, [([], [5, 5])]))
    assert ei.value.code == crdtgpu.CRDT_E_ACTOR_RANGE


# ---------------------------------------------------------------- fold

def fold_case(rng, n_docs, R, dst_n, n_src, src_n, tomb_n, universe, max_c, delta):
    dsts, per_doc = [], []
    for _ in range(n_docs):
        dsts.append(random_state(rng, R, dst_n(), universe, max_c))
        chain = []
        for _ in range(n_src()):
            e, vv = random_state(rng, R, src_n(), universe, max_c)
            t = random_state(rng, R, tomb_n(), universe, max_c)[0] if delta else []
            chain.append((rng.randrange(R), vv, e, t))
        per_doc.append(chain)
    return batch_of(R, dsts), src_batch_of(R, per_doc)


@pytest.mark.parametrize("mode", [CRDT_FOLD_AWSET, CRDT_FOLD_DELTA])
def test_fold_wave_path_random(eng, mode):
    rng = random.Random(20 + mode)
    R = 4
    dst, srcs = fold_case(rng, 3000, R, lambda: rng.randint(0, 64), lambda: rng.randint(0, 10),
                          lambda: rng.randint(0, 8), lambda: rng.randint(0, 3), 120, 8, mode == CRDT_FOLD_DELTA)
    rc, want = oracle.fold(mode, dst, srcs)
    assert rc == 0
    assert_same(eng.fold(mode, dst, srcs), want, dst.n_docs, R)


@pytest.mark.parametrize("universe,max_src", [(16, 4), (40, 15), (64, 15), (64, 16), (65, 8)])
@pytest.mark.parametrize("mode", [CRDT_FOLD_AWSET, CRDT_FOLD_DELTA])
def test_fold_dense_key_spans(eng, mode, universe, max_src):
    """Documents whose keys span few ids -- the per-slot AWSet walk (span < 64,
    <= 15 sources) and the counting sort (span < 256) -- at and around their
    limits (64 ids, 15/16 sources, 65 ids fall back), with entries that cover
    or not the clocks so that adds, skips, removals and src-wins all occur."""
    rng = random.Random(universe * 100 + max_src + mode)
    R = 4
    dst, srcs = fold_case(rng, 4000, R, lambda: rng.randint(0, min(universe, 60)), lambda: rng.randint(0, max_src),
                          lambda: rng.randint(0, min(universe, 12)), lambda: rng.randint(0, 3), universe, 9,
                          mode == CRDT_FOLD_DELTA)
    rc, want = oracle.fold(mode, dst, srcs)
    assert rc == 0
    assert_same(eng.fold(mode, dst, srcs), want, dst.n_docs, R)


@pytest.mark.parametrize("mode", [CRDT_FOLD_AWSET, CRDT_FOLD_DELTA])
def test_fold_block_path_and_overflow(eng, mode):
    """Docs that start above CAP, grow above CAP mid-fold, or carry > 64 entries/tombstones per source."""
    rng = random.Random(30 + mode)
    R = 3
    dst, srcs = fold_case(rng, 200, R, lambda: rng.choice([10, 100, 127, 128, 129, 600]), lambda: rng.randint(0, 6),
                          lambda: rng.choice([5, 40, 64, 65, 300]), lambda: rng.choice([0, 2, 64, 65, 200]), 5000, 50,
                          mode == CRDT_FOLD_DELTA)
    rc, want = oracle.fold(mode, dst, srcs)
    assert rc == 0
    assert_same(eng.fold(mode, dst, srcs), want, dst.n_docs, R)


@pytest.mark.parametrize("mode", [CRDT_FOLD_AWSET, CRDT_FOLD_DELTA])
def test_fold_wide_key_spans(eng, mode):
    """The in-register sort packs (key, tag) into 32 bits when a document's keys
    lie within 2^15 of its first kept key, into 64 bits within 2^47, and falls
    back to the 80-bit comparison beyond: every tier, mixed in one batch, and
    keys at both ends of the u64 range."""
    rng = random.Random(40 + mode)
    R = 4
    delta = mode == CRDT_FOLD_DELTA
    top = (1 << 64) - 1
    # per-document monotone key maps: dense, spread beyond 2^16, beyond 2^48, the whole range
    maps = [lambda k: k, lambda k: (1 << 40) + k * 1021, lambda k: (1 << 62) + k * (1 << 41),
            lambda k: min(top, k * (top // 199))]
    dsts, per_doc = [], []
    for d in range(1200):
        f = maps[d % len(maps)]
        mp = lambda es: [(f(k), a, c) for k, a, c in es]
        e, vv = random_state(rng, R, rng.randint(0, 64), 200, 8)
        dsts.append((mp(e), vv))
        chain = []
        for _ in range(rng.randint(0, 8)):
            se, svv = random_state(rng, R, rng.randint(0, 10), 200, 8)
            t = mp(random_state(rng, R, rng.randint(0, 3), 200, 8)[0]) if delta else []
            chain.append((rng.randrange(R), svv, mp(se), t))
        per_doc.append(chain)
    dst, srcs = batch_of(R, dsts), src_batch_of(R, per_doc)
    rc, want = oracle.fold(mode, dst, srcs)
    assert rc == 0
    assert_same(eng.fold(mode, dst, srcs), want, dst.n_docs, R)


@pytest.mark.parametrize("lean", [1, 0])
def test_delta_fold_lean_pass_defers(eng, lean):
    """Delta folds run a lean slot-walk pass first (fold.hip LEAN) and defer every
    document it cannot walk to the general kernel: interleaved in one batch,
    dense documents next to key spans >= 256, 16+ sources, clocks beyond the lean
    pass's 192 words (R = 16 x 13 sources), tuples beyond 256 (block path) and
    empty documents -- the same bits as the general kernel alone and the oracle."""
    rng = random.Random(77)
    R = 16
    dsts, per_doc = [], []
    for d in range(3000):
        kind = d % 6
        universe = 200 if kind == 0 else (5000 if kind == 1 else 150)
        n_src = {0: rng.randint(0, 10), 1: rng.randint(0, 8), 2: 16, 3: 13, 4: 3, 5: 0}[kind]
        dn = 0 if kind == 5 else (rng.randint(100, 140) if kind == 4 else rng.randint(0, 60))
        sn = 60 if kind == 4 else rng.randint(0, 8)
        dsts.append(random_state(rng, R, dn, universe, 9))
        chain = []
        for _ in range(n_src):
            e, vv = random_state(rng, R, sn, universe, 9)
            t = random_state(rng, R, rng.randint(0, 3), universe, 9)[0]
            chain.append((rng.randrange(R), vv, e, t))
        per_doc.append(chain)
    dst, srcs = batch_of(R, dsts), src_batch_of(R, per_doc)
    rc, want = oracle.fold(CRDT_FOLD_DELTA, dst, srcs)
    assert rc == 0
    try:
        eng.set_option("fold_lean_first", lean)
        assert_same(eng.fold(CRDT_FOLD_DELTA, dst, srcs), want, dst.n_docs, R)
    finally:
        eng.set_option("fold_lean_first", 1)


@pytest.mark.parametrize("mode", [CRDT_FOLD_AWSET, CRDT_FOLD_DELTA])
def test_fold_panic_parity_per_doc(eng, mode):
    """actor == len(VV) panics exactly where the reference evaluates HasDot on
    it (a full step's add check, a tombstone's check, a gap step's removal
    check, the path select), and actor > len(VV) is "never seen": one
    document per call, the oracle's verdict against the kernel's."""
    rng = random.Random(50 + mode)
    R = 3
    delta = mode == CRDT_FOLD_DELTA
    seen_err = seen_ok = 0

    def ah():  # now and then a state whose dots name actors R and R + 1
        return R + 1 if rng.random() < 0.12 else None

    for _ in range(240):
        e, vv = random_state(rng, R, rng.randint(0, 12), 24, 6, actor_hi=ah())
        if rng.random() < 0.3:
            vv[rng.randrange(R)] = 0
        chain = []
        for _ in range(rng.randint(1, 5)):
            se, svv = random_state(rng, R, rng.randint(0, 8), 24, 6, actor_hi=ah())
            t = random_state(rng, R, rng.randint(0, 3), 24, 6, actor_hi=ah())[0] if delta else []
            chain.append((rng.randrange(R + 1) if rng.random() < 0.1 else rng.randrange(R), svv, se, t))
        dst, srcs = batch_of(R, [(e, vv)]), src_batch_of(R, [chain])
        rc, want = oracle.fold(mode, dst, srcs)
        if rc != 0:
            with pytest.raises(crdtgpu.CrdtError) as ei:
                eng.fold(mode, dst, srcs)
            assert ei.value.code == crdtgpu.CRDT_E_ACTOR_RANGE, (e, vv, chain)
            seen_err += 1
        else:
            assert_same(eng.fold(mode, dst, srcs), want, 1, R)
            seen_ok += 1
    assert seen_err > 10 and seen_ok > 10


def test_delta_fold_noop_and_first_contact(eng):
    R = 2
    # dst has seen actor 1 up to 5: src (actor 1) entries covered, no tombstones -> no-op, VV untouched
    dst = batch_of(R, [([(1, 0, 1)], [1, 5]), ([(1, 0, 1)], [1, 0]), ([(1, 0, 1), (2, 1, 1)], [1, 5])])
    per = [[(1, [9, 5], [(3, 1, 4)], [])],              # no-op
           [(1, [9, 5], [(3, 1, 4)], [(1, 0, 9)])],     # first contact: tombstone ignored, (A 1) removed (9>=1)
           [(1, [1, 6], [(3, 1, 6)], [(2, 1, 6)])]]     # delta: add (B 6), tombstone removes key 2
    srcs = src_batch_of(R, per)
    rc, want = oracle.fold(CRDT_FOLD_DELTA, dst, srcs)
    assert rc == 0
    got = eng.fold(CRDT_FOLD_DELTA, dst, srcs)
    assert_same(got, want, 3, R)
    assert out_doc(got, 0, R) == ([(1, 0, 1)], [1, 5])
    assert out_doc(got, 1, R) == ([(3, 1, 4)], [9, 5])
    assert out_doc(got, 2, R) == ([(1, 0, 1), (3, 1, 6)], [1, 6])


def test_delta_fold_actor_range(eng):
    R = 2
    with pytest.raises(crdtgpu.CrdtError) as ei:
        eng.fold(CRDT_FOLD_DELTA, batch_of(R, [([], [1, 1])]), src_batch_of(R, [[(2, [1, 1], [], [])]]))
    assert ei.value.code == crdtgpu.CRDT_E_ACTOR_RANGE


# ---------------------------------------------------------------- reductions

def test_causal_context_and_vv_max(eng, torch):
    rng = np.random.default_rng(3)
    dev = torch.device("cuda:0")
    for n_docs, R in [(1, 1), (5, 2), (1000, 16), (300001, 8), (77, 64)]:
        vv = rng.integers(0, 2**63, size=n_docs * R, dtype=np.uint64)
        want = oracle.causal_context(vv, n_docs, R)
        dv = torch.from_numpy(vv.view(np.int64)).to(dev)
        out = torch.zeros(R, dtype=torch.int64, device=dev)
        eng.causal_context_async(dv, n_docs, R, out)
        eng.sync()
        assert out.cpu().numpy().view(np.uint64).tolist() == want.tolist()
    a = rng.integers(0, 2**64 - 1, size=1000, dtype=np.uint64)
    b = rng.integers(0, 2**64 - 1, size=1000, dtype=np.uint64)
    da, db = torch.from_numpy(a.view(np.int64)).to(dev), torch.from_numpy(b.view(np.int64)).to(dev)
    eng.vv_max_async(da, db, 1000)
    eng.sync()
    assert (da.cpu().numpy().view(np.uint64) == np.maximum(a, b)).all()


# ---------------------------------------------------------------- workload + config 2

def gen_pair(eng, torch, n_docs, seed):
    dev = torch.device("cuda:0")
    A = OutBuffers(n_docs, 2, n_docs * 64, device=dev)
    B = OutBuffers(n_docs, 2, n_docs * 64, device=dev)
    eng.gen_pair_async(seed, n_docs, A, B)
    eng.sync()
    return A, B


def test_gen_pair_matches_host_restatement(eng, torch):
    A, B = gen_pair(eng, torch, 5000, 0x5EED)
    ha, hb = host_out(A, torch), host_out(B, torch)
    docs = list(range(0, 5000, 37)) + [4999]
    wa, wb = workloads.pair_docs(0x5EED, docs)
    for i, d in enumerate(docs):
        assert out_doc(ha, d, 2) == wa[i]
        assert out_doc(hb, d, 2) == wb[i]


def test_config2_full_size(eng, torch):
    """1,048,576 docs x 2 replicas x 64 entries, both directions, on the device.
    Exact against the oracle on a doc sample; size-independent properties on all docs."""
    n = 1 << 20
    A, B = gen_pair(eng, torch, n, 0x5EED)
    dev = torch.device("cuda:0")
    a, b = A.as_batch(), B.as_batch()
    oab = OutBuffers(n, 2, 2 * n * 64, device=dev)
    oba = OutBuffers(n, 2, 2 * n * 64, device=dev)
    eng.join_async(a, b, oab)
    eng.join_async(b, a, oba)
    eng.sync()
    # every document exact vs the oracle run on the same (device-generated) inputs
    ha, hb = host_out(A, torch).as_batch(), host_out(B, torch).as_batch()
    hab, hba = host_out(oab, torch), host_out(oba, torch)
    rc, want_ab = oracle.join(ha, hb)
    assert rc == 0
    assert_same_all(hab, want_ab, n, 2)
    rc, want_ba = oracle.join(hb, ha)
    assert rc == 0
    assert_same_all(hba, want_ba, n, 2)
    # all docs: slot bounds, element-set symmetry (A<-B and B<-A hold the same keys), VV = max
    offs = hab.offsets.astype(np.int64)
    assert (offs == np.arange(n + 1, dtype=np.int64) * 128).all()
    assert (hab.counts == hba.counts).all()
    mask = np.zeros(hab.keys.shape[0], dtype=bool)
    cnt = hab.counts.astype(np.int64)
    starts = offs[:-1]
    idx = np.repeat(starts, cnt) + (np.arange(cnt.sum()) - np.repeat(np.cumsum(cnt) - cnt, cnt))
    mask[idx] = True
    assert (hab.keys[mask] == hba.keys[mask]).all()
    k = hab.keys[idx].astype(np.uint64)
    same_doc = np.repeat(np.arange(n), cnt)
    inner = same_doc[1:] == same_doc[:-1]
    assert (k[1:][inner] > k[:-1][inner]).all(), "keys not strictly ascending inside a doc"
    va = host_out(A, torch).vv.reshape(n, 2)
    vb = host_out(B, torch).vv.reshape(n, 2)
    assert (hab.vv.reshape(n, 2) == np.maximum(va, vb)).all()
    # idempotence: X <- X == X on the whole output
    ob = oab.as_batch()
    oxx = OutBuffers(n, 2, 4 * n * 64, device=dev)
    eng.join_async(ob, ob, oxx)
    eng.sync()
    hxx = host_out(oxx, torch)
    assert (hxx.counts == hab.counts).all()
    idx2 = np.repeat(hxx.offsets[:-1].astype(np.int64), cnt) + (idx - np.repeat(starts, cnt))
    assert (hxx.keys[idx2] == hab.keys[idx]).all()
    assert (hxx.actors[idx2] == hab.actors[idx]).all()
    assert (hxx.counters[idx2] == hab.counters[idx]).all()


def host_src(S, torch):
    torch.cuda.synchronize()
    return S.numpy()


def test_gen_delta_matches_host_restatement(eng, torch):
    n, R, M = 3000, 16, 10
    dev = torch.device("cuda:0")
    D = OutBuffers(n, R, n * 64, device=dev)
    S = SrcBuffers(R, n, n * M, n * M * 8, n * M * 2, device=dev)
    eng.gen_delta_async(0x5EED, n, R, M, D, S)
    eng.sync()
    hd, hs = host_out(D, torch), host_src(S, torch)
    docs = list(range(0, n, 29)) + [n - 1]
    wd, ws = workloads.delta_docs(0x5EED, docs, R, M)
    for i, d in enumerate(docs):
        assert out_doc(hd, d, R) == wd[i]
        for j, (a, vv, e, t) in enumerate(ws[i]):
            k = d * M + j
            assert int(hs.src_actor[k]) == a
            assert hs.vv[k * R:(k + 1) * R].tolist() == vv
            o, p = int(hs.entry_off[k]), int(hs.tomb_off[k])
            assert list(zip(hs.keys[o:o + 8].tolist(), hs.actors[o:o + 8].tolist(), hs.counters[o:o + 8].tolist())) == e
            assert list(zip(hs.tkeys[p:p + 2].tolist(), hs.tactors[p:p + 2].tolist(),
                            hs.tcounters[p:p + 2].tolist())) == t


def test_config3_full_size(eng, torch):
    """1,048,576 docs x 64 entries, R=16, 10 ordered AWSetDelta sources each
    (10,485,760 deltas): every document bit-exact vs the oracle on the same inputs."""
    n, R, M = 1 << 20, 16, 10
    dev = torch.device("cuda:0")
    D = OutBuffers(n, R, n * 64, device=dev)
    S = SrcBuffers(R, n, n * M, n * M * 8, n * M * 2, device=dev)
    eng.gen_delta_async(0x5EED, n, R, M, D, S)
    out = OutBuffers(n, R, n * 64 + n * M * 8, device=dev)
    eng.reserve(n, out.slots)
    eng.fold_async(CRDT_FOLD_DELTA, D.as_batch(), S, out)
    eng.sync()
    hd, hs = host_out(D, torch).as_batch(), host_src(S, torch)
    rc, want = oracle.fold(CRDT_FOLD_DELTA, hd, hs)
    assert rc == 0
    assert_same_all(host_out(out, torch), want, n, R)


def test_gen_replicas_and_config5_fold(eng, torch):
    """Config 5 shape (8 replicas x 16 entries, R=8, fold r0<-..<-r7) on 1,048,576
    docs: generator vs host restatement on a sample; every doc's fold exact vs
    the oracle; the causal-context summary vs the oracle."""
    n, P, E, R = 1 << 20, 8, 16, 8
    dev = torch.device("cuda:0")
    D = OutBuffers(n, R, n * E, device=dev)
    S = SrcBuffers(R, n, n * (P - 1), n * (P - 1) * E, 0, device=dev)
    eng.gen_replicas_async(0x5EED, n, P, E, D, S)
    out = OutBuffers(n, R, n * E * P, device=dev)
    eng.fold_async(CRDT_FOLD_AWSET, D.as_batch(), S, out)
    ctx = torch.zeros(R, dtype=torch.int64, device=dev)
    eng.causal_context_async(out.vv, n, R, ctx)
    eng.sync()
    hd, hs = host_out(D, torch), host_src(S, torch)
    docs = list(range(0, n, 104729)) + [n - 1]
    wd, ws = workloads.replica_docs(0x5EED, docs, P, E)
    for i, d in enumerate(docs):
        assert out_doc(hd, d, R) == wd[i]
        for j, (a, vv, e, _) in enumerate(ws[i]):
            k = d * (P - 1) + j
            assert int(hs.src_actor[k]) == a and hs.vv[k * R:(k + 1) * R].tolist() == vv
            o = int(hs.entry_off[k])
            assert list(zip(hs.keys[o:o + E].tolist(), hs.actors[o:o + E].tolist(),
                            hs.counters[o:o + E].tolist())) == e
    rc, want = oracle.fold(CRDT_FOLD_AWSET, hd.as_batch(), hs)
    assert rc == 0
    ho = host_out(out, torch)
    assert_same_all(ho, want, n, R)
    assert ctx.cpu().numpy().view(np.uint64).tolist() == oracle.causal_context(want.vv, n, R).tolist()


def test_config5_bench_size(eng, torch):
    """Config 5 exactly as bench.py times it on one GPU: 12,500,000 docs
    (DEFAULT_DOCS[5], the bench seed 0x5EED of rank 0) x 8 replicas x 16
    entries, R = 8, fold r0 <- r1 <- ... <- r7, then the causal-context summary.
    - every 11th doc across the whole range (1,136,364 docs) plus the last one,
      bit-exact vs the oracle run on the same device-generated inputs;
    - every doc: its output clock is the u64 max of its 8 input clocks (each
      step merges its source clock, awset.go:160 -> crdt-misc.go:43-55) and its
      live count is <= 128;
    - the summary crdt_causal_context_async over all 12.5 M outputs == the
      oracle's max over the downloaded output clocks (crdt-misc.go:43-55)."""
    n, P, E, R = 12_500_000, 8, 16, 8
    dev = torch.device("cuda:0")
    D = OutBuffers(n, R, n * E, device=dev)
    S = SrcBuffers(R, n, n * (P - 1), n * (P - 1) * E, 0, device=dev)
    eng.gen_replicas_async(0x5EED, n, P, E, D, S)
    out = OutBuffers(n, R, n * E * P, device=dev)
    eng.fold_async(CRDT_FOLD_AWSET, D.as_batch(), S, out)
    ctx = torch.zeros(R, dtype=torch.int64, device=dev)
    eng.causal_context_async(out.vv, n, R, ctx)
    eng.sync()
    torch.cuda.synchronize()
    ar = torch.arange(n + 1, dtype=torch.int64, device=dev)
    # the generator's and the fold's fixed slot layout, which the gathers below rely on
    assert bool((D.offsets.to(torch.int64) == ar * E).all())
    assert bool((S.doc_srcs.to(torch.int64) == ar * (P - 1)).all())
    assert bool((S.entry_off.to(torch.int64) == torch.arange(n * (P - 1) + 1, device=dev) * E).all())
    assert bool((out.offsets.to(torch.int64) == ar * E * P).all())
    # every doc: output clock == u64 max of the input clocks; live count within capacity
    flip = torch.tensor(-(1 << 63), dtype=torch.int64, device=dev)
    vin = torch.maximum(D.vv.view(n, R) ^ flip, (S.vv.view(n, P - 1, R) ^ flip).amax(dim=1))
    assert bool(((out.vv.view(n, R) ^ flip) == vin).all()), "output clock != max of input clocks"
    del vin
    assert int(out.counts.max()) <= E * P and int(out.counts.min()) >= 0
    # the strided sample, gathered on the device into a batch of its own
    docs = torch.cat([torch.arange(0, n, 11, device=dev), torch.tensor([n - 1], device=dev)])
    m = int(docs.numel())
    assert m >= 1 << 20
    u32, u64 = np.uint32, np.uint64

    def rows(t, w, dt):
        return t[: n * w].view(n, w).index_select(0, docs).reshape(-1).cpu().numpy().view(dt)

    hd = AWSetBatch(R, np.arange(m + 1, dtype=u32) * E, rows(D.keys, E, u64), rows(D.actors, E, u32),
                    rows(D.counters, E, u64), rows(D.vv, R, u64), counts=rows(D.counts, 1, u32))
    ns = m * (P - 1)
    hs = SrcBatch(R, np.arange(m + 1, dtype=u32) * (P - 1), rows(S.src_actor, P - 1, u32),
                  rows(S.vv, (P - 1) * R, u64), np.arange(ns + 1, dtype=u32) * E,
                  rows(S.keys, (P - 1) * E, u64), rows(S.actors, (P - 1) * E, u32),
                  rows(S.counters, (P - 1) * E, u64), np.zeros(ns + 1, dtype=u32), np.zeros(1, dtype=u64),
                  np.zeros(1, dtype=u32), np.zeros(1, dtype=u64))
    got = OutBuffers(m, R, 0)
    got.offsets = np.arange(m + 1, dtype=u32) * E * P
    got.counts = rows(out.counts, 1, u32)
    got.keys, got.actors = rows(out.keys, E * P, u64), rows(out.actors, E * P, u32)
    got.counters, got.vv = rows(out.counters, E * P, u64), rows(out.vv, R, u64)
    rc, want = oracle.fold(CRDT_FOLD_AWSET, hd, hs)
    assert rc == 0
    assert_same_all(got, want, m, R)
    # the summary over all 12.5 M docs
    all_vv = out.vv[: n * R].cpu().numpy().view(u64)
    assert ctx.cpu().numpy().view(u64).tolist() == oracle.causal_context(all_vv, n, R).tolist()


def gen_zipf(eng, torch, n, seed=0x5EED):
    from crdtgpu.engine import zipf_sizes

    dev = torch.device("cuda:0")
    sizes = zipf_sizes(seed, n)
    offs = np.zeros(n + 1, dtype=np.uint32)
    np.cumsum(sizes, out=offs[1:])
    total = int(offs[-1])
    d_offs = torch.from_numpy(offs.view(np.int32).copy()).to(dev)
    A = OutBuffers(n, 2, total, device=dev)
    B = OutBuffers(n, 2, total, device=dev)
    eng.gen_zipf_async(seed, n, d_offs, A, B)
    eng.sync()
    return A, B, total


def test_config4_zipf_slice_exact(eng, torch):
    """Config 4 (Zipf sizes up to 2^20, 50% add/remove conflicts) on the first
    1,024 docs: generator vs host restatement on small docs; both join
    directions exact on every doc (wave + block paths) vs the oracle."""
    n = 1024
    A, B, total = gen_zipf(eng, torch, n)
    ha, hb = host_out(A, torch), host_out(B, torch)
    small = [d for d in range(64) if workloads.zipf_size(0x5EED, d) <= 3000][:12]
    wa, wb = workloads.zipf_docs(0x5EED, small)
    for i, d in enumerate(small):
        assert out_doc(ha, d, 2) == wa[i] and out_doc(hb, d, 2) == wb[i]
    dev = torch.device("cuda:0")
    for x, y, hx, hy in ((A, B, ha, hb), (B, A, hb, ha)):
        o = OutBuffers(n, 2, 2 * total, device=dev)
        eng.join_async(x.as_batch(), y.as_batch(), o)
        eng.sync()
        rc, want = oracle.join(hx.as_batch(), hy.as_batch())
        assert rc == 0
        assert_same_all(host_out(o, torch), want, n, 2)


def test_two_streams_share_one_context(eng, torch):
    """A fold on one stream and a join on another, issued back to back on one
    context with no host sync between: the context orders them (its workspace
    -- worklist, counters, scratch, status -- is shared), so both are exact.
    Large documents put both calls on the block path, which uses the worklist."""
    rng = random.Random(61)
    R = 3
    fdst, fsrc = fold_case(rng, 120, R, lambda: rng.choice([100, 600]), lambda: rng.randint(1, 4),
                           lambda: rng.choice([40, 300]), lambda: 0, 5000, 50, False)
    jd = [random_state(rng, R, rng.choice([5, 900]), 4000, 30) for _ in range(150)]
    js = [random_state(rng, R, rng.choice([5, 900]), 4000, 30) for _ in range(150)]
    jdst, jsrc = batch_of(R, jd), batch_of(R, js)
    rc1, want_f = oracle.fold(CRDT_FOLD_AWSET, fdst, fsrc)
    rc2, want_j = oracle.join(jdst, jsrc)
    assert rc1 == rc2 == 0
    dev = torch.device("cuda:0")
    fd, fs = fdst.to(dev), fsrc.to(dev)
    jdd, jds = jdst.to(dev), jsrc.to(dev)
    fout = OutBuffers(fdst.n_docs, R, fsrc.out_slots(fdst), device=dev)
    jout = OutBuffers(jdst.n_docs, R, int(jdst.offsets[-1]) + int(jsrc.offsets[-1]), device=dev)
    eng.reserve(max(fdst.n_docs, jdst.n_docs), fout.slots)
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    for _ in range(3):
        eng.fold_async(CRDT_FOLD_AWSET, fd, fs, fout, stream=sa)
        eng.join_async(jdd, jds, jout, stream=sb)
    eng.sync(sa)
    eng.sync(sb)
    assert_same(host_out(fout, torch), want_f, fdst.n_docs, R)
    assert_same(host_out(jout, torch), want_j, jdst.n_docs, R)


def test_capture_never_allocates_and_old_graphs_survive_growth(torch):
    """While a stream captures, a call that would grow the workspace returns
    CRDT_E_WORKSPACE; a graph captured before the workspace grows still replays
    correctly afterwards (outgrown buffers are kept until destroy)."""
    rng = random.Random(62)
    R = 2
    e = crdtgpu.Engine(0)
    try:
        dev = torch.device("cuda:0")
        small = [random_state(rng, R, rng.randint(0, 90), 500, 9) for _ in range(600)]
        small2 = [random_state(rng, R, rng.randint(0, 90), 500, 9) for _ in range(600)]
        d1, s1 = batch_of(R, small), batch_of(R, small2)
        rc, want = oracle.join(d1, s1)
        assert rc == 0
        dd, ds = d1.to(dev), s1.to(dev)
        out = OutBuffers(d1.n_docs, R, int(d1.offsets[-1]) + int(s1.offsets[-1]), device=dev)
        e.join_async(dd, ds, out, stream=torch.cuda.current_stream())  # sizes the workspace for 600 docs
        e.sync(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            e.join_async(dd, ds, out, stream=torch.cuda.current_stream())
        # a bigger batch cannot be captured: it would need a bigger worklist
        big = [random_state(rng, R, 3, 500, 9) for _ in range(5000)]
        bd, bs = batch_of(R, big).to(dev), batch_of(R, big).to(dev)
        bout = OutBuffers(5000, R, 6 * 5000, device=dev)
        g2 = torch.cuda.CUDAGraph()
        with pytest.raises(crdtgpu.CrdtError) as ei:
            with torch.cuda.graph(g2):
                e.join_async(bd, bs, bout, stream=torch.cuda.current_stream())
        assert ei.value.code == crdtgpu.CRDT_E_WORKSPACE
        # eagerly it grows the workspace; the first graph still replays correctly
        e.join_async(bd, bs, bout, stream=torch.cuda.current_stream())
        e.sync(torch.cuda.current_stream())
        for t in (out.keys, out.actors, out.counters, out.vv, out.counts, out.offsets):
            t.fill_(-1)
        g.replay()
        e.sync(torch.cuda.current_stream())
        assert_same(host_out(out, torch), want, d1.n_docs, R)
    finally:
        e.close()


@pytest.mark.parametrize("sizes", ["small", "mixed"])
def test_exchange_equals_two_joins(eng, torch, sizes):
    """crdt_awset_exchange_*: one pass, out_ab = a <- b and out_ba = b <- a,
    each bit-exact vs the oracle join (wave path, and block path for > 64)."""
    rng = random.Random(40 if sizes == "small" else 41)
    R = 3
    pick = (lambda: rng.randint(0, 64)) if sizes == "small" else (lambda: rng.choice([0, 5, 64, 65, 300, 2000]))
    a, b = join_case(rng, 1500 if sizes == "small" else 300, R, pick, 5000, 9)
    o1, o2 = eng.exchange(a, b)
    rc, w1 = oracle.join(a, b)
    assert rc == 0
    rc, w2 = oracle.join(b, a)
    assert rc == 0
    assert_same(o1, w1, a.n_docs, R)
    assert_same(o2, w2, a.n_docs, R)


@pytest.mark.parametrize("stage,shared,slab", [(1, 0, 0), (1, 1, 0), (0, 0, 0), (0, 1, 0), (1, 1, 7)])
def test_exchange_config2_full_size(eng, torch, stage, shared, slab):
    """All 1,048,576 config-2 docs, both directions, vs the oracle joins: LDS-
    staged contiguous stores (the default) and the lane-scattered stores, each
    with its own and with one shared key column (out_ba.keys = out_ab.keys);
    and the slab block order (join_slab_blocks_per_cu = 7: blocks remapped to
    contiguous chunks per CU, padding blocks exiting at once)."""
    n = 1 << 20
    A, B = gen_pair(eng, torch, n, 0x5EED)
    dev = torch.device("cuda:0")
    oab = OutBuffers(n, 2, 2 * n * 64, device=dev)
    oba = OutBuffers(n, 2, 2 * n * 64, device=dev, shared_keys=oab if shared else None)
    eng.set_max_doc_entries(64)
    eng.set_option("join_stage_stores", stage)
    eng.set_option("join_slab_blocks_per_cu", slab)
    try:
        eng.exchange_async(A.as_batch(), B.as_batch(), oab, oba)
        eng.sync()
    finally:
        eng.set_max_doc_entries()
        eng.set_option("join_stage_stores", 1)
        eng.set_option("join_slab_blocks_per_cu", 0)
    ha, hb = host_out(A, torch).as_batch(), host_out(B, torch).as_batch()
    rc, want = oracle.join(ha, hb)
    assert rc == 0
    assert_same_all(host_out(oab, torch), want, n, 2)
    rc, want = oracle.join(hb, ha)
    assert rc == 0
    assert_same_all(host_out(oba, torch), want, n, 2)


def test_exchange_rejects_overlapping_outputs(eng, torch):
    """crdt_awset_exchange_async: only keys == keys may be shared; two arrays at
    one address, or per-document arrays overlapping, are CRDT_E_INVALID."""
    n, R = 64, 2
    dev = torch.device("cuda:0")
    A, B = gen_pair(eng, torch, n, 7)
    o1 = OutBuffers(n, R, 2 * n * 64, device=dev)
    big = torch.empty(3 * n * R, dtype=torch.int64, device=dev)
    cases = {
        "actors": lambda o2: setattr(o2, "actors", o1.actors),
        "keys=counters": lambda o2: setattr(o2, "counters", o1.keys),
        "vv partial": None,
        "offsets=counts": lambda o2: setattr(o2, "offsets", o1.counts),
    }
    for what, mut in cases.items():
        o2 = OutBuffers(n, R, 2 * n * 64, device=dev)
        if mut is None:  # two VV arrays overlapping by one document
            o1v, o2.vv = o1.vv, big[(n - 1) * R:]
            o1.vv = big[: n * R]
        else:
            mut(o2)
        with pytest.raises(crdtgpu.CrdtError) as ei:
            eng.exchange_async(A.as_batch(), B.as_batch(), o1, o2)
        assert ei.value.code == crdtgpu.CRDT_E_INVALID, what
        if mut is None:
            o1.vv = o1v
    eng.sync()


@pytest.mark.parametrize("packed", [0, 1])
def test_exchange_batch_shared_key_column(eng, packed):
    """crdt_awset_exchange_batch with host outputs sharing one key column (the
    C++ mirror's and the Go binding's ExchangeBatch): fetched once, both
    directions exact (wave, tile and block paths; packed and slot layouts)."""
    rng = random.Random(44)
    R = 3
    a, b = join_case(rng, 300, R, lambda: rng.choice([0, 5, 64, 65, 300, 2000]), 5000, 9)
    eng.set_option("pack_batch_outputs", packed)
    try:
        o1, o2 = eng.exchange(a, b, shared_keys=True)
    finally:
        eng.set_option("pack_batch_outputs", 0)
    assert o1.keys is o2.keys
    rc, w1 = oracle.join(a, b)
    assert rc == 0
    rc, w2 = oracle.join(b, a)
    assert rc == 0
    for got, want in ((o1, w1), (o2, w2)):  # per document (a packed output has its own slot bounds)
        for d in range(a.n_docs):
            assert out_doc(got, d, R) == out_doc(want, d, R), d


@pytest.mark.parametrize("stage", [1, 0])
def test_exchange_shared_key_column_mixed_sizes(eng, torch, stage):
    """One shared key column for both exchange outputs on the wave, tile and
    block paths (documents of 0 ... 2000 entries per side), device buffers."""
    rng = random.Random(43)
    R = 3
    a, b = join_case(rng, 300, R, lambda: rng.choice([0, 5, 63, 64, 65, 300, 2000]), 5000, 9)
    dev = torch.device("cuda:0")
    da, db = a.to(dev), b.to(dev)
    slots = int(a.offsets[-1]) + int(b.offsets[-1])
    o1 = OutBuffers(a.n_docs, R, slots, device=dev)
    o2 = OutBuffers(a.n_docs, R, slots, device=dev, shared_keys=o1)
    eng.set_option("join_stage_stores", stage)
    try:
        eng.exchange_async(da, db, o1, o2)
        eng.sync()
    finally:
        eng.set_option("join_stage_stores", 1)
    rc, w1 = oracle.join(a, b)
    assert rc == 0
    rc, w2 = oracle.join(b, a)
    assert rc == 0
    assert_same(host_out(o1, torch), w1, a.n_docs, R)
    assert_same(host_out(o2, torch), w2, a.n_docs, R)


def test_max_doc_entries_promise_is_checked(eng):
    R = 2
    dst = batch_of(R, [([(k, 0, 1) for k in range(70)], [1, 0])])
    src = batch_of(R, [([], [0, 0])])
    eng.set_max_doc_entries(64)
    try:
        with pytest.raises(crdtgpu.CrdtError) as ei:
            eng.join(dst, src)
        assert ei.value.code == crdtgpu.CRDT_E_INVALID
    finally:
        eng.set_max_doc_entries()
    rc, want = oracle.join(dst, src)
    assert_same(eng.join(dst, src), want, 1, R)


@pytest.mark.parametrize("kind", ["fold_delta", "join_tiles"])
def test_graph_replay_stress_worklist_paths(torch, kind):
    """The paths that share the worklist (push_work / work_total) and the
    per-call counters zeroed by reset_work_kernel, captured ONCE into a HIP
    graph and replayed 30 times, the outputs poisoned before every replay and
    checked bit-exactly against the oracle after each: a fold whose documents
    go to both the wave pipeline and the block kernel, and a join whose large
    documents go through the tile plan (count / scan / split / look-back).
    (The round-1 fold fault under replay was in a kernel since replaced; this
    pins the shared machinery under repeated replay.)"""
    rng = random.Random(91 if kind == "fold_delta" else 92)
    R = 4
    dev = torch.device("cuda:0")
    e = crdtgpu.Engine(0)
    try:
        if kind == "fold_delta":
            dsts, per_doc = [], []
            for d in range(900):
                big = d % 97 == 0  # > 256 tuples: the block kernel's worklist
                dsts.append(random_state(rng, R, rng.randint(200, 600) if big else rng.randint(0, 60), 4000, 9))
                srcs = []
                for _ in range(rng.randint(0, 6)):
                    ents = random_state(rng, R, rng.randint(0, 30), 4000, 12)
                    tom = random_state(rng, R, rng.randint(0, 4), 4000, 12)[0]
                    srcs.append((rng.randrange(R), [rng.randint(1, 12) for _ in range(R)], ents[0], tom))
                per_doc.append(srcs)
            hd, hs = batch_of(R, dsts), src_batch_of(R, per_doc)
            rc, want = oracle.fold(CRDT_FOLD_DELTA, hd, hs)
            assert rc == 0
            dd, ds = hd.to(dev), hs.to(dev)
            out = OutBuffers(hd.n_docs, R, hs.out_slots(hd), device=dev)
            e.reserve(hd.n_docs, out.slots)

            def call(s):
                e.fold_async(CRDT_FOLD_DELTA, dd, ds, out, stream=s)
        else:
            a, b = join_case(rng, 400, R, lambda: rng.choice([0, 3, 64, 65, 900, 5000]), 20000, 9)
            rc, want = oracle.join(a, b)
            assert rc == 0
            dd, ds = a.to(dev), b.to(dev)
            out = OutBuffers(a.n_docs, R, int(a.offsets[-1]) + int(b.offsets[-1]), device=dev)
            e.set_option("join_tile_capacity", 1 << 16)

            def call(s):
                e.join_async(dd, ds, out, stream=s)
        s = torch.cuda.current_stream()
        call(s)  # eager first: sizes every workspace
        e.sync(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            call(torch.cuda.current_stream())
        n = want.n_docs if hasattr(want, "n_docs") else len(want.counts)
        for _ in range(30):
            for t in (out.keys, out.actors, out.counters, out.vv, out.counts, out.offsets):
                t.fill_(-1)
            g.replay()
            e.sync(s)
            assert_same_all(host_out(out, torch), want, n, R)
    finally:
        e.close()


# ------------------------------------------------ host path: packed outputs, device order check

@pytest.mark.parametrize("pinned", [False, True], ids=["copied", "pinned"])
@pytest.mark.parametrize("what", ["join", "exchange", "fold_awset", "fold_delta"])
def test_packed_batch_outputs(torch, what, pinned):
    """crdt_ctx_set_option("pack_batch_outputs", 1): the *_batch calls return
    only live entries, doc d at the prefix sum of the counts (computed on the
    device, pack_scan_kernel); every document bit-exact vs the oracle (large
    documents take the tile / block paths).  pinned: the host outputs lie in
    crdt_host_alloc blocks, so the gather kernel writes them itself (api.cpp
    fetch_outputs) and the call's one sync is its last; copied: ordinary host
    memory, gathered on the device and copied after one read-back of the totals."""
    rng = random.Random(hash(what) % 1000)
    R = 3
    e = crdtgpu.Engine(0)
    try:
        e.set_option("pack_batch_outputs", 1)
        if what in ("join", "exchange"):
            dst, src = join_case(rng, 1500, R, lambda: rng.choice([0, 1, 30, 64, 65, 300, 3000]), 10 ** 6, 40)
            if what == "join":
                pairs = [(e.join(dst, src, pinned=pinned), oracle.join(dst, src))]
            else:
                g1, g2 = e.exchange(dst, src, pinned=pinned)
                pairs = [(g1, oracle.join(dst, src)), (g2, oracle.join(src, dst))]
        else:
            mode = CRDT_FOLD_AWSET if what == "fold_awset" else CRDT_FOLD_DELTA
            dst, srcs = fold_case(rng, 1500, R, lambda: rng.randint(0, 80), lambda: rng.randint(0, 6),
                                  lambda: rng.randint(0, 12), lambda: rng.randint(0, 3), 300, 9, mode == CRDT_FOLD_DELTA)
            pairs = [(e.fold(mode, dst, srcs, pinned=pinned), oracle.fold(mode, dst, srcs))]
        for got, (rc, want) in pairs:
            assert rc == 0
            n = dst.n_docs
            cnt = np.asarray(got.counts[:n]).astype(np.int64)
            assert (np.asarray(got.offsets[: n + 1]) == np.concatenate([[0], np.cumsum(cnt)])).all()
            for d in range(n):
                assert out_doc(got, d, R) == out_doc(want, d, R), d
    finally:
        e.close()


@pytest.mark.parametrize("pinned", [False, True], ids=["copied", "pinned"])
def test_packed_outputs_scan_chunks(torch, pinned):
    """The packed offsets are scanned in chunks of 8,192 documents (pack.hip,
    pack_scan_kernel): an exchange of 2 x 8,192 + 37 small documents crosses
    two chunk carries in each output; offsets and every document bit-exact."""
    rng = random.Random(8229)
    R = 2
    e = crdtgpu.Engine(0)
    try:
        e.set_option("pack_batch_outputs", 1)
        dst, src = join_case(rng, 2 * 8192 + 37, R, lambda: rng.choice([0, 1, 2, 5, 9]), 10 ** 4, 12)
        g1, g2 = e.exchange(dst, src, pinned=pinned)
        for got, (rc, want) in ((g1, oracle.join(dst, src)), (g2, oracle.join(src, dst))):
            assert rc == 0
            n = dst.n_docs
            cnt = np.asarray(got.counts[:n]).astype(np.int64)
            assert (np.asarray(got.offsets[: n + 1]) == np.concatenate([[0], np.cumsum(cnt)])).all()
            for d in range(0, n, 7):
                assert out_doc(got, d, R) == out_doc(want, d, R), d
    finally:
        e.close()


@pytest.mark.parametrize("span", [1, 0], ids=["span", "per_array"])
@pytest.mark.parametrize("shared", [False, True], ids=["own_keys", "shared_keys"])
@pytest.mark.parametrize("pinned_out", [False, True], ids=["copied", "pinned"])
def test_packed_exchange_counts_inputs(torch, span, shared, pinned_out):
    """The host path's most staging-hungry call: crdt_awset_exchange_batch with
    counts-bearing inputs (slack slots: 12 input arrays) in ordinary host
    memory, packed outputs (two output rooms of six arrays, the packed offsets
    and gathers), staged span-wise or array by array ("span_staging"): every
    document of both directions exact, counts and offsets as packed."""
    rng = random.Random(61)
    R = 3
    sz = lambda: rng.choice([0, 2, 40, 64, 65, 500, 2100])  # noqa: E731
    dst = batch_of(R, [random_state(rng, R, sz(), 10 ** 6, 30) for _ in range(700)], slack=3)
    src = batch_of(R, [random_state(rng, R, sz(), 10 ** 6, 30) for _ in range(700)], slack=1)
    assert dst.counts is not None and src.counts is not None
    e = crdtgpu.Engine(0)
    try:
        e.set_option("pack_batch_outputs", 1)
        e.set_option("span_staging", span)
        for _ in range(2):  # twice: the second call reuses every staging buffer
            g1, g2 = e.exchange(dst, src, shared_keys=shared, pinned=pinned_out)
        rc, w1 = oracle.join(dst, src)
        assert rc == 0
        rc, w2 = oracle.join(src, dst)
        assert rc == 0
        n = dst.n_docs
        for got, want in ((g1, w1), (g2, w2)):
            cnt = np.asarray(got.counts[:n]).astype(np.int64)
            assert (cnt == np.asarray(want.counts[:n])).all()
            assert (np.asarray(got.offsets[: n + 1]) == np.concatenate([[0], np.cumsum(cnt)])).all()
            for d in range(n):
                assert out_doc(got, d, R) == out_doc(want, d, R), d
    finally:
        e.close()


@pytest.mark.parametrize("what", ["exchange_shared", "exchange", "join"])
def test_padded_stores_stay_in_each_document(eng, torch, what):
    """The wave kernel's padded whole-sector stores (join.hip,
    CRDT_JOIN_PAD_STORES) write zeros into a document's slack slots past its
    live entries (include/crdtgpu.h: slots past counts[d] are unspecified).
    Outputs pre-filled with a sentinel: every document's live entries exact,
    every slot a padded store wrote lies inside its own document's capacity
    [dst.offsets[d] + src.offsets[d], dst.offsets[d+1] + src.offsets[d+1])
    below 128 slots past its live count, and nothing past the batch's capacity
    changed.  Inputs with slack (counts < slots) and without."""
    rng = random.Random(63)
    R = 2
    sz = lambda: rng.choice([0, 1, 3, 7, 16, 33, 64])  # noqa: E731
    docs_d = [random_state(rng, R, sz(), 400, 9) for _ in range(3000)]
    docs_s = [random_state(rng, R, sz(), 400, 9) for _ in range(3000)]
    dev = torch.device("cuda:0")
    SENT = -0x5A5A5A5A5A5A5A5B
    for slack in (0, 5):
        a, b = batch_of(R, docs_d, slack=slack), batch_of(R, docs_s, slack=slack)
        slots = int(a.offsets[-1]) + int(b.offsets[-1])
        extra = 4096
        outs = []
        for k in range(2 if what.startswith("exchange") else 1):
            o = OutBuffers(a.n_docs, R, slots + extra, device=dev,
                           shared_keys=outs[0] if (k == 1 and what == "exchange_shared") else None)
            for t in (o.keys, o.counters):
                t.fill_(SENT)
            o.actors.fill_(-0x5A5A5A5B)
            outs.append(o)
        if what == "join":
            eng.join_async(a.to(dev), b.to(dev), outs[0])
        else:
            eng.exchange_async(a.to(dev), b.to(dev), outs[0], outs[1])
        eng.sync()
        wants = [oracle.join(a, b)[1]] + ([oracle.join(b, a)[1]] if len(outs) == 2 else [])
        cap_lo = (np.asarray(a.offsets[:-1]).astype(np.int64) + np.asarray(b.offsets[:-1]))
        cap_hi = (np.asarray(a.offsets[1:]).astype(np.int64) + np.asarray(b.offsets[1:]))
        for o, want in zip(outs, wants):
            h = host_out(o, torch)
            assert_same(h, want, a.n_docs, R)
            cnt = np.asarray(h.counts[: a.n_docs]).astype(np.int64)
            for f, sent in (("keys", SENT & ((1 << 64) - 1)), ("counters", SENT & ((1 << 64) - 1)),
                            ("actors", -0x5A5A5A5B & 0xFFFFFFFF)):
                arr = np.asarray(getattr(h, f)).astype(np.uint64)
                assert (arr[slots:] == sent).all(), (f, "written past the batch's capacity")
                written = np.nonzero(arr[:slots] != sent)[0]
                doc = np.searchsorted(cap_hi, written, side="right")  # the document whose capacity holds the slot
                assert (written >= cap_lo[doc]).all()
                rel = written - cap_lo[doc]
                assert (rel < np.maximum(cnt[doc], 128)).all(), (f, "a padded store past 128 slots")


def test_batch_key_order_checked_on_device(eng):
    """The *_batch calls check the key order after the upload (pack.hip): an
    unsorted or repeated key in any document, source or tombstone list is
    CRDT_E_UNSORTED, as crdt_validate_batch reports on the host."""
    rng = random.Random(5)
    R = 2
    dst, src = join_case(rng, 300, R, lambda: rng.randint(2, 90), 10 ** 6, 9)
    for which in ("dst", "src", "dup"):
        d2, s2 = dst.numpy(), src.numpy()
        b = d2 if which != "src" else s2
        b = AWSetBatch(b.R, b.offsets.copy(), b.keys.copy(), b.actors, b.counters, b.vv, b.counts)
        o = int(b.offsets[123])
        if which == "dup":
            b.keys[o + 1] = b.keys[o]
        else:
            b.keys[o], b.keys[o + 1] = b.keys[o + 1], b.keys[o]
        assert crdtgpu.validate(b) == crdtgpu.CRDT_E_UNSORTED
        with pytest.raises(crdtgpu.CrdtError) as ei:
            if which == "src":
                eng.join(d2, b)
            else:
                eng.exchange(b, s2)
        assert ei.value.code == crdtgpu.CRDT_E_UNSORTED
    fd, fs = fold_case(rng, 200, R, lambda: rng.randint(0, 20), lambda: rng.randint(1, 4), lambda: rng.randint(2, 9),
                       lambda: rng.randint(2, 4), 300, 9, True)
    for arr in ("keys", "tkeys"):
        s = fs.numpy() if hasattr(fs, "numpy") else fs
        bad = getattr(s, arr).copy()
        k = int((s.entry_off if arr == "keys" else s.tomb_off)[5])
        bad[k], bad[k + 1] = bad[k + 1], bad[k]
        kw = {a: getattr(s, a) for a in ("doc_srcs", "src_actor", "vv", "entry_off", "keys", "actors", "counters",
                                         "tomb_off", "tkeys", "tactors", "tcounters")}
        kw[arr] = bad
        s2 = SrcBatch(s.R, **kw)
        with pytest.raises(crdtgpu.CrdtError) as ei:
            eng.fold(CRDT_FOLD_DELTA, fd, s2)
        assert ei.value.code == crdtgpu.CRDT_E_UNSORTED


@pytest.mark.parametrize("what", ["tile_join", "tile_exchange", "block_fold_awset", "block_fold_delta"])
def test_unsorted_large_documents_never_reach_the_merge(eng, what):
    """An unsorted key in a tile-sized document (join / exchange: merge-path
    tiles) or in a block-fold-sized document (> 256 tuples): the device order
    check closes the merge's gate, so the merge's first kernel returns at once
    and nothing reaches the tile / block paths (Work::gate; no host read-back
    before the launch); the *_batch call returns CRDT_E_UNSORTED and the
    context stays usable."""
    rng = random.Random(77)
    R = 3
    if what.startswith("tile"):
        dst, src = join_case(rng, 40, R, lambda: rng.choice([3, 70, 3000]), 10 ** 6, 9)
        d2, s2 = dst.numpy(), src.numpy()
        big = max(range(40), key=lambda d: int(d2.offsets[d + 1] - d2.offsets[d]))
        b = AWSetBatch(d2.R, d2.offsets.copy(), d2.keys.copy(), d2.actors, d2.counters, d2.vv, d2.counts)
        o = int(b.offsets[big]) + 1500
        b.keys[o], b.keys[o + 1] = b.keys[o + 1], b.keys[o]
        with pytest.raises(crdtgpu.CrdtError) as ei:
            eng.join(b, s2) if what == "tile_join" else eng.exchange(b, s2)
        assert ei.value.code == crdtgpu.CRDT_E_UNSORTED
        rc, want = oracle.join(d2, s2)  # the same context, sorted input: exact
        assert rc == 0
        assert_same(eng.join(d2, s2), want, d2.n_docs, R)
        return
    mode = CRDT_FOLD_AWSET if what.endswith("awset") else CRDT_FOLD_DELTA
    fd, fs = fold_case(rng, 30, R, lambda: rng.choice([10, 400]), lambda: rng.randint(1, 4),
                       lambda: rng.choice([5, 300]), lambda: rng.randint(0, 3), 5000, 9, mode == CRDT_FOLD_DELTA)
    d2 = fd.numpy()
    big = max(range(30), key=lambda d: int(d2.offsets[d + 1] - d2.offsets[d]))
    b = AWSetBatch(d2.R, d2.offsets.copy(), d2.keys.copy(), d2.actors, d2.counters, d2.vv, d2.counts)
    o = int(b.offsets[big]) + 200
    b.keys[o], b.keys[o + 1] = b.keys[o + 1], b.keys[o]
    with pytest.raises(crdtgpu.CrdtError) as ei:
        eng.fold(mode, b, fs)
    assert ei.value.code == crdtgpu.CRDT_E_UNSORTED
    rc, want = oracle.fold(mode, fd, fs)
    assert rc == 0
    assert_same(eng.fold(mode, fd, fs), want, fd.n_docs, R)
