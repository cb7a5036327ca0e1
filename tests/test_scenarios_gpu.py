"""GPU: the reference's scenario tests, replayed through the host mirror of the
Go API (crdtgpu.awset) whose Merge runs on the device.  Each test reads like
its Go counterpart (awset_test.go, awset-delta_test.go); the final states are
also compared, dots and clocks included, with tests/golden/kat_scenarios.json."""

import json

import pytest

from crdtgpu.awset import AWSet, AWSetDelta, DeltaMergeBatch, Dot, FoldBatch, MergeBatch, VersionVector
from helpers import GOLDEN

pytestmark = pytest.mark.gpu


def init(cls=AWSet):
    return cls(0, [0, 0]), cls(1, [0, 0])


def assert_entries(s, *values):
    assert s.SortedValues() == sorted(values)


def golden_final(name):
    for sc in json.load(open(GOLDEN))["scenarios"]:
        if sc["name"].startswith(name):
            return sc["final"]
    raise KeyError(name)


def assert_golden(name, **reps):
    fin = golden_final(name)
    for r, s in reps.items():
        want = fin[r]
        assert list(s.VersionVector) == want["vv"], r
        assert sorted((k, d.Actor, d.Counter) for k, d in s.Entries.items()) == [tuple(e) for e in want["entries"]], r


def test_AWSetXXX():  # awset_test.go:10-29
    A, B = init()
    A.Add("A", "B", "C")
    B.Add("A", "B", "C")
    A.Merge(B)
    B.Merge(A)
    assert_entries(A, "A", "B", "C")
    assert_entries(B, "A", "B", "C")
    A.Del("B")
    B.Add("B")
    B.Merge(A)
    A.Merge(B)
    assert_entries(A, "A", "B", "C")
    assert_entries(B, "A", "B", "C")  # concurrent writer wins
    assert_golden("KAT-1", A=A, B=B)


def test_AWSet():  # awset_test.go:31-83
    A, B = init()
    assert_entries(A)
    assert_entries(B)
    A.Add("Shelly")
    assert_entries(A, "Shelly")
    B.Merge(A)
    assert_entries(B, "Shelly")
    B.Add("Bob", "Phil", "Pete")
    A.Merge(B)
    assert_entries(A, "Shelly", "Bob", "Phil", "Pete")
    A.Del("Phil")
    A.Add("Bob")
    A.Add("Anna")
    assert_entries(A, "Shelly", "Bob", "Pete", "Anna")
    B.Merge(A)
    assert_entries(B, "Shelly", "Bob", "Pete", "Anna")
    A.Del("Bob", "Pete")
    B.Del("Bob", "Shelly")
    A.Merge(B)
    B.Merge(A)
    assert_entries(A, "Anna")
    assert_entries(B, "Anna")
    A.Add("A", "B", "C")
    A.Del("A")
    A.Add("A")
    B.Merge(A)
    assert_entries(A, "Anna", "A", "B", "C")
    assert_entries(B, "Anna", "A", "B", "C")
    assert_golden("KAT-2", A=A, B=B)


def test_AWSetConcurrentAddWinsOverDelete():  # awset_test.go:85-122
    A, B = init()
    A.Add("Anne", "Bob")
    B.Add("Anne")
    A2, B2 = A.Clone(), B.Clone()
    B2.Add("Bob")
    A2.Del("Bob")
    B2.Merge(A2)
    A2.Merge(B2)
    assert_entries(B2, "Anne", "Bob")  # writer wins
    assert_entries(A2, "Anne", "Bob")
    B.Add("Bob")
    B.Merge(A)
    A.Del("Bob")
    B.Merge(A)
    A.Merge(B)
    assert_entries(B, "Anne")
    assert_entries(A, "Anne")
    assert_golden("KAT-3", A=A, B=B, **{"A'": A2, "B'": B2})


def test_AWSetCommutativity():  # awset_test.go:124-154
    A, B = init()
    A.Add("Shelly", "Bob", "Pete", "Anna")
    B.Add("Shelly", "Bob", "Pete", "Anna")
    A.Del("Anna")
    B.Add("Anna")
    want = ["Shelly", "Bob", "Pete", "Anna"]
    A2, B2 = A.Clone(), B.Clone()
    B2.Merge(A2)
    A2.Merge(B2)
    assert_entries(A2, *want)
    assert_entries(B2, *want)
    A.Merge(B)
    B.Merge(A)
    assert_entries(A, *want)
    assert_entries(B, *want)
    assert_golden("KAT-4", A=A, B=B, **{"A'": A2, "B'": B2})


def test_AWSetDelta():  # awset-delta_test.go:168-189
    A, B = init(AWSetDelta)
    A.Add("A", "B")
    B.Add("A", "C")
    A.Merge(B)
    B.Merge(A)
    assert_entries(A, "A", "B", "C")
    assert_entries(B, "A", "B", "C")
    A.Del("B")
    A.Add("D", "E")
    B.Add("E")
    B.Merge(A)
    assert_entries(B, "A", "C", "D", "E")
    A.Merge(B)
    assert_entries(A, "A", "C", "D", "E")
    assert A.VersionVector == [5, 2]  # the no-op delta leaves A's clock alone
    assert_golden("KAT-5", A=A, B=B)


def test_VersionVector():  # crdt-misc_test.go:5-28
    A, B = VersionVector([1, 1, 0, 4]), VersionVector([2, 0, 3, 0])
    A.Merge(B)
    assert A == [2, 1, 3, 4]
    B.Merge(A)
    assert B == [2, 1, 3, 4]


def test_batch_entry_points():
    """MergeBatch / FoldBatch / DeltaMergeBatch over many independent docs at once."""
    dsts, srcs = [], []
    for i in range(50):
        a, b = AWSet(0, [0, 0]), AWSet(1, [0, 0])
        a.Add(*["x%d" % j for j in range(i % 7)])
        b.Add(*["x%d" % j for j in range(i % 5)])
        dsts.append(a)
        srcs.append(b)
    MergeBatch(dsts, srcs)
    for i, a in enumerate(dsts):
        assert a.SortedValues() == sorted("x%d" % j for j in range(max(i % 7, i % 5)))
        assert list(a.VersionVector) == [i % 7, i % 5]
    # fold: dst <- b1 <- b2 in order
    d = AWSet(0, [0, 0, 0])
    b1, b2 = AWSet(1, [0, 0, 0]), AWSet(2, [0, 0, 0])
    b1.Add("p", "q")
    b2.Add("q")
    FoldBatch([d], [[b1, b2]])
    assert d.Entries == {"p": Dot(1, 1), "q": Dot(2, 1)}
    # delta fold
    x, y = AWSetDelta(0, [0, 0]), AWSetDelta(1, [0, 0])
    y.Add("k")
    DeltaMergeBatch([x], [[y]])
    assert x.Entries == {"k": Dot(1, 1)} and list(x.VersionVector) == [0, 1]


def test_apply_batch_matches_reference_calls():
    """ApplyBatch (batched Add / Del / AWSetDelta.Del on the GPU) leaves every
    replica exactly as the same calls on the map-based restatement
    (oracle/awset_ref.py) do: entries, Deleted, clocks; panics raise and leave
    the replica untouched."""
    import random

    from crdtgpu import CrdtError
    from crdtgpu.awset import ApplyBatch
    from oracle import awset_ref as ref

    rng = random.Random(9)
    keys = ["k%02d" % i for i in range(30)]
    mirrors, refs, scripts = [], [], []
    for i in range(300):
        R = rng.randint(1, 4)
        actor = rng.randrange(R)
        delta = i % 2 == 0
        m = (AWSetDelta if delta else AWSet)(actor, [rng.randint(0, 5) for _ in range(R)])
        r = (ref.AWSetDelta if delta else ref.AWSet)(actor, ref.VersionVector(list(m.VersionVector)))
        for k in rng.sample(keys, rng.randint(0, 10)):  # a starting state, same on both
            m.Add(k)
            r.Add(k)
        calls = []
        for _ in range(rng.randint(0, 12)):
            name = rng.choice(["Add", "Del", "AWSet.Del"] if delta else ["Add", "Del"])
            calls.append((name,) + tuple(rng.sample(keys, rng.randint(0, 3))))
        for c in calls:
            if c[0] == "Add":
                r.Add(*c[1:])
            elif c[0] == "AWSet.Del":
                ref.AWSet.Del(r, *c[1:])
            else:
                r.Del(*c[1:])
        mirrors.append(m)
        refs.append(r)
        scripts.append(calls)
    ApplyBatch(mirrors, scripts)
    for m, r in zip(mirrors, refs):
        assert {k: (d.Actor, d.Counter) for k, d in m.Entries.items()} == \
            {k: (d.actor, d.counter) for k, d in r.Entries.items()}
        assert list(m.VersionVector) == list(r.VersionVector)
        if isinstance(m, AWSetDelta):
            assert {k: (d.Actor, d.Counter) for k, d in (m.Deleted or {}).items()} == \
                {k: (d.actor, d.counter) for k, d in (r.Deleted or {}).items()}
    # panic: Add with the actor outside a shorter vector (the batch pads to R = 3)
    a, b = AWSet(2, [0, 0]), AWSet(0, [0, 0, 0])
    with pytest.raises(CrdtError):
        ApplyBatch([a, b], [[("Add", "x")], [("Add", "y")]])
    assert a.Entries == {} and list(a.VersionVector) == [0, 0]


@pytest.mark.parametrize("kind", ["join", "fold", "delta"])
def test_ragged_version_vectors_match_reference(kind):
    """Version vectors of unequal lengths in one batch (padded to one width on
    the device): every document ends exactly as the map restatement of the
    reference leaves it (entries, dots, clock and its length), and a document
    whose merge panics in Go (HasDot / Counter at actor == len(vv) of the
    unpadded vector) raises CRDT_E_ACTOR_RANGE with its destination untouched."""
    import random

    from crdtgpu import CrdtError, abi
    from helpers import ref_state
    from oracle import awset_ref as ref
    from test_mirror_width import _ragged_chain

    rng = random.Random({"join": 81, "fold": 82, "delta": 83}[kind])
    delta = kind == "delta"
    cls, rcls = (AWSetDelta, ref.AWSetDelta) if delta else (AWSet, ref.AWSet)

    def mirror(actor, e, vv, dele):
        m = cls(actor, vv, {"%012d" % k: Dot(a, c) for k, a, c in e})
        if delta and dele:
            m.Deleted = {"%012d" % k: Dot(a, c) for k, a, c in dele}
        return m

    ok, panics = [], []
    for _ in range(600):
        (e0, v0, _), chain = _ragged_chain(rng, delta, 1 if kind == "join" else rng.randint(1, 4))
        x = ref_state(e0, v0, cls=rcls)
        try:
            for act, e, svv, dele in chain:
                x.Merge(ref_state(e, svv, actor=act, cls=rcls, deleted=dele if delta else None))
            ok.append((e0, v0, chain, x))
        except ref.GoPanic:
            panics.append((e0, v0, chain))
    assert len(ok) > 100 and len(panics) > 50

    def run(dsts, chains):
        srcs = [[mirror(a, e, v, d) for a, e, v, d in ch] for ch in chains]
        if kind == "join":
            MergeBatch(dsts, [s[0] for s in srcs])
        elif kind == "fold":
            FoldBatch(dsts, srcs)
        else:
            DeltaMergeBatch(dsts, srcs)

    dsts = [mirror(0, e0, v0, []) for e0, v0, _, _ in ok]
    run(dsts, [ch for _, _, ch, _ in ok])
    for m, (_, _, _, x) in zip(dsts, ok):
        assert {k: (d.Actor, d.Counter) for k, d in m.Entries.items()} == \
            {k: (d.actor, d.counter) for k, d in x.Entries.items()}
        assert list(m.VersionVector) == list(x.VersionVector)
    for e0, v0, chain in panics[:40]:
        d = mirror(0, e0, v0, [])
        with pytest.raises(CrdtError) as ei:
            run([d], [chain])
        assert ei.value.code == abi.CRDT_E_ACTOR_RANGE
        assert list(d.VersionVector) == v0 and len(d.Entries) == len(e0)
    # the one input the padded layout cannot express: a counter-0 dot between a
    # shorter vector's end and the batch width (Go: HasDot false; pad: true)
    a, b = AWSet(0, [1], {}), AWSet(1, [1, 1, 1], {"q": Dot(2, 0)})
    with pytest.raises(CrdtError) as ei:
        MergeBatch([a], [b])
    assert ei.value.code == abi.CRDT_E_INVALID


def _mirror_of(x):
    """map-restatement state -> Python-mirror state (same actor, clock, maps)."""
    m = (AWSetDelta if hasattr(x, "Deleted") else AWSet)(x.Actor, list(x.VersionVector),
                                                          {k: Dot(d.actor, d.counter) for k, d in x.Entries.items()})
    if hasattr(x, "Deleted") and x.Deleted is not None:
        m.Deleted = {k: Dot(d.actor, d.counter) for k, d in x.Deleted.items()}
    return m


def _same(m, x):
    assert {k: (d.Actor, d.Counter) for k, d in m.Entries.items()} == \
        {k: (d.actor, d.counter) for k, d in x.Entries.items()}
    assert list(m.VersionVector) == list(x.VersionVector)


@pytest.mark.parametrize("delta", [False, True])
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_config1_two_replica_history(delta, seed):
    """BASELINE config 1 on the GPU, as SURVEY.md 8d states it: a reachable
    1,000-element two-replica history (each side deletes 10 %, adds 10 % new
    keys, re-adds 5 %), merged both ways, full-state (AWSet) and AWSetDelta:
      * the two merges of one snapshot, x = A<-B and y = B<-A, in one batch;
      * the reference's sequential round trip A.Merge(B); B.Merge(A)
        (awset_test.go:15-16), each merge one GPU call.
    Exact vs the map restatement of the reference: element sets, dots, clocks."""
    import random

    from helpers import config1_history

    A, B = config1_history(random.Random(seed), delta)
    assert 1000 <= len(A.Entries) <= 1100 and A.Entries != B.Entries
    merge = DeltaMergeBatch if delta else None
    # two merges of one snapshot
    x, y = A.Clone(), B.Clone()
    x.Merge(B)
    y.Merge(A)
    mx, my = _mirror_of(A), _mirror_of(B)
    if delta:
        merge([mx, my], [[_mirror_of(B)], [_mirror_of(A)]])
    else:
        MergeBatch([mx, my], [_mirror_of(B), _mirror_of(A)])
    _same(mx, x)
    _same(my, y)
    # sequential round trip: the second merge sees the merged A
    ma, mb = _mirror_of(A), _mirror_of(B)
    A.Merge(B)
    B.Merge(A)
    ma.Merge(mb)
    mb.Merge(ma)
    _same(ma, A)
    _same(mb, B)
    if not delta:
        assert sorted(A.Entries) == sorted(B.Entries)  # full-state round trip: converged element sets
    # (the AWSetDelta round trip does NOT converge here, in the reference as on
    # the GPU: B.Merge(A) takes the delta path, and A's Deleted holds only A's
    # own deletes -- the keys B deleted and A had never seen deleted stay in A)
