"""CPU: the synthetic "pair" workload (BASELINE config 2) is a set of
reachable states -- replaying its definition through the reference semantics
(map-based oracle: Add / Merge / Del in the stated order) yields exactly the
states the generator formulas produce -- and the byte counts follow 8d."""

import pytest

from crdtgpu import workloads
from helpers import ref


def replay_pair(seed, d):
    """The op history that defines doc d of the pair workload."""
    name = lambda u: (d << 8) | u  # noqa: E731
    A = ref.AWSet(0, ref.VersionVector([0, 0]))
    B = ref.AWSet(1, ref.VersionVector([0, 0]))
    A.Add(*[name(u) for u in range(48)])  # base, dots (A, u+1)
    B.Merge(A)
    for X, rep, new in ((0, A, range(48, 72)), (1, B, range(72, 96))):
        fates = workloads.pair_fates(seed, d, X)
        rep.Del(*[name(u) for u in range(48) if fates[u] == "del"])
        ops = [u for u in range(48) if fates[u] == "re"] + list(new)
        for u in sorted(ops):
            rep.Add(name(u))
    return A, B


def as_doc(s):
    return sorted((k, dt.actor, dt.counter) for k, dt in s.Entries.items()), list(s.VersionVector)


@pytest.mark.parametrize("seed", [0x5EED, 1, 12345])
def test_pair_workload_is_reachable(seed):
    docs = [0, 1, 2, 3, 7, 1000, 123456, 1048575]
    A, B = workloads.pair_docs(seed, docs)
    for i, d in enumerate(docs):
        a, b = replay_pair(seed, d)
        assert A[i] == as_doc(a)
        assert B[i] == as_doc(b)
        assert len(A[i][0]) == 64 and len(B[i][0]) == 64


def test_pair_workload_mix():
    """~25% of replicas re-add; deletes are exactly 8 per replica."""
    readd = 0
    for d in range(400):
        for X in (0, 1):
            f = workloads.pair_fates(0x5EED, d, X)
            assert f.count("del") == 8
            readd += "re" in f
    assert 120 < readd < 280


def test_byte_formulas():
    # one join of 64+64 -> 96 at R=2 is 20*224 + 24*2 + 12 = 4540 B
    assert workloads.join_bytes([64], [64], [96], 2) == 4540
    # delta fold, one doc: 20*64 + 8R+4 + [20*(8+2) + 8R+12]*10 + 20*n_out + 8R+4
    R = 16
    want = 20 * 64 + 8 * R + 4 + 10 * (20 * 10 + 8 * R + 12) + 20 * 100 + 8 * R + 4
    assert workloads.fold_bytes([64], [100], 80, 20, 10, R) == want


def test_delta_workload_shape_and_mix():
    dsts, srcs = workloads.delta_docs(0x5EED, list(range(300)), R=16, M=10)
    covered = total = first = 0
    for (ents, vv), chain in zip(dsts, srcs):
        assert len(ents) == 64 and [k for k, _, _ in ents] == sorted(k for k, _, _ in ents)
        assert all(a < 16 and c >= 1 for _, a, c in ents)
        first += min(vv) == 0
        assert len(chain) == 10
        for actor, svv, e, t in chain:
            assert len(e) == 8 and len(t) == 2 and actor < 16
            assert [k for k, _, _ in e] == sorted(k for k, _, _ in e)
            for _, a, c in e:
                total += 1
                covered += vv[a] >= c
    assert 0.4 < covered / total < 0.6
    assert 0 < first < 12


def test_replica_workload_is_consistent():
    """Config 5 states: every dot is covered by its own replica's clock, E keys each."""
    dsts, srcs = workloads.replica_docs(0x5EED, list(range(200)), P=8, E=16)
    for (ents, vv), chain in zip(dsts, srcs):
        states = [(0, vv, ents, [])] + chain
        assert [c[0] for c in states] == list(range(8))
        for r, v, e, t in states:
            assert len(e) == 16 and not t and v[r] >= 16
            assert all(v[a] >= c >= 1 for _, a, c in e)


def replay_zipf(seed, d):
    """The op history that defines doc d of the zipf workload (config 4)."""
    size = workloads.zipf_size(seed, d)
    key = lambda u: (d << 21) | u  # noqa: E731
    A = ref.AWSet(0, ref.VersionVector([0, 0]))
    B = ref.AWSet(1, ref.VersionVector([0, 0]))
    A.Add(*[key(u) for u in range(size)])
    B.Merge(A)
    g = [workloads._sm(seed ^ ((d << 24) | (u << 4) | 1)) for u in range(size)]
    a_del = [u for u in range(size) if g[u] & 1 and not g[u] & 2]
    b_del = [u for u in range(size) if g[u] & 1 and g[u] & 2]
    A.Del(*[key(u) for u in a_del])
    B.Del(*[key(u) for u in b_del])
    A.Add(*[key(u) for u in b_del])  # concurrent re-add wins over the other side's delete
    B.Add(*[key(u) for u in a_del])
    return A, B


def test_zipf_workload_is_reachable_and_skewed():
    docs = [d for d in range(64) if workloads.zipf_size(0x5EED, d) <= 5000][:25]
    A, B = workloads.zipf_docs(0x5EED, docs)
    for i, d in enumerate(docs):
        a, b = replay_zipf(0x5EED, d)
        assert A[i] == as_doc(a) and B[i] == as_doc(b)
    sizes = [workloads.zipf_size(0x5EED, d) for d in range(4096)]
    assert 1 <= min(sizes) and max(sizes) < (1 << 20)
    assert 20_000 < sum(sizes) / len(sizes) < 50_000
    assert sorted(sizes)[len(sizes) // 2] < 5000  # heavy tail: median far below the mean
