"""Host restatement of the synthetic workloads and the algorithmic byte counts.

``pair_docs`` recomputes, on the host, the states ``crdt_gen_pair_async``
writes on the device (csrc/gen.hip), for any sample of document ids: GPU tests
compare the two, and tests/test_workloads.py replays the same documents as
reference op sequences (Add / Del / Merge) to show the states are reachable.

Byte counts are the metric definitions of BASELINE.md / SURVEY.md 8d.
"""

from __future__ import annotations

import numpy as np

UNITS48 = np.array([1, 5, 7, 11, 13, 17, 19, 23, 25, 29, 31, 35, 37, 41, 43, 47], dtype=np.uint64)
M64 = (1 << 64) - 1


def splitmix64(x):
    """Vectorised splitmix64 over a uint64 array."""
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return x ^ (x >> np.uint64(31))


def pair_fates(seed: int, d: int, X: int):
    """Per base key u < 48 of replica X of doc d: 'del' | 're' | 'keep'."""
    s = int(splitmix64(np.uint64(seed) ^ np.uint64(2 * d + X)))
    mul, add = int(UNITS48[s & 15]), (s >> 4) % 48
    readd = ((s >> 12) & 3) == 0
    out = []
    for u in range(48):
        p = (mul * u + add) % 48
        out.append("del" if p < 8 else ("re" if readd and 8 <= p < 16 else "keep"))
    return out


def pair_docs(seed: int, docs):
    """Host copy of the pair workload for doc ids `docs`: two lists of (entries, vv)."""
    A, B = [], []
    for d in docs:
        for X, dst in ((0, A), (1, B)):
            fates = pair_fates(seed, d, X)
            c0 = 48 if X == 0 else 0
            ops = 0
            ents = []
            for u in range(48):
                if fates[u] == "del":
                    continue
                if fates[u] == "re":
                    ops += 1
                    ents.append(((d << 8) | u, X, c0 + ops))
                else:
                    ents.append(((d << 8) | u, 0, u + 1))
            n_re = ops
            lo = 48 if X == 0 else 72
            for r in range(24):
                ents.append(((d << 8) | (lo + r), X, c0 + n_re + r + 1))
            vv = [48 + n_re + 24, 0] if X == 0 else [48, n_re + 24]
            dst.append((ents, vv))
    return A, B


def _H(seed, d, tag, i):
    return int(splitmix64(np.uint64((seed ^ (d << 20) ^ (tag << 12) ^ i) & M64)))


def _subset256(h, k):
    mul, add = (h & 0xFF) | 1, (h >> 8) & 0xFF
    return [u for u in range(256) if ((mul * u + add) & 255) < k]


def delta_docs(seed: int, docs, R: int = 16, M: int = 10):
    """Host copy of the "delta" workload (csrc/gen.hip) for doc ids `docs`:
    (dst docs [(entries, vv)], per-doc sources [(actor, vv, entries, tombstones)])."""
    dsts, srcs = [], []
    for d in docs:
        first = _H(seed, d, 1, 0) % 100 == 0
        astar = _H(seed, d, 1, 1) % R
        vv0 = [0 if (first and r == astar) else 64 + _H(seed, d, 3, r) % 32 for r in range(R)]
        ents = []
        for u in _subset256(_H(seed, d, 0, 0), 64):
            hu = _H(seed, d, 2, u)
            a = hu % R
            if first and a == astar:
                a = (a + 1) % R
            ents.append(((d << 8) | u, a, 1 + (hu >> 8) % 64))
        dsts.append((ents, vv0))
        chain = []
        for j in range(M):
            aj = astar if (first and j == 0) else _H(seed, d, 4, j) % R
            svv = [vv0[r] + 1 + _H(seed, d, 5, j * R + r) % 16 for r in range(R)]
            e = []
            for u in _subset256(_H(seed, d, 6, j), 8):
                he = _H(seed, d, 7, j * 256 + u)
                a = (he >> 2) % R if (he & 3) == 0 else aj
                v0, sv = vv0[a], svv[a]
                c = 1 + (he >> 16) % (v0 if v0 > 0 else 1) if ((he >> 8) & 1) == 0 else v0 + 1 + (he >> 16) % (sv - v0)
                e.append(((d << 8) | u, a, c))
            t = []
            for u in _subset256(_H(seed, d, 8, j), 2):
                back = _H(seed, d, 9, j * 256 + u) % 8
                t.append(((d << 8) | u, aj, svv[aj] - back if svv[aj] > back else 1))
            chain.append((aj, svv, e, t))
        srcs.append(chain)
    return dsts, srcs


def replica_docs(seed: int, docs, P: int = 8, E: int = 16):
    """Host copy of the "replicas" workload (csrc/gen.hip): (dst docs = replica 0,
    per-doc sources = replicas 1..P-1 as (actor, vv, entries, []))."""
    U, R = 2 * E, P
    dsts, srcs = [], []
    for d in docs:
        chain = []
        for r in range(P):
            vv = [E + _H(seed, d, 20, r * 64 + a) % E if a == r else _H(seed, d, 20, r * 64 + a) % (E + E // 2)
                  for a in range(R)]
            h = _H(seed, d, 21, r)
            mul, add = (h & 0xFF) | 1, (h >> 8) & 0xFF
            ents = []
            for u in range(U):
                if ((mul * u + add) & (U - 1)) >= E:
                    continue
                he = _H(seed, d, 22, r * 64 + u)
                a = (he >> 2) % R if (he & 3) == 0 else r
                if vv[a] == 0:
                    a = r
                ents.append(((d << 8) | u, a, 1 + (he >> 16) % vv[a]))
            if r == 0:
                dsts.append((ents, vv))
            else:
                chain.append((r, vv, ents, []))
        srcs.append(chain)
    return dsts, srcs


ZIPF_W = [65536, 61147, 57052, 53232, 49667, 46341, 43238, 40342, 37641, 35120,
          32768, 30574, 28526, 26616, 24834, 23170, 21619, 20171, 18820, 17560]


def _sm(x):
    return int(splitmix64(np.uint64(x & M64)))


def zipf_size(seed: int, d: int) -> int:
    """Host restatement of zipf_doc_size (csrc/gen.hip)."""
    h = _sm(seed ^ ((d << 24) | 0xF))
    r, k = h % 733974, 0
    while k < 19 and r >= ZIPF_W[k]:
        r -= ZIPF_W[k]
        k += 1
    h2 = _sm(h)
    span = 1 << k
    a, b = (h2 & 0xFFFFF) % span, ((h2 >> 20) & 0xFFFFF) % span
    return span + ((a * b) >> k)


def zipf_docs(seed: int, docs):
    """Host copy of the "zipf" workload (csrc/gen.hip) for doc ids `docs`."""
    A, B = [], []
    for d in docs:
        size = zipf_size(seed, d)
        g = [_sm(seed ^ ((d << 24) | (u << 4) | 1)) for u in range(size)]
        a_del = [(x & 1) == 1 and (x & 2) == 0 for x in g]
        b_del = [(x & 1) == 1 and (x & 2) != 0 for x in g]
        na, nb = sum(b_del), sum(a_del)  # A re-adds where B deletes and vice versa
        ea, eb, ra, rb = [], [], 0, 0
        for u in range(size):
            key = (d << 21) | u
            if not a_del[u]:
                if b_del[u]:
                    ra += 1
                    ea.append((key, 0, size + ra))
                else:
                    ea.append((key, 0, u + 1))
            if not b_del[u]:
                if a_del[u]:
                    rb += 1
                    eb.append((key, 1, rb))
                else:
                    eb.append((key, 0, u + 1))
        A.append((ea, [size + na, 0]))
        B.append((eb, [size, nb]))
    return A, B


def join_bytes(n_dst, n_src, n_out, R) -> int:
    """Σ over docs of 20(n_dst + n_src + n_out) + 24R + 12."""
    n_dst, n_src, n_out = (np.asarray(x, dtype=np.int64) for x in (n_dst, n_src, n_out))
    return int(20 * (n_dst.sum() + n_src.sum() + n_out.sum()) + (24 * R + 12) * n_dst.size)


def exchange_bytes(n_a, n_b, n_ab, n_ba, R, shared_keys=False) -> int:
    """One exchange launch (A <- B and B <- A from one read of both states):
    Σ over docs of 20(n_a + n_b) read once + 20(n_ab + n_ba) written +
    32R (two VVs read, two written) + 32 (offsets and counts: two read, two written).
    shared_keys: the two outputs share one key column (n_ab == n_ba, the same
    keys at the same slots), so B <- A writes 12 B per entry (actor, counter)."""
    n_a, n_b, n_ab, n_ba = (np.asarray(x, dtype=np.int64) for x in (n_a, n_b, n_ab, n_ba))
    out_b = 12 if shared_keys else 20
    return int(20 * (n_a.sum() + n_b.sum() + n_ab.sum()) + out_b * n_ba.sum() + (32 * R + 32) * n_a.size)


def fold_bytes(n_dst, n_out, src_entries, src_tombs, n_srcs_total, R) -> int:
    """Σ over docs of 20 n_dst + 8R + 4 + Σ_j [20 (c_j + x_j) + 8R + 12] + 20 n_out + 8R + 4."""
    n_dst, n_out = np.asarray(n_dst, dtype=np.int64), np.asarray(n_out, dtype=np.int64)
    per_doc = 20 * (n_dst.sum() + n_out.sum()) + (16 * R + 8) * n_dst.size
    per_src = 20 * (int(src_entries) + int(src_tombs)) + (8 * R + 12) * int(n_srcs_total)
    return int(per_doc + per_src)
