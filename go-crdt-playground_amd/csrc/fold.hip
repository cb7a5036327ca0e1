// Ordered fold of source states into each document:
//   out[d] = (((dst[d] <- src[d][0]) <- src[d][1]) ... )
// mode CRDT_FOLD_AWSET : each step is (*AWSet).Merge        awset.go:103-161
// mode CRDT_FOLD_DELTA : each step is (*AWSetDelta).Merge   awset-delta_test.go:51-166
//   path select  Counter(src.Actor) == 0 -> full merge, src.Deleted ignored (:53-56)
//   otherwise    changed = src entries dst's clock has not seen, deleted =
//                tombstones not re-added (:79-105); both empty -> nothing,
//                not even the VV merge (:60); else deltaMerge (:107-166).
// Steps into one document are applied in order: the
// document stays on chip for the whole fold and is written to HBM once.
//
//  * fold_sort_kernel: one wavefront per document while document + source
//    entries + tombstones fit 256 tuples (<= 64 sources, sources x R <= 256
//    clock words).  The fold is replayed per key (see below), not per step.
//  * fold_block_kernel: every other document (worklist); persistent
//    workgroups, merge-path walk per step (merge_block.hpp), ping-pong
//    between the output slots and a scratch copy.
#include "crdt_device.hpp"
#include "merge_block.hpp"

namespace crdt {

// ---- fold_sort_kernel: the fold restated per key --------------------------
// A key's fate over the whole fold depends only on its own tuples (its dot in
// the document, its entry in each source, its tombstone in each source) and on
// three per-step facts of the document: V_j, the clock before step j; full_j,
// the awset path (or Counter(src.Actor) == 0, awset-delta_test.go:53); noop_j,
// a delta step with nothing changed and nothing deleted (:60, no VV merge).
// V_j/full_j/noop_j need only the clocks and one "anything changed?" ballot
// per step.  So one wavefront per document:
//   1. schedule  V_j, full_j, noop_j for j < M; mark the tuples that can act
//                on their key (entries of full steps, changed entries and
//                effective tombstones of delta steps);
//   2. group     those tuples by (key, step, kind): a bitonic network held in
//                registers, EPL tuples per lane, cross-lane stages by lane
//                shuffles;
//   3. walk      one lane per distinct key replays its events in step order
//                (its tuples, and -- while present -- every full step, whose
//                phase 2 may remove it: awset.go:147-158);
//   4. write     the survivors, already in key order, ballot-compacted.
// Work per document is a few ballots per step plus one sort of <= 256 tuples,
// instead of one sorted merge (binary searches, barriers) per step.
struct FoldSortSmem {
    static constexpr int NCAP = 256;  // document entries + source entries + tombstones
    static constexpr int VCAP = 256;  // sources x R clock words
    static constexpr int MCAP = 64;   // sources per document
    uint64_t tk[NCAP];      // tuple keys; after the sort: the key of each segment
    uint64_t tc[NCAP];      // tuple counters (document, entries, tombstones)
    uint32_t ta[NCAP];      // tuple actors
    uint16_t stag[NCAP];    // kept tuples' tags, then the sorted tags
    uint16_t seg[NCAP + 1]; // first sorted position of each distinct key
    uint8_t keep[NCAP];     // delta steps: entry changed / tombstone effective
    uint8_t step[NCAP];     // source index of an entry / tombstone tuple
    uint64_t vs[VCAP];      // V_j (j < M), R words each
    uint64_t svv[VCAP];     // source clocks, R words each
    uint32_t soff[MCAP + 1];
    uint32_t toff[MCAP + 1];
    uint32_t sact[MCAP];
    uint64_t emask;         // steps holding an effective tombstone
};

// Tuple tag: bits 15..8 = 0 for a document entry, (j+1)*2 for an entry of
// source j, (j+1)*2+1 for its tombstone; bits 7..0 = tuple index in LDS.  The
// sort order (key, tag) puts a key's tuples in replay order.
constexpr uint32_t kPadTag = 0xFFFFu;

__device__ __forceinline__ bool tup_less(uint64_t ka, uint32_t ta, uint64_t kb, uint32_t tb) {
    return ka < kb || (ka == kb && ta < tb);
}

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m) {
    return (uint64_t)__shfl_xor((unsigned long long)v, m);
}

// Bitonic sort of EPL*64 (key, tag) pairs; element i = lane*EPL + q.
template <int EPL>
__device__ __forceinline__ void wave_bitonic(uint64_t (&k)[EPL], uint32_t (&t)[EPL], uint32_t lane) {
    constexpr int P = EPL * 64;
#pragma unroll
    for (int kk = 2; kk <= P; kk <<= 1) {
#pragma unroll
        for (int jj = kk >> 1; jj > 0; jj >>= 1) {
            if (jj >= EPL) {
                const int lm = jj / EPL;
                const bool lower = (lane & lm) == 0;
#pragma unroll
                for (int q = 0; q < EPL; ++q) {
                    const bool asc = (((lane * EPL + q) & kk) == 0);
                    const uint64_t pk = shfl_xor64(k[q], lm);
                    const uint32_t pt = (uint32_t)__shfl_xor((int)t[q], lm);
                    const bool take = (lower == asc) ? tup_less(pk, pt, k[q], t[q]) : tup_less(k[q], t[q], pk, pt);
                    k[q] = take ? pk : k[q];
                    t[q] = take ? pt : t[q];
                }
            } else {
#pragma unroll
                for (int q = 0; q < EPL; ++q) {
                    if (q & jj) continue;
                    const int r = q | jj;
                    const bool asc = (((lane * EPL + q) & kk) == 0);
                    const bool sw = asc ? tup_less(k[r], t[r], k[q], t[q]) : tup_less(k[q], t[q], k[r], t[r]);
                    const uint64_t k0 = k[q], k1 = k[r];
                    const uint32_t t0 = t[q], t1 = t[r];
                    k[q] = sw ? k1 : k0;
                    k[r] = sw ? k0 : k1;
                    t[q] = sw ? t1 : t0;
                    t[r] = sw ? t0 : t1;
                }
            }
        }
    }
}

// Load cnt (key, actor, counter) triples from global [o, o+cnt) into LDS at
// [base, base+cnt), cnt <= 256: all loads first (unused chunks skipped by a
// uniform branch, lanes past cnt read 0), then the LDS stores.
__device__ __forceinline__ void load_tuples(FoldSortSmem& m, uint32_t base, const uint64_t* gk, const uint32_t* ga,
                                            const uint64_t* gc, uint32_t o, uint32_t cnt, uint32_t lane) {
    const rsrc_t rk = make_rsrc(gk + o, cnt * 8u), ra = make_rsrc(ga + o, cnt * 4u), rc = make_rsrc(gc + o, cnt * 8u);
    uint64_t kk[4], cc[4];
    uint32_t aa[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        if (q * 64u >= cnt) break;
        const uint32_t i = q * 64 + lane;
        kk[q] = ld64(rk, i * 8u);
        aa[q] = ld32(ra, i * 4u);
        cc[q] = ld64(rc, i * 8u);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        if (q * 64u >= cnt) break;
        const uint32_t i = q * 64 + lane;
        if (i < cnt) {
            m.tk[base + i] = kk[q];
            m.ta[base + i] = aa[q];
            m.tc[base + i] = cc[q];
        }
    }
}

// Walk one round of up to 64 keys (segments r0 + lane) and write the survivors.
template <bool DELTA>
__device__ __forceinline__ uint32_t walk_round(FoldSortSmem& m, uint32_t r0, uint32_t U, uint32_t K, uint32_t R,
                                               uint64_t full_mask, uint32_t lane, uint64_t lt, rsrc_t ok, rsrc_t oa,
                                               rsrc_t oc, uint32_t carry, uint32_t& err) {
    const uint32_t s = r0 + lane;
    const bool act = s < U;
    uint32_t p = act ? m.seg[s] : 0u;
    const uint32_t p1 = act ? m.seg[s + 1] : 0u;
    const uint64_t key = m.tk[act ? s : 0u];
    uint32_t tg = act ? m.stag[p] : kPadTag;
    bool pres = false;
    uint32_t a = 0;
    uint64_t c = 0;
    if ((tg >> 8) == 0) {  // the document's own entry
        pres = true;
        a = m.ta[tg & 0xFF];
        c = m.tc[tg & 0xFF];
        ++p;
        tg = p < p1 ? m.stag[p] : kPadTag;
    }
    uint32_t jn = 0;  // first step not yet replayed
    for (;;) {
        // next event: this key's next tuple, or (while present) the next full step
        const uint32_t ts = tg == kPadTag ? 64u : ((tg >> 9) - 1u);
        const uint64_t fm = pres && jn < 64 ? (full_mask & (~0ull << jn)) : 0ull;
        const uint32_t nf = fm ? (uint32_t)__builtin_ctzll(fm) : 64u;
        const uint32_t je = ts < nf ? ts : nf;
        const bool go = act && je < 64;
        if (!ballot(go)) break;
        if (go) {
            const bool full = (full_mask >> je) & 1ull;
            bool is_e = false, is_t = false;
            uint32_t ea = 0, xa = 0;
            uint64_t ec = 0, xc = 0;
            if (ts == je && !((tg >> 8) & 1u)) {
                is_e = true;
                ea = m.ta[tg & 0xFF];
                ec = m.tc[tg & 0xFF];
                ++p;
                tg = p < p1 ? m.stag[p] : kPadTag;
            }
            if (DELTA && tg != kPadTag && ((tg >> 9) - 1u) == je) {  // tombstone of the same step
                is_t = true;
                xa = m.ta[tg & 0xFF];
                xc = m.tc[tg & 0xFF];
                ++p;
                tg = p < p1 ? m.stag[p] : kPadTag;
            }
            if (full) {
                if (is_e) {
                    // awset.go:117-141: common key -> src dot; src-only -> added iff dst clock lacks it
                    if (pres || !has_dot_bf(m.vs + je * R, R, ea, ec, true, err)) {
                        pres = true;
                        a = ea;
                        c = ec;
                    }
                } else if (pres && has_dot_bf(m.svv + je * R, R, a, c, true, err)) {
                    pres = false;  // awset.go:150-153: src saw it and dropped it
                }
            } else {
                if (is_e) {  // changed entry: deltaMerge phase 1 (awset-delta_test.go:126-144)
                    pres = true;
                    a = ea;
                    c = ec;
                }
                // phase 2 (:146-163): an effective tombstone removes a present
                // key unless the clock before this step already holds its dot
                if (is_t && pres && !has_dot_bf(m.vs + je * R, R, xa, xc, true, err)) pres = false;
            }
            jn = je + 1;
        }
    }
    const bool emit = act && pres;
    const uint64_t em = ballot(emit);
    const uint32_t pos = carry + popc(em & lt);
    const uint32_t ko = emit ? pos * 8u : kOOB, ao = emit ? pos * 4u : kOOB;
    st64<kAuxNT>(key, ok, ko);
    st32<kAuxNT>(a, oa, ao);
    st64<kAuxNT>(c, oc, ko);
    return carry + popc(em);
}

template <int EPL, bool DELTA>
__device__ __forceinline__ uint32_t sort_and_walk(FoldSortSmem& m, uint32_t K, uint32_t R, uint64_t full_mask,
                                                  uint32_t lane, uint64_t lt, rsrc_t ok, rsrc_t oa, rsrc_t oc,
                                                  uint32_t& err) {
    uint64_t k[EPL];
    uint32_t t[EPL];
#pragma unroll
    for (int q = 0; q < EPL; ++q) {
        const uint32_t i = lane * EPL + q;
        k[q] = i < K ? m.tk[i] : ~0ull;
        t[q] = i < K ? (uint32_t)m.stag[i] : kPadTag;
    }
    wave_sync();
    wave_bitonic<EPL>(k, t, lane);
    // segment heads: first tuple of each distinct key
    const uint64_t prev = (uint64_t)__shfl_up((unsigned long long)k[EPL - 1], 1);
    bool head[EPL];
    uint32_t hc = 0;
#pragma unroll
    for (int q = 0; q < EPL; ++q) {
        const uint32_t i = lane * EPL + q;
        const uint64_t pk = q == 0 ? prev : k[q - 1];
        head[q] = t[q] != kPadTag && (i == 0 || k[q] != pk);
        hc += head[q];
    }
    uint32_t pre = 0, U = 0;
#pragma unroll
    for (int b = 0; b < 3; ++b) {
        const uint64_t mb = ballot((hc >> b) & 1u);
        pre += popc(mb & lt) << b;
        U += popc(mb) << b;
    }
#pragma unroll
    for (int q = 0; q < EPL; ++q) {
        const uint32_t i = lane * EPL + q;
        if (i < K) m.stag[i] = (uint16_t)t[q];
        if (head[q]) {
            m.seg[pre] = (uint16_t)i;
            m.tk[pre] = k[q];
            ++pre;
        }
    }
    if (lane == 0) m.seg[U] = (uint16_t)K;
    wave_sync();
    uint32_t carry = 0;
    for (uint32_t r0 = 0; r0 < U; r0 += 64)
        carry = walk_round<DELTA>(m, r0, U, K, R, full_mask, lane, lt, ok, oa, oc, carry, err);
    return carry;
}

template <int WAVES, bool DELTA>
__global__ __launch_bounds__(WAVES * 64) void fold_sort_kernel(BatchView dst, SrcView sb, OutView out, Work wk) {
    using Smem = FoldSortSmem;
    __shared__ Smem smem[WAVES];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t w = threadIdx.x >> 6;
    Smem& m = smem[w];
    const uint32_t R = dst.R;
    const uint32_t n_docs = dst.n_docs;
    const uint64_t lt = low_mask(lane);
    const bool tombs = DELTA && sb.tomb_off != nullptr;
    uint32_t err = 0;

    for (uint32_t d0 = blockIdx.x * WAVES + w; d0 < n_docs; d0 += gridDim.x * WAVES) {
        const uint32_t d = uniform(d0);
        const uint32_t s0 = sb.doc_srcs[d], s1 = sb.doc_srcs[d + 1];
        const uint32_t ms = s1 - s0;
        const uint32_t doff = dst.offsets[d];
        const uint32_t e0 = sb.entry_off[s0], E = sb.entry_off[s1] - e0;
        const uint32_t t0 = tombs ? sb.tomb_off[s0] : 0u;
        const uint32_t X = tombs ? sb.tomb_off[s1] - t0 : 0u;
        const uint32_t obase = doff + e0;
        const uint32_t cap = dst.offsets[d + 1] - doff + E;
        const uint32_t n = live_count(dst.offsets, dst.counts, d);
        if (lane == 0) {
            out.offsets[d] = obase;
            if (d == n_docs - 1) out.offsets[n_docs] = dst.offsets[n_docs] + sb.entry_off[sb.doc_srcs[n_docs]];
        }
        const uint32_t N = n + E + X;
        if (N > Smem::NCAP || ms > Smem::MCAP || ms * R > Smem::VCAP) {  // block path
            if (lane == 0) push_work(wk, d, n_docs);
            continue;
        }
        // ---- load: document, source entries, tombstones, clocks, offsets, actors
        load_tuples(m, 0, dst.keys, dst.actors, dst.counters, doff, n, lane);
        load_tuples(m, n, sb.keys, sb.actors, sb.counters, e0, E, lane);
        if (X) load_tuples(m, n + E, sb.tkeys, sb.tactors, sb.tcounters, t0, X, lane);
        {
            const rsrc_t rv = make_rsrc(sb.vv + (size_t)s0 * R, ms * R * 8u);
            uint64_t vq[Smem::VCAP / 64];
#pragma unroll
            for (int q = 0; q < Smem::VCAP / 64; ++q) vq[q] = ld64(rv, (q * 64 + lane) * 8u);
            const rsrc_t re = make_rsrc(sb.entry_off + s0, (ms + 1) * 4u);
            const uint32_t eo = ld32(re, lane * 4u), eo2 = ld32(re, (64 + lane) * 4u);
            uint32_t to = 0, to2 = 0;
            if (tombs) {
                const rsrc_t rt = make_rsrc(sb.tomb_off + s0, (ms + 1) * 4u);
                to = ld32(rt, lane * 4u);
                to2 = ld32(rt, (64 + lane) * 4u);
            }
            const uint32_t ac = ld32(make_rsrc(sb.src_actor + s0, ms * 4u), lane * 4u);
#pragma unroll
            for (int q = 0; q < Smem::VCAP / 64; ++q) m.svv[q * 64 + lane] = vq[q];
            m.soff[lane] = eo - e0;
            m.toff[lane] = to - t0;
            if (lane == 0) {
                m.soff[64] = eo2 - e0;
                m.toff[64] = to2 - t0;
                m.emask = 0;
            }
            m.sact[lane] = ac;
        }
        uint64_t vreg = ld64(make_rsrc(dst.vv + (size_t)d * R, R * 8u), lane * 8u);  // lane r: V[r]
        wave_sync();
        // ---- source index of every entry / tombstone tuple (lane j fills source j's range)
        if (lane < ms) {
            const uint32_t a0 = m.soff[lane], a1 = m.soff[lane + 1];
            for (uint32_t i = a0; i < a1; ++i) m.step[n + i] = (uint8_t)lane;
            if (X) {
                const uint32_t b0 = m.toff[lane], b1 = m.toff[lane + 1];
                for (uint32_t i = b0; i < b1; ++i) m.step[n + E + i] = (uint8_t)lane;
            }
        }
        wave_sync();
        // ---- effective tombstones (MakeDeltaMergeData, awset-delta_test.go:93-104):
        // not re-added in the same source.  Clock-independent, so all at once.
        if (X) {
            uint32_t cmax = 0;  // longest source: search depth
            for (uint32_t j = lane; j < ms; j += 64) cmax = max(cmax, m.soff[j + 1] - m.soff[j]);
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) cmax = max(cmax, (uint32_t)__shfl_xor((int)cmax, o));
            for (uint32_t q = 0; q * 64 < X; ++q) {
                const uint32_t x = q * 64 + lane;
                if (x < X) {
                    const uint32_t ti = n + E + x;
                    const uint32_t j = m.step[ti];
                    const uint32_t lo = n + m.soff[j], len = m.soff[j + 1] - m.soff[j];
                    const uint64_t tkey = m.tk[ti];
                    uint32_t pos = 0;
                    for (uint32_t st = 256; st > 0; st >>= 1) {
                        if (st > cmax) continue;
                        const bool in = pos + st <= len;
                        const uint64_t v = m.tk[in ? lo + pos + st - 1 : 0u];
                        pos += (in && v < tkey) ? st : 0u;
                    }
                    const bool in_s = pos < len && m.tk[lo + pos] == tkey;
                    const bool eff = !(in_s && (m.ta[lo + pos] != m.ta[ti] || m.tc[lo + pos] > m.tc[ti]));
                    m.keep[ti] = eff;
                    if (eff) atomicOr((unsigned long long*)&m.emask, 1ull << j);
                }
            }
            wave_sync();
        }
        // ---- schedule: V_j, full_j, noop_j (one ballot per delta step)
        uint64_t full_mask = 0, noop_mask = 0;
        const uint64_t emask = X ? m.emask : 0ull;
        for (uint32_t j = 0; j < ms; ++j) {
            if (lane < R) m.vs[j * R + lane] = vreg;
            bool full = true;
            if (DELTA) {
                const uint32_t aj = m.sact[j];
                // VersionVector.Counter (crdt-misc.go:36-41); actor == len panics
                if (aj == R) err |= kErrActorRange;
                const uint64_t cnt = aj < R ? (uint64_t)__shfl((unsigned long long)vreg, (int)aj) : 0ull;
                full = cnt == 0;
            }
            bool noop = false;
            if (!full) {
                const uint32_t a0 = m.soff[j], a1 = m.soff[j + 1];
                bool any = false;
                for (uint32_t b = a0; b < a1; b += 64) {
                    const uint32_t i = b + lane;
                    const bool v = i < a1;
                    const uint32_t ea = v ? m.ta[n + i] : 0u;
                    const uint64_t ec = v ? m.tc[n + i] : 0ull;
                    const uint64_t have = (uint64_t)__shfl((unsigned long long)vreg, (int)(ea < R ? ea : 0u));
                    if (v && ea == R) err |= kErrActorRange;  // HasDot panics (crdt-misc.go:28-34)
                    const bool chg = v && !(ea < R && have >= ec);
                    if (v) m.keep[n + i] = chg;
                    any |= chg;
                }
                noop = !ballot(any) && !((emask >> j) & 1ull);
            }
            full_mask |= (uint64_t)full << j;
            noop_mask |= (uint64_t)noop << j;
            if (!noop && lane < R) vreg = max(vreg, m.svv[j * R + lane]);
        }
        wave_sync();
        // ---- keep only tuples that act on their key; stage (key, tag) compacted
        uint32_t K = 0;
        for (uint32_t q = 0; q * 64 < N; ++q) {
            const uint32_t i = q * 64 + lane;
            bool kept = i < N;
            uint32_t tag = i;
            const uint64_t key = m.tk[kept ? i : 0u];
            if (kept && i >= n) {
                const uint32_t j = m.step[i];
                const bool tomb = i >= n + E;
                const bool full = (full_mask >> j) & 1ull;
                kept = !((noop_mask >> j) & 1ull) && (tomb ? (!full && m.keep[i]) : (full || m.keep[i]));
                tag |= (((j + 1) * 2 + (tomb ? 1u : 0u)) << 8);
            }
            const uint64_t km = ballot(kept);
            const uint32_t pos = K + popc(km & lt);
            if (kept) {
                m.tk[pos] = key;
                m.stag[pos] = (uint16_t)tag;
            }
            K += popc(km);
        }
        wave_sync();
        // ---- sort, walk, write
        const uint32_t oc_n = cap < Smem::NCAP ? cap : Smem::NCAP;  // survivors <= n + E <= 256
        const rsrc_t ok = make_rsrc(out.keys + obase, oc_n * 8u), oa = make_rsrc(out.actors + obase, oc_n * 4u),
                     oc = make_rsrc(out.counters + obase, oc_n * 8u);
        const uint32_t cnt = K <= 128 ? sort_and_walk<2, DELTA>(m, K, R, full_mask, lane, lt, ok, oa, oc, err)
                                      : sort_and_walk<4, DELTA>(m, K, R, full_mask, lane, lt, ok, oa, oc, err);
        if (lane == 0) out.counts[d] = cnt;
        if (lane < R) out.vv[(size_t)d * R + lane] = vreg;
        wave_sync();
    }
    flag_error(wk.status, err);
}

template <int NT, int IPT>
__global__ __launch_bounds__(NT) void fold_block_kernel(int mode, BatchView dst, SrcView sb, OutView out, Scratch scr,
                                                        Work wk) {
    __shared__ MergeSmem<NT, IPT> sm;
    const uint32_t tid = threadIdx.x;
    const uint32_t R = dst.R;
    uint32_t err = 0;
    for (;;) {
        if (tid == 0) sm.word[0] = atomicAdd(wk.wl_head, 1u);
        __syncthreads();
        const uint32_t slot = sm.word[0];
        const uint32_t total = work_total(wk, dst.n_docs);
        __syncthreads();
        if (slot >= total) break;
        const uint32_t d = wk.worklist[slot];
        if (d >= dst.n_docs) {  // not a document of this call: never dereferenced
            if (tid == 0) atomicOr(wk.status, kErrWorkspace);
            continue;
        }
        const uint32_t s0 = sb.doc_srcs[d], s1 = sb.doc_srcs[d + 1];
        const uint32_t doff = dst.offsets[d];
        const uint32_t obase = doff + sb.entry_off[s0];
        const uint64_t cap = (uint64_t)(dst.offsets[d + 1] - doff) + (sb.entry_off[s1] - sb.entry_off[s0]);
        if ((uint64_t)obase + cap > scr.slots) {  // crdt_ctx_reserve was not told enough slots
            if (tid == 0) atomicOr(wk.status, kErrWorkspace);
            __syncthreads();
            continue;
        }
        const EntriesOut O{out.keys + obase, out.actors + obase, out.counters + obase};
        const EntriesOut X{scr.keys + obase, scr.actors + obase, scr.counters + obase};
        Entries cur{dst.keys + doff, dst.actors + doff, dst.counters + doff, live_count(dst.offsets, dst.counts, d)};
        int where = 0;  // 0 = input, 1 = out, 2 = scratch
        if (tid < R) sm.dvv[tid] = dst.vv[(size_t)d * R + tid];
        __syncthreads();
        bool stop = false;
        for (uint32_t k = s0; k < s1 && !stop; ++k) {
            const uint32_t e0 = sb.entry_off[k];
            const Entries S{sb.keys + e0, sb.actors + e0, sb.counters + e0, sb.entry_off[k + 1] - e0};
            Entries Tm{nullptr, nullptr, nullptr, 0};
            if (sb.tomb_off && mode == CRDT_FOLD_DELTA) {
                const uint32_t t0 = sb.tomb_off[k];
                Tm = Entries{sb.tkeys + t0, sb.tactors + t0, sb.tcounters + t0, sb.tomb_off[k + 1] - t0};
            }
            if (tid < R) sm.svv[tid] = sb.vv[(size_t)k * R + tid];
            __syncthreads();
            uint32_t perr = 0;
            const bool full = (mode != CRDT_FOLD_DELTA) || vv_counter(sm.dvv, R, sb.src_actor[k], perr) == 0;
            if (perr) {
                err |= perr;
                stop = true;
                break;
            }
            if (!full) {
                bool any = false;
                for (uint32_t e = tid; e < S.n; e += NT) any |= !has_dot(sm.dvv, R, S.a[e], S.c[e], err);
                for (uint32_t t = tid; t < Tm.n; t += NT) {
                    const uint32_t g = lower_bound(S.k, S.n, Tm.k[t]);
                    const bool in_s = g < S.n && S.k[g] == Tm.k[t];
                    any |= !(in_s && (S.a[g] != Tm.a[t] || S.c[g] > Tm.c[t]));
                }
                if (!__syncthreads_or(any)) continue;
            }
            const EntriesOut& tgt = (where == 1) ? X : O;
            const uint32_t n = block_merge<NT, IPT>(cur, S, full ? Entries{nullptr, nullptr, nullptr, 0} : Tm, full, R,
                                                    sm, tgt, err);
            if (tid < R) sm.dvv[tid] = max(sm.dvv[tid], sm.svv[tid]);
            where = (where == 1) ? 2 : 1;
            cur = Entries{tgt.k, tgt.a, tgt.c, n};
            __syncthreads();
        }
        if (where != 1) {  // result still in the input or the scratch copy
            for (uint32_t i = tid; i < cur.n; i += NT) {
                O.k[i] = cur.k[i];
                O.a[i] = cur.a[i];
                O.c[i] = cur.c[i];
            }
        }
        if (tid == 0) out.counts[d] = cur.n;
        if (tid < R) out.vv[(size_t)d * R + tid] = sm.dvv[tid];
        __syncthreads();
    }
    if (__syncthreads_or(err != 0) && tid == 0) atomicOr(wk.status, kErrActorRange);
}

constexpr int kFoldWaves = 2;
constexpr int kFoldNT = 256;
constexpr int kFoldIPT = 4;

hipError_t launch_fold(int mode, const BatchView& dst, const SrcView& sb, const OutView& out, const Scratch& scr,
                       const Work& wk, uint32_t block_grid, hipStream_t stream) {
    if (dst.n_docs == 0) return hipSuccess;
    uint32_t grid = (dst.n_docs + kFoldWaves - 1) / kFoldWaves;
    if (grid > (1u << 20)) grid = 1u << 20;
    if (mode == CRDT_FOLD_DELTA)
        hipLaunchKernelGGL((fold_sort_kernel<kFoldWaves, true>), dim3(grid), dim3(kFoldWaves * 64), 0, stream, dst, sb,
                           out, wk);
    else
        hipLaunchKernelGGL((fold_sort_kernel<kFoldWaves, false>), dim3(grid), dim3(kFoldWaves * 64), 0, stream, dst,
                           sb, out, wk);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((fold_block_kernel<kFoldNT, kFoldIPT>), dim3(block_grid), dim3(kFoldNT), 0, stream, mode, dst,
                       sb, out, scr, wk);
    return hipGetLastError();
}

}  // namespace crdt
