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
//  * fold_wave_kernel: one wavefront per document while the document fits
//    CAP slots and each source has <= 64 entries and <= 64 tombstones.  The
//    document lives in two LDS ping-pong buffers; a step is one wave-wide
//    sorted merge (binary searches in LDS + ballot compaction).  A document
//    that outgrows CAP mid-fold is handed to the block path (nothing was
//    written yet, so it restarts there).
//  * fold_block_kernel: persistent workgroups, merge-path walk per step
//    (merge_block.hpp), ping-pong between the output slots and a scratch copy.
#include "crdt_device.hpp"
#include "merge_block.hpp"

namespace crdt {

// LDS of one wavefront: the document (two ping-pong buffers of CAP slots) and
// ALL of its sources (entries, tombstones, version vectors), loaded in one
// burst so that no fold step waits on HBM.
template <int CAP>
struct FoldWaveSmem {
    static constexpr int SCAP = 128;  // Σ source entries of a doc
    static constexpr int TCAP = 64;   // Σ tombstones of a doc
    static constexpr int VCAP = 256;  // Σ source VV words (sources x R)
    static constexpr int MCAP = 64;   // sources per doc
    uint64_t bk[2][CAP];
    uint64_t bc[2][CAP];
    uint32_t ba[2][CAP];
    uint32_t kp[CAP + 1];   // exclusive prefix of surviving document entries
    uint32_t mark[CAP];     // doc slot -> (src lane + 1) that owns it this step
    uint32_t tmark[CAP];    // doc slot -> (tombstone lane + 1) that hits it
    uint32_t stomb[64];     // src lane -> (tombstone lane + 1) on the same key
    uint64_t sk[SCAP];
    uint64_t sc[SCAP];
    uint32_t sa[SCAP];
    uint64_t tk[TCAP];
    uint64_t tc[TCAP];
    uint32_t ta[TCAP];
    uint64_t svv[VCAP];
    uint32_t soff[MCAP + 1];  // source j: entries [soff[j], soff[j+1]) relative to the doc
    uint32_t toff[MCAP + 1];
    uint32_t sact[MCAP];
    uint64_t dvv[CRDT_MAX_R];
};

// Burst-load n_elems 8/4/8-byte entry triples starting at o into LDS (lanes
// stride 64; unconditional buffer loads, out-of-range lanes read 0).
template <int CHUNKS>
__device__ __forceinline__ void burst_entries(uint64_t* k, uint32_t* a, uint64_t* c, const uint64_t* gk,
                                              const uint32_t* ga, const uint64_t* gc, uint32_t o, uint32_t n,
                                              uint32_t lane) {
    const rsrc_t rk = make_rsrc(gk + o, n * 8u), ra = make_rsrc(ga + o, n * 4u), rc = make_rsrc(gc + o, n * 8u);
    uint64_t kk[CHUNKS], cc[CHUNKS];
    uint32_t aa[CHUNKS];
#pragma unroll
    for (int q = 0; q < CHUNKS; ++q) {
        const uint32_t i = q * 64 + lane;
        kk[q] = ld64(rk, i * 8u);
        aa[q] = ld32(ra, i * 4u);
        cc[q] = ld64(rc, i * 8u);
    }
#pragma unroll
    for (int q = 0; q < CHUNKS; ++q) {
        const uint32_t i = q * 64 + lane;
        k[i] = kk[q];
        a[i] = aa[q];
        c[i] = cc[q];
    }
}

template <int WAVES, int CAP, int LOGCAP>
__global__ __launch_bounds__(WAVES * 64) void fold_wave_kernel(int mode, BatchView dst, SrcView sb, OutView out,
                                                                 Work wk) {
    using Smem = FoldWaveSmem<CAP>;
    __shared__ Smem smem[WAVES];
    constexpr int NCH = CAP / 64;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t w = threadIdx.x >> 6;
    Smem& m = smem[w];
    const uint32_t R = dst.R;
    const uint32_t n_docs = dst.n_docs;
    const uint64_t lt = low_mask(lane);
    const bool delta = mode == CRDT_FOLD_DELTA;
    uint32_t err = 0;

    for (uint32_t d0 = blockIdx.x * WAVES + w; d0 < n_docs; d0 += gridDim.x * WAVES) {
        const uint32_t d = uniform(d0);
        const uint32_t s0 = sb.doc_srcs[d], s1 = sb.doc_srcs[d + 1];
        const uint32_t ms = s1 - s0;
        const uint32_t doff = dst.offsets[d];
        const uint32_t e0 = sb.entry_off[s0], E = sb.entry_off[s1] - e0;
        const uint32_t t0 = (sb.tomb_off && delta) ? sb.tomb_off[s0] : 0u;
        const uint32_t X = (sb.tomb_off && delta) ? sb.tomb_off[s1] - t0 : 0u;
        const uint32_t obase = doff + e0;
        uint32_t n = live_count(dst.offsets, dst.counts, d);
        if (lane == 0) {
            out.offsets[d] = obase;
            if (d == n_docs - 1) out.offsets[n_docs] = dst.offsets[n_docs] + sb.entry_off[sb.doc_srcs[n_docs]];
        }
        // eligibility for the LDS path (else: block path, nothing written yet)
        bool bad = n > CAP || E > Smem::SCAP || X > Smem::TCAP || ms > Smem::MCAP || ms * R > Smem::VCAP;
        if (!bad) {
            const uint32_t k = s0 + lane;
            const uint32_t c = lane < ms ? sb.entry_off[k + 1] - sb.entry_off[k] : 0u;
            const uint32_t x = (lane < ms && X) ? sb.tomb_off[k + 1] - sb.tomb_off[k] : 0u;
            bad = ballot(c > 64 || x > 64) != 0;
        }
        if (bad) {
            if (lane == 0) wk.worklist[atomicAdd(wk.wl_count, 1u)] = d;
            continue;
        }
        // ---- one burst: document, source entries, tombstones, VVs, actors, offsets
        burst_entries<NCH>(m.bk[0], m.ba[0], m.bc[0], dst.keys, dst.actors, dst.counters, doff, n, lane);
        burst_entries<Smem::SCAP / 64>(m.sk, m.sa, m.sc, sb.keys, sb.actors, sb.counters, e0, E, lane);
        if (delta) burst_entries<Smem::TCAP / 64>(m.tk, m.ta, m.tc, sb.tkeys, sb.tactors, sb.tcounters, t0, X, lane);
        {
            const rsrc_t rv = make_rsrc(sb.vv + (size_t)s0 * R, ms * R * 8u);
            uint64_t vq[Smem::VCAP / 64];
#pragma unroll
            for (int q = 0; q < Smem::VCAP / 64; ++q) vq[q] = ld64(rv, (q * 64 + lane) * 8u);
            const uint32_t eo = ld32(make_rsrc(sb.entry_off + s0, (ms + 1) * 4u), lane * 4u);
            const uint32_t eo2 = ld32(make_rsrc(sb.entry_off + s0, (ms + 1) * 4u), (64 + lane) * 4u);
            const uint32_t to = X ? ld32(make_rsrc(sb.tomb_off + s0, (ms + 1) * 4u), lane * 4u) : 0u;
            const uint32_t to2 = X ? ld32(make_rsrc(sb.tomb_off + s0, (ms + 1) * 4u), (64 + lane) * 4u) : 0u;
            const uint32_t ac = ld32(make_rsrc(sb.src_actor + s0, ms * 4u), lane * 4u);
            const uint64_t dv = ld64(make_rsrc(dst.vv + (size_t)d * R, R * 8u), lane * 8u);
#pragma unroll
            for (int q = 0; q < Smem::VCAP / 64; ++q) m.svv[q * 64 + lane] = vq[q];
            m.soff[lane] = eo - e0;
            if (lane == 0) m.soff[64] = eo2 - e0;
            m.toff[lane] = to - t0;
            if (lane == 0) m.toff[64] = to2 - t0;
            m.sact[lane] = ac;
            m.dvv[lane] = dv;
        }
        m.stomb[lane] = 0;
#pragma unroll
        for (int q = 0; q < NCH; ++q) {
            m.mark[q * 64 + lane] = 0;
            m.tmark[q * 64 + lane] = 0;
        }
        wave_sync();

        uint32_t cur = 0;
        bool bailed = false;
        for (uint32_t j = 0; j < ms; ++j) {
            const uint32_t ej = m.soff[j], c = m.soff[j + 1] - ej;
            const uint32_t tj = delta ? m.toff[j] : 0u;
            const uint64_t* svv = m.svv + j * R;
            const bool sv = lane < c;
            const uint64_t skey = sv ? m.sk[ej + lane] : 0ull;
            const uint32_t sact = sv ? m.sa[ej + lane] : 0u;
            const uint64_t scnt = sv ? m.sc[ej + lane] : 0ull;

            // path select (awset-delta_test.go:53)
            uint32_t perr = 0;
            const bool full = !delta || vv_counter(m.dvv, R, m.sact[j], perr) == 0;
            err |= perr;
            if (perr) break;  // the reference panics here; outputs undefined
            const uint32_t x = full ? 0u : m.toff[j + 1] - tj;  // tombstones matter only on the delta path
            const bool tv = lane < x;
            const uint64_t tkey = tv ? m.tk[tj + lane] : 0ull;
            const uint32_t tact = tv ? m.ta[tj + lane] : 0u;
            const uint64_t tcnt = tv ? m.tc[tj + lane] : 0ull;

            // searches: src key in the doc; tombstone key in the doc and in src
            const uint32_t f = lower_bound_adapt<LOGCAP>(m.bk[cur], n, skey);
            const bool in_d = sv && f < n && m.bk[cur][f < CAP ? f : 0] == skey;
            const bool changed = sv && (full || !has_dot(m.dvv, R, sact, scnt, err));
            bool eff = false, t_in_d = false;
            uint32_t g = 0, q = 0;
            if (x) {
                g = lower_bound_adapt<6>(m.sk + ej, c, tkey);
                q = lower_bound_adapt<LOGCAP>(m.bk[cur], n, tkey);
                const bool in_s = tv && g < c && m.sk[ej + (g & 63)] == tkey;
                t_in_d = tv && q < n && m.bk[cur][q < CAP ? q : 0] == tkey;
                // awset-delta_test.go:93-102: a tombstone re-added since is dropped
                eff = tv && !(in_s && (m.sa[ej + (g & 63)] != tact || m.sc[ej + (g & 63)] > tcnt));
                if (eff && in_s) m.stomb[g & 63] = lane + 1;
                if (eff && t_in_d) m.tmark[q] = lane + 1;
            }
            if (!full && !ballot(changed) && !ballot(eff)) {  // :60 no-op, VV untouched
                wave_sync();
                if (eff && t_in_d) m.tmark[q] = 0;
                if (eff && g < 64) m.stomb[g & 63] = 0;
                continue;
            }
            if (in_d) m.mark[f] = lane + 1;
            wave_sync();

            // decisions for src lanes (they own every key present in src)
            bool pres_s = false;
            uint32_t oa_s = sact;
            uint64_t oc_s = scnt;
            if (sv) {
                if (in_d) {
                    pres_s = true;
                    if (!changed) {
                        oa_s = m.ba[cur][f];
                        oc_s = m.bc[cur][f];
                    }
                } else {
                    pres_s = changed && !has_dot(m.dvv, R, sact, scnt, err);
                }
                const uint32_t h = m.stomb[lane];
                if (pres_s && h) pres_s = has_dot(m.dvv, R, m.ta[tj + h - 1], m.tc[tj + h - 1], err);
            }
            const uint64_t emit_s = ballot(pres_s);

            // decisions for document entries not present in src
            bool emit_d[NCH];
            uint32_t g_d[NCH];
            uint32_t carry = 0;
#pragma unroll
            for (int qq = 0; qq < NCH; ++qq) {
                const uint32_t idx = qq * 64 + lane;
                const bool valid = idx < n;
                const uint64_t key = m.bk[cur][idx];
                const bool owned = m.mark[idx] != 0;
                const uint32_t th = m.tmark[idx];
                bool pres = false;
                if (valid && !owned) {
                    pres = full ? !has_dot(svv, R, m.ba[cur][idx], m.bc[cur][idx], err) : true;
                    if (pres && th) pres = has_dot(m.dvv, R, m.ta[tj + th - 1], m.tc[tj + th - 1], err);
                }
                // # src keys < key (its shift by inserted src entries)
                g_d[qq] = lower_bound_adapt<6>(m.sk + ej, c, key);
                const uint64_t bm = ballot(pres);
                if (valid) m.kp[idx] = carry + popc(bm & lt);
                emit_d[qq] = pres;
                carry += popc(bm);
            }
            if (lane == 0) m.kp[n] = carry;
            wave_sync();
            const uint32_t new_n = carry + popc(emit_s);
            if (new_n > CAP) {
                bailed = true;
                break;
            }
            const uint32_t nx = cur ^ 1u;
            if (pres_s) {
                const uint32_t pos = popc(emit_s & lt) + m.kp[f];
                m.bk[nx][pos] = skey;
                m.ba[nx][pos] = oa_s;
                m.bc[nx][pos] = oc_s;
            }
#pragma unroll
            for (int qq = 0; qq < NCH; ++qq) {
                if (emit_d[qq]) {
                    const uint32_t idx = qq * 64 + lane;
                    const uint32_t pos = m.kp[idx] + popc(emit_s & low_mask(g_d[qq]));
                    m.bk[nx][pos] = m.bk[cur][idx];
                    m.ba[nx][pos] = m.ba[cur][idx];
                    m.bc[nx][pos] = m.bc[cur][idx];
                }
            }
            // clear this step's marks
            if (in_d) m.mark[f] = 0;
            if (eff && t_in_d) m.tmark[q] = 0;
            if (eff && g < 64) m.stomb[g & 63] = 0;
            if (lane < R) m.dvv[lane] = max(m.dvv[lane], svv[lane]);
            n = new_n;
            cur = nx;
            wave_sync();
        }
        if (bailed) {
            if (lane == 0) wk.worklist[atomicAdd(wk.wl_count, 1u)] = d;
            wave_sync();
            continue;
        }
        const rsrc_t ok = make_rsrc(out.keys + obase, n * 8u), oa = make_rsrc(out.actors + obase, n * 4u),
                     oc = make_rsrc(out.counters + obase, n * 8u);
#pragma unroll
        for (int qq = 0; qq < NCH; ++qq) {
            const uint32_t i = qq * 64 + lane;
            st64<kAuxNT>(m.bk[cur][i], ok, i * 8u);
            st32<kAuxNT>(m.ba[cur][i], oa, i * 4u);
            st64<kAuxNT>(m.bc[cur][i], oc, i * 8u);
        }
        if (lane == 0) out.counts[d] = n;
        if (lane < R) out.vv[(size_t)d * R + lane] = m.dvv[lane];
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
        const uint32_t total = __hip_atomic_load(wk.wl_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        if (slot >= total) break;
        const uint32_t d = wk.worklist[slot];
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
constexpr int kFoldCap = 128;
constexpr int kFoldLogCap = 7;
constexpr int kFoldNT = 256;
constexpr int kFoldIPT = 4;

hipError_t launch_fold(int mode, const BatchView& dst, const SrcView& sb, const OutView& out, const Scratch& scr,
                       const Work& wk, uint32_t block_grid, hipStream_t stream) {
    if (dst.n_docs == 0) return hipSuccess;
    uint32_t grid = (dst.n_docs + kFoldWaves - 1) / kFoldWaves;
    if (grid > (1u << 20)) grid = 1u << 20;
    hipLaunchKernelGGL((fold_wave_kernel<kFoldWaves, kFoldCap, kFoldLogCap>), dim3(grid), dim3(kFoldWaves * 64), 0,
                       stream, mode, dst, sb, out, wk);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((fold_block_kernel<kFoldNT, kFoldIPT>), dim3(block_grid), dim3(kFoldNT), 0, stream, mode, dst,
                       sb, out, scr, wk);
    return hipGetLastError();
}

}  // namespace crdt
