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

template <int CAP>
struct FoldWaveSmem {
    uint64_t bk[2][CAP];
    uint64_t bc[2][CAP];
    uint32_t ba[2][CAP];
    uint32_t kp[CAP + 1];
    uint64_t sk[64];
    uint64_t sc[64];
    uint64_t tk[64];
    uint64_t tc[64];
    uint32_t sa[64];
    uint32_t ta[64];
    uint32_t teff[64];
    uint64_t dvv[CRDT_MAX_R];
    uint64_t svv[CRDT_MAX_R];
};

template <int WAVES, int CAP, int LOGCAP>
__global__ __launch_bounds__(WAVES * 64) void fold_wave_kernel(int mode, BatchView dst, SrcView sb, OutView out,
                                                                 Work wk) {
    __shared__ FoldWaveSmem<CAP> smem[WAVES];
    constexpr int NCH = CAP / 64;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t w = threadIdx.x >> 6;
    FoldWaveSmem<CAP>& m = smem[w];
    const uint32_t R = dst.R;
    const uint32_t n_docs = dst.n_docs;
    const uint64_t lt = low_mask(lane);
    uint32_t err = 0;

    for (uint32_t d0 = blockIdx.x * WAVES + w; d0 < n_docs; d0 += gridDim.x * WAVES) {
        const uint32_t d = uniform(d0);
        const uint32_t s0 = sb.doc_srcs[d], s1 = sb.doc_srcs[d + 1];
        const uint32_t doff = dst.offsets[d];
        const uint32_t obase = doff + sb.entry_off[s0];
        uint32_t n = live_count(dst.offsets, dst.counts, d);
        if (lane == 0) {
            out.offsets[d] = obase;
            if (d == n_docs - 1) out.offsets[n_docs] = dst.offsets[n_docs] + sb.entry_off[sb.doc_srcs[n_docs]];
        }
        // eligibility for the wave path
        bool bad = n > CAP;
        for (uint32_t k = s0 + lane; k < s1; k += 64) {
            const uint32_t c = sb.entry_off[k + 1] - sb.entry_off[k];
            const uint32_t x = sb.tomb_off ? sb.tomb_off[k + 1] - sb.tomb_off[k] : 0u;
            bad |= (c > 64) || (x > 64);
        }
        if (ballot(bad)) {
            if (lane == 0) wk.worklist[atomicAdd(wk.wl_count, 1u)] = d;
            continue;
        }
        for (uint32_t i = lane; i < n; i += 64) {
            m.bk[0][i] = dst.keys[doff + i];
            m.ba[0][i] = dst.actors[doff + i];
            m.bc[0][i] = dst.counters[doff + i];
        }
        if (lane < R) m.dvv[lane] = dst.vv[(size_t)d * R + lane];
        uint32_t cur = 0;
        bool bailed = false;

        for (uint32_t k = s0; k < s1; ++k) {
            const uint32_t e0 = sb.entry_off[k];
            const uint32_t c = sb.entry_off[k + 1] - e0;
            const uint32_t t0 = sb.tomb_off ? sb.tomb_off[k] : 0u;
            const uint32_t x = sb.tomb_off ? sb.tomb_off[k + 1] - t0 : 0u;
            const bool sv = lane < c, tv = lane < x;
            uint64_t skey = 0, scnt = 0;
            uint32_t sact = 0;
            if (sv) {
                skey = sb.keys[e0 + lane];
                sact = sb.actors[e0 + lane];
                scnt = sb.counters[e0 + lane];
            }
            m.sk[lane] = skey;
            m.sa[lane] = sact;
            m.sc[lane] = scnt;
            uint64_t tkey = 0, tcnt = 0;
            uint32_t tact = 0;
            if (tv && mode == CRDT_FOLD_DELTA) {
                tkey = sb.tkeys[t0 + lane];
                tact = sb.tactors[t0 + lane];
                tcnt = sb.tcounters[t0 + lane];
            }
            m.tk[lane] = tkey;
            m.ta[lane] = tact;
            m.tc[lane] = tcnt;
            if (lane < R) m.svv[lane] = sb.vv[(size_t)k * R + lane];
            wave_sync();

            // path select (awset-delta_test.go:53)
            uint32_t perr = 0;
            const bool full = (mode != CRDT_FOLD_DELTA) || vv_counter(m.dvv, R, sb.src_actor[k], perr) == 0;
            err |= perr;
            if (perr) {  // the reference panics here; stop this document
                wave_sync();
                break;
            }
            const uint32_t xd = full ? 0u : x;  // tombstones matter only on the delta path

            // src entry lanes: position in the document, "changed" (dot pruning)
            const uint32_t f = lower_bound_pow<LOGCAP>(m.bk[cur], n, skey);
            const bool in_d = sv && f < n && m.bk[cur][f] == skey;
            const bool changed = sv && (full || !has_dot(m.dvv, R, sact, scnt, err));
            // tombstone lanes: effective unless re-added (awset-delta_test.go:93-102)
            bool eff = false;
            if (lane < xd) {
                const uint32_t g = lower_bound_pow<6>(m.sk, c, tkey);
                const bool in_s = g < c && m.sk[g] == tkey;
                eff = !(in_s && (m.sa[g] != tact || m.sc[g] > tcnt));
            }
            m.teff[lane] = eff ? 1u : 0u;
            if (!full && !ballot(changed) && !ballot(eff)) {  // :60 no-op, VV untouched
                wave_sync();
                continue;
            }
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
                if (pres_s && xd) {
                    const uint32_t h = lower_bound_pow<6>(m.tk, xd, skey);
                    if (h < xd && m.tk[h] == skey && m.teff[h]) pres_s = has_dot(m.dvv, R, m.ta[h], m.tc[h], err);
                }
            }
            const uint64_t emit_s = ballot(pres_s);

            // decisions for document entries not present in src
            bool emit_d[NCH];
            uint32_t g_d[NCH];
            uint32_t carry = 0;
#pragma unroll
            for (int q = 0; q < NCH; ++q) {
                const uint32_t idx = q * 64 + lane;
                const bool valid = idx < n;
                const uint64_t key = valid ? m.bk[cur][idx] : 0ull;
                const uint32_t g = lower_bound_pow<6>(m.sk, c, key);
                const bool in_s = valid && g < c && m.sk[g] == key;
                bool pres = false;
                if (valid && !in_s) {
                    pres = full ? !has_dot(m.svv, R, m.ba[cur][idx], m.bc[cur][idx], err) : true;
                    if (pres && xd) {
                        const uint32_t h = lower_bound_pow<6>(m.tk, xd, key);
                        if (h < xd && m.tk[h] == key && m.teff[h]) pres = has_dot(m.dvv, R, m.ta[h], m.tc[h], err);
                    }
                }
                const uint64_t bm = ballot(pres);
                if (valid) m.kp[idx] = carry + popc(bm & lt);
                emit_d[q] = pres;
                g_d[q] = g;
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
            for (int q = 0; q < NCH; ++q) {
                if (emit_d[q]) {
                    const uint32_t idx = q * 64 + lane;
                    const uint32_t pos = m.kp[idx] + popc(emit_s & low_mask(g_d[q]));
                    m.bk[nx][pos] = m.bk[cur][idx];
                    m.ba[nx][pos] = m.ba[cur][idx];
                    m.bc[nx][pos] = m.bc[cur][idx];
                }
            }
            if (lane < R) m.dvv[lane] = max(m.dvv[lane], m.svv[lane]);
            n = new_n;
            cur = nx;
            wave_sync();
        }
        if (bailed) {
            if (lane == 0) wk.worklist[atomicAdd(wk.wl_count, 1u)] = d;
            wave_sync();
            continue;
        }
        for (uint32_t i = lane; i < n; i += 64) {
            out.keys[obase + i] = m.bk[cur][i];
            out.actors[obase + i] = m.ba[cur][i];
            out.counters[obase + i] = m.bc[cur][i];
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

constexpr int kFoldWaves = 4;
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
