// Full-state AWSet join over a batch of documents: out[d] = dst[d] <- src[d].
// Replaces (*AWSet).Merge / merge, awset.go:103-161, for millions of docs.
//
// Two paths, one launch each:
//  * join_wave_kernel: one wavefront per document when both sides hold <= 64
//    entries.  Lane i owns dst entry i and src entry i; both key lists are
//    staged in LDS; each lane binary-searches its key in the other side
//    (7 LDS probes), decides with HasDot against the other side's VV in LDS,
//    and the survivors are compacted with two 64-bit ballots: a survivor's
//    output slot is (kept lanes of its own side below it) + (kept entries of
//    the other side with a smaller key), both popcounts.  Output is sorted by
//    key, written once.  Larger documents are pushed to a worklist.
//  * join_block_kernel: persistent workgroups pop the worklist and merge each
//    large document with the merge-path walk of merge_block.hpp.
#include "crdt_device.hpp"
#include "merge_block.hpp"

namespace crdt {

// CRDT_JOIN_PAD_STORES (default 1): the staged stores (STG) of each output
// array run on past the last survivor to the end of its 64-byte sector,
// within the document's own output capacity, writing zeros there (slack
// slots, whose contents the ABI leaves unspecified), so no sector of a
// document's output is written partially.  A partially written sector costs
// the memory far more than its bytes: the config-2 exchange 1.216 -> 1.124 ms
// per launch padded to 128-byte lines (-7.6 %, three interleaved rounds,
// identical live outputs; profiles/r05b_exchange_pad_ab.log), 1.125 -> 1.108
// ms more padded to 64-byte sectors (profiles/r05d_exchange_pad_ab.log; 2 =
// 128-byte lines, 0 = off).  The folds gain nothing from it (their stores are
// not what binds them: profiles/r05b_fold_stage_pad_ab.log), so they keep
// their own store forms.
#ifndef CRDT_JOIN_WAVE_PUSH
#define CRDT_JOIN_WAVE_PUSH 1  // 0: one worklist atomic per large document (A/B builds)
#endif
#ifndef CRDT_JOIN_PAD_STORES
#define CRDT_JOIN_PAD_STORES 1
#endif

struct JoinMeta {
    uint32_t doff, soff, dn, sn, cap;
};

// Metadata of up to 64 documents, lane i = document first + i*stride: one
// unconditional vector load per field (indices clamped).
struct MetaVec {
    uint32_t doff, soff, dend, send, dnx, snx;
};

__device__ __forceinline__ MetaVec meta_vec_issue(const BatchView& dst, const BatchView& src, uint32_t first,
                                                  uint32_t stride, uint32_t lane) {
    const uint32_t n = dst.n_docs;
    const uint32_t d0 = first + lane * stride;
    const uint32_t dd = d0 < n ? d0 : n - 1;
    MetaVec v;
    v.doff = dst.offsets[dd];
    v.soff = src.offsets[dd];
    v.dend = dst.counts ? dst.counts[dd] : dst.offsets[dd + 1];
    v.send = src.counts ? src.counts[dd] : src.offsets[dd + 1];
    if (CRDT_JOIN_PAD_STORES) {  // slot bounds of the next document: the output capacity
        v.dnx = dst.counts ? dst.offsets[dd + 1] : v.dend;
        v.snx = src.counts ? src.offsets[dd + 1] : v.send;
    } else {
        v.dnx = v.snx = 0;
    }
    return v;
}

__device__ __forceinline__ JoinMeta meta_of(const BatchView& dst, const BatchView& src, const MetaVec& v,
                                            uint32_t i) {
    JoinMeta m;
    m.doff = (uint32_t)__builtin_amdgcn_readlane((int)v.doff, (int)i);
    m.soff = (uint32_t)__builtin_amdgcn_readlane((int)v.soff, (int)i);
    const uint32_t a = (uint32_t)__builtin_amdgcn_readlane((int)v.dend, (int)i);
    const uint32_t b = (uint32_t)__builtin_amdgcn_readlane((int)v.send, (int)i);
    m.dn = dst.counts ? a : a - m.doff;
    m.sn = src.counts ? b : b - m.soff;
    m.cap = 0;
    if (CRDT_JOIN_PAD_STORES)
        m.cap = (uint32_t)__builtin_amdgcn_readlane((int)v.dnx, (int)i) - m.doff +
                (uint32_t)__builtin_amdgcn_readlane((int)v.snx, (int)i) - m.soff;
    return m;
}

// One document's entries, one per lane (lane i: dst entry i, src entry i, VV[i]).
struct JoinLanes {
    uint64_t dk, dc, sk, sc, vd, vs;
    uint32_t da, sa;
};

// ld = false (document on the block path, or none): every lane reads 0, no traffic.
__device__ __forceinline__ void lanes_issue(JoinLanes& L, const BatchView& dst, const BatchView& src,
                                            const JoinMeta& m, uint32_t d, bool ld, uint32_t lane, uint32_t R) {
    const uint32_t dn = ld ? m.dn : 0u, sn = ld ? m.sn : 0u, rv = ld ? R : 0u;
    const uint32_t o8 = lane * 8u, o4 = lane * 4u;
    // non-temporal entry loads: each entry is read once (1.3 % faster than the
    // default policy, and than aux 1 / 3, measured on one box)
    constexpr int LA = kAuxNT;
    auto l64 = [](rsrc_t r, uint32_t off) {
        return __builtin_bit_cast(uint64_t, __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, LA));
    };
    auto l32 = [](rsrc_t r, uint32_t off) { return (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, LA); };
    L.dk = l64(make_rsrc(dst.keys + m.doff, dn * 8u), o8);
    L.da = l32(make_rsrc(dst.actors + m.doff, dn * 4u), o4);
    L.dc = l64(make_rsrc(dst.counters + m.doff, dn * 8u), o8);
    L.sk = l64(make_rsrc(src.keys + m.soff, sn * 8u), o8);
    L.sa = l32(make_rsrc(src.actors + m.soff, sn * 4u), o4);
    L.sc = l64(make_rsrc(src.counters + m.soff, sn * 8u), o8);
    const size_t vo = ld ? (size_t)d * R : 0;
    L.vd = ld64(make_rsrc(dst.vv + vo, rv * 8u), o8);
    L.vs = ld64(make_rsrc(src.vv + vo, rv * 8u), o8);
}

// Per wave: key[0..64) dst keys, key[64..128) src keys; vv[0..64) dst VV,
// vv[64..128) src VV.  Staged stores (STG) then reuse key/vv/act as the
// document's output image: keys, counters and actors by output slot.
template <int WAVES>
struct JoinWaveSmem {
    uint64_t key[WAVES][128];
    uint64_t vv[WAVES][128];
    uint32_t act[WAVES][128];
};

// Merge document d whose entries are in L (awset.go:107-161).  AUX: cache
// policy of the entry stores (0 plain, kAuxNT non-temporal).
// EXCH: also write out2 = src <- dst (the exchange's other direction).  Both
// directions keep the same keys at the same slots (a dst-only key survives iff
// srcVV has not seen it, a src-only key iff dstVV has not, in either
// direction); only a common key's dot differs -- the src dot wins
// (awset.go:142), so out2 takes the dst lane's own dot.  out2.keys may be
// out.keys (one shared key column): its key stores are then skipped.
// STG: survivors are placed in LDS by output slot first and each output array
// is written lane l -> slot l (and l + 64): every store instruction covers
// whole contiguous cache lines, instead of the dst lanes and the src lanes
// each writing an interleaved subset of the same lines.
template <int WAVES, int AUX, bool EXCH, bool STG>
__device__ __forceinline__ void join_doc(JoinWaveSmem<WAVES>& sm, uint32_t w, const JoinLanes& L, const JoinMeta& m,
                                         uint32_t d, bool small, const OutView& out, const OutView& out2,
                                         uint32_t n_docs, uint32_t end_off, uint32_t R, uint32_t lane, uint64_t lt,
                                         uint32_t& err) {
    const uint32_t obase = m.doff + m.soff;
    const uint32_t dnn = small ? m.dn : 0u, snn = small ? m.sn : 0u;
    const bool dv = lane < dnn, sv = lane < snn;
    uint64_t* const dkey = sm.key[w];
    uint64_t* const skey = sm.key[w] + 64;
    uint64_t* const dvv = sm.vv[w];
    uint64_t* const svv = sm.vv[w] + 64;
    dvv[lane] = L.vd;
    svv[lane] = L.vs;
    dkey[lane] = L.dk;
    skey[lane] = L.sk;
    wave_sync();
    // # src keys < dk, # dst keys < sk
    const uint32_t j = lower_bound_pow<6>(skey, snn, L.dk);
    const uint32_t i = lower_bound_pow<6>(dkey, dnn, L.sk);
    const bool dmatch = dv && j < snn && skey[j & 63] == L.dk;
    const bool smatch = sv && i < dnn && dkey[i & 63] == L.sk;
    // awset.go:145-159: a dst-only key survives unless src's clock covers it.
    const bool dh = has_dot_bf(svv, R, L.da, L.dc, dv && !dmatch, err);
    // awset.go:130-140: a src-only key is added unless dst's clock covers it.
    const bool sh = has_dot_bf(dvv, R, L.sa, L.sc, sv && !smatch, err);
    const bool dkeep = dv && (dmatch || !dh);
    const bool skeep = sv && !smatch && !sh;
    const uint64_t dm = ballot(dkeep), smk = ballot(skeep);
    // awset.go:142: the src dot wins on a common key (lane j holds it).
    const uint32_t ma = __shfl(L.sa, (int)(j & 63));
    const uint64_t mc = __shfl(L.sc, (int)(j & 63));
    const uint32_t dpos = below(dm) + popc(smk & low_mask(j));
    const uint32_t spos = below(smk) + popc(dm & low_mask(i));
    const uint32_t n_out = popc(dm) + popc(smk);
    const bool kshare = EXCH && out2.keys == out.keys;
    if (STG) {
        // the output image: slot -> key / counter / actor (out = dst <- src)
        uint64_t* const ik = sm.key[w];
        uint64_t* const ic = sm.vv[w];
        uint32_t* const ia = sm.act[w];
        wave_sync();  // every lane's probes of this document are done
        if (dkeep) {
            ik[dpos] = L.dk;
            ic[dpos] = dmatch ? mc : L.dc;
            ia[dpos] = dmatch ? ma : L.da;
        }
        if (skeep) {
            ik[spos] = L.sk;
            ic[spos] = L.sc;
            ia[spos] = L.sa;
        }
        wave_sync();
        // (slots past the survivors read as 0: the padding below writes zeros)
        const bool l0 = lane < n_out, l1 = lane + 64u < n_out;
        const uint64_t k0 = l0 ? ik[lane] : 0ull, k1 = l1 ? ik[lane + 64] : 0ull;
        const uint64_t c0 = l0 ? ic[lane] : 0ull, c1 = l1 ? ic[lane + 64] : 0ull;
        const uint32_t a0 = l0 ? ia[lane] : 0u, a1 = l1 ? ia[lane + 64] : 0u;
        // slots each array's stores cover: the survivors, or (padded) through
        // the end of the last survivor's cache line, within the capacity
        uint32_t n8 = n_out, n4 = n_out;
        if (CRDT_JOIN_PAD_STORES && small && n_out != 0) {  // (a large document: the block / tile path writes it)
            const uint32_t lim = min(m.cap, 128u);
            // 1: to the end of the 64-byte sector; 2 (diagnostic): of the 128-byte line
            constexpr uint32_t m8 = CRDT_JOIN_PAD_STORES == 2 ? 15u : 7u, m4 = CRDT_JOIN_PAD_STORES == 2 ? 31u : 15u;
            n8 = min(((obase + n_out + m8) & ~m8) - obase, lim);
            n4 = min(((obase + n_out + m4) & ~m4) - obase, lim);
            n8 = max(n8, n_out);
            n4 = max(n4, n_out);
        }
        const rsrc_t ok = make_rsrc(out.keys + obase, n8 * 8u);
        const rsrc_t oa = make_rsrc(out.actors + obase, n4 * 4u);
        const rsrc_t oc = make_rsrc(out.counters + obase, n8 * 8u);
        st64<AUX>(k0, ok, lane * 8u);
        st64<AUX>(k1, ok, lane * 8u + 512u);
        st32<AUX>(a0, oa, lane * 4u);
        st32<AUX>(a1, oa, lane * 4u + 256u);
        st64<AUX>(c0, oc, lane * 8u);
        st64<AUX>(c1, oc, lane * 8u + 512u);
        if (EXCH) {
            // out2 = src <- dst: the same image but a common key keeps the dst dot
            wave_sync();
            if (dmatch) {
                ic[dpos] = L.dc;
                ia[dpos] = L.da;
            }
            wave_sync();
            const uint64_t e0 = l0 ? ic[lane] : 0ull, e1 = l1 ? ic[lane + 64] : 0ull;
            const uint32_t b0 = l0 ? ia[lane] : 0u, b1 = l1 ? ia[lane + 64] : 0u;
            const rsrc_t pk = make_rsrc(out2.keys + obase, kshare ? 0u : n8 * 8u);
            const rsrc_t pa = make_rsrc(out2.actors + obase, n4 * 4u);
            const rsrc_t pc = make_rsrc(out2.counters + obase, n8 * 8u);
            if (!kshare) {
                st64<AUX>(k0, pk, lane * 8u);
                st64<AUX>(k1, pk, lane * 8u + 512u);
            }
            st32<AUX>(b0, pa, lane * 4u);
            st32<AUX>(b1, pa, lane * 4u + 256u);
            st64<AUX>(e0, pc, lane * 8u);
            st64<AUX>(e1, pc, lane * 8u + 512u);
        }
    } else {
        const uint32_t cap = dnn + snn;
        const rsrc_t ok = make_rsrc(out.keys + obase, cap * 8u);
        const rsrc_t oa = make_rsrc(out.actors + obase, cap * 4u);
        const rsrc_t oc = make_rsrc(out.counters + obase, cap * 8u);
        const uint32_t d8 = dkeep ? dpos * 8u : kOOB, d4 = dkeep ? dpos * 4u : kOOB;
        const uint32_t s8 = skeep ? spos * 8u : kOOB, s4 = skeep ? spos * 4u : kOOB;
        st64<AUX>(L.dk, ok, d8);
        st32<AUX>(dmatch ? ma : L.da, oa, d4);
        st64<AUX>(dmatch ? mc : L.dc, oc, d8);
        st64<AUX>(L.sk, ok, s8);
        st32<AUX>(L.sa, oa, s4);
        st64<AUX>(L.sc, oc, s8);
        if (EXCH) {
            const rsrc_t pk = make_rsrc(out2.keys + obase, kshare ? 0u : cap * 8u);
            const rsrc_t pa = make_rsrc(out2.actors + obase, cap * 4u);
            const rsrc_t pc = make_rsrc(out2.counters + obase, cap * 8u);
            if (!kshare) {
                st64<AUX>(L.dk, pk, d8);
                st64<AUX>(L.sk, pk, s8);
            }
            st32<AUX>(L.da, pa, d4);
            st64<AUX>(L.dc, pc, d8);
            st32<AUX>(L.sa, pa, s4);
            st64<AUX>(L.sc, pc, s8);
        }
    }
    // slot bounds (every doc), live count and VV (wave path only)
    const bool last = d == n_docs - 1;
    const uint64_t vmax = L.vd > L.vs ? L.vd : L.vs;  // awset.go:160 -> crdt-misc.go:43-55
    st32(lane == 0 ? obase : end_off, make_rsrc(out.offsets + d, last ? 8u : 4u), lane < 2 ? lane * 4u : kOOB);
    st32(n_out, make_rsrc(out.counts + d, small ? 4u : 0u), lane == 0 ? 0u : kOOB);
    st64(vmax, make_rsrc(out.vv + (size_t)d * R, small ? R * 8u : 0u), lane * 8u);
    if (EXCH) {
        st32(lane == 0 ? obase : end_off, make_rsrc(out2.offsets + d, last ? 8u : 4u), lane < 2 ? lane * 4u : kOOB);
        st32(n_out, make_rsrc(out2.counts + d, small ? 4u : 0u), lane == 0 ? 0u : kOOB);
        st64(vmax, make_rsrc(out2.vv + (size_t)d * R, small ? R * 8u : 0u), lane * 8u);
    }
    wave_sync();
}

// A block covers the contiguous documents [blockIdx*WAVES*K, +WAVES*K); wave w
// takes documents base + w + k*WAVES, k < K, so the documents in flight across
// the GPU form one contiguous window (the dispatcher runs blocks roughly in
// order).  Per wave: one metadata vector load for its K documents, then a
// ping-pong pipeline -- the next document's entries are issued before this
// one is merged.  The body is straight-line buffer VMEM, so the compiler's
// vmcnt waits count exactly and the prefetch stays in flight.
#ifndef CRDT_JOIN_WPE  // waves per SIMD the compiler must fit (0: its own choice -- 106 SGPRs, 7 waves)
#define CRDT_JOIN_WPE 0
#endif
#if CRDT_JOIN_WPE
#define CRDT_JOIN_WPE_ATTR __attribute__((amdgpu_waves_per_eu(CRDT_JOIN_WPE)))
#else
#define CRDT_JOIN_WPE_ATTR
#endif
template <int WAVES, int K, int AUX, bool EXCH, bool STG>
__global__ __launch_bounds__(WAVES * 64) CRDT_JOIN_WPE_ATTR void join_wave_kernel(BatchView dst, BatchView src, OutView out, OutView out2,
                                                               Work wk, uint32_t no_large, SlabMap slabs) {
    __shared__ JoinWaveSmem<WAVES> sm;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t w = threadIdx.x >> 6;
    const uint32_t R = dst.R;
    const uint32_t n_docs = dst.n_docs;
    const uint64_t lt = low_mask(lane);
    const uint32_t end_off = dst.offsets[n_docs] + src.offsets[n_docs];
    uint32_t err = 0;

    const uint32_t chunk = slab_chunk(slabs, blockIdx.x);
    if (chunk == 0xFFFFFFFFu || !gate_open(wk)) return;  // (a closed gate: nothing reaches the worklist either)
    const uint32_t first = uniform(chunk * (WAVES * K) + w);
    if (first >= n_docs) return;
    const uint32_t cnt = min((uint32_t)K, (n_docs - first + WAVES - 1) / WAVES);
    const MetaVec mv = meta_vec_issue(dst, src, first, WAVES, lane);

    auto push_large = [&](uint32_t dd) {
        if (CRDT_JOIN_WAVE_PUSH) return;  // pushed below, all at once
        if (lane == 0) {
            if (no_large)
                atomicOr(wk.status, kErrHint);
            else
                push_work(wk, dd, n_docs);
        }
    };
    if (CRDT_JOIN_WAVE_PUSH) {
        // The wave's large documents (lane i: document first + i * WAVES) go to
        // the worklist with ONE atomic on its counter: config 4 pushes 10,800
        // documents, and one counter word takes ~88 M atomics/s, so a push per
        // document serialised ~0.1 ms of the launch on that word.
        const uint32_t dn_l = dst.counts ? mv.dend : mv.dend - mv.doff;
        const uint32_t sn_l = src.counts ? mv.send : mv.send - mv.soff;
        const bool large = lane < cnt && (dn_l > 64 || sn_l > 64);
        const uint64_t bl = ballot(large);
        if (bl) {
            if (no_large) {
                if (lane == 0) atomicOr(wk.status, kErrHint);
            } else {
                uint32_t base = 0;
                if (lane == 0) base = atomicAdd(wk.wl_count, (uint32_t)__builtin_popcountll(bl));
                base = (uint32_t)__builtin_amdgcn_readfirstlane((int)base);
                const uint32_t slot = base + (uint32_t)__builtin_popcountll(bl & lt);
                if (large) {  // bounded as push_work
                    if (slot < n_docs)
                        wk.worklist[slot] = first + lane * WAVES;
                    else
                        atomicOr(wk.status, kErrWorkspace);
                }
            }
        }
    }

    JoinMeta m = meta_of(dst, src, mv, 0);
    uint32_t d = first;
    bool small = m.dn <= 64 && m.sn <= 64;
    JoinLanes LA, LB;
    lanes_issue(LA, dst, src, m, d, small, lane, R);
#pragma unroll 1
    for (uint32_t k = 0;;) {
        // A: issue k+1 into LB, merge LA
        bool more = k + 1 < cnt;
        JoinMeta mn = meta_of(dst, src, mv, more ? k + 1 : 0);
        uint32_t dn = d + WAVES;
        bool small_n = more && mn.dn <= 64 && mn.sn <= 64;
        lanes_issue(LB, dst, src, mn, dn, small_n, lane, R);
        join_doc<WAVES, AUX, EXCH, STG>(sm, w, LA, m, d, small, out, out2, n_docs, end_off, R, lane, lt, err);
        if (!small) push_large(d);
        if (!more) break;
        ++k;
        m = mn;
        d = dn;
        small = small_n;
        // B: issue k+1 into LA, merge LB
        more = k + 1 < cnt;
        mn = meta_of(dst, src, mv, more ? k + 1 : 0);
        dn = d + WAVES;
        small_n = more && mn.dn <= 64 && mn.sn <= 64;
        lanes_issue(LA, dst, src, mn, dn, small_n, lane, R);
        join_doc<WAVES, AUX, EXCH, STG>(sm, w, LB, m, d, small, out, out2, n_docs, end_off, R, lane, lt, err);
        if (!small) push_large(d);
        if (!more) break;
        ++k;
        m = mn;
        d = dn;
        small = small_n;
    }
    flag_error(wk.status, err);
}

// head: which dequeue counter this pass uses (the exchange runs the worklist
// twice, once per direction).
template <int NT, int IPT>
__global__ __launch_bounds__(NT) void join_block_kernel(BatchView dst, BatchView src, OutView out, Work wk,
                                                        uint32_t head, const uint32_t* gate) {
    // gate != nullptr: the tile path (tile.hip) took the worklist unless it set *gate
    if (gate && *gate == 0u) return;
    __shared__ MergeSmem<NT, IPT> sm;
    const uint32_t tid = threadIdx.x;
    const uint32_t R = dst.R;
    uint32_t err = 0;
    const Entries none{nullptr, nullptr, nullptr, 0};
    if (work_total(wk, dst.n_docs) == 0) return;  // empty worklist (set by the previous launch): no dispensing atomics
    for (;;) {
        if (tid == 0) sm.word[0] = atomicAdd(wk.wl_head + head, 1u);
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
        const uint32_t doff = dst.offsets[d], soff = src.offsets[d];
        const Entries D{dst.keys + doff, dst.actors + doff, dst.counters + doff, live_count(dst.offsets, dst.counts, d)};
        const Entries S{src.keys + soff, src.actors + soff, src.counters + soff, live_count(src.offsets, src.counts, d)};
        if (tid < R) {
            sm.dvv[tid] = dst.vv[(size_t)d * R + tid];
            sm.svv[tid] = src.vv[(size_t)d * R + tid];
        }
        __syncthreads();
        const uint32_t obase = doff + soff;
        const EntriesOut O{out.keys + obase, out.actors + obase, out.counters + obase};
        const uint32_t n = block_merge<NT, IPT>(D, S, none, true, R, sm, O, err);
        if (tid == 0) out.counts[d] = n;
        if (tid < R) out.vv[(size_t)d * R + tid] = max(sm.dvv[tid], sm.svv[tid]);
        __syncthreads();
    }
    if (__syncthreads_or(err != 0) && tid == 0) atomicOr(wk.status, kErrActorRange);
}

constexpr int kJoinWaves = 4;
constexpr int kBlockNT = 256;
constexpr int kBlockIPT = 4;

// slab_blocks: G of the block order (crdt_device.hpp SlabMap), 0 = in order
template <int K, int AUX, bool EXCH, bool STG>
static void launch_wave(const BatchView& dst, const BatchView& src, const OutView& out, const OutView& out2,
                        const Work& wk, bool no_large, uint32_t slab_blocks, hipStream_t stream) {
    const uint32_t per_block = kJoinWaves * K;
    const SlabMap sm = slab_map((dst.n_docs + per_block - 1) / per_block, slab_blocks);
    hipLaunchKernelGGL((join_wave_kernel<kJoinWaves, K, AUX, EXCH, STG>), dim3(slab_grid(sm)), dim3(kJoinWaves * 64), 0,
                       stream, dst, src, out, out2, wk, (uint32_t)no_large, sm);
}

template <int AUX, bool EXCH, bool STG>
static void launch_wave_k(uint32_t k, const BatchView& dst, const BatchView& src, const OutView& out,
                          const OutView& out2, const Work& wk, bool no_large, uint32_t sb, hipStream_t stream) {
    switch (k) {
        case 1: launch_wave<1, AUX, EXCH, STG>(dst, src, out, out2, wk, no_large, sb, stream); break;
        case 2: launch_wave<2, AUX, EXCH, STG>(dst, src, out, out2, wk, no_large, sb, stream); break;
        case 4: launch_wave<4, AUX, EXCH, STG>(dst, src, out, out2, wk, no_large, sb, stream); break;
        case 16: launch_wave<16, AUX, EXCH, STG>(dst, src, out, out2, wk, no_large, sb, stream); break;
        default: launch_wave<8, AUX, EXCH, STG>(dst, src, out, out2, wk, no_large, sb, stream); break;
    }
}

template <bool EXCH, bool STG>
static void launch_wave_ks(uint32_t k, bool nt_stores, const BatchView& dst, const BatchView& src, const OutView& out,
                           const OutView& out2, const Work& wk, bool no_large, uint32_t sb, hipStream_t stream) {
    if (nt_stores)
        launch_wave_k<kAuxNT, EXCH, STG>(k, dst, src, out, out2, wk, no_large, sb, stream);
    else
        launch_wave_k<0, EXCH, STG>(k, dst, src, out, out2, wk, no_large, sb, stream);
}

// docs_per_wave: K of join_wave_kernel (1, 2, 4, 8 or 16); nt_stores: write the
// output with non-temporal stores; stage_stores: place the survivors in LDS by
// output slot and write whole contiguous lines (join_doc's STG); slab_blocks:
// the wave kernel's block order (SlabMap G; 0 = in order); no_large: the caller promised every doc has
// <= 64 entries per side, so the block path is not launched (a larger doc then
// raises CRDT_E_INVALID).  out2 != nullptr: exchange -- also out2 = src <- dst.
hipError_t launch_join_tiles(const BatchView& A, const BatchView& B, const OutView& o1, const OutView* o2,
                             const Work& wk, const TileWork& tw, uint32_t n_cu, hipStream_t stream);

// tw != nullptr: large documents go through the merge-path tile path
// (tile.hip); the per-document block kernel then only runs when the tiles
// exceed the workspace (tw->fallback).
hipError_t launch_join(const BatchView& dst, const BatchView& src, const OutView& out, const OutView* out2,
                       const Work& wk, uint32_t docs_per_wave, bool nt_stores, bool stage_stores, uint32_t slab_blocks,
                       uint32_t block_grid, bool no_large, const TileWork* tw, uint32_t n_cu, hipStream_t stream) {
    if (dst.n_docs == 0) return hipSuccess;
    const OutView& o2 = out2 ? *out2 : out;
    if (out2) {
        if (stage_stores)
            launch_wave_ks<true, true>(docs_per_wave, nt_stores, dst, src, out, o2, wk, no_large, slab_blocks, stream);
        else
            launch_wave_ks<true, false>(docs_per_wave, nt_stores, dst, src, out, o2, wk, no_large, slab_blocks, stream);
    } else {
        if (stage_stores)
            launch_wave_ks<false, true>(docs_per_wave, nt_stores, dst, src, out, o2, wk, no_large, slab_blocks, stream);
        else
            launch_wave_ks<false, false>(docs_per_wave, nt_stores, dst, src, out, o2, wk, no_large, slab_blocks,
                                         stream);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || no_large) return e;
    const uint32_t* gate = nullptr;
    if (tw) {
        e = launch_join_tiles(dst, src, out, out2, wk, *tw, n_cu, stream);
        if (e != hipSuccess || tw->covered) return e;  // covered: the passes hold every tile, no fallback
        gate = tw->fallback;
    }
    hipLaunchKernelGGL((join_block_kernel<kBlockNT, kBlockIPT>), dim3(block_grid), dim3(kBlockNT), 0, stream, dst,
                       src, out, wk, 0u, gate);
    if (out2) {
        e = hipGetLastError();
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL((join_block_kernel<kBlockNT, kBlockIPT>), dim3(block_grid), dim3(kBlockNT), 0, stream,
                           src, dst, *out2, wk, 1u, gate);
    }
    return hipGetLastError();
}

}  // namespace crdt
