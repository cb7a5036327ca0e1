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

// Per-doc metadata, fetched by lanes 0..3 with ONE vector load (in-order vmcnt,
// so it can run ahead of the LDS traffic without forcing lgkmcnt(0) waits).
// Unconditional: lanes >= 4 repeat lane 3's address, d is clamped.
struct JoinMeta {
    uint32_t doff, soff, dn, sn;
};

__device__ __forceinline__ uint32_t meta_issue(const BatchView& dst, const BatchView& src, uint32_t d,
                                               uint32_t lane) {
    const uint32_t dd = d < dst.n_docs ? d : dst.n_docs - 1;
    const uint32_t* p2 = dst.counts ? dst.counts + dd : dst.offsets + dd + 1;
    const uint32_t* p3 = src.counts ? src.counts + dd : src.offsets + dd + 1;
    const uint32_t* p = lane == 0 ? dst.offsets + dd : lane == 1 ? src.offsets + dd : lane == 2 ? p2 : p3;
    return *p;
}

__device__ __forceinline__ JoinMeta meta_decode(const BatchView& dst, const BatchView& src, uint32_t v) {
    JoinMeta m;
    m.doff = (uint32_t)__builtin_amdgcn_readlane((int)v, 0);
    m.soff = (uint32_t)__builtin_amdgcn_readlane((int)v, 1);
    const uint32_t a = (uint32_t)__builtin_amdgcn_readlane((int)v, 2);
    const uint32_t b = (uint32_t)__builtin_amdgcn_readlane((int)v, 3);
    m.dn = dst.counts ? a : a - m.doff;
    m.sn = src.counts ? b : b - m.soff;
    return m;
}

// One document's entries, one per lane (lane i: dst entry i, src entry i, VV[i]).
struct JoinLanes {
    uint64_t dk, dc, sk, sc, vd, vs;
    uint32_t da, sa;
};

// ld = false (document on the block path, or past the end): every lane reads 0.
__device__ __forceinline__ void lanes_issue(JoinLanes& L, const BatchView& dst, const BatchView& src,
                                            const JoinMeta& m, uint32_t d, bool ld, uint32_t lane, uint32_t R) {
    const uint32_t dn = ld ? m.dn : 0u, sn = ld ? m.sn : 0u, rv = ld ? R : 0u;
    const uint32_t o8 = lane * 8u, o4 = lane * 4u;
    L.dk = ld64(make_rsrc(dst.keys + m.doff, dn * 8u), o8);
    L.da = ld32(make_rsrc(dst.actors + m.doff, dn * 4u), o4);
    L.dc = ld64(make_rsrc(dst.counters + m.doff, dn * 8u), o8);
    L.sk = ld64(make_rsrc(src.keys + m.soff, sn * 8u), o8);
    L.sa = ld32(make_rsrc(src.actors + m.soff, sn * 4u), o4);
    L.sc = ld64(make_rsrc(src.counters + m.soff, sn * 8u), o8);
    const size_t vo = ld ? (size_t)d * R : 0;
    L.vd = ld64(make_rsrc(dst.vv + vo, rv * 8u), o8);
    L.vs = ld64(make_rsrc(src.vv + vo, rv * 8u), o8);
}

// Persistent waves, software-pipelined over the documents d = gw, gw + nw, ...:
// metadata two documents ahead, entries one document ahead, so the loads of
// the next document are in flight while this one is merged.  The loop body is
// straight-line VMEM (buffer ops, no exec-masked branches) so the compiler's
// vmcnt waits count exactly instead of draining to 0.
template <int WAVES>
__global__ __launch_bounds__(WAVES * 64) void join_wave_kernel(BatchView dst, BatchView src, OutView out, Work wk,
                                                               uint32_t no_large) {
    __shared__ uint64_t s_dkey[WAVES][64];
    __shared__ uint64_t s_skey[WAVES][64];
    __shared__ uint64_t s_dvv[WAVES][64];
    __shared__ uint64_t s_svv[WAVES][64];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t w = threadIdx.x >> 6;
    const uint32_t R = dst.R;
    const uint32_t n_docs = dst.n_docs;
    const uint32_t nw = gridDim.x * WAVES;
    const uint64_t lt = low_mask(lane);
    const uint32_t end_off = dst.offsets[n_docs] + src.offsets[n_docs];
    uint32_t err = 0;

    uint32_t d = uniform(blockIdx.x * WAVES + w);
    if (d >= n_docs) return;
    JoinMeta m = meta_decode(dst, src, meta_issue(dst, src, d, lane));
    uint32_t mv_next = meta_issue(dst, src, d + nw, lane);
    JoinLanes cur;
    bool small = m.dn <= 64 && m.sn <= 64;
    lanes_issue(cur, dst, src, m, d, small, lane, R);

    for (;;) {
        const uint32_t dn = d + nw;
        const bool more = dn < n_docs;
        // stage 1: next document's metadata is back; issue its entries and the
        // metadata after it.
        const JoinMeta mn = meta_decode(dst, src, mv_next);
        const bool small_n = more && mn.dn <= 64 && mn.sn <= 64;
        const uint32_t mv_next2 = meta_issue(dst, src, dn + nw, lane);
        JoinLanes nxt;
        lanes_issue(nxt, dst, src, mn, dn, small_n, lane, R);

        // stage 2: merge document d (awset.go:107-161).
        const uint32_t obase = m.doff + m.soff;
        const uint32_t dnn = small ? m.dn : 0u, snn = small ? m.sn : 0u;
        const bool dv = lane < dnn, sv = lane < snn;
        s_dvv[w][lane] = cur.vd;
        s_svv[w][lane] = cur.vs;
        s_dkey[w][lane] = cur.dk;
        s_skey[w][lane] = cur.sk;
        wave_sync();
        // # src keys < dk, # dst keys < sk
        const uint32_t j = lower_bound_pow<6>(s_skey[w], snn, cur.dk);
        const uint32_t i = lower_bound_pow<6>(s_dkey[w], dnn, cur.sk);
        const bool dmatch = dv && j < snn && s_skey[w][j & 63] == cur.dk;
        const bool smatch = sv && i < dnn && s_dkey[w][i & 63] == cur.sk;
        // awset.go:145-159: a dst-only key survives unless src's clock covers it.
        const bool dh = has_dot_bf(s_svv[w], R, cur.da, cur.dc, dv && !dmatch, err);
        // awset.go:130-140: a src-only key is added unless dst's clock covers it.
        const bool sh = has_dot_bf(s_dvv[w], R, cur.sa, cur.sc, sv && !smatch, err);
        const bool dkeep = dv && (dmatch || !dh);
        const bool skeep = sv && !smatch && !sh;
        const uint64_t dm = ballot(dkeep), sm = ballot(skeep);
        // awset.go:142: the src dot wins on a common key (lane j holds it).
        const uint32_t ma = __shfl(cur.sa, (int)(j & 63));
        const uint64_t mc = __shfl(cur.sc, (int)(j & 63));
        const uint32_t dpos = popc(dm & lt) + popc(sm & low_mask(j));
        const uint32_t spos = popc(sm & lt) + popc(dm & low_mask(i));
        const uint32_t cap = dnn + snn;
        const rsrc_t ok = make_rsrc(out.keys + obase, cap * 8u);
        const rsrc_t oa = make_rsrc(out.actors + obase, cap * 4u);
        const rsrc_t oc = make_rsrc(out.counters + obase, cap * 8u);
        const uint32_t d8 = dkeep ? dpos * 8u : kOOB, d4 = dkeep ? dpos * 4u : kOOB;
        const uint32_t s8 = skeep ? spos * 8u : kOOB, s4 = skeep ? spos * 4u : kOOB;
        st64(cur.dk, ok, d8);
        st32(dmatch ? ma : cur.da, oa, d4);
        st64(dmatch ? mc : cur.dc, oc, d8);
        st64(cur.sk, ok, s8);
        st32(cur.sa, oa, s4);
        st64(cur.sc, oc, s8);
        // slot bounds (every doc), live count and VV (wave path only)
        const bool last = d == n_docs - 1;
        st32(lane == 0 ? obase : end_off, make_rsrc(out.offsets + d, last ? 8u : 4u), lane < 2 ? lane * 4u : kOOB);
        st32(popc(dm) + popc(sm), make_rsrc(out.counts + d, small ? 4u : 0u), lane == 0 ? 0u : kOOB);
        // awset.go:160 -> crdt-misc.go:43-55
        st64(cur.vd > cur.vs ? cur.vd : cur.vs, make_rsrc(out.vv + (size_t)d * R, small ? R * 8u : 0u), lane * 8u);
        wave_sync();
        if (!small) {
            if (lane == 0) {
                if (no_large)
                    atomicOr(wk.status, kErrHint);
                else
                    wk.worklist[atomicAdd(wk.wl_count, 1u)] = d;
            }
        }
        if (!more) break;
        d = dn;
        m = mn;
        cur = nxt;
        small = small_n;
        mv_next = mv_next2;
    }
    flag_error(wk.status, err);
}

template <int NT, int IPT>
__global__ __launch_bounds__(NT) void join_block_kernel(BatchView dst, BatchView src, OutView out, Work wk) {
    __shared__ MergeSmem<NT, IPT> sm;
    const uint32_t tid = threadIdx.x;
    const uint32_t R = dst.R;
    uint32_t err = 0;
    const Entries none{nullptr, nullptr, nullptr, 0};
    for (;;) {
        if (tid == 0) sm.word[0] = atomicAdd(wk.wl_head, 1u);
        __syncthreads();
        const uint32_t slot = sm.word[0];
        const uint32_t total = __hip_atomic_load(wk.wl_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        if (slot >= total) break;
        const uint32_t d = wk.worklist[slot];
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

// wave_grid: persistent blocks of the wave path (a few per CU); no_large: the
// caller promised every doc has <= 64 entries per side, so the block path is
// not launched (a larger doc then raises CRDT_E_INVALID).
hipError_t launch_join(const BatchView& dst, const BatchView& src, const OutView& out, const Work& wk,
                       uint32_t wave_grid, uint32_t block_grid, bool no_large, hipStream_t stream) {
    if (dst.n_docs == 0) return hipSuccess;
    uint32_t grid = (dst.n_docs + kJoinWaves - 1) / kJoinWaves;
    if (grid > wave_grid) grid = wave_grid;
    hipLaunchKernelGGL((join_wave_kernel<kJoinWaves>), dim3(grid), dim3(kJoinWaves * 64), 0, stream, dst, src, out,
                       wk, (uint32_t)no_large);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || no_large) return e;
    hipLaunchKernelGGL((join_block_kernel<kBlockNT, kBlockIPT>), dim3(block_grid), dim3(kBlockNT), 0, stream, dst,
                       src, out, wk);
    return hipGetLastError();
}

}  // namespace crdt
