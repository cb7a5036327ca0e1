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

template <int WAVES>
__global__ __launch_bounds__(WAVES * 64) void join_wave_kernel(BatchView dst, BatchView src, OutView out, Work wk) {
    __shared__ uint64_t s_dkey[WAVES][64];
    __shared__ uint64_t s_skey[WAVES][64];
    __shared__ uint64_t s_dvv[WAVES][CRDT_MAX_R];
    __shared__ uint64_t s_svv[WAVES][CRDT_MAX_R];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t w = threadIdx.x >> 6;
    const uint32_t R = dst.R;
    const uint32_t n_docs = dst.n_docs;
    uint32_t err = 0;
    const uint64_t lt = low_mask(lane);

    for (uint32_t d0 = blockIdx.x * WAVES + w; d0 < n_docs; d0 += gridDim.x * WAVES) {
        const uint32_t d = uniform(d0);
        const uint32_t doff = dst.offsets[d], soff = src.offsets[d];
        const uint32_t dn = live_count(dst.offsets, dst.counts, d);
        const uint32_t sn = live_count(src.offsets, src.counts, d);
        const uint32_t obase = doff + soff;
        if (lane == 0) {
            out.offsets[d] = obase;
            if (d == n_docs - 1) out.offsets[n_docs] = dst.offsets[n_docs] + src.offsets[n_docs];
        }
        if (dn > 64 || sn > 64) {
            if (lane == 0) wk.worklist[atomicAdd(wk.wl_count, 1u)] = d;
            continue;
        }
        const bool dv = lane < dn, sv = lane < sn;
        uint64_t dk = 0, dc = 0, sk = 0, sc = 0;
        uint32_t da = 0, sa = 0;
        if (dv) {
            dk = dst.keys[doff + lane];
            da = dst.actors[doff + lane];
            dc = dst.counters[doff + lane];
        }
        if (sv) {
            sk = src.keys[soff + lane];
            sa = src.actors[soff + lane];
            sc = src.counters[soff + lane];
        }
        uint64_t vd = 0, vs = 0;
        if (lane < R) {
            vd = dst.vv[(size_t)d * R + lane];
            vs = src.vv[(size_t)d * R + lane];
            s_dvv[w][lane] = vd;
            s_svv[w][lane] = vs;
        }
        s_dkey[w][lane] = dk;
        s_skey[w][lane] = sk;
        wave_sync();

        // # src keys < dk, # dst keys < sk
        const uint32_t j = lower_bound_pow<6>(s_skey[w], sn, dk);
        const uint32_t i = lower_bound_pow<6>(s_dkey[w], dn, sk);
        const bool dmatch = dv && j < sn && s_skey[w][j] == dk;
        const bool smatch = sv && i < dn && s_dkey[w][i] == sk;
        // awset.go:145-159: a dst-only key survives unless src's clock covers it.
        bool dkeep = false, skeep = false;
        if (dv) dkeep = dmatch || !has_dot(s_svv[w], R, da, dc, err);
        // awset.go:130-140: a src-only key is added unless dst's clock covers it.
        if (sv && !smatch) skeep = !has_dot(s_dvv[w], R, sa, sc, err);
        const uint64_t dm = ballot(dkeep), sm = ballot(skeep);
        // awset.go:142: the src dot wins on a common key (lane j holds it).
        const uint32_t ma = __shfl(sa, (int)(j & 63));
        const uint64_t mc = __shfl(sc, (int)(j & 63));
        if (dkeep) {
            const uint32_t pos = obase + popc(dm & lt) + popc(sm & low_mask(j));
            out.keys[pos] = dk;
            out.actors[pos] = dmatch ? ma : da;
            out.counters[pos] = dmatch ? mc : dc;
        }
        if (skeep) {
            const uint32_t pos = obase + popc(sm & lt) + popc(dm & low_mask(i));
            out.keys[pos] = sk;
            out.actors[pos] = sa;
            out.counters[pos] = sc;
        }
        if (lane == 0) out.counts[d] = popc(dm) + popc(sm);
        // awset.go:160 -> crdt-misc.go:43-55
        if (lane < R) out.vv[(size_t)d * R + lane] = vd > vs ? vd : vs;
        wave_sync();
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

hipError_t launch_join(const BatchView& dst, const BatchView& src, const OutView& out, const Work& wk,
                       uint32_t block_grid, hipStream_t stream) {
    if (dst.n_docs == 0) return hipSuccess;
    const uint32_t max_grid = 1u << 20;
    uint32_t grid = (dst.n_docs + kJoinWaves - 1) / kJoinWaves;
    if (grid > max_grid) grid = max_grid;
    hipLaunchKernelGGL((join_wave_kernel<kJoinWaves>), dim3(grid), dim3(kJoinWaves * 64), 0, stream, dst, src, out,
                       wk);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((join_block_kernel<kBlockNT, kBlockIPT>), dim3(block_grid), dim3(kBlockNT), 0, stream, dst,
                       src, out, wk);
    return hipGetLastError();
}

}  // namespace crdt
