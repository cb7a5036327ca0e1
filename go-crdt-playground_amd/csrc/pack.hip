// Host-path helpers around the merge kernels (the *_batch calls of api.cpp):
//  * check_order_kernel: every document's (or source's) live keys strictly
//    ascending -- the merge kernels' input contract (include/crdtgpu.h) --
//    checked on the device after the upload instead of by one host thread
//    before it; a violation sets kErrUnsorted (CRDT_E_UNSORTED).
//  * pack_scan_kernel: the packed offsets of a merge output -- the exclusive
//    prefix over documents of the live counts, each clamped to the document's
//    output capacity -- on the device, so the host path needs no count
//    read-back before it can gather.
//  * pack_out_kernel: a merge output (document d at its capacity offset)
//    gathered into consecutive live entries at those offsets, so the download
//    moves only live entries (crdt_ctx_set_option "pack_batch_outputs"); with
//    the counts and clocks too when the destination is the caller's page-locked
//    host output (written over PCIe by the kernel, no copy call at all).
// One wavefront per range, grid-stride; coalesced 64-lane runs.
#include "crdt_device.hpp"
#include "merge_block.hpp"

namespace crdt {

constexpr int kPackScanNT = 1024;

// One workgroup: thread t sums a contiguous run of documents, a block scan
// places the runs, then each thread writes its run's prefixes (poff[n] =
// total).  host_off (may be NULL): the same offsets, into the caller's
// page-locked output.
// gate: the call's status word -- after a failed order check the merge never
// ran, so the output's slot bounds and counts were never written: every
// offset is 0 and pack_out_kernel writes nothing.
__global__ __launch_bounds__(kPackScanNT) void pack_scan_kernel(const uint32_t* off, const uint32_t* cnt, uint32_t n,
                                                                uint32_t* poff, uint32_t* host_off,
                                                                const uint32_t* gate) {
    __shared__ uint32_t wave_tot[kPackScanNT / 64];
    const uint32_t t = threadIdx.x;
    const bool open = (*gate & kErrUnsorted) == 0u;
    const uint32_t per = (n + kPackScanNT - 1) / kPackScanNT;
    const uint32_t d0 = min(t * per, n), d1 = min(d0 + per, n);
    auto live = [&](uint32_t d) -> uint32_t {  // clamped to the capacity (a larger count only follows a failed merge)
        if (!open) return 0u;
        const uint32_t c = off[d + 1] - off[d];
        return min(cnt[d], c);
    };
    uint32_t sum = 0;
    for (uint32_t d = d0; d < d1; ++d) sum += live(d);
    uint32_t tot = 0;
    uint32_t p = block_exclusive_scan<kPackScanNT>(sum, wave_tot, &tot);
    for (uint32_t d = d0; d < d1; ++d) {
        poff[d] = p;
        if (host_off) host_off[d] = p;
        p += live(d);
    }
    if (t == 0) {
        poff[n] = tot;
        if (host_off) host_off[n] = tot;
    }
}

__global__ __launch_bounds__(256) void check_order_kernel(const uint32_t* off, const uint32_t* cnt, uint32_t n,
                                                          const uint64_t* keys, uint32_t* status) {
    const uint32_t lane = threadIdx.x & 63;
    uint32_t err = 0;
    for (uint32_t r = uniform(blockIdx.x * 4 + (threadIdx.x >> 6)); r < n; r += gridDim.x * 4) {
        const uint32_t o = off[r];
        const uint32_t m = cnt ? cnt[r] : off[r + 1] - o;  // counts <= slots: checked on the host
        for (uint32_t i = 1 + lane; i < m; i += 64)
            if (keys[o + i] <= keys[o + i - 1]) err |= kErrUnsorted;
    }
    flag_error(status, err);
}

// out.keys == NULL: no key column (an exchange's second output sharing the
// first's); out.counts / out.vv != NULL: each document's count and clock too.
__global__ __launch_bounds__(256) void pack_out_kernel(OutView in, const uint32_t* poff, uint32_t n, uint32_t R,
                                                       OutView out, const uint32_t* gate) {
    const uint32_t lane = threadIdx.x & 63;
    if (*gate & kErrUnsorted) return;  // the merge never ran (pack_scan_kernel)
    for (uint32_t d = uniform(blockIdx.x * 4 + (threadIdx.x >> 6)); d < n; d += gridDim.x * 4) {
        // a count above the document's own capacity (only after a failed merge)
        // is clamped to it: the gather never leaves the document's region
        const uint32_t o = in.offsets[d], p = poff[d], m = min(poff[d + 1] - p, in.offsets[d + 1] - o);
        for (uint32_t i = lane; i < m; i += 64) {
            if (out.keys) out.keys[p + i] = in.keys[o + i];
            out.actors[p + i] = in.actors[o + i];
            out.counters[p + i] = in.counters[o + i];
        }
        if (out.counts && lane == 0) out.counts[d] = in.counts[d];
        if (out.vv && lane < R) out.vv[(size_t)d * R + lane] = in.vv[(size_t)d * R + lane];
    }
}

hipError_t launch_check_order(const uint32_t* off, const uint32_t* cnt, uint32_t n, const uint64_t* keys,
                              uint32_t* status, uint32_t n_cu, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const uint32_t grid = min((n + 3) / 4, n_cu * 16u);
    hipLaunchKernelGGL(check_order_kernel, dim3(grid), dim3(256), 0, stream, off, cnt, n, keys, status);
    return hipGetLastError();
}

hipError_t launch_pack_scan(const uint32_t* off, const uint32_t* cnt, uint32_t n, uint32_t* poff, uint32_t* host_off,
                            const uint32_t* gate, hipStream_t stream) {
    hipLaunchKernelGGL(pack_scan_kernel, dim3(1), dim3(kPackScanNT), 0, stream, off, cnt, n, poff, host_off, gate);
    return hipGetLastError();
}

hipError_t launch_pack_out(const OutView& in, const uint32_t* poff, uint32_t n, uint32_t R, const OutView& out,
                           const uint32_t* gate, uint32_t n_cu, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const uint32_t grid = min((n + 3) / 4, n_cu * 16u);
    hipLaunchKernelGGL(pack_out_kernel, dim3(grid), dim3(256), 0, stream, in, poff, n, R, out, gate);
    return hipGetLastError();
}

}  // namespace crdt
