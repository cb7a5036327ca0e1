// Host-path helpers around the merge kernels (the *_batch calls of api.cpp):
//  * check_order_kernel: every document's (or source's) live keys strictly
//    ascending -- the merge kernels' input contract (include/crdtgpu.h) --
//    checked on the device after the upload instead of by one host thread
//    before it; a violation sets kErrUnsorted (CRDT_E_UNSORTED).
//  * pack_out_kernel: a merge output (document d at its capacity offset)
//    gathered into consecutive live entries at caller-computed offsets, so
//    the download moves only live entries (crdt_ctx_set_option
//    "pack_batch_outputs").
// One wavefront per range, grid-stride; coalesced 64-lane runs.
#include "crdt_device.hpp"

namespace crdt {

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

__global__ __launch_bounds__(256) void pack_out_kernel(OutView in, const uint32_t* poff, uint32_t n, OutView out) {
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t d = uniform(blockIdx.x * 4 + (threadIdx.x >> 6)); d < n; d += gridDim.x * 4) {
        // a count above the document's own capacity (only after a failed merge)
        // is clamped to it: the gather never leaves the document's region
        const uint32_t o = in.offsets[d], p = poff[d], m = min(poff[d + 1] - p, in.offsets[d + 1] - o);
        for (uint32_t i = lane; i < m; i += 64) {
            out.keys[p + i] = in.keys[o + i];
            out.actors[p + i] = in.actors[o + i];
            out.counters[p + i] = in.counters[o + i];
        }
    }
}

hipError_t launch_check_order(const uint32_t* off, const uint32_t* cnt, uint32_t n, const uint64_t* keys,
                              uint32_t* status, uint32_t n_cu, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const uint32_t grid = min((n + 3) / 4, n_cu * 16u);
    hipLaunchKernelGGL(check_order_kernel, dim3(grid), dim3(256), 0, stream, off, cnt, n, keys, status);
    return hipGetLastError();
}

hipError_t launch_pack_out(const OutView& in, const uint32_t* poff, uint32_t n, const OutView& out, uint32_t n_cu,
                           hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const uint32_t grid = min((n + 3) / 4, n_cu * 16u);
    hipLaunchKernelGGL(pack_out_kernel, dim3(grid), dim3(256), 0, stream, in, poff, n, out);
    return hipGetLastError();
}

}  // namespace crdt
