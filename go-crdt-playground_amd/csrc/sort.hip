// Ingest sort: each document's live entries ordered by key on the device, so a
// producer that packs a map (Go iterates map[string]Dot in random order,
// awset.go:55-59) need not sort on the host before the merge kernels, which
// require strictly ascending keys per document (include/crdtgpu.h).
//
// rocPRIM's segmented radix sort orders (key, slot index) pairs per document
// (one segment = one document's live range); a gather kernel then moves the
// dots, copies the version vectors, and flags a key that appears twice in one
// document (CRDT_E_DUP_KEY: interned ids of one map are distinct).
#include <rocprim/device/device_segmented_radix_sort.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include "crdt_device.hpp"

namespace crdt {

__global__ void sort_ends_kernel(BatchView in, uint32_t* ends) {
    for (uint32_t d = blockIdx.x * blockDim.x + threadIdx.x; d < in.n_docs; d += gridDim.x * blockDim.x)
        ends[d] = in.offsets[d] + live_count(in.offsets, in.counts, d);
}

// One wave per document: gather the dots of the sorted order, check for
// repeated keys, copy the VV and the slot bounds.
__global__ __launch_bounds__(256) void sort_gather_kernel(BatchView in, const uint32_t* idx, OutView out,
                                                          uint32_t* status) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t R = in.R;
    uint32_t err = 0;
    for (uint32_t d = uniform(blockIdx.x * 4 + (threadIdx.x >> 6)); d < in.n_docs; d += gridDim.x * 4) {
        const uint32_t o = in.offsets[d], n = live_count(in.offsets, in.counts, d);
        for (uint32_t i = lane; i < n; i += 64) {
            const uint32_t src = idx[o + i];
            out.actors[o + i] = in.actors[src];
            out.counters[o + i] = in.counters[src];
            if (i > 0 && out.keys[o + i] == out.keys[o + i - 1]) err |= kErrDupKey;
        }
        if (lane < R) out.vv[(size_t)d * R + lane] = in.vv[(size_t)d * R + lane];
        if (lane == 0) {
            out.counts[d] = n;
            out.offsets[d] = o;
            if (d == in.n_docs - 1) out.offsets[in.n_docs] = in.offsets[in.n_docs];
        }
    }
    flag_error(status, err);
}

// Temporary storage rocPRIM needs for n_slots pairs in n_docs segments.
hipError_t sort_storage(uint32_t n_docs, uint32_t n_slots, size_t* bytes) {
    rocprim::counting_iterator<uint32_t> iota(0u);
    return rocprim::segmented_radix_sort_pairs(nullptr, *bytes, (const uint64_t*)nullptr, (uint64_t*)nullptr, iota,
                                               (uint32_t*)nullptr, n_slots, n_docs, (const uint32_t*)nullptr,
                                               (const uint32_t*)nullptr);
}

hipError_t launch_sort(const BatchView& in, uint32_t n_slots, const OutView& out, void* temp, size_t temp_bytes,
                       uint32_t* ends, uint32_t* idx, uint32_t* status, uint32_t n_cu, hipStream_t stream) {
    if (in.n_docs == 0) return hipSuccess;
    const uint32_t grid = min((in.n_docs + 255) / 256, n_cu * 8u);
    hipLaunchKernelGGL(sort_ends_kernel, dim3(grid), dim3(256), 0, stream, in, ends);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    rocprim::counting_iterator<uint32_t> iota(0u);
    size_t tb = temp_bytes;
    e = rocprim::segmented_radix_sort_pairs(temp, tb, in.keys, out.keys, iota, idx, n_slots, in.n_docs, in.offsets,
                                            (const uint32_t*)ends, 0u, 64u, stream);
    if (e != hipSuccess) return e;
    const uint32_t g2 = min((in.n_docs + 3) / 4, n_cu * 16u);
    hipLaunchKernelGGL(sort_gather_kernel, dim3(g2), dim3(256), 0, stream, in, (const uint32_t*)idx, out, status);
    return hipGetLastError();
}

}  // namespace crdt
