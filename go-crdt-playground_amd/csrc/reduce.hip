// Version-vector reductions.
//  * vv_max_kernel: dst[i] = max(dst[i], src[i]) -- (*VersionVector).Merge,
//    crdt-misc.go:43-55, over equal-length vectors (R-padded).
//  * causal-context summary: elementwise max over n_docs VVs of length R, the
//    per-GPU clock summary that bench.py all-reduces (max, u64) across GPUs.
//    Two launches: per-block partial maxima, then one block folds the partials
//    (deterministic, no global atomics).
#include "crdt_device.hpp"

namespace crdt {

__global__ void vv_max_kernel(uint64_t* __restrict__ dst, const uint64_t* __restrict__ src, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint64_t a = dst[i], b = src[i];
        dst[i] = a > b ? a : b;
    }
}

// Thread t of a block handles actor r = t % R over docs t/R, t/R + NT/R, ...
// (threads t >= (NT/R)*R idle).  Block partial -> part[block*R + r].
template <int NT>
__global__ __launch_bounds__(NT) void context_partial_kernel(const uint64_t* __restrict__ vv, uint32_t n_docs,
                                                             uint32_t R, uint64_t* __restrict__ part) {
    __shared__ uint64_t red[NT];
    const uint32_t t = threadIdx.x;
    const uint32_t per = NT / R;  // docs per block-stride
    const uint32_t r = t % R, lane_doc = t / R;
    uint64_t m = 0;
    if (lane_doc < per) {
        const size_t stride = (size_t)gridDim.x * per;
        // eight independent loads in flight per round (a plain strided loop
        // waits out one HBM latency per document)
        for (size_t d0 = (size_t)blockIdx.x * per + lane_doc; d0 < n_docs; d0 += 8 * stride) {
            uint64_t v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const size_t d = d0 + u * stride;
                v[u] = d < n_docs ? vv[d * R + r] : 0ull;
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) m = v[u] > m ? v[u] : m;
        }
    }
    red[t] = m;
    __syncthreads();
    if (t < R) {
        uint64_t acc = 0;
        for (uint32_t q = 0; q < per; ++q) {
            const uint64_t v = red[q * R + t];
            acc = v > acc ? v : acc;
        }
        part[(size_t)blockIdx.x * R + t] = acc;
    }
}

// One block folds the n_part partials: thread t takes actor t % R over
// partial rows t / R, t / R + NT / R, ...; then R threads fold the LDS row.
template <int NT>
__global__ __launch_bounds__(NT) void context_final_kernel(const uint64_t* __restrict__ part, uint32_t n_part,
                                                           uint32_t R, uint64_t* __restrict__ out) {
    __shared__ uint64_t red[NT];
    const uint32_t t = threadIdx.x;
    const uint32_t per = NT / R;
    const uint32_t r = t % R, row = t / R;
    uint64_t m = 0;
    if (row < per)
        for (uint32_t b0 = row; b0 < n_part; b0 += 8 * per) {
            uint64_t v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const uint32_t b = b0 + u * per;
                v[u] = b < n_part ? part[(size_t)b * R + r] : 0ull;
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) m = v[u] > m ? v[u] : m;
        }
    red[t] = m;
    __syncthreads();
    if (t < R) {
        uint64_t acc = 0;
        for (uint32_t q = 0; q < per; ++q) {
            const uint64_t v = red[q * R + t];
            acc = v > acc ? v : acc;
        }
        out[t] = acc;
    }
}

constexpr int kCtxNT = 256;

// Zero the per-call work counters (workspace words [0, 16)).  A kernel rather
// than hipMemsetAsync so a captured call is a graph of kernel nodes only.
__global__ void reset_work_kernel(uint32_t* ws) { ws[threadIdx.x] = 0u; }

hipError_t launch_reset_work(uint32_t* ws, hipStream_t stream) {
    hipLaunchKernelGGL(reset_work_kernel, dim3(1), dim3(16), 0, stream, ws);
    return hipGetLastError();
}

__global__ void vv_min_kernel(uint64_t* dst, const uint64_t* src, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint64_t a = dst[i], b = src[i];
        dst[i] = a < b ? a : b;
    }
}

hipError_t launch_vv_min(uint64_t* dst, const uint64_t* src, size_t n, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    size_t grid = (n + 255) / 256;
    if (grid > 4096) grid = 4096;
    hipLaunchKernelGGL(vv_min_kernel, dim3((uint32_t)grid), dim3(256), 0, stream, dst, src, n);
    return hipGetLastError();
}

hipError_t launch_vv_max(uint64_t* dst, const uint64_t* src, size_t n, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    size_t grid = (n + 255) / 256;
    if (grid > 4096) grid = 4096;
    hipLaunchKernelGGL(vv_max_kernel, dim3((uint32_t)grid), dim3(256), 0, stream, dst, src, n);
    return hipGetLastError();
}

// part must hold n_part*R u64; n_part <= caller's bound.
hipError_t launch_context(const uint64_t* vv, uint32_t n_docs, uint32_t R, uint64_t* part, uint32_t n_part,
                          uint64_t* out, hipStream_t stream) {
    hipLaunchKernelGGL((context_partial_kernel<kCtxNT>), dim3(n_part), dim3(kCtxNT), 0, stream, vv, n_docs, R, part);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((context_final_kernel<kCtxNT>), dim3(1), dim3(kCtxNT), 0, stream, part, n_part, R, out);
    return hipGetLastError();
}

}  // namespace crdt
