// Bandwidth probes: what this box's HBM moves with no merge work at all.
// Not a merge.  bench.py runs them before timing so that a bench line carries
// the ceiling of the box it ran on next to the 8 TB/s spec figure (boxes of one
// pool differ by up to 25 % in copy bandwidth).
//
//   read : 16 B per lane loads, four in flight per lane, grid-stride
//   write: 16 B per lane non-temporal stores (the merge kernels' output stores)
//   copy : both, one read and one write per 16 B
//   mix  : 3 reads : 4 writes of 16 B (the config-2 exchange's round-3 mix,
//          2.85 GB read : 3.72 GB written per launch)
// each in two block orders: grid-stride, and one contiguous slab per
// workgroup ("probe_slab"), which reaches 8-30 % more on MI355X.
#include "crdt_device.hpp"

namespace crdt {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Index range of one thread.  SLAB = false: grid-stride (the whole grid
// sweeps one advancing window); SLAB = true: workgroup b streams its own
// contiguous slab b of the buffer (the form that reaches the box's ceiling,
// tools/bw_layout.hip).
template <bool SLAB>
__device__ __forceinline__ void probe_range(size_t n, size_t& begin, size_t& step, size_t& end) {
    if (SLAB) {
        const size_t per = (n + gridDim.x - 1) / gridDim.x;
        begin = (size_t)blockIdx.x * per + threadIdx.x;
        step = blockDim.x;
        end = min(n, (size_t)(blockIdx.x + 1) * per);
    } else {
        begin = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
        step = (size_t)gridDim.x * blockDim.x;
        end = n;
    }
}

template <bool SLAB>
__global__ __launch_bounds__(256) void probe_read_kernel(const u32x4* __restrict__ a, size_t n, uint32_t* sink) {
    size_t i, stride, end;
    probe_range<SLAB>(n, i, stride, end);
    u32x4 acc = {0u, 0u, 0u, 0u};
    for (; i + 3 * stride < end; i += 4 * stride) {
        const u32x4 x0 = a[i], x1 = a[i + stride], x2 = a[i + 2 * stride], x3 = a[i + 3 * stride];
        acc ^= x0 ^ x1 ^ x2 ^ x3;
    }
    for (; i < end; i += stride) acc ^= a[i];
    // never true for the probe's fill pattern; keeps the loads live
    if (acc.x == 0x9E3779B9u && acc.y == 0x7F4A7C15u) sink[0] = acc.z ^ acc.w;
}

template <bool NT>
__device__ __forceinline__ void put16(u32x4 v, u32x4* p) {
    if (NT)
        __builtin_nontemporal_store(v, p);
    else
        *p = v;
}

template <bool NT, bool SLAB>
__global__ __launch_bounds__(256) void probe_write_kernel(u32x4* __restrict__ b, size_t n) {
    size_t i, stride, end;
    probe_range<SLAB>(n, i, stride, end);
    for (; i < end; i += stride) {
        const u32x4 v = {(uint32_t)i, (uint32_t)(i >> 32), 0x5EEDu, 1u};
        put16<NT>(v, b + i);
    }
}

template <bool NT, bool SLAB>
__global__ __launch_bounds__(256) void probe_copy_kernel(const u32x4* __restrict__ a, u32x4* __restrict__ b,
                                                         size_t n) {
    size_t i, stride, end;
    probe_range<SLAB>(n, i, stride, end);
    for (; i + 3 * stride < end; i += 4 * stride) {
        const u32x4 x0 = a[i], x1 = a[i + stride], x2 = a[i + 2 * stride], x3 = a[i + 3 * stride];
        put16<NT>(x0, b + i);
        put16<NT>(x1, b + i + stride);
        put16<NT>(x2, b + i + 2 * stride);
        put16<NT>(x3, b + i + 3 * stride);
    }
    for (; i < end; i += stride) put16<NT>(a[i], b + i);
}

// q = a quarter of the buffer in 16-byte words: reads a[i], a[i+q], a[i+2q],
// writes b[i], b[i+q], b[i+2q], b[i+3q] -- 7 x 16 B moved per i, 3:4.
template <bool NT, bool SLAB>
__global__ __launch_bounds__(256) void probe_mix_kernel(const u32x4* __restrict__ a, u32x4* __restrict__ b, size_t q) {
    size_t i, stride, end;
    probe_range<SLAB>(q, i, stride, end);
    for (; i < end; i += stride) {
        const u32x4 x0 = a[i], x1 = a[i + q], x2 = a[i + 2 * q];
        put16<NT>(x0, b + i);
        put16<NT>(x1, b + i + q);
        put16<NT>(x2, b + i + 2 * q);
        put16<NT>(x0 ^ x1 ^ x2, b + i + 3 * q);
    }
}

// Shader clock under load: every CU runs dependent VALU chains; wave 0 of
// block 0 reads the shader-cycle counter (s_memtime) and the fixed-rate
// wall clock (s_memrealtime) around its loop.  out[0] = cycles, out[1] =
// wall ticks.  Issue-bound kernels scale with this clock, streaming ones do
// not -- boxes of one pool differ in both.
__global__ __launch_bounds__(256) void probe_clock_kernel(uint64_t* out, uint32_t iters, uint32_t seed) {
    uint32_t x = threadIdx.x ^ seed, y = x * 7u + 1u;
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (uint32_t i = 0; i < iters; ++i) {
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            x = x * 0x9E3779B1u + y;
            y = y ^ (x >> 7);
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        out[0] = t1 - t0;
        out[1] = r1 - r0;
    }
    if (x == 0x12345678u && y == 0x9ABCDEF0u) out[2] = x;  // keeps the chain live
}

hipError_t launch_clock_probe(uint64_t* out, uint32_t n_cu, hipStream_t stream) {
    hipLaunchKernelGGL(probe_clock_kernel, dim3(n_cu * 8u), dim3(256), 0, stream, out, 20000u, 0x5EEDu);
    return hipGetLastError();
}

// kind (crdtgpu.h CRDT_PROBE_*): 0 read a, 1 write b (nt), 2 copy a -> b (nt),
// 3 write b (plain stores), 4 copy (plain stores), 5 mix 3 reads : 4 writes
// (nt), 6 mix (plain stores); n16 = 16-byte words; blocks_per_cu workgroups
// of 256 threads per CU; slab: each workgroup streams its own contiguous slab.
template <bool SLAB>
static void launch_probe_s(int kind, const u32x4* src, u32x4* dst, size_t n16, uint32_t grid, hipStream_t stream) {
    switch (kind) {
        case 0: hipLaunchKernelGGL((probe_read_kernel<SLAB>), dim3(grid), dim3(256), 0, stream, src, n16, (uint32_t*)dst); break;
        case 1: hipLaunchKernelGGL((probe_write_kernel<true, SLAB>), dim3(grid), dim3(256), 0, stream, dst, n16); break;
        case 2: hipLaunchKernelGGL((probe_copy_kernel<true, SLAB>), dim3(grid), dim3(256), 0, stream, src, dst, n16); break;
        case 3: hipLaunchKernelGGL((probe_write_kernel<false, SLAB>), dim3(grid), dim3(256), 0, stream, dst, n16); break;
        case 5: hipLaunchKernelGGL((probe_mix_kernel<true, SLAB>), dim3(grid), dim3(256), 0, stream, src, dst, n16 / 4); break;
        case 6: hipLaunchKernelGGL((probe_mix_kernel<false, SLAB>), dim3(grid), dim3(256), 0, stream, src, dst, n16 / 4); break;
        default: hipLaunchKernelGGL((probe_copy_kernel<false, SLAB>), dim3(grid), dim3(256), 0, stream, src, dst, n16); break;
    }
}

hipError_t launch_probe(int kind, const void* a, void* b, size_t n16, uint32_t n_cu, uint32_t blocks_per_cu, bool slab,
                        hipStream_t stream) {
    const uint32_t grid = n_cu * blocks_per_cu;
    const u32x4* src = (const u32x4*)a;
    u32x4* dst = (u32x4*)b;
    if (slab)
        launch_probe_s<true>(kind, src, dst, n16, grid, stream);
    else
        launch_probe_s<false>(kind, src, dst, n16, grid, stream);
    return hipGetLastError();
}

}  // namespace crdt
