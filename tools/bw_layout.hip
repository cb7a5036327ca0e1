// Bandwidth probe (diagnostic, not product): does the HBM rate depend on how
// a streaming kernel's workgroups map to addresses?  Three mappings of the
// same 16-B-per-lane read / write / copy over 2 GiB:
//   stride : grid-stride loop (crdt_bw_probe's form): the whole grid sweeps
//            one contiguous window per iteration
//   slab   : workgroup b streams its own contiguous slab b (1/grid of the buffer)
//   xcd    : as slab, but the slabs of one XCD (workgroups b = x mod 8, the
//            dispatcher's round-robin) are adjacent: XCD x owns 1/8 of the
//            buffer as one region
// Build: hipcc --offload-arch=gfx950 -O3 tools/bw_layout.hip -o tools/bw_layout
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e = (x);                                                            \
        if (e != hipSuccess) {                                                         \
            printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__);                \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// MAP 0 stride, 1 slab, 2 xcd; OP 0 read, 1 write (nt), 2 copy (nt stores)
template <int MAP, int OP>
__global__ __launch_bounds__(256) void stream_kernel(const u32x4* __restrict__ a, u32x4* __restrict__ b, size_t n,
                                                     uint32_t* sink) {
    const uint32_t G = gridDim.x, blk = blockIdx.x;
    size_t begin, step, end;
    if (MAP == 0) {
        begin = (size_t)blk * 256 + threadIdx.x;
        step = (size_t)G * 256;
        end = n;
    } else {
        // slab index: MAP 1 = blk; MAP 2 = blocks of XCD x (blk % 8) first, in order
        const uint32_t s = MAP == 1 ? blk : (blk % 8) * (G / 8) + blk / 8;
        const size_t per = n / G;
        begin = (size_t)s * per + threadIdx.x;
        step = 256;
        end = (size_t)(s + 1) * per;
    }
    u32x4 acc = {0u, 0u, 0u, 0u};
    size_t i = begin;
    for (; i + 3 * step < end; i += 4 * step) {
        if (OP == 1) {
            const u32x4 v = {(uint32_t)i, 1u, 2u, 3u};
            __builtin_nontemporal_store(v, b + i);
            __builtin_nontemporal_store(v, b + i + step);
            __builtin_nontemporal_store(v, b + i + 2 * step);
            __builtin_nontemporal_store(v, b + i + 3 * step);
        } else {
            const u32x4 x0 = a[i], x1 = a[i + step], x2 = a[i + 2 * step], x3 = a[i + 3 * step];
            if (OP == 2) {
                __builtin_nontemporal_store(x0, b + i);
                __builtin_nontemporal_store(x1, b + i + step);
                __builtin_nontemporal_store(x2, b + i + 2 * step);
                __builtin_nontemporal_store(x3, b + i + 3 * step);
            } else {
                acc ^= x0 ^ x1 ^ x2 ^ x3;
            }
        }
    }
    for (; i < end; i += step) {
        if (OP == 1) {
            const u32x4 v = {(uint32_t)i, 1u, 2u, 3u};
            __builtin_nontemporal_store(v, b + i);
        } else if (OP == 2) {
            __builtin_nontemporal_store(a[i], b + i);
        } else {
            acc ^= a[i];
        }
    }
    if (OP == 0 && acc.x == 0x9E3779B9u && acc.y == 0x7F4A7C15u) sink[0] = acc.z;
}

template <int MAP, int OP>
static int run(const char* name, const u32x4* a, u32x4* b, size_t n, uint32_t grid, hipEvent_t e0, hipEvent_t e1) {
    const int reps = 10;
    hipLaunchKernelGGL((stream_kernel<MAP, OP>), dim3(grid), dim3(256), 0, 0, a, b, n, (uint32_t*)b);
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL((stream_kernel<MAP, OP>), dim3(grid), dim3(256), 0, 0, a, b, n, (uint32_t*)b);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double bytes = (double)n * 16 * (OP == 2 ? 2 : 1);
    printf("%-6s %-5s grid %6u  %.3f ms  %.0f GB/s\n", name, OP == 0 ? "read" : (OP == 1 ? "write" : "copy"), grid,
           ms / reps, bytes * reps / (ms * 1e-3) / 1e9);
    return 0;
}

int main() {
    const size_t bytes = (size_t)2 << 30, n = bytes / 16;
    u32x4 *a, *b;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMemset(a, 0x5A, bytes));
    CK(hipMemset(b, 0, bytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int round = 0; round < 2; ++round) {
        for (uint32_t grid : {256u * 8, 256u * 16, 256u * 32}) {
            if (run<0, 0>("stride", a, b, n, grid, e0, e1) || run<1, 0>("slab", a, b, n, grid, e0, e1) ||
                run<2, 0>("xcd", a, b, n, grid, e0, e1))
                return 1;
            if (run<0, 1>("stride", a, b, n, grid, e0, e1) || run<1, 1>("slab", a, b, n, grid, e0, e1) ||
                run<2, 1>("xcd", a, b, n, grid, e0, e1))
                return 1;
            if (run<0, 2>("stride", a, b, n, grid, e0, e1) || run<1, 2>("slab", a, b, n, grid, e0, e1) ||
                run<2, 2>("xcd", a, b, n, grid, e0, e1))
                return 1;
        }
    }
    return 0;
}
