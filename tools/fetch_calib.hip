// Known-byte reads for the FETCH_SIZE correction of the tile kernel's access
// pattern (diagnostic, GPU box only, never part of the product).  tools/calib.py
// calibrates 8-byte-per-lane streaming (vv_max_kernel, the join's key/counter
// width); the config-4 tile kernel reads each element as an 8-byte key, a
// 4-byte actor and an 8-byte counter, per-lane addresses, non-temporal.  Three
// kernels, each streaming a known number of bytes once per launch:
//   read8    u64 per lane
//   read4    u32 per lane
//   readmix  u64 + u32 + u64 per lane from three arrays (the tile's element)
// Run under `rocprofv3 --pmc FETCH_SIZE` (tools/pmc.sh, config 4): the
// correction of a pattern = its bytes / (FETCH_SIZE x 1024).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/fetch_calib.hip -o tools/fetch_calib
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                          \
    do {                                                                                               \
        hipError_t e_ = (x);                                                                           \
        if (e_ != hipSuccess) {                                                                        \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));          \
            exit(2);                                                                                   \
        }                                                                                              \
    } while (0)

template <typename T>
__global__ void read1(const T* a, size_t n, unsigned long long* sink) {
    unsigned long long acc = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        acc += __builtin_nontemporal_load(a + i);
    if (acc == 0x1234567ull) sink[0] = acc;  // (never: keeps the loads)
}

__global__ void readmix(const unsigned long long* k, const unsigned* a, const unsigned long long* c, size_t n,
                        unsigned long long* sink) {
    unsigned long long acc = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        acc += __builtin_nontemporal_load(k + i) ^ __builtin_nontemporal_load(a + i) ^
               __builtin_nontemporal_load(c + i);
    if (acc == 0x1234567ull) sink[0] = acc;
}

int main() {
    const size_t n = 64ull << 20;  // elements: 512 MiB of u64, 256 MiB of u32
    unsigned long long *k, *c, *sink;
    unsigned* a;
    CK(hipMalloc(&k, n * 8));
    CK(hipMalloc(&c, n * 8));
    CK(hipMalloc(&a, n * 4));
    CK(hipMalloc(&sink, 8));
    CK(hipMemset(k, 1, n * 8));
    CK(hipMemset(c, 2, n * 8));
    CK(hipMemset(a, 3, n * 4));
    const dim3 grid(256 * 16), block(256);
    for (int r = 0; r < 3; ++r) {
        hipLaunchKernelGGL(read1<unsigned long long>, grid, block, 0, 0, k, n, sink);
        hipLaunchKernelGGL(read1<unsigned>, grid, block, 0, 0, a, n, sink);
        hipLaunchKernelGGL(readmix, grid, block, 0, 0, k, a, c, n, sink);
    }
    CK(hipDeviceSynchronize());
    printf("fetch_calib: read1<u64> %zu B, read1<u32> %zu B, readmix %zu B per launch\n", n * 8, n * 4, n * 20);
    return 0;
}
