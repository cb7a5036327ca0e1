// Diagnostic probe (GPU box only, never part of the product): host -> device
// staging of one boundary-sized batch (the byte sizes the exchange call stages
// for 65,536 documents x 64 entries per replica) from page-locked memory, timed
// per hipMemcpyAsync call and in total, with the host buffers written just
// before by 1 or 16 threads (as the mirror's pack phase does).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/h2d_probe.hip -o tools/h2d_probe -pthread
//   tools/h2d_probe [flags: 0 default, 1 non-coherent, 2 write-combined]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(2);                                                                           \
        }                                                                                      \
    } while (0)

using clk = std::chrono::steady_clock;
static double ms_since(clk::time_point t) { return std::chrono::duration<double, std::milli>(clk::now() - t).count(); }

int main(int argc, char** argv) {
    const int mode = argc > 1 ? atoi(argv[1]) : 0;
    const unsigned flags = mode == 1 ? hipHostMallocNonCoherent : (mode == 2 ? hipHostMallocWriteCombined : 0u);
    const size_t n = 65536, e = 64, slots = n * e;
    const std::vector<size_t> sizes = {(n + 1) * 4, slots * 8, slots * 4, slots * 8, n * 16 * 8,
                                       (n + 1) * 4, slots * 8, slots * 4, slots * 8, n * 16 * 8};
    std::vector<void*> h(sizes.size()), d(sizes.size());
    for (size_t i = 0; i < sizes.size(); ++i) {
        CK(hipHostMalloc(&h[i], sizes[i], flags));
        CK(hipMalloc(&d[i], sizes[i]));
    }
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    for (int rep = 0; rep < 6; ++rep) {
        const int threads = rep % 2 ? 16 : 1;
        {
            std::vector<std::thread> pool;
            for (int t = 0; t < threads; ++t)
                pool.emplace_back([&, t] {
                    for (size_t i = 0; i < sizes.size(); ++i) {
                        const size_t lo = sizes[i] * t / threads, hi = sizes[i] * (t + 1) / threads;
                        memset((char*)h[i] + lo, rep + 1, hi - lo);
                    }
                });
            for (auto& th : pool) th.join();
        }
        const auto t0 = clk::now();
        double worst = 0;
        for (size_t i = 0; i < sizes.size(); ++i) {
            const auto t1 = clk::now();
            CK(hipMemcpyAsync(d[i], h[i], sizes[i], hipMemcpyHostToDevice, s));
            worst = std::max(worst, ms_since(t1));
        }
        const double issue = ms_since(t0);
        CK(hipStreamSynchronize(s));
        const double tot = ms_since(t0);
        size_t bytes = 0;
        for (size_t z : sizes) bytes += z;
        printf("flags %u, filled by %2d threads: issue %.3f ms (worst call %.3f), total %.3f ms, %.1f GB/s\n", flags,
               threads, issue, worst, tot, bytes / (tot * 1e-3) / 1e9);
    }
    return 0;
}
