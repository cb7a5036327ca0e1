// Diagnostic (GPU box only, not part of the product): how long do
// host->device copies from page-locked buffers take when the buffers were
// just written by many host threads, as the C++ mirror's pack does before a
// *_batch call?  Times the host call and the copy separately.
//   hipcc -O2 -std=c++17 -pthread tools/h2d_probe.cpp -o tools/h2d_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                \
    do {                                                                     \
        hipError_t e_ = (x);                                                 \
        if (e_ != hipSuccess) {                                              \
            printf("%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            return 1;                                                        \
        }                                                                    \
    } while (0)

using clk = std::chrono::steady_clock;
static double ms_since(clk::time_point t) { return std::chrono::duration<double, std::milli>(clk::now() - t).count(); }

int main() {
    const size_t sizes[] = {33554432, 16777216, 33554432, 1048576};  // keys, actors, counters, vv of 65,536 docs
    std::vector<void*> h(4), d(4);
    for (int i = 0; i < 4; ++i) {
        CK(hipHostMalloc(&h[i], sizes[i], hipHostMallocDefault));
        CK(hipMalloc(&d[i], sizes[i]));
    }
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    for (int round = 0; round < 4; ++round) {
        const unsigned T = round < 2 ? 16 : 1;
        auto t0 = clk::now();
        std::vector<std::thread> pool;
        for (unsigned t = 0; t < T; ++t)
            pool.emplace_back([&, t] {
                for (int i = 0; i < 4; ++i) {
                    const size_t chunk = sizes[i] / T;
                    memset((char*)h[i] + t * chunk, round + 1, chunk);
                }
            });
        for (auto& th : pool) th.join();
        const double fill = ms_since(t0);
        double call[4];
        t0 = clk::now();
        for (int i = 0; i < 4; ++i) {
            auto t1 = clk::now();
            CK(hipMemcpyAsync(d[i], h[i], sizes[i], hipMemcpyHostToDevice, s));
            call[i] = ms_since(t1);
        }
        CK(hipStreamSynchronize(s));
        const double total = ms_since(t0);
        printf("round %d (fill %u threads %.2f ms): calls %.3f %.3f %.3f %.3f ms, all copies done %.3f ms (%.1f GB/s)\n",
               round, T, fill, call[0], call[1], call[2], call[3], total,
               (sizes[0] + sizes[1] + sizes[2] + sizes[3]) / (total * 1e6));
    }
    return 0;
}
