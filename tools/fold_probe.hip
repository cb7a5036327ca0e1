// Diagnostic probe (GPU box only, never part of the product): builds the
// fold kernels with CRDT_STAMPS and reports where a wave's cycles go, phase by
// phase, for the config-3 (delta) and config-5 (replicas) workloads.  The
// stamped build is slower than the real kernel; read the SHARES, not the
// time (cdna_hip_programming.md s7, "In-kernel stamps").
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DCRDT_STAMPS tools/fold_probe.hip -o tools/fold_probe
//   tools/fold_probe [config 3|5] [docs]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#ifndef FOLD_SRC  // A/B builds may compile another copy of the fold kernels
#define FOLD_SRC "../go-crdt-playground_amd/csrc/fold.hip"
#endif
#include FOLD_SRC
#include "../go-crdt-playground_amd/csrc/gen.hip"
#include "../go-crdt-playground_amd/csrc/reduce.hip"

using namespace crdt;

// order-independent checksum of an output (the live entries of every document,
// their slot bounds, counts and clocks; slack slots are unspecified and some
// variants write them): variants of the fold must print the same value
__global__ void checksum_kernel(const uint32_t* offsets, const uint32_t* counts, const uint64_t* vv, size_t n_vv,
                                const uint64_t* keys, const uint32_t* actors, const uint64_t* ctrs, uint32_t n,
                                unsigned long long* out) {
    unsigned long long h = 0;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t d = blockIdx.x * (size_t)blockDim.x + threadIdx.x; d < n; d += stride) {
        const size_t o = offsets[d];
        h += o * 0x2545F4914F6CDD1Dull;
        for (uint32_t j = 0; j < counts[d]; ++j) {
            const size_t i = o + j;
            h += (keys[i] * 0x9E3779B97F4A7C15ull) ^ (ctrs[i] * 0xC2B2AE3D27D4EB4Full) ^ ((uint64_t)actors[i] << 17) ^ i;
        }
    }
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n_vv; i += stride)
        h += (vv[i] + 0x165667B19E3779F9ull) * (i + 1);
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += stride) h += (uint64_t)counts[i] << (i & 31);
    atomicAdd(out, h);
}

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(2);                                                                 \
        }                                                                            \
    } while (0)

template <typename T>
T* dalloc(size_t n) {
    void* p = nullptr;
    CK(hipMalloc(&p, (n ? n : 1) * sizeof(T)));
    return (T*)p;
}

OutView make_out(uint32_t n, uint32_t R, size_t slots) {
    return OutView{dalloc<uint32_t>(n + 1), dalloc<uint32_t>(n), dalloc<uint64_t>(slots),
                   dalloc<uint32_t>(slots), dalloc<uint64_t>(slots), dalloc<uint64_t>((size_t)n * R)};
}

int main(int argc, char** argv) {
    const int config = argc > 1 ? atoi(argv[1]) : 3;
    const uint32_t n = argc > 2 ? (uint32_t)atoi(argv[2]) : (config == 5 ? 4000000u : 1048576u);
    const uint32_t R = config == 5 ? 8 : 16, M = config == 5 ? 7 : 10;
    const uint32_t E = config == 5 ? 16 : 8, X = config == 5 ? 0 : 2, nd = config == 5 ? 16 : 64;
    OutView D = make_out(n, R, (size_t)n * nd);
    const size_t ns = (size_t)n * M;
    SrcOutView S{dalloc<uint32_t>(n + 1),   dalloc<uint32_t>(ns),          dalloc<uint64_t>(ns * R),
                 dalloc<uint32_t>(ns + 1),  dalloc<uint64_t>(ns * E),      dalloc<uint32_t>(ns * E),
                 dalloc<uint64_t>(ns * E),  dalloc<uint32_t>(ns + 1),      dalloc<uint64_t>(ns * X + 1),
                 dalloc<uint32_t>(ns * X + 1), dalloc<uint64_t>(ns * X + 1)};
    if (config == 5)
        CK(launch_gen_replicas(0x5EED, n, M + 1, E, D, S, 0));
    else
        CK(launch_gen_delta(0x5EED, n, R, M, D, S, 0));
    const size_t oslots = (size_t)n * nd + ns * E;
    OutView O = make_out(n, R, oslots);
    CK(hipMemset(O.keys, 0, oslots * 8));
    CK(hipMemset(O.counters, 0, oslots * 8));
    CK(hipMemset(O.actors, 0, oslots * 4));
    CK(hipMemset(O.vv, 0, (size_t)n * R * 8));
    CK(hipMemset(O.counts, 0, (size_t)n * 4));
    uint32_t* ws = dalloc<uint32_t>(64);
    CK(hipMemset(ws, 0, 64 * 4));
    Work wk{ws + 16, ws, ws + 1, dalloc<uint32_t>(n), ws + 8, dalloc<uint32_t>(n), ws + 2};
    Scratch scr{dalloc<uint64_t>(oslots), dalloc<uint32_t>(oslots), dalloc<uint64_t>(oslots), oslots};
    BatchView dv{n, R, D.offsets, D.counts, D.keys, D.actors, D.counters, D.vv};
    SrcView sv{n, R, S.doc_srcs, S.src_actor, S.vv, S.entry_off, S.keys, S.actors, S.counters,
               X ? S.tomb_off : nullptr, S.tkeys, S.tactors, S.tcounters};
    const int mode = config == 5 ? CRDT_FOLD_AWSET : CRDT_FOLD_DELTA;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int reps = 5;
    unsigned long long zero[16] = {0};
    for (int r = 0; r < reps + 1; ++r) {
        if (r == 1) {
#ifdef CRDT_STAMPS
            CK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), zero, sizeof(zero)));
#endif
            CK(hipEventRecord(e0, 0));
        }
        CK(launch_reset_work(ws, 0));
        CK(launch_fold(mode, dv, sv, O, scr, wk, 512, getenv("FOLD_GENERAL") == nullptr, 0));
    }
    CK(hipEventRecord(e1, 0));
    CK(hipDeviceSynchronize());
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    unsigned long long st[16] = {0};
#ifdef CRDT_STAMPS
    CK(hipMemcpyFromSymbol(st, HIP_SYMBOL(g_stamps), sizeof(st)));
#endif
    uint32_t status = 0;
    CK(hipMemcpy(&status, ws + 16, 4, hipMemcpyDeviceToHost));
    unsigned long long* dsum = dalloc<unsigned long long>(1);
    CK(hipMemset(dsum, 0, 8));
    hipLaunchKernelGGL(checksum_kernel, dim3(4096), dim3(256), 0, 0, O.offsets, O.counts, O.vv, (size_t)n * R, O.keys,
                       O.actors, O.counters, n, dsum);
    unsigned long long hsum = 0;
    CK(hipMemcpy(&hsum, dsum, 8, hipMemcpyDeviceToHost));
    printf("output checksum %016llx\n", hsum);
    const char* names[16] = {"stage", "prefetch", "schedule", "classify", "noop+keep", "sort-group", "write",
                             "sort|walk-span", "elem-flags|walk-rows", "dot-scan+gaps|walk-bits", "step-of-tuple", "cmax",
                             "meta-next", "noop", "", "doc-loop"};
    double tot = 0;
    for (int i = 0; i < 16; ++i) tot += (double)st[i];
    printf("config %d: %u docs, %.3f ms per stamped launch, status %u\n", config, n, ms / reps, status);
    if (tot == 0) return 0;  // timing build (no stamps)
    printf("wave-cycles per doc (all waves): %.0f\n", tot / reps / n);
    for (int i = 0; i < 16; ++i)
        if (st[i]) printf("  %-14s %6.1f%%  %8.0f cyc/doc\n", names[i], 100.0 * st[i] / tot, (double)st[i] / reps / n);
    return 0;
}
