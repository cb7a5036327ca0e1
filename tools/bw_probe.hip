// Bandwidth probe (diagnostic, not product): what does the join's SoA access
// pattern cost with NO merge work?  Build: hipcc --offload-arch=gfx950 -O3
// tools/bw_probe.hip -o tools/bw_probe ; run on the GPU box.
//   copy16   : float4 streaming copy (the chip's copy ceiling)
//   doc8     : per doc, read dst/src keys(8B)/actors(4B)/counters(8B) x 64
//              lanes, write keys/actors/counters for n_out = 81 slots of a
//              128-slot region -- the join's exact traffic, 8 B per lane
//   doc16    : same bytes, 16 B per lane loads (keys, counters), stores 8 B
//   docread  : reads only (the join's 2.7 GB), writes nothing
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void copy16(const float4* __restrict__ a, float4* __restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) b[i] = a[i];
}

// 4 independent float4 per thread per iteration; NT = non-temporal stores
typedef float f4v __attribute__((ext_vector_type(4)));
template <bool NT>
__global__ void copy16x4(const f4v* __restrict__ a, f4v* __restrict__ b, size_t n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i + 3 * stride < n; i += 4 * stride) {
        f4v x0 = a[i], x1 = a[i + stride], x2 = a[i + 2 * stride], x3 = a[i + 3 * stride];
        if (NT) {
            __builtin_nontemporal_store(x0, b + i);
            __builtin_nontemporal_store(x1, b + i + stride);
            __builtin_nontemporal_store(x2, b + i + 2 * stride);
            __builtin_nontemporal_store(x3, b + i + 3 * stride);
        } else {
            b[i] = x0; b[i + stride] = x1; b[i + 2 * stride] = x2; b[i + 3 * stride] = x3;
        }
    }
}

// read-only float4 stream
__global__ void read16(const float4* __restrict__ a, float* out, size_t n) {
    float acc = 0.f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        float4 x = a[i];
        acc += x.x + x.y + x.z + x.w;
    }
    if (acc == 1.2345f) out[0] = acc;
}

// write-only float4 stream
__global__ void write16(float4* __restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        b[i] = make_float4(1.f, 2.f, 3.f, (float)i);
}

template <int MODE>
__global__ __launch_bounds__(256) void doc_kernel(const uint64_t* __restrict__ dk, const uint32_t* __restrict__ da,
                                                  const uint64_t* __restrict__ dc, const uint64_t* __restrict__ sk,
                                                  const uint32_t* __restrict__ sa, const uint64_t* __restrict__ sc,
                                                  uint64_t* __restrict__ ok, uint32_t* __restrict__ oa,
                                                  uint64_t* __restrict__ oc, uint32_t n_docs, uint32_t n_out) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t d = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (d >= n_docs) return;
    const size_t i = (size_t)d * 64 + lane;
    uint64_t k0, c0, k1, c1;
    uint32_t a0 = da[i], a1 = sa[i];
    if (MODE == 1) {  // 16 B per lane: lanes 0..31 read 2 keys each
        const uint4* p = reinterpret_cast<const uint4*>(dk + (size_t)d * 64);
        const uint4* q = reinterpret_cast<const uint4*>(sk + (size_t)d * 64);
        const uint4* r = reinterpret_cast<const uint4*>(dc + (size_t)d * 64);
        const uint4* t = reinterpret_cast<const uint4*>(sc + (size_t)d * 64);
        uint4 x = p[lane & 31], y = q[lane & 31], z = r[lane & 31], u = t[lane & 31];
        k0 = ((uint64_t)x.y << 32) | x.x;
        k1 = ((uint64_t)y.y << 32) | y.x;
        c0 = ((uint64_t)z.w << 32) | z.z;
        c1 = ((uint64_t)u.w << 32) | u.z;
    } else {
        k0 = dk[i];
        c0 = dc[i];
        k1 = sk[i];
        c1 = sc[i];
    }
    if (MODE == 2) {  // reads only; keep values live
        if ((k0 ^ c0 ^ k1 ^ c1 ^ a0 ^ a1) == 0x123456789ull) ok[0] = 1;
        return;
    }
    const size_t o = (size_t)d * 128;
    // dst lanes write slots [0, 64) minus holes, src lanes the rest up to n_out
    if (MODE == 3) {  // non-temporal stores
        if (lane < 48) {
            __builtin_nontemporal_store(k0 ^ k1, ok + o + lane);
            __builtin_nontemporal_store(a0, oa + o + lane);
            __builtin_nontemporal_store(c0, oc + o + lane);
        }
        if (lane < n_out - 48) {
            __builtin_nontemporal_store(k1, ok + o + 48 + lane);
            __builtin_nontemporal_store(a1, oa + o + 48 + lane);
            __builtin_nontemporal_store(c1, oc + o + 48 + lane);
        }
        return;
    }
    if (lane < 48) {
        ok[o + lane] = k0 ^ k1;
        oa[o + lane] = a0;
        oc[o + lane] = c0;
    }
    if (lane < n_out - 48) {
        ok[o + 48 + lane] = k1;
        oa[o + 48 + lane] = a1;
        oc[o + 48 + lane] = c1;
    }
}

int main() {
    const uint32_t n_docs = 1u << 20;
    const size_t ne = (size_t)n_docs * 64, no = (size_t)n_docs * 128;
    uint64_t *dk, *dc, *sk, *sc, *ok, *oc;
    uint32_t *da, *sa, *oa;
    CK(hipMalloc(&dk, ne * 8)); CK(hipMalloc(&dc, ne * 8)); CK(hipMalloc(&sk, ne * 8)); CK(hipMalloc(&sc, ne * 8));
    CK(hipMalloc(&da, ne * 4)); CK(hipMalloc(&sa, ne * 4));
    CK(hipMalloc(&ok, no * 8)); CK(hipMalloc(&oc, no * 8)); CK(hipMalloc(&oa, no * 4));
    CK(hipMemset(dk, 1, ne * 8)); CK(hipMemset(dc, 2, ne * 8)); CK(hipMemset(sk, 3, ne * 8)); CK(hipMemset(sc, 4, ne * 8));
    CK(hipMemset(da, 5, ne * 4)); CK(hipMemset(sa, 6, ne * 4));
    const size_t cn = (size_t)1 << 28;  // 4 GiB float4 copy
    float4 *ca, *cb;
    CK(hipMalloc(&ca, cn * 16 / 2)); CK(hipMalloc(&cb, cn * 16 / 2));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const uint32_t n_out = 81;
    const double rd = 20.0 * 128 * n_docs, wr = 20.0 * n_out * n_docs;
    for (int round = 0; round < 2; ++round) {
        float ms;
        CK(hipEventRecord(e0));
        for (int r = 0; r < 5; ++r) copy16<<<8192, 256>>>(ca, cb, cn / 2);
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
        printf("copy16   %.3f ms  %.0f GB/s (r+w)\n", ms / 5, 2.0 * cn / 2 * 16 / (ms / 5 / 1e3) / 1e9);
        for (int g : {2048, 8192, 32768}) {
            CK(hipEventRecord(e0));
            for (int r = 0; r < 5; ++r) copy16x4<false><<<g, 256>>>((const f4v*)ca, (f4v*)cb, cn / 2);
            CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
            printf("copy16x4 grid %5d  %.3f ms  %.0f GB/s (r+w)\n", g, ms / 5, 2.0 * cn / 2 * 16 / (ms / 5 / 1e3) / 1e9);
            CK(hipEventRecord(e0));
            for (int r = 0; r < 5; ++r) copy16x4<true><<<g, 256>>>((const f4v*)ca, (f4v*)cb, cn / 2);
            CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
            printf("copy16x4nt grid %5d %.3f ms  %.0f GB/s (r+w)\n", g, ms / 5, 2.0 * cn / 2 * 16 / (ms / 5 / 1e3) / 1e9);
        }
        CK(hipEventRecord(e0));
        for (int r = 0; r < 5; ++r) read16<<<8192, 256>>>(ca, (float*)cb, cn / 2);
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
        printf("read16   %.3f ms  %.0f GB/s\n", ms / 5, 1.0 * cn / 2 * 16 / (ms / 5 / 1e3) / 1e9);
        CK(hipEventRecord(e0));
        for (int r = 0; r < 5; ++r) write16<<<8192, 256>>>(cb, cn / 2);
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
        printf("write16  %.3f ms  %.0f GB/s\n", ms / 5, 1.0 * cn / 2 * 16 / (ms / 5 / 1e3) / 1e9);
        const char* names[4] = {"doc8    ", "doc16   ", "docread ", "doc8nt  "};
        for (int m = 0; m < 4; ++m) {
            CK(hipEventRecord(e0));
            for (int r = 0; r < 5; ++r) {
                if (m == 0) doc_kernel<0><<<n_docs / 4, 256>>>(dk, da, dc, sk, sa, sc, ok, oa, oc, n_docs, n_out);
                if (m == 1) doc_kernel<1><<<n_docs / 4, 256>>>(dk, da, dc, sk, sa, sc, ok, oa, oc, n_docs, n_out);
                if (m == 2) doc_kernel<2><<<n_docs / 4, 256>>>(dk, da, dc, sk, sa, sc, ok, oa, oc, n_docs, n_out);
                if (m == 3) doc_kernel<3><<<n_docs / 4, 256>>>(dk, da, dc, sk, sa, sc, ok, oa, oc, n_docs, n_out);
            }
            CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
            const double bytes = (m == 2) ? rd : rd + wr;
            printf("%s %.3f ms  %.0f GB/s\n", names[m], ms / 5, bytes / (ms / 5 / 1e3) / 1e9);
        }
    }
    return 0;
}
