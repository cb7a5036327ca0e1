// Boundary cost of the drop-in ("pack and H2D are reported
// separately"; §8f-1): what a caller holding reference-shaped states
// (map[string]Dot per replica, awset.go:55-59) pays around the kernels, phase
// by phase, through the C++ host mirror (go-crdt-playground_amd/host/crdt.hpp,
// the same interning and packing its MergeBatch uses):
//   intern   string keys -> order-preserving u64 ids (per document: the ranks
//            of the document's keys; documents spread over host threads)
//   pack     maps -> sorted SoA arrays (keys, actors, counters, offsets, vv)
//   h2d      pageable host -> HBM copies of both states
//   kernel   the exchange (A<-B and B<-A from one read), device time
//   d2h      both outputs back
//   unpack   SoA -> map[string]Dot per doc, both outputs
// Workload: config-2-shaped docs (2 replicas x 64 entries, R = 2, ~50% common
// keys, string keys of 12-16 bytes), n docs (default 65,536).  Prints one
// JSON object.  GPU box only.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../../go-crdt-playground_amd/host/crdt.hpp"

using namespace crdt;
using clk = std::chrono::steady_clock;

static double secs(clk::time_point a, clk::time_point b) { return std::chrono::duration<double>(b - a).count(); }

static uint64_t mix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

#define HIPCHECK(x)                                                   \
    do {                                                              \
        if ((x) != hipSuccess) {                                      \
            fprintf(stderr, "HIP error at %s:%d\n", __FILE__, __LINE__); \
            return 1;                                                 \
        }                                                             \
    } while (0)

template <typename T>
static T* dev_copy(const std::vector<T>& v) {
    T* p = nullptr;
    if (hipMalloc(&p, std::max<size_t>(v.size(), 1) * sizeof(T)) != hipSuccess) return nullptr;
    if (!v.empty() && hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice) != hipSuccess) return nullptr;
    return p;
}

template <typename T>
static T* dev_alloc(size_t n) {
    T* p = nullptr;
    return hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(T)) == hipSuccess ? p : nullptr;
}

static size_t keys_interned(const detail::Batch& b) {
    size_t k = 0;
    for (auto& v : b.names) k += v.size();
    return k;
}

int main(int argc, char** argv) {
    const size_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 65536;
    const int E = 64;
    // reference-shaped states (not timed)
    std::vector<AWSet> A(n, AWSet(0, VersionVector{0, 0})), B(n, AWSet(1, VersionVector{0, 0}));
    for (size_t d = 0; d < n; ++d) {
        for (int i = 0; i < E; ++i) {
            const uint64_t h = mix(d * 1315423911ull + i);
            A[d].entries["doc" + std::to_string(d) + "/a" + std::to_string(i)] = Dot{0, 1 + (h % 40)};
            const bool common = i < E / 2;
            const std::string kb = common ? "doc" + std::to_string(d) + "/a" + std::to_string(i)
                                          : "doc" + std::to_string(d) + "/b" + std::to_string(i);
            B[d].entries[kb] = Dot{(uint32_t)(h >> 40) & 1u, 1 + ((h >> 8) % 40)};
        }
        A[d].versionVector = VersionVector{40, 20};
        B[d].versionVector = VersionVector{20, 40};
    }
    std::vector<AWSet*> pa, pb;
    for (size_t d = 0; d < n; ++d) {
        pa.push_back(&A[d]);
        pb.push_back(&B[d]);
    }
    crdt_ctx* ctx = nullptr;
    if (crdt_ctx_create(0, &ctx) != CRDT_OK) return 1;

    auto t0 = clk::now();
    detail::Batch b;
    b.R = 2;
    detail::intern_all(b, n, [&](size_t d) { return std::vector<const AWSet*>{pa[d], pb[d]}; });
    auto t1 = clk::now();
    detail::Packed xa = b.pack(pa), xb = b.pack(pb);
    auto t2 = clk::now();
    crdt_awset_batch ha = b.view(xa), hb = b.view(xb);
    const size_t slots = xa.keys.size() + xb.keys.size();
    crdt_awset_batch da = ha, db = hb;
    da.offsets = dev_copy(xa.offsets);
    da.keys = dev_copy(xa.keys);
    da.actors = dev_copy(xa.actors);
    da.counters = dev_copy(xa.counters);
    da.vv = dev_copy(xa.vv);
    db.offsets = dev_copy(xb.offsets);
    db.keys = dev_copy(xb.keys);
    db.actors = dev_copy(xb.actors);
    db.counters = dev_copy(xb.counters);
    db.vv = dev_copy(xb.vv);
    HIPCHECK(hipDeviceSynchronize());
    auto t3 = clk::now();
    crdt_awset_out o[2];
    for (auto& x : o)
        x = crdt_awset_out{dev_alloc<uint32_t>(n + 1), dev_alloc<uint32_t>(n), dev_alloc<uint64_t>(slots),
                           dev_alloc<uint32_t>(slots), dev_alloc<uint64_t>(slots), dev_alloc<uint64_t>(n * b.R)};
    // one untimed exchange warms the context's workspace
    if (crdt_awset_exchange_async(ctx, &da, &db, &o[0], &o[1], nullptr) != CRDT_OK) return 1;
    if (crdt_ctx_sync(ctx, nullptr) != CRDT_OK) return 1;
    hipEvent_t e0, e1;
    HIPCHECK(hipEventCreate(&e0));
    HIPCHECK(hipEventCreate(&e1));
    HIPCHECK(hipEventRecord(e0, nullptr));
    if (crdt_awset_exchange_async(ctx, &da, &db, &o[0], &o[1], nullptr) != CRDT_OK) return 1;
    HIPCHECK(hipEventRecord(e1, nullptr));
    if (crdt_ctx_sync(ctx, nullptr) != CRDT_OK) return 1;
    float kms = 0;
    HIPCHECK(hipEventElapsedTime(&kms, e0, e1));
    auto t4 = clk::now();
    std::vector<uint32_t> counts[2];
    detail::Packed po[2];
    for (int i = 0; i < 2; ++i) {
        crdt_awset_out h;
        po[i] = detail::make_out(n, b.R, slots, counts[i], h);
        HIPCHECK(hipMemcpy(h.offsets, o[i].offsets, (n + 1) * 4, hipMemcpyDeviceToHost));
        HIPCHECK(hipMemcpy(h.counts, o[i].counts, n * 4, hipMemcpyDeviceToHost));
        HIPCHECK(hipMemcpy(h.keys, o[i].keys, slots * 8, hipMemcpyDeviceToHost));
        HIPCHECK(hipMemcpy(h.actors, o[i].actors, slots * 4, hipMemcpyDeviceToHost));
        HIPCHECK(hipMemcpy(h.counters, o[i].counters, slots * 8, hipMemcpyDeviceToHost));
        HIPCHECK(hipMemcpy(h.vv, o[i].vv, n * b.R * 8, hipMemcpyDeviceToHost));
    }
    auto t5 = clk::now();
    std::vector<size_t> widths(n, 2);
    std::vector<AWSet> OA(n), OB(n);
    std::vector<AWSet*> poa, pob;
    for (size_t d = 0; d < n; ++d) {
        poa.push_back(&OA[d]);
        pob.push_back(&OB[d]);
    }
    b.unpack(poa, po[0], counts[0], widths);
    b.unpack(pob, po[1], counts[1], widths);
    auto t6 = clk::now();
    // sanity: common keys take the src dot in A<-B
    size_t live = 0;
    for (size_t d = 0; d < n; ++d) live += OA[d].entries.size();
    const double intern = secs(t0, t1), pack = secs(t1, t2), h2d = secs(t2, t3), d2h = secs(t4, t5),
                 unpack = secs(t5, t6), kernel = kms / 1e3;
    const double merges = 2.0 * n;
    const double total = intern + pack + h2d + kernel + d2h + unpack;
    printf("{\"docs\": %zu, \"entries_per_replica\": %d, \"keys_interned\": %zu, \"out_entries_per_doc\": %.2f, "
           "\"intern_s\": %.6f, \"pack_s\": %.6f, \"h2d_s\": %.6f, \"kernel_s\": %.6f, \"d2h_s\": %.6f, "
           "\"unpack_s\": %.6f, \"host_threads\": %u, \"end_to_end_merges_per_s\": %.1f, \"kernel_only_merges_per_s\": %.1f, "
           "\"pcie_inclusive_merges_per_s\": %.1f}\n",
           n, E, keys_interned(b), (double)live / n, intern, pack, h2d, kernel, d2h, unpack, detail::host_threads(), merges / total,
           merges / kernel, merges / (h2d + kernel + d2h));
    crdt_ctx_destroy(ctx);
    return 0;
}
