// CPU-only profile of the C++ mirror's host path (tools, not a test of the
// engine): ExchangeBatch's pack and apply phases on config-2-shaped maps with
// the device call replaced by the C oracle's join (oracle/awset_oracle.c), so
// the host work can be measured and tuned on a machine with no GPU.  The C ABI
// symbols the mirror uses are defined here; nothing of libcrdtgpu.so is linked.
//   g++ -O2 -std=c++17 -pthread tests/cpp/host_path_prof.cpp -Loracle/build -loracle -Wl,-rpath,oracle/build
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "../../go-crdt-playground_amd/host/crdt.hpp"

extern "C" {
int oracle_awset_join(const crdt_awset_batch* dst, const crdt_awset_batch* src, const crdt_awset_out* out);
struct crdt_ctx {
    int dummy;
};
int crdt_ctx_create(int, crdt_ctx** out) {
    *out = new crdt_ctx{0};
    return CRDT_OK;
}
void crdt_ctx_destroy(crdt_ctx* c) { delete c; }
int crdt_ctx_set_option(crdt_ctx*, const char*, int64_t) { return CRDT_OK; }
const char* crdt_strerror(int) { return "error"; }
int crdt_host_alloc(size_t bytes, void** out) {
    *out = malloc(bytes);
    return *out ? CRDT_OK : CRDT_E_NOMEM;
}
void crdt_host_free(void* p) { free(p); }
int crdt_awset_exchange_batch(crdt_ctx*, const crdt_awset_batch* a, const crdt_awset_batch* b,
                              const crdt_awset_out* oab, const crdt_awset_out* oba) {
    int rc = oracle_awset_join(a, b, oab);
    return rc ? rc : oracle_awset_join(b, a, oba);
}
int crdt_awset_join_batch(crdt_ctx*, const crdt_awset_batch* d, const crdt_awset_batch* s, const crdt_awset_out* o) {
    return oracle_awset_join(d, s, o);
}
int crdt_awset_fold_batch(crdt_ctx*, int, const crdt_awset_batch*, const crdt_src_batch*, const crdt_awset_out*) {
    return CRDT_E_INVALID;
}
}

using namespace crdt;

static uint64_t mix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

int main(int argc, char** argv) {
    const size_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 65536;
    const int E = 64;
    std::vector<AWSet> A(n, AWSet(0, VersionVector{0, 0})), B(n, AWSet(1, VersionVector{0, 0}));
    for (size_t d = 0; d < n; ++d) {
        for (int i = 0; i < E; ++i) {
            const uint64_t h = mix(d * 1315423911ull + i);
            A[d].entries["doc" + std::to_string(d) + "/a" + std::to_string(i)] = Dot{0, 1 + (h % 40)};
            const std::string kb = i < E / 2 ? "doc" + std::to_string(d) + "/a" + std::to_string(i)
                                             : "doc" + std::to_string(d) + "/b" + std::to_string(i);
            B[d].entries[kb] = Dot{(uint32_t)(h >> 40) & 1u, 1 + ((h >> 8) % 40)};
        }
        A[d].versionVector = VersionVector{40, 20};
        B[d].versionVector = VersionVector{20, 40};
    }
    std::vector<AWSet> WA = A, WB = B;
    auto ptrs = [](std::vector<AWSet>& v) {
        std::vector<AWSet*> p;
        for (auto& x : v) p.push_back(&x);
        return p;
    };
    Engine eng(0);
    ExchangeBatch(ptrs(WA), ptrs(WB), eng);
    auto t0 = std::chrono::steady_clock::now();
    ExchangeBatch(ptrs(A), ptrs(B), eng);
    const double total = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    const BoundaryStats st = LastStats();
    printf("threads %u docs %zu: pack %.4f oracle %.4f apply %.4f in-call %.4f total %.4f\n", detail::host_threads(), n,
           st.pack_s, st.device_s, st.apply_s, st.call_s, total);
    return 0;
}
