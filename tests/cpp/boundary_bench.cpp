// Boundary cost of the drop-in ("pack and H2D are reported
// separately"; §8f-1): what a caller holding reference-shaped states
// (map[string]Dot per replica, awset.go:55-59) pays end to end for the two
// merges A <- B and B <- A of every document, through the C++ host mirror's
// ExchangeBatch (go-crdt-playground_amd/host/crdt.hpp), phase by phase:
//   pack     string keys -> 64-bit hash ids (exact per-document collision
//            check), entries sorted by id into page-locked SoA arrays
//   device   crdt_awset_exchange_batch: H2D, the exchange kernel, D2H
//   apply    each result applied to its map in place (erase / overwrite /
//            insert), as the reference's merge mutates dst.Entries
// Workload: config-2-shaped docs (2 replicas x 64 entries, R = 2, ~50% common
// keys, string keys of 12-16 bytes), n docs (default 65,536).  One untimed
// call on a copy of the states first (it sizes the page-locked staging and the
// host scratch, which a long-running caller keeps).  Both the GPU path and the
// CPU reference merge run on copy-constructed maps of the same states, and
// every document of both directions is compared between them afterwards
// (sample_docs_checked = docs), plus 64 documents against single Merge calls.
// Prints one JSON object.  GPU box only.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "../../go-crdt-playground_amd/host/crdt.hpp"

using namespace crdt;
using clk = std::chrono::steady_clock;

static uint64_t mix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

static void make_states(size_t n, int E, std::vector<AWSet>& A, std::vector<AWSet>& B) {
    A.assign(n, AWSet(0, VersionVector{0, 0}));
    B.assign(n, AWSet(1, VersionVector{0, 0}));
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
}

// The reference merge on the same maps, for the CPU comparison on identical
// states (test infrastructure: a restatement of awset.go:107-161 without the
// decision log; HasDot crdt-misc.go:28-34, VersionVector.Merge :43-55).
static void cpu_merge(AWSet& dst, const AWSet& src) {
    for (auto& kv : src.entries) {
        auto it = dst.entries.find(kv.first);
        if (it != dst.entries.end()) {
            it->second = kv.second;  // awset.go:142: the src dot wins
        } else if (!dst.versionVector.HasDot(kv.second)) {
            dst.entries.emplace(kv.first, kv.second);
        }
    }
    for (auto it = dst.entries.begin(); it != dst.entries.end();) {
        if (!src.entries.count(it->first) && src.versionVector.HasDot(it->second))
            it = dst.entries.erase(it);
        else
            ++it;
    }
    dst.versionVector.Merge(src.versionVector);
}

int main(int argc, char** argv) {
    const size_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 65536;
    const int E = 64;
    std::vector<AWSet> A0, B0, A, B, WA, WB;
    make_states(n, E, A0, B0);
    // every timed path (GPU and CPU) works on copy-constructed maps of the same
    // states, so node layouts in memory are alike
    A = A0, B = B0, WA = A0, WB = B0;
    // reference answer for a sample of documents: x := a.Clone(); x.Merge(b) on the GPU one by one later
    std::vector<size_t> sample;
    for (size_t d = 0; d < n; d += std::max<size_t>(1, n / 64)) sample.push_back(d);
    std::vector<AWSet> SA, SB;
    for (size_t d : sample) {
        SA.push_back(A[d]);
        SB.push_back(B[d]);
    }
    auto ptrs = [](std::vector<AWSet>& v) {
        std::vector<AWSet*> p;
        for (auto& x : v) p.push_back(&x);
        return p;
    };
    Engine eng(0);
    ExchangeBatch(ptrs(WA), ptrs(WB), eng);  // untimed: sizes the page-locked staging
    const std::vector<AWSet*> pa = ptrs(A), pb = ptrs(B);  // the caller's own arrays, made before timing
    auto t0 = clk::now();
    ExchangeBatch(pa, pb, eng);
    const double total = std::chrono::duration<double>(clk::now() - t0).count();
    const BoundaryStats st = LastStats();
    // check the sample against single merges of the same snapshot
    size_t bad = 0;
    for (size_t i = 0; i < sample.size(); ++i) {
        AWSet x = SA[i], y = SB[i];
        x.Merge(SB[i], eng);
        y.Merge(SA[i], eng);
        const size_t d = sample[i];
        bad += x.entries != A[d].entries || x.versionVector != A[d].versionVector;
        bad += y.entries != B[d].entries || y.versionVector != B[d].versionVector;
    }
    size_t live = 0;
    for (size_t d = 0; d < n; ++d) live += A[d].entries.size();
    // CPU: the reference merge, both directions, on the same (untouched) states,
    // every host thread over documents; the clones are made untimed
    std::vector<AWSet> CA, CB;
    double cpu_s = 0;
    {
        CA = A0;
        CB = B0;
        auto c0 = clk::now();
        detail::parallel_docs(n, [&](size_t lo, size_t hi) {
            for (size_t d = lo; d < hi; ++d) {
                cpu_merge(CA[d], B0[d]);
                cpu_merge(CB[d], A0[d]);
            }
        });
        cpu_s = std::chrono::duration<double>(clk::now() - c0).count();
    }
    // every document of both directions against the reference merge on the
    // same states (untimed; one thread per document range)
    std::vector<size_t> bad_of(detail::host_threads() + 1, 0);
    {
        std::vector<std::thread> pool;
        const size_t t = bad_of.size(), chunk = (n + t - 1) / t;
        for (size_t i = 0; i < t; ++i)
            pool.emplace_back([&, i] {
                for (size_t d = i * chunk; d < std::min(n, (i + 1) * chunk); ++d) {
                    bad_of[i] += CA[d].entries != A[d].entries || CA[d].versionVector != A[d].versionVector;
                    bad_of[i] += CB[d].entries != B[d].entries || CB[d].versionVector != B[d].versionVector;
                }
            });
        for (auto& th : pool) th.join();
    }
    for (size_t b : bad_of) bad += b;
    const double merges = 2.0 * n;
    printf("{\"docs\": %zu, \"entries_per_replica\": %d, \"out_entries_per_doc\": %.2f, \"pack_s\": %.6f, "
           "\"device_s\": %.6f, \"apply_s\": %.6f, \"call_s\": %.6f, \"total_s\": %.6f, \"rank_docs\": %zu, \"host_threads\": %u, "
           "\"host_phases_s\": {\"batch\": %.6f, \"layout\": %.6f, \"pack_docs\": %.6f, \"distinct\": %.6f}, "
           "\"end_to_end_merges_per_s\": %.1f, \"pcie_inclusive_merges_per_s\": %.1f, "
           "\"cpu_same_states_merges_per_s\": %.1f, \"sample_docs_checked\": %zu, \"single_merge_docs_checked\": %zu, "
           "\"sample_mismatches\": %zu}\n",
           n, E, (double)live / n, st.pack_s, st.device_s, st.apply_s, st.call_s, total, st.rank_docs, detail::host_threads(),
           st.batch_s, st.layout_s, st.docs_s, st.distinct_s,
           merges / total, merges / st.device_s, merges / cpu_s, n, sample.size(), bad);
    return bad ? 1 : 0;
}
