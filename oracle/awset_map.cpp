// TEST INFRASTRUCTURE ONLY -- the CPU baseline and a second, independent
// oracle: a C++ restatement of the reference merge over hash maps keyed by
// strings, the same data structure as the reference (map[string]Dot,
// awset.go:55-59; Deleted map, awset-delta_test.go:9-12).
//
// Only tests/ and bench.py's cpu_baseline leg load it.  It is labelled as
// C++ everywhere it is reported -- never as "Go": the image and the GPU box
// have no Go toolchain, so the reference itself cannot run.
//
// Restated, in the reference's own loop order:
//   HasDot / Counter              crdt-misc.go:28-41 (actor == len panics in
//                                  Go: here CRDT_E_ACTOR_RANGE, state dropped)
//   VersionVector.Merge           crdt-misc.go:43-55 (append semantics)
//   AWSet.merge                   awset.go:107-161 (loop over src entries,
//                                  then over dst entries, then the VV merge)
//   AWSetDelta.Merge              awset-delta_test.go:51-65
//   MakeDeltaMergeData            awset-delta_test.go:79-105
//   deltaMerge                    awset-delta_test.go:107-166
// The per-key decision log (fmt.Printf) is left out: it has no effect on the
// state (SURVEY.md 8d excludes it from the baseline).
//
// Keys: interned ids from the SoA batch are turned into strings ("e" + the
// decimal id) before any timing, so the timed merges hash and compare strings
// as the Go maps do.
#include <stdint.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../include/crdtgpu.h"

namespace {

struct Dot {
    uint32_t actor = 0;
    uint64_t counter = 0;
    bool operator==(const Dot& o) const { return actor == o.actor && counter == o.counter; }
};

using Map = std::unordered_map<std::string, Dot>;
using VV = std::vector<uint64_t>;

struct State {
    uint32_t actor = 0;
    VV vv;
    Map entries;
    Map deleted;  // AWSetDelta.Deleted (sources of a delta fold)
};

// crdt-misc.go:28-34
bool has_dot(const VV& vv, const Dot& d, int& err) {
    if (vv.size() < d.actor) return false;
    if (vv.size() == d.actor) {
        err = CRDT_E_ACTOR_RANGE;
        return false;
    }
    return vv[d.actor] >= d.counter;
}

// crdt-misc.go:36-41
uint64_t counter_of(const VV& vv, uint32_t a, int& err) {
    if (vv.size() < a) return 0;
    if (vv.size() == a) {
        err = CRDT_E_ACTOR_RANGE;
        return 0;
    }
    return vv[a];
}

// crdt-misc.go:43-55
void vv_merge(VV& dst, const VV& src) {
    for (size_t i = 0; i < src.size(); ++i) {
        if (i < dst.size()) {
            if (dst[i] < src[i]) dst[i] = src[i];
        } else {
            dst.push_back(src[i]);
        }
    }
}

// awset.go:107-161
void merge(State& dst, const VV& src_vv, const Map& src_entries, int& err) {
    for (const auto& kv : src_entries) {
        auto it = dst.entries.find(kv.first);
        if (it == dst.entries.end()) {
            if (has_dot(dst.vv, kv.second, err)) continue;  // skip
            dst.entries.emplace(kv.first, kv.second);       // add
        } else {
            it->second = kv.second;  // update / keep: the src dot wins
        }
    }
    for (auto it = dst.entries.begin(); it != dst.entries.end();) {
        if (src_entries.count(it->first) == 0 && has_dot(src_vv, it->second, err))
            it = dst.entries.erase(it);  // remove
        else
            ++it;
    }
    vv_merge(dst.vv, src_vv);
}

// awset-delta_test.go:107-166
void delta_merge(State& dst, const VV& src_vv, const Map& changes, const Map& deleted, int& err) {
    for (const auto& kv : changes) {
        auto it = dst.entries.find(kv.first);
        if (it == dst.entries.end()) {
            if (has_dot(dst.vv, kv.second, err)) continue;
            dst.entries.emplace(kv.first, kv.second);
        } else {
            it->second = kv.second;
        }
    }
    for (const auto& kv : deleted) {
        auto it = dst.entries.find(kv.first);
        if (it != dst.entries.end()) {
            if (!has_dot(dst.vv, kv.second, err)) dst.entries.erase(it);
        }
    }
    vv_merge(dst.vv, src_vv);
}

// awset-delta_test.go:51-65 with MakeDeltaMergeData (:79-105) inlined.
void delta_step(State& dst, const State& src, int& err) {
    if (counter_of(dst.vv, src.actor, err) <= 0) {  // full merge, src.Deleted ignored
        merge(dst, src.vv, src.entries, err);
        return;
    }
    Map changed, deleted;
    for (const auto& kv : src.entries)
        if (!has_dot(dst.vv, kv.second, err)) changed.emplace(kv.first, kv.second);
    for (const auto& kv : src.deleted) {
        auto it = src.entries.find(kv.first);
        if (it != src.entries.end() &&
            (it->second.actor != kv.second.actor || it->second.counter > kv.second.counter))
            continue;  // removed and then added again
        deleted.emplace(kv.first, kv.second);
    }
    if (!changed.empty() || !deleted.empty()) delta_merge(dst, src.vv, changed, deleted, err);
    // gcDeleted (:67-77) is empty
}

std::string key_string(uint64_t id) { return "e" + std::to_string(id); }

uint64_t key_id(const std::string& s) { return std::strtoull(s.c_str() + 1, nullptr, 10); }

State state_of(const crdt_awset_batch* b, uint32_t d) {
    State s;
    const uint32_t o = b->offsets[d];
    const uint32_t n = b->counts ? b->counts[d] : b->offsets[d + 1] - o;
    s.vv.assign(b->vv + (size_t)d * b->R, b->vv + (size_t)(d + 1) * b->R);
    s.entries.reserve(n);
    for (uint32_t i = o; i < o + n; ++i) s.entries.emplace(key_string(b->keys[i]), Dot{b->actors[i], b->counters[i]});
    return s;
}

State src_state_of(const crdt_src_batch* s, uint32_t k, bool tombs) {
    State st;
    st.actor = s->src_actor[k];
    st.vv.assign(s->vv + (size_t)k * s->R, s->vv + (size_t)(k + 1) * s->R);
    for (uint32_t i = s->entry_off[k]; i < s->entry_off[k + 1]; ++i)
        st.entries.emplace(key_string(s->keys[i]), Dot{s->actors[i], s->counters[i]});
    if (tombs && s->tomb_off)
        for (uint32_t i = s->tomb_off[k]; i < s->tomb_off[k + 1]; ++i)
            st.deleted.emplace(key_string(s->tkeys[i]), Dot{s->tactors[i], s->tcounters[i]});
    return st;
}

// Writes a state as doc d of an SoA output at slot offset o (entries sorted by key id).
void write_state(const State& s, crdt_awset_out* out, uint32_t d, uint32_t o, uint32_t R) {
    std::vector<std::pair<uint64_t, Dot>> v;
    v.reserve(s.entries.size());
    for (const auto& kv : s.entries) v.emplace_back(key_id(kv.first), kv.second);
    std::sort(v.begin(), v.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
    for (size_t i = 0; i < v.size(); ++i) {
        out->keys[o + i] = v[i].first;
        out->actors[o + i] = v[i].second.actor;
        out->counters[o + i] = v[i].second.counter;
    }
    out->offsets[d] = o;
    out->counts[d] = (uint32_t)v.size();
    for (uint32_t r = 0; r < R; ++r) out->vv[(size_t)d * R + r] = r < s.vv.size() ? s.vv[r] : 0;
}

// Run f(lo, hi) over [0, n) split across `threads` std::threads.
template <typename F>
void parallel(uint32_t n, int threads, F f) {
    if (threads <= 1 || n < 2) {
        f(0u, n);
        return;
    }
    std::vector<std::thread> ts;
    const uint32_t per = (n + threads - 1) / threads;
    for (int t = 0; t < threads; ++t) {
        const uint32_t lo = std::min(n, t * per), hi = std::min(n, lo + per);
        if (lo < hi) ts.emplace_back(f, lo, hi);
    }
    for (auto& t : ts) t.join();
}

double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace

extern "C" {

// out[d] = dst[d] <- src[d] (AWSet.Merge); out capacity as the product's join.
int awmap_join(const crdt_awset_batch* dst, const crdt_awset_batch* src, crdt_awset_out* out) {
    int rc = CRDT_OK;
    for (uint32_t d = 0; d < dst->n_docs; ++d) {
        State s = state_of(dst, d);
        State t = state_of(src, d);
        int err = CRDT_OK;
        merge(s, t.vv, t.entries, err);
        if (err != CRDT_OK) rc = err;
        write_state(s, out, d, dst->offsets[d] + src->offsets[d], dst->R);
    }
    out->offsets[dst->n_docs] = dst->offsets[dst->n_docs] + src->offsets[src->n_docs];
    return rc;
}

// Ordered fold of each doc's sources (mode 0: AWSet.Merge, 1: AWSetDelta.Merge).
int awmap_fold(int mode, const crdt_awset_batch* dst, const crdt_src_batch* srcs, crdt_awset_out* out) {
    int rc = CRDT_OK;
    for (uint32_t d = 0; d < dst->n_docs; ++d) {
        State s = state_of(dst, d);
        int err = CRDT_OK;
        for (uint32_t k = srcs->doc_srcs[d]; k < srcs->doc_srcs[d + 1] && err == CRDT_OK; ++k) {
            State t = src_state_of(srcs, k, mode == CRDT_FOLD_DELTA);
            if (mode == CRDT_FOLD_DELTA)
                delta_step(s, t, err);
            else
                merge(s, t.vv, t.entries, err);
        }
        if (err != CRDT_OK) rc = err;
        write_state(s, out, d, dst->offsets[d] + srcs->entry_off[srcs->doc_srcs[d]], dst->R);
    }
    const uint32_t ns = srcs->doc_srcs[srcs->n_docs];
    out->offsets[dst->n_docs] = dst->offsets[dst->n_docs] + srcs->entry_off[ns];
    return rc;
}

// CPU baseline, full-state join: per pass, every doc's dst map is cloned
// (untimed, AWSet.Clone) and merged (timed): a <- b, and b <- a too when
// both_dirs.  Passes repeat until the timed merges reach budget_s.  Returns
// the timed seconds; *merges = merges done in them.
double awmap_bench_join(const crdt_awset_batch* a, const crdt_awset_batch* b, int both_dirs, int threads,
                        double budget_s, uint64_t* merges) {
    const uint32_t n = a->n_docs;
    std::vector<State> A(n), B(n), WA(n), WB(n);
    parallel(n, threads, [&](uint32_t lo, uint32_t hi) {
        for (uint32_t d = lo; d < hi; ++d) {
            A[d] = state_of(a, d);
            B[d] = state_of(b, d);
        }
    });
    std::atomic<int> err{0};
    double timed = 0;
    uint64_t m = 0;
    while (timed < budget_s) {
        parallel(n, threads, [&](uint32_t lo, uint32_t hi) {
            for (uint32_t d = lo; d < hi; ++d) {
                WA[d] = A[d];
                if (both_dirs) WB[d] = B[d];
            }
        });
        const double t0 = now_s();
        parallel(n, threads, [&](uint32_t lo, uint32_t hi) {
            int e = 0;
            for (uint32_t d = lo; d < hi; ++d) {
                merge(WA[d], B[d].vv, B[d].entries, e);
                if (both_dirs) merge(WB[d], A[d].vv, A[d].entries, e);
            }
            if (e) err = e;
        });
        timed += now_s() - t0;
        m += (uint64_t)n * (both_dirs ? 2 : 1);
    }
    *merges = m;
    return err ? -1.0 : timed;
}

// CPU baseline, ordered fold (mode as awmap_fold): per pass the dst maps are
// cloned (untimed) and every doc's sources folded in order (timed).
double awmap_bench_fold(int mode, const crdt_awset_batch* dst, const crdt_src_batch* srcs, int threads,
                        double budget_s, uint64_t* merges) {
    const uint32_t n = dst->n_docs;
    const uint32_t ns = srcs->doc_srcs[n] - srcs->doc_srcs[0];
    std::vector<State> D(n), W(n), S(srcs->doc_srcs[n]);
    parallel(n, threads, [&](uint32_t lo, uint32_t hi) {
        for (uint32_t d = lo; d < hi; ++d) {
            D[d] = state_of(dst, d);
            for (uint32_t k = srcs->doc_srcs[d]; k < srcs->doc_srcs[d + 1]; ++k)
                S[k] = src_state_of(srcs, k, mode == CRDT_FOLD_DELTA);
        }
    });
    std::atomic<int> err{0};
    double timed = 0;
    uint64_t m = 0;
    while (timed < budget_s) {
        parallel(n, threads, [&](uint32_t lo, uint32_t hi) {
            for (uint32_t d = lo; d < hi; ++d) W[d] = D[d];
        });
        const double t0 = now_s();
        parallel(n, threads, [&](uint32_t lo, uint32_t hi) {
            int e = 0;
            for (uint32_t d = lo; d < hi; ++d)
                for (uint32_t k = srcs->doc_srcs[d]; k < srcs->doc_srcs[d + 1]; ++k) {
                    if (mode == CRDT_FOLD_DELTA)
                        delta_step(W[d], S[k], e);
                    else
                        merge(W[d], S[k].vv, S[k].entries, e);
                }
            if (e) err = e;
        });
        timed += now_s() - t0;
        m += ns;
    }
    *merges = m;
    return err ? -1.0 : timed;
}

}  // extern "C"
