// crdt.hpp -- C++ host mirror of the reference's Go API, merging on the GPU.
//
// Same types and method names as package crdt (rsms/go-crdt-playground):
//   Actor, Dot                        crdt-misc.go:8-19
//   VersionVector                     crdt-misc.go:21-74
//   AWSet                             awset.go:55-171
//   AWSetDelta                        awset-delta_test.go:9-77
// Merge() and the batch entry points (MergeBatch, FoldBatch, DeltaMergeBatch)
// intern the string keys of each document into order-preserving u64 ids (the
// ranks of the document's keys; host work spread over threads), pack the
// structure-of-arrays buffers of include/crdtgpu.h, run the HIP kernels through
// crdt_awset_join_batch / crdt_awset_fold_batch and unpack the result.  Local
// ops (Add, Del, Clone, ...) are per-replica host state, as in the reference.
//
// Where the Go code panics (HasDot/Counter at actor == len(vv), Add with the
// actor outside the vector), this API throws crdt::Error carrying the C ABI
// code (CRDT_E_ACTOR_RANGE); a failed merge leaves its destinations untouched.
// Version vectors of one batch are zero-padded to one width R (<= 64).  A
// document with a vector shorter than R is replayed on the host before the
// launch (detail::replay_checks: every HasDot / Counter call of the reference
// on the unpadded vectors), so Go's panic at actor == len(vv) is found exactly;
// R is chosen clear of such documents' actors (the kernels flag actor == R).
// A counter-0 dot between a shorter vector's end and R (unreachable: Add bumps
// first) is refused with CRDT_E_INVALID: the zero pad cannot express it.
#pragma once

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <map>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/crdtgpu.h"

namespace crdt {

using Actor = uint32_t;  // crdt-misc.go:9 (uint; the engine stores u32 actors)

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string& what) : std::runtime_error(what + ": " + crdt_strerror(c)), code(c) {}
};

inline void check(int rc, const char* what) {
    if (rc != CRDT_OK) throw Error(rc, what);
}

// crdt-misc.go:12-19
struct Dot {
    Actor actor = 0;
    uint64_t counter = 0;
    bool operator==(const Dot& o) const { return actor == o.actor && counter == o.counter; }
    bool operator!=(const Dot& o) const { return !(*this == o); }
    std::string String() const { return "(" + std::string(1, char('A' + actor)) + " " + std::to_string(counter) + ")"; }
};

// crdt-misc.go:23-74
struct VersionVector : std::vector<uint64_t> {
    using std::vector<uint64_t>::vector;
    bool HasDot(const Dot& d) const {  // crdt-misc.go:28-34
        if (size() < d.actor) return false;
        if (d.actor == size()) throw Error(CRDT_E_ACTOR_RANGE, "HasDot");
        return (*this)[d.actor] >= d.counter;
    }
    uint64_t Counter(Actor a) const {  // crdt-misc.go:36-41
        if (size() < a) return 0;
        if (a == size()) throw Error(CRDT_E_ACTOR_RANGE, "Counter");
        return (*this)[a];
    }
    void Merge(const VersionVector& src) {  // crdt-misc.go:43-55
        for (size_t i = 0; i < src.size(); ++i) {
            if (i < size()) {
                if ((*this)[i] < src[i]) (*this)[i] = src[i];
            } else {
                push_back(src[i]);
            }
        }
    }
    VersionVector Clone() const { return *this; }
    std::string String() const {  // crdt-misc.go:57-68
        std::string s = "[";
        for (size_t i = 0; i < size(); ++i) {
            if (i) s += ", ";
            s += "(" + std::string(1, char('A' + i)) + " " + std::to_string((*this)[i]) + ")";
        }
        return s + "]";
    }
};

using Entries = std::unordered_map<std::string, Dot>;

// One context per host thread (crdt_ctx).
class Engine {
   public:
    explicit Engine(int device = 0) { check(crdt_ctx_create(device, &ctx_), "crdt_ctx_create"); }
    ~Engine() { crdt_ctx_destroy(ctx_); }
    Engine(const Engine&) = delete;
    Engine& operator=(const Engine&) = delete;
    crdt_ctx* ctx() const { return ctx_; }
    static Engine& Default() {
        static thread_local Engine e(0);
        return e;
    }

   private:
    crdt_ctx* ctx_ = nullptr;
};

class AWSetDelta;

// awset.go:55-59
class AWSet {
   public:
    Actor actor = 0;
    VersionVector versionVector;
    Entries entries;

    AWSet() = default;
    AWSet(Actor a, VersionVector vv) : actor(a), versionVector(std::move(vv)) {}
    virtual ~AWSet() = default;

    std::vector<std::string> SortedValues() const {  // awset.go:61-70
        std::vector<std::string> v;
        v.reserve(entries.size());
        for (auto& kv : entries) v.push_back(kv.first);
        std::sort(v.begin(), v.end());
        return v;
    }
    void Reset() {  // awset.go:72-75
        versionVector = VersionVector{0};
        entries.clear();
    }
    AWSet Clone() const { return *this; }                                     // awset.go:77-85
    bool Has(const std::string& k) const { return entries.count(k) != 0; }    // awset.go:87
    void Add(std::initializer_list<std::string> keys) {                       // awset.go:89-94
        for (auto& k : keys) {
            if (actor >= versionVector.size()) throw Error(CRDT_E_ACTOR_RANGE, "Add");
            versionVector[actor]++;
            entries[k] = Dot{actor, versionVector[actor]};
        }
    }
    void Del(std::initializer_list<std::string> keys) {  // awset.go:96-101 (no clock bump)
        for (auto& k : keys) entries.erase(k);
    }
    void Merge(const AWSet& src, Engine& e = Engine::Default());  // awset.go:103-105, on the GPU
    std::string String() const {                                    // awset.go:163-171
        std::string s = versionVector.String();
        for (auto& v : SortedValues()) s += "\n  " + entries.at(v).String() + "  \"" + v + "\"";
        return s;
    }
    virtual const Entries* deleted_map() const { return nullptr; }
};

// awset-delta_test.go:9-12
class AWSetDelta : public AWSet {
   public:
    Entries deleted;

    AWSetDelta() = default;
    AWSetDelta(Actor a, VersionVector vv) : AWSet(a, std::move(vv)) {}
    void Del(std::initializer_list<std::string> keys) {  // awset-delta_test.go:14-33
        if (actor >= versionVector.size()) throw Error(CRDT_E_ACTOR_RANGE, "Del");
        versionVector[actor]++;
        const Dot dot2{actor, versionVector[actor]};
        for (auto& k : keys) {
            auto it = entries.find(k);
            if (it != entries.end()) {
                deleted[k] = dot2;
                entries.erase(it);
            }
        }
    }
    AWSetDelta Clone() const { return *this; }                        // awset-delta_test.go:35-49
    void Merge(const AWSetDelta& src, Engine& e = Engine::Default());  // awset-delta_test.go:51-65, on the GPU
    void gcDeleted(const VersionVector&) {}                            // awset-delta_test.go:67-77: empty
    const Entries* deleted_map() const override { return &deleted; }
};

namespace detail {

struct Packed {
    std::vector<uint32_t> offsets{0};
    std::vector<uint64_t> keys;
    std::vector<uint32_t> actors;
    std::vector<uint64_t> counters;
    std::vector<uint64_t> vv;
};

template <typename T>
T* data_or_null(std::vector<T>& v) {
    return v.empty() ? nullptr : v.data();
}

// Worker threads for the per-document host work (interning, packing,
// unpacking): CRDT_HOST_THREADS, else OMP_NUM_THREADS, else the hardware
// threads (at most 16); 1 = serial.
inline unsigned host_threads() {
    static const unsigned n = [] {
        for (const char* name : {"CRDT_HOST_THREADS", "OMP_NUM_THREADS"}) {
            const char* e = std::getenv(name);
            const long v = e ? std::strtol(e, nullptr, 10) : 0;
            if (v > 0) return (unsigned)std::min(v, 256L);
        }
        return std::min(std::max(1u, std::thread::hardware_concurrency()), 16u);
    }();
    return n;
}

template <typename F>
void parallel_docs(size_t n, F&& fn) {
    const unsigned t = (unsigned)std::min<size_t>(host_threads(), std::max<size_t>(1, n / 256));
    if (t <= 1) {
        fn(0, n);
        return;
    }
    std::vector<std::thread> pool;
    const size_t chunk = (n + t - 1) / t;
    for (unsigned i = 0; i < t; ++i) {
        const size_t lo = i * chunk, hi = std::min(n, lo + chunk);
        if (lo < hi) pool.emplace_back([&fn, lo, hi] { fn(lo, hi); });
    }
    for (auto& th : pool) th.join();
}

// Interning + packing shared by the batch entry points.  Keys are interned
// per document: the merge only ever compares keys of one document, so a
// document's ids are the ranks of its keys (over every state of that document
// in the batch) in string order -- an exact, order-preserving bijection per
// document, as the C ABI requires, built from a small sort per document.
struct Batch {
    size_t R = 1;
    std::vector<std::vector<const std::string*>> names;  // doc -> id -> key

    // doc d's states: every key of each (entries and Deleted) becomes an id
    void intern(size_t d, const std::vector<const AWSet*>& states) {
        auto& v = names[d];
        v.clear();
        for (auto* s : states) {
            for (auto& kv : s->entries) v.push_back(&kv.first);
            if (auto* del = s->deleted_map())
                for (auto& kv : *del) v.push_back(&kv.first);
        }
        std::sort(v.begin(), v.end(), [](const std::string* a, const std::string* b) { return *a < *b; });
        v.erase(std::unique(v.begin(), v.end(), [](const std::string* a, const std::string* b) { return *a == *b; }),
                v.end());
    }
    uint64_t id(size_t d, const std::string& k) const {
        const auto& v = names[d];
        return (uint64_t)(std::lower_bound(v.begin(), v.end(), &k,
                                           [](const std::string* a, const std::string* b) { return *a < *b; }) -
                          v.begin());
    }
    // write map m of doc d at k/a/c[at..], sorted by id
    void put_entries(size_t d, const Entries& m, uint64_t* k, uint32_t* a, uint64_t* c) const {
        std::vector<std::pair<uint64_t, Dot>> v;
        v.reserve(m.size());
        for (auto& kv : m) v.emplace_back(id(d, kv.first), kv.second);
        std::sort(v.begin(), v.end(), [](auto& x, auto& y) { return x.first < y.first; });
        for (size_t i = 0; i < v.size(); ++i) {
            k[i] = v[i].first;
            a[i] = v[i].second.actor;
            c[i] = v[i].second.counter;
        }
    }
    // one state per doc (states[d] of doc d), offsets = prefix of entry counts
    Packed pack(const std::vector<AWSet*>& states) const {
        Packed p;
        const size_t n = states.size();
        p.offsets.assign(n + 1, 0);
        for (size_t d = 0; d < n; ++d) p.offsets[d + 1] = p.offsets[d] + (uint32_t)states[d]->entries.size();
        const size_t tot = p.offsets[n];
        p.keys.resize(tot);
        p.actors.resize(tot);
        p.counters.resize(tot);
        p.vv.assign(n * R, 0);
        parallel_docs(n, [&](size_t lo, size_t hi) {
            for (size_t d = lo; d < hi; ++d) {
                const uint32_t o = p.offsets[d];
                put_entries(d, states[d]->entries, p.keys.data() + o, p.actors.data() + o, p.counters.data() + o);
                const auto& v = states[d]->versionVector;
                for (size_t r = 0; r < std::min(R, v.size()); ++r) p.vv[d * R + r] = v[r];
            }
        });
        return p;
    }
    crdt_awset_batch view(Packed& p) const {
        return crdt_awset_batch{(uint32_t)(p.offsets.size() - 1), (uint32_t)R, p.offsets.data(), nullptr,
                                data_or_null(p.keys), data_or_null(p.actors), data_or_null(p.counters),
                                data_or_null(p.vv)};
    }
    void unpack(const std::vector<AWSet*>& dsts, const Packed& out, const std::vector<uint32_t>& counts,
                const std::vector<size_t>& widths) const {
        parallel_docs(dsts.size(), [&](size_t lo, size_t hi) {
            for (size_t d = lo; d < hi; ++d) {
                Entries m;
                m.reserve(counts[d]);
                for (uint32_t j = out.offsets[d]; j < out.offsets[d] + counts[d]; ++j)
                    m.emplace(*names[d][out.keys[j]], Dot{out.actors[j], out.counters[j]});
                dsts[d]->entries = std::move(m);
                VersionVector vv(widths[d]);
                for (size_t r = 0; r < widths[d]; ++r) vv[r] = out.vv[d * R + r];
                dsts[d]->versionVector = std::move(vv);
            }
        });
    }
};

inline Packed make_out(size_t n_docs, size_t R, size_t slots, std::vector<uint32_t>& counts, crdt_awset_out& o) {
    Packed p;
    p.offsets.assign(n_docs + 1, 0);
    p.keys.assign(slots + 1, 0);
    p.actors.assign(slots + 1, 0);
    p.counters.assign(slots + 1, 0);
    p.vv.assign(std::max<size_t>(n_docs * R, 1), 0);
    counts.assign(std::max<size_t>(n_docs, 1), 0);
    o = crdt_awset_out{p.offsets.data(), counts.data(), p.keys.data(), p.actors.data(), p.counters.data(), p.vv.data()};
    return p;
}

// Intern a batch: doc d's states are states_of(d).
template <typename F>
void intern_all(Batch& b, size_t n, F&& states_of) {
    b.names.assign(n, {});
    parallel_docs(n, [&](size_t lo, size_t hi) {
        for (size_t d = lo; d < hi; ++d) b.intern(d, states_of(d));
    });
}

}  // namespace detail

namespace detail {
struct GoPanic {};

// HasDot / Counter as Go evaluates them on the unpadded vectors
// (crdt-misc.go:28-41), noting where the zero-padded width R answers
// differently (a counter-0 dot at len(vv) < actor < R).
struct Checks {
    size_t R;
    bool pad_differs = false;
    bool has(const std::vector<uint64_t>& vv, const Dot& d) {
        const size_t n = vv.size();
        if (n < d.actor) {
            if (d.actor < R && d.counter == 0) pad_differs = true;
            return false;
        }
        if (d.actor == n) throw GoPanic{};
        return vv[d.actor] >= d.counter;
    }
    static uint64_t counter(const std::vector<uint64_t>& vv, Actor a) {
        if (vv.size() < a) return 0;
        if (a == vv.size()) throw GoPanic{};
        return vv[a];
    }
};

enum { kReplayOk = 0, kReplayPanic = 1, kReplayPad = 2 };

// Replay dst.Merge(src) for src in srcs, in order, on maps with the
// reference's rules -- (*AWSet).merge awset.go:107-161, (*AWSetDelta).Merge
// awset-delta_test.go:51-65, MakeDeltaMergeData :79-105, deltaMerge :107-166
// -- only to find whether Go panics or the padded layout would differ.
// Whether Go panics does not depend on its random map order.
inline int replay_checks(int mode, const AWSet& dst, const std::vector<const AWSet*>& srcs, size_t R) {
    Checks ck{R};
    std::vector<uint64_t> V(dst.versionVector.begin(), dst.versionVector.end());
    Entries E = dst.entries;
    try {
        for (const AWSet* s : srcs) {
            const bool full = mode != CRDT_FOLD_DELTA || Checks::counter(V, s->actor) == 0;
            Entries changed, dele;
            if (!full) {
                for (auto& kv : s->entries)
                    if (!ck.has(V, kv.second)) changed.emplace(kv.first, kv.second);
                if (auto* del = s->deleted_map())
                    for (auto& kv : *del) {
                        auto it = s->entries.find(kv.first);
                        if (it == s->entries.end() ||
                            !(it->second.actor != kv.second.actor || it->second.counter > kv.second.counter))
                            dele.emplace(kv.first, kv.second);
                    }
                if (changed.empty() && dele.empty()) continue;  // awset-delta_test.go:60: nothing, not even the VV
            }
            for (auto& kv : full ? s->entries : changed)
                if (E.count(kv.first) || !ck.has(V, kv.second)) E[kv.first] = kv.second;
            if (full) {
                for (auto it = E.begin(); it != E.end();) {
                    if (!s->entries.count(it->first) && ck.has(s->versionVector, it->second))
                        it = E.erase(it);
                    else
                        ++it;
                }
            } else {
                for (auto& kv : dele) {
                    auto it = E.find(kv.first);
                    if (it != E.end() && !ck.has(V, kv.second)) E.erase(it);
                }
            }
            const auto& sv = s->versionVector;
            for (size_t i = 0; i < sv.size(); ++i) {
                if (i < V.size())
                    V[i] = std::max<uint64_t>(V[i], sv[i]);
                else
                    V.push_back(sv[i]);
            }
        }
    } catch (const GoPanic&) {
        return kReplayPanic;
    }
    return ck.pad_differs ? kReplayPad : kReplayOk;
}

// The padded width R of a batch whose document d holds states_of(d) (dst
// first), after the host checks of its documents with a vector shorter than R.
template <typename F>
size_t ragged_checks(int mode, size_t n_docs, F&& states_of, const char* what) {
    size_t R = 1;
    for (size_t d = 0; d < n_docs; ++d)
        for (const AWSet* s : states_of(d)) R = std::max(R, s->versionVector.size());
    if (R > CRDT_MAX_R) throw Error(CRDT_E_INVALID, "version vector longer than CRDT_MAX_R");
    auto is_short = [](const std::vector<const AWSet*>& doc, size_t w) {
        for (const AWSet* s : doc)
            if (s->versionVector.size() < w) return true;
        return false;
    };
    auto has_actor = [mode](const std::vector<const AWSet*>& doc, size_t w) {
        for (size_t i = 0; i < doc.size(); ++i) {
            if (i && mode == CRDT_FOLD_DELTA && doc[i]->actor == w) return true;
            for (auto& kv : doc[i]->entries)
                if (kv.second.actor == w) return true;
            if (auto* del = doc[i]->deleted_map())
                for (auto& kv : *del)
                    if (kv.second.actor == w) return true;
        }
        return false;
    };
    size_t w = R;
    for (;; ++w) {
        if (w > CRDT_MAX_R) throw Error(CRDT_E_INVALID, std::string(what) + ": every padded width collides with an actor");
        bool clash = false;
        for (size_t d = 0; d < n_docs && !clash; ++d) {
            const auto doc = states_of(d);
            clash = is_short(doc, w) && has_actor(doc, w);
        }
        if (!clash) break;
    }
    for (size_t d = 0; d < n_docs; ++d) {
        const auto doc = states_of(d);
        if (!is_short(doc, w)) continue;
        const int r = replay_checks(mode, *doc[0], std::vector<const AWSet*>(doc.begin() + 1, doc.end()), w);
        if (r == kReplayPanic) throw Error(CRDT_E_ACTOR_RANGE, std::string(what) + ": HasDot/Counter at actor == len(vv)");
        if (r == kReplayPad) throw Error(CRDT_E_INVALID, std::string(what) + ": counter-0 dot beyond a shorter version vector");
    }
    return w;
}
}  // namespace detail

// dsts[i].Merge(*srcs[i]) for every i, as one batched GPU join.
inline void MergeBatch(const std::vector<AWSet*>& dsts, const std::vector<const AWSet*>& srcs,
                       Engine& e = Engine::Default()) {
    if (dsts.size() != srcs.size()) throw Error(CRDT_E_INVALID, "MergeBatch: length mismatch");
    if (dsts.empty()) return;
    detail::Batch b;
    b.R = detail::ragged_checks(
        CRDT_FOLD_AWSET, dsts.size(), [&](size_t d) { return std::vector<const AWSet*>{dsts[d], srcs[d]}; },
        "MergeBatch");
    detail::intern_all(b, dsts.size(), [&](size_t d) { return std::vector<const AWSet*>{dsts[d], srcs[d]}; });
    std::vector<AWSet*> sv;
    for (auto* s : srcs) sv.push_back(const_cast<AWSet*>(s));
    detail::Packed pd = b.pack(dsts), ps = b.pack(sv);
    crdt_awset_batch cd = b.view(pd), cs = b.view(ps);
    std::vector<uint32_t> counts;
    crdt_awset_out co;
    detail::Packed po = detail::make_out(dsts.size(), b.R, pd.keys.size() + ps.keys.size(), counts, co);
    check(crdt_awset_join_batch(e.ctx(), &cd, &cs, &co), "crdt_awset_join_batch");
    std::vector<size_t> widths;
    for (size_t i = 0; i < dsts.size(); ++i)
        widths.push_back(std::max(dsts[i]->versionVector.size(), srcs[i]->versionVector.size()));
    b.unpack(dsts, po, counts, widths);
}

namespace detail {
// len(dst.versionVector) after the fold, replayed on the VVs alone: a delta
// step that brings nothing (awset-delta_test.go:60) skips VersionVector.Merge.
// A step merges iff Counter(src.Actor) == 0 (:53) or MakeDeltaMergeData finds
// a changed entry or an effective tombstone (:79-105).
inline size_t fold_width(int mode, const AWSet& dst, const std::vector<const AWSet*>& srcs) {
    size_t n = dst.versionVector.size();
    if (mode != CRDT_FOLD_DELTA) {
        for (auto* s : srcs) n = std::max(n, s->versionVector.size());
        return n;
    }
    std::vector<uint64_t> V(dst.versionVector.begin(), dst.versionVector.end());
    for (auto* s : srcs) {
        if ((s->actor < V.size() ? V[s->actor] : 0) != 0) {
            bool any = false;
            for (auto& kv : s->entries)
                if (!(kv.second.actor < V.size() && V[kv.second.actor] >= kv.second.counter)) any = true;
            if (auto* del = s->deleted_map())
                for (auto& kv : *del) {
                    auto it = s->entries.find(kv.first);
                    if (!(it != s->entries.end() &&
                          (it->second.actor != kv.second.actor || it->second.counter > kv.second.counter)))
                        any = true;
                }
            if (!any) continue;
        }
        const auto& sv = s->versionVector;
        for (size_t i = 0; i < sv.size(); ++i) {
            if (i < V.size())
                V[i] = std::max(V[i], sv[i]);
            else
                V.push_back(sv[i]);
        }
    }
    return V.size();
}

inline void fold(int mode, const std::vector<AWSet*>& dsts, const std::vector<std::vector<const AWSet*>>& srcs,
                 Engine& e) {
    if (dsts.size() != srcs.size()) throw Error(CRDT_E_INVALID, "fold: length mismatch");
    if (dsts.empty()) return;
    Batch b;
    b.R = ragged_checks(
        mode, dsts.size(),
        [&](size_t d) {
            std::vector<const AWSet*> v{dsts[d]};
            v.insert(v.end(), srcs[d].begin(), srcs[d].end());
            return v;
        },
        mode == CRDT_FOLD_DELTA ? "DeltaMergeBatch" : "FoldBatch");
    intern_all(b, dsts.size(), [&](size_t d) {
        std::vector<const AWSet*> v{dsts[d]};
        v.insert(v.end(), srcs[d].begin(), srcs[d].end());
        return v;
    });
    Packed pd = b.pack(dsts);
    std::vector<uint32_t> doc_srcs{0}, src_actor, entry_off{0}, tomb_off{0};
    std::vector<uint64_t> vv, keys, counters, tkeys, tcounters;
    std::vector<uint32_t> actors, tactors;
    for (size_t d = 0; d < srcs.size(); ++d) {
        for (auto* s : srcs[d]) {
            src_actor.push_back(s->actor);
            for (size_t r = 0; r < b.R; ++r) vv.push_back(r < s->versionVector.size() ? s->versionVector[r] : 0);
            const size_t o = keys.size(), m = s->entries.size();
            keys.resize(o + m);
            actors.resize(o + m);
            counters.resize(o + m);
            b.put_entries(d, s->entries, keys.data() + o, actors.data() + o, counters.data() + o);
            entry_off.push_back((uint32_t)keys.size());
            if (auto* del = s->deleted_map()) {
                const size_t t = tkeys.size(), x = del->size();
                tkeys.resize(t + x);
                tactors.resize(t + x);
                tcounters.resize(t + x);
                b.put_entries(d, *del, tkeys.data() + t, tactors.data() + t, tcounters.data() + t);
            }
            tomb_off.push_back((uint32_t)tkeys.size());
        }
        doc_srcs.push_back((uint32_t)src_actor.size());
    }
    crdt_awset_batch cd = b.view(pd);
    const bool tombs = !tkeys.empty();  // no tombstones at all: tomb_off = NULL
    crdt_src_batch cs{(uint32_t)dsts.size(), (uint32_t)b.R, doc_srcs.data(), data_or_null(src_actor),
                      data_or_null(vv), entry_off.data(), data_or_null(keys), data_or_null(actors),
                      data_or_null(counters), tombs ? tomb_off.data() : nullptr, data_or_null(tkeys),
                      data_or_null(tactors), data_or_null(tcounters)};
    std::vector<uint32_t> counts;
    crdt_awset_out co;
    Packed po = make_out(dsts.size(), b.R, pd.keys.size() + keys.size(), counts, co);
    check(crdt_awset_fold_batch(e.ctx(), mode, &cd, &cs, &co), "crdt_awset_fold_batch");
    std::vector<size_t> widths;
    for (size_t i = 0; i < dsts.size(); ++i) widths.push_back(fold_width(mode, *dsts[i], srcs[i]));
    b.unpack(dsts, po, counts, widths);
}
}  // namespace detail

// for each i, for src in srcs[i] in order: dsts[i]->Merge(*src)  (AWSet semantics)
inline void FoldBatch(const std::vector<AWSet*>& dsts, const std::vector<std::vector<const AWSet*>>& srcs,
                      Engine& e = Engine::Default()) {
    detail::fold(CRDT_FOLD_AWSET, dsts, srcs, e);
}

// for each i, for src in srcs[i] in order: dsts[i]->Merge(*src)  (AWSetDelta semantics)
inline void DeltaMergeBatch(const std::vector<AWSetDelta*>& dsts,
                            const std::vector<std::vector<const AWSetDelta*>>& srcs, Engine& e = Engine::Default()) {
    std::vector<AWSet*> d(dsts.begin(), dsts.end());
    std::vector<std::vector<const AWSet*>> s;
    for (auto& l : srcs) s.emplace_back(l.begin(), l.end());
    detail::fold(CRDT_FOLD_DELTA, d, s, e);
}

inline void AWSet::Merge(const AWSet& src, Engine& e) { MergeBatch({this}, {&src}, e); }
inline void AWSetDelta::Merge(const AWSetDelta& src, Engine& e) { DeltaMergeBatch({this}, {{&src}}, e); }

}  // namespace crdt
