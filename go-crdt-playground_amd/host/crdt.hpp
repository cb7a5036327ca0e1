// crdt.hpp -- C++ host mirror of the reference's Go API, merging on the GPU.
//
// Same types and method names as package crdt (rsms/go-crdt-playground):
//   Actor, Dot                        crdt-misc.go:8-19
//   VersionVector                     crdt-misc.go:21-74
//   AWSet                             awset.go:55-171
//   AWSetDelta                        awset-delta_test.go:9-77
// Merge() and the batch entry points (MergeBatch, ExchangeBatch, FoldBatch,
// DeltaMergeBatch) move map[string]Dot-shaped states through the C ABI
// (include/crdtgpu.h) and back, per document on host threads:
//   intern  each key -> a 64-bit hash id; a document whose states hold two
//           different keys with one id (checked exactly, by string compare on
//           equal ids) falls back to rank ids (its keys' ranks in string
//           order), so ids are always an exact bijection per document
//   pack    entries sorted by id straight into page-locked SoA arrays
//           (crdt_host_alloc, kept by the Engine and reused across calls)
//   merge   crdt_awset_join_batch / _exchange_batch / _fold_batch
//   apply   the result applied to each destination map IN PLACE, as the
//           reference's merge mutates dst.Entries (awset.go:142,154): removed
//           keys erased, changed dots overwritten, new keys inserted -- no
//           map is rebuilt
// Local ops (Add, Del, Clone, ...) are per-replica host state, as in the
// reference.
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
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

namespace detail {
// Page-locked host buffer (crdt_host_alloc), grown on demand, kept for reuse:
// allocating page-locked memory costs far more than filling it.
struct PinnedBuf {
    void* p = nullptr;
    size_t bytes = 0;
    PinnedBuf() = default;
    PinnedBuf(const PinnedBuf&) = delete;
    PinnedBuf& operator=(const PinnedBuf&) = delete;
    ~PinnedBuf() { crdt_host_free(p); }
    void* get(size_t want) {
        want = std::max<size_t>(want, 64);
        if (want > bytes) {
            crdt_host_free(p);
            p = nullptr;
            bytes = 0;
            want += want / 8;
            check(crdt_host_alloc(want, &p), "crdt_host_alloc");
            bytes = want;
        }
        return p;
    }
};

// staging roles of one batch call
enum Pin {
    kD_OFF, kD_KEY, kD_ACT, kD_CTR, kD_VV,        // destinations
    kS_OFF, kS_KEY, kS_ACT, kS_CTR, kS_VV,        // sources (join / exchange: one per doc)
    kS_DOC, kS_SACT, kS_TOFF, kS_TKEY, kS_TACT, kS_TCTR,  // fold sources: doc_srcs, src_actor, tombstones
    kO_OFF, kO_CNT, kO_KEY, kO_ACT, kO_CTR, kO_VV,  // output
    kP_OFF, kP_CNT, kP_KEY, kP_ACT, kP_CTR, kP_VV,  // second output (exchange)
    kPinSlots
};
}  // namespace detail

namespace detail {
struct Batch;
}

// One context per host thread (crdt_ctx), plus the page-locked staging and
// the host scratch its batch calls reuse (nothing large is allocated or freed
// per call).
class Engine {
   public:
    explicit Engine(int device = 0);
    ~Engine();
    Engine(const Engine&) = delete;
    Engine& operator=(const Engine&) = delete;
    crdt_ctx* ctx() const { return ctx_; }
    static Engine& Default() {
        static thread_local Engine e(0);
        return e;
    }
    template <typename T>
    T* pinned(int role, size_t n) {
        if (carved_[role] && n * sizeof(T) <= carved_n_[role]) return static_cast<T*>(carved_[role]);
        return static_cast<T*>(pin_[role].get(n * sizeof(T)));
    }
    // Place the given roles' arrays in ONE page-locked block (256-byte aligned
    // sub-arrays): the C ABI stages arrays that lie in one crdt_host_alloc
    // block with a single copy (api.cpp, Stager::flush) instead of one runtime
    // copy call each.  Replaces the previous call's carving.
    void carve(std::initializer_list<std::pair<int, size_t>> roles) {
        for (auto& c : carved_) c = nullptr;
        size_t total = 0;
        for (const auto& r : roles) total += (r.second + 255) & ~(size_t)255;
        char* base = static_cast<char*>(arena_.get(total));
        size_t off = 0;
        for (const auto& r : roles) {
            carved_[r.first] = base + off;
            carved_n_[r.first] = r.second;
            off += (r.second + 255) & ~(size_t)255;
        }
    }
    // host arrays of map iterators per slot (0: destinations, 1: sources),
    // grown on demand and reused: no per-call allocation or first touch
    Entries::iterator* iters(int role, size_t n) {
        if (its_[role].size() < n) its_[role].resize(n + n / 8);
        return its_[role].data();
    }

    detail::Batch& batch() { return *batch_; }

   private:
    crdt_ctx* ctx_ = nullptr;
    detail::PinnedBuf pin_[detail::kPinSlots];
    detail::PinnedBuf arena_;  // the carved input block
    void* carved_[detail::kPinSlots] = {};
    size_t carved_n_[detail::kPinSlots] = {};
    std::vector<Entries::iterator> its_[2];
    detail::Batch* batch_ = nullptr;
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

// Seconds per phase of the last batch call on this thread (boundary cost).
struct BoundaryStats {
    double pack_s = 0, device_s = 0, apply_s = 0, call_s = 0;
    // inside pack_s: the batch's checks (join_batch), the layout (slot offsets),
    // the per-document packing; inside apply_s: the distinct-states check
    double batch_s = 0, layout_s = 0, docs_s = 0, distinct_s = 0;
    size_t rank_docs = 0;  // documents interned by rank after a hash collision
};
inline BoundaryStats& LastStats() {
    static thread_local BoundaryStats s;
    return s;
}

namespace detail {

using clk = std::chrono::steady_clock;
inline double secs_since(clk::time_point t) { return std::chrono::duration<double>(clk::now() - t).count(); }

// Worker threads for the per-document host work (interning, packing,
// applying): CRDT_HOST_THREADS, else OMP_NUM_THREADS, else the hardware
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

// The worker threads, started once and kept, with their scratch (thread_local
// below): a steady stream of batch calls then starts no thread and allocates
// almost nothing on the host.  Threads started and joined per phase cost the
// 65,536-document pack ~20 ms (34 -> 13-16 ms with kept threads,
// profiles/r06n_boundary_malloc_arenas.log vs profiles/r06r_boundary_calls_*.log).
class WorkerPool {
   public:
    explicit WorkerPool(unsigned n) {
        for (unsigned i = 0; i < n; ++i) th_.emplace_back([this, i] { loop(i); });
    }
    ~WorkerPool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    unsigned size() const { return (unsigned)th_.size(); }
    // run(i) for i in [0, jobs) -- job 0 on the calling thread, job i on worker i - 1
    // (callers on several threads take turns; jobs <= size() + 1)
    void run(unsigned jobs, const std::function<void(unsigned)>& f) {
        std::lock_guard<std::mutex> turn(run_mu_);
        {
            std::lock_guard<std::mutex> lk(mu_);
            job_ = &f;
            jobs_ = jobs;
            left_ = jobs - 1;
            ++round_;
        }
        cv_.notify_all();
        f(0);
        std::unique_lock<std::mutex> lk(mu_);
        done_.wait(lk, [this] { return left_ == 0; });
        job_ = nullptr;
    }

   private:
    void loop(unsigned i) {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(unsigned)>* f = nullptr;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || round_ != seen; });
                if (stop_) return;
                seen = round_;
                if (i + 1 >= jobs_) continue;
                f = job_;
            }
            (*f)(i + 1);
            std::lock_guard<std::mutex> lk(mu_);
            if (--left_ == 0) done_.notify_one();
        }
    }
    std::vector<std::thread> th_;
    std::mutex run_mu_, mu_;
    std::condition_variable cv_, done_;
    const std::function<void(unsigned)>* job_ = nullptr;
    unsigned jobs_ = 0, left_ = 0;
    uint64_t round_ = 0;
    bool stop_ = false;
};

inline WorkerPool& worker_pool() {
    static WorkerPool pool(host_threads() > 1 ? host_threads() - 1 : 0);
    return pool;
}

template <typename F>
void parallel_docs(size_t n, F&& fn) {
    const unsigned t = (unsigned)std::min<size_t>(host_threads(), std::max<size_t>(1, n / 256));
    if (t <= 1) {
        fn(0, n);
        return;
    }
    const size_t chunk = (n + t - 1) / t;
    const std::function<void(unsigned)> job = [&fn, n, chunk](unsigned i) {
        const size_t lo = i * chunk, hi = std::min(n, lo + chunk);
        if (lo < hi) fn(lo, hi);
    };
    worker_pool().run(t, job);
}

// 64-bit key hash (8-byte words, multiply-xorshift mixing).  Collisions are
// detected exactly per document, so the quality only sets how often the rank
// fallback runs.
inline uint64_t key_hash(const std::string& s) {
    const unsigned char* p = (const unsigned char*)s.data();
    size_t n = s.size();
    uint64_t h = 0x9E3779B97F4A7C15ull ^ (n * 0xC2B2AE3D27D4EB4Full);
    while (n >= 8) {
        uint64_t w;
        memcpy(&w, p, 8);
        h = (h ^ w) * 0xFF51AFD7ED558CCDull;
        h ^= h >> 29;
        p += 8;
        n -= 8;
    }
    uint64_t w = 0;
    memcpy(&w, p, n);
    h = (h ^ w ^ ((uint64_t)n << 56)) * 0xC4CEB9FE1A85EC53ull;
    h ^= h >> 32;
    h *= 0xD6E8FEB86659FD93ull;
    return h ^ (h >> 32);
}

// CRDT_HOST_RANK_IDS=1: every document takes the collision fallback (tests).
inline bool force_rank_ids() {
    static const bool f = [] {
        const char* e = std::getenv("CRDT_HOST_RANK_IDS");
        return e && e[0] == '1';
    }();
    return f;
}

// One packed slot while a state is sorted: key id, the dot, and the map
// element it came from (its key string; for a destination, the element the
// result updates in place).
struct SlotRef {
    uint64_t id;
    Dot dot;
    Entries::iterator it;
};

// The states of a batch: role 0 = destinations (one per document), role 1 =
// the sources (one per document for a join, any number for a fold); each
// state's slots are contiguous and sorted by id at dfirst[state] /
// sfirst[state] of the page-locked SoA arrays (dk/da/dc, sk/sa/sc) and of the
// element iterators (dit, sit: the Engine's reusable host arrays).
struct Batch {
    size_t R = 1;
    size_t n_docs = 0;
    std::vector<AWSet*> dst;                   // [n_docs]
    std::vector<const AWSet*> src;             // all sources, doc-major
    std::vector<uint32_t> src_beg{0};          // doc d's sources: [src_beg[d], src_beg[d+1])
    std::vector<uint32_t> dfirst, sfirst;      // per state: first slot (prefix of entry counts)
    std::vector<uint32_t> tfirst;              // per source: first tombstone slot
    std::vector<uint8_t> rank_doc;             // 1: ids of doc d are ranks (CRDT_HOST_RANK_IDS)
    std::vector<AWSet*> all;                   // scratch of the aliasing check
    std::vector<const AWSet*> sorted_states;   // scratch of the aliasing check
    uint64_t *dk = nullptr, *dc = nullptr, *sk = nullptr, *sc = nullptr;
    uint32_t *da = nullptr, *sa = nullptr;
    Entries::iterator *dit = nullptr, *sit = nullptr;
    void reset() {  // keeps every vector's capacity
        R = 1;
        n_docs = 0;
        dst.clear();
        src.clear();
        src_beg.assign(1, 0);
    }
};

}  // namespace detail

inline Engine::Engine(int device) : batch_(new detail::Batch()) {
    const int rc = crdt_ctx_create(device, &ctx_);
    if (rc != CRDT_OK) {
        delete batch_;
        throw Error(rc, "crdt_ctx_create");
    }
    // results come back packed (live entries only): less to download, and the
    // apply reads each document at out.offsets[d] either way
    check(crdt_ctx_set_option(ctx_, "pack_batch_outputs", 1), "crdt_ctx_set_option");
}
inline Engine::~Engine() {
    crdt_ctx_destroy(ctx_);
    delete batch_;
}

namespace detail {

// CRDT_HOST_NO_PREFETCH=1: the apply requests nothing ahead (A/B diagnostics).
inline bool host_prefetch() {
    static const bool on = [] {
        const char* e = std::getenv("CRDT_HOST_NO_PREFETCH");
        return !(e && e[0] == '1');
    }();
    return on;
}

// Fill doc d's slots.  A document's key ids are the order in which its keys
// first appear over its states (the destination's keys in map order, then
// each new key of each source): exact -- keys are matched by string, through
// a small per-document open-addressing table of (hash, key) -- and small, so
// every state is placed in ascending id order by direct addressing, with no
// comparison sort.  The destination's ids are its map order, already
// ascending.  (CRDT_HOST_RANK_IDS=1 instead gives the keys' ranks in string
// order, the fallback path of the earlier hash-id scheme, kept for tests.)
// A packing thread's scratch, kept across calls (the worker threads persist).
struct PackScratch {
    struct Cell {
        uint64_t h;
        const std::string* key;
        uint32_t id, gen;
    };
    std::vector<Cell> cells;
    uint32_t gen = 0;
    std::vector<Entries::iterator> by_id;  // a state's element per id (or end)
    std::vector<uint8_t> has;
    std::vector<const std::string*> sorted;
};

struct DocPacker {
    Batch& b;
    uint64_t* tk;
    uint64_t* tc;
    uint32_t* ta;
    PackScratch& s;
    using Cell = PackScratch::Cell;
    std::vector<Cell>& cells = s.cells;
    uint32_t& gen = s.gen;
    std::vector<Entries::iterator>& by_id = s.by_id;
    std::vector<uint8_t>& has = s.has;
    std::vector<const std::string*>& sorted = s.sorted;
    uint32_t mask = 0, next = 0;

    uint32_t intern(const std::string& k) {
        const uint64_t h = key_hash(k);
        for (uint32_t i = (uint32_t)h & mask;; i = (i + 1) & mask) {
            Cell& c = cells[i];
            if (c.gen != gen) {
                c = Cell{h, &k, next, gen};
                return next++;
            }
            if (c.h == h && *c.key == k) return c.id;
        }
    }
    void begin_doc(size_t n_keys) {
        size_t cap = 64;
        while (cap < 2 * n_keys) cap <<= 1;
        if (cells.size() < cap) cells.assign(cap, Cell{0, nullptr, 0, 0}), gen = 0;
        mask = (uint32_t)cap - 1;
        if (++gen == 0) {  // generation wrap: clear once
            std::fill(cells.begin(), cells.end(), Cell{0, nullptr, 0, 0});
            gen = 1;
        }
        next = 0;
    }
    // One state: ids via `id_of`, written in ascending id order (direct
    // addressing over the ids given out so far).
    template <typename IdOf>
    void put_state(const Entries& m, uint32_t first, uint64_t* k, uint32_t* a, uint64_t* c, Entries::iterator* its,
                   IdOf&& id_of) {
        const Entries::iterator end = const_cast<Entries&>(m).end();
        for (auto it = const_cast<Entries&>(m).begin(); it != end; ++it) {
            const uint32_t id = id_of(it->first);
            if (id >= by_id.size()) {
                by_id.resize(id + 1 + id / 2);
                has.resize(by_id.size(), 0);
            }
            by_id[id] = it;
            has[id] = 1;
        }
        const uint32_t stop = first + (uint32_t)m.size();
        for (uint32_t id = 0, o = first; o < stop; ++id) {
            if (!has[id]) continue;
            has[id] = 0;
            const Entries::iterator it = by_id[id];
            k[o] = id;
            a[o] = it->second.actor;
            c[o] = it->second.counter;
            if (its) its[o] = it;
            ++o;
        }
    }
    template <typename IdOf>
    void put_doc(size_t d, IdOf&& id_of) {
        put_state(b.dst[d]->entries, b.dfirst[d], b.dk, b.da, b.dc, b.dit, id_of);
        for (uint32_t s = b.src_beg[d]; s < b.src_beg[d + 1]; ++s) {
            put_state(b.src[s]->entries, b.sfirst[s], b.sk, b.sa, b.sc, b.sit, id_of);
            if (tk)
                if (auto* del = b.src[s]->deleted_map()) put_state(*del, b.tfirst[s], tk, ta, tc, nullptr, id_of);
        }
    }
    void doc(size_t d) {
        if (!force_rank_ids()) {
            size_t n_keys = b.dst[d]->entries.size();
            for (uint32_t s = b.src_beg[d]; s < b.src_beg[d + 1]; ++s) {
                n_keys += b.src[s]->entries.size();
                if (tk)
                    if (auto* del = b.src[s]->deleted_map()) n_keys += del->size();
            }
            begin_doc(n_keys);
            put_doc(d, [this](const std::string& k) { return intern(k); });
            return;
        }
        // rank ids: the key's rank in string order over the doc's states
        b.rank_doc[d] = 1;
        sorted.clear();
        auto add = [&](const Entries& m) {
            for (auto& kv : m) sorted.push_back(&kv.first);
        };
        add(b.dst[d]->entries);
        for (uint32_t s = b.src_beg[d]; s < b.src_beg[d + 1]; ++s) {
            add(b.src[s]->entries);
            if (auto* del = b.src[s]->deleted_map()) add(*del);
        }
        auto lt = [](const std::string* x, const std::string* y) { return *x < *y; };
        std::sort(sorted.begin(), sorted.end(), lt);
        sorted.erase(std::unique(sorted.begin(), sorted.end(), [](auto* x, auto* y) { return *x == *y; }), sorted.end());
        next = (uint32_t)sorted.size();
        put_doc(d, [&](const std::string& k) {
            return (uint32_t)(std::lower_bound(sorted.begin(), sorted.end(), &k, lt) - sorted.begin());
        });
    }
};

// Slot counts and offsets of every state (serial: prefix sums).
inline void layout(Batch& b, bool tombs) {
    b.dfirst.assign(b.n_docs + 1, 0);
    for (size_t d = 0; d < b.n_docs; ++d) b.dfirst[d + 1] = b.dfirst[d] + (uint32_t)b.dst[d]->entries.size();
    const size_t ns = b.src.size();
    b.sfirst.assign(ns + 1, 0);
    b.tfirst.assign(ns + 1, 0);
    for (size_t s = 0; s < ns; ++s) {
        b.sfirst[s + 1] = b.sfirst[s] + (uint32_t)b.src[s]->entries.size();
        const Entries* del = tombs ? b.src[s]->deleted_map() : nullptr;
        b.tfirst[s + 1] = b.tfirst[s] + (uint32_t)(del ? del->size() : 0);
    }
    if ((uint64_t)b.dfirst[b.n_docs] + b.sfirst[ns] >= (1ull << 32)) throw Error(CRDT_E_INVALID, "batch too large");
    b.rank_doc.assign(b.n_docs, 0);
}

// The merged doc (out entries [o, o + c), sorted by id) applied to its
// destination map in place, as the reference's merge mutates dst.Entries:
// keys absent from the result are erased, dots that differ are overwritten,
// new keys inserted -- their strings come from the sources' elements.  plan()
// only reads (the iterators taken when packing are still valid); commit()
// erases, overwrites, then inserts.
struct Plan {
    std::vector<Entries::iterator> erase;
    std::vector<std::pair<Entries::iterator, Dot>> upd;
    std::vector<std::pair<const std::string*, Dot>> ins;
    bool own = false;  // aliased batch: copy the strings (their map may change before commit)
    std::vector<std::pair<std::string, Dot>> ins_own;

    // dst's slots [f, f + m) of (dk, da, dc, dit); sources: slots
    // [sfirst[q], sfirst[q + 1]) of (sk, sit) for q in [s0, s1)
    void plan(const uint64_t* dk, const uint32_t* da, const uint64_t* dc, const Entries::iterator* dit, uint32_t f,
              uint32_t m, const uint64_t* ok, const uint32_t* oa, const uint64_t* oc, uint32_t o, uint32_t c,
              const uint64_t* sk, const Entries::iterator* sit, const uint32_t* sfirst, uint32_t s0, uint32_t s1) {
        erase.clear();
        upd.clear();
        ins.clear();
        ins_own.clear();
        dk += f, da += f, dc += f, dit += f;
        uint32_t i = 0, j = 0;
        uint32_t js = sfirst[s0];  // one source: its slots are walked along the output (both sorted)
        const bool one = s1 - s0 == 1;
        while (i < c || j < m) {
            if (j < m && (i == c || dk[j] < ok[o + i])) {
                erase.push_back(dit[j]);
                ++j;
            } else if (j < m && dk[j] == ok[o + i]) {
                if (da[j] != oa[o + i] || dc[j] != oc[o + i]) upd.emplace_back(dit[j], Dot{oa[o + i], oc[o + i]});
                ++i, ++j;
            } else {  // a key the destination did not hold: its string is a source's
                const uint64_t id = ok[o + i];
                const std::string* name = nullptr;
                if (one) {
                    const uint32_t je = sfirst[s0 + 1];
                    while (js < je && sk[js] < id) ++js;
                    if (js < je && sk[js] == id) name = &sit[js]->first;
                }
                for (uint32_t q = s0; q < s1 && !name && !one; ++q) {
                    const uint64_t* lo = sk + sfirst[q];
                    const uint64_t* hi = sk + sfirst[q + 1];
                    const uint64_t* at = std::lower_bound(lo, hi, id);
                    if (at != hi && *at == id) name = &sit[at - sk]->first;
                }
                if (!name) throw Error(CRDT_E_INVALID, "merge result holds a key no state of its document had");
                if (own)
                    ins_own.emplace_back(*name, Dot{oa[o + i], oc[o + i]});
                else
                    ins.emplace_back(name, Dot{oa[o + i], oc[o + i]});
                ++i;
            }
        }
    }
    // A removed key's node is reused for an added key (extract, rename,
    // reinsert): no free/allocate pair, and the map's size -- hence its bucket
    // array -- does not change, so no rehash invalidates the iterators still
    // to be used.  Only the adds beyond the removals allocate, after every
    // iterator has been used.  (No reserve(): libstdc++'s rehash(n) also
    // SHRINKS to n's bucket count, relinking every node.)
    void commit(AWSet& dst) {
        for (auto& u : upd) u.first->second = u.second;
        size_t k = 0;
        auto put = [&](auto&& key, const Dot& dot) {
            if (k < erase.size()) {
                auto nh = dst.entries.extract(erase[k++]);
                nh.key() = std::forward<decltype(key)>(key);
                nh.mapped() = dot;
                dst.entries.insert(std::move(nh));
            } else {
                dst.entries.emplace(std::forward<decltype(key)>(key), dot);
            }
        };
        for (auto& x : ins) put(*x.first, x.second);
        for (auto& x : ins_own) put(std::move(x.first), x.second);
        for (; k < erase.size(); ++k) dst.entries.erase(erase[k]);
    }
};

// Destinations must be distinct; true when some source is also a destination
// of the batch, so that every plan must be made before any map changes.
inline bool aliased(const std::vector<AWSet*>& dsts, const std::vector<const AWSet*>& srcs, const char* what,
                    std::vector<const AWSet*>& v) {
    v.assign(dsts.begin(), dsts.end());
    std::sort(v.begin(), v.end());
    if (std::adjacent_find(v.begin(), v.end()) != v.end())
        throw Error(CRDT_E_INVALID, std::string(what) + ": a destination appears twice");
    for (auto* s : srcs)
        if (std::binary_search(v.begin(), v.end(), s)) return true;
    return false;
}

// Per document: plan (read only) then commit (the destination maps change).
// Unaliased batches do both per document on its thread; aliased ones make
// every plan first (strings copied), then commit.
// The plan phase also takes the result's VersionVector width from the
// pre-merge states: in an aliased batch another document's commit may be
// rewriting a source's VV while this document commits.
struct DocPlan {
    Plan a, b;      // b: the second direction of an exchange
    size_t w = 0;   // len(dst.versionVector) after the merge
};

// The map elements document d's plan and commit touch -- its destination's
// and its sources' (their strings name the inserted keys) -- requested ahead:
// the maps' nodes are scattered over the heap, so the apply is a chain of cache
// misses unless several are in flight.
inline void prefetch_doc(const Batch& b, size_t d) {
    for (uint32_t j = b.dfirst[d], e = b.dfirst[d + 1]; j < e; ++j) __builtin_prefetch(&*b.dit[j], 1);
    for (uint32_t j = b.sfirst[b.src_beg[d]], e = b.sfirst[b.src_beg[d + 1]]; j < e; ++j)
        __builtin_prefetch(&*b.sit[j], 0);
}

template <typename PlanFn, typename CommitFn>
void apply_docs(const Batch& b, size_t n, bool alias, PlanFn&& plan_fn, CommitFn&& commit_fn) {
    if (!alias) {
        const bool pf = host_prefetch();
        parallel_docs(n, [&](size_t lo, size_t hi) {
            static thread_local DocPlan p;  // (kept with its thread: its vectors keep their capacity)
            if (pf && lo < hi) prefetch_doc(b, lo);
            for (size_t d = lo; d < hi; ++d) {
                if (pf && d + 1 < hi) prefetch_doc(b, d + 1);  // one document ahead (2 or 3: no better)
                plan_fn(d, p);
                commit_fn(d, p);
            }
        });
        return;
    }
    std::vector<DocPlan> plans(n);
    parallel_docs(n, [&](size_t lo, size_t hi) {
        for (size_t d = lo; d < hi; ++d) {
            plans[d].a.own = plans[d].b.own = true;
            plan_fn(d, plans[d]);
        }
    });
    parallel_docs(n, [&](size_t lo, size_t hi) {
        for (size_t d = lo; d < hi; ++d) commit_fn(d, plans[d]);
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
size_t ragged_checks(int mode, size_t n_docs, F&& states_of, const char* what, size_t lo_len, size_t hi_len) {
    // every vector of the batch has one length >= 1: the kernels are exact at R
    if (lo_len == hi_len && hi_len >= 1) {
        if (hi_len > CRDT_MAX_R) throw Error(CRDT_E_INVALID, "version vector longer than CRDT_MAX_R");
        return hi_len;
    }
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

namespace detail {
// len(dst.versionVector) after the fold, replayed on the VVs alone: a delta
// step that brings nothing (awset-delta_test.go:60) skips VersionVector.Merge.
// A step merges iff Counter(src.Actor) == 0 (:53) or MakeDeltaMergeData finds
// a changed entry or an effective tombstone (:79-105).
inline size_t fold_width(int mode, const AWSet& dst, const AWSet* const* srcs, size_t ns) {
    size_t n = dst.versionVector.size();
    if (mode != CRDT_FOLD_DELTA) {
        for (size_t i = 0; i < ns; ++i) n = std::max(n, srcs[i]->versionVector.size());
        return n;
    }
    std::vector<uint64_t> V(dst.versionVector.begin(), dst.versionVector.end());
    for (size_t q = 0; q < ns; ++q) {
        const AWSet* s = srcs[q];
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

// Lay out and pack a batch into the engine's page-locked SoA arrays.
// Returns the destination batch; the sources' arrays are left in the
// engine's kS_* staging.
inline crdt_awset_batch pack(Batch& b, Engine& e, bool tombs) {
    auto t0 = clk::now();
    layout(b, tombs);
    LastStats().layout_s = secs_since(t0);
    const size_t n = b.n_docs, ns = b.src.size(), R = b.R;
    const size_t nd = b.dfirst[n], nse = b.sfirst[ns], nt = b.tfirst[ns];
    // every input array of the call in one page-locked block: staged by one copy
    e.carve({{kD_OFF, (n + 1) * 4}, {kS_OFF, (ns + 1) * 4}, {kD_KEY, nd * 8}, {kD_ACT, nd * 4}, {kD_CTR, nd * 8},
             {kD_VV, n * R * 8}, {kS_KEY, nse * 8}, {kS_ACT, nse * 4}, {kS_CTR, nse * 8}, {kS_VV, ns * R * 8},
             {kS_TKEY, (tombs ? nt : 0) * 8}, {kS_TACT, (tombs ? nt : 0) * 4}, {kS_TCTR, (tombs ? nt : 0) * 8},
             {kS_DOC, (n + 1) * 4}, {kS_SACT, ns * 4}, {kS_TOFF, (ns + 1) * 4}});
    uint32_t* doff = e.pinned<uint32_t>(kD_OFF, n + 1);
    std::copy(b.dfirst.begin(), b.dfirst.end(), doff);
    uint32_t* soff = e.pinned<uint32_t>(kS_OFF, ns + 1);
    std::copy(b.sfirst.begin(), b.sfirst.end(), soff);
    uint64_t* dk = e.pinned<uint64_t>(kD_KEY, nd);
    uint32_t* da = e.pinned<uint32_t>(kD_ACT, nd);
    uint64_t* dc = e.pinned<uint64_t>(kD_CTR, nd);
    uint64_t* dv = e.pinned<uint64_t>(kD_VV, n * R);
    uint64_t* sk = e.pinned<uint64_t>(kS_KEY, nse);
    uint32_t* sa = e.pinned<uint32_t>(kS_ACT, nse);
    uint64_t* sc = e.pinned<uint64_t>(kS_CTR, nse);
    uint64_t* sv = e.pinned<uint64_t>(kS_VV, ns * R);
    uint64_t *tk = nullptr, *tc = nullptr;
    uint32_t* ta = nullptr;
    if (tombs && nt) {
        tk = e.pinned<uint64_t>(kS_TKEY, nt);
        ta = e.pinned<uint32_t>(kS_TACT, nt);
        tc = e.pinned<uint64_t>(kS_TCTR, nt);
    }
    b.dk = dk, b.da = da, b.dc = dc, b.sk = sk, b.sa = sa, b.sc = sc;
    b.dit = e.iters(0, nd);
    b.sit = e.iters(1, nse);
    t0 = clk::now();
    parallel_docs(n, [&](size_t lo, size_t hi) {
        static thread_local PackScratch scratch;
        DocPacker pk{b, tk, tc, ta, scratch};
        for (size_t d = lo; d < hi; ++d) {
            pk.doc(d);
            const auto& v = b.dst[d]->versionVector;
            for (size_t r = 0; r < R; ++r) dv[d * R + r] = r < v.size() ? v[r] : 0;
            for (uint32_t q = b.src_beg[d]; q < b.src_beg[d + 1]; ++q) {
                const auto& w = b.src[q]->versionVector;
                for (size_t r = 0; r < R; ++r) sv[q * R + r] = r < w.size() ? w[r] : 0;
            }
        }
    });
    LastStats().docs_s = secs_since(t0);
    size_t ranks = 0;
    for (auto x : b.rank_doc) ranks += x;
    LastStats().rank_docs = ranks;
    return crdt_awset_batch{(uint32_t)n, (uint32_t)R, doff, nullptr, dk, da, dc, dv};
}

inline crdt_awset_out out_arrays(Engine& e, int first_role, size_t n, size_t R, size_t slots) {
    return crdt_awset_out{e.pinned<uint32_t>(first_role + 0, n + 1), e.pinned<uint32_t>(first_role + 1, n),
                          e.pinned<uint64_t>(first_role + 2, slots), e.pinned<uint32_t>(first_role + 3, slots),
                          e.pinned<uint64_t>(first_role + 4, slots), e.pinned<uint64_t>(first_role + 5, n * R)};
}

inline crdt_awset_batch src_view(const Batch& b, Engine& e) {
    const size_t n = b.n_docs, R = b.R;
    return crdt_awset_batch{(uint32_t)n,
                            (uint32_t)R,
                            e.pinned<uint32_t>(kS_OFF, n + 1),
                            nullptr,
                            e.pinned<uint64_t>(kS_KEY, 0),
                            e.pinned<uint32_t>(kS_ACT, 0),
                            e.pinned<uint64_t>(kS_CTR, 0),
                            e.pinned<uint64_t>(kS_VV, 0)};
}

inline void set_vv(AWSet& dst, const uint64_t* vv, size_t width) { dst.versionVector.assign(vv, vv + width); }

// shortest and longest VersionVector of some states
template <typename V>
void vv_range(const V& states, size_t& lo, size_t& hi) {
    for (const AWSet* x : states) {
        lo = std::min(lo, x->versionVector.size());
        hi = std::max(hi, x->versionVector.size());
    }
}

template <typename SrcVec>
Batch& join_batch(Engine& e, const std::vector<AWSet*>& dsts, const SrcVec& srcs, const char* what) {
    if (dsts.size() != srcs.size()) throw Error(CRDT_E_INVALID, std::string(what) + ": length mismatch");
    Batch& b = e.batch();
    b.reset();
    b.n_docs = dsts.size();
    size_t lo = ~(size_t)0, hi = 0;
    vv_range(dsts, lo, hi);
    vv_range(srcs, lo, hi);
    b.R = ragged_checks(
        CRDT_FOLD_AWSET, b.n_docs, [&](size_t d) { return std::vector<const AWSet*>{dsts[d], srcs[d]}; }, what, lo,
        hi);
    b.dst.assign(dsts.begin(), dsts.end());
    b.src.assign(srcs.begin(), srcs.end());
    b.src_beg.resize(b.n_docs + 1);
    for (size_t d = 0; d <= b.n_docs; ++d) b.src_beg[d] = (uint32_t)d;
    return b;
}
}  // namespace detail

// dsts[i].Merge(*srcs[i]) for every i, as one batched GPU join (dsts distinct).
inline void MergeBatch(const std::vector<AWSet*>& dsts, const std::vector<const AWSet*>& srcs,
                       Engine& e = Engine::Default()) {
    using namespace detail;
    if (dsts.empty() && srcs.empty()) return;
    LastStats() = BoundaryStats{};
    auto t0 = clk::now();
    Batch& b = join_batch(e, dsts, srcs, "MergeBatch");
    const crdt_awset_batch cd = pack(b, e, false), cs = src_view(b, e);
    const size_t n = b.n_docs, slots = (size_t)b.dfirst[n] + b.sfirst[n];
    const crdt_awset_out co = out_arrays(e, kO_OFF, n, b.R, slots);
    LastStats().pack_s = secs_since(t0);
    t0 = clk::now();
    check(crdt_awset_join_batch(e.ctx(), &cd, &cs, &co), "crdt_awset_join_batch");
    LastStats().device_s = secs_since(t0);
    t0 = clk::now();
    apply_docs(
        b, n, aliased(b.dst, b.src, "MergeBatch", b.sorted_states),
        [&](size_t d, DocPlan& p) {
            p.a.plan(b.dk, b.da, b.dc, b.dit, b.dfirst[d], b.dfirst[d + 1] - b.dfirst[d], co.keys, co.actors,
                     co.counters, co.offsets[d], co.counts[d], b.sk, b.sit, b.sfirst.data(), (uint32_t)d,
                     (uint32_t)d + 1);
            p.w = std::max(b.dst[d]->versionVector.size(), b.src[d]->versionVector.size());
        },
        [&](size_t d, DocPlan& p) {  // writes only
            p.a.commit(*b.dst[d]);
            set_vv(*b.dst[d], co.vv + d * b.R, p.w);
        });
    LastStats().apply_s = secs_since(t0);
}

// Anti-entropy both ways: for every i, as[i] <- bs[i] and bs[i] <- as[i],
// the two merges of ONE snapshot (crdt_awset_exchange_batch; each equals
// x := a.Clone(); x.Merge(b) resp. y := b.Clone(); y.Merge(a)), applied in
// place to both maps.
inline void ExchangeBatch(const std::vector<AWSet*>& as, const std::vector<AWSet*>& bs,
                          Engine& e = Engine::Default()) {
    using namespace detail;
    if (as.empty() && bs.empty()) return;
    LastStats() = BoundaryStats{};
    auto t0 = clk::now();
    const auto t_call = t0;
    Batch& b = join_batch(e, as, bs, "ExchangeBatch");
    LastStats().batch_s = secs_since(t0);
    const crdt_awset_batch ca = pack(b, e, false), cb = src_view(b, e);
    const size_t n = b.n_docs, slots = (size_t)b.dfirst[n] + b.sfirst[n];
    const crdt_awset_out oab = out_arrays(e, kO_OFF, n, b.R, slots);
    crdt_awset_out oba = out_arrays(e, kP_OFF, n, b.R, slots);
    oba.keys = oab.keys;  // both directions hold the same keys at the same slots: one column, fetched once
    LastStats().pack_s = secs_since(t0);
    if (const char* ms = std::getenv("CRDT_HOST_PAUSE_MS"))  // diagnostics: host idle before the device phase
        std::this_thread::sleep_for(std::chrono::milliseconds(std::atoi(ms)));
    t0 = clk::now();
    check(crdt_awset_exchange_batch(e.ctx(), &ca, &cb, &oab, &oba), "crdt_awset_exchange_batch");
    if (const char* rep = std::getenv("CRDT_HOST_DEVICE_REPEAT")) {  // diagnostics: the same device call again
        const double first = secs_since(t0);
        for (int r = 0; r < std::atoi(rep); ++r) {
            const auto tr = clk::now();
            check(crdt_awset_exchange_batch(e.ctx(), &ca, &cb, &oab, &oba), "crdt_awset_exchange_batch");
            fprintf(stderr, "device call repeat %d: %.3f ms (first %.3f ms)\n", r, secs_since(tr) * 1e3, first * 1e3);
        }
        t0 = clk::now() - std::chrono::duration_cast<clk::duration>(std::chrono::duration<double>(first));
    }
    LastStats().device_s = secs_since(t0);
    t0 = clk::now();
    {
        std::vector<AWSet*>& all = e.batch().all;  // reused scratch: no large free inside the call
        all.assign(as.begin(), as.end());
        all.insert(all.end(), bs.begin(), bs.end());
        aliased(all, {}, "ExchangeBatch", e.batch().sorted_states);  // every state distinct
    }
    LastStats().distinct_s = secs_since(t0);
    apply_docs(
        b, n, false,
        [&](size_t d, DocPlan& p) {  // both plans read the untouched maps ...
            p.a.plan(b.dk, b.da, b.dc, b.dit, b.dfirst[d], b.dfirst[d + 1] - b.dfirst[d], oab.keys, oab.actors,
                     oab.counters, oab.offsets[d], oab.counts[d], b.sk, b.sit, b.sfirst.data(), (uint32_t)d,
                     (uint32_t)d + 1);
            p.b.plan(b.sk, b.sa, b.sc, b.sit, b.sfirst[d], b.sfirst[d + 1] - b.sfirst[d], oba.keys, oba.actors,
                     oba.counters, oba.offsets[d], oba.counts[d], b.dk, b.dit, b.dfirst.data(), (uint32_t)d,
                     (uint32_t)d + 1);
            p.w = std::max(as[d]->versionVector.size(), bs[d]->versionVector.size());
        },
        [&](size_t d, DocPlan& p) {  // ... then each map changes
            p.a.commit(*as[d]);
            p.b.commit(*bs[d]);
            set_vv(*as[d], oab.vv + d * b.R, p.w);
            set_vv(*bs[d], oba.vv + d * b.R, p.w);
        });
    LastStats().apply_s = secs_since(t0);
    LastStats().call_s = secs_since(t_call);
}

namespace detail {
inline void fold(int mode, const std::vector<AWSet*>& dsts, const std::vector<std::vector<const AWSet*>>& srcs,
                 Engine& e) {
    if (dsts.size() != srcs.size()) throw Error(CRDT_E_INVALID, "fold: length mismatch");
    if (dsts.empty()) return;
    LastStats() = BoundaryStats{};
    auto t0 = clk::now();
    Batch& b = e.batch();
    b.reset();
    b.n_docs = dsts.size();
    size_t lo = ~(size_t)0, hi = 0;
    vv_range(dsts, lo, hi);
    for (auto& l : srcs) vv_range(l, lo, hi);
    b.R = ragged_checks(
        mode, b.n_docs,
        [&](size_t d) {
            std::vector<const AWSet*> v{dsts[d]};
            v.insert(v.end(), srcs[d].begin(), srcs[d].end());
            return v;
        },
        mode == CRDT_FOLD_DELTA ? "DeltaMergeBatch" : "FoldBatch", lo, hi);
    b.dst.assign(dsts.begin(), dsts.end());
    for (auto& l : srcs) {
        b.src.insert(b.src.end(), l.begin(), l.end());
        b.src_beg.push_back((uint32_t)b.src.size());
    }
    const bool tomb_mode = mode == CRDT_FOLD_DELTA;
    const crdt_awset_batch cd = pack(b, e, tomb_mode);
    const size_t n = b.n_docs, ns = b.src.size(), R = b.R;
    uint32_t* doc_srcs = e.pinned<uint32_t>(kS_DOC, n + 1);
    std::copy(b.src_beg.begin(), b.src_beg.end(), doc_srcs);
    uint32_t* sact = e.pinned<uint32_t>(kS_SACT, ns);
    for (size_t q = 0; q < ns; ++q) sact[q] = b.src[q]->actor;
    const bool tombs = tomb_mode && b.tfirst[ns] > 0;  // no tombstones at all: tomb_off = NULL
    uint32_t* toff = nullptr;
    if (tombs) {
        toff = e.pinned<uint32_t>(kS_TOFF, ns + 1);
        std::copy(b.tfirst.begin(), b.tfirst.end(), toff);
    }
    const crdt_src_batch cs{(uint32_t)n,
                            (uint32_t)R,
                            doc_srcs,
                            sact,
                            e.pinned<uint64_t>(kS_VV, 0),
                            e.pinned<uint32_t>(kS_OFF, 0),
                            e.pinned<uint64_t>(kS_KEY, 0),
                            e.pinned<uint32_t>(kS_ACT, 0),
                            e.pinned<uint64_t>(kS_CTR, 0),
                            toff,
                            tombs ? e.pinned<uint64_t>(kS_TKEY, 0) : nullptr,
                            tombs ? e.pinned<uint32_t>(kS_TACT, 0) : nullptr,
                            tombs ? e.pinned<uint64_t>(kS_TCTR, 0) : nullptr};
    const size_t slots = (size_t)b.dfirst[n] + b.sfirst[ns];
    const crdt_awset_out co = out_arrays(e, kO_OFF, n, R, slots);
    LastStats().pack_s = secs_since(t0);
    t0 = clk::now();
    check(crdt_awset_fold_batch(e.ctx(), mode, &cd, &cs, &co), "crdt_awset_fold_batch");
    LastStats().device_s = secs_since(t0);
    t0 = clk::now();
    apply_docs(
        b, n, aliased(b.dst, b.src, "fold", b.sorted_states),
        [&](size_t d, DocPlan& p) {
            p.a.plan(b.dk, b.da, b.dc, b.dit, b.dfirst[d], b.dfirst[d + 1] - b.dfirst[d], co.keys, co.actors,
                     co.counters, co.offsets[d], co.counts[d], b.sk, b.sit, b.sfirst.data(), b.src_beg[d],
                     b.src_beg[d + 1]);
            const uint32_t s0 = b.src_beg[d], s1 = b.src_beg[d + 1];
            p.w = fold_width(mode, *b.dst[d], b.src.data() + s0, s1 - s0);
        },
        [&](size_t d, DocPlan& p) {  // writes only
            p.a.commit(*b.dst[d]);
            set_vv(*b.dst[d], co.vv + d * R, p.w);
        });
    LastStats().apply_s = secs_since(t0);
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
