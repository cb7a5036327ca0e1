// Device-side building blocks shared by the join and fold kernels (gfx950).
//
// The per-key rule these helpers serve is the reference's merge
// (awset.go:107-161) and delta merge (awset-delta_test.go:51-166); see
// DESIGN.md "Per-key rule" for how one rule covers both.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/crdtgpu.h"

namespace crdt {

constexpr int kWave = 64;

// Device status bits (OR-ed into the context's status word).
constexpr uint32_t kErrActorRange = 1u;
constexpr uint32_t kErrWorkspace = 2u;  // fold scratch smaller than the output slots
constexpr uint32_t kErrHint = 4u;       // a doc broke the crdt_ctx_set_max_doc_entries promise
constexpr uint32_t kErrCapacity = 8u;   // a doc's live count exceeds its slots (clamped)
constexpr uint32_t kErrDupKey = 16u;    // a key appears twice in one document (ingest sort)
constexpr uint32_t kErrUnsorted = 32u;  // keys not strictly ascending in a document (host path check)

// Kernel-side view of an AWSet batch (same fields as crdt_awset_batch).
struct BatchView {
    uint32_t n_docs, R;
    const uint32_t* offsets;
    const uint32_t* counts;
    const uint64_t* keys;
    const uint32_t* actors;
    const uint64_t* counters;
    const uint64_t* vv;
};

struct OutView {
    uint32_t* offsets;
    uint32_t* counts;
    uint64_t* keys;
    uint32_t* actors;
    uint64_t* counters;
    uint64_t* vv;
};

struct SrcView {
    uint32_t n_docs, R;
    const uint32_t* doc_srcs;
    const uint32_t* src_actor;
    const uint64_t* vv;
    const uint32_t* entry_off;
    const uint64_t* keys;
    const uint32_t* actors;
    const uint64_t* counters;
    const uint32_t* tomb_off;
    const uint64_t* tkeys;
    const uint32_t* tactors;
    const uint64_t* tcounters;
};

// Scratch copy of the output slots (fold block path ping-pong), `slots` long.
struct Scratch {
    uint64_t* keys;
    uint32_t* actors;
    uint64_t* counters;
    uint64_t slots;
};

// Workspace shared by the launches of one call.
struct Work {
    uint32_t* status;      // device status word (kErr* bits)
    uint32_t* wl_count;    // number of docs pushed to the block-path worklist
    uint32_t* wl_head;     // dequeue head of the block path
    uint32_t* worklist;    // [n_docs]
    uint32_t* chunk_ctr;   // [8] dispenser shards (the tile path's, TileWork::head)
    uint32_t* defer;       // [n_docs] folds: documents the lean pass leaves to the general one
    uint32_t* defer_count; // number of deferred documents
    // Host-path calls (crdt_awset_*_batch): the status word their device key-order
    // checks (pack.hip) wrote.  The first kernel of the merge returns at once when
    // it holds kErrUnsorted, so a batch whose keys are out of order never reaches
    // a merge and no host read-back gates the launch.  NULL: no gate.
    const uint32_t* gate;
};

// The merge's first kernel: false when the host path's order checks failed (Work::gate).
__device__ __forceinline__ bool gate_open(const Work& wk) {
    return !wk.gate || (*wk.gate & kErrUnsorted) == 0u;
}

// Batched local ops (apply.hip): the op lists, tombstones in and out.
struct ApplyOps {
    uint32_t n_docs;
    const uint32_t* op_off;
    const uint8_t* kind;
    const uint64_t* keys;
    const uint32_t* doc_actor;
};

struct TombView {  // AWSetDelta.Deleted of each doc (NULL offsets: none)
    const uint32_t* offsets;
    const uint32_t* counts;
    const uint64_t* keys;
    const uint32_t* actors;
    const uint64_t* counters;
};

struct TombOut {
    uint32_t* offsets;
    uint32_t* counts;
    uint64_t* keys;
    uint32_t* actors;
    uint64_t* counters;
};

// Workspace of the large-document tile path (tile.hip).  A call's tiles are
// numbered 0 .. total-1 over all its documents and run in passes of at most
// `cap` tiles (pass p: tiles [p*cap, p*cap + cap)); the per-tile arrays hold
// one pass, indexed by the tile's position within it.
struct TileWork {
    uint4* desc;          // [cap + 1] {doc, tile index in doc, i0, j0}; + the next pass's first tile
    uint4* geo;           // [2*cap] per-tile geometry (tile.hip, tile_geo_kernel)
    uint64_t* flags;      // [cap] look-back words
    uint32_t* slot_incl;  // [n_docs] inclusive tile count within the slot's run
    uint32_t* run;        // [ceil(n_docs/kRun)] run sums -> exclusive prefixes
    uint32_t* total;      // workspace word: tiles of this call (every pass)
    uint32_t* head;       // workspace words [shards]: tile dispensers (tile.hip, tile_take)
    uint32_t* fallback;   // workspace word: 1 = tiles exceed passes x cap, block kernel runs
    uint32_t* carry;      // workspace words [2]: survivors a document's tiles of the previous pass
                          // placed, for its tiles in this pass (indexed by pass parity)
    uint32_t cap;
    uint32_t tile;   // merged positions per tile (= the tile kernel's NT * IPT)
    uint32_t shape;  // tile kernel shape (tile.hip, tile_positions)
    uint32_t nt_stores;  // non-temporal output stores ("join_tile_nt_stores")
    uint32_t split_bpc;  // tile_split_kernel workgroups per CU ("join_tile_split_blocks_per_cu")
    uint32_t shards;     // tile dispenser words, 1 or 8 ("join_tile_dispensers")
    uint32_t pass;       // the pass this launch runs
    uint32_t passes;     // passes the host launches (more tiles than passes x cap: fallback)
    uint32_t covered;    // 1: passes x cap holds every tile the call can have (no block-kernel fallback launched)
};

// ---- slab order of a grid's blocks.  A streaming kernel whose concurrently
// running workgroups stream separate, distant regions moves more HBM bytes
// per second than one whose running workgroups share one advancing frontier
// (tools/bw_layout.hip on MI355X: copy 5.75 vs 4.9 TB/s, writes 6.0 vs 4.4,
// reads 6.0 vs 5.5).  SlabMap reorders the blocks of a launch so that block c
// takes chunk (c mod G) * S + c / G: the G blocks that run together (G ~ the
// resident blocks of the whole GPU) start G slabs of S chunks apart, and the
// blocks dispatched after them continue each slab in order.  G == 0: identity.
struct SlabMap {
    uint32_t G, S, C;  // slabs, chunks per slab, real chunks
};
inline SlabMap slab_map(uint32_t C, uint32_t G) {
    if (G == 0 || C <= G) return SlabMap{0u, 0u, C};
    return SlabMap{G, (C + G - 1) / G, C};
}
inline uint32_t slab_grid(const SlabMap& m) { return m.G ? m.G * m.S : m.C; }
// chunk of block c, or 0xFFFFFFFF for a padding block (G * S > C) that exits
__device__ __forceinline__ uint32_t slab_chunk(const SlabMap& m, uint32_t c) {
    if (m.G == 0) return c;
    const uint32_t ch = (c % m.G) * m.S + c / m.G;
    return ch < m.C ? ch : 0xFFFFFFFFu;
}

__device__ __forceinline__ uint32_t live_count(const uint32_t* offsets, const uint32_t* counts, uint32_t d) {
    return counts ? counts[d] : offsets[d + 1] - offsets[d];
}

// VersionVector.HasDot (crdt-misc.go:28-34) against a VV of length R held in
// LDS.  actor > R: "never seen"; actor == R: the Go slice index panics, flagged.
__device__ __forceinline__ bool has_dot(const uint64_t* vv, uint32_t R, uint32_t actor, uint64_t counter,
                                        uint32_t& err) {
    if (actor >= R) {
        if (actor == R) err |= kErrActorRange;
        return false;
    }
    return vv[actor] >= counter;
}

// VersionVector.Counter (crdt-misc.go:36-41).
__device__ __forceinline__ uint64_t vv_counter(const uint64_t* vv, uint32_t R, uint32_t actor, uint32_t& err) {
    if (actor >= R) {
        if (actor == R) err |= kErrActorRange;
        return 0;
    }
    return vv[actor];
}

// Intra-wave ordering of LDS traffic (all lanes of one wave).
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }

__device__ __forceinline__ uint32_t popc(uint64_t m) { return (uint32_t)__popcll(m); }

// Bits [0, n) set, n in [0, 64].
// Set bits of m below this lane (popc(m & low_mask(lane))), by mbcnt: two VALU
// ops and no lane-mask register.
__device__ __forceinline__ uint32_t below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ uint64_t low_mask(uint32_t n) { return n >= 64 ? ~0ull : ((1ull << n) - 1ull); }

// Number of elements of the sorted a[0..n) strictly less than key; n <= 2^LOG.
// Branch-free: every probe reads (index 0 when the step is out of range), so a
// wave runs LOG+1 LDS reads with no exec-mask juggling.
template <int LOG>
__device__ __forceinline__ uint32_t lower_bound_pow(const uint64_t* a, uint32_t n, uint64_t key) {
    uint32_t pos = 0;
#pragma unroll
    for (int s = LOG; s >= 0; --s) {
        const uint32_t step = 1u << s;
        const bool in = pos + step <= n;
        const uint64_t v = a[in ? pos + step - 1 : 0u];
        pos += (in && v < key) ? step : 0u;
    }
    return pos;
}

// As lower_bound_pow, but probes only the steps that fit n (n wave-uniform:
// the skipped steps are scalar branches), so short lists cost few LDS reads.
template <int LOG>
__device__ __forceinline__ uint32_t lower_bound_adapt(const uint64_t* a, uint32_t n, uint64_t key) {
    uint32_t pos = 0;
#pragma unroll
    for (int s = LOG; s >= 0; --s) {
        const uint32_t step = 1u << s;
        if (step > n) continue;
        const bool in = pos + step <= n;
        const uint64_t v = a[in ? pos + step - 1 : 0u];
        pos += (in && v < key) ? step : 0u;
    }
    return pos;
}

// Generic lower bound for any n (global or LDS memory).
__device__ __forceinline__ uint32_t lower_bound(const uint64_t* a, uint32_t n, uint64_t key) {
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        uint32_t mid = (lo + hi) >> 1;
        if (a[mid] < key)
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo;
}

// Wave-uniform value (forces a scalar register).
template <typename T>
__device__ __forceinline__ T uniform(T v) {
    return (T)__builtin_amdgcn_readfirstlane((int)v);
}

// ---- buffer resources (T8): per-document descriptors built from wave-uniform
// values.  A lane whose byte offset falls outside the descriptor reads 0 and
// its store is dropped, so partially filled documents need no exec masking and
// every memory op of a loop body can issue unconditionally.
using rsrc_t = __amdgpu_buffer_rsrc_t;
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
constexpr uint32_t kOOB = 0x80000000u;  // byte offset past any descriptor

__device__ __forceinline__ rsrc_t make_rsrc(const void* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
// The same from values the compiler cannot prove wave-uniform but that are: the
// base and size are read from the first lane, so the descriptor is scalar (a
// divergent descriptor makes the compiler loop over its distinct values).
__device__ __forceinline__ rsrc_t make_rsrc_u(const void* p, uint32_t bytes) {
    const uint64_t a = reinterpret_cast<uint64_t>(p);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    return make_rsrc(reinterpret_cast<const void*>(((uint64_t)hi << 32) | lo), __builtin_amdgcn_readfirstlane(bytes));
}
__device__ __forceinline__ uint64_t ld64(rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(uint64_t, __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, 0));
}
__device__ __forceinline__ uint32_t ld32(rsrc_t r, uint32_t off) {
    return (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, 0);
}
// AUX = cache policy bits of the buffer instruction (gfx950: 2 = nt,
// non-temporal: streaming output that no kernel of this launch re-reads).
constexpr int kAuxNT = 2;
template <int AUX = 0>
__device__ __forceinline__ void st64(uint64_t v, rsrc_t r, uint32_t off) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, (int)off, 0, AUX);
}
template <int AUX = 0>
__device__ __forceinline__ void st32(uint32_t v, rsrc_t r, uint32_t off) {
    __builtin_amdgcn_raw_buffer_store_b32(v, r, (int)off, 0, AUX);
}

// HasDot without branches (LDS read always issued); `call` says whether the
// reference evaluates HasDot here, i.e. whether actor == R is its panic.
__device__ __forceinline__ bool has_dot_bf(const uint64_t* vv, uint32_t R, uint32_t actor, uint64_t counter,
                                           bool call, uint32_t& err) {
    const uint64_t v = vv[actor < R ? actor : 0u];
    err |= (call && actor == R) ? kErrActorRange : 0u;
    return actor < R && v >= counter;
}

// Worklist push: the slot and the doc index are checked against the worklist
// capacity (n_docs), so a counter that was not reset can never turn into an
// out-of-bounds address -- it surfaces as CRDT_E_WORKSPACE instead.
__device__ __forceinline__ void push_work(const Work& wk, uint32_t d, uint32_t n_docs) {
    const uint32_t slot = atomicAdd(wk.wl_count, 1u);
    if (slot < n_docs)
        wk.worklist[slot] = d;
    else
        atomicOr(wk.status, kErrWorkspace);
}

// Defer a document from the lean fold pass to the general one (same bounds as push_work).
__device__ __forceinline__ void push_defer(const Work& wk, uint32_t d, uint32_t n_docs) {
    const uint32_t slot = atomicAdd(wk.defer_count, 1u);
    if (slot < n_docs)
        wk.defer[slot] = d;
    else
        atomicOr(wk.status, kErrWorkspace);
}

// Number of worklist entries a consumer may read (clamped to the capacity).
__device__ __forceinline__ uint32_t work_total(const Work& wk, uint32_t n_docs) {
    const uint32_t t = __hip_atomic_load(wk.wl_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return t < n_docs ? t : n_docs;
}

__device__ __forceinline__ void flag_error(uint32_t* status, uint32_t err) {
    // OR of every lane's bits, one atomic per wave that saw an error
    if (ballot(err != 0)) {
        uint32_t e = err;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) e |= (uint32_t)__shfl_xor((int)e, o);
        if (lane_id() == 0) atomicOr(status, e);
    }
}

// ---- diagnostic phase stamps (tools/fold_probe.hip builds with
// CRDT_STAMPS; the product library never does).  Each wave sums the cycles
// between consecutive STAMP(i) points into scalar accumulators and lane 0
// adds them to g_stamps once at the end (cdna_hip_programming.md s7 stamps).
#ifdef CRDT_STAMPS
__device__ unsigned long long g_stamps[16];
__device__ __forceinline__ uint64_t stamp_now() {
    uint64_t t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define STAMP_DECL                    \
    uint64_t st_acc[16] = {0};        \
    uint64_t st_prev = stamp_now();
#define STAMP(i)                      \
    {                                 \
        const uint64_t t_ = stamp_now(); \
        st_acc[i] += t_ - st_prev;    \
        st_prev = t_;                 \
    }
#define STAMP_PARAM , uint64_t(&st_acc)[16], uint64_t& st_prev
#define STAMP_ARGS , st_acc, st_prev
#define STAMP_FLUSH                                                          \
    if ((threadIdx.x & 63) == 0)                                             \
        for (int i_ = 0; i_ < 16; ++i_)                                      \
            if (st_acc[i_]) atomicAdd(&g_stamps[i_], (unsigned long long)st_acc[i_]);
#else
#define STAMP_PARAM
#define STAMP_ARGS
#define STAMP_DECL
#define STAMP(i)
#define STAMP_FLUSH
#endif

}  // namespace crdt
