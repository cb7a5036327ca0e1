// Large-document join split across workgroups: merge-path tiles.
//
// (*AWSet).Merge (awset.go:103-161) of a document with up to millions of
// entries per side.  The wave kernel (join.hip) pushes every document with
// more than 64 entries on a side to the worklist; this path cuts each such
// document into tiles of kTile merged positions so that one large document is
// spread over the whole GPU instead of one workgroup:
//
//   tile_count_kernel   per worklist slot: tiles = ceil((nd + ns) / kTile),
//                       inclusive scan within each run of 1024 slots
//   tile_scan_kernel    one workgroup: exclusive scan of the run sums, the
//                       total tile count; more tiles than the workspace holds
//                       -> the per-document block kernel takes the worklist
//   tile_split_kernel   one thread per tile: the tile's document and its
//                       merge-path split (i0, j0) at diagonal t*kTile, found
//                       by binary search over the two key arrays in HBM
//   join_tile_kernel    persistent workgroups take tiles in order from an
//                       atomic dispenser, stage the tile's dst and src runs in
//                       LDS, decide every union key with the per-key rule,
//                       place the survivors with a decoupled look-back prefix
//                       within the document, and write them coalesced
//
// Merge order puts the dst element first on equal keys, so a common key's
// pair is adjacent; a tile boundary may fall between the two.  The dst element
// then peeks the first src element past its tile (staged at LDS index n), and
// the src element sees the previous dst key (the element before i0).
//
// Exchange (EXCH): out1 = A <- B and out2 = B <- A from one read.  Both keep
// the same keys at the same slots (join.hip, join_doc); only a common key's
// dot differs, the src dot wins (awset.go:142), so each survivor stages two
// LDS indices: the dot for out1 and the dot for out2.
#include "crdt_device.hpp"
#include "wave_sort.hpp"
#include "merge_block.hpp"

namespace crdt {

constexpr uint32_t kRun = 1024;                 // worklist slots per count/scan run

// look-back word: status in bits 32-33, survivors in bits 0-31
constexpr uint64_t kFlagAgg = 1ull << 32;
constexpr uint64_t kFlagInc = 2ull << 32;


__device__ __forceinline__ uint32_t doc_tiles(uint32_t nd, uint32_t ns, uint32_t tile) {
    const uint32_t n = nd + ns;
    return n == 0 ? 1u : (n + tile - 1) / tile;
}

template <int NT>
__global__ __launch_bounds__(NT) void tile_count_kernel(BatchView A, BatchView B, Work wk, TileWork tw) {
    __shared__ uint32_t wave_tot[NT / 64];
    const uint32_t total_slots = work_total(wk, A.n_docs);
    const uint32_t n_runs = (total_slots + kRun - 1) / kRun;
    for (uint32_t r = blockIdx.x; r < n_runs; r += gridDim.x) {
        uint32_t carry = 0;
        for (uint32_t base = r * kRun; base < min((r + 1) * kRun, total_slots); base += NT) {
            const uint32_t slot = base + threadIdx.x;
            uint32_t n = 0;
            if (slot < total_slots && slot < (r + 1) * kRun) {
                const uint32_t d = wk.worklist[slot];
                n = d < A.n_docs ? doc_tiles(live_count(A.offsets, A.counts, d), live_count(B.offsets, B.counts, d),
                                             tw.tile)
                                 : 1u;
            }
            uint32_t tot;
            const uint32_t ex = block_exclusive_scan<NT>(n, wave_tot, &tot);
            if (slot < total_slots && slot < (r + 1) * kRun) tw.slot_incl[slot] = carry + ex + n;
            carry += tot;
        }
        if (threadIdx.x == 0) tw.run[r] = carry;
    }
}

template <int NT>
__global__ __launch_bounds__(NT) void tile_scan_kernel(uint32_t n_docs, Work wk, TileWork tw) {
    __shared__ uint32_t wave_tot[NT / 64];
    const uint32_t total_slots = work_total(wk, n_docs);
    const uint32_t n_runs = (total_slots + kRun - 1) / kRun;
    uint64_t carry = 0;
    for (uint32_t base = 0; base < n_runs; base += NT) {
        const uint32_t r = base + threadIdx.x;
        const uint32_t v = r < n_runs ? tw.run[r] : 0u;
        uint32_t tot;
        const uint32_t ex = block_exclusive_scan<NT>(v, wave_tot, &tot);
        if (r < n_runs) tw.run[r] = (uint32_t)min<uint64_t>(carry + ex, 0xFFFFFFFFull);
        carry += tot;
    }
    if (threadIdx.x == 0) {  // more tiles than the launched passes hold: the block kernel takes the worklist
        const bool over = carry > (uint64_t)tw.cap * tw.passes;
        *tw.fallback = over ? 1u : 0u;
        *tw.total = over ? 0u : (uint32_t)carry;
    }
}

// This launch's pass: tiles [base, base + count) of the call's `total`.
struct TilePass {
    uint32_t base, count;
};
__device__ __forceinline__ TilePass tile_pass(const TileWork& tw, uint32_t total) {
    const uint64_t b = (uint64_t)tw.pass * tw.cap;
    TilePass p{0u, 0u};
    if (b < total) {
        p.base = (uint32_t)b;
        p.count = min(tw.cap, total - p.base);
    }
    return p;
}

// Merge-path split at diagonal k whose answer is known to lie in [lo, hi]
// (merge_path searches the whole diagonal).
__device__ __forceinline__ uint32_t merge_path_in(const uint64_t* dk, const uint64_t* sk, uint32_t k, uint32_t lo,
                                                  uint32_t hi) {
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (dk[mid] <= sk[k - 1 - mid])
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo;
}

#ifndef CRDT_TILE_GALLOP
#define CRDT_TILE_GALLOP 1  // 0: every split bisects its whole diagonal (A/B builds)
#endif
#ifndef CRDT_TILE_GALLOP_HEAD
#define CRDT_TILE_GALLOP_HEAD CRDT_TILE_GALLOP  // 0: a run's first split bisects (A/B builds)
#endif

// merge_path_in from a guess g in [lo, hi): probes g, then steps 1, 2, 4 ...
// away from it until the answer is bracketed, then bisects the bracket.  A
// tile after its predecessor moves about tile * nd / (nd + ns) along the dst
// run, so the bracket is a few elements wide and the probes share lines.
__device__ __forceinline__ uint32_t merge_path_gallop(const uint64_t* dk, const uint64_t* sk, uint32_t k,
                                                      uint32_t lo, uint32_t hi, uint32_t g) {
    if (lo >= hi)
        return lo;
    g = min(max(g, lo), hi - 1u);
    if (dk[g] <= sk[k - 1 - g]) {
        lo = g + 1u;
        for (uint32_t step = 1;; step <<= 1) {
            const uint32_t j = g + step;
            if (j >= hi)
                break;
            if (!(dk[j] <= sk[k - 1 - j])) {
                hi = j;
                break;
            }
            lo = j + 1u;
        }
    } else {
        hi = g;
        for (uint32_t step = 1;; step <<= 1) {
            if (step > g - lo)
                break;
            const uint32_t j = g - step;
            if (dk[j] <= sk[k - 1 - j]) {
                lo = j + 1u;
                break;
            }
            hi = j;
        }
    }
    return merge_path_in(dk, sk, k, lo, hi);
}

// kSplitRun consecutive tiles per thread: a tile after its document's previous
// tile searches only the window its predecessor's split bounds (the split
// moves by at most one tile along each array: i(t) <= i(t+1) <= i(t) + tile),
// so the deep levels of the search -- a line fetched per level -- are fewer.
#ifndef CRDT_TILE_SPLIT_RUN
#define CRDT_TILE_SPLIT_RUN 4  // (A/B builds)
#endif
constexpr uint32_t kSplitRun = CRDT_TILE_SPLIT_RUN;

// Tiles of one pass, plus the first tile of the next pass: its split is where
// this pass's last tile ends (tile_geo_kernel).
template <int NT>
__global__ __launch_bounds__(NT) void tile_split_kernel(BatchView A, BatchView B, Work wk, TileWork tw) {
    const uint32_t total = *tw.total;
    const TilePass ps = tile_pass(tw, total);
    if (ps.count == 0) return;
    const uint32_t n_split = min(ps.count + 1u, total - ps.base);
    const uint32_t total_slots = work_total(wk, A.n_docs);
    const uint32_t n_runs = (total_slots + kRun - 1) / kRun;
    uint32_t pd = 0xFFFFFFFFu, pt = 0, pi = 0;  // this thread's previous tile: document, index, split
    for (uint32_t l0 = (blockIdx.x * NT + threadIdx.x) * kSplitRun; l0 < n_split; l0 += gridDim.x * NT * kSplitRun)
    for (uint32_t l = l0; l < min(l0 + kSplitRun, n_split); ++l) {
        const uint32_t g = ps.base + l;  // the call's tile number
        // run: last r with run[r] <= g (run prefixes strictly increase: every slot has >= 1 tile)
        uint32_t lo = 0, hi = n_runs;
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (tw.run[mid] <= g)
                lo = mid;
            else
                hi = mid;
        }
        const uint32_t r = lo, rbase = tw.run[r], rel = g - rbase;
        // slot: first slot of the run whose inclusive count exceeds rel
        uint32_t s0 = r * kRun, s1 = min(s0 + kRun, total_slots);
        while (s0 < s1) {
            const uint32_t mid = (s0 + s1) >> 1;
            if (tw.slot_incl[mid] <= rel)
                s0 = mid + 1;
            else
                s1 = mid;
        }
        const uint32_t slot = s0;
        const uint32_t first = (slot % kRun) ? tw.slot_incl[slot - 1] : 0u;
        const uint32_t t = rel - first;
        const uint32_t d = wk.worklist[slot];
        uint32_t i0 = 0, j0 = 0;
        if (d < A.n_docs) {
            const uint32_t nd = live_count(A.offsets, A.counts, d), ns = live_count(B.offsets, B.counts, d);
            const uint32_t k0 = min(t * tw.tile, nd + ns);
            uint32_t lo = k0 > ns ? k0 - ns : 0u, hi = k0 < nd ? k0 : nd;
            const uint64_t* dk = A.keys + A.offsets[d];
            const uint64_t* sk = B.keys + B.offsets[d];
            if (CRDT_TILE_GALLOP && d == pd && t == pt + 1u) {  // the previous tile's split bounds this one's
                lo = max(lo, pi);
                hi = min(hi, pi + tw.tile);
                const uint32_t g = pi + (uint32_t)(((uint64_t)tw.tile * nd) / max(nd + ns, 1u));
                i0 = merge_path_gallop(dk, sk, k0, lo, hi, g);
            } else if (CRDT_TILE_GALLOP_HEAD) {  // a run's first tile: from the proportional point of its diagonal
                i0 = merge_path_gallop(dk, sk, k0, lo, hi, (uint32_t)(((uint64_t)k0 * nd) / max(nd + ns, 1u)));
            } else {
                i0 = merge_path_in(dk, sk, k0, lo, hi);
            }
            j0 = k0 - i0;
        }
        pd = d;
        pt = t;
        pi = i0;
        tw.desc[l] = make_uint4(d, t, i0, j0);
        if (l < ps.count) tw.flags[l] = 0ull;
    }
}

template <int NT, int IPT>
struct TileSmem {
    static constexpr uint32_t T = NT * IPT;
    uint64_t key[T + 1];  // dst run at [0, nA), src run at [nA, nA+nB), peeked src element at nA+nB
    uint64_t ctr[T + 1];
    uint32_t act[T + 1];
    uint32_t stage[T];  // survivor p: LDS index of its out1 dot | out2 dot << 16
    uint64_t va[CRDT_MAX_R];
    uint64_t vb[CRDT_MAX_R];
    uint32_t wave_tot[NT / 64];
    uint32_t word[4];
    uint64_t prev_key;
};

// The tile dispenser, sharded: workgroup b takes the tiles s, s + S, s + 2S, ...
// (s = b mod S, S = tw.shards) in order from head word s.  One word taken by
// every workgroup saturates near 88 M takes/s (MI355X_MICROARCH.md, 'dequeue')
// -- config 4 takes 1.1 M tiles per launch -- while S = 8 words, one per XCD
// (workgroups are dispatched to the XCDs round-robin, so b mod 8 is the XCD),
// spread the takes.  Progress: a taken tile is published without waiting; a
// look-back waits only on smaller tiles, and the smallest tile not yet
// published is either held by a workgroup whose pending look-back concerns
// smaller, published tiles only, or not taken yet, in which case the resident
// workgroups of its shard (blocks 0..S-1 start first) are not held by it
// either and reach it.  Needs S resident workgroups, as the persistent grid
// (the occupancy query) always has.
__device__ __forceinline__ uint32_t tile_take(const TileWork& tw) {
    const uint32_t S = tw.shards, s = blockIdx.x % S;
    return atomicAdd(tw.head + s, 1u) * S + s;
}

__device__ __forceinline__ uint64_t flag_load(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void flag_store(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Exclusive prefix of tile g (index t within its document) by decoupled
// look-back over tiles g-1 .. g-t, 64 predecessors per poll (wave 0 only).
// Tile 0 of a document publishes its inclusive count at once, so the walk
// ends inside the document; a predecessor not yet published is polled again
// (it was dispensed before g and publishes its aggregate without waiting).
__device__ __forceinline__ uint32_t look_back(uint64_t* flags, uint32_t g, uint32_t t, uint32_t lane,
                                              uint64_t* polls = nullptr) {
    uint32_t prefix = 0;
    uint32_t look = g - 1;
    int32_t rem = (int32_t)t;
    for (;;) {
        const uint64_t f = (int32_t)lane < rem ? flag_load(flags + (look - lane)) : kFlagInc;
        const uint32_t st = (uint32_t)(f >> 32);
        const uint64_t inc = ballot(st == 2u);
        const uint32_t first_inc = inc ? (uint32_t)__builtin_ctzll(inc) : 64u;
        const uint64_t pending = ballot(st == 0u) & low_mask(first_inc + 1u);
        if (polls) polls[pending ? 1 : 0] += 1;  // diagnostic builds: polls that found a gap / that summed
        if (pending) {
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        uint32_t v = lane <= first_inc ? (uint32_t)f : 0u;
        v += dpp<0x111>(0u, v);  // wave sum: DPP inclusive scan (no LDS round trips) ...
        v += dpp<0x112>(0u, v);
        v += dpp<0x114>(0u, v);
        v += dpp<0x118>(0u, v);
        v += dpp<0x142, 0xA>(0u, v);
        v += dpp<0x143, 0xC>(0u, v);
        prefix += (uint32_t)__builtin_amdgcn_readlane((int)v, 63);  // ... whose last lane holds the total
        if (first_inc < 64u) break;
        look -= 64;
        rem -= 64;
    }
    return prefix;
}

// A tile's coordinates, from its descriptor and its successor's (uniform loads).
struct TileGeo {
    uint32_t d, t, ga, gb, nA, nB, obase;  // ga/gb: absolute slot of the tile's first dst/src element
    bool last, has_next, has_prev, bad;
    bool cont_in, cont_out;  // the document continues from the previous pass / into the next
};

// A tile's geometry record sits with those of its dispenser shard (tile_take):
// the shard's tiles, taken in order by the workgroups of one XCD, then share
// cache lines (four 32-byte records a line) in that XCD's L2, so the geometry
// load of most taken tiles hits L2 instead of going to memory.
__device__ __forceinline__ size_t geo_slot(const TileWork& tw, uint32_t g) {
    const uint32_t S = tw.shards;
    return (size_t)(g % S) * ((tw.cap + S - 1) / S) + g / S;
}

// Per-tile geometry, precomputed once per call (tile_geo_kernel) so that a
// workgroup's dependent chain per tile is dispense -> one 32-byte record ->
// data loads.
// Flags of a tile's geometry record (r1.z): the document's last tile, a src
// element past the tile, a dst element before it; the first tile of this pass
// continuing a document of the previous pass (its tiles there placed
// tw.carry[pass & 1] survivors), the last tile of this pass whose document
// continues in the next (it hands on its inclusive count).
constexpr uint32_t kGeoLast = 1u, kGeoNext = 2u, kGeoPrev = 4u, kGeoContIn = 8u, kGeoContOut = 16u;

__global__ __launch_bounds__(256) void tile_geo_kernel(BatchView A, BatchView B, TileWork tw) {
    const uint32_t total = *tw.total;
    const TilePass ps = tile_pass(tw, total);
    // this pass's dispensers start at 0 (the previous pass's tile kernel, which
    // advanced them, has finished; pass 0's were zeroed with the call's counters)
    if (tw.pass && blockIdx.x == 0 && threadIdx.x < tw.shards) tw.head[threadIdx.x] = 0u;
    for (uint32_t l = blockIdx.x * 256 + threadIdx.x; l < ps.count; l += gridDim.x * 256) {
        const uint4 ds = tw.desc[l];
        const uint32_t d = ds.x, t = ds.y, i0 = ds.z, j0 = ds.w;
        uint4 r0 = make_uint4(d, t, 0u, 0u), r1 = make_uint4(0u, 0u, kGeoLast, 0u);
        if (d < A.n_docs) {
            const uint32_t nd = live_count(A.offsets, A.counts, d), ns = live_count(B.offsets, B.counts, d);
            const uint32_t aoff = A.offsets[d], boff = B.offsets[d];
            uint32_t i1 = nd, j1 = ns, last = kGeoLast;
            if (ps.base + l + 1 < total) {  // (desc[count] is the next pass's first tile)
                const uint4 nx = tw.desc[l + 1];
                if (nx.x == d && nx.y == t + 1) {
                    i1 = nx.z;
                    j1 = nx.w;
                    last = 0u;
                }
            }
            r0.z = aoff + i0;
            r0.w = boff + j0;
            r1.x = i1 - i0;
            r1.y = j1 - j0;
            r1.z = last | (j1 < ns ? kGeoNext : 0u) | (i0 > 0 ? kGeoPrev : 0u) |
                   ((l == 0 && t > 0) ? kGeoContIn : 0u) | ((l + 1 == ps.count && !last) ? kGeoContOut : 0u);
            r1.w = aoff + boff;
        }
        const size_t at = geo_slot(tw, l);
        tw.geo[2 * at] = r0;
        tw.geo[2 * at + 1] = r1;
    }
}

__device__ __forceinline__ TileGeo tile_geo(const BatchView& A, const TileWork& tw, uint32_t g) {
    TileGeo x{};
    const size_t at = geo_slot(tw, g);
    const uint4 r0 = tw.geo[2 * at], r1 = tw.geo[2 * at + 1];
    x.d = r0.x;
    x.t = r0.y;
    x.ga = r0.z;
    x.gb = r0.w;
    x.nA = r1.x;
    x.nB = r1.y;
    x.last = (r1.z & kGeoLast) != 0;
    x.has_next = (r1.z & kGeoNext) != 0;
    x.has_prev = (r1.z & kGeoPrev) != 0;
    x.cont_in = (r1.z & kGeoContIn) != 0;
    x.cont_out = (r1.z & kGeoContOut) != 0;
    x.obase = r1.w;
    x.bad = x.d >= A.n_docs;  // not a document of this call: never dereferenced
    if (x.bad) x.nA = x.nB = 0, x.has_next = x.has_prev = x.cont_in = x.cont_out = false;
    return x;
}

// One tile's operands in registers, loaded a tile ahead: thread tid holds staged
// positions p = tid + q*NT -- the dst run [0, nA), the src run [nA, n), and at
// p == n the src element past the tile (a common key's twin across the
// boundary); the last thread also the element past a full tile (p == T) and the
// dst key before the tile; lanes < R the two clocks.
template <int IPT>
struct TileRegs {
    uint64_t k[IPT], c[IPT], xk, xc, pk, va, vb;
    uint32_t a[IPT], xa;
};

template <int NT, int IPT>
__device__ __forceinline__ void tile_issue(const BatchView& A, const BatchView& B, const TileGeo& x, uint32_t tid,
                                           const void* dummy, TileRegs<IPT>& r) {
    constexpr uint32_t T = NT * IPT;
    const uint32_t n = x.nA + x.nB;
    const bool peek = x.has_next;
    const uint64_t* ak = A.keys + x.ga;
    const uint32_t* aa = A.actors + x.ga;
    const uint64_t* ac = A.counters + x.ga;
    const uint64_t* bk = B.keys + x.gb;
    const uint32_t* ba = B.actors + x.gb;
    const uint64_t* bc = B.counters + x.gb;
#pragma unroll
    for (int q = 0; q < IPT; ++q) {
        const uint32_t p = tid + q * NT;
        const bool inA = !x.bad && p < x.nA;
        const uint32_t pb = p - x.nA;
        const bool inB = !x.bad && !inA && (p < n || (p == n && peek));
        // one load per array for every lane (address selected; `dummy` for none)
        const uint64_t* kp = inA ? ak + p : (inB ? bk + pb : static_cast<const uint64_t*>(dummy));
        const uint32_t* ap = inA ? aa + p : (inB ? ba + pb : static_cast<const uint32_t*>(dummy));
        const uint64_t* cp = inA ? ac + p : (inB ? bc + pb : static_cast<const uint64_t*>(dummy));
        // (no select on the values: a lane without an element holds a dummy that
        // nothing reads, and a select here would wait for the load)
        r.k[q] = __builtin_nontemporal_load(kp);
        r.a[q] = __builtin_nontemporal_load(ap);
        r.c[q] = __builtin_nontemporal_load(cp);
    }
    // the rest unconditionally (a lane with nothing to load reads `dummy`): the
    // number of loads issued after the runs' is fixed, so the stage's vmcnt
    // wait is exact and never waits out the stores issued after them
    const uint64_t* dk = static_cast<const uint64_t*>(dummy);
    const uint32_t* da = static_cast<const uint32_t*>(dummy);
    const bool px = tid == NT - 1 && n == T && peek, pp = tid == NT - 1 && x.has_prev;
    const bool vl = !x.bad && tid < A.R;
    // (read only where they exist: the peeked element when the tile is full and
    // has a successor, the key before it when it has a predecessor, the clocks
    // of a real tile)
    r.xk = *(px ? bk + x.nB : dk);
    r.xa = *(px ? ba + x.nB : da);
    r.xc = *(px ? bc + x.nB : dk);
    r.pk = *(pp ? ak - 1 : dk);
    r.va = *(vl ? A.vv + (size_t)x.d * A.R + tid : dk);
    r.vb = *(vl ? B.vv + (size_t)x.d * A.R + tid : dk);
}

// Front of a tile: stage its registers in LDS, merge IPT positions per thread
// from the thread's diagonal split deciding every union key, and compact the
// survivors' LDS indices (out1 dot | out2 dot << 16) into sm.stage in merged
// order.  Returns the tile's survivor count (every thread).  Ends with the
// workgroup barrier of the scan.
template <int NT, int IPT>
__device__ __forceinline__ void tile_stage(TileSmem<NT, IPT>& sm, const TileGeo& cur, const TileRegs<IPT>& r,
                                           uint32_t R, uint32_t tid) {
    constexpr uint32_t T = NT * IPT;
    const uint32_t nA = cur.nA, nB = cur.nB, n = nA + nB;  // n <= T
#pragma unroll
    for (int q = 0; q < IPT; ++q) {
        const uint32_t p = tid + q * NT;
        if (p <= n && p < T) {
            sm.key[p] = r.k[q];
            sm.act[p] = r.a[q];
            sm.ctr[p] = r.c[q];
        }
    }
    if (tid == NT - 1) {
        if (n == T) {
            sm.key[T] = r.xk;
            sm.act[T] = r.xa;
            sm.ctr[T] = r.xc;
        }
        sm.prev_key = r.pk;
    }
    if (tid < R) {
        sm.va[tid] = r.va;
        sm.vb[tid] = r.vb;
    }
}

// The decide half of a tile's front (after tile_stage and a barrier).
template <int NT, int IPT>
__device__ __forceinline__ uint32_t tile_decide(TileSmem<NT, IPT>& sm, const TileGeo& cur, uint32_t R, uint32_t tid,
                                                uint32_t& err) {
    const uint32_t nA = cur.nA, nB = cur.nB, n = nA + nB;
    const bool has_next = cur.has_next, has_prev = cur.has_prev;
    const uint64_t prev_key = sm.prev_key;
    const uint32_t k0 = min(tid * IPT, n);
    uint32_t a = merge_path(sm.key, nA, sm.key + nA, nB, k0);
    uint32_t b = k0 - a;
    uint32_t pick[IPT];
    bool keep[IPT];
    uint32_t cnt = 0;
#pragma unroll
    for (int q = 0; q < IPT; ++q) {
        keep[q] = false;
        pick[q] = 0;
        if (k0 + q < n) {
            const bool take_a = a < nA && (b >= nB || sm.key[a] <= sm.key[nA + b]);
            if (take_a) {
                const uint64_t key = sm.key[a];
                const uint32_t nb = b < nB ? nA + b : n;  // next src element (peeked past the tile)
                const bool match = (b < nB || has_next) && sm.key[nb] == key;
                if (match) {  // common key: present, src dot wins (awset.go:123-129,142)
                    keep[q] = true;
                    pick[q] = nb | (a << 16);
                } else {  // dst-only: removed iff srcVV.HasDot(d) (awset.go:146-158)
                    keep[q] = !has_dot(sm.vb, R, sm.act[a], sm.ctr[a], err);
                    pick[q] = a | (a << 16);
                }
                ++a;
            } else {
                const uint32_t sb = nA + b;
                const uint64_t key = sm.key[sb];
                const bool match = a > 0 ? sm.key[a - 1] == key : (has_prev && prev_key == key);
                if (!match) {  // src-only: added iff !dstVV.HasDot(s) (awset.go:130-140)
                    keep[q] = !has_dot(sm.va, R, sm.act[sb], sm.ctr[sb], err);
                    pick[q] = sb | (sb << 16);
                }
                ++b;
            }
            cnt += keep[q] ? 1u : 0u;
        }
    }
    uint32_t agg;
    const uint32_t lpos = block_exclusive_scan<NT>(cnt, sm.wave_tot, &agg);
    uint32_t p = lpos;
#pragma unroll
    for (int q = 0; q < IPT; ++q)
        if (keep[q]) sm.stage[p++] = pick[q];
    return agg;
}

template <int NT, int IPT>
__device__ __forceinline__ uint32_t tile_front(TileSmem<NT, IPT>& sm, const TileGeo& cur, const TileRegs<IPT>& r,
                                               uint32_t R, uint32_t tid, uint32_t& err) {
    tile_stage<NT, IPT>(sm, cur, r, R, tid);
    __syncthreads();
    return tile_decide<NT, IPT>(sm, cur, R, tid, err);
}

// Survivors of a staged tile written coalesced at the document's output base +
// prefix; the last tile writes the count, tile 0 the merged clock.  Every
// store is issued by every thread (buffer stores; out-of-range offsets where
// there is nothing to write, and for `none`), so the count of memory operations
// after the next tile's loads is fixed and the wait for them is exact.
//
// ALIGN: lane l of every store instruction writes an output slot = l (mod 64),
// so each wave-instruction covers one aligned 64-slot window (whole cache
// lines; the tile's first and last windows are shared with its neighbours);
// one more round of stores than positions per thread.
template <int NT, int IPT, bool EXCH, bool NTS, bool ALIGN = false>
__device__ __forceinline__ void tile_stores(const TileSmem<NT, IPT>& sm, const TileGeo& cur, bool none,
                                            uint32_t prefix, uint32_t agg, uint32_t R, uint32_t tid,
                                            const OutView& o1, const OutView& o2) {
    constexpr int AUX = NTS ? kAuxNT : 0;
    // descriptors from wave-uniform values (a divergent descriptor would make
    // the compiler loop over its distinct values around every store)
    const bool w = !none && !cur.bad;
    const size_t obase = (size_t)uniform(cur.obase + prefix);
    const uint32_t nb = uniform(w ? agg : 0u);
    const uint32_t d = uniform(cur.d);
    const rsrc_t k1 = make_rsrc_u(o1.keys + obase, nb * 8u), a1 = make_rsrc_u(o1.actors + obase, nb * 4u),
                 c1 = make_rsrc_u(o1.counters + obase, nb * 8u);
    // o2.keys == o1.keys: one shared key column, written once (the store
    // still issues, out of range, so the count of memory operations is fixed)
    const rsrc_t k2 = make_rsrc_u(o2.keys + obase, (EXCH && o2.keys != o1.keys) ? nb * 8u : 0u),
                 a2 = make_rsrc_u(o2.actors + obase, EXCH ? nb * 4u : 0u),
                 c2 = make_rsrc_u(o2.counters + obase, EXCH ? nb * 8u : 0u);
    const uint32_t shift = ALIGN ? (uint32_t)(obase & 63u) : 0u;
#pragma unroll
    for (int q = 0; q < IPT + (ALIGN ? 1 : 0); ++q) {
        const uint32_t p = tid + q * NT - shift;  // wraps below 0: out of range
        const bool in = p < nb;
        const uint32_t v = sm.stage[in ? p : 0u];
        const uint32_t x1 = in ? (v & 0xFFFFu) : 0u, x2 = in ? (v >> 16) : 0u;
        const uint64_t key = sm.key[x1];
        const uint32_t o8 = in ? p * 8u : kOOB, o4 = in ? p * 4u : kOOB;
        st64<AUX>(key, k1, o8);
        st32<AUX>(sm.act[x1], a1, o4);
        st64<AUX>(sm.ctr[x1], c1, o8);
        if (EXCH) {
            st64<AUX>(key, k2, o8);
            st32<AUX>(sm.act[x2], a2, o4);
            st64<AUX>(sm.ctr[x2], c2, o8);
        }
    }
    const uint32_t co = (w && cur.last && tid == 0) ? 0u : kOOB;
    st32(prefix + agg, make_rsrc_u(o1.counts + d, 4u), co);
    if (EXCH) st32(prefix + agg, make_rsrc_u(o2.counts + d, 4u), co);
    // awset.go:160 -> crdt-misc.go:43-55, the same max both ways
    const uint64_t m = max(sm.va[tid < R ? tid : 0u], sm.vb[tid < R ? tid : 0u]);
    const uint32_t vo = (w && cur.t == 0 && tid < R) ? tid * 8u : kOOB;
    st64(m, make_rsrc_u(o1.vv + (size_t)d * R, R * 8u), vo);
    if (EXCH) st64(m, make_rsrc_u(o2.vv + (size_t)d * R, R * 8u), vo);
}

// Persistent workgroups take tiles in order from an atomic dispenser.  The
// next tile is taken once this tile's look-back is done (from then on nothing
// of this tile waits on another workgroup, so a taken tile is never held
// behind a wait), and its loads are issued before this tile's output stores,
// which they overlap.
template <int NT, int IPT, bool EXCH, bool NTS>
__global__ __launch_bounds__(NT) void join_tile_kernel(BatchView A, BatchView B, OutView o1, OutView o2,
                                                       TileWork tw, Work wk) {
    __shared__ TileSmem<NT, IPT> sm;
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    const uint32_t R = A.R;
    const uint32_t total = tile_pass(tw, *tw.total).count;  // this pass's tiles, numbered from 0
    if (total == 0) return;  // a pass past the call's tiles
    const uint32_t carry_in = tw.pass ? tw.carry[tw.pass & 1u] : 0u;
    uint32_t err = 0;
    TileRegs<IPT> rg;
    STAMP_DECL

    if (tid == 0) sm.word[0] = tile_take(tw);
    __syncthreads();
    uint32_t g = sm.word[0];
    TileGeo x{};
    if (g < total) x = tile_geo(A, tw, g);
    else x.bad = true;
    tile_issue<NT, IPT>(A, B, x, tid, tw.desc, rg);
    tile_stores<NT, IPT, EXCH, NTS>(sm, x, true, 0u, 0u, R, tid, o1, o2);  // (as in the pipelined kernel)
    while (g < total) {
        const TileGeo cur = x;
        const uint32_t agg = tile_front<NT, IPT>(sm, cur, rg, R, tid, err);
        STAMP(1)
        if (tid < 64) {
            uint32_t prefix = 0;
            if (cur.bad) {
                if (lane == 0) {
                    atomicOr(wk.status, kErrWorkspace);
                    flag_store(tw.flags + g, kFlagInc);
                }
            } else if (cur.t == 0 || cur.cont_in) {  // a document's first tile (in this pass): inclusive at once
                prefix = cur.t == 0 ? 0u : carry_in;
                if (lane == 0) flag_store(tw.flags + g, kFlagInc | (prefix + agg));
            } else {
                if (lane == 0) flag_store(tw.flags + g, kFlagAgg | agg);
                prefix = look_back(tw.flags, g, min(cur.t, g), lane);
                if (lane == 0) flag_store(tw.flags + g, kFlagInc | (prefix + agg));
            }
            if (cur.cont_out && lane == 0) tw.carry[(tw.pass + 1u) & 1u] = prefix + agg;  // for the next pass
            // nothing of this tile waits on another workgroup any more: take the
            // next tile now (a tile taken earlier would be held while this one's
            // look-back waits, and its successors would wait on that in turn)
            if (lane == 0) {
                sm.word[0] = tile_take(tw);
                sm.word[1] = prefix;
            }
        }
        __syncthreads();
        STAMP(3)
        const uint32_t prefix = sm.word[1];
        const uint32_t gn = sm.word[0];
        // the next tile's loads overlap this tile's stores (past the end: dummy
        // loads, so their number never depends on the path)
        if (gn < total) x = tile_geo(A, tw, gn);
        else x = TileGeo{}, x.bad = true;
        tile_issue<NT, IPT>(A, B, x, tid, tw.desc, rg);
        STAMP(4)
        tile_stores<NT, IPT, EXCH, NTS>(sm, cur, false, prefix, agg, R, tid, o1, o2);
        __syncthreads();
        STAMP(5)
        g = gn;
    }
    STAMP_FLUSH
    if (__syncthreads_or(err != 0) && tid == 0) atomicOr(wk.status, kErrActorRange);
}

// Pipelined tiles: a tile's look-back is deferred by one tile.  Per round the
// workgroup (1) decides tile g1 (its loads arrived during the previous round)
// and publishes g1's aggregate at once, (2) runs the look-back of the tile
// before it, g0, whose predecessors have had a whole front to publish, (3) takes
// the next tile g2 and issues its loads, (4) writes g0's survivors.  Two LDS
// tile buffers alternate.  Holding: g1 is held through g0's look-back with its
// aggregate already published (successors sum past it); g2 is taken after the
// look-back and decided next round with nothing to wait on in between -- so
// every walk ends (each tile's aggregate is published without waiting, and
// tile 0 of a document publishes its inclusive count).
template <int NT, int IPT, bool EXCH, bool NTS, bool ALIGN>
__device__ __forceinline__ void tile_pipe_body(const BatchView& A, const BatchView& B, const OutView& o1,
                                               const OutView& o2, const TileWork& tw, const Work& wk) {
    __shared__ TileSmem<NT, IPT> sm[2];
    __shared__ uint32_t word[2];
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    const uint32_t R = A.R;
    const uint32_t total = tile_pass(tw, *tw.total).count;  // this pass's tiles, numbered from 0
    if (total == 0) return;  // a pass past the call's tiles
    const uint32_t carry_in = tw.pass ? tw.carry[tw.pass & 1u] : 0u;
    uint32_t err = 0;
    TileRegs<IPT> rg;
    STAMP_DECL

    if (tid == 0) word[0] = tile_take(tw);
    __syncthreads();
    uint32_t g1 = word[0];
    if (g1 >= total) return;
    TileGeo x1 = tile_geo(A, tw, g1);
    tile_issue<NT, IPT>(A, B, x1, tid, tw.desc, rg);
    // as many (dropped) stores as a round issues after its loads: the loop is
    // entered with the same memory operations behind them on both paths, so the
    // stage's wait for them is an exact vmcnt
    tile_stores<NT, IPT, EXCH, NTS, ALIGN>(sm[1], x1, true, 0u, 0u, R, tid, o1, o2);
    uint32_t g0 = total, agg0 = 0;  // g0 >= total: no tile waiting for its stores
    TileGeo x0{};
    uint32_t buf = 0;
    // g0's look-back (wave 0), then the next tile; every thread gets both
    auto resolve0 = [&](uint32_t& prefix0, uint32_t& g2) {
        if (tid < 64) {
            uint32_t p0 = 0;
            const bool live0 = g0 < total && !x0.bad;
            if (live0 && x0.cont_in) {
                p0 = carry_in;  // (published inclusive by publish1)
            } else if (live0 && x0.t != 0) {
#ifdef CRDT_STAMPS
                p0 = look_back(tw.flags, g0, min(x0.t, g0), lane, st_acc + 8);
#else
                p0 = look_back(tw.flags, g0, min(x0.t, g0), lane);
#endif
                if (lane == 0) flag_store(tw.flags + g0, kFlagInc | (p0 + agg0));
            }
            if (live0 && x0.cont_out && lane == 0) tw.carry[(tw.pass + 1u) & 1u] = p0 + agg0;  // for the next pass
            if (lane == 0) {
                word[1] = p0;
                word[0] = tile_take(tw);
            }
        }
        __syncthreads();
        prefix0 = word[1];
        g2 = word[0];
    };
    auto publish1 = [&](uint32_t agg1) {
        if (tid == 0) {  // publish g1 at once: inclusive for a document's first tile
            if (x1.bad) {
                atomicOr(wk.status, kErrWorkspace);
                flag_store(tw.flags + g1, kFlagInc);
            } else if (x1.cont_in) {  // first tile of this pass, its document begun in the previous one
                flag_store(tw.flags + g1, kFlagInc | (carry_in + agg1));
            } else {
                flag_store(tw.flags + g1, (x1.t == 0 ? kFlagInc : kFlagAgg) | agg1);
            }
        }
    };
    for (;;) {
        const bool have1 = g1 < total, have0 = g0 < total;
        uint32_t agg1 = 0, prefix0 = 0, g2 = total;
        if (have1) {
            agg1 = tile_front<NT, IPT>(sm[buf], x1, rg, R, tid, err);
            publish1(agg1);
        }
        STAMP(1)
        resolve0(prefix0, g2);
        STAMP(3)
        TileGeo x2{};
        // g2's loads overlap g0's stores; issued even past the end (a tile marked
        // bad: dummy loads only), so their number never depends on the path
        if (g2 < total) x2 = tile_geo(A, tw, g2);
        else x2.bad = true;
        tile_issue<NT, IPT>(A, B, x2, tid, tw.desc, rg);
        STAMP(4)
        tile_stores<NT, IPT, EXCH, NTS, ALIGN>(sm[buf ^ 1], x0, !have0, prefix0, agg0, R, tid, o1, o2);
        if (!have1 && g2 >= total) break;  // (g2 >= total whenever g1 is: the dispenser only grows)
        __syncthreads();
        STAMP(5)
        g0 = g1;
        x0 = x1;
        agg0 = agg1;
        g1 = g2;
        x1 = x2;
        buf ^= 1u;
    }
    STAMP_FLUSH
    if (__syncthreads_or(err != 0) && tid == 0) atomicOr(wk.status, kErrActorRange);
}

// Pass 0 of a call, and its later passes under their own name: a call whose
// tiles the host cannot count (an _async call) launches passes up to a bound,
// and the later ones usually return at once -- kept apart in kernel traces and
// counter means, the first pass's figures stay those of the call's tiles.
// (waves_per_eu(6) is met by the default shape, 512 x 2; the other shapes' LDS
// holds them below it, which the compiler reports as a failed occupancy target)
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Wpass-failed"
template <int NT, int IPT, bool EXCH, bool NTS, bool ALIGN>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(6))) void join_tile_pipe_kernel(
    BatchView A, BatchView B, OutView o1, OutView o2, TileWork tw, Work wk) {
    tile_pipe_body<NT, IPT, EXCH, NTS, ALIGN>(A, B, o1, o2, tw, wk);
}
template <int NT, int IPT, bool EXCH, bool NTS, bool ALIGN>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(6))) void join_tile_pipe_later_kernel(
    BatchView A, BatchView B, OutView o1, OutView o2, TileWork tw, Work wk) {
    tile_pipe_body<NT, IPT, EXCH, NTS, ALIGN>(A, B, o1, o2, tw, wk);
}
#pragma clang diagnostic pop

// Tile shapes (workgroup size x positions per thread); "join_tile_shape".
template <int NT, int IPT, bool NTS>
static hipError_t launch_tile_kernel_s(const BatchView& A, const BatchView& B, const OutView& o1, const OutView* o2,
                                       const Work& wk, const TileWork& tw, uint32_t n_cu, hipStream_t stream) {
    static int per_cu = 0;  // resident workgroups per CU (occupancy query, once per shape)
    if (per_cu == 0) {
        int nb = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, join_tile_kernel<NT, IPT, true, NTS>, NT, 0) !=
                hipSuccess ||
            nb < 1)
            nb = 1;
        per_cu = nb;
    }
    const dim3 grid(n_cu * per_cu);
    if (o2)
        hipLaunchKernelGGL((join_tile_kernel<NT, IPT, true, NTS>), grid, dim3(NT), 0, stream, A, B, o1, *o2, tw,
                           wk);
    else
        hipLaunchKernelGGL((join_tile_kernel<NT, IPT, false, NTS>), grid, dim3(NT), 0, stream, A, B, o1, o1, tw,
                           wk);
    return hipGetLastError();
}

template <int NT, int IPT, bool NTS, bool ALIGN>
static hipError_t launch_tile_pipe_s(const BatchView& A, const BatchView& B, const OutView& o1, const OutView* o2,
                                     const Work& wk, const TileWork& tw, uint32_t n_cu, hipStream_t stream) {
    static int per_cu = 0;  // resident workgroups per CU (occupancy query, once per shape)
    if (per_cu == 0) {
        int nb = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, join_tile_pipe_kernel<NT, IPT, true, NTS, ALIGN>, NT, 0) !=
                hipSuccess ||
            nb < 1)
            nb = 1;
        per_cu = nb;
    }
    const dim3 grid(n_cu * per_cu);
    if (tw.pass == 0 && o2)
        hipLaunchKernelGGL((join_tile_pipe_kernel<NT, IPT, true, NTS, ALIGN>), grid, dim3(NT), 0, stream, A, B, o1, *o2, tw,
                           wk);
    else if (tw.pass == 0)
        hipLaunchKernelGGL((join_tile_pipe_kernel<NT, IPT, false, NTS, ALIGN>), grid, dim3(NT), 0, stream, A, B, o1, o1, tw,
                           wk);
    else if (o2)
        hipLaunchKernelGGL((join_tile_pipe_later_kernel<NT, IPT, true, NTS, ALIGN>), grid, dim3(NT), 0, stream, A, B, o1,
                           *o2, tw, wk);
    else
        hipLaunchKernelGGL((join_tile_pipe_later_kernel<NT, IPT, false, NTS, ALIGN>), grid, dim3(NT), 0, stream, A, B, o1,
                           o1, tw, wk);
    return hipGetLastError();
}

template <int NT, int IPT, bool ALIGN = false>
static hipError_t launch_tile_pipe(const BatchView& A, const BatchView& B, const OutView& o1, const OutView* o2,
                                   const Work& wk, const TileWork& tw, uint32_t n_cu, hipStream_t stream) {
    return tw.nt_stores ? launch_tile_pipe_s<NT, IPT, true, ALIGN>(A, B, o1, o2, wk, tw, n_cu, stream)
                        : launch_tile_pipe_s<NT, IPT, false, ALIGN>(A, B, o1, o2, wk, tw, n_cu, stream);
}

template <int NT, int IPT>
static hipError_t launch_tile_kernel(const BatchView& A, const BatchView& B, const OutView& o1, const OutView* o2,
                                     const Work& wk, const TileWork& tw, uint32_t n_cu, hipStream_t stream) {
    return tw.nt_stores ? launch_tile_kernel_s<NT, IPT, true>(A, B, o1, o2, wk, tw, n_cu, stream)
                        : launch_tile_kernel_s<NT, IPT, false>(A, B, o1, o2, wk, tw, n_cu, stream);
}

uint32_t tile_positions(uint32_t shape) {
    switch (shape) {
        case 1: return 256 * 4;
        case 2: return 256 * 8;
        case 3: return 1024 * 2;
        case 4: return 256 * 4;  // pipelined look-back (join_tile_pipe_kernel)
        case 5: return 512 * 2;
        case 6: return 256 * 8;
        case 7: return 128 * 8;
        case 8: return 256 * 4;  // aligned store windows
        case 9: return 512 * 2;
        case 10: return 256 * 2;  // aligned store windows, half tiles (six workgroups per CU by LDS)
        default: return 512 * 4;
    }
}

// Launch the tile path for the worklist the wave kernel filled.  n_cu sizes the
// persistent grid.  out2 != nullptr: exchange.
static hipError_t launch_tile_pass(const BatchView& A, const BatchView& B, const OutView& o1, const OutView* o2,
                                   const Work& wk, const TileWork& tw, uint32_t n_cu, hipStream_t stream) {
    hipLaunchKernelGGL((tile_split_kernel<256>), dim3(n_cu * tw.split_bpc), dim3(256), 0, stream, A, B, wk, tw);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(tile_geo_kernel, dim3(n_cu * 4), dim3(256), 0, stream, A, B, tw);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    switch (tw.shape) {
        case 1: return launch_tile_kernel<256, 4>(A, B, o1, o2, wk, tw, n_cu, stream);
        case 2: return launch_tile_kernel<256, 8>(A, B, o1, o2, wk, tw, n_cu, stream);
        case 3: return launch_tile_kernel<1024, 2>(A, B, o1, o2, wk, tw, n_cu, stream);
        case 4: return launch_tile_pipe<256, 4>(A, B, o1, o2, wk, tw, n_cu, stream);
        case 5: return launch_tile_pipe<512, 2>(A, B, o1, o2, wk, tw, n_cu, stream);
        case 6: return launch_tile_pipe<256, 8>(A, B, o1, o2, wk, tw, n_cu, stream);
        case 7: return launch_tile_pipe<128, 8>(A, B, o1, o2, wk, tw, n_cu, stream);
        case 8: return launch_tile_pipe<256, 4, true>(A, B, o1, o2, wk, tw, n_cu, stream);
        case 9: return launch_tile_pipe<512, 2, true>(A, B, o1, o2, wk, tw, n_cu, stream);
        case 10: return launch_tile_pipe<256, 2, true>(A, B, o1, o2, wk, tw, n_cu, stream);
        default: return launch_tile_kernel<512, 4>(A, B, o1, o2, wk, tw, n_cu, stream);
    }
}

// The plan, then tw.passes passes of at most tw.cap tiles each (split, geometry,
// tile kernel): a call's tiles need no workspace beyond one pass, and a pass
// may end inside a document (tw.carry hands its placed count on).  Passes past
// the call's tiles return at once; more tiles than tw.passes * tw.cap set
// tw.fallback and leave the worklist to the block kernel.
hipError_t launch_join_tiles(const BatchView& A, const BatchView& B, const OutView& o1, const OutView* o2,
                             const Work& wk, const TileWork& tw_in, uint32_t n_cu, hipStream_t stream) {
    TileWork tw = tw_in;
    // every dispenser shard needs a resident workgroup (tile_take); the
    // persistent grid has n_cu x occupancy >= n_cu of them
    tw.shards = max(1u, min(tw.shards, n_cu));
    const uint32_t n_runs = (A.n_docs + kRun - 1) / kRun;
    hipLaunchKernelGGL((tile_count_kernel<256>), dim3(min(n_runs, 2048u)), dim3(256), 0, stream, A, B, wk, tw);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((tile_scan_kernel<1024>), dim3(1), dim3(1024), 0, stream, A.n_docs, wk, tw);
    e = hipGetLastError();
    for (uint32_t p = 0; p < tw.passes && e == hipSuccess; ++p) {
        tw.pass = p;
        e = launch_tile_pass(A, B, o1, o2, wk, tw, n_cu, stream);
    }
    return e;
}

}  // namespace crdt

#ifdef CRDT_STAMPS
// Diagnostic builds only (Makefile target "stamps"): the tile kernel's phase
// cycles summed over waves, read and optionally cleared.
extern "C" int crdt_probe_tile_stamps(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(crdt::g_stamps), 16 * sizeof(unsigned long long)) != hipSuccess) return -1;
    if (reset) {
        static const unsigned long long z[16] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(crdt::g_stamps), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif
