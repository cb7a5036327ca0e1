// Ordered fold of source states into each document:
//   out[d] = (((dst[d] <- src[d][0]) <- src[d][1]) ... )
// mode CRDT_FOLD_AWSET : each step is (*AWSet).Merge        awset.go:103-161
// mode CRDT_FOLD_DELTA : each step is (*AWSetDelta).Merge   awset-delta_test.go:51-166
//   path select  Counter(src.Actor) == 0 -> full merge, src.Deleted ignored (:53-56)
//   otherwise    changed = src entries dst's clock has not seen, deleted =
//                tombstones not re-added (:79-105); both empty -> nothing,
//                not even the VV merge (:60); else deltaMerge (:107-166).
// Steps into one document are applied in order: the
// document stays on chip for the whole fold and is written to HBM once.
//
//  * fold_pipe_kernel: one wavefront per run of K consecutive documents, while
//    a document + its source entries + tombstones fit 256 tuples (<= 64
//    sources, sources x R <= 256 clock words).  The fold is replayed per key
//    (below), not per step, and the next document's loads are in flight while
//    the current one is folded.
//  * fold_block_kernel: every other document (worklist); persistent
//    workgroups, merge-path walk per step (merge_block.hpp), ping-pong
//    between the output slots and a scratch copy.
#include "crdt_device.hpp"
#include "merge_block.hpp"
#include "wave_sort.hpp"

namespace crdt {

// ---- build options (tools/fold_probe.hip timing builds override them) ----
// Measured on config 3 / 5 with timing builds, three interleaved rounds each,
// outputs checksummed equal (round 4):
//  * CRDT_FOLD_PAD_VALU / _SALU = 200 (diagnostic: 200 dependent VALU or SALU
//    instructions per document): +8 % / +7 % on config 3, +20 % / +26 % on
//    config 5 -- config 5 (6 waves per SIMD) is near issue-bound, config 3
//    (4 waves per SIMD) is bound by its per-document dependent chain;
//  * CRDT_FOLD_PURE_CHUNKS (buffer loads for a chunk inside one region instead
//    of per-lane pointer selects): no change (-0.5 % / +1 %), off;
//  * branch-free slot walks (every lane issues the atomics and reads, no
//    per-lane branch): +8 % / +5 %, dropped; branch-free staging (below): -2 %
//    on config 5, kept;
//  * CRDT_FOLD_LDS_PAD (diagnostic: LDS padding, fewer waves per CU): config 3
//    16 -> 14 -> 12 waves per CU costs +9 % / +35 %, config 5 24 -> 22 -> 16
//    costs +9 % / +18 % -- both folds scale with resident waves, i.e. they are
//    bound by each document's dependent chain, not by bytes or issue;
//  * more waves by squeezing registers: the lean delta pass at 5 waves per SIMD
//    (95 VGPRs, 40 spilled) +59 %, the lean AWSet pass at 7 (72 VGPRs) +13 %;
//    counters and clocks staged as u32 (half the LDS of tc / vs / svv, the
//    documents with a word >= 2^32 deferred) +2.5 % at the same occupancy;
//    dropped;
//  * the lean passes defer > 15 sources before their prefetch and keep no
//    registers for words they never load (the second offset chunk, the lean
//    AWSet pass's second clock chunk): config 5 -1.5 %, kept; the lean AWSet
//    pass then fits 7 waves per SIMD in 72 VGPRs (3 spilled): another -0.5 %,
//    within noise, not taken;
//  * the lean delta pass's survivors written per slot quad inside the walk (no
//    Emit registers) with u32 staging: 128 -> 109 VGPRs, but +7.5 % at 4 waves
//    per SIMD, and at 5 waves (96 VGPRs, 3 spilled) still +5.6 % on config 3
//    (+3 % config 5); dropped;
//  * tombstone check by reading a short source's <= 8 entries at once instead
//    of binary-search probes: +8 % on config 3 (one VGPR spills); the source
//    actors kept in a register instead of re-read from LDS: no change; dropped;
//  * CRDT_FOLD_NOFULL_PASS: a delta document with no full step (every step a
//    delta) walks its slots once -- the entry/add/drop time words and the last
//    entry row in one pass, one wave barrier fewer in the chain: config 3
//    1.87 -> 1.81 ms (-3.7 %), config 5 unchanged, on (profiles/r04y_*);
//  * the per-step "has a changed entry / an effective tombstone" flags OR-ed
//    over the wave with DPP instead of written to LDS and read back: no change
//    (within 0.3 %), kept as the simpler form;
//  * tuple loads by region (one descriptor per region and array, the regions'
//    zero-filled out-of-range loads OR-ed): +30 % on both -- three times the
//    load instructions of a straddling chunk, plus spills; dropped.  HasDot of
//    every source tuple computed in the classify pass (the walk then reads no
//    clocks): +0.5 %, dropped.  8 more (out-of-range) store instructions per
//    document: +0.7 % config 3, +7 % config 5 -- config 3 is not bound by its
//    memory-instruction count;
//  * CRDT_FOLD_STAGE_STORES 2 (survivors staged by slot in LDS, then 16-byte
//    stores: 5 store instructions a document instead of 12; the range check
//    drops each dword past the last survivor, tools/buf_probe):
//    -1.8 % config 3, +2.5 % config 5 (profiles/r04z_fold_variants.log), off;
//  * CRDT_FOLD_PTAB (the prefetch reads its region's base pointers from a
//    12-entry LDS table instead of a 3-way select of scalar pointers: 330
//    fewer static VALU in the lean delta kernel): -1.8 % config 3, +0.9 %
//    config 5; on for the delta folds only;
//  * CRDT_FOLD_IDX32 (the AWSet prefetch selects 32-bit slot indices and knows
//    it has no tombstone region: no exec-masked 64-bit arithmetic; -74 static
//    VALU, -33 SALU): config 5 -3 % (noisy), on;
//  * CRDT_FOLD_CLASSIFY_UNIFORM (chunk-uniform guards + predicated per-lane
//    entry / tombstone checks in the delta classify, -80 static SALU): +1.3 %
//    on config 3, off.  PMC of the lean delta pass at HEAD: 691 VALU, 485 SALU,
//    97 LDS instructions a document (round 3: 837 / 533 / 104;
//    profiles/r04c3_pmc_summary.txt);
//  * documents per wave (CRDT_FOLD_K_DELTA / CRDT_FOLD_K) 8 / 16 and 24 / 48
//    against 16 / 32: equal or slower on both configs, 16 / 32 kept (round 4);
//    with the fused delta walk (round 6, profiles/r06zj_fold_docs_per_wave.log,
//    three interleaved rounds each): delta 8 and 6 -1.3-1.9 %, 4 +1.2 %, 12
//    -0.4 % against 16 -- 8 kept; AWSet 16 / 24 against 32 within noise, 32 kept.
// 1: survivors staged through LDS and written as contiguous lines -- measured
// 4 % slower on config 3 and 5 % on config 5 (tools/fold_probe.hip timing
// builds, three interleaved rounds), so off: each lane stores its own
// survivors at their slots.  (CRDT_FOLD_NO_STORES, a diagnostic bound that
// writes nothing, is only 4 % faster: the folds are not bound by their stores.)
#ifndef CRDT_FOLD_STAGE_STORES
#define CRDT_FOLD_STAGE_STORES 0
#endif
#ifndef CRDT_FOLD_NO_STORES
#define CRDT_FOLD_NO_STORES 0
#endif
// diagnostic bounds (timing builds only): no per-document fold / no loads after the first document
#ifndef CRDT_FOLD_DIAG_NOCOMPUTE
#define CRDT_FOLD_DIAG_NOCOMPUTE 0
#endif
#ifndef CRDT_FOLD_DIAG_NOLOAD
#define CRDT_FOLD_DIAG_NOLOAD 0
#endif
#ifndef CRDT_FOLD_DIAG_SKIP_CLASSIFY  // diagnostic: no classify pass (keys read, nothing kept but the document)
#define CRDT_FOLD_DIAG_SKIP_CLASSIFY 0
#endif
#ifndef CRDT_FOLD_DIAG_SKIP_WALK  // diagnostic: no slot walk (nothing written)
#define CRDT_FOLD_DIAG_SKIP_WALK 0
#endif
// CRDT_FOLD_PAD_STORES (with CRDT_FOLD_STAGE_STORES 1, diagnostic): each array's
// staged stores run on to the end of the last survivor's cache line, within
// the document's output capacity (slack past the live count is unspecified),
// so no output line is written partially.
#ifndef CRDT_FOLD_PAD_STORES
#define CRDT_FOLD_PAD_STORES 0
#endif
#ifndef CRDT_FOLD_PURE_CHUNKS
#define CRDT_FOLD_PURE_CHUNKS 0
#endif
#ifndef CRDT_FOLD_AWSET_ONE_ROUND
#define CRDT_FOLD_AWSET_ONE_ROUND 1
#endif
#ifndef CRDT_FOLD_CLASSIFY_UNIFORM
#define CRDT_FOLD_CLASSIFY_UNIFORM 0
#endif
#ifndef CRDT_FOLD_IDX32
#define CRDT_FOLD_IDX32 1
#endif
#ifndef CRDT_FOLD_PTAB
#define CRDT_FOLD_PTAB 1
#endif
#ifndef CRDT_FOLD_NOFULL_PASS
#define CRDT_FOLD_NOFULL_PASS 1
#endif
#ifndef CRDT_FOLD_LDS_PAD
#define CRDT_FOLD_LDS_PAD 0
#endif
// CRDT_FOLD_GLOBAL_PTAB: the PTAB prefetch's tuple loads through global-address-
// space pointers (global_load) instead of generic ones (flat_load, which also
// counts in lgkmcnt: every LDS wait of the fold then waited for the prefetch).
#ifndef CRDT_FOLD_GLOBAL_PTAB
#define CRDT_FOLD_GLOBAL_PTAB 1
#endif
// CRDT_FOLD_TOMB_TAB: the delta classify's "re-added in the same source" check
// (awset-delta_test.go:93-102) through a per-low-key-byte step bitmap, searching
// the source's entries only on a possible hit (see the classify pass).
#ifndef CRDT_FOLD_TOMB_TAB
#define CRDT_FOLD_TOMB_TAB 1
#endif
// CRDT_FOLD_FUSED: the lean delta pass's documents with no full step classified
// and walked in one pass (fused_delta_walk)
#ifndef CRDT_FOLD_LIST_SPREAD
#define CRDT_FOLD_LIST_SPREAD 1  // 0: the deferred list in runs of K (A/B builds)
#endif
#ifndef CRDT_FOLD_XCD_MAP
#define CRDT_FOLD_XCD_MAP 1  // XCD-contiguous document ranges: 0 none, 1 AWSet lean pass, 2 both lean passes
#endif
#ifndef CRDT_FOLD_FUSED
#define CRDT_FOLD_FUSED 1
#endif
// pointer to global (address space 1) memory
template <typename T>
using gptr = const T __attribute__((address_space(1)))*;
#ifndef CRDT_FOLD_PAD_VALU
#define CRDT_FOLD_PAD_VALU 0
#endif
#ifndef CRDT_FOLD_PAD_SALU
#define CRDT_FOLD_PAD_SALU 0
#endif
#ifndef CRDT_FOLD_PAD_VMEM
#define CRDT_FOLD_PAD_VMEM 0
#endif

// ---- the fold restated per key ---------------------------------------------
// A key's fate over the whole fold depends only on its own tuples (its dot in
// the document, its entry in each source, its tombstone in each source) and on
// three per-step facts of the document: V_j, the clock before step j; full_j,
// the awset path (or Counter(src.Actor) == 0, awset-delta_test.go:53); noop_j,
// a delta step with nothing changed and nothing deleted (:60, no VV merge).
//
// Schedule.  U_j = V_0 max svv_0 max ... max svv_{j-1} (a prefix max, one lane
// per actor) equals V_j as long as no step is a no-op: if no step is a no-op
// under U, then by induction on j every V_j = U_j, so full_j, the changed bits
// and every clock computed from U are the exact ones.  Otherwise (rare: a
// delta that brings nothing) the steps are replayed one at a time.
//
// Per document, one wavefront:
//   stage     the tuples (loaded while the previous document was folded) -> LDS
//   schedule  U_j, full_j; changed entries and effective tombstones; no-op check
//   keep      the tuples that can act on their key (document entries, entries
//             of full steps, changed entries and effective tombstones of delta
//             steps), tagged (step, kind), ballot-compacted
//   group     a bitonic network over (key, tag) in registers (wave_sort.hpp:
//             DPP and permlane lane exchanges, no LDS)
//   walk      one lane per distinct key replays its events in step order (its
//             tuples and, while present, every full step, whose phase 2 may
//             remove it: awset.go:147-158)
//   write     the survivors, already in key order, ballot-compacted.  Every
//             store is issued unconditionally (out-of-range offsets where there
//             is nothing to write), so the count of memory operations after the
//             next document's prefetch is fixed and its wait is an exact vmcnt.
// Waves per SIMD: the delta fold needs 168 VGPRs (3 waves); the AWSet fold
// fits 128 (4 waves), which also needs its LDS trimmed to 16 waves per CU
// (160 KiB): 224 clock words per document instead of 256.
#ifndef CRDT_FOLD_DELTA_WPE
#define CRDT_FOLD_DELTA_WPE 3  // probe builds may override (tools/fold_probe.hip)
#endif
#ifndef CRDT_FOLD_AWSET_WPE
#define CRDT_FOLD_AWSET_WPE 5  // 96 VGPRs: 3 loop-invariant values spill (measured 11 % faster than 4)
#endif
// NCH: 64-tuple chunks a document may fill on this path (AWSet folds: 128
// tuples -- fewer registers for the prefetch and the walk, so the kernel fits
// 128 VGPRs with no spills; larger documents take the block kernel).  VCH:
// 64-word chunks of source clocks.
//
// LEAN (delta folds): the pass that resolves a document only by the slot walk
// (dense_delta_walk) -- no sort paths, so 128 VGPRs and 192 clock words: 4 waves
// per SIMD.  A document it cannot walk (key span >= 256, > 15 sources, an
// actor == len(VV), or beyond its tuple / clock capacity) is deferred, untouched,
// to the general kernel, which takes the deferred list (LIST) afterwards.
// The AWSet fold has a lean pass too (dense_awset_walk only).
#ifndef CRDT_FOLD_LEAN_WPE
#define CRDT_FOLD_LEAN_WPE 4
#endif
#ifndef CRDT_FOLD_AWSET_LEAN_WPE
#define CRDT_FOLD_AWSET_LEAN_WPE 6
#endif
template <bool DELTA, bool LEAN = false>
struct FoldShape {
    static constexpr int WPE = LEAN ? (DELTA ? CRDT_FOLD_LEAN_WPE : CRDT_FOLD_AWSET_LEAN_WPE)
                                    : (DELTA ? CRDT_FOLD_DELTA_WPE : CRDT_FOLD_AWSET_WPE);
    static constexpr int NCH = DELTA ? 4 : 2;
    // the lean AWSet pass stages one chunk of clock words (sources x R <= 64;
    // config 5: 7 x 8): two fewer prefetch registers
    static constexpr int VCH = (LEAN && DELTA) ? 3 : (DELTA ? 4 : (LEAN ? 1 : 2));
    static constexpr int VCAP =
        (LEAN && DELTA) ? 192 : ((DELTA && CRDT_FOLD_DELTA_WPE < 4) ? 256 : (DELTA ? 224 : (LEAN ? 64 : 128)));
};

template <int VCAP_, int NCAP_>
struct alignas(16) FoldSmem {
    static constexpr int NCAP = NCAP_;  // document entries + source entries + tombstones
    static constexpr int VCAP = VCAP_;  // sources x R clock words
    static constexpr int MCAP = 64;   // sources per document
    uint64_t tk[NCAP];        // tuple keys; compacted kept keys; after the sort: segment keys
    uint64_t tc[NCAP];        // tuple counters
    uint64_t vs[VCAP];        // V_j (j < M), R words each
    uint64_t svv[VCAP];       // source clocks, R words each
    uint32_t ta[NCAP];        // tuple actors
    uint32_t soff[MCAP + 1];  // source entry ranges, relative to the first source
    uint32_t sact[MCAP];      // source actors (AWSetDelta.Actor)
    // 8-byte aligned: the AWSet walk keeps 64-bit slot masks here, updated
    // with 64-bit LDS atomics, which fault on a misaligned address
    alignas(16) uint16_t stag[NCAP];  // kept tuples' tags
    uint8_t anye[MCAP];              // the prefetch's per-region base table (CRDT_FOLD_PTAB: 12 x 8 bytes
    uint8_t anyt[MCAP];              //  over both; dead during a fold, whose walk tables reach over them)
    alignas(4) uint8_t smark[NCAP];  // s + 1 where source s's entries / tombstones end (step of a tuple)
    alignas(8) uint16_t dbase[256];  // dense_sort: first sorted position of each key slot (64-bit stores)
#if CRDT_FOLD_LDS_PAD
    uint8_t pad[CRDT_FOLD_LDS_PAD];  // diagnostic builds: fewer waves per CU by LDS (occupancy slope)
#endif
};

// The members reached by 64-bit LDS accesses (atomics on stag, stores on
// dbase, u64 arrays) must sit on 8-byte boundaries for every shape in use.
template <int V, int N>
constexpr bool fold_smem_aligned() {
    using S = FoldSmem<V, N>;
    return offsetof(S, tk) % 8 == 0 && offsetof(S, tc) % 8 == 0 && offsetof(S, vs) % 8 == 0 &&
           offsetof(S, svv) % 8 == 0 && offsetof(S, stag) % 8 == 0 && offsetof(S, dbase) % 8 == 0 &&
           offsetof(S, anye) % 8 == 0 && offsetof(S, anyt) == offsetof(S, anye) + S::MCAP && 2 * S::MCAP >= 96 &&
           alignof(S) >= 8;
}
// (checked where each kernel instantiates its shape, fold_pipe_kernel)

// A value every lane must load: consumed by an empty asm, so the compiler
// cannot sink its (LDS) load into an exec-masked block of the lanes that use it.
__device__ __forceinline__ uint64_t issued(uint64_t v) {
    asm volatile("" : "+v"(v));
    return v;
}
__device__ __forceinline__ uint32_t issued(uint32_t v) {
    asm volatile("" : "+v"(v));
    return v;
}

// Tuple tag: bits 15..8 = 0 for a document entry, (j+1)*2 for an entry of
// source j, (j+1)*2+1 for its tombstone; bits 7..0 = tuple index in LDS.  The
// sort order (key, tag) puts a key's tuples in replay order.
constexpr uint32_t kPadTag = 0xFFFFu;

// A document's survivors, at most 4 per lane, in key order: element q of this
// lane goes to output position off[q] (kOOB: nothing to write).
template <int NQ>
struct Emit {
    uint64_t k[NQ], c[NQ];
    uint32_t a[NQ], off[NQ];
};

// Resolve every key of the document at once, element-parallel.  After the sort
// a key's kept tuples are consecutive, in replay order (document entry, then by
// step, an entry before its step's tombstone).  Each tuple acts on the key's
// presence as a constant or the identity:
//   document entry                     present (dot := its own)
//   entry of a full step     (awset.go:122-143) present if the clock before the
//                            step lacks it, else unchanged (dot := its own)
//   changed entry, delta step (awset-delta_test.go:126-147) present (dot := own)
//   effective tombstone      (:149-164) absent if the clock before the step
//                            lacks it, else unchanged (dot unchanged)
// and between a tuple and the key's next one (or the end), every full step
// whose source clock has seen the current dot removes it (awset.go:147-158).
// The current dot is the last entry's, whatever the presence, so it is one
// segmented scan; with the gap folded in, each tuple is again constant or
// identity, and the final presence is the last constant: a second scan.
// Wave reductions over u32 lanes (DPP row shifts and broadcasts; lanes with no
// source take the identity); every lane gets the result.
template <bool MAX>
__device__ __forceinline__ uint32_t wave_minmax(uint32_t x) {
    const uint32_t id = MAX ? 0u : ~0u;
    auto op = [](uint32_t a, uint32_t b) { return MAX ? max(a, b) : min(a, b); };
    x = op(x, dpp<0x111>(id, x));       // row_shr:1
    x = op(x, dpp<0x112>(id, x));       // row_shr:2
    x = op(x, dpp<0x114>(id, x));       // row_shr:4
    x = op(x, dpp<0x118>(id, x));       // row_shr:8
    x = op(x, dpp<0x142, 0xA>(id, x));  // row_bcast:15
    x = op(x, dpp<0x143, 0xC>(id, x));  // row_bcast:31
    return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}

// OR of a u64 over every lane (DPP scan; every lane gets the result).
__device__ __forceinline__ uint64_t wave_or64(uint64_t v) {
    uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    lo |= dpp<0x111>(0u, lo);
    hi |= dpp<0x111>(0u, hi);
    lo |= dpp<0x112>(0u, lo);
    hi |= dpp<0x112>(0u, hi);
    lo |= dpp<0x114>(0u, lo);
    hi |= dpp<0x114>(0u, hi);
    lo |= dpp<0x118>(0u, lo);
    hi |= dpp<0x118>(0u, hi);
    lo |= dpp<0x142, 0xA>(0u, lo);
    hi |= dpp<0x142, 0xA>(0u, hi);
    lo |= dpp<0x143, 0xC>(0u, lo);
    hi |= dpp<0x143, 0xC>(0u, hi);
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)hi, 63) << 32) |
           (uint32_t)__builtin_amdgcn_readlane((int)lo, 63);
}

// Inclusive prefix sum over lanes (DPP).
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t x) {
    x += dpp<0x111>(0u, x);
    x += dpp<0x112>(0u, x);
    x += dpp<0x114>(0u, x);
    x += dpp<0x118>(0u, x);
    x += dpp<0x142, 0xA>(0u, x);
    x += dpp<0x143, 0xC>(0u, x);
    return x;
}

// Counting sort of the kept (key, tag) pairs, used instead of the bitonic
// network when the document's kept keys span fewer than 256 ids and every
// tag's step field (tag >> 8) is below 32 -- the common case for keys
// interned per document (host/crdt.hpp: ranks, or the generator's dense ids).
// ev[s] = the set of step fields present at key slot s (keys of one document
// are distinct per state, so a (slot, step field) pair occurs once); a pair's
// sorted position is the exclusive prefix over slots of popc(ev) plus its rank
// in its slot's mask, which is (key, tag) order.  Scratch aliases tk, stag and
// smark, all dead once k / t are in registers.  Returns false (nothing
// changed) when the document does not qualify.
template <int EPL, class Smem>
__device__ __forceinline__ bool dense_sort(Smem& m, uint64_t (&k)[EPL], uint32_t (&t)[EPL], uint32_t n,
                                           uint32_t lane) {
    if (n == 0) return true;
    const uint64_t b = readlane64(k[0], 0);  // element 0 is valid
    bool bad = false;
    uint32_t lo = ~0u, hi = 0u;
#pragma unroll
    for (int q = 0; q < EPL; ++q) {
        const bool valid = lane * EPL + q < n;
        const uint64_t d = k[q] - b + 0x80000000ull;  // biased: u32 order = signed offset order
        bad |= valid && ((d >> 32) != 0 || (t[q] >> 8) >= 32u);
        lo = valid ? min(lo, (uint32_t)d) : lo;
        hi = valid ? max(hi, (uint32_t)d) : hi;
    }
    if (ballot(bad)) return false;
    lo = wave_minmax<false>(lo);
    hi = wave_minmax<true>(hi);
    if (hi - lo >= 256u) return false;
    uint32_t* ev = reinterpret_cast<uint32_t*>(m.tk);
    uint16_t* base = m.dbase;
    // slot and step field are recomputed from k / t where needed (no extra
    // registers live across the sort: the AWSet fold runs at 128 VGPRs)
    const uint64_t bs = b - 0x80000000ull + uniform(lo);  // key of slot 0
    static_assert(sizeof(m.tk) >= 1024, "dense_sort: tk holds the 256 slot masks");
    ev[lane] = 0u;
    ev[64 + lane] = 0u;
    ev[128 + lane] = 0u;
    ev[192 + lane] = 0u;
    wave_sync();
#pragma unroll
    for (int q = 0; q < EPL; ++q)
        if (lane * EPL + q < n) atomicOr(&ev[(uint32_t)(k[q] - bs) & 255u], 1u << ((t[q] >> 8) & 31u));
    wave_sync();
    const uint4 e4 = reinterpret_cast<const uint4*>(ev)[lane];
    const uint32_t c0 = __popc(e4.x), c1 = __popc(e4.y), c2 = __popc(e4.z), c3 = __popc(e4.w);
    const uint32_t tot = c0 + c1 + c2 + c3;
    const uint32_t pre = wave_incl_sum(tot) - tot;
    reinterpret_cast<ushort4*>(base)[lane] =
        make_ushort4((uint16_t)pre, (uint16_t)(pre + c0), (uint16_t)(pre + c0 + c1), (uint16_t)(pre + c0 + c1 + c2));
    wave_sync();
#pragma unroll
    for (int q = 0; q < EPL; ++q) {
        if (lane * EPL + q < n) {
            const uint32_t sl = (uint32_t)(k[q] - bs) & 255u;
            const uint32_t pos = base[sl] + __popc(ev[sl] & ((1u << ((t[q] >> 8) & 31u)) - 1u));
            m.stag[pos] = (uint16_t)t[q];
            m.smark[pos] = (uint8_t)sl;
        }
    }
    wave_sync();
#pragma unroll
    for (int q = 0; q < EPL; ++q) {
        const uint32_t i = lane * EPL + q;
        const bool valid = i < n;
        t[q] = valid ? (uint32_t)m.stag[i] : kPadTag;
        k[q] = valid ? bs + m.smark[i] : ~0ull;
    }
    return true;
}

// The AWSet fold (every step a full (*AWSet).Merge, awset.go:107-161)
// resolved per key slot when the document's keys span fewer than 64 ids and it
// has at most 15 sources: lane s owns key kmin + s.  The reference's rule, one
// key at a time, over the steps in order:
//   key in source j:  present -> dot := the source's dot (awset.go:123-129,142)
//                     absent  -> added iff !HasDot(V_j, dot) (:133-140)
//   not in source j:  present -> removed iff HasDot(svv_j, dot) (:146-158)
// V_j is the clock before step j (the schedule's prefix max: an AWSet fold has
// no no-op steps).  Rows: row 0 the document, row j + 1 source j.  A key's
// tuples, in row order, each hold the current dot from their row until the
// key's next row; so, per tuple t at row r:
//   add_t  = t is the document's, or !HasDot(V_{r-1}, dot_t)
//   drop_t = HasDot(svv_j, dot_t) for some step j in [r, next row - 1)
// and the key survives iff some tuple has add set and no tuple from the last
// such row on has drop set (an add makes the key present whatever it was
// before; a drop removes it while present; a tuple without add keeps the
// state it finds).  The survivor's dot is its last tuple's.  Each tuple's
// bits are independent, so every check is one lane-parallel LDS read instead
// of a step-by-step chain; the per-slot words (rows, add, drop, last tuple)
// live in tk, dead once the keys are in registers.  Go evaluates HasDot only
// where the step-by-step walk does, and panics at actor == len(VV): a document
// holding such an actor takes that walk instead (dense_awset_walk_seq), so
// the reference's panics are flagged exactly.  Survivors come out in slot =
// key order, one store round.  Returns false (nothing changed) when the
// document does not qualify.
template <int NCH, class Smem>
__device__ __forceinline__ void dense_awset_walk_seq(Smem& m, const uint64_t (&key)[NCH], const uint32_t (&step)[NCH],
                                                     uint64_t kb, uint32_t N, uint32_t n, uint32_t ms, uint32_t R,
                                                     uint32_t lane, bool& P, uint32_t& da, uint64_t& dc,
                                                     uint32_t& err) {
    // mask[row] = the slots present in a row, idx[row * 64 + slot] = the tuple
    uint64_t* mask = reinterpret_cast<uint64_t*>(m.stag);
    uint8_t* idx = reinterpret_cast<uint8_t*>(m.tk);
    if (lane <= ms) mask[lane] = 0ull;
    wave_sync();
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
        const uint32_t i = c * 64u + lane;
        if (i < N) {
            const uint32_t sl = (uint32_t)(key[c] - kb) & 63u;
            const uint32_t row = i < n ? 0u : (step[c] & 63u) + 1u;
            atomicOr(reinterpret_cast<unsigned long long*>(&mask[row]), 1ull << sl);
            idx[row * 64u + sl] = (uint8_t)i;
        }
    }
    wave_sync();
    P = (mask[0] >> lane) & 1ull;
    da = 0;
    dc = 0;
    if (P) {
        const uint32_t t = idx[lane];
        da = m.ta[t];
        dc = m.tc[t];
    }
    uint32_t perr = 0;
    for (uint32_t j = 0; j < ms; ++j) {
        const bool has = (mask[j + 1] >> lane) & 1ull;
        if (has) {
            const uint32_t t = idx[(j + 1) * 64u + lane];
            const uint32_t ea = m.ta[t];
            const uint64_t ec = m.tc[t];
            if (!P) {  // src-only: HasDot(dstVV, s), awset.go:133
                perr |= ea == R ? 1u : 0u;
                P = !(ea < R && m.vs[j * R + ea] >= ec);
            }
            da = ea;  // the source's dot wins when present (an absent key's dot is never read)
            dc = ec;
        } else if (P) {  // dst-only: HasDot(srcVV, d), awset.go:152
            perr |= da == R ? 1u : 0u;
            P = !(da < R && m.svv[j * R + da] >= dc);
        }
    }
    if (perr) err |= kErrActorRange;
}

template <int NCH, class Smem>
__device__ __forceinline__ bool dense_awset_walk(Smem& m, const uint64_t (&key)[NCH], const uint32_t (&step)[NCH],
                                                 uint32_t N, uint32_t n, uint32_t ms, uint32_t R, uint32_t lane,
                                                 uint64_t lt, Emit<NCH>& e, uint32_t& U, uint32_t& err) {
    static_assert(sizeof(m.tk) >= 16 * 64 && sizeof(m.stag) >= 16 * 8, "dense_awset_walk: table space");
    if (N == 0 || ms > 15) return false;
    const uint64_t b = readlane64(key[0], 0);  // element 0 is valid
    bool bad = false;
    uint32_t lo = ~0u, hi = 0u;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
        const bool valid = c * 64u + lane < N;
        const uint64_t d = key[c] - b + 0x80000000ull;
        bad |= valid && (d >> 32) != 0;
        lo = valid ? min(lo, (uint32_t)d) : lo;
        hi = valid ? max(hi, (uint32_t)d) : hi;
    }
    if (ballot(bad)) return false;
    lo = wave_minmax<false>(lo);
    hi = wave_minmax<true>(hi);
    if (hi - lo >= 64u) return false;
    const uint64_t kb = b - 0x80000000ull + lo;  // key of slot 0
    uint32_t a[NCH], sl[NCH], row[NCH];
    uint64_t cc[NCH];
    bool anyR = false;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
        const uint32_t i = c * 64u + lane;
        const bool valid = i < N;
        a[c] = m.ta[valid ? i : 0u];
        cc[c] = m.tc[valid ? i : 0u];
        sl[c] = (uint32_t)(key[c] - kb) & 63u;
        row[c] = i < n ? 0u : (step[c] & 63u) + 1u;
        anyR |= valid && a[c] == R;
    }
    bool P;
    uint32_t da;
    uint64_t dc;
    if (ballot(anyR)) {
        dense_awset_walk_seq<NCH>(m, key, step, kb, N, n, ms, R, lane, P, da, dc, err);
    } else {
        uint32_t* rows = reinterpret_cast<uint32_t*>(m.tk);  // [64] rows holding the slot
        uint32_t* addw = rows + 64;                          // [64] rows with add set
        uint32_t* dropw = rows + 128;                        // [64] rows with drop set
        uint8_t* last = reinterpret_cast<uint8_t*>(rows + 192);  // [64] the slot's last tuple
        rows[lane] = 0u;
        addw[lane] = 0u;
        dropw[lane] = 0u;
        wave_sync();
#pragma unroll
        for (int c = 0; c < NCH; ++c)
            if (c * 64u + lane < N) atomicOr(&rows[sl[c]], 1u << row[c]);
        wave_sync();
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            const uint32_t i = c * 64u + lane;
            if (i < N) {
                const uint32_t r = row[c], above = rows[sl[c]] >> (r + 1u);
                const uint32_t nr = above ? r + (uint32_t)__ffs(above) : ms + 1u;  // the key's next row
                const bool cov = a[c] < R;  // actor > R: HasDot false (actor == R: the step walk)
                const bool add = r == 0u || !(cov && m.vs[(r - 1u) * R + (cov ? a[c] : 0u)] >= cc[c]);
                bool drop = false;
                for (uint32_t j = r; j + 1u < nr; j += 4u) {  // four independent clock reads per round
#pragma unroll
                    for (uint32_t u = 0; u < 4u; ++u) {
                        const bool in = cov && j + u + 1u < nr;
                        drop |= in && m.svv[in ? (j + u) * R + a[c] : 0u] >= cc[c];
                    }
                }
                if (add) atomicOr(&addw[sl[c]], 1u << r);
                if (drop) atomicOr(&dropw[sl[c]], 1u << r);
                if (!above) last[sl[c]] = (uint8_t)i;
            }
        }
        wave_sync();
        const uint32_t aw = addw[lane], dw = dropw[lane];
        P = aw != 0u && (dw >> (31u - (uint32_t)__clz(aw))) == 0u;
        da = 0;
        dc = 0;
        if (P) {
            const uint32_t t = last[lane];
            da = m.ta[t];
            dc = m.tc[t];
        }
    }
    const uint64_t pm = ballot(P);
    U = popc(pm);
    e.k[0] = kb + lane;
    e.a[0] = da;
    e.c[0] = dc;
    e.off[0] = P ? below(pm) : kOOB;
#pragma unroll
    for (int q = 1; q < NCH; ++q) {
        e.k[q] = 0;
        e.a[q] = 0;
        e.c[q] = 0;
        e.off[q] = kOOB;
    }
    return true;
}

// The delta fold's kept tuples resolved per key slot, as dense_awset_walk does
// for the AWSet fold, when the keys span fewer than 256 ids (4 slots per lane:
// slot q * 64 + lane) and there are at most 15 sources.  The rule of
// sort_resolve, slot-wise: times 0 (document), 2j + 1 (entry of step j),
// 2j + 2 (tombstone of step j); per kept tuple t
//   document entry        add;  drop = a full step of its gap covers its dot
//   entry, full step j    add iff !HasDot(V_j, dot);  drop as above
//   changed entry, delta  add;  drop as above
//   effective tombstone   drop iff !HasDot(V_j, dot) (awset-delta_test.go:149-164)
// where an entry's gap is the full steps after it up to the key's next entry
// (tombstones do not move the dot; a removal there precedes any later add, so
// attributing it to the entry's time is exact).  The key survives iff some
// tuple adds and none from the last add's time on drops; its dot is the last
// entry's.  Per-slot words: entry times and add times in tk, drop times and the
// last entry in stag..dbase (all dead by now).  A document with a kept tuple of
// actor == len(VV) is left to the sort path (exact panics).
template <class Smem>
__device__ __forceinline__ bool dense_delta_walk(Smem& m, const uint64_t (&key)[4], const uint32_t (&step)[4],
                                                 const bool (&isE)[4], const bool (&isT)[4], uint32_t flag,
                                                 uint64_t full_mask, uint64_t noop_mask, uint32_t N, uint32_t n,
                                                 uint32_t ms, uint32_t R, uint32_t lane, uint64_t lt, Emit<4>& e,
                                                 uint32_t& U STAMP_PARAM) {
    static_assert(sizeof(m.tk) >= 2 * 256 * 4, "dense_delta_walk: entry/add words");
    static_assert(offsetof(Smem, dbase) + sizeof(m.dbase) - offsetof(Smem, stag) >= 256 * 5,
                  "dense_delta_walk: drop words + last entry");
    if (N == 0 || ms > 15) return false;
    bool kept[4];
    uint32_t a[4];
    bool anyR = false, bad = false;
    const uint64_t b = readlane64(key[0], 0);  // element 0 is valid
    uint32_t lo = ~0u, hi = 0u;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        if ((uint32_t)c * 64u >= N) {  // a chunk past the document's tuples (wave-uniform): nothing kept
            kept[c] = false;
            a[c] = 0;
            continue;
        }
        const uint32_t i = c * 64u + lane;
        const uint32_t j = step[c] & 63u;
        const bool fj = (full_mask >> j) & 1ull, nj = (noop_mask >> j) & 1ull, f = (flag >> c) & 1u;
        kept[c] = i < N && ((i < n) || (isE[c] && !nj && (fj || f)) || (isT[c] && !nj && !fj && f));
        a[c] = issued(m.ta[i < N ? i : 0u]);  // every lane: no exec region around the load
        anyR |= kept[c] && a[c] == R;
        const uint64_t d = key[c] - b + 0x80000000ull;
        bad |= kept[c] && (d >> 32) != 0;
        lo = kept[c] ? min(lo, (uint32_t)d) : lo;
        hi = kept[c] ? max(hi, (uint32_t)d) : hi;
    }
    if (ballot(anyR || bad)) return false;
    lo = wave_minmax<false>(lo);
    hi = wave_minmax<true>(hi);
    if (lo > hi || hi - lo >= 256u) return false;  // lo > hi: nothing kept
    const uint64_t kb = b - 0x80000000ull + lo;   // key of slot 0
    uint32_t* erows = reinterpret_cast<uint32_t*>(m.tk);  // [256] entry times of the slot
    uint32_t* addw = erows + 256;                          // [256] add times
    uint32_t* dropw = reinterpret_cast<uint32_t*>(m.stag);  // [256] drop times
    uint8_t* last = reinterpret_cast<uint8_t*>(dropw + 256);  // [256] the slot's last entry
    STAMP(7)
    const uint4 z4 = make_uint4(0u, 0u, 0u, 0u);
    reinterpret_cast<uint4*>(erows)[lane] = z4;
    reinterpret_cast<uint4*>(addw)[lane] = z4;
    reinterpret_cast<uint4*>(dropw)[lane] = z4;
    wave_sync();
    uint32_t tm[4], sl[4];
    // No full step (wave-uniform; the common case of delta anti-entropy): every
    // kept entry adds and no gap can drop it, so the entry-time pass is not
    // needed -- the slot's last entry is an atomic max of (time << 8 | tuple)
    // in erows' words, in the same pass as the add and drop bits.
    const bool nofull = CRDT_FOLD_NOFULL_PASS && full_mask == 0ull;
    if (nofull) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const uint32_t i = c * 64u + lane;
            sl[c] = (uint32_t)(key[c] - kb) & 255u;
            tm[c] = i < n ? 0u : (step[c] & 63u) * 2u + (isT[c] ? 2u : 1u);
            if (!kept[c]) continue;
            const uint32_t r = tm[c];
            if (isT[c]) {
                const uint64_t cc = m.tc[i];
                const bool cov = a[c] < R;  // actor > R: HasDot false
                const uint32_t j = (r - 1u) >> 1;
                if (!(cov && m.vs[j * R + (cov ? a[c] : 0u)] >= cc)) atomicOr(&dropw[sl[c]], 1u << r);
            } else {
                atomicOr(&addw[sl[c]], 1u << r);
                atomicMax(&erows[sl[c]], (r << 8) | i);
            }
        }
    } else {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const uint32_t i = c * 64u + lane;
        sl[c] = (uint32_t)(key[c] - kb) & 255u;
        tm[c] = i < n ? 0u : (step[c] & 63u) * 2u + (isT[c] ? 2u : 1u);
        if (kept[c] && !isT[c]) atomicOr(&erows[sl[c]], 1u << tm[c]);
    }
    wave_sync();
    STAMP(8)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        if (!kept[c]) continue;
        const uint32_t i = c * 64u + lane;
        const uint64_t cc = m.tc[i];
        const bool cov = a[c] < R;  // actor > R: HasDot false
        const uint32_t r = tm[c], j = (r - 1u) >> 1;  // j: the tuple's step (unused for the document)
        if (isT[c]) {
            if (!(cov && m.vs[j * R + (cov ? a[c] : 0u)] >= cc)) atomicOr(&dropw[sl[c]], 1u << r);
            continue;
        }
        const uint32_t above = erows[sl[c]] >> (r + 1u);
        const uint32_t jn = above ? (r + (uint32_t)__ffs(above) - 1u) >> 1 : ms;  // the key's next entry step
        const uint32_t j0 = r == 0u ? 0u : j + 1u;
        uint64_t gap = cov ? full_mask & low_mask(jn) & ~low_mask(j0) : 0ull;
        bool drop = false;
        while (gap) {  // full steps of the gap: HasDot(svv_g, dot) (awset.go:146-158)
            const uint32_t g = (uint32_t)__ffsll((unsigned long long)gap) - 1u;
            gap &= gap - 1ull;
            drop |= m.svv[g * R + a[c]] >= cc;
        }
        const bool fj = r != 0u && ((full_mask >> j) & 1ull);
        const bool add = !fj || !(cov && m.vs[j * R + (cov ? a[c] : 0u)] >= cc);
        if (add) atomicOr(&addw[sl[c]], 1u << r);
        if (drop) atomicOr(&dropw[sl[c]], 1u << r);
        if (!above) last[sl[c]] = (uint8_t)i;
    }
    }
    wave_sync();
    STAMP(9)
    // every slot's words first, then its last entry's dot (reads issued
    // unconditionally: a slot without an entry reads a stale index < 256)
    uint32_t aw[4], dw[4], lt8[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t s = q * 64u + lane;
        aw[q] = addw[s];
        dw[q] = dropw[s];
        lt8[q] = nofull ? (erows[s] & 0xFFu) : last[s];
    }
    uint32_t ea[4];
    uint64_t ec[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        ea[q] = m.ta[lt8[q]];
        ec[q] = m.tc[lt8[q]];
    }
    uint32_t base = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t s = q * 64u + lane;
        const bool P = aw[q] != 0u && (dw[q] >> (31u - (uint32_t)__clz(aw[q]))) == 0u;
        const uint32_t da = P ? ea[q] : 0u;
        const uint64_t dc = P ? ec[q] : 0ull;
        const uint64_t pm = ballot(P);
        e.k[q] = kb + s;
        e.a[q] = da;
        e.c[q] = dc;
        e.off[q] = P ? base + below(pm) : kOOB;
        base += popc(pm);
    }
    U = base;
    return true;
}

// The lean delta pass's common case in one pass over the tuples: no step is a
// full merge (every Counter(src.Actor) > 0, awset-delta_test.go:53), at most
// 15 sources, every key of the document within 256 ids and no actor == len(VV).
// The classify (MakeDeltaMergeData, awset-delta_test.go:79-105: changed
// entries, tombstones not re-added in their source) and the slot walk's add /
// drop times (dense_delta_walk, no-full form) are computed from the same
// registers, so the tuples and clocks are read from LDS once:
//   1. every tuple's key, actor and counter into registers; the span and actor
//      checks (a document that fails one is left to the two-pass form, LDS
//      untouched: returns 0);
//   2. the re-add check: a table of the steps with an entry per key slot
//      (est, in svv -- dead without a full step), then each tombstone looks its
//      slot up, searching its source's entries only when the bit is set (an
//      entry of that key in the source, whose dot decides);
//   3. the slot words (tk and svv, dead now): document entries add at time 0,
//      changed entries (!HasDot(V_j, dot)) add at 2j+1, effective tombstones
//      whose dot V_j lacks drop at 2j+2 (awset-delta_test.go:126-164); the
//      slot's last entry is an atomic max of (time << 8 | tuple);
//   4. a step with neither a changed entry nor an effective tombstone is a no-op
//      (:60), under which the prefix-max clocks are not the exact ones: the
//      document is left to the general kernel (returns 2);
//   5. each slot resolves as in dense_delta_walk (returns 1).
// Exactly the rule of the two-pass form (same times, same words).
template <class Smem>
__device__ __forceinline__ int fused_delta_walk(Smem& m, const uint32_t (&step)[4], const bool (&isE)[4],
                                                const bool (&isT)[4], uint32_t N, uint32_t n, uint32_t ms, uint32_t R,
                                                uint32_t cmax, uint32_t lane, Emit<4>& e, uint32_t& U) {
    static_assert(sizeof(m.tk) >= 2 * 256 * 4 && sizeof(m.svv) >= 256 * 4, "fused_delta_walk: slot words");
    if (N == 0 || ms > 15) return 0;
    // (registers: only the slots stay live across the passes; actors and
    // counters are re-read from ta / tc, which no pass below overwrites)
    uint32_t sl[4];
    uint64_t b;
    {
        uint64_t key[4];
        bool bad = false;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const uint32_t i = c * 64u + lane, ii = i < N ? i : N - 1u;  // (lanes past N: copies of the last tuple)
            const bool in = (uint32_t)c * 64u < N;
            key[c] = in ? m.tk[ii] : 0ull;
            bad |= in && m.ta[ii] == R;
        }
        b = readlane64(key[0], 0);
        uint32_t lo = ~0u, hi = 0u;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            if ((uint32_t)c * 64u >= N) continue;
            const uint64_t d = key[c] - b + 0x80000000ull;
            bad |= (d >> 32) != 0;
            lo = min(lo, (uint32_t)d);
            hi = max(hi, (uint32_t)d);
        }
        if (ballot(bad)) return 0;
        lo = wave_minmax<false>(lo);
        hi = wave_minmax<true>(hi);
        if (hi - lo >= 256u) return 0;
        b = b - 0x80000000ull + lo;  // key of slot 0
#pragma unroll
        for (int c = 0; c < 4; ++c) sl[c] = (uint32_t)(key[c] - b) & 255u;
    }
    const uint64_t kb = b;
    // 2. re-add check
    uint32_t* est = reinterpret_cast<uint32_t*>(m.svv);
    reinterpret_cast<uint4*>(est)[lane] = make_uint4(0u, 0u, 0u, 0u);
    wave_sync();
#pragma unroll
    for (int c = 0; c < 4; ++c)
        if ((uint32_t)c * 64u < N && isE[c]) atomicOr(&est[sl[c]], 1u << (step[c] & 63u));
    wave_sync();
    uint32_t eff = 0;  // bit c: the lane's tuple of chunk c is an effective tombstone
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        if ((uint32_t)c * 64u >= N || !isT[c]) continue;
        const uint32_t j = step[c] & 63u;
        bool f = true;
        if ((est[sl[c]] >> j) & 1u) {  // an entry of this slot in source j: is it this key, re-added?
            const uint32_t i = c * 64u + lane;
            const uint64_t k = m.tk[i];
            const uint32_t s0 = m.soff[j], lo2 = n + s0, len = m.soff[j + 1] - s0;
            uint32_t pos = 0;
            for (uint32_t st = 256; st > 0; st >>= 1) {
                if (st > cmax) continue;
                const bool in = pos + st <= len;
                const uint64_t v2 = m.tk[in ? lo2 + pos + st - 1 : 0u];
                pos += (in && v2 < k) ? st : 0u;
            }
            const bool in_s = pos < len && m.tk[lo2 + pos] == k;
            f = !(in_s && (m.ta[lo2 + pos] != m.ta[i] || m.tc[lo2 + pos] > m.tc[i]));
        }
        eff |= f ? (1u << c) : 0u;
    }
    // 3. slot words (every read of tk and est is issued above: LDS runs a wave's operations in order)
    uint32_t* erows = reinterpret_cast<uint32_t*>(m.tk);  // [256] last entry: time << 8 | tuple
    uint32_t* addw = erows + 256;                          // [256] add times
    uint32_t* dropw = est;                                 // [256] drop times
    const uint4 z4 = make_uint4(0u, 0u, 0u, 0u);
    reinterpret_cast<uint4*>(erows)[lane] = z4;
    reinterpret_cast<uint4*>(addw)[lane] = z4;
    reinterpret_cast<uint4*>(dropw)[lane] = z4;
    wave_sync();
    uint64_t me = 0, mt = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const uint32_t i = c * 64u + lane;
        if ((uint32_t)c * 64u >= N) continue;
        const uint32_t ii = i < N ? i : 0u;
        const uint32_t a = m.ta[ii];
        const uint64_t cc = m.tc[ii];
        if (i >= N) continue;
        const uint32_t j = step[c] & 63u;
        const bool cov = a < R;  // (actor > R: HasDot false; == R was excluded)
        const bool seen = cov && m.vs[j * R + (cov ? a : 0u)] >= cc;  // HasDot(V_j, dot)
        if (i < n) {
            atomicOr(&addw[sl[c]], 1u);
            atomicMax(&erows[sl[c]], i);
        } else if (isE[c]) {
            if (!seen) {
                const uint32_t r = 2u * j + 1u;
                me |= 1ull << j;
                atomicOr(&addw[sl[c]], 1u << r);
                atomicMax(&erows[sl[c]], (r << 8) | i);
            }
        } else if ((eff >> c) & 1u) {
            mt |= 1ull << j;
            if (!seen) atomicOr(&dropw[sl[c]], 1u << (2u * j + 2u));
        }
    }
    // 4. a no-op step: the general kernel replays the steps one by one
    if (low_mask(ms) & ~wave_or64(me) & ~wave_or64(mt)) return 2;
    wave_sync();
    // 5. resolve each slot
    uint32_t aw[4], dw[4], lt8[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t s = q * 64u + lane;
        aw[q] = addw[s];
        dw[q] = dropw[s];
        lt8[q] = erows[s] & 0xFFu;
    }
    uint32_t ea[4];
    uint64_t ec[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        ea[q] = m.ta[lt8[q]];
        ec[q] = m.tc[lt8[q]];
    }
    uint32_t base = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t s = q * 64u + lane;
        const bool P = aw[q] != 0u && (dw[q] >> (31u - (uint32_t)__clz(aw[q]))) == 0u;
        const uint64_t pm = ballot(P);
        e.k[q] = kb + s;
        e.a[q] = P ? ea[q] : 0u;
        e.c[q] = P ? ec[q] : 0ull;
        e.off[q] = P ? base + below(pm) : kOOB;
        base += popc(pm);
    }
    U = base;
    return 1;
}

template <int EPL, bool DELTA, int NQ, class Smem>
__device__ __forceinline__ uint32_t sort_resolve(Smem& m, uint32_t Kc, uint32_t ms, uint32_t R,
                                                 uint64_t full_mask, uint32_t lane, uint64_t lt, Emit<NQ>& e,
                                                 uint32_t& err STAMP_PARAM) {
    uint64_t k[EPL];
    uint32_t t[EPL];
#pragma unroll
    for (int q = 0; q < EPL; ++q) {
        const uint32_t i = lane * EPL + q;
        k[q] = i < Kc ? m.tk[i] : ~0ull;
        t[q] = i < Kc ? (uint32_t)m.stag[i] : kPadTag;
    }
    if (!dense_sort<EPL>(m, k, t, Kc, lane)) wave_sort_pairs<EPL>(k, t, Kc, lane);
    STAMP(7)
    // the element after each one (the next lane's first for the last slot)
    const uint64_t k_nl = from_next_lane64(~0ull, k[0]);
    const uint32_t t_nl = from_next_lane(kPadTag, t[0]);
    const uint64_t k_pl = (uint64_t)__shfl_up((unsigned long long)k[EPL - 1], 1);

    // per element: flags, the current dot (da, dc) and the gap's full steps g
    enum : uint32_t {
        F_PRES = 1u, F_ABS = 2u,  // presence code of the tuple alone (neither: unchanged)
        F_HEAD = 4u, F_TAIL = 8u, F_ENT = 16u, F_TOMB = 32u, F_SRC = 64u, F_FULL = 128u,
        F_AR = 256u,   // the tuple's actor == R (HasDot panics if the reference evaluates it)
        F_GAP = 512u,  // a full step lies between this tuple and the key's next one
        F_G = 1024u    // a gap step's source clock has seen the current dot
    };
    uint32_t fl[EPL], da[EPL], xd[EPL], dinc[EPL], dexc[EPL];
    uint64_t dc[EPL], g[EPL];
#pragma unroll
    for (int q = 0; q < EPL; ++q) {
        const uint32_t i = lane * EPL + q;
        const bool valid = t[q] != kPadTag;
        const uint32_t hi = t[q] >> 8, ti = valid ? t[q] & 0xFFu : 0u;
        const bool src = valid && hi != 0, tomb = valid && (hi & 1u);
        const uint32_t j = src ? ((hi >> 1) - 1u) & 63u : 0u;
        const bool head = !valid || i == 0 || k[q] != (q == 0 ? k_pl : k[q - 1]);
        const uint64_t kn = q + 1 < EPL ? k[q + 1] : k_nl;
        const uint32_t tn = q + 1 < EPL ? t[q + 1] : t_nl;
        const bool tl = valid && (tn == kPadTag || kn != k[q]);
        const uint32_t jn = tl ? ms : ((tn >> 9) - 1u);
        const uint32_t j0 = src ? j + 1u : 0u;
        g[q] = valid ? (full_mask & low_mask(jn) & ~low_mask(j0)) : 0ull;
        da[q] = m.ta[ti];
        dc[q] = m.tc[ti];
        const uint32_t ar = da[q] < R ? da[q] : 0u;
        const bool hv = src && da[q] < R && m.vs[j * R + ar] >= dc[q];  // clock before the step has it
        const bool full = src && ((full_mask >> j) & 1ull);
        uint32_t f = F_PRES;
        if (tomb) f = hv ? 0u : F_ABS;
        else if (full) f = hv ? 0u : F_PRES;
        f |= (head ? F_HEAD : 0u) | (tl ? F_TAIL : 0u) | ((valid && !tomb) ? F_ENT : 0u) | (tomb ? F_TOMB : 0u) |
             (src ? F_SRC : 0u) | (full ? F_FULL : 0u) | (da[q] == R ? F_AR : 0u) | (g[q] ? F_GAP : 0u);
        fl[q] = f;
        xd[q] = (head || (f & F_ENT)) ? (0x80000000u | ((f & F_ENT) ? 0x100u | ti : 0u)) : 0u;
    }
    STAMP(8)
    scan_last_marked<EPL>(xd, dinc, dexc);
    // current dot: the key's last entry at or before the tuple
#pragma unroll
    for (int q = 0; q < EPL; ++q) {
        if (!(fl[q] & F_ENT)) {
            const bool has = dinc[q] & 0x100u;
            const uint32_t src = dinc[q] & 0xFFu;
            da[q] = has ? m.ta[src] : 0u;
            dc[q] = has ? m.tc[src] : 0ull;
        }
        if (da[q] >= R) g[q] = 0;  // never seen: no gap step removes it
    }
    // the gaps' full steps, one step per element per round, until one has seen the dot
    for (;;) {
        bool any = false;
#pragma unroll
        for (int q = 0; q < EPL; ++q) any |= g[q] != 0;
        if (!ballot(any)) break;
#pragma unroll
        for (int q = 0; q < EPL; ++q) {
            const uint32_t j = g[q] ? (uint32_t)__builtin_ctzll(g[q]) : 0u;
            const bool seen = g[q] && m.svv[j * R + (da[q] < R ? da[q] : 0u)] >= dc[q];
            fl[q] |= seen ? F_G : 0u;
            g[q] = seen ? 0ull : (g[q] & (g[q] - 1ull));
        }
    }
    STAMP(9)
    uint32_t xp[EPL], pinc[EPL], pexc[EPL];
#pragma unroll
    for (int q = 0; q < EPL; ++q) {
        const uint32_t h = (fl[q] & F_G) ? F_ABS : (fl[q] & (F_PRES | F_ABS));
        xp[q] = ((fl[q] & F_HEAD) || h) ? (0x80000000u | (h == F_PRES ? 1u : 0u)) : 0u;
    }
    scan_last_marked<EPL>(xp, pinc, pexc);
    uint32_t ne = 0, perr = 0;
    bool em[EPL];
#pragma unroll
    for (int q = 0; q < EPL; ++q) {
        const uint32_t f = fl[q];
        const bool before = !(f & F_HEAD) && (pexc[q] & 1u);  // present before the tuple
        const bool after = (f & F_PRES) || (!(f & (F_PRES | F_ABS)) && before);
        if ((f & F_FULL) && (f & F_ENT) && !before && (f & F_AR)) perr = 1;  // awset.go:129 HasDot
        if (DELTA && (f & F_TOMB) && before && (f & F_AR)) perr = 1;         // delta phase 2 HasDot
        if (after && da[q] == R && (f & F_GAP)) perr = 1;                    // awset.go:151 HasDot
        em[q] = (f & F_TAIL) && (pinc[q] & 1u);
        ne += em[q] ? 1u : 0u;
    }
    if (perr) err |= kErrActorRange;
    uint32_t pre = 0;
    const uint32_t tot = lane_prefix_small(ne, lt, pre);
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        if (q < EPL) {
            e.k[q] = k[q];
            e.a[q] = da[q];
            e.c[q] = dc[q];
            e.off[q] = em[q] ? pre : kOOB;
            pre += em[q] ? 1u : 0u;
        } else {
            e.k[q] = 0;
            e.a[q] = 0;
            e.c[q] = 0;
            e.off[q] = kOOB;
        }
    }
    return tot;
}

// One document's inputs, loaded a document ahead.
template <int NCH, int VCH>
struct FoldPref {
    uint64_t k[NCH], c[NCH], sv[VCH], dv;
    uint32_t a[NCH], eo, eo2, to, to2, act;
};

struct DocMeta {
    uint32_t d, doff, slots, n, s0, ms, e0, E, t0, X, N, big;
};

#ifndef CRDT_FOLD_WAVES
#define CRDT_FOLD_WAVES 2
#endif
#ifndef CRDT_FOLD_K
#define CRDT_FOLD_K 32
#endif
#ifndef CRDT_FOLD_K_DELTA
#define CRDT_FOLD_K_DELTA 8
#endif
#ifndef CRDT_FOLD_WAVES_DELTA
#define CRDT_FOLD_WAVES_DELTA 1
#endif
// wavefronts per workgroup (independent): AWSet folds 2; delta folds 1 (2 %
// faster than 2 on config 3, measured; the AWSet fold is the same either way)
constexpr int kFoldWaves = CRDT_FOLD_WAVES;
constexpr int kFoldWavesD = CRDT_FOLD_WAVES_DELTA;
template <bool DELTA>
constexpr int fold_waves() { return DELTA ? kFoldWavesD : kFoldWaves; }
// survivors' stores: non-temporal (plain stores measured no faster)
constexpr int kFoldStoreAux = kAuxNT;
constexpr int kFoldK = CRDT_FOLD_K;  // consecutive documents per wavefront (AWSet folds)
constexpr int kFoldKD = CRDT_FOLD_K_DELTA;  // (delta folds: 8; 16 was 2 % faster than 32, 8 1.3-1.9 % than 16)
// stores of one document's write-out: walk rounds x 3 + count + VV
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
// lane E of (hi:lo) := the wave-uniform x (v_writelane: no select, no exec change)
template <int E>
__device__ __forceinline__ void lane_put(uint32_t& lo, uint32_t& hi, uint64_t x) {
    asm("v_writelane_b32 %0, %1, %2" : "+v"(lo) : "s"((uint32_t)x), "i"(E));
    asm("v_writelane_b32 %0, %1, %2" : "+v"(hi) : "s"((uint32_t)(x >> 32)), "i"(E));
}
// (CRDT_FOLD_STAGE_STORES 2: 16-byte stores, two keys / counters or four actors a lane)
__host__ __device__ constexpr int fold_stores(int nch) {
    return CRDT_FOLD_STAGE_STORES == 2 ? 2 * ((nch + 1) / 2) + (nch + 3) / 4 + 2 : nch * 3 + 2;
}

template <int K, bool DELTA, bool LEAN, bool LIST>
__global__ __launch_bounds__(fold_waves<DELTA>() * 64) __attribute__((amdgpu_waves_per_eu(FoldShape<DELTA, LEAN>::WPE))) void fold_pipe_kernel(BatchView dst, SrcView sb, OutView out, Work wk) {
    static_assert(!(LEAN && LIST), "the lean pass runs over consecutive documents");
    static_assert(K >= 1 && K < 64, "a run's end bounds live in lane K: K < 64");
    constexpr int NCH = FoldShape<DELTA, LEAN>::NCH, VCH = FoldShape<DELTA, LEAN>::VCH;
    // store rounds of a write-out: the lean AWSet pass emits only through
    // dense_awset_walk (slots < 64: one round; a document it cannot walk is
    // deferred, nothing written), so its second round would be all out of
    // range -- not issued (config 5: 3 fewer store instructions a document)
    constexpr int WQ = (LEAN && !DELTA && CRDT_FOLD_AWSET_ONE_ROUND) ? 1 : NCH;
    using Smem = FoldSmem<FoldShape<DELTA, LEAN>::VCAP, 64 * NCH>;
    static_assert(fold_smem_aligned<FoldShape<DELTA, LEAN>::VCAP, 64 * NCH>(),
                  "FoldSmem: a 64-bit LDS access target is not 8-byte aligned");
    __shared__ Smem smem[fold_waves<DELTA>()];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t w = threadIdx.x >> 6;
    Smem& m = smem[w];
    const uint32_t R = dst.R;
    const uint32_t n_docs = dst.n_docs;
    const uint64_t lt = low_mask(lane);
    const bool tombs = DELTA && sb.tomb_off != nullptr;
    uint32_t err = 0;
    STAMP_DECL

    // LIST: the run is entries [first, first + kr) of the deferred list.  Delta
    // folds: kr = the fewest per wave that cover it (the grid is sized for every
    // document at K a wave: config 3's list, ~1 % of its documents, is spread one
    // document a wave over the chip instead of K-long latency chains on ~700
    // waves -- the call 1.717 -> 1.630 ms, profiles/r06za_lab.log); AWSet folds
    // keep runs of K (config 5: spread 0.2 % slower)
    const uint32_t n_run = LIST ? min(__hip_atomic_load(wk.defer_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                                      n_docs)
                                : n_docs;
    uint32_t kr = (uint32_t)K;
    if constexpr (LIST && DELTA && CRDT_FOLD_LIST_SPREAD) {
        const uint32_t waves = gridDim.x * (uint32_t)fold_waves<DELTA>();
        kr = uniform(max(1u, min((uint32_t)K, (n_run + waves - 1u) / waves)));
    }
    // CRDT_FOLD_XCD_MAP: the lean pass's workgroups renumbered so that each XCD
    // (workgroups are dispatched to the 8 XCDs round-robin) takes one contiguous
    // range of documents, and neighbouring runs share their edge lines in one
    // L2.  AWSet lean pass (1, default): config 5 8.52-8.74 ms against 8.55-9.41
    // for the round-robin order, nine interleaved rounds on two boxes, and far
    // less spread; the delta pass (2: both) gained nothing on config 3
    // (profiles/r06zl_fold_xcd_map_ab.log).
    uint32_t blk = blockIdx.x;
    if constexpr (LEAN && (CRDT_FOLD_XCD_MAP == 2 || (CRDT_FOLD_XCD_MAP == 1 && !DELTA))) {
        const uint32_t q = gridDim.x / 8u, r = gridDim.x % 8u, x = blk % 8u;
        blk = x * q + min(x, r) + blk / 8u;
    }
    const uint32_t first = uniform((blk * fold_waves<DELTA>() + w) * kr);
    if (first >= n_run || !gate_open(wk)) return;  // (a closed gate: nothing deferred or pushed either)
    const uint32_t cnt = min(kr, n_run - first);

    // ---- metadata of the run: lane i <= cnt describes document first + i (LIST:
    // lane i < cnt describes deferred document i, with its end bounds loaded)
    const uint32_t di = LIST ? wk.defer[first + min(lane, cnt - 1u)] : first + min(lane, cnt);
    const uint32_t mv_ds = sb.doc_srcs[di];
    const uint32_t mv_off = dst.offsets[di];
    const uint32_t mv_cnt = dst.counts ? dst.counts[min(di, n_docs - 1u)] : 0u;
    const uint32_t mv_eo = sb.entry_off[mv_ds];
    const uint32_t mv_to = tombs ? sb.tomb_off[mv_ds] : 0u;
    uint32_t ds_hi, off_hi, eo_hi, to_hi, mv_doc = 0;
    if constexpr (LIST) {
        mv_doc = di;
        ds_hi = sb.doc_srcs[di + 1];
        off_hi = dst.offsets[di + 1];
        eo_hi = sb.entry_off[ds_hi];
        to_hi = tombs ? sb.tomb_off[ds_hi] : 0u;
    } else {
        ds_hi = (uint32_t)__shfl_down((int)mv_ds, 1);
        off_hi = (uint32_t)__shfl_down((int)mv_off, 1);
        eo_hi = (uint32_t)__shfl_down((int)mv_eo, 1);
        to_hi = (uint32_t)__shfl_down((int)mv_to, 1);
    }
    const uint32_t slots_i = off_hi - mv_off;
    uint32_t n_i = dst.counts ? mv_cnt : slots_i;
    if (lane < cnt && n_i > slots_i) {  // live count beyond the slots: clamped, reported
        err |= kErrCapacity;
        n_i = slots_i;
    }
    const uint32_t ms_i = ds_hi - mv_ds;
    const uint32_t E_i = eo_hi - mv_eo;
    const uint32_t X_i = to_hi - mv_to;
    const bool big_i = lane < cnt && ((uint64_t)n_i + E_i + X_i > (uint64_t)Smem::NCAP ||
                                      ms_i > (uint32_t)(LEAN ? 15 : Smem::MCAP) || ms_i * R > (uint32_t)Smem::VCAP);
    const uint64_t bigm = ballot(big_i);
    if (big_i) {
        if (LEAN)
            push_defer(wk, first + lane, n_docs);
        else
            push_work(wk, di, n_docs);
    }
    if (!LIST) {  // output slot bounds of the run's documents (+ the batch end after the last one)
        const bool wr = lane < cnt || (lane == cnt && first + cnt == n_docs);
        st32(mv_off + mv_eo, make_rsrc(out.offsets + first, (cnt + 1u) * 4u), wr ? lane * 4u : kOOB);
    }

    auto rl = [](uint32_t v, uint32_t i) { return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)i); };
    auto meta = [&](uint32_t k) {
        DocMeta q;
        if constexpr (LIST) {
            q.d = rl(mv_doc, k);
            q.doff = rl(mv_off, k);
            q.slots = rl(off_hi, k) - q.doff;
            q.s0 = rl(mv_ds, k);
            q.ms = rl(ds_hi, k) - q.s0;
            q.e0 = rl(mv_eo, k);
            q.E = rl(eo_hi, k) - q.e0;
            q.t0 = rl(mv_to, k);
            q.X = rl(to_hi, k) - q.t0;
        } else {
            q.d = first + k;
            // bounds of lanes k and k + 1 (lane cnt holds the run's end): only the
            // base vectors stay live through the loop, not their differences
            q.doff = rl(mv_off, k);
            q.slots = rl(mv_off, k + 1) - q.doff;
            q.s0 = rl(mv_ds, k);
            q.ms = rl(mv_ds, k + 1) - q.s0;
            q.e0 = rl(mv_eo, k);
            q.E = rl(mv_eo, k + 1) - q.e0;
            q.t0 = rl(mv_to, k);
            q.X = rl(mv_to, k + 1) - q.t0;
        }
        q.n = rl(n_i, k);
        q.N = q.n + q.E + q.X;
        q.big = (uint32_t)((bigm >> k) & 1ull);
        return q;
    };
    // Issue every load of document q (no waits): tuples [document | source
    // entries | tombstones] by per-lane address (lanes past N re-read the last
    // tuple, so no load is exec-masked), clocks and offsets by buffer loads.
    auto prefetch = [&](FoldPref<NCH, VCH>& P, const DocMeta& q) {
        // (delta folds only: -1.8 % on config 3; the AWSet folds select between
        // two regions, +0.9 % on config 5 -- profiles/r04z_fold_variants.log)
        if constexpr (DELTA && CRDT_FOLD_PTAB) {
        // Per-region base table in LDS (the 128 spare bytes at anye / anyt,
        // dead here): entry r * 4 + {0 keys, 1 counters, 2 actors} points at
        // tuple 0 of the document's index space in region r's array, so a lane
        // reads its region's three bases (two LDS reads) instead of selecting
        // among nine scalar pointers in vector registers.  Built lane by lane
        // from scalar values (v_writelane), written by one LDS store.
        {
            uint64_t* ptab = reinterpret_cast<uint64_t*>(m.anye);
            const uint64_t dn = (uint64_t)q.doff, en = (uint64_t)q.e0 - q.n, tn = (uint64_t)q.t0 - q.n - q.E;
            uint32_t lo = 0, hi = 0;
            lane_put<0>(lo, hi, reinterpret_cast<uint64_t>(dst.keys) + 8u * dn);
            lane_put<1>(lo, hi, reinterpret_cast<uint64_t>(dst.counters) + 8u * dn);
            lane_put<2>(lo, hi, reinterpret_cast<uint64_t>(dst.actors) + 4u * dn);
            lane_put<4>(lo, hi, reinterpret_cast<uint64_t>(sb.keys) + 8u * en);
            lane_put<5>(lo, hi, reinterpret_cast<uint64_t>(sb.counters) + 8u * en);
            lane_put<6>(lo, hi, reinterpret_cast<uint64_t>(sb.actors) + 4u * en);
            if (DELTA) {
                lane_put<8>(lo, hi, reinterpret_cast<uint64_t>(sb.tkeys) + 8u * tn);
                lane_put<9>(lo, hi, reinterpret_cast<uint64_t>(sb.tcounters) + 8u * tn);
                lane_put<10>(lo, hi, reinterpret_cast<uint64_t>(sb.tactors) + 4u * tn);
            }
            if (lane < 12) ptab[lane] = ((uint64_t)hi << 32) | lo;
            wave_sync();
        }
        const uint64_t* ptab = reinterpret_cast<const uint64_t*>(m.anye);
        const uint32_t nE = q.n + q.E;
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            if ((uint32_t)c * 64u < q.N) {
                uint32_t i = c * 64u + lane;
                i = i < q.N ? i : q.N - 1u;
                const uint32_t r4 = (i >= q.n ? 4u : 0u) + (i >= nE ? 4u : 0u);
                const uint64_t kb = ptab[r4], cb = ptab[r4 + 1], ab = ptab[r4 + 2];
#if CRDT_FOLD_GLOBAL_PTAB
                // Global (not generic) loads: a FLAT load also counts in lgkmcnt, so
                // every LDS wait of the current document's fold -- the first comes
                // right after this prefetch -- would wait for the next document's
                // HBM loads too, and the prefetch would overlap nothing.
                P.k[c] = __builtin_nontemporal_load(reinterpret_cast<gptr<uint64_t>>(kb) + i);
                P.a[c] = __builtin_nontemporal_load(reinterpret_cast<gptr<uint32_t>>(ab) + i);
                P.c[c] = __builtin_nontemporal_load(reinterpret_cast<gptr<uint64_t>>(cb) + i);
#else
                P.k[c] = __builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(kb) + i);
                P.a[c] = __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(ab) + i);
                P.c[c] = __builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(cb) + i);
#endif
            }
        }
        } else {
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
#if CRDT_FOLD_PURE_CHUNKS
            // a chunk inside one region (the document's entries, the source
            // entries or the tombstones): buffer loads from that region's
            // scalar base, no per-lane pointer select
            const uint32_t lo = c * 64u, hi = lo + 64u;
            const bool pure_d = hi <= q.n, pure_e = lo >= q.n && hi <= q.n + q.E;
            if (lo < q.N && (pure_d || pure_e)) {
                const uint32_t r0 = pure_d ? q.doff + lo : q.e0 + (lo - q.n);
                const uint32_t o8 = lane * 8u, o4 = lane * 4u;
                const rsrc_t rk = make_rsrc(pure_d ? dst.keys + r0 : sb.keys + r0, 512u);
                const rsrc_t ra = make_rsrc(pure_d ? dst.actors + r0 : sb.actors + r0, 256u);
                const rsrc_t rc = make_rsrc(pure_d ? dst.counters + r0 : sb.counters + r0, 512u);
                P.k[c] = __builtin_bit_cast(uint64_t, __builtin_amdgcn_raw_buffer_load_b64(rk, (int)o8, 0, kAuxNT));
                P.a[c] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(ra, (int)o4, 0, kAuxNT);
                P.c[c] = __builtin_bit_cast(uint64_t, __builtin_amdgcn_raw_buffer_load_b64(rc, (int)o8, 0, kAuxNT));
            } else
#endif
            if ((uint32_t)c * 64u < q.N) {
                uint32_t i = c * 64u + lane;
                i = i < q.N ? i : q.N - 1u;
#if CRDT_FOLD_IDX32
                // 32-bit index selects (slot indices are u32), no tombstone region
                // in an AWSet fold: no exec-masked 64-bit arithmetic per region
                const bool isd = i < q.n, iss = !DELTA || i < q.n + q.E;
                const size_t idx = isd ? q.doff + i : (iss ? q.e0 + (i - q.n) : q.t0 + (i - q.n - q.E));
#else
                const bool isd = i < q.n, iss = i < q.n + q.E;
                const size_t idx = isd ? (size_t)q.doff + i
                                       : (iss ? (size_t)q.e0 + (i - q.n) : (size_t)q.t0 + (i - q.n - q.E));
#endif
                const uint64_t* kb = isd ? dst.keys : (iss ? sb.keys : sb.tkeys);
                const uint32_t* ab = isd ? dst.actors : (iss ? sb.actors : sb.tactors);
                const uint64_t* cb = isd ? dst.counters : (iss ? sb.counters : sb.tcounters);
                // non-temporal: every tuple is read once (0.5 % faster, measured)
                P.k[c] = __builtin_nontemporal_load(kb + idx);
                P.a[c] = __builtin_nontemporal_load(ab + idx);
                P.c[c] = __builtin_nontemporal_load(cb + idx);
            }
        }
        }
        const rsrc_t rv = make_rsrc(sb.vv + (size_t)q.s0 * R, q.ms * R * 8u);
#pragma unroll
        for (int c = 0; c < VCH; ++c)
            if ((uint32_t)c * 64u < q.ms * R) P.sv[c] = ld64(rv, (c * 64u + lane) * 8u);
        P.dv = ld64(make_rsrc(dst.vv + (size_t)q.d * R, R * 8u), lane * 8u);
        const rsrc_t re = make_rsrc(sb.entry_off + q.s0, (q.ms + 1u) * 4u);
        P.eo = ld32(re, lane * 4u);
        if (!LEAN && q.ms >= 64) P.eo2 = ld32(re, (64u + lane) * 4u);
        if (tombs) {
            const rsrc_t rt = make_rsrc(sb.tomb_off + q.s0, (q.ms + 1u) * 4u);
            P.to = ld32(rt, lane * 4u);
            if (!LEAN && q.ms >= 64) P.to2 = ld32(rt, (64u + lane) * 4u);
        }
        P.act = ld32(make_rsrc(sb.src_actor + q.s0, q.ms * 4u), lane * 4u);
    };

    FoldPref<NCH, VCH> P{};
    {
        const DocMeta q0 = meta(0);
        if (!q0.big) prefetch(P, q0);
    }
    {   // As many (out-of-range, no-traffic) stores as a document's write-out
        // issues, so the loop is entered with the same memory operations
        // behind the prefetch as every later iteration: the compiler's vmcnt
        // for the staged registers is then exact on both paths into the loop.
        const rsrc_t none = make_rsrc(out.counts, 0u);
#pragma unroll
        for (int i = 0; i < fold_stores(WQ); ++i) st32(0u, none, kOOB + 4u * i);  // distinct: not merged
    }
#pragma unroll 1
    for (uint32_t k = 0; k < cnt; ++k) {
        STAMP(15)
        // metadata re-read per document (lane k of the run's vectors), not carried
        // across the fold: fewer scalar registers live through the loop body
        const DocMeta cur = meta(k);
        // Every prefetch register is consumed here, on every path: its load
        // (issued one document ago, before the last write-out's stores) is then
        // known complete, so the next prefetch may overwrite it without a
        // vmcnt wait -- which, counted in order, would wait out those stores.
#pragma unroll
        for (int c = 0; c < NCH; ++c) asm volatile("" ::"v"(P.k[c]), "v"(P.c[c]), "v"(P.a[c]));
#pragma unroll
        for (int c = 0; c < VCH; ++c) asm volatile("" ::"v"(P.sv[c]));
        asm volatile("" ::"v"(P.dv), "v"(P.eo), "v"(P.act));
        if constexpr (!LEAN) asm volatile("" ::"v"(P.eo2));  // (the lean passes defer > 15 sources)
        if constexpr (DELTA) asm volatile("" ::"v"(P.to));
        if constexpr (DELTA && !LEAN) asm volatile("" ::"v"(P.to2));
#if CRDT_FOLD_PAD_VALU || CRDT_FOLD_PAD_SALU
        {   // diagnostic (tools/fold_probe timing builds): N dependent VALU / SALU
            // instructions per document -- the slope says which issue port binds
            uint32_t pv = lane, ps = k;
#pragma unroll
            for (int i = 0; i < CRDT_FOLD_PAD_VALU; ++i) asm volatile("v_add_u32 %0, %0, 1" : "+v"(pv));
#pragma unroll
            for (int i = 0; i < CRDT_FOLD_PAD_SALU; ++i) asm volatile("s_add_u32 %0, %0, 1" : "+s"(ps));
            err |= (pv == 0xFFFFFFFFu && ps == 0xFFFFFFFFu) ? kErrWorkspace : 0u;
        }
#endif
        // ---- stage document k (its loads were issued one document ago)
        uint64_t vreg = 0;              // lane r < R: V_0[r]
        uint32_t soffv = 0, toffv = 0;  // lane s: end of source s's entries / tombstones
        if (!cur.big) {
            const uint32_t N = cur.N, msR = cur.ms * R;
            // Whole chunks are written (wave-uniform guards only, no per-lane
            // branch: each divergent branch costs scalar exec-mask work): the
            // lanes past N store a copy of the last tuple (the prefetch
            // clamps), which nothing reads.
#pragma unroll
            for (int c = 0; c < NCH; ++c) {
                const uint32_t i = c * 64u + lane;
                if ((uint32_t)c * 64u < N) {
                    m.tk[i] = P.k[c];
                    m.ta[i] = P.a[c];
                    m.tc[i] = P.c[c];
                }
            }
#pragma unroll
            for (int c = 0; c < VCH; ++c) {
                const uint32_t i = c * 64u + lane;
                if constexpr (Smem::VCAP >= 64 * VCH) {  // whole chunks fit: the words past ms*R are never read
                    if ((uint32_t)c * 64u < msR) m.svv[i] = P.sv[c];
                } else {
                    if ((uint32_t)c * 64u < msR && i < msR) m.svv[i] = P.sv[c];
                }
            }
            // (CRDT_FOLD_DIAG_NOLOAD: the offsets held are the run's first document's)
            const uint32_t e0 = CRDT_FOLD_DIAG_NOLOAD ? rl(P.eo, 0) : cur.e0;
            const uint32_t t0 = CRDT_FOLD_DIAG_NOLOAD ? rl(P.to, 0) : cur.t0;
            const uint32_t nso = from_next_lane(LEAN ? 0u : rl(P.eo2, 0), P.eo);
            soffv = nso - e0;
            // per-source words of every lane (MCAP = 64: lanes past ms write words no step reads)
            m.soff[lane] = P.eo - e0;
            if (cur.ms >= 64 && lane == 0) m.soff[64] = P.eo2 - e0;
            if (tombs) {
                const uint32_t nto = from_next_lane(LEAN ? 0u : rl(P.to2, 0), P.to);
                toffv = nto - t0;
            }
            m.sact[lane] = P.act;
            reinterpret_cast<uint32_t*>(m.smark)[lane & (Smem::NCAP / 4 - 1)] = 0u;
            wave_sync();
            // Source s's tuples end at soffv / toffv (nondecreasing in s): mark
            // s + 1 at that position (the last source ending there), so a tuple's
            // step is the largest mark at or before it within its region.
            const uint32_t nse = from_next_lane(0u, soffv), nte = from_next_lane(0u, toffv);
            const bool lasts = lane + 1u == cur.ms;
            if (lane < cur.ms && soffv < cur.E && (lasts || nse != soffv)) m.smark[cur.n + soffv] = (uint8_t)(lane + 1u);
            if (lane < cur.ms && toffv < cur.X && (lasts || nte != toffv))
                m.smark[cur.n + cur.E + toffv] = (uint8_t)(lane + 1u);
            vreg = P.dv;
        }
        wave_sync();
        STAMP(0)
        // ---- issue document k+1's loads; they fly while document k is folded
        // (CRDT_FOLD_DIAG_NOLOAD, diagnostic: none -- every document of the run folds
        // the first one's tuples, which in configs 3 and 5 have the same shape)
        if (k + 1 < cnt && !CRDT_FOLD_DIAG_NOLOAD) {
            const DocMeta nxt = meta(k + 1);
            STAMP(12)
            if (!nxt.big) prefetch(P, nxt);
        }
        STAMP(1)

        // ---- fold document k
        uint64_t vfin = 0, full_mask = 0;
        uint32_t U = 0;  // survivors
        bool deferred = false;  // LEAN: the document is left to the general kernel
        Emit<NCH> em;
#if CRDT_FOLD_DIAG_NOCOMPUTE
        // diagnostic bound (tools/fold_probe timing builds): no fold at all -- the
        // document's own entries written back as its survivors (memory traffic and
        // the pipeline, without the per-document chain)
        if (!cur.big) {
#pragma unroll
            for (int q = 0; q < NCH; ++q) {
                const uint32_t i = q * 64u + lane;
                em.k[q] = m.tk[i];
                em.a[q] = m.ta[i];
                em.c[q] = m.tc[i];
                em.off[q] = i < cur.n ? i : kOOB;
            }
            U = cur.n;
            vfin = vreg;
        }
        if (false) {
#else
        if (!cur.big) {
#endif
            const uint32_t n = cur.n, E = cur.E, N = cur.N, ms = cur.ms;
            // schedule: U_j, one lane per actor
            uint64_t v = vreg;
            uint32_t j = 0;
            if (lane < R) {
                for (; j + 4u <= ms; j += 4u) {  // four clock loads in flight per round
                    uint64_t sw[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) sw[u] = m.svv[(j + u) * R + lane];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        m.vs[(j + u) * R + lane] = v;
                        v = v > sw[u] ? v : sw[u];
                    }
                }
                for (; j < ms; ++j) {
                    m.vs[j * R + lane] = v;
                    const uint64_t sw = m.svv[j * R + lane];
                    v = v > sw ? v : sw;
                }
            }
            vfin = v;
            wave_sync();
            full_mask = low_mask(ms);  // AWSet fold: every step is a full merge
            if (DELTA) {
                // path select (awset-delta_test.go:53): Counter(src.Actor) of the
                // clock before the step; actor == len(VV) panics in Go
                const uint32_t aj = lane < ms ? m.sact[lane] : 0u;
                if (lane < ms && aj == R) err |= kErrActorRange;
                const uint64_t cj = (lane < ms && aj < R) ? m.vs[lane * R + aj] : 0ull;
                full_mask = ballot(lane < ms && cj == 0);
            }
            STAMP(2)
            // classify the tuples: kind, step, changed / effective
            const uint32_t NQ = (N + 63u) >> 6;
            uint32_t step[NCH];
            bool isE[NCH], isT[NCH];
#pragma unroll
            for (int c = 0; c < NCH; ++c) {
                const uint32_t i = c * 64u + lane;
                isE[c] = i >= n && i < n + E;
                isT[c] = i >= n + E && i < N;
                step[c] = 0;
            }
            // step of a source tuple = number of sources whose range ends at or
            // before it = the largest mark at or before it in its region: a max-scan
            // of (region << 8 | mark) (regions ascend, so the scan never looks back
            // into an earlier region's marks)
            {
                const uint32_t c0 = n >> 6;  // first chunk holding a source tuple
                uint32_t carry = 0;
#pragma unroll
                for (int c = 0; c < NCH; ++c) {
                    if ((uint32_t)c >= c0 && (uint32_t)c < NQ) {
                        const uint32_t i = c * 64u + lane;
                        uint32_t x = ((isT[c] ? 2u : (isE[c] ? 1u : 0u)) << 8) | m.smark[i];
                        x = max(x, dpp<0x111>(0u, x));         // row_shr:1
                        x = max(x, dpp<0x112>(0u, x));         // row_shr:2
                        x = max(x, dpp<0x114>(0u, x));         // row_shr:4
                        x = max(x, dpp<0x118>(0u, x));         // row_shr:8
                        x = max(x, dpp<0x142, 0xA>(0u, x));    // row_bcast:15
                        x = max(x, dpp<0x143, 0xC>(0u, x));    // row_bcast:31
                        x = max(x, carry);
                        carry = (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
                        step[c] = x & 0xFFu;
                    }
                }
            }
            STAMP(10)
            // (the fused pass searches a source's entries only on a table hit, rare:
            // it probes every level instead, and the scan below is skipped)
            constexpr bool kFused = DELTA && LEAN && NCH == 4 && CRDT_FOLD_FUSED;
            uint32_t cmax = kFused ? 256u : 0u;  // longest source: depth of the re-add search
            if (DELTA && cur.X && !kFused) {
                const uint32_t prv = dpp<0x138>(0u, soffv);  // wave_shr:1
                cmax = lane < ms ? soffv - (lane ? prv : 0u) : 0u;
                cmax = max(cmax, dpp<0x111>(0u, cmax));  // inclusive max-scan (DPP, no LDS) ...
                cmax = max(cmax, dpp<0x112>(0u, cmax));
                cmax = max(cmax, dpp<0x114>(0u, cmax));
                cmax = max(cmax, dpp<0x118>(0u, cmax));
                cmax = max(cmax, dpp<0x142, 0xA>(0u, cmax));
                cmax = max(cmax, dpp<0x143, 0xC>(0u, cmax));
                cmax = (uint32_t)__builtin_amdgcn_readlane((int)cmax, 63);  // ... whose last lane has the maximum
            }
            STAMP(11)
            // CRDT_FOLD_FUSED: the lean delta pass's common case, classify and slot
            // walk in one pass (fused_delta_walk); 0: the two-pass form below
            // The lean delta pass then holds nothing else: a document the fused pass
            // does not take (a full step, a no-op step, > 15 sources, a key span of
            // 256 or more, an actor == len(VV)) is left to the general kernel.
            if constexpr (kFused) {
                const int fused =
                    full_mask == 0ull ? fused_delta_walk(m, step, isE, isT, N, n, ms, R, cmax, lane, em, U) : 0;
                if (fused != 1) {  // left to the general kernel, nothing written here
                    deferred = true;
                    if (lane == 0) push_defer(wk, cur.d, n_docs);
#pragma unroll
                    for (int q = 0; q < NCH; ++q) em.off[q] = kOOB;
                    U = 0;
                }
            }
            if constexpr (!kFused) {
            // CRDT_FOLD_TOMB_TAB: est[key & 255] = the steps (< 32) with an entry of that
            // low key byte, so a tombstone whose step bit is clear was not re-added in
            // its source (effective) without the binary search below; a set bit (the
            // key, or another one with the same low byte) still searches.  Scratch:
            // stag onwards, dead until the keep phase / the walk.
            const bool tab = CRDT_FOLD_TOMB_TAB && DELTA && cur.X != 0 && ms <= 32;
            uint32_t* est = reinterpret_cast<uint32_t*>(m.stag);
            static_assert(offsetof(Smem, dbase) + sizeof(m.dbase) - offsetof(Smem, stag) >= 1024,
                          "fold: step table space");
            if (tab) {
                reinterpret_cast<uint4*>(est)[lane] = make_uint4(0u, 0u, 0u, 0u);
                wave_sync();
            }
            uint64_t key[NCH];
            uint32_t flag = 0, perr = 0;  // flag bit c: changed entry / effective tombstone
            uint64_t me = 0, mt = 0;      // steps of this lane's changed entries / effective tombstones
#pragma unroll
            for (int c = 0; c < NCH; ++c) {
                key[c] = 0;
                if (CRDT_FOLD_DIAG_SKIP_CLASSIFY && (uint32_t)c < NQ) {  // diagnostic: keys only
                    key[c] = m.tk[c * 64u + lane < N ? c * 64u + lane : 0u];
                    continue;
                }
                if ((uint32_t)c < NQ) {
                    const uint32_t i = c * 64u + lane;
                    const uint32_t ii = i < N ? i : 0u;
                    key[c] = m.tk[ii];
                    const uint32_t a = m.ta[ii];
                    const uint64_t cc = m.tc[ii];
                    const uint32_t j = step[c] & 63u;
                    bool f = false;
#if CRDT_FOLD_CLASSIFY_UNIFORM
                    // Wave-uniform guards (does the chunk hold entries / tombstones)
                    // and predicated per-lane work: no exec-mask regions per chunk.
                    const uint32_t c64 = c * 64u;
                    if (DELTA && c64 < n + E && c64 + 64u > n) {
                        // MakeDeltaMergeData (:84-92): dst's clock has not seen the entry
                        const bool ce = isE[c] && !((full_mask >> j) & 1ull);
                        perr |= (ce && a == R) ? kErrActorRange : 0u;
                        const bool cov = a < R;
                        const uint64_t vj = issued(m.vs[j * R + (cov ? a : 0u)]);
                        const bool fe = ce && !(cov && vj >= cc);
                        me |= fe ? 1ull << j : 0ull;
                        f = fe;
                    }
                    if (DELTA && c64 + 64u > n + E && c64 < N) {
                        // effective: not re-added in the same source (:93-102); lanes
                        // that are not tombstones search an empty range
                        const uint32_t s0 = m.soff[j], lo = n + s0, len = isT[c] ? m.soff[j + 1] - s0 : 0u;
                        uint32_t pos = 0;
                        for (uint32_t st = 256; st > 0; st >>= 1) {
                            if (st > cmax) continue;
                            const bool in = pos + st <= len;
                            const uint64_t v2 = issued(m.tk[in ? lo + pos + st - 1 : 0u]);
                            pos += (in && v2 < key[c]) ? st : 0u;
                        }
                        const bool hit = pos < len;
                        const uint32_t at = hit ? lo + pos : 0u;
                        const uint64_t hk = issued(m.tk[at]), hc = issued(m.tc[at]);
                        const uint32_t ha = issued(m.ta[at]);
                        const bool in_s = hit && hk == key[c];
                        const bool ft = isT[c] && !(in_s && (ha != a || hc > cc));
                        mt |= ft ? 1ull << j : 0ull;
                        f = f || ft;
                    }
#else
                    if (DELTA && isE[c] && !((full_mask >> j) & 1ull)) {
                        // MakeDeltaMergeData (:84-92): dst's clock has not seen the entry
                        if (a == R) perr |= kErrActorRange;
                        f = !(a < R && m.vs[j * R + a] >= cc);
                        me |= f ? 1ull << j : 0ull;
                    }
                    // (before the tombstones' reads: this chunk's and every earlier one's
                    // entries are in the table when a tombstone of the chunk looks)
                    if (tab && isE[c]) atomicOr(&est[(uint32_t)key[c] & 255u], 1u << j);
                    if (DELTA && isT[c] && tab && !((est[(uint32_t)key[c] & 255u] >> j) & 1u)) {
                        f = true;  // no entry of this key in source j: effective (:93-102)
                        mt |= 1ull << j;
                    } else if (DELTA && isT[c]) {
                        // effective: not re-added in the same source (:93-102)
                        const uint32_t lo = n + m.soff[j], len = m.soff[j + 1] - m.soff[j];
                        uint32_t pos = 0;
                        for (uint32_t st = 256; st > 0; st >>= 1) {
                            if (st > cmax) continue;
                            const bool in = pos + st <= len;
                            const uint64_t v2 = m.tk[in ? lo + pos + st - 1 : 0u];
                            pos += (in && v2 < key[c]) ? st : 0u;
                        }
                        const bool in_s = pos < len && m.tk[lo + pos] == key[c];
                        f = !(in_s && (m.ta[lo + pos] != a || m.tc[lo + pos] > cc));
                        mt |= f ? 1ull << j : 0ull;
                    }
#endif
                    flag |= f ? (1u << c) : 0u;
                }
            }
            wave_sync();
            STAMP(3)
            uint64_t noop_mask = 0, tmask = 0;
            if (DELTA) {
                // steps with a changed entry / an effective tombstone, OR-ed over the
                // wave in registers (DPP): no LDS round trip
                const uint64_t anye = wave_or64(me);
                tmask = wave_or64(mt) & low_mask(ms);
                noop_mask = low_mask(ms) & ~full_mask & ~anye & ~tmask;
                if (CRDT_FOLD_DIAG_SKIP_CLASSIFY) noop_mask = 0;  // (diagnostic: no replay either)
            }
            if (DELTA && noop_mask) {
                // a step brings nothing: replay the schedule step by step with the exact clocks
                const uint64_t emask = tmask;
                v = vreg;
                full_mask = 0;
                noop_mask = 0;
                perr = 0;
                uint32_t fe = 0;  // changed bits of the entries, rebuilt
                for (uint32_t j = 0; j < ms; ++j) {
                    if (lane < R) m.vs[j * R + lane] = v;
                    const uint32_t aj = uniform(m.sact[j]);
                    const uint64_t cj = aj < R ? readlane64(v, aj) : 0ull;
                    const bool full = cj == 0;
                    bool noop = false;
                    if (!full) {
                        bool any = false;
#pragma unroll
                        for (int c = 0; c < NCH; ++c) {
                            if ((uint32_t)c < NQ) {
                                const uint32_t i = c * 64u + lane;
                                const bool mine = isE[c] && step[c] == j;
                                const uint32_t a = m.ta[mine ? i : 0u];
                                const uint64_t cc = m.tc[mine ? i : 0u];
                                const uint64_t have = (uint64_t)__shfl((unsigned long long)v, (int)(a < R ? a : 0u));
                                if (mine && a == R) perr |= kErrActorRange;
                                const bool chg = mine && !(a < R && have >= cc);
                                fe |= chg ? (1u << c) : 0u;
                                any |= chg;
                            }
                        }
                        noop = !ballot(any) && !((emask >> j) & 1ull);
                    }
                    full_mask |= (uint64_t)full << j;
                    noop_mask |= (uint64_t)noop << j;
                    if (!noop && lane < R) {
                        const uint64_t s = m.svv[j * R + lane];
                        v = v > s ? v : s;
                    }
                }
                vfin = v;
                // entries take their rebuilt bits, tombstones keep their effective bits
                uint32_t tb = 0;
#pragma unroll
                for (int c = 0; c < NCH; ++c) tb |= isT[c] ? (flag & (1u << c)) : 0u;
                flag = fe | tb;
                wave_sync();
            }
            err |= perr;
            STAMP(13)
            bool walked = false;
            if constexpr (!DELTA)
                walked = dense_awset_walk<NCH>(m, key, step, N, n, ms, R, lane, lt, em, U, err);
            else if constexpr (NCH == 4) {
                if (CRDT_FOLD_DIAG_SKIP_WALK) {  // diagnostic: nothing resolved, nothing written
                    walked = true;
                    U = 0;
#pragma unroll
                    for (int q = 0; q < NCH; ++q) em.off[q] = kOOB, em.k[q] = key[q], em.a[q] = flag, em.c[q] = 0;
                } else {
                    walked = dense_delta_walk(m, key, step, isE, isT, flag, full_mask, noop_mask, N, n, ms, R, lane,
                                              lt, em, U STAMP_ARGS);
                }
            }
            if (LEAN && !walked) {  // left to the general kernel: nothing written here
                deferred = true;
                if (lane == 0) push_defer(wk, cur.d, n_docs);
#pragma unroll
                for (int q = 0; q < NCH; ++q) em.off[q] = kOOB;
                U = 0;
            }
            if constexpr (!LEAN) if (!walked) {
            // keep + tag, compacted in place over m.tk (every read of m.tk is done)
            uint32_t Kc = 0;
#pragma unroll
            for (int c = 0; c < NCH; ++c) {
                if ((uint32_t)c < NQ) {
                    const uint32_t i = c * 64u + lane;
                    const uint32_t j = step[c] & 63u;
                    const bool fj = (full_mask >> j) & 1ull, nj = (noop_mask >> j) & 1ull;
                    const bool f = (flag >> c) & 1u;
                    const bool kept =
                        (i < n) || (isE[c] && !nj && (fj || f)) || (DELTA && isT[c] && !nj && !fj && f);
                    const uint32_t tag =
                        (isE[c] || isT[c]) ? ((((j + 1u) * 2u + (isT[c] ? 1u : 0u)) << 8) | i) : i;
                    const uint64_t km = ballot(kept);
                    const uint32_t pos = Kc + below(km);
                    if (kept) {
                        m.tk[pos] = key[c];
                        m.stag[pos] = (uint16_t)tag;
                    }
                    Kc += popc(km);
                }
            }
            wave_sync();
            STAMP(4)
            if constexpr (NCH == 4)
                U = Kc <= 64    ? sort_resolve<1, DELTA>(m, Kc, ms, R, full_mask, lane, lt, em, err STAMP_ARGS)
                    : Kc <= 128 ? sort_resolve<2, DELTA>(m, Kc, ms, R, full_mask, lane, lt, em, err STAMP_ARGS)
                                : sort_resolve<4, DELTA>(m, Kc, ms, R, full_mask, lane, lt, em, err STAMP_ARGS);
            else
                U = Kc <= 64 ? sort_resolve<1, DELTA>(m, Kc, ms, R, full_mask, lane, lt, em, err STAMP_ARGS)
                             : sort_resolve<2, DELTA>(m, Kc, ms, R, full_mask, lane, lt, em, err STAMP_ARGS);
            }
            }  // !kFused
            STAMP(5)
        }
        // ---- write the survivors (every store unconditional)
        const uint32_t obase = cur.doff + cur.e0;
        const uint32_t capo = cur.big ? 0u : min(cur.slots + cur.E, (uint32_t)Smem::NCAP);
        const rsrc_t ok = make_rsrc(out.keys + obase, capo * 8u), oa = make_rsrc(out.actors + obase, capo * 4u),
                     oc = make_rsrc(out.counters + obase, capo * 8u);
        if (cur.big) {
#pragma unroll
            for (int q = 0; q < NCH; ++q) em.off[q] = kOOB;
            U = 0;
        }
#if CRDT_FOLD_NO_STORES  // diagnostic bound (tools/fold_probe): the survivors are not written
#pragma unroll
        for (int q = 0; q < NCH; ++q) {
            st64<kFoldStoreAux>(em.k[q], ok, kOOB);
            st32<kFoldStoreAux>(em.a[q], oa, kOOB);
            st64<kFoldStoreAux>(em.c[q], oc, kOOB);
        }
#elif CRDT_FOLD_STAGE_STORES
        // The survivors are placed by output slot in LDS (tk / ta / tc are dead
        // once the resolve is done), then each array is written lane l -> slot
        // c * 64 + l: every store instruction covers contiguous whole lines.
        wave_sync();
#pragma unroll
        for (int q = 0; q < NCH; ++q) {
            const uint32_t o = em.off[q];
            if (o != kOOB) {
                m.tk[o] = em.k[q];
                m.ta[o] = em.a[q];
                m.tc[o] = em.c[q];
            }
        }
        wave_sync();
        if constexpr (CRDT_FOLD_STAGE_STORES == 2) {
            // 16 bytes a lane: 128 keys / counters or 256 actors per store
            // instruction (the descriptors end at the last survivor, and the
            // range check drops each dword past it)
            const rsrc_t sk = make_rsrc(out.keys + obase, min(U, capo) * 8u);
            const rsrc_t sa = make_rsrc(out.actors + obase, min(U, capo) * 4u);
            const rsrc_t sc = make_rsrc(out.counters + obase, min(U, capo) * 8u);
#pragma unroll
            for (int h = 0; h < (NCH + 1) / 2; ++h) {
                const uint32_t i = h * 128u + 2u * lane;
                const bool in = i < (uint32_t)Smem::NCAP;
                const uint32_t ii = in ? i : 0u;
                const u32x4 kv = *reinterpret_cast<const u32x4*>(&m.tk[ii]);
                const u32x4 cv = *reinterpret_cast<const u32x4*>(&m.tc[ii]);
                __builtin_amdgcn_raw_buffer_store_b128(kv, sk, (int)(in ? i * 8u : kOOB), 0, kFoldStoreAux);
                __builtin_amdgcn_raw_buffer_store_b128(cv, sc, (int)(in ? i * 8u : kOOB), 0, kFoldStoreAux);
            }
#pragma unroll
            for (int g = 0; g < (NCH + 3) / 4; ++g) {
                const uint32_t i = g * 256u + 4u * lane;
                const bool in = i < (uint32_t)Smem::NCAP;
                const u32x4 av = *reinterpret_cast<const u32x4*>(&m.ta[in ? i : 0u]);
                __builtin_amdgcn_raw_buffer_store_b128(av, sa, (int)(in ? i * 4u : kOOB), 0, kFoldStoreAux);
            }
        } else {
            const uint32_t nw = min(U, capo);
            uint32_t n8 = nw, n4 = nw;
            if (CRDT_FOLD_PAD_STORES && nw != 0) {
                n8 = min(((obase + nw + 15u) & ~15u) - obase, capo);
                n4 = min(((obase + nw + 31u) & ~31u) - obase, capo);
            }
            const rsrc_t sk = make_rsrc(out.keys + obase, n8 * 8u);
            const rsrc_t sa = make_rsrc(out.actors + obase, n4 * 4u);
            const rsrc_t sc = make_rsrc(out.counters + obase, n8 * 8u);
#pragma unroll
            for (int q = 0; q < NCH; ++q) {
                const uint32_t i = q * 64u + lane;
                st64<kFoldStoreAux>(m.tk[i], sk, i * 8u);
                st32<kFoldStoreAux>(m.ta[i], sa, i * 4u);
                st64<kFoldStoreAux>(m.tc[i], sc, i * 8u);
            }
        }
#else
#pragma unroll
        for (int q = 0; q < WQ; ++q) {
            const uint32_t o = em.off[q];
            const uint32_t o8 = o == kOOB ? kOOB : o * 8u, o4 = o == kOOB ? kOOB : o * 4u;
            st64<kFoldStoreAux>(em.k[q], ok, o8);
            st32<kFoldStoreAux>(em.a[q], oa, o4);
            st64<kFoldStoreAux>(em.c[q], oc, o8);
        }
#endif
#if CRDT_FOLD_PAD_VMEM  // diagnostic: N more (all out-of-range) store instructions per document
#pragma unroll
        for (int i = 0; i < CRDT_FOLD_PAD_VMEM; ++i) st64<kFoldStoreAux>(em.k[0], ok, kOOB + 8u * i);
#endif
        const uint32_t carry = U;
        const bool none = cur.big || deferred;
        st32(carry, make_rsrc(out.counts + cur.d, none ? 0u : 4u), lane == 0 ? 0u : kOOB);
        st64(vfin, make_rsrc(out.vv + (size_t)cur.d * R, none ? 0u : R * 8u), lane * 8u);
        wave_sync();
        STAMP(6)
    }
    STAMP_FLUSH
    flag_error(wk.status, err);
}

template <int NT, int IPT>
__global__ __launch_bounds__(NT) void fold_block_kernel(int mode, BatchView dst, SrcView sb, OutView out, Scratch scr,
                                                        Work wk) {
    __shared__ MergeSmem<NT, IPT> sm;
    const uint32_t tid = threadIdx.x;
    const uint32_t R = dst.R;
    uint32_t err = 0;
    if (work_total(wk, dst.n_docs) == 0) return;  // empty worklist (set by the previous launch): no dispensing atomics
    for (;;) {
        if (tid == 0) sm.word[0] = atomicAdd(wk.wl_head, 1u);
        __syncthreads();
        const uint32_t slot = sm.word[0];
        const uint32_t total = work_total(wk, dst.n_docs);
        __syncthreads();
        if (slot >= total) break;
        const uint32_t d = wk.worklist[slot];
        if (d >= dst.n_docs) {  // not a document of this call: never dereferenced
            if (tid == 0) atomicOr(wk.status, kErrWorkspace);
            continue;
        }
        const uint32_t s0 = sb.doc_srcs[d], s1 = sb.doc_srcs[d + 1];
        const uint32_t doff = dst.offsets[d];
        const uint32_t dslots = dst.offsets[d + 1] - doff;
        const uint32_t obase = doff + sb.entry_off[s0];
        const uint64_t cap = (uint64_t)dslots + (sb.entry_off[s1] - sb.entry_off[s0]);
        if ((uint64_t)obase + cap > scr.slots) {  // crdt_ctx_reserve was not told enough slots
            if (tid == 0) atomicOr(wk.status, kErrWorkspace);
            __syncthreads();
            continue;
        }
        const EntriesOut O{out.keys + obase, out.actors + obase, out.counters + obase};
        const EntriesOut X{scr.keys + obase, scr.actors + obase, scr.counters + obase};
        const uint32_t live = live_count(dst.offsets, dst.counts, d);
        if (live > dslots && tid == 0) atomicOr(wk.status, kErrCapacity);
        Entries cur{dst.keys + doff, dst.actors + doff, dst.counters + doff, live < dslots ? live : dslots};
        int where = 0;  // 0 = input, 1 = out, 2 = scratch
        if (tid < R) sm.dvv[tid] = dst.vv[(size_t)d * R + tid];
        __syncthreads();
        bool stop = false;
        for (uint32_t k = s0; k < s1 && !stop; ++k) {
            const uint32_t e0 = sb.entry_off[k];
            const Entries S{sb.keys + e0, sb.actors + e0, sb.counters + e0, sb.entry_off[k + 1] - e0};
            Entries Tm{nullptr, nullptr, nullptr, 0};
            if (sb.tomb_off && mode == CRDT_FOLD_DELTA) {
                const uint32_t t0 = sb.tomb_off[k];
                Tm = Entries{sb.tkeys + t0, sb.tactors + t0, sb.tcounters + t0, sb.tomb_off[k + 1] - t0};
            }
            if (tid < R) sm.svv[tid] = sb.vv[(size_t)k * R + tid];
            __syncthreads();
            uint32_t perr = 0;
            const bool full = (mode != CRDT_FOLD_DELTA) || vv_counter(sm.dvv, R, sb.src_actor[k], perr) == 0;
            if (perr) {
                err |= perr;
                stop = true;
                break;
            }
            if (!full) {
                bool any = false;
                for (uint32_t e = tid; e < S.n; e += NT) any |= !has_dot(sm.dvv, R, S.a[e], S.c[e], err);
                for (uint32_t t = tid; t < Tm.n; t += NT) {
                    const uint32_t g = lower_bound(S.k, S.n, Tm.k[t]);
                    const bool in_s = g < S.n && S.k[g] == Tm.k[t];
                    any |= !(in_s && (S.a[g] != Tm.a[t] || S.c[g] > Tm.c[t]));
                }
                if (!__syncthreads_or(any)) continue;
            }
            const EntriesOut& tgt = (where == 1) ? X : O;
            const uint32_t n = block_merge<NT, IPT>(cur, S, full ? Entries{nullptr, nullptr, nullptr, 0} : Tm, full, R,
                                                    sm, tgt, err);
            if (tid < R) sm.dvv[tid] = max(sm.dvv[tid], sm.svv[tid]);
            where = (where == 1) ? 2 : 1;
            cur = Entries{tgt.k, tgt.a, tgt.c, n};
            __syncthreads();
        }
        if (where != 1) {  // result still in the input or the scratch copy
            for (uint32_t i = tid; i < cur.n; i += NT) {
                O.k[i] = cur.k[i];
                O.a[i] = cur.a[i];
                O.c[i] = cur.c[i];
            }
        }
        if (tid == 0) out.counts[d] = cur.n;
        if (tid < R) out.vv[(size_t)d * R + tid] = sm.dvv[tid];
        __syncthreads();
    }
    if (__syncthreads_or(err != 0) && tid == 0) atomicOr(wk.status, kErrActorRange);
}

constexpr int kFoldNT = 256;
constexpr int kFoldIPT = 4;

// lean_first: the lean slot-walk pass over every document, then
// the general kernel over the documents it deferred (grid sized for all of
// them; runs past the deferred count exit at once); otherwise the general
// kernel over every document.
hipError_t launch_fold(int mode, const BatchView& dst, const SrcView& sb, const OutView& out, const Scratch& scr,
                       const Work& wk, uint32_t block_grid, bool lean_first, hipStream_t stream) {
    if (dst.n_docs == 0) return hipSuccess;
    const uint32_t grid = (dst.n_docs + kFoldWaves * kFoldK - 1) / (kFoldWaves * kFoldK);
    const uint32_t grid_d = (dst.n_docs + kFoldWavesD * kFoldKD - 1) / (kFoldWavesD * kFoldKD);
    if (mode == CRDT_FOLD_DELTA && lean_first) {
        hipLaunchKernelGGL((fold_pipe_kernel<kFoldKD, true, true, false>), dim3(grid_d), dim3(kFoldWavesD * 64), 0,
                           stream, dst, sb, out, wk);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL((fold_pipe_kernel<kFoldKD, true, false, true>), dim3(grid_d), dim3(kFoldWavesD * 64), 0,
                           stream, dst, sb, out, wk);
    } else if (mode == CRDT_FOLD_DELTA) {
        hipLaunchKernelGGL((fold_pipe_kernel<kFoldKD, true, false, false>), dim3(grid_d), dim3(kFoldWavesD * 64), 0,
                           stream, dst, sb, out, wk);
    } else if (lean_first) {
        hipLaunchKernelGGL((fold_pipe_kernel<kFoldK, false, true, false>), dim3(grid), dim3(kFoldWaves * 64), 0,
                           stream, dst, sb, out, wk);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL((fold_pipe_kernel<kFoldK, false, false, true>), dim3(grid), dim3(kFoldWaves * 64), 0,
                           stream, dst, sb, out, wk);
    } else {
        hipLaunchKernelGGL((fold_pipe_kernel<kFoldK, false, false, false>), dim3(grid), dim3(kFoldWaves * 64), 0,
                           stream, dst, sb, out, wk);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((fold_block_kernel<kFoldNT, kFoldIPT>), dim3(block_grid), dim3(kFoldNT), 0, stream, mode, dst,
                       sb, out, scr, wk);
    return hipGetLastError();
}

}  // namespace crdt
