// Batched local operations on the device: the state producers of the merge
// path, applied to many documents at once.
//
//   CRDT_OP_ADD            (*AWSet).Add(k)          awset.go:89-94
//                          vv[actor]++; entries[k] = {actor, vv[actor]}
//   CRDT_OP_DEL            (*AWSet).Del(k)          awset.go:96-101
//                          delete(entries, k); the clock is not bumped
//   CRDT_OP_DELTA_DEL      (*AWSetDelta).Del(k...)  awset-delta_test.go:14-33:
//                          one call: vv[actor]++ once, dot2 = {actor, vv[actor]}
//   CRDT_OP_DELTA_DEL_KEY  a key of that call: if k is in entries,
//                          Deleted[k] = dot2 and the entry is removed
//
// The per-key view (one wavefront per document, <= 256 ops per call):
//   * a bumping op's clock is vv0[actor] + the number of bumping ops up to and
//     including it (a prefix count in op order);
//   * a key's fate depends only on its own ops, in op order: presence after
//     its last op is "that op is an ADD" (no ops: unchanged); a DELTA_DEL_KEY
//     is effective (records a tombstone) iff the key is present just before
//     it, i.e. its previous op on the key is an ADD, or it is the key's first
//     op and the key is in the state;
// so the ops are sorted by (key, op index) in registers (wave_sort.hpp), each
// key's run is resolved with neighbour tests and one segmented scan, and the
// state is then streamed once: every state entry and tombstone computes its
// own output slot from the resolved keys (a lower bound in LDS plus prefix
// counts), with no scan over the state.
#include "crdt_device.hpp"
#include "wave_sort.hpp"

namespace crdt {

constexpr int kApplyWaves = 2;
constexpr int kApplyEPL = 4;
constexpr uint32_t kApplyMaxOps = kApplyEPL * 64;  // CRDT_MAX_OPS_PER_DOC

constexpr uint32_t kOpAdd = CRDT_OP_ADD, kOpDel = CRDT_OP_DEL, kOpDDel = CRDT_OP_DELTA_DEL,
                   kOpDDelKey = CRDT_OP_DELTA_DEL_KEY;

struct ApplyWaveSmem {
    uint64_t okey[kApplyMaxOps];  // by op index
    uint64_t octr[kApplyMaxOps];  // clock of a bumping op / tombstone dot of a DELTA_DEL_KEY
    uint32_t okind[kApplyMaxOps];
    uint64_t skey[kApplyMaxOps + 1];  // sorted (key, op index); element n_keyed = sentinel
    uint32_t stag[kApplyMaxOps + 1];
    uint32_t slb[kApplyMaxOps];   // at a run head: # state entries with key < k; bit 31: k in state
    // resolved keys (one per run), key order
    uint64_t rkey[kApplyMaxOps];
    uint64_t rctr[kApplyMaxOps];   // dot counter when present
    uint64_t rtctr[kApplyMaxOps];  // new tombstone counter
    uint32_t rflag[kApplyMaxOps];  // bit0 in state, bit1 present after, bit2 new tombstone, bit3 key in tombs
    uint32_t rlb[kApplyMaxOps];    // # state entries < key
    uint32_t rtlb[kApplyMaxOps];   // # tombstones < key (new tombstones only)
    uint32_t rem_before[kApplyMaxOps + 1];  // removed state entries among resolved keys before r
    uint32_t ins_before[kApplyMaxOps + 1];  // inserted entries before r
    uint32_t tins_before[kApplyMaxOps + 1]; // inserted tombstones before r
    uint64_t vv[CRDT_MAX_R];
};

// lower bound in a sorted global array (the document's state keys)
__device__ __forceinline__ uint32_t lb_global(const uint64_t* a, uint32_t n, uint64_t key) {
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a[mid] < key)
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo;
}

// Exclusive prefix over EPL*64 elements (element e = lane*EPL + q) of 0/1 flags;
// writes pre[e] for e <= n (pre[n] = total).
template <int EPL>
__device__ __forceinline__ void flag_prefix(const bool (&f)[EPL], uint32_t* pre, uint32_t n, uint32_t lane,
                                            uint64_t lt) {
    uint32_t c = 0;
#pragma unroll
    for (int q = 0; q < EPL; ++q) c += f[q] ? 1u : 0u;
    uint32_t base;
    const uint32_t tot = lane_prefix_small(c, lt, base);
#pragma unroll
    for (int q = 0; q < EPL; ++q) {
        const uint32_t e = lane * EPL + q;
        if (e < n) pre[e] = base;
        base += f[q] ? 1u : 0u;
    }
    if (lane == 0) pre[n] = tot;
}

template <int WAVES>
__global__ __launch_bounds__(WAVES * 64) void apply_kernel(BatchView st, TombView tb, ApplyOps ops, OutView out,
                                                           TombOut tout, uint32_t has_tout, Work wk) {
    constexpr int EPL = kApplyEPL;
    __shared__ ApplyWaveSmem smem[WAVES];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    ApplyWaveSmem& sm = smem[w];
    const uint64_t lt = low_mask(lane);
    const uint32_t R = st.R, n_docs = st.n_docs;
    uint32_t err = 0;
    const uint32_t end_off = st.offsets[n_docs] + ops.op_off[n_docs];
    const uint32_t tend_off = (tb.offsets ? tb.offsets[n_docs] : 0u) + ops.op_off[n_docs];

    for (uint32_t d = uniform(blockIdx.x * WAVES + w); d < n_docs; d += gridDim.x * WAVES) {
        const uint32_t o0 = ops.op_off[d], nops = ops.op_off[d + 1] - o0;
        const uint32_t actor = ops.doc_actor[d];
        const uint32_t soff = st.offsets[d], ns = live_count(st.offsets, st.counts, d);
        const uint32_t toff = tb.offsets ? tb.offsets[d] : 0u, nt = tb.offsets ? live_count(tb.offsets, tb.counts, d) : 0u;
        const uint32_t obase = soff + o0, tbase = toff + o0;
        // slot bounds of every doc (outputs are valid input batches)
        if (lane == 0) {
            out.offsets[d] = obase;
            if (d == n_docs - 1) out.offsets[n_docs] = end_off;
            if (has_tout) {
                tout.offsets[d] = tbase;
                if (d == n_docs - 1) tout.offsets[n_docs] = tend_off;
            }
        }
        if (nops > kApplyMaxOps) {  // one call holds at most 256 ops per doc (outputs of d undefined)
            err |= kErrHint;
            continue;
        }
        uint32_t derr = 0;
        if (lane < R) sm.vv[lane] = st.vv[(size_t)d * R + lane];
        // ---- ops by index: kind, key
#pragma unroll
        for (int q = 0; q < EPL; ++q) {
            const uint32_t j = lane + q * 64;
            if (j < nops) {
                sm.okind[j] = ops.kind[o0 + j];
                sm.okey[j] = ops.keys[o0 + j];
            }
        }
        wave_sync();
        // ---- clocks: prefix count of bumping ops in op order (element j = lane*EPL + q)
        const uint64_t clock0 = actor < R ? sm.vv[actor] : 0ull;
        bool bump[EPL], keyed[EPL];
        uint32_t kind[EPL];
        uint32_t nb = 0, nk = 0;
#pragma unroll
        for (int q = 0; q < EPL; ++q) {
            const uint32_t j = lane * EPL + q;
            const bool v = j < nops;
            kind[q] = v ? sm.okind[j] : kOpDel;
            bump[q] = v && (kind[q] == kOpAdd || kind[q] == kOpDDel);
            keyed[q] = v && kind[q] != kOpDDel;
            nb += bump[q] ? 1u : 0u;
            nk += keyed[q] ? 1u : 0u;
            if (v) {
                // a DELTA_DEL_KEY belongs to the DELTA_DEL call just before it
                const uint32_t pk = j > 0 ? sm.okind[j - 1] : 0xFFu;
                if (kind[q] > kOpDDelKey || (kind[q] == kOpDDelKey && pk != kOpDDel && pk != kOpDDelKey) ||
                    (kind[q] == kOpDDelKey && !has_tout))
                    derr |= kErrHint;
                if (bump[q] && actor >= R) derr |= kErrActorRange;  // VersionVector[actor]++ out of range
            }
        }
        if (ballot(derr != 0)) {  // the reference panics (or the ops are malformed): outputs of d undefined
            err |= derr;
            wave_sync();
            continue;
        }
        uint32_t bpre, kpre;
        const uint32_t nbumps = lane_prefix_small(nb, lt, bpre);
        const uint32_t n_keyed = lane_prefix_small(nk, lt, kpre);
        // per op: its dot counter; keyed ops compacted into the sort input
#pragma unroll
        for (int q = 0; q < EPL; ++q) {
            const uint32_t j = lane * EPL + q;
            bpre += bump[q] ? 1u : 0u;
            if (j < nops) sm.octr[j] = clock0 + bpre;  // ADD: its own bump; DDK: its call's bump
            if (keyed[q]) {
                sm.skey[kpre] = sm.okey[j];
                sm.stag[kpre] = j;
            }
            kpre += keyed[q] ? 1u : 0u;
        }
        wave_sync();
        // ---- sort keyed ops by (key, op index)
        uint64_t k[EPL];
        uint32_t t[EPL];
#pragma unroll
        for (int q = 0; q < EPL; ++q) {
            const uint32_t e = lane * EPL + q;
            k[q] = e < n_keyed ? sm.skey[e] : ~0ull;
            t[q] = e < n_keyed ? sm.stag[e] : 0xFFFFu;
        }
        wave_sync();
        wave_sort_pairs<EPL>(k, t, n_keyed, lane);
#pragma unroll
        for (int q = 0; q < EPL; ++q) {
            const uint32_t e = lane * EPL + q;
            sm.skey[e] = k[q];
            sm.stag[e] = t[q];
        }
        if (lane == 0) {
            sm.skey[n_keyed] = ~0ull;
            sm.stag[n_keyed] = 0xFFFFu;
        }
        wave_sync();
        // ---- runs: heads look the key up in the state
        const uint64_t* skeys = st.keys + soff;
        bool head[EPL], last[EPL];
#pragma unroll
        for (int q = 0; q < EPL; ++q) {
            const uint32_t e = lane * EPL + q;
            const bool v = e < n_keyed;
            head[q] = v && (e == 0 || sm.skey[e - 1] != k[q]);
            last[q] = v && (e + 1 == n_keyed || sm.skey[e + 1] != k[q]);
            if (head[q]) {
                const uint32_t lb = lb_global(skeys, ns, k[q]);
                const bool in = lb < ns && skeys[lb] == k[q];
                sm.slb[e] = lb | (in ? 0x80000000u : 0u);
            }
        }
        wave_sync();
        // effective tombstones: mark heads (run boundary) and effective DELTA_DEL_KEYs
        uint32_t mk[EPL], hd[EPL], inc[EPL], exc[EPL], hinc[EPL], hexc[EPL];
#pragma unroll
        for (int q = 0; q < EPL; ++q) {
            const uint32_t e = lane * EPL + q;
            bool eff = false;
            if (e < n_keyed && sm.okind[t[q]] == kOpDDelKey) {
                const bool present_before =
                    head[q] ? (sm.slb[e] >> 31) != 0 : sm.okind[sm.stag[e - 1]] == kOpAdd;
                eff = present_before;
            }
            mk[q] = eff ? (0x80000000u | e) : (head[q] ? 0xFFFFFFFFu : 0u);  // 0x7FFFFFFF payload = none
            hd[q] = head[q] ? (0x80000000u | e) : 0u;
        }
        scan_last_marked<EPL>(mk, inc, exc);
        scan_last_marked<EPL>(hd, hinc, hexc);
        // ---- one resolved key per run (at its last op), compacted in key order
        uint32_t nl = 0;
#pragma unroll
        for (int q = 0; q < EPL; ++q) nl += last[q] ? 1u : 0u;
        uint32_t rpos;
        const uint32_t m = lane_prefix_small(nl, lt, rpos);
#pragma unroll
        for (int q = 0; q < EPL; ++q) {
            if (last[q]) {
                const uint32_t he = hinc[q] & 0x7FFFFFFFu;
                const uint32_t lbw = sm.slb[he];
                const bool in = (lbw >> 31) != 0;
                const uint32_t lk = sm.okind[t[q]];
                const bool present = lk == kOpAdd;
                const uint32_t te = inc[q] & 0x7FFFFFFFu;
                const bool ntomb = te != 0x7FFFFFFFu;
                uint32_t f = (in ? 1u : 0u) | (present ? 2u : 0u) | (ntomb ? 4u : 0u);
                uint32_t tlb = 0;
                if (ntomb) {
                    tlb = lb_global(tb.keys + toff, nt, k[q]);
                    if (tlb < nt && tb.keys[toff + tlb] == k[q]) f |= 8u;
                }
                sm.rkey[rpos] = k[q];
                sm.rctr[rpos] = sm.octr[t[q]];
                sm.rtctr[rpos] = ntomb ? sm.octr[sm.stag[te]] : 0ull;
                sm.rflag[rpos] = f;
                sm.rlb[rpos] = lbw & 0x7FFFFFFFu;
                sm.rtlb[rpos] = tlb;
                ++rpos;
            }
        }
        wave_sync();
        // ---- prefix counts over the resolved keys
        {
            bool rem[EPL], ins[EPL], tins[EPL];
#pragma unroll
            for (int q = 0; q < EPL; ++q) {
                const uint32_t r = lane * EPL + q;
                const uint32_t f = r < m ? sm.rflag[r] : 0u;
                rem[q] = (f & 3u) == 1u;   // in state, absent after
                ins[q] = (f & 3u) == 2u;   // not in state, present after
                tins[q] = (f & 12u) == 4u; // new tombstone for a key without one
            }
            flag_prefix<EPL>(rem, sm.rem_before, m, lane, lt);
            flag_prefix<EPL>(ins, sm.ins_before, m, lane, lt);
            flag_prefix<EPL>(tins, sm.tins_before, m, lane, lt);
        }
        wave_sync();
        // ---- inserted entries and tombstones
#pragma unroll
        for (int q = 0; q < EPL; ++q) {
            const uint32_t r = lane + q * 64;
            if (r < m) {
                const uint32_t f = sm.rflag[r];
                if ((f & 3u) == 2u) {
                    const uint32_t pos = sm.rlb[r] - sm.rem_before[r] + sm.ins_before[r];
                    out.keys[obase + pos] = sm.rkey[r];
                    out.actors[obase + pos] = actor;
                    out.counters[obase + pos] = sm.rctr[r];
                }
                if ((f & 12u) == 4u) {
                    const uint32_t pos = sm.rtlb[r] + sm.tins_before[r];
                    tout.keys[tbase + pos] = sm.rkey[r];
                    tout.actors[tbase + pos] = actor;
                    tout.counters[tbase + pos] = sm.rtctr[r];
                }
            }
        }
        // ---- stream the state: each entry finds its resolved key (if any) and its slot
        for (uint32_t i = lane; i < ns; i += 64) {
            const uint64_t key = st.keys[soff + i];
            const uint32_t r = lower_bound(sm.rkey, m, key);
            const bool hit = r < m && sm.rkey[r] == key;
            const uint32_t f = hit ? sm.rflag[r] : 0u;
            if (hit && !(f & 2u)) continue;  // deleted by an op
            const uint32_t pos = i - sm.rem_before[r] + sm.ins_before[r];
            out.keys[obase + pos] = key;
            out.actors[obase + pos] = hit ? actor : st.actors[soff + i];
            out.counters[obase + pos] = hit ? sm.rctr[r] : st.counters[soff + i];
        }
        for (uint32_t i = lane; i < nt; i += 64) {
            const uint64_t key = tb.keys[toff + i];
            const uint32_t r = lower_bound(sm.rkey, m, key);
            const bool hit = r < m && sm.rkey[r] == key && (sm.rflag[r] & 4u);
            const uint32_t pos = i + sm.tins_before[r];
            tout.keys[tbase + pos] = key;
            tout.actors[tbase + pos] = hit ? actor : tb.actors[toff + i];
            tout.counters[tbase + pos] = hit ? sm.rtctr[r] : tb.counters[toff + i];
        }
        if (lane == 0) {
            out.counts[d] = ns - sm.rem_before[m] + sm.ins_before[m];
            if (has_tout) tout.counts[d] = nt + sm.tins_before[m];
        }
        if (lane < R) out.vv[(size_t)d * R + lane] = sm.vv[lane] + (lane == actor ? (uint64_t)nbumps : 0ull);
        wave_sync();
    }
    flag_error(wk.status, err);
}

// Opt-in tombstone GC (crdt_tombstone_gc_async): one wavefront per doc keeps
// the tombstones the doc's stable clock has not covered, compacted in order
// with one ballot per 64 (gcDeleted, awset-delta_test.go:67-77, is empty in the
// reference; see include/crdtgpu.h for the rule).
__global__ __launch_bounds__(256) void tomb_gc_kernel(TombView tb, uint32_t n_docs, uint32_t R, const uint64_t* stable,
                                                      TombOut out) {
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t d = uniform(blockIdx.x * 4 + (threadIdx.x >> 6)); d < n_docs; d += gridDim.x * 4) {
        const uint32_t o = tb.offsets[d], n = live_count(tb.offsets, tb.counts, d);
        const uint64_t* vv = stable + (size_t)d * R;
        uint32_t kept = 0;
        for (uint32_t base = 0; base < n; base += 64) {
            const uint32_t i = base + lane;
            const bool v = i < n;
            uint64_t k = 0, c = 0;
            uint32_t a = 0;
            if (v) {
                k = tb.keys[o + i];
                a = tb.actors[o + i];
                c = tb.counters[o + i];
            }
            const bool covered = v && a < R && vv[a] >= c;  // HasDot, crdt-misc.go:28-34
            const bool keep = v && !covered;
            const uint64_t m = ballot(keep);
            if (keep) {
                const uint32_t pos = kept + below(m);
                out.keys[o + pos] = k;
                out.actors[o + pos] = a;
                out.counters[o + pos] = c;
            }
            kept += popc(m);
        }
        if (lane == 0) {
            out.counts[d] = kept;
            out.offsets[d] = o;
            if (d == n_docs - 1) out.offsets[n_docs] = tb.offsets[n_docs];
        }
    }
}

hipError_t launch_tomb_gc(const TombView& tb, uint32_t n_docs, uint32_t R, const uint64_t* stable, const TombOut& out,
                          uint32_t n_cu, hipStream_t stream) {
    if (n_docs == 0) return hipSuccess;
    const uint32_t grid = min((n_docs + 3) / 4, n_cu * 16u);
    hipLaunchKernelGGL(tomb_gc_kernel, dim3(grid), dim3(256), 0, stream, tb, n_docs, R, stable, out);
    return hipGetLastError();
}

hipError_t launch_apply(const BatchView& st, const TombView& tb, const ApplyOps& ops, const OutView& out,
                        const TombOut& tout, bool has_tout, const Work& wk, uint32_t n_cu, hipStream_t stream) {
    if (st.n_docs == 0) return hipSuccess;
    const uint32_t need = (st.n_docs + kApplyWaves - 1) / kApplyWaves;
    const uint32_t grid = min(need, n_cu * 16u);
    hipLaunchKernelGGL((apply_kernel<kApplyWaves>), dim3(grid), dim3(kApplyWaves * 64), 0, stream, st, tb, ops, out,
                       tout, (uint32_t)has_tout, wk);
    return hipGetLastError();
}

}  // namespace crdt
