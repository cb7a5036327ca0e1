// In-register sorting of one wavefront's (key, tag) pairs on gfx950, shared by
// the fold (fold.hip) and the batched local ops (apply.hip).  Element i of a
// wavefront's EPL*64 pairs lives in lane i / EPL, slot i % EPL.  Lane
// exchanges use DPP inside rows of 16 lanes and the gfx950 permlane swaps
// across rows: VALU only, no LDS traffic.
#pragma once

#include "crdt_device.hpp"

namespace crdt {

__device__ __forceinline__ bool tup_less(uint64_t ka, uint32_t ta, uint64_t kb, uint32_t tb) {
    return ka < kb || (ka == kb && ta < tb);
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, uint32_t i) {
    return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, (int)i) |
           ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), (int)i) << 32);
}

// The value of lane (lane ^ LM).
template <int LM>
__device__ __forceinline__ uint32_t lane_xor(uint32_t v, uint32_t lane) {
    if constexpr (LM == 1) {
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
    } else if constexpr (LM == 2) {
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
    } else if constexpr (LM == 4) {
        const int h = __builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, false);  // row_half_mirror: i -> 7-i
        return (uint32_t)__builtin_amdgcn_mov_dpp(h, 0x1B, 0xF, 0xF, false);       // quad_perm [3,2,1,0]
    } else if constexpr (LM == 8) {
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xF, 0xF, false);  // row_ror:8
    } else if constexpr (LM == 16) {
        // swaps row 1 of the first operand with row 0 of the second (and rows 3 / 2)
        const auto p = __builtin_amdgcn_permlane16_swap(v, v, false, false);
        return (lane & 16) ? p[0] : p[1];
    } else {
        static_assert(LM == 32, "lane_xor: LM must be a power of two below 64");
        const auto p = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        return (lane & 32) ? p[0] : p[1];
    }
}

// Element i keeps the smaller of its pair at stage (KK, JJ) iff its position
// in the pair (lower: bit JJ of i clear) agrees with the merge's direction
// (ascending: bit KK of i clear).
template <int EPL, int KK, int JJ>
__device__ __forceinline__ bool keeps_min(uint32_t lane, int q) {
    const uint32_t i = lane * EPL + (uint32_t)q;
    return ((i & JJ) == 0) == ((i & KK) == 0);
}

// Bitonic network over EPL*64 (key, tag) pairs: stage (KK, JJ) and every later
// stage of the same merge.  Pairs are distinct or identical, so "take the
// partner" is simply (partner < own) == keeps_min: one comparison per element.
template <int EPL, int KK, int JJ>
__device__ __forceinline__ void bitonic_step(uint64_t (&k)[EPL], uint32_t (&t)[EPL], uint32_t lane) {
    if constexpr (JJ >= EPL) {
        constexpr int LM = JJ / EPL;
#pragma unroll
        for (int q = 0; q < EPL; ++q) {
            const uint64_t pk = (uint64_t)lane_xor<LM>((uint32_t)k[q], lane) |
                                ((uint64_t)lane_xor<LM>((uint32_t)(k[q] >> 32), lane) << 32);
            const uint32_t pt = lane_xor<LM>(t[q], lane);
            const bool take = tup_less(pk, pt, k[q], t[q]) == keeps_min<EPL, KK, JJ>(lane, q);
            k[q] = take ? pk : k[q];
            t[q] = take ? pt : t[q];
        }
    } else {
#pragma unroll
        for (int q = 0; q < EPL; ++q) {
            if (q & JJ) continue;
            const int r = q | JJ;
            const bool asc = ((lane * EPL + q) & KK) == 0;
            const bool sw = tup_less(k[r], t[r], k[q], t[q]) == asc;
            const uint64_t k0 = k[q], k1 = k[r];
            const uint32_t t0 = t[q], t1 = t[r];
            k[q] = sw ? k1 : k0;
            k[r] = sw ? k0 : k1;
            t[q] = sw ? t1 : t0;
            t[r] = sw ? t0 : t1;
        }
    }
    if constexpr (JJ > 1) bitonic_step<EPL, KK, JJ / 2>(k, t, lane);
}

// The same network over packed 64-bit values (key offset << 16 | tag): one
// 64-bit compare and one pair of selects per element and stage.
template <int EPL, int KK, int JJ>
__device__ __forceinline__ void bitonic_step_packed(uint64_t (&v)[EPL], uint32_t lane) {
    if constexpr (JJ >= EPL) {
        constexpr int LM = JJ / EPL;
#pragma unroll
        for (int q = 0; q < EPL; ++q) {
            const uint64_t pv = (uint64_t)lane_xor<LM>((uint32_t)v[q], lane) |
                                ((uint64_t)lane_xor<LM>((uint32_t)(v[q] >> 32), lane) << 32);
            const bool take = (pv < v[q]) == keeps_min<EPL, KK, JJ>(lane, q);
            v[q] = take ? pv : v[q];
        }
    } else {
#pragma unroll
        for (int q = 0; q < EPL; ++q) {
            if (q & JJ) continue;
            const int r = q | JJ;
            const bool asc = ((lane * EPL + q) & KK) == 0;
            const uint64_t lo = v[q] < v[r] ? v[q] : v[r], hi = v[q] < v[r] ? v[r] : v[q];
            v[q] = asc ? lo : hi;
            v[r] = asc ? hi : lo;
        }
    }
    if constexpr (JJ > 1) bitonic_step_packed<EPL, KK, JJ / 2>(v, lane);
}

// The network over packed 32-bit values ((key offset) << 16 | tag): one DPP
// exchange, one compare and one select per element and stage.
template <int EPL, int KK, int JJ>
__device__ __forceinline__ void bitonic_step32(uint32_t (&v)[EPL], uint32_t lane) {
    if constexpr (JJ >= EPL) {
        constexpr int LM = JJ / EPL;
#pragma unroll
        for (int q = 0; q < EPL; ++q) {
            const uint32_t pv = lane_xor<LM>(v[q], lane);
            const bool take = (pv < v[q]) == keeps_min<EPL, KK, JJ>(lane, q);
            v[q] = take ? pv : v[q];
        }
    } else {
#pragma unroll
        for (int q = 0; q < EPL; ++q) {
            if (q & JJ) continue;
            const int r = q | JJ;
            const bool asc = ((lane * EPL + q) & KK) == 0;
            const uint32_t lo = min(v[q], v[r]), hi = max(v[q], v[r]);
            v[q] = asc ? lo : hi;
            v[r] = asc ? hi : lo;
        }
    }
    if constexpr (JJ > 1) bitonic_step32<EPL, KK, JJ / 2>(v, lane);
}

// Sort the wavefront's EPL*64 pairs ascending by (key, tag).
template <int EPL, int KK = 2>
__device__ __forceinline__ void wave_bitonic(uint64_t (&k)[EPL], uint32_t (&t)[EPL], uint32_t lane) {
    bitonic_step<EPL, KK, KK / 2>(k, t, lane);
    if constexpr (KK < EPL * 64) wave_bitonic<EPL, KK * 2>(k, t, lane);
}

template <int EPL, int KK = 2>
__device__ __forceinline__ void wave_bitonic32(uint32_t (&v)[EPL], uint32_t lane) {
    bitonic_step32<EPL, KK, KK / 2>(v, lane);
    if constexpr (KK < EPL * 64) wave_bitonic32<EPL, KK * 2>(v, lane);
}

template <int EPL, int KK = 2>
__device__ __forceinline__ void wave_bitonic_packed(uint64_t (&v)[EPL], uint32_t lane) {
    bitonic_step_packed<EPL, KK, KK / 2>(v, lane);
    if constexpr (KK < EPL * 64) wave_bitonic_packed<EPL, KK * 2>(v, lane);
}

// Sort n <= EPL*64 (key, tag) pairs (tags < 0xFFFF, unique per key; slots past
// n are padding).  Keys are taken relative to the first pair's key b: when
// every key lies in [b - 2^15, b + 2^15) the pair packs into 32 bits (offset
// << 16 | tag), when within [b - 2^47, b + 2^47) into 64 bits, both
// order-preserving; otherwise the 80-bit comparison runs.  Returns with the
// pairs in element order and pads (key ~0, tag 0xFFFF) last.
template <int EPL>
__device__ __forceinline__ void wave_sort_pairs(uint64_t (&k)[EPL], uint32_t (&t)[EPL], uint32_t n, uint32_t lane) {
    const uint64_t b = readlane64(k[0], 0);
    bool o16 = false, o48 = false;
#pragma unroll
    for (int q = 0; q < EPL; ++q) {
        const bool valid = lane * EPL + q < n;
        const uint64_t d = k[q] - b;
        o16 |= valid && d + 0x8000ull >= 0x10000ull;
        o48 |= valid && d + (1ull << 47) >= (1ull << 48);
    }
    if (!ballot(o16)) {
        uint32_t v[EPL];
#pragma unroll
        for (int q = 0; q < EPL; ++q)
            v[q] = lane * EPL + q < n ? ((uint32_t)(k[q] - b + 0x8000ull) << 16) | (t[q] & 0xFFFFu) : ~0u;
        wave_bitonic32<EPL>(v, lane);
#pragma unroll
        for (int q = 0; q < EPL; ++q) {
            const bool pad = v[q] == ~0u;
            k[q] = pad ? ~0ull : b - 0x8000ull + (v[q] >> 16);
            t[q] = pad ? 0xFFFFu : (v[q] & 0xFFFFu);
        }
    } else if (!ballot(o48)) {
        uint64_t v[EPL];
#pragma unroll
        for (int q = 0; q < EPL; ++q)
            v[q] = lane * EPL + q < n ? ((k[q] - b + (1ull << 47)) << 16) | (uint64_t)(t[q] & 0xFFFFu) : ~0ull;
        wave_bitonic_packed<EPL>(v, lane);
#pragma unroll
        for (int q = 0; q < EPL; ++q) {
            const bool pad = v[q] == ~0ull;
            k[q] = pad ? ~0ull : b - (1ull << 47) + (v[q] >> 16);
            t[q] = pad ? 0xFFFFu : (uint32_t)(v[q] & 0xFFFFu);
        }
    } else {
        wave_bitonic<EPL>(k, t, lane);
    }
}

// ---- DPP lane shifts and the segmented "last marked value" scan (gfx9 DPP:
// row_shr, row_bcast, wave_shl/shr; lanes with no source take `old`).
template <int CTRL, int ROWS = 0xF>
__device__ __forceinline__ uint32_t dpp(uint32_t old, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, CTRL, ROWS, 0xF, false);
}
// value of lane + 1 (lane 63: old)
__device__ __forceinline__ uint32_t from_next_lane(uint32_t old, uint32_t v) { return dpp<0x130>(old, v); }
__device__ __forceinline__ uint64_t from_next_lane64(uint64_t old, uint64_t v) {
    return (uint64_t)from_next_lane((uint32_t)old, (uint32_t)v) |
           ((uint64_t)from_next_lane((uint32_t)(old >> 32), (uint32_t)(v >> 32)) << 32);
}

// Elements carry x = 0 (unmarked) or 0x80000000 | value (marked).  incl[q] =
// the x of the last marked element at or before element q (0 if none);
// excl[q] = the same strictly before q.  Segment heads are marked by the
// caller, so nothing crosses a segment boundary.  Lane-local pass, then a
// Hillis-Steele pass over lanes with DPP (no LDS).
template <int EPL>
__device__ __forceinline__ void scan_last_marked(const uint32_t (&x)[EPL], uint32_t (&incl)[EPL], uint32_t (&excl)[EPL]) {
    uint32_t loc[EPL], acc = 0;
#pragma unroll
    for (int q = 0; q < EPL; ++q) {
        acc = (x[q] >> 31) ? x[q] : acc;
        loc[q] = acc;
    }
    uint32_t s = acc, y;
    y = dpp<0x111>(0u, s); s = (s >> 31) ? s : y;        // row_shr:1
    y = dpp<0x112>(0u, s); s = (s >> 31) ? s : y;        // row_shr:2
    y = dpp<0x114>(0u, s); s = (s >> 31) ? s : y;        // row_shr:4
    y = dpp<0x118>(0u, s); s = (s >> 31) ? s : y;        // row_shr:8
    y = dpp<0x142, 0xA>(0u, s); s = (s >> 31) ? s : y;   // row_bcast:15 -> rows 1, 3
    y = dpp<0x143, 0xC>(0u, s); s = (s >> 31) ? s : y;   // row_bcast:31 -> rows 2, 3
    uint32_t prev = dpp<0x138>(0u, s);                    // wave_shr:1: lanes before this one
#pragma unroll
    for (int q = 0; q < EPL; ++q) {
        excl[q] = prev;
        incl[q] = (loc[q] >> 31) ? loc[q] : prev;
        prev = incl[q];
    }
}

// Exclusive prefix count of per-lane counts c (<= 7) in lane order; returns the total.
__device__ __forceinline__ uint32_t lane_prefix_small(uint32_t c, uint64_t lt, uint32_t& pre) {
    uint32_t tot = 0;
    pre = 0;
#pragma unroll
    for (int b = 0; b < 3; ++b) {
        const uint64_t mb = ballot((c >> b) & 1u);
        pre += below(mb) << b;
        tot += popc(mb) << b;
    }
    return tot;
}

}  // namespace crdt
