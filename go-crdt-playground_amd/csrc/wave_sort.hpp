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

// Sort the wavefront's EPL*64 pairs ascending by (key, tag).
template <int EPL, int KK = 2>
__device__ __forceinline__ void wave_bitonic(uint64_t (&k)[EPL], uint32_t (&t)[EPL], uint32_t lane) {
    bitonic_step<EPL, KK, KK / 2>(k, t, lane);
    if constexpr (KK < EPL * 64) wave_bitonic<EPL, KK * 2>(k, t, lane);
}

template <int EPL, int KK = 2>
__device__ __forceinline__ void wave_bitonic_packed(uint64_t (&v)[EPL], uint32_t lane) {
    bitonic_step_packed<EPL, KK, KK / 2>(v, lane);
    if constexpr (KK < EPL * 64) wave_bitonic_packed<EPL, KK * 2>(v, lane);
}

// 64-bit min / max over the wavefront (every lane gets the result).
__device__ __forceinline__ uint64_t wave_min64(uint64_t x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t y = (uint64_t)__shfl_xor((unsigned long long)x, o);
        x = y < x ? y : x;
    }
    return x;
}
__device__ __forceinline__ uint64_t wave_max64(uint64_t x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t y = (uint64_t)__shfl_xor((unsigned long long)x, o);
        x = y > x ? y : x;
    }
    return x;
}

// Sort n <= EPL*64 (key, tag) pairs (tags < 0xFFFF, unique per key; slots past
// n are padding): packed into one 64-bit value when the keys span less than
// 2^48, the general 80-bit comparison otherwise.  Returns with the pairs in
// element order and pads (key ~0, tag 0xFFFF) at the end.
template <int EPL>
__device__ __forceinline__ void wave_sort_pairs(uint64_t (&k)[EPL], uint32_t (&t)[EPL], uint32_t n, uint32_t lane) {
    uint64_t lo = ~0ull, hi = 0;
#pragma unroll
    for (int q = 0; q < EPL; ++q) {
        const bool v = lane * EPL + q < n;
        lo = v && k[q] < lo ? k[q] : lo;
        hi = v && k[q] > hi ? k[q] : hi;
    }
    const uint64_t kmin = wave_min64(lo), kmax = wave_max64(hi);
    if (n == 0 || kmax - kmin < (1ull << 48)) {
        uint64_t v[EPL];
#pragma unroll
        for (int q = 0; q < EPL; ++q)
            v[q] = lane * EPL + q < n ? ((k[q] - kmin) << 16) | (uint64_t)(t[q] & 0xFFFFu) : ~0ull;
        wave_bitonic_packed<EPL>(v, lane);
#pragma unroll
        for (int q = 0; q < EPL; ++q) {
            const bool pad = v[q] == ~0ull;
            k[q] = pad ? ~0ull : (v[q] >> 16) + kmin;
            t[q] = pad ? 0xFFFFu : (uint32_t)(v[q] & 0xFFFFu);
        }
    } else {
        wave_bitonic<EPL>(k, t, lane);
    }
}

// Heads of the sorted pairs: the first pair of each distinct key (pads, tag ==
// pad, are never heads).  head[q] per element; pre = number of heads before
// this lane's elements (bit-sliced ballots of the per-lane counts, <= 4).
// Returns the number of heads.
template <int EPL>
__device__ __forceinline__ uint32_t segment_heads(const uint64_t (&k)[EPL], const uint32_t (&t)[EPL], uint32_t pad,
                                                  uint32_t lane, uint64_t lt, bool (&head)[EPL], uint32_t& pre) {
    static_assert(EPL <= 4, "segment_heads: at most 4 elements per lane");
    const uint64_t prev = (uint64_t)__shfl_up((unsigned long long)k[EPL - 1], 1);
    uint32_t hc = 0;
#pragma unroll
    for (int q = 0; q < EPL; ++q) {
        const uint32_t i = lane * EPL + q;
        const uint64_t pk = q == 0 ? prev : k[q - 1];
        head[q] = t[q] != pad && (i == 0 || k[q] != pk);
        hc += head[q] ? 1u : 0u;
    }
    uint32_t U = 0;
    pre = 0;
#pragma unroll
    for (int b = 0; b < 3; ++b) {
        const uint64_t mb = ballot((hc >> b) & 1u);
        pre += popc(mb & lt) << b;
        U += popc(mb) << b;
    }
    return U;
}

}  // namespace crdt
