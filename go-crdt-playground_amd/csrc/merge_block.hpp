// Block-level merge of one large document: dst <- src (+ tombstones).
//
// One workgroup of NT threads walks the two sorted entry lists with a
// merge-path window of T = NT*IPT merged positions per iteration.  Each thread
// finds its own diagonal split inside the LDS windows, decides IPT union keys
// with the per-key rule (DESIGN.md "Per-key rule"), and the workgroup scans the
// kept counts to place the survivors contiguously in key order.
//
// The rule (union key k, dst dot d if present, src dot s if present):
//   changed  = has_s && (full || !dstVV.HasDot(s))   awset-delta_test.go:84-92
//   has_d && has_s : present, dot = changed ? s : d   awset.go:123-129,142
//   has_d only     : present = full ? !srcVV.HasDot(d) : true      awset.go:146-158
//   has_s only     : present = changed && !dstVV.HasDot(s)         awset.go:133-140
//   delta mode, present, k in src.Deleted as x and x "effective"
//   (not re-added, awset-delta_test.go:93-102): present = dstVV.HasDot(x)
//                                                     awset-delta_test.go:149-164
#pragma once

#include "crdt_device.hpp"

namespace crdt {

template <int NT, int IPT>
struct MergeSmem {
    static constexpr int T = NT * IPT;
    uint64_t dk[T];
    uint64_t dc[T];
    uint64_t sk[T];
    uint64_t sc[T];
    uint32_t da[T];
    uint32_t sa[T];
    uint64_t dvv[CRDT_MAX_R];
    uint64_t svv[CRDT_MAX_R];
    uint32_t wave_tot[NT / 64];
    uint32_t word[4];
};

struct Entries {
    const uint64_t* k;
    const uint32_t* a;
    const uint64_t* c;
    uint32_t n;
};

struct EntriesOut {
    uint64_t* k;
    uint32_t* a;
    uint64_t* c;
};

// # of dst elements among the first k merged (dst first on equal keys).
__device__ __forceinline__ uint32_t merge_path(const uint64_t* dk, uint32_t nd, const uint64_t* sk, uint32_t ns,
                                               uint32_t k) {
    uint32_t lo = k > ns ? k - ns : 0;
    uint32_t hi = k < nd ? k : nd;
    while (lo < hi) {
        uint32_t mid = (lo + hi) >> 1;
        if (dk[mid] <= sk[k - 1 - mid])
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo;
}

// Tombstone probe for delta mode: returns true and (xa, xc) when key is in t.
__device__ __forceinline__ bool tomb_find(const Entries& t, uint64_t key, uint32_t& xa, uint64_t& xc) {
    if (t.n == 0) return false;
    uint32_t h = lower_bound(t.k, t.n, key);
    if (h < t.n && t.k[h] == key) {
        xa = t.a[h];
        xc = t.c[h];
        return true;
    }
    return false;
}

// Per-key rule shared by every path.  Returns whether the key survives and its dot.
__device__ __forceinline__ bool decide(bool has_d, uint32_t d_a, uint64_t d_c, bool has_s, uint32_t s_a, uint64_t s_c,
                                       bool full, const uint64_t* dvv, const uint64_t* svv, uint32_t R,
                                       const Entries& tomb, uint64_t key, uint32_t& o_a, uint64_t& o_c,
                                       uint32_t& err) {
    const bool changed = has_s && (full || !has_dot(dvv, R, s_a, s_c, err));
    bool present;
    if (has_d) {
        present = has_s ? true : (full ? !has_dot(svv, R, d_a, d_c, err) : true);
        const bool take_s = has_s && changed;
        o_a = take_s ? s_a : d_a;
        o_c = take_s ? s_c : d_c;
    } else {
        present = changed && !has_dot(dvv, R, s_a, s_c, err);
        o_a = s_a;
        o_c = s_c;
    }
    if (!full && present) {
        uint32_t xa;
        uint64_t xc;
        if (tomb_find(tomb, key, xa, xc)) {
            const bool readded = has_s && (s_a != xa || s_c > xc);
            if (!readded) present = has_dot(dvv, R, xa, xc, err);
        }
    }
    return present;
}

// Block-wide exclusive scan of v (per thread); returns exclusive prefix, total in *tot.
template <int NT>
__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t* wave_tot, uint32_t* tot) {
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t y = __shfl_up(x, o);
        if (lane >= (uint32_t)o) x += y;
    }
    if (lane == 63) wave_tot[w] = x;
    __syncthreads();
    uint32_t base = 0, all = 0;
#pragma unroll
    for (int i = 0; i < NT / 64; ++i) {
        uint32_t t = wave_tot[i];
        base += (i < (int)w) ? t : 0u;
        all += t;
    }
    __syncthreads();
    *tot = all;
    return base + x - v;
}

// Merge one document.  sm.dvv / sm.svv must hold the two version vectors.
// Returns the number of entries written to out.
template <int NT, int IPT>
__device__ uint32_t block_merge(const Entries& D, const Entries& S, const Entries& tomb, bool full, uint32_t R,
                                MergeSmem<NT, IPT>& sm, const EntriesOut& out, uint32_t& err) {
    constexpr uint32_t T = NT * IPT;
    const uint32_t tid = threadIdx.x;
    uint32_t i = 0, j = 0, o = 0;
    while (i < D.n || j < S.n) {
        const uint32_t nd = min(T, D.n - i), ns = min(T, S.n - j);
        const uint32_t K = min(T, nd + ns);
        for (uint32_t t = tid; t < nd; t += NT) {
            sm.dk[t] = D.k[i + t];
            sm.da[t] = D.a[i + t];
            sm.dc[t] = D.c[i + t];
        }
        for (uint32_t t = tid; t < ns; t += NT) {
            sm.sk[t] = S.k[j + t];
            sm.sa[t] = S.a[j + t];
            sm.sc[t] = S.c[j + t];
        }
        const bool has_prev = i > 0;
        const uint64_t prev_dk = has_prev ? D.k[i - 1] : 0ull;
        __syncthreads();

        const uint32_t k0 = min(tid * IPT, K), k1 = min(k0 + IPT, K);
        uint32_t a = merge_path(sm.dk, nd, sm.sk, ns, k0);
        uint32_t b = k0 - a;

        uint64_t ok[IPT];
        uint32_t oa[IPT];
        uint64_t oc[IPT];
        bool kp[IPT];
        uint32_t cnt = 0;
#pragma unroll
        for (int q = 0; q < IPT; ++q) {
            kp[q] = false;
            ok[q] = 0;
            oa[q] = 0;
            oc[q] = 0;
            if (k0 + q < k1) {
                const bool take_d = (a < nd) && (b >= ns || sm.dk[a] <= sm.sk[b]);
                if (take_d) {
                    const uint64_t key = sm.dk[a];
                    const bool match = (b < ns) && sm.sk[b] == key;
                    uint32_t s_a = match ? sm.sa[b] : 0u;
                    uint64_t s_c = match ? sm.sc[b] : 0ull;
                    kp[q] = decide(true, sm.da[a], sm.dc[a], match, s_a, s_c, full, sm.dvv, sm.svv, R, tomb, key,
                                   oa[q], oc[q], err);
                    ok[q] = key;
                    ++a;
                } else {
                    const uint64_t key = sm.sk[b];
                    const bool match = (a > 0) ? (sm.dk[a - 1] == key) : (has_prev && prev_dk == key);
                    if (!match) {
                        kp[q] = decide(false, 0u, 0ull, true, sm.sa[b], sm.sc[b], full, sm.dvv, sm.svv, R, tomb, key,
                                       oa[q], oc[q], err);
                        ok[q] = key;
                    }
                    ++b;
                }
                cnt += kp[q] ? 1u : 0u;
            }
        }
        uint32_t total;
        uint32_t pos = o + block_exclusive_scan<NT>(cnt, sm.wave_tot, &total);
#pragma unroll
        for (int q = 0; q < IPT; ++q) {
            if (kp[q]) {
                out.k[pos] = ok[q];
                out.a[pos] = oa[q];
                out.c[pos] = oc[q];
                ++pos;
            }
        }
        const uint32_t aK = merge_path(sm.dk, nd, sm.sk, ns, K);
        i += aK;
        j += K - aK;
        o += total;
        __syncthreads();
    }
    return o;
}

}  // namespace crdt
