// Synthetic, reachable replica states generated on the device (bench and
// GPU-test workloads; never part of a merge).  Each document's states are a
// pure function of (seed, doc), so any sample can be regenerated on the host
// (crdtgpu/workloads.py restates the same formulas and replays them through
// the reference semantics to prove reachability).
//
// "pair" workload (BASELINE config 2: 2 replicas, 64 entries each, R = 2):
//   key universe of doc d: u in [0, 96), key id = d << 8 | u
//   base: A adds u = 0..47 in order (dots (A, u+1)), B merges A.
//   then, concurrently, replica X in {A, B} with s = splitmix64(seed ^ (2d+X)):
//     p(u) = (mul*u + add) mod 48, mul = kUnits48[s & 15], add = (s >> 4) % 48
//     p < 8            : X deletes u                    (awset.go:96-101)
//     8 <= p < 16      : X re-adds u if ((s >> 12) & 3) == 0 (25% of replicas)
//     X adds its 24 new keys: A u = 48..71, B u = 72..95
//   X's re-adds and new adds are applied in key order (awset.go:89-94), so
//   A's counters continue from 48 and B's start at 1.
#include "crdt_device.hpp"

namespace crdt {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__constant__ uint32_t kUnits48[16] = {1, 5, 7, 11, 13, 17, 19, 23, 25, 29, 31, 35, 37, 41, 43, 47};

template <int WAVES>
__global__ __launch_bounds__(WAVES * 64) void gen_pair_kernel(uint64_t seed, uint32_t n_docs, OutView A, OutView B) {
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t d0 = blockIdx.x * WAVES + (threadIdx.x >> 6); d0 < n_docs; d0 += gridDim.x * WAVES) {
        const uint32_t d = uniform(d0);
        const uint32_t base = d * 64u;
#pragma unroll
        for (int X = 0; X < 2; ++X) {
            OutView& O = X == 0 ? A : B;
            const uint64_t s = splitmix64(seed ^ (2ull * d + (uint64_t)X));
            const uint32_t mul = kUnits48[s & 15], add = (uint32_t)((s >> 4) % 48);
            const bool readd = ((s >> 12) & 3) == 0;
            // pass 1: base keys u = lane (< 48)
            const uint32_t u1 = lane;
            const uint32_t p = (mul * u1 + add) % 48u;
            const bool in_base = u1 < 48;
            const bool del = in_base && p < 8;
            const bool re = in_base && readd && p >= 8 && p < 16;
            const uint64_t ops1 = ballot(re);
            const uint64_t pres1 = ballot(in_base && !del);
            const uint32_t n_ops1 = popc(ops1), n_pres1 = popc(pres1);  // n_pres1 == 40
            const uint64_t c0 = X == 0 ? 48ull : 0ull;                    // X's counter before its ops
            if (in_base && !del) {
                const uint32_t idx = base + below(pres1);
                O.keys[idx] = ((uint64_t)d << 8) | u1;
                if (re) {
                    O.actors[idx] = (uint32_t)X;
                    O.counters[idx] = c0 + below(ops1) + 1;
                } else {
                    O.actors[idx] = 0;
                    O.counters[idx] = u1 + 1;
                }
            }
            // pass 2: X's 24 new keys
            const uint32_t lo = X == 0 ? 0u : 24u;
            if (lane >= lo && lane < lo + 24) {
                const uint32_t r = lane - lo;
                const uint32_t idx = base + n_pres1 + r;
                O.keys[idx] = ((uint64_t)d << 8) | (48u + lane);
                O.actors[idx] = (uint32_t)X;
                O.counters[idx] = c0 + n_ops1 + r + 1;
            }
            if (lane == 0) {
                O.offsets[d] = base;
                O.counts[d] = n_pres1 + 24;
                if (d == n_docs - 1) O.offsets[n_docs] = base + 64;
                O.vv[(size_t)d * 2 + 0] = X == 0 ? 48ull + n_ops1 + 24 : 48ull;
                O.vv[(size_t)d * 2 + 1] = X == 0 ? 0ull : (uint64_t)n_ops1 + 24;
            }
        }
    }
}

// ---------------------------------------------------------------------------
// "delta" workload (BASELINE config 3): n_docs dst docs x 64 entries, R actors,
// M ordered AWSetDelta sources per doc, each 8 entries + 2 tombstones.  Valid
// random states with a controlled path mix (not simulated histories):
//   H(d, tag, i) = splitmix64(seed ^ d << 20 ^ tag << 12 ^ i)
//   universe u in [0, 256), key = d << 8 | u; a subset of size k is
//   {u : (mul*u + add) & 255 < k}, mul odd, from one H draw
//   dst: 64 keys, dot (H%R, 1 + (H>>8)%64), VV[r] = 64 + H%32
//   1% of docs ("first contact"): dst VV[a*] = 0, no dst dot of actor a*,
//   source 0 has actor a* -> full-merge path (awset-delta_test.go:53-56)
//   source j: actor a_j = H%R, VV[r] = VV0[r] + 1 + H%16,
//     8 entries: actor a_j (75%) or H%R; counter covered by VV0 (50%, pruned
//     by MakeDeltaMergeData) or in (VV0, srcVV] (new)
//     2 tombstones: actor a_j, counter srcVV[a_j] - H%8 (>= 1)
// workloads.delta_docs restates these formulas on the host.
__device__ __forceinline__ uint64_t Hx(uint64_t seed, uint64_t d, uint32_t tag, uint32_t i) {
    return splitmix64(seed ^ (d << 20) ^ ((uint64_t)tag << 12) ^ (uint64_t)i);
}

struct SrcOutView {
    uint32_t* doc_srcs;
    uint32_t* src_actor;
    uint64_t* vv;
    uint32_t* entry_off;
    uint64_t* keys;
    uint32_t* actors;
    uint64_t* counters;
    uint32_t* tomb_off;
    uint64_t* tkeys;
    uint32_t* tactors;
    uint64_t* tcounters;
};

// Writes the k-subset of the 256-key universe selected by draw h, sorted, at
// base; f(u, slot) gives each selected key's fields.
template <typename F>
__device__ __forceinline__ void subset256(uint64_t h, uint32_t k, uint32_t lane, F f) {
    const uint32_t mul = (uint32_t)(h & 0xFF) | 1u, add = (uint32_t)((h >> 8) & 0xFF);
    uint32_t base = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t u = q * 64 + lane;
        const bool sel = ((mul * u + add) & 255u) < k;
        const uint64_t m = ballot(sel);
        if (sel) f(u, base + popc(m & low_mask(lane)));
        base += popc(m);
    }
}

template <int WAVES>
__global__ __launch_bounds__(WAVES * 64) void gen_delta_kernel(uint64_t seed, uint32_t n_docs, uint32_t R, uint32_t M,
                                                              OutView D, SrcOutView S) {
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t d0 = blockIdx.x * WAVES + (threadIdx.x >> 6); d0 < n_docs; d0 += gridDim.x * WAVES) {
        const uint32_t d = uniform(d0);
        const bool first = Hx(seed, d, 1, 0) % 100 == 0;
        const uint32_t astar = (uint32_t)(Hx(seed, d, 1, 1) % R);
        // dst VV0 (lane r)
        uint64_t vv0 = 0;
        if (lane < R) vv0 = (first && lane == astar) ? 0ull : 64 + Hx(seed, d, 3, lane) % 32;
        subset256(Hx(seed, d, 0, 0), 64, lane, [&](uint32_t u, uint32_t slot) {
            const uint64_t hu = Hx(seed, d, 2, u);
            uint32_t a = (uint32_t)(hu % R);
            if (first && a == astar) a = (a + 1) % R;
            D.keys[(size_t)d * 64 + slot] = ((uint64_t)d << 8) | u;
            D.actors[(size_t)d * 64 + slot] = a;
            D.counters[(size_t)d * 64 + slot] = 1 + (hu >> 8) % 64;
        });
        if (lane < R) D.vv[(size_t)d * R + lane] = vv0;
        if (lane == 0) {
            D.offsets[d] = d * 64;
            D.counts[d] = 64;
            S.doc_srcs[d] = d * M;
            if (d == n_docs - 1) {
                D.offsets[n_docs] = n_docs * 64;
                S.doc_srcs[n_docs] = n_docs * M;
                S.entry_off[(size_t)n_docs * M] = n_docs * M * 8;
                S.tomb_off[(size_t)n_docs * M] = n_docs * M * 2;
            }
        }
        for (uint32_t j = 0; j < M; ++j) {
            const uint32_t sidx = d * M + j;
            const uint32_t aj = (first && j == 0) ? astar : (uint32_t)(Hx(seed, d, 4, j) % R);
            uint64_t svv = 0;
            if (lane < R) svv = vv0 + 1 + Hx(seed, d, 5, j * R + lane) % 16;
            if (lane < R) S.vv[(size_t)sidx * R + lane] = svv;
            const uint64_t svv_aj = __shfl(svv, (int)aj);
            if (lane == 0) {
                S.src_actor[sidx] = aj;
                S.entry_off[sidx] = sidx * 8;
                S.tomb_off[sidx] = sidx * 2;
            }
            subset256(Hx(seed, d, 6, j), 8, lane, [&](uint32_t u, uint32_t slot) {
                const uint64_t he = Hx(seed, d, 7, j * 256 + u);
                const uint32_t a = (he & 3) == 0 ? (uint32_t)((he >> 2) % R) : aj;
                // VV0[a], srcVV[a] live in lane a: fetch through LDS-free shuffles
                // is not possible inside a divergent lambda, so recompute them.
                const uint64_t v0 = (first && a == astar) ? 0ull : 64 + Hx(seed, d, 3, a) % 32;
                const uint64_t sv = v0 + 1 + Hx(seed, d, 5, j * R + a) % 16;
                const uint64_t c = ((he >> 8) & 1) == 0 ? 1 + (he >> 16) % (v0 > 0 ? v0 : 1)
                                                       : v0 + 1 + (he >> 16) % (sv - v0);
                S.keys[(size_t)sidx * 8 + slot] = ((uint64_t)d << 8) | u;
                S.actors[(size_t)sidx * 8 + slot] = a;
                S.counters[(size_t)sidx * 8 + slot] = c;
            });
            subset256(Hx(seed, d, 8, j), 2, lane, [&](uint32_t u, uint32_t slot) {
                const uint64_t ht = Hx(seed, d, 9, j * 256 + u);
                const uint64_t back = ht % 8;
                S.tkeys[(size_t)sidx * 2 + slot] = ((uint64_t)d << 8) | u;
                S.tactors[(size_t)sidx * 2 + slot] = aj;
                S.tcounters[(size_t)sidx * 2 + slot] = svv_aj > back ? svv_aj - back : 1;
            });
        }
    }
}

hipError_t launch_gen_delta(uint64_t seed, uint32_t n_docs, uint32_t R, uint32_t M, const OutView& D,
                            const SrcOutView& S, hipStream_t stream) {
    if (n_docs == 0) return hipSuccess;
    uint32_t grid = (n_docs + 3) / 4;
    if (grid > (1u << 20)) grid = 1u << 20;
    hipLaunchKernelGGL((gen_delta_kernel<4>), dim3(grid), dim3(256), 0, stream, seed, n_docs, R, M, D, S);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// "replicas" workload (BASELINE config 5): per document, P replica states of E
// entries each over R = P actors, to be folded r0 <- r1 <- ... <- r(P-1).
//   universe u in [0, 2E), key = d << 8 | u; replica r holds the E keys
//   {u : (mul*u + add) mod 2E < E} (mul odd, one H draw; 2E a power of two)
//   replica r's VV: own VV[r] = E + H%E, others VV[a] = H % (E + E/2)
//   each entry's dot: actor r (75%) or H%R when that actor's VV > 0, counter
//   1 + H % VV[actor] (covered by the replica's own clock)
// dst = replica 0 (batch D), sources = replicas 1..P-1 (batch S, no tombstones).
// workloads.replica_docs restates these formulas on the host.
template <int WAVES>
__global__ __launch_bounds__(WAVES * 64) void gen_replicas_kernel(uint64_t seed, uint32_t n_docs, uint32_t P,
                                                                 uint32_t E, OutView D, SrcOutView S) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t U = 2 * E;  // universe, power of two, <= 64
    const uint32_t R = P;
    for (uint32_t d0 = blockIdx.x * WAVES + (threadIdx.x >> 6); d0 < n_docs; d0 += gridDim.x * WAVES) {
        const uint32_t d = uniform(d0);
        if (lane == 0) {
            D.offsets[d] = d * E;
            D.counts[d] = E;
            S.doc_srcs[d] = d * (P - 1);
            if (d == n_docs - 1) {
                D.offsets[n_docs] = n_docs * E;
                S.doc_srcs[n_docs] = n_docs * (P - 1);
                S.entry_off[(size_t)n_docs * (P - 1)] = n_docs * (P - 1) * E;
                S.tomb_off[(size_t)n_docs * (P - 1)] = 0;
            }
        }
        for (uint32_t r = 0; r < P; ++r) {
            // VV of replica r: lane a holds VV[a]
            uint64_t vv = 0;
            if (lane < R) vv = lane == r ? E + Hx(seed, d, 20, r * 64 + lane) % E : Hx(seed, d, 20, r * 64 + lane) % (E + E / 2);
            const uint64_t h = Hx(seed, d, 21, r);
            const uint32_t mul = (uint32_t)(h & 0xFF) | 1u, add = (uint32_t)((h >> 8) & 0xFF);
            const uint32_t u = lane;
            const bool sel = u < U && ((mul * u + add) & (U - 1)) < E;
            const uint64_t m = ballot(sel);
            const uint32_t slot = popc(m & low_mask(lane));
            const uint64_t he = Hx(seed, d, 22, r * 64 + u);
            uint32_t a = (he & 3) == 0 ? (uint32_t)((he >> 2) % R) : r;
            // both shuffles run in every lane (a shuffle inside a divergent branch
            // reads inactive source lanes)
            const uint64_t va_a = __shfl(vv, (int)a), va_r = __shfl(vv, (int)r);
            uint64_t va = va_a;
            if (va_a == 0) {  // never seen that actor: fall back to own dot
                a = r;
                va = va_r;
            }
            const uint64_t c = 1 + (he >> 16) % va;
            const uint64_t key = ((uint64_t)d << 8) | u;
            if (r == 0) {
                if (sel) {
                    D.keys[(size_t)d * E + slot] = key;
                    D.actors[(size_t)d * E + slot] = a;
                    D.counters[(size_t)d * E + slot] = c;
                }
                if (lane < R) D.vv[(size_t)d * R + lane] = vv;
            } else {
                const size_t sidx = (size_t)d * (P - 1) + (r - 1);
                if (sel) {
                    S.keys[sidx * E + slot] = key;
                    S.actors[sidx * E + slot] = a;
                    S.counters[sidx * E + slot] = c;
                }
                if (lane < R) S.vv[sidx * R + lane] = vv;
                if (lane == 0) {
                    S.src_actor[sidx] = r;
                    S.entry_off[sidx] = (uint32_t)(sidx * E);
                    S.tomb_off[sidx] = 0;
                }
            }
        }
    }
}

hipError_t launch_gen_replicas(uint64_t seed, uint32_t n_docs, uint32_t P, uint32_t E, const OutView& D,
                               const SrcOutView& S, hipStream_t stream) {
    if (n_docs == 0) return hipSuccess;
    uint32_t grid = (n_docs + 3) / 4;
    if (grid > (1u << 20)) grid = 1u << 20;
    hipLaunchKernelGGL((gen_replicas_kernel<4>), dim3(grid), dim3(256), 0, stream, seed, n_docs, P, E, D, S);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// "zipf" workload (BASELINE config 4): skewed document sizes, 50% concurrent
// add/remove conflicts, R = 2.
//   size of doc d: octave k drawn with weight kZipfW[k] ~ 2^(-0.1k), k < 20
//   (the Zipf(1.1) mass per octave), then 2^k + (a*b >> k) with a, b uniform
//   in [0, 2^k) -- mean 3.4e4, max 2^20 - 1 (crdt_zipf_doc_size, host+device)
//   base keys u < size (key = d << 21 | u): A added them in order (dots
//   (A, u+1)), B merged A.  Then for each base key, G = splitmix64(seed ^
//   (d << 24 | u << 4 | tag)): bit 0 of G(.,1) = conflict; bit 1 picks the
//   side that deletes; the other side re-adds with a fresh dot (its re-adds in
//   key order: A's counters continue from size, B's start at 1).
__host__ __device__ inline uint64_t splitmix64_hd(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__host__ __device__ inline uint32_t zipf_doc_size(uint64_t seed, uint32_t d) {
    const uint32_t W[20] = {65536, 61147, 57052, 53232, 49667, 46341, 43238, 40342, 37641, 35120,
                            32768, 30574, 28526, 26616, 24834, 23170, 21619, 20171, 18820, 17560};
    const uint64_t h = splitmix64_hd(seed ^ (((uint64_t)d << 24) | 0xFull));
    uint32_t r = (uint32_t)(h % 733974u), k = 0;
    while (k < 19 && r >= W[k]) r -= W[k++];
    const uint64_t h2 = splitmix64_hd(h);
    const uint64_t span = 1ull << k;
    const uint64_t a = (h2 & 0xFFFFFull) % span, b = ((h2 >> 20) & 0xFFFFFull) % span;
    return (uint32_t)(span + ((a * b) >> k));
}

__device__ __forceinline__ uint64_t zipf_G(uint64_t seed, uint32_t d, uint32_t u, uint32_t tag) {
    return splitmix64(seed ^ (((uint64_t)d << 24) | ((uint64_t)u << 4) | tag));
}

// One wave per document, 64 base keys per iteration (ballot prefix carries).
__global__ __launch_bounds__(256) void gen_zipf_kernel(uint64_t seed, uint32_t n_docs, const uint32_t* offsets,
                                                        OutView A, OutView B) {
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t d0 = blockIdx.x * 4 + (threadIdx.x >> 6); d0 < n_docs; d0 += gridDim.x * 4) {
        const uint32_t d = uniform(d0);
        const uint32_t size = zipf_doc_size(seed, d);
        const uint32_t base = offsets[d];
        uint32_t pa = 0, pb = 0, ra = 0, rb = 0;  // present so far (A, B); re-adds so far (A, B)
        // pass 1: count re-adds of each side (VV and counters need the totals)
        uint32_t na = 0, nb = 0;
        for (uint32_t u0 = 0; u0 < size; u0 += 64) {
            const uint32_t u = u0 + lane;
            const uint64_t g = u < size ? zipf_G(seed, d, u, 1) : 0ull;
            const bool conflict = u < size && (g & 1);
            const bool a_del = conflict && !(g & 2);  // A deletes, B re-adds
            na += popc(ballot(conflict && !a_del));
            nb += popc(ballot(a_del));
        }
        for (uint32_t u0 = 0; u0 < size; u0 += 64) {
            const uint32_t u = u0 + lane;
            const bool in = u < size;
            const uint64_t g = in ? zipf_G(seed, d, u, 1) : 0ull;
            const bool conflict = in && (g & 1);
            const bool a_del = conflict && !(g & 2);
            const bool b_del = conflict && (g & 2);
            const uint64_t key = ((uint64_t)d << 21) | u;
            const uint64_t ma = ballot(in && !a_del), mb = ballot(in && !b_del);
            const uint64_t mra = ballot(b_del), mrb = ballot(a_del);  // A re-adds where B deletes
            if (in && !a_del) {
                const uint32_t i = base + pa + below(ma);
                A.keys[i] = key;
                A.actors[i] = 0;
                A.counters[i] = b_del ? (uint64_t)size + ra + below(mra) + 1 : (uint64_t)u + 1;
            }
            if (in && !b_del) {
                const uint32_t i = base + pb + below(mb);
                B.keys[i] = key;
                B.actors[i] = a_del ? 1u : 0u;
                B.counters[i] = a_del ? (uint64_t)rb + below(mrb) + 1 : (uint64_t)u + 1;
            }
            pa += popc(ma);
            pb += popc(mb);
            ra += popc(mra);
            rb += popc(mrb);
        }
        if (lane == 0) {
            A.offsets[d] = base;
            B.offsets[d] = base;
            A.counts[d] = pa;
            B.counts[d] = pb;
            if (d == n_docs - 1) {
                A.offsets[n_docs] = base + size;
                B.offsets[n_docs] = base + size;
            }
            A.vv[(size_t)d * 2] = (uint64_t)size + na;
            A.vv[(size_t)d * 2 + 1] = 0;
            B.vv[(size_t)d * 2] = size;
            B.vv[(size_t)d * 2 + 1] = nb;
        }
    }
}

hipError_t launch_gen_zipf(uint64_t seed, uint32_t n_docs, const uint32_t* offsets, const OutView& A,
                           const OutView& B, hipStream_t stream) {
    if (n_docs == 0) return hipSuccess;
    const uint32_t grid = (n_docs + 3) / 4;
    hipLaunchKernelGGL(gen_zipf_kernel, dim3(grid), dim3(256), 0, stream, seed, n_docs, offsets, A, B);
    return hipGetLastError();
}

uint32_t host_zipf_doc_size(uint64_t seed, uint32_t d) { return zipf_doc_size(seed, d); }

hipError_t launch_gen_pair(uint64_t seed, uint32_t n_docs, const OutView& A, const OutView& B, hipStream_t stream) {
    if (n_docs == 0) return hipSuccess;
    uint32_t grid = (n_docs + 3) / 4;
    if (grid > (1u << 20)) grid = 1u << 20;
    hipLaunchKernelGGL((gen_pair_kernel<4>), dim3(grid), dim3(256), 0, stream, seed, n_docs, A, B);
    return hipGetLastError();
}

}  // namespace crdt
