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
    const uint64_t lt = low_mask(lane);
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
                const uint32_t idx = base + popc(pres1 & lt);
                O.keys[idx] = ((uint64_t)d << 8) | u1;
                if (re) {
                    O.actors[idx] = (uint32_t)X;
                    O.counters[idx] = c0 + popc(ops1 & lt) + 1;
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

hipError_t launch_gen_pair(uint64_t seed, uint32_t n_docs, const OutView& A, const OutView& B, hipStream_t stream) {
    if (n_docs == 0) return hipSuccess;
    uint32_t grid = (n_docs + 3) / 4;
    if (grid > (1u << 20)) grid = 1u << 20;
    hipLaunchKernelGGL((gen_pair_kernel<4>), dim3(grid), dim3(256), 0, stream, seed, n_docs, A, B);
    return hipGetLastError();
}

}  // namespace crdt
