// Ingest sort: each document's live entries ordered by key on the device, so a
// producer that packs a map (Go iterates map[string]Dot in random order,
// awset.go:55-59) need not sort on the host before the merge kernels, which
// require strictly ascending keys per document (include/crdtgpu.h).
//
// Hand-written for gfx950, two launches:
//  * sort_wave_kernel: one wavefront per document.  A document of <= 256 live
//    entries is sorted in registers (wave_sort_pairs, wave_sort.hpp: bitonic
//    network over DPP / permlane exchanges, no LDS), with the compare width
//    cut to the document's key span -- 32-bit packed (key offset, index) pairs
//    when the keys span < 2^15 ids (interned ids of one map are small and
//    dense), 64-bit when < 2^47 -- and the dots gathered by the sorted index.
//    It also copies the VV and slot bounds, and queues larger documents.
//  * sort_block_kernel: one workgroup per queued document.  Its wavefronts sort
//    256-entry runs in registers as above, then merge-path passes double the
//    run length (each thread: one co-rank search, then 8 outputs merged
//    sequentially), ping-ponging (key, index) between two buffers chosen so
//    the last pass lands in out.keys; the dots are gathered at the end.
// A key twice in one document: CRDT_E_DUP_KEY (adjacent after the sort).
#include "crdt_device.hpp"
#include "wave_sort.hpp"

namespace crdt {

constexpr uint32_t kSortWaveMax = 256;  // live entries sorted by one wavefront in registers
constexpr int kSortNT = 256;            // sort_block_kernel threads
constexpr uint32_t kSortItems = 8;      // outputs per thread per merge-path pass

struct SortWork {
    uint32_t* count;  // documents queued for the block path
    uint32_t* head;   // next queued document to take
    uint32_t* list;   // [n_docs] queued documents
};

// Live entries of doc d, clamped to its slots (a larger count is reported).
__device__ __forceinline__ uint32_t sort_live(const BatchView& in, uint32_t d, uint32_t& err) {
    const uint32_t slots = in.offsets[d + 1] - in.offsets[d];
    const uint32_t n = live_count(in.offsets, in.counts, d);
    if (n > slots) err |= kErrCapacity;
    return n > slots ? slots : n;
}

// Sort the n <= EPL*64 entries at `keys` (element i = lane*EPL + q); returns
// them with the index each came from.  Pads (i >= n) come last.
template <int EPL>
__device__ __forceinline__ void sort_run(const uint64_t* keys, uint32_t n, uint32_t lane, uint64_t (&k)[EPL],
                                         uint32_t (&t)[EPL]) {
#pragma unroll
    for (int q = 0; q < EPL; ++q) {
        const uint32_t i = lane * EPL + q;
        k[q] = i < n ? keys[i] : ~0ull;
        t[q] = i;
    }
    wave_sort_pairs<EPL>(k, t, n, lane);
}

// The key of the element before each lane's first one (lane 0: none).
template <int EPL>
__device__ __forceinline__ uint64_t prev_lane_last(const uint64_t (&k)[EPL]) {
    const uint64_t v = k[EPL - 1];
    return (uint64_t)dpp<0x138>(0u, (uint32_t)v) | ((uint64_t)dpp<0x138>(0u, (uint32_t)(v >> 32)) << 32);  // wave_shr:1
}

template <int EPL>
__device__ __forceinline__ uint32_t sort_doc_wave(const BatchView& in, const OutView& out, uint32_t o, uint32_t n,
                                                  uint32_t lane) {
    uint64_t k[EPL];
    uint32_t t[EPL];
    sort_run<EPL>(in.keys + o, n, lane, k, t);
    const uint64_t pl = prev_lane_last<EPL>(k);
    uint32_t err = 0;
#pragma unroll
    for (int q = 0; q < EPL; ++q) {
        const uint32_t i = lane * EPL + q;
        if (i < n) {
            const uint32_t src = o + t[q];
            out.keys[o + i] = k[q];
            out.actors[o + i] = in.actors[src];
            out.counters[o + i] = in.counters[src];
            const uint64_t pk = q ? k[q ? q - 1 : 0] : pl;
            if (i > 0 && pk == k[q]) err |= kErrDupKey;
        }
    }
    return err;
}

__global__ __launch_bounds__(256) void sort_wave_kernel(BatchView in, OutView out, SortWork sw, uint32_t* status) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t R = in.R;
    uint32_t err = 0;
    for (uint32_t d = uniform(blockIdx.x * 4 + (threadIdx.x >> 6)); d < in.n_docs; d += gridDim.x * 4) {
        const uint32_t o = uniform(in.offsets[d]);
        const uint32_t n = uniform(sort_live(in, d, err));
        if (n <= 64)
            err |= sort_doc_wave<1>(in, out, o, n, lane);
        else if (n <= 128)
            err |= sort_doc_wave<2>(in, out, o, n, lane);
        else if (n <= kSortWaveMax)
            err |= sort_doc_wave<4>(in, out, o, n, lane);
        else if (lane == 0)
            sw.list[atomicAdd(sw.count, 1u)] = d;  // each document once: < n_docs
        if (lane < R) out.vv[(size_t)d * R + lane] = in.vv[(size_t)d * R + lane];
        if (lane == 0) {
            out.counts[d] = n;
            out.offsets[d] = o;
            if (d == in.n_docs - 1) out.offsets[in.n_docs] = in.offsets[in.n_docs];
        }
    }
    flag_error(status, err);
}

// Merge-path co-rank: how many of the first `diag` outputs of merging a[0, la)
// and b[0, lb) come from a (a first on equal keys, so the merge is stable).
__device__ __forceinline__ uint32_t co_rank(const uint64_t* a, uint32_t la, const uint64_t* b, uint32_t lb,
                                            uint32_t diag) {
    uint32_t lo = diag > lb ? diag - lb : 0u, hi = diag < la ? diag : la;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a[mid] <= b[diag - 1u - mid])
            lo = mid + 1u;
        else
            hi = mid;
    }
    return lo;
}

__global__ __launch_bounds__(kSortNT) void sort_block_kernel(BatchView in, OutView out, uint64_t* tk, uint32_t* ti0,
                                                             uint32_t* ti1, SortWork sw, uint32_t* status) {
    __shared__ uint32_t sh_slot;
    const uint32_t total = __hip_atomic_load(sw.count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (total == 0) return;  // nothing queued: no dispensing atomics
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    uint32_t err = 0;
    for (;;) {
        if (tid == 0) sh_slot = atomicAdd(sw.head, 1u);
        __syncthreads();
        const uint32_t slot = sh_slot;
        __syncthreads();  // every thread has read sh_slot before the next doc overwrites it
        if (slot >= total) break;
        const uint32_t d = sw.list[slot];
        const uint32_t o = in.offsets[d];
        uint32_t e0 = 0;
        const uint32_t n = sort_live(in, d, e0);  // > kSortWaveMax (reported by the wave kernel)
        const uint32_t runs = (n + kSortWaveMax - 1) / kSortWaveMax;
        const uint32_t passes = 32u - (uint32_t)__clz(runs - 1u);
        // (key, index) ping-pong: an odd number of passes starts in the scratch
        // keys, so the last pass always writes out.keys
        uint64_t* ka = (passes & 1u) ? tk + o : out.keys + o;
        uint64_t* kb = (passes & 1u) ? out.keys + o : tk + o;
        uint32_t* ia = (passes & 1u) ? ti1 + o : ti0 + o;
        uint32_t* ib = (passes & 1u) ? ti0 + o : ti1 + o;
        for (uint32_t c = w; c < runs; c += kSortNT / 64) {  // 256-entry runs, one per wavefront
            const uint32_t base = c * kSortWaveMax, m = min(kSortWaveMax, n - base);
            uint64_t k[4];
            uint32_t t[4];
            sort_run<4>(in.keys + o + base, m, lane, k, t);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t i = lane * 4 + q;
                if (i < m) {
                    ka[base + i] = k[q];
                    ia[base + i] = base + t[q];
                }
            }
        }
        __syncthreads();
        for (uint32_t width = kSortWaveMax; width < n; width *= 2) {
            const uint32_t units = (n + kSortItems - 1) / kSortItems;
            for (uint32_t u = tid; u < units; u += kSortNT) {
                const uint32_t s = u * kSortItems;
                const uint32_t pb = s / (2 * width) * (2 * width);  // the pair of runs holding output s
                const uint32_t la = min(width, n - pb);
                const uint32_t lb = n - pb > width ? min(width, n - pb - width) : 0u;
                const uint64_t* A = ka + pb;
                const uint64_t* B = A + la;
                const uint32_t diag = s - pb, end = min(diag + kSortItems, la + lb);
                uint32_t i = co_rank(A, la, B, lb, diag), j = diag - i;
                uint64_t va = i < la ? A[i] : ~0ull, vb = j < lb ? B[j] : ~0ull;
                for (uint32_t r = diag; r < end; ++r) {
                    const bool takea = j >= lb || (i < la && va <= vb);
                    if (takea) {
                        kb[pb + r] = va;
                        ib[pb + r] = ia[pb + i];
                        ++i;
                        va = i < la ? A[i] : ~0ull;
                    } else {
                        kb[pb + r] = vb;
                        ib[pb + r] = ia[pb + la + j];
                        ++j;
                        vb = j < lb ? B[j] : ~0ull;
                    }
                }
            }
            __syncthreads();
            uint64_t* tk2 = ka;
            ka = kb;
            kb = tk2;
            uint32_t* ti2 = ia;
            ia = ib;
            ib = ti2;
        }
        // ka == out.keys + o: gather the dots, flag repeated keys
        for (uint32_t e = tid; e < n; e += kSortNT) {
            const uint32_t src = o + ia[e];
            out.actors[o + e] = in.actors[src];
            out.counters[o + e] = in.counters[src];
            if (e > 0 && ka[e] == ka[e - 1]) err |= kErrDupKey;
        }
    }
    flag_error(status, err);
}

// Scratch the sort needs for n_slots entries: a key and an index plane for
// the ping-pong (the other index plane is the caller's idx array), and the
// queue counters.  The queue list itself is the caller's `ends` array.
hipError_t sort_storage(uint32_t n_docs, uint32_t n_slots, size_t* bytes) {
    (void)n_docs;
    *bytes = (size_t)n_slots * 12u + 64u;
    return hipSuccess;
}

hipError_t launch_sort(const BatchView& in, uint32_t n_slots, const OutView& out, void* temp, size_t temp_bytes,
                       uint32_t* ends, uint32_t* idx, uint32_t* status, uint32_t n_cu, hipStream_t stream) {
    if (in.n_docs == 0) return hipSuccess;
    if (temp_bytes < (size_t)n_slots * 12u + 64u) return hipErrorInvalidValue;
    uint64_t* tk = static_cast<uint64_t*>(temp);
    uint32_t* ti1 = reinterpret_cast<uint32_t*>(tk + n_slots);
    uint32_t* ctr = ti1 + n_slots;
    hipError_t e = hipMemsetAsync(ctr, 0, 2 * sizeof(uint32_t), stream);
    if (e != hipSuccess) return e;
    const SortWork sw{ctr, ctr + 1, ends};
    const uint32_t g1 = min((in.n_docs + 3) / 4, n_cu * 16u);
    hipLaunchKernelGGL(sort_wave_kernel, dim3(g1), dim3(256), 0, stream, in, out, sw, status);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(sort_block_kernel, dim3(min(in.n_docs, n_cu * 4u)), dim3(kSortNT), 0, stream, in, out, tk, idx,
                       ti1, sw, status);
    return hipGetLastError();
}

}  // namespace crdt
