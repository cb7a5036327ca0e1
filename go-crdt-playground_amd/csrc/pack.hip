// Host-path helpers around the merge kernels (the *_batch calls of api.cpp):
//  * check_order_kernel: every document's (or source's) live keys strictly
//    ascending -- the merge kernels' input contract (include/crdtgpu.h) --
//    checked on the device after the upload instead of by one host thread
//    before it; a violation sets kErrUnsorted (CRDT_E_UNSORTED).
//  * pack_scan_kernel: the packed offsets of a merge output -- the exclusive
//    prefix over documents of the live counts, each clamped to the document's
//    output capacity -- on the device, so the host path needs no count
//    read-back before it can gather.
//  * pack_out_kernel: a merge output (document d at its capacity offset)
//    gathered into consecutive live entries at those offsets, so the download
//    moves only live entries (crdt_ctx_set_option "pack_batch_outputs"); with
//    the counts and clocks too when the destination is the caller's page-locked
//    host output (written over PCIe by the kernel, no copy call at all).
// One wavefront per range, grid-stride; coalesced 64-lane runs.
#include "crdt_device.hpp"
#include "merge_block.hpp"

namespace crdt {

constexpr int kPackScanNT = 1024;

// One workgroup, in chunks of kPackScanNT x kPackScanV documents: the chunk's
// live counts are loaded coalesced into LDS, each thread sums kPackScanV
// consecutive ones, a block scan places the thread runs, the prefixes go back
// to LDS and out coalesced (poff[n] = total).  Threads reading and writing
// their own runs straight from memory -- 4-byte accesses 256 bytes apart,
// through one CU -- took 0.43-0.47 ms for an exchange's 2 x 65,536 documents.
// host_off (may be NULL): the same offsets, into the caller's page-locked
// output.
// gate: the call's status word -- after a failed order check the merge never
// ran, so the output's slot bounds and counts were never written: every
// offset is 0 and pack_out_kernel writes nothing.
// Up to two outputs (an exchange's), one after the other; host_status (may
// be NULL): the call's status word, copied for the host to read after its sync
// (the merges that set it have all run; nothing after this kernel sets it).
constexpr int kPackScanV = 8;
struct PackScanOut {
    const uint32_t* off;
    const uint32_t* cnt;
    uint32_t* poff;
    uint32_t* host_off;
};
__global__ __launch_bounds__(kPackScanNT) void pack_scan_kernel(PackScanOut o0, PackScanOut o1, uint32_t nout,
                                                                uint32_t n, const uint32_t* gate,
                                                                uint32_t* host_status) {
    constexpr uint32_t C = kPackScanNT * kPackScanV;
    __shared__ uint32_t wave_tot[kPackScanNT / 64];
    __shared__ uint32_t run[C];
    const uint32_t t = threadIdx.x;
    const bool open = (*gate & kErrUnsorted) == 0u;
    if (host_status && t == 0) *host_status = *gate;
    for (uint32_t k = 0; k < nout; ++k) {
        const PackScanOut& po = k ? o1 : o0;
        uint32_t carry = 0;
        for (uint32_t base = 0; base < n; base += C) {
            const uint32_t m = min(C, n - base);
            for (uint32_t i = t; i < C; i += kPackScanNT) {
                const uint32_t d = base + i;
                // clamped to the capacity (a larger count only follows a failed merge)
                run[i] = (open && i < m) ? min(po.cnt[d], po.off[d + 1] - po.off[d]) : 0u;
            }
            __syncthreads();
            uint32_t v[kPackScanV], sum = 0;
#pragma unroll
            for (int j = 0; j < kPackScanV; ++j) {
                v[j] = run[t * kPackScanV + j];
                sum += v[j];
            }
            uint32_t tot = 0;
            uint32_t p = carry + block_exclusive_scan<kPackScanNT>(sum, wave_tot, &tot);
            // (the scan's barriers order every read of run above before these writes)
#pragma unroll
            for (int j = 0; j < kPackScanV; ++j) {
                run[t * kPackScanV + j] = p;
                p += v[j];
            }
            __syncthreads();
            for (uint32_t i = t; i < m; i += kPackScanNT) {
                po.poff[base + i] = run[i];
                if (po.host_off) po.host_off[base + i] = run[i];
            }
            carry += tot;
            __syncthreads();  // (run and wave_tot are reused by the next chunk)
        }
        if (t == 0) {
            po.poff[n] = carry;
            if (po.host_off) po.host_off[n] = carry;
        }
    }
}

// Up to three lists of ranges in one launch (a batch call's dst and src, or a
// fold's documents, source entries and tombstones): each launch is a runtime
// call the host waits on.
struct OrderRanges {
    const uint32_t* off;
    const uint32_t* cnt;  // NULL: off[r + 1] ends range r
    uint32_t n;
    const uint64_t* keys;
};
struct OrderSets {
    OrderRanges set[3];
    uint32_t n_sets;
};

__global__ __launch_bounds__(256) void check_order_kernel(OrderSets sets, uint32_t total, uint32_t* status) {
    const uint32_t lane = threadIdx.x & 63;
    uint32_t err = 0;
    for (uint32_t g = uniform(blockIdx.x * 4 + (threadIdx.x >> 6)); g < total; g += gridDim.x * 4) {
        uint32_t r = g, k = 0;
        while (k + 1 < sets.n_sets && r >= sets.set[k].n) r -= sets.set[k++].n;
        const OrderRanges& q = sets.set[k];
        const uint32_t o = q.off[r];
        const uint32_t m = q.cnt ? q.cnt[r] : q.off[r + 1] - o;  // counts <= slots: checked on the host
        for (uint32_t i = 1 + lane; i < m; i += 64)
            if (q.keys[o + i] <= q.keys[o + i - 1]) err |= kErrUnsorted;
    }
    flag_error(status, err);
}

// out.keys == NULL: no key column (an exchange's second output sharing the
// first's); out.counts / out.vv != NULL: each document's count and clock too.
// Up to two outputs in one launch: documents [0, n) of output 0, then of output 1.
struct PackOut {
    OutView in;
    const uint32_t* poff;
    OutView out;
};
__global__ __launch_bounds__(256) void pack_out_kernel(PackOut p0, PackOut p1, uint32_t nout, uint32_t n, uint32_t R,
                                                       const uint32_t* gate) {
    const uint32_t lane = threadIdx.x & 63;
    if (*gate & kErrUnsorted) return;  // the merge never ran (pack_scan_kernel)
    for (uint32_t g = uniform(blockIdx.x * 4 + (threadIdx.x >> 6)); g < nout * n; g += gridDim.x * 4) {
        const PackOut& po = g < n ? p0 : p1;
        const OutView& in = po.in;
        const OutView& out = po.out;
        const uint32_t* poff = po.poff;
        const uint32_t d = g < n ? g : g - n;
        // a count above the document's own capacity (only after a failed merge)
        // is clamped to it: the gather never leaves the document's region
        const uint32_t o = in.offsets[d], p = poff[d], m = min(poff[d + 1] - p, in.offsets[d + 1] - o);
        for (uint32_t i = lane; i < m; i += 64) {
            if (out.keys) out.keys[p + i] = in.keys[o + i];
            out.actors[p + i] = in.actors[o + i];
            out.counters[p + i] = in.counters[o + i];
        }
        if (out.counts && lane == 0) out.counts[d] = in.counts[d];
        if (out.vv && lane < R) out.vv[(size_t)d * R + lane] = in.vv[(size_t)d * R + lane];
    }
}

// sets[k] = {off, cnt, n, keys}, k < n_sets <= 3
hipError_t launch_check_order(const void* sets_in, uint32_t n_sets, uint32_t* status, uint32_t n_cu,
                              hipStream_t stream) {
    OrderSets sets{};
    const OrderRanges* r = static_cast<const OrderRanges*>(sets_in);
    uint32_t total = 0;
    for (uint32_t k = 0; k < n_sets && k < 3; ++k) {
        sets.set[k] = r[k];
        total += r[k].n;
    }
    sets.n_sets = n_sets;
    if (total == 0) return hipSuccess;
    const uint32_t grid = min((total + 3) / 4, n_cu * 16u);
    hipLaunchKernelGGL(check_order_kernel, dim3(grid), dim3(256), 0, stream, sets, total, status);
    return hipGetLastError();
}

// nout <= 2 outputs: in[k] (the merge's), poff[k] (device), host_off[k] and
// out[k] (the gather's destinations)
hipError_t launch_pack(uint32_t nout, const OutView* in, uint32_t* const* poff, uint32_t* const* host_off,
                       const OutView* out, uint32_t n, uint32_t R, const uint32_t* gate, uint32_t* host_status,
                       uint32_t n_cu, hipStream_t stream) {
    PackScanOut s[2] = {};
    PackOut p[2] = {};
    for (uint32_t k = 0; k < nout && k < 2; ++k) {
        s[k] = PackScanOut{in[k].offsets, in[k].counts, poff[k], host_off[k]};
        p[k] = PackOut{in[k], poff[k], out[k]};
    }
    hipLaunchKernelGGL(pack_scan_kernel, dim3(1), dim3(kPackScanNT), 0, stream, s[0], s[1], nout, n, gate,
                       host_status);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || n == 0) return e;
    const uint32_t grid = min((nout * n + 3) / 4, n_cu * 16u);
    hipLaunchKernelGGL(pack_out_kernel, dim3(grid), dim3(256), 0, stream, p[0], p[1], nout, n, R, gate);
    return hipGetLastError();
}

}  // namespace crdt
