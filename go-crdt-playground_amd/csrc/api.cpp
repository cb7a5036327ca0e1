// C ABI of the engine (include/crdtgpu.h): context, validation, launches and
// the synchronous host-buffer path used by the cgo drop-in.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <initializer_list>
#include <map>
#include <mutex>
#include <new>
#include <vector>

#include "../../include/crdtgpu.h"
#include "crdt_device.hpp"

namespace crdt {
hipError_t launch_join(const BatchView& dst, const BatchView& src, const OutView& out, const OutView* out2,
                       const Work& wk, uint32_t docs_per_wave, bool nt_stores, bool stage_stores, uint32_t slab_blocks,
                       uint32_t block_grid, bool no_large,
                       const TileWork* tw, uint32_t n_cu, hipStream_t stream);
hipError_t launch_fold(int mode, const BatchView& dst, const SrcView& sb, const OutView& out, const Scratch& scr,
                       const Work& wk, uint32_t block_grid, bool lean_first, hipStream_t stream);
uint32_t tile_positions(uint32_t shape);
hipError_t sort_storage(uint32_t n_docs, uint32_t n_slots, size_t* bytes);
struct OrderRanges {  // pack.hip: one list of key ranges whose order is checked
    const uint32_t* off;
    const uint32_t* cnt;
    uint32_t n;
    const uint64_t* keys;
};
hipError_t launch_check_order(const void* sets, uint32_t n_sets, uint32_t* status, uint32_t n_cu, hipStream_t stream);
hipError_t launch_pack(uint32_t nout, const OutView* in, uint32_t* const* poff, uint32_t* const* host_off,
                       const OutView* out, uint32_t n, uint32_t R, const uint32_t* gate, uint32_t* host_status,
                       uint32_t n_cu, hipStream_t stream);
hipError_t launch_sort(const BatchView& in, uint32_t n_slots, const OutView& out, void* temp, size_t temp_bytes,
                       uint32_t* ends, uint32_t* idx, uint32_t* status, uint32_t n_cu, hipStream_t stream);
hipError_t launch_apply(const BatchView& st, const TombView& tb, const ApplyOps& ops, const OutView& out,
                        const TombOut& tout, bool has_tout, const Work& wk, uint32_t n_cu, hipStream_t stream);
hipError_t launch_vv_max(uint64_t* dst, const uint64_t* src, size_t n, hipStream_t stream);
hipError_t launch_vv_min(uint64_t* dst, const uint64_t* src, size_t n, hipStream_t stream);
hipError_t launch_tomb_gc(const TombView& tb, uint32_t n_docs, uint32_t R, const uint64_t* stable, const TombOut& out,
                          uint32_t n_cu, hipStream_t stream);
hipError_t launch_reset_work(uint32_t* ws, hipStream_t stream);
hipError_t launch_context(const uint64_t* vv, uint32_t n_docs, uint32_t R, uint64_t* part, uint32_t n_part,
                          uint64_t* out, hipStream_t stream);
hipError_t launch_gen_pair(uint64_t seed, uint32_t n_docs, const OutView& A, const OutView& B, hipStream_t stream);
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
hipError_t launch_gen_delta(uint64_t seed, uint32_t n_docs, uint32_t R, uint32_t M, const OutView& D,
                            const SrcOutView& S, hipStream_t stream);
hipError_t launch_gen_replicas(uint64_t seed, uint32_t n_docs, uint32_t P, uint32_t E, const OutView& D,
                               const SrcOutView& S, hipStream_t stream);
hipError_t launch_gen_zipf(uint64_t seed, uint32_t n_docs, const uint32_t* offsets, const OutView& A,
                           const OutView& B, hipStream_t stream);
uint32_t host_zipf_doc_size(uint64_t seed, uint32_t d);
hipError_t launch_clock_probe(uint64_t* out, uint32_t n_cu, hipStream_t stream);
hipError_t launch_probe(int kind, const void* a, void* b, size_t n16, uint32_t n_cu, uint32_t blocks_per_cu, bool slab,
                        hipStream_t stream);
}  // namespace crdt

using namespace crdt;

namespace {

constexpr uint32_t kCtxParts = 1024;

// Device buffer that only grows.  A buffer it outgrows is retired, not freed:
// a HIP graph captured earlier may still name it, so retired buffers live
// until crdt_ctx_destroy.
struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    std::vector<void*>* retired = nullptr;
    int reserve(size_t want) {
        if (want <= bytes) return CRDT_OK;
        if (p) {
            if (retired)
                retired->push_back(p);
            else
                (void)hipFree(p);
        }
        p = nullptr;
        bytes = 0;
        if (hipMalloc(&p, want) != hipSuccess) return CRDT_E_NOMEM;
        bytes = want;
        return CRDT_OK;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    template <typename T>
    T* as(size_t byte_off = 0) const {
        return reinterpret_cast<T*>(static_cast<char*>(p) + byte_off);
    }
};

// The page-locked blocks crdt_host_alloc made (base -> size): a *_batch call
// whose input arrays all lie in one of them is staged by ONE copy of the span
// they cover (Stager), because each runtime H2D copy call costs the host 1-7
// ms before its DMA is even submitted, whatever its size
// (profiles/r05i_boundary_timeline.txt), while the span moves at PCIe rate.
// Each block also keeps its device-side address: a host-path call whose outputs
// lie in such blocks has its packed results written there by the gather kernel
// (pack.hip) instead of copied back by runtime copy calls.
struct HostBlock {
    size_t size;
    uintptr_t dev;  // hipHostGetDevicePointer of the base (0: none)
};
std::mutex g_host_mu;
std::map<uintptr_t, HostBlock> g_host_blocks;

bool host_block(const void* p, uintptr_t& base, size_t& size, uintptr_t* dev = nullptr) {
    const uintptr_t a = (uintptr_t)p;
    std::lock_guard<std::mutex> lk(g_host_mu);
    auto it = g_host_blocks.upper_bound(a);
    if (it == g_host_blocks.begin()) return false;
    --it;
    if (a >= it->first + it->second.size) return false;
    base = it->first;
    size = it->second.size;
    if (dev) *dev = it->second.dev;
    return true;
}

// The device address of host range [p, p + bytes) when all of it lies in one
// crdt_host_alloc block (0 otherwise).
uintptr_t host_dev_addr(const void* p, size_t bytes) {
    uintptr_t base = 0, dev = 0;
    size_t size = 0;
    if (!p || !host_block(p, base, size, &dev) || !dev) return 0;
    const uintptr_t a = (uintptr_t)p;
    if (a + bytes > base + size) return 0;
    return dev + (a - base);
}


}  // namespace

struct crdt_ctx {
    int device = 0;
    int n_cu = 256;
    // [0,64): per-call counters {wl_count, wl_head, -, ..., chunk_ctr[8] at 32}
    // zeroed by every call; [64,68): status word, cleared by crdt_ctx_sync.
    DevBuf ws;
    DevBuf worklist;
    DevBuf defer;  // folds: documents the lean pass leaves to the general kernel
    DevBuf parts;
    DevBuf scratch;  // fold block path ping-pong: keys | actors | counters
    // large-document join tiles (tile.hip): descriptors + look-back words for
    // tile_cap tiles, per-slot and per-run tile counts for the worklist
    DevBuf tile_desc, tile_geo, tile_flags, tile_slot, tile_run;
    DevBuf sort_tmp, sort_idx, sort_ends;  // ingest sort (sort.hip)
    // crdt_ctx_set_option("join_tile_capacity"): 2^22 tiles (235 MB of tile workspace, on
    // first use); config 4 needs 1.035 M tiles of 1,024 positions, 2.07 M of 512
    uint32_t tile_cap = 1u << 22;
    bool join_tiles = true;                   // crdt_ctx_set_option("join_tiles")
    uint32_t tile_shape = 9;                  // crdt_ctx_set_option("join_tile_shape")
    bool tile_nt_stores = true;               // crdt_ctx_set_option("join_tile_nt_stores")
    uint32_t tile_split_bpc = 4;              // crdt_ctx_set_option("join_tile_split_blocks_per_cu")
    uint32_t tile_shards = 8;                 // crdt_ctx_set_option("join_tile_dispensers")
    uint32_t tile_max_passes = 256;           // crdt_ctx_set_option("join_tile_max_passes")
    // the tiles of the join this host-path call is about to launch, counted from
    // its host arrays (0: unknown, an _async call: bounded instead, join_common)
    uint64_t call_tiles = 0;
    size_t scratch_slots = 0;
    uint32_t max_doc_entries = 0xFFFFFFFFu;  // caller's promise (crdt_ctx_set_max_doc_entries)
    uint32_t join_docs_per_wave = 8;          // crdt_ctx_set_option("join_docs_per_wave")
    bool join_nt_stores = true;               // crdt_ctx_set_option("join_nt_stores")
    bool join_stage_stores = true;            // crdt_ctx_set_option("join_stage_stores")
    uint32_t join_slab_per_cu = 0;            // crdt_ctx_set_option("join_slab_blocks_per_cu"): 0 = blocks in order
    bool fold_lean_first = true;              // crdt_ctx_set_option("fold_lean_first")
    uint32_t probe_blocks_per_cu = 16;        // crdt_ctx_set_option("probe_blocks_per_cu")
    bool probe_slab = false;                  // crdt_ctx_set_option("probe_slab")
    bool pack_outputs = false;                // crdt_ctx_set_option("pack_batch_outputs")
    bool span_staging = true;                 // crdt_ctx_set_option("span_staging")
    // staging for the *_batch host path: per-array buffers, and the device image
    // of the part of one crdt_host_alloc block a call's inputs cover (Stager)
    DevBuf stage[48];
    DevBuf span_img;
    // set by a *_batch call around its merge launch: the merge's first kernel is
    // gated on the status word its order checks wrote (Work::gate)
    bool call_gate = false;
    // set by a *_batch call whose host arrays show no document above 64 live
    // entries on a side: the join launches no large-document path at all
    bool call_small = false;
    // page-locked word the packed-output gather copies the status word into, so
    // a host-path call reads its verdict without another runtime call
    uint32_t* host_status = nullptr;
    hipStream_t stream = nullptr;
    // Ordering of the shared workspace across streams: the last call's stream
    // and an event recorded after its launches.  A call on another stream
    // waits for that event first (see enter()).
    hipEvent_t last_ev = nullptr;
    hipStream_t last_stream = nullptr;
    bool has_last = false;
    std::vector<void*> retired;  // outgrown workspace buffers, freed at destroy
    void* comm = nullptr;        // RCCL communicator (comm.cpp)
    void* comm_group = nullptr;  // single-process group it belongs to (comm.cpp)
};

void crdt_internal_comm_release(crdt_ctx* ctx);
int crdt_internal_device(crdt_ctx* ctx) { return ctx->device; }
hipStream_t crdt_internal_stream(crdt_ctx* ctx) { return ctx->stream; }
void** crdt_internal_comm(crdt_ctx* ctx) { return &ctx->comm; }
void** crdt_internal_comm_group(crdt_ctx* ctx) { return &ctx->comm_group; }
// Order stream s after the context's last call (when that ran on another stream).
int crdt_internal_order(crdt_ctx* ctx, hipStream_t s) {
    if (ctx->has_last && ctx->last_stream != s && hipStreamWaitEvent(s, ctx->last_ev, 0) != hipSuccess)
        return CRDT_E_HIP;
    return CRDT_OK;
}

namespace {

int hip_err(hipError_t e) { return e == hipSuccess ? CRDT_OK : CRDT_E_HIP; }

int set_device(crdt_ctx* ctx) { return hip_err(hipSetDevice(ctx->device)); }

uint32_t block_grid(const crdt_ctx* ctx) { return (uint32_t)ctx->n_cu * 2u; }

Work make_work(crdt_ctx* ctx) {
    Work w;
    w.wl_count = ctx->ws.as<uint32_t>(0);
    w.wl_head = ctx->ws.as<uint32_t>(4);
    w.status = ctx->ws.as<uint32_t>(64);
    w.chunk_ctr = ctx->ws.as<uint32_t>(32);
    w.worklist = ctx->worklist.as<uint32_t>();
    w.defer_count = ctx->ws.as<uint32_t>(8);
    w.defer = ctx->defer.as<uint32_t>();
    w.gate = ctx->call_gate ? w.status : nullptr;
    return w;
}

// Start of a call that uses the context's shared workspace (worklist,
// counters, scratch, status word, context partials) on stream s.  Work of an
// earlier call on a different stream is ordered before it with a stream wait
// on that call's event.  While s is capturing a graph no wait is recorded
// (the caller orders the capture; the capture itself must not allocate, see
// grow()).
int enter(crdt_ctx* ctx, hipStream_t s, bool& capturing) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &st) != hipSuccess) return CRDT_E_HIP;
    capturing = st != hipStreamCaptureStatusNone;
    if (!capturing && ctx->has_last && ctx->last_stream != s)
        if (hipStreamWaitEvent(s, ctx->last_ev, 0) != hipSuccess) return CRDT_E_HIP;
    return CRDT_OK;
}

// End of such a call: its launches are what the next call on another stream waits for.
int leave(crdt_ctx* ctx, hipStream_t s, bool capturing, int rc) {
    if (rc != CRDT_OK || capturing) return rc;
    if (hipEventRecord(ctx->last_ev, s) != hipSuccess) return CRDT_E_HIP;
    ctx->last_stream = s;
    ctx->has_last = true;
    return CRDT_OK;
}

// Grow a workspace buffer; refused while capturing (an allocation would break
// the capture, and the graph would keep the old address).
int grow(DevBuf& b, size_t want, bool capturing) {
    if (want <= b.bytes) return CRDT_OK;
    if (capturing) return CRDT_E_WORKSPACE;
    return b.reserve(want);
}

int reserve_worklist(crdt_ctx* ctx, uint32_t n_docs) {
    int rc = ctx->worklist.reserve(std::max<size_t>((size_t)n_docs, 1) * sizeof(uint32_t));
    if (rc == CRDT_OK) rc = ctx->defer.reserve(std::max<size_t>((size_t)n_docs, 1) * sizeof(uint32_t));
    return rc;
}

int reserve_scratch(crdt_ctx* ctx, uint64_t slots) {
    if (slots <= ctx->scratch_slots) return CRDT_OK;
    int rc = ctx->scratch.reserve(slots * 20 + 64);
    if (rc == CRDT_OK) ctx->scratch_slots = slots;
    return rc;
}

BatchView view(const crdt_awset_batch* b) {
    return BatchView{b->n_docs, b->R, b->offsets, b->counts, b->keys, b->actors, b->counters, b->vv};
}

OutView view(const crdt_awset_out* o) {
    return OutView{o->offsets, o->counts, o->keys, o->actors, o->counters, o->vv};
}

SrcView view(const crdt_src_batch* s) {
    return SrcView{s->n_docs,    s->R,       s->doc_srcs, s->src_actor, s->vv,    s->entry_off, s->keys,
                   s->actors,    s->counters, s->tomb_off, s->tkeys,     s->tactors, s->tcounters};
}

bool batch_ptrs_ok(const crdt_awset_batch* b) {
    return b && b->offsets && (b->n_docs == 0 || b->vv) && b->R > 0 && b->R <= CRDT_MAX_R;
}

bool out_ptrs_ok(const crdt_awset_out* o) {
    return o && o->offsets && o->counts && o->keys && o->actors && o->counters && o->vv;
}

bool src_ptrs_ok(const crdt_src_batch* s) {
    return s && s->doc_srcs && s->src_actor && s->entry_off && s->R > 0 && s->R <= CRDT_MAX_R &&
           (!s->tomb_off || (s->tkeys && s->tactors && s->tcounters));
}

}  // namespace

extern "C" {

int crdt_abi_version(void) { return CRDTGPU_ABI_VERSION; }

const char* crdt_strerror(int code) {
    switch (code) {
        case CRDT_OK: return "ok";
        case CRDT_E_INVALID: return "invalid argument";
        case CRDT_E_ACTOR_RANGE: return "dot actor == len(VersionVector): the reference panics (index out of range)";
        case CRDT_E_UNSORTED: return "keys of a document are not strictly ascending";
        case CRDT_E_CAPACITY: return "live count exceeds the document's slots";
        case CRDT_E_HIP: return "HIP runtime error";
        case CRDT_E_NOMEM: return "device allocation failed";
        case CRDT_E_WORKSPACE: return "fold scratch too small: call crdt_ctx_reserve with the output slot count";
        case CRDT_E_RCCL: return "RCCL unavailable or a collective failed";
        case CRDT_E_DUP_KEY: return "a key appears twice in one document";
        default: return "unknown error";
    }
}

int crdt_ctx_create(int device, crdt_ctx** out) {
    if (!out) return CRDT_E_INVALID;
    *out = nullptr;
    crdt_ctx* ctx = new (std::nothrow) crdt_ctx();
    if (!ctx) return CRDT_E_NOMEM;
    ctx->device = device;
    for (DevBuf* b : {&ctx->ws, &ctx->worklist, &ctx->defer, &ctx->parts, &ctx->scratch, &ctx->tile_desc, &ctx->tile_geo, &ctx->tile_flags,
                      &ctx->tile_slot, &ctx->tile_run, &ctx->sort_tmp, &ctx->sort_idx, &ctx->sort_ends})
        b->retired = &ctx->retired;
    for (auto& b : ctx->stage) b.retired = &ctx->retired;
    ctx->span_img.retired = &ctx->retired;
    int rc = set_device(ctx);
    hipDeviceProp_t prop;
    if (rc == CRDT_OK && hipGetDeviceProperties(&prop, device) == hipSuccess) ctx->n_cu = prop.multiProcessorCount;
    if (rc == CRDT_OK) rc = ctx->ws.reserve(128);
    if (rc == CRDT_OK) rc = hip_err(hipMemset(ctx->ws.p, 0, 128));
    if (rc == CRDT_OK) rc = reserve_worklist(ctx, 1024);
    if (rc == CRDT_OK) rc = ctx->parts.reserve((size_t)kCtxParts * CRDT_MAX_R * sizeof(uint64_t));
    if (rc == CRDT_OK) rc = hip_err(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
    if (rc == CRDT_OK) rc = hip_err(hipEventCreateWithFlags(&ctx->last_ev, hipEventDisableTiming));
    if (rc == CRDT_OK && hipHostMalloc(reinterpret_cast<void**>(&ctx->host_status), 64, hipHostMallocDefault) != hipSuccess)
        ctx->host_status = nullptr;  // (then the host path reads the status word back instead)
    if (rc != CRDT_OK) {
        crdt_ctx_destroy(ctx);
        return rc;
    }
    *out = ctx;
    return CRDT_OK;
}

void crdt_ctx_destroy(crdt_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    // drain every queued call (an all-reduce on the communicator included)
    // before the communicator and the workspaces go away
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    if (ctx->last_ev) (void)hipEventSynchronize(ctx->last_ev);
    crdt_internal_comm_release(ctx);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    if (ctx->last_ev) (void)hipEventDestroy(ctx->last_ev);
    for (void* p : ctx->retired) (void)hipFree(p);
    ctx->retired.clear();
    if (ctx->host_status) (void)hipHostFree(ctx->host_status);
    ctx->ws.release();
    ctx->worklist.release();
    ctx->defer.release();
    ctx->parts.release();
    ctx->scratch.release();
    for (DevBuf* b : {&ctx->tile_desc, &ctx->tile_geo, &ctx->tile_flags, &ctx->tile_slot, &ctx->tile_run,
                      &ctx->sort_tmp, &ctx->sort_idx, &ctx->sort_ends})
        b->release();
    for (auto& b : ctx->stage) b.release();
    ctx->span_img.release();
    delete ctx;
}

int crdt_ctx_reserve(crdt_ctx* ctx, uint32_t max_docs, uint64_t max_fold_slots) {
    if (!ctx) return CRDT_E_INVALID;
    int rc = set_device(ctx);
    if (rc == CRDT_OK) rc = reserve_worklist(ctx, max_docs);
    if (rc == CRDT_OK) rc = reserve_scratch(ctx, max_fold_slots);
    return rc;
}

int crdt_ctx_set_max_doc_entries(crdt_ctx* ctx, uint32_t max_entries) {
    if (!ctx) return CRDT_E_INVALID;
    ctx->max_doc_entries = max_entries;
    return CRDT_OK;
}

int crdt_ctx_set_option(crdt_ctx* ctx, const char* name, int64_t value) {
    if (!ctx || !name) return CRDT_E_INVALID;
    if (!strcmp(name, "join_docs_per_wave")) {
        if (value != 1 && value != 2 && value != 4 && value != 8 && value != 16) return CRDT_E_INVALID;
        ctx->join_docs_per_wave = (uint32_t)value;
        return CRDT_OK;
    }
    if (!strcmp(name, "join_tile_capacity")) {  // tiles per pass of the tile path (workspace: 56 B a tile)
        if (value < 1 || value > (1ll << 28)) return CRDT_E_INVALID;
        ctx->tile_cap = (uint32_t)value;
        return CRDT_OK;
    }
    if (!strcmp(name, "join_tile_max_passes")) {  // more tiles than passes x capacity -> block kernel
        if (value < 1 || value > 65536) return CRDT_E_INVALID;
        ctx->tile_max_passes = (uint32_t)value;
        return CRDT_OK;
    }
    if (!strcmp(name, "join_tile_shape")) {  // threads x positions: look-back per tile 0: 512x4, 1: 256x4, 2: 256x8,
                                             // 3: 1024x2; deferred by a tile 4: 256x4, 5: 512x2, 6: 256x8, 7: 128x8,
                                             // and aligned store windows 8: 256x4, 9: 512x2 (default), 10: 256x2
        if (value < 0 || value > 10) return CRDT_E_INVALID;
        ctx->tile_shape = (uint32_t)value;
        return CRDT_OK;
    }
    if (!strcmp(name, "join_tile_dispensers")) {  // tile dispenser words: 1, or 8 (one per XCD, tile.hip)
        if (value != 1 && value != 8) return CRDT_E_INVALID;
        ctx->tile_shards = (uint32_t)value;
        return CRDT_OK;
    }
    if (!strcmp(name, "join_tile_split_blocks_per_cu")) {  // grid of the tile plan's merge-path search
        if (value < 1 || value > 64) return CRDT_E_INVALID;
        ctx->tile_split_bpc = (uint32_t)value;
        return CRDT_OK;
    }
    if (!strcmp(name, "join_tile_nt_stores")) {
        ctx->tile_nt_stores = value != 0;
        return CRDT_OK;
    }
    if (!strcmp(name, "join_tiles")) {  // 0: large documents one workgroup each (join_block_kernel)
        ctx->join_tiles = value != 0;
        return CRDT_OK;
    }
    if (!strcmp(name, "pack_batch_outputs")) {  // *_batch joins / exchanges / folds: live entries only, packed
        ctx->pack_outputs = value != 0;
        return CRDT_OK;
    }
    if (!strcmp(name, "span_staging")) {  // *_batch inputs in one crdt_host_alloc block: one copy of their span
        ctx->span_staging = value != 0;
        return CRDT_OK;
    }
    if (!strcmp(name, "probe_slab")) {  // bandwidth probes: one contiguous slab per workgroup
        ctx->probe_slab = value != 0;
        return CRDT_OK;
    }
    if (!strcmp(name, "probe_blocks_per_cu")) {
        if (value < 1 || value > 64) return CRDT_E_INVALID;
        ctx->probe_blocks_per_cu = (uint32_t)value;
        return CRDT_OK;
    }
    if (!strcmp(name, "fold_lean_first")) {  // delta folds: slot-walk pass first, the rest deferred (fold.hip)
        ctx->fold_lean_first = value != 0;
        return CRDT_OK;
    }
    if (!strcmp(name, "join_nt_stores")) {
        ctx->join_nt_stores = value != 0;
        return CRDT_OK;
    }
    if (!strcmp(name, "join_stage_stores")) {
        ctx->join_stage_stores = value != 0;
        return CRDT_OK;
    }
    if (!strcmp(name, "join_slab_blocks_per_cu")) {  // slab order of the wave kernel's blocks (SlabMap G per CU)
        if (value < 0 || value > 64) return CRDT_E_INVALID;
        ctx->join_slab_per_cu = (uint32_t)value;
        return CRDT_OK;
    }
    return CRDT_E_INVALID;
}

int crdt_ctx_sync(crdt_ctx* ctx, void* stream) {
    if (!ctx) return CRDT_E_INVALID;
    int rc = set_device(ctx);
    if (rc != CRDT_OK) return rc;
    hipStream_t s = (hipStream_t)stream;
    if (hipStreamSynchronize(s) != hipSuccess) return CRDT_E_HIP;
    // the status word is shared: also wait for the last call if it ran elsewhere
    if (ctx->has_last && ctx->last_stream != s && hipEventSynchronize(ctx->last_ev) != hipSuccess) return CRDT_E_HIP;
    uint32_t status = 0;
    if (hipMemcpy(&status, ctx->ws.as<uint32_t>(64), sizeof(status), hipMemcpyDeviceToHost) != hipSuccess)
        return CRDT_E_HIP;
    if (status) {
        if (hipMemset(ctx->ws.as<uint32_t>(64), 0, sizeof(uint32_t)) != hipSuccess) return CRDT_E_HIP;
        if (status & kErrUnsorted) return CRDT_E_UNSORTED;
        if (status & kErrActorRange) return CRDT_E_ACTOR_RANGE;
        if (status & kErrWorkspace) return CRDT_E_WORKSPACE;
        if (status & kErrHint) return CRDT_E_INVALID;
        if (status & kErrCapacity) return CRDT_E_CAPACITY;
        if (status & kErrDupKey) return CRDT_E_DUP_KEY;
    }
    return CRDT_OK;
}

static int join_common(crdt_ctx* ctx, const crdt_awset_batch* dst, const crdt_awset_batch* src,
                       const crdt_awset_out* out, const crdt_awset_out* out2, void* stream) {
    if (!ctx || !batch_ptrs_ok(dst) || !batch_ptrs_ok(src) || !out_ptrs_ok(out) || (out2 && !out_ptrs_ok(out2)))
        return CRDT_E_INVALID;
    if (dst->n_docs != src->n_docs || dst->R != src->R) return CRDT_E_INVALID;
    int rc = set_device(ctx);
    if (rc != CRDT_OK) return rc;
    hipStream_t s = (hipStream_t)stream;
    bool cap = false;
    rc = enter(ctx, s, cap);
    if (rc == CRDT_OK) rc = grow(ctx->worklist, std::max<size_t>(dst->n_docs, 1) * sizeof(uint32_t), cap);
    if (rc != CRDT_OK) return rc;
    const bool no_large = ctx->max_doc_entries <= 64 || ctx->call_small;
    TileWork tw{};
    const bool tiles = !no_large && ctx->join_tiles;
    if (tiles) {
        const size_t n = std::max<size_t>(dst->n_docs, 1);
        rc = grow(ctx->tile_desc, ((size_t)ctx->tile_cap + 1) * 16, cap);  // (+1: the next pass's first split)
        if (rc == CRDT_OK) rc = grow(ctx->tile_geo, ((size_t)ctx->tile_cap + 8) * 32, cap);  // (+8: geo_slot)
        if (rc == CRDT_OK) rc = grow(ctx->tile_flags, (size_t)ctx->tile_cap * 8, cap);
        if (rc == CRDT_OK) rc = grow(ctx->tile_slot, n * 4, cap);
        if (rc == CRDT_OK) rc = grow(ctx->tile_run, ((n + 1023) / 1024) * 4, cap);
        if (rc != CRDT_OK) return rc;
        uint32_t* w = ctx->ws.as<uint32_t>(0);
        // Passes of tile_cap tiles: as many as the call's tiles can need.  A host-path
        // call counted them (ctx->call_tiles); otherwise a document of nd + ns merged
        // positions has ceil((nd + ns) / T) tiles, and a batch's slots are < 2^32 per
        // side, so a call has at most 2^33 / T + n_docs -- or, under the caller's
        // max_doc_entries promise, n_docs * ceil(2 max / T).  Passes past the call's
        // tiles return at once.  The block kernel is launched behind them (gated on
        // the plan's fallback word) unless the passes hold every tile a call can have
        // without trusting the promise: beyond them (tile_max_passes, or a broken
        // promise) it takes the worklist.
        const uint64_t T = tile_positions(ctx->tile_shape);
        const uint64_t hard = ctx->call_tiles ? ctx->call_tiles : (1ull << 33) / T + dst->n_docs;
        uint64_t bound = hard;
        if (!ctx->call_tiles && ctx->max_doc_entries != 0xFFFFFFFFu)
            bound = std::min<uint64_t>(bound, (uint64_t)dst->n_docs * ((2ull * ctx->max_doc_entries + T - 1) / T));
        auto passes_for = [&](uint64_t t) { return std::max<uint64_t>(1, (t + ctx->tile_cap - 1) / ctx->tile_cap); };
        const uint32_t passes = (uint32_t)std::min<uint64_t>(passes_for(bound), ctx->tile_max_passes);
        tw = TileWork{ctx->tile_desc.as<uint4>(), ctx->tile_geo.as<uint4>(), ctx->tile_flags.as<uint64_t>(), ctx->tile_slot.as<uint32_t>(),
                      ctx->tile_run.as<uint32_t>(), w + 3, w + 8, w + 5, w + 6, ctx->tile_cap,
                      tile_positions(ctx->tile_shape), ctx->tile_shape, ctx->tile_nt_stores ? 1u : 0u,
                      ctx->tile_split_bpc, ctx->tile_shards, 0u, passes, passes_for(hard) <= passes ? 1u : 0u};
    }
    // the per-call counters are read only by the large-document paths
    if (!no_large && launch_reset_work(ctx->ws.as<uint32_t>(0), s) != hipSuccess) return CRDT_E_HIP;
    OutView o2v;
    if (out2) o2v = view(out2);
    rc = hip_err(launch_join(view(dst), view(src), view(out), out2 ? &o2v : nullptr, make_work(ctx),
                             ctx->join_docs_per_wave, ctx->join_nt_stores, ctx->join_stage_stores,
                             ctx->join_slab_per_cu * (uint32_t)ctx->n_cu, block_grid(ctx), no_large,
                             tiles ? &tw : nullptr, (uint32_t)ctx->n_cu, s));
    return leave(ctx, s, cap, rc);
}

int crdt_awset_join_async(crdt_ctx* ctx, const crdt_awset_batch* dst, const crdt_awset_batch* src,
                          const crdt_awset_out* out, void* stream) {
    return join_common(ctx, dst, src, out, nullptr, stream);
}

int crdt_awset_exchange_async(crdt_ctx* ctx, const crdt_awset_batch* a, const crdt_awset_batch* b,
                              const crdt_awset_out* out_ab, const crdt_awset_out* out_ba, void* stream) {
    // out_ba->keys == out_ab->keys: one shared key column (both directions hold
    // the same keys at the same slots); every other array must be its own.
    // Checked here: no two of the twelve arrays start at the same address
    // (keys == keys excepted), and the per-document arrays, whose sizes the
    // host knows (offsets, counts, vv), do not overlap at all.  The entry
    // arrays' capacity lives in device memory, so a partial overlap of them
    // cannot be checked and is undefined (include/crdtgpu.h).
    if (!out_ab || !out_ba || !a) return CRDT_E_INVALID;
    const size_t n = a->n_docs, R = a->R;
    struct Range {
        uintptr_t p;
        size_t bytes;  // 0: size unknown here (entry arrays)
    };
    const Range r[12] = {{(uintptr_t)out_ab->offsets, (n + 1) * 4}, {(uintptr_t)out_ab->counts, n * 4},
                         {(uintptr_t)out_ab->vv, n * R * 8},       {(uintptr_t)out_ab->keys, 0},
                         {(uintptr_t)out_ab->actors, 0},           {(uintptr_t)out_ab->counters, 0},
                         {(uintptr_t)out_ba->offsets, (n + 1) * 4}, {(uintptr_t)out_ba->counts, n * 4},
                         {(uintptr_t)out_ba->vv, n * R * 8},       {(uintptr_t)out_ba->keys, 0},
                         {(uintptr_t)out_ba->actors, 0},           {(uintptr_t)out_ba->counters, 0}};
    for (int i = 0; i < 12; ++i)
        for (int j = i + 1; j < 12; ++j) {
            if (i == 3 && j == 9) continue;  // the shared key column
            if (!r[i].p || !r[j].p) continue;  // NULL pointers are rejected by join_common
            if (r[i].p == r[j].p) return CRDT_E_INVALID;
            if (r[i].bytes && r[j].bytes && r[i].p < r[j].p + r[j].bytes && r[j].p < r[i].p + r[i].bytes)
                return CRDT_E_INVALID;
        }
    return join_common(ctx, a, b, out_ab, out_ba, stream);
}

int crdt_awset_fold_async(crdt_ctx* ctx, int mode, const crdt_awset_batch* dst, const crdt_src_batch* srcs,
                          const crdt_awset_out* out, void* stream) {
    if (!ctx || !batch_ptrs_ok(dst) || !src_ptrs_ok(srcs) || !out_ptrs_ok(out)) return CRDT_E_INVALID;
    if (mode != CRDT_FOLD_AWSET && mode != CRDT_FOLD_DELTA) return CRDT_E_INVALID;
    if (dst->n_docs != srcs->n_docs || dst->R != srcs->R) return CRDT_E_INVALID;
    int rc = set_device(ctx);
    if (rc != CRDT_OK) return rc;
    hipStream_t s = (hipStream_t)stream;
    bool cap = false;
    rc = enter(ctx, s, cap);
    if (rc == CRDT_OK) rc = grow(ctx->worklist, std::max<size_t>(dst->n_docs, 1) * sizeof(uint32_t), cap);
    if (rc == CRDT_OK) rc = grow(ctx->defer, std::max<size_t>(dst->n_docs, 1) * sizeof(uint32_t), cap);
    if (rc != CRDT_OK) return rc;
    if (ctx->scratch_slots == 0) {
        if (cap) return CRDT_E_WORKSPACE;
        if (reserve_scratch(ctx, 1) != CRDT_OK) return CRDT_E_NOMEM;
    }
    if (launch_reset_work(ctx->ws.as<uint32_t>(0), s) != hipSuccess) return CRDT_E_HIP;
    const size_t slots = ctx->scratch_slots;
    Scratch scr{ctx->scratch.as<uint64_t>(0), ctx->scratch.as<uint32_t>(slots * 16), ctx->scratch.as<uint64_t>(slots * 8),
                slots};
    rc = hip_err(launch_fold(mode, view(dst), view(srcs), view(out), scr, make_work(ctx), block_grid(ctx),
                             ctx->fold_lean_first, s));
    return leave(ctx, s, cap, rc);
}

int crdt_awset_apply_async(crdt_ctx* ctx, const crdt_awset_batch* state, const crdt_tomb_batch* tombs,
                           const crdt_op_batch* ops, const crdt_awset_out* out, const crdt_tomb_out* tomb_out,
                           void* stream) {
    if (!ctx || !batch_ptrs_ok(state) || !ops || !ops->op_off || !ops->doc_actor || !out_ptrs_ok(out))
        return CRDT_E_INVALID;
    if (ops->n_docs != state->n_docs) return CRDT_E_INVALID;
    if (tombs && (!tombs->offsets || !tombs->keys || !tombs->actors || !tombs->counters)) return CRDT_E_INVALID;
    if (tomb_out && (!tomb_out->offsets || !tomb_out->counts || !tomb_out->keys || !tomb_out->actors ||
                     !tomb_out->counters))
        return CRDT_E_INVALID;
    int rc = set_device(ctx);
    if (rc != CRDT_OK) return rc;
    hipStream_t s = (hipStream_t)stream;
    bool cap = false;
    rc = enter(ctx, s, cap);
    if (rc != CRDT_OK) return rc;
    TombView tv{};
    if (tombs) tv = TombView{tombs->offsets, tombs->counts, tombs->keys, tombs->actors, tombs->counters};
    TombOut to{};
    if (tomb_out) to = TombOut{tomb_out->offsets, tomb_out->counts, tomb_out->keys, tomb_out->actors, tomb_out->counters};
    const ApplyOps av{ops->n_docs, ops->op_off, ops->kind, ops->keys, ops->doc_actor};
    rc = hip_err(launch_apply(view(state), tv, av, view(out), to, tomb_out != nullptr, make_work(ctx),
                              (uint32_t)ctx->n_cu, s));
    return leave(ctx, s, cap, rc);
}

int crdt_awset_sort_async(crdt_ctx* ctx, const crdt_awset_batch* in, uint32_t n_slots, const crdt_awset_out* out,
                          void* stream) {
    if (!ctx || !batch_ptrs_ok(in) || !out_ptrs_ok(out) || out->keys == in->keys) return CRDT_E_INVALID;
    if (n_slots && (!in->keys || !in->actors || !in->counters)) return CRDT_E_INVALID;
    int rc = set_device(ctx);
    if (rc != CRDT_OK) return rc;
    hipStream_t s = (hipStream_t)stream;
    bool cap = false;
    rc = enter(ctx, s, cap);
    if (rc != CRDT_OK) return rc;
    size_t tb = 0;
    if (sort_storage(in->n_docs, n_slots, &tb) != hipSuccess) return CRDT_E_HIP;
    rc = grow(ctx->sort_tmp, std::max<size_t>(tb, 16), cap);
    if (rc == CRDT_OK) rc = grow(ctx->sort_idx, std::max<size_t>(n_slots, 1) * 4, cap);
    if (rc == CRDT_OK) rc = grow(ctx->sort_ends, std::max<size_t>(in->n_docs, 1) * 4, cap);
    if (rc != CRDT_OK) return rc;
    rc = hip_err(launch_sort(view(in), n_slots, view(out), ctx->sort_tmp.p, ctx->sort_tmp.bytes,
                             ctx->sort_ends.as<uint32_t>(), ctx->sort_idx.as<uint32_t>(), ctx->ws.as<uint32_t>(64),
                             (uint32_t)ctx->n_cu, s));
    return leave(ctx, s, cap, rc);
}

int crdt_vv_min_async(crdt_ctx* ctx, uint64_t* dst, const uint64_t* src, size_t n, void* stream) {
    if (!ctx || (n && (!dst || !src))) return CRDT_E_INVALID;
    int rc = set_device(ctx);
    if (rc != CRDT_OK) return rc;
    return hip_err(launch_vv_min(dst, src, n, (hipStream_t)stream));
}

int crdt_tombstone_gc_async(crdt_ctx* ctx, const crdt_tomb_batch* tombs, uint32_t n_docs, uint32_t R,
                            const uint64_t* stable_vv, const crdt_tomb_out* out, void* stream) {
    if (!ctx || !tombs || !tombs->offsets || !out || !out->offsets || !out->counts || R == 0 || R > CRDT_MAX_R ||
        (n_docs && !stable_vv))
        return CRDT_E_INVALID;
    int rc = set_device(ctx);
    if (rc != CRDT_OK) return rc;
    const TombView tv{tombs->offsets, tombs->counts, tombs->keys, tombs->actors, tombs->counters};
    const TombOut to{out->offsets, out->counts, out->keys, out->actors, out->counters};
    return hip_err(launch_tomb_gc(tv, n_docs, R, stable_vv, to, (uint32_t)ctx->n_cu, (hipStream_t)stream));
}

int crdt_vv_max_async(crdt_ctx* ctx, uint64_t* dst, const uint64_t* src, size_t n, void* stream) {
    if (!ctx || (n && (!dst || !src))) return CRDT_E_INVALID;
    int rc = set_device(ctx);
    if (rc != CRDT_OK) return rc;
    return hip_err(launch_vv_max(dst, src, n, (hipStream_t)stream));
}

int crdt_causal_context_async(crdt_ctx* ctx, const uint64_t* vv, uint32_t n_docs, uint32_t R, uint64_t* out,
                              void* stream) {
    if (!ctx || !out || R == 0 || R > CRDT_MAX_R || (n_docs && !vv)) return CRDT_E_INVALID;
    int rc = set_device(ctx);
    if (rc != CRDT_OK) return rc;
    uint32_t n_part = std::min<uint32_t>(kCtxParts, std::max<uint32_t>(1u, (n_docs + 255) / 256));
    hipStream_t s = (hipStream_t)stream;
    bool cap = false;
    rc = enter(ctx, s, cap);
    if (rc != CRDT_OK) return rc;
    rc = hip_err(launch_context(vv, n_docs, R, ctx->parts.as<uint64_t>(), n_part, out, s));
    return leave(ctx, s, cap, rc);
}

int crdt_gen_pair_async(crdt_ctx* ctx, uint64_t seed, uint32_t n_docs, const crdt_awset_out* a,
                        const crdt_awset_out* b, void* stream) {
    if (!ctx || !out_ptrs_ok(a) || !out_ptrs_ok(b)) return CRDT_E_INVALID;
    if ((uint64_t)n_docs * 64ull >= (1ull << 32)) return CRDT_E_INVALID;
    int rc = set_device(ctx);
    if (rc != CRDT_OK) return rc;
    return hip_err(launch_gen_pair(seed, n_docs, view(a), view(b), (hipStream_t)stream));
}

int crdt_gen_delta_async(crdt_ctx* ctx, uint64_t seed, uint32_t n_docs, uint32_t R, uint32_t n_srcs_per_doc,
                         const crdt_awset_out* dst, const crdt_src_batch* srcs, void* stream) {
    if (!ctx || !out_ptrs_ok(dst) || !src_ptrs_ok(srcs) || !srcs->tomb_off || R == 0 || R > CRDT_MAX_R ||
        n_srcs_per_doc == 0)
        return CRDT_E_INVALID;
    if ((uint64_t)n_docs * n_srcs_per_doc * 8ull >= (1ull << 32) || (uint64_t)n_docs * 64ull >= (1ull << 32))
        return CRDT_E_INVALID;
    int rc = set_device(ctx);
    if (rc != CRDT_OK) return rc;
    auto w = [](const void* p) { return const_cast<void*>(p); };
    SrcOutView S{(uint32_t*)w(srcs->doc_srcs), (uint32_t*)w(srcs->src_actor), (uint64_t*)w(srcs->vv),
                 (uint32_t*)w(srcs->entry_off), (uint64_t*)w(srcs->keys), (uint32_t*)w(srcs->actors),
                 (uint64_t*)w(srcs->counters), (uint32_t*)w(srcs->tomb_off), (uint64_t*)w(srcs->tkeys),
                 (uint32_t*)w(srcs->tactors), (uint64_t*)w(srcs->tcounters)};
    return hip_err(launch_gen_delta(seed, n_docs, R, n_srcs_per_doc, view(dst), S, (hipStream_t)stream));
}

int crdt_gen_replicas_async(crdt_ctx* ctx, uint64_t seed, uint32_t n_docs, uint32_t replicas, uint32_t entries,
                            const crdt_awset_out* dst, const crdt_src_batch* srcs, void* stream) {
    if (!ctx || !out_ptrs_ok(dst) || !src_ptrs_ok(srcs) || !srcs->tomb_off) return CRDT_E_INVALID;
    if (replicas < 2 || replicas > CRDT_MAX_R || entries < 1 || entries > 32 || (entries & (entries - 1)))
        return CRDT_E_INVALID;
    if ((uint64_t)n_docs * replicas * entries >= (1ull << 32)) return CRDT_E_INVALID;
    int rc = set_device(ctx);
    if (rc != CRDT_OK) return rc;
    auto w = [](const void* p) { return const_cast<void*>(p); };
    SrcOutView S{(uint32_t*)w(srcs->doc_srcs), (uint32_t*)w(srcs->src_actor), (uint64_t*)w(srcs->vv),
                 (uint32_t*)w(srcs->entry_off), (uint64_t*)w(srcs->keys), (uint32_t*)w(srcs->actors),
                 (uint64_t*)w(srcs->counters), (uint32_t*)w(srcs->tomb_off), (uint64_t*)w(srcs->tkeys),
                 (uint32_t*)w(srcs->tactors), (uint64_t*)w(srcs->tcounters)};
    return hip_err(launch_gen_replicas(seed, n_docs, replicas, entries, view(dst), S, (hipStream_t)stream));
}

int crdt_gen_zipf_sizes(uint64_t seed, uint32_t n_docs, uint32_t* sizes) {
    if (n_docs && !sizes) return CRDT_E_INVALID;
    for (uint32_t d = 0; d < n_docs; ++d) sizes[d] = host_zipf_doc_size(seed, d);
    return CRDT_OK;
}

int crdt_gen_zipf_async(crdt_ctx* ctx, uint64_t seed, uint32_t n_docs, const uint32_t* offsets,
                        const crdt_awset_out* a, const crdt_awset_out* b, void* stream) {
    if (!ctx || !offsets || !out_ptrs_ok(a) || !out_ptrs_ok(b) || n_docs >= (1u << 24)) return CRDT_E_INVALID;
    int rc = set_device(ctx);
    if (rc != CRDT_OK) return rc;
    return hip_err(launch_gen_zipf(seed, n_docs, offsets, view(a), view(b), (hipStream_t)stream));
}

int crdt_bw_probe(crdt_ctx* ctx, int kind, const void* a, void* b, size_t bytes, int reps, double* gbs) {
    if (!ctx || !gbs || kind < CRDT_PROBE_READ || kind > CRDT_PROBE_MIX_PLAIN || reps < 1 || bytes < 16 || !b ||
        (kind != CRDT_PROBE_WRITE && kind != CRDT_PROBE_WRITE_PLAIN && !a))
        return CRDT_E_INVALID;
    int rc = set_device(ctx);
    if (rc != CRDT_OK) return rc;
    hipStream_t s = ctx->stream;
    bool cap = false;
    if ((rc = enter(ctx, s, cap)) != CRDT_OK) return rc;
    if (cap) return CRDT_E_INVALID;
    const size_t n16 = bytes / 16;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    rc = hip_err(hipEventCreate(&e0));
    if (rc == CRDT_OK) rc = hip_err(hipEventCreate(&e1));
    // one untimed launch (first touch, clocks up), then reps timed back to back
    if (rc == CRDT_OK) rc = hip_err(launch_probe(kind, a, b, n16, (uint32_t)ctx->n_cu, ctx->probe_blocks_per_cu, ctx->probe_slab, s));
    if (rc == CRDT_OK) rc = hip_err(hipEventRecord(e0, s));
    for (int r = 0; r < reps && rc == CRDT_OK; ++r)
        rc = hip_err(launch_probe(kind, a, b, n16, (uint32_t)ctx->n_cu, ctx->probe_blocks_per_cu, ctx->probe_slab, s));
    if (rc == CRDT_OK) rc = hip_err(hipEventRecord(e1, s));
    if (rc == CRDT_OK) rc = hip_err(hipEventSynchronize(e1));
    float ms = 0.f;
    if (rc == CRDT_OK) rc = hip_err(hipEventElapsedTime(&ms, e0, e1));
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (rc == CRDT_OK) {
        const bool mix = kind == CRDT_PROBE_MIX || kind == CRDT_PROBE_MIX_PLAIN;
        const double moved = mix ? (double)(n16 / 4) * 16.0 * 7.0
                                 : (double)n16 * 16.0 * ((kind == CRDT_PROBE_COPY || kind == CRDT_PROBE_COPY_PLAIN) ? 2.0 : 1.0);
        *gbs = ms > 0.f ? moved * reps / (ms * 1e-3) / 1e9 : 0.0;
    }
    return leave(ctx, s, cap, rc);
}

int crdt_host_alloc(size_t bytes, void** out) {
    if (!out) return CRDT_E_INVALID;
    *out = nullptr;
    if (bytes == 0) bytes = 1;
    // CRDT_HOST_MALLOC_FLAGS (diagnostics): hipHostMalloc flags instead of the default
    static const unsigned flags = [] {
        const char* e = std::getenv("CRDT_HOST_MALLOC_FLAGS");
        return e ? (unsigned)std::strtoul(e, nullptr, 0) : (unsigned)hipHostMallocDefault;
    }();
    if (hipHostMalloc(out, bytes, flags) != hipSuccess) return CRDT_E_NOMEM;
    void* dev = nullptr;
    if (hipHostGetDevicePointer(&dev, *out, 0) != hipSuccess) dev = nullptr;
    std::lock_guard<std::mutex> lk(g_host_mu);
    g_host_blocks[(uintptr_t)*out] = HostBlock{bytes, (uintptr_t)dev};
    return CRDT_OK;
}

void crdt_host_free(void* p) {
    if (p) {
        {
            std::lock_guard<std::mutex> lk(g_host_mu);
            g_host_blocks.erase((uintptr_t)p);
        }
        (void)hipHostFree(p);
    }
}

int crdt_clock_probe(crdt_ctx* ctx, double* mhz) {
    if (!ctx || !mhz) return CRDT_E_INVALID;
    int rc = set_device(ctx);
    if (rc != CRDT_OK) return rc;
    hipStream_t s = ctx->stream;
    bool cap = false;
    if ((rc = enter(ctx, s, cap)) != CRDT_OK) return rc;
    if (cap) return CRDT_E_INVALID;
    int wall_khz = 0;
    if (hipDeviceGetAttribute(&wall_khz, hipDeviceAttributeWallClockRate, ctx->device) != hipSuccess || wall_khz <= 0)
        return CRDT_E_HIP;
    uint64_t* dev = ctx->parts.as<uint64_t>();  // 3 words of the context-summary partials, free between calls
    uint64_t host[2] = {0, 0};
    rc = hip_err(launch_clock_probe(dev, (uint32_t)ctx->n_cu, s));  // warm-up: clocks ramp up
    if (rc == CRDT_OK) rc = hip_err(launch_clock_probe(dev, (uint32_t)ctx->n_cu, s));
    if (rc == CRDT_OK) rc = hip_err(hipMemcpyAsync(host, dev, sizeof(host), hipMemcpyDeviceToHost, s));
    if (rc == CRDT_OK) rc = hip_err(hipStreamSynchronize(s));
    if (rc == CRDT_OK) *mhz = host[1] ? (double)host[0] / ((double)host[1] / ((double)wall_khz * 1e3)) / 1e6 : 0.0;
    return leave(ctx, s, cap, rc);
}

/* ---------------- validation (host) ---------------- */

}  // extern "C"

// Pointers, slot bounds, live counts and (keys = true) the key order.  The
// *_batch calls check only the layout here (O(documents)) and the key order
// on the device after the upload (pack.hip, check_order_kernel), whose verdict
// the merge's first kernel reads before doing anything (Work::gate).
static int validate_batch(const crdt_awset_batch* b, bool keys) {
    if (!b || !b->offsets || b->R == 0 || b->R > CRDT_MAX_R) return CRDT_E_INVALID;
    if (b->n_docs && (!b->vv || ((b->offsets[b->n_docs] > b->offsets[0]) && (!b->keys || !b->actors || !b->counters))))
        return CRDT_E_INVALID;
    for (uint32_t d = 0; d < b->n_docs; d++) {
        const uint32_t o = b->offsets[d], e = b->offsets[d + 1];
        if (e < o) return CRDT_E_INVALID;
        const uint32_t n = b->counts ? b->counts[d] : e - o;
        if (n > e - o) return CRDT_E_CAPACITY;
        if (keys)
            for (uint32_t i = o + 1; i < o + n; i++)
                if (b->keys[i] <= b->keys[i - 1]) return CRDT_E_UNSORTED;
    }
    return CRDT_OK;
}

static int validate_src_batch(const crdt_src_batch* s, bool keys) {
    if (!src_ptrs_ok(s)) return CRDT_E_INVALID;
    const uint32_t ns = s->doc_srcs[s->n_docs];
    for (uint32_t d = 0; d < s->n_docs; d++)
        if (s->doc_srcs[d + 1] < s->doc_srcs[d]) return CRDT_E_INVALID;
    if (ns && !s->vv) return CRDT_E_INVALID;
    for (uint32_t k = 0; k < ns; k++) {
        const uint32_t o = s->entry_off[k], e = s->entry_off[k + 1];
        if (e < o) return CRDT_E_INVALID;
        if (keys)
            for (uint32_t i = o + 1; i < e; i++)
                if (s->keys[i] <= s->keys[i - 1]) return CRDT_E_UNSORTED;
        if (s->tomb_off) {
            const uint32_t to = s->tomb_off[k], te = s->tomb_off[k + 1];
            if (te < to) return CRDT_E_INVALID;
            if (keys)
                for (uint32_t i = to + 1; i < te; i++)
                    if (s->tkeys[i] <= s->tkeys[i - 1]) return CRDT_E_UNSORTED;
        }
    }
    return CRDT_OK;
}

extern "C" {

int crdt_validate_batch(const crdt_awset_batch* b) { return validate_batch(b, true); }

int crdt_validate_src_batch(const crdt_src_batch* s) { return validate_src_batch(s, true); }

int crdt_validate_tomb_batch(const crdt_tomb_batch* t, uint32_t n_docs) {
    if (!t || !t->offsets) return CRDT_E_INVALID;
    if (n_docs && t->offsets[n_docs] > t->offsets[0] && (!t->keys || !t->actors || !t->counters))
        return CRDT_E_INVALID;
    for (uint32_t d = 0; d < n_docs; d++) {
        const uint32_t o = t->offsets[d], e = t->offsets[d + 1];
        if (e < o) return CRDT_E_INVALID;
        const uint32_t n = t->counts ? t->counts[d] : e - o;
        if (n > e - o) return CRDT_E_CAPACITY;
        for (uint32_t i = o + 1; i < o + n; i++)
            if (t->keys[i] <= t->keys[i - 1]) return CRDT_E_UNSORTED;
    }
    return CRDT_OK;
}

/* ---------------- synchronous host-buffer path ---------------- */

}  // extern "C"

namespace {

// Diagnostics (CRDT_TRACE_STAGE): host time between the phases of a batch call.
struct PhaseClock {
    const char* what;
    bool on = std::getenv("CRDT_TRACE_STAGE") != nullptr;
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    explicit PhaseClock(const char* w) : what(w) {}
    void mark(const char* phase) {
        if (!on) return;
        const auto n = std::chrono::steady_clock::now();
        fprintf(stderr, "%s: %s %.3f ms\n", what, phase, std::chrono::duration<double, std::milli>(n - t).count());
        t = n;
    }
};

constexpr int kStageSlots = 48;  // ctx->stage: per-array device buffers of one call

// The device copies of a host-path call's arrays.  Input arrays that lie in one
// crdt_host_alloc block are staged by ONE copy of the span they cover: each
// runtime H2D copy call costs the host 1-7 ms before its DMA is even
// submitted, whatever its size (profiles/r05i_boundary_timeline.txt), while
// the span moves at PCIe rate.  Other arrays, and output rooms, get a buffer of
// their own.  A call runs its input staging twice: first planning (plan():
// nothing is allocated, only the span the call's arrays cover is measured),
// then for real, so the device image is the size of that span, not of the
// whole block.
struct Stager {
    crdt_ctx* ctx;
    bool planning = false;
    int next = 0;
    int rc = CRDT_OK;
    uintptr_t blk = 0;  // the host block of the call's inputs (the first one met)
    size_t blk_size = 0;
    size_t lo = SIZE_MAX, hi = 0;  // the span of it the call covers
    size_t img_lo = 0;             // block offset of the device image's first byte
    char* dimg = nullptr;
    bool flushed = false;
    template <typename T>
    T* put(const T* host, size_t n) {  // allocate + copy in (n elements)
        if (rc != CRDT_OK) return nullptr;
        static const bool trace = std::getenv("CRDT_TRACE_STAGE") != nullptr;  // diagnostics: host time per step
        static const bool span = std::getenv("CRDT_NO_SPAN_STAGING") == nullptr;
        const uintptr_t a = (uintptr_t)host;
        const size_t bytes = n * sizeof(T);
        if (planning) {
            if (span && ctx->span_staging && host && n) {
                uintptr_t b0 = 0;
                size_t sz = 0;
                if (!blk && host_block(host, b0, sz)) {
                    blk = b0;
                    blk_size = sz;
                }
                if (blk && a >= blk && a + bytes <= blk + blk_size) {
                    lo = std::min(lo, (size_t)(a - blk));
                    hi = std::max(hi, (size_t)(a - blk) + bytes);
                }
            }
            return nullptr;
        }
        if (dimg && host && n && a >= blk + img_lo && a + bytes <= blk + hi) {
            const size_t off = a - blk - img_lo;
            // staged after the span went: its own copy, into the same image
            if (flushed && hipMemcpyAsync(dimg + off, host, bytes, hipMemcpyHostToDevice, ctx->stream) != hipSuccess)
                rc = CRDT_E_HIP;
            return reinterpret_cast<T*>(dimg + off);
        }
        if (next >= kStageSlots) {
            rc = CRDT_E_INVALID;
            return nullptr;
        }
        const auto t0 = std::chrono::steady_clock::now();
        DevBuf& b = ctx->stage[next++];
        rc = b.reserve(std::max<size_t>(n, 1) * sizeof(T));
        if (rc != CRDT_OK) return nullptr;
        const auto t1 = std::chrono::steady_clock::now();
        if (host && n && hipMemcpyAsync(b.p, host, bytes, hipMemcpyHostToDevice, ctx->stream) != hipSuccess)
            rc = CRDT_E_HIP;
        if (trace) {
            const auto t2 = std::chrono::steady_clock::now();
            fprintf(stderr, "stage[%d] %zu B: reserve %.3f ms, copy call %.3f ms\n", next - 1, bytes,
                    std::chrono::duration<double, std::milli>(t1 - t0).count(),
                    std::chrono::duration<double, std::milli>(t2 - t1).count());
        }
        return b.as<T>();
    }
    template <typename T>
    T* room(size_t n) {
        return put<T>(nullptr, n);
    }
    // Run the call's input staging `f` planning, size the span's image, then run it for real.
    template <typename F>
    void plan(F&& f) {
        planning = true;
        f();
        planning = false;
        if (rc == CRDT_OK && blk && hi > lo) {
            img_lo = lo & ~(size_t)255;  // (the image keeps the block's 256-byte alignment)
            if (hi - img_lo <= ((size_t)4 << 30)) {  // (a larger span: array by array)
                rc = ctx->span_img.reserve(hi - img_lo);
                if (rc == CRDT_OK) dimg = ctx->span_img.as<char>();
            }
        }
        f();
    }
    // Copy the span of the host block that this call's arrays cover (one call).
    void flush() {
        if (rc == CRDT_OK && !flushed && dimg &&
            hipMemcpyAsync(dimg, reinterpret_cast<const char*>(blk) + img_lo, hi - img_lo, hipMemcpyHostToDevice,
                           ctx->stream) != hipSuccess)
            rc = CRDT_E_HIP;
        flushed = true;
    }
};

template <typename T>
int get(T* host, const T* dev, size_t n, hipStream_t s) {
    if (!n) return CRDT_OK;
    return hip_err(hipMemcpyAsync(host, dev, n * sizeof(T), hipMemcpyDeviceToHost, s));
}

crdt_awset_batch stage_batch(Stager& st, const crdt_awset_batch* h) {
    crdt_awset_batch d = *h;
    const size_t slots = h->offsets[h->n_docs];
    d.offsets = st.put(h->offsets, (size_t)h->n_docs + 1);
    d.counts = h->counts ? st.put(h->counts, h->n_docs) : nullptr;
    d.keys = st.put(h->keys, slots);
    d.actors = st.put(h->actors, slots);
    d.counters = st.put(h->counters, slots);
    d.vv = st.put(h->vv, (size_t)h->n_docs * h->R);
    return d;
}

crdt_awset_out stage_out(Stager& st, uint32_t n_docs, uint32_t R, size_t slots) {
    crdt_awset_out o;
    o.offsets = st.room<uint32_t>((size_t)n_docs + 1);
    o.counts = st.room<uint32_t>(n_docs);
    o.keys = st.room<uint64_t>(slots);
    o.actors = st.room<uint32_t>(slots);
    o.counters = st.room<uint64_t>(slots);
    o.vv = st.room<uint64_t>((size_t)n_docs * R);
    return o;
}

// keys = false: the key column is shared with an output fetched before (exchange)
int fetch_out(const crdt_awset_out* h, const crdt_awset_out& d, uint32_t n_docs, uint32_t R, size_t slots,
              hipStream_t s, bool keys = true) {
    int rc = get(h->offsets, d.offsets, (size_t)n_docs + 1, s);
    if (rc == CRDT_OK) rc = get(h->counts, d.counts, n_docs, s);
    if (rc == CRDT_OK && keys) rc = get(h->keys, d.keys, slots, s);
    if (rc == CRDT_OK) rc = get(h->actors, d.actors, slots, s);
    if (rc == CRDT_OK) rc = get(h->counters, d.counters, slots, s);
    if (rc == CRDT_OK) rc = get(h->vv, d.vv, (size_t)n_docs * R, s);
    return rc;
}

// The key order of a staged batch (ranges off[r] .. + counts or off[r + 1]),
// checked on the device; a violation sets kErrUnsorted in the status word, which
// closes the merge's gate (Work::gate) and reads back as CRDT_E_UNSORTED.
int check_order(crdt_ctx* ctx, std::initializer_list<OrderRanges> sets) {
    return hip_err(launch_check_order(sets.begin(), (uint32_t)sets.size(), ctx->ws.as<uint32_t>(64),
                                      (uint32_t)ctx->n_cu, ctx->stream));
}

// The merge launch of a host-path call, gated on the device by its order checks.
template <typename F>
int gated(crdt_ctx* ctx, F&& launch) {
    ctx->call_gate = true;
    const int rc = launch();
    ctx->call_gate = false;
    ctx->call_tiles = 0;
    ctx->call_small = false;
    return rc;
}

// Tiles the join of host batches a <- b launches (tile.hip: ceil((nd + ns) / T)
// per document with more than 64 live entries on a side), so the tile path
// launches exactly the passes it needs (join_common).
uint64_t host_tiles(const crdt_ctx* ctx, const crdt_awset_batch* a, const crdt_awset_batch* b) {
    const uint64_t T = tile_positions(ctx->tile_shape);
    uint64_t t = 0;
    for (uint32_t d = 0; d < a->n_docs; ++d) {
        const uint64_t nd = a->counts ? a->counts[d] : a->offsets[d + 1] - a->offsets[d];
        const uint64_t ns = b->counts ? b->counts[d] : b->offsets[d + 1] - b->offsets[d];
        if (nd > 64 || ns > 64) t += (nd + ns + T - 1) / T;
    }
    return t;
}

// Before a host-path join's launch: the exact tile count, or no large-document
// path at all when no document has one (six launches fewer; 0 tiles <=> no
// document above 64 live entries on a side, whatever the tile options).
void plan_tiles(crdt_ctx* ctx, const crdt_awset_batch* a, const crdt_awset_batch* b) {
    const uint64_t t = host_tiles(ctx, a, b);
    ctx->call_small = t == 0;
    ctx->call_tiles = std::max<uint64_t>(t, 1);
}

// The end of a host-path call: its one sync, then its status (read from the
// page-locked copy the gather kernel made when `copied`, else read back).
int finish(crdt_ctx* ctx, bool copied) {
    if (!copied || !ctx->host_status) return crdt_ctx_sync(ctx, ctx->stream);
    if (hipStreamSynchronize(ctx->stream) != hipSuccess) return CRDT_E_HIP;
    const uint32_t st = __atomic_load_n(ctx->host_status, __ATOMIC_ACQUIRE);
    return st ? crdt_ctx_sync(ctx, ctx->stream) : CRDT_OK;  // (an error: the usual read-back and reset)
}

// Download merge outputs.  Default: at their capacity offsets, as the kernels
// wrote them.  pack_batch_outputs: only the live entries, gathered on the
// device at offsets computed on the device (pack_scan_kernel) -- an output
// whose host arrays all lie in crdt_host_alloc blocks is written there by the
// gather kernel itself (no copy call, no read-back: the call's one sync is its
// last); any other is gathered on the device, and the totals of all such
// outputs come back in ONE read-back before their copies.  keys[i] = false: an
// exchange's second output sharing the first's key column.
int fetch_outputs(crdt_ctx* ctx, Stager& st, int nout, const crdt_awset_out* const* h, const crdt_awset_out* d,
                  const bool* keys, uint32_t n, uint32_t R, size_t slots, bool* status_copied) {
    *status_copied = false;
    if (!ctx->pack_outputs) {
        int rc = CRDT_OK;
        for (int i = 0; i < nout && rc == CRDT_OK; ++i) rc = fetch_out(h[i], d[i], n, R, slots, ctx->stream, keys[i]);
        return rc;
    }
    static const bool no_zc = std::getenv("CRDT_NO_ZERO_COPY") != nullptr;  // diagnostics: copies only
    uint32_t* poff[2] = {nullptr, nullptr};
    uint32_t* hoff[2] = {nullptr, nullptr};
    OutView pk[2];
    bool zc[2] = {false, false};
    for (int i = 0; i < nout; ++i) {
        poff[i] = st.room<uint32_t>((size_t)n + 1);
        const uintptr_t ho = host_dev_addr(h[i]->offsets, ((size_t)n + 1) * 4),
                        hc = host_dev_addr(h[i]->counts, (size_t)n * 4),
                        hk = keys[i] ? host_dev_addr(h[i]->keys, slots * 8) : 1,
                        ha = host_dev_addr(h[i]->actors, slots * 4), hcc = host_dev_addr(h[i]->counters, slots * 8),
                        hv = host_dev_addr(h[i]->vv, (size_t)n * R * 8);
        zc[i] = !no_zc && ho && hc && hk && ha && hcc && hv;
        if (zc[i]) {
            hoff[i] = reinterpret_cast<uint32_t*>(ho);
            pk[i] = OutView{nullptr, reinterpret_cast<uint32_t*>(hc),
                            keys[i] ? reinterpret_cast<uint64_t*>(hk) : nullptr, reinterpret_cast<uint32_t*>(ha),
                            reinterpret_cast<uint64_t*>(hcc), reinterpret_cast<uint64_t*>(hv)};
        } else {
            pk[i] = OutView{nullptr, nullptr, keys[i] ? st.room<uint64_t>(slots) : nullptr, st.room<uint32_t>(slots),
                            st.room<uint64_t>(slots), nullptr};
        }
    }
    if (st.rc != CRDT_OK) return st.rc;
    const OutView in[2] = {view(&d[0]), nout > 1 ? view(&d[1]) : OutView{}};
    int rc = hip_err(launch_pack((uint32_t)nout, in, poff, hoff, pk, n, R, ctx->ws.as<uint32_t>(64), ctx->host_status,
                                 (uint32_t)ctx->n_cu, ctx->stream));
    *status_copied = rc == CRDT_OK && ctx->host_status != nullptr;
    if (rc != CRDT_OK || (zc[0] && (nout < 2 || zc[1]))) return rc;
    uint32_t tot[2] = {0, 0};
    for (int i = 0; i < nout && rc == CRDT_OK; ++i)
        if (!zc[i]) rc = get(&tot[i], poff[i] + n, 1, ctx->stream);
    if (rc == CRDT_OK && hipStreamSynchronize(ctx->stream) != hipSuccess) rc = CRDT_E_HIP;
    for (int i = 0; i < nout && rc == CRDT_OK; ++i) {
        if (zc[i]) continue;
        if (tot[i] > slots) return CRDT_E_CAPACITY;  // (the scan clamps to capacity: never)
        rc = get(h[i]->offsets, poff[i], (size_t)n + 1, ctx->stream);
        if (rc == CRDT_OK) rc = get(h[i]->counts, d[i].counts, n, ctx->stream);
        if (rc == CRDT_OK && keys[i]) rc = get(h[i]->keys, pk[i].keys, tot[i], ctx->stream);
        if (rc == CRDT_OK) rc = get(h[i]->actors, pk[i].actors, tot[i], ctx->stream);
        if (rc == CRDT_OK) rc = get(h[i]->counters, pk[i].counters, tot[i], ctx->stream);
        if (rc == CRDT_OK) rc = get(h[i]->vv, d[i].vv, (size_t)n * R, ctx->stream);
    }
    return rc;
}

}  // namespace

extern "C" {

int crdt_awset_sort_batch(crdt_ctx* ctx, const crdt_awset_batch* in, const crdt_awset_out* out) {
    if (!ctx || !in || !in->offsets || !out_ptrs_ok(out) || in->R == 0 || in->R > CRDT_MAX_R) return CRDT_E_INVALID;
    const uint32_t n = in->n_docs;
    const size_t slots = in->offsets[n];
    int rc = set_device(ctx);
    if (rc != CRDT_OK) return rc;
    Stager st{ctx};
    crdt_awset_batch di{};
    st.plan([&] { di = stage_batch(st, in); });
    crdt_awset_out dout = stage_out(st, n, in->R, slots);
    st.flush();  // the inputs' span, if they lie in one crdt_host_alloc block
    if (st.rc != CRDT_OK) return st.rc;
    rc = crdt_awset_sort_async(ctx, &di, (uint32_t)slots, &dout, ctx->stream);
    if (rc == CRDT_OK) rc = fetch_out(out, dout, n, in->R, slots, ctx->stream);
    const int sync = crdt_ctx_sync(ctx, ctx->stream);
    return rc != CRDT_OK ? rc : sync;
}

int crdt_awset_apply_batch(crdt_ctx* ctx, const crdt_awset_batch* state, const crdt_tomb_batch* tombs,
                           const crdt_op_batch* ops, const crdt_awset_out* out, const crdt_tomb_out* tomb_out) {
    if (!ctx || !ops || !ops->op_off || !ops->doc_actor || !out_ptrs_ok(out)) return CRDT_E_INVALID;
    int rc = crdt_validate_batch(state);
    if (rc != CRDT_OK) return rc;
    if (ops->n_docs != state->n_docs) return CRDT_E_INVALID;
    const uint32_t n = state->n_docs;
    if (tombs && (rc = crdt_validate_tomb_batch(tombs, n)) != CRDT_OK) return rc;
    const size_t nops = ops->op_off[n];
    if (nops && (!ops->kind || !ops->keys)) return CRDT_E_INVALID;
    const uint64_t slots = (uint64_t)state->offsets[n] + nops;
    const uint64_t tin = tombs ? tombs->offsets[n] : 0;
    if (slots >= (1ull << 32) || tin + nops >= (1ull << 32)) return CRDT_E_INVALID;
    if ((rc = set_device(ctx)) != CRDT_OK) return rc;
    Stager st{ctx};
    crdt_awset_batch ds{};
    crdt_op_batch dops = *ops;
    crdt_tomb_batch dt{};
    st.plan([&] {
        ds = stage_batch(st, state);
        dops.op_off = st.put(ops->op_off, (size_t)n + 1);
        dops.kind = st.put(ops->kind, nops);
        dops.keys = st.put(ops->keys, nops);
        dops.doc_actor = st.put(ops->doc_actor, n);
        if (tombs) {
            dt.offsets = st.put(tombs->offsets, (size_t)n + 1);
            dt.counts = tombs->counts ? st.put(tombs->counts, n) : nullptr;
            dt.keys = st.put(tombs->keys, tin);
            dt.actors = st.put(tombs->actors, tin);
            dt.counters = st.put(tombs->counters, tin);
        }
    });
    crdt_awset_out dout = stage_out(st, n, state->R, slots);
    crdt_tomb_out dto{};
    if (tomb_out) {
        dto.offsets = st.room<uint32_t>((size_t)n + 1);
        dto.counts = st.room<uint32_t>(n);
        dto.keys = st.room<uint64_t>(tin + nops);
        dto.actors = st.room<uint32_t>(tin + nops);
        dto.counters = st.room<uint64_t>(tin + nops);
    }
    st.flush();  // the inputs' span, if they lie in one crdt_host_alloc block
    if (st.rc != CRDT_OK) return st.rc;
    rc = crdt_awset_apply_async(ctx, &ds, tombs ? &dt : nullptr, &dops, &dout, tomb_out ? &dto : nullptr,
                                ctx->stream);
    if (rc == CRDT_OK) rc = fetch_out(out, dout, n, state->R, slots, ctx->stream);
    if (rc == CRDT_OK && tomb_out) {
        rc = get(tomb_out->offsets, dto.offsets, (size_t)n + 1, ctx->stream);
        if (rc == CRDT_OK) rc = get(tomb_out->counts, dto.counts, n, ctx->stream);
        if (rc == CRDT_OK) rc = get(tomb_out->keys, dto.keys, tin + nops, ctx->stream);
        if (rc == CRDT_OK) rc = get(tomb_out->actors, dto.actors, tin + nops, ctx->stream);
        if (rc == CRDT_OK) rc = get(tomb_out->counters, dto.counters, tin + nops, ctx->stream);
    }
    const int sync = crdt_ctx_sync(ctx, ctx->stream);
    return rc != CRDT_OK ? rc : sync;
}

// The merge calls below make one host sync each (their last): the inputs go up
// (one copy of their span when they lie in one crdt_host_alloc block), the key
// order is checked on the device, the merge's first kernel reads that verdict
// (a batch out of order reaches no merge, Work::gate), and the outputs come
// back (fetch_outputs: with pack_batch_outputs into page-locked outputs, by
// the gather kernel itself).
int crdt_awset_join_batch(crdt_ctx* ctx, const crdt_awset_batch* dst, const crdt_awset_batch* src,
                          const crdt_awset_out* out) {
    if (!ctx || !out_ptrs_ok(out)) return CRDT_E_INVALID;
    int rc = validate_batch(dst, false);
    if (rc == CRDT_OK) rc = validate_batch(src, false);
    if (rc != CRDT_OK) return rc;
    if (dst->n_docs != src->n_docs || dst->R != src->R) return CRDT_E_INVALID;
    if ((uint64_t)dst->offsets[dst->n_docs] + src->offsets[src->n_docs] >= (1ull << 32)) return CRDT_E_INVALID;
    if ((rc = set_device(ctx)) != CRDT_OK) return rc;
    Stager st{ctx};
    crdt_awset_batch dd{}, ds{};
    st.plan([&] {
        dd = stage_batch(st, dst);
        ds = stage_batch(st, src);
    });
    const size_t slots = (size_t)dst->offsets[dst->n_docs] + src->offsets[src->n_docs];
    crdt_awset_out dout = stage_out(st, dst->n_docs, dst->R, slots);
    st.flush();  // the inputs' span, if they lie in one crdt_host_alloc block
    if (st.rc != CRDT_OK) return st.rc;
    rc = check_order(ctx, {{dd.offsets, dd.counts, dd.n_docs, dd.keys}, {ds.offsets, ds.counts, ds.n_docs, ds.keys}});
    plan_tiles(ctx, dst, src);
    if (rc == CRDT_OK) rc = gated(ctx, [&] { return crdt_awset_join_async(ctx, &dd, &ds, &dout, ctx->stream); });
    const crdt_awset_out* hs[1] = {out};
    const bool keys[1] = {true};
    bool copied = false;
    if (rc == CRDT_OK) rc = fetch_outputs(ctx, st, 1, hs, &dout, keys, dst->n_docs, dst->R, slots, &copied);
    ctx->call_tiles = 0;
    ctx->call_small = false;
    const int sync = finish(ctx, copied);
    return rc != CRDT_OK ? rc : sync;
}

int crdt_awset_exchange_batch(crdt_ctx* ctx, const crdt_awset_batch* a, const crdt_awset_batch* b,
                              const crdt_awset_out* out_ab, const crdt_awset_out* out_ba) {
    if (!ctx || !out_ptrs_ok(out_ab) || !out_ptrs_ok(out_ba)) return CRDT_E_INVALID;
    int rc = validate_batch(a, false);
    if (rc == CRDT_OK) rc = validate_batch(b, false);
    if (rc != CRDT_OK) return rc;
    if (a->n_docs != b->n_docs || a->R != b->R) return CRDT_E_INVALID;
    if ((uint64_t)a->offsets[a->n_docs] + b->offsets[b->n_docs] >= (1ull << 32)) return CRDT_E_INVALID;
    if ((rc = set_device(ctx)) != CRDT_OK) return rc;
    PhaseClock pc("exchange_batch");
    Stager st{ctx};
    crdt_awset_batch da{}, db{};
    st.plan([&] {
        da = stage_batch(st, a);
        db = stage_batch(st, b);
    });
    const size_t slots = (size_t)a->offsets[a->n_docs] + b->offsets[b->n_docs];
    crdt_awset_out o[2] = {stage_out(st, a->n_docs, a->R, slots), stage_out(st, a->n_docs, a->R, slots)};
    st.flush();  // the inputs' span, if they lie in one crdt_host_alloc block
    if (st.rc != CRDT_OK) return st.rc;
    // host outputs sharing one key column: one device column, written and fetched once
    const bool share = out_ab->keys == out_ba->keys;
    if (share) o[1].keys = o[0].keys;
    pc.mark("stage issued");
    rc = check_order(ctx, {{da.offsets, da.counts, da.n_docs, da.keys}, {db.offsets, db.counts, db.n_docs, db.keys}});
    plan_tiles(ctx, a, b);
    if (rc == CRDT_OK) rc = gated(ctx, [&] { return crdt_awset_exchange_async(ctx, &da, &db, &o[0], &o[1], ctx->stream); });
    pc.mark("order checks + kernels issued");
    const crdt_awset_out* hs[2] = {out_ab, out_ba};
    const bool keys[2] = {true, !share};
    bool copied = false;
    if (rc == CRDT_OK) rc = fetch_outputs(ctx, st, 2, hs, o, keys, a->n_docs, a->R, slots, &copied);
    ctx->call_tiles = 0;
    ctx->call_small = false;
    pc.mark("fetches issued");
    const int sync = finish(ctx, copied);
    pc.mark("synced");
    return rc != CRDT_OK ? rc : sync;
}

int crdt_awset_fold_batch(crdt_ctx* ctx, int mode, const crdt_awset_batch* dst, const crdt_src_batch* srcs,
                          const crdt_awset_out* out) {
    if (!ctx || !out_ptrs_ok(out)) return CRDT_E_INVALID;
    int rc = validate_batch(dst, false);
    if (rc == CRDT_OK) rc = validate_src_batch(srcs, false);
    if (rc != CRDT_OK) return rc;
    if (dst->n_docs != srcs->n_docs || dst->R != srcs->R) return CRDT_E_INVALID;
    const uint32_t ns = srcs->doc_srcs[srcs->n_docs];
    const uint64_t total = (uint64_t)dst->offsets[dst->n_docs] + srcs->entry_off[ns];
    if (total >= (1ull << 32)) return CRDT_E_INVALID;
    if ((rc = set_device(ctx)) != CRDT_OK) return rc;
    if ((rc = reserve_scratch(ctx, total)) != CRDT_OK) return rc;
    Stager st{ctx};
    crdt_awset_batch dd{};
    crdt_src_batch ds = *srcs;
    const size_t ne = srcs->entry_off[ns];
    const size_t nt = srcs->tomb_off ? srcs->tomb_off[ns] : 0;
    st.plan([&] {
        dd = stage_batch(st, dst);
        ds.doc_srcs = st.put(srcs->doc_srcs, (size_t)srcs->n_docs + 1);
        ds.src_actor = st.put(srcs->src_actor, ns);
        ds.vv = st.put(srcs->vv, (size_t)ns * srcs->R);
        ds.entry_off = st.put(srcs->entry_off, (size_t)ns + 1);
        ds.keys = st.put(srcs->keys, ne);
        ds.actors = st.put(srcs->actors, ne);
        ds.counters = st.put(srcs->counters, ne);
        if (srcs->tomb_off) {
            ds.tomb_off = st.put(srcs->tomb_off, (size_t)ns + 1);
            ds.tkeys = st.put(srcs->tkeys, nt);
            ds.tactors = st.put(srcs->tactors, nt);
            ds.tcounters = st.put(srcs->tcounters, nt);
        }
    });
    crdt_awset_out dout = stage_out(st, dst->n_docs, dst->R, total);
    st.flush();  // the inputs' span, if they lie in one crdt_host_alloc block
    if (st.rc != CRDT_OK) return st.rc;
    rc = srcs->tomb_off ? check_order(ctx, {{dd.offsets, dd.counts, dd.n_docs, dd.keys}, {ds.entry_off, nullptr, ns, ds.keys},
                                            {ds.tomb_off, nullptr, ns, ds.tkeys}})
                        : check_order(ctx, {{dd.offsets, dd.counts, dd.n_docs, dd.keys}, {ds.entry_off, nullptr, ns, ds.keys}});
    if (rc == CRDT_OK) rc = gated(ctx, [&] { return crdt_awset_fold_async(ctx, mode, &dd, &ds, &dout, ctx->stream); });
    const crdt_awset_out* hs[1] = {out};
    const bool keys[1] = {true};
    bool copied = false;
    if (rc == CRDT_OK) rc = fetch_outputs(ctx, st, 1, hs, &dout, keys, dst->n_docs, dst->R, total, &copied);
    const int sync = finish(ctx, copied);
    return rc != CRDT_OK ? rc : sync;
}

}  // extern "C"
