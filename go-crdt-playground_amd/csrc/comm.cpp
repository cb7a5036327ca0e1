// Global causal context across GPUs over RCCL.
//
// Documents shard over the GPUs with no data-path exchange; the one
// collective is the causal-context summary: every GPU reduces its output
// version vectors to R u64 (crdt_causal_context_async) and the GPUs combine
// them with ncclAllReduce(ncclUint64, ncclMax) over xGMI.  The reference has
// no such object (it is single-process Go); its counterpart is the CPU max
// over every merged VersionVector (crdt-misc.go:43-55 applied across docs).
//
// RCCL is bound at run time (dlopen) rather than linked: under PyTorch the
// already-loaded RCCL (torch/lib/librccl.so) is reused, so one process never
// maps two copies; elsewhere the system librccl.so.1 is loaded.  A host
// without RCCL still loads libcrdtgpu.so; only these calls fail (CRDT_E_RCCL).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <mutex>
#include <vector>

#include "../../include/crdtgpu.h"

// internal accessors (api.cpp)
int crdt_internal_device(crdt_ctx* ctx);
hipStream_t crdt_internal_stream(crdt_ctx* ctx);
int crdt_internal_order(crdt_ctx* ctx, hipStream_t s);  // s waits for the ctx's last call
void** crdt_internal_comm(crdt_ctx* ctx);
void** crdt_internal_comm_group(crdt_ctx* ctx);

namespace {

struct Rccl {
    bool tried = false;
    void* h = nullptr;
    ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
    ncclResult_t (*init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*init_all)(ncclComm_t*, int, const int*) = nullptr;
    ncclResult_t (*destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*abort)(ncclComm_t) = nullptr;
    ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                               hipStream_t) = nullptr;
    ncclResult_t (*group_start)() = nullptr;
    ncclResult_t (*group_end)() = nullptr;
};

std::mutex g_mu;
Rccl g_rccl;

template <typename F>
bool bind(void* h, const char* name, F& f) {
    f = reinterpret_cast<F>(dlsym(h, name));
    return f != nullptr;
}

const Rccl* rccl() {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_rccl.tried) return g_rccl.h ? &g_rccl : nullptr;
    g_rccl.tried = true;
    void* h = dlopen("librccl.so", RTLD_NOW | RTLD_NOLOAD);  // PyTorch's copy, if mapped
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) return nullptr;
    Rccl r;
    r.h = h;
    r.tried = true;
    if (!bind(h, "ncclGetUniqueId", r.get_unique_id) || !bind(h, "ncclCommInitRank", r.init_rank) ||
        !bind(h, "ncclCommInitAll", r.init_all) || !bind(h, "ncclCommDestroy", r.destroy) ||
        !bind(h, "ncclCommAbort", r.abort) ||
        !bind(h, "ncclAllReduce", r.all_reduce) || !bind(h, "ncclGroupStart", r.group_start) ||
        !bind(h, "ncclGroupEnd", r.group_end))
        return nullptr;
    g_rccl = r;
    return &g_rccl;
}

// A single-process group of contexts sharing communicators (crdt_global_context_allreduce).
struct Group {
    std::vector<crdt_ctx*> members;
};

void drop_comm(const Rccl* r, crdt_ctx* c, bool abort = false) {
    void** comm = crdt_internal_comm(c);
    if (*comm && r) (void)(abort ? r->abort : r->destroy)((ncclComm_t)*comm);
    *comm = nullptr;
    void** grp = crdt_internal_comm_group(c);
    if (*grp) {
        Group* g = (Group*)*grp;
        for (auto*& m : g->members)
            if (m == c) m = nullptr;
        bool empty = true;
        for (auto* m : g->members) empty = empty && m == nullptr;
        if (empty) delete g;
        *grp = nullptr;
    }
}

// Restores the calling thread's current HIP device on every return path.
struct DeviceGuard {
    int dev = -1;
    DeviceGuard() {
        if (hipGetDevice(&dev) != hipSuccess) dev = -1;
    }
    ~DeviceGuard() {
        if (dev >= 0) (void)hipSetDevice(dev);
    }
};

}  // namespace

// Called by crdt_ctx_destroy.
void crdt_internal_comm_release(crdt_ctx* ctx) {
    if (!*crdt_internal_comm(ctx) && !*crdt_internal_comm_group(ctx)) return;
    drop_comm(g_rccl.h ? &g_rccl : nullptr, ctx);
}

extern "C" {

int crdt_comm_unique_id(uint8_t* id) {
    if (!id) return CRDT_E_INVALID;
    const Rccl* r = rccl();
    if (!r) return CRDT_E_RCCL;
    ncclUniqueId u;
    if (r->get_unique_id(&u) != ncclSuccess) return CRDT_E_RCCL;
    static_assert(sizeof(u) == CRDT_COMM_ID_BYTES, "ncclUniqueId size");
    memcpy(id, &u, sizeof(u));
    return CRDT_OK;
}

int crdt_comm_init(crdt_ctx* ctx, int n_ranks, int rank, const uint8_t* id) {
    if (!ctx || !id || n_ranks < 1 || rank < 0 || rank >= n_ranks) return CRDT_E_INVALID;
    DeviceGuard keep;
    const Rccl* r = rccl();
    if (!r) return CRDT_E_RCCL;
    if (hipSetDevice(crdt_internal_device(ctx)) != hipSuccess) return CRDT_E_HIP;
    drop_comm(r, ctx);
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    ncclComm_t c = nullptr;
    if (r->init_rank(&c, n_ranks, u, rank) != ncclSuccess) return CRDT_E_RCCL;
    *crdt_internal_comm(ctx) = c;
    return CRDT_OK;
}

int crdt_context_allreduce_async(crdt_ctx* ctx, uint64_t* vv_R, uint32_t R, void* stream) {
    if (!ctx || !vv_R || R == 0 || R > CRDT_MAX_R) return CRDT_E_INVALID;
    const Rccl* r = rccl();
    if (!r) return CRDT_E_RCCL;
    ncclComm_t c = (ncclComm_t)*crdt_internal_comm(ctx);
    if (!c) return CRDT_E_INVALID;  // crdt_comm_init first
    DeviceGuard keep;
    if (hipSetDevice(crdt_internal_device(ctx)) != hipSuccess) return CRDT_E_HIP;
    hipStream_t s = (hipStream_t)stream;
    int rc = crdt_internal_order(ctx, s);
    if (rc != CRDT_OK) return rc;
    return r->all_reduce(vv_R, vv_R, R, ncclUint64, ncclMax, c, s) == ncclSuccess ? CRDT_OK : CRDT_E_RCCL;
}

int crdt_global_context_allreduce(crdt_ctx* const* per_gpu, int n_gpus, uint64_t* const* vv_R, uint32_t R,
                                  uint64_t* out_vv_R) {
    if (!per_gpu || !vv_R || n_gpus < 1 || R == 0 || R > CRDT_MAX_R) return CRDT_E_INVALID;
    DeviceGuard keep;  // the caller's current device is unchanged on return
    std::vector<int> devs(n_gpus);
    for (int i = 0; i < n_gpus; ++i) {
        if (!per_gpu[i] || !vv_R[i]) return CRDT_E_INVALID;
        devs[i] = crdt_internal_device(per_gpu[i]);
        for (int j = 0; j < i; ++j)
            if (devs[j] == devs[i] || per_gpu[j] == per_gpu[i]) return CRDT_E_INVALID;  // one context per GPU
    }
    const Rccl* r = rccl();
    if (!r) return CRDT_E_RCCL;
    // communicators: reuse the group these contexts already form, else build one
    Group* g = (Group*)*crdt_internal_comm_group(per_gpu[0]);
    bool same = g && (int)g->members.size() == n_gpus;
    for (int i = 0; same && i < n_gpus; ++i) same = g->members[i] == per_gpu[i];
    if (!same) {
        for (int i = 0; i < n_gpus; ++i) drop_comm(r, per_gpu[i]);
        std::vector<ncclComm_t> comms(n_gpus, nullptr);
        if (r->init_all(comms.data(), n_gpus, devs.data()) != ncclSuccess) return CRDT_E_RCCL;
        g = new Group{std::vector<crdt_ctx*>(per_gpu, per_gpu + n_gpus)};
        for (int i = 0; i < n_gpus; ++i) {
            *crdt_internal_comm(per_gpu[i]) = comms[i];
            *crdt_internal_comm_group(per_gpu[i]) = g;
        }
    }
    for (int i = 0; i < n_gpus; ++i) {
        if (hipSetDevice(devs[i]) != hipSuccess) return CRDT_E_HIP;
        int rc = crdt_internal_order(per_gpu[i], crdt_internal_stream(per_gpu[i]));
        if (rc != CRDT_OK) return rc;
    }
    // A group that was started must be ended even when an enqueue failed (an
    // open group would swallow the caller's next RCCL calls); after the first
    // failure no further all-reduce is enqueued. A partly issued collective
    // would leave the enqueued ranks' streams waiting for the missing ones, so
    // the communicators are then aborted (their pending work is dropped) and
    // the group dissolved: the next call builds fresh communicators.
    if (r->group_start() != ncclSuccess) return CRDT_E_RCCL;
    bool ok = true;
    for (int i = 0; i < n_gpus; ++i) {
        if (hipSetDevice(devs[i]) != hipSuccess) ok = false;
        ok = ok && r->all_reduce(vv_R[i], vv_R[i], R, ncclUint64, ncclMax, (ncclComm_t)*crdt_internal_comm(per_gpu[i]),
                                 crdt_internal_stream(per_gpu[i])) == ncclSuccess;
    }
    const bool ended = r->group_end() == ncclSuccess;
    if (!ok || !ended) {
        for (int i = 0; i < n_gpus; ++i) drop_comm(r, per_gpu[i], true);
        return CRDT_E_RCCL;
    }
    for (int i = 0; i < n_gpus; ++i) {
        if (hipSetDevice(devs[i]) != hipSuccess) return CRDT_E_HIP;
        if (hipStreamSynchronize(crdt_internal_stream(per_gpu[i])) != hipSuccess) return CRDT_E_HIP;
    }
    if (out_vv_R) {
        if (hipSetDevice(devs[0]) != hipSuccess) return CRDT_E_HIP;
        if (hipMemcpy(out_vv_R, vv_R[0], R * sizeof(uint64_t), hipMemcpyDeviceToHost) != hipSuccess)
            return CRDT_E_HIP;
    }
    return CRDT_OK;
}

}  // extern "C"
