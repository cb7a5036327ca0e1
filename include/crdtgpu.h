/*
 * crdtgpu.h -- C ABI of the MI355X batched AWSet merge engine.
 *
 * The reference (rsms/go-crdt-playground, package crdt) has no FFI: its merge
 * path is a Go method set called in-process.  Each entry point below replaces
 * one of those methods, applied to a whole batch of independent documents at
 * once; a cgo package with the reference's types calls them.
 *
 *   crdt_awset_join_async / crdt_awset_join_batch
 *       replace (*AWSet).Merge / merge                 awset.go:103-161
 *   crdt_awset_fold_async / crdt_awset_fold_batch, mode CRDT_FOLD_AWSET
 *       replace an ordered sequence of (*AWSet).Merge  awset.go:103-161
 *   crdt_awset_fold_async / crdt_awset_fold_batch, mode CRDT_FOLD_DELTA
 *       replace (*AWSetDelta).Merge with MakeDeltaMergeData, deltaMerge and
 *       the (no-op) gcDeleted                          awset-delta_test.go:51-166
 *   crdt_vv_max_async
 *       replaces (*VersionVector).Merge                crdt-misc.go:43-55
 *   crdt_causal_context_async
 *       the elementwise max over many version vectors (no reference
 *       counterpart: the per-GPU summary reduced across GPUs by RCCL)
 *   crdt_awset_apply_async / crdt_awset_apply_batch
 *       replace the state producers (*AWSet).Add / Del  awset.go:89-101
 *       and (*AWSetDelta).Del                          awset-delta_test.go:14-33
 *       applied as ordered op lists to a batch of documents
 *   crdt_global_context_allreduce / crdt_context_allreduce_async
 *       that summary combined across GPUs: RCCL all-reduce(max, u64)
 *       (the reference's counterpart is the CPU max over
 *       every merged VersionVector, crdt-misc.go:43-55)
 *
 * HasDot (crdt-misc.go:28-34) and Counter (:36-41) run inside the kernels.
 *
 * Encoding (SoA, all little-endian):
 *   entry  = key id u64 + dot actor u32 + dot counter u64   (20 B)
 *   VV     = R x u64 per state, R identical for every state of a call
 *   doc d of a batch owns the slots [offsets[d], offsets[d+1]); its live
 *   entries are the first counts[d] of them (counts == NULL: all slots live),
 *   keys strictly ascending.  Strings are interned to key ids by the caller.
 *
 * HasDot / Counter with actor == R index one past the reference's slice and
 * panic in Go; here the call returns CRDT_E_ACTOR_RANGE instead (outputs then
 * undefined).  actor > R is "never seen" (false / 0), as in the reference.
 *
 * Output: doc d of a join is written at out offset dst.offsets[d] +
 * src.offsets[d] (capacity = both inputs' capacities), its live count to
 * out->counts[d], its slot bounds to out->offsets[d] (n_docs+1 values) and its
 * VV to out->vv.  Entries come out sorted by key.  No scan over documents is
 * needed, so one launch finishes the batch, and the output is directly a valid
 * input batch for the next merge.  A document's slots past its live count
 * (counts[d] .. its capacity) are unspecified and may be written (the joins'
 * whole-sector stores pad them with zeros); slots of other documents never are.
 *
 * Threading: one crdt_ctx per host thread; *_async calls are ordered on the
 * given HIP stream; crdt_ctx_sync returns device-side errors.  Device buffers
 * passed to *_async are caller-owned (device-resident, e.g. torch tensors).
 * The *_batch calls take host buffers and are synchronous.
 *
 * Streams and graphs: the calls of one context share its workspace (worklist,
 * counters, fold scratch, status word).  A call issued on a different stream
 * than the previous call of the same context first waits (hipStreamWaitEvent)
 * for that call's launches, so calls of one context never overlap on the
 * device, whatever streams they use; crdt_ctx_sync also waits for them.  A
 * call made while its stream is capturing a HIP graph records no such wait
 * (the capture is ordered by its caller) and never allocates: if the
 * workspace would have to grow it returns CRDT_E_WORKSPACE (reserve first,
 * or run the call once eagerly).  Buffers the workspace outgrows are kept
 * until crdt_ctx_destroy, so graphs captured earlier stay valid.
 */
#ifndef CRDTGPU_H
#define CRDTGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CRDTGPU_ABI_VERSION 1

/* status codes */
#define CRDT_OK 0
#define CRDT_E_INVALID (-1)     /* null pointer, R==0 or R>CRDT_MAX_R, bad sizes       */
#define CRDT_E_ACTOR_RANGE (-2) /* HasDot/Counter at actor == R: reference panics     */
#define CRDT_E_UNSORTED (-3)    /* keys of a doc not strictly ascending (validation)  */
#define CRDT_E_CAPACITY (-4)    /* a doc's live count exceeds its slots               */
#define CRDT_E_HIP (-5)         /* HIP runtime error                                   */
#define CRDT_E_NOMEM (-6)       /* device allocation failed                            */
#define CRDT_E_WORKSPACE (-7)   /* fold block path needs crdt_ctx_reserve(max_fold_slots) */
#define CRDT_E_RCCL (-8)        /* RCCL not loadable, or a collective failed          */
#define CRDT_E_DUP_KEY (-9)     /* a key appears twice in one document (ingest sort)  */

#define CRDT_MAX_R 64 /* version-vector length limit (one wave lane per actor) */

/* fold modes */
#define CRDT_FOLD_AWSET 0 /* each step = (*AWSet).Merge: tombstones ignored       */
#define CRDT_FOLD_DELTA 1 /* each step = (*AWSetDelta).Merge                       */

typedef struct crdt_ctx crdt_ctx;

/* A batch of AWSet states (read-only view). */
typedef struct {
    uint32_t n_docs;
    uint32_t R;
    const uint32_t* offsets;  /* [n_docs+1] slot bounds                          */
    const uint32_t* counts;   /* [n_docs] live entries, or NULL = all slots live */
    const uint64_t* keys;     /* [offsets[n_docs]]                              */
    const uint32_t* actors;   /* [offsets[n_docs]]                              */
    const uint64_t* counters; /* [offsets[n_docs]]                              */
    const uint64_t* vv;       /* [n_docs*R]                                     */
} crdt_awset_batch;

/* Output of a join or fold (written). */
typedef struct {
    uint32_t* offsets;  /* [n_docs+1]                          */
    uint32_t* counts;   /* [n_docs]                            */
    uint64_t* keys;     /* capacity = Σ input slots            */
    uint32_t* actors;
    uint64_t* counters;
    uint64_t* vv;       /* [n_docs*R]                          */
} crdt_awset_out;

/*
 * Ordered source states folded into each dst doc (AWSet or AWSetDelta
 * states).  Doc d receives sources [doc_srcs[d], doc_srcs[d+1]) in that order.
 * Source s: replica actor src_actor[s] (AWSetDelta.Actor, read by the path
 * select of awset-delta_test.go:53), VV vv[s*R..], entries
 * [entry_off[s], entry_off[s+1]) and tombstones (AWSetDelta.Deleted)
 * [tomb_off[s], tomb_off[s+1]), each sorted by key.  tomb_off may be NULL.
 * Fold output capacity of doc d: dst slots + Σ its sources' entry slots, at
 * offset dst.offsets[d] + entry_off[doc_srcs[d]].
 */
typedef struct {
    uint32_t n_docs;
    uint32_t R;
    const uint32_t* doc_srcs;   /* [n_docs+1]  */
    const uint32_t* src_actor;  /* [n_srcs]    */
    const uint64_t* vv;         /* [n_srcs*R]  */
    const uint32_t* entry_off;  /* [n_srcs+1]  */
    const uint64_t* keys;
    const uint32_t* actors;
    const uint64_t* counters;
    const uint32_t* tomb_off;   /* [n_srcs+1] or NULL */
    const uint64_t* tkeys;
    const uint32_t* tactors;
    const uint64_t* tcounters;
} crdt_src_batch;

/* ---- context ---------------------------------------------------------- */
int crdt_ctx_create(int device, crdt_ctx** out);
void crdt_ctx_destroy(crdt_ctx* ctx);
/* Pre-size workspaces so that *_async calls never allocate (graph capture). */
int crdt_ctx_reserve(crdt_ctx* ctx, uint32_t max_docs, uint64_t max_fold_slots);
/* Promise that every doc of later joins holds <= max_entries live entries per
 * side (0xFFFFFFFF = no promise, the default).  At <= 64 the large-document
 * path is not launched; a doc that breaks the promise makes crdt_ctx_sync
 * return CRDT_E_INVALID. */
int crdt_ctx_set_max_doc_entries(crdt_ctx* ctx, uint32_t max_entries);
/* Tuning knobs (performance only, never results):
 *   "join_docs_per_wave"  1|2|4|8|16  documents one wavefront pipelines (default 8)
 *   "join_nt_stores"      0|1         non-temporal output stores (default 1)
 *   "probe_blocks_per_cu" 1..64       crdt_bw_probe grid (default 16)
 *   "probe_slab"          0|1         crdt_bw_probe: one contiguous slab per workgroup
 *                                     instead of a grid-stride sweep (default 0)
 *   "join_stage_stores"   0|1         survivors staged in LDS, whole-line stores (default 1)
 *   "join_slab_blocks_per_cu" 0..64   wave kernel block order: slabs of G = this x CUs
 *                                     blocks (crdt_device.hpp SlabMap; 0 = in order)
 *   "fold_lean_first"     0|1         folds: slot-walk pass first, the rest deferred (default 1)
 *   "join_tile_capacity"  1..2^28     large documents: merge-path tiles of 1,024 merged
 *                                     positions per pass (default 2^22, 56 B each,
 *                                     allocated on first use); a call with more tiles runs
 *                                     in passes of this many, a pass may end inside a
 *                                     document
 *   "join_tile_max_passes" 1..65536   passes launched at most (default 256): a call with
 *                                     more tiles than this x capacity takes the
 *                                     per-document block kernel instead
 *   "join_tile_dispensers" 1|8        tile dispenser words (default 8, one per XCD)
 *   (also "join_tile_shape", "join_tile_nt_stores", "join_tile_split_blocks_per_cu",
 *   "join_tiles": see api.cpp)
 * and one layout option of the host-buffer (*_batch) joins, exchanges and folds:
 *   "pack_batch_outputs"  0|1         1: out holds only the live entries, doc d
 *                                     at offsets[d] = counts[0] + .. + counts[d-1]
 *                                     (less to download; the offsets are computed on the
 *                                     device, and outputs in crdt_host_alloc memory are
 *                                     written there by the device, no copy call); 0
 *                                     (default): at its capacity offset, as the *_async
 *                                     calls write.
 *   "span_staging"        0|1         inputs lying in one crdt_host_alloc block go up as
 *                                     one copy of the span they cover (default 1)
 * The *_batch calls check the slot layout on the host and the key order on the
 * device after the upload; a batch out of order reaches no merge kernel (the
 * merge's first kernel reads the check's verdict on the device) and the call
 * returns CRDT_E_UNSORTED with the outputs unspecified; crdt_validate_batch
 * checks everything on the host. */
int crdt_ctx_set_option(crdt_ctx* ctx, const char* name, int64_t value);
/* Wait for `stream`, return (and clear) the first device-side error. */
int crdt_ctx_sync(crdt_ctx* ctx, void* stream);
const char* crdt_strerror(int code);
int crdt_abi_version(void);

/* ---- device-resident, asynchronous on a HIP stream (NULL = default) ---- */
int crdt_awset_join_async(crdt_ctx* ctx, const crdt_awset_batch* dst, const crdt_awset_batch* src,
                          const crdt_awset_out* out, void* stream);
/* Anti-entropy exchange: out_ab[d] = a[d] <- b[d] AND out_ba[d] = b[d] <- a[d]
 * (two (*AWSet).Merge calls per doc, awset.go:103-161) from ONE read of both
 * states.  Both directions keep the same keys at the same slots; only a
 * common key's dot differs (the src dot wins, awset.go:142).  So the two
 * outputs may share one key column: out_ba->keys == out_ab->keys is allowed
 * and writes the keys once; every other output array must be distinct and
 * must not overlap another (CRDT_E_INVALID when two arrays start at the same
 * address or the per-document arrays overlap; a partial overlap of the entry
 * arrays, whose capacity is in device memory, is undefined behaviour).
 * (crdt_awset_exchange_batch: the same for host outputs -- the shared column
 * is also downloaded once.) */
int crdt_awset_exchange_async(crdt_ctx* ctx, const crdt_awset_batch* a, const crdt_awset_batch* b,
                              const crdt_awset_out* out_ab, const crdt_awset_out* out_ba, void* stream);
int crdt_awset_fold_async(crdt_ctx* ctx, int mode, const crdt_awset_batch* dst, const crdt_src_batch* srcs,
                          const crdt_awset_out* out, void* stream);
/* dst[i] = max(dst[i], src[i]) for i < n (u64). */
int crdt_vv_max_async(crdt_ctx* ctx, uint64_t* dst, const uint64_t* src, size_t n, void* stream);
/* out[r] = max over d < n_docs of vv[d*R + r]  (the per-GPU causal-context summary). */
int crdt_causal_context_async(crdt_ctx* ctx, const uint64_t* vv, uint32_t n_docs, uint32_t R, uint64_t* out,
                              void* stream);

/* ---- synthetic workloads (bench / GPU tests; not part of a merge) ----------
 * "pair" (BASELINE config 2): n_docs documents x 2 replicas (A actor 0, B
 * actor 1), R = 2, 64 live entries each in 64 slots per doc; reachable states
 * (formulas: go-crdt-playground_amd/csrc/gen.hip).  a/b need n_docs*64 slots. */
int crdt_gen_pair_async(crdt_ctx* ctx, uint64_t seed, uint32_t n_docs, const crdt_awset_out* a,
                        const crdt_awset_out* b, void* stream);
/* "delta" (BASELINE config 3): n_docs dst docs x 64 entries (64 slots each),
 * R actors, n_srcs_per_doc ordered AWSetDelta sources per doc of 8 entries and
 * 2 tombstones.  Writes through srcs' pointers (all must be allocated:
 * n_docs*M sources, 8 and 2 slots each).  Formulas: csrc/gen.hip. */
int crdt_gen_delta_async(crdt_ctx* ctx, uint64_t seed, uint32_t n_docs, uint32_t R, uint32_t n_srcs_per_doc,
                         const crdt_awset_out* dst, const crdt_src_batch* srcs, void* stream);
/* "replicas" (BASELINE config 5): per doc `replicas` AWSet states of `entries`
 * entries (a power of two <= 32), R = replicas; dst = replica 0 (entries slots
 * per doc), srcs = replicas 1.. in order (entries slots each, 0 tombstones;
 * tomb_off must be allocated).  Fold with CRDT_FOLD_AWSET. */
/* "zipf" (BASELINE config 4): n_docs (< 2^24) docs, sizes from
 * crdt_gen_zipf_sizes (host, no GPU), A/B replicas with 50% concurrent
 * add/remove conflicts, R = 2.  offsets: device array [n_docs+1], the prefix
 * sum of the sizes (each side gets `size` slots per doc).  Formulas: gen.hip. */
int crdt_gen_zipf_sizes(uint64_t seed, uint32_t n_docs, uint32_t* sizes);
int crdt_gen_zipf_async(crdt_ctx* ctx, uint64_t seed, uint32_t n_docs, const uint32_t* offsets,
                        const crdt_awset_out* a, const crdt_awset_out* b, void* stream);
int crdt_gen_replicas_async(crdt_ctx* ctx, uint64_t seed, uint32_t n_docs, uint32_t replicas, uint32_t entries,
                            const crdt_awset_out* dst, const crdt_src_batch* srcs, void* stream);

/* ---- box bandwidth probes (not a merge; bench.py's roofline context) ------
 * Times `reps` launches of a streaming kernel over caller-owned device memory
 * on the context's stream (after one untimed launch) and returns the HBM rate
 * in GB/s (1e9 B/s): READ reads `bytes` of a (16 B per lane, four loads in
 * flight), WRITE writes `bytes` to b (16 B non-temporal stores; _PLAIN: plain
 * stores), COPY reads a and writes b (counts 2 x bytes).  READ needs b as a
 * 4-byte sink.  Grid: crdt_ctx_set_option("probe_blocks_per_cu", 1..64,
 * default 16) workgroups of 256 per CU.  Use buffers well above the 256 MiB
 * Infinity Cache.  Synchronous. */
#define CRDT_PROBE_READ 0
#define CRDT_PROBE_WRITE 1
#define CRDT_PROBE_COPY 2
#define CRDT_PROBE_WRITE_PLAIN 3
#define CRDT_PROBE_COPY_PLAIN 4
#define CRDT_PROBE_MIX 5       /* 3 reads : 4 writes of 16 B (the exchange's mix), nt stores; GB/s = all 7 */
#define CRDT_PROBE_MIX_PLAIN 6 /* the same, plain stores */
int crdt_bw_probe(crdt_ctx* ctx, int kind, const void* a, void* b, size_t bytes, int reps, double* gbs);
/* The shader clock (MHz) while every CU runs dependent integer chains:
 * shader-cycle counter over the fixed-rate wall clock on one wave.  Kernels
 * bound by instruction issue scale with it; streaming ones do not. */
int crdt_clock_probe(crdt_ctx* ctx, double* mhz);

/* ---- batched local operations: the state producers -----
 * Each document receives an ordered op list, applied to its replica state
 * (AWSet entries + VV, and for AWSetDelta its Deleted tombstones) as the
 * reference's calls would be, in order:
 *   CRDT_OP_ADD            (*AWSet).Add(k)            awset.go:89-94
 *                          vv[actor]++; entries[k] = {actor, vv[actor]}
 *   CRDT_OP_DEL            (*AWSet).Del(k)            awset.go:96-101
 *                          delete(entries, k); no clock bump
 *   CRDT_OP_DELTA_DEL      starts one (*AWSetDelta).Del(k...) call,
 *                          awset-delta_test.go:14-33: vv[actor]++ once
 *   CRDT_OP_DELTA_DEL_KEY  one key of that call (must follow the
 *                          DELTA_DEL or another DELTA_DEL_KEY): if k is in
 *                          entries, Deleted[k] = {actor, vv[actor]} and the
 *                          entry is deleted; otherwise nothing
 * Add(k1, k2) / Del(k1, k2) are one op per key in order.  `keys` of
 * CRDT_OP_DELTA_DEL ops are ignored.  The doc's replica actor is doc_actor[d];
 * an op that bumps the clock with actor >= R is Go's index-out-of-range panic:
 * CRDT_E_ACTOR_RANGE.  At most CRDT_MAX_OPS_PER_DOC ops per doc per call
 * (longer lists: successive calls); malformed lists: CRDT_E_INVALID.
 * Outputs: doc d's entries at out offset state.offsets[d] + op_off[d]
 * (capacity = state slots + ops), its tombstones at tombs.offsets[d] +
 * op_off[d] (tombs NULL: no Deleted yet, offsets 0); tomb_out may be NULL when
 * no DELTA_DEL_KEY op occurs.  Offsets/counts are written for every doc. */
#define CRDT_OP_ADD 0
#define CRDT_OP_DEL 1
#define CRDT_OP_DELTA_DEL 2
#define CRDT_OP_DELTA_DEL_KEY 3
#define CRDT_MAX_OPS_PER_DOC 256

typedef struct {
    uint32_t n_docs;
    const uint32_t* op_off;    /* [n_docs+1]  */
    const uint8_t* kind;       /* [n_ops]     */
    const uint64_t* keys;      /* [n_ops]     */
    const uint32_t* doc_actor; /* [n_docs]  AWSet.Actor of each doc's replica */
} crdt_op_batch;

/* AWSetDelta.Deleted of each doc of a batch (sorted by key). */
typedef struct {
    const uint32_t* offsets;  /* [n_docs+1] */
    const uint32_t* counts;   /* [n_docs] or NULL */
    const uint64_t* keys;
    const uint32_t* actors;
    const uint64_t* counters;
} crdt_tomb_batch;

typedef struct {
    uint32_t* offsets;  /* [n_docs+1] */
    uint32_t* counts;   /* [n_docs]   */
    uint64_t* keys;
    uint32_t* actors;
    uint64_t* counters;
} crdt_tomb_out;

int crdt_awset_apply_async(crdt_ctx* ctx, const crdt_awset_batch* state, const crdt_tomb_batch* tombs,
                           const crdt_op_batch* ops, const crdt_awset_out* out, const crdt_tomb_out* tomb_out,
                           void* stream);
int crdt_awset_apply_batch(crdt_ctx* ctx, const crdt_awset_batch* state, const crdt_tomb_batch* tombs,
                           const crdt_op_batch* ops, const crdt_awset_out* out, const crdt_tomb_out* tomb_out);

/* ---- ingest sort ---------------------------------------------------------
 * The merge kernels need each document's keys strictly ascending; a producer
 * that packs Go maps (random iteration order) can hand them over unsorted and
 * sort on the device: out gets each document's live entries ordered by key, at
 * the same slot offsets as `in` (out must not alias in; capacity = in's
 * slots), counts = live counts, VVs copied.  A key twice in one document:
 * CRDT_E_DUP_KEY.  n_slots = in->offsets[n_docs] (host-known for async). */
int crdt_awset_sort_async(crdt_ctx* ctx, const crdt_awset_batch* in, uint32_t n_slots, const crdt_awset_out* out,
                          void* stream);
int crdt_awset_sort_batch(crdt_ctx* ctx, const crdt_awset_batch* in, const crdt_awset_out* out);

/* ---- opt-in tombstone GC -------------------------------
 * The reference never collects tombstones: (*AWSetDelta).gcDeleted is an
 * empty stub (awset-delta_test.go:67-77) whose comment states the intent,
 * "remove entries in s.Deleted for srcVersionVector".  Nothing calls this
 * implicitly.  Doc d keeps tombstone (k, x) unless stable[d*R..].HasDot(x)
 * (crdt-misc.go:28-34; actor >= R is "not covered", kept).  Pass per doc the
 * clock every replica has reached (the elementwise min of the replicas' VVs,
 * crdt_vv_min_async) so that no replica can still need the delete, or the
 * source VV of the last merge for the stub's literal reading.  Output at the
 * input's slot offsets, compacted, in key order. */
int crdt_tombstone_gc_async(crdt_ctx* ctx, const crdt_tomb_batch* tombs, uint32_t n_docs, uint32_t R,
                            const uint64_t* stable_vv, const crdt_tomb_out* out, void* stream);
/* dst[i] = min(dst[i], src[i]) for i < n (u64): causal stability across replicas. */
int crdt_vv_min_async(crdt_ctx* ctx, uint64_t* dst, const uint64_t* src, size_t n, void* stream);

/* ---- fixture dumps and debug text, host buffers -------
 * crdt_awset_format: Go's (AWSet).String() of doc `doc` (awset.go:163-171:
 * VersionVector.String crdt-misc.go:57-68, then "
  %s  %q" per entry in
 * sorted key order, Dot.String crdt-misc.go:17-19).  names[id] is the string
 * of key id (ids order-preserving); names == NULL prints "#<id>".  The VV
 * prints all R words.  Writes at most cap bytes including the NUL; *len = the
 * full length.
 * crdt_batch_dump: a self-checking binary image of a batch (live entries
 * only, compact offsets); buf == NULL: *len = the size needed.
 * crdt_batch_info / crdt_batch_undump: check an image and read its sizes, then
 * fill caller arrays (offsets n_docs+1, counts, n_entries entries, n_docs*R vv). */
int crdt_awset_format(const crdt_awset_batch* b, uint32_t doc, const char* const* names, char* buf, size_t cap,
                      size_t* len);
int crdt_batch_dump(const crdt_awset_batch* b, void* buf, size_t cap, size_t* len);
int crdt_batch_info(const void* buf, size_t len, uint32_t* n_docs, uint32_t* R, uint64_t* n_entries);
int crdt_batch_undump(const void* buf, size_t len, const crdt_awset_out* out);

/* ---- multi-GPU: the global causal context over RCCL (xGMI) --------------
 * Documents shard over GPUs with no exchange; the one collective is the
 * causal-context summary, R u64 per GPU, combined with
 * ncclAllReduce(ncclUint64, ncclMax).  RCCL is bound at run time (an RCCL
 * already mapped by the process is reused); without it these return
 * CRDT_E_RCCL.
 *
 * One process, several GPUs: per_gpu[i] is a context on its own device and
 * vv_R[i] a device pointer on that device holding its summary (e.g. the
 * output of crdt_causal_context_async); every vv_R[i] is replaced by the
 * elementwise max over all of them, and out_vv_R (host, may be NULL)
 * receives a copy.  Synchronous.  The communicators are built on the first
 * call and kept while the same contexts are passed in the same order.
 *
 * One process per GPU: rank 0 makes an id (crdt_comm_unique_id), every rank
 * receives it out of band and calls crdt_comm_init; then
 * crdt_context_allreduce_async reduces vv_R in place on `stream`. */
#define CRDT_COMM_ID_BYTES 128
int crdt_global_context_allreduce(crdt_ctx* const* per_gpu, int n_gpus, uint64_t* const* vv_R, uint32_t R,
                                  uint64_t* out_vv_R);
int crdt_comm_unique_id(uint8_t* id /* [CRDT_COMM_ID_BYTES] */);
int crdt_comm_init(crdt_ctx* ctx, int n_ranks, int rank, const uint8_t* id);
int crdt_context_allreduce_async(crdt_ctx* ctx, uint64_t* vv_R, uint32_t R, void* stream);

/* ---- host buffers, synchronous: copies in, runs, copies out -------------
 * Host arrays from crdt_host_alloc (page-locked) cross PCIe by DMA at full
 * link rate; pageable arrays work too, staged by the HIP runtime.  A caller
 * packing many batches keeps its page-locked arrays and reuses them. */
int crdt_host_alloc(size_t bytes, void** out);
void crdt_host_free(void* p);
int crdt_awset_join_batch(crdt_ctx* ctx, const crdt_awset_batch* dst, const crdt_awset_batch* src,
                          const crdt_awset_out* out);
int crdt_awset_exchange_batch(crdt_ctx* ctx, const crdt_awset_batch* a, const crdt_awset_batch* b,
                              const crdt_awset_out* out_ab, const crdt_awset_out* out_ba);
int crdt_awset_fold_batch(crdt_ctx* ctx, int mode, const crdt_awset_batch* dst, const crdt_src_batch* srcs,
                          const crdt_awset_out* out);

/* ---- host-side validation of a packed batch (no GPU) -------------------- */
int crdt_validate_batch(const crdt_awset_batch* b);
int crdt_validate_src_batch(const crdt_src_batch* s);
/* tombstones of n_docs documents: monotone offsets, counts <= slots, keys
 * strictly ascending per document (crdt_awset_apply_batch runs it first). */
int crdt_validate_tomb_batch(const crdt_tomb_batch* t, uint32_t n_docs);

#ifdef __cplusplus
}
#endif
#endif /* CRDTGPU_H */
