/*
 * TEST INFRASTRUCTURE ONLY -- CPU restatement of the reference merge over the
 * engine's SoA batch layout (include/crdtgpu.h).
 *
 * This is the ORACLE the HIP kernels are checked against.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it; the
 * product library never links it.
 *
 * It follows the reference phase by phase, with a document held as sorted
 * arrays standing in for Go's map[string]Dot (a map lookup becomes a binary
 * search):
 *   has_dot / counter            crdt-misc.go:28-41 (actor == len panics there:
 *                                 here CRDT_E_ACTOR_RANGE)
 *   vv merge                     crdt-misc.go:43-55
 *   join_doc                     awset.go:107-161  (phase 1 :122-143,
 *                                 phase 2 :145-159, VV merge :160)
 *   make_delta / delta_merge     awset-delta_test.go:79-105, 107-166
 *   delta step (path select)     awset-delta_test.go:51-65
 * Pinned against tests/golden/kat_scenarios.json (tests/test_oracle.py).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/crdtgpu.h"

typedef struct {
    uint64_t key;
    uint32_t actor;
    uint64_t counter;
} ent;

/* crdt-misc.go:28-34 */
static int has_dot(const uint64_t* vv, uint32_t R, uint32_t actor, uint64_t counter, int* err) {
    if (R < actor) return 0;
    if (actor == R) {
        *err = CRDT_E_ACTOR_RANGE;
        return 0;
    }
    return vv[actor] >= counter;
}

/* crdt-misc.go:36-41 */
static uint64_t counter_of(const uint64_t* vv, uint32_t R, uint32_t actor, int* err) {
    if (R < actor) return 0;
    if (actor == R) {
        *err = CRDT_E_ACTOR_RANGE;
        return 0;
    }
    return vv[actor];
}

/* crdt-misc.go:43-55 with equal lengths */
static void vv_merge(uint64_t* dst, const uint64_t* src, uint32_t R) {
    for (uint32_t i = 0; i < R; i++)
        if (dst[i] < src[i]) dst[i] = src[i];
}

/* map lookup: index of key in e[0..n) or -1 */
static long find(const ent* e, size_t n, uint64_t key) {
    size_t lo = 0, hi = n;
    while (lo < hi) {
        size_t mid = lo + (hi - lo) / 2;
        if (e[mid].key < key)
            lo = mid + 1;
        else
            hi = mid;
    }
    return (lo < n && e[lo].key == key) ? (long)lo : -1;
}

/* A working document: sorted entries with a capacity. */
typedef struct {
    ent* e;
    size_t n, cap;
} doc_t;

/* Rebuild d from kept d-entries (flag keep[i]) merged with sorted `add` list. */
static int rebuild(doc_t* d, const unsigned char* keep, const ent* add, size_t nadd, ent* scratch) {
    size_t i = 0, j = 0, o = 0;
    while (i < d->n || j < nadd) {
        if (i < d->n && !keep[i]) {
            i++;
            continue;
        }
        if (j >= nadd || (i < d->n && d->e[i].key < add[j].key))
            scratch[o++] = d->e[i++];
        else
            scratch[o++] = add[j++];
    }
    memcpy(d->e, scratch, o * sizeof(ent));
    d->n = o;
    return 0;
}

typedef struct {
    ent* buf_add;
    ent* scratch;
    unsigned char* keep;
    size_t cap;
} work_t;

static int work_reserve(work_t* w, size_t cap) {
    if (cap <= w->cap) return 0;
    free(w->buf_add);
    free(w->scratch);
    free(w->keep);
    w->buf_add = (ent*)malloc(cap * sizeof(ent));
    w->scratch = (ent*)malloc(cap * sizeof(ent));
    w->keep = (unsigned char*)malloc(cap);
    w->cap = cap;
    return (w->buf_add && w->scratch && w->keep) ? 0 : CRDT_E_NOMEM;
}

static void work_free(work_t* w) {
    free(w->buf_add);
    free(w->scratch);
    free(w->keep);
}

/*
 * awset.go:107-161: dst <- (srcVV, src entries).  d holds dst, dvv its VV
 * (updated in place).
 */
static int join_doc(doc_t* d, uint64_t* dvv, const uint64_t* svv, const ent* s, size_t ns, uint32_t R, work_t* w) {
    int err = 0;
    size_t nadd = 0;
    /* phase 1 (awset.go:122-143): src dot wins on common keys, a src-only key
       is added unless dst's clock covers its dot.  Decisions use the pre-merge
       dst VV (merged only at :160). */
    for (size_t j = 0; j < ns; j++) {
        long i = find(d->e, d->n, s[j].key);
        if (i >= 0) {
            d->e[i].actor = s[j].actor;
            d->e[i].counter = s[j].counter;
        } else if (!has_dot(dvv, R, s[j].actor, s[j].counter, &err)) {
            w->buf_add[nadd++] = s[j];
        }
    }
    /* phase 2 (awset.go:145-159): every entry of dst (the added ones are all
       in src and are kept) -- a dst-only key src has seen is removed. */
    for (size_t i = 0; i < d->n; i++) {
        w->keep[i] = 1;
        if (find(s, ns, d->e[i].key) < 0 && has_dot(svv, R, d->e[i].actor, d->e[i].counter, &err)) w->keep[i] = 0;
    }
    rebuild(d, w->keep, w->buf_add, nadd, w->scratch);
    vv_merge(dvv, svv, R); /* awset.go:160 */
    return err;
}

/*
 * awset-delta_test.go:51-65 (*AWSetDelta).Merge of one source into d.
 * s/ns = src.Entries, t/nt = src.Deleted, sactor = src.Actor.
 */
static int delta_step(doc_t* d, uint64_t* dvv, const uint64_t* svv, uint32_t sactor, const ent* s, size_t ns,
                      const ent* t, size_t nt, uint32_t R, work_t* w) {
    int err = 0;
    uint64_t c = counter_of(dvv, R, sactor, &err);
    if (err) return err;
    if (c <= 0) return join_doc(d, dvv, svv, s, ns, R, w); /* first contact, :53-56 */

    /* MakeDeltaMergeData (:79-105).  changed = src entries dst has not seen;
       deleted = tombstones minus keys re-added since (no dst-VV filter). */
    ent* changed = (ent*)malloc((ns ? ns : 1) * sizeof(ent));
    ent* deleted = (ent*)malloc((nt ? nt : 1) * sizeof(ent));
    size_t nc = 0, nd = 0;
    for (size_t j = 0; j < ns; j++)
        if (!has_dot(dvv, R, s[j].actor, s[j].counter, &err)) changed[nc++] = s[j];
    for (size_t j = 0; j < nt; j++) {
        long m = find(s, ns, t[j].key);
        if (m >= 0 && (s[m].actor != t[j].actor || s[m].counter > t[j].counter)) continue;
        deleted[nd++] = t[j];
    }
    if (nc == 0 && nd == 0) { /* :60 both maps nil -> nothing at all, VV included */
        free(changed);
        free(deleted);
        return err;
    }
    /* deltaMerge (:107-166).  Phase 1 (:126-147) same rule as merge phase 1. */
    size_t nadd = 0;
    for (size_t j = 0; j < nc; j++) {
        long i = find(d->e, d->n, changed[j].key);
        if (i >= 0) {
            d->e[i].actor = changed[j].actor;
            d->e[i].counter = changed[j].counter;
        } else if (!has_dot(dvv, R, changed[j].actor, changed[j].counter, &err)) {
            w->buf_add[nadd++] = changed[j];
        }
    }
    /* phase 2 (:149-164) runs over the map after phase 1, so an entry added in
       phase 1 can be deleted by a tombstone of the same key. */
    for (size_t i = 0; i < d->n; i++) w->keep[i] = 1;
    unsigned char* add_keep = (unsigned char*)malloc(nadd ? nadd : 1);
    for (size_t j = 0; j < nadd; j++) add_keep[j] = 1;
    for (size_t j = 0; j < nd; j++) {
        long i = find(d->e, d->n, deleted[j].key);
        long a = (i < 0) ? find(w->buf_add, nadd, deleted[j].key) : -1;
        if (i < 0 && a < 0) continue; /* absent: no-op */
        if (has_dot(dvv, R, deleted[j].actor, deleted[j].counter, &err)) continue; /* updated in dst: keep */
        if (i >= 0)
            w->keep[i] = 0;
        else
            add_keep[a] = 0;
    }
    size_t na = 0;
    for (size_t j = 0; j < nadd; j++)
        if (add_keep[j]) w->buf_add[na++] = w->buf_add[j];
    rebuild(d, w->keep, w->buf_add, na, w->scratch);
    vv_merge(dvv, svv, R); /* :165; gcDeleted (:63, :67-77) is empty */
    free(add_keep);
    free(changed);
    free(deleted);
    return err;
}

static uint32_t live(const crdt_awset_batch* b, uint32_t d) {
    return b->counts ? b->counts[d] : b->offsets[d + 1] - b->offsets[d];
}

static void load_doc(doc_t* doc, const crdt_awset_batch* b, uint32_t d) {
    uint32_t o = b->offsets[d], n = live(b, d);
    for (uint32_t i = 0; i < n; i++) {
        doc->e[i].key = b->keys[o + i];
        doc->e[i].actor = b->actors[o + i];
        doc->e[i].counter = b->counters[o + i];
    }
    doc->n = n;
}

static void store_doc(const doc_t* doc, const crdt_awset_out* out, uint32_t base) {
    for (size_t i = 0; i < doc->n; i++) {
        out->keys[base + i] = doc->e[i].key;
        out->actors[base + i] = doc->e[i].actor;
        out->counters[base + i] = doc->e[i].counter;
    }
}

static void gather(ent* e, const uint64_t* k, const uint32_t* a, const uint64_t* c, uint32_t lo, uint32_t hi) {
    for (uint32_t i = lo; i < hi; i++) {
        e[i - lo].key = k[i];
        e[i - lo].actor = a[i];
        e[i - lo].counter = c[i];
    }
}

/* Full-state join of every doc: out[d] = dst[d] <- src[d].  Same output layout
   as crdt_awset_join_async. */
int oracle_awset_join(const crdt_awset_batch* dst, const crdt_awset_batch* src, const crdt_awset_out* out) {
    uint32_t R = dst->R;
    if (R == 0 || src->R != R || src->n_docs != dst->n_docs) return CRDT_E_INVALID;
    work_t w = {0};
    doc_t doc = {0};
    ent* s = NULL;
    size_t scap = 0;
    int first_err = 0;
    for (uint32_t d = 0; d < dst->n_docs; d++) {
        uint32_t nd = live(dst, d), ns = live(src, d);
        size_t cap = (size_t)nd + ns + 1;
        if (work_reserve(&w, cap)) return CRDT_E_NOMEM;
        if (cap > doc.cap) {
            free(doc.e);
            doc.e = (ent*)malloc(cap * sizeof(ent));
            doc.cap = cap;
        }
        if (cap > scap) {
            free(s);
            s = (ent*)malloc(cap * sizeof(ent));
            scap = cap;
        }
        load_doc(&doc, dst, d);
        gather(s, src->keys, src->actors, src->counters, src->offsets[d], src->offsets[d] + ns);
        uint64_t* vv = out->vv + (size_t)d * R;
        memcpy(vv, dst->vv + (size_t)d * R, R * sizeof(uint64_t));
        int e = join_doc(&doc, vv, src->vv + (size_t)d * R, s, ns, R, &w);
        if (e && !first_err) first_err = e;
        uint32_t base = dst->offsets[d] + src->offsets[d];
        out->offsets[d] = base;
        out->counts[d] = (uint32_t)doc.n;
        store_doc(&doc, out, base);
    }
    out->offsets[dst->n_docs] = dst->offsets[dst->n_docs] + src->offsets[src->n_docs];
    free(doc.e);
    free(s);
    work_free(&w);
    return first_err;
}

/* Ordered fold of sources into each dst doc (mode CRDT_FOLD_AWSET or
   CRDT_FOLD_DELTA), same output layout as crdt_awset_fold_async. */
int oracle_awset_fold(int mode, const crdt_awset_batch* dst, const crdt_src_batch* sb, const crdt_awset_out* out) {
    uint32_t R = dst->R;
    if (R == 0 || sb->R != R || sb->n_docs != dst->n_docs) return CRDT_E_INVALID;
    work_t w = {0};
    doc_t doc = {0};
    ent *s = NULL, *t = NULL;
    size_t scap = 0, tcap = 0;
    int first_err = 0;
    for (uint32_t d = 0; d < dst->n_docs; d++) {
        uint32_t s0 = sb->doc_srcs[d], s1 = sb->doc_srcs[d + 1];
        size_t cap = (size_t)live(dst, d) + (sb->entry_off[s1] - sb->entry_off[s0]) + 1;
        if (work_reserve(&w, cap)) return CRDT_E_NOMEM;
        if (cap > doc.cap) {
            free(doc.e);
            doc.e = (ent*)malloc(cap * sizeof(ent));
            doc.cap = cap;
        }
        load_doc(&doc, dst, d);
        uint64_t* vv = out->vv + (size_t)d * R;
        memcpy(vv, dst->vv + (size_t)d * R, R * sizeof(uint64_t));
        int err = 0;
        for (uint32_t k = s0; k < s1 && !err; k++) {
            uint32_t e0 = sb->entry_off[k], e1 = sb->entry_off[k + 1];
            uint32_t t0 = sb->tomb_off ? sb->tomb_off[k] : 0, t1 = sb->tomb_off ? sb->tomb_off[k + 1] : 0;
            if (e1 - e0 + 1 > scap) {
                free(s);
                scap = e1 - e0 + 1;
                s = (ent*)malloc(scap * sizeof(ent));
            }
            if (t1 - t0 + 1 > tcap) {
                free(t);
                tcap = t1 - t0 + 1;
                t = (ent*)malloc(tcap * sizeof(ent));
            }
            gather(s, sb->keys, sb->actors, sb->counters, e0, e1);
            if (t1 > t0) gather(t, sb->tkeys, sb->tactors, sb->tcounters, t0, t1);
            const uint64_t* svv = sb->vv + (size_t)k * R;
            if (mode == CRDT_FOLD_DELTA)
                err = delta_step(&doc, vv, svv, sb->src_actor[k], s, e1 - e0, t, t1 - t0, R, &w);
            else
                err = join_doc(&doc, vv, svv, s, e1 - e0, R, &w);
        }
        if (err && !first_err) first_err = err;
        uint32_t base = dst->offsets[d] + sb->entry_off[s0];
        out->offsets[d] = base;
        out->counts[d] = (uint32_t)doc.n;
        store_doc(&doc, out, base);
    }
    out->offsets[dst->n_docs] = dst->offsets[dst->n_docs] + sb->entry_off[sb->doc_srcs[sb->n_docs]];
    free(doc.e);
    free(s);
    free(t);
    work_free(&w);
    return first_err;
}

/* Elementwise max over docs' VVs: the causal-context summary. */
void oracle_causal_context(const uint64_t* vv, uint32_t n_docs, uint32_t R, uint64_t* out) {
    for (uint32_t r = 0; r < R; r++) out[r] = 0;
    for (uint32_t d = 0; d < n_docs; d++) vv_merge(out, vv + (size_t)d * R, R);
}

/* ---- batched local ops: the state producers, op by op ------------------- */

/* sorted-array map: set e[key] = v (insert or overwrite); cap must allow n+1 */
static void map_set(ent* e, size_t* n, ent v) {
    size_t lo = 0, hi = *n;
    while (lo < hi) {
        size_t mid = lo + (hi - lo) / 2;
        if (e[mid].key < v.key)
            lo = mid + 1;
        else
            hi = mid;
    }
    if (lo < *n && e[lo].key == v.key) {
        e[lo] = v;
        return;
    }
    memmove(e + lo + 1, e + lo, (*n - lo) * sizeof(ent));
    e[lo] = v;
    (*n)++;
}

/* delete(e, key) */
static void map_del(ent* e, size_t* n, uint64_t key) {
    long i = find(e, *n, key);
    if (i < 0) return;
    memmove(e + i, e + i + 1, (*n - (size_t)i - 1) * sizeof(ent));
    (*n)--;
}

/*
 * Each doc's ops, in order, on its replica state (entries, VV, Deleted):
 *   CRDT_OP_ADD            awset.go:89-94   vv[actor]++; entries[k] = {actor, vv[actor]}
 *   CRDT_OP_DEL            awset.go:96-101  delete(entries, k)
 *   CRDT_OP_DELTA_DEL      awset-delta_test.go:14-16  vv[actor]++; dot2 = {actor, vv[actor]}
 *   CRDT_OP_DELTA_DEL_KEY  awset-delta_test.go:17-31  if k in entries: Deleted[k] = dot2, delete
 * VersionVector[actor]++ with actor >= len(vv) is Go's index panic:
 * CRDT_E_ACTOR_RANGE.  The device limit of CRDT_MAX_OPS_PER_DOC ops per doc
 * and the DELTA_DEL_KEY placement rule are checked too (CRDT_E_INVALID).
 */
int oracle_awset_apply(const crdt_awset_batch* st, const crdt_tomb_batch* tb, const crdt_op_batch* ops,
                       const crdt_awset_out* out, const crdt_tomb_out* tout) {
    const uint32_t R = st->R, n = st->n_docs;
    int rc = 0;
    size_t cap = 1;
    for (uint32_t d = 0; d < n; d++) {
        size_t c = (size_t)(st->offsets[d + 1] - st->offsets[d]) + (tb ? tb->offsets[d + 1] - tb->offsets[d] : 0) +
                   (ops->op_off[d + 1] - ops->op_off[d]) + 1;
        if (c > cap) cap = c;
    }
    ent* e = (ent*)malloc(cap * sizeof(ent));
    ent* t = (ent*)malloc(cap * sizeof(ent));
    uint64_t* vv = (uint64_t*)malloc((R ? R : 1) * sizeof(uint64_t));
    if (!e || !t || !vv) {
        free(e);
        free(t);
        free(vv);
        return CRDT_E_NOMEM;
    }
    for (uint32_t d = 0; d < n && !rc; d++) {
        const uint32_t so = st->offsets[d];
        size_t ne = st->counts ? st->counts[d] : st->offsets[d + 1] - so;
        gather(e, st->keys, st->actors, st->counters, so, so + (uint32_t)ne);
        size_t nt = 0;
        uint32_t to = 0;
        if (tb) {
            to = tb->offsets[d];
            nt = tb->counts ? tb->counts[d] : tb->offsets[d + 1] - to;
            gather(t, tb->keys, tb->actors, tb->counters, to, to + (uint32_t)nt);
        }
        memcpy(vv, st->vv + (size_t)d * R, R * sizeof(uint64_t));
        const uint32_t o0 = ops->op_off[d], no = ops->op_off[d + 1] - o0;
        const uint32_t actor = ops->doc_actor[d];
        if (no > CRDT_MAX_OPS_PER_DOC) rc = CRDT_E_INVALID;
        uint64_t dot2 = 0;
        for (uint32_t j = 0; j < no && !rc; j++) {
            const uint32_t kind = ops->kind[o0 + j];
            const uint64_t key = ops->keys[o0 + j];
            const uint32_t prev = j ? ops->kind[o0 + j - 1] : 0xFFu;
            if (kind == CRDT_OP_ADD || kind == CRDT_OP_DELTA_DEL) {
                if (actor >= R) {
                    rc = CRDT_E_ACTOR_RANGE;
                    break;
                }
                vv[actor]++;
            }
            if (kind == CRDT_OP_ADD) {
                ent v = {key, actor, vv[actor]};
                map_set(e, &ne, v);
            } else if (kind == CRDT_OP_DEL) {
                map_del(e, &ne, key);
            } else if (kind == CRDT_OP_DELTA_DEL) {
                dot2 = vv[actor];
            } else if (kind == CRDT_OP_DELTA_DEL_KEY) {
                if ((prev != CRDT_OP_DELTA_DEL && prev != CRDT_OP_DELTA_DEL_KEY) || !tout) {
                    rc = CRDT_E_INVALID;
                    break;
                }
                if (find(e, ne, key) >= 0) {
                    ent v = {key, actor, dot2};
                    map_set(t, &nt, v);
                    map_del(e, &ne, key);
                }
            } else {
                rc = CRDT_E_INVALID;
            }
        }
        if (rc) break;
        const uint32_t base = so + o0;
        out->offsets[d] = base;
        out->counts[d] = (uint32_t)ne;
        for (size_t i = 0; i < ne; i++) {
            out->keys[base + i] = e[i].key;
            out->actors[base + i] = e[i].actor;
            out->counters[base + i] = e[i].counter;
        }
        memcpy(out->vv + (size_t)d * R, vv, R * sizeof(uint64_t));
        if (tout) {
            const uint32_t tbase = to + o0;
            tout->offsets[d] = tbase;
            tout->counts[d] = (uint32_t)nt;
            for (size_t i = 0; i < nt; i++) {
                tout->keys[tbase + i] = t[i].key;
                tout->actors[tbase + i] = t[i].actor;
                tout->counters[tbase + i] = t[i].counter;
            }
        }
    }
    if (!rc) {
        out->offsets[n] = st->offsets[n] + ops->op_off[n];
        if (tout) tout->offsets[n] = (tb ? tb->offsets[n] : 0) + ops->op_off[n];
    }
    free(e);
    free(t);
    free(vv);
    return rc;
}

/* Opt-in tombstone GC (no reference counterpart: gcDeleted is empty,
 * awset-delta_test.go:67-77): keep (k, x) unless stable.HasDot(x), with
 * actor >= R kept.  Same layout as crdt_tombstone_gc_async. */
int oracle_tomb_gc(const crdt_tomb_batch* tb, uint32_t n_docs, uint32_t R, const uint64_t* stable,
                   const crdt_tomb_out* out) {
    for (uint32_t d = 0; d < n_docs; d++) {
        const uint32_t o = tb->offsets[d];
        const uint32_t n = tb->counts ? tb->counts[d] : tb->offsets[d + 1] - o;
        uint32_t k = 0;
        for (uint32_t i = 0; i < n; i++) {
            const uint32_t a = tb->actors[o + i];
            if (a < R && stable[(size_t)d * R + a] >= tb->counters[o + i]) continue;
            out->keys[o + k] = tb->keys[o + i];
            out->actors[o + k] = a;
            out->counters[o + k] = tb->counters[o + i];
            k++;
        }
        out->offsets[d] = o;
        out->counts[d] = k;
    }
    out->offsets[n_docs] = tb->offsets[n_docs];
    return 0;
}
