/*
 * orc_ring.c — CPU restatement of ringpop's HashRing. TEST INFRASTRUCTURE ONLY.
 *
 * Restates lib/ring/index.js (HashRing, lines 25-189) on top of the *semantics* of
 * lib/ring/rbtree.js: the red-black tree is used as an ordered map uint32 -> owner with
 *   - insert-if-absent: RBTree.insert returns false on a duplicate and keeps the existing
 *     payload (rbtree.js:112-116),
 *   - erase-by-key: RBTree.remove(val) ignores the owner argument (rbtree.js:152; called
 *     as remove(hash, server) at lib/ring/index.js:141),
 *   - upperBound(h) == first key >= h (rbtree.js:235-271, pinned by rbtree_test.js:575-592).
 * Here the map is an open-addressing hash table plus a lazily rebuilt sorted array.
 */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

#define NIL 0xFFFFFFFFu

typedef struct {
    uint32_t *keys;   /* token */
    uint32_t *vals;   /* owner id, NIL = empty, NIL-1 = tombstone */
    uint32_t cap;     /* power of two */
    uint32_t used;    /* live + tombstones */
    uint32_t live;
} tokmap;

struct orc_ring {
    uint32_t R;
    /* interned names */
    char *nb;
    uint64_t nb_len, nb_cap;
    uint64_t *noff; /* noff[id], noff[id+1] */
    uint32_t nnames, ncap;
    uint8_t *in_ring;
    uint32_t *ht; /* name hash table -> id, NIL empty */
    uint32_t ht_cap;
    uint32_t server_count;
    /* token map */
    tokmap tm;
    /* sorted view */
    int dirty;
    uint32_t *T, *O;
    uint32_t M;
    /* checksum */
    int has_checksum;
    uint32_t checksum;
};

static uint64_t fnv64(const char *s, uint32_t n) {
    uint64_t h = 1469598103934665603ull;
    for (uint32_t i = 0; i < n; i++) {
        h ^= (uint8_t)s[i];
        h *= 1099511628211ull;
    }
    return h;
}

static void ht_rebuild(orc_ring *r, uint32_t cap) {
    free(r->ht);
    r->ht = (uint32_t *)malloc(sizeof(uint32_t) * cap);
    memset(r->ht, 0xff, sizeof(uint32_t) * cap);
    r->ht_cap = cap;
    for (uint32_t id = 0; id < r->nnames; id++) {
        const char *s = r->nb + r->noff[id];
        uint32_t n = (uint32_t)(r->noff[id + 1] - r->noff[id]);
        uint32_t p = (uint32_t)fnv64(s, n) & (cap - 1);
        while (r->ht[p] != NIL) p = (p + 1) & (cap - 1);
        r->ht[p] = id;
    }
}

static uint32_t name_find(const orc_ring *r, const char *s, uint32_t n) {
    uint32_t p = (uint32_t)fnv64(s, n) & (r->ht_cap - 1);
    while (r->ht[p] != NIL) {
        uint32_t id = r->ht[p];
        uint32_t ln = (uint32_t)(r->noff[id + 1] - r->noff[id]);
        if (ln == n && memcmp(r->nb + r->noff[id], s, n) == 0) return id;
        p = (p + 1) & (r->ht_cap - 1);
    }
    return NIL;
}

static uint32_t name_intern(orc_ring *r, const char *s, uint32_t n) {
    uint32_t id = name_find(r, s, n);
    if (id != NIL) return id;
    if (r->nnames + 1 >= r->ncap) {
        r->ncap = r->ncap ? r->ncap * 2 : 64;
        r->noff = (uint64_t *)realloc(r->noff, sizeof(uint64_t) * (r->ncap + 1));
        r->in_ring = (uint8_t *)realloc(r->in_ring, r->ncap);
    }
    if (r->nb_len + n > r->nb_cap) {
        while (r->nb_len + n > r->nb_cap) r->nb_cap = r->nb_cap ? r->nb_cap * 2 : 4096;
        r->nb = (char *)realloc(r->nb, r->nb_cap);
    }
    memcpy(r->nb + r->nb_len, s, n);
    id = r->nnames++;
    r->noff[id] = r->nb_len;
    r->nb_len += n;
    r->noff[id + 1] = r->nb_len;
    r->in_ring[id] = 0;
    if ((uint64_t)r->nnames * 2 > r->ht_cap) ht_rebuild(r, r->ht_cap * 2);
    else {
        uint32_t p = (uint32_t)fnv64(s, n) & (r->ht_cap - 1);
        while (r->ht[p] != NIL) p = (p + 1) & (r->ht_cap - 1);
        r->ht[p] = id;
    }
    return id;
}

static uint32_t mix32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

static void tm_init(tokmap *m, uint32_t cap) {
    m->cap = cap;
    m->keys = (uint32_t *)calloc(cap, sizeof(uint32_t));
    m->vals = (uint32_t *)malloc(sizeof(uint32_t) * cap);
    memset(m->vals, 0xff, sizeof(uint32_t) * cap);
    m->used = m->live = 0;
}

static void tm_insert_raw(tokmap *m, uint32_t k, uint32_t v);

static void tm_grow(tokmap *m) {
    tokmap old = *m;
    uint32_t cap = old.cap;
    if (old.live * 2 >= cap / 2) cap *= 2;
    tm_init(m, cap);
    for (uint32_t i = 0; i < old.cap; i++)
        if (old.vals[i] < NIL - 1) tm_insert_raw(m, old.keys[i], old.vals[i]);
    free(old.keys);
    free(old.vals);
}

static void tm_insert_raw(tokmap *m, uint32_t k, uint32_t v) {
    uint32_t p = mix32(k) & (m->cap - 1);
    while (m->vals[p] != NIL) p = (p + 1) & (m->cap - 1);
    m->keys[p] = k;
    m->vals[p] = v;
    m->used++;
    m->live++;
}

/* RBTree.insert: insert-if-absent, returns 1 if inserted (rbtree.js:70-144). */
static int tm_insert(tokmap *m, uint32_t k, uint32_t v) {
    if ((uint64_t)(m->used + 1) * 4 > (uint64_t)m->cap * 3) tm_grow(m);
    uint32_t p = mix32(k) & (m->cap - 1);
    uint32_t tomb = NIL;
    while (m->vals[p] != NIL) {
        if (m->vals[p] == NIL - 1) {
            if (tomb == NIL) tomb = p;
        } else if (m->keys[p] == k) {
            return 0; /* duplicate: existing owner kept */
        }
        p = (p + 1) & (m->cap - 1);
    }
    if (tomb != NIL) p = tomb; else m->used++;
    m->keys[p] = k;
    m->vals[p] = v;
    m->live++;
    return 1;
}

/* RBTree.remove: erase-by-key whatever the owner (rbtree.js:152-232). */
static int tm_remove(tokmap *m, uint32_t k) {
    uint32_t p = mix32(k) & (m->cap - 1);
    while (m->vals[p] != NIL) {
        if (m->vals[p] != NIL - 1 && m->keys[p] == k) {
            m->vals[p] = NIL - 1;
            m->live--;
            return 1;
        }
        p = (p + 1) & (m->cap - 1);
    }
    return 0;
}

orc_ring *orc_ring_new(uint32_t replica_points) {
    orc_ring *r = (orc_ring *)calloc(1, sizeof(orc_ring));
    r->R = replica_points ? replica_points : 100; /* lib/ring/index.js:28 */
    r->ht_cap = 0;
    r->ht = NULL;
    ht_rebuild(r, 128);
    tm_init(&r->tm, 1024);
    r->dirty = 1;
    return r;
}

void orc_ring_free(orc_ring *r) {
    if (!r) return;
    free(r->nb); free(r->noff); free(r->in_ring); free(r->ht);
    free(r->tm.keys); free(r->tm.vals);
    free(r->T); free(r->O);
    free(r);
}

/* hashFunc(server + i): decimal concatenation (lib/ring/index.js:55,140) */
static uint32_t replica_hash(const char *s, uint32_t n, uint32_t i) {
    char buf[4096 + 16];
    char dig[16];
    int nd = 0;
    do { dig[nd++] = (char)('0' + i % 10); i /= 10; } while (i);
    uint32_t L = n < 4096 ? n : 4096;
    memcpy(buf, s, L);
    for (int k = 0; k < nd; k++) buf[L + k] = dig[nd - 1 - k];
    return orc_hash32((const uint8_t *)buf, L + (uint32_t)nd);
}

static int cmp_names(const orc_ring *r, uint32_t a, uint32_t b) {
    const char *sa = r->nb + r->noff[a];
    const char *sb = r->nb + r->noff[b];
    uint32_t la = (uint32_t)(r->noff[a + 1] - r->noff[a]);
    uint32_t lb = (uint32_t)(r->noff[b + 1] - r->noff[b]);
    uint32_t l = la < lb ? la : lb;
    int c = memcmp(sa, sb, l);
    if (c) return c;
    return la < lb ? -1 : (la > lb ? 1 : 0);
}

static const orc_ring *g_sort_ring; /* qsort context (oracle is single-threaded here) */
static int qcmp_ids(const void *x, const void *y) {
    return cmp_names(g_sort_ring, *(const uint32_t *)x, *(const uint32_t *)y);
}

/* HashRing.computeChecksum (lib/ring/index.js:96-105):
 * hash32(Object.keys(servers).sort().join(';')) */
static void compute_checksum(orc_ring *r) {
    uint32_t *ids = (uint32_t *)malloc(sizeof(uint32_t) * (r->server_count + 1));
    uint32_t k = 0;
    uint64_t total = 0;
    for (uint32_t id = 0; id < r->nnames; id++)
        if (r->in_ring[id]) {
            ids[k++] = id;
            total += r->noff[id + 1] - r->noff[id] + 1;
        }
    g_sort_ring = r;
    qsort(ids, k, sizeof(uint32_t), qcmp_ids);
    char *buf = (char *)malloc(total + 1);
    uint64_t o = 0;
    for (uint32_t j = 0; j < k; j++) {
        uint32_t id = ids[j];
        uint64_t ln = r->noff[id + 1] - r->noff[id];
        if (j) buf[o++] = ';';
        memcpy(buf + o, r->nb + r->noff[id], ln);
        o += ln;
    }
    r->checksum = orc_hash32((const uint8_t *)buf, o);
    r->has_checksum = 1;
    free(buf);
    free(ids);
}

int orc_ring_add_remove(orc_ring *r,
                        const char *add_bytes, const uint32_t *add_off, uint32_t n_add,
                        const uint32_t *add_tokens,
                        const char *rem_bytes, const uint32_t *rem_off, uint32_t n_rem,
                        const uint32_t *rem_tokens) {
    int added = 0, removed = 0;
    /* lib/ring/index.js:69-76: adds first, in array order, skipping present servers */
    for (uint32_t j = 0; j < n_add; j++) {
        const char *s = add_bytes + add_off[j];
        uint32_t n = add_off[j + 1] - add_off[j];
        uint32_t id = name_intern(r, s, n);
        if (r->in_ring[id]) continue;            /* hasServer (118-120) */
        r->in_ring[id] = 1;                       /* servers[server] = true (52) */
        r->server_count++;
        for (uint32_t i = 0; i < r->R; i++) {    /* addServerReplicas (54-57) */
            uint32_t t = add_tokens ? add_tokens[(uint64_t)j * r->R + i] : replica_hash(s, n, i);
            tm_insert(&r->tm, t, id);
        }
        added = 1;
    }
    /* lib/ring/index.js:78-85: then removes, in array order, skipping absent servers */
    for (uint32_t j = 0; j < n_rem; j++) {
        const char *s = rem_bytes + rem_off[j];
        uint32_t n = rem_off[j + 1] - rem_off[j];
        uint32_t id = name_find(r, s, n);
        if (id == NIL || !r->in_ring[id]) continue;
        r->in_ring[id] = 0;                       /* delete servers[server] (137) */
        r->server_count--;
        for (uint32_t i = 0; i < r->R; i++) {    /* removeServerReplicas (139-142) */
            uint32_t t = rem_tokens ? rem_tokens[(uint64_t)j * r->R + i] : replica_hash(s, n, i);
            tm_remove(&r->tm, t);
        }
        removed = 1;
    }
    if (added || removed) {
        r->dirty = 1;
        compute_checksum(r);                      /* (89-91) */
        return 1;
    }
    return 0;
}

int orc_ring_checksum(const orc_ring *r, uint32_t *out) {
    if (!r->has_checksum) return 0;
    *out = r->checksum;
    return 1;
}

uint32_t orc_ring_server_count(const orc_ring *r) { return r->server_count; }

const char *orc_ring_name(const orc_ring *r, uint32_t id, uint32_t *len) {
    if (id >= r->nnames) { *len = 0; return NULL; }
    *len = (uint32_t)(r->noff[id + 1] - r->noff[id]);
    return r->nb + r->noff[id];
}

static int cmp_u64(const void *a, const void *b) {
    uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
    return x < y ? -1 : x > y;
}

static void ensure_sorted(orc_ring *r) {
    if (!r->dirty) return;
    uint32_t M = r->tm.live;
    uint64_t *kv = (uint64_t *)malloc(sizeof(uint64_t) * (M + 1));
    uint32_t k = 0;
    for (uint32_t i = 0; i < r->tm.cap; i++)
        if (r->tm.vals[i] < NIL - 1) kv[k++] = ((uint64_t)r->tm.keys[i] << 32) | r->tm.vals[i];
    qsort(kv, k, sizeof(uint64_t), cmp_u64);
    free(r->T); free(r->O);
    r->T = (uint32_t *)malloc(sizeof(uint32_t) * (k + 1));
    r->O = (uint32_t *)malloc(sizeof(uint32_t) * (k + 1));
    for (uint32_t i = 0; i < k; i++) { r->T[i] = (uint32_t)(kv[i] >> 32); r->O[i] = (uint32_t)kv[i]; }
    r->M = k;
    free(kv);
    r->dirty = 0;
}

uint32_t orc_ring_token_count(orc_ring *r) { ensure_sorted(r); return r->M; }

void orc_ring_dump(orc_ring *r, uint32_t *tokens, uint32_t *owners) {
    ensure_sorted(r);
    memcpy(tokens, r->T, sizeof(uint32_t) * r->M);
    memcpy(owners, r->O, sizeof(uint32_t) * r->M);
}

/* first index with T[i] >= h (rbtree upperBound == lowerBound, rbtree.js:235-271) */
static uint32_t lower_bound(const uint32_t *T, uint32_t M, uint32_t h) {
    uint32_t lo = 0, hi = M;
    while (lo < hi) {
        uint32_t mid = lo + ((hi - lo) >> 1);
        if (T[mid] < h) lo = mid + 1; else hi = mid;
    }
    return lo;
}

/* HashRing.lookup (lib/ring/index.js:145-154) */
static uint32_t lookup_sorted(const orc_ring *r, uint32_t h) {
    if (r->M == 0) return NIL;                   /* min() null -> null */
    uint32_t i = lower_bound(r->T, r->M, h);
    return r->O[i == r->M ? 0 : i];              /* past-the-end -> rbtree.min() */
}

uint32_t orc_ring_lookup_hash(orc_ring *r, uint32_t h) {
    ensure_sorted(r);
    return lookup_sorted(r, h);
}

/* HashRing.lookupN (lib/ring/index.js:157-189), restated as an index walk.
 * The do/while visits positions i, i+1, ..., M-1, (null: wrap to min), 0, ..., i-1 and
 * stops when the cursor is back at firstVal; the count test runs after each visit. */
static uint32_t lookupn_sorted(const orc_ring *r, uint32_t h, int64_t n, uint32_t *out, uint32_t cap) {
    int64_t sc = r->server_count;                /* getServerCount (159, 108) */
    if (n > sc) n = sc;
    uint32_t M = r->M;
    uint32_t cnt = 0;
    if (M == 0) return 0;                        /* iter stays null; val()===firstVal===null */
    uint32_t i = lower_bound(r->T, M, h);
    if (n <= 0) {
        /* one loop body, then `resultArray.length < n` is false */
        if (i < M) { if (cap) out[0] = r->O[i]; return 1; }
        return 0;                                /* the body only wrapped the iterator */
    }
    uint32_t j = (i == M) ? 0 : i;
    for (uint32_t steps = 0; steps < M; steps++) {
        uint32_t o = r->O[j];
        int dup = 0;
        for (uint32_t q = 0; q < cnt; q++) if (out[q] == o) { dup = 1; break; }
        if (!dup) {
            if (cnt < cap) out[cnt] = o;
            cnt++;
            if ((int64_t)cnt >= n) break;
        }
        j = (j + 1 == M) ? 0 : j + 1;
    }
    return cnt;
}

uint32_t orc_ring_lookupn_hash(orc_ring *r, uint32_t h, int64_t n, uint32_t *out, uint32_t cap) {
    ensure_sorted(r);
    return lookupn_sorted(r, h, n, out, cap);
}

static void key_at(const char *keys, uint32_t stride, const uint64_t *off, uint64_t i,
                   const uint8_t **p, size_t *n) {
    if (stride) { *p = (const uint8_t *)keys + i * stride; *n = stride; }
    else { *p = (const uint8_t *)keys + off[i]; *n = (size_t)(off[i + 1] - off[i]); }
}

void orc_ring_lookup_keys(orc_ring *r, const char *keys, uint32_t stride, const uint64_t *off,
                          uint64_t n, uint32_t *owners) {
    ensure_sorted(r);
    for (uint64_t i = 0; i < n; i++) {
        const uint8_t *p; size_t ln;
        key_at(keys, stride, off, i, &p, &ln);
        owners[i] = lookup_sorted(r, orc_hash32(p, ln));
    }
}

void orc_ring_lookupn_keys(orc_ring *r, const char *keys, uint32_t stride, const uint64_t *off,
                           uint64_t n, int64_t nrep, uint32_t *owners, uint8_t *counts) {
    ensure_sorted(r);
    uint32_t w = nrep > 0 ? (uint32_t)nrep : 1;
    uint32_t *tmp = (uint32_t *)malloc(sizeof(uint32_t) * (r->server_count + 2));
    for (uint64_t i = 0; i < n; i++) {
        const uint8_t *p; size_t ln;
        key_at(keys, stride, off, i, &p, &ln);
        uint32_t c = lookupn_sorted(r, orc_hash32(p, ln), nrep, tmp, r->server_count + 1);
        for (uint32_t q = 0; q < w; q++) owners[i * w + q] = q < c ? tmp[q] : NIL;
        if (counts) counts[i] = (uint8_t)(c > 255 ? 255 : c);
    }
    free(tmp);
}

typedef struct {
    orc_ring *r; const char *keys; uint32_t stride; uint64_t b, e; int64_t nrep;
    uint32_t *owners; uint8_t *counts;
} mt_arg;

static void *mt_body(void *p) {
    mt_arg *a = (mt_arg *)p;
    uint32_t w = a->nrep > 0 ? (uint32_t)a->nrep : 1;
    orc_ring_lookupn_keys(a->r, a->keys + a->b * a->stride, a->stride, NULL, a->e - a->b, a->nrep,
                          a->owners + a->b * w, a->counts ? a->counts + a->b : NULL);
    return NULL;
}

void orc_ring_lookupn_keys_mt(orc_ring *r, const char *keys, uint32_t stride, uint64_t n,
                              int64_t nrep, uint32_t *owners, uint8_t *counts, int threads) {
    ensure_sorted(r);
    if (threads < 1) threads = 1;
    pthread_t th[256];
    mt_arg args[256];
    if (threads > 256) threads = 256;
    for (int t = 0; t < threads; t++) {
        args[t].r = r; args[t].keys = keys; args[t].stride = stride; args[t].nrep = nrep;
        args[t].owners = owners; args[t].counts = counts;
        args[t].b = n * (uint64_t)t / (uint64_t)threads;
        args[t].e = n * (uint64_t)(t + 1) / (uint64_t)threads;
        pthread_create(&th[t], NULL, mt_body, &args[t]);
    }
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
}
