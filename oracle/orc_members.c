/*
 * orc_members.c — CPU restatement of ringpop's membership merge and checksum.
 * TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Restates:
 *   Member.evaluateUpdate / _isLocalOverride / _isOtherOverride  lib/membership/member.js:71-122,155-202
 *   Membership.update (sequential fold, new members, stash)      lib/membership/index.js:249-324
 *   Membership.set + mergeMembershipChangesets                   lib/membership/index.js:208-247, merge.js:22-51
 *   Membership.computeChecksum / generateChecksumString          lib/membership/index.js:48-75,100-123
 *   Membership.getJoinPosition (Math.random injected: Philox)    lib/membership/index.js:129-131
 * Members are identified by interned address ids 0..n_names-1 (names given up front).
 */
#include <stdint.h>
#include <stdio.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

static const char *const STATUS_STR[4] = {"alive", "suspect", "faulty", "leave"};
static const uint32_t STATUS_LEN[4] = {5, 7, 6, 5};

struct orc_members {
    uint32_t n_names;
    char *nb;
    uint64_t *noff;
    uint32_t local_id;
    int is_ready;
    uint32_t join_seed;
    uint64_t join_ctr;
    /* per id */
    uint8_t *exists, *status;
    int64_t *inc;
    /* members array order (ids): order[0 .. ord_n) is materialised; the inserts since then are
       logged (id, position at insert time) and placed by materialise_order, so a bulk fill of
       millions of members is O(n log n) instead of one memmove per insert */
    uint32_t *order;
    uint32_t count, ord_n;
    uint32_t *pend_id, *pend_pos;
    uint32_t pend_n;
    /* stash (ring of change batches, flattened) */
    uint32_t *st_id; uint8_t *st_status; int64_t *st_inc; uint32_t *st_batch_end;
    uint32_t st_n, st_cap, st_batches, st_bcap;
    int stash_nulled;
    /* checksum */
    int has_checksum;
    uint32_t checksum;
    uint32_t *sorted; /* ids sorted by address */
    char *buf;
    uint64_t buf_cap;
    /* compute_checksum_mt: per-thread segment buffers, kept across calls (fresh pages per call
       would serialise the threads on page faults) */
    char *tbuf[256];
    uint64_t tcap[256];
};

static int cmp_addr(const orc_members *m, uint32_t a, uint32_t b) {
    uint64_t la = m->noff[a + 1] - m->noff[a], lb = m->noff[b + 1] - m->noff[b];
    uint64_t l = la < lb ? la : lb;
    int c = memcmp(m->nb + m->noff[a], m->nb + m->noff[b], l);
    if (c) return c;
    return la < lb ? -1 : (la > lb ? 1 : 0);
}

static const orc_members *g_m;
static int qcmp(const void *x, const void *y) { return cmp_addr(g_m, *(const uint32_t *)x, *(const uint32_t *)y); }

orc_members *orc_members_new(const char *names, const uint32_t *off, uint32_t n, uint32_t local_id,
                             uint32_t join_seed) {
    orc_members *m = (orc_members *)calloc(1, sizeof(orc_members));
    m->n_names = n;
    m->nb = (char *)malloc(off[n] + 1);
    memcpy(m->nb, names, off[n]);
    m->noff = (uint64_t *)malloc(sizeof(uint64_t) * (n + 1));
    for (uint32_t i = 0; i <= n; i++) m->noff[i] = off[i];
    m->local_id = local_id;
    m->is_ready = 1;
    m->join_seed = join_seed;
    m->exists = (uint8_t *)calloc(n, 1);
    m->status = (uint8_t *)calloc(n, 1);
    m->inc = (int64_t *)calloc(n, sizeof(int64_t));
    m->order = (uint32_t *)malloc(sizeof(uint32_t) * (n + 1));
    m->pend_id = (uint32_t *)malloc(sizeof(uint32_t) * (n + 1));
    m->pend_pos = (uint32_t *)malloc(sizeof(uint32_t) * (n + 1));
    m->sorted = (uint32_t *)malloc(sizeof(uint32_t) * (n + 1));
    for (uint32_t i = 0; i < n; i++) m->sorted[i] = i;
    g_m = m;
    qsort(m->sorted, n, sizeof(uint32_t), qcmp);
    return m;
}

void orc_members_free(orc_members *m) {
    if (!m) return;
    free(m->nb); free(m->noff); free(m->exists); free(m->status); free(m->inc); free(m->order); free(m->pend_id); free(m->pend_pos);
    free(m->st_id); free(m->st_status); free(m->st_inc); free(m->st_batch_end);
    free(m->sorted); free(m->buf);
    for (int t = 0; t < 256; t++) free(m->tbuf[t]);
    free(m);
}

void orc_members_set_ready(orc_members *m, int ready) { m->is_ready = ready; }

/* Math.floor(Math.random() * members.length) with Math.random := philox_u32 / 2^32 */
static uint32_t join_position(orc_members *m) {
    uint32_t ctr[4] = {(uint32_t)m->join_ctr, (uint32_t)(m->join_ctr >> 32), 0, 0};
    uint32_t key[2] = {m->join_seed, 0x4a4f494eu /* 'JOIN' */};
    uint32_t r[4];
    orc_philox4x32_10(ctr, key, r);
    m->join_ctr++;
    return (uint32_t)(((uint64_t)r[0] * m->count) >> 32);
}

/* members.splice(pos, 0, member) (index.js:286-291), logged; each id is inserted at most once */
static void insert_member(orc_members *m, uint32_t id, uint8_t st, int64_t inc, uint32_t pos) {
    m->exists[id] = 1;
    m->status[id] = st;
    m->inc[id] = inc;
    m->pend_id[m->pend_n] = id;
    m->pend_pos[m->pend_n] = pos;
    m->pend_n++;
    m->count++;
}

/* The array the logged splices produce: taken in reverse, a splice at position p owns the p-th
 * (0-based) slot not owned by a later splice (a Fenwick tree over the final slots finds it); the
 * materialised members fill the slots left, in their order. */
static void materialise_order(orc_members *m) {
    const uint32_t P = m->pend_n, N = m->count;
    if (P == 0) return;
    uint32_t *fw = (uint32_t *)calloc(N + 1, sizeof(uint32_t));
    uint32_t *out = (uint32_t *)malloc(sizeof(uint32_t) * (N + 1));
    uint8_t *taken = (uint8_t *)calloc(N, 1);
    for (uint32_t i = 1; i <= N; i++) { /* all slots free: fw = prefix counts of ones */
        fw[i] += 1;
        const uint32_t j = i + (i & (0u - i));
        if (j <= N) fw[j] += fw[i];
    }
    uint32_t top = 1;
    while ((top << 1) <= N) top <<= 1;
    for (uint32_t q = P; q-- > 0;) {
        uint32_t want = m->pend_pos[q] + 1, at = 0; /* the want-th free slot (1-based) */
        for (uint32_t b = top; b; b >>= 1)
            if (at + b <= N && fw[at + b] < want) {
                at += b;
                want -= fw[at];
            }
        out[at] = m->pend_id[q]; /* slot at (0-based) */
        taken[at] = 1;
        for (uint32_t i = at + 1; i <= N; i += i & (0u - i)) fw[i] -= 1;
    }
    uint32_t r = 0;
    for (uint32_t i = 0; i < N; i++)
        if (!taken[i]) out[i] = m->order[r++];
    memcpy(m->order, out, sizeof(uint32_t) * N);
    m->ord_n = N;
    m->pend_n = 0;
    free(fw);
    free(out);
    free(taken);
}

/* Member._isOtherOverride (member.js:171-202) */
static int other_override(uint8_t cur, int64_t cur_inc, uint8_t st, int64_t inc) {
    switch (st) {
    case 0: return inc > cur_inc;                                        /* isAliveOverride */
    case 1: return (cur == 1 && inc > cur_inc) || (cur == 2 && inc > cur_inc) ||
                   (cur == 0 && inc >= cur_inc);                         /* isSuspectOverride */
    case 2: return (cur == 1 && inc >= cur_inc) || (cur == 2 && inc > cur_inc) ||
                   (cur == 0 && inc >= cur_inc);                         /* isFaultyOverride */
    case 3: return cur != 3 && inc >= cur_inc;                           /* isLeaveOverride */
    }
    return 0;
}

/* String(inc) for an integral Number (decimal, '-' for negatives); returns the length. */
static uint32_t fmt_i64(char *o, int64_t v) {
    char t[24];
    uint32_t n = 0;
    uint64_t u = v < 0 ? (uint64_t)(-(v + 1)) + 1 : (uint64_t)v;
    do {
        t[n++] = (char)('0' + (u % 10));
        u /= 10;
    } while (u);
    uint32_t w = 0;
    if (v < 0) o[w++] = '-';
    while (n) o[w++] = t[--n];
    return w;
}

/* generateChecksumString's pieces (index.js:115-120) of the members sorted[k0..k1), each
 * followed by ';' (the caller drops the string's last ';'). Returns the bytes written. */
static uint64_t format_pieces(const orc_members *m, uint32_t k0, uint32_t k1, char *o) {
    uint64_t w = 0;
    for (uint32_t k = k0; k < k1; k++) {
        uint32_t id = m->sorted[k];
        if (!m->exists[id]) continue;
        uint64_t ln = m->noff[id + 1] - m->noff[id];
        memcpy(o + w, m->nb + m->noff[id], ln);
        w += ln;
        memcpy(o + w, STATUS_STR[m->status[id]], STATUS_LEN[m->status[id]]);
        w += STATUS_LEN[m->status[id]];
        w += fmt_i64(o + w, m->inc[id]);
        o[w++] = ';';
    }
    return w;
}

static void ensure_buf(orc_members *m) {
    uint64_t need = 0;
    for (uint32_t i = 0; i < m->n_names; i++)
        if (m->exists[i]) need += (m->noff[i + 1] - m->noff[i]) + 7 + 21 + 1;
    if (need + 1 > m->buf_cap) {
        m->buf_cap = need + 64;
        m->buf = (char *)realloc(m->buf, m->buf_cap);
    }
}

static void compute_checksum(orc_members *m) {
    ensure_buf(m);
    uint64_t o = format_pieces(m, 0, m->n_names, m->buf);
    if (o) o--; /* the joined string has no trailing ';' */
    m->checksum = orc_hash32((const uint8_t *)m->buf, o);
    m->has_checksum = 1;
}

/* The same checksum with the string formatted by T threads (segments of the address order in
 * private buffers, then copied into place); the hash itself is one serial chain. */
typedef struct {
    const orc_members *m;
    uint32_t k0, k1;
    char *tmp;
    uint64_t len, off;
    char *dst;
} fmt_job;

static void *fmt_worker(void *p) {
    fmt_job *j = (fmt_job *)p;
    j->len = format_pieces(j->m, j->k0, j->k1, j->tmp);
    return NULL;
}

static void *copy_worker(void *p) {
    fmt_job *j = (fmt_job *)p;
    memcpy(j->dst + j->off, j->tmp, j->len);
    return NULL;
}

/* A persistent pool for the *_mt paths: T - 1 workers parked on a barrier, the caller is
 * thread 0. Creating threads per phase (three phases per batch) cost more than the phases
 * (bench C3 baseline, round 4: 16 threads slower than 1). */
typedef void *(*pool_fn)(void *);
static struct {
    int T;
    pthread_t th[256];
    pthread_barrier_t start, done;
    pool_fn fn;
    void *arg[256];
    int quit;
} g_pool;

static void *pool_main(void *p) {
    const int t = (int)(intptr_t)p;
    for (;;) {
        pthread_barrier_wait(&g_pool.start);
        if (g_pool.quit) return NULL;
        g_pool.fn(g_pool.arg[t]);
        pthread_barrier_wait(&g_pool.done);
    }
}

static void pool_stop(void) {
    if (g_pool.T <= 1) return;
    g_pool.quit = 1;
    pthread_barrier_wait(&g_pool.start);
    for (int t = 1; t < g_pool.T; t++) pthread_join(g_pool.th[t], NULL);
    pthread_barrier_destroy(&g_pool.start);
    pthread_barrier_destroy(&g_pool.done);
    g_pool.T = 0;
    g_pool.quit = 0;
}

/* fn(args[t]) for t < T on the pool, the caller running t = 0; returns when all are done. */
static void pool_run(int T, pool_fn fn, void *const *args) {
    if (T <= 1) {
        fn(args[0]);
        return;
    }
    if (g_pool.T != T) {
        pool_stop();
        pthread_barrier_init(&g_pool.start, NULL, (unsigned)T);
        pthread_barrier_init(&g_pool.done, NULL, (unsigned)T);
        g_pool.T = T;
        for (int t = 1; t < T; t++) pthread_create(&g_pool.th[t], NULL, pool_main, (void *)(intptr_t)t);
    }
    g_pool.fn = fn;
    for (int t = 0; t < T; t++) g_pool.arg[t] = args[t];
    pthread_barrier_wait(&g_pool.start);
    fn(args[0]);
    pthread_barrier_wait(&g_pool.done);
}

static void compute_checksum_mt(orc_members *m, int T) {
    if (T <= 1 || m->n_names < 4096) {
        compute_checksum(m);
        return;
    }
    ensure_buf(m);
    fmt_job jobs[256];
    void *args[256] = {0};
    const uint32_t per = (m->n_names + T - 1) / T;
    for (int t = 0; t < T; t++) {
        uint32_t k0 = (uint32_t)t * per, k1 = k0 + per;
        if (k0 > m->n_names) k0 = m->n_names;
        if (k1 > m->n_names) k1 = m->n_names;
        uint64_t cap = 0;
        for (uint32_t k = k0; k < k1; k++) cap += (m->noff[m->sorted[k] + 1] - m->noff[m->sorted[k]]) + 7 + 21 + 1;
        if (cap + 1 > m->tcap[t]) {
            free(m->tbuf[t]);
            m->tcap[t] = cap + 1;
            m->tbuf[t] = (char *)malloc(m->tcap[t]);
        }
        jobs[t] = (fmt_job){m, k0, k1, m->tbuf[t], 0, 0, m->buf};
        args[t] = &jobs[t];
    }
    pool_run(T, fmt_worker, args);
    uint64_t o = 0;
    for (int t = 0; t < T; t++) {
        jobs[t].off = o;
        o += jobs[t].len;
    }
    pool_run(T, copy_worker, args);
    if (o) o--;
    m->checksum = orc_hash32((const uint8_t *)m->buf, o);
    m->has_checksum = 1;
}

/* Membership.update (lib/membership/index.js:249-324). Returns the number of applied updates;
 * applied_out[k] flags them, new_*_out[k] hold the applied (possibly rewritten) update. */
uint32_t orc_members_update(orc_members *m, const uint32_t *ids, const uint8_t *status, const int64_t *inc,
                            uint32_t k, int is_local, int64_t now_ms, uint8_t *applied_out,
                            uint8_t *new_status_out, int64_t *new_inc_out) {
    if (k == 0) return 0;
    if (!is_local && !m->is_ready) { /* stash (259-265) */
        if (!m->stash_nulled) {
            if (m->st_n + k > m->st_cap) {
                while (m->st_n + k > m->st_cap) m->st_cap = m->st_cap ? 2 * m->st_cap : 1024;
                m->st_id = (uint32_t *)realloc(m->st_id, sizeof(uint32_t) * m->st_cap);
                m->st_status = (uint8_t *)realloc(m->st_status, m->st_cap);
                m->st_inc = (int64_t *)realloc(m->st_inc, sizeof(int64_t) * m->st_cap);
            }
            if (m->st_batches + 1 > m->st_bcap) {
                m->st_bcap = m->st_bcap ? 2 * m->st_bcap : 64;
                m->st_batch_end = (uint32_t *)realloc(m->st_batch_end, sizeof(uint32_t) * m->st_bcap);
            }
            memcpy(m->st_id + m->st_n, ids, sizeof(uint32_t) * k);
            memcpy(m->st_status + m->st_n, status, k);
            memcpy(m->st_inc + m->st_n, inc, sizeof(int64_t) * k);
            m->st_n += k;
            m->st_batch_end[m->st_batches++] = m->st_n;
        }
        if (applied_out) memset(applied_out, 0, k);
        return 0;
    }
    uint32_t napplied = 0;
    for (uint32_t i = 0; i < k; i++) { /* (272-304) sequential fold */
        uint32_t id = ids[i];
        uint8_t st = status[i];
        int64_t in = inc[i];
        int applied = 0;
        if (!m->exists[id]) { /* new member: verbatim, random join position (277-291) */
            insert_member(m, id, st, in, join_position(m));
            applied = 1;
        } else if (id == m->local_id && (st == 1 || st == 2)) { /* _isLocalOverride (155-169) */
            st = 0;
            in = now_ms;
            applied = 1;
        } else if (other_override(m->status[id], m->inc[id], st, in)) {
            applied = 1;
        }
        if (applied) {
            m->status[id] = st;
            m->inc[id] = in;
            napplied++;
        }
        if (applied_out) applied_out[i] = (uint8_t)applied;
        if (new_status_out) new_status_out[i] = st;
        if (new_inc_out) new_inc_out[i] = in;
    }
    if (napplied) compute_checksum(m); /* (306-309) */
    return napplied;
}

/* The same fold on T threads for a batch that creates no member (the C3 CPU baseline on all
 * host cores): the fold is order-sensitive only within one address, so thread t folds, in
 * arrival order, the changes whose id % T == t; the checksum is then computed once (serial). */
typedef struct {
    orc_members *m;
    const uint32_t *ids;
    const uint8_t *status;
    const int64_t *inc;
    uint32_t k, lo, hi; /* this thread's ids: [lo, hi) */
    int64_t now_ms;
    uint8_t *applied;
    uint32_t napplied;
} fold_job;

static void *fold_worker(void *p) {
    fold_job *j = (fold_job *)p;
    orc_members *m = j->m;
    for (uint32_t i = 0; i < j->k; i++) {
        uint32_t id = j->ids[i];
        if (id < j->lo || id >= j->hi) continue; /* contiguous id ranges: no false sharing */
        uint8_t st = j->status[i];
        int64_t in = j->inc[i];
        int applied = 0;
        if (id == m->local_id && (st == 1 || st == 2)) {
            st = 0;
            in = j->now_ms;
            applied = 1;
        } else if (other_override(m->status[id], m->inc[id], st, in)) {
            applied = 1;
        }
        if (applied) {
            m->status[id] = st;
            m->inc[id] = in;
            j->napplied++;
        }
        if (j->applied) j->applied[i] = (uint8_t)applied;
    }
    return NULL;
}

uint32_t orc_members_update_mt(orc_members *m, const uint32_t *ids, const uint8_t *status, const int64_t *inc,
                               uint32_t k, int64_t now_ms, int threads, uint8_t *applied_out) {
    for (uint32_t i = 0; i < k; i++)
        if (!m->exists[ids[i]] || !m->is_ready) return 0xFFFFFFFFu; /* only the no-create, ready case */
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    fold_job jobs[256];
    void *args[256] = {0};
    const uint32_t per = (m->n_names + threads - 1) / threads;
    for (int t = 0; t < threads; t++) {
        const uint32_t lo = (uint32_t)t * per, hi = lo + per;
        jobs[t] = (fold_job){m, ids, status, inc, k, lo < m->n_names ? lo : m->n_names,
                             hi < m->n_names ? hi : m->n_names, now_ms, applied_out, 0};
        args[t] = &jobs[t];
    }
    pool_run(threads, fold_worker, args);
    uint32_t napplied = 0;
    for (int t = 0; t < threads; t++) napplied += jobs[t].napplied;
    if (napplied) compute_checksum_mt(m, threads);
    return napplied;
}

/* Membership.set (208-247): mergeMembershipChangesets (merge.js:22-51) over the stash, then
 * append in first-seen order, checksum once. Returns the number of members set. */
uint32_t orc_members_set(orc_members *m) {
    if (m->is_ready || m->stash_nulled || m->st_n == 0) return 0;
    uint32_t *best = (uint32_t *)malloc(sizeof(uint32_t) * m->n_names);
    uint32_t *seen = (uint32_t *)malloc(sizeof(uint32_t) * (m->st_n + 1));
    uint32_t nseen = 0;
    for (uint32_t i = 0; i < m->n_names; i++) best[i] = 0xFFFFFFFFu;
    for (uint32_t i = 0; i < m->st_n; i++) {
        uint32_t id = m->st_id[i];
        if (id == m->local_id) continue; /* skip whoami */
        if (best[id] == 0xFFFFFFFFu) { best[id] = i; seen[nseen++] = id; }
        else if (m->st_inc[best[id]] < m->st_inc[i]) best[id] = i; /* strictly greater wins */
    }
    for (uint32_t j = 0; j < nseen; j++) {
        uint32_t id = seen[j];
        uint32_t i = best[id];
        if (m->exists[id]) { m->status[id] = m->st_status[i]; m->inc[id] = m->st_inc[i]; continue; }
        insert_member(m, id, m->st_status[i], m->st_inc[i], m->count);
    }
    free(best);
    free(seen);
    m->stash_nulled = 1;
    compute_checksum(m);
    return nseen;
}

int orc_members_checksum(const orc_members *m, uint32_t *out) {
    if (!m->has_checksum) return 0;
    *out = m->checksum;
    return 1;
}

uint32_t orc_members_count(const orc_members *m) { return m->count; }

void orc_members_order(orc_members *m, uint32_t *ids_out) {
    materialise_order(m);
    memcpy(ids_out, m->order, sizeof(uint32_t) * m->count);
}

int orc_members_get(const orc_members *m, uint32_t id, uint8_t *status, int64_t *inc) {
    if (id >= m->n_names || !m->exists[id]) return 0;
    *status = m->status[id];
    *inc = m->inc[id];
    return 1;
}

/* Write the checksum string (generateChecksumString) into buf (cap bytes); returns length. */
uint64_t orc_members_checksum_string(orc_members *m, char *buf, uint64_t cap) {
    compute_checksum(m);
    uint64_t n = 0;
    /* recompute length: buf holds the last string */
    for (uint32_t k = 0, first = 1; k < m->n_names; k++) {
        uint32_t id = m->sorted[k];
        if (!m->exists[id]) continue;
        char tmp[32];
        n += (first ? 0 : 1) + (m->noff[id + 1] - m->noff[id]) + STATUS_LEN[m->status[id]] +
             (uint64_t)sprintf(tmp, "%lld", (long long)m->inc[id]);
        first = 0;
    }
    if (buf) memcpy(buf, m->buf, n < cap ? n : cap);
    return n;
}

/* Membership.computeChecksum on T threads (bench.py's CPU baseline probes it). */
void orc_members_compute_checksum_mt(orc_members *m, int threads) { compute_checksum_mt(m, threads); }
