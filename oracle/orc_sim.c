/*
 * orc_sim.c — CPU restatement of ringpop's gossip protocol as a deterministic round model.
 * TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Every node is a full ringpop membership view (lib/membership), dissemination buffer
 * (lib/gossip/dissemination.js), ring membership (lib/ring, for maxPiggybackCount),
 * iterator (lib/membership/iterator.js) and suspicion timers (lib/gossip/suspicion.js),
 * wired as lib/on_membership_event.js does. The reference runs these asynchronously over
 * TChannel; the model fixes one order (the "round model", DESIGN.md §SWIM round model), and
 * tests/golden/ref_sim.js drives the REFERENCE modules through the same order so per-round
 * checksums can be compared bit-for-bit.
 *
 * Round r (nodes that are down neither act nor answer):
 *   events  scheduled by the caller before the round (orc_sim_event): a node goes down
 *      (SIGSTOP / crash, scripts/tick-cluster.js:417-470), comes back with its state intact
 *      (SIGCONT), or leaves: makeLeave(whoami, own incarnation) (server/admin/member.js:92-93,
 *      lib/membership/index.js:191-195), as benchmarks/convergence-time/scenarios/ send
 *   A  each node v: t = iterator.next() (iterator.js:28-51); ping = issueAsSender()
 *      (dissemination.js:78-84) + v's checksum + v's incarnation (ping-sender.js:70-76)
 *   B  each live target j, its pings in sender order: update(changes) (ping.js:44), response
 *      = issueAsReceiver(sender, senderInc, senderChecksum) (ping.js:46-49)
 *   C  each sender with a live target: update(response) twice (ping-sender.js:38,
 *      gossip/index.js:165)
 *   D1 each sender with a dead target: k=3 helpers = getRandomPingableMembers(3, [t])
 *      (ping-req-sender.js:293-296); none -> makeSuspect(t, t.inc) (162-169); else one
 *      issueAsSender() per leg (ping-req-sender.js:75-81)
 *   D2 each helper, legs in (sender, leg) order: dead helper -> network error; else
 *      update(changes) (ping-req.js:45), its own ping of t: issueAsSender() (ping-req.js:50),
 *      t is dead -> pingStatus false; response = issueAsReceiver(...) (ping-req.js:61-66)
 *   D3 each sender, legs in order: update(response) for answered legs (ping-req-sender.js:130);
 *      if any leg answered with a bad ping status: makeSuspect(t, t.inc) (239-268)
 *   E  each node: suspicion timers due this round fire in member-id order:
 *      makeFaulty(addr, inc captured at start) (suspicion.js:67-70)
 * Randomness: iterator shuffles and ping-req samples are Philox streams (SHUF, SAMP);
 * Date.now() (local override, member.js:80) is now0 + 200 * round.
 *
 * Representation (sized for the C5 config, 10^5 full views, on a 64 GB host): a view is the
 * all-alive bootstrap state plus a sparse table of the members whose row ever changed (view
 * row, ring bit, dissemination entry, suspicion timer), indexed by an open-addressing hash. A
 * view's checksum string is the base string with the deviated pieces substituted; it is
 * hashed lazily when read, and identical views (same deviated pieces) share one hash through a
 * memo keyed by a 128-bit fingerprint of the pieces. The members-array order is kept whole
 * when N^2 * 4 bytes fit ORC_SIM_ORDER_BYTES (default 2 GiB), else as a window regenerated from
 * the Philox shuffles. Phases run on a pthread pool: every phase's per-node work is
 * independent once pings / legs are grouped by receiver (in sender order).
 */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

#define TAG_SHUF 0x53485546u
#define TAG_SAMP 0x53414d50u
#define TAG_JOIN 0x4a4f494eu
#define NONE 0xFFFFFFFFu
#define WIN 1024u

typedef struct {
    uint32_t addr;
    uint8_t st;
    int64_t inc;
    uint32_t src;     /* NONE = undefined */
    int64_t srcinc;   /* 0 = undefined */
} chg;

typedef struct {
    chg *v;
    uint32_t n, cap;
} chgvec;

static void cv_push(chgvec *c, chg x) {
    if (c->n == c->cap) {
        c->cap = c->cap ? c->cap * 2 : 16;
        c->v = (chg *)realloc(c->v, sizeof(chg) * c->cap);
    }
    c->v[c->n++] = x;
}

/* A member whose row in this view ever left the bootstrap state (alive, inc0, in the ring). */
typedef struct {
    uint32_t addr;
    uint8_t st, in_ring, d_on, t_on;
    uint32_t d_cnt, d_src;  /* dissemination entry: piggybackCount, source */
    int64_t inc, d_srcinc;
    int64_t deadline, s_inc; /* suspicion timer: round it fires at, captured incarnation */
} ent;

typedef struct {
    ent *e;
    uint32_t ne, ecap;
    uint32_t *ix; /* addr -> entry index + 1 (0 = empty); linear probing */
    uint32_t ixcap;
    uint32_t max_piggy, ring_count;
    int64_t it_idx;
    uint32_t n_shuffles;
    uint32_t *order; /* whole members array, or the window [w0, w0 + WIN) */
    uint32_t *base;  /* the members array a join's set() built (NULL: the bootstrap one) */
    uint32_t w0;
    uint32_t checksum;
    uint8_t dirty;
} node;

/* per-worker scratch */
typedef struct {
    uint32_t *perm, *vis, *cand;
    uint64_t *bits;
    char *buf;
    uint64_t bufcap;
    uint32_t *dk;   /* deviated ranks */
    uint32_t dkcap;
    chg *app;
    uint32_t appcap;
    chgvec scratch;
} wctx;

#define MEMO_BITS 20
typedef struct {
    uint64_t a, b;
    uint32_t ck, ok;
} memo_slot;

struct orc_sim {
    uint32_t N;
    uint32_t seed;
    uint32_t susp_rounds;
    int64_t now0;
    int64_t round;
    uint8_t *down;    /* not acting this round */
    uint8_t *left;    /* sent makeLeave */
    uint8_t *stopped; /* own status became leave: gossip.stop() + suspicion.stopAll() */
    char *nb;
    uint64_t *noff;
    int64_t *inc0;
    uint32_t *sorted; /* ids in address order */
    uint32_t *rank;
    char *sbase;      /* all-alive checksum string */
    uint64_t *boff;   /* [N+1] piece offsets in sbase */
    uint32_t base_ck;
    int full_order;
    node *nodes;
    int threads;
    wctx *ctx;
    memo_slot *memo;
    pthread_mutex_t memo_mu[64];
    /* per-round scratch */
    int64_t *target;
    chgvec *ping, *resp;
    uint32_t *ping_ck;
    int64_t *ping_inc;
    uint32_t *csr_off, *csr_idx;
    uint32_t (*helpers)[3];
    uint32_t *nh;
    chgvec (*legs)[3], (*lresp)[3];
    uint8_t (*lok)[3];
    uint32_t *leg_ck;
    int64_t *leg_inc;
    /* stats */
    uint64_t stat_pings, stat_pingreqs, stat_fullsyncs, stat_applied;
};

static const char *const ST[4] = {"alive", "suspect", "faulty", "leave"};
static const uint32_t STL[4] = {5, 7, 6, 5};

static uint32_t philox_u32(uint32_t seed, uint32_t tag, uint32_t c0, uint32_t c1, uint32_t c2) {
    uint32_t ctr[4] = {c0, c1, c2, 0}, key[2] = {seed, tag}, r[4];
    orc_philox4x32_10(ctr, key, r);
    return r[0];
}

static int digits(uint32_t n) {
    int d = 0;
    while (n) { d++; n /= 10; }
    return d;
}

static void add_u64(uint64_t *p, uint64_t v) { __atomic_fetch_add(p, v, __ATOMIC_RELAXED); }

/* ---- thread pool: fn(s, i, ctx) for i in [0, n), dynamic chunks */
typedef void (*work_fn)(orc_sim *s, uint32_t i, wctx *c);
typedef struct {
    orc_sim *s;
    work_fn fn;
    uint32_t n, chunk;
    uint32_t next;
    int t;
} job;
typedef struct {
    job *j;
    int t;
} jarg;

static void *worker(void *p) {
    jarg *a = (jarg *)p;
    job *j = a->j;
    for (;;) {
        uint32_t b = __atomic_fetch_add(&j->next, j->chunk, __ATOMIC_RELAXED);
        if (b >= j->n) break;
        uint32_t e = b + j->chunk < j->n ? b + j->chunk : j->n;
        for (uint32_t i = b; i < e; i++) j->fn(j->s, i, &j->s->ctx[a->t]);
    }
    return NULL;
}

static void parallel_for(orc_sim *s, uint32_t n, uint32_t chunk, work_fn fn) {
    job j = {s, fn, n, chunk ? chunk : 1, 0, 0};
    int T = s->threads;
    if (T <= 1 || n <= j.chunk) {
        for (uint32_t i = 0; i < n; i++) fn(s, i, &s->ctx[0]);
        return;
    }
    pthread_t th[256];
    jarg args[256];
    if (T > 256) T = 256;
    for (int t = 0; t < T; t++) {
        args[t].j = &j;
        args[t].t = t;
        pthread_create(&th[t], NULL, worker, &args[t]);
    }
    for (int t = 0; t < T; t++) pthread_join(th[t], NULL);
}

/* ---- a view's sparse rows */
static ent *find(const node *nd, uint32_t a) {
    if (!nd->ixcap) return NULL;
    uint32_t m = nd->ixcap - 1, h = (a * 0x9E3779B1u) & m;
    for (;;) {
        uint32_t x = nd->ix[h];
        if (!x) return NULL;
        if (nd->e[x - 1].addr == a) return &nd->e[x - 1];
        h = (h + 1) & m;
    }
}

static void ix_put(node *nd, uint32_t a, uint32_t idx1) {
    uint32_t m = nd->ixcap - 1, h = (a * 0x9E3779B1u) & m;
    while (nd->ix[h]) h = (h + 1) & m;
    nd->ix[h] = idx1;
}

/* the entry of a (created in the bootstrap state if absent) */
static ent *get(const orc_sim *s, node *nd, uint32_t a) {
    ent *x = find(nd, a);
    if (x) return x;
    if (nd->ne == nd->ecap) {
        nd->ecap = nd->ecap ? nd->ecap * 2 : 8;
        nd->e = (ent *)realloc(nd->e, sizeof(ent) * nd->ecap);
    }
    if (2 * (nd->ne + 1) > nd->ixcap) {
        uint32_t nc = nd->ixcap ? nd->ixcap * 2 : 16;
        while (2 * (nd->ne + 1) > nc) nc *= 2;
        free(nd->ix);
        nd->ix = (uint32_t *)calloc(nc, 4);
        nd->ixcap = nc;
        for (uint32_t i = 0; i < nd->ne; i++) ix_put(nd, nd->e[i].addr, i + 1);
    }
    ent *e = &nd->e[nd->ne];
    memset(e, 0, sizeof *e);
    e->addr = a;
    e->st = 0;
    e->inc = s->inc0[a];
    e->in_ring = 1;
    e->deadline = -1;
    ix_put(nd, a, ++nd->ne);
    return e;
}

static uint8_t st_of(const node *nd, uint32_t a) {
    const ent *e = find(nd, a);
    return e ? e->st : 0;
}

static int64_t inc_of(const orc_sim *s, const node *nd, uint32_t a) {
    const ent *e = find(nd, a);
    return e ? e->inc : s->inc0[a];
}

/* ---- members array (Membership.members) and _.shuffle */
static void perm_initial(uint32_t N, uint32_t v, uint32_t *o) {
    /* after bootstrap: self (makeAlive, index.js:270) then set() in id order */
    o[0] = v;
    for (uint32_t i = 0, k = 1; i < N; i++)
        if (i != v) o[k++] = i;
}

/* _.shuffle replaced by Fisher-Yates over a Philox stream (SHUF, shuffle#, i, view) */
static void perm_shuffle(const orc_sim *s, uint32_t v, uint32_t sh, uint32_t *o) {
    for (uint32_t i = s->N - 1; i >= 1; i--) {
        uint32_t r = philox_u32(s->seed, TAG_SHUF, sh, i, v);
        uint32_t j = (uint32_t)(((uint64_t)r * (i + 1)) >> 32);
        uint32_t t = o[i]; o[i] = o[j]; o[j] = t;
    }
}

/* the whole current members array of view v (pointer valid until the next call) */
static const uint32_t *perm_full(const orc_sim *s, uint32_t v, const node *nd, wctx *c) {
    if (s->full_order) return nd->order;
    if (nd->base)
        memcpy(c->perm, nd->base, 4ull * s->N);
    else
        perm_initial(s->N, v, c->perm);
    for (uint32_t sh = 0; sh < nd->n_shuffles; sh++) perm_shuffle(s, v, sh, c->perm);
    return c->perm;
}

static void set_window(const orc_sim *s, node *nd, const uint32_t *perm, uint32_t w0) {
    uint32_t n = s->N - w0 < WIN ? s->N - w0 : WIN;
    nd->w0 = w0;
    memcpy(nd->order, perm + w0, 4ull * n);
}

/* Membership.shuffle (membership/index.js:326-328) */
static void node_shuffle(orc_sim *s, uint32_t v, node *nd, wctx *c) {
    if (s->full_order) {
        perm_shuffle(s, v, nd->n_shuffles++, nd->order);
        return;
    }
    nd->n_shuffles++;
    set_window(s, nd, perm_full(s, v, nd, c), 0);
}

static uint32_t order_at(orc_sim *s, uint32_t v, node *nd, uint32_t k, wctx *c) {
    if (s->full_order) return nd->order[k];
    if (k < nd->w0 || k >= nd->w0 + WIN) set_window(s, nd, perm_full(s, v, nd, c), k);
    return nd->order[k - nd->w0];
}

static int pingable(const node *nd, uint32_t v, uint32_t m) {
    if (m == v) return 0;
    uint8_t st = st_of(nd, m);
    return st == 0 || st == 1; /* isPingable (index.js:173-177) */
}

/* MembershipIterator.next (iterator.js:28-51); -1 = no pingable member. The loop runs until
 * every distinct address has been visited; before the walk wraps its positions are distinct,
 * after a wrap (a reshuffle) a bitmap tracks distinct visits. */
static int64_t iter_next(orc_sim *s, uint32_t v, node *nd, wctx *c) {
    const uint32_t N = s->N;
    uint32_t nseen = 0, steps = 0;
    int wrapped = 0;
    while (nseen < N) {
        nd->it_idx++;
        if (nd->it_idx >= (int64_t)N) {
            nd->it_idx = 0;
            if (!wrapped) {
                memset(c->bits, 0, 8ull * ((N + 63) / 64));
                for (uint32_t q = 0; q < steps; q++) c->bits[c->vis[q] >> 6] |= 1ull << (c->vis[q] & 63);
                wrapped = 1;
            }
            node_shuffle(s, v, nd, c);
        }
        uint32_t m = order_at(s, v, nd, (uint32_t)nd->it_idx, c);
        if (!wrapped) {
            c->vis[steps] = m;
            nseen++;
        } else if (!(c->bits[m >> 6] & (1ull << (m & 63)))) {
            c->bits[m >> 6] |= 1ull << (m & 63);
            nseen++;
        }
        steps++;
        if (pingable(nd, v, m)) return m;
    }
    return -1;
}

/* ---- checksums: Membership.computeChecksum (lib/membership/index.js:48-75) +
 * generateChecksumString (100-123): members sorted by address, address + status + inc, ';' */
static int cmp_u32(const void *x, const void *y) {
    uint32_t a = *(const uint32_t *)x, b = *(const uint32_t *)y;
    return a < b ? -1 : a > b;
}

static int dec(int64_t v, char *out) {
    char tmp[24];
    int n = 0, neg = v < 0, o = 0;
    uint64_t u = neg ? (uint64_t)(-(v + 1)) + 1 : (uint64_t)v;
    do { tmp[n++] = (char)('0' + u % 10); u /= 10; } while (u);
    if (neg) out[o++] = '-';
    while (n) out[o++] = tmp[--n];
    return o;
}

static uint64_t mix64(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}

static uint32_t view_checksum(orc_sim *s, node *nd, wctx *c) {
    /* deviated pieces, in address order */
    uint32_t nd_ = 0;
    if (c->dkcap < nd->ne) {
        c->dkcap = nd->ne * 2;
        c->dk = (uint32_t *)realloc(c->dk, 4ull * c->dkcap);
    }
    for (uint32_t i = 0; i < nd->ne; i++) {
        const ent *e = &nd->e[i];
        if (e->st != 0 || e->inc != s->inc0[e->addr]) c->dk[nd_++] = s->rank[e->addr];
    }
    if (!nd_) return s->base_ck;
    qsort(c->dk, nd_, 4, cmp_u32);
    uint64_t fa = 0x9E3779B97F4A7C15ull ^ nd_, fb = 0xC2B2AE3D27D4EB4Full + nd_;
    for (uint32_t q = 0; q < nd_; q++) {
        const ent *e = find(nd, s->sorted[c->dk[q]]);
        uint64_t w = ((uint64_t)c->dk[q] << 2) | e->st;
        fa = mix64(fa ^ w) + (uint64_t)e->inc;
        fb = mix64(fb + (uint64_t)e->inc * 0x100000001B3ull) ^ w;
    }
    fa = mix64(fa);
    fb = mix64(fb ^ fa);
    memo_slot *m = &s->memo[fa & ((1u << MEMO_BITS) - 1)];
    pthread_mutex_t *mu = &s->memo_mu[fa & 63];
    pthread_mutex_lock(mu);
    if (m->ok && m->a == fa && m->b == fb) {
        uint32_t ck = m->ck;
        pthread_mutex_unlock(mu);
        return ck;
    }
    pthread_mutex_unlock(mu);
    uint64_t need = s->boff[s->N] + 32ull * nd_ + 64;
    if (c->bufcap < need) {
        c->bufcap = need * 2;
        c->buf = (char *)realloc(c->buf, c->bufcap);
    }
    uint64_t o = 0, b = 0;
    for (uint32_t q = 0; q < nd_; q++) {
        uint32_t k = c->dk[q], a = s->sorted[k];
        const ent *e = find(nd, a);
        memcpy(c->buf + o, s->sbase + b, s->boff[k] - b);
        o += s->boff[k] - b;
        uint64_t ln = s->noff[a + 1] - s->noff[a];
        memcpy(c->buf + o, s->nb + s->noff[a], ln);
        o += ln;
        memcpy(c->buf + o, ST[e->st], STL[e->st]);
        o += STL[e->st];
        o += (uint64_t)dec(e->inc, c->buf + o);
        if (k + 1 < s->N) c->buf[o++] = ';';
        b = s->boff[k + 1];
    }
    memcpy(c->buf + o, s->sbase + b, s->boff[s->N] - b);
    o += s->boff[s->N] - b;
    uint32_t ck = orc_hash32((const uint8_t *)c->buf, o);
    pthread_mutex_lock(mu);
    m->a = fa; m->b = fb; m->ck = ck; m->ok = 1;
    pthread_mutex_unlock(mu);
    return ck;
}

static uint32_t checksum(orc_sim *s, node *nd, wctx *c) {
    if (nd->dirty) {
        nd->checksum = view_checksum(s, nd, c);
        nd->dirty = 0;
    }
    return nd->checksum;
}

/* ---- Dissemination._issueAs (dissemination.js:133-176). filter: sender id or NONE. */
static void issue(orc_sim *s, node *nd, uint32_t sender, int64_t sender_inc, chgvec *out) {
    out->n = 0;
    for (uint32_t i = 0; i < nd->ne; i++) {
        ent *e = &nd->e[i];
        if (!e->d_on) continue;
        if (sender != NONE && sender_inc != 0 && e->d_src != NONE && e->d_srcinc != 0 && e->d_src == sender &&
            e->d_srcinc == sender_inc)
            continue; /* filtered: no count bump (150-153) */
        e->d_cnt += 1;
        if (e->d_cnt > nd->max_piggy) { e->d_on = 0; continue; }
        chg c = {e->addr, e->st, e->inc, e->d_src, e->d_srcinc};
        cv_push(out, c);
    }
}

static void issue_as_receiver(orc_sim *s, uint32_t v, node *nd, uint32_t sender, int64_t sender_inc,
                              uint32_t sender_ck, chgvec *out, wctx *c) {
    issue(s, nd, sender, sender_inc, out);
    if (out->n == 0 && checksum(s, nd, c) != sender_ck) { /* fullSync (61-76, 100-113) */
        add_u64(&s->stat_fullsyncs, 1);
        const uint32_t *perm = perm_full(s, v, nd, c);
        for (uint32_t k = 0; k < s->N; k++) {
            uint32_t a = perm[k];
            chg x = {a, st_of(nd, a), inc_of(s, nd, a), v, 0};
            cv_push(out, x);
        }
    }
}

/* Membership.update + the 'updated' listeners of lib/on_membership_event.js */
static uint32_t update(orc_sim *s, uint32_t v, const chg *ch, uint32_t n, wctx *c) {
    node *nd = &s->nodes[v];
    if (c->appcap < n) {
        c->appcap = n * 2;
        c->app = (chg *)realloc(c->app, sizeof(chg) * c->appcap);
    }
    uint32_t na = 0;
    int64_t now = s->now0 + 200 * s->round;
    for (uint32_t i = 0; i < n; i++) {
        chg u = ch[i];
        uint32_t a = u.addr;
        ent *e = find(nd, a);
        uint8_t cur = e ? e->st : 0;
        int64_t ci = e ? e->inc : s->inc0[a];
        int ok;
        if (a == v && (u.st == 1 || u.st == 2)) { /* local override (member.js:76-81) */
            u.st = 0;
            u.inc = now;
            ok = 1;
        } else {
            switch (u.st) { /* _isOtherOverride (member.js:171-202) */
            case 0: ok = u.inc > ci; break;
            case 1: ok = (cur == 1 && u.inc > ci) || (cur == 2 && u.inc > ci) || (cur == 0 && u.inc >= ci); break;
            case 2: ok = (cur == 1 && u.inc >= ci) || (cur == 2 && u.inc > ci) || (cur == 0 && u.inc >= ci); break;
            default: ok = cur != 3 && u.inc >= ci; break;
            }
        }
        if (!ok) continue;
        e = get(s, nd, a);
        e->st = u.st;
        e->inc = u.inc;
        c->app[na++] = u;
    }
    if (na) {
        nd->dirty = 1;
        int added = 0, removed = 0;
        /* the local member becoming `leave` emits LocalMemberLeaveEvent while the batch is evaluated
         * (member.js:87-95): gossip.stop() and suspicion.stopAll() (on_membership_event.js:32-40),
         * so no timer starts from this batch on and the running ones are cleared */
        for (uint32_t i = 0; i < na; i++)
            if (c->app[i].addr == v && c->app[i].st == 3 && !s->stopped[v]) {
                s->stopped[v] = 1;
                for (uint32_t q = 0; q < nd->ne; q++) { nd->e[q].t_on = 0; nd->e[q].deadline = -1; }
            }
        for (uint32_t i = 0; i < na; i++) {
            chg u = c->app[i];
            ent *e = find(nd, u.addr);
            /* createUpdatedHandlerForGossip (on_membership_event.js:86-104) */
            if (u.st == 1) {
                if (u.addr != v && !s->stopped[v]) { e->t_on = 1; e->deadline = s->round + s->susp_rounds; e->s_inc = u.inc; }
            } else {
                e->t_on = 0;
                e->deadline = -1;
            }
            e->d_on = 1;
            e->d_cnt = 0;
            e->d_src = u.src;
            e->d_srcinc = u.srcinc;
        }
        /* createUpdatedHandlerForRing (106-134): all adds, then all removes */
        for (uint32_t i = 0; i < na; i++) {
            ent *e = find(nd, c->app[i].addr);
            if (c->app[i].st == 0 && !e->in_ring) { e->in_ring = 1; nd->ring_count++; added = 1; }
        }
        for (uint32_t i = 0; i < na; i++) {
            ent *e = find(nd, c->app[i].addr);
            if ((c->app[i].st == 2 || c->app[i].st == 3) && e->in_ring) { e->in_ring = 0; nd->ring_count--; removed = 1; }
        }
        if (added || removed) /* ringChanged -> adjustMaxPiggybackCount (dissemination.js:38-55) */
            nd->max_piggy = 15u * (uint32_t)digits(nd->ring_count);
        add_u64(&s->stat_applied, na);
    }
    return na;
}

static void make_change(orc_sim *s, uint32_t v, uint32_t a, uint8_t st, int64_t inc, wctx *c) {
    node *nd = &s->nodes[v];
    chg x = {a, st, inc, v, inc_of(s, nd, v)}; /* new Update(..., localMember) (update.js:26-35) */
    update(s, v, &x, 1, c);
}

/* ---- creation */
static const orc_sim *g_sim;
static int qcmp_addr(const void *x, const void *y) {
    uint32_t a = *(const uint32_t *)x, b = *(const uint32_t *)y;
    uint64_t la = g_sim->noff[a + 1] - g_sim->noff[a], lb = g_sim->noff[b + 1] - g_sim->noff[b];
    int c = memcmp(g_sim->nb + g_sim->noff[a], g_sim->nb + g_sim->noff[b], la < lb ? la : lb);
    if (c) return c;
    return la < lb ? -1 : la > lb;
}

static void w_init(orc_sim *s, uint32_t v, wctx *c) {
    node *nd = &s->nodes[v];
    nd->max_piggy = 15u * (uint32_t)digits(s->N);
    nd->ring_count = s->N;
    nd->it_idx = -1;
    nd->checksum = s->base_ck;
    if (s->full_order) {
        nd->order = (uint32_t *)malloc(4ull * s->N);
        perm_initial(s->N, v, nd->order);
        if (!s->down[v]) node_shuffle(s, v, nd, c); /* gossip.start (gossip/index.js:97) */
    } else {
        nd->order = (uint32_t *)malloc(4ull * WIN);
        if (!s->down[v]) node_shuffle(s, v, nd, c);
        else set_window(s, nd, perm_full(s, v, nd, c), 0);
    }
}

static int env_threads(void) {
    const char *e = getenv("ORC_SIM_THREADS");
    if (e && *e) return atoi(e) > 0 ? atoi(e) : 1;
    return 1;
}

orc_sim *orc_sim_new(uint32_t N, uint32_t seed, uint32_t susp_rounds, int64_t now0, const char *names,
                     const uint32_t *off, const int64_t *inc0, const uint8_t *dead) {
    orc_sim *s = (orc_sim *)calloc(1, sizeof(orc_sim));
    s->N = N;
    s->seed = seed;
    s->susp_rounds = susp_rounds;
    s->now0 = now0;
    s->down = (uint8_t *)malloc(N);
    memcpy(s->down, dead, N);
    s->left = (uint8_t *)calloc(N, 1);
    s->stopped = (uint8_t *)calloc(N, 1);
    s->nb = (char *)malloc(off[N] + 1);
    memcpy(s->nb, names, off[N]);
    s->noff = (uint64_t *)malloc(sizeof(uint64_t) * (N + 1));
    for (uint32_t i = 0; i <= N; i++) s->noff[i] = off[i];
    s->inc0 = (int64_t *)malloc(8ull * N);
    memcpy(s->inc0, inc0, 8ull * N);
    s->sorted = (uint32_t *)malloc(sizeof(uint32_t) * N);
    s->rank = (uint32_t *)malloc(sizeof(uint32_t) * N);
    for (uint32_t i = 0; i < N; i++) s->sorted[i] = i;
    g_sim = s;
    qsort(s->sorted, N, sizeof(uint32_t), qcmp_addr);
    for (uint32_t k = 0; k < N; k++) s->rank[s->sorted[k]] = k;
    /* the all-alive base string */
    uint64_t cap = off[N] + 32ull * N + 64, o = 0;
    s->sbase = (char *)malloc(cap);
    s->boff = (uint64_t *)malloc(8ull * (N + 1));
    for (uint32_t k = 0; k < N; k++) {
        uint32_t a = s->sorted[k];
        s->boff[k] = o;
        memcpy(s->sbase + o, s->nb + s->noff[a], s->noff[a + 1] - s->noff[a]);
        o += s->noff[a + 1] - s->noff[a];
        memcpy(s->sbase + o, "alive", 5);
        o += 5;
        o += (uint64_t)dec(inc0[a], s->sbase + o);
        if (k + 1 < N) s->sbase[o++] = ';';
    }
    s->boff[N] = o;
    s->base_ck = orc_hash32((const uint8_t *)s->sbase, o);
    const char *ob = getenv("ORC_SIM_ORDER_BYTES");
    uint64_t obytes = ob && *ob ? strtoull(ob, NULL, 10) : (2ull << 30);
    s->full_order = (uint64_t)N * N * 4 <= obytes;
    s->threads = env_threads();
    s->ctx = (wctx *)calloc((size_t)s->threads, sizeof(wctx));
    for (int t = 0; t < s->threads; t++) {
        s->ctx[t].perm = (uint32_t *)malloc(4ull * N);
        s->ctx[t].vis = (uint32_t *)malloc(4ull * N);
        s->ctx[t].cand = (uint32_t *)malloc(4ull * N);
        s->ctx[t].bits = (uint64_t *)malloc(8ull * ((N + 63) / 64));
    }
    s->memo = (memo_slot *)calloc(1u << MEMO_BITS, sizeof(memo_slot));
    for (int i = 0; i < 64; i++) pthread_mutex_init(&s->memo_mu[i], NULL);
    s->nodes = (node *)calloc(N, sizeof(node));
    parallel_for(s, N, 16, w_init);
    s->target = (int64_t *)malloc(sizeof(int64_t) * N);
    s->ping = (chgvec *)calloc(N, sizeof(chgvec));
    s->resp = (chgvec *)calloc(N, sizeof(chgvec));
    s->ping_ck = (uint32_t *)malloc(sizeof(uint32_t) * N);
    s->ping_inc = (int64_t *)malloc(sizeof(int64_t) * N);
    s->csr_off = (uint32_t *)malloc(sizeof(uint32_t) * (N + 1));
    s->csr_idx = (uint32_t *)malloc(sizeof(uint32_t) * 3ull * N);
    s->helpers = (uint32_t(*)[3])malloc(sizeof(uint32_t[3]) * N);
    s->nh = (uint32_t *)calloc(N, sizeof(uint32_t));
    s->legs = (chgvec(*)[3])calloc(N, sizeof(chgvec[3]));
    s->lresp = (chgvec(*)[3])calloc(N, sizeof(chgvec[3]));
    s->lok = (uint8_t(*)[3])calloc(N, 3);
    s->leg_ck = (uint32_t *)malloc(sizeof(uint32_t) * N);
    s->leg_inc = (int64_t *)malloc(sizeof(int64_t) * N);
    return s;
}

void orc_sim_set_threads(orc_sim *s, int threads) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    for (int t = threads; t < s->threads; t++) {
        wctx *c = &s->ctx[t];
        free(c->perm); free(c->vis); free(c->cand); free(c->bits); free(c->buf); free(c->dk); free(c->app);
        free(c->scratch.v);
    }
    s->ctx = (wctx *)realloc(s->ctx, sizeof(wctx) * (size_t)threads);
    for (int t = s->threads; t < threads; t++) {
        memset(&s->ctx[t], 0, sizeof(wctx));
        s->ctx[t].perm = (uint32_t *)malloc(4ull * s->N);
        s->ctx[t].vis = (uint32_t *)malloc(4ull * s->N);
        s->ctx[t].cand = (uint32_t *)malloc(4ull * s->N);
        s->ctx[t].bits = (uint64_t *)malloc(8ull * ((s->N + 63) / 64));
    }
    s->threads = threads;
}

void orc_sim_free(orc_sim *s) {
    if (!s) return;
    for (uint32_t v = 0; v < s->N; v++) {
        node *nd = &s->nodes[v];
        free(nd->e); free(nd->ix); free(nd->order); free(nd->base);
        free(s->ping[v].v); free(s->resp[v].v);
        for (int k = 0; k < 3; k++) { free(s->legs[v][k].v); free(s->lresp[v][k].v); }
    }
    for (int t = 0; t < s->threads; t++) {
        wctx *c = &s->ctx[t];
        free(c->perm); free(c->vis); free(c->cand); free(c->bits); free(c->buf); free(c->dk); free(c->app);
        free(c->scratch.v);
    }
    for (int i = 0; i < 64; i++) pthread_mutex_destroy(&s->memo_mu[i]);
    free(s->ctx); free(s->memo);
    free(s->nodes); free(s->target); free(s->ping); free(s->resp); free(s->ping_ck); free(s->ping_inc);
    free(s->csr_off); free(s->csr_idx); free(s->helpers); free(s->nh); free(s->legs); free(s->lresp); free(s->lok);
    free(s->leg_ck); free(s->leg_inc);
    free(s->down); free(s->left); free(s->stopped); free(s->nb); free(s->noff); free(s->inc0); free(s->sorted); free(s->rank);
    free(s->sbase); free(s->boff);
    free(s);
}

/* A fresh process for node v bootstraps into the running cluster (index.js:240-322):
 * makeAlive(self, Date.now()); three live nodes other than v (a partial Fisher-Yates over them
 * in id order, JOIN stream) answer the join: each applies makeAlive(v, that incarnation)
 * (server/protocol/join.js:126) and returns its fullSync; mergeJoinResponses
 * (join-response-merge.js:40-56: the first response when every checksum agrees, else
 * mergeMembershipChangesets; the same rows either way) is stashed and set() (index.js:208-247)
 * builds the view: self first, then the others in the first response's members-array order,
 * each at the greatest incarnation any response holds (the first on ties). The set handler
 * (on_membership_event.js:42-67) adds alive / suspect members to the ring without a
 * ringChanged (maxPiggybackCount stays at the one-server value of makeAlive(self)) and starts a
 * suspicion timer per suspect member. The dissemination is cleared as at bootstrap; gossip.start
 * shuffles. */
static void node_join(orc_sim *s, uint32_t v, wctx *c) {
    const uint32_t N = s->N;
    const int64_t now = s->now0 + 200 * s->round;
    uint32_t len = 0;
    for (uint32_t u = 0; u < N; u++)
        if (u != v && !s->down[u]) c->cand[len++] = u;
    const uint32_t nj = len < 3 ? len : 3;
    uint32_t resp[3];
    for (uint32_t q = 0; q < nj; q++) {
        uint32_t r = philox_u32(s->seed, TAG_JOIN, (uint32_t)s->round, q, v);
        uint32_t j = q + (uint32_t)(((uint64_t)r * (len - q)) >> 32);
        uint32_t t = c->cand[q]; c->cand[q] = c->cand[j]; c->cand[j] = t;
        resp[q] = c->cand[q];
    }
    for (uint32_t q = 0; q < nj; q++) make_change(s, resp[q], v, 0, now, c);
    node *nd = &s->nodes[v];
    /* the members array: self, then the first response's order without self */
    uint32_t *base = nd->base ? nd->base : (uint32_t *)malloc(4ull * N);
    base[0] = v;
    if (nj) {
        const uint32_t *p0 = perm_full(s, resp[0], &s->nodes[resp[0]], c);
        for (uint32_t k = 0, o = 1; k < N; k++)
            if (p0[k] != v) base[o++] = p0[k];
    } else {
        for (uint32_t k = 0, o = 1; k < N; k++)
            if (k != v) base[o++] = k;
    }
    /* the rows: a fresh sparse view, then every member some response holds off its base state */
    nd->ne = 0;
    if (nd->ixcap) memset(nd->ix, 0, 4ull * nd->ixcap);
    uint32_t nrem = 0;
    for (uint32_t q = 0; q < nj; q++) {
        const node *rq = &s->nodes[resp[q]];
        for (uint32_t i = 0; i < rq->ne; i++) {
            const uint32_t a = rq->e[i].addr;
            if (a == v || find(nd, a)) continue;
            uint8_t st = 0;
            int64_t inc = s->inc0[a];
            for (uint32_t q2 = 0; q2 < nj; q2++) { /* greatest incarnation, the first on ties */
                const ent *x = find(&s->nodes[resp[q2]], a);
                const uint8_t st2 = x ? x->st : 0;
                const int64_t in2 = x ? x->inc : s->inc0[a];
                if (q2 == 0 || in2 > inc) { st = st2; inc = in2; }
            }
            ent *e = get(s, nd, a);
            e->st = st;
            e->inc = inc;
            e->in_ring = st == 0 || st == 1;
            if (!e->in_ring) nrem++;
            if (st == 1) { e->t_on = 1; e->deadline = s->round + s->susp_rounds; e->s_inc = inc; }
        }
    }
    ent *self = get(s, nd, v);
    self->st = 0;
    self->inc = now;
    self->in_ring = 1;
    nd->ring_count = N - nrem;
    nd->max_piggy = 15u * (uint32_t)digits(1);
    nd->it_idx = -1;
    nd->n_shuffles = 0;
    nd->dirty = 1;
    if (s->full_order) {
        memcpy(nd->order, base, 4ull * N);
        free(base);
        nd->base = NULL;
    } else {
        nd->base = base;
    }
    s->down[v] = 0;
    s->stopped[v] = 0;
    s->left[v] = 0;
    node_shuffle(s, v, nd, c); /* gossip.start */
}

/* Scenario events, applied before the next round (see the header). */
int orc_sim_event(orc_sim *s, int kind, uint32_t v) {
    if (v >= s->N) return -1;
    switch (kind) {
    case ORC_SIM_KILL: s->down[v] = 1; return 0;
    case ORC_SIM_REVIVE: s->down[v] = 0; return 0;
    case ORC_SIM_JOIN: node_join(s, v, &s->ctx[0]); return 0;
    case ORC_SIM_LEAVE: {
        node *nd = &s->nodes[v];
        /* the admin handler refuses a redundant leave (server/admin/member.js:84-89); a node that
         * is down cannot be asked */
        if (s->down[v] || st_of(nd, v) == 3) return 0;
        s->left[v] = 1;
        make_change(s, v, v, 3, inc_of(s, nd, v), &s->ctx[0]);
        return 0;
    }
    default: return -1;
    }
}

/* _.sample(pingable members excluding target, 3) as a partial Fisher-Yates (SAMP stream) */
static uint32_t sample_helpers(orc_sim *s, uint32_t v, uint32_t t, uint32_t *out, wctx *c) {
    node *nd = &s->nodes[v];
    const uint32_t *perm = perm_full(s, v, nd, c);
    uint32_t len = 0;
    for (uint32_t k = 0; k < s->N; k++) {
        uint32_t m = perm[k]; /* members array order (index.js:145-149) */
        if (m != t && pingable(nd, v, m)) c->cand[len++] = m;
    }
    uint32_t n = len < 3 ? len : 3;
    for (uint32_t i = 0; i < n; i++) {
        uint32_t r = philox_u32(s->seed, TAG_SAMP, (uint32_t)s->round, i, v);
        uint32_t j = i + (uint32_t)(((uint64_t)r * (len - i)) >> 32);
        uint32_t x = c->cand[i]; c->cand[i] = c->cand[j]; c->cand[j] = x;
        out[i] = c->cand[i];
    }
    return n;
}

/* ---- phases (one node per work item) */
static void w_a(orc_sim *s, uint32_t v, wctx *c) {
    s->target[v] = -1;
    if (s->down[v] || s->stopped[v]) return;
    node *nd = &s->nodes[v];
    int64_t t = iter_next(s, v, nd, c);
    s->target[v] = t;
    if (t < 0) return;
    issue(s, nd, NONE, 0, &s->ping[v]);
    s->ping_ck[v] = checksum(s, nd, c);
    s->ping_inc[v] = inc_of(s, nd, v);
    add_u64(&s->stat_pings, 1);
}

static void w_b(orc_sim *s, uint32_t j, wctx *c) { /* target j: its pings in sender order */
    for (uint32_t q = s->csr_off[j]; q < s->csr_off[j + 1]; q++) {
        uint32_t v = s->csr_idx[q];
        update(s, j, s->ping[v].v, s->ping[v].n, c);
        issue_as_receiver(s, j, &s->nodes[j], v, s->ping_inc[v], s->ping_ck[v], &s->resp[v], c);
    }
}

static void w_c(orc_sim *s, uint32_t v, wctx *c) {
    int64_t t = s->target[v];
    if (t < 0 || s->down[t]) return;
    update(s, v, s->resp[v].v, s->resp[v].n, c);
    update(s, v, s->resp[v].v, s->resp[v].n, c);
}

static void w_d1(orc_sim *s, uint32_t v, wctx *c) {
    s->nh[v] = 0;
    int64_t t = s->target[v];
    if (t < 0 || !s->down[t]) return;
    node *nd = &s->nodes[v];
    add_u64(&s->stat_pingreqs, 1);
    s->nh[v] = sample_helpers(s, v, (uint32_t)t, s->helpers[v], c);
    if (s->nh[v] == 0) { make_change(s, v, (uint32_t)t, 1, inc_of(s, nd, (uint32_t)t), c); return; }
    s->leg_ck[v] = checksum(s, nd, c);
    s->leg_inc[v] = inc_of(s, nd, v);
    for (uint32_t k = 0; k < s->nh[v]; k++) issue(s, nd, NONE, 0, &s->legs[v][k]);
}

static void w_d2(orc_sim *s, uint32_t h, wctx *c) { /* helper h: legs in (sender, leg) order */
    for (uint32_t q = s->csr_off[h]; q < s->csr_off[h + 1]; q++) {
        uint32_t v = s->csr_idx[q] / 3, k = s->csr_idx[q] % 3;
        update(s, h, s->legs[v][k].v, s->legs[v][k].n, c);
        issue(s, &s->nodes[h], NONE, 0, &c->scratch); /* the helper's own ping of t */
        issue_as_receiver(s, h, &s->nodes[h], v, s->leg_inc[v], s->leg_ck[v], &s->lresp[v][k], c);
        s->lok[v][k] = 1;
    }
}

static void w_d3(orc_sim *s, uint32_t v, wctx *c) {
    if (s->nh[v] == 0) return;
    int bad = 0;
    for (uint32_t k = 0; k < s->nh[v]; k++) {
        if (!s->lok[v][k]) continue;
        update(s, v, s->lresp[v][k].v, s->lresp[v][k].n, c);
        bad = 1;
    }
    if (bad) {
        uint32_t t = (uint32_t)s->target[v];
        make_change(s, v, t, 1, inc_of(s, &s->nodes[v], t), c);
    }
}

static void w_e(orc_sim *s, uint32_t v, wctx *c) {
    if (s->down[v]) return;
    node *nd = &s->nodes[v];
    uint32_t nd_ = 0;
    if (c->dkcap < nd->ne) {
        c->dkcap = nd->ne * 2;
        c->dk = (uint32_t *)realloc(c->dk, 4ull * c->dkcap);
    }
    for (uint32_t i = 0; i < nd->ne; i++)
        if (nd->e[i].t_on && nd->e[i].deadline <= s->round) c->dk[nd_++] = nd->e[i].addr;
    qsort(c->dk, nd_, 4, cmp_u32); /* member-id order */
    for (uint32_t q = 0; q < nd_; q++) {
        ent *e = find(nd, c->dk[q]);
        if (!e->t_on || e->deadline > s->round) continue;
        e->t_on = 0;
        e->deadline = -1;
        make_change(s, v, e->addr, 2, e->s_inc, c);
    }
}

static void w_ck(orc_sim *s, uint32_t v, wctx *c) {
    if (!s->down[v]) checksum(s, &s->nodes[v], c);
}

void orc_sim_step(orc_sim *s) {
    const uint32_t N = s->N;
    /* A: pings */
    parallel_for(s, N, 64, w_a);
    /* B: deliveries, per target in sender order */
    memset(s->csr_off, 0, 4ull * (N + 1));
    for (uint32_t v = 0; v < N; v++) {
        int64_t t = s->target[v];
        if (t >= 0 && !s->down[t]) s->csr_off[t + 1]++;
    }
    for (uint32_t j = 0; j < N; j++) s->csr_off[j + 1] += s->csr_off[j];
    {
        uint32_t *fill = s->nh; /* scratch: per-target cursor */
        memcpy(fill, s->csr_off, 4ull * N);
        for (uint32_t v = 0; v < N; v++) {
            int64_t t = s->target[v];
            if (t >= 0 && !s->down[t]) s->csr_idx[fill[t]++] = v;
        }
    }
    parallel_for(s, N, 16, w_b);
    /* C: responses, applied twice */
    parallel_for(s, N, 64, w_c);
    /* D: ping-req for dead targets */
    parallel_for(s, N, 64, w_d1);
    memset(s->lok, 0, 3ull * N);
    memset(s->csr_off, 0, 4ull * (N + 1));
    for (uint32_t v = 0; v < N; v++)
        for (uint32_t k = 0; k < s->nh[v]; k++)
            if (!s->down[s->helpers[v][k]]) s->csr_off[s->helpers[v][k] + 1]++;
    for (uint32_t j = 0; j < N; j++) s->csr_off[j + 1] += s->csr_off[j];
    {
        uint32_t *fill = (uint32_t *)malloc(4ull * N);
        memcpy(fill, s->csr_off, 4ull * N);
        for (uint32_t v = 0; v < N; v++)
            for (uint32_t k = 0; k < s->nh[v]; k++) {
                uint32_t h = s->helpers[v][k];
                if (!s->down[h]) s->csr_idx[fill[h]++] = 3 * v + k; /* network error otherwise */
            }
        free(fill);
    }
    parallel_for(s, N, 16, w_d2);
    parallel_for(s, N, 64, w_d3);
    /* E: suspicion timers */
    parallel_for(s, N, 64, w_e);
    /* every view's checksum as of the end of the round */
    parallel_for(s, N, 16, w_ck);
    s->round++;
}

int64_t orc_sim_round(const orc_sim *s) { return s->round; }

void orc_sim_checksums(orc_sim *s, uint32_t *out) {
    parallel_for(s, s->N, 16, w_ck);
    for (uint32_t v = 0; v < s->N; v++) out[v] = s->down[v] ? 0 : s->nodes[v].checksum;
}

void orc_sim_view(const orc_sim *s, uint32_t v, uint8_t *st, int64_t *inc) {
    const node *nd = &s->nodes[v];
    memset(st, 0, s->N);
    memcpy(inc, s->inc0, sizeof(int64_t) * s->N);
    for (uint32_t i = 0; i < nd->ne; i++) {
        st[nd->e[i].addr] = nd->e[i].st;
        inc[nd->e[i].addr] = nd->e[i].inc;
    }
}

/* scenario-runner.js:152-170 over the nodes that are up and have not left (its
 * hostToAliveWorker), plus: every member that left is `leave`, and every other member that is
 * down is `faulty`, in each of those views */
int orc_sim_converged(orc_sim *s) {
    parallel_for(s, s->N, 16, w_ck);
    uint32_t *want = (uint32_t *)malloc(4ull * s->N + 4), nw = 0;
    for (uint32_t a = 0; a < s->N; a++)
        if (s->left[a] || s->down[a]) want[nw++] = a;
    int64_t ck = -1;
    int ok = 1;
    for (uint32_t v = 0; v < s->N && ok; v++) {
        if (s->down[v] || s->left[v]) continue;
        const node *nd = &s->nodes[v];
        if (ck < 0) ck = nd->checksum;
        else if ((uint32_t)ck != nd->checksum) ok = 0;
        for (uint32_t q = 0; q < nw && ok; q++)
            if (st_of(nd, want[q]) != (s->left[want[q]] ? 3 : 2)) ok = 0;
    }
    free(want);
    return ok;
}

void orc_sim_stats(const orc_sim *s, uint64_t *out4) {
    out4[0] = s->stat_pings;
    out4[1] = s->stat_pingreqs;
    out4[2] = s->stat_fullsyncs;
    out4[3] = s->stat_applied;
}

void orc_sim_piggyback(const orc_sim *s, uint32_t *out) {
    for (uint32_t v = 0; v < s->N; v++) out[v] = s->nodes[v].max_piggy;
}
