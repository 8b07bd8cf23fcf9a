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
 * Round r (live nodes only act; killed nodes never answer):
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
 */
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

#define TAG_SHUF 0x53485546u
#define TAG_SAMP 0x53414d50u

typedef struct {
    uint32_t addr;
    uint8_t st;
    int64_t inc;
    uint32_t src;     /* NONE = 0xFFFFFFFF */
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

typedef struct {
    /* view */
    uint8_t *st;
    int64_t *inc;
    /* dissemination records, by member */
    uint8_t *d_on, *d_st;
    uint32_t *d_cnt, *d_src;
    int64_t *d_inc, *d_srcinc;
    uint32_t max_piggy;
    /* ring */
    uint8_t *in_ring;
    uint32_t ring_count;
    /* members array order + iterator */
    uint32_t *order;
    int64_t it_idx;
    uint32_t n_shuffles;
    /* suspicion */
    int64_t *deadline; /* -1 none */
    int64_t *s_inc;
    /* checksum */
    uint32_t checksum;
} node;

struct orc_sim {
    uint32_t N;
    uint32_t seed;
    uint32_t susp_rounds;
    int64_t now0;
    int64_t round;
    uint8_t *dead;
    char *nb;
    uint64_t *noff;
    uint32_t *sorted; /* ids in address order */
    char *buf;
    uint64_t buf_cap;
    node *nodes;
    /* per-round scratch */
    int64_t *target;
    chgvec *ping, *resp;
    uint32_t *ping_ck;
    int64_t *ping_inc;
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

static const orc_sim *g_sim;
static int qcmp_addr(const void *x, const void *y) {
    uint32_t a = *(const uint32_t *)x, b = *(const uint32_t *)y;
    uint64_t la = g_sim->noff[a + 1] - g_sim->noff[a], lb = g_sim->noff[b + 1] - g_sim->noff[b];
    int c = memcmp(g_sim->nb + g_sim->noff[a], g_sim->nb + g_sim->noff[b], la < lb ? la : lb);
    if (c) return c;
    return la < lb ? -1 : la > lb;
}

/* Membership.computeChecksum (lib/membership/index.js:48-75) */
static void compute_checksum(orc_sim *s, node *nd) {
    uint64_t o = 0;
    for (uint32_t k = 0; k < s->N; k++) {
        uint32_t id = s->sorted[k];
        uint64_t ln = s->noff[id + 1] - s->noff[id];
        if (o + ln + 40 > s->buf_cap) {
            s->buf_cap = (o + ln + 40) * 2;
            s->buf = (char *)realloc(s->buf, s->buf_cap);
        }
        if (k) s->buf[o++] = ';';
        memcpy(s->buf + o, s->nb + s->noff[id], ln);
        o += ln;
        memcpy(s->buf + o, ST[nd->st[id]], STL[nd->st[id]]);
        o += STL[nd->st[id]];
        char tmp[24];
        int64_t v = nd->inc[id];
        int n = 0, neg = v < 0;
        uint64_t u = neg ? (uint64_t)(-(v + 1)) + 1 : (uint64_t)v;
        do { tmp[n++] = (char)('0' + u % 10); u /= 10; } while (u);
        if (neg) s->buf[o++] = '-';
        while (n) s->buf[o++] = tmp[--n];
    }
    nd->checksum = orc_hash32((const uint8_t *)s->buf, o);
}

/* _.shuffle replaced by Fisher-Yates over a Philox stream (SHUF, shuffle#, i, view) */
static void shuffle(orc_sim *s, uint32_t v, node *nd) {
    uint32_t sh = nd->n_shuffles++;
    for (uint32_t i = s->N - 1; i >= 1; i--) {
        uint32_t r = philox_u32(s->seed, TAG_SHUF, sh, i, v);
        uint32_t j = (uint32_t)(((uint64_t)r * (i + 1)) >> 32);
        uint32_t t = nd->order[i]; nd->order[i] = nd->order[j]; nd->order[j] = t;
    }
}

static int pingable(const orc_sim *s, uint32_t v, const node *nd, uint32_t m) {
    (void)s;
    return m != v && (nd->st[m] == 0 || nd->st[m] == 1); /* isPingable (index.js:173-177) */
}

/* MembershipIterator.next (iterator.js:28-51); -1 = no pingable member. The loop runs until
 * every distinct address has been visited (a reshuffle mid-walk can revisit members). */
static int64_t iter_next(orc_sim *s, uint32_t v, node *nd) {
    uint8_t *seen = (uint8_t *)calloc(s->N, 1);
    uint32_t nseen = 0;
    int64_t found = -1;
    while (nseen < s->N) {
        nd->it_idx++;
        if (nd->it_idx >= (int64_t)s->N) {
            nd->it_idx = 0;
            shuffle(s, v, nd);
        }
        uint32_t m = nd->order[nd->it_idx];
        if (!seen[m]) { seen[m] = 1; nseen++; }
        if (pingable(s, v, nd, m)) { found = m; break; }
    }
    free(seen);
    return found;
}

/* Dissemination._issueAs (dissemination.js:133-176). filter: sender id or NONE. */
static void issue(orc_sim *s, node *nd, uint32_t sender, int64_t sender_inc, chgvec *out) {
    out->n = 0;
    for (uint32_t a = 0; a < s->N; a++) {
        if (!nd->d_on[a]) continue;
        if (sender != 0xFFFFFFFFu && sender_inc != 0 && nd->d_src[a] != 0xFFFFFFFFu && nd->d_srcinc[a] != 0 &&
            nd->d_src[a] == sender && nd->d_srcinc[a] == sender_inc)
            continue; /* filtered: no count bump (150-153) */
        nd->d_cnt[a] += 1;
        if (nd->d_cnt[a] > nd->max_piggy) { nd->d_on[a] = 0; continue; }
        chg c = {a, nd->d_st[a], nd->d_inc[a], nd->d_src[a], nd->d_srcinc[a]};
        cv_push(out, c);
    }
}

static void issue_as_receiver(orc_sim *s, uint32_t v, node *nd, uint32_t sender, int64_t sender_inc,
                              uint32_t sender_ck, chgvec *out) {
    issue(s, nd, sender, sender_inc, out);
    if (out->n == 0 && nd->checksum != sender_ck) { /* fullSync (61-76, 100-113) */
        s->stat_fullsyncs++;
        for (uint32_t k = 0; k < s->N; k++) {
            uint32_t a = nd->order[k];
            chg c = {a, nd->st[a], nd->inc[a], v, 0};
            cv_push(out, c);
        }
    }
}

/* Membership.update + the 'updated' listeners of lib/on_membership_event.js */
static uint32_t update(orc_sim *s, uint32_t v, const chg *ch, uint32_t n) {
    node *nd = &s->nodes[v];
    chg *applied = n ? (chg *)malloc(sizeof(chg) * n) : NULL;
    uint32_t na = 0;
    int64_t now = s->now0 + 200 * s->round;
    for (uint32_t i = 0; i < n; i++) {
        chg u = ch[i];
        uint32_t a = u.addr;
        uint8_t cur = nd->st[a];
        int64_t ci = nd->inc[a];
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
        nd->st[a] = u.st;
        nd->inc[a] = u.inc;
        applied[na++] = u;
    }
    if (na) {
        compute_checksum(s, nd);
        int added = 0, removed = 0;
        for (uint32_t i = 0; i < na; i++) {
            chg u = applied[i];
            uint32_t a = u.addr;
            /* createUpdatedHandlerForGossip (on_membership_event.js:86-104) */
            if (u.st == 1) {
                if (a != v) { nd->deadline[a] = s->round + s->susp_rounds; nd->s_inc[a] = u.inc; }
            } else {
                nd->deadline[a] = -1;
            }
            nd->d_on[a] = 1;
            nd->d_cnt[a] = 0;
            nd->d_st[a] = u.st;
            nd->d_inc[a] = u.inc;
            nd->d_src[a] = u.src;
            nd->d_srcinc[a] = u.srcinc;
        }
        /* createUpdatedHandlerForRing (106-134): all adds, then all removes */
        for (uint32_t i = 0; i < na; i++)
            if (applied[i].st == 0 && !nd->in_ring[applied[i].addr]) {
                nd->in_ring[applied[i].addr] = 1; nd->ring_count++; added = 1;
            }
        for (uint32_t i = 0; i < na; i++)
            if ((applied[i].st == 2 || applied[i].st == 3) && nd->in_ring[applied[i].addr]) {
                nd->in_ring[applied[i].addr] = 0; nd->ring_count--; removed = 1;
            }
        if (added || removed) /* ringChanged -> adjustMaxPiggybackCount (dissemination.js:38-55) */
            nd->max_piggy = 15u * (uint32_t)digits(nd->ring_count);
        s->stat_applied += na;
    }
    free(applied);
    return na;
}

static void make_change(orc_sim *s, uint32_t v, uint32_t a, uint8_t st, int64_t inc) {
    node *nd = &s->nodes[v];
    chg c = {a, st, inc, v, nd->inc[v]}; /* new Update(..., localMember) (update.js:26-35) */
    update(s, v, &c, 1);
}

orc_sim *orc_sim_new(uint32_t N, uint32_t seed, uint32_t susp_rounds, int64_t now0, const char *names,
                     const uint32_t *off, const int64_t *inc0, const uint8_t *dead) {
    orc_sim *s = (orc_sim *)calloc(1, sizeof(orc_sim));
    s->N = N;
    s->seed = seed;
    s->susp_rounds = susp_rounds;
    s->now0 = now0;
    s->dead = (uint8_t *)malloc(N);
    memcpy(s->dead, dead, N);
    s->nb = (char *)malloc(off[N] + 1);
    memcpy(s->nb, names, off[N]);
    s->noff = (uint64_t *)malloc(sizeof(uint64_t) * (N + 1));
    for (uint32_t i = 0; i <= N; i++) s->noff[i] = off[i];
    s->sorted = (uint32_t *)malloc(sizeof(uint32_t) * N);
    for (uint32_t i = 0; i < N; i++) s->sorted[i] = i;
    g_sim = s;
    qsort(s->sorted, N, sizeof(uint32_t), qcmp_addr);
    s->nodes = (node *)calloc(N, sizeof(node));
    s->target = (int64_t *)malloc(sizeof(int64_t) * N);
    s->ping = (chgvec *)calloc(N, sizeof(chgvec));
    s->resp = (chgvec *)calloc(N, sizeof(chgvec));
    s->ping_ck = (uint32_t *)malloc(sizeof(uint32_t) * N);
    s->ping_inc = (int64_t *)malloc(sizeof(int64_t) * N);
    uint32_t mp = 15u * (uint32_t)digits(N);
    for (uint32_t v = 0; v < N; v++) {
        node *nd = &s->nodes[v];
        nd->st = (uint8_t *)calloc(N, 1);
        nd->inc = (int64_t *)malloc(sizeof(int64_t) * N);
        memcpy(nd->inc, inc0, sizeof(int64_t) * N);
        nd->d_on = (uint8_t *)calloc(N, 1);
        nd->d_st = (uint8_t *)calloc(N, 1);
        nd->d_cnt = (uint32_t *)calloc(N, sizeof(uint32_t));
        nd->d_src = (uint32_t *)calloc(N, sizeof(uint32_t));
        nd->d_inc = (int64_t *)calloc(N, sizeof(int64_t));
        nd->d_srcinc = (int64_t *)calloc(N, sizeof(int64_t));
        nd->max_piggy = mp;
        nd->in_ring = (uint8_t *)malloc(N);
        memset(nd->in_ring, 1, N);
        nd->ring_count = N;
        /* members array after bootstrap: self (makeAlive) then set() in id order */
        nd->order = (uint32_t *)malloc(sizeof(uint32_t) * N);
        nd->order[0] = v;
        for (uint32_t i = 0, k = 1; i < N; i++) if (i != v) nd->order[k++] = i;
        nd->it_idx = -1;
        nd->deadline = (int64_t *)malloc(sizeof(int64_t) * N);
        for (uint32_t i = 0; i < N; i++) nd->deadline[i] = -1;
        nd->s_inc = (int64_t *)calloc(N, sizeof(int64_t));
        if (dead[v]) continue;
        shuffle(s, v, nd); /* gossip.start (gossip/index.js:97) */
    }
    /* every view starts identical */
    compute_checksum(s, &s->nodes[0]);
    for (uint32_t v = 1; v < N; v++) s->nodes[v].checksum = s->nodes[0].checksum;
    return s;
}

void orc_sim_free(orc_sim *s) {
    if (!s) return;
    for (uint32_t v = 0; v < s->N; v++) {
        node *nd = &s->nodes[v];
        free(nd->st); free(nd->inc); free(nd->d_on); free(nd->d_st); free(nd->d_cnt); free(nd->d_src);
        free(nd->d_inc); free(nd->d_srcinc); free(nd->in_ring); free(nd->order); free(nd->deadline); free(nd->s_inc);
        free(s->ping[v].v); free(s->resp[v].v);
    }
    free(s->nodes); free(s->target); free(s->ping); free(s->resp); free(s->ping_ck); free(s->ping_inc);
    free(s->dead); free(s->nb); free(s->noff); free(s->sorted); free(s->buf);
    free(s);
}

/* _.sample(pingable members excluding target, 3) as a partial Fisher-Yates (SAMP stream) */
static uint32_t sample_helpers(orc_sim *s, uint32_t v, uint32_t t, uint32_t *out) {
    node *nd = &s->nodes[v];
    uint32_t *c = (uint32_t *)malloc(sizeof(uint32_t) * s->N);
    uint32_t len = 0;
    for (uint32_t k = 0; k < s->N; k++) {
        uint32_t m = nd->order[k]; /* members array order (index.js:145-149) */
        if (m != t && pingable(s, v, nd, m)) c[len++] = m;
    }
    uint32_t n = len < 3 ? len : 3;
    for (uint32_t i = 0; i < n; i++) {
        uint32_t r = philox_u32(s->seed, TAG_SAMP, (uint32_t)s->round, i, v);
        uint32_t j = i + (uint32_t)(((uint64_t)r * (len - i)) >> 32);
        uint32_t x = c[i]; c[i] = c[j]; c[j] = x;
        out[i] = c[i];
    }
    free(c);
    return n;
}

void orc_sim_step(orc_sim *s) {
    const uint32_t N = s->N;
    /* A: pings */
    for (uint32_t v = 0; v < N; v++) {
        s->target[v] = -1;
        if (s->dead[v]) continue;
        node *nd = &s->nodes[v];
        int64_t t = iter_next(s, v, nd);
        s->target[v] = t;
        if (t < 0) continue;
        issue(s, nd, 0xFFFFFFFFu, 0, &s->ping[v]);
        s->ping_ck[v] = nd->checksum;
        s->ping_inc[v] = nd->inc[v];
        s->stat_pings++;
    }
    /* B: deliveries, per target in sender order (targets are independent) */
    for (uint32_t v = 0; v < N; v++) {
        int64_t t = s->target[v];
        if (t < 0 || s->dead[t]) continue;
        update(s, (uint32_t)t, s->ping[v].v, s->ping[v].n);
        issue_as_receiver(s, (uint32_t)t, &s->nodes[t], v, s->ping_inc[v], s->ping_ck[v], &s->resp[v]);
    }
    /* C: responses, applied twice */
    for (uint32_t v = 0; v < N; v++) {
        int64_t t = s->target[v];
        if (t < 0 || s->dead[t]) continue;
        update(s, v, s->resp[v].v, s->resp[v].n);
        update(s, v, s->resp[v].v, s->resp[v].n);
    }
    /* D: ping-req for dead targets */
    uint32_t (*helpers)[3] = (uint32_t(*)[3])malloc(sizeof(uint32_t[3]) * N);
    uint32_t *nh = (uint32_t *)calloc(N, sizeof(uint32_t));
    chgvec(*legs)[3] = (chgvec(*)[3])calloc(N, sizeof(chgvec[3]));
    chgvec(*lresp)[3] = (chgvec(*)[3])calloc(N, sizeof(chgvec[3]));
    uint8_t(*lok)[3] = (uint8_t(*)[3])calloc(N, 3);
    uint32_t *leg_ck = (uint32_t *)malloc(sizeof(uint32_t) * N);
    int64_t *leg_inc = (int64_t *)malloc(sizeof(int64_t) * N);
    chgvec scratch = {0, 0, 0};
    for (uint32_t v = 0; v < N; v++) { /* D1 */
        int64_t t = s->target[v];
        if (t < 0 || !s->dead[t]) continue;
        node *nd = &s->nodes[v];
        s->stat_pingreqs++;
        nh[v] = sample_helpers(s, v, (uint32_t)t, helpers[v]);
        if (nh[v] == 0) { make_change(s, v, (uint32_t)t, 1, nd->inc[t]); continue; }
        leg_ck[v] = nd->checksum;
        leg_inc[v] = nd->inc[v];
        for (uint32_t k = 0; k < nh[v]; k++) issue(s, nd, 0xFFFFFFFFu, 0, &legs[v][k]);
    }
    for (uint32_t v = 0; v < N; v++) { /* D2, in (sender, leg) order */
        for (uint32_t k = 0; k < nh[v]; k++) {
            uint32_t h = helpers[v][k];
            if (s->dead[h]) continue; /* network error */
            update(s, h, legs[v][k].v, legs[v][k].n);
            issue(s, &s->nodes[h], 0xFFFFFFFFu, 0, &scratch); /* the helper's own ping of t */
            issue_as_receiver(s, h, &s->nodes[h], v, leg_inc[v], leg_ck[v], &lresp[v][k]);
            lok[v][k] = 1;
        }
    }
    for (uint32_t v = 0; v < N; v++) { /* D3 */
        if (nh[v] == 0) continue;
        int bad = 0;
        for (uint32_t k = 0; k < nh[v]; k++) {
            if (!lok[v][k]) continue;
            update(s, v, lresp[v][k].v, lresp[v][k].n);
            bad = 1;
        }
        if (bad) {
            uint32_t t = (uint32_t)s->target[v];
            make_change(s, v, t, 1, s->nodes[v].inc[t]);
        }
    }
    for (uint32_t v = 0; v < N; v++)
        for (int k = 0; k < 3; k++) { free(legs[v][k].v); free(lresp[v][k].v); }
    free(legs); free(lresp); free(lok); free(helpers); free(nh); free(leg_ck); free(leg_inc); free(scratch.v);
    /* E: suspicion timers */
    for (uint32_t v = 0; v < N; v++) {
        if (s->dead[v]) continue;
        node *nd = &s->nodes[v];
        for (uint32_t a = 0; a < N; a++)
            if (nd->deadline[a] >= 0 && nd->deadline[a] <= s->round) {
                nd->deadline[a] = -1;
                make_change(s, v, a, 2, nd->s_inc[a]);
            }
    }
    s->round++;
}

int64_t orc_sim_round(const orc_sim *s) { return s->round; }

void orc_sim_checksums(const orc_sim *s, uint32_t *out) {
    for (uint32_t v = 0; v < s->N; v++) out[v] = s->dead[v] ? 0 : s->nodes[v].checksum;
}

void orc_sim_view(const orc_sim *s, uint32_t v, uint8_t *st, int64_t *inc) {
    memcpy(st, s->nodes[v].st, s->N);
    memcpy(inc, s->nodes[v].inc, sizeof(int64_t) * s->N);
}

/* scenario-runner.js:152-170 + every killed member faulty in every live view */
int orc_sim_converged(const orc_sim *s) {
    int64_t ck = -1;
    for (uint32_t v = 0; v < s->N; v++) {
        if (s->dead[v]) continue;
        if (ck < 0) ck = s->nodes[v].checksum;
        else if ((uint32_t)ck != s->nodes[v].checksum) return 0;
        for (uint32_t a = 0; a < s->N; a++)
            if (s->dead[a] && s->nodes[v].st[a] != 2) return 0;
    }
    return 1;
}

void orc_sim_stats(const orc_sim *s, uint64_t *out4) {
    out4[0] = s->stat_pings;
    out4[1] = s->stat_pingreqs;
    out4[2] = s->stat_fullsyncs;
    out4[3] = s->stat_applied;
}
