// rp_sim.hip — the gossip protocol of N full ringpop nodes as a batched round simulator,
// optionally sharded by node over several GPUs.
//
// Every node v keeps what a ringpop process keeps: its membership view (lib/membership), its
// dissemination buffer (lib/gossip/dissemination.js), its ring membership + server count (only
// for maxPiggybackCount; lib/ring), its members-array order + iterator
// (lib/membership/iterator.js) and its suspicion timers (lib/gossip/suspicion.js), wired as
// lib/on_membership_event.js. Rounds follow the model of oracle/orc_sim.c (phases A, B, C,
// D1-D3, E). Within a phase every node's work is independent of the others, so
// one workgroup owns one node at a time (persistent grid); inside a node the records of one
// message carry distinct addresses and are applied by all 256 lanes at once.
//
// Sharding (C5). A handle owns the nodes [v0, v0 + NL) of a partition `bounds` of [0, N) into
// G contiguous shards; its views still cover all N members. Everything that crosses nodes is a
// MESSAGE (header Msg + piggybacked records Rec): pings (A -> B), their responses (B -> C),
// ping-req legs (D1 -> D2) and their responses (D2 -> D3). A round is five stages separated by
// four exchanges; each stage ends by building an outbox grouped by destination shard (local
// senders in id order, so the concatenation of the shards' outboxes is in global sender order,
// which is the order the reference's receivers process them in), and the next stage imports
// the inbox (the sources' outboxes for this shard, concatenated in shard order). The host moves
// the bytes: an in-process swap for one shard (rp_sim_step), device copies between handles of
// one process (rp_sim_exchange_local), or RCCL all-to-all-v between processes (the Python
// ShardedGossipSim over torch.distributed).
//
// HBM layout (sized for 10^5 members on one MI355X):
//   dense rows [lv][a]  status u8 (bit 7: in this node's ring) | incarnation i64 | members-array
//                       order u32 | dissemination slot u32  (17 B per (node, member))
//   per node            deviation bitmap over address ranks (which rows ever changed), sparse
//                       change list (dissemination's `changes` map: address, piggyback count,
//                       source, source incarnation; the status/incarnation of a change always
//                       equal the view row's), sparse timer list (address, due round, captured
//                       incarnation); capacities checked, overflow is a loud error
//   messages            fixed per-sender slots (ping, ping-req legs), a per-round arena
//                       (responses, full syncs), out/in message buffers (headers + records)
// Checksums: the membership checksum string of a view is the all-alive base string (address
// order, built once) with the deviated rows' pieces substituted. Nodes whose views changed are
// re-checksummed in batch with ONE NODE PER LANE (64 independent farmhash chains per wave,
// reading the shared base string plus the node's few deviated rows), or, when a reader needs
// one node's checksum in the middle of a phase, by one workgroup (one chain lane fed by
// pre-mixing lanes).
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/ringpop_amd.h"
#include "rp_farmhash.h"
#include "rp_names.h"
#include "rp_philox.h"
#include "rp_prims.h"
#include "rp_swim.h"

namespace rp {

namespace {

constexpr int kT = 256;            // threads per node-workgroup
constexpr uint32_t NONE = 0xFFFFFFFFu;
constexpr uint32_t TAG_SHUF = 0x53485546u;
constexpr uint32_t TAG_SAMP = 0x53414d50u;
constexpr uint32_t TAG_JOIN = 0x4a4f494eu;
constexpr int kHashWin = 512;      // LDS window of pre-mixed chunks for the block checksum chain
constexpr uint8_t ST_MASK = 3, IN_RING = 0x80;
constexpr uint32_t kMaxShards = 64;
// error flags (rp_sim_step reports them)
constexpr uint32_t ERR_CHANGES = 1, ERR_TIMERS = 2, ERR_ARENA = 4, ERR_TWINFP = 8;

// One piggybacked change on the wire (dissemination.js:163-170): 24 bytes.
// w0 = address (bits 0-22) | status (bits 23-24) | aux (bits 25-31: a ping-req leg record's
// piggyback count after the first of the three issues).
struct Rec {
    uint32_t w0;
    uint32_t src;  // NONE = undefined
    int64_t inc;
    int64_t srcinc;  // 0 = undefined
};
__device__ __forceinline__ uint32_t rec_addr(const Rec& r) { return r.w0 & 0x7FFFFFu; }
__device__ __forceinline__ uint8_t rec_st(const Rec& r) { return (uint8_t)((r.w0 >> 23) & 3u); }
__device__ __forceinline__ uint32_t rec_aux(const Rec& r) { return r.w0 >> 25; }
__device__ __forceinline__ uint32_t rec_w0(uint32_t a, uint8_t st, uint32_t aux) {
    return a | ((uint32_t)st << 23) | (aux << 25);
}

// A message header (40 bytes): a ping (from sender to target, with the sender's checksum and
// incarnation: ping-sender.js:71-76), a ping-req leg (tag = leg index; ping-req-sender.js:75-81)
// or a response (to = the original sender). n = records (NONE = network error); roff = where its
// records are: in an outbox, the index of the first one in its destination's record area; once
// imported, the byte offset of the first one in the inbox buffer.
struct Msg {
    uint32_t from, to, n, tag;
    uint32_t ck, pad;
    int64_t inc;
    uint64_t roff;
};
static_assert(sizeof(Msg) == 40, "Msg layout is part of the exchange format");
static_assert(sizeof(Rec) == 24, "Rec layout is part of the exchange format");

// An entry of dissemination's changes map. It also carries the member's current status and
// incarnation: every row update goes through block_apply, which records the change in the same
// step (on_membership_event.js:86-134 -> recordChange), so an issue reads the records it sends
// sequentially from the list instead of at random from the view's rows.
struct Change {
    uint32_t addr;
    uint32_t cnt;  // piggybackCount
    uint32_t src;
    uint32_t st;   // the member's status (ST_MASK bits)
    int64_t srcinc;
    int64_t inc;   // the member's incarnation
};

struct P1 {  // a view's pass-1 results (lane_pass1 / seg_pass1)
    int64_t dtot, dlo, dhi;
    uint32_t last, nd;
};

struct Timer {  // a suspicion timer (suspicion.js:55-84)
    uint32_t addr;
    int32_t due;  // round at whose end it fires
    int64_t inc;  // incarnation captured at start (== the row's while the episode lasts)
};

enum MsgKind : int { K_PING = 0, K_RESP = 1, K_LEG = 2, K_LRESP = 3 };

struct SimDev {
    uint32_t N, W;   // members, bitmap words per node
    uint32_t v0, NL;  // this shard's nodes [v0, v0 + NL)
    uint32_t G;       // shards
    const uint32_t* bounds;  // [G + 1]
    uint32_t seed, susp, Cd, Ct, Cm;
    int64_t now0;
    int64_t round;
    // dense rows [lv][N]
    uint8_t* st;
    int64_t* inc;
    uint32_t* order;
    uint32_t* opos;  // inverse of order (each member's members-array position), or null
    uint32_t xcap;   // D1 non-candidate list capacity (<= kXCap; RP_SIM_D1_XCAP lowers it)
    uint32_t* slot;  // 0 = no change, else index + 1 into the node's change list
    uint32_t* dev;   // [lv][W] rows ever changed, by address rank
    // sparse per node
    Change* chg;  // [lv][Cd]
    uint32_t* n_chg;
    Timer* tim;  // [lv][Ct] appended in due order; [t_head, n_tim) are pending
    uint32_t* n_tim;
    uint32_t* t_head;  // first pending timer (the ones before it have fired or lapsed)
    uint64_t* vfp;     // [NL] twin fingerprint of each view, kept by block_apply (see twin_mix)
    int64_t* vdt;      // [NL] each view's checksum-string length minus the base's, kept by block_apply
                       // (the refresh's order, RP_SIM_CK_SORT; joined views are not updated)
    // per local node
    int64_t* it_idx;
    uint32_t *n_shuf, *ring_count, *max_piggy, *checksum;
    uint8_t* dirty;
    const uint8_t* dead;  // [N] (global): down this round (never started, crashed, suspended)
    uint8_t* stopped;     // [NL] own status became leave: gossip.stop() + suspicion.stopAll()
    // names in address order; base checksum string (global)
    const uint32_t* sorted;
    const uint32_t* rank;
    const uint8_t* names;
    const uint64_t* noff;
    const uint8_t* sbase;
    const uint64_t* boff;  // [N+1], boff[N] = base length
    const int64_t* inc0;
    // sender side (per local node)
    int32_t* target;
    uint32_t* ck_snap;
    int64_t* inc_snap;
    Rec* pool;  // [2][NL][Cm] fixed slots (ping, leg) + arena
    uint64_t arena0, arena_cap;
    unsigned long long* cursor;  // arena bump pointer (reset every round)
    uint32_t* work;              // [8] per-phase node counters (dynamic node order, reset every round)
    uint32_t *ping_n, *leg_n;
    uint32_t* helpers;  // [NL*3] (global ids)
    uint32_t* nhelp;    // [NL]
    uint32_t* leg_nk;   // [NL*3] records of leg k
    uint32_t* cand;     // [grid*N] scratch for ping-req candidate lists
    uint8_t* strbuf;    // [grid * strcap]
    uint64_t strcap;
    uint4* dlist;       // [NL][dcap] a lane checksum's deviated pieces, address order
    uint32_t dcap;
    P1* p1;              // [NL] pass-1 results k_pass1 left for the refresh kernel
    uint32_t p1_pre;     // 1: the lane kernels read p1 instead of running lane_pass1
    uint32_t ck_ablate;  // timing ablation of k_ck_lanes (RP_SIM_CK_ABLATE=1; results are wrong): no
                         // piece fixups
    // inbound messages of the current stage
    const Msg* in_msg;      // headers, gathered in arrival order
    const uint8_t* in_buf;  // the inbox: per source shard [headers | records]
    uint32_t nin;
    const uint32_t* ib_off;  // [NL+1] inbox CSR (pings / legs) by local receiver
    const uint32_t* ib_idx;  // message indices, (receiver, arrival) order
    // receiver side: the response to each inbound message (pool offset; n NONE = network error)
    uint32_t* rsp_n;
    uint64_t* rsp_off;
    // sender side: the inbound response message of each local sender / (sender, leg)
    uint32_t* resp_idx;   // [NL]
    uint32_t* lresp_idx;  // [NL*3]
    // stats: pings, pingreqs, fullsyncs, applied
    unsigned long long* stats;
    uint32_t* err;
};

__device__ __forceinline__ Rec* ping_slot(const SimDev& S, uint32_t lv) { return S.pool + (uint64_t)lv * S.Cm; }
__device__ __forceinline__ Rec* leg_slot(const SimDev& S, uint32_t lv) {
    return S.pool + ((uint64_t)S.NL + lv) * S.Cm;
}

__device__ __forceinline__ const Rec* msg_recs(const SimDev& S, const Msg& m) {
    return reinterpret_cast<const Rec*>(S.in_buf + m.roff);
}

__device__ __forceinline__ uint32_t shard_of(const SimDev& S, uint32_t v) {
    uint32_t s = 0;
    while (s + 1 < S.G && v >= S.bounds[s + 1]) s++;
    return s;
}

__device__ __forceinline__ uint32_t philox_u32(uint32_t seed, uint32_t tag, uint32_t c0, uint32_t c1, uint32_t c2) {
    return philox4x32_10(U4{c0, c1, c2, 0u}, seed, tag).x;
}

__device__ __forceinline__ uint32_t digits(uint32_t n) {
    uint32_t d = 0;
    while (n) {
        d++;
        n /= 10;
    }
    return d;
}

__device__ __forceinline__ void set_err(const SimDev& S, uint32_t e) { atomicOr(S.err, e); }

// ---- block primitives (256 threads)

__device__ uint32_t block_sum(uint32_t v, uint32_t* lds) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    __syncthreads();
    if (lane == 0) lds[w] = v;
    __syncthreads();
    const uint32_t t = lds[0] + lds[1] + lds[2] + lds[3];
    __syncthreads();
    return t;
}

// exclusive prefix of v over the block (thread order); *total = sum
__device__ uint32_t block_scan(uint32_t v, uint32_t* lds, uint32_t* total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    __syncthreads();
    if (lane == 63) lds[w] = x;
    __syncthreads();
    uint32_t base = 0, tot = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const uint32_t s = lds[q];
        if (q < w) base += s;
        tot += s;
    }
    __syncthreads();
    *total = tot;
    return base + x - v;
}

// thread 0 allocates n records from the round arena; broadcast to the block (~0 on overflow,
// with the error flag set)
__device__ uint64_t block_alloc(const SimDev& S, uint64_t n, uint64_t* lds64) {
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long o = atomicAdd(S.cursor, (unsigned long long)n);
        if (o + n > S.arena_cap) {
            set_err(S, ERR_ARENA);
            *lds64 = ~0ull;
        } else {
            *lds64 = S.arena0 + o;
        }
    }
    __syncthreads();
    const uint64_t r = *lds64;
    __syncthreads();
    return r;
}

__device__ __forceinline__ uint32_t premix(uint32_t x) { return fh::rotr(x * fh::kC1, 17) * fh::kC2; }

__device__ __forceinline__ uint32_t ld32(const uint8_t* p, uint64_t o) {
    return (uint32_t)p[o] | ((uint32_t)p[o + 1] << 8) | ((uint32_t)p[o + 2] << 16) | ((uint32_t)p[o + 3] << 24);
}

struct Lds {
    uint32_t u[16];
    uint64_t u64;
    unsigned long long fpd;  // block_apply: the batch's twin-fingerprint delta
    unsigned long long dtd;  // block_apply: the batch's string-length delta (vdt)
    uint32_t win[2][kHashWin][8] __attribute__((aligned(16)));
    uint32_t pad[8];  // the chain's one-chunk lookahead past win[1]
};

// ---- checksums

// One node's checksum string, seen by one lane: the base string with the deviated rows'
// pieces substituted. Piece k (address rank k) of the view is name + status + incarnation
// (+ ';' unless last); clean pieces equal the base string's. A deviated piece is described once
// (Piece), when the lane's cursor reaches it; in this model a deviated piece almost always keeps
// the base incarnation, so it differs from the base piece only in its status word.
struct Piece {
    uint32_t k;      // address rank (N: none)
    uint32_t nl;     // name bytes
    uint32_t sl;     // status bytes
    uint32_t blen;   // base piece bytes
    uint32_t plen;   // this view's piece bytes
    uint32_t dl;     // digit count
    uint64_t bpos;   // base offset of the piece
    uint64_t st64;   // status characters, little-endian
    int64_t x;       // incarnation
    bool basedig;    // the digits are the base piece's (incarnation == inc0)
};

// the status's checksum spelling as little-endian bytes ("alive" "suspect" "faulty" "leave")
__device__ __forceinline__ uint64_t status_u64(uint8_t s) {
    uint64_t v = 0x6576696c61ull;        // alive
    v = s == 1 ? 0x74636570737573ull : v;  // suspect
    v = s == 2 ? 0x79746c756166ull : v;    // faulty
    v = s == 3 ? 0x657661656cull : v;      // leave
    return v;
}
// status_len without branches: lengths 5 7 6 5 as nibbles
__device__ __forceinline__ uint32_t status_len_nb(uint32_t s) { return (0x5675u >> (4 * (s & 3))) & 15u; }

struct LaneView {
    const SimDev& S;
    const uint8_t* strow;
    const int64_t* incrow;
    const uint32_t* dev;

    __device__ Piece piece(uint32_t k) const {
        Piece P;
        P.k = k;
        if (k >= S.N) {
            P.nl = P.sl = P.blen = P.plen = P.dl = 0;
            P.bpos = S.boff[S.N];
            P.st64 = 0;
            P.x = 0;
            P.basedig = true;
            return P;
        }
        const uint32_t a = S.sorted[k];
        const uint8_t s = strow[a] & ST_MASK;
        P.nl = (uint32_t)(S.noff[a + 1] - S.noff[a]);
        P.sl = status_len(s);
        P.st64 = status_u64(s);
        P.bpos = S.boff[k];
        P.blen = (uint32_t)(S.boff[k + 1] - P.bpos);
        const uint32_t sep = k + 1 < S.N ? 1u : 0u;
        P.x = incrow[a];
        P.basedig = P.x == S.inc0[a];
        P.dl = P.basedig ? P.blen - P.nl - 5u - sep : dec_len(P.x);
        P.plen = P.nl + P.sl + P.dl + sep;
        return P;
    }
    // lane length - base length of deviated piece k (4 loads)
    __device__ int64_t piece_delta(uint32_t k) const {
        const uint32_t a = S.sorted[k];
        const int64_t x = incrow[a], x0 = S.inc0[a];
        int64_t d = (int64_t)status_len(strow[a] & ST_MASK) - 5;
        if (x != x0) d += (int64_t)dec_len(x) - (int64_t)dec_len(x0);
        return d;
    }
    __device__ uint8_t piece_byte(const Piece& P, uint32_t j) const {
        if (j < P.nl) return S.sbase[P.bpos + j];
        j -= P.nl;
        if (j < P.sl) return (uint8_t)(P.st64 >> (8 * j));
        j -= P.sl;
        if (P.basedig) return S.sbase[P.bpos + P.nl + 5u + j];  // digits (+ ';') of the base piece
        if (j >= P.dl) return (uint8_t)';';
        uint8_t tmp[24];
        dec_write(P.x, tmp, P.dl);
        return tmp[j];
    }
    // next deviated rank >= k (N if none)
    __device__ uint32_t next_dev(uint32_t k) const {
        if (k >= S.N) return S.N;
        uint32_t w = k >> 5;
        uint32_t bits = dev[w] & (0xFFFFFFFFu << (k & 31));
        while (!bits) {
            if (++w >= S.W) return S.N;
            bits = dev[w];
        }
        const uint32_t r = (w << 5) + __builtin_ctz(bits);
        return r < S.N ? r : S.N;
    }
    // previous deviated rank < k (NONE if none)
    __device__ uint32_t prev_dev(uint32_t k) const {
        if (k == 0) return NONE;
        const uint32_t q = k - 1;
        uint32_t w = q >> 5;
        uint32_t bits = dev[w] & (0xFFFFFFFFu >> (31 - (q & 31)));
        while (!bits) {
            if (w == 0) return NONE;
            bits = dev[--w];
        }
        return (w << 5) + 31 - __builtin_clz(bits);
    }
};

// Forward cursor over a lane's string (positions queried in non-decreasing order): the current
// (or next) deviated piece P at lane offset pos, the shift delta of the clean bytes before it,
// and the base offset of the deviated piece after it.
struct Fwd {
    Piece P;
    uint64_t pos;
    int64_t delta;
    uint64_t nb2;  // base offset of the next deviated piece after P (base length if none)

    __device__ void load(const LaneView& V, uint32_t k) {
        P = V.piece(k);
        pos = (uint64_t)((int64_t)P.bpos + delta);
        nb2 = V.S.boff[V.next_dev(k < V.S.N ? k + 1 : V.S.N)];
    }
    __device__ void init(const LaneView& V) {
        delta = 0;
        load(V, V.next_dev(0));
    }
    __device__ void skip_to(const LaneView& V, uint64_t q) {
        while (P.k < V.S.N && q >= pos + P.plen) {
            delta += (int64_t)P.plen - (int64_t)P.blen;
            load(V, V.next_dev(P.k + 1));
        }
    }
    __device__ uint8_t byte(const LaneView& V, uint64_t q) {
        skip_to(V, q);
        if (q < pos) return V.S.sbase[(uint64_t)((int64_t)q - delta)];
        return V.piece_byte(P, (uint32_t)(q - pos));
    }
};

__device__ __forceinline__ uint32_t ldw(const uint8_t* p) { return *reinterpret_cast<const uint32_t*>(p); }

// the 5 words of base bytes [o, o + 20)
__device__ __forceinline__ void base_words(const uint8_t* sbase, uint64_t o, uint32_t (&w)[5]) {
    const uint8_t* p = sbase + (o & ~3ull);
    const uint32_t sh = (uint32_t)(o & 3);
    const uint32_t w0 = ldw(p), w1 = ldw(p + 4), w2 = ldw(p + 8), w3 = ldw(p + 12), w4 = ldw(p + 16),
                   w5 = ldw(p + 20);
    w[0] = __builtin_amdgcn_alignbyte(w1, w0, sh);
    w[1] = __builtin_amdgcn_alignbyte(w2, w1, sh);
    w[2] = __builtin_amdgcn_alignbyte(w3, w2, sh);
    w[3] = __builtin_amdgcn_alignbyte(w4, w3, sh);
    w[4] = __builtin_amdgcn_alignbyte(w5, w4, sh);
}

// mask of the low bytes of a word whose lane offsets q (= base + b) are < lim
__device__ __forceinline__ uint32_t below_mask(int64_t lim, uint64_t base) {
    const int64_t m = lim - (int64_t)base;
    return m <= 0 ? 0u : m >= 4 ? 0xFFFFFFFFu : (1u << (8 * m)) - 1u;
}

// Membership checksum of local node lv computed by this lane alone.
__device__ uint32_t lane_checksum(const SimDev& S, uint32_t lv) {
    const uint32_t N = S.N;
    const uint64_t row = (uint64_t)lv * N;
    const LaneView V{S, S.st + row, S.inc + row, S.dev + (uint64_t)lv * S.W};
    // pass 1: length (base length + the deviated pieces' differences) and the last deviation
    int64_t dtot = 0;
    uint32_t last = NONE;
    for (uint32_t w = 0; w < S.W; w++) {
        uint32_t bits = V.dev[w];
        while (bits) {
            const uint32_t k = (w << 5) + __builtin_ctz(bits);
            bits &= bits - 1;
            dtot += V.piece_delta(k);
            last = k;
        }
    }
    const uint64_t len = (uint64_t)((int64_t)S.boff[N] + dtot);
    if (len <= 24) {
        uint8_t buf[24];
        Fwd F;
        F.init(V);
        for (uint32_t q = 0; q < (uint32_t)len; q++) buf[q] = F.byte(V, q);
        return fh::hash32(fh::PtrSrc{buf}, (uint32_t)len);
    }
    // the last 20 bytes, walking deviated pieces backwards from the end
    uint8_t tail[20];
    {
        uint32_t kd = last;
        int64_t da = dtot;  // delta of the clean bytes after piece kd
        Piece P{};
        uint64_t E = 0, B = 0;
        if (kd != NONE) {
            P = V.piece(kd);
            E = (uint64_t)((int64_t)S.boff[kd + 1] + da);
            B = E - P.plen;
        }
        for (int i = 19; i >= 0; i--) {
            const uint64_t q = len - 20 + (uint64_t)i;
            while (kd != NONE && q < B) {
                da -= (int64_t)P.plen - (int64_t)P.blen;
                kd = V.prev_dev(kd);
                if (kd != NONE) {
                    P = V.piece(kd);
                    E = (uint64_t)((int64_t)S.boff[kd + 1] + da);
                    B = E - P.plen;
                }
            }
            tail[i] = (kd != NONE && q >= B && q < E) ? V.piece_byte(P, (uint32_t)(q - B))
                                                       : S.sbase[(uint64_t)((int64_t)q - da)];
        }
    }
    auto tw = [&](int o) {
        return (uint32_t)tail[o] | ((uint32_t)tail[o + 1] << 8) | ((uint32_t)tail[o + 2] << 16) |
               ((uint32_t)tail[o + 3] << 24);
    };
    uint32_t h = (uint32_t)len, g = fh::kC1 * (uint32_t)len, f = g;
    h ^= premix(tw(16));
    h = fh::rotr(h, 19) * 5 + 0xe6546b64u;
    h ^= premix(tw(4));
    h = fh::rotr(h, 19) * 5 + 0xe6546b64u;
    g ^= premix(tw(12));
    g = fh::rotr(g, 19) * 5 + 0xe6546b64u;
    g ^= premix(tw(8));
    g = fh::rotr(g, 19) * 5 + 0xe6546b64u;
    f += premix(tw(0));
    f = fh::rotr(f, 19) + 113;
    const uint64_t iters = (len - 1) / 20;
    Fwd F;
    F.init(V);
    for (uint64_t c = 0; c < iters; c++) {
        const uint64_t q0 = c * 20;
        F.skip_to(V, q0);
        uint32_t wd[5];
        if (q0 + 20 <= F.pos) {  // clean: 20 base bytes at this lane's shift
            base_words(S.sbase, (uint64_t)((int64_t)q0 - F.delta), wd);
        } else if (F.P.basedig &&
                   q0 + 20 <= (uint64_t)((int64_t)F.nb2 + F.delta + (int64_t)F.P.plen - (int64_t)F.P.blen)) {
            // one deviated piece whose only difference is its status: base bytes at shift delta
            // before the status, the status characters, base bytes at shift delta + sl - 5 after
            const int64_t s0 = (int64_t)F.pos + F.P.nl, s1 = s0 + F.P.sl;
            uint32_t w1[5], w2[5];
            base_words(S.sbase, (uint64_t)((int64_t)q0 - F.delta), w1);
            base_words(S.sbase, (uint64_t)((int64_t)q0 - F.delta - (int64_t)F.P.sl + 5), w2);
#pragma unroll
            for (int i = 0; i < 5; i++) {
                const uint64_t qb = q0 + 4 * i;
                const uint32_t m1 = below_mask(s0, qb), m2 = below_mask(s1, qb);
                const int64_t so = (int64_t)qb - s0;  // status byte index of this word's byte 0
                const uint32_t sw = so >= 0 ? (so < 8 ? (uint32_t)(F.P.st64 >> (8 * so)) : 0u)
                                            : (so > -4 ? (uint32_t)(F.P.st64 << (8 * -so)) : 0u);
                wd[i] = (w1[i] & m1) | (sw & m2 & ~m1) | (w2[i] & ~m2);
            }
        } else {
            for (int i = 0; i < 5; i++) {
                uint32_t x = 0;
                for (int j = 0; j < 4; j++) x |= (uint32_t)F.byte(V, q0 + 4 * i + j) << (8 * j);
                wd[i] = x;
            }
        }
        const uint32_t a = wd[0], b = wd[1], cc = wd[2], d = wd[3], e = wd[4];
        h += a;
        g += b;
        f += cc;
        h = fh::rotr(h ^ premix(d), 19) * 5 + 0xe6546b64u + e;
        g = fh::rotr(g ^ premix(cc), 19) * 5 + 0xe6546b64u + a;
        f = fh::rotr(f ^ premix(b + e * fh::kC1), 19) * 5 + 0xe6546b64u + d;
        f += g;
        g += f;
    }
    g = fh::rotr(g, 11) * fh::kC1;
    g = fh::rotr(g, 17) * fh::kC1;
    f = fh::rotr(f, 11) * fh::kC1;
    f = fh::rotr(f, 17) * fh::kC1;
    h = fh::rotr(h + g, 19);
    h = h * 5 + 0xe6546b64u;
    h = fh::rotr(h, 17) * fh::kC1;
    h = fh::rotr(h + f, 19);
    h = h * 5 + 0xe6546b64u;
    h = fh::rotr(h, 17) * fh::kC1;
    return h;
}

// (a << SH) + b as one v_lshl_add_u32 (inline asm: the compiler would re-associate the chain's
// sums into a longer dependent sequence)
template <int SH>
__device__ __forceinline__ uint32_t lshl_add(uint32_t a, uint32_t b) {
    uint32_t r;
    asm("v_lshl_add_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "i"(SH), "v"(b));
    return r;
}
__device__ __forceinline__ uint32_t lshl_add_v(uint32_t a, uint32_t sh, uint32_t b) {  // (a << sh) + b
    uint32_t r;
    asm("v_lshl_add_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(sh), "v"(b));
    return r;
}
// a * c + b with a 32-bit v_mul_lo_u32 (hipcc fuses `a * c + b` into a 64-bit v_mad_u64_u32)
__device__ __forceinline__ uint32_t mul_lo_add(uint32_t a, uint32_t c, uint32_t b) {
    uint32_t r;
    asm("v_mul_lo_u32 %0, %1, %2" : "=v"(r) : "v"(a), "s"(c));
    return r + b;
}
__device__ __forceinline__ uint32_t swap_pair(uint32_t v) {  // lanes 2i <-> 2i+1 (quad_perm 1,0,3,2)
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, true);
}

// Membership.computeChecksum (index.js:48-75) of local node lv by one workgroup, without
// materialising the string: the view's deviated pieces are listed in address order with their
// lane offsets (a scan of the deviation bitmap + a prefix sum of the length differences), then
// 192 lanes produce the 20-byte chunks (base words at the right shift, or bytes of a deviated
// piece) and pre-mix them into double-buffered LDS windows while one lane runs the serial chain.
struct DevTab {  // per-block scratch in strbuf
    uint32_t* k;     // deviated ranks, address order
    int64_t* db;     // lane - base shift of the clean bytes before piece i
    uint64_t* pos;   // lane offset of piece i
    uint64_t* end;   // lane offset past piece i
    uint32_t n;
    int64_t dtot;    // shift after the last piece
};

// first piece i whose lane end is > q (n if none)
__device__ __forceinline__ uint32_t tab_find(const DevTab& T, uint64_t q) {
    uint32_t lo = 0, hi = T.n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (T.end[mid] <= q) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// byte cursor over the table (positions in non-decreasing order)
struct TabCursor {
    uint32_t i;
    uint32_t pk;  // rank whose Piece is cached (NONE: none)
    Piece P;
    __device__ uint8_t byte(const LaneView& V, const DevTab& T, uint64_t q) {
        while (i < T.n && q >= T.end[i]) i++;
        const int64_t db = i < T.n ? T.db[i] : T.dtot;
        if (i >= T.n || q < T.pos[i]) return V.S.sbase[(uint64_t)((int64_t)q - db)];
        if (pk != T.k[i]) {
            pk = T.k[i];
            P = V.piece(pk);
        }
        return V.piece_byte(P, (uint32_t)(q - T.pos[i]));
    }
};

__device__ void block_checksum(const SimDev& S, uint32_t lv, uint8_t* scratch, Lds& L) {
#ifdef RP_CK_PROF
    const uint64_t bt0 = clock64();
    uint64_t bt_chain = 0, bt_fill = 0;
#endif
    const uint32_t N = S.N;
    const uint64_t row = (uint64_t)lv * N;
    const LaneView V{S, S.st + row, S.inc + row, S.dev + (uint64_t)lv * S.W};
    const int tid = threadIdx.x;
    const uint64_t o1 = ((4ull * N) + 7) & ~7ull;
    DevTab T;
    T.k = reinterpret_cast<uint32_t*>(scratch);
    T.db = reinterpret_cast<int64_t*>(scratch + o1);
    T.pos = reinterpret_cast<uint64_t*>(scratch + o1 + 8ull * N);
    T.end = reinterpret_cast<uint64_t*>(scratch + o1 + 16ull * N);
    // deviated ranks in address order (contiguous bitmap words per thread)
    {
        const uint32_t per = (S.W + kT - 1) / kT;
        const uint32_t w0 = min(S.W, per * tid), w1 = min(S.W, w0 + per);
        uint32_t cnt = 0;
        for (uint32_t w = w0; w < w1; w++) cnt += __builtin_popcount(V.dev[w]);
        uint32_t nd;
        uint32_t o = block_scan(cnt, L.u, &nd);
        for (uint32_t w = w0; w < w1; w++) {
            uint32_t bits = V.dev[w];
            while (bits) {
                T.k[o++] = (w << 5) + __builtin_ctz(bits);
                bits &= bits - 1;
            }
        }
        T.n = nd;
    }
    __threadfence_block();
    __syncthreads();
    // shifts: prefix sums of the pieces' length differences (|sum| < 2^31)
    int32_t run = 0;
    for (uint32_t base = 0; base < T.n; base += kT) {
        const uint32_t i = base + tid;
        int32_t d = 0;
        uint32_t k = 0;
        if (i < T.n) {
            k = T.k[i];
            d = (int32_t)V.piece_delta(k);
        }
        uint32_t tot;
        const int32_t ex = (int32_t)block_scan((uint32_t)d, L.u, &tot);
        if (i < T.n) {
            const int64_t db = (int64_t)run + ex;
            T.db[i] = db;
            T.pos[i] = (uint64_t)((int64_t)S.boff[k] + db);
            T.end[i] = (uint64_t)((int64_t)S.boff[k + 1] + db + d);
        }
        run += (int32_t)tot;
    }
    T.dtot = run;
#ifdef RP_CK_PROF
    const uint64_t bt1 = clock64();
#endif
    __threadfence_block();
    __syncthreads();
    const uint64_t len = (uint64_t)((int64_t)S.boff[N] + run);
    uint32_t h = 0;
    if (len <= 24) {
        if (tid == 0) {
            uint8_t b[24];
            TabCursor C{0, NONE, Piece{}};
            for (uint32_t q = 0; q < (uint32_t)len; q++) b[q] = C.byte(V, T, q);
            h = fh::hash32(fh::PtrSrc{b}, (uint32_t)len);
        }
    } else {
        const uint64_t iters = (len - 1) / 20;
        uint32_t g = 0, f = 0;
        if (tid == 0) {
            uint8_t tb[20];
            TabCursor C{tab_find(T, len - 20), NONE, Piece{}};
            for (int i = 0; i < 20; i++) tb[i] = C.byte(V, T, len - 20 + i);
            auto tw = [&](int o) {
                return (uint32_t)tb[o] | ((uint32_t)tb[o + 1] << 8) | ((uint32_t)tb[o + 2] << 16) |
                       ((uint32_t)tb[o + 3] << 24);
            };
            const uint32_t L32 = (uint32_t)len;
            h = L32;
            g = fh::kC1 * L32;
            f = g;
            h ^= premix(tw(16));
            h = fh::rotr(h, 19) * 5 + 0xe6546b64u;
            h ^= premix(tw(4));
            h = fh::rotr(h, 19) * 5 + 0xe6546b64u;
            g ^= premix(tw(12));
            g = fh::rotr(g, 19) * 5 + 0xe6546b64u;
            g ^= premix(tw(8));
            g = fh::rotr(g, 19) * 5 + 0xe6546b64u;
            f += premix(tw(0));
            f = fh::rotr(f, 19) + 113;
        }
        // The chain in pre-added form (as rp_hashlong.hip): the state enters chunk j as
        // hp = h + a_j, gp = g + b_j, fp = f + c_j, and chunk j's record holds one {premix,
        // addend} pair per chain word: h {premix(d), K + e + a'}, g {premix(c), 3K + 2a + d + b'},
        // f {premix(b + e c1), 2K + a + d + c'}, with a', b', c' the next chunk's first words (0
        // after the last chunk).
        constexpr uint32_t kK = 0xe6546b64u;
        // the 20 bytes of chunk c as words (TabCursor C is advanced to c)
        auto chunk_words = [&](TabCursor& C, uint64_t c, uint32_t (&wd)[5]) {
            const uint64_t q0 = c * 20;
            while (C.i < T.n && q0 >= T.end[C.i]) C.i++;
            if (C.i >= T.n || q0 + 20 <= T.pos[C.i]) {
                const int64_t db = C.i < T.n ? T.db[C.i] : T.dtot;
                base_words(S.sbase, (uint64_t)((int64_t)q0 - db), wd);
            } else {
                TabCursor D = C;
                for (int i = 0; i < 5; i++) {
                    uint32_t x = 0;
                    for (int b = 0; b < 4; b++) x |= (uint32_t)D.byte(V, T, q0 + 4 * i + b) << (8 * b);
                    wd[i] = x;
                }
                C.pk = D.pk;
                C.P = D.P;
            }
        };
        // lanes [t0, t0 + nt) produce window wb = chunks [c0, c0 + kHashWin), a contiguous run each
        auto fill = [&](int wb, uint64_t c0, int idx, int nt) {
            const uint64_t n = (iters - c0) < (uint64_t)kHashWin ? (iters - c0) : kHashWin;
            const uint64_t per = (n + nt - 1) / nt;
            const uint64_t ja = (uint64_t)idx * per, jb = ja + per < n ? ja + per : n;
            if (ja >= jb) return;
            TabCursor C{tab_find(T, (c0 + ja) * 20), NONE, Piece{}};
            uint32_t wd[5];
            chunk_words(C, c0 + ja, wd);
            for (uint64_t j = ja; j < jb; j++) {
                uint32_t nx[5] = {0, 0, 0, 0, 0};
                if (c0 + j + 1 < iters) chunk_words(C, c0 + j + 1, nx);
                uint32_t* r = L.win[wb][j];
                *reinterpret_cast<uint2*>(r) = uint2{premix(wd[3]), kK + wd[4] + nx[0]};
                *reinterpret_cast<uint2*>(r + 2) = uint2{premix(wd[2]), 3u * kK + 2u * wd[0] + wd[3] + nx[1]};
                *reinterpret_cast<uint2*>(r + 4) =
                    uint2{premix(wd[1] + wd[4] * fh::kC1), 2u * kK + wd[0] + wd[3] + nx[2]};
#pragma unroll
                for (int i = 0; i < 5; i++) wd[i] = nx[i];
            }
        };
        // chunk 0's addends, then the h chain moves to lane 64 (it never mixes with g and f
        // before the finalisation; one wave issues ~1 VALU op per 4 cycles, so splitting the
        // chain over two waves shortens it)
        if (tid == 0) {
            TabCursor C0{0, NONE, Piece{}};
            uint32_t w0[5];
            chunk_words(C0, 0, w0);
            L.u[0] = g + w0[1];
            L.u[1] = f + w0[2];
            L.u[2] = h + w0[0];
        }
        fill(0, 0, tid, kT);
        __syncthreads();
        // the coupled (g, f) pair on lanes 0 and 1 of wave 0 (one instruction advances both, as
        // rp_hashlong.hip), h on lane 64
        const int ln = tid < 2 ? tid : 2;
        uint32_t cv = (tid < 2 || tid == 64) ? L.u[ln] : 0u;
        const uint32_t sh = tid == 0 ? 1u : 0u, sh2 = sh + 2u;
        __syncthreads();
        const uint64_t nwin = (iters + kHashWin - 1) / kHashWin;
        for (uint64_t w = 0; w < nwin; w++) {
            const int cur = (int)(w & 1);
            if (tid >= 128) {
#ifdef RP_CK_PROF
                const uint64_t tf0 = clock64();
#endif
                if (w + 1 < nwin) fill(cur ^ 1, (w + 1) * kHashWin, tid - 128, kT - 128);
#ifdef RP_CK_PROF
                bt_fill += clock64() - tf0;
#endif
            } else if (tid < 2 || tid == 64) {
#ifdef RP_CK_PROF
                const uint64_t tc0 = clock64();
#endif
                const uint64_t c0 = w * kHashWin;
                const int n = (int)((iters - c0) < (uint64_t)kHashWin ? (iters - c0) : kHashWin);
                // lane 0 (g) reads record words 2-3, lane 1 (f) words 4-5, lane 64 (h) words 0-1;
                // the pair: v' = 5 r_other + (5 (r_self << sh) + addend); h: 5 r + addend. LDS
                // reads 8 chunks ahead of their steps.
                if (tid < 2) {
                    const int wo = 2 + 2 * tid;
                    auto step = [&](const uint2 x) {
                        const uint32_t y = cv ^ x.x;
                        const uint32_t r = __builtin_amdgcn_alignbit(y, y, 19);
                        const uint32_t r5 = lshl_add<2>(r, r);
                        const uint32_t own = lshl_add_v(r, sh2, lshl_add_v(r, sh, x.y));
                        cv = swap_pair(r5) + own;
                    };
                    int j = 0;
                    for (; j + 8 <= n; j += 8) {
                        uint2 x[8];
#pragma unroll
                        for (int q = 0; q < 8; q++) x[q] = *reinterpret_cast<const uint2*>(L.win[cur][j + q] + wo);
#pragma unroll
                        for (int q = 0; q < 8; q++) step(x[q]);
                    }
                    for (; j < n; j++) step(*reinterpret_cast<const uint2*>(L.win[cur][j] + wo));
                } else {
                    auto step = [&](const uint2 x) {
                        const uint32_t y = cv ^ x.x;
                        const uint32_t r = __builtin_amdgcn_alignbit(y, y, 19);
                        cv = lshl_add<2>(r, r + x.y);
                    };
                    int j = 0;
                    for (; j + 8 <= n; j += 8) {
                        uint2 x[8];
#pragma unroll
                        for (int q = 0; q < 8; q++) x[q] = *reinterpret_cast<const uint2*>(L.win[cur][j + q]);
#pragma unroll
                        for (int q = 0; q < 8; q++) step(x[q]);
                    }
                    for (; j < n; j++) step(*reinterpret_cast<const uint2*>(L.win[cur][j]));
                }
#ifdef RP_CK_PROF
                if (tid == 0) bt_chain += clock64() - tc0;
#endif
            }
            __syncthreads();
        }
        if (tid < 2 || tid == 64) L.u[ln] = cv;
        __syncthreads();
        if (tid == 0) {
            g = L.u[0];  // the last chunk's next-words were 0: plain h, g, f
            f = L.u[1];
            h = L.u[2];
            g = fh::rotr(g, 11) * fh::kC1;
            g = fh::rotr(g, 17) * fh::kC1;
            f = fh::rotr(f, 11) * fh::kC1;
            f = fh::rotr(f, 17) * fh::kC1;
            h = fh::rotr(h + g, 19);
            h = h * 5 + 0xe6546b64u;
            h = fh::rotr(h, 17) * fh::kC1;
            h = fh::rotr(h + f, 19);
            h = h * 5 + 0xe6546b64u;
            h = fh::rotr(h, 17) * fh::kC1;
        }
    }
    if (tid == 0) {
        S.checksum[lv] = h;
        S.dirty[lv] = 0;
    }
#ifdef RP_CK_PROF
    if ((tid == 0 || tid == 64) && blockIdx.x == 0)
        printf("bckprof tid %d lv %u: table %llu total %llu chain %llu fill %llu cycles\n", tid, lv,
               (unsigned long long)(bt1 - bt0), (unsigned long long)(clock64() - bt0), (unsigned long long)bt_chain,
               (unsigned long long)bt_fill);
#endif
    __syncthreads();
}

__device__ __forceinline__ void checksum_if_dirty(const SimDev& S, uint32_t lv, Lds& L) {
    __syncthreads();
    if (S.dirty[lv]) {
        if (threadIdx.x == 0) atomicAdd(&S.stats[4], 1ull);  // views hashed
        block_checksum(S, lv, S.strbuf + (uint64_t)blockIdx.x * S.strcap, L);
    }
}

// Base-string ring of one wave in LDS. The wave's lanes hash different views in lockstep (chunk
// c of every lane's string at the same time); their base offsets differ only by each lane's
// running shift, within [q0 - DHI, q0 + 112 - DLO]. The ring keeps base bytes [hi - kRing, hi)
// (its first 24 words mirrored past its end, so a group's 21 words never wrap) and one more 1-KB
// slice in flight in registers (16 B per lane): every chunk's words come from LDS instead of an
// L2 round trip.
constexpr uint32_t kRing = 16384, kSlice = 1024, kRingW = kRing / 4;
typedef uint32_t u32x4s __attribute__((ext_vector_type(4)));

struct BaseRing {
    uint32_t* ring;  // kRingW + 24 words
    uint32_t hi;
    u32x4s pend;
    __device__ void start(const uint8_t* sbase, int lane) {
        hi = 0;
        pend = *reinterpret_cast<const u32x4s*>(sbase + lane * 16);
    }
    // wave-uniform: make base bytes [.., need) resident
    __device__ void ensure(const uint8_t* sbase, uint32_t need, int lane) {
        while (hi < need) {
            const uint32_t w = ((hi >> 2) + lane * 4) & (kRingW - 1);
            *reinterpret_cast<u32x4s*>(&ring[w]) = pend;
            if (w < 24) *reinterpret_cast<u32x4s*>(&ring[kRingW + w]) = pend;
            hi += kSlice;
            pend = *reinterpret_cast<const u32x4s*>(sbase + hi + lane * 16);
        }
    }
    __device__ __forceinline__ void words(uint32_t o, uint32_t (&w)[5]) const {
        const uint32_t* p = ring + ((o >> 2) & (kRingW - 1));
        const uint32_t sh = o & 3;
        const uint32_t x0 = p[0], x1 = p[1], x2 = p[2], x3 = p[3], x4 = p[4], x5 = p[5];
        w[0] = __builtin_amdgcn_alignbyte(x1, x0, sh);
        w[1] = __builtin_amdgcn_alignbyte(x2, x1, sh);
        w[2] = __builtin_amdgcn_alignbyte(x3, x2, sh);
        w[3] = __builtin_amdgcn_alignbyte(x4, x3, sh);
        w[4] = __builtin_amdgcn_alignbyte(x5, x4, sh);
    }
};

__device__ __forceinline__ int64_t wave_min64(int64_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const int64_t u = __shfl_xor(v, o, 64);
        v = u < v ? u : v;
    }
    return v;
}
__device__ __forceinline__ int64_t wave_max64(int64_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const int64_t u = __shfl_xor(v, o, 64);
        v = u > v ? u : v;
    }
    return v;
}

// A lane's cursor over its listed deviated pieces (uint4 {base offset, member, blen | nl << 8 |
// status << 16 | basedig << 18, rank}), in 32-bit lane coordinates: the current piece spans
// [pos, pend) at shift delta before it; nxt (the next entry) is loaded one piece ahead, so a
// piece boundary costs no dependent memory round trip.
struct LaneCursor {
    const uint4* dl;
    uint32_t i, n;
    uint4 cur, nxt, nn;  // nn: prefetched one piece ahead, first used by the advance after next
    uint32_t pos, pend, nl, sl, blen, nstart;  // nstart: lane offset of the next piece
    int32_t delta;
    uint64_t st64;
    bool basedig;

    __device__ uint4 entry(const SimDev& S, uint32_t j) const {
        return j < n ? dl[j] : uint4{(uint32_t)S.boff[S.N], 0u, 0u, S.N};
    }
    // everything from the list record (pass 1 packed the view's piece length in): no loads
    __device__ void set(const SimDev& S) {
        if (cur.w >= S.N) {  // past the last deviated piece
            pos = pend = nstart = 0xFFFFFFF0u;
            nl = sl = blen = 0;
            st64 = 0;
            basedig = true;
            return;
        }
        blen = cur.z & 0xFFu;
        nl = (cur.z >> 8) & 0xFFu;
        const uint8_t s = (uint8_t)((cur.z >> 16) & 3u);
        sl = status_len_nb(s);
        st64 = status_u64(s);
        basedig = (cur.z >> 18) & 1u;
        const uint32_t plen = (cur.z >> 19) & 0xFFu;
        pos = (uint32_t)((int32_t)cur.x + delta);
        pend = pos + plen;
        nstart = nxt.w >= S.N ? 0xFFFFFFF0u : (uint32_t)((int32_t)nxt.x + delta + (int32_t)plen - (int32_t)blen);
    }
    __device__ void init(const SimDev& S, const LaneView&, const uint4* list, uint32_t cnt) {
        dl = list;
        n = cnt;
        i = 0;
        delta = 0;
        cur = entry(S, 0);
        nxt = entry(S, 1);
        nn = entry(S, 2);
        set(S);
    }
    __device__ void advance(const SimDev& S, const LaneView&) {
        delta += (int32_t)(pend - pos) - (int32_t)blen;
        cur = nxt;
        nxt = nn;
        i++;
        nn = entry(S, i + 2);
        set(S);
    }
    __device__ Piece piece(const SimDev& S, const LaneView& V) const { return V.piece(cur.w); }
};

// byte q of a lane's string by a cursor copy that may walk past several pieces (rare path)
__device__ uint8_t lane_byte(const SimDev& S, const LaneView& V, LaneCursor& C, uint32_t q) {
    while (q >= C.pend && C.cur.w < S.N) C.advance(S, V);
    if (q < C.pos || C.cur.w >= S.N) return S.sbase[(uint32_t)((int32_t)q - C.delta)];
    return V.piece_byte(V.piece(C.cur.w), q - C.pos);
}

// Pass 1 of a lane checksum: list the view's deviated pieces (address order; the uint4 records
// of LaneCursor) and return the string's shift range, total, last deviated rank and count.
__device__ void lane_pass1(const SimDev& S, const LaneView& V, uint4* dl, int64_t& dtot, int64_t& dlo,
                           int64_t& dhi, uint32_t& last, uint32_t& nd) {
    dtot = dlo = dhi = 0;
    last = NONE;
    nd = 0;
    for (uint32_t w = 0; w < S.W; w++) {
        uint32_t bits = V.dev[w];
        while (bits) {
            const uint32_t k = (w << 5) + __builtin_ctz(bits);
            bits &= bits - 1;
            const uint32_t a = S.sorted[k];
            const uint8_t st = V.strow[a] & ST_MASK;
            const int64_t x = V.incrow[a], x0 = S.inc0[a];
            int64_t d = (int64_t)status_len(st) - 5;
            if (x != x0) d += (int64_t)dec_len(x) - (int64_t)dec_len(x0);
            if (nd < S.dcap) {
                const uint32_t bpos = (uint32_t)S.boff[k];
                const uint32_t blen = (uint32_t)(S.boff[k + 1] - bpos);
                const uint32_t nl = (uint32_t)(S.noff[a + 1] - S.noff[a]);
                const uint32_t plen = (uint32_t)((int64_t)blen + d);
                if (plen > 0xFFu) nd = S.dcap;  // a piece too long for the record: this lane falls back
                dl[nd < S.dcap ? nd : 0] =
                    uint4{bpos, a, blen | (nl << 8) | ((uint32_t)st << 16) | ((x == x0 ? 1u : 0u) << 18) | (plen << 19), k};
            }
            nd++;
            dtot += d;
            dlo = dtot < dlo ? dtot : dlo;
            dhi = dtot > dhi ? dtot : dhi;
            last = k;
        }
    }
}

// lane_pass1 by a segment of SEG lanes of one wave (lane sl of the segment; act and the view are
// segment-uniform, every lane of the segment calls it). Each lane takes a contiguous run of
// bitmap words; the record offsets and the running shift come from segment scans, so the list is
// the one lane_pass1 writes (a piece too long for its record makes nd exceed dcap the same way).
// One lane walking ~1,000 deviated members through their dependent loads took milliseconds (the
// D1 senders at C5); SEG lanes take 1/SEG of it.
template <int SEG>
__device__ void seg_pass1(const SimDev& S, const LaneView& V, uint4* dl, bool act, uint32_t sl, int64_t& dtot,
                          int64_t& dlo, int64_t& dhi, uint32_t& last, uint32_t& nd) {
    const uint32_t per = (S.W + SEG - 1) / SEG;
    const uint32_t w0 = min(S.W, sl * per), w1 = min(S.W, w0 + per);
    uint32_t cnt = 0;
    if (act)
        for (uint32_t w = w0; w < w1; w++) cnt += __builtin_popcount(V.dev[w]);
    // exclusive scan of the counts over the segment
    uint32_t inc = cnt;
#pragma unroll
    for (int o = 1; o < SEG; o <<= 1) {
        const uint32_t t = __shfl_up(inc, o, SEG);
        if (sl >= (uint32_t)o) inc += t;
    }
    const uint32_t total = __shfl(inc, SEG - 1, SEG);
    uint32_t idx = inc - cnt;
    int64_t run = 0, lmin = 0, lmax = 0;
    uint32_t llast = NONE;
    bool big = false;
    if (act) {
        for (uint32_t w = w0; w < w1; w++) {
            uint32_t bits = V.dev[w];
            while (bits) {
                const uint32_t k = (w << 5) + __builtin_ctz(bits);
                bits &= bits - 1;
                const uint32_t a = S.sorted[k];
                const uint8_t st = V.strow[a] & ST_MASK;
                const int64_t x = V.incrow[a], x0 = S.inc0[a];
                int64_t d = (int64_t)status_len(st) - 5;
                if (x != x0) d += (int64_t)dec_len(x) - (int64_t)dec_len(x0);
                if (idx < S.dcap) {
                    const uint32_t bpos = (uint32_t)S.boff[k];
                    const uint32_t blen = (uint32_t)(S.boff[k + 1] - bpos);
                    const uint32_t nl = (uint32_t)(S.noff[a + 1] - S.noff[a]);
                    const uint32_t plen = (uint32_t)((int64_t)blen + d);
                    if (plen > 0xFFu) big = true;
                    dl[idx] = uint4{bpos, a, blen | (nl << 8) | ((uint32_t)st << 16) | ((x == x0 ? 1u : 0u) << 18) |
                                                 (plen << 19),
                                    k};
                }
                idx++;
                run += d;
                lmin = run < lmin ? run : lmin;
                lmax = run > lmax ? run : lmax;
                llast = k;
            }
        }
    }
    // the running shift: exclusive scan of the lanes' sums, then min / max over the segment
    int64_t rin = run;
#pragma unroll
    for (int o = 1; o < SEG; o <<= 1) {
        const int64_t t = __shfl_up(rin, o, SEG);
        if (sl >= (uint32_t)o) rin += t;
    }
    const int64_t ex = rin - run;
    int64_t mn = ex + lmin, mx = ex + lmax;
    uint32_t lst = llast == NONE ? 0u : llast + 1u;
    uint32_t bg = big ? 1u : 0u;
#pragma unroll
    for (int o = SEG / 2; o > 0; o >>= 1) {
        const int64_t a = __shfl_xor(mn, o, SEG), b = __shfl_xor(mx, o, SEG);
        mn = a < mn ? a : mn;
        mx = b > mx ? b : mx;
        const uint32_t c = __shfl_xor(lst, o, SEG);
        lst = c > lst ? c : lst;
        bg |= __shfl_xor(bg, o, SEG);
    }
    dtot = __shfl(rin, SEG - 1, SEG);
    dlo = mn < 0 ? mn : 0;
    dhi = mx > 0 ? mx : 0;
    last = lst ? lst - 1u : NONE;
    nd = bg && total <= S.dcap ? S.dcap + 1u : total;  // an oversize piece: the lane path's fallback
}

// Pass 1 of the refresh's views ahead of the lane kernels, one wave per view (seg_pass1<64>):
// a lane walking its own view's bitmap (3,125 words at C5) and ~1,000 deviated members through
// dependent loads spent milliseconds before its chain started; 64 lanes take 1/64 of that.
__global__ __launch_bounds__(256) void k_pass1(SimDev S, const uint32_t* __restrict__ sel,
                                               const uint32_t* __restrict__ nsel) {
    const int lane = threadIdx.x & 63;
    const uint32_t nw = gridDim.x * blockDim.x / 64;
    const uint32_t n = sel ? *nsel : S.NL;
    for (uint32_t i = (blockIdx.x * blockDim.x + threadIdx.x) / 64; i < n; i += nw) {
        const uint32_t lv = sel ? sel[i] : i;
        if (lv >= S.NL || S.dead[S.v0 + lv] || !S.dirty[lv]) continue;  // wave-uniform
        const uint64_t row = (uint64_t)lv * S.N;
        const LaneView V{S, S.st + row, S.inc + row, S.dev + (uint64_t)lv * S.W};
        P1 r;
        seg_pass1<64>(S, V, S.dlist + (uint64_t)lv * S.dcap, true, (uint32_t)lane, r.dtot, r.dlo, r.dhi, r.last, r.nd);
        if (lane == 0) S.p1[lv] = r;
    }
}

// The compacted views to hash ordered by their string's total shift (refresh_checksums,
// RP_SIM_CK_SORT), so that a wave's 64 lanes meet their deviated pieces in the same chunk groups
// (the fixup path runs for the whole wave when any lane needs it). keys[i] from vdt (block_apply)
// or from the view's pass-1 record.
__global__ void k_ck_sort_keys(SimDev S, const uint32_t* __restrict__ sel, const uint32_t* __restrict__ nsel,
                               uint32_t* __restrict__ keys, uint32_t* __restrict__ vals, int from_vdt) {
    const uint32_t n = *nsel;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint32_t lv = sel[i];
        const int64_t t = lv >= S.NL ? 0 : from_vdt ? S.vdt[lv] : S.p1[lv].dtot;
        keys[i] = (uint32_t)(t + 0x80000000ll);
        vals[i] = lv;
    }
}

// Every live local node whose view changed: one node per lane, the wave's 64 chains in lockstep
// over a shared LDS ring of the base string. A view with more deviated pieces than its list holds,
// or a wave whose lanes drift further apart than the ring allows, uses the L2 path
// (lane_checksum).
// Fixup statistics of k_ck_lanes (diagnostics only, -DRP_CKL_STAT; printed per launch under
// RP_CKL_STAT_PRINT): [0] wave-groups, [1] wave-groups that ran a fixup, [2] lane-groups with a
// fixup, [3] active lane-groups, [4] waves
#ifdef RP_CKL_STAT
__device__ unsigned long long g_ckl_stat[8];
#endif
__global__ __launch_bounds__(256) void k_ck_lanes(SimDev S, const uint32_t* __restrict__ sel,
                                                  const uint32_t* __restrict__ nsel) {
    __shared__ __attribute__((aligned(16))) uint32_t rings[4][kRingW + 24];
    const int lane = threadIdx.x & 63;
    uint32_t lv = blockIdx.x * blockDim.x + threadIdx.x;
    if (sel) lv = lv < *nsel ? sel[lv] : NONE;  // a compacted list of the views to hash
    const bool act = lv < S.NL && !S.dead[S.v0 + lv] && S.dirty[lv];
    if (__ballot(act) == 0) return;  // wave-uniform
    const uint32_t N = S.N;
    const uint64_t row = (uint64_t)(act ? lv : 0) * N;
    const LaneView V{S, S.st + row, S.inc + row, S.dev + (uint64_t)(act ? lv : 0) * S.W};
    // pass 1: length, last deviation, the running shift's range; the deviated pieces are listed
    // (address order) for the main loop, which then never scans the bitmap or chases member
    // tables at a piece boundary
    int64_t dtot = 0, dlo = 0, dhi = 0;
    uint32_t last = NONE, nd = 0;
    uint4* dl = S.dlist + (uint64_t)(act ? lv : 0) * S.dcap;
    if (act) {
        if (S.p1_pre) {
            const P1 r = S.p1[lv];
            dtot = r.dtot;
            dlo = r.dlo;
            dhi = r.dhi;
            last = r.last;
            nd = r.nd;
        } else {
            lane_pass1(S, V, dl, dtot, dlo, dhi, last, nd);
        }
    }
    const uint64_t len = (uint64_t)((int64_t)S.boff[N] + dtot);
    const bool ring_ok = __ballot(act && (nd > S.dcap || len > 0x7FFFFFF0ull)) == 0 &&
                         wave_max64(act ? dhi : 0) - wave_min64(act ? dlo : 0) <= (int64_t)(kRing - 2 * kSlice - 256);
    if (!ring_ok) {  // wave-uniform
        if (act) {
            S.checksum[lv] = lane_checksum(S, lv);
            S.dirty[lv] = 0;
        }
        return;
    }
    const int64_t DLO = wave_min64(act ? dlo : 0);
    uint32_t h = 0, g = 0, f = 0;
    uint32_t iters = 0;
    if (act) {
        if (len <= 24) {
            uint8_t buf[24];
            Fwd F;
            F.init(V);
            for (uint32_t q = 0; q < (uint32_t)len; q++) buf[q] = F.byte(V, q);
            h = fh::hash32(fh::PtrSrc{buf}, (uint32_t)len);
        } else {
            uint8_t tail[20];
            uint32_t kd = last;
            int64_t da = dtot;
            Piece P{};
            uint64_t E = 0, B = 0;
            if (kd != NONE) {
                P = V.piece(kd);
                E = (uint64_t)((int64_t)S.boff[kd + 1] + da);
                B = E - P.plen;
            }
            for (int i = 19; i >= 0; i--) {
                const uint64_t q = len - 20 + (uint64_t)i;
                while (kd != NONE && q < B) {
                    da -= (int64_t)P.plen - (int64_t)P.blen;
                    kd = V.prev_dev(kd);
                    if (kd != NONE) {
                        P = V.piece(kd);
                        E = (uint64_t)((int64_t)S.boff[kd + 1] + da);
                        B = E - P.plen;
                    }
                }
                tail[i] = (kd != NONE && q >= B && q < E) ? V.piece_byte(P, (uint32_t)(q - B))
                                                           : S.sbase[(uint64_t)((int64_t)q - da)];
            }
            auto tw = [&](int o) {
                return (uint32_t)tail[o] | ((uint32_t)tail[o + 1] << 8) | ((uint32_t)tail[o + 2] << 16) |
                       ((uint32_t)tail[o + 3] << 24);
            };
            h = (uint32_t)len;
            g = fh::kC1 * (uint32_t)len;
            f = g;
            h ^= premix(tw(16));
            h = fh::rotr(h, 19) * 5 + 0xe6546b64u;
            h ^= premix(tw(4));
            h = fh::rotr(h, 19) * 5 + 0xe6546b64u;
            g ^= premix(tw(12));
            g = fh::rotr(g, 19) * 5 + 0xe6546b64u;
            g ^= premix(tw(8));
            g = fh::rotr(g, 19) * 5 + 0xe6546b64u;
            f += premix(tw(0));
            f = fh::rotr(f, 19) + 113;
            iters = (uint32_t)((len - 1) / 20);
        }
    }
    const uint32_t maxit = (uint32_t)wave_max64((int64_t)iters);
    BaseRing R{rings[threadIdx.x >> 6], 0, {}};
    R.start(S.sbase, lane);
    LaneCursor C;
    if (act) C.init(S, V, dl, nd);
    const uint32_t lead = (uint32_t)(240 - DLO) + kSlice;  // ring lookahead past a group's q0
    // Groups of 4 chunks, software-pipelined: while the serial chain consumes group g, group g+1's
    // words are read from the ring assuming they are clean (one straight run of 21 LDS words at
    // the current shift) and pre-mixed, in the same basic block, so the two independent
    // instruction streams hide each other's latency (a lone wave per SIMD). The rare chunks that
    // touch a deviated piece are then redone through the cursor.
    uint32_t wd[4][5], p5[4], p6[4], p7[4];
    // group words at the cursor's shift (speculative) + their pre-mixes
    auto produce = [&](uint32_t q, uint32_t (&w)[4][5], uint32_t (&a5)[4], uint32_t (&a6)[4], uint32_t (&a7)[4]) {
        const uint32_t o = (uint32_t)((int32_t)q - C.delta);
        const uint32_t* p = R.ring + ((o >> 2) & (kRingW - 1));
        const uint32_t sh = o & 3;
        uint32_t x[21];
#pragma unroll
        for (int i = 0; i < 21; i++) x[i] = p[i];  // (the ring mirrors 24 words past its end)
#pragma unroll
        for (int j = 0; j < 4; j++) {
#pragma unroll
            for (int i = 0; i < 5; i++) w[j][i] = __builtin_amdgcn_alignbyte(x[5 * j + i + 1], x[5 * j + i], sh);
            a5[j] = premix(w[j][3]);
            a6[j] = premix(w[j][2]);
            a7[j] = premix(mul_lo_add(w[j][4], fh::kC1, w[j][1]));
        }
    };
    // redo the chunks of the group at q that touch the piece under the cursor (and later ones)
    auto fixup = [&](uint32_t q, uint32_t ng, uint32_t (&w4)[4][5], uint32_t (&a5)[4], uint32_t (&a6)[4],
                     uint32_t (&a7)[4]) {
        const uint32_t j0 = C.pos > q ? (C.pos - q) / 20 : 0;
        for (uint32_t j = j0; j < ng; j++) {
            const uint32_t qj = q + 20 * j;
            while (qj >= C.pend && C.cur.w < N) C.advance(S, V);
            uint32_t w[5];
#ifdef RP_CKL_STAT
            atomicAdd(&g_ckl_stat[(qj + 20 <= C.pos) ? 5 : (C.basedig && qj + 20 <= C.nstart) ? 6 : 7], 1ull);
#endif
            if (qj + 20 <= C.pos) {
                R.words((uint32_t)((int32_t)qj - C.delta), w);
            } else if (C.basedig && qj + 20 <= C.nstart) {
                // one deviated piece whose only difference is its status: base bytes at shift
                // delta before the status, the status characters, base bytes at shift
                // delta + sl - 5 after
                const int32_t s0 = (int32_t)(C.pos + C.nl), s1 = s0 + (int32_t)C.sl;
                uint32_t w1[5], w2[5];
                const uint32_t o1 = (uint32_t)((int32_t)qj - C.delta);
                R.words(o1, w1);
                R.words(o1 - C.sl + 5u, w2);
#pragma unroll
                for (int i = 0; i < 5; i++) {
                    const int32_t qb = (int32_t)qj + 4 * i;
                    const int32_t m1 = s0 - qb, m2 = s1 - qb;
                    const uint32_t k1 = m1 <= 0 ? 0u : m1 >= 4 ? 0xFFFFFFFFu : (1u << (8 * m1)) - 1u;
                    const uint32_t k2 = m2 <= 0 ? 0u : m2 >= 4 ? 0xFFFFFFFFu : (1u << (8 * m2)) - 1u;
                    const int32_t so = -m1;  // status byte index of this word's byte 0
                    const uint32_t sw = so >= 0 ? (so < 8 ? (uint32_t)(C.st64 >> (8 * so)) : 0u)
                                                : (so > -4 ? (uint32_t)(C.st64 << (8 * -so)) : 0u);
                    w[i] = (w1[i] & k1) | (sw & k2 & ~k1) | (w2[i] & ~k2);
                }
            } else {
                LaneCursor T = C;  // bytes across piece boundaries: a copy walks ahead
                for (int i = 0; i < 5; i++) {
                    uint32_t x = 0;
                    for (int b = 0; b < 4; b++) x |= (uint32_t)lane_byte(S, V, T, qj + 4 * i + b) << (8 * b);
                    w[i] = x;
                }
            }
#pragma unroll
            for (int jj = 0; jj < 4; jj++)
                if ((uint32_t)jj == j) {
#pragma unroll
                    for (int i = 0; i < 5; i++) w4[jj][i] = w[i];
                    a5[jj] = premix(w[3]);
                    a6[jj] = premix(w[2]);
                    a7[jj] = premix(w[1] + w[4] * fh::kC1);
                }
        }
    };
    auto ngroup = [&](uint32_t c0) { return c0 >= iters ? 0u : (iters - c0 < 4 ? iters - c0 : 4u); };
    // group 0
    R.ensure(S.sbase, lead, lane);
    if (act && iters) {
        while (0 >= C.pend && C.cur.w < N) C.advance(S, V);
        produce(0, wd, p5, p6, p7);
        if (__builtin_expect(20 * ngroup(0) > C.pos, 0)) fixup(0, ngroup(0), wd, p5, p6, p7);
    }
    for (uint32_t c0 = 0; c0 < maxit; c0 += 4) {
        const uint32_t q1 = (c0 + 4) * 20;  // the next group
        R.ensure(S.sbase, q1 + lead, lane);
        const uint32_t ng = ngroup(c0), ng1 = ngroup(c0 + 4);
        uint32_t nw[4][5], n5[4], n6[4], n7[4];
        if (ng1) {
            while (__builtin_expect(q1 >= C.pend, 0) && C.cur.w < N) C.advance(S, V);
        }
        // one chunk of the chain (5 r as one v_lshl_add_u32)
        auto chunk = [&](int j) {
            h += wd[j][0];
            g += wd[j][1];
            f += wd[j][2];
            const uint32_t rh = fh::rotr(h ^ p5[j], 19), rg = fh::rotr(g ^ p6[j], 19), rf = fh::rotr(f ^ p7[j], 19);
            h = lshl_add<2>(rh, rh) + 0xe6546b64u + wd[j][4];
            g = lshl_add<2>(rg, rg) + 0xe6546b64u + wd[j][0];
            f = lshl_add<2>(rf, rf) + 0xe6546b64u + wd[j][3];
            f += g;
            g += f;
        };
        // one basic block: the next group's words + pre-mixes beside this group's chain. The arms
        // differ only in masking; each holds its own copy of produce (a block boundary between
        // the two streams would serialise them; without the compiler barriers hipcc hoists the
        // common copy out of the arms). Every live lane takes a whole group except in
        // its last one.
        // (the pins keep the pre-mixes computed in the arm: hipcc would sink the arms' common
        // multiplies into the join block)
        auto pin = [&]() {
#pragma unroll
            for (int j = 0; j < 4; j++) asm volatile("" : "+v"(n5[j]), "+v"(n6[j]), "+v"(n7[j]));
        };
        if (__ballot(act && ng < 4) == 0) {
            asm volatile("" ::: "memory");  // keeps the arm's ring reads (and all that uses them) in the arm
            produce(q1, nw, n5, n6, n7);
#pragma unroll
            for (int j = 0; j < 4; j++) chunk(j);
            pin();
        } else {
            asm volatile("" ::: "memory");
            produce(q1, nw, n5, n6, n7);
#pragma unroll
            for (int j = 0; j < 4; j++)
                if ((uint32_t)j < ng) chunk(j);
            pin();
        }
#ifdef RP_CKL_STAT
        {
            const uint64_t fx = __ballot(ng1 && q1 + 20 * ng1 > C.pos), av = __ballot(act && ng1);
            if (lane == 0 && av) {
                atomicAdd(&g_ckl_stat[0], 1ull);
                atomicAdd(&g_ckl_stat[1], fx ? 1ull : 0ull);
                atomicAdd(&g_ckl_stat[2], (unsigned long long)__popcll(fx));
                atomicAdd(&g_ckl_stat[3], (unsigned long long)__popcll(av));
            }
        }
#endif
        if (__builtin_expect(ng1 && q1 + 20 * ng1 > C.pos, 0) && S.ck_ablate == 0) fixup(q1, ng1, nw, n5, n6, n7);
#pragma unroll
        for (int j = 0; j < 4; j++) {
#pragma unroll
            for (int i = 0; i < 5; i++) wd[j][i] = nw[j][i];
            p5[j] = n5[j];
            p6[j] = n6[j];
            p7[j] = n7[j];
        }
    }
    if (!act) return;
    if (len > 24) {
        g = fh::rotr(g, 11) * fh::kC1;
        g = fh::rotr(g, 17) * fh::kC1;
        f = fh::rotr(f, 11) * fh::kC1;
        f = fh::rotr(f, 17) * fh::kC1;
        h = fh::rotr(h + g, 19);
        h = h * 5 + 0xe6546b64u;
        h = fh::rotr(h, 17) * fh::kC1;
        h = fh::rotr(h + f, 19);
        h = h * 5 + 0xe6546b64u;
        h = fh::rotr(h, 17) * fh::kC1;
    }
    S.checksum[lv] = h;
    S.dirty[lv] = 0;
}

// ---- producer/consumer lane checksums

// The chain's initial state from the string's last 20 bytes (farmhashmk Hash32, len > 24), or
// the whole hash for len <= 24 (returned in h with *done).
__device__ void lane_chain_init(const SimDev& S, const LaneView& V, uint64_t len, int64_t dtot, uint32_t last,
                                uint32_t& h, uint32_t& g, uint32_t& f, bool& done) {
    done = false;
    if (len <= 24) {
        uint8_t buf[24];
        Fwd F;
        F.init(V);
        for (uint32_t q = 0; q < (uint32_t)len; q++) buf[q] = F.byte(V, q);
        h = fh::hash32(fh::PtrSrc{buf}, (uint32_t)len);
        done = true;
        return;
    }
    uint8_t tail[20];
    uint32_t kd = last;
    int64_t da = dtot;
    Piece P{};
    uint64_t E = 0, B = 0;
    if (kd != NONE) {
        P = V.piece(kd);
        E = (uint64_t)((int64_t)S.boff[kd + 1] + da);
        B = E - P.plen;
    }
    for (int i = 19; i >= 0; i--) {
        const uint64_t q = len - 20 + (uint64_t)i;
        while (kd != NONE && q < B) {
            da -= (int64_t)P.plen - (int64_t)P.blen;
            kd = V.prev_dev(kd);
            if (kd != NONE) {
                P = V.piece(kd);
                E = (uint64_t)((int64_t)S.boff[kd + 1] + da);
                B = E - P.plen;
            }
        }
        tail[i] = (kd != NONE && q >= B && q < E) ? V.piece_byte(P, (uint32_t)(q - B))
                                                   : S.sbase[(uint64_t)((int64_t)q - da)];
    }
    auto tw = [&](int o) {
        return (uint32_t)tail[o] | ((uint32_t)tail[o + 1] << 8) | ((uint32_t)tail[o + 2] << 16) |
               ((uint32_t)tail[o + 3] << 24);
    };
    h = (uint32_t)len;
    g = fh::kC1 * (uint32_t)len;
    f = g;
    h ^= premix(tw(16));
    h = fh::rotr(h, 19) * 5 + 0xe6546b64u;
    h ^= premix(tw(4));
    h = fh::rotr(h, 19) * 5 + 0xe6546b64u;
    g ^= premix(tw(12));
    g = fh::rotr(g, 19) * 5 + 0xe6546b64u;
    g ^= premix(tw(8));
    g = fh::rotr(g, 19) * 5 + 0xe6546b64u;
    f += premix(tw(0));
    f = fh::rotr(f, 19) + 113;
}

// x * 5 as one full-rate shift-add (the compiler otherwise may pick a 64-bit multiply-add)
__device__ __forceinline__ uint32_t mul5(uint32_t x) {
    uint32_t r;
    asm("v_lshl_add_u32 %0, %1, 2, %1" : "=v"(r) : "v"(x));
    return r;
}

__device__ __forceinline__ uint32_t chain_final(uint32_t h, uint32_t g, uint32_t f) {
    g = fh::rotr(g, 11) * fh::kC1;
    g = fh::rotr(g, 17) * fh::kC1;
    f = fh::rotr(f, 11) * fh::kC1;
    f = fh::rotr(f, 17) * fh::kC1;
    h = fh::rotr(h + g, 19);
    h = h * 5 + 0xe6546b64u;
    h = fh::rotr(h, 17) * fh::kC1;
    h = fh::rotr(h + f, 19);
    h = h * 5 + 0xe6546b64u;
    h = fh::rotr(h, 17) * fh::kC1;
    return h;
}

// The 20-byte chunk of a lane's string at qj through its cursor (advancing it): base words at
// the cursor's shift, a status-only piece as a word overlay, or bytes across pieces.
__device__ void cursor_chunk(const SimDev& S, const LaneView& V, LaneCursor& C, const BaseRing& R, uint32_t qj,
                             uint32_t (&w)[5]) {
    while (qj >= C.pend && C.cur.w < S.N) C.advance(S, V);
    if (qj + 20 <= C.pos) {
        R.words((uint32_t)((int32_t)qj - C.delta), w);
    } else if (C.basedig && qj + 20 <= C.nstart) {
        const int32_t s0 = (int32_t)(C.pos + C.nl), s1 = s0 + (int32_t)C.sl;
        uint32_t w1[5], w2[5];
        const uint32_t o1 = (uint32_t)((int32_t)qj - C.delta);
        R.words(o1, w1);
        R.words(o1 - C.sl + 5u, w2);
#pragma unroll
        for (int i = 0; i < 5; i++) {
            const int32_t qb = (int32_t)qj + 4 * i;
            const int32_t m1 = s0 - qb, m2 = s1 - qb;
            const uint32_t k1 = m1 <= 0 ? 0u : m1 >= 4 ? 0xFFFFFFFFu : (1u << (8 * m1)) - 1u;
            const uint32_t k2 = m2 <= 0 ? 0u : m2 >= 4 ? 0xFFFFFFFFu : (1u << (8 * m2)) - 1u;
            const int32_t so = -m1;
            const uint32_t sw = so >= 0 ? (so < 8 ? (uint32_t)(C.st64 >> (8 * so)) : 0u)
                                        : (so > -4 ? (uint32_t)(C.st64 << (8 * -so)) : 0u);
            w[i] = (w1[i] & k1) | (sw & k2 & ~k1) | (w2[i] & ~k2);
        }
    } else {
        LaneCursor T = C;
        for (int i = 0; i < 5; i++) {
            uint32_t x = 0;
            for (int b = 0; b < 4; b++) x |= (uint32_t)lane_byte(S, V, T, qj + 4 * i + b) << (8 * b);
            w[i] = x;
        }
    }
}

// Every live local node whose view changed, 64 nodes per workgroup: wave 0 runs the 64 serial
// chains (only the chain's ~17 dependent-ish ops per chunk), waves 1-3 produce the chunks' words
// and pre-mixes one epoch ahead (each a 4-chunk group per epoch, from a shared LDS ring of the
// base string kept by wave 1) into double-buffered LDS. A view's checksum is one serial chain,
// so this is what bounds a refresh when few waves share a SIMD (the sharded case).
// NP producer waves (3: 256-thread blocks; 7: 512-thread blocks, two waves per SIMD), each
// producing 4 chunks per epoch.
// sel != null: only the nodes listed in sel[0..*nsel) (the ping-req senders of D1, whose
// views phases B and C just changed), 64 per workgroup in list order.
// CP chunks per producer per epoch: the LDS stage is 4 KB x NP x CP, so a smaller epoch lets
// several groups share a CU (C5 on one GPU: ~635 dirty groups for 256 CUs).
template <int NP, int CP = 4>
__global__ __launch_bounds__(64 * (NP + 1)) void k_ck_pc(SimDev S, const uint32_t* __restrict__ sel,
                                                         const uint32_t* __restrict__ nsel) {
    constexpr int kEp = CP * NP;  // chunks per epoch
    __shared__ __attribute__((aligned(16))) uint32_t ring[kRingW + 24];
    __shared__ __attribute__((aligned(16))) u32x4s stage[2][kEp][2][64];
    __shared__ uint32_t s_nd[64], s_iters[64];
    __shared__ int32_t s_red[4];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint32_t lv = blockIdx.x * 64 + lane;
    if (sel) lv = lv < *nsel ? sel[lv] : NONE;
    const bool act = lv < S.NL && !S.dead[S.v0 + lv] && S.dirty[lv];
    if (!__syncthreads_or(act ? 1 : 0)) return;
    const uint32_t N = S.N;
    const uint64_t row = (uint64_t)(act ? lv : 0) * N;
    const LaneView V{S, S.st + row, S.inc + row, S.dev + (uint64_t)(act ? lv : 0) * S.W};
    uint4* dl = S.dlist + (uint64_t)(act ? lv : 0) * S.dcap;
    uint32_t h = 0, g = 0, f = 0;
    uint64_t len = 0;
    bool done = false;
    if (wv == 0) {
        int64_t dtot = 0, dlo = 0, dhi = 0;
        uint32_t last = NONE, nd = 0;
        if (act) {
            if (S.p1_pre) {
                const P1 r = S.p1[lv];
                dtot = r.dtot;
                dlo = r.dlo;
                dhi = r.dhi;
                last = r.last;
                nd = r.nd;
            } else {
                lane_pass1(S, V, dl, dtot, dlo, dhi, last, nd);
            }
        }
        len = (uint64_t)((int64_t)S.boff[N] + dtot);
        const bool bad = act && (nd > S.dcap || len > 0x7FFFFFF0ull);
        uint32_t iters = 0;
        if (act && !bad) {
            lane_chain_init(S, V, len, dtot, last, h, g, f, done);
            iters = done ? 0u : (uint32_t)((len - 1) / 20);
        }
        s_nd[lane] = nd;
        s_iters[lane] = iters;
        const int64_t DLO = wave_min64(act ? dlo : 0), DHI = wave_max64(act ? dhi : 0);
        // the ring holds two epochs ahead of the producers plus a slice being refilled
        const bool okw = __ballot(bad) == 0 && DHI - DLO <= (int64_t)(kRing - 3 * kSlice - 4 * kEp * 20 - 256);
        const int64_t MX = wave_max64((int64_t)iters);
        if (lane == 0) {
            s_red[0] = okw ? 1 : 0;
            s_red[1] = (int32_t)DLO;
            s_red[2] = (int32_t)MX;
        }
    }
    __syncthreads();
    if (!s_red[0]) {  // block-uniform: too many deviations for the list or the ring
        if (wv == 0 && act) {
            S.checksum[lv] = lane_checksum(S, lv);
            S.dirty[lv] = 0;
        }
        return;
    }
    const int32_t DLO = s_red[1];
    const uint32_t maxit = (uint32_t)s_red[2];
    const uint32_t nep = (maxit + kEp - 1) / kEp;
    const uint32_t lead = (uint32_t)(2 * kEp * 20 + 64 - DLO) + kSlice;
    BaseRing R;
    R.ring = ring;
    R.hi = 0;
    LaneCursor C;
    uint32_t iters = s_iters[lane];
    if (wv >= 1) {
        if (act && iters) C.init(S, V, dl, s_nd[lane]);
        if (wv == 1) {
            R.start(S.sbase, lane);
            R.ensure(S.sbase, lead, lane);  // epochs 0 and 1
        }
    }
    // producer p (1..NP) owns chunks [e*kEp + CP(p-1), +CP) of epoch e
    auto produce = [&](uint32_t e) {
        const uint32_t c0 = e * kEp + CP * (wv - 1);
        const uint32_t ng = c0 >= iters ? 0u : (iters - c0 < (uint32_t)CP ? iters - c0 : (uint32_t)CP);
        if (!ng) return;
        const uint32_t q = c0 * 20;
        while (q >= C.pend && C.cur.w < N) C.advance(S, V);
        uint32_t w4[CP][5];
        {
            const uint32_t o = (uint32_t)((int32_t)q - C.delta);
            const uint32_t* p = R.ring + ((o >> 2) & (kRingW - 1));
            const uint32_t sh = o & 3;
            uint32_t x[5 * CP + 1];
#pragma unroll
            for (int i = 0; i < 5 * CP + 1; i++) x[i] = p[i];
#pragma unroll
            for (int j = 0; j < CP; j++)
#pragma unroll
                for (int i = 0; i < 5; i++) w4[j][i] = __builtin_amdgcn_alignbyte(x[5 * j + i + 1], x[5 * j + i], sh);
        }
        if (__builtin_expect(q + 20 * ng > C.pos, 0)) {
            const uint32_t j0 = C.pos > q ? (C.pos - q) / 20 : 0;
            for (uint32_t j = j0; j < ng; j++) {
                uint32_t w[5];
                cursor_chunk(S, V, C, R, q + 20 * j, w);
#pragma unroll
                for (int jj = 0; jj < CP; jj++)
                    if ((uint32_t)jj == j)
#pragma unroll
                        for (int i = 0; i < 5; i++) w4[jj][i] = w[i];
            }
        }
        const int b = e & 1;
#pragma unroll
        for (int j = 0; j < CP; j++) {
            const int slot = CP * (wv - 1) + j;
            stage[b][slot][0][lane] = u32x4s{w4[j][0], w4[j][1], w4[j][2], w4[j][3]};
            stage[b][slot][1][lane] = u32x4s{w4[j][4], premix(w4[j][3]), premix(w4[j][2]),
                                             premix(w4[j][1] + w4[j][4] * fh::kC1)};
        }
    };
    __syncthreads();  // the ring holds epochs 0 and 1
    if (wv >= 1 && act) produce(0);
    __syncthreads();
#ifdef RP_CK_PROF
    uint64_t t_work = 0, t_bar = 0, t0 = clock64();
#endif
    for (uint32_t e = 0; e < nep; e++) {
#ifdef RP_CK_PROF
        const uint64_t ta = clock64();
#endif
        if (wv == 0) {
            if (act) {
                const int b = e & 1;
                const uint32_t c0 = e * kEp;
                auto step = [&](const u32x4s& x0, const u32x4s& x1) {
                    h += x0.x;
                    g += x0.y;
                    f += x0.z;
                    h = mul5(fh::rotr(h ^ x1.y, 19)) + 0xe6546b64u + x1.x;
                    g = mul5(fh::rotr(g ^ x1.z, 19)) + 0xe6546b64u + x0.x;
                    f = mul5(fh::rotr(f ^ x1.w, 19)) + 0xe6546b64u + x0.w;
                    f += g;
                    g += f;
                };
                if (__ballot(c0 + kEp > iters) == 0) {
                    // every lane takes the whole epoch: loads issued a 4-chunk group ahead, no
                    // branches
                    u32x4s x[2][CP][2];
#pragma unroll
                    for (int j = 0; j < CP; j++) {
                        x[0][j][0] = stage[b][j][0][lane];
                        x[0][j][1] = stage[b][j][1][lane];
                    }
#pragma unroll
                    for (int q = 0; q < NP; q++) {
                        if (q + 1 < NP) {
#pragma unroll
                            for (int j = 0; j < CP; j++) {
                                x[(q + 1) & 1][j][0] = stage[b][CP * (q + 1) + j][0][lane];
                                x[(q + 1) & 1][j][1] = stage[b][CP * (q + 1) + j][1][lane];
                            }
                        }
#pragma unroll
                        for (int j = 0; j < CP; j++) step(x[q & 1][j][0], x[q & 1][j][1]);
                    }
                } else {
#pragma unroll
                    for (int j = 0; j < kEp; j++)
                        if (c0 + j < iters) step(stage[b][j][0][lane], stage[b][j][1][lane]);
                }
            }
        } else {
            if (act && e + 1 < nep) produce(e + 1);
            // the ring one epoch further ahead (the producers of the next iteration read it after
            // the barrier; nobody reads the slices being replaced any more)
            if (wv == 1) R.ensure(S.sbase, (e + 2) * kEp * 20 + lead, lane);
        }
#ifdef RP_CK_PROF
        const uint64_t tb = clock64();
        t_work += tb - ta;
#endif
        __syncthreads();
#ifdef RP_CK_PROF
        t_bar += clock64() - tb;
#endif
    }
#ifdef RP_CK_PROF
    if (lane == 0 && (blockIdx.x == 0 || blockIdx.x == gridDim.x / 2))
        printf("ckprof blk %u wave %d: epochs %u maxit %u total %llu work %llu bar %llu (cyc/chunk %.1f)\n", blockIdx.x,
               wv, nep, maxit, (unsigned long long)(clock64() - t0), (unsigned long long)t_work,
               (unsigned long long)t_bar, (double)(clock64() - t0) / (maxit ? maxit : 1));
#endif
    if (wv == 0 && act) {
        S.checksum[lv] = done ? h : chain_final(h, g, f);
        S.dirty[lv] = 0;
    }
}

// The chains of k_ck_pc for a short list of views (D1's ping-req senders, whose checksums their
// ping-req bodies carry: ~1 % of the nodes, so a few groups on an idle machine and the refresh is
// a latency bound). The coupled (g, f) pair runs on two lanes in the pre-added form of
// rp_hashlong.hip (one instruction advances both: six VALU ops per chunk, four of them on the
// dependent path, against k_ck_pc's one lane per view), so a workgroup holds VPG <= 32 views.
// Waves: 0 = the pairs (lane 2i: g of view i, lane 2i + 1: f); 1 = the h chains (lane i < VPG;
// also the chain init per view; pass 1 runs on every wave, SEG lanes per view: seg_pass1); 2..NP+1 = producers, lane = (view lane % VPG, part
// lane / VPG): producer p's part hf makes chunks [e kEp + CP (NPART p + hf), + CP) of epoch e.
// Producers are the bound when views carry many deviated pieces (a wave waits for its slowest
// lane's piece overlay every call), so D1 takes 16 views per group: twice the chunks per epoch
// for the same producer calls, and the chain waves set the pace. A chunk's
// record per chain word: h {premix(d), K + e + a'}, g {premix(c), 3K + 2a + d + b'}, f
// {premix(b + e c1), 2K + a + d + c'} with a', b', c' the next chunk's first words (0 after the
// last), so a producer also reads the first words of the chunk after its run.
template <int NP, int CP, int VPG>
__global__ __launch_bounds__(64 * (NP + 2)) void k_ck_pair(SimDev S, const uint32_t* __restrict__ sel,
                                                          const uint32_t* __restrict__ nsel) {
    static_assert(VPG == 8 || VPG == 16 || VPG == 32, "views per group");
    constexpr int NPART = 64 / VPG;       // producer lanes per view in a wave
    constexpr int kEp = NPART * CP * NP;  // chunks per epoch
    static_assert(kEp % 8 == 0, "the chain loads 8 records ahead");
    constexpr uint32_t kK = 0xe6546b64u;
    __shared__ __attribute__((aligned(16))) uint32_t ring[kRingW + 24];
    __shared__ __attribute__((aligned(16))) uint2 stage[2][kEp][3][VPG];  // role 0: h, 1: g, 2: f
    __shared__ uint32_t s_nd[VPG], s_iters[VPG], s_st[3][VPG], s_w0[3][VPG], s_last[VPG];
    __shared__ int64_t s_dtot[VPG], s_dlo[VPG], s_dhi[VPG];
    constexpr int SEG = 64 * (NP + 2) / VPG;  // lanes per view for pass 1
    static_assert(SEG <= 64 && (SEG & (SEG - 1)) == 0, "pass-1 segments within a wave");
    __shared__ int32_t s_red[4];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    // the lane's view (wave 0: lanes >= 2 VPG idle; wave 1: lanes >= VPG idle)
    const uint32_t vi = wv == 0 ? (uint32_t)lane >> 1 : wv == 1 ? (uint32_t)lane : (uint32_t)lane % VPG;
    uint32_t lv = vi < VPG ? blockIdx.x * VPG + vi : NONE;
    if (sel && lv != NONE) lv = lv < *nsel ? sel[lv] : NONE;
    const bool act = lv < S.NL && !S.dead[S.v0 + lv] && S.dirty[lv];
    if (!__syncthreads_or(act ? 1 : 0)) return;
    const uint32_t N = S.N;
    const uint64_t row = (uint64_t)(act ? lv : 0) * N;
    const LaneView V{S, S.st + row, S.inc + row, S.dev + (uint64_t)(act ? lv : 0) * S.W};
    uint4* dl = S.dlist + (uint64_t)(act ? lv : 0) * S.dcap;
    {  // pass 1, SEG lanes per view
        const uint32_t sv = threadIdx.x / SEG, sl = threadIdx.x % SEG;
        uint32_t slv = blockIdx.x * VPG + sv;
        if (sel) slv = slv < *nsel ? sel[slv] : NONE;
        const bool sact = slv < S.NL && !S.dead[S.v0 + slv] && S.dirty[slv];
        const uint64_t srow = (uint64_t)(sact ? slv : 0) * N;
        const LaneView SV{S, S.st + srow, S.inc + srow, S.dev + (uint64_t)(sact ? slv : 0) * S.W};
        int64_t dt, dlo1, dhi1;
        uint32_t la, nd1;
        seg_pass1<SEG>(S, SV, S.dlist + (uint64_t)(sact ? slv : 0) * S.dcap, sact, sl, dt, dlo1, dhi1, la, nd1);
        if (sl == 0) {
            s_dtot[sv] = dt;
            s_dlo[sv] = dlo1;
            s_dhi[sv] = dhi1;
            s_last[sv] = la;
            s_nd[sv] = nd1;
        }
    }
    __syncthreads();
    uint32_t hdone = 0;
    if (wv == 1) {
        int64_t dtot = 0, dlo = 0, dhi = 0;
        uint32_t last = NONE, nd = 0;
        if (act) {
            dtot = s_dtot[lane];
            dlo = s_dlo[lane];
            dhi = s_dhi[lane];
            last = s_last[lane];
            nd = s_nd[lane];
        }
        const uint64_t len = (uint64_t)((int64_t)S.boff[N] + dtot);
        const bool bad = act && (nd > S.dcap || len > 0x7FFFFFF0ull);
        uint32_t iters = 0, h = 0, g = 0, f = 0;
        bool done = false;
        if (act && !bad) {
            lane_chain_init(S, V, len, dtot, last, h, g, f, done);
            iters = done ? 0u : (uint32_t)((len - 1) / 20);
        }
        hdone = h;
        if (lane < VPG) {
            s_iters[lane] = iters;
            s_st[0][lane] = h;
            s_st[1][lane] = g;
            s_st[2][lane] = f;
        }
        const int64_t DLO = wave_min64(act ? dlo : 0), DHI = wave_max64(act ? dhi : 0);
        const bool okw = __ballot(bad) == 0 && DHI - DLO <= (int64_t)(kRing - 3 * kSlice - 4 * kEp * 20 - 256);
        const int64_t MX = wave_max64((int64_t)iters);
        if (lane == 0) {
            s_red[0] = okw ? 1 : 0;
            s_red[1] = (int32_t)DLO;
            s_red[2] = (int32_t)MX;
        }
    }
    __syncthreads();
    if (!s_red[0]) {  // block-uniform: too many deviations for the list or the ring
        if (wv == 1 && act) {
            S.checksum[lv] = lane_checksum(S, lv);
            S.dirty[lv] = 0;
        }
        return;
    }
    const int32_t DLO = s_red[1];
    const uint32_t maxit = (uint32_t)s_red[2];
    const uint32_t nep = (maxit + kEp - 1) / kEp;
    const uint32_t lead = (uint32_t)(2 * kEp * 20 + 64 - DLO) + kSlice;
    const uint32_t iters = vi < VPG ? s_iters[vi] : 0u;
    BaseRing R;
    R.ring = ring;
    R.hi = 0;
    LaneCursor C;
    const int pw = wv - 2, hf = lane / VPG;
    if (wv >= 2) {
        if (act && iters) C.init(S, V, dl, s_nd[vi]);
        if (wv == 2) {
            R.start(S.sbase, lane);
            R.ensure(S.sbase, lead, lane);  // epochs 0 and 1
        }
    }
    auto produce = [&](uint32_t e) {
        const uint32_t c0 = e * kEp + CP * (NPART * pw + hf);
        const uint32_t ng = c0 >= iters ? 0u : (iters - c0 < (uint32_t)CP ? iters - c0 : (uint32_t)CP);
        if (!ng) return;
        const uint32_t ngx = ng + (c0 + ng < iters ? 1u : 0u);  // + the next chunk, if any
        const uint32_t q = c0 * 20;
        while (q >= C.pend && C.cur.w < N) C.advance(S, V);
        uint32_t w4[CP + 1][5];
        {
            const uint32_t o = (uint32_t)((int32_t)q - C.delta);
            const uint32_t* p = R.ring + ((o >> 2) & (kRingW - 1));
            const uint32_t sh = o & 3;
            uint32_t x[5 * CP + 4];
#pragma unroll
            for (int i = 0; i < 5 * CP + 4; i++) x[i] = p[i];
#pragma unroll
            for (int j = 0; j < CP; j++)
#pragma unroll
                for (int i = 0; i < 5; i++) w4[j][i] = __builtin_amdgcn_alignbyte(x[5 * j + i + 1], x[5 * j + i], sh);
#pragma unroll
            for (int i = 0; i < 3; i++) w4[CP][i] = __builtin_amdgcn_alignbyte(x[5 * CP + i + 1], x[5 * CP + i], sh);
            w4[CP][3] = w4[CP][4] = 0;
        }
        if (__builtin_expect(q + 20 * ngx > C.pos, 0)) {
            const uint32_t j0 = C.pos > q ? (C.pos - q) / 20 : 0;
            for (uint32_t j = j0; j < ngx; j++) {
                uint32_t w[5];
                cursor_chunk(S, V, C, R, q + 20 * j, w);
#pragma unroll
                for (int jj = 0; jj <= CP; jj++)
                    if ((uint32_t)jj == j)
#pragma unroll
                        for (int i = 0; i < 5; i++) w4[jj][i] = w[i];
            }
        }
        if (c0 == 0) {  // chunk 0's first words pre-add the chain state
            s_w0[0][vi] = w4[0][0];
            s_w0[1][vi] = w4[0][1];
            s_w0[2][vi] = w4[0][2];
        }
        const int b = e & 1;
#pragma unroll
        for (int j = 0; j < CP; j++) {
            if ((uint32_t)j < ng) {
                const bool nx = (uint32_t)j + 1 < ngx;
                const uint32_t a1 = nx ? w4[j + 1][0] : 0u, b1 = nx ? w4[j + 1][1] : 0u, c1 = nx ? w4[j + 1][2] : 0u;
                const uint32_t a = w4[j][0], bb = w4[j][1], cc = w4[j][2], d = w4[j][3], ee = w4[j][4];
                const int slot = CP * (NPART * pw + hf) + j;
                stage[b][slot][0][vi] = uint2{premix(d), kK + ee + a1};
                stage[b][slot][1][vi] = uint2{premix(cc), 3u * kK + 2u * a + d + b1};
                stage[b][slot][2][vi] = uint2{premix(bb + ee * fh::kC1), 2u * kK + a + d + c1};
            }
        }
    };
    __syncthreads();  // the ring holds epochs 0 and 1
    if (wv >= 2 && act) produce(0);
    __syncthreads();
    const uint32_t role = wv == 0 ? 1u + ((uint32_t)lane & 1u) : 0u;
    const uint32_t sh = (wv == 0 && (lane & 1) == 0) ? 1u : 0u, sh2 = sh + 2u;
    uint32_t cv = 0;
    if ((wv == 0 || wv == 1) && act && iters) cv = s_st[role][vi] + s_w0[role][vi];
    auto step_pair = [&](const uint2 x) {
        const uint32_t y = cv ^ x.x;
        const uint32_t r = __builtin_amdgcn_alignbit(y, y, 19);
        const uint32_t r5 = lshl_add<2>(r, r);
        const uint32_t own = lshl_add_v(r, sh2, lshl_add_v(r, sh, x.y));
        cv = swap_pair(r5) + own;
    };
    auto step_h = [&](const uint2 x) {
        const uint32_t y = cv ^ x.x;
        const uint32_t r = __builtin_amdgcn_alignbit(y, y, 19);
        cv = lshl_add<2>(r, r + x.y);
    };
    for (uint32_t e = 0; e < nep; e++) {
        const int b = e & 1;
        const uint32_t c0 = e * kEp;
        if (wv <= 1) {
            if (act) {
                if (__ballot(c0 + kEp > iters) == 0) {  // every lane takes the whole epoch
#pragma unroll
                    for (int j = 0; j < kEp; j += 8) {
                        uint2 x[8];
#pragma unroll
                        for (int q = 0; q < 8; q++) x[q] = stage[b][j + q][role][vi];
                        if (wv == 0) {
#pragma unroll
                            for (int q = 0; q < 8; q++) step_pair(x[q]);
                        } else {
#pragma unroll
                            for (int q = 0; q < 8; q++) step_h(x[q]);
                        }
                    }
                } else {
                    for (int j = 0; j < kEp; j++) {
                        if (c0 + j < iters) {  // (a pair's lanes share the view: both or neither)
                            if (wv == 0) step_pair(stage[b][j][role][vi]);
                            else step_h(stage[b][j][role][vi]);
                        }
                    }
                }
            }
        } else {
            if (act && e + 1 < nep) produce(e + 1);
            // the ring one epoch further ahead (the producers of the next iteration read it
            // after the barrier; nobody reads the slices being replaced any more)
            if (wv == 2) R.ensure(S.sbase, (e + 2) * kEp * 20 + lead, lane);
        }
        __syncthreads();
    }
    if (wv <= 1 && act) s_st[role][vi] = cv;
    __syncthreads();
    if (wv == 1 && act) {  // the last chunk's next-words were 0: plain h, g, f
        S.checksum[lv] = iters == 0 ? hdone : chain_final(s_st[0][lane], s_st[1][lane], s_st[2][lane]);
        S.dirty[lv] = 0;
    }
}

// ---- membership / dissemination / suspicion on one node

// A view's twin fingerprint: the sum over its deviated members (rank k; rows not at the base
// values) of a 64-bit mix of (rank, status, incarnation). Order-free, so block_apply keeps it
// per view as rows change (vfp) and the twin pass reads it instead of scanning the bitmap.
__device__ __forceinline__ uint64_t twin_mix(uint32_t k, uint8_t st, int64_t inc) {
    uint64_t x = ((uint64_t)k << 2 | st) * 0x9E3779B97F4A7C15ull ^ (uint64_t)inc * 0xC2B2AE3D27D4EB4Full;
    x ^= x >> 29;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 32;
    return x;
}

// the mix of a member's row, 0 at the base values (alive, the initial incarnation)
__device__ __forceinline__ uint64_t twin_term(uint32_t k, uint8_t st, int64_t inc, int64_t inc0) {
    return (st != ST_ALIVE || inc != inc0) ? twin_mix(k, st, inc) : 0ull;
}

// The node's change list as an LDS hash table (addr -> status, incarnation) for block_apply's
// no-op test: a list entry always holds its member's row values (block_apply writes both in the
// same step; an issue only deletes entries), so a record about a listed member is evaluated
// without reading the view's row, which is a random HBM access per record. Overlays Lds::win.
constexpr uint32_t kApHash = 2048;          // slots (a power of 2)
constexpr uint32_t kApHashMax = 1536;       // list entries it takes (load <= 0.75)
constexpr uint32_t kApHashMin = 64;         // records that pay for building it
constexpr uint32_t kApEmpty = 0xFFFFFFFFu;  // key: addr | status << 30
struct ApHash {
    uint32_t key[kApHash];
    int64_t inc[kApHash];
};
static_assert(sizeof(ApHash) <= sizeof(Lds::win), "the change-list hash overlays the checksum window");
__device__ __forceinline__ uint32_t ap_slot(uint32_t a) { return (a * 0x9E3779B1u) >> (32 - 11); }
static_assert(kApHash == 1u << 11, "ap_slot shift");

// Membership.update(records) on local node lv + the 'updated' listeners
// (on_membership_event.js:86-134): view row, recordChange (dissemination.js:56-72), suspicion
// start (a suspect update about another member), ring add/remove -> maxPiggybackCount. Records
// carry distinct addresses (one message), so lanes apply them independently. Returns the number
// applied (block-uniform). A record about a member on the node's change list is tested against
// the list entry first (ApHash); only the records that apply, or whose member is not listed,
// read the view's row.
__device__ uint32_t block_apply(const SimDev& S, uint32_t lv, const Rec* recs, uint32_t n, Lds& L, int64_t now) {
    const uint32_t v = S.v0 + lv;
    const uint64_t row = (uint64_t)lv * S.N;
    uint32_t napp = 0, nadd = 0, nrem = 0, nleave = 0;
    Change* chg = S.chg + (uint64_t)lv * S.Cd;
    Timer* tim = S.tim + (uint64_t)lv * S.Ct;
    __syncthreads();
    uint32_t nc = S.n_chg[lv], nt = S.n_tim[lv];
    const bool stopped = S.stopped[lv] != 0;
    ApHash& HT = *reinterpret_cast<ApHash*>(&L.win[0][0][0]);
    if (threadIdx.x == 0) L.fpd = L.dtd = 0;  // (visible after the loop's first block_scan)
    const bool hashed = n >= kApHashMin && nc > 0 && nc <= kApHashMax && S.N < (1u << 30);
    if (hashed) {  // block-uniform
        for (uint32_t q = threadIdx.x; q < kApHash; q += kT) HT.key[q] = kApEmpty;
        __syncthreads();
        for (uint32_t j = threadIdx.x; j < nc; j += kT) {
            const uint32_t a = chg[j].addr;
            const uint32_t k = a | (chg[j].st << 30);
            uint32_t q = ap_slot(a);
            while (atomicCAS(&HT.key[q], kApEmpty, k) != kApEmpty) q = (q + 1) & (kApHash - 1);
            HT.inc[q] = chg[j].inc;
        }
        __syncthreads();
    }
    for (uint32_t base = 0; base < n; base += kT) {
        const uint32_t i = base + threadIdx.x;
        bool applied = false, need_timer = false, need_new = false;
        uint32_t a = 0, slot = 0;
        uint64_t fpd = 0;
        int64_t dtd = 0;
        uint8_t us = 0;
        int64_t ui = 0;
        Rec r{};
        if (i < n) {
            r = recs[i];
            a = rec_addr(r);
            us = rec_st(r);
            ui = r.inc;
            bool noop = false;
            if (hashed) {
                uint32_t q = ap_slot(a), k;
                while ((k = HT.key[q]) != kApEmpty && (k & 0x3FFFFFFFu) != a) q = (q + 1) & (kApHash - 1);
                if (k != kApEmpty) {
                    uint8_t s2 = us;
                    int64_t i2 = ui;
                    noop = !evaluate_update((uint8_t)(k >> 30), HT.inc[q], a == v, s2, i2, now);
                }
            }
            const uint8_t cur = noop ? (uint8_t)0 : S.st[row + a];
            const int64_t oi = noop ? 0 : S.inc[row + a];
            if (!noop && evaluate_update(cur & ST_MASK, oi, a == v, us, ui, now)) {
                applied = true;
                napp++;
                // createUpdatedHandlerForRing: alive -> add, faulty/leave -> remove
                uint8_t ir = cur & IN_RING;
                if (us == ST_ALIVE && !ir) {
                    ir = IN_RING;
                    nadd++;
                } else if ((us == ST_FAULTY || us == ST_LEAVE) && ir) {
                    ir = 0;
                    nrem++;
                }
                S.st[row + a] = us | ir;
                S.inc[row + a] = ui;
                const uint32_t k = S.rank[a];
                atomicOr(&S.dev[(uint64_t)lv * S.W + (k >> 5)], 1u << (k & 31));
                fpd = twin_term(k, us, ui, S.inc0[a]) - twin_term(k, cur & ST_MASK, oi, S.inc0[a]);
                {
                    const int64_t i0 = S.inc0[a];
                    dtd = (int64_t)status_len(us) - (int64_t)status_len(cur & ST_MASK);
                    if (ui != i0) dtd += (int64_t)dec_len(ui) - (int64_t)dec_len(i0);
                    if (oi != i0) dtd -= (int64_t)dec_len(oi) - (int64_t)dec_len(i0);
                }
                need_timer = us == ST_SUSPECT && a != v && !stopped;
                // the local member becoming `leave` (LocalMemberLeaveEvent, member.js:87-95)
                if (a == v && us == ST_LEAVE && (cur & ST_MASK) != ST_LEAVE) nleave++;
                slot = S.slot[row + a];
                need_new = slot == 0;
            }
        }
        uint32_t ttot, ctot;
        const uint32_t tpos = block_scan(need_timer ? 1u : 0u, L.u, &ttot);
        const uint32_t cpos = block_scan(need_new ? 1u : 0u, L.u, &ctot);
        if (need_timer) {
            const uint32_t idx = nt + tpos;
            if (idx < S.Ct) tim[idx] = Timer{a, (int32_t)(S.round + S.susp), ui};
            else set_err(S, ERR_TIMERS);
        }
        if (applied) {
            if (fpd) atomicAdd(&L.fpd, (unsigned long long)fpd);
            if (dtd) atomicAdd(&L.dtd, (unsigned long long)dtd);
            if (!need_new) {
                Change& c = chg[slot - 1];
                c.cnt = 0;
                c.src = r.src;
                c.st = us;
                c.srcinc = r.srcinc;
                c.inc = ui;
            } else {
                const uint32_t idx = nc + cpos;
                if (idx < S.Cd) {
                    chg[idx] = Change{a, 0u, r.src, us, r.srcinc, ui};
                    S.slot[row + a] = idx + 1;
                } else {
                    set_err(S, ERR_CHANGES);
                }
            }
        }
        nt = min(nt + ttot, S.Ct);
        nc = min(nc + ctot, S.Cd);
    }
    const uint32_t tot = block_sum(napp, L.u);
    const uint32_t adds = block_sum(nadd, L.u);
    const uint32_t rems = block_sum(nrem, L.u);
    const uint32_t leaves = block_sum(nleave, L.u);
    if (threadIdx.x == 0) {
        S.n_chg[lv] = nc;
        // gossip.stop() + suspicion.stopAll() (on_membership_event.js:32-40): every timer is
        // cleared, the ones this batch started included (they start after the event)
        S.n_tim[lv] = leaves ? 0u : nt;
        if (leaves) S.t_head[lv] = 0;
        if (leaves) S.stopped[lv] = 1;
        if (tot) {
            S.vfp[lv] += L.fpd;
            S.vdt[lv] += (int64_t)L.dtd;
            S.dirty[lv] = 1;
            atomicAdd(&S.stats[3], (unsigned long long)tot);
            if (adds || rems) {  // ringChanged -> adjustMaxPiggybackCount (dissemination.js:38-55)
                const uint32_t rc = S.ring_count[lv] + adds - rems;
                S.ring_count[lv] = rc;
                S.max_piggy[lv] = 15u * digits(rc);
            }
        }
    }
    __syncthreads();
    return tot;
}

// Dissemination._issueAs (dissemination.js:133-176) for local node lv into out (nullable:
// discard). Filter: sender != NONE. Entries over maxPiggybackCount are deleted; the list is
// compacted in place (order kept). Returns the count emitted (block-uniform).
__device__ uint32_t block_issue(const SimDev& S, uint32_t lv, uint32_t sender, int64_t sinc, Rec* out, Lds& L) {
    const uint64_t row = (uint64_t)lv * S.N;
    Change* chg = S.chg + (uint64_t)lv * S.Cd;
    uint32_t emitted = 0, kept = 0;
    __syncthreads();
    const uint32_t maxp = S.max_piggy[lv];
    const uint32_t nc = S.n_chg[lv];
    for (uint32_t base = 0; base < nc; base += kT) {
        const uint32_t j = base + threadIdx.x;
        bool keep = false, emit = false;
        Change c{};
        if (j < nc) {
            c = chg[j];
            const bool filtered = sender != NONE && sinc != 0 && c.src != NONE && c.srcinc != 0 && c.src == sender &&
                                  c.srcinc == sinc;
            keep = true;
            if (!filtered) {
                if (c.cnt + 1u > maxp) {
                    keep = false;
                } else {
                    c.cnt++;
                    emit = true;
                }
            }
        }
        uint32_t ktot, etot;
        const uint32_t kpos = block_scan(keep ? 1u : 0u, L.u, &ktot);  // (syncs: reads above are done)
        const uint32_t epos = block_scan(emit ? 1u : 0u, L.u, &etot);
        if (j < nc) {
            if (keep) {
                chg[kept + kpos] = c;
                if (kept + kpos != j) S.slot[row + c.addr] = kept + kpos + 1;  // moved up
            } else {
                S.slot[row + c.addr] = 0;
            }
            if (emit && out) out[emitted + epos] = Rec{rec_w0(c.addr, (uint8_t)c.st, 0), c.src, c.inc, c.srcinc};
        }
        kept += ktot;
        emitted += etot;
        __syncthreads();
    }
    if (threadIdx.x == 0) S.n_chg[lv] = kept;
    __syncthreads();
    return emitted;
}

// issueAsReceiver (dissemination.js:86-119) of local node lv answering `sender`: the filtered
// issue, else a full sync when the checksums differ. The answer is written to the round arena;
// *off_out = its pool offset. Returns the record count, or NONE on arena overflow (the sender
// then sees a network error; rp_sim_step reports the overflow).
__device__ uint32_t block_issue_receiver(const SimDev& S, uint32_t lv, uint32_t sender, int64_t sinc, uint32_t sck,
                                         uint64_t* off_out, Lds& L) {
    const uint64_t ro = block_alloc(S, S.n_chg[lv], &L.u64);
    if (ro == ~0ull) return NONE;
    const uint32_t n = block_issue(S, lv, sender, sinc, S.pool + ro, L);
    *off_out = ro;
    if (n > 0) return n;
    checksum_if_dirty(S, lv, L);
    if (S.checksum[lv] == sck) return 0;
    const uint64_t fo = block_alloc(S, S.N, &L.u64);
    if (fo == ~0ull) return NONE;
    const uint64_t row = (uint64_t)lv * S.N;
    const uint32_t v = S.v0 + lv;
    Rec* out = S.pool + fo;
    for (uint32_t k = threadIdx.x; k < S.N; k += kT) {  // fullSync: members-array order, source = v
        const uint32_t a = S.order[row + k];
        out[k] = Rec{rec_w0(a, S.st[row + a] & ST_MASK, 0), v, S.inc[row + a], 0};
    }
    if (threadIdx.x == 0) atomicAdd(&S.stats[2], 1ull);
    *off_out = fo;
    __syncthreads();
    return S.N;
}

// makeSuspect / makeFaulty (index.js:179-202): one update from the local member
__device__ void block_make(const SimDev& S, uint32_t lv, uint32_t a, uint8_t st, int64_t inc, Lds& L, int64_t now,
                           Rec* tmp) {
    if (threadIdx.x == 0) *tmp = Rec{rec_w0(a, st, 0), S.v0 + lv, inc, S.inc[(uint64_t)lv * S.N + S.v0 + lv]};
    __syncthreads();
    block_apply(S, lv, tmp, 1, L, now);
}

// inv: also rewrite the row's inverse (k_opos_build does it for the start-up shuffle)
__device__ void lane0_shuffle(const SimDev& S, uint32_t lv, bool inv) {
    const uint64_t row = (uint64_t)lv * S.N;
    const uint32_t v = S.v0 + lv;
    const uint32_t sh = S.n_shuf[lv]++;
    for (uint32_t i = S.N - 1; i >= 1; i--) {
        const uint32_t r = philox_u32(S.seed, TAG_SHUF, sh, i, v);
        const uint32_t j = (uint32_t)(((uint64_t)r * (i + 1)) >> 32);
        const uint32_t t = S.order[row + i];
        S.order[row + i] = S.order[row + j];
        S.order[row + j] = t;
    }
    if (inv && S.opos)
        for (uint32_t k = 0; k < S.N; k++) S.opos[row + S.order[row + k]] = k;
}

__device__ __forceinline__ bool pingable(const SimDev& S, uint64_t row, uint32_t v, uint32_t m) {
    const uint8_t s = S.st[row + m] & ST_MASK;
    return m != v && (s == ST_ALIVE || s == ST_SUSPECT);  // isPingable (index.js:173-177)
}

// MembershipIterator.next (iterator.js:28-51) by one lane: walk the members array (reshuffling
// on wrap) until a pingable member, or until every distinct address has been visited. Before
// the first wrap of a walk positions are distinct; after it a bitmap tracks distinct visits.
__device__ int32_t lane0_iter_next(const SimDev& S, uint32_t lv, uint32_t* list, uint32_t* bits) {
    const uint32_t N = S.N;
    const uint64_t row = (uint64_t)lv * N;
    const uint32_t v = S.v0 + lv;
    uint32_t nseen = 0, steps = 0;
    bool wrapped = false;
    while (nseen < N) {
        int64_t idx = S.it_idx[lv] + 1;
        if (idx >= (int64_t)N) {
            idx = 0;
            if (!wrapped) {
                for (uint32_t w = 0; w < (N + 31) / 32; w++) bits[w] = 0;
                for (uint32_t q = 0; q < steps; q++) bits[list[q] >> 5] |= 1u << (list[q] & 31);
                wrapped = true;
            }
            lane0_shuffle(S, lv, true);
        }
        S.it_idx[lv] = idx;
        const uint32_t m = S.order[row + idx];
        if (!wrapped) {
            list[steps] = m;
            nseen++;
        } else if (!(bits[m >> 5] & (1u << (m & 31)))) {
            bits[m >> 5] |= 1u << (m & 31);
            nseen++;
        }
        steps++;
        if (pingable(S, row, v, m)) return (int32_t)m;
    }
    return -1;
}

// ---- phases (each over this shard's nodes)

__global__ void k_round_begin(SimDev S) {
    if (blockIdx.x == 0 && threadIdx.x == 0) *S.cursor = 0;
    if (blockIdx.x == 0 && threadIdx.x < 8) S.work[threadIdx.x] = 0;
}

// Phases A, B and D2 take their local nodes from a counter, kNodeChunk at a time, instead of a
// fixed stride: a node whose answer needs a checksum chain (block_checksum) holds its
// workgroup for milliseconds, and a fixed assignment left the workgroups that drew several of
// them running long after the rest (C5, early rounds: phase B 41-49 -> 14-18 ms). One atomic
// per node cost ~1 ms per phase on one counter, hence the chunks; the cheap phases keep the
// stride. Every node's work in a phase is independent of the others', so the order does not
// matter (only where the arena places a response, never its content).
constexpr uint32_t kNodeChunk = 4;
struct NodeIter {
    uint32_t cur = 0, end = 0;
};
__device__ __forceinline__ uint32_t next_node(const SimDev& S, int ph, uint32_t* slot, NodeIter& it) {
    if (it.cur == it.end) {
        __syncthreads();  // every thread has read the previous chunk's base
        if (threadIdx.x == 0) *slot = atomicAdd(&S.work[ph], kNodeChunk);
        __syncthreads();
        it.cur = *slot;
        it.end = it.cur + kNodeChunk;
    }
    return it.cur++;
}

// views the batch refresh is about to hash (stats[4])
__global__ void k_count_dirty(SimDev S) {
    uint32_t c = 0;
    for (uint32_t lv = blockIdx.x * blockDim.x + threadIdx.x; lv < S.NL; lv += gridDim.x * blockDim.x)
        c += (!S.dead[S.v0 + lv] && S.dirty[lv]) ? 1u : 0u;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(&S.stats[4], (unsigned long long)c);
}

// ---- twin views: dirty views whose checksum strings are equal hash once (refresh_checksums)
//
// A view's string is fixed by its members' (status, incarnation); a member whose bitmap bit is
// clear holds the base values. The fingerprint is a sum over the view's deviated members of a
// 64-bit mix of (rank, status, incarnation): order-free, so a wave sums it lane-parallel over
// the bitmap. Views land in an open-addressing table by fingerprint; the lowest view id of each
// fingerprint is the representative. Every other view verifies its content against the
// representative's member by member over the union of both bitmaps (exact: a fingerprint
// collision only costs the verification), and an equal view is marked clean and takes the
// representative's checksum after the chains.

constexpr unsigned long long kTwinEmpty = ~0ull;

__device__ __forceinline__ uint32_t twin_slot(uint64_t f, uint32_t tmask) { return (uint32_t)(f ^ (f >> 32)) & tmask; }

// a view's fingerprint from its rows (one wave; the result in every lane)
__device__ uint64_t view_fp_scan(const SimDev& S, uint32_t lv, int lane) {
    const uint64_t row = (uint64_t)lv * S.N;
    const uint32_t* dv = S.dev + (uint64_t)lv * S.W;
    uint64_t sum = 0;
    for (uint32_t w = lane; w < S.W; w += 64) {
        uint32_t bits = dv[w];
        while (bits) {
            const uint32_t k = (w << 5) + __builtin_ctz(bits);
            bits &= bits - 1;
            const uint32_t a = S.sorted[k];
            sum += twin_term(k, S.st[row + a] & ST_MASK, S.inc[row + a], S.inc0[a]);
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
    return sum;
}

// the kept fingerprint of a view whose rows were rewritten wholesale (a join)
__global__ void k_vfp_view(SimDev S, uint32_t lv) {
    const uint64_t f = view_fp_scan(S, lv, threadIdx.x & 63);
    if (threadIdx.x == 0) S.vfp[lv] = f;
}

// Every dirty live view into the fingerprint table (one lane per view; verify: one wave per
// view also recomputes it from the rows and flags a difference).
__global__ void k_twin_fp(SimDev S, uint64_t* __restrict__ fp, unsigned long long* __restrict__ tkey,
                          uint32_t* __restrict__ trep, uint32_t tmask, int verify) {
    const int lane = threadIdx.x & 63;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < (verify ? S.NL * 64u : S.NL);
         i += gridDim.x * blockDim.x) {
        const uint32_t lv = verify ? i >> 6 : i;
        if (!S.dirty[lv] || S.dead[S.v0 + lv]) continue;  // (wave-uniform when verifying)
        const uint64_t sum = S.vfp[lv];
        if (verify && view_fp_scan(S, lv, lane) != sum && lane == 0) set_err(S, ERR_TWINFP);
        if (!verify || lane == 0) {
            const uint64_t f = sum == kTwinEmpty ? 0x5bd1e995ull : sum;
            fp[lv] = f;
            for (uint32_t h = twin_slot(f, tmask);; h = (h + 1) & tmask) {
                const unsigned long long prev = atomicCAS(&tkey[h], kTwinEmpty, (unsigned long long)f);
                if (prev == kTwinEmpty || prev == f) {
                    atomicMin(&trep[h], lv);
                    break;
                }
            }
        }
    }
}

__global__ void k_twin_check(SimDev S, const uint64_t* __restrict__ fp, const unsigned long long* __restrict__ tkey,
                             const uint32_t* __restrict__ trep, uint32_t tmask, uint32_t* __restrict__ twin_of,
                             uint32_t* __restrict__ ntwins) {
    const int lane = threadIdx.x & 63;
    const uint32_t nw = (gridDim.x * blockDim.x) >> 6;
    for (uint32_t lv = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; lv < S.NL; lv += nw) {
        if (!S.dirty[lv] || S.dead[S.v0 + lv]) continue;  // wave-uniform
        const uint64_t f = fp[lv];
        uint32_t h = twin_slot(f, tmask);
        while (tkey[h] != f) h = (h + 1) & tmask;
        const uint32_t rep = trep[h];
        if (rep == lv) continue;
        const uint64_t ra = (uint64_t)lv * S.N, rb = (uint64_t)rep * S.N;
        const uint32_t* da = S.dev + (uint64_t)lv * S.W;
        const uint32_t* db = S.dev + (uint64_t)rep * S.W;
        bool same = true;
        for (uint32_t w = lane; w < S.W && same; w += 64) {
            uint32_t bits = da[w] | db[w];
            while (bits && same) {
                const uint32_t k = (w << 5) + __builtin_ctz(bits);
                bits &= bits - 1;
                const uint32_t a = S.sorted[k];
                same = (S.st[ra + a] & ST_MASK) == (S.st[rb + a] & ST_MASK) && S.inc[ra + a] == S.inc[rb + a];
            }
        }
        if (__all(same) && lane == 0) {
            twin_of[lv] = rep;
            S.dirty[lv] = 0;
            atomicAdd(ntwins, 1u);
            atomicAdd(&S.stats[4], ~0ull);  // not hashed after all (views-hashed counter)
        }
    }
}

// the live dirty views, compacted (one atomic per wave; order immaterial: one chain per view)
__global__ void k_dirty_list(SimDev S, uint32_t* __restrict__ list, uint32_t* __restrict__ n) {
    const int lane = threadIdx.x & 63;
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t i0 = blockIdx.x * blockDim.x; i0 < S.NL; i0 += stride) {
        const uint32_t lv = i0 + threadIdx.x;
        const bool on = lv < S.NL && S.dirty[lv] && !S.dead[S.v0 + lv];
        const uint64_t m = __ballot(on);
        if (!m) continue;
        uint32_t base = 0;
        if (lane == __ffsll((long long)m) - 1) base = atomicAdd(n, (uint32_t)__popcll(m));
        base = __shfl(base, __ffsll((long long)m) - 1, 64);
        if (on) list[base + __popcll(m & ((1ull << lane) - 1))] = lv;
    }
}

// The early refresh's views (stage 2, beside the D1 sender chains): the live dirty views except
// the round's ping-req senders (k_d1_list's predicate: their chains run in k_ck_pc over the D1
// list, and phase D1 reads and may change those views meanwhile). The count goes to the
// views-hashed counter (stats[4]) as k_count_dirty's would.
__global__ void k_early_list(SimDev S, uint32_t* __restrict__ list, uint32_t* __restrict__ n) {
    const int lane = threadIdx.x & 63;
    const uint32_t stride = gridDim.x * blockDim.x;
    uint32_t cnt = 0;
    for (uint32_t i0 = blockIdx.x * blockDim.x; i0 < S.NL; i0 += stride) {
        const uint32_t lv = i0 + threadIdx.x;
        bool on = lv < S.NL && S.dirty[lv] && !S.dead[S.v0 + lv];
        if (on) {
            const int32_t t = S.target[lv];
            on = !(t >= 0 && S.dead[t]);
            // a view whose earliest suspicion timer is due fires it in phase E and changes again
            // (timers are appended with due = round + susp, so the head timer is the earliest)
            const uint32_t th = S.t_head[lv];
            if (on && S.n_tim[lv] > th && S.tim[(uint64_t)lv * S.Ct + th].due <= S.round) on = false;
        }
        const uint64_t m = __ballot(on);
        if (!m) continue;
        uint32_t base = 0;
        if (lane == __ffsll((long long)m) - 1) base = atomicAdd(n, (uint32_t)__popcll(m));
        base = __shfl(base, __ffsll((long long)m) - 1, 64);
        if (on) list[base + __popcll(m & ((1ull << lane) - 1))] = lv;
        cnt += lane == 0 ? (uint32_t)__popcll(m) : 0u;
    }
    if (lane == 0 && cnt) atomicAdd(&S.stats[4], (unsigned long long)cnt);
}

__global__ void k_twin_copy(SimDev S, uint32_t* __restrict__ twin_of) {
    for (uint32_t lv = blockIdx.x * blockDim.x + threadIdx.x; lv < S.NL; lv += gridDim.x * blockDim.x) {
        const uint32_t r = twin_of[lv];
        if (r != NONE) {
            S.checksum[lv] = S.checksum[r];
            twin_of[lv] = NONE;
        }
    }
}

// A: iterator.next() + issueAsSender() for every live node (checksums are fresh: k_ck_lanes ran)
__global__ __launch_bounds__(kT) void k_phase_a(SimDev S) {
    __shared__ Lds L;
    __shared__ int32_t tgt;
    __shared__ uint32_t s_w;
    NodeIter it;
    for (uint32_t lv = next_node(S, 0, &s_w, it); lv < S.NL; lv = next_node(S, 0, &s_w, it)) {
        const uint32_t v = S.v0 + lv;
        if (S.dead[v] || S.stopped[lv]) {  // down, or its gossip loop stopped by a leave
            if (threadIdx.x == 0) S.target[lv] = -1;
            continue;
        }
        const uint64_t row = (uint64_t)lv * S.N;
        if (threadIdx.x == 0) {
            uint8_t* scratch = S.strbuf + (uint64_t)blockIdx.x * S.strcap;
            const int32_t found = lane0_iter_next(S, lv, reinterpret_cast<uint32_t*>(scratch),
                                                  reinterpret_cast<uint32_t*>(scratch + 4ull * S.N));
            tgt = found;
            S.target[lv] = found;
        }
        __syncthreads();
        if (tgt >= 0) {
            checksum_if_dirty(S, lv, L);
            const uint32_t n = block_issue(S, lv, NONE, 0, ping_slot(S, lv), L);
            if (threadIdx.x == 0) {
                S.ping_n[lv] = n;
                S.ck_snap[lv] = S.checksum[lv];
                S.inc_snap[lv] = S.inc[row + v];
                atomicAdd(&S.stats[0], 1ull);
            }
        }
        __syncthreads();
    }
}

// B: each live local target applies its pings in sender order and answers each one
__global__ __launch_bounds__(kT, 4) void k_phase_b(SimDev S) {
    __shared__ Lds L;
    const int64_t now = S.now0 + 200 * S.round;
    __shared__ uint32_t s_w;
    NodeIter it;
    for (uint32_t lj = next_node(S, 1, &s_w, it); lj < S.NL; lj = next_node(S, 1, &s_w, it)) {
        const uint32_t b = S.ib_off[lj], e = S.ib_off[lj + 1];
        for (uint32_t q = b; q < e; q++) {
            const uint32_t i = S.ib_idx[q];
            const Msg m = S.in_msg[i];
            block_apply(S, lj, msg_recs(S, m), m.n, L, now);
            uint64_t o = 0;
            const uint32_t n = block_issue_receiver(S, lj, m.from, m.inc, m.ck, &o, L);
            if (threadIdx.x == 0) {
                S.rsp_n[i] = n;
                S.rsp_off[i] = o;
            }
            __syncthreads();
        }
    }
}

// C: each sender with a live target applies the response (ping-sender.js:38). The reference
// applies it a second time (gossip/index.js:165); that pass changes no state, so it is not run.
// The records have distinct addresses, evaluate_update of a record depends only on its own
// address's row, and every rule applies only a strictly newer incarnation or a strictly higher
// status at the same incarnation, so after the first pass a record meets a row that it does
// not override. The one exception is a suspect/faulty record about the local member: the local
// override (member.js:76-81) applies it again, as alive at the same Date.now(), which rewrites
// the same row and change values and only counts one more applied update; that count is added
// here. The oracle keeps both passes, so the parity tests check this.
__global__ __launch_bounds__(kT) void k_phase_c(SimDev S) {
    __shared__ Lds L;
    const int64_t now = S.now0 + 200 * S.round;
    for (uint32_t lv = blockIdx.x; lv < S.NL; lv += gridDim.x) {
        const uint32_t i = S.resp_idx[lv];
        if (i == NONE) continue;  // dead sender, no target, dead target
        const Msg m = S.in_msg[i];
        if (m.n == NONE) continue;  // the target's arena overflowed (reported)
        const Rec* r = msg_recs(S, m);
        block_apply(S, lv, r, m.n, L, now);
        const uint32_t v = S.v0 + lv;
        for (uint32_t k = threadIdx.x; k < m.n; k += kT) {
            const uint8_t us = rec_st(r[k]);
            if (rec_addr(r[k]) == v && (us == ST_SUSPECT || us == ST_FAULTY)) atomicAdd(&S.stats[3], 1ull);
        }
    }
}

// The live local senders whose target is dead (the ping-req senders of D1), in any order (their
// work is independent); every node's helper count is reset.
__global__ void k_d1_list(SimDev S, uint32_t* __restrict__ list, uint32_t* __restrict__ n) {
    for (uint32_t lv = blockIdx.x * blockDim.x + threadIdx.x; lv < S.NL; lv += gridDim.x * blockDim.x) {
        S.nhelp[lv] = 0;
        const int32_t t = S.target[lv];
        if (!S.dead[S.v0 + lv] && t >= 0 && S.dead[t]) list[atomicAdd(n, 1u)] = lv;
    }
}

constexpr uint32_t kXCap = 2048;  // non-candidates a D1 sender sorts in LDS (more: the scan path)

// The k-th (0-based) members-array position outside the sorted position set xs[0..n): with
// y_i = xs[i] - i (non-decreasing), it is k + #{i : y_i <= k}.
__device__ __forceinline__ uint32_t d1_select(const uint32_t* xs, uint32_t n, uint32_t k) {
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (xs[mid] - mid <= k)
            lo = mid + 1;
        else
            hi = mid;
    }
    return k + lo;
}

// D1: ping-req fan-out for senders whose target is dead (one workgroup per listed sender).
// getRandomPingableMembers(3, [target]) (index.js:141-150) is _.sample over the members array
// minus the non-candidates: self, the target, and members whose status is faulty / leave. Only
// members whose row ever changed can be faulty / leave, so the non-candidates come from the
// view's deviation bitmap (N/32 words), their positions from the inverse permutation; sorted in
// LDS they turn each index the partial Fisher-Yates draws into a position by a binary search.
// The draws, the swaps and so the helpers are the scan path's (kept for views with more than
// kXCap non-candidates, or when the inverse is not allocated).
__global__ __launch_bounds__(kT) void k_phase_d1(SimDev S, const uint32_t* __restrict__ list,
                                                 const uint32_t* __restrict__ nlist) {
    __shared__ Lds L;
    __shared__ Rec tmp;
    __shared__ uint32_t ncand, nx;
    __shared__ uint32_t xs[kXCap];
    const int64_t now = S.now0 + 200 * S.round;
    uint32_t* cand = S.cand + (uint64_t)blockIdx.x * S.N;
    const uint32_t nl = *nlist;
    for (uint32_t li = blockIdx.x; li < nl; li += gridDim.x) {
        const uint32_t lv = list[li];
        const uint32_t v = S.v0 + lv;
        const int32_t t = S.target[lv];
        const uint64_t row = (uint64_t)lv * S.N;
        if (threadIdx.x == 0) atomicAdd(&S.stats[1], 1ull);
        bool fast = S.opos != nullptr;
        if (fast) {
            if (threadIdx.x == 0) {
                xs[0] = S.opos[row + v];
                xs[1] = S.opos[row + (uint32_t)t];
                nx = 2;
            }
            __syncthreads();
            const uint32_t* dv = S.dev + (uint64_t)lv * S.W;
            for (uint32_t w = threadIdx.x; w < S.W; w += kT) {
                uint32_t bits = dv[w];
                while (bits) {
                    const uint32_t m = S.sorted[w * 32u + (uint32_t)__builtin_ctz(bits)];
                    bits &= bits - 1u;
                    if (m != v && m != (uint32_t)t && !pingable(S, row, v, m)) {
                        const uint32_t q = atomicAdd(&nx, 1u);
                        if (q < S.xcap) xs[q] = S.opos[row + m];
                    }
                }
            }
            __syncthreads();
            fast = nx <= S.xcap;
        }
        if (fast) {
            const uint32_t n = nx;
            uint32_t P = 1;
            while (P < n) P <<= 1;
            for (uint32_t i = n + threadIdx.x; i < P; i += kT) xs[i] = 0xFFFFFFFFu;
            __syncthreads();
            for (uint32_t size = 2; size <= P; size <<= 1) {  // bitonic sort, ascending
                for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
                    for (uint32_t i = threadIdx.x; i < P; i += kT) {
                        const uint32_t j = i ^ stride;
                        if (j > i) {
                            const uint32_t a = xs[i], b = xs[j];
                            if ((a > b) == ((i & size) == 0)) {
                                xs[i] = b;
                                xs[j] = a;
                            }
                        }
                    }
                    __syncthreads();
                }
            }
            if (threadIdx.x == 0) {
                const uint32_t len = S.N - n;
                const uint32_t nh = len < 3 ? len : 3;
                uint32_t key[6], val[6], nk = 0;  // the candidate slots the swaps have rewritten
                auto get = [&](uint32_t q) -> uint32_t {
                    for (uint32_t z = 0; z < nk; z++)
                        if (key[z] == q) return val[z];
                    return S.order[row + d1_select(xs, n, q)];
                };
                auto put = [&](uint32_t q, uint32_t x) {
                    for (uint32_t z = 0; z < nk; z++)
                        if (key[z] == q) {
                            val[z] = x;
                            return;
                        }
                    key[nk] = q;
                    val[nk] = x;
                    nk++;
                };
                for (uint32_t i = 0; i < nh; i++) {  // _.sample -> partial Fisher-Yates (SAMP stream)
                    const uint32_t r = philox_u32(S.seed, TAG_SAMP, (uint32_t)S.round, i, v);
                    const uint32_t j = i + (uint32_t)(((uint64_t)r * (len - i)) >> 32);
                    const uint32_t a = get(i), b = get(j);
                    put(i, b);
                    put(j, a);
                    S.helpers[lv * 3 + i] = b;
                }
                S.nhelp[lv] = nh;
                ncand = nh;
            }
        } else {
            // candidates: members-array order, pingable, not the target (index.js:141-150)
            uint32_t written = 0;
            for (uint32_t base = 0; base < S.N; base += kT) {
                const uint32_t k = base + threadIdx.x;
                bool ok = false;
                uint32_t m = 0;
                if (k < S.N) {
                    m = S.order[row + k];
                    ok = m != (uint32_t)t && pingable(S, row, v, m);
                }
                uint32_t tot;
                const uint32_t p = block_scan(ok ? 1u : 0u, L.u, &tot);
                if (ok) cand[written + p] = m;
                written += tot;
            }
            if (threadIdx.x == 0) ncand = written;
            __syncthreads();
            __threadfence_block();
            if (threadIdx.x == 0) {
                const uint32_t len = ncand;
                const uint32_t nh = len < 3 ? len : 3;
                for (uint32_t i = 0; i < nh; i++) {  // _.sample -> partial Fisher-Yates (SAMP stream)
                    const uint32_t r = philox_u32(S.seed, TAG_SAMP, (uint32_t)S.round, i, v);
                    const uint32_t j = i + (uint32_t)(((uint64_t)r * (len - i)) >> 32);
                    const uint32_t x = cand[i];
                    cand[i] = cand[j];
                    cand[j] = x;
                    S.helpers[lv * 3 + i] = cand[i];
                }
                S.nhelp[lv] = nh;
                ncand = nh;
            }
        }
        __syncthreads();
        if (ncand == 0) {
            block_make(S, lv, (uint32_t)t, ST_SUSPECT, S.inc[row + t], L, now, &tmp);
            if (threadIdx.x == 0) S.nhelp[lv] = 0;
            __syncthreads();
            continue;
        }
        checksum_if_dirty(S, lv, L);
        if (threadIdx.x == 0) {
            S.ck_snap[lv] = S.checksum[lv];
            S.inc_snap[lv] = S.inc[row + v];
        }
        // three issueAsSender() calls; records carry the count after the first one (aux); leg k
        // carries the records whose count after the first issue + k <= maxPiggybackCount
        const uint32_t maxp = S.max_piggy[lv];
        const uint32_t nc = S.n_chg[lv];
        Change* chg = S.chg + (uint64_t)lv * S.Cd;
        Rec* leg = leg_slot(S, lv);
        uint32_t written2 = 0, kept = 0, nk1 = 0, nk2 = 0;
        for (uint32_t base = 0; base < nc; base += kT) {
            const uint32_t j = base + threadIdx.x;
            bool emit = false, keep = false;
            Change c{};
            uint32_t c1 = 0;
            if (j < nc) {
                c = chg[j];
                c1 = c.cnt + 1;
                if (c1 <= maxp) {
                    emit = true;
                    if (c.cnt + 3 <= maxp) {
                        keep = true;
                        c.cnt += 3;
                    }
                }
            }
            nk1 += (emit && c1 + 1 <= maxp) ? 1u : 0u;
            nk2 += (emit && c1 + 2 <= maxp) ? 1u : 0u;
            uint32_t ktot, etot;
            const uint32_t kpos = block_scan(keep ? 1u : 0u, L.u, &ktot);
            const uint32_t p = block_scan(emit ? 1u : 0u, L.u, &etot);
            if (j < nc) {
                if (keep) {
                    chg[kept + kpos] = c;
                    if (kept + kpos != j) S.slot[row + c.addr] = kept + kpos + 1;  // moved up
                } else {
                    S.slot[row + c.addr] = 0;
                }
                if (emit) leg[written2 + p] = Rec{rec_w0(c.addr, (uint8_t)c.st, c1), c.src, c.inc, c.srcinc};
            }
            written2 += etot;
            kept += ktot;
            __syncthreads();
        }
        const uint32_t t1 = block_sum(nk1, L.u), t2 = block_sum(nk2, L.u);
        if (threadIdx.x == 0) {
            S.leg_n[lv] = written2;
            S.leg_nk[lv * 3 + 0] = written2;
            S.leg_nk[lv * 3 + 1] = t1;
            S.leg_nk[lv * 3 + 2] = t2;
            S.n_chg[lv] = kept;
        }
        __syncthreads();
    }
}

// D2: local helpers handle their ping-req legs in (sender, leg) order (ping-req.js:26-68). The
// legs to dead helpers were never sent (the sender sees a network error).
__global__ __launch_bounds__(kT, 4) void k_phase_d2(SimDev S) {
    __shared__ Lds L;
    const int64_t now = S.now0 + 200 * S.round;
    __shared__ uint32_t s_w;
    NodeIter it;
    for (uint32_t lh = next_node(S, 3, &s_w, it); lh < S.NL; lh = next_node(S, 3, &s_w, it)) {
        const uint32_t b = S.ib_off[lh], e = S.ib_off[lh + 1];
        for (uint32_t q = b; q < e; q++) {
            const uint32_t i = S.ib_idx[q];
            const Msg m = S.in_msg[i];
            block_apply(S, lh, msg_recs(S, m), m.n, L, now);
            block_issue(S, lh, NONE, 0, nullptr, L);  // the helper's own ping of the dead target
            uint64_t o = 0;
            const uint32_t n = block_issue_receiver(S, lh, m.from, m.inc, m.ck, &o, L);
            if (threadIdx.x == 0) {
                S.rsp_n[i] = n;
                S.rsp_off[i] = o;
            }
            __syncthreads();
        }
    }
}

// D3: senders apply answered legs, then the verdict (ping-req-sender.js:190-284)
__global__ __launch_bounds__(kT) void k_phase_d3(SimDev S) {
    __shared__ Lds L;
    __shared__ Rec tmp;
    const int64_t now = S.now0 + 200 * S.round;
    for (uint32_t lv = blockIdx.x; lv < S.NL; lv += gridDim.x) {
        const uint32_t nh = S.nhelp[lv];
        if (S.dead[S.v0 + lv] || nh == 0) continue;
        const uint64_t row = (uint64_t)lv * S.N;
        bool bad = false;
        for (uint32_t k = 0; k < nh; k++) {
            const uint32_t i = S.lresp_idx[lv * 3 + k];
            if (i == NONE) continue;  // dead helper: network error
            const Msg m = S.in_msg[i];
            if (m.n == NONE) continue;
            block_apply(S, lv, msg_recs(S, m), m.n, L, now);
            bad = true;
        }
        if (bad) {
            const uint32_t t = (uint32_t)S.target[lv];
            block_make(S, lv, t, ST_SUSPECT, S.inc[row + t], L, now, &tmp);
        }
    }
}

// E: suspicion timers due this round fire (makeFaulty with the captured incarnation). A timer
// is live while its member is still suspect at the captured incarnation (a newer suspicion
// started a newer timer; any other status stopped it); the rest are dropped. The firings touch
// distinct members, so they are applied together.
// Timers are appended with due = round + susp, so a node's list is in due order and the timers
// due this round are a prefix of its pending part [t_head, n_tim): only that prefix is read
// (a lapsed timer that is not due yet waits in the list; at its due round it is dropped, as the
// reference's cleared timeout never fires). A list past half its capacity is pruned whole and
// compacted instead, so the appends of later rounds keep their room.
__global__ __launch_bounds__(kT) void k_phase_e(SimDev S) {
    __shared__ Lds L;
    const int64_t now = S.now0 + 200 * S.round;
    for (uint32_t lv = blockIdx.x; lv < S.NL; lv += gridDim.x) {
        const uint32_t v = S.v0 + lv;
        if (S.dead[v] || S.stopped[lv]) continue;
        const uint32_t nt = S.n_tim[lv], h0 = S.t_head[lv];
        if (h0 >= nt) continue;  // nothing pending
        const uint64_t row = (uint64_t)lv * S.N;
        const int64_t srci = S.inc[row + v];
        Rec* stage = ping_slot(S, lv);  // free: the ping left in the exchange after phase A
        Timer* tim = S.tim + (uint64_t)lv * S.Ct;
        const bool whole = nt > S.Ct / 2;
        uint32_t written = 0, kept = 0, h = h0;
        for (uint32_t base = h0; base < nt; base += kT) {
            const uint32_t i = base + threadIdx.x;
            bool keep = false, fire = false, due = false;
            Timer t{};
            if (i < nt) {
                t = tim[i];
                due = t.due <= S.round;
                if (due || whole) {
                    const bool live = (S.st[row + t.addr] & ST_MASK) == ST_SUSPECT && S.inc[row + t.addr] == t.inc;
                    fire = live && due;
                    keep = live && !due;
                }
            }
            uint32_t ktot, ftot, dtot;
            const uint32_t kpos = block_scan(keep ? 1u : 0u, L.u, &ktot);
            const uint32_t fpos = block_scan(fire ? 1u : 0u, L.u, &ftot);
            block_scan(due ? 1u : 0u, L.u, &dtot);
            if (whole && keep) tim[kept + kpos] = t;
            if (fire && written + fpos < S.Cm) stage[written + fpos] = Rec{rec_w0(t.addr, ST_FAULTY, 0), v, t.inc, srci};
            kept += ktot;
            written += ftot;
            h += dtot;
            __syncthreads();
            if (!whole && dtot < kT) break;  // the due prefix ended in this chunk (block-uniform)
        }
        if (threadIdx.x == 0) {
            if (whole) {
                S.n_tim[lv] = kept;
                S.t_head[lv] = 0;
            } else if (h >= nt) {
                S.n_tim[lv] = 0;
                S.t_head[lv] = 0;
            } else {
                S.t_head[lv] = h;
            }
        }
        __threadfence_block();
        __syncthreads();
        if (written > S.Cm) {
            if (threadIdx.x == 0) set_err(S, ERR_TIMERS);
            written = S.Cm;
        }
        if (written) block_apply(S, lv, stage, written, L, now);
    }
}

// Scenario leaves (server/admin/member.js:92-93): makeLeave(whoami, own incarnation) on each
// listed local node whose own status is not `leave` yet (a redundant leave is refused, :84-89)
__global__ __launch_bounds__(kT) void k_leave(SimDev S, const uint32_t* __restrict__ list, uint32_t n) {
    __shared__ Lds L;
    __shared__ Rec tmp;
    const int64_t now = S.now0 + 200 * S.round;
    for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
        const uint32_t lv = list[i], v = S.v0 + lv;
        const uint64_t row = (uint64_t)lv * S.N;
        if ((S.st[row + v] & ST_MASK) == ST_LEAVE) continue;
        block_make(S, lv, v, ST_LEAVE, S.inc[row + v], L, now, &tmp);
    }
}

// ---- a fresh process joining from join responses (RP_SIM_JOIN)
//
// index.js:240-322 for node v: makeAlive(self, Date.now()); each responder (chosen on the host)
// answers the join with makeAlive(v, that incarnation) (server/protocol/join.js:126) and its
// fullSync; mergeJoinResponses (join-response-merge.js:40-56) + set() (index.js:208-247) give
// self first, then the first response's members-array order without self, each member at the
// greatest incarnation any response holds (the first on ties); the set handler
// (on_membership_event.js:42-67) puts alive / suspect members in the ring without a ringChanged
// and starts a timer per suspect member. The dissemination is cleared as at bootstrap.

// Where the joiner reads its responders' rows: the shard's own view rows when every responder
// is local (one shard), else a join exchange buffer (JoinBuf layout) that the shards filled with
// their responders' rows.
struct JoinSrc {
    const uint8_t* st[3];   // status (masked or not: read through ST_MASK)
    const int64_t* inc[3];
    const uint32_t* order0;  // the first responder's members array
};

// Join exchange buffer: [3][N] statuses, [3][N] incarnations (16-B aligned), [N] order of r0.
struct JoinBuf {
    uint64_t o_inc, o_ord, bytes;
    explicit JoinBuf(uint32_t N) {
        o_inc = (3ull * N + 15) & ~15ull;
        o_ord = o_inc + 24ull * N;
        bytes = o_ord + 4ull * N;
    }
    JoinSrc src(const uint8_t* b, uint32_t N) const {
        JoinSrc j{};
        for (int q = 0; q < 3; q++) {
            j.st[q] = b + (uint64_t)q * N;
            j.inc[q] = reinterpret_cast<const int64_t*>(b + o_inc) + (uint64_t)q * N;
        }
        j.order0 = reinterpret_cast<const uint32_t*>(b + o_ord);
        return j;
    }
};

// the responders' join handler, on the shard that owns each (bit q of `local`)
__global__ __launch_bounds__(kT) void k_join_resp(SimDev S, uint32_t v, int64_t incv, uint32_t r0, uint32_t r1,
                                                  uint32_t r2, uint32_t nj, uint32_t local) {
    __shared__ Lds L;
    __shared__ Rec tmp;
    const int64_t now = S.now0 + 200 * S.round;
    for (uint32_t q = blockIdx.x; q < nj; q += gridDim.x) {
        if (!((local >> q) & 1u)) continue;
        const uint32_t r = q == 0 ? r0 : q == 1 ? r1 : r2;
        block_make(S, r - S.v0, v, ST_ALIVE, incv, L, now, &tmp);
    }
}

// this shard's responders' rows into the (zeroed) join exchange buffer
__global__ void k_join_export(SimDev S, uint32_t r0, uint32_t r1, uint32_t r2, uint32_t nj, uint32_t local,
                              uint8_t* __restrict__ jst, int64_t* __restrict__ jinc, uint32_t* __restrict__ jord) {
    for (uint32_t m = blockIdx.x * blockDim.x + threadIdx.x; m < S.N; m += gridDim.x * blockDim.x)
        for (uint32_t q = 0; q < nj; q++) {
            if (!((local >> q) & 1u)) continue;
            const uint64_t row = (uint64_t)((q == 0 ? r0 : q == 1 ? r1 : r2) - S.v0) * S.N;
            jst[(uint64_t)q * S.N + m] = S.st[row + m] & ST_MASK;
            jinc[(uint64_t)q * S.N + m] = S.inc[row + m];
            if (q == 0) jord[m] = S.order[row + m];
        }
}

// v's position in the first response's members array; the joiner's deviation words cleared
__global__ void k_join_prep(SimDev S, uint32_t v, JoinSrc J, uint32_t* __restrict__ scratch) {
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < S.N; k += gridDim.x * blockDim.x)
        if (J.order0[k] == v) scratch[0] = k;
    for (uint32_t w = blockIdx.x * blockDim.x + threadIdx.x; w < S.W; w += gridDim.x * blockDim.x)
        S.dev[(uint64_t)(v - S.v0) * S.W + w] = 0;
}

// the joiner's rows, members array, timers; scratch[0] = v's position in r0's array,
// scratch[1] accumulates the members outside the ring
__global__ void k_join_view(SimDev S, uint32_t v, int64_t incv, uint32_t nj, JoinSrc J,
                            uint32_t* __restrict__ scratch) {
    const uint32_t lv = v - S.v0;
    const uint64_t row = (uint64_t)lv * S.N;
    const uint32_t pv = scratch[0];
    Timer* tim = S.tim + (uint64_t)lv * S.Ct;
    for (uint32_t m = blockIdx.x * blockDim.x + threadIdx.x; m < S.N; m += gridDim.x * blockDim.x) {
        uint8_t st = ST_ALIVE;
        int64_t inc = incv;
        if (m != v) {
            for (uint32_t q = 0; q < nj; q++) {
                const uint8_t s2 = J.st[q][m] & ST_MASK;
                const int64_t i2 = J.inc[q][m];
                if (q == 0 || i2 > inc) {
                    st = s2;
                    inc = i2;
                }
            }
        }
        const bool ring = st == ST_ALIVE || st == ST_SUSPECT;
        S.st[row + m] = st | (ring ? IN_RING : 0);
        S.inc[row + m] = inc;
        S.slot[row + m] = 0;
        if (!ring) atomicAdd(&scratch[1], 1u);
        if (st != ST_ALIVE || inc != S.inc0[m]) {
            const uint32_t k = S.rank[m];
            atomicOr(&S.dev[(uint64_t)lv * S.W + (k >> 5)], 1u << (k & 31));
        }
        if (st == ST_SUSPECT && m != v) {
            const uint32_t q = atomicAdd(&S.n_tim[lv], 1u);
            if (q < S.Ct) tim[q] = Timer{m, (int32_t)(S.round + S.susp), inc};
            else set_err(S, ERR_TIMERS);
        }
        // members array: self, then r0's without self
        if (m == 0) S.order[row] = v;
        const uint32_t k = m;  // position k of r0's array goes to k + 1 (before v) or k (after)
        const uint32_t a = J.order0[k];
        if (a != v) S.order[row + (k < pv ? k + 1 : k)] = a;
    }
}

// the joiner's scalars, then gossip.start's shuffle (one lane)
__global__ void k_join_finish(SimDev S, uint32_t v, uint32_t* __restrict__ scratch) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    const uint32_t lv = v - S.v0;
    S.ring_count[lv] = S.N - scratch[1];
    S.max_piggy[lv] = 15u * digits(1);  // makeAlive(self)'s ringChanged; set() emits none
    S.n_chg[lv] = 0;
    S.it_idx[lv] = -1;
    S.n_shuf[lv] = 0;
    S.stopped[lv] = 0;
    S.dirty[lv] = 1;
    S.target[lv] = -1;
    lane0_shuffle(S, lv, true);
}

// ---- outboxes: messages grouped by destination shard

// Candidate c of a message kind: its destination shard (G = none) and the sort value c.
//   K_PING  c = local sender        -> shard of its live target
//   K_LEG   c = local sender * 3 + k -> shard of helper k (live helpers only)
//   K_RESP / K_LRESP c = inbound message (receive order) -> shard of its sender
__global__ void k_out_keys(SimDev S, int kind, uint32_t C, uint32_t* __restrict__ key, uint32_t* __restrict__ val) {
    for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < C; c += gridDim.x * blockDim.x) {
        uint32_t k = S.G;
        if (kind == K_PING) {
            const int32_t t = S.target[c];
            if (!S.dead[S.v0 + c] && t >= 0 && !S.dead[t]) k = shard_of(S, (uint32_t)t);
        } else if (kind == K_LEG) {
            const uint32_t lv = c / 3, j = c % 3;
            if (j < S.nhelp[lv] && !S.dead[S.helpers[c]]) k = shard_of(S, S.helpers[c]);
        } else {
            k = shard_of(S, S.in_msg[c].from);
        }
        key[c] = k;
        val[c] = c;
    }
}

__device__ __forceinline__ uint32_t out_count(const SimDev& S, int kind, uint32_t c) {
    if (kind == K_PING) return S.ping_n[c];
    if (kind == K_LEG) return S.leg_nk[c];
    const uint32_t n = S.rsp_n[c];
    return n == NONE ? 0u : n;
}

// records of each sorted message (0 past the last real one)
__global__ void k_out_counts(SimDev S, int kind, const uint32_t* __restrict__ key, const uint32_t* __restrict__ val,
                             uint32_t C, uint32_t* __restrict__ cnt) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < C; i += gridDim.x * blockDim.x)
        cnt[i] = key[i] < S.G ? out_count(S, kind, val[i]) : 0u;
}

// one workgroup per message: header + records (leg records filtered by the leg's count rule),
// into the packed outbox: destination d's segment at byte seg[d] holds its headers, then its
// records
__global__ __launch_bounds__(kT) void k_out_fill(SimDev S, int kind, const uint32_t* __restrict__ key,
                                                 const uint32_t* __restrict__ val, uint32_t nmsg,
                                                 const uint32_t* __restrict__ roff, const uint32_t* __restrict__ moff,
                                                 const uint64_t* __restrict__ seg, uint8_t* __restrict__ out) {
    __shared__ uint32_t lds[16];
    for (uint32_t i = blockIdx.x; i < nmsg; i += gridDim.x) {
        const uint32_t c = val[i], d = key[i];
        const uint64_t r0 = roff[i], dbase = roff[moff[d]];
        Msg* out_msg = reinterpret_cast<Msg*>(out + seg[d]) - moff[d];
        Rec* out_rec = reinterpret_cast<Rec*>(out + seg[d] + sizeof(Msg) * (uint64_t)(moff[d + 1] - moff[d])) - dbase;
        Msg m{};
        const Rec* src = nullptr;
        uint32_t nsrc = 0, k = 0, maxp = 0;
        if (kind == K_PING) {
            m = Msg{S.v0 + c, (uint32_t)S.target[c], S.ping_n[c], 0u, S.ck_snap[c], 0u, S.inc_snap[c], r0 - dbase};
            src = ping_slot(S, c);
            nsrc = m.n;
        } else if (kind == K_LEG) {
            const uint32_t lv = c / 3;
            k = c % 3;
            m = Msg{S.v0 + lv, S.helpers[c], S.leg_nk[c], k, S.ck_snap[lv], 0u, S.inc_snap[lv], r0 - dbase};
            src = leg_slot(S, lv);
            nsrc = S.leg_n[lv];
            maxp = S.max_piggy[lv];
        } else {
            const Msg q = S.in_msg[c];
            m = Msg{q.to, q.from, S.rsp_n[c], q.tag, 0u, 0u, 0, r0 - dbase};
            src = S.pool + S.rsp_off[c];
            nsrc = m.n == NONE ? 0u : m.n;
        }
        if (threadIdx.x == 0) out_msg[i] = m;
        Rec* dst = out_rec + r0;
        if (kind != K_LEG || k == 0) {
            for (uint32_t j = threadIdx.x; j < nsrc; j += kT) dst[j] = src[j];
        } else {
            uint32_t w = 0;
            for (uint32_t base = 0; base < nsrc; base += kT) {
                const uint32_t j = base + threadIdx.x;
                Rec r{};
                bool ok = false;
                if (j < nsrc) {
                    r = src[j];
                    ok = rec_aux(r) + k <= maxp;
                }
                uint32_t tot;
                const uint32_t p = block_scan(ok ? 1u : 0u, lds, &tot);
                if (ok) dst[w + p] = r;
                w += tot;
            }
        }
        __syncthreads();
    }
}

// ---- inboxes

// the inbox's headers in arrival order (sources in shard order), their record offsets made
// absolute byte offsets into the inbox. tab = {message base [G + 1], segment byte offset [G]}
__global__ void k_in_gather(Msg* __restrict__ msg, uint32_t n, const uint8_t* __restrict__ buf,
                            const uint64_t* __restrict__ tab, uint32_t G) {
    const uint64_t* mbase = tab;
    const uint64_t* segb = tab + G + 1;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        uint32_t s = 0;
        while (s + 1 < G && i >= mbase[s + 1]) s++;
        const uint64_t nm = mbase[s + 1] - mbase[s];
        Msg m = reinterpret_cast<const Msg*>(buf + segb[s])[i - mbase[s]];
        m.roff = segb[s] + sizeof(Msg) * nm + sizeof(Rec) * m.roff;
        msg[i] = m;
    }
}

__global__ void k_in_keys(SimDev S, uint32_t* __restrict__ key, uint32_t* __restrict__ val) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < S.nin; i += gridDim.x * blockDim.x) {
        key[i] = S.in_msg[i].to - S.v0;
        val[i] = i;
    }
}

__global__ void k_fill_none(uint32_t* p, uint32_t n) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) p[i] = NONE;
}

// responses: the inbound message index of each local sender (K_RESP) or (sender, leg) (K_LRESP)
__global__ void k_in_scatter(SimDev S, int kind) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < S.nin; i += gridDim.x * blockDim.x) {
        const Msg m = S.in_msg[i];
        const uint32_t lv = m.to - S.v0;
        if (kind == K_RESP) S.resp_idx[lv] = i;
        else S.lresp_idx[lv * 3 + m.tag] = i;
    }
}

__global__ void k_csr(const uint32_t* __restrict__ keys, uint32_t n, uint32_t N, uint32_t* __restrict__ off) {
    for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j <= N; j += gridDim.x * blockDim.x) {
        uint32_t lo = 0, hi = n;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (keys[mid] < j) lo = mid + 1;
            else hi = mid;
        }
        off[j] = lo;
    }
}

// The outbox's per-destination message offsets and the record offsets at them, in one array the
// host reads with one copy (build_out's one host wait of a stage).
__global__ void k_out_cnt_pack(const uint32_t* __restrict__ moff, const uint32_t* __restrict__ ooff, uint32_t G,
                               uint32_t* __restrict__ out) {
    for (uint32_t g = threadIdx.x; g <= G; g += blockDim.x) {
        const uint32_t m = moff[g];
        out[g] = m;
        out[G + 1 + g] = ooff[m];
    }
}

// ---- convergence over this shard's nodes that are up and have not left (scenario-runner.js's
// hostToAliveWorker): {count, min checksum, max checksum, some wanted member not at its wanted
// status in one of those views}. want[i] = member | status << 24: a member that left must be
// `leave`, any other member that is down `faulty`.
// Two launches: the live count and checksum range (one atomic of each kind per wave), then the
// wanted statuses, which the second launch reads only when this shard's live checksums are all
// equal (otherwise the handle has not converged whatever they are: conv_reduce needs min == max).
__global__ void k_conv_ck(SimDev S, const uint8_t* __restrict__ skip, uint32_t* __restrict__ out) {
    uint32_t cnt = 0, lo = 0xFFFFFFFFu, hi = 0;
    for (uint32_t lv = blockIdx.x * blockDim.x + threadIdx.x; lv < S.NL; lv += gridDim.x * blockDim.x) {
        if (skip[S.v0 + lv]) continue;
        const uint32_t c = S.checksum[lv];
        cnt++;
        lo = c < lo ? c : lo;
        hi = c > hi ? c : hi;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        cnt += __shfl_xor(cnt, o, 64);
        const uint32_t l2 = __shfl_xor(lo, o, 64), h2 = __shfl_xor(hi, o, 64);
        lo = l2 < lo ? l2 : lo;
        hi = h2 > hi ? h2 : hi;
    }
    if ((threadIdx.x & 63) == 0 && cnt) {
        atomicAdd(&out[0], cnt);
        atomicMin(&out[1], lo);
        atomicMax(&out[2], hi);
    }
}
__global__ void k_conv_local(SimDev S, const uint8_t* __restrict__ skip, const uint32_t* __restrict__ want,
                             uint32_t nk, uint32_t* __restrict__ out) {
    if (out[0] == 0 || out[1] != out[2]) return;  // block-uniform
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (uint64_t)S.NL * nk;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t lv = (uint32_t)(i / nk), w = want[i % nk], a = w & 0xFFFFFFu;
        if (skip[S.v0 + lv]) continue;
        if ((S.st[(uint64_t)lv * S.N + a] & ST_MASK) != (w >> 24)) out[3] = 1;
    }
}

__global__ void k_sim_init(SimDev S) {
    const uint64_t NN = (uint64_t)S.NL * S.N;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < NN; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t v = S.v0 + (uint32_t)(i / S.N), a = (uint32_t)(i % S.N);
        S.st[i] = ST_ALIVE | IN_RING;
        S.inc[i] = S.inc0[a];
        S.slot[i] = 0;
        // members array after bootstrap: self first (makeAlive), then set() in id order
        S.order[i] = a == 0 ? v : (a <= v ? a - 1 : a);
    }
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (uint64_t)S.NL * S.W;
         i += (uint64_t)gridDim.x * blockDim.x)
        S.dev[i] = 0;
    for (uint32_t lv = blockIdx.x * blockDim.x + threadIdx.x; lv < S.NL; lv += gridDim.x * blockDim.x) {
        S.it_idx[lv] = -1;
        S.n_shuf[lv] = 0;
        S.ring_count[lv] = S.N;
        S.max_piggy[lv] = 15u * digits(S.N);
        S.dirty[lv] = 1;  // first checksum by k_ck_lanes
        S.n_chg[lv] = 0;
        S.n_tim[lv] = 0;
        S.t_head[lv] = 0;
        S.vfp[lv] = 0;
        S.vdt[lv] = 0;
        S.target[lv] = -1;
        S.nhelp[lv] = 0;
        S.stopped[lv] = 0;
    }
}

__global__ void k_sim_start(SimDev S) {  // gossip.start -> membership.shuffle() on live nodes
    for (uint32_t lv = blockIdx.x * blockDim.x + threadIdx.x; lv < S.NL; lv += gridDim.x * blockDim.x)
        if (!S.dead[S.v0 + lv]) lane0_shuffle(S, lv, false);
}

// opos = the inverse of every row of order (one workgroup per row)
__global__ void k_opos_build(SimDev S) {
    for (uint32_t lv = blockIdx.x; lv < S.NL; lv += gridDim.x) {
        const uint64_t row = (uint64_t)lv * S.N;
        for (uint32_t k = threadIdx.x; k < S.N; k += blockDim.x) S.opos[row + S.order[row + k]] = k;
    }
}

// every node starts with the same view: hash it once, copy to all
__global__ void k_sim_first_checksum(SimDev S) {
    if (blockIdx.x == 0 && threadIdx.x == 0) S.checksum[0] = lane_checksum(S, 0);
}

__global__ void k_sim_bcast_checksum(SimDev S) {
    for (uint32_t lv = blockIdx.x * blockDim.x + threadIdx.x; lv < S.NL; lv += gridDim.x * blockDim.x) {
        S.checksum[lv] = S.checksum[0];
        S.dirty[lv] = 0;
    }
}

}  // namespace

// An exchange buffer: one segment per peer shard, in shard order, each holding that peer's
// 40-byte headers then its 24-byte records (nmsg/nrec[G]). The outbox is sent and the inbox
// received as they lie (one all-to-all-v), kept across rounds and grown geometrically.
struct MsgBuf {
    DevBuf<uint8_t> buf;
    std::vector<uint64_t> nmsg, nrec;
    uint64_t tot_msg = 0, tot_rec = 0;
    uint64_t seg_bytes(uint32_t g) const { return sizeof(Msg) * nmsg[g] + sizeof(Rec) * nrec[g]; }
    uint64_t seg_off(uint32_t g) const {
        uint64_t o = 0;
        for (uint32_t h = 0; h < g; h++) o += seg_bytes(h);
        return o;
    }
    uint64_t bytes() const { return sizeof(Msg) * tot_msg + sizeof(Rec) * tot_rec; }
    void size_for(uint64_t b) {
        if (b + 8 > buf.cap) {
            const uint64_t c = std::max<uint64_t>(b + 8, 2 * buf.cap);
            buf.reserve(c);
        }
    }
    void swap(MsgBuf& o) {
        buf.swap(o.buf);
        std::swap(nmsg, o.nmsg);
        std::swap(nrec, o.nrec);
        std::swap(tot_msg, o.tot_msg);
        std::swap(tot_rec, o.tot_rec);
    }
};

struct Sim {
    int device = 0;
    hipStream_t st = nullptr;
    // the early refresh (stage 2): dirty views hashed on a side stream beside the D1 sender
    // chains; stage 3 waits for it before phase D2 changes views again (RP_SIM_EARLY=1: on)
    hipStream_t st2 = nullptr;
    hipEvent_t ev_c = nullptr, ev_early = nullptr;
    hipEvent_t ev_ext = nullptr;  // rp_sim_wait_stream: the next stage waits for a caller's stream
    hipEvent_t ev_ord = nullptr;  // rp_sim_order_stream: a caller's stream waits for this handle's
    // Pinned host staging (round 6): a stage's outbox counts come back with one
    // copy and one event wait, and the segment and inbox tables go up from a ring of pinned slots,
    // so the host waits neither for the outbox fill nor for an import. A slot is rewritten
    // kPinSlots uses later; every stage with an outbox waits for its counts, which follow every
    // earlier copy on the stream, so no slot is rewritten before its copy ran.
    static constexpr uint32_t kPinSlots = 8;
    uint64_t* h_pin = nullptr;
    uint32_t pin_next = 0;
    hipEvent_t ev_cnt = nullptr;
    DevBuf<uint32_t> ocnt_pack;
    uint64_t* pin_slot() {  // 2G + 2 words
        if (!h_pin) {
            RP_HIP(hipHostMalloc(reinterpret_cast<void**>(&h_pin), 8ull * kPinSlots * (2 * G + 2), hipHostMallocDefault));
            RP_HIP(hipEventCreateWithFlags(&ev_cnt, hipEventDisableTiming));
        }
        uint64_t* p = h_pin + (uint64_t)(pin_next % kPinSlots) * (2 * G + 2);
        pin_next++;
        return p;
    }
    bool early_pending = false;
    bool early_on = [] {
        const char* e = getenv("RP_SIM_EARLY");
        return e && *e == '1';
    }();
    DevBuf<uint32_t> elist;
    uint32_t N = 0, NL = 0, v0 = 0, G = 1, shard = 0;
    unsigned grid = 0;
    NameTable nt;
    SimDev d{};
    DevBuf<uint8_t> st_, dirty, dead, strbuf, sbase, stopped, cskip;
    DevBuf<int64_t> inc, it_idx, inc_snap, inc0;
    DevBuf<int32_t> target;
    DevBuf<uint32_t> slot;
    DevBuf<uint32_t> opos;
    DevBuf<uint32_t> order, dev, n_chg, n_tim, t_head, n_shuf, ring_count, max_piggy, checksum, ck_snap, ping_n, leg_n,
        helpers, nhelp, leg_nk, cand, rank, err, bounds, want, conv, leave_list;
    DevBuf<uint32_t> okey, oval, ocnt, ooff, omoff;  // outbox build
    DevBuf<uint64_t> oseg;                           // outbox segment offsets
    DevBuf<Msg> imsg;                                // inbox headers, gathered
    DevBuf<uint32_t> ib_off, ib_idx, ikey;         // inbox build
    DevBuf<uint32_t> rsp_n, resp_idx, lresp_idx, d1list;
    DevBuf<uint64_t> boff, rsp_off, ibase, vfp;
    DevBuf<int64_t> vdt;
    DevBuf<Change> chg;
    DevBuf<Timer> tim;
    DevBuf<Rec> pool;
    DevBuf<uint4> dlist;
    DevBuf<P1> p1buf;
    DevBuf<unsigned long long> stats, cursor;
    MsgBuf out, in;
    Scratch ws;
    std::vector<uint8_t> h_dead, h_left;
    std::vector<uint32_t> h_bounds;
    std::vector<rp_sim_event> events;  // the scenario, by round
    size_t next_event = 0;
    uint32_t nwant = 0;
    bool conv_dirty = true;
    uint64_t sent_msgs = 0, sent_recs = 0, base_len = 0;  // traffic counters (rp_sim_counters)
    int64_t round = 0;
    int next_stage = 0;  // 0..4 within a round

    uint32_t cus = 0;  // compute units of the device (first refresh)
    void refresh_checksums() {
        if (NL == 0) return;
        // One chain per lane either way. With no more 64-node groups than CUs (a shard, C4) each
        // group gets a whole CU: its chain wave plus three producer waves (k_ck_pc, ~130 cycles
        // per chunk). With more groups than CUs the machine is issue-bound on the chunks'
        // multiplies, and one wave per group without producers (k_ck_lanes) does less work.
        // RP_SIM_CK=pc|lanes overrides.
        if (cus == 0) {
            int dev = 0, n = 0;
            RP_HIP(hipGetDevice(&dev));
            RP_HIP(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev));
            cus = (uint32_t)(n > 0 ? n : 1);
        }
        const uint32_t groups = (NL + 63) / 64;
        {
            const char* ab = getenv("RP_SIM_CK_ABLATE");
            d.ck_ablate = ab && *ab ? (uint32_t)atoi(ab) : 0u;
        }
        hipLaunchKernelGGL(k_count_dirty, dim3(grid_for(NL, 256, 1024)), dim3(256), 0, st, d);
        const char* m = getenv("RP_SIM_CK");
        const bool pc = m ? strcmp(m, "lanes") != 0 : groups <= cus;
        // twins pay on the lane path (C5 on one GPU: 76.7 vs 78.2 ms per round, 31 % fewer
        // chains); at a shard's size (C4, the producer/consumer path) the two passes cost about
        // what they save (3.25 vs 3.14 ms), so RP_SIM_TWINS=1 forces them there
        const char* tw = getenv("RP_SIM_TWINS");
        const bool twins = tw && *tw ? *tw != '0' : !pc;
        if (twins) {
            uint32_t T = 1024;
            while (T < 2 * NL) T <<= 1;
            if (twin_cap < T) {
                twin_key.release();
                twin_rep.release();
                twin_key.reserve(T);
                twin_rep.reserve(T);
                twin_cap = T;
            }
            if (!twin_of.p) {
                twin_of.reserve(NL);
                twin_fp.reserve(NL);
                twin_cnt.reserve(1);
                RP_HIP(hipMemsetAsync(twin_of.p, 0xFF, 4ull * NL, st));
                RP_HIP(hipMemsetAsync(twin_cnt.p, 0, 4, st));
            }
            RP_HIP(hipMemsetAsync(twin_key.p, 0xFF, 8ull * T, st));
            RP_HIP(hipMemsetAsync(twin_rep.p, 0xFF, 4ull * T, st));
            const unsigned gw = grid_for((uint64_t)NL * 64, 256, 4096);
            // RP_SIM_TWIN_VERIFY=1: recompute every fingerprint from the rows (a check of vfp)
            const char* tv = getenv("RP_SIM_TWIN_VERIFY");
            const int verify = tv && *tv && *tv != '0';
            hipLaunchKernelGGL(k_twin_fp, dim3(verify ? gw : grid_for(NL, 256, 4096)), dim3(256), 0, st, d, twin_fp.p,
                               twin_key.p, twin_rep.p, T - 1, verify);
            hipLaunchKernelGGL(k_twin_check, dim3(gw), dim3(256), 0, st, d, twin_fp.p, twin_key.p, twin_rep.p, T - 1,
                               twin_of.p, twin_cnt.p);
            RP_HIP(hipGetLastError());
        }
        // with twins marked clean, the views left to hash are compacted so that waves hold
        // only real chains (a wave runs as long as its longest lane)
        const uint32_t* sel = nullptr;
        const uint32_t* nsel = nullptr;
        if (twins) {
            twin_list.reserve(NL + 1);
            RP_HIP(hipMemsetAsync(twin_list.p + NL, 0, 4, st));
            hipLaunchKernelGGL(k_dirty_list, dim3(grid_for(NL, 256, 1024)), dim3(256), 0, st, d, twin_list.p,
                               twin_list.p + NL);
            sel = twin_list.p;
            nsel = twin_list.p + NL;
        }
        // pc32 (3 producers x 2 chunks per epoch, 41 KB of LDS) puts 3 groups on a CU. On the
        // lane path it takes the rounds whose compacted dirty views fill at most 3 groups per CU
        // (C5 on one GPU: median round 64 against 68 ms); the peak rounds, where nearly every
        // view is dirty and the machine is issue-bound, stay on k_ck_lanes (pc32 there: 111
        // against 96 ms). Choosing reads the dirty count back (one small copy per round).
        bool use32 = m && !strcmp(m, "pc32");
        uint32_t nd_host = 0;
        bool nd_known = false;
        if (!m && !pc && sel) {
            uint32_t nd = 0;
            RP_HIP(hipMemcpyAsync(&nd, nsel, 4, hipMemcpyDeviceToHost, st));
            RP_HIP(hipStreamSynchronize(st));
            nd_host = nd;
            nd_known = true;
            static const uint32_t per_cu = [] {  // A/B: RP_SIM_PC32_PER_CU
                const char* e = getenv("RP_SIM_PC32_PER_CU");
                return e && *e ? (uint32_t)atoi(e) : 3u;
            }();
            use32 = (nd + 63) / 64 <= per_cu * cus;
        }
        // Pass 1 of every view to hash, a wave per view, ahead of the producer/consumer kernels,
        // whose chain wave otherwise walks its 64 views' bitmaps and deviated members before any
        // chunk is produced (C5: k_ck_pc<3, 2> 375 -> 324 ms over a run for 13 ms of k_pass1).
        // k_ck_lanes hides its own lane walks behind other waves: there k_pass1 costs more than
        // it saves (153 against 49 ms), so it stays in the kernel (RP_SIM_PASS1=0|1 overrides).
        const bool lanes_path = !use32 && !pc && !(m && !strcmp(m, "pair"));
        const char* p1e = getenv("RP_SIM_PASS1");
        // The lane path's order (round 6): the views to hash sorted by their string's length delta
        // (vdt, kept by block_apply), so that a wave's 64 lanes reach their deviated pieces in the
        // same chunk groups: the fixup path runs for a whole wave when any lane needs it, and in
        // C5's peak refreshes list order put a fixup in 10-13 % of wave-groups against 3-4 %
        // sorted (-DRP_CKL_STAT, profiles/r06/r06ab, r06ac); C5 p95 round 78 -> 68 ms (r06ae).
        // RP_SIM_CK_SORT: 3 (default) that order, 1 = by this round's shifts from a pass-1
        // launch (slower: the launch), 0 = list order.
        const char* cks = getenv("RP_SIM_CK_SORT");
        const int sort_mode = cks && *cks ? atoi(cks) : 3;
        const bool is_pair = m && !strcmp(m, "pair");
        // The same order on the producer/consumer paths when this handle is one shard of several
        // (each rank of a sharded C5 refreshes on them): C5 in 8 shards on one GPU 147.7 -> 142.6
        // ms per round; C4 on one GPU (not sharded) 2.41 -> 2.46, so not there (profiles/r06/
        // r06ah, r06ai). RP_SIM_CK_SORT_PC=0|1 overrides.
        const char* ckp = getenv("RP_SIM_CK_SORT_PC");
        const bool pc_on = ckp && *ckp ? *ckp == '1' : G > 1;
        const bool sort_pc = !lanes_path && !is_pair && sort_mode == 3 && pc_on;
        if (sort_pc && !sel) {
            twin_list.reserve(NL + 1);
            RP_HIP(hipMemsetAsync(twin_list.p + NL, 0, 4, st));
            hipLaunchKernelGGL(k_dirty_list, dim3(grid_for(NL, 256, 1024)), dim3(256), 0, st, d, twin_list.p,
                               twin_list.p + NL);
            sel = twin_list.p;
            nsel = twin_list.p + NL;
        }
        const bool sort_sel = (lanes_path || sort_pc) && sel && sort_mode > 0;
        const bool pre1 = (sort_sel && sort_mode == 1) || (p1e && *p1e ? *p1e != '0' : !lanes_path);
        if (pre1 && !(m && !strcmp(m, "pair"))) {
            hipLaunchKernelGGL(k_pass1, dim3(grid_for((uint64_t)NL * 64, 256, 4096)), dim3(256), 0, st, d, sel, nsel);
            d.p1_pre = 1;
        }
        if (sort_sel) {
            if (!nd_known) {
                RP_HIP(hipMemcpyAsync(&nd_host, nsel, 4, hipMemcpyDeviceToHost, st));
                RP_HIP(hipStreamSynchronize(st));
            }
            ck_sort_key.reserve(NL + 1);
            ck_sort_sel.reserve(NL + 1);
            hipLaunchKernelGGL(k_ck_sort_keys, dim3(grid_for(NL, 256, 1024)), dim3(256), 0, st, d, sel, nsel,
                               ck_sort_key.p, ck_sort_sel.p, sort_mode == 3 ? 1 : 0);
            if (nd_host > 1) radix_sort_pairs(ck_sort_key.p, ck_sort_sel.p, nd_host, 0, 32, st, ws);
            sel = ck_sort_sel.p;  // (the count stays *nsel)
        }
        if (m && !strcmp(m, "pair"))  // A/B: the lane-pair chains, 32 views per workgroup
            hipLaunchKernelGGL((k_ck_pair<6, 2, 32>), dim3((NL + 31) / 32), dim3(512), 0, st, d, sel, nsel);
        else if (use32)
            hipLaunchKernelGGL((k_ck_pc<3, 2>), dim3(groups), dim3(256), 0, st, d, sel, nsel);
        else if (pc && !(m && !strcmp(m, "pc3")))
            hipLaunchKernelGGL(k_ck_pc<7>, dim3(groups), dim3(512), 0, st, d, sel, nsel);
        else if (pc)
            hipLaunchKernelGGL(k_ck_pc<3>, dim3(groups), dim3(256), 0, st, d, sel, nsel);
        else
            hipLaunchKernelGGL(k_ck_lanes, dim3(grid_for(NL, 256, 1u << 20)), dim3(256), 0, st, d, sel, nsel);
#ifdef RP_CKL_STAT
        if (getenv("RP_CKL_STAT_PRINT")) {
            unsigned long long v[8];
            RP_HIP(hipStreamSynchronize(st));
            RP_HIP(hipMemcpyFromSymbol(v, HIP_SYMBOL(g_ckl_stat), sizeof v));
            if (v[0])
                fprintf(stderr, "[rp] k_ck_lanes: %llu wave-groups, %.1f %% with a fixup; lane-groups %.2f %% with one; "
                                "redone lane-chunks: clean %llu, status overlay %llu, byte-wise %llu\n",
                        v[0], 100.0 * v[1] / v[0], v[3] ? 100.0 * v[2] / v[3] : 0.0, v[5], v[6], v[7]);
            memset(v, 0, sizeof v);
            RP_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_ckl_stat), v, sizeof v));
        }
#endif
        d.p1_pre = 0;
        if (twins) hipLaunchKernelGGL(k_twin_copy, dim3(grid_for(NL, 256)), dim3(256), 0, st, d, twin_of.p);
        RP_HIP(hipGetLastError());
    }
    // dirty views with equal content hash once (k_twin_*); RP_SIM_TWINS=0|1 overrides
    DevBuf<uint64_t> twin_fp;
    DevBuf<unsigned long long> twin_key;
    DevBuf<uint32_t> twin_rep, twin_of, twin_cnt, twin_list;
    DevBuf<uint32_t> ck_sort_key, ck_sort_sel;  // RP_SIM_CK_SORT
    uint32_t twin_cap = 0;

    // Outbox of a message kind: sort candidates by destination shard (stable), scan the record
    // counts, fill headers + records. Leaves out.nmsg/nrec per destination.
    void build_out(int kind) {
        const uint32_t C = kind == K_PING ? NL : kind == K_LEG ? 3 * NL : (uint32_t)in.tot_msg;
        out.nmsg.assign(G, 0);
        out.nrec.assign(G, 0);
        out.tot_msg = out.tot_rec = 0;
        if (C == 0) return;
        okey.reserve(C + 1);
        oval.reserve(C + 1);
        ocnt.reserve(C + 1);
        ooff.reserve(C + 1);
        omoff.reserve(G + 1);
        hipLaunchKernelGGL(k_out_keys, dim3(grid_for(C, 256)), dim3(256), 0, st, d, kind, C, okey.p, oval.p);
        if (kind == K_PING || kind == K_LEG) radix_sort_pairs(okey.p, oval.p, C, 0, 8, st, ws);
        hipLaunchKernelGGL(k_out_counts, dim3(grid_for(C, 256)), dim3(256), 0, st, d, kind, okey.p, oval.p, C, ocnt.p);
        scan_exclusive_u32(ocnt.p, ooff.p, C, st, ws);
        hipLaunchKernelGGL(k_csr, dim3(1), dim3(128), 0, st, okey.p, C, G, omoff.p);
        ocnt_pack.reserve(2 * G + 2);
        hipLaunchKernelGGL(k_out_cnt_pack, dim3(1), dim3(64), 0, st, omoff.p, ooff.p, G, ocnt_pack.p);
        RP_HIP(hipGetLastError());
        const uint32_t* hc = reinterpret_cast<const uint32_t*>(pin_slot());
        RP_HIP(hipMemcpyAsync(const_cast<uint32_t*>(hc), ocnt_pack.p, 4ull * (2 * G + 2), hipMemcpyDeviceToHost, st));
        RP_HIP(hipEventRecord(ev_cnt, st));
        RP_HIP(hipEventSynchronize(ev_cnt));  // the stage's one host wait: its counts
        const uint32_t *moff = hc, *roff = hc + G + 1;
        out.tot_msg = moff[G];
        out.tot_rec = roff[G];
        sent_msgs += out.tot_msg;
        sent_recs += out.tot_rec;
        for (uint32_t g = 0; g < G; g++) {
            out.nmsg[g] = moff[g + 1] - moff[g];
            out.nrec[g] = roff[g + 1] - roff[g];
        }
        uint64_t* seg = pin_slot();
        for (uint32_t g = 0; g <= G; g++) seg[g] = out.seg_off(g);
        out.size_for(out.bytes());
        oseg.reserve(G + 1);
        RP_HIP(hipMemcpyAsync(oseg.p, seg, 8ull * (G + 1), hipMemcpyHostToDevice, st));
        if (out.tot_msg)
            hipLaunchKernelGGL(k_out_fill, dim3(grid_for(out.tot_msg, 1, 4096)), dim3(kT), 0, st, d, kind, okey.p,
                               oval.p, (uint32_t)out.tot_msg, ooff.p, omoff.p, oseg.p, out.buf.p);
        RP_HIP(hipGetLastError());  // no wait for the fill: rp_sim_order_stream orders its readers
    }

    // Size the inbox for per-source counts (the caller then fills in.buf, segments in source order).
    void prepare_in(const uint64_t* nmsg, const uint64_t* nrec) {
        in.nmsg.assign(nmsg, nmsg + G);
        in.nrec.assign(nrec, nrec + G);
        in.tot_msg = in.tot_rec = 0;
        for (uint32_t g = 0; g < G; g++) {
            in.tot_msg += nmsg[g];
            in.tot_rec += nrec[g];
        }
        RP_REQUIRE(in.tot_msg < (1ull << 32), "sim: too many inbound messages");
        in.size_for(in.bytes());
    }

    // One shard: the outbox is the inbox.
    void self_exchange() {
        std::vector<uint64_t> nm = out.nmsg, nr = out.nrec;
        in.swap(out);
        in.nmsg = nm;
        in.nrec = nr;
    }

    // Bind the inbox to the device view: gather the headers (absolute record offsets), index them.
    void import_in(int kind) {
        imsg.reserve(in.tot_msg + 1);
        d.in_msg = imsg.p;
        d.in_buf = in.buf.p;
        d.nin = (uint32_t)in.tot_msg;
        if (in.tot_msg) {
            uint64_t* tab = pin_slot();
            uint64_t m = 0;
            for (uint32_t g = 0; g < G; g++) {
                tab[g] = m;
                m += in.nmsg[g];
                tab[G + 1 + g] = in.seg_off(g);
            }
            tab[G] = m;
            ibase.reserve(2 * G + 1);
            RP_HIP(hipMemcpyAsync(ibase.p, tab, 8ull * (2 * G + 1), hipMemcpyHostToDevice, st));
            hipLaunchKernelGGL(k_in_gather, dim3(grid_for(in.tot_msg, 256)), dim3(256), 0, st, imsg.p,
                               (uint32_t)in.tot_msg, in.buf.p, ibase.p, G);
        }
        const uint32_t n = (uint32_t)in.tot_msg;
        if (kind == K_PING || kind == K_LEG) {
            ikey.reserve(n + 1);
            ib_idx.reserve(n + 1);
            ib_off.reserve(NL + 1);
            rsp_n.reserve(n + 1);
            rsp_off.reserve(n + 1);
            if (n) {
                hipLaunchKernelGGL(k_in_keys, dim3(grid_for(n, 256)), dim3(256), 0, st, d, ikey.p, ib_idx.p);
                int bits = 8;
                while (bits < 32 && (1ull << bits) <= NL) bits += 8;
                radix_sort_pairs(ikey.p, ib_idx.p, n, 0, bits, st, ws);
            }
            hipLaunchKernelGGL(k_csr, dim3(grid_for(NL + 1, 256)), dim3(256), 0, st, ikey.p, n, NL, ib_off.p);
            d.ib_off = ib_off.p;
            d.ib_idx = ib_idx.p;
            d.rsp_n = rsp_n.p;
            d.rsp_off = rsp_off.p;
        } else {
            uint32_t* idx = kind == K_RESP ? resp_idx.p : lresp_idx.p;
            const uint32_t cnt = kind == K_RESP ? NL : 3 * NL;
            hipLaunchKernelGGL(k_fill_none, dim3(grid_for(cnt, 256)), dim3(256), 0, st, idx, cnt);
            if (n) hipLaunchKernelGGL(k_in_scatter, dim3(grid_for(n, 256)), dim3(256), 0, st, d, kind);
        }
        RP_HIP(hipGetLastError());
    }

    // Stage k of a round. 0: checksums + A -> pings out. 1: pings in, B -> responses out.
    // 2: responses in, C, D1 -> legs out. 3: legs in, D2 -> leg responses out.
    // 4: leg responses in, D3, E; the round ends.
    void stage(int k) {
        RP_REQUIRE(k == next_stage, "sim: stages must run in order 0..4");
        d.round = round;
        const unsigned g = grid;
        switch (k) {
        case 0:
            apply_events();
            hipLaunchKernelGGL(k_round_begin, dim3(1), dim3(64), 0, st, d);
            refresh_checksums();
            if (NL) hipLaunchKernelGGL(k_phase_a, dim3(g), dim3(kT), 0, st, d);
            build_out(K_PING);
            break;
        case 1:
            import_in(K_PING);
            if (NL) hipLaunchKernelGGL(k_phase_b, dim3(g), dim3(kT), 0, st, d);
            build_out(K_RESP);
            break;
        case 2:
            import_in(K_RESP);
            if (NL) {
                hipLaunchKernelGGL(k_phase_c, dim3(g), dim3(kT), 0, st, d);
                d1list.reserve(NL + 1);
                RP_HIP(hipMemsetAsync(d1list.p + NL, 0, 4, st));
                hipLaunchKernelGGL(k_d1_list, dim3(grid_for(NL, 256)), dim3(256), 0, st, d, d1list.p, d1list.p + NL);
                const bool early = early_on;
                if (early) {  // this round's dirty views except the D1 senders, listed after C
                    elist.reserve(NL + 1);
                    RP_HIP(hipMemsetAsync(elist.p + NL, 0, 4, st));
                    hipLaunchKernelGGL(k_early_list, dim3(grid_for(NL, 256, 1024)), dim3(256), 0, st, d, elist.p,
                                       elist.p + NL);
                    if (!st2) {
                        RP_HIP(hipStreamCreateWithFlags(&st2, hipStreamNonBlocking));
                        RP_HIP(hipEventCreateWithFlags(&ev_c, hipEventDisableTiming));
                        RP_HIP(hipEventCreateWithFlags(&ev_early, hipEventDisableTiming));
                    }
                    RP_HIP(hipEventRecord(ev_c, st));
                }
                // the senders' checksums (their ping-req bodies carry them) as side-by-side chains
                // first, so D1's workgroups find their views clean
                // (RP_SIM_D1_CK=pc: k_ck_pc's one lane per view; blockck: a workgroup per sender
                // inside D1)
                const char* d1ck = getenv("RP_SIM_D1_CK");
                if (d1ck && !strcmp(d1ck, "pc"))
                    hipLaunchKernelGGL(k_ck_pc<7>, dim3((NL + 63) / 64), dim3(512), 0, st, d, d1list.p, d1list.p + NL);
                else if (!(d1ck && !strcmp(d1ck, "blockck")) && !getenv("RP_SIM_D1_BLOCKCK"))
                {
                    static const int vpg = [] {  // A/B: RP_SIM_D1_VPG = 8 | 16
                        const char* e = getenv("RP_SIM_D1_VPG");
                        return e && *e ? atoi(e) : 8;
                    }();
                    if (vpg == 16)
                        hipLaunchKernelGGL((k_ck_pair<6, 2, 16>), dim3((NL + 15) / 16), dim3(512), 0, st, d, d1list.p,
                                           d1list.p + NL);
                    else
                        hipLaunchKernelGGL((k_ck_pair<6, 2, 8>), dim3((NL + 7) / 8), dim3(512), 0, st, d, d1list.p,
                                           d1list.p + NL);
                }
                hipLaunchKernelGGL(k_phase_d1, dim3(g), dim3(kT), 0, st, d, d1list.p, d1list.p + NL);
                if (early) {
                    // The D1 chains hold a few CUs for milliseconds (one 64-view group per CU);
                    // the rest of the machine hashes the views B and C dirtied, which the next
                    // round's refresh would otherwise hash after E. A view that D2, D3 or E
                    // changes again is dirty again and is hashed again then.
                    RP_HIP(hipStreamWaitEvent(st2, ev_c, 0));
                    const uint32_t groups = (NL + 63) / 64;
                    if (groups <= cus)
                        hipLaunchKernelGGL(k_ck_pc<7>, dim3(groups), dim3(512), 0, st2, d, elist.p, elist.p + NL);
                    else
                        hipLaunchKernelGGL(k_ck_lanes, dim3(grid_for(NL, 256, 1u << 20)), dim3(256), 0, st2, d,
                                           elist.p, elist.p + NL);
                    RP_HIP(hipGetLastError());
                    RP_HIP(hipEventRecord(ev_early, st2));
                    early_pending = true;
                }
            }
            build_out(K_LEG);
            break;
        case 3:
            import_in(K_LEG);
            if (early_pending) {  // D2 changes helper views: the early refresh must be done
                RP_HIP(hipStreamWaitEvent(st, ev_early, 0));
                early_pending = false;
            }
            if (NL) hipLaunchKernelGGL(k_phase_d2, dim3(g), dim3(kT), 0, st, d);
            build_out(K_LRESP);
            break;
        case 4:
            import_in(K_LRESP);
            if (NL) {
                hipLaunchKernelGGL(k_phase_d3, dim3(g), dim3(kT), 0, st, d);
                hipLaunchKernelGGL(k_phase_e, dim3(g), dim3(kT), 0, st, d);
            }
            round++;
            break;
        }
        RP_HIP(hipGetLastError());
        next_stage = (k + 1) % 5;
    }

    void step() {  // one shard: a whole round
        RP_REQUIRE(G == 1, "sim: a sharded handle advances through rp_sim_stage + an exchange");
        for (int k = 0; k < 5; k++) {
            stage(k);
            if (k < 4) self_exchange();
        }
    }

    void check_err() {
        uint32_t e = 0;
        RP_HIP(hipMemcpyAsync(&e, err.p, 4, hipMemcpyDeviceToHost, st));
        RP_HIP(hipStreamSynchronize(st));
        if (e & ERR_CHANGES)
            throw Error(RP_ESTATE, "sim: a node's dissemination list exceeded its capacity (RP_SIM_CAP)");
        if (e & ERR_TIMERS) throw Error(RP_ESTATE, "sim: a node's suspicion timers exceeded their capacity (RP_SIM_CAP)");
        if (e & ERR_ARENA) throw Error(RP_ESTATE, "sim: the per-round message arena overflowed (RP_SIM_ARENA)");
        if (e & ERR_TWINFP)
            throw Error(RP_ESTATE, "sim: a view's kept twin fingerprint differs from its rows (RP_SIM_TWIN_VERIFY)");
    }

    // The scenario's events of this round, before phase A: a node goes down or comes back (every
    // shard keeps the global down flags), or leaves (on the shard that owns it).
    DevBuf<uint32_t> join_scratch;

    // leaves collected so far run before anything that reads the views (a join)
    void flush_leaves(std::vector<uint32_t>& leaves) {
        if (leaves.empty()) return;
        leave_list.reserve(leaves.size());
        RP_HIP(hipMemcpyAsync(leave_list.p, leaves.data(), 4 * leaves.size(), hipMemcpyHostToDevice, st));
        d.round = round;
        hipLaunchKernelGGL(k_leave, dim3((unsigned)std::min<size_t>(leaves.size(), 1024)), dim3(kT), 0, st, d,
                           leave_list.p, (uint32_t)leaves.size());
        RP_HIP(hipGetLastError());
        RP_HIP(hipStreamSynchronize(st));  // the host vector is reused
        leaves.clear();
    }

    // A join in progress: the joiner, its responders (host-chosen, identical on every shard)
    // and the incarnation its responders give it.
    struct Join {
        uint32_t v = 0, r[3] = {0, 0, 0}, nj = 0;
        int64_t incv = 0;
        bool active = false;
    } pj;
    DevBuf<uint8_t> jx;  // join exchange buffer (JoinBuf layout)

    bool local_node(uint32_t u) const { return u >= v0 && u < v0 + NL; }

    void join_begin(uint32_t v) {
        std::vector<uint32_t> cand;
        for (uint32_t u = 0; u < N; u++)
            if (u != v && !h_dead[u]) cand.push_back(u);
        const uint32_t nj = (uint32_t)std::min<size_t>(3, cand.size());
        RP_REQUIRE(nj > 0, "sim: a join needs at least one live node to answer it");
        for (uint32_t q = 0; q < nj; q++) {  // partial Fisher-Yates, JOIN stream
            const uint32_t r = philox4x32_10(U4{(uint32_t)round, q, v, 0u}, d.seed, TAG_JOIN).x;
            const uint32_t j = q + (uint32_t)(((uint64_t)r * (cand.size() - q)) >> 32);
            std::swap(cand[q], cand[j]);
        }
        pj.v = v;
        pj.nj = nj;
        for (uint32_t q = 0; q < 3; q++) pj.r[q] = q < nj ? cand[q] : 0;
        pj.incv = d.now0 + 200 * round;
        pj.active = true;
        d.round = round;
        uint32_t local = 0;
        for (uint32_t q = 0; q < nj; q++) local |= (local_node(pj.r[q]) ? 1u : 0u) << q;
        if (local)
            hipLaunchKernelGGL(k_join_resp, dim3(nj), dim3(kT), 0, st, d, v, pj.incv, pj.r[0], pj.r[1], pj.r[2], nj,
                               local);
        RP_HIP(hipGetLastError());
    }

    // the joiner's view from its responders' rows (on the joiner's shard), then the global flags
    void join_finish(const JoinSrc& J) {
        const uint32_t v = pj.v;
        if (local_node(v)) {
            join_scratch.reserve(2);
            RP_HIP(hipMemsetAsync(join_scratch.p, 0, 8, st));
            RP_HIP(hipMemsetAsync(n_tim.p + (v - v0), 0, 4, st));
            RP_HIP(hipMemsetAsync(t_head.p + (v - v0), 0, 4, st));
            hipLaunchKernelGGL(k_join_prep, dim3(grid_for(std::max(N, d.W), 256)), dim3(256), 0, st, d, v, J,
                               join_scratch.p);
            hipLaunchKernelGGL(k_join_view, dim3(grid_for(N, 256)), dim3(256), 0, st, d, v, pj.incv, pj.nj, J,
                               join_scratch.p);
            hipLaunchKernelGGL(k_join_finish, dim3(1), dim3(64), 0, st, d, v, join_scratch.p);
            hipLaunchKernelGGL(k_vfp_view, dim3(1), dim3(64), 0, st, d, v - v0);
            RP_HIP(hipGetLastError());
        }
        h_dead[v] = 0;
        h_left[v] = 0;
        RP_HIP(hipMemcpyAsync(dead.p, h_dead.data(), N, hipMemcpyHostToDevice, st));
        RP_HIP(hipStreamSynchronize(st));
        pj.active = false;
        conv_dirty = true;
    }

    // one shard holding every responder: the joiner reads their rows in place
    void join(uint32_t v) {
        join_begin(v);
        JoinSrc J{};
        for (uint32_t q = 0; q < 3; q++) {
            const uint64_t row = (uint64_t)((q < pj.nj ? pj.r[q] : pj.r[0]) - v0) * N;
            J.st[q] = d.st + row;
            J.inc[q] = d.inc + row;
        }
        J.order0 = d.order + (uint64_t)(pj.r[0] - v0) * N;
        join_finish(J);
    }

    // The round's events up to the next join: kills, revives and leaves are applied; a join is
    // applied in place when this handle holds every node (stop_at_join false), else it is
    // begun (responders answer) and left for the join exchange. Returns true at such a join.
    bool apply_events_until_join(bool stop_at_join) {
        bool down_changed = false;
        std::vector<uint32_t> leaves;
        bool stopped = false;
        while (next_event < events.size() && events[next_event].round <= (uint64_t)round) {
            const rp_sim_event& e = events[next_event];
            if (e.round != (uint64_t)round) {
                next_event++;
                continue;
            }
            if (e.kind == RP_SIM_JOIN) {
                flush_leaves(leaves);
                if (down_changed) RP_HIP(hipMemcpyAsync(dead.p, h_dead.data(), N, hipMemcpyHostToDevice, st));
                down_changed = false;
                if (stop_at_join) {
                    next_event++;
                    join_begin(e.node);
                    stopped = true;
                    break;
                }
                RP_REQUIRE(G == 1, "sim: a sharded simulator takes join events through rp_sim_join_export / "
                                   "rp_sim_join_import before stage 0 (the joiner reads its responders' views)");
                next_event++;
                join(e.node);
                continue;
            }
            next_event++;
            if (e.kind == RP_SIM_KILL || e.kind == RP_SIM_REVIVE) {
                const uint8_t dv = e.kind == RP_SIM_KILL ? 1 : 0;
                down_changed |= h_dead[e.node] != dv;
                h_dead[e.node] = dv;
            } else if (!h_dead[e.node] && !h_left[e.node]) {
                h_left[e.node] = 1;
                if (e.node >= v0 && e.node < v0 + NL) leaves.push_back(e.node - v0);
            }
            conv_dirty = true;
        }
        if (down_changed) RP_HIP(hipMemcpyAsync(dead.p, h_dead.data(), N, hipMemcpyHostToDevice, st));
        flush_leaves(leaves);
        if (down_changed) RP_HIP(hipStreamSynchronize(st));  // host vectors reused
        return stopped;
    }
    void apply_events() { apply_events_until_join(false); }

    // rp_sim_join_export: up to the next join of this round; its responders' rows on this shard
    // go into jx (zeros elsewhere)
    bool join_export() {
        RP_REQUIRE(next_stage == 0, "sim_join_export: call before stage 0 of a round");
        RP_REQUIRE(!pj.active, "sim_join_export: the previous join was not imported");
        if (!apply_events_until_join(true)) return false;
        const JoinBuf B(N);
        jx.reserve(B.bytes);
        RP_HIP(hipMemsetAsync(jx.p, 0, B.bytes, st));
        uint32_t local = 0;
        for (uint32_t q = 0; q < pj.nj; q++) local |= (local_node(pj.r[q]) ? 1u : 0u) << q;
        if (local)
            hipLaunchKernelGGL(k_join_export, dim3(grid_for(N, 256)), dim3(256), 0, st, d, pj.r[0], pj.r[1], pj.r[2],
                               pj.nj, local, jx.p, reinterpret_cast<int64_t*>(jx.p + B.o_inc),
                               reinterpret_cast<uint32_t*>(jx.p + B.o_ord));
        RP_HIP(hipGetLastError());
        RP_HIP(hipStreamSynchronize(st));
        return true;
    }
    // rp_sim_join_import: jx now holds every responder's rows
    void join_import() {
        RP_REQUIRE(pj.active, "sim_join_import: no join exported");
        const JoinBuf B(N);
        join_finish(B.src(jx.p, N));
    }

    // {live, min checksum, max checksum, some wanted member not at its wanted status}
    void conv_local(uint32_t* out4) {
        refresh_checksums();
        if (conv_dirty) {
            std::vector<uint32_t> w;
            std::vector<uint8_t> skip(N);
            for (uint32_t a = 0; a < N; a++) {
                if (h_left[a]) w.push_back(a | ((uint32_t)ST_LEAVE << 24));
                else if (h_dead[a]) w.push_back(a | ((uint32_t)ST_FAULTY << 24));
                skip[a] = h_dead[a] | h_left[a];
            }
            nwant = (uint32_t)w.size();
            want.reserve(nwant + 1);
            cskip.reserve(N);
            if (nwant) RP_HIP(hipMemcpyAsync(want.p, w.data(), 4ull * nwant, hipMemcpyHostToDevice, st));
            RP_HIP(hipMemcpyAsync(cskip.p, skip.data(), N, hipMemcpyHostToDevice, st));
            RP_HIP(hipStreamSynchronize(st));
            conv_dirty = false;
        }
        const uint32_t init[4] = {0u, 0xFFFFFFFFu, 0u, 0u};
        RP_HIP(hipMemcpyAsync(conv.p, init, sizeof init, hipMemcpyHostToDevice, st));
        if (NL) {
            hipLaunchKernelGGL(k_conv_ck, dim3(grid_for(NL, 256, 1024)), dim3(256), 0, st, d, cskip.p, conv.p);
            if (nwant)
                hipLaunchKernelGGL(k_conv_local, dim3(grid_for((uint64_t)NL * nwant, 256, 8192)), dim3(256), 0, st, d,
                                   cskip.p, want.p, nwant, conv.p);
        }
        RP_HIP(hipGetLastError());
        RP_HIP(hipMemcpyAsync(out4, conv.p, 16, hipMemcpyDeviceToHost, st));
        RP_HIP(hipStreamSynchronize(st));
    }
};

}  // namespace rp

// ==================================================================================== C ABI

struct rp_sim {
    rp::Sim impl;
};

using rp::guard;

static rp::Sim& SM(rp_sim* s) {
    if (!s) throw rp::Error(rp::RP_EINVAL, "null sim handle");
    RP_HIP(hipSetDevice(s->impl.device));
    return s->impl;
}

static uint64_t env_u64(const char* name, uint64_t dflt) {
    const char* s = getenv(name);
    if (!s || !*s) return dflt;
    return strtoull(s, nullptr, 10);
}

static void sim_create(uint32_t n, const char* names, const uint32_t* off, const int64_t* inc0, const uint8_t* dead,
                       uint32_t seed, uint32_t suspicion_rounds, int64_t now0, int device, const uint32_t* bounds,
                       uint32_t nshards, uint32_t shard, const rp_sim_event* events, uint32_t n_events,
                       rp_sim** out) {
    RP_REQUIRE(out && n >= 2 && names && off && inc0 && dead, "sim_create: bad arguments");
    RP_REQUIRE(n_events == 0 || events, "sim_create: events missing");
    for (uint32_t i = 0; i < n_events; i++)
        RP_REQUIRE(events[i].node < n && events[i].kind <= RP_SIM_JOIN, "sim_create: bad event");
    RP_REQUIRE(n < (1u << 23), "sim_create: at most 2^23 members");
    RP_REQUIRE(nshards >= 1 && nshards <= rp::kMaxShards && shard < nshards, "sim_create: bad shard");
    std::vector<uint32_t> bnd(nshards + 1);
    if (bounds) {
        bnd.assign(bounds, bounds + nshards + 1);
    } else {
        for (uint32_t g = 0; g <= nshards; g++) bnd[g] = (uint32_t)((uint64_t)n * g / nshards);
    }
    RP_REQUIRE(bnd[0] == 0 && bnd[nshards] == n, "sim_create: shard bounds must cover [0, n)");
    for (uint32_t g = 0; g < nshards; g++) RP_REQUIRE(bnd[g] <= bnd[g + 1], "sim_create: shard bounds must be sorted");
    int nd = 0;
    RP_HIP(hipGetDeviceCount(&nd));
    RP_REQUIRE(device >= 0 && device < nd, "no such HIP device");
    RP_HIP(hipSetDevice(device));
    auto* h = new rp_sim();
    rp::Sim& S = h->impl;
    S.device = device;
    S.N = n;
    S.G = nshards;
    S.shard = shard;
    S.v0 = bnd[shard];
    S.NL = bnd[shard + 1] - bnd[shard];
    S.h_bounds = bnd;
    if (hipStreamCreateWithFlags(&S.st, hipStreamNonBlocking) != hipSuccess) {
        delete h;
        throw rp::Error(rp::RP_EDEVICE, "hipStreamCreate failed");
    }
    try {
        const uint32_t NL = S.NL, v0 = S.v0;
        for (uint32_t i = 0; i < n; i++) {
            const uint32_t id = S.nt.intern(names + off[i], off[i + 1] - off[i]);
            RP_REQUIRE(id == i, "sim_create: member addresses must be distinct");
        }
        S.nt.sort(S.st, S.ws);
        // address order on the host: the all-alive base checksum string and its piece offsets
        std::vector<uint32_t> sorted(n), rank(n);
        RP_HIP(hipMemcpyAsync(sorted.data(), S.nt.sorted.p, 4ull * n, hipMemcpyDeviceToHost, S.st));
        RP_HIP(hipStreamSynchronize(S.st));
        std::vector<uint8_t> base;
        std::vector<uint64_t> boff(n + 1ull);
        base.reserve(S.nt.h_bytes.size() + 20ull * n + 64);
        for (uint32_t k = 0; k < n; k++) {
            const uint32_t a = sorted[k];
            rank[a] = k;
            boff[k] = base.size();
            base.insert(base.end(), S.nt.h_bytes.begin() + (long)S.nt.h_noff[a],
                        S.nt.h_bytes.begin() + (long)S.nt.h_noff[a + 1]);
            const char* alive = "alive";
            base.insert(base.end(), alive, alive + 5);
            uint8_t dig[24];
            const uint32_t dl = rp::dec_len(inc0[a]);
            rp::dec_write(inc0[a], dig, dl);
            base.insert(base.end(), dig, dig + dl);
            if (k + 1 < n) base.push_back(';');
        }
        boff[n] = base.size();
        // the lane chain reads up to 24 bytes past a chunk; the LDS ring loads whole 1-KB slices
        // up to ~3 KB past the end
        base.resize(((base.size() + 64 + 1023) & ~1023ull) + 32768, 0);

        const uint64_t NN = (uint64_t)NL * n;
        // Capacities. Only the members the scenario touches ever change state in any view (a
        // node is suspected only when it stops answering; only a suspected or leaving member's
        // row moves, refutations included), so a node's changes and timers are bounded by them.
        std::vector<uint8_t> touched(dead, dead + n);
        uint32_t nrevive = 0;
        for (uint32_t i = 0; i < n_events; i++) {
            touched[events[i].node] = 1;
            nrevive += events[i].kind == RP_SIM_REVIVE;
        }
        uint32_t ndead = 0;
        for (uint32_t i = 0; i < n; i++) ndead += touched[i];
        const uint64_t cap = std::min<uint64_t>(n, env_u64("RP_SIM_CAP", 2ull * ndead + 256));
        RP_REQUIRE(cap >= 1 && cap <= 0xFFFFFFFEull, "sim_create: RP_SIM_CAP out of range");
        S.events.assign(events, events + n_events);
        std::stable_sort(S.events.begin(), S.events.end(),
                         [](const rp_sim_event& a, const rp_sim_event& b) { return a.round < b.round; });
        S.h_left.assign(n, 0);
        S.grid = std::max<uint32_t>(1, std::min<uint32_t>(NL, 256u * 4u));
        const uint32_t W = (n + 31) / 32;
        // arena: the round's responses (B and D2 answers of up to cap records, +25 % for shards
        // receiving more than their share of pings), full syncs (a handful per round, more while
        // revived nodes catch up) and slack
        const uint64_t arena =
            env_u64("RP_SIM_ARENA", (NL + NL / 4 + 256) * cap + (8ull + 2ull * nrevive) * n + 4096);
        const uint64_t L1 = NL ? NL : 1;
        S.st_.reserve(NN + 1); S.inc.reserve(NN + 1); S.order.reserve(NN + 1); S.slot.reserve(NN + 1);
        S.dev.reserve(L1 * W);
        S.chg.reserve(L1 * cap); S.tim.reserve(L1 * cap);
        S.n_chg.reserve(L1); S.n_tim.reserve(L1); S.t_head.reserve(L1); S.vfp.reserve(L1); S.vdt.reserve(L1); S.p1buf.reserve(L1);
        S.it_idx.reserve(L1); S.n_shuf.reserve(L1); S.ring_count.reserve(L1); S.max_piggy.reserve(L1);
        S.checksum.reserve(L1); S.dirty.reserve(L1); S.dead.reserve(n); S.target.reserve(L1); S.ck_snap.reserve(L1);
        S.inc_snap.reserve(L1); S.ping_n.reserve(L1); S.leg_n.reserve(L1);
        S.helpers.reserve(3 * L1); S.nhelp.reserve(L1); S.leg_nk.reserve(3 * L1);
        S.resp_idx.reserve(L1); S.lresp_idx.reserve(3 * L1);
        S.ib_off.reserve(L1 + 1);
        S.conv.reserve(4);
        S.stopped.reserve(L1);
        S.bounds.reserve(nshards + 1);
        S.pool.reserve(2 * L1 * cap + arena);
        // The message buffers up front for a stage where every local node sends a full change list
        // (C5: 5.4 GB each): growing them mid-run (a hipFree + hipMalloc of gigabytes) stalled a
        // peak round by 0.1 s. RP_SIM_MSG_BYTES caps the reservation (they still grow past it).
        {
            const uint64_t want = (uint64_t)L1 * (sizeof(rp::Msg) + sizeof(rp::Rec) * cap) + 4096;
            const uint64_t lim = env_u64("RP_SIM_MSG_BYTES", 16ull << 30);
            S.out.size_for(std::min(want, lim));
            S.in.size_for(std::min(want, lim));
        }
        S.cand.reserve((uint64_t)S.grid * n);
        // the inverse permutation that makes D1 sub-linear (RP_SIM_OPOS_BYTES = 0 turns it off:
        // every ping-req sender then scans its members array)
        const bool use_opos = NN * 4ull <= env_u64("RP_SIM_OPOS_BYTES", 64ull << 30);
        if (use_opos) S.opos.reserve(NN + 1);
        // lane checksums list each view's deviated pieces (16 B each); a view with more than dcap
        // falls back to scanning its bitmap
        uint64_t dcap = std::min<uint64_t>(n, 2ull * ndead + 256);
        const uint64_t dbudget = env_u64("RP_SIM_DLIST_BYTES", 16ull << 30);
        if (L1 * dcap * 16 > dbudget) dcap = std::max<uint64_t>(1, dbudget / (16 * L1));
        S.dlist.reserve(L1 * dcap);
        // per-block string buffer: names + ';' + "suspect" + 20 digits per member (also the
        // iterator's scratch)
        const uint64_t strcap = std::max<uint64_t>(S.nt.h_bytes.size() + 29ull * n + 64, 5ull * n + 64);
        S.strbuf.reserve((uint64_t)S.grid * ((strcap + 255) & ~255ull));
        S.stats.reserve(8); S.cursor.reserve(1 + 4); S.err.reserve(1);
        S.base_len = boff[n];
        S.inc0.reserve(n); S.rank.reserve(n); S.boff.reserve(n + 1ull); S.sbase.reserve(base.size());
        RP_HIP(hipMemcpyAsync(S.inc0.p, inc0, 8ull * n, hipMemcpyHostToDevice, S.st));
        RP_HIP(hipMemcpyAsync(S.rank.p, rank.data(), 4ull * n, hipMemcpyHostToDevice, S.st));
        RP_HIP(hipMemcpyAsync(S.boff.p, boff.data(), 8ull * (n + 1), hipMemcpyHostToDevice, S.st));
        RP_HIP(hipMemcpyAsync(S.sbase.p, base.data(), base.size(), hipMemcpyHostToDevice, S.st));
        RP_HIP(hipMemcpyAsync(S.bounds.p, bnd.data(), 4ull * (nshards + 1), hipMemcpyHostToDevice, S.st));
        S.h_dead.assign(dead, dead + n);
        RP_HIP(hipMemcpyAsync(S.dead.p, S.h_dead.data(), n, hipMemcpyHostToDevice, S.st));
        RP_HIP(hipMemsetAsync(S.stats.p, 0, 8 * sizeof(unsigned long long), S.st));
        RP_HIP(hipMemsetAsync(S.err.p, 0, 4, S.st));
        RP_HIP(hipMemsetAsync(S.cursor.p, 0, 8, S.st));
        rp::SimDev& d = S.d;
        d.N = n; d.W = W; d.v0 = v0; d.NL = NL; d.G = nshards; d.bounds = S.bounds.p;
        d.seed = seed; d.susp = suspicion_rounds; d.now0 = now0;
        d.Cd = (uint32_t)cap; d.Ct = (uint32_t)cap; d.Cm = (uint32_t)cap;
        d.st = S.st_.p; d.inc = S.inc.p; d.order = S.order.p; d.slot = S.slot.p; d.dev = S.dev.p;
        d.opos = use_opos ? S.opos.p : nullptr;
        d.xcap = (uint32_t)std::max<uint64_t>(2, std::min<uint64_t>(rp::kXCap, env_u64("RP_SIM_D1_XCAP", rp::kXCap)));
        d.chg = S.chg.p; d.n_chg = S.n_chg.p; d.tim = S.tim.p; d.n_tim = S.n_tim.p; d.t_head = S.t_head.p; d.vfp = S.vfp.p; d.vdt = S.vdt.p; d.p1 = S.p1buf.p; d.p1_pre = 0;
        d.it_idx = S.it_idx.p; d.n_shuf = S.n_shuf.p; d.ring_count = S.ring_count.p; d.max_piggy = S.max_piggy.p;
        d.checksum = S.checksum.p; d.dirty = S.dirty.p; d.dead = S.dead.p; d.stopped = S.stopped.p;
        d.sorted = S.nt.sorted.p; d.rank = S.rank.p; d.names = S.nt.d_bytes.p; d.noff = S.nt.d_noff.p;
        d.sbase = S.sbase.p; d.boff = S.boff.p; d.inc0 = S.inc0.p;
        d.target = S.target.p; d.ck_snap = S.ck_snap.p; d.inc_snap = S.inc_snap.p;
        d.pool = S.pool.p; d.arena0 = 2ull * L1 * cap; d.arena_cap = arena; d.cursor = S.cursor.p; d.work = reinterpret_cast<uint32_t*>(S.cursor.p + 1);
        d.ping_n = S.ping_n.p; d.leg_n = S.leg_n.p; d.helpers = S.helpers.p; d.nhelp = S.nhelp.p;
        d.leg_nk = S.leg_nk.p; d.cand = S.cand.p;
        d.strbuf = S.strbuf.p; d.strcap = (strcap + 255) & ~255ull;
        d.dlist = S.dlist.p; d.dcap = (uint32_t)dcap;
        d.resp_idx = S.resp_idx.p; d.lresp_idx = S.lresp_idx.p;
        d.stats = S.stats.p; d.err = S.err.p; d.round = 0;
        {
            const void* ptrs[] = {d.st, d.inc, d.order, d.slot, d.dev, d.chg, d.n_chg, d.tim, d.n_tim, d.t_head, d.vfp, d.it_idx,
                                  d.n_shuf, d.ring_count, d.max_piggy, d.checksum, d.dirty, d.dead, d.sorted,
                                  d.rank, d.names, d.noff, d.sbase, d.boff, d.inc0, d.target, d.ck_snap,
                                  d.inc_snap, d.pool, d.cursor, d.ping_n, d.leg_n, d.helpers, d.nhelp, d.leg_nk,
                                  d.cand, d.strbuf, d.resp_idx, d.lresp_idx, d.stats, d.err, d.bounds, d.stopped};
            for (const void* p : ptrs) RP_REQUIRE(p != nullptr, "sim_create: internal buffer not allocated");
        }
        hipLaunchKernelGGL(rp::k_sim_init, dim3(rp::grid_for(NN + 1, 256, 8192)), dim3(256), 0, S.st, d);
        if (NL) {
            hipLaunchKernelGGL(rp::k_sim_start, dim3(rp::grid_for(NL, 64)), dim3(64), 0, S.st, d);
            if (d.opos)
                hipLaunchKernelGGL(rp::k_opos_build, dim3(std::min<uint32_t>(NL, 4096)), dim3(256), 0, S.st, d);
            hipLaunchKernelGGL(rp::k_sim_first_checksum, dim3(1), dim3(64), 0, S.st, d);
            hipLaunchKernelGGL(rp::k_sim_bcast_checksum, dim3(rp::grid_for(NL, 256)), dim3(256), 0, S.st, d);
        }
        RP_HIP(hipGetLastError());
        RP_HIP(hipStreamSynchronize(S.st));
    } catch (...) {
        (void)hipStreamSynchronize(S.st);
        (void)hipStreamDestroy(S.st);
        delete h;
        throw;
    }
    *out = h;
}

extern "C" {

int rp_sim_create(uint32_t n, const char* names, const uint32_t* off, const int64_t* inc0, const uint8_t* dead,
                  uint32_t seed, uint32_t suspicion_rounds, int64_t now0, int device, rp_sim** out) {
    return guard([&] {
        sim_create(n, names, off, inc0, dead, seed, suspicion_rounds, now0, device, nullptr, 1, 0, nullptr, 0, out);
    });
}

int rp_sim_create_shard(uint32_t n, const char* names, const uint32_t* off, const int64_t* inc0, const uint8_t* dead,
                        uint32_t seed, uint32_t suspicion_rounds, int64_t now0, int device, const uint32_t* bounds,
                        uint32_t nshards, uint32_t shard, rp_sim** out) {
    return guard([&] {
        sim_create(n, names, off, inc0, dead, seed, suspicion_rounds, now0, device, bounds, nshards, shard, nullptr, 0,
                   out);
    });
}

int rp_sim_create_scenario(uint32_t n, const char* names, const uint32_t* off, const int64_t* inc0, const uint8_t* dead,
                           uint32_t seed, uint32_t suspicion_rounds, int64_t now0, int device, const uint32_t* bounds,
                           uint32_t nshards, uint32_t shard, const rp_sim_event* events, uint32_t n_events,
                           rp_sim** out) {
    return guard([&] {
        sim_create(n, names, off, inc0, dead, seed, suspicion_rounds, now0, device, bounds, nshards, shard, events,
                   n_events, out);
    });
}

int rp_sim_counters(rp_sim* s, uint64_t* out8) {
    return guard([&] {
        rp::Sim& S = SM(s);
        unsigned long long v[8];
        RP_HIP(hipMemcpyAsync(v, S.stats.p, sizeof v, hipMemcpyDeviceToHost, S.st));
        RP_HIP(hipStreamSynchronize(S.st));
        for (int i = 0; i < 4; i++) out8[i] = v[i];
        out8[4] = S.sent_msgs;
        out8[5] = S.sent_recs;
        out8[6] = v[4];
        out8[7] = S.base_len;
    });
}

int rp_sim_piggyback(rp_sim* s, uint32_t* out) {
    return guard([&] {
        rp::Sim& S = SM(s);
        if (S.NL) RP_HIP(hipMemcpyAsync(out, S.max_piggy.p, 4ull * S.NL, hipMemcpyDeviceToHost, S.st));
        RP_HIP(hipStreamSynchronize(S.st));
    });
}

int rp_sim_destroy(rp_sim* s) {
    return guard([&] {
        if (!s) return;
        (void)hipSetDevice(s->impl.device);
        if (s->impl.st) {
            (void)hipStreamSynchronize(s->impl.st);
            (void)hipStreamDestroy(s->impl.st);
        }
        if (s->impl.st2) {
            (void)hipStreamSynchronize(s->impl.st2);
            (void)hipStreamDestroy(s->impl.st2);
            (void)hipEventDestroy(s->impl.ev_c);
            (void)hipEventDestroy(s->impl.ev_early);
        }
        if (s->impl.ev_ext) (void)hipEventDestroy(s->impl.ev_ext);
        if (s->impl.ev_ord) (void)hipEventDestroy(s->impl.ev_ord);
        if (s->impl.h_pin) {
            (void)hipHostFree(s->impl.h_pin);
            (void)hipEventDestroy(s->impl.ev_cnt);
        }
        delete s;
    });
}

int rp_sim_shard_info(rp_sim* s, uint32_t* v0, uint32_t* nl, uint32_t* nshards, uint32_t* shard) {
    return guard([&] {
        rp::Sim& S = SM(s);
        if (v0) *v0 = S.v0;
        if (nl) *nl = S.NL;
        if (nshards) *nshards = S.G;
        if (shard) *shard = S.shard;
    });
}

int rp_sim_step(rp_sim* s, uint32_t rounds) {
    return guard([&] {
        rp::Sim& S = SM(s);
        for (uint32_t r = 0; r < rounds; r++) S.step();
        S.check_err();
    });
}

int rp_sim_step_async(rp_sim* s, uint32_t rounds) {
    return guard([&] {
        rp::Sim& S = SM(s);
        for (uint32_t r = 0; r < rounds; r++) S.step();
    });
}

int rp_sim_sync(rp_sim* s) {
    return guard([&] { SM(s).check_err(); });
}

int rp_sim_stage(rp_sim* s, int stage) {
    return guard([&] {
        rp::Sim& S = SM(s);
        RP_REQUIRE(stage >= 0 && stage <= 4, "sim_stage: stage must be 0..4");
        S.stage(stage);
        if (stage == 4) S.check_err();
    });
}

int rp_sim_outbox(rp_sim* s, uint64_t* nmsg, uint64_t* nrec, void** buf) {
    return guard([&] {
        rp::Sim& S = SM(s);
        for (uint32_t g = 0; g < S.G; g++) {
            if (nmsg) nmsg[g] = S.out.nmsg.empty() ? 0 : S.out.nmsg[g];
            if (nrec) nrec[g] = S.out.nrec.empty() ? 0 : S.out.nrec[g];
        }
        if (buf) *buf = S.out.buf.p;
    });
}

int rp_sim_inbox(rp_sim* s, const uint64_t* nmsg, const uint64_t* nrec, void** buf) {
    return guard([&] {
        rp::Sim& S = SM(s);
        RP_REQUIRE(nmsg && nrec, "sim_inbox: counts required");
        S.prepare_in(nmsg, nrec);
        if (buf) *buf = S.in.buf.p;
    });
}

int rp_sim_order_stream(rp_sim* s, void* stream) {
    return guard([&] {
        rp::Sim& S = SM(s);
        if (!stream) {
            RP_HIP(hipStreamSynchronize(S.st));
            return;
        }
        if (!S.ev_ord) RP_HIP(hipEventCreateWithFlags(&S.ev_ord, hipEventDisableTiming));
        RP_HIP(hipEventRecord(S.ev_ord, S.st));
        RP_HIP(hipStreamWaitEvent((hipStream_t)stream, S.ev_ord, 0));
    });
}

int rp_sim_wait_stream(rp_sim* s, void* stream) {
    return guard([&] {
        rp::Sim& S = SM(s);
        if (!S.ev_ext) RP_HIP(hipEventCreateWithFlags(&S.ev_ext, hipEventDisableTiming));
        RP_HIP(hipEventRecord(S.ev_ext, (hipStream_t)stream));
        RP_HIP(hipStreamWaitEvent(S.st, S.ev_ext, 0));
    });
}

int rp_sim_exchange_local(rp_sim* const* shards, uint32_t nshards) {
    return guard([&] {
        RP_REQUIRE(shards && nshards >= 1, "sim_exchange_local: bad arguments");
        for (uint32_t i = 0; i < nshards; i++) {
            RP_REQUIRE(shards[i] && shards[i]->impl.G == nshards && shards[i]->impl.shard == i,
                       "sim_exchange_local: handles must be shards 0..G-1 of one partition");
            RP_HIP(hipSetDevice(shards[i]->impl.device));
            RP_HIP(hipStreamSynchronize(shards[i]->impl.st));
        }
        for (uint32_t dst = 0; dst < nshards; dst++) {
            rp::Sim& D = shards[dst]->impl;
            std::vector<uint64_t> nm(nshards), nr(nshards);
            for (uint32_t src = 0; src < nshards; src++) {
                nm[src] = shards[src]->impl.out.nmsg[dst];
                nr[src] = shards[src]->impl.out.nrec[dst];
            }
            D.prepare_in(nm.data(), nr.data());
            for (uint32_t src = 0; src < nshards; src++) {
                rp::Sim& Sx = shards[src]->impl;
                const uint64_t b = Sx.out.seg_bytes(dst);
                if (b)
                    RP_HIP(hipMemcpyAsync(D.in.buf.p + D.in.seg_off(src), Sx.out.buf.p + Sx.out.seg_off(dst), b,
                                          hipMemcpyDeviceToDevice, D.st));
            }
        }
        for (uint32_t i = 0; i < nshards; i++) RP_HIP(hipStreamSynchronize(shards[i]->impl.st));
    });
}

int rp_sim_join_export(rp_sim* s, int* has, void** buf, uint64_t* bytes) {
    return guard([&] {
        rp::Sim& S = SM(s);
        const bool h = S.join_export();
        if (has) *has = h ? 1 : 0;
        if (buf) *buf = h ? S.jx.p : nullptr;
        if (bytes) *bytes = h ? rp::JoinBuf(S.N).bytes : 0;
    });
}

int rp_sim_join_import(rp_sim* s) {
    return guard([&] { SM(s).join_import(); });
}

int rp_sim_join_exchange_local(rp_sim* const* shards, uint32_t nshards) {
    return guard([&] {
        RP_REQUIRE(shards && nshards >= 1, "sim_join_exchange_local: bad arguments");
        for (uint32_t i = 0; i < nshards; i++) {
            RP_REQUIRE(shards[i] && shards[i]->impl.G == nshards && shards[i]->impl.shard == i,
                       "sim_join_exchange_local: handles must be shards 0..G-1 of one partition");
            RP_REQUIRE(shards[i]->impl.pj.active, "sim_join_exchange_local: every shard must have exported the join");
            RP_HIP(hipSetDevice(shards[i]->impl.device));
            RP_HIP(hipStreamSynchronize(shards[i]->impl.st));
        }
        const rp::Sim& S0 = shards[0]->impl;
        const rp::JoinBuf B(S0.N);
        const uint64_t N = S0.N;
        for (uint32_t q = 0; q < S0.pj.nj; q++) {
            uint32_t o = 0;  // the shard owning responder q wrote its rows
            while (o < nshards && !shards[o]->impl.local_node(S0.pj.r[q])) o++;
            RP_REQUIRE(o < nshards, "sim_join_exchange_local: a responder belongs to no shard");
            const uint8_t* src = shards[o]->impl.jx.p;
            for (uint32_t g = 0; g < nshards; g++) {
                if (g == o) continue;
                rp::Sim& D = shards[g]->impl;
                RP_HIP(hipMemcpyAsync(D.jx.p + q * N, src + q * N, N, hipMemcpyDefault, D.st));
                RP_HIP(hipMemcpyAsync(D.jx.p + B.o_inc + 8 * q * N, src + B.o_inc + 8 * q * N, 8 * N, hipMemcpyDefault,
                                      D.st));
                if (q == 0) RP_HIP(hipMemcpyAsync(D.jx.p + B.o_ord, src + B.o_ord, 4 * N, hipMemcpyDefault, D.st));
            }
        }
        for (uint32_t i = 0; i < nshards; i++) RP_HIP(hipStreamSynchronize(shards[i]->impl.st));
    });
}

int rp_sim_round(rp_sim* s, int64_t* out) {
    return guard([&] { *out = SM(s).round; });
}

int rp_sim_checksums(rp_sim* s, uint32_t* out) {
    return guard([&] {
        rp::Sim& S = SM(s);
        S.refresh_checksums();
        if (S.NL) RP_HIP(hipMemcpyAsync(out, S.checksum.p, 4ull * S.NL, hipMemcpyDeviceToHost, S.st));
        RP_HIP(hipStreamSynchronize(S.st));
        for (uint32_t lv = 0; lv < S.NL; lv++)
            if (S.h_dead[S.v0 + lv]) out[lv] = 0;
    });
}

int rp_sim_view(rp_sim* s, uint32_t v, uint8_t* status, int64_t* inc) {
    return guard([&] {
        rp::Sim& S = SM(s);
        RP_REQUIRE(v >= S.v0 && v < S.v0 + S.NL, "sim_view: node not in this shard");
        const uint64_t row = (uint64_t)(v - S.v0) * S.N;
        if (status) {
            RP_HIP(hipMemcpyAsync(status, S.st_.p + row, S.N, hipMemcpyDeviceToHost, S.st));
        }
        if (inc) RP_HIP(hipMemcpyAsync(inc, S.inc.p + row, 8ull * S.N, hipMemcpyDeviceToHost, S.st));
        RP_HIP(hipStreamSynchronize(S.st));
        if (status)
            for (uint32_t a = 0; a < S.N; a++) status[a] &= rp::ST_MASK;
    });
}

int rp_sim_converged_local(rp_sim* s, uint32_t* out4) {
    return guard([&] { SM(s).conv_local(out4); });
}

int rp_sim_converged(rp_sim* s, int* out) {
    return guard([&] {
        rp::Sim& S = SM(s);
        RP_REQUIRE(S.G == 1, "sim_converged: a sharded handle reduces rp_sim_converged_local over its shards");
        uint32_t c[4];
        S.conv_local(c);
        *out = (c[0] == 0 || (c[1] == c[2] && c[3] == 0)) ? 1 : 0;
    });
}

int rp_sim_stats(rp_sim* s, uint64_t* out4) {
    return guard([&] {
        rp::Sim& S = SM(s);
        unsigned long long v[4];
        RP_HIP(hipMemcpyAsync(v, S.stats.p, sizeof v, hipMemcpyDeviceToHost, S.st));
        RP_HIP(hipStreamSynchronize(S.st));
        for (int i = 0; i < 4; i++) out4[i] = v[i];
    });
}

}  // extern "C"
