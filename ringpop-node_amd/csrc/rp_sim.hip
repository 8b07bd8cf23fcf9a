// rp_sim.hip — the gossip protocol of N full ringpop nodes as a batched round simulator.
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
// HBM layout (sized for 10^5 members on one MI355X):
//   dense rows [v][a]   status u8 (bit 7: in this node's ring) | incarnation i64 | members-array
//                       order u32 | dissemination slot u16  (15 B per (node, member))
//   per node            deviation bitmap over address ranks (which rows ever changed), sparse
//                       change list (dissemination's `changes` map: address, piggyback count,
//                       source, source incarnation; the status/incarnation of a change always
//                       equal the view row's), sparse timer list (address, due round, captured
//                       incarnation); capacities checked, overflow is a loud error
//   messages            fixed per-sender slots (ping, response, ping-req legs) + a per-round
//                       arena (ping-req responses, full syncs, staging)
// Checksums: the membership checksum string of a view is the all-alive base string (address
// order, built once) with the deviated rows' pieces substituted. Nodes whose views changed are
// re-checksummed in batch with ONE NODE PER LANE (64 independent farmhash chains per wave,
// reading the shared base string plus the node's few deviated rows), or, when a reader needs
// one node's checksum in the middle of a phase, by one workgroup (one chain lane fed by
// pre-mixing lanes).
#include <algorithm>
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
constexpr int kHashWin = 512;      // LDS window of pre-mixed chunks for the block checksum chain
constexpr uint8_t ST_MASK = 3, IN_RING = 0x80;
// error flags (rp_sim_step reports them)
constexpr uint32_t ERR_CHANGES = 1, ERR_TIMERS = 2, ERR_ARENA = 4;

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

struct Change {  // an entry of dissemination's changes map
    uint32_t addr;
    uint32_t cnt;  // piggybackCount
    uint32_t src;
    uint32_t pad;
    int64_t srcinc;
};

struct Timer {  // a suspicion timer (suspicion.js:55-84)
    uint32_t addr;
    int32_t due;  // round at whose end it fires
    int64_t inc;  // incarnation captured at start (== the row's while the episode lasts)
};

struct SimDev {
    uint32_t N, W;  // members, bitmap words per node
    uint32_t seed, susp, Cd, Ct, Cm;
    int64_t now0;
    int64_t round;
    // dense rows [v][N]
    uint8_t* st;
    int64_t* inc;
    uint32_t* order;
    uint16_t* slot;  // 0 = no change, else index + 1 into the node's change list
    uint32_t* dev;   // [v][W] rows ever changed, by address rank
    // sparse per node
    Change* chg;  // [v][Cd]
    uint32_t* n_chg;
    Timer* tim;  // [v][Ct]
    uint32_t* n_tim;
    // per node
    int64_t* it_idx;
    uint32_t *n_shuf, *ring_count, *max_piggy, *checksum;
    uint8_t* dirty;
    const uint8_t* dead;
    // names in address order; base checksum string
    const uint32_t* sorted;
    const uint32_t* rank;
    const uint8_t* names;
    const uint64_t* noff;
    const uint8_t* sbase;
    const uint64_t* boff;  // [N+1], boff[N] = base length
    const int64_t* inc0;
    // round scratch and messages
    int32_t* target;
    uint32_t* ck_snap;
    int64_t* inc_snap;
    Rec* pool;  // [3][N][Cm] fixed slots (ping, response, leg) + arena
    uint64_t arena0, arena_cap;
    unsigned long long* cursor;  // arena bump pointer (reset every round)
    uint64_t *resp_off, *lresp_off;
    uint32_t *ping_n, *resp_n, *leg_n;
    uint32_t* helpers;  // [N*3]
    uint32_t* nhelp;    // [N]
    uint32_t* lresp_n;  // [N*3]  (NONE = network error)
    uint32_t* cand;     // [grid*N] scratch for ping-req candidate lists
    uint8_t* strbuf;    // [grid * strcap]
    uint64_t strcap;
    // CSR inboxes
    const uint32_t* in_off;  // receivers: [N+1]
    const uint32_t* in_src;  // senders sorted by (target, sender)
    const uint32_t* h_off;   // helpers: [N+1]
    const uint32_t* h_src;   // (sender*3 + leg) sorted by (helper, sender, leg)
    // stats: pings, pingreqs, fullsyncs, applied
    unsigned long long* stats;
    uint32_t* err;
};

__device__ __forceinline__ Rec* ping_slot(const SimDev& S, uint32_t v) { return S.pool + (uint64_t)v * S.Cm; }
__device__ __forceinline__ Rec* resp_slot(const SimDev& S, uint32_t v) {
    return S.pool + ((uint64_t)S.N + v) * S.Cm;
}
__device__ __forceinline__ Rec* leg_slot(const SimDev& S, uint32_t v) {
    return S.pool + (2ull * S.N + v) * S.Cm;
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

// thread 0 allocates n records from the round arena; broadcast to the block (NONE-offset on
// overflow, with the error flag set)
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
    uint32_t win[2][kHashWin][8];
};

// ---- checksums

// Membership.computeChecksum (index.js:48-75) of node v by one workgroup: the string is
// written to buf in address order, then hashed (one chain lane, 192 pre-mixing lanes).
__device__ void block_checksum(const SimDev& S, uint32_t v, uint8_t* buf, Lds& L) {
    const uint32_t N = S.N;
    const uint64_t row = (uint64_t)v * N;
    const int tid = threadIdx.x;
    // contiguous member range per thread keeps address order inside each thread's piece
    const uint32_t per = (N + kT - 1) / kT;
    const uint32_t b0 = min(N, per * tid), b1 = min(N, b0 + per);
    uint32_t mine = 0;
    for (uint32_t k = b0; k < b1; k++) {
        const uint32_t a = S.sorted[k];
        mine += (uint32_t)(S.noff[a + 1] - S.noff[a]) + status_len(S.st[row + a] & ST_MASK) + dec_len(S.inc[row + a]) +
                1u;
    }
    uint32_t total;
    uint32_t o = block_scan(mine, L.u, &total);
    for (uint32_t k = b0; k < b1; k++) {
        const uint32_t a = S.sorted[k];
        const uint64_t nb = S.noff[a];
        const uint32_t nl = (uint32_t)(S.noff[a + 1] - nb);
        for (uint32_t q = 0; q < nl; q++) buf[o++] = S.names[nb + q];
        const uint8_t st = S.st[row + a] & ST_MASK;
        const uint32_t sl = status_len(st);
        for (uint32_t q = 0; q < sl; q++) buf[o++] = status_char(st, q);
        const int64_t in = S.inc[row + a];
        const uint32_t dl = dec_len(in);
        dec_write(in, buf + o, dl);
        o += dl;
        buf[o++] = ';';
    }
    __threadfence_block();
    __syncthreads();
    const uint64_t len = total ? total - 1 : 0;
    uint32_t h = 0;
    if (len <= 24) {
        if (tid == 0) h = fh::hash32(fh::PtrSrc{buf}, (uint32_t)len);
    } else {
        const uint64_t iters = (len - 1) / 20;
        uint32_t g = 0, f = 0;
        if (tid == 0) {
            const uint32_t L = (uint32_t)len;
            h = L;
            g = fh::kC1 * L;
            f = g;
            const uint32_t a0 = premix(ld32(buf, len - 4)), a1 = premix(ld32(buf, len - 8)),
                           a2 = premix(ld32(buf, len - 16)), a3 = premix(ld32(buf, len - 12)),
                           a4 = premix(ld32(buf, len - 20));
            h ^= a0;
            h = fh::rotr(h, 19) * 5 + 0xe6546b64u;
            h ^= a2;
            h = fh::rotr(h, 19) * 5 + 0xe6546b64u;
            g ^= a1;
            g = fh::rotr(g, 19) * 5 + 0xe6546b64u;
            g ^= a3;
            g = fh::rotr(g, 19) * 5 + 0xe6546b64u;
            f += a4;
            f = fh::rotr(f, 19) + 113;
        }
        auto fill = [&](int wb, uint64_t c0, int t0, int nt) {
            for (int j = t0; j < kHashWin; j += nt) {
                const uint64_t c = c0 + j;
                if (c >= iters) break;
                const uint64_t off = c * 20;
                const uint32_t a = ld32(buf, off), b = ld32(buf, off + 4), cc = ld32(buf, off + 8),
                               d = ld32(buf, off + 12), e = ld32(buf, off + 16);
                uint32_t* r = L.win[wb][j];
                r[0] = a; r[1] = b; r[2] = cc; r[3] = d;
                r[4] = e; r[5] = premix(d); r[6] = premix(cc); r[7] = premix(b + e * fh::kC1);
            }
        };
        fill(0, 0, tid, kT);
        __syncthreads();
        const uint64_t nwin = (iters + kHashWin - 1) / kHashWin;
        for (uint64_t w = 0; w < nwin; w++) {
            const int cur = (int)(w & 1);
            if (tid >= 64) {
                if (w + 1 < nwin) fill(cur ^ 1, (w + 1) * kHashWin, tid - 64, kT - 64);
            } else if (tid == 0) {
                const uint64_t c0 = w * kHashWin;
                const int n = (int)((iters - c0) < (uint64_t)kHashWin ? (iters - c0) : kHashWin);
                for (int j = 0; j < n; j++) {
                    const uint32_t* r = L.win[cur][j];
                    const uint32_t a = r[0], b = r[1], c = r[2], d = r[3], e = r[4];
                    h += a;
                    g += b;
                    f += c;
                    h = fh::rotr(h ^ r[5], 19) * 5 + 0xe6546b64u + e;
                    g = fh::rotr(g ^ r[6], 19) * 5 + 0xe6546b64u + a;
                    f = fh::rotr(f ^ r[7], 19) * 5 + 0xe6546b64u + d;
                    f += g;
                    g += f;
                }
            }
            __syncthreads();
        }
        if (tid == 0) {
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
        S.checksum[v] = h;
        S.dirty[v] = 0;
    }
    __syncthreads();
}

__device__ __forceinline__ void checksum_if_dirty(const SimDev& S, uint32_t v, Lds& L) {
    __syncthreads();
    if (S.dirty[v]) block_checksum(S, v, S.strbuf + (uint64_t)blockIdx.x * S.strcap, L);
}

// One node's checksum string, seen by one lane: the base string with the deviated rows'
// pieces substituted. Piece k (address rank k) of the view is name + status + incarnation
// (+ ';' unless last); clean pieces equal the base string's.
struct LaneView {
    const SimDev& S;
    const uint8_t* strow;
    const int64_t* incrow;
    const uint32_t* dev;

    __device__ uint32_t blen(uint32_t k) const { return (uint32_t)(S.boff[k + 1] - S.boff[k]); }
    __device__ uint32_t plen(uint32_t k) const {
        const uint32_t a = S.sorted[k];
        return (uint32_t)(S.noff[a + 1] - S.noff[a]) + status_len(strow[a] & ST_MASK) + dec_len(incrow[a]) +
               (k + 1 < S.N ? 1u : 0u);
    }
    __device__ uint8_t piece_byte(uint32_t k, uint32_t j) const {
        const uint32_t a = S.sorted[k];
        const uint64_t nb = S.noff[a];
        const uint32_t nl = (uint32_t)(S.noff[a + 1] - nb);
        if (j < nl) return S.names[nb + j];
        j -= nl;
        const uint8_t s = strow[a] & ST_MASK;
        const uint32_t sl = status_len(s);
        if (j < sl) return status_char(s, j);
        j -= sl;
        const int64_t x = incrow[a];
        if (x == S.inc0[a]) {  // the base piece holds these digits after "alive"
            const uint64_t p = S.boff[k] + nl + 5u;
            const uint32_t dl = blen(k) - nl - 5u - (k + 1 < S.N ? 1u : 0u);
            return j < dl ? S.sbase[p + j] : (uint8_t)';';
        }
        const uint32_t dl = dec_len(x);
        if (j >= dl) return (uint8_t)';';
        uint8_t tmp[24];
        dec_write(x, tmp, dl);
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

// Forward byte cursor over a lane's string (positions queried in non-decreasing order).
struct Fwd {
    uint32_t nd;    // next (or current) deviated rank
    uint64_t pos;   // its start in the lane string
    uint32_t pl;    // its length in the lane string
    int64_t delta;  // lane position - base position for clean bytes before `pos`

    __device__ void init(const LaneView& V) {
        delta = 0;
        nd = V.next_dev(0);
        if (nd < V.S.N) {
            pos = V.S.boff[nd];
            pl = V.plen(nd);
        } else {
            pos = ~0ull >> 1;
            pl = 0;
        }
    }
    __device__ void skip_to(const LaneView& V, uint64_t q) {
        while (nd < V.S.N && q >= pos + pl) {
            delta += (int64_t)pl - (int64_t)V.blen(nd);
            nd = V.next_dev(nd + 1);
            if (nd < V.S.N) {
                pos = (uint64_t)((int64_t)V.S.boff[nd] + delta);
                pl = V.plen(nd);
            } else {
                pos = ~0ull >> 1;
                pl = 0;
            }
        }
    }
    __device__ uint8_t byte(const LaneView& V, uint64_t q) {
        skip_to(V, q);
        if (q < pos) return V.S.sbase[(uint64_t)((int64_t)q - delta)];
        return V.piece_byte(nd, (uint32_t)(q - pos));
    }
};

__device__ __forceinline__ uint32_t ldw(const uint8_t* p) { return *reinterpret_cast<const uint32_t*>(p); }

// Membership checksum of node v computed by this lane alone.
__device__ uint32_t lane_checksum(const SimDev& S, uint32_t v) {
    const uint32_t N = S.N;
    const uint64_t row = (uint64_t)v * N;
    const LaneView V{S, S.st + row, S.inc + row, S.dev + (uint64_t)v * S.W};
    // pass 1: length (base length + the deviated pieces' differences) and the last deviation
    int64_t dtot = 0;
    uint32_t last = NONE;
    for (uint32_t w = 0; w < S.W; w++) {
        uint32_t bits = V.dev[w];
        while (bits) {
            const uint32_t k = (w << 5) + __builtin_ctz(bits);
            bits &= bits - 1;
            dtot += (int64_t)V.plen(k) - (int64_t)V.blen(k);
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
        uint64_t E = 0, B = 0;
        if (kd != NONE) {
            E = (uint64_t)((int64_t)S.boff[kd + 1] + da);
            B = E - V.plen(kd);
        }
        for (int i = 19; i >= 0; i--) {
            const uint64_t q = len - 20 + (uint64_t)i;
            while (kd != NONE && q < B) {
                da -= (int64_t)V.plen(kd) - (int64_t)V.blen(kd);
                kd = V.prev_dev(kd);
                if (kd != NONE) {
                    E = (uint64_t)((int64_t)S.boff[kd + 1] + da);
                    B = E - V.plen(kd);
                }
            }
            tail[i] = (kd != NONE && q >= B && q < E) ? V.piece_byte(kd, (uint32_t)(q - B))
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
        uint32_t a, b, cc, d, e;
        if (q0 + 20 <= F.pos) {  // clean: 20 bytes of the base string at a lane-specific shift
            const uint64_t o = (uint64_t)((int64_t)q0 - F.delta);
            const uint8_t* p = S.sbase + (o & ~3ull);
            const uint32_t sh = (uint32_t)(o & 3);
            const uint32_t w0 = ldw(p), w1 = ldw(p + 4), w2 = ldw(p + 8), w3 = ldw(p + 12), w4 = ldw(p + 16),
                           w5 = ldw(p + 20);
            a = __builtin_amdgcn_alignbyte(w1, w0, sh);
            b = __builtin_amdgcn_alignbyte(w2, w1, sh);
            cc = __builtin_amdgcn_alignbyte(w3, w2, sh);
            d = __builtin_amdgcn_alignbyte(w4, w3, sh);
            e = __builtin_amdgcn_alignbyte(w5, w4, sh);
        } else {
            uint32_t wd[5];
            for (int i = 0; i < 5; i++) {
                uint32_t x = 0;
                for (int j = 0; j < 4; j++) x |= (uint32_t)F.byte(V, q0 + 4 * i + j) << (8 * j);
                wd[i] = x;
            }
            a = wd[0]; b = wd[1]; cc = wd[2]; d = wd[3]; e = wd[4];
        }
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

// every live node whose view changed: one node per lane
__global__ __launch_bounds__(256) void k_ck_lanes(SimDev S) {
    const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= S.N || S.dead[v] || !S.dirty[v]) return;
    S.checksum[v] = lane_checksum(S, v);
    S.dirty[v] = 0;
}

// ---- membership / dissemination / suspicion on one node

// Membership.update(records) on node v + the 'updated' listeners (on_membership_event.js:86-134):
// view row, recordChange (dissemination.js:56-72), suspicion start (a suspect update about
// another member), ring add/remove -> maxPiggybackCount. Records carry distinct addresses (one
// message), so lanes apply them independently. Returns the number applied (block-uniform).
__device__ uint32_t block_apply(const SimDev& S, uint32_t v, const Rec* recs, uint32_t n, Lds& L, int64_t now) {
    const uint64_t row = (uint64_t)v * S.N;
    uint32_t napp = 0, nadd = 0, nrem = 0;
    Change* chg = S.chg + (uint64_t)v * S.Cd;
    Timer* tim = S.tim + (uint64_t)v * S.Ct;
    __syncthreads();
    uint32_t nc = S.n_chg[v], nt = S.n_tim[v];
    for (uint32_t base = 0; base < n; base += kT) {
        const uint32_t i = base + threadIdx.x;
        bool applied = false, need_timer = false, need_new = false;
        uint32_t a = 0, slot = 0;
        uint8_t us = 0;
        int64_t ui = 0;
        Rec r{};
        if (i < n) {
            r = recs[i];
            a = rec_addr(r);
            us = rec_st(r);
            ui = r.inc;
            const uint8_t cur = S.st[row + a];
            if (evaluate_update(cur & ST_MASK, S.inc[row + a], a == v, us, ui, now)) {
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
                atomicOr(&S.dev[(uint64_t)v * S.W + (k >> 5)], 1u << (k & 31));
                need_timer = us == ST_SUSPECT && a != v;
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
            if (!need_new) {
                Change& c = chg[slot - 1];
                c.cnt = 0;
                c.src = r.src;
                c.srcinc = r.srcinc;
            } else {
                const uint32_t idx = nc + cpos;
                if (idx < S.Cd) {
                    chg[idx] = Change{a, 0u, r.src, 0u, r.srcinc};
                    S.slot[row + a] = (uint16_t)(idx + 1);
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
    if (threadIdx.x == 0) {
        S.n_chg[v] = nc;
        S.n_tim[v] = nt;
        if (tot) {
            S.dirty[v] = 1;
            atomicAdd(&S.stats[3], (unsigned long long)tot);
            if (adds || rems) {  // ringChanged -> adjustMaxPiggybackCount (dissemination.js:38-55)
                const uint32_t rc = S.ring_count[v] + adds - rems;
                S.ring_count[v] = rc;
                S.max_piggy[v] = 15u * digits(rc);
            }
        }
    }
    __syncthreads();
    return tot;
}

// Dissemination._issueAs (dissemination.js:133-176) for node v into out (nullable: discard).
// Filter: sender != NONE. Entries over maxPiggybackCount are deleted; the list is compacted in
// place (order kept). Returns the count emitted (block-uniform).
__device__ uint32_t block_issue(const SimDev& S, uint32_t v, uint32_t sender, int64_t sinc, Rec* out, Lds& L) {
    const uint64_t row = (uint64_t)v * S.N;
    Change* chg = S.chg + (uint64_t)v * S.Cd;
    uint32_t emitted = 0, kept = 0;
    __syncthreads();
    const uint32_t maxp = S.max_piggy[v];
    const uint32_t nc = S.n_chg[v];
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
                S.slot[row + c.addr] = (uint16_t)(kept + kpos + 1);
            } else {
                S.slot[row + c.addr] = 0;
            }
            if (emit && out) {
                const uint8_t st = S.st[row + c.addr] & ST_MASK;
                out[emitted + epos] = Rec{rec_w0(c.addr, st, 0), c.src, S.inc[row + c.addr], c.srcinc};
            }
        }
        kept += ktot;
        emitted += etot;
        __syncthreads();
    }
    if (threadIdx.x == 0) S.n_chg[v] = kept;
    __syncthreads();
    return emitted;
}

// issueAsReceiver (dissemination.js:86-119): filtered issue into `out`, else a full sync (into
// the arena) when the checksums differ. *off_out = pool offset of the message.
__device__ uint32_t block_issue_receiver(const SimDev& S, uint32_t v, uint32_t sender, int64_t sinc, uint32_t sck,
                                         uint64_t out_off, uint64_t* off_out, Lds& L) {
    const uint32_t n = block_issue(S, v, sender, sinc, S.pool + out_off, L);
    *off_out = out_off;
    if (n > 0) return n;
    checksum_if_dirty(S, v, L);
    if (S.checksum[v] == sck) return 0;
    const uint64_t fo = block_alloc(S, S.N, &L.u64);
    if (fo == ~0ull) return 0;
    const uint64_t row = (uint64_t)v * S.N;
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
__device__ void block_make(const SimDev& S, uint32_t v, uint32_t a, uint8_t st, int64_t inc, Lds& L, int64_t now,
                           Rec* tmp) {
    if (threadIdx.x == 0) *tmp = Rec{rec_w0(a, st, 0), v, inc, S.inc[(uint64_t)v * S.N + v]};
    __syncthreads();
    block_apply(S, v, tmp, 1, L, now);
}

__device__ void lane0_shuffle(const SimDev& S, uint32_t v) {
    const uint64_t row = (uint64_t)v * S.N;
    const uint32_t sh = S.n_shuf[v]++;
    for (uint32_t i = S.N - 1; i >= 1; i--) {
        const uint32_t r = philox_u32(S.seed, TAG_SHUF, sh, i, v);
        const uint32_t j = (uint32_t)(((uint64_t)r * (i + 1)) >> 32);
        const uint32_t t = S.order[row + i];
        S.order[row + i] = S.order[row + j];
        S.order[row + j] = t;
    }
}

__device__ __forceinline__ bool pingable(const SimDev& S, uint64_t row, uint32_t v, uint32_t m) {
    const uint8_t s = S.st[row + m] & ST_MASK;
    return m != v && (s == ST_ALIVE || s == ST_SUSPECT);  // isPingable (index.js:173-177)
}

// MembershipIterator.next (iterator.js:28-51) by one lane: walk the members array (reshuffling
// on wrap) until a pingable member, or until every distinct address has been visited. Before
// the first wrap of a walk positions are distinct; after it a bitmap tracks distinct visits.
__device__ int32_t lane0_iter_next(const SimDev& S, uint32_t v, uint32_t* list, uint32_t* bits) {
    const uint32_t N = S.N;
    const uint64_t row = (uint64_t)v * N;
    uint32_t nseen = 0, steps = 0;
    bool wrapped = false;
    while (nseen < N) {
        int64_t idx = S.it_idx[v] + 1;
        if (idx >= (int64_t)N) {
            idx = 0;
            if (!wrapped) {
                for (uint32_t w = 0; w < (N + 31) / 32; w++) bits[w] = 0;
                for (uint32_t q = 0; q < steps; q++) bits[list[q] >> 5] |= 1u << (list[q] & 31);
                wrapped = true;
            }
            lane0_shuffle(S, v);
        }
        S.it_idx[v] = idx;
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

// ---- phases

__global__ void k_round_begin(SimDev S) {
    if (blockIdx.x == 0 && threadIdx.x == 0) *S.cursor = 0;
}

// A: iterator.next() + issueAsSender() for every live node (checksums are fresh: k_ck_lanes ran)
__global__ __launch_bounds__(kT) void k_phase_a(SimDev S) {
    __shared__ Lds L;
    __shared__ int32_t tgt;
    for (uint32_t v = blockIdx.x; v < S.N; v += gridDim.x) {
        if (S.dead[v]) {
            if (threadIdx.x == 0) S.target[v] = -1;
            continue;
        }
        const uint64_t row = (uint64_t)v * S.N;
        if (threadIdx.x == 0) {
            uint8_t* scratch = S.strbuf + (uint64_t)blockIdx.x * S.strcap;
            const int32_t found = lane0_iter_next(S, v, reinterpret_cast<uint32_t*>(scratch),
                                                  reinterpret_cast<uint32_t*>(scratch + 4ull * S.N));
            tgt = found;
            S.target[v] = found;
        }
        __syncthreads();
        if (tgt >= 0) {
            checksum_if_dirty(S, v, L);
            const uint32_t n = block_issue(S, v, NONE, 0, ping_slot(S, v), L);
            if (threadIdx.x == 0) {
                S.ping_n[v] = n;
                S.ck_snap[v] = S.checksum[v];
                S.inc_snap[v] = S.inc[row + v];
                atomicAdd(&S.stats[0], 1ull);
            }
        }
        __syncthreads();
    }
}

// B: each live target applies its pings in sender order and answers each one
__global__ __launch_bounds__(kT) void k_phase_b(SimDev S) {
    __shared__ Lds L;
    const int64_t now = S.now0 + 200 * S.round;
    for (uint32_t j = blockIdx.x; j < S.N; j += gridDim.x) {
        if (S.dead[j]) continue;
        const uint32_t b = S.in_off[j], e = S.in_off[j + 1];
        for (uint32_t q = b; q < e; q++) {
            const uint32_t v = S.in_src[q];
            block_apply(S, j, ping_slot(S, v), S.ping_n[v], L, now);
            uint64_t o;
            const uint32_t n = block_issue_receiver(S, j, v, S.inc_snap[v], S.ck_snap[v],
                                                    (uint64_t)(resp_slot(S, v) - S.pool), &o, L);
            if (threadIdx.x == 0) {
                S.resp_n[v] = n;
                S.resp_off[v] = o;
            }
            __syncthreads();
        }
    }
}

// C: each sender with a live target applies the response (ping-sender.js:38; the second
// application at gossip/index.js:165 is idempotent: see DESIGN.md)
__global__ __launch_bounds__(kT) void k_phase_c(SimDev S) {
    __shared__ Lds L;
    const int64_t now = S.now0 + 200 * S.round;
    for (uint32_t v = blockIdx.x; v < S.N; v += gridDim.x) {
        const int32_t t = S.target[v];
        if (S.dead[v] || t < 0 || S.dead[t]) continue;
        const Rec* r = S.pool + S.resp_off[v];
        block_apply(S, v, r, S.resp_n[v], L, now);
        block_apply(S, v, r, S.resp_n[v], L, now);
    }
}

// D1: ping-req fan-out for senders whose target is dead
__global__ __launch_bounds__(kT) void k_phase_d1(SimDev S) {
    __shared__ Lds L;
    __shared__ Rec tmp;
    __shared__ uint32_t ncand;
    const int64_t now = S.now0 + 200 * S.round;
    uint32_t* cand = S.cand + (uint64_t)blockIdx.x * S.N;
    for (uint32_t v = blockIdx.x; v < S.N; v += gridDim.x) {
        const int32_t t = S.target[v];
        if (threadIdx.x == 0) S.nhelp[v] = 0;
        if (S.dead[v] || t < 0 || !S.dead[t]) continue;
        const uint64_t row = (uint64_t)v * S.N;
        if (threadIdx.x == 0) atomicAdd(&S.stats[1], 1ull);
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
                S.helpers[v * 3 + i] = cand[i];
            }
            S.nhelp[v] = nh;
            ncand = nh;
        }
        __syncthreads();
        if (ncand == 0) {
            block_make(S, v, (uint32_t)t, ST_SUSPECT, S.inc[row + t], L, now, &tmp);
            if (threadIdx.x == 0) S.nhelp[v] = 0;
            __syncthreads();
            continue;
        }
        checksum_if_dirty(S, v, L);
        if (threadIdx.x == 0) {
            S.ck_snap[v] = S.checksum[v];
            S.inc_snap[v] = S.inc[row + v];
        }
        // three issueAsSender() calls; records carry the count after the first one (aux)
        const uint32_t maxp = S.max_piggy[v];
        const uint32_t nc = S.n_chg[v];
        Change* chg = S.chg + (uint64_t)v * S.Cd;
        Rec* leg = leg_slot(S, v);
        uint32_t written2 = 0, kept = 0;
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
            uint32_t ktot, etot;
            const uint32_t kpos = block_scan(keep ? 1u : 0u, L.u, &ktot);
            const uint32_t p = block_scan(emit ? 1u : 0u, L.u, &etot);
            if (j < nc) {
                if (keep) {
                    chg[kept + kpos] = c;
                    S.slot[row + c.addr] = (uint16_t)(kept + kpos + 1);
                } else {
                    S.slot[row + c.addr] = 0;
                }
                if (emit)
                    leg[written2 + p] = Rec{rec_w0(c.addr, S.st[row + c.addr] & ST_MASK, c1), c.src,
                                            S.inc[row + c.addr], c.srcinc};
            }
            written2 += etot;
            kept += ktot;
            __syncthreads();
        }
        if (threadIdx.x == 0) {
            S.leg_n[v] = written2;
            S.n_chg[v] = kept;
        }
        __syncthreads();
    }
}

// D2: helpers handle ping-req legs in (sender, leg) order (ping-req.js:26-68)
__global__ __launch_bounds__(kT) void k_phase_d2(SimDev S) {
    __shared__ Lds L;
    const int64_t now = S.now0 + 200 * S.round;
    for (uint32_t h = blockIdx.x; h < S.N; h += gridDim.x) {
        const uint32_t b = S.h_off[h], e = S.h_off[h + 1];
        for (uint32_t q = b; q < e; q++) {
            const uint32_t code = S.h_src[q];
            const uint32_t v = code / 3, k = code % 3;
            if (S.dead[h]) {
                if (threadIdx.x == 0) S.lresp_n[code] = NONE;  // network error
                continue;
            }
            // leg k carries the records whose count after the first issue + k <= maxPiggy
            const uint32_t maxp = S.max_piggy[v];
            const uint32_t nleg = S.leg_n[v];
            const Rec* leg = leg_slot(S, v);
            const uint64_t so = block_alloc(S, nleg, &L.u64);
            if (so == ~0ull) {  // arena overflow: reported by rp_sim_step; answer as a network error
                if (threadIdx.x == 0) S.lresp_n[code] = NONE;
                __syncthreads();
                continue;
            }
            Rec* stage = S.pool + so;
            uint32_t written = 0;
            for (uint32_t base = 0; base < nleg; base += kT) {
                const uint32_t i = base + threadIdx.x;
                bool ok = false;
                Rec r{};
                if (i < nleg) {
                    r = leg[i];
                    ok = rec_aux(r) + k <= maxp;
                }
                uint32_t tot;
                const uint32_t p = block_scan(ok ? 1u : 0u, L.u, &tot);
                if (ok) stage[written + p] = r;
                written += tot;
            }
            __threadfence_block();
            __syncthreads();
            block_apply(S, h, stage, written, L, now);
            block_issue(S, h, NONE, 0, nullptr, L);  // the helper's own ping of the dead target
            const uint64_t ro = block_alloc(S, S.n_chg[h], &L.u64);
            if (ro == ~0ull) {
                if (threadIdx.x == 0) S.lresp_n[code] = NONE;
                __syncthreads();
                continue;
            }
            uint64_t o;
            const uint32_t n = block_issue_receiver(S, h, v, S.inc_snap[v], S.ck_snap[v], ro, &o, L);
            if (threadIdx.x == 0) {
                S.lresp_n[code] = n;
                S.lresp_off[code] = o;
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
    for (uint32_t v = blockIdx.x; v < S.N; v += gridDim.x) {
        const uint32_t nh = S.nhelp[v];
        if (S.dead[v] || nh == 0) continue;
        const uint64_t row = (uint64_t)v * S.N;
        bool bad = false;
        for (uint32_t k = 0; k < nh; k++) {
            const uint32_t code = v * 3 + k;
            const uint32_t n = S.lresp_n[code];
            if (n == NONE) continue;
            block_apply(S, v, S.pool + S.lresp_off[code], n, L, now);
            bad = true;
        }
        if (bad) {
            const uint32_t t = (uint32_t)S.target[v];
            block_make(S, v, t, ST_SUSPECT, S.inc[row + t], L, now, &tmp);
        }
    }
}

// E: suspicion timers due this round fire (makeFaulty with the captured incarnation). A timer
// is live while its member is still suspect at the captured incarnation (a newer suspicion
// started a newer timer; any other status stopped it); the rest are dropped. The firings touch
// distinct members, so they are applied together.
__global__ __launch_bounds__(kT) void k_phase_e(SimDev S) {
    __shared__ Lds L;
    const int64_t now = S.now0 + 200 * S.round;
    for (uint32_t v = blockIdx.x; v < S.N; v += gridDim.x) {
        if (S.dead[v]) continue;
        const uint64_t row = (uint64_t)v * S.N;
        const int64_t srci = S.inc[row + v];
        Rec* stage = ping_slot(S, v);  // free after phase B
        Timer* tim = S.tim + (uint64_t)v * S.Ct;
        const uint32_t nt = S.n_tim[v];
        uint32_t written = 0, kept = 0;
        for (uint32_t base = 0; base < nt; base += kT) {
            const uint32_t i = base + threadIdx.x;
            bool keep = false, fire = false;
            Timer t{};
            if (i < nt) {
                t = tim[i];
                const bool live = (S.st[row + t.addr] & ST_MASK) == ST_SUSPECT && S.inc[row + t.addr] == t.inc;
                fire = live && t.due <= S.round;
                keep = live && !fire;
            }
            uint32_t ktot, ftot;
            const uint32_t kpos = block_scan(keep ? 1u : 0u, L.u, &ktot);
            const uint32_t fpos = block_scan(fire ? 1u : 0u, L.u, &ftot);
            if (keep) tim[kept + kpos] = t;
            if (fire && written + fpos < S.Cm) stage[written + fpos] = Rec{rec_w0(t.addr, ST_FAULTY, 0), v, t.inc, srci};
            kept += ktot;
            written += ftot;
            __syncthreads();
        }
        if (threadIdx.x == 0) S.n_tim[v] = kept;
        __threadfence_block();
        __syncthreads();
        if (written > S.Cm) {
            if (threadIdx.x == 0) set_err(S, ERR_TIMERS);
            written = S.Cm;
        }
        if (written) block_apply(S, v, stage, written, L, now);
    }
}

__global__ void k_sim_keys(const int32_t* __restrict__ target, const uint8_t* __restrict__ dead, uint32_t N,
                           uint32_t* __restrict__ key, uint32_t* __restrict__ val) {
    for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < N; v += gridDim.x * blockDim.x) {
        const int32_t t = target[v];
        key[v] = (dead[v] || t < 0) ? NONE : (uint32_t)t;
        val[v] = v;
    }
}

__global__ void k_help_keys(const uint32_t* __restrict__ helpers, const uint32_t* __restrict__ nhelp, uint32_t N,
                            uint32_t* __restrict__ key, uint32_t* __restrict__ val) {
    for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < 3 * N; c += gridDim.x * blockDim.x) {
        const uint32_t v = c / 3, k = c % 3;
        key[c] = k < nhelp[v] ? helpers[c] : NONE;
        val[c] = c;
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

// convergence: every live checksum equal, every killed member faulty in every live view
// (checksums are fresh: k_ck_lanes ran)
__global__ void k_converged(SimDev S, uint32_t first_live, uint32_t* __restrict__ flag) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (uint64_t)S.N * S.N;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t v = (uint32_t)(i / S.N), a = (uint32_t)(i % S.N);
        if (S.dead[v]) continue;
        if (S.dead[a] && (S.st[i] & ST_MASK) != ST_FAULTY) *flag = 0;
        if (a == 0 && S.checksum[v] != S.checksum[first_live]) *flag = 0;
    }
}

__global__ void k_sim_init(SimDev S) {
    const uint64_t NN = (uint64_t)S.N * S.N;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < NN; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t v = (uint32_t)(i / S.N), a = (uint32_t)(i % S.N);
        S.st[i] = ST_ALIVE | IN_RING;
        S.inc[i] = S.inc0[a];
        S.slot[i] = 0;
        // members array after bootstrap: self first (makeAlive), then set() in id order
        S.order[i] = a == 0 ? v : (a <= v ? a - 1 : a);
    }
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (uint64_t)S.N * S.W;
         i += (uint64_t)gridDim.x * blockDim.x)
        S.dev[i] = 0;
    for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < S.N; v += gridDim.x * blockDim.x) {
        S.it_idx[v] = -1;
        S.n_shuf[v] = 0;
        S.ring_count[v] = S.N;
        S.max_piggy[v] = 15u * digits(S.N);
        S.dirty[v] = 1;  // first checksum by k_ck_lanes
        S.n_chg[v] = 0;
        S.n_tim[v] = 0;
    }
}

__global__ void k_sim_start(SimDev S) {  // gossip.start -> membership.shuffle() on live nodes
    for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < S.N; v += gridDim.x * blockDim.x)
        if (!S.dead[v]) lane0_shuffle(S, v);
}

// every node starts with the same view: hash it once, copy to all
__global__ void k_sim_first_checksum(SimDev S) {
    if (blockIdx.x == 0 && threadIdx.x == 0) S.checksum[0] = lane_checksum(S, 0);
}

__global__ void k_sim_bcast_checksum(SimDev S) {
    for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < S.N; v += gridDim.x * blockDim.x) {
        S.checksum[v] = S.checksum[0];
        S.dirty[v] = 0;
    }
}

}  // namespace

struct Sim {
    int device = 0;
    hipStream_t st = nullptr;
    uint32_t N = 0;
    unsigned grid = 0;
    NameTable nt;
    SimDev d{};
    DevBuf<uint8_t> st_, dirty, dead, strbuf, sbase;
    DevBuf<int64_t> inc, it_idx, inc_snap, inc0;
    DevBuf<int32_t> target;
    DevBuf<uint16_t> slot;
    DevBuf<uint32_t> order, dev, n_chg, n_tim, n_shuf, ring_count, max_piggy, checksum, ck_snap, ping_n, resp_n,
        leg_n, helpers, nhelp, lresp_n, cand, in_off, in_src, h_off, h_src, keys, conv, rank, err;
    DevBuf<uint64_t> boff, resp_off, lresp_off;
    DevBuf<Change> chg;
    DevBuf<Timer> tim;
    DevBuf<Rec> pool;
    DevBuf<unsigned long long> stats, cursor;
    Scratch ws;
    std::vector<uint8_t> h_dead;
    uint32_t first_live = 0;
    int64_t round = 0;

    void build_inboxes() {
        const uint32_t n = N;
        hipLaunchKernelGGL(k_sim_keys, dim3(grid_for(n, 256)), dim3(256), 0, st, target.p, dead.p, n, keys.p, in_src.p);
        radix_sort_pairs(keys.p, in_src.p, n, 0, 32, st, ws);
        hipLaunchKernelGGL(k_csr, dim3(grid_for(n + 1, 256)), dim3(256), 0, st, keys.p, n, n, in_off.p);
        RP_HIP(hipGetLastError());
    }
    void build_helper_inboxes() {
        const uint32_t n = 3 * N;
        hipLaunchKernelGGL(k_help_keys, dim3(grid_for(n, 256)), dim3(256), 0, st, helpers.p, nhelp.p, N, keys.p,
                           h_src.p);
        radix_sort_pairs(keys.p, h_src.p, n, 0, 32, st, ws);
        hipLaunchKernelGGL(k_csr, dim3(grid_for(N + 1, 256)), dim3(256), 0, st, keys.p, n, N, h_off.p);
        RP_HIP(hipGetLastError());
    }
    void refresh_checksums() {
        hipLaunchKernelGGL(k_ck_lanes, dim3(grid_for(N, 256, 1u << 20)), dim3(256), 0, st, d);
        RP_HIP(hipGetLastError());
    }
    void step() {
        d.round = round;
        hipLaunchKernelGGL(k_round_begin, dim3(1), dim3(64), 0, st, d);
        refresh_checksums();
        hipLaunchKernelGGL(k_phase_a, dim3(grid), dim3(kT), 0, st, d);
        build_inboxes();
        hipLaunchKernelGGL(k_phase_b, dim3(grid), dim3(kT), 0, st, d);
        hipLaunchKernelGGL(k_phase_c, dim3(grid), dim3(kT), 0, st, d);
        hipLaunchKernelGGL(k_phase_d1, dim3(grid), dim3(kT), 0, st, d);
        build_helper_inboxes();
        hipLaunchKernelGGL(k_phase_d2, dim3(grid), dim3(kT), 0, st, d);
        hipLaunchKernelGGL(k_phase_d3, dim3(grid), dim3(kT), 0, st, d);
        hipLaunchKernelGGL(k_phase_e, dim3(grid), dim3(kT), 0, st, d);
        RP_HIP(hipGetLastError());
        round++;
    }
    void check_err() {
        uint32_t e = 0;
        RP_HIP(hipMemcpyAsync(&e, err.p, 4, hipMemcpyDeviceToHost, st));
        RP_HIP(hipStreamSynchronize(st));
        if (e & ERR_CHANGES)
            throw Error(RP_ESTATE, "sim: a node's dissemination list exceeded its capacity (RP_SIM_CAP)");
        if (e & ERR_TIMERS) throw Error(RP_ESTATE, "sim: a node's suspicion timers exceeded their capacity (RP_SIM_CAP)");
        if (e & ERR_ARENA) throw Error(RP_ESTATE, "sim: the per-round message arena overflowed (RP_SIM_ARENA)");
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

extern "C" {

int rp_sim_create(uint32_t n, const char* names, const uint32_t* off, const int64_t* inc0, const uint8_t* dead,
                  uint32_t seed, uint32_t suspicion_rounds, int64_t now0, int device, rp_sim** out) {
    return guard([&] {
        RP_REQUIRE(out && n >= 2 && names && off && inc0 && dead, "sim_create: bad arguments");
        RP_REQUIRE(n < (1u << 23), "sim_create: at most 2^23 members");
        int nd = 0;
        RP_HIP(hipGetDeviceCount(&nd));
        RP_REQUIRE(device >= 0 && device < nd, "no such HIP device");
        RP_HIP(hipSetDevice(device));
        auto* h = new rp_sim();
        rp::Sim& S = h->impl;
        S.device = device;
        S.N = n;
        if (hipStreamCreateWithFlags(&S.st, hipStreamNonBlocking) != hipSuccess) {
            delete h;
            throw rp::Error(rp::RP_EDEVICE, "hipStreamCreate failed");
        }
        try {
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
            base.resize(base.size() + 64, 0);  // the lane chain reads up to 24 bytes past a chunk

            const uint64_t NN = (uint64_t)n * n;
            uint32_t ndead = 0;
            for (uint32_t i = 0; i < n; i++) ndead += dead[i] ? 1 : 0;
            // Capacities. In this model only killed members change state (only they are suspected;
            // nobody refutes), so a node's changes and timers are bounded by the killed count.
            const uint64_t cap = std::min<uint64_t>(n, env_u64("RP_SIM_CAP", 2ull * ndead + 256));
            RP_REQUIRE(cap >= 1 && cap < 65535, "sim_create: RP_SIM_CAP must be in [1, 65534]");
            S.grid = std::min<uint32_t>(n, 256u * 4u);
            const uint32_t W = (n + 31) / 32;
            const uint64_t arena =
                env_u64("RP_SIM_ARENA", 6ull * cap * (2ull * ndead + 64) + 32ull * n + 4096);
            S.st_.reserve(NN); S.inc.reserve(NN); S.order.reserve(NN); S.slot.reserve(NN);
            S.dev.reserve((uint64_t)n * W);
            S.chg.reserve((uint64_t)n * cap); S.tim.reserve((uint64_t)n * cap);
            S.n_chg.reserve(n); S.n_tim.reserve(n);
            S.it_idx.reserve(n); S.n_shuf.reserve(n); S.ring_count.reserve(n); S.max_piggy.reserve(n);
            S.checksum.reserve(n); S.dirty.reserve(n); S.dead.reserve(n); S.target.reserve(n); S.ck_snap.reserve(n);
            S.inc_snap.reserve(n); S.ping_n.reserve(n); S.resp_n.reserve(n); S.leg_n.reserve(n);
            S.resp_off.reserve(n); S.lresp_off.reserve(3ull * n);
            S.helpers.reserve(3ull * n); S.nhelp.reserve(n); S.lresp_n.reserve(3ull * n);
            S.in_off.reserve(n + 1ull); S.in_src.reserve(n + 1ull); S.h_off.reserve(n + 1ull);
            S.h_src.reserve(3ull * n + 1); S.keys.reserve(3ull * n + 1); S.conv.reserve(1);
            S.pool.reserve(3ull * n * cap + arena);
            S.cand.reserve((uint64_t)S.grid * n);
            // per-block string buffer: names + ';' + "suspect" + 20 digits per member (also the
            // iterator's scratch)
            const uint64_t strcap = std::max<uint64_t>(S.nt.h_bytes.size() + 29ull * n + 64, 5ull * n + 64);
            S.strbuf.reserve((uint64_t)S.grid * ((strcap + 255) & ~255ull));
            S.stats.reserve(4); S.cursor.reserve(1); S.err.reserve(1);
            S.inc0.reserve(n); S.rank.reserve(n); S.boff.reserve(n + 1ull); S.sbase.reserve(base.size());
            RP_HIP(hipMemcpyAsync(S.inc0.p, inc0, 8ull * n, hipMemcpyHostToDevice, S.st));
            RP_HIP(hipMemcpyAsync(S.rank.p, rank.data(), 4ull * n, hipMemcpyHostToDevice, S.st));
            RP_HIP(hipMemcpyAsync(S.boff.p, boff.data(), 8ull * (n + 1), hipMemcpyHostToDevice, S.st));
            RP_HIP(hipMemcpyAsync(S.sbase.p, base.data(), base.size(), hipMemcpyHostToDevice, S.st));
            S.h_dead.assign(dead, dead + n);
            RP_HIP(hipMemcpyAsync(S.dead.p, S.h_dead.data(), n, hipMemcpyHostToDevice, S.st));
            RP_HIP(hipMemsetAsync(S.stats.p, 0, 4 * sizeof(unsigned long long), S.st));
            RP_HIP(hipMemsetAsync(S.err.p, 0, 4, S.st));
            RP_HIP(hipMemsetAsync(S.cursor.p, 0, 8, S.st));
            S.first_live = 0;
            while (S.first_live < n && dead[S.first_live]) S.first_live++;
            rp::SimDev& d = S.d;
            d.N = n; d.W = W; d.seed = seed; d.susp = suspicion_rounds; d.now0 = now0;
            d.Cd = (uint32_t)cap; d.Ct = (uint32_t)cap; d.Cm = (uint32_t)cap;
            d.st = S.st_.p; d.inc = S.inc.p; d.order = S.order.p; d.slot = S.slot.p; d.dev = S.dev.p;
            d.chg = S.chg.p; d.n_chg = S.n_chg.p; d.tim = S.tim.p; d.n_tim = S.n_tim.p;
            d.it_idx = S.it_idx.p; d.n_shuf = S.n_shuf.p; d.ring_count = S.ring_count.p; d.max_piggy = S.max_piggy.p;
            d.checksum = S.checksum.p; d.dirty = S.dirty.p; d.dead = S.dead.p;
            d.sorted = S.nt.sorted.p; d.rank = S.rank.p; d.names = S.nt.d_bytes.p; d.noff = S.nt.d_noff.p;
            d.sbase = S.sbase.p; d.boff = S.boff.p; d.inc0 = S.inc0.p;
            d.target = S.target.p; d.ck_snap = S.ck_snap.p; d.inc_snap = S.inc_snap.p;
            d.pool = S.pool.p; d.arena0 = 3ull * n * cap; d.arena_cap = arena; d.cursor = S.cursor.p;
            d.resp_off = S.resp_off.p; d.lresp_off = S.lresp_off.p;
            d.ping_n = S.ping_n.p; d.resp_n = S.resp_n.p; d.leg_n = S.leg_n.p; d.helpers = S.helpers.p;
            d.nhelp = S.nhelp.p; d.lresp_n = S.lresp_n.p; d.cand = S.cand.p;
            d.strbuf = S.strbuf.p; d.strcap = (strcap + 255) & ~255ull;
            d.in_off = S.in_off.p; d.in_src = S.in_src.p; d.h_off = S.h_off.p; d.h_src = S.h_src.p;
            d.stats = S.stats.p; d.err = S.err.p; d.round = 0;
            {
                const void* ptrs[] = {d.st, d.inc, d.order, d.slot, d.dev, d.chg, d.n_chg, d.tim, d.n_tim, d.it_idx,
                                      d.n_shuf, d.ring_count, d.max_piggy, d.checksum, d.dirty, d.dead, d.sorted,
                                      d.rank, d.names, d.noff, d.sbase, d.boff, d.inc0, d.target, d.ck_snap,
                                      d.inc_snap, d.pool, d.cursor, d.resp_off, d.lresp_off, d.ping_n, d.resp_n,
                                      d.leg_n, d.helpers, d.nhelp, d.lresp_n, d.cand, d.strbuf, d.in_off, d.in_src,
                                      d.h_off, d.h_src, d.stats, d.err};
                for (const void* p : ptrs) RP_REQUIRE(p != nullptr, "sim_create: internal buffer not allocated");
            }
            hipLaunchKernelGGL(rp::k_sim_init, dim3(rp::grid_for(NN, 256, 8192)), dim3(256), 0, S.st, d);
            hipLaunchKernelGGL(rp::k_sim_start, dim3(rp::grid_for(n, 64)), dim3(64), 0, S.st, d);
            hipLaunchKernelGGL(rp::k_sim_first_checksum, dim3(1), dim3(64), 0, S.st, d);
            hipLaunchKernelGGL(rp::k_sim_bcast_checksum, dim3(rp::grid_for(n, 256)), dim3(256), 0, S.st, d);
            RP_HIP(hipGetLastError());
            RP_HIP(hipStreamSynchronize(S.st));
        } catch (...) {
            (void)hipStreamSynchronize(S.st);
            (void)hipStreamDestroy(S.st);
            delete h;
            throw;
        }
        *out = h;
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
        delete s;
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

int rp_sim_round(rp_sim* s, int64_t* out) {
    return guard([&] { *out = SM(s).round; });
}

int rp_sim_checksums(rp_sim* s, uint32_t* out) {
    return guard([&] {
        rp::Sim& S = SM(s);
        S.refresh_checksums();
        RP_HIP(hipMemcpyAsync(out, S.checksum.p, 4ull * S.N, hipMemcpyDeviceToHost, S.st));
        RP_HIP(hipStreamSynchronize(S.st));
        for (uint32_t v = 0; v < S.N; v++)
            if (S.h_dead[v]) out[v] = 0;
    });
}

int rp_sim_view(rp_sim* s, uint32_t v, uint8_t* status, int64_t* inc) {
    return guard([&] {
        rp::Sim& S = SM(s);
        RP_REQUIRE(v < S.N, "sim_view: no such node");
        const uint64_t row = (uint64_t)v * S.N;
        if (status) {
            RP_HIP(hipMemcpyAsync(status, S.st_.p + row, S.N, hipMemcpyDeviceToHost, S.st));
        }
        if (inc) RP_HIP(hipMemcpyAsync(inc, S.inc.p + row, 8ull * S.N, hipMemcpyDeviceToHost, S.st));
        RP_HIP(hipStreamSynchronize(S.st));
        if (status)
            for (uint32_t a = 0; a < S.N; a++) status[a] &= rp::ST_MASK;
    });
}

int rp_sim_converged(rp_sim* s, int* out) {
    return guard([&] {
        rp::Sim& S = SM(s);
        if (S.first_live >= S.N) {
            *out = 1;
            return;
        }
        S.refresh_checksums();
        const uint32_t one = 1;
        RP_HIP(hipMemcpyAsync(S.conv.p, &one, 4, hipMemcpyHostToDevice, S.st));
        hipLaunchKernelGGL(rp::k_converged, dim3(rp::grid_for((uint64_t)S.N * S.N, 256, 8192)), dim3(256), 0, S.st,
                           S.d, S.first_live, S.conv.p);
        uint32_t f = 0;
        RP_HIP(hipMemcpyAsync(&f, S.conv.p, 4, hipMemcpyDeviceToHost, S.st));
        RP_HIP(hipStreamSynchronize(S.st));
        *out = (int)f;
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
