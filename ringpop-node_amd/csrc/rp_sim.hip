// rp_sim.hip — the gossip protocol of N full ringpop nodes as a batched round simulator.
//
// Every node v keeps what a ringpop process keeps (SoA rows [v][member] in HBM): its membership
// view (status, incarnation; lib/membership), its dissemination buffer (piggyback records and
// counts; lib/gossip/dissemination.js), its ring membership bits + server count (only for
// maxPiggybackCount; lib/ring), its members-array order + iterator (lib/membership/iterator.js)
// and its suspicion deadlines (lib/gossip/suspicion.js), wired as lib/on_membership_event.js.
// Rounds follow the model of oracle/orc_sim.c (phases A, B, C, D1-D3, E; DESIGN.md §SWIM round
// model). Within a phase every node's work is independent of the others, so one workgroup owns
// one node at a time (persistent grid), and inside a node the records of one message (distinct
// addresses) are applied by all 256 lanes at once. Messages are fixed-capacity outboxes of
// 32-byte records. Checksums are rebuilt only for nodes whose view changed, with the
// workgroup writing the checksum string and one lane running the farmhash chain over
// LDS-staged, pre-mixed 20-byte chunks.
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
constexpr int kHashWin = 512;      // LDS window of pre-mixed chunks for the checksum chain

struct Rec {  // one piggybacked change (dissemination.js:163-170)
    uint32_t addr;
    uint32_t st;
    int64_t inc;
    uint32_t src;  // NONE = undefined
    uint32_t pad;
    int64_t srcinc;  // 0 = undefined
};

struct SimDev {
    uint32_t N;
    uint32_t seed, susp;
    int64_t now0;
    // [N*N] rows
    uint8_t* st;
    int64_t* inc;
    uint8_t *d_on, *d_st, *d_cnt;
    uint32_t* d_src;
    int64_t *d_inc, *d_srcinc;
    int32_t* deadline;
    int64_t* s_inc;
    uint8_t* in_ring;
    uint32_t* order;
    // [N]
    int64_t* it_idx;
    uint32_t *n_shuf, *ring_count, *max_piggy, *checksum;
    uint8_t* dirty;
    const uint8_t* dead;
    // names in address order
    const uint32_t* sorted;
    const uint8_t* names;
    const uint64_t* noff;
    // round scratch
    int32_t* target;
    uint32_t* ck_snap;
    int64_t* inc_snap;
    Rec* ping;
    uint32_t* ping_n;
    Rec* resp;
    uint32_t* resp_n;
    Rec* leg;  // leg records of pingreq senders, with their count after the first issue in pad
    uint32_t* leg_n;
    uint32_t* helpers;  // [N*3]
    uint32_t* nhelp;    // [N]
    Rec* lresp;         // [N*3*N]
    uint32_t* lresp_n;  // [N*3]  (NONE = network error)
    uint32_t* cand;     // [grid*N] scratch for ping-req candidate lists
    uint8_t* strbuf;    // [grid * strcap]
    uint64_t strcap;
    // CSR inboxes
    const uint32_t* in_off;   // receivers: [N+1]
    const uint32_t* in_src;   // senders sorted by (target, sender)
    const uint32_t* h_off;    // helpers: [N+1]
    const uint32_t* h_src;    // (sender*3 + leg) sorted by (helper, sender, leg)
    // stats: pings, pingreqs, fullsyncs, applied
    unsigned long long* stats;
    int64_t round;
};

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

__device__ __forceinline__ uint32_t premix(uint32_t x) { return fh::rotr(x * fh::kC1, 17) * fh::kC2; }

__device__ __forceinline__ uint32_t ld32(const uint8_t* p, uint64_t o) {
    return (uint32_t)p[o] | ((uint32_t)p[o + 1] << 8) | ((uint32_t)p[o + 2] << 16) | ((uint32_t)p[o + 3] << 24);
}

// Membership.computeChecksum (index.js:48-75) of node v by one workgroup: the string is
// written to buf in address order, then hashed (one chain lane, 192 pre-mixing lanes).
__device__ void block_checksum(const SimDev& S, uint32_t v, uint8_t* buf, uint32_t* lds_u32,
                               uint32_t (*win)[kHashWin][8]) {
    const uint32_t N = S.N;
    const uint64_t row = (uint64_t)v * N;
    const int tid = threadIdx.x;
    // contiguous member range per thread keeps address order inside each thread's piece
    const uint32_t per = (N + kT - 1) / kT;
    const uint32_t b0 = min(N, per * tid), b1 = min(N, b0 + per);
    uint32_t mine = 0;
    for (uint32_t k = b0; k < b1; k++) {
        const uint32_t a = S.sorted[k];
        mine += (uint32_t)(S.noff[a + 1] - S.noff[a]) + status_len(S.st[row + a]) + dec_len(S.inc[row + a]) + 1u;
    }
    uint32_t total;
    uint32_t o = block_scan(mine, lds_u32, &total);
    for (uint32_t k = b0; k < b1; k++) {
        const uint32_t a = S.sorted[k];
        const uint64_t nb = S.noff[a];
        const uint32_t L = (uint32_t)(S.noff[a + 1] - nb);
        for (uint32_t q = 0; q < L; q++) buf[o++] = S.names[nb + q];
        const uint8_t st = S.st[row + a];
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
                uint32_t* r = win[wb][j];
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
                    const uint32_t* r = win[cur][j];
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

struct Lds {
    uint32_t u[16];
    uint32_t win[2][kHashWin][8];
};

__device__ __forceinline__ void checksum_if_dirty(const SimDev& S, uint32_t v, Lds& L) {
    __syncthreads();
    if (S.dirty[v]) block_checksum(S, v, S.strbuf + (uint64_t)blockIdx.x * S.strcap, L.u, L.win);
}

// Membership.update(records) on node v + the 'updated' listeners (on_membership_event.js:86-134).
// Records carry distinct addresses (one message), so lanes apply them independently.
// Returns the number applied (block-uniform).
__device__ uint32_t block_apply(const SimDev& S, uint32_t v, const Rec* recs, uint32_t n, Lds& L, int64_t now) {
    const uint64_t row = (uint64_t)v * S.N;
    uint32_t napp = 0, nadd = 0, nrem = 0;
    for (uint32_t i = threadIdx.x; i < n; i += kT) {
        const Rec r = recs[i];
        const uint32_t a = r.addr;
        uint8_t us = (uint8_t)r.st;
        int64_t ui = r.inc;
        if (!evaluate_update(S.st[row + a], S.inc[row + a], a == v, us, ui, now)) continue;
        S.st[row + a] = us;
        S.inc[row + a] = ui;
        napp++;
        // createUpdatedHandlerForGossip: suspicion + recordChange
        if (us == ST_SUSPECT) {
            if (a != v) {
                S.deadline[row + a] = (int32_t)(S.round + S.susp);
                S.s_inc[row + a] = ui;
            }
        } else {
            S.deadline[row + a] = -1;
        }
        S.d_on[row + a] = 1;
        S.d_cnt[row + a] = 0;
        S.d_st[row + a] = us;
        S.d_inc[row + a] = ui;
        S.d_src[row + a] = r.src;
        S.d_srcinc[row + a] = r.srcinc;
        // createUpdatedHandlerForRing: alive -> add, faulty/leave -> remove
        if (us == ST_ALIVE && !S.in_ring[row + a]) {
            S.in_ring[row + a] = 1;
            nadd++;
        } else if ((us == ST_FAULTY || us == ST_LEAVE) && S.in_ring[row + a]) {
            S.in_ring[row + a] = 0;
            nrem++;
        }
    }
    const uint32_t tot = block_sum(napp, L.u);
    const uint32_t adds = block_sum(nadd, L.u);
    const uint32_t rems = block_sum(nrem, L.u);
    if (threadIdx.x == 0 && tot) {
        S.dirty[v] = 1;
        atomicAdd(&S.stats[3], (unsigned long long)tot);
        if (adds || rems) {  // ringChanged -> adjustMaxPiggybackCount (dissemination.js:38-55)
            const uint32_t rc = S.ring_count[v] + adds - rems;
            S.ring_count[v] = rc;
            S.max_piggy[v] = 15u * digits(rc);
        }
    }
    __syncthreads();
    return tot;
}

// Dissemination._issueAs (dissemination.js:133-176) for node v into out (nullable: discard).
// Filter: sender != NONE. Returns the count emitted (block-uniform).
__device__ uint32_t block_issue(const SimDev& S, uint32_t v, uint32_t sender, int64_t sinc, Rec* out, Lds& L) {
    const uint32_t N = S.N;
    const uint64_t row = (uint64_t)v * N;
    const uint32_t maxp = S.max_piggy[v];
    uint32_t emitted = 0;
    for (uint32_t base = 0; base < N; base += kT) {
        const uint32_t a = base + threadIdx.x;
        bool emit = false;
        if (a < N && S.d_on[row + a]) {
            const uint32_t src = S.d_src[row + a];
            const int64_t si = S.d_srcinc[row + a];
            const bool filtered = sender != NONE && sinc != 0 && src != NONE && si != 0 && src == sender && si == sinc;
            if (!filtered) {
                const uint32_t c = S.d_cnt[row + a] + 1u;
                if (c > maxp) {
                    S.d_on[row + a] = 0;
                } else {
                    S.d_cnt[row + a] = (uint8_t)c;
                    emit = true;
                }
            }
        }
        uint32_t tot;
        const uint32_t pos = block_scan(emit ? 1u : 0u, L.u, &tot);
        if (emit && out) {
            Rec r;
            r.addr = a;
            r.st = S.d_st[row + a];
            r.inc = S.d_inc[row + a];
            r.src = S.d_src[row + a];
            r.pad = 0;
            r.srcinc = S.d_srcinc[row + a];
            out[emitted + pos] = r;
        }
        emitted += tot;
    }
    return emitted;
}

// issueAsReceiver (dissemination.js:86-119): filtered issue, else fullSync when checksums differ.
__device__ uint32_t block_issue_receiver(const SimDev& S, uint32_t v, uint32_t sender, int64_t sinc, uint32_t sck,
                                         Rec* out, Lds& L) {
    const uint32_t n = block_issue(S, v, sender, sinc, out, L);
    if (n > 0) return n;
    checksum_if_dirty(S, v, L);
    if (S.checksum[v] == sck) return 0;
    const uint64_t row = (uint64_t)v * S.N;
    for (uint32_t k = threadIdx.x; k < S.N; k += kT) {  // fullSync: members-array order, source = v
        const uint32_t a = S.order[row + k];
        Rec r;
        r.addr = a;
        r.st = S.st[row + a];
        r.inc = S.inc[row + a];
        r.src = v;
        r.pad = 0;
        r.srcinc = 0;
        out[k] = r;
    }
    if (threadIdx.x == 0) atomicAdd(&S.stats[2], 1ull);
    __syncthreads();
    return S.N;
}

// makeSuspect / makeFaulty (index.js:179-202): one update from the local member
__device__ void block_make(const SimDev& S, uint32_t v, uint32_t a, uint8_t st, int64_t inc, Lds& L, int64_t now,
                           Rec* tmp) {
    if (threadIdx.x == 0) {
        Rec r;
        r.addr = a;
        r.st = st;
        r.inc = inc;
        r.src = v;
        r.pad = 0;
        r.srcinc = S.inc[(uint64_t)v * S.N + v];
        *tmp = r;
    }
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
    const uint8_t s = S.st[row + m];
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

// A: iterator.next() + issueAsSender() for every live node
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
            const uint32_t n = block_issue(S, v, NONE, 0, S.ping + row, L);
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
            const uint64_t vrow = (uint64_t)v * S.N;
            block_apply(S, j, S.ping + vrow, S.ping_n[v], L, now);
            const uint32_t n = block_issue_receiver(S, j, v, S.inc_snap[v], S.ck_snap[v], S.resp + vrow, L);
            if (threadIdx.x == 0) S.resp_n[v] = n;
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
        const uint64_t row = (uint64_t)v * S.N;
        block_apply(S, v, S.resp + row, S.resp_n[v], L, now);
        block_apply(S, v, S.resp + row, S.resp_n[v], L, now);
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
        // three issueAsSender() calls; records carry the count after the first one in .pad
        const uint32_t maxp = S.max_piggy[v];
        uint32_t written2 = 0;
        for (uint32_t base = 0; base < S.N; base += kT) {
            const uint32_t a = base + threadIdx.x;
            bool emit = false;
            uint32_t c1 = 0;
            if (a < S.N && S.d_on[row + a]) {
                const uint32_t c = S.d_cnt[row + a];
                c1 = c + 1;
                if (c + 1 > maxp) {
                    S.d_on[row + a] = 0;
                } else {
                    emit = true;
                    const uint32_t legs = (c + 3 <= maxp) ? 3u : (c + 2 <= maxp ? 2u : 1u);
                    if (legs == 3) S.d_cnt[row + a] = (uint8_t)(c + 3);
                    else S.d_on[row + a] = 0;
                }
            }
            uint32_t tot;
            const uint32_t p = block_scan(emit ? 1u : 0u, L.u, &tot);
            if (emit) {
                Rec r;
                r.addr = a;
                r.st = S.d_st[row + a];
                r.inc = S.d_inc[row + a];
                r.src = S.d_src[row + a];
                r.pad = c1;
                r.srcinc = S.d_srcinc[row + a];
                S.leg[row + written2 + p] = r;
            }
            written2 += tot;
        }
        if (threadIdx.x == 0) S.leg_n[v] = written2;
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
            const uint64_t vrow = (uint64_t)v * S.N;
            // leg k carries the records whose count after the first issue + k <= maxPiggy
            const uint32_t maxp = S.max_piggy[v];
            // compact leg k into the response buffer's tail as a staging area, then apply
            Rec* stage = S.lresp + ((uint64_t)code) * S.N;
            const uint32_t nleg = S.leg_n[v];
            uint32_t written = 0;
            for (uint32_t base = 0; base < nleg; base += kT) {
                const uint32_t i = base + threadIdx.x;
                bool ok = false;
                Rec r;
                if (i < nleg) {
                    r = S.leg[vrow + i];
                    ok = r.pad + k <= maxp;
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
            const uint32_t n = block_issue_receiver(S, h, v, S.inc_snap[v], S.ck_snap[v], stage, L);
            if (threadIdx.x == 0) S.lresp_n[code] = n;
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
            block_apply(S, v, S.lresp + (uint64_t)code * S.N, n, L, now);
            bad = true;
        }
        if (bad) {
            const uint32_t t = (uint32_t)S.target[v];
            block_make(S, v, t, ST_SUSPECT, S.inc[row + t], L, now, &tmp);
        }
    }
}

// E: suspicion timers due this round fire (makeFaulty with the captured incarnation); the
// firings touch distinct members, so they are applied together; then refresh checksums.
__global__ __launch_bounds__(kT) void k_phase_e(SimDev S) {
    __shared__ Lds L;
    const int64_t now = S.now0 + 200 * S.round;
    Rec* stage = reinterpret_cast<Rec*>(S.strbuf + (uint64_t)blockIdx.x * S.strcap);
    for (uint32_t v = blockIdx.x; v < S.N; v += gridDim.x) {
        if (S.dead[v]) continue;
        const uint64_t row = (uint64_t)v * S.N;
        const int64_t srci = S.inc[row + v];
        uint32_t written = 0;
        for (uint32_t base = 0; base < S.N; base += kT) {
            const uint32_t a = base + threadIdx.x;
            const bool due = a < S.N && S.deadline[row + a] >= 0 && S.deadline[row + a] <= S.round;
            uint32_t tot;
            const uint32_t p = block_scan(due ? 1u : 0u, L.u, &tot);
            if (due) {
                S.deadline[row + a] = -1;
                Rec r;
                r.addr = a;
                r.st = ST_FAULTY;
                r.inc = S.s_inc[row + a];
                r.src = v;
                r.pad = 0;
                r.srcinc = srci;
                stage[written + p] = r;
            }
            written += tot;
        }
        __threadfence_block();
        __syncthreads();
        if (written) block_apply(S, v, stage, written, L, now);
        checksum_if_dirty(S, v, L);
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
__global__ void k_converged(SimDev S, uint32_t* __restrict__ flag) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (uint64_t)S.N * S.N;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t v = (uint32_t)(i / S.N), a = (uint32_t)(i % S.N);
        if (S.dead[v]) continue;
        if (S.dead[a] && S.st[i] != ST_FAULTY) *flag = 0;
        if (a == 0) {
            // compare with the first live node's checksum
            uint32_t first = 0;
            while (first < S.N && S.dead[first]) first++;
            if (S.checksum[v] != S.checksum[first]) *flag = 0;
        }
    }
}

__global__ void k_sim_init(SimDev S, const int64_t* __restrict__ inc0) {
    const uint64_t NN = (uint64_t)S.N * S.N;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < NN; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t v = (uint32_t)(i / S.N), a = (uint32_t)(i % S.N);
        S.st[i] = ST_ALIVE;
        S.inc[i] = inc0[a];
        S.d_on[i] = 0;
        S.d_cnt[i] = 0;
        S.d_st[i] = 0;
        S.d_src[i] = NONE;
        S.d_inc[i] = 0;
        S.d_srcinc[i] = 0;
        S.deadline[i] = -1;
        S.s_inc[i] = 0;
        S.in_ring[i] = 1;
        // members array after bootstrap: self first (makeAlive), then set() in id order
        S.order[i] = a == 0 ? v : (a <= v ? a - 1 : a);
    }
    for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < S.N; v += gridDim.x * blockDim.x) {
        S.it_idx[v] = -1;
        S.n_shuf[v] = 0;
        S.ring_count[v] = S.N;
        S.max_piggy[v] = 15u * digits(S.N);
        S.dirty[v] = 0;
    }
}

__global__ void k_sim_start(SimDev S) {  // gossip.start -> membership.shuffle() on live nodes
    for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < S.N; v += gridDim.x * blockDim.x)
        if (!S.dead[v]) lane0_shuffle(S, v);
}

__global__ __launch_bounds__(kT) void k_sim_first_checksum(SimDev S) {
    __shared__ Lds L;
    if (blockIdx.x == 0) block_checksum(S, 0, S.strbuf, L.u, L.win);
}

__global__ void k_sim_bcast_checksum(SimDev S) {
    for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < S.N; v += gridDim.x * blockDim.x)
        S.checksum[v] = S.checksum[0];
}

}  // namespace

struct Sim {
    int device = 0;
    hipStream_t st = nullptr;
    uint32_t N = 0;
    unsigned grid = 0;
    NameTable nt;
    SimDev d{};
    DevBuf<uint8_t> st_, d_on, d_st, d_cnt, in_ring, dirty, dead, strbuf;
    DevBuf<int64_t> inc, d_inc, d_srcinc, s_inc, it_idx, inc_snap, inc0;
    DevBuf<int32_t> deadline, target;
    DevBuf<uint32_t> d_src, order, n_shuf, ring_count, max_piggy, checksum, ck_snap, ping_n, resp_n, leg_n,
        helpers, nhelp, lresp_n, cand, in_off, in_src, h_off, h_src, keys, conv;
    DevBuf<Rec> ping, resp, leg, lresp;
    DevBuf<unsigned long long> stats;
    Scratch ws;
    std::vector<uint8_t> h_dead;

    void build_inboxes() {
        const uint32_t n = N;
        // every buffer the kernels see through `d` is allocated once in rp_sim_create
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
    void step() {
        d.round = round;
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
    int64_t round = 0;
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

extern "C" {

int rp_sim_create(uint32_t n, const char* names, const uint32_t* off, const int64_t* inc0, const uint8_t* dead,
                  uint32_t seed, uint32_t suspicion_rounds, int64_t now0, int device, rp_sim** out) {
    return guard([&] {
        RP_REQUIRE(out && n >= 2 && names && off && inc0 && dead, "sim_create: bad arguments");
        RP_REQUIRE(n < (1u << 24), "sim_create: at most 2^24 members");
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
        for (uint32_t i = 0; i < n; i++) {
            const uint32_t id = S.nt.intern(names + off[i], off[i + 1] - off[i]);
            RP_REQUIRE(id == i, "sim_create: member addresses must be distinct");
        }
        S.nt.sort(S.st, S.ws);
        const uint64_t NN = (uint64_t)n * n;
        S.grid = std::min<uint32_t>(n, 256u * 4u);
        S.st_.reserve(NN); S.inc.reserve(NN); S.d_on.reserve(NN); S.d_st.reserve(NN); S.d_cnt.reserve(NN);
        S.d_src.reserve(NN); S.d_inc.reserve(NN); S.d_srcinc.reserve(NN); S.deadline.reserve(NN);
        S.s_inc.reserve(NN); S.in_ring.reserve(NN); S.order.reserve(NN);
        S.it_idx.reserve(n); S.n_shuf.reserve(n); S.ring_count.reserve(n); S.max_piggy.reserve(n);
        S.checksum.reserve(n); S.dirty.reserve(n); S.dead.reserve(n); S.target.reserve(n); S.ck_snap.reserve(n);
        S.inc_snap.reserve(n); S.ping_n.reserve(n); S.resp_n.reserve(n); S.leg_n.reserve(n);
        S.helpers.reserve(3ull * n); S.nhelp.reserve(n); S.lresp_n.reserve(3ull * n);
        S.in_off.reserve(n + 1ull); S.in_src.reserve(n + 1ull); S.h_off.reserve(n + 1ull);
        S.h_src.reserve(3ull * n + 1); S.keys.reserve(3ull * n + 1); S.conv.reserve(1);
        S.ping.reserve(NN); S.resp.reserve(NN); S.leg.reserve(NN); S.lresp.reserve(3 * NN);
        S.cand.reserve((uint64_t)S.grid * n);
        // per-block string buffer: names + ';' + "suspect" + 20 digits per member (also E's staging)
        const uint64_t strcap = std::max<uint64_t>(S.nt.h_bytes.size() + 29ull * n + 64, 32ull * n + 64);
        S.strbuf.reserve((uint64_t)S.grid * ((strcap + 255) & ~255ull));
        S.stats.reserve(4);
        S.inc0.reserve(n);
        RP_HIP(hipMemcpyAsync(S.inc0.p, inc0, 8ull * n, hipMemcpyHostToDevice, S.st));
        S.h_dead.assign(dead, dead + n);
        RP_HIP(hipMemcpyAsync(S.dead.p, S.h_dead.data(), n, hipMemcpyHostToDevice, S.st));
        RP_HIP(hipMemsetAsync(S.stats.p, 0, 4 * sizeof(unsigned long long), S.st));
        rp::SimDev& d = S.d;
        d.N = n; d.seed = seed; d.susp = suspicion_rounds; d.now0 = now0;
        d.st = S.st_.p; d.inc = S.inc.p; d.d_on = S.d_on.p; d.d_st = S.d_st.p; d.d_cnt = S.d_cnt.p;
        d.d_src = S.d_src.p; d.d_inc = S.d_inc.p; d.d_srcinc = S.d_srcinc.p; d.deadline = S.deadline.p;
        d.s_inc = S.s_inc.p; d.in_ring = S.in_ring.p; d.order = S.order.p;
        d.it_idx = S.it_idx.p; d.n_shuf = S.n_shuf.p; d.ring_count = S.ring_count.p; d.max_piggy = S.max_piggy.p;
        d.checksum = S.checksum.p; d.dirty = S.dirty.p; d.dead = S.dead.p;
        d.sorted = S.nt.sorted.p; d.names = S.nt.d_bytes.p; d.noff = S.nt.d_noff.p;
        d.target = S.target.p; d.ck_snap = S.ck_snap.p; d.inc_snap = S.inc_snap.p;
        d.ping = S.ping.p; d.ping_n = S.ping_n.p; d.resp = S.resp.p; d.resp_n = S.resp_n.p;
        d.leg = S.leg.p; d.leg_n = S.leg_n.p; d.helpers = S.helpers.p; d.nhelp = S.nhelp.p;
        d.lresp = S.lresp.p; d.lresp_n = S.lresp_n.p; d.cand = S.cand.p;
        d.strbuf = S.strbuf.p; d.strcap = (strcap + 255) & ~255ull;
        d.in_off = S.in_off.p; d.in_src = S.in_src.p; d.h_off = S.h_off.p; d.h_src = S.h_src.p;
        d.stats = S.stats.p; d.round = 0;
        {
            const void* ptrs[] = {d.st, d.inc, d.d_on, d.d_st, d.d_cnt, d.d_src, d.d_inc, d.d_srcinc, d.deadline,
                                  d.s_inc, d.in_ring, d.order, d.it_idx, d.n_shuf, d.ring_count, d.max_piggy,
                                  d.checksum, d.dirty, d.dead, d.sorted, d.names, d.noff, d.target, d.ck_snap,
                                  d.inc_snap, d.ping, d.ping_n, d.resp, d.resp_n, d.leg, d.leg_n, d.helpers, d.nhelp,
                                  d.lresp, d.lresp_n, d.cand, d.strbuf, d.in_off, d.in_src, d.h_off, d.h_src, d.stats};
            for (const void* p : ptrs) RP_REQUIRE(p != nullptr, "sim_create: internal buffer not allocated");
        }
        hipLaunchKernelGGL(rp::k_sim_init, dim3(rp::grid_for(NN, 256, 8192)), dim3(256), 0, S.st, d, S.inc0.p);
        hipLaunchKernelGGL(rp::k_sim_start, dim3(rp::grid_for(n, 64)), dim3(64), 0, S.st, d);
        hipLaunchKernelGGL(rp::k_sim_first_checksum, dim3(1), dim3(rp::kT), 0, S.st, d);
        hipLaunchKernelGGL(rp::k_sim_bcast_checksum, dim3(rp::grid_for(n, 256)), dim3(256), 0, S.st, d);
        RP_HIP(hipGetLastError());
        RP_HIP(hipStreamSynchronize(S.st));
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
        RP_HIP(hipStreamSynchronize(S.st));
    });
}

int rp_sim_step_async(rp_sim* s, uint32_t rounds) {
    return guard([&] {
        rp::Sim& S = SM(s);
        for (uint32_t r = 0; r < rounds; r++) S.step();
    });
}

int rp_sim_sync(rp_sim* s) {
    return guard([&] { RP_HIP(hipStreamSynchronize(SM(s).st)); });
}

int rp_sim_round(rp_sim* s, int64_t* out) {
    return guard([&] { *out = SM(s).round; });
}

int rp_sim_checksums(rp_sim* s, uint32_t* out) {
    return guard([&] {
        rp::Sim& S = SM(s);
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
        if (status) RP_HIP(hipMemcpyAsync(status, S.st_.p + row, S.N, hipMemcpyDeviceToHost, S.st));
        if (inc) RP_HIP(hipMemcpyAsync(inc, S.inc.p + row, 8ull * S.N, hipMemcpyDeviceToHost, S.st));
        RP_HIP(hipStreamSynchronize(S.st));
    });
}

int rp_sim_converged(rp_sim* s, int* out) {
    return guard([&] {
        rp::Sim& S = SM(s);
        const uint32_t one = 1;
        RP_HIP(hipMemcpyAsync(S.conv.p, &one, 4, hipMemcpyHostToDevice, S.st));
        hipLaunchKernelGGL(rp::k_converged, dim3(rp::grid_for((uint64_t)S.N * S.N, 256, 8192)), dim3(256), 0, S.st,
                           S.d, S.conv.p);
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
