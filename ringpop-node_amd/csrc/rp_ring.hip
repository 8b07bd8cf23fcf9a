// rp_ring.hip — the consistent hash ring on MI355X.
//
// Replaces lib/ring/index.js (HashRing) + lib/ring/rbtree.js (RBTree). The red-black tree is
// an ordered map token -> owner with insert-if-absent and erase-by-key (rbtree.js:112-116,
// 152-232); here it is a sorted uint32 token array + owner array in HBM, rebuilt per
// addRemoveServers batch by: device farmhash of every replica string -> stable radix sort
// -> drop in-batch duplicates and tokens already present (first insert wins) -> parallel
// merge with the live array; removals mark-and-compact by token regardless of owner.
// A 2^B bucket index over the top token bits bounds each lookup's search.
//
// Hot path: batched lookup / lookupN (lib/ring/index.js:145-189). One thread per key;
// fixed-stride keys are staged through LDS with coalesced 16-B loads, hashed from
// registers (fh::hash32_words), searched bucket-first, walked for distinct owners, and the
// owner rows are staged back through LDS for coalesced stores.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/ringpop_amd.h"
#include "rp_farmhash.h"
#include "rp_philox.h"
#include "rp_hashlong.h"
#include "rp_names.h"
#include "rp_prims.h"

namespace rp {

constexpr uint32_t NIL = 0xFFFFFFFFu;

static bool getenv_flag(const char* name) {
    const char* v = getenv(name);
    return v && *v && *v != '0';
}

struct RingView {
    const uint32_t* tok;
    const uint32_t* own;
    const uint32_t* bstart;  // 2^bbits + 1 entries
    uint32_t M;
    uint32_t shift;  // 32 - bbits

    // first index i in [0, M] with tok[i] >= h (RBTree upperBound semantics, rbtree.js:235-271)
    __device__ __forceinline__ uint32_t find(uint32_t h) const {
        const uint32_t b = h >> shift;
        uint32_t lo = bstart[b], hi = bstart[b + 1];
        while (lo < hi) {
            uint32_t mid = (lo + hi) >> 1;
            if (tok[mid] < h) lo = mid + 1;
            else hi = mid;
        }
        return lo;
    }
    __device__ __forceinline__ uint32_t owner(uint32_t j) const { return own[j]; }
};

// Packed lookup layout: 2^B buckets on the top B token bits (B chosen for ~4 tokens per
// bucket); each entry is one uint32 = (token low 32-B bits) << B | owner, so owner ids must be
// < 2^B. A bucket plus its lookupN successors usually sits inside one 16-entry (64-B) window.
// The entry array is padded with 0xFFFFFFFF so window loads past M stay in bounds.
struct PackedView {
    const uint32_t* ent;
    const uint32_t* bstart;  // 2^B + 1 entries
    uint32_t M;
    uint32_t B;

    __device__ __forceinline__ uint32_t key_of(uint32_t h) const { return (h << B) >> 0; }
    __device__ __forceinline__ uint32_t find(uint32_t h) const {
        const uint32_t b = h >> (32 - B);
        const uint32_t key = h << B;  // the low 32-B bits of h, shifted over the owner field
        uint32_t lo = bstart[b], hi = bstart[b + 1];
        while (lo < hi) {
            uint32_t mid = (lo + hi) >> 1;
            if (ent[mid] < key) lo = mid + 1;
            else hi = mid;
        }
        return lo;
    }
    __device__ __forceinline__ uint32_t owner(uint32_t j) const { return ent[j] & ((1u << B) - 1u); }
};

// Compact lookup layout (the C2 hot path). Sized so the whole table stays in one XCD's 4 MB L2
// (≈3.5 MB at 10k servers x 100 replicas; the packed layout's 8 MB missed ~half the time):
//   2^cb buckets on the top cb token bits, cb = floor(log2 M) (1-2 tokens per bucket);
//   idx[g] = {position of the first token of bucket 8g, 8 x 4-bit token counts of buckets
//   8g..8g+7} (8 B per 8 buckets); ent = 3 bytes per token, (fp << ob) | owner, where fp is
//   the top (24 - ob) bits of the token's low 32 - cb bits (all of them when they fit) and
//   owner < 2^ob. A key's bucket start is one 8-B load plus a nibble sum; its position and
//   successor owners come from one unaligned 16-B load of 5 entries. A key whose fingerprint
//   equals one in its bucket (only when fp drops bits) is deferred to the exact fix path.
struct CompactView {
    const uint8_t* ent;   // 3 B per token, M + kEnt3Pad entries (+16 B)
    const uint32_t* idx;  // 2 u32 per group of 8 buckets
    uint32_t M;
    uint32_t cb;   // bucket bits (>= 3)
    uint32_t ob;   // owner bits
    uint32_t fsh;  // fingerprint = (low 32 - cb bits of the hash) >> fsh
    uint32_t exact;  // fsh == 0: fingerprints are the whole residual
    uint32_t ablate;  // diagnostics only (RP_LOOKUP_ABLATE): 1 = no second windows, 2 = aligned windows
    uint32_t ent_bytes;  // allocated bytes of ent / idx (buffer-descriptor ranges of the lean kernel)
    uint32_t idx_bytes;
    uint32_t wpred;  // lean kernel: window 1 starts where the key's hash falls in its bucket (A/B:
                     // RP_LOOKUP_WPRED=0 starts it at the bucket start)
    // round 5: the hinted index (lookupN(3) in the lean kernel): per group of 8 buckets
    // {14-bit signed base - pred(g) | 8 x 2-bit window-start hints, nibble counts}, pred(g) =
    // g * M >> (cb - 3); hint h moves window 1's start by h - 1 entries (chosen at build time per
    // bucket so that the most of its hash range resolves in window 1). idxh null: no hints.
    const uint32_t* idxh;
};

// Exact view for the compact kernel's deferred keys: the bucket start comes from the compact
// index (one load) and the position from the exact wide tokens of that bucket, so a deferred
// key costs ~4 dependent loads instead of a full binary search.
struct CompactFixView {
    const uint32_t* tok;
    const uint32_t* own;
    const uint32_t* idx;
    RingView wide;  // buckets of 16+ tokens
    uint32_t M;
    uint32_t cb;

    __device__ __forceinline__ uint32_t find(uint32_t h) const {
        const uint32_t bsh = 32u - cb;
        const uint32_t g = h >> (bsh + 3u), s4 = ((h >> bsh) & 7u) * 4u;
        const uint32_t base = idx[2 * g], nib = idx[2 * g + 1];
        const uint32_t bc = (nib >> s4) & 15u;
        if (bc == 15u) return wide.find(h);
        const uint32_t below = nib & ((1u << s4) - 1u);
        const uint32_t x = (below & 0x0F0F0F0Fu) + ((below >> 4) & 0x0F0F0F0Fu);
        uint32_t i = base + ((x * 0x01010101u) >> 24);
        for (uint32_t j = 0; j < bc && tok[i] < h; j++) i++;
        return i;
    }
    __device__ __forceinline__ uint32_t owner(uint32_t j) const { return own[j]; }
};

// lookupN walk (lib/ring/index.js:157-189) with the result kept in registers (np <= MAXN).
// Visits positions i%M, i%M+1, ... cyclically, at most M of them, stopping once np
// distinct owners are collected. np <= 0 reproduces the reference's single loop body.
template <int MAXN, class View>
__device__ __forceinline__ int ring_walk(const View& rv, uint32_t i, int np, uint32_t (&res)[MAXN]) {
#pragma unroll
    for (int q = 0; q < MAXN; q++) res[q] = NIL;
    if (rv.M == 0) return 0;
    if (np <= 0) {
        if (i < rv.M) {
            res[0] = rv.owner(i);
            return 1;
        }
        return 0;
    }
    uint32_t j = (i == rv.M) ? 0u : i;
    if (MAXN == 1) {
        res[0] = rv.owner(j);
        return 1;
    }
    int cnt = 0;
    for (uint32_t steps = 0; steps < rv.M; steps++) {
        const uint32_t o = rv.owner(j);
        bool dup = false;
#pragma unroll
        for (int q = 0; q < MAXN; q++) dup |= (q < cnt) & (res[q] == o);
        if (!dup) {
#pragma unroll
            for (int q = 0; q < MAXN; q++) res[q] = (q == cnt) ? o : res[q];
            cnt++;
            if (cnt >= np) break;
        }
        j = (j + 1 == rv.M) ? 0u : j + 1;
    }
    return cnt;
}

// Unbounded walk writing straight to the output row (np > 8).
template <class View>
__device__ int ring_walk_global(const View& rv, uint32_t i, int np, uint32_t* row, uint32_t W) {
    for (uint32_t q = 0; q < W; q++) row[q] = NIL;
    if (rv.M == 0) return 0;
    if (np <= 0) {
        if (i < rv.M) {
            row[0] = rv.owner(i);
            return 1;
        }
        return 0;
    }
    uint32_t j = (i == rv.M) ? 0u : i;
    int cnt = 0;
    for (uint32_t steps = 0; steps < rv.M; steps++) {
        const uint32_t o = rv.owner(j);
        bool dup = false;
        for (int q = 0; q < cnt; q++)
            if (row[q] == o) {
                dup = true;
                break;
            }
        if (!dup) {
            row[cnt++] = o;
            if (cnt >= np) break;
        }
        j = (j + 1 == rv.M) ? 0u : j + 1;
    }
    return cnt;
}

namespace {

constexpr int kLkThreads = 256;
constexpr uint32_t kEntPad = 32;  // padding entries after M in the packed array
constexpr uint32_t kEnt3Pad = 16;  // padding entries after M in the compact array (+16 bytes)
constexpr int kDefaultKPL = 2;     // keys per lane in the probe kernel (RP_LOOKUP_KPL overrides)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Fixed-stride keys (LEN % 4 == 0, LEN > 24, e.g. 36-byte UUIDs): the hot kernel.
// Keys stream HBM -> registers -> LDS with 16-B non-temporal loads (read once; they must not
// evict the ring table from L2). The next tile's loads are issued before the current tile is
// hashed, so their HBM latency hides under the search. Each lane hashes its key from
// registers, searches, walks, and the owner rows leave through LDS as 16-B non-temporal stores.
// MODE is a diagnostic ablation (0 = full; 1 = write the hash; 2 = write the ring index).
template <int LEN, int MAXN, class View, int MODE = 0>
__global__ __launch_bounds__(kLkThreads) void k_lookupn_fixed(const uint8_t* __restrict__ keys, uint64_t n,
                                                              View rv, int np, uint32_t W,
                                                              uint32_t* __restrict__ out,
                                                              uint8_t* __restrict__ counts) {
    constexpr int W4 = LEN / 4;                       // dwords per key
    constexpr int V4 = kLkThreads * W4 / 4;           // 16-B vectors per tile
    constexpr int PER = (V4 + kLkThreads - 1) / kLkThreads;
    static_assert((kLkThreads * W4) % 4 == 0, "tile must be a whole number of 16-B vectors");
    __shared__ __attribute__((aligned(16))) uint32_t sk[kLkThreads * W4];
    __shared__ __attribute__((aligned(16))) uint32_t so[kLkThreads * MAXN];
    const int tid = threadIdx.x;
    const bool kvec = ((reinterpret_cast<uintptr_t>(keys) & 15) == 0);
    const bool ovec = ((reinterpret_cast<uintptr_t>(out) & 15) == 0);
    const uint64_t ntiles = (n + kLkThreads - 1) / kLkThreads;
    const uint64_t nfull = n / kLkThreads;  // tiles with all 256 keys

    u32x4 pre[PER];
    auto issue = [&](uint64_t t) {
        const u32x4* s4 = reinterpret_cast<const u32x4*>(keys + t * kLkThreads * LEN);
#pragma unroll
        for (int q = 0; q < PER; q++) {
            const int k = tid + q * kLkThreads;
            if (k < V4) pre[q] = __builtin_nontemporal_load(s4 + k);
        }
    };
    uint64_t t = blockIdx.x;
    if (kvec && t < nfull) issue(t);
    for (; t < ntiles; t += gridDim.x) {
        const uint64_t base = t * kLkThreads;
        const uint32_t cnt = (uint32_t)((n - base) < (uint64_t)kLkThreads ? (n - base) : kLkThreads);
        if (kvec && t < nfull) {
            u32x4* d4 = reinterpret_cast<u32x4*>(sk);
#pragma unroll
            for (int q = 0; q < PER; q++) {
                const int k = tid + q * kLkThreads;
                if (k < V4) d4[k] = pre[q];
            }
        } else {
            const uint32_t* src = reinterpret_cast<const uint32_t*>(keys + base * LEN);
            for (uint32_t k = tid; k < cnt * W4; k += kLkThreads) sk[k] = src[k];
        }
        __syncthreads();
        const uint64_t tn = t + gridDim.x;
        if (kvec && tn < nfull) issue(tn);  // in flight while this tile is searched
        int c = 0;
        uint32_t res[MAXN];
        if ((uint32_t)tid < cnt) {
            uint32_t w[W4];
#pragma unroll
            for (int j = 0; j < W4; j++) w[j] = sk[tid * W4 + j];
            const uint32_t h = fh::hash32_words<LEN>(w);
            if constexpr (MODE == 1) {
#pragma unroll
                for (int q = 0; q < MAXN; q++) res[q] = h + q;
                c = 1;
            } else if constexpr (MODE == 2) {
                const uint32_t i = rv.find(h);
#pragma unroll
                for (int q = 0; q < MAXN; q++) res[q] = i + q;
                c = 1;
            } else {
                const uint32_t i = rv.find(h);
                c = ring_walk<MAXN>(rv, i, np, res);
            }
#pragma unroll
            for (int q = 0; q < MAXN; q++)
                if ((uint32_t)q < W) so[tid * W + q] = res[q];
            if (counts) counts[base + tid] = (uint8_t)c;
        }
        __syncthreads();
        uint32_t* dst = out + base * W;
        const uint32_t tot = cnt * W;
        if (ovec && cnt == kLkThreads && (tot & 3) == 0) {
            u32x4* d4 = reinterpret_cast<u32x4*>(dst);
            const u32x4* s4 = reinterpret_cast<const u32x4*>(so);
            for (uint32_t k = tid; k < tot / 4; k += kLkThreads) __builtin_nontemporal_store(s4[k], d4 + k);
        } else {
            for (uint32_t k = tid; k < tot; k += kLkThreads) dst[k] = so[k];
        }
        __syncthreads();
    }
}

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));
typedef uint32_t u32x2_a4 __attribute__((ext_vector_type(2), aligned(4)));

// The C2 hot kernel (packed layout with ~1 token per bucket; lookup / lookupN with n <= 4;
// 36-byte keys). Every random access is ONE load instruction per key, so it costs one
// L1->L2 request (each lane of a wave instruction touching a different line is a separate
// request; PMC showed ~6 requests/key for a binary search + walk):
//   LDS key words -> farmhash32 -> [bucket lo, hi) as one 8-B load -> the 4 entries at lo as
//   one 16-B load -> position i = lo + #(entries < key) and the successor owners, from
//   registers; only when the successors run past those 4 entries, one more 16-B load at i.
// Each lane owns KPL keys of a 256*KPL-key tile, so each dependent trip serves KPL keys.
// Keys the 4-entry window cannot answer exactly (bucket longer than 4 with every entry below
// the key, positions within 3 of the end of the ring, repeated owners among the successors)
// are appended to a slow list and finished by k_lookupn_fix (binary search + the exact walk).
template <int LEN, int KPL, int MODE = 0>
__global__ __launch_bounds__(kLkThreads) void k_lookupn_probe(const uint8_t* __restrict__ keys, uint64_t n,
                                                              PackedView rv, int np, uint32_t W,
                                                              uint32_t* __restrict__ out,
                                                              uint8_t* __restrict__ counts,
                                                              uint32_t* __restrict__ slow_list,
                                                              uint32_t* __restrict__ nslow) {
    constexpr int W4 = LEN / 4;
    constexpr int TK = kLkThreads * KPL;
    constexpr int V4 = TK * W4 / 4;
    constexpr int PER = (V4 + kLkThreads - 1) / kLkThreads;
    static_assert((TK * W4) % 4 == 0, "tile must be whole 16-B vectors");
    // one LDS buffer: key words until every lane has hashed, then the owner rows
    constexpr int SK = TK * W4, SO = TK * 4;
    __shared__ __attribute__((aligned(16))) uint32_t lds[SK > SO ? SK : SO];
    uint32_t* const sk = lds;
    uint32_t* const so = lds;
    const int tid = threadIdx.x;
    const bool kvec = ((reinterpret_cast<uintptr_t>(keys) & 15) == 0);
    const bool ovec = ((reinterpret_cast<uintptr_t>(out) & 15) == 0);
    const uint64_t ntiles = (n + TK - 1) / TK;
    const uint32_t B = rv.B;
    const uint32_t omask = (1u << B) - 1u;
    const int need = np <= 0 ? 1 : np;
    for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const uint64_t base = t * TK;
        const uint32_t cnt = (uint32_t)((n - base) < (uint64_t)TK ? (n - base) : TK);
        if (kvec && cnt == TK) {
            const u32x4* s4 = reinterpret_cast<const u32x4*>(keys + base * LEN);
            u32x4 pre[PER];
#pragma unroll
            for (int q = 0; q < PER; q++) {
                const int k = tid + q * kLkThreads;
                if (k < V4) pre[q] = __builtin_nontemporal_load(s4 + k);
            }
            u32x4* d4 = reinterpret_cast<u32x4*>(sk);
#pragma unroll
            for (int q = 0; q < PER; q++) {
                const int k = tid + q * kLkThreads;
                if (k < V4) d4[k] = pre[q];
            }
        } else {
            const uint32_t* src = reinterpret_cast<const uint32_t*>(keys + base * LEN);
            for (uint32_t k = tid; k < cnt * W4; k += kLkThreads) sk[k] = src[k];
        }
        __syncthreads();
        uint32_t h[KPL];
#pragma unroll
        for (int k = 0; k < KPL; k++) {
            const uint32_t kk = tid + k * kLkThreads;
            uint32_t w[W4];
#pragma unroll
            for (int j = 0; j < W4; j++) w[j] = sk[(kk < cnt ? kk : 0) * W4 + j];
            h[k] = fh::hash32_words<LEN>(w);
        }
        __syncthreads();  // sk is reused as so below
        if constexpr (MODE == 1) {
#pragma unroll
            for (int k = 0; k < KPL; k++) {
                const uint32_t kk = tid + k * kLkThreads;
                if (kk < cnt) {
#pragma unroll
                    for (int q = 0; q < 4; q++)
                        if ((uint32_t)q < W) so[kk * W + q] = h[k] + q;
                }
            }
        } else {
            u32x2 bb[KPL];
#pragma unroll
            for (int k = 0; k < KPL; k++)
                bb[k] = *reinterpret_cast<const u32x2_a4*>(rv.bstart + (h[k] >> (32 - B)));
            u32x4 win[KPL];
#pragma unroll
            for (int k = 0; k < KPL; k++) win[k] = *reinterpret_cast<const u32x4_a4*>(rv.ent + bb[k].x);
#pragma unroll
            for (int k = 0; k < KPL; k++) {
                const uint32_t kk = tid + k * kLkThreads;
                const uint32_t lo = bb[k].x, hi = bb[k].y;
                const uint32_t key = h[k] << B;
                const uint32_t len = hi - lo;
                const uint32_t c = (0u < len && win[k].x < key) + (1u < len && win[k].y < key) +
                                   (2u < len && win[k].z < key) + (3u < len && win[k].w < key);
                const uint32_t i = lo + c;
                bool slow = (c == 4u && len > 4u) | (i + 3u >= rv.M);
                uint32_t e0, e1, e2, e3;
                if (4u - c >= (uint32_t)need) {
                    // successors i.. are win[c..3]
                    const uint32_t a0 = (c & 1) ? win[k].y : win[k].x, a1 = (c & 1) ? win[k].z : win[k].y;
                    const uint32_t a2 = (c & 1) ? win[k].w : win[k].z, a3 = win[k].w;
                    e0 = (c & 2) ? a2 : a0;
                    e1 = (c & 2) ? a3 : a1;
                    e2 = a2;
                    e3 = a3;
                } else {
                    const u32x4 sc = *reinterpret_cast<const u32x4_a4*>(rv.ent + (i < rv.M ? i : 0u));
                    e0 = sc.x;
                    e1 = sc.y;
                    e2 = sc.z;
                    e3 = sc.w;
                }
                uint32_t res[4] = {NIL, NIL, NIL, NIL};
                uint32_t rc = 1;
                if constexpr (MODE == 2) {
                    res[0] = i;
                    res[1] = i + 1;
                    res[2] = i + 2;
                    res[3] = i + 3;
                } else {
                    const uint32_t o0 = e0 & omask, o1 = e1 & omask, o2 = e2 & omask, o3 = e3 & omask;
                    // distinct owners in visit order (lib/ring/index.js:173-186)
                    res[0] = o0;
                    const uint32_t oq[3] = {o1, o2, o3};
#pragma unroll
                    for (int q = 0; q < 3; q++) {
                        const uint32_t o = oq[q];
                        const bool dup = (o == res[0]) | (rc > 1 && o == res[1]) | (rc > 2 && o == res[2]);
                        if (!dup && (int)rc < need) {
                            res[1] = rc == 1 ? o : res[1];
                            res[2] = rc == 2 ? o : res[2];
                            res[3] = rc == 3 ? o : res[3];
                            rc++;
                        }
                    }
                    slow |= (int)rc < need;  // repeated owners: the walk must go further
                }
                if (kk < cnt) {
                    if (slow) {
                        const uint32_t pos = atomicAdd(nslow, 1u);
                        slow_list[pos] = (uint32_t)(base + kk);
                    }
#pragma unroll
                    for (int q = 0; q < 4; q++)
                        if ((uint32_t)q < W) so[kk * W + q] = res[q];
                    if (counts) counts[base + kk] = (uint8_t)rc;
                }
            }
        }
        __syncthreads();
        uint32_t* dst = out + base * W;
        const uint32_t tot = cnt * W;
        if (ovec && cnt == TK && (tot & 3) == 0) {
            u32x4* d4 = reinterpret_cast<u32x4*>(dst);
            const u32x4* s4 = reinterpret_cast<const u32x4*>(so);
            for (uint32_t k = tid; k < tot / 4; k += kLkThreads) __builtin_nontemporal_store(s4[k], d4 + k);
        } else {
            for (uint32_t k = tid; k < tot; k += kLkThreads) dst[k] = so[k];
        }
        __syncthreads();
    }
}

typedef uint32_t u32x4_a1 __attribute__((ext_vector_type(4), aligned(1)));

// the 5 whole 3-byte entries in a 16-byte window
__device__ __forceinline__ void ent5(const u32x4_a1 v, uint32_t (&e)[5]) {
    e[0] = v.x & 0xFFFFFFu;
    e[1] = (v.x >> 24) | ((v.y & 0xFFFFu) << 8);
    e[2] = (v.y >> 16) | ((v.z & 0xFFu) << 16);
    e[3] = v.z >> 8;
    e[4] = v.w & 0xFFFFFFu;
}

// distinct owners in visit order (lib/ring/index.js:173-186) from window entries j >= off
__device__ __forceinline__ uint32_t dedupe5(const uint32_t (&e)[5], uint32_t off, uint32_t omask, uint32_t need,
                                            uint32_t (&res)[4]) {
    uint32_t rc = 0;
#pragma unroll
    for (int j = 0; j < 5; j++) {
        const uint32_t o = e[j] & omask;
        const bool dup = (rc > 0 && o == res[0]) | (rc > 1 && o == res[1]) | (rc > 2 && o == res[2]);
        if ((uint32_t)j >= off && !dup && rc < need) {
            res[0] = rc == 0 ? o : res[0];
            res[1] = rc == 1 ? o : res[1];
            res[2] = rc == 2 ? o : res[2];
            res[3] = rc == 3 ? o : res[3];
            rc++;
        }
    }
    return rc;
}

constexpr uint32_t kSlowPerTile = 32;  // deferred-key slots per tile of the compact kernel

// The C2 hot kernel over the compact layout: KPL keys per lane, all of a lane's random loads
// issued together (the index records, then the entry windows, then any second windows), so
// each dependent trip overlaps KPL keys. Whole tiles only (the launcher sends the tail to the
// generic kernel), 16-B aligned keys and output rows of NEED owners. Keys stream HBM -> LDS
// with 16-B non-temporal loads; owner rows leave through LDS as 16-B non-temporal stores.
// Per key: window 1 = the 5 entries at the bucket start. If the bucket has more than 5 tokens
// and all 5 are below the key, window 2 continues the search at lo + 5; if the owners run
// past window 1, window 2 starts at the position. Deferred to the exact fix path (per-tile
// slot lists, no global atomics): a fingerprint tie, a bucket of more than 10 tokens, a
// position within 10 of the ring end (wrap), more repeated owners than the windows cover.
template <int KPL, int NEED>
__global__ __launch_bounds__(kLkThreads) void k_lookupn_compact(const uint8_t* __restrict__ keys, uint64_t ntiles,
                                                                CompactView cv, uint32_t* __restrict__ out,
                                                                uint8_t* __restrict__ counts,
                                                                uint32_t* __restrict__ slow_list,
                                                                uint32_t* __restrict__ slow_cnt) {
    constexpr int LEN = 36, W4 = LEN / 4;
    constexpr int TK = kLkThreads * KPL;
    constexpr int V4 = TK * W4 / 4;
    constexpr int PER = (V4 + kLkThreads - 1) / kLkThreads;
    static_assert((TK * W4) % 4 == 0 && (TK * NEED) % 4 == 0, "tile must be whole 16-B vectors");
    constexpr int SK = TK * W4, SO = TK * NEED;
    __shared__ __attribute__((aligned(16))) uint32_t lds[SK > SO ? SK : SO];
    __shared__ uint32_t nslow_tile;
    uint32_t* const sk = lds;
    uint32_t* const so = lds;
    const int tid = threadIdx.x;
    const uint32_t omask = (1u << cv.ob) - 1u;
    const uint32_t bsh = 32u - cv.cb;
    const uint32_t rmask = (1u << bsh) - 1u;
    const u32x2* idx2 = reinterpret_cast<const u32x2*>(cv.idx);
    for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const uint64_t base = t * TK;
        {
            const u32x4* s4 = reinterpret_cast<const u32x4*>(keys + base * LEN);
            u32x4 pre[PER];
#pragma unroll
            for (int q = 0; q < PER; q++) {
                const int k = tid + q * kLkThreads;
                if (k < V4) pre[q] = __builtin_nontemporal_load(s4 + k);
            }
#pragma unroll
            for (int q = 0; q < PER; q++) {
                const int k = tid + q * kLkThreads;
                if (k < V4) reinterpret_cast<u32x4*>(sk)[k] = pre[q];
            }
        }
        if (tid == 0) nslow_tile = 0;
        __syncthreads();
        uint32_t h[KPL];
#pragma unroll
        for (int k = 0; k < KPL; k++) {
            uint32_t w[W4];
#pragma unroll
            for (int j = 0; j < W4; j++) w[j] = sk[(tid + k * kLkThreads) * W4 + j];
            h[k] = fh::hash32_words<LEN>(w);
        }
        __syncthreads();  // sk is reused as so below
        u32x2 rec[KPL];
#pragma unroll
        for (int k = 0; k < KPL; k++) rec[k] = idx2[h[k] >> (bsh + 3u)];
        uint32_t lo[KPL], bc[KPL];
        u32x4_a1 win[KPL];
#pragma unroll
        for (int k = 0; k < KPL; k++) {
            const uint32_t s4 = ((h[k] >> bsh) & 7u) * 4u;
            const uint32_t below = rec[k].y & ((1u << s4) - 1u);
            const uint32_t x = (below & 0x0F0F0F0Fu) + ((below >> 4) & 0x0F0F0F0Fu);
            lo[k] = rec[k].x + ((x * 0x01010101u) >> 24);
            bc[k] = (rec[k].y >> s4) & 15u;
            win[k] = *reinterpret_cast<const u32x4_a1*>(cv.ent + ((3ull * lo[k]) & (cv.ablate == 2 ? ~15ull : ~0ull)));
        }
        uint32_t res[KPL][4], rc[KPL], ipos[KPL], kfp[KPL];
        bool slow[KPL], search[KPL], again[KPL];
#pragma unroll
        for (int k = 0; k < KPL; k++) {
            uint32_t e[5];
            ent5(win[k], e);
            kfp[k] = (h[k] & rmask) >> cv.fsh;
            uint32_t lt = 0;
            bool tie = false;
#pragma unroll
            for (int j = 0; j < 5; j++) {
                const uint32_t f = e[j] >> cv.ob;
                const bool inb = (uint32_t)j < bc[k];
                lt += (inb && f < kfp[k]);
                tie |= (inb && f == kfp[k]);
            }
            search[k] = lt == 5u && bc[k] > 5u;  // the position lies past window 1
            ipos[k] = lo[k] + lt;
            slow[k] = (tie && !cv.exact) | (lo[k] + 10u > cv.M);
            res[k][0] = res[k][1] = res[k][2] = res[k][3] = NIL;
            rc[k] = search[k] ? 0u : dedupe5(e, lt, omask, NEED, res[k]);
            again[k] = !slow[k] && (search[k] || rc[k] < (uint32_t)NEED) && cv.ablate != 1;
        }
#pragma unroll
        for (int k = 0; k < KPL; k++)
            if (again[k]) win[k] = *reinterpret_cast<const u32x4_a1*>(cv.ent + 3ull * ipos[k]);
#pragma unroll
        for (int k = 0; k < KPL; k++) {
            if (again[k]) {
                uint32_t e[5];
                ent5(win[k], e);
                uint32_t off = 0;
                if (search[k]) {  // window 2 holds bucket entries 5..9
                    bool tie = false;
#pragma unroll
                    for (int j = 0; j < 5; j++) {
                        const uint32_t f = e[j] >> cv.ob;
                        const bool inb = (uint32_t)j + 5u < bc[k];
                        off += (inb && f < kfp[k]);
                        tie |= (inb && f == kfp[k]);
                    }
                    slow[k] |= (tie && !cv.exact) | (off == 5u && bc[k] > 10u);
                }
                res[k][0] = res[k][1] = res[k][2] = res[k][3] = NIL;
                rc[k] = dedupe5(e, off, omask, NEED, res[k]);
                slow[k] |= rc[k] < (uint32_t)NEED;
            }
            const uint32_t kk = tid + k * kLkThreads;
            if (slow[k]) {
                const uint32_t pos = atomicAdd(&nslow_tile, 1u);
                if (pos < kSlowPerTile) slow_list[t * kSlowPerTile + pos] = (uint32_t)kk;
            }
#pragma unroll
            for (int q = 0; q < NEED; q++) so[kk * NEED + q] = res[k][q];
            if (counts) counts[base + kk] = (uint8_t)rc[k];
        }
        __syncthreads();
        if (tid == 0) slow_cnt[t] = nslow_tile;
        u32x4* d4 = reinterpret_cast<u32x4*>(out + base * NEED);
        const u32x4* s4 = reinterpret_cast<const u32x4*>(so);
#pragma unroll
        for (int k = tid; k < TK * NEED / 4; k += kLkThreads) __builtin_nontemporal_store(s4[k], d4 + k);
        __syncthreads();
    }
}

// The exact position and walk of a deferred key on the compact layout with the dependent trips
// cut: the bucket's tokens are compared four at a time (one vector load for a bucket of <= 4) and
// the next 8 owners come in two vector loads; the result equals ring_walk's (the general walk
// takes over when 8 entries do not hold np distinct owners or the ring end is near).
__device__ __forceinline__ int compact_fix_walk(const CompactFixView& fv, uint32_t h, int np, uint32_t (&res)[4]) {
    if (np < 1 || np > 4) return ring_walk<4>(fv, fv.find(h), np, res);
    const uint32_t bsh = 32u - fv.cb;
    const uint32_t g = h >> (bsh + 3u), s4 = ((h >> bsh) & 7u) * 4u;
    const u32x2 rec = *reinterpret_cast<const u32x2*>(fv.idx + 2ull * g);
    const uint32_t bc = (rec.y >> s4) & 15u;
    uint32_t i;
    if (bc == 15u) {
        i = fv.wide.find(h);
    } else {
        const uint32_t below = rec.y & ((1u << s4) - 1u);
        const uint32_t x = (below & 0x0F0F0F0Fu) + ((below >> 4) & 0x0F0F0F0Fu);
        i = rec.x + ((x * 0x01010101u) >> 24);
        uint32_t lt = 0;
        for (uint32_t j = 0; j < bc; j += 4) {
            if (i + j + 4 <= fv.M) {
                const u32x4_a1 v = *reinterpret_cast<const u32x4_a1*>(fv.tok + i + j);
                lt += (j < bc && v.x < h) + (j + 1 < bc && v.y < h) + (j + 2 < bc && v.z < h) + (j + 3 < bc && v.w < h);
            } else {
                for (uint32_t q = j; q < bc && q < j + 4; q++) lt += fv.tok[i + q] < h;
            }
        }
        i += lt;  // tokens are sorted: the count below h is the position
    }
    const uint32_t p = (i == fv.M) ? 0u : i;
    if (p + 8 <= fv.M) {
        const u32x4_a1 a = *reinterpret_cast<const u32x4_a1*>(fv.own + p);
        const u32x4_a1 b = *reinterpret_cast<const u32x4_a1*>(fv.own + p + 4);
        const uint32_t o[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
        for (int q = 0; q < 4; q++) res[q] = NIL;
        int cnt = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            bool dup = false;
#pragma unroll
            for (int q = 0; q < 4; q++) dup |= (q < cnt) & (res[q] == o[j]);
            if (!dup && cnt < np) {
#pragma unroll
                for (int q = 0; q < 4; q++) res[q] = (q == cnt) ? o[j] : res[q];
                cnt++;
            }
        }
        if (cnt >= np) return cnt;
    }
    return ring_walk<4>(fv, i, np, res);
}

template <class View>
__device__ __forceinline__ int fix_walk(const View& rv, uint32_t h, int np, uint32_t (&res)[4]) {
    if constexpr (std::is_same<View, CompactFixView>::value)
        return compact_fix_walk(rv, h, np, res);
    else
        return ring_walk<4>(rv, rv.find(h), np, res);
}

// One deferred key redone exactly: hash, exact position, the reference walk; its row and count
// overwrite what the compact kernel stored.
template <class View>
__device__ __forceinline__ void lookupn_redo(const uint8_t* __restrict__ keys, const View& rv, int np, uint32_t W,
                                             uint32_t* __restrict__ out, uint8_t* __restrict__ counts, uint64_t k) {
    uint32_t w[9];
    const uint32_t* src = reinterpret_cast<const uint32_t*>(keys + k * 36);
#pragma unroll
    for (int j = 0; j < 9; j++) w[j] = src[j];
    const uint32_t h = fh::hash32_words<36>(w);
    uint32_t res[4];
    const int cnt = fix_walk(rv, h, np, res);
    uint32_t* row = out + k * W;
#pragma unroll
    for (int q = 0; q < 4; q++)
        if ((uint32_t)q < W) row[q] = res[q];
    if (counts) counts[k] = (uint8_t)cnt;
}

// Phase cycle counters of the lean kernel (diagnostics only: built with -DRP_LK_PROF by
// tools/build_prof.sh; the product build has none of this). A wave stamps s_memtime at each
// phase boundary, the stamp depending on the phase's last result; the per-phase sums over all
// waves land in g_lk_prof (printed by launch_lookupn under RP_LK_PROF_PRINT).
#ifdef RP_LK_PROF
__device__ unsigned long long g_lk_prof[10];
#define LK_T(var, dep) \
    uint64_t var;      \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(var) : "v"(dep))
#else
#define LK_T(var, dep)
#endif

// The C2 hot kernel, lean form (round 2): the same layout, loads and results as
// k_lookupn_compact, with fewer vector instructions per key (the SQ counters put that kernel at
// ~2.9x the VALU issue of the hash-only ablation).
//   - The index record and the window come through buffer descriptors with 32-bit offsets (no
//     64-bit address arithmetic); the nibble sum is two v_sad_u8.
//   - Window 1 resolves a key in one straight-line pass when its position is at most 5 - NEED
//     entries into the window and the NEED owners there are distinct: the fingerprint tests
//     compare whole entries against kfp << ob, the owners are picked by the position.
//   - The ~8 % of keys that need a second window (the position lies further, a long bucket, or
//     a repeated owner) are appended to a per-wave list (ballot + mbcnt, 64 slots in LDS); the
//     wave then finishes them one key per lane, so the second-window code runs once per wave
//     instead of once per key slot. Keys past the list go to the exact fix path, like ties and
//     positions near the ring end.
// HS: the tile's keys pass through LDS in HS slices (all loads issued first, held in registers),
// so the key stage takes 1/HS of the LDS and more workgroups fit a CU (A/B).
// (Forcing 5 waves per SIMD with __launch_bounds__ spills 8 VGPRs and ran 1.05 against 0.91 ms,
// profiles/r03/ab_lookup_occ.json: the 119-121 VGPRs and 4 waves per SIMD stay.)
// FUSE: the workgroup finishes its own tiles' deferred keys after its last tile (one thread per
// list slot, 8 tiles at a time) instead of k_lookupn_fix_tiles (A/B: RP_LOOKUP_FUSEFIX).
// STG: how the key tile reaches LDS. 0: every lane loads all its 16-B pieces of the tile into
// registers first (PER x u32x4 held), then the slices go through LDS one after another. 1: the
// slices are DMA'd global -> LDS (global_load_lds_dwordx4, no VGPR destination) into a ring of
// two slice buffers, slice s + 2 issued as soon as slice s is hashed (A/B: RP_LOOKUP_STG=1).
// The lean kernel's timing ablations (RP_LOOKUP_ABLATE, round 5) exist only in a diagnostics
// build (-DRP_LK_ABLATE, tools/build_prof.sh). Read at run time (as from r05a to r05au), their
// uniform branches around the index and window loads split the loads' clusters: 3,394
// instructions and 181 branches against 3,191 and 139, 0.926 against 0.886 ms per 2^26-key step
// on one box, below round 4's kernel (0.903; profiles/r05/r05aw/).
#ifdef RP_LK_ABLATE
#define RP_LKA(cv) ((cv).ablate)
#else
#define RP_LKA(cv) 0u
#endif
template <int KPL, int NEED, int HS = 1, bool FUSE = false, int STG = 0, int LH = 1>
__global__ __launch_bounds__(kLkThreads) __attribute__((amdgpu_waves_per_eu(4))) void k_lookupn_lean(const uint8_t* __restrict__ keys, uint64_t ntiles,
                                                             CompactView cv, uint32_t* __restrict__ out,
                                                             uint8_t* __restrict__ counts,
                                                             uint32_t* __restrict__ slow_list,
                                                             uint32_t* __restrict__ slow_cnt, CompactFixView fv,
                                                             int np) {
    constexpr int LEN = 36, W4 = LEN / 4;
    constexpr int TK = kLkThreads * KPL;
    constexpr int V4 = TK * W4 / 4;
    constexpr int PER = (V4 + kLkThreads - 1) / kLkThreads;
    constexpr int NW = kLkThreads / 64;
    constexpr uint32_t SPAN = 5 - NEED;  // last window-1 position that still holds NEED entries
    static_assert((TK * W4) % 4 == 0 && (TK * NEED) % 4 == 0 && NEED >= 1 && NEED <= 4, "tile shape");
    static_assert(KPL % HS == 0 && V4 % HS == 0, "slices of whole keys");
    constexpr int SK = TK * W4 / HS, SO = TK * NEED;
    constexpr int VS = V4 / HS;  // 16-B vectors per slice
    constexpr int SKR = STG ? 2 * SK : SK;  // STG 1 / 2: two slice buffers
    static_assert(STG == 0 || (SK * 4) % 1024 == 0, "DMA slices of whole 1-KB wave pieces");
    __shared__ __attribute__((aligned(16))) uint32_t lds[SKR > SO ? SKR : SO];
    constexpr uint32_t AG = 64;  // list slots per wave (8 % of 64 * KPL keys: ~41 at KPL 8)
    __shared__ uint32_t ag[NW][3][AG];  // per-wave second-window list: start, K, kk | bc << 12 | search << 16
    __shared__ uint32_t nslow_tile;
    uint32_t* const sk = lds;
    uint32_t* const so = lds;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint32_t omask = (1u << cv.ob) - 1u, obit = 1u << cv.ob;
    const uint32_t bsh = 32u - cv.cb;
    const uint32_t rmask = (1u << bsh) - 1u;
    const __amdgpu_buffer_rsrc_t ent_r =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(cv.ent), 0, (int)cv.ent_bytes, 0x00020000);
    // lookupN(3) reads the hinted index when the ring has one (round 5; RP_LOOKUP_HINT=0: A/B)
    const bool hinted = NEED == 3 && cv.idxh != nullptr && !(RP_LKA(cv) & 4u);
    const __amdgpu_buffer_rsrc_t idx_r = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint32_t*>(hinted ? cv.idxh : cv.idx), 0, (int)cv.idx_bytes, 0x00020000);
    auto load16 = [&](uint32_t pos) {
        return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(ent_r, (int)(3u * pos), 0, 0));
    };
    auto ent5v = [&](const u32x4 v, uint32_t (&e)[5]) {
        e[0] = v.x & 0xFFFFFFu;
        e[1] = (v.x >> 24) | ((v.y & 0xFFFFu) << 8);
        e[2] = (v.y >> 16) | ((v.z & 0xFFu) << 16);
        e[3] = v.z >> 8;
        e[4] = v.w & 0xFFFFFFu;
    };
    // Window 1's first entry within the bucket (round 3): the key's position in a bucket of bc
    // tokens is about bc times its place in the bucket's hash range (r), so the window starts at
    // max(0, floor(r bc) - 1). A window at w > 0 resolves positions w+1..w+2 (entry w below the key
    // is the guard), one at 0 positions 0..2: 3.6 % of keys need a second window instead of 9.9 %
    // (Poisson buckets of 1.9 tokens; lookupN(2): 3.3 % -> 1.6 %). Long buckets (> 10) keep w = 0,
    // and so does lookup (NEED 1), whose window at 0 already resolves positions 0..4 (0.9 % of keys
    // past it against 1.5 % with the predicted start).
    // hint (the hinted index): the start moves by hint - 1 entries (1 = the plain prediction)
    auto wstart = [&](uint32_t hk, uint32_t bck, uint32_t hint) -> uint32_t {
        const int fl = (int)((((hk << cv.cb) >> 24) * bck) >> 8) - 2 + (int)hint;
        return (NEED >= 2 && cv.wpred && bck <= 10u && fl > 0) ? (uint32_t)fl : 0u;
    };
    // a listed key's second window (held by one lane): finish it, write its row into `row`
    auto finish2 = [&](const u32x4 win, uint32_t K, uint32_t w2, uint32_t* row, uint8_t* cnt, uint32_t* nsl,
                       uint32_t* slist) {
        const uint32_t kk = w2 & 0xFFFu, bck = (w2 >> 12) & 15u, b0 = (w2 >> 17) & 15u;
        uint32_t e2[5];
        ent5v(win, e2);
        uint32_t off = 0;
        bool slow = false;
        if ((w2 >> 16) & 1u) {  // window 2 holds bucket entries b0..b0+4: search it
            bool tie = false;
#pragma unroll
            for (int j = 0; j < 5; j++) {
                const bool inb = (uint32_t)j + b0 < bck;
                off += (inb && e2[j] < K);
                tie |= (inb && e2[j] - K < obit);
            }
            // past this window too; or (guard) the key may lie before entry b0
            slow = (tie && !cv.exact) | (off == 5u && bck > b0 + 5u) | (((w2 >> 21) & 1u) && off == 0u);
        }
        uint32_t res[4] = {NIL, NIL, NIL, NIL};
        const uint32_t rc = dedupe5(e2, off, omask, NEED, res);
        slow |= rc < (uint32_t)NEED;
        if (slow) {
            const uint32_t sp = atomicAdd(nsl, 1u);
            if (sp < kSlowPerTile) slist[sp] = kk;
        }
#pragma unroll
        for (int q = 0; q < NEED; q++) row[kk * NEED + q] = res[q];
        if (cnt) cnt[kk] = (uint8_t)rc;
    };
#ifdef RP_LK_PROF
    uint64_t pa[6] = {0, 0, 0, 0, 0, 0}, ntl = 0;
#endif
    for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const uint64_t base = t * TK;
        uint32_t h[KPL];
        LK_T(t0, tid);
        if constexpr (STG == 1 || STG == 2) {
            // DMA ring: slice s in buffer s & 1; a slice is SLI 1-KB wave pieces dealt over the
            // waves (wave w takes pieces w, w + NW, ...), so wave w waits for its own pieces of
            // slice s with a counted vmcnt (its pieces of slice s + 1 may stay in flight), then
            // the workgroup barrier makes every wave's pieces visible
            constexpr int SLB = SK * 4, SLI = SLB / 1024, PW = SLI / NW, PX = SLI % NW;
            const uint8_t* src = keys + base * LEN;
            uint8_t* ring = reinterpret_cast<uint8_t*>(lds);
            auto dma = [&](int sl) {
#pragma unroll
                for (int i = 0; i < PW + 1; i++)
                    if (i < PW || wv < PX) {
                        const void* g = reinterpret_cast<const void*>(src + sl * SLB + (i * NW + wv) * 1024 + lane * 16);
                        uint8_t* l = ring + (sl & 1) * SLB + (i * NW + wv) * 1024;
                        if constexpr (STG == 1) {
                            __builtin_amdgcn_global_load_lds(g, l, 16, 0, 0);
                        } else {
                            // the same DMA in asm: the compiler does not see an LDS write in flight,
                            // so it does not drain vmcnt(0) before the next slice's ds_reads (the
                            // counted waits below order them)
                            const uint32_t lo = __builtin_amdgcn_readfirstlane(
                                (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)l);
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"  // m0 is set here; the kernel has no other m0 use
                            asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
                                         :
                                         : "v"(g), "s"(lo)
                                         : "memory", "m0");
#pragma clang diagnostic pop
                        }
                    }
            };
            if (tid == 0) nslow_tile = 0;
            dma(0);
            if (HS > 1) dma(1);
#pragma unroll
            for (int hs = 0; hs < HS; hs++) {
                if (hs + 1 < HS) {
                    if (wv < PX)
                        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PW + 1) : "memory");
                    else
                        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PW) : "memory");
                } else {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
                asm volatile("" ::: "memory");
#ifdef RP_LK_PROF
                if (hs == 0) {
                    LK_T(tk, lds[tid]);
                    pa[0] += tk - t0;
                }
#endif
                const uint32_t* sb = lds + (hs & 1) * SK;
#pragma unroll
                for (int k = hs * (KPL / HS); k < (hs + 1) * (KPL / HS); k++) {
                    uint32_t w[W4];
#pragma unroll
                    for (int j = 0; j < W4; j++) w[j] = sb[(tid + (k - hs * (KPL / HS)) * kLkThreads) * W4 + j];
                    h[k] = fh::hash32_words<LEN>(w);
                }
                if (hs + 2 < HS) {  // this buffer is free once every wave has hashed from it
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    __builtin_amdgcn_s_barrier();
                    asm volatile("" ::: "memory");
                    dma(hs + 2);
                }
            }
        } else {
            const u32x4* s4 = reinterpret_cast<const u32x4*>(keys + base * LEN);
            u32x4 pre[PER];
#pragma unroll
            for (int q = 0; q < PER; q++) {
                const int k = tid + q * kLkThreads;
                if (k < V4) pre[q] = __builtin_nontemporal_load(s4 + k);
            }
            if (tid == 0) nslow_tile = 0;
#pragma unroll
            for (int hs = 0; hs < HS; hs++) {
                if (hs) __syncthreads();  // the previous slice is hashed
#pragma unroll
                for (int q = 0; q < PER; q++) {
                    const int k = tid + q * kLkThreads;
                    if (k >= hs * VS && k < (hs + 1) * VS) reinterpret_cast<u32x4*>(sk)[k - hs * VS] = pre[q];
                }
                __syncthreads();
#ifdef RP_LK_PROF
                if (hs == 0) {
                    LK_T(tk, sk[tid]);
                    pa[0] += tk - t0;
                }
#endif
#pragma unroll
                for (int k = hs * (KPL / HS); k < (hs + 1) * (KPL / HS); k++) {
                    uint32_t w[W4];
#pragma unroll
                    for (int j = 0; j < W4; j++) w[j] = sk[(tid + (k - hs * (KPL / HS)) * kLkThreads) * W4 + j];
                    h[k] = fh::hash32_words<LEN>(w);
                }
            }
        }
        LK_T(t2, h[KPL - 1]);
        __syncthreads();  // sk is reused as so below
        uint32_t nag = 0;  // wave-uniform length of this wave's list
        // LH > 1: the index and window trips run for KPL / LH keys at a time (fewer live
        // registers in this phase; A/B: RP_LOOKUP_LH)
        constexpr int KH = KPL / LH;
        static_assert(KPL % LH == 0, "whole halves");
#ifdef RP_LK_PROF
        uint64_t t3 = 0;
#endif
#pragma unroll
        for (int hh = 0; hh < LH; hh++) {
        if (hh) __builtin_amdgcn_sched_barrier(0);
        u32x2 rec[KH];
#pragma unroll
        for (int kq = 0; kq < KH; kq++) {
            const int k = hh * KH + kq;
            if (RP_LKA(cv) & 4u)  // diagnostics: no index trip (a record made from the hash)
                rec[kq] = u32x2{(uint32_t)(((uint64_t)h[k] * (cv.M - 32u)) >> 32), h[k] & 0x11111111u};
            else
                rec[kq] = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(idx_r, (int)((h[k] >> (bsh + 3u)) * 8u), 0, 0));
        }
        uint32_t lo[KH], bc[KH], ws[KH];
        u32x4 win[KH];
#pragma unroll
        for (int kq = 0; kq < KH; kq++) {
            const int k = hh * KH + kq;
            const uint32_t s4 = ((h[k] >> bsh) & 7u) * 4u;
            const uint32_t below = rec[kq].y & ((1u << s4) - 1u);
            uint32_t base = rec[kq].x, hint = 1u;
            if (hinted) {  // base = pred(g) + the 14-bit delta; the bucket's 2-bit hint
                const uint32_t g = h[k] >> (bsh + 3u);
                base = (uint32_t)(((uint64_t)g * cv.M) >> (cv.cb - 3u)) + (uint32_t)((int32_t)(rec[kq].x << 18) >> 18);
                hint = (rec[kq].x >> (14u + (s4 >> 1))) & 3u;
            }
            lo[kq] = base + __builtin_amdgcn_sad_u8(below & 0x0F0F0F0Fu, 0u,
                                                    __builtin_amdgcn_sad_u8((below >> 4) & 0x0F0F0F0Fu, 0u, 0u));
            bc[kq] = (rec[kq].y >> s4) & 15u;
            ws[kq] = wstart(h[k], bc[kq], hint);
            if (RP_LKA(cv) & 26u) {  // diagnostics: 2 = windows rounded down to 16 B (no line crossing);
                                    // 8 = no window trip (entries made from the record); 16 = windows
                                    // rounded down to 4 B (dword-aligned, still crossing lines)
                const uint32_t pos = lo[kq] + ws[kq];
                win[kq] = (RP_LKA(cv) & 8u) ? u32x4{rec[kq].x, rec[kq].y, h[k], pos}
                                           : __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                                          ent_r, (int)((3u * pos) & ((RP_LKA(cv) & 2u) ? ~15u : ~3u)), 0, 0));
            } else {
                win[kq] = load16(lo[kq] + ws[kq]);
            }
        }
#ifdef RP_LK_PROF
        if (hh == 0) {
            LK_T(t3h, lo[KH - 1]);
            t3 = t3h;
        }
#endif
#pragma unroll
        for (int kq = 0; kq < KH; kq++) {
            const int k = hh * KH + kq;
            uint32_t e[5];
            ent5v(win[kq], e);
            const uint32_t K = ((h[k] & rmask) >> cv.fsh) << cv.ob;
            const uint32_t w = ws[kq];
            uint32_t lt = 0;  // in-bucket window entries below the key: the position is lo + w + lt
            bool tie = false;
#pragma unroll
            for (int j = 0; j < 5; j++) {
                const bool inb = (uint32_t)j + w < bc[kq];
                lt += (inb && e[j] < K);
                tie |= (inb && e[j] - K < obit);
            }
            uint32_t r[NEED];
#pragma unroll
            for (int q = 0; q < NEED; q++) {
                uint32_t v = e[q] & omask;
#pragma unroll
                for (uint32_t d = 1; d <= SPAN; d++) v = lt == d ? (e[q + d] & omask) : v;
                r[q] = v;
            }
            bool dup = false;
#pragma unroll
            for (int a = 0; a < NEED; a++)
#pragma unroll
                for (int b = a + 1; b < NEED; b++) dup |= r[a] == r[b];
            const uint32_t kk = tid + k * kLkThreads;
            bool slow = (tie && !cv.exact) | (lo[kq] + 20u > cv.M);
            const bool under = w > 0u && lt == 0u;  // the key lies before window 1's first entry
            const bool again = !slow && (lt > SPAN || dup || under) && !(RP_LKA(cv) & 1u);  // 1: diagnostics
            const uint64_t m = __ballot(again);
            const uint32_t pos = nag + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            nag += (uint32_t)__popcll(m);
            if (again) {
                if (pos < AG) {
                    // under: search from w - 2 (the position is at most w), guarded when > 0; past
                    // window 1 inside the bucket: search on from w + 5; else the position is known
                    const uint32_t b0 = under ? (w > 2u ? w - 2u : 0u) : w + 5u;
                    const bool search = under || (lt == 5u && bc[kq] > w + 5u);
                    ag[wv][0][pos] = lo[kq] + (search ? b0 : w + lt);
                    ag[wv][1][pos] = K;
                    ag[wv][2][pos] = kk | (bc[kq] << 12) | ((uint32_t)search << 16) | ((search ? b0 : 0u) << 17) |
                                     ((uint32_t)(under && b0 > 0u) << 21);
                } else {
                    slow = true;
                }
            } else {
#pragma unroll
                for (int q = 0; q < NEED; q++) so[kk * NEED + q] = r[q];
                if (counts) counts[base + kk] = (uint8_t)NEED;
            }
            if (slow) {
                const uint32_t sp = atomicAdd(&nslow_tile, 1u);
                if (sp < kSlowPerTile) slow_list[t * kSlowPerTile + sp] = kk;
            }
        }
        }  // halves
        LK_T(t4, nag);
        // second windows, one listed key per lane (the list is this wave's own LDS rows)
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        for (uint32_t j = lane; j < (nag < AG ? nag : AG); j += 64)
            finish2(load16(ag[wv][0][j]), ag[wv][1][j], ag[wv][2][j], so, counts ? counts + base : nullptr,
                    &nslow_tile, slow_list + t * kSlowPerTile);
        LK_T(t5a, nag);
        __syncthreads();
        LK_T(t5, tid);
        if (tid == 0) slow_cnt[t] = nslow_tile;
        u32x4* d4 = reinterpret_cast<u32x4*>(out + base * NEED);
        const u32x4* s4 = reinterpret_cast<const u32x4*>(so);
#pragma unroll
        for (int k = tid; k < TK * NEED / 4; k += kLkThreads) __builtin_nontemporal_store(s4[k], d4 + k);
        __syncthreads();
#ifdef RP_LK_PROF
        LK_T(t6, tid);
        pa[1] += t2 - t0;
        pa[2] += t3 - t2;
        pa[3] += t4 - t3;
        pa[4] += t5a - t4;
        pa[5] += t6 - t5;
        ntl += 1;
        (void)t5;
#endif
    }
#ifdef RP_LK_PROF
    if (lane == 0) {
        for (int i = 0; i < 6; i++) atomicAdd(&g_lk_prof[i], (unsigned long long)pa[i]);
        atomicAdd(&g_lk_prof[6], (unsigned long long)ntl);
    }
#endif
    if constexpr (FUSE) {
        // this workgroup's tiles t = blockIdx.x + i * gridDim.x; their rows are stored (the barrier
        // above orders the overwrites after them)
        constexpr uint32_t TPP = kLkThreads / kSlowPerTile;
        const uint64_t nt = ntiles > blockIdx.x ? (ntiles - blockIdx.x + gridDim.x - 1) / gridDim.x : 0;
        for (uint64_t i0 = 0; i0 < nt; i0 += TPP) {
            const uint64_t i = i0 + (uint32_t)tid / kSlowPerTile;
            const uint32_t q = (uint32_t)tid % kSlowPerTile;
            if (i < nt) {
                const uint64_t t = blockIdx.x + i * gridDim.x;
                const uint32_t c = slow_cnt[t];
                if (c <= kSlowPerTile) {
                    if (q < c) lookupn_redo(keys, fv, np, (uint32_t)NEED, out, counts, t * TK + slow_list[t * kSlowPerTile + q]);
                } else {
                    for (uint32_t k = q; k < (uint32_t)TK; k += kSlowPerTile) lookupn_redo(keys, fv, np, (uint32_t)NEED, out, counts, t * TK + k);
                }
            }
        }
    }
}

// ---- The wave-specialised lean kernel (round 6, A/B: RP_LOOKUP_WS). The lean kernel's waves run
// every phase in turn (key stream, hash, index trip, window trip, stores), and s_waitcnt vmcnt
// retires in issue order, so a wave cannot keep its next keys in flight behind its lookups. Here
// the NP producer waves of a workgroup only stream keys (16-B non-temporal loads, transposed
// through an 18-KB LDS tile per producer, the next tile's loads in flight) and hash them into an
// LDS ring (slots of 512 hashes), and the NC consumer waves only take the index and window trips
// and store the rows (a 12-B
// buffer store per key: 768 contiguous bytes per wave instruction; second-window keys' rows
// from the lane that finishes them). Producer p serves consumers p, p + NP, ...; the ring's
// counters are LDS words (prod[c]: wave-tiles filled, cons[c]: wave-tiles read). Every wait is
// bounded (kWsSpin polls): past it the wave stops waiting and sets *err, so the grid always
// drains (the launch's results are then wrong; the launcher reports it under RP_LOOKUP_DEBUG).
// Deferred keys go to per-wave-tile lists (k_lookupn_fix_tiles with TK 512).
// Measured (profiles/r06/r06at-r06aw): 1.10 ms per 2^26 C2 keys at 4:12 against the lean kernel's
// 0.88; alone, the producers take 0.58 ms and the consumers 0.68, and split this way the two add
// up (both move their bytes through the L2 -> CU return path). The lean kernel stays the default.
constexpr int kWsSlots = 2;
constexpr uint32_t kWsSpin = 1u << 22;
typedef uint32_t u32x3v __attribute__((ext_vector_type(3)));

// ABL (diagnostics, RP_LOOKUP_WS_ABL; results wrong, times only): 1 = producers load no keys (the
// hashes are made from the key index), 2 = consumers take no trips (the row is the hash).
template <int NP, int NC, int ABL = 0>
__global__ __launch_bounds__((NP + NC) * 64) __attribute__((amdgpu_waves_per_eu(4))) void k_lookupn_ws(const uint8_t* __restrict__ keys, uint64_t nwt,
                                                               CompactView cv, uint32_t* __restrict__ out,
                                                               uint32_t out_bytes, uint8_t* __restrict__ counts,
                                                               uint32_t* __restrict__ slow_list,
                                                               uint32_t* __restrict__ slow_cnt,
                                                               uint32_t* __restrict__ err) {
    constexpr int NEED = 3, KPL = 8, LEN = 36, W4 = LEN / 4;
    constexpr int TK = 64 * KPL;         // keys a wave-tile
    constexpr int V4 = TK * W4 / 4;      // its 16-B pieces
    constexpr int PER = V4 / 64;         // per producer lane
    constexpr uint32_t SPAN = 5 - NEED;
    constexpr uint32_t AG = 64;
    static_assert(V4 % 64 == 0, "wave-tile shape");
    __shared__ __attribute__((aligned(16))) uint32_t stg[NP][V4 * 4];
    __shared__ uint32_t ring[NC][kWsSlots][TK];
    __shared__ uint32_t ag[NC][3][AG];
    __shared__ uint32_t prod[NC], cons[NC], nsl[NC];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    if (tid < NC) {
        prod[tid] = 0;
        cons[tid] = 0;
    }
    __syncthreads();
    const uint64_t nwg = (nwt + NC - 1) / NC;  // workgroup tiles: NC wave-tiles each
    // until *p >= target (wave-uniform: one LDS word read by the whole wave)
    auto wait_ge = [&](uint32_t* p, uint32_t target) {
        for (uint32_t n = 0;; n++) {
            const uint32_t v = __builtin_amdgcn_readfirstlane(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
            if (v >= target) break;
            if (n == kWsSpin) {
                if (lane == 0) atomicOr(err, 1u);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
            asm volatile("" ::: "memory");
        }
        asm volatile("" ::: "memory");
    };
    if (wv < NP) {
        // producer: item j is consumer c = wv + (j % cnt) NP's wave-tile of workgroup tile
        // blockIdx.x + (j / cnt) gridDim.x (ring sequence j / cnt). The whole wave-tile's keys go
        // to LDS at once, and the next item's 18 loads a lane are issued before this one is
        // hashed, so the key stream stays in flight behind the hashing and the ring waits.
        const int cnt = (NC - wv + NP - 1) / NP;
        auto item_wt = [&](uint32_t j) -> uint64_t {
            const uint64_t T = blockIdx.x + (uint64_t)(j / cnt) * gridDim.x;
            const uint64_t wt = T * NC + wv + (j % cnt) * NP;
            return T < nwg && wt < nwt ? wt : ~0ull;
        };
        u32x4 pre[PER];
        auto issue = [&](uint64_t wt) {
            const u32x4* s4 = reinterpret_cast<const u32x4*>(keys + wt * (uint64_t)(TK * LEN));
#pragma unroll
            for (int q = 0; q < PER; q++) pre[q] = __builtin_nontemporal_load(s4 + lane + 64 * q);
        };
        uint64_t wt = item_wt(0);
        if (ABL != 1 && wt != ~0ull) issue(wt);
        for (uint32_t j = 0; wt != ~0ull; j++) {
            const uint64_t wn = item_wt(j + 1);
            uint32_t h[KPL];
            if constexpr (ABL == 1) {
#pragma unroll
                for (int k = 0; k < KPL; k++) h[k] = (uint32_t)(wt * TK + lane + 64 * k) * 0x9E3779B1u;
            } else {
                u32x4* st4 = reinterpret_cast<u32x4*>(stg[wv]);
#pragma unroll
                for (int q = 0; q < PER; q++) st4[lane + 64 * q] = pre[q];
                __builtin_amdgcn_wave_barrier();
                if (wn != ~0ull) issue(wn);
#pragma unroll
                for (int k = 0; k < KPL; k++) {
                    uint32_t w[W4];
#pragma unroll
                    for (int x = 0; x < W4; x++) w[x] = stg[wv][(lane + 64 * k) * W4 + x];
                    h[k] = fh::hash32_words<LEN>(w);
                }
            }
            __builtin_amdgcn_wave_barrier();
            const int c = wv + (int)(j % cnt) * NP;
            const uint32_t i = j / cnt;
            wait_ge(&cons[c], i + 1 > (uint32_t)kWsSlots ? i + 1 - kWsSlots : 0u);
            uint32_t* slot = ring[c][i % kWsSlots];
#pragma unroll
            for (int k = 0; k < KPL; k++) slot[lane + 64 * k] = h[k];
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (lane == 0) __hip_atomic_store(&prod[c], i + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            wt = wn;
        }
        return;
    }
    // consumer c: its wave-tile of every workgroup tile
    const int c = wv - NP;
    const uint32_t omask = (1u << cv.ob) - 1u, obit = 1u << cv.ob;
    const uint32_t bsh = 32u - cv.cb;
    const uint32_t rmask = (1u << bsh) - 1u;
    const __amdgpu_buffer_rsrc_t ent_r =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(cv.ent), 0, (int)cv.ent_bytes, 0x00020000);
    const bool hinted = cv.idxh != nullptr;
    const __amdgpu_buffer_rsrc_t idx_r = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint32_t*>(hinted ? cv.idxh : cv.idx), 0, (int)cv.idx_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t out_r = __builtin_amdgcn_make_buffer_rsrc(out, 0, (int)out_bytes, 0x00020000);
    auto load16 = [&](uint32_t pos) {
        return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(ent_r, (int)(3u * pos), 0, 0));
    };
    auto ent5v = [&](const u32x4 v, uint32_t (&e)[5]) {
        e[0] = v.x & 0xFFFFFFu;
        e[1] = (v.x >> 24) | ((v.y & 0xFFFFu) << 8);
        e[2] = (v.y >> 16) | ((v.z & 0xFFu) << 16);
        e[3] = v.z >> 8;
        e[4] = v.w & 0xFFFFFFu;
    };
    auto wstart = [&](uint32_t hk, uint32_t bck, uint32_t hint) -> uint32_t {
        const int fl = (int)((((hk << cv.cb) >> 24) * bck) >> 8) - 2 + (int)hint;
        return (cv.wpred && bck <= 10u && fl > 0) ? (uint32_t)fl : 0u;
    };
    auto store_row = [&](uint64_t key, uint32_t a, uint32_t b, uint32_t d) {
        const u32x3v v = {a, b, d};
        __builtin_amdgcn_raw_buffer_store_b96(v, out_r, (int)(key * 12u), 0, 2);
    };
    uint32_t i = 0;
    for (uint64_t T = blockIdx.x; T < nwg; T += gridDim.x, i++) {
        const uint64_t wt = T * NC + c;
        if (wt >= nwt) break;
        const uint64_t base = wt * TK;
        wait_ge(&prod[c], i + 1);
        uint32_t h[KPL];
        const uint32_t* slot = ring[c][i % kWsSlots];
#pragma unroll
        for (int k = 0; k < KPL; k++) h[k] = slot[lane + 64 * k];
        if (lane == 0) nsl[c] = 0;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane == 0) __hip_atomic_store(&cons[c], i + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if constexpr (ABL == 2) {
#pragma unroll
            for (int k = 0; k < KPL; k++) store_row(base + lane + 64 * k, h[k], h[k] + 1u, h[k] + 2u);
            if (lane == 0) slow_cnt[wt] = 0;
            continue;
        }
        u32x2 rec[KPL];
#pragma unroll
        for (int k = 0; k < KPL; k++)
            rec[k] = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(idx_r, (int)((h[k] >> (bsh + 3u)) * 8u), 0, 0));
        uint32_t lo[KPL], bc[KPL], ws[KPL];
        u32x4 win[KPL];
#pragma unroll
        for (int k = 0; k < KPL; k++) {
            const uint32_t s4 = ((h[k] >> bsh) & 7u) * 4u;
            const uint32_t below = rec[k].y & ((1u << s4) - 1u);
            uint32_t b0 = rec[k].x, hint = 1u;
            if (hinted) {
                const uint32_t g = h[k] >> (bsh + 3u);
                b0 = (uint32_t)(((uint64_t)g * cv.M) >> (cv.cb - 3u)) + (uint32_t)((int32_t)(rec[k].x << 18) >> 18);
                hint = (rec[k].x >> (14u + (s4 >> 1))) & 3u;
            }
            lo[k] = b0 + __builtin_amdgcn_sad_u8(below & 0x0F0F0F0Fu, 0u, __builtin_amdgcn_sad_u8((below >> 4) & 0x0F0F0F0Fu, 0u, 0u));
            bc[k] = (rec[k].y >> s4) & 15u;
            ws[k] = wstart(h[k], bc[k], hint);
            win[k] = load16(lo[k] + ws[k]);
        }
        uint32_t nag = 0;
#pragma unroll
        for (int k = 0; k < KPL; k++) {
            uint32_t e[5];
            ent5v(win[k], e);
            const uint32_t K = ((h[k] & rmask) >> cv.fsh) << cv.ob;
            const uint32_t w = ws[k];
            uint32_t lt = 0;
            bool tie = false;
#pragma unroll
            for (int j = 0; j < 5; j++) {
                const bool inb = (uint32_t)j + w < bc[k];
                lt += (inb && e[j] < K);
                tie |= (inb && e[j] - K < obit);
            }
            uint32_t r[NEED];
#pragma unroll
            for (int q = 0; q < NEED; q++) {
                uint32_t v = e[q] & omask;
#pragma unroll
                for (uint32_t d = 1; d <= SPAN; d++) v = lt == d ? (e[q + d] & omask) : v;
                r[q] = v;
            }
            const bool dup = r[0] == r[1] || r[0] == r[2] || r[1] == r[2];
            const uint32_t kk = lane + 64 * k;
            bool slow = (tie && !cv.exact) | (lo[k] + 20u > cv.M);
            const bool under = w > 0u && lt == 0u;
            const bool again = !slow && (lt > SPAN || dup || under);
            const uint64_t m = __ballot(again);
            const uint32_t pos = nag + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            nag += (uint32_t)__popcll(m);
            if (again) {
                if (pos < AG) {
                    const uint32_t b0 = under ? (w > 2u ? w - 2u : 0u) : w + 5u;
                    const bool search = under || (lt == 5u && bc[k] > w + 5u);
                    ag[c][0][pos] = lo[k] + (search ? b0 : w + lt);
                    ag[c][1][pos] = K;
                    ag[c][2][pos] = kk | (bc[k] << 12) | ((uint32_t)search << 16) | ((search ? b0 : 0u) << 17) |
                                    ((uint32_t)(under && b0 > 0u) << 21);
                } else {
                    slow = true;
                }
            }
            if (!again || pos >= AG) {
                store_row(base + kk, r[0], r[1], r[2]);
                if (counts) counts[base + kk] = (uint8_t)NEED;
            }
            if (slow) {
                const uint32_t sp = atomicAdd(&nsl[c], 1u);
                if (sp < kSlowPerTile) slow_list[wt * kSlowPerTile + sp] = kk;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        for (uint32_t j = lane; j < (nag < AG ? nag : AG); j += 64) {
            const u32x4 wn = load16(ag[c][0][j]);
            const uint32_t K = ag[c][1][j], w2 = ag[c][2][j];
            const uint32_t kk = w2 & 0xFFFu, bck = (w2 >> 12) & 15u, b0 = (w2 >> 17) & 15u;
            uint32_t e2[5];
            ent5v(wn, e2);
            uint32_t off = 0;
            bool slow = false;
            if ((w2 >> 16) & 1u) {
                bool tie = false;
#pragma unroll
                for (int j2 = 0; j2 < 5; j2++) {
                    const bool inb = (uint32_t)j2 + b0 < bck;
                    off += (inb && e2[j2] < K);
                    tie |= (inb && e2[j2] - K < obit);
                }
                slow = (tie && !cv.exact) | (off == 5u && bck > b0 + 5u) | (((w2 >> 21) & 1u) && off == 0u);
            }
            uint32_t res[4] = {NIL, NIL, NIL, NIL};
            const uint32_t rc = dedupe5(e2, off, omask, NEED, res);
            slow |= rc < (uint32_t)NEED;
            if (slow) {
                const uint32_t sp = atomicAdd(&nsl[c], 1u);
                if (sp < kSlowPerTile) slow_list[wt * kSlowPerTile + sp] = kk;
            }
            store_row(base + kk, res[0], res[1], res[2]);
            if (counts) counts[base + kk] = (uint8_t)rc;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        if (lane == 0) slow_cnt[wt] = __hip_atomic_load(&nsl[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
}

// ---- The LDS-index kernel (round 6). The lean kernel above takes two dependent L2 trips per key
// (the index record, then the window); its ablations price the index trip at 0.21 of 0.93 ms, and
// the access-pattern microbenchmark (profiles/r01c/ub_access_patterns.txt) puts one random 16-B
// load per key from a 3 MB table at 0.62 ms against 0.80 for two dependent ones. Here the index
// lives in LDS: one 768-thread workgroup per CU loads the NG group records (<= 128 KB, k_lidx_build)
// once, and each wave then streams its own tiles of 64 x KPL keys: 16-B non-temporal key loads,
// transposed through the wave's 2.3-KB LDS slice (one key per lane per slice) and hashed; the
// group record from LDS gives the bucket's first position and token count; the window is 10
// entries (32 B, two 16-B loads) from max(0, floor(u c) - 4) into the bucket (u: the key's place in
// the bucket's hash range), which holds the key's position and its NEED owners for all but ~0.45 %
// of C2 keys (a fingerprint tie: 0.43 %; a window that misses; a group with a bucket of 16+
// tokens; the ring end: the numpy emulation of the C2 ring in tools/emu_lds.py). Those
// are deferred to k_lookupn_fix_tiles (the exact tokens) through the per-tile lists, as in the
// compact kernels.
struct LdsView {
    const uint8_t* ent;  // 3 B per token (k_lpack3), M + kEnt3Pad + 6 entries (+16 B)
    const uint4* idx;    // ng group records (k_lidx_build)
    uint32_t M, ng, lg, fb, ob;
    uint32_t ent_bytes;
};
constexpr bool kLdsDefault = false;      // RP_LOOKUP_LDS=1 selects it (A/B)
constexpr int kLdsThreads = 768;          // 12 waves: one workgroup a CU (the index takes up to 128 KB)
constexpr uint32_t kLdsMaxGroups = 8192;  // 128 KB of group records

// STG 0: each lane loads its own keys (three loads per 36-B key: 16 + 16 + 4 B at a 36-B stride;
// the lines a wave touches are the same as the coalesced form's), no LDS transposition; STG 1:
// 16-B coalesced loads transposed through the wave's LDS slice (A/B: RP_LOOKUP_LDS_STG).
// ABL (diagnostics, RP_LOOKUP_LDS_ABL; results wrong, times only): 1 = no window loads (entries
// made from the group record), 2 = no LDS index read (a record made from the hash), 4 = rows not
// stored (one store of their xor per lane-tile).
template <int KPL, int NEED, int STG = 0, int ABL = 0>
__global__ __launch_bounds__(kLdsThreads) __attribute__((amdgpu_waves_per_eu(3))) void k_lookupn_lds(
    const uint8_t* __restrict__ keys, uint64_t nwt, LdsView lv, uint32_t* __restrict__ out,
    uint8_t* __restrict__ counts, uint32_t* __restrict__ slow_list, uint32_t* __restrict__ slow_cnt) {
    constexpr int LEN = 36, W4 = LEN / 4, NWV = kLdsThreads / 64;
    constexpr int TK = 64 * KPL;       // keys per wave-tile
    constexpr int V4 = TK * W4 / 4;    // 16-B key vectors per wave-tile
    constexpr int PER = V4 / 64;       // per lane
    constexpr int SV = 64 * W4 / 4;    // vectors per slice of 64 keys
    static_assert(V4 % 64 == 0 && NEED >= 1 && NEED <= 4, "tile shape");
    __shared__ uint4 s_idx[kLdsMaxGroups];
    __shared__ __attribute__((aligned(16))) uint32_t s_key[STG ? NWV : 1][64 * W4];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    for (uint32_t i = tid; i < lv.ng; i += kLdsThreads) s_idx[i] = lv.idx[i];
    __syncthreads();
    const uint32_t omask = (1u << lv.ob) - 1u, obit = 1u << lv.ob, lg = lv.lg, gsh = 32u - lv.lg;
    const uint32_t fsh = 32u - lv.fb;
    const __amdgpu_buffer_rsrc_t ent_r =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(lv.ent), 0, (int)lv.ent_bytes, 0x00020000);
    uint32_t* const sk = s_key[STG ? wv : 0];
    const uint64_t nwaves = (uint64_t)gridDim.x * NWV;
    auto nsum = [](uint32_t w, uint32_t acc) {  // the sum of w's eight nibbles, plus acc
        return __builtin_amdgcn_sad_u8(w & 0x0F0F0F0Fu, 0u, __builtin_amdgcn_sad_u8((w >> 4) & 0x0F0F0F0Fu, 0u, acc));
    };
    for (uint64_t wt = (uint64_t)blockIdx.x * NWV + wv; wt < nwt; wt += nwaves) {
        const uint64_t base = wt * TK;
        uint32_t h[KPL];
        if constexpr (STG == 0) {
            uint32_t kw[KPL][W4];
#pragma unroll
            for (int k = 0; k < KPL; k++) {
                const uint32_t* src = reinterpret_cast<const uint32_t*>(keys + (base + (uint64_t)k * 64 + lane) * LEN);
                const u32x4_a4 a = *reinterpret_cast<const u32x4_a4*>(src);
                const u32x4_a4 b = *reinterpret_cast<const u32x4_a4*>(src + 4);
                kw[k][0] = a.x; kw[k][1] = a.y; kw[k][2] = a.z; kw[k][3] = a.w;
                kw[k][4] = b.x; kw[k][5] = b.y; kw[k][6] = b.z; kw[k][7] = b.w;
                kw[k][8] = src[8];
            }
#pragma unroll
            for (int k = 0; k < KPL; k++) h[k] = fh::hash32_words<LEN>(kw[k]);
        } else {
        const u32x4* s4 = reinterpret_cast<const u32x4*>(keys + base * LEN);
        u32x4 pre[PER];
#pragma unroll
        for (int q = 0; q < PER; q++) pre[q] = __builtin_nontemporal_load(s4 + lane + 64 * q);
#pragma unroll
        for (int k = 0; k < KPL; k++) {  // slice k: keys k * 64 + lane, one per lane
#pragma unroll
            for (int q = 0; q < PER; q++) {
                const int v = (int)lane + 64 * q;
                if (v >= SV * k && v < SV * (k + 1)) reinterpret_cast<u32x4*>(sk)[v - SV * k] = pre[q];
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            uint32_t w[W4];
#pragma unroll
            for (int j = 0; j < W4; j++) w[j] = sk[lane * W4 + j];
            h[k] = fh::hash32_words<LEN>(w);
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        }
        }  // STG
        // the group records (LDS), every key's window start, both window loads in flight
        uint32_t w0[KPL], bc[KPL], sw[KPL], K[KPL];
        bool gfull[KPL];
        u32x4 wa[KPL], wb[KPL];
#pragma unroll
        for (int k = 0; k < KPL; k++) {
            const uint32_t x = h[k] << lg;
            const uint64_t t = (uint64_t)x * 28u;
            const uint32_t j = (uint32_t)(t >> 32), fr = (uint32_t)t, g = h[k] >> gsh;
            const uint4 rec = (ABL & 2) ? uint4{h[k] & 0x11111111u, h[k] & 0x22222222u, fr & 0x11111111u,
                                                (h[k] & 0x00FF1111u)}
                                        : s_idx[g];
            const uint32_t jb = 4u * j;  // the bucket's bit offset among the 112 count bits
            const uint32_t m0 = jb >= 32u ? ~0u : (1u << jb) - 1u;
            const uint32_t m1 = jb >= 64u ? ~0u : jb <= 32u ? 0u : (1u << (jb - 32u)) - 1u;
            const uint32_t m2 = jb >= 96u ? ~0u : jb <= 64u ? 0u : (1u << (jb - 64u)) - 1u;
            const uint32_t m3 = jb <= 96u ? 0u : (1u << (jb - 96u)) - 1u;
            const uint32_t below = nsum(rec.x & m0, nsum(rec.y & m1, nsum(rec.z & m2, nsum(rec.w & m3, 0u))));
            const uint32_t cw = jb < 32u ? rec.x : jb < 64u ? rec.y : jb < 96u ? rec.z : rec.w;
            const uint32_t c = (cw >> (jb & 31u)) & 15u;
            const uint32_t st = (uint32_t)(((uint64_t)g * lv.M) >> lg) + (uint32_t)((int32_t)rec.w >> 16) + below;
            const uint32_t fl = ((fr >> 24) * c) >> 8;  // about the key's position in the bucket
            const uint32_t s = fl > 4u ? fl - 4u : 0u;
            gfull[k] = (rec.w >> 16) == 0x8000u;
            w0[k] = gfull[k] ? 0u : st + s;
            sw[k] = s;
            bc[k] = c;
            K[k] = (fr >> fsh) << lv.ob;
            if constexpr ((ABL & 1) != 0) {
                wa[k] = u32x4{rec.x, rec.y, rec.z, w0[k]};
                wb[k] = u32x4{rec.w, K[k], fr, st};
            } else {
                wa[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(ent_r, (int)(3u * w0[k]), 0, 0));
                wb[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(ent_r, (int)(3u * w0[k] + 16u), 0, 0));
            }
        }
        uint32_t nsl = 0;  // wave-uniform: this wave-tile's deferred keys
        uint32_t sink = 0;
#pragma unroll
        for (int k = 0; k < KPL; k++) {
            const u32x4 a = wa[k], b = wb[k];
            const uint32_t e[10] = {a.x & 0xFFFFFFu,
                                    (a.x >> 24) | ((a.y & 0xFFFFu) << 8),
                                    (a.y >> 16) | ((a.z & 0xFFu) << 16),
                                    a.z >> 8,
                                    a.w & 0xFFFFFFu,
                                    (a.w >> 24) | ((b.x & 0xFFFFu) << 8),
                                    (b.x >> 16) | ((b.y & 0xFFu) << 16),
                                    b.y >> 8,
                                    b.z & 0xFFFFFFu,
                                    (b.z >> 24) | ((b.w & 0xFFFFu) << 8)};
            uint32_t lt = 0;  // in-bucket window entries below the key
            bool tie = false;
#pragma unroll
            for (int j = 0; j < 10; j++) {
                const bool inb = sw[k] + (uint32_t)j < bc[k];
                lt += (inb && e[j] < K[k]);
                tie |= (inb && e[j] - K[k] < obit);
            }
            uint32_t res[4] = {NIL, NIL, NIL, NIL}, rc = 0;
#pragma unroll
            for (int j = 0; j < 10; j++) {  // the first NEED distinct owners from the key's position
                const uint32_t o = e[j] & omask;
                const bool dup = (rc > 0 && o == res[0]) | (rc > 1 && o == res[1]) | (rc > 2 && o == res[2]);
                if ((uint32_t)j >= lt && !dup && rc < (uint32_t)NEED) {
                    res[0] = rc == 0 ? o : res[0];
                    res[1] = rc == 1 ? o : res[1];
                    res[2] = rc == 2 ? o : res[2];
                    res[3] = rc == 3 ? o : res[3];
                    rc++;
                }
            }
            // deferred: a tie, a group with a bucket of 16+ tokens, the key before the window (its guard entry
            // is not below it) or past it, owners not distinct inside it, the ring end
            const bool slow = tie | gfull[k] | (sw[k] > 0u && lt == 0u) | (lt == 10u) | (rc < (uint32_t)NEED) |
                              (w0[k] + 12u > lv.M);
            const uint32_t kk = (uint32_t)k * 64u + lane;
            uint32_t* row = out + (base + kk) * NEED;
            if constexpr ((ABL & 4) != 0) {
                sink ^= res[0] ^ res[1] ^ res[2] ^ res[3];
            } else {
#pragma unroll
                for (int q = 0; q < NEED; q++) __builtin_nontemporal_store(res[q], row + q);
                if (counts) counts[base + kk] = (uint8_t)NEED;
            }
            const uint64_t m = __ballot(slow);
            const uint32_t pos = nsl + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            if (slow && pos < kSlowPerTile) slow_list[wt * kSlowPerTile + pos] = kk;
            nsl += (uint32_t)__popcll(m);
        }
        if (lane == 0) slow_cnt[wt] = nsl;
        if constexpr ((ABL & 4) != 0) out[(base + lane) * NEED] = sink;
    }
}

// Exact completion of the keys the compact kernels deferred: one thread per list slot
// (kSlowPerTile per tile) redoes its key; the slots of a tile whose list overflowed share the
// whole tile. (One thread per tile, redoing its list serially, took 0.043 ms per C2 launch.)
template <class View>
__global__ __launch_bounds__(256) void k_lookupn_fix_tiles(const uint8_t* __restrict__ keys, View rv, int np,
                                                           uint32_t W, uint32_t* __restrict__ out,
                                                           uint8_t* __restrict__ counts,
                                                           const uint32_t* __restrict__ slow_list,
                                                           const uint32_t* __restrict__ slow_cnt, uint64_t ntiles,
                                                           uint32_t TK) {
    const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t t = gid / kSlowPerTile;
    const uint32_t q = (uint32_t)(gid % kSlowPerTile);
    if (t >= ntiles) return;
    // the count and the slot are independent loads (one trip); the slot is used only when q < count
    const uint32_t c = slow_cnt[t];
    const uint32_t kq = slow_list[t * kSlowPerTile + q];
    if (c == 0) return;
    auto redo = [&](uint64_t k) { lookupn_redo(keys, rv, np, W, out, counts, k); };
    if (c <= kSlowPerTile) {
        if (q < c) lookupn_redo(keys, rv, np, W, out, counts, t * TK + kq);
    } else {
        for (uint32_t k = q; k < TK; k += kSlowPerTile) redo(t * TK + k);
    }
}

// Exact completion of the keys k_lookupn_probe / k_lookupn_compact deferred (same stream, so it
// sees the list and overwrites those rows): binary search in the bucket + the reference walk.
template <int LEN, int MODE = 0, class View = PackedView>
__global__ __launch_bounds__(256) void k_lookupn_fix(const uint8_t* __restrict__ keys, View rv, int np,
                                                     uint32_t W, uint32_t* __restrict__ out,
                                                     uint8_t* __restrict__ counts,
                                                     const uint32_t* __restrict__ slow,
                                                     const uint32_t* __restrict__ nslow) {
    const uint32_t total = *nslow;
    const uint32_t gstride = gridDim.x * blockDim.x;
    for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < total; s += gstride) {
        const uint64_t k = slow[s];
        uint32_t w[LEN / 4];
        const uint32_t* src = reinterpret_cast<const uint32_t*>(keys + k * LEN);
#pragma unroll
        for (int j = 0; j < LEN / 4; j++) w[j] = src[j];
        const uint32_t h = fh::hash32_words<LEN>(w);
        const uint32_t i = rv.find(h);
        uint32_t res[4];
        int c;
        if constexpr (MODE == 2) {
            res[0] = i; res[1] = i + 1; res[2] = i + 2; res[3] = i + 3;
            c = 1;
        } else {
            c = ring_walk<4>(rv, i, np, res);
        }
        uint32_t* row = out + k * W;
#pragma unroll
        for (int q = 0; q < 4; q++)
            if ((uint32_t)q < W) row[q] = res[q];
        if (counts) counts[k] = (uint8_t)c;
    }
}

// Generic keys: per-thread byte fetches (variable length via uint64 offsets, or any stride),
// or precomputed hashes (hashes != null).
template <int MAXN, class View>
__global__ __launch_bounds__(kLkThreads) void k_lookupn_generic(const uint8_t* __restrict__ keys,
                                                                const uint64_t* __restrict__ off,
                                                                uint32_t stride,
                                                                const uint32_t* __restrict__ hashes,
                                                                uint64_t n, View rv, int np, uint32_t W,
                                                                uint32_t* __restrict__ out,
                                                                uint8_t* __restrict__ counts) {
    const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gstride) {
        uint32_t h;
        if (hashes) {
            h = hashes[k];
        } else {
            uint64_t b, e;
            if (stride) {
                b = k * stride;
                e = b + stride;
            } else {
                b = off[k];
                e = off[k + 1];
            }
            h = fh::hash32(fh::PtrSrc{keys + b}, (uint32_t)(e - b));
        }
        const uint32_t i = rv.find(h);
        uint32_t* row = out + k * W;
        int c;
        if constexpr (MAXN > 0) {
            uint32_t res[MAXN];
            c = ring_walk<MAXN>(rv, i, np, res);
#pragma unroll
            for (int q = 0; q < MAXN; q++)
                if ((uint32_t)q < W) row[q] = res[q];
            for (uint32_t q = MAXN; q < W; q++) row[q] = NIL;
        } else {
            c = ring_walk_global(rv, i, np, row, W);
        }
        if (counts) counts[k] = (uint8_t)(c > 255 ? 255 : c);
    }
}

// Small host batches (the drop-in's one-key lookup / lookupN calls, index.js:434-471): the keys
// travel in the kernel arguments and the rows go straight to pinned host memory, so a call is
// one launch and one stream sync instead of two copies each way (host_lookup).
constexpr uint32_t kSmallKeys = 64, kSmallBytes = 3072, kSmallW = 16;
struct SmallKeys {
    uint32_t n;
    uint16_t off[kSmallKeys + 1];
    uint8_t b[kSmallBytes];
};
template <int MAXN, class View>
__global__ __launch_bounds__(64) void k_lookupn_small(const SmallKeys sk, View rv, int np, uint32_t W,
                                                      uint32_t* __restrict__ out, uint8_t* __restrict__ counts) {
    __shared__ uint8_t kb[kSmallBytes];
    const uint32_t k = threadIdx.x, nb = sk.off[sk.n];
    for (uint32_t i = k; i < nb; i += 64) kb[i] = sk.b[i];
    __syncthreads();
    if (k >= sk.n) return;
    const uint32_t b = sk.off[k], e = sk.off[k + 1];
    const uint32_t i = rv.find(fh::hash32(fh::PtrSrc{kb + b}, e - b));
    uint32_t res[MAXN];
    const int c = ring_walk<MAXN>(rv, i, np, res);
    for (uint32_t q = 0; q < W; q++) out[k * W + q] = q < (uint32_t)MAXN ? res[q] : NIL;
    if (counts) counts[k] = (uint8_t)(c > 255 ? 255 : c);
}

// The lookup service (rp_ring_service): one resident wave answers single-key lookup / lookupN
// calls (RingPop.lookup per request, index.js:434-451) through pinned, device-mapped host lines,
// so a call costs the PCIe round trips instead of a launch and a stream sync. Request: a header
// line {seq, len, np, W, stop} and up to kSvcChunks key lines of 60 B + their copy of seq in the
// last dword (the host writes a line's bytes before its seq, so a line read with the expected
// seq holds the new bytes). Response: owners + count, then seq in its own line, released at
// system scope. The wave exits on the stop flag, after idle_ticks of no request, or after
// max_ticks in all (s_memrealtime, 100 MHz), so it always drains; the host relaunches it when a
// request finds it gone.
constexpr uint32_t kSvcChunks = 3, kSvcKeyMax = kSvcChunks * 60;
constexpr uint32_t kSvcWaves = 8;     // k_lookup_service3's independent pollers (RP_SVC_WAVES)
constexpr uint32_t kSvcPeriod = 120;  // their common poll period, 100 MHz ticks (RP_SVC_PERIOD)
struct SvcLines {
    uint32_t req[16 * (1 + kSvcChunks)];  // header line + key lines
    uint32_t resp[16];                    // owners[0..W), count at [15]
    uint32_t resp_seq[16];                // [0] = the answered seq
    uint64_t resp2[8][8];                 // k_lookup_service3: slot seq % 8, owner q | seq << 32 (64-B lines)
    uint32_t diag[16];                    // k_lookup_service3 with prof: seq, then phase ticks (100 MHz)
};
// With the compact layout built, a key with 1..4 owners wanted takes compact_fix_walk (the
// index record, the bucket's tokens, the next 8 owners: three dependent trips) instead of the
// wide binary search and walk.
template <class View>
__global__ __launch_bounds__(64) void k_lookup_service(SvcLines* io, View rv, CompactFixView fv, uint32_t use_compact,
                                                       uint32_t last, uint64_t idle_ticks, uint64_t max_ticks) {
    __shared__ uint32_t kw[kSvcChunks * 15];
    const uint32_t lane = threadIdx.x;
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
    uint64_t t_idle = t_start;
    while (true) {
        const uint32_t v = lane < 16 * (1 + kSvcChunks)
                               ? __hip_atomic_load(&io->req[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                               : 0u;
        const uint32_t seq = __builtin_amdgcn_readfirstlane(__shfl(v, 0, 64));
        const uint32_t stop = __builtin_amdgcn_readfirstlane(__shfl(v, 4, 64));
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        if (stop || now - t_start > max_ticks) break;
        if (seq == last) {
            if (now - t_idle > idle_ticks) break;
            __builtin_amdgcn_s_sleep(2);
            continue;
        }
        const uint32_t len = __builtin_amdgcn_readfirstlane(__shfl(v, 1, 64));
        const int np = (int)__builtin_amdgcn_readfirstlane(__shfl(v, 2, 64));
        const uint32_t W = __builtin_amdgcn_readfirstlane(__shfl(v, 3, 64));
        const uint32_t nch = (len + 59) / 60;
        // every key line the request uses must carry this seq (else re-read)
        const bool line_ok = lane < 16 || (lane >> 4) > nch || (lane & 15) != 15 || v == seq;
        if (__ballot(!line_ok) != 0 || len > kSvcKeyMax || W > 16) {
            if (len > kSvcKeyMax || W > 16) {  // malformed: answer empty
                if (lane < 16) __hip_atomic_store(&io->resp[lane], lane == 15 ? 0u : NIL, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_SYSTEM);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
                if (lane == 0) __hip_atomic_store(&io->resp_seq[0], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
                last = seq;
                t_idle = now;
            }
            continue;
        }
        if (lane >= 16 && (lane & 15) < 15) kw[((lane >> 4) - 1) * 15 + (lane & 15)] = v;
        __syncthreads();
        uint32_t res[8] = {NIL, NIL, NIL, NIL, NIL, NIL, NIL, NIL};
        int c = 0;
        if (lane == 0) {
            const uint32_t hk = fh::hash32(fh::PtrSrc{reinterpret_cast<const uint8_t*>(kw)}, len);
            if (use_compact && np >= 1 && np <= 4) {
                uint32_t r4[4];
                c = compact_fix_walk(fv, hk, np, r4);
#pragma unroll
                for (int q = 0; q < 4; q++) res[q] = r4[q];
            } else {
                c = ring_walk<8>(rv, rv.find(hk), np > 8 ? 8 : np, res);
            }
        }
        // lane 0's row to lanes 0..W-1, then the seq after it (system-scope release)
        uint32_t mine = NIL;
#pragma unroll
        for (uint32_t q = 0; q < 8; q++) {
            const uint32_t x = __shfl(res[q], 0, 64);
            mine = lane == q ? x : mine;
        }
        const uint32_t cnt = (uint32_t)__shfl(c, 0, 64);
        if (lane < 16) __hip_atomic_store(&io->resp[lane], lane == 15 ? cnt : (lane < W ? mine : NIL), __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_SYSTEM);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        if (lane == 0) __hip_atomic_store(&io->resp_seq[0], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        __syncthreads();
        last = seq;
        t_idle = __builtin_amdgcn_s_memrealtime();
    }
}

// One key on the compact layout in two dependent trips (the index record, one 5-entry window at
// the predicted start, as k_lookupn_lean): true with the first `need` distinct owners when window 1
// holds them; false when the key needs more (a fingerprint tie, a long bucket, the ring end, a
// position or repeated owners past the window), and the caller takes the exact walk.
__device__ __forceinline__ bool svc_compact_window(const CompactView& cv, uint32_t h, int need, uint32_t (&res)[4],
                                                   int& cnt) {
    const uint32_t bsh = 32u - cv.cb;
    const uint32_t g = h >> (bsh + 3u), s4 = ((h >> bsh) & 7u) * 4u;
    const u32x2 rec = *reinterpret_cast<const u32x2*>(cv.idx + 2ull * g);
    const uint32_t below = rec.y & ((1u << s4) - 1u);
    const uint32_t x = (below & 0x0F0F0F0Fu) + ((below >> 4) & 0x0F0F0F0Fu);
    const uint32_t lo = rec.x + ((x * 0x01010101u) >> 24);
    const uint32_t bc = (rec.y >> s4) & 15u;
    if (bc > 10u || lo + 20u > cv.M) return false;
    const uint32_t fl = (((h << cv.cb) >> 24) * bc) >> 8;
    const uint32_t w = (need >= 2 && fl > 1u) ? fl - 1u : 0u;
    const u32x4_a1 v = *reinterpret_cast<const u32x4_a1*>(cv.ent + 3ull * (lo + w));
    const uint32_t e[5] = {v.x & 0xFFFFFFu, (v.x >> 24) | ((v.y & 0xFFFFu) << 8), (v.y >> 16) | ((v.z & 0xFFu) << 16),
                           v.z >> 8, v.w & 0xFFFFFFu};
    const uint32_t omask = (1u << cv.ob) - 1u, obit = 1u << cv.ob;
    const uint32_t K = ((h & ((1u << bsh) - 1u)) >> cv.fsh) << cv.ob;
    uint32_t lt = 0;
    bool tie = false;
#pragma unroll
    for (int j = 0; j < 5; j++) {
        const bool inb = (uint32_t)j + w < bc;
        lt += (inb && e[j] < K);
        tie |= (inb && e[j] - K < obit);
    }
    if ((tie && !cv.exact) || (w > 0u && lt == 0u)) return false;
    const uint32_t rc = dedupe5(e, lt, omask, (uint32_t)need, res);
    if (rc < (uint32_t)need) return false;
    cnt = (int)rc;
    return true;
}

// The service's direct table (round 5): one 64-B record per bucket of the top B hash bits (2^B >= M,
// B >= 16, so the bucket fixes all but <= 16 token bits and a record answers exactly, no
// fingerprints), read as one aligned line: the lookup is one dependent trip instead of the compact
// layout's two. Record words:
//   [0]     token count c (<= 7; 15: more, the caller takes the other paths) | successors s << 8 |
//           complete << 16 (s < 16 only because the ring has fewer distinct owners)
//   [1..7]  the bucket's tokens in ring order: low 32 - B bits | owner << 16
//   [8..15] the first 16 distinct owners from the first token after the bucket onwards (cyclic),
//           two 16-bit ids a word
// lookupN(h, n <= 8) = the first n distinct of (owners of the bucket's tokens >= h, then the
// successors): the successors are the distinct owners of the rest of the walk in first-seen order,
// so deduplicating the concatenation gives the walk's answer (lib/ring/index.js:157-189). Only
// for rings whose interned ids fit 16 bits. tools/svc_latency.js prices it (r05w).
constexpr uint32_t kDtEnt = 7, kDtSucc = 16, kDtWalk = 4096;
__global__ __launch_bounds__(256) void k_dt_build(const uint32_t* __restrict__ tok, const uint32_t* __restrict__ own,
                                                  uint32_t M, uint32_t B, uint4* __restrict__ dt) {
    const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >> B) return;
    const uint32_t sh = 32u - B;
    auto lower = [&](uint64_t key) {  // first i with tok[i] >= key
        uint32_t lo = 0, hi = M;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if ((uint64_t)tok[mid] < key) lo = mid + 1;
            else hi = mid;
        }
        return lo;
    };
    const uint32_t lo = lower(b << sh), hi = lower((b + 1) << sh);
    const uint32_t c = hi - lo;
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 16; i++) w[i] = 0xFFFFFFFFu;
    if (c > kDtEnt) {
        w[0] = 15u;
    } else {
        for (uint32_t i = 0; i < c; i++) w[1 + i] = (tok[lo + i] & ((1u << sh) - 1u)) | (own[lo + i] << 16);
        uint32_t su[kDtSucc], ns = 0, k = 0;
        const uint32_t lim = M < kDtWalk ? M : kDtWalk;
        for (; k < lim && ns < kDtSucc; k++) {
            const uint32_t j = hi + k >= M ? hi + k - M : hi + k;
            const uint32_t o = own[j];
            bool seen = false;
            for (uint32_t q = 0; q < ns; q++) seen |= su[q] == o;
            if (!seen) su[ns++] = o;
        }
        const uint32_t complete = (ns < kDtSucc && k == M) ? 1u : 0u;
        w[0] = c | (ns << 8) | (complete << 16);
        for (uint32_t q = 0; q < kDtSucc; q += 2)
            w[8 + q / 2] = (q < ns ? su[q] : 0xFFFFu) | ((q + 1 < ns ? su[q + 1] : 0xFFFFu) << 16);
    }
    uint4* d = dt + 4 * b;
#pragma unroll
    for (int q = 0; q < 4; q++) d[q] = uint4{w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]};
}

// The answer from a record, across the wave: lane i < 16 holds record word i (x). Lane i takes
// item i of (owners of the bucket's tokens >= h, then the successors), flags it when no earlier
// item has its owner, and the flagged items' ranks are their slots. Returns false (wave-uniform)
// when the record cannot say (an overflowing bucket, too few successors); else cnt and, in lane
// q < 8, the q-th owner (NIL past cnt).
__device__ __forceinline__ bool dt_answer(uint32_t x, uint32_t lane, uint32_t h, uint32_t B, uint32_t need,
                                          uint32_t* slot, uint32_t& mine, int& cnt) {
    const uint32_t w0 = __builtin_amdgcn_readfirstlane(x);
    const uint32_t c = w0 & 15u, ns = (w0 >> 8) & 31u, complete = (w0 >> 16) & 1u;
    if (c > kDtEnt) return false;
    const uint32_t rmask = (1u << (32u - B)) - 1u, hr = h & rmask;
    const uint32_t e = __shfl(x, 1 + (lane < kDtEnt ? lane : 0), 64);
    const uint32_t f = (uint32_t)__popcll(__ballot(lane < c && (e & 0xFFFFu & rmask) < hr));  // tokens below h
    const uint32_t na = c - f;
    const uint32_t ea = __shfl(x, 1 + f + (lane < na ? lane : 0), 64);
    const uint32_t k = lane - na;
    const uint32_t sw = __shfl(x, 8 + ((lane >= na && k < kDtSucc ? k : 0) >> 1), 64);
    const bool valid = lane < na || (lane >= na && k < ns);
    const uint32_t t = lane < na ? (ea >> 16) : ((sw >> (16 * (k & 1))) & 0xFFFFu);
    bool dup = false;
#pragma unroll
    for (uint32_t j = 0; j < kDtEnt + kDtSucc; j++) {
        const uint32_t tj = __builtin_amdgcn_readlane(t, j);
        dup |= j < lane && tj == t;
    }
    const uint64_t fb = __ballot(valid && !dup);
    const uint32_t total = (uint32_t)__popcll(fb);
    if (total < need && !complete) return false;
    const uint32_t rank = (uint32_t)__popcll(fb & ((1ull << lane) - 1ull));
    if (valid && !dup && rank < 8) slot[rank] = t;
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the slots are written (one wave: no barrier)
    __builtin_amdgcn_wave_barrier();
    const uint32_t got = total < need ? total : need;
    mine = lane < got ? slot[lane] : NIL;
    cnt = (int)got;
    return true;
}

// dt_answer without LDS (round 6, the default; RP_SVC_ANS=0 keeps dt_answer): the items stay where
// the record puts them, in item order by lane (the bucket's tokens >= h in lanes 1..c, the
// successors spread to lanes 16..31 by one shuffle), and the first `need` distinct owners are
// taken one at a time: the first remaining lane's owner, then every lane holding it dropped by a
// ballot. A lookup (need 1) is one step; no 23-step duplicate scan, no LDS slots.
__device__ __forceinline__ bool dt_answer_fast(uint32_t x, uint32_t lane, uint32_t h, uint32_t B, uint32_t need,
                                               uint32_t& mine, int& cnt) {
    const uint32_t w0 = __builtin_amdgcn_readlane(x, 0);
    const uint32_t c = w0 & 15u, ns = (w0 >> 8) & 31u, complete = (w0 >> 16) & 1u;
    if (c > kDtEnt) return false;
    const uint32_t rmask = (1u << (32u - B)) - 1u, hr = h & rmask;
    const uint32_t k = lane - 16u;
    const bool sl = lane >= 16u && k < kDtSucc;
    const uint32_t sw = __shfl(x, 8u + ((sl ? k : 0u) >> 1), 64);
    const bool tk = lane >= 1u && lane <= c && (x & 0xFFFFu & rmask) >= hr;
    const bool su = sl && k < ns;
    const uint32_t t = tk ? (x >> 16) : ((sw >> (16u * (k & 1u))) & 0xFFFFu);
    uint64_t rem = __ballot(tk || su);
    uint32_t got = 0;
    mine = NIL;
    while (got < need && rem) {
        const uint32_t v = __builtin_amdgcn_readlane(t, (uint32_t)__builtin_ctzll(rem));
        mine = lane == got ? v : mine;
        rem &= ~__ballot(t == v);
        got++;
    }
    if (got < need && !complete) return false;
    cnt = (int)got;
    return true;
}

// The lookup service, round 5 form (RP_RING_SVC=2, the default). Round 5 measured the round-4
// kernel's call (5.0 us in node) with device stamps (RP_SVC_PROF): the poll's PCIe round trip
// ~1.1 us, the key's farmhash on one lane from LDS ~0.5 us, three dependent table trips, the
// answer's line and its seq line. A three-wave form (a poller with 8 reads in flight, a worker,
// an L2-warming wave) was slower (6.0 us): the poller's PCIe reads in flight delayed the worker's
// table loads on the same CU (lookup 1.4 us at 1 read in flight, 2.8 at 8) and the LDS hand-off
// cost 0.4 us. So this form is one wave again, and:
//   - the host hashes the key (farmhash32, as the reference's lookup does on the CPU) and sends
//     {seq, hash, np, W, stop, ..., seq} in one 64-B header line: no key lines, no device hash,
//     and no key-length limit;
//   - one poll in flight, and nothing else outstanding when a request is seen;
//   - the compact layout answers in two trips (svc_compact_window: the index record and one
//     window), the exact walk otherwise;
//   - the answer is one 64-B line of 8 words {owner | seq << 32} (no fence, no second line: the
//     host takes the line when every word carries its seq);
//   - RP_SVC_WARM=1: while idle, after each poll is issued, the wave touches 32 KB of the compact
//     tables (the whole 3.5 MB about every 0.15 ms) to keep them in its XCD's L2. Measured without
//     effect on the lookup's two trips (1.08 us either way, r05g) and 0.1 us slower polls: off.
// Round 6: the wait for a request is the poll's phase, on average half a PCIe round trip before
// the read that sees the line plus the return. So the service is kSvcWaves independent waves of
// this same loop, one workgroup each (so on different CUs and XCDs, none delaying another's table
// read), each with its one poll in flight at its own phase: the first to see a request answers
// it, the later ones answer it again with the same line (a pure function of the request), and no
// wave waits on another. The answer goes to line seq % 8, so a late duplicate can only land on
// the line of a request eight calls old, never on the one the host is waiting for.
// RP_SVC_PROF=1 writes per-call device phase ticks into diag (poll round trip, lookup).
template <class View>
__global__ __launch_bounds__(64) void k_lookup_service3(SvcLines* io, View rv, CompactFixView fv, CompactView cv,
                                                       uint32_t use_compact, uint32_t last, uint64_t idle_ticks,
                                                       uint64_t max_ticks, uint32_t warm, uint32_t prof,
                                                       const uint32_t* __restrict__ dt, uint32_t dtb,
                                                       uint32_t period, uint32_t ans_old) {
    __shared__ uint32_t dslot[8];
    const uint32_t lane = threadIdx.x;
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
    uint64_t t_idle = t_start;
    const uint64_t nidx = cv.idx_bytes, nwarm = nidx + cv.ent_bytes;
    uint64_t woff = 0;
    uint32_t acc = 0;
    // period > 0 (several waves): wave i issues its polls on the device clock's slots
    // n * period + i * period / waves, so the waves' reads reach the host line evenly spread
    // instead of in step (launched together, they would otherwise poll at one phase)
    uint64_t slot = period ? (t_start / period + 1) * period + (uint64_t)blockIdx.x * period / gridDim.x : 0;
    while (true) {
        if (period) {
            while (__builtin_amdgcn_s_memrealtime() < slot) __builtin_amdgcn_s_sleep(1);
            const uint64_t t = __builtin_amdgcn_s_memrealtime();
            do slot += period;
            while (slot <= t);
        }
        if (warm == 2 && dt) {  // this wave's slice of the direct table, a record a lane per poll, issued
            // before the poll (loads return in order: one behind the poll would hold up the lookup's)
            const uint64_t nrec = 1ull << dtb, r0 = nrec * blockIdx.x / gridDim.x, r1 = nrec * (blockIdx.x + 1) / gridDim.x;
            const uint64_t r = r0 + woff + lane;
            acc ^= r < r1 ? dt[16ull * r] : 0u;
            woff = r0 + woff + 64 >= r1 ? 0 : woff + 64;
        }
        const uint64_t tp = __builtin_amdgcn_s_memrealtime();
        const uint32_t v = lane < 16 ? __hip_atomic_load(&io->req[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0u;
        if (warm == 1 && use_compact) {  // issued after the poll, done within its round trip
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const uint64_t o = woff + 64ull * lane;
                const uint32_t x = o < nidx ? cv.idx[o >> 2]
                                   : o + 4 <= nwarm ? *reinterpret_cast<const uint32_t*>(cv.ent + ((o - nidx) & ~3ull))
                                                    : 0u;
                acc ^= x;
                woff = woff + 4096 >= nwarm ? 0 : woff + 4096;
            }
        }
        const uint32_t seq = __builtin_amdgcn_readlane(v, 0);  // (register reads, no LDS trip)
        const uint32_t stop = __builtin_amdgcn_readlane(v, 4);
        const uint32_t tail = __builtin_amdgcn_readlane(v, 15);
        if (prof) asm volatile("s_waitcnt vmcnt(0)" ::"s"(seq) : "memory");  // (stamps) the clock after the poll
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        if (stop || now - t_start > max_ticks) break;
        if (seq == last || tail != seq) {
            if (seq == last && now - t_idle > idle_ticks) break;
            __builtin_amdgcn_s_sleep(2);
            continue;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the warm load, before the lookup's own
        asm volatile("" ::"v"(acc));
        const uint32_t hk = __builtin_amdgcn_readlane(v, 1);
        const int np = (int)__builtin_amdgcn_readlane(v, 2);
        const uint32_t W = __builtin_amdgcn_readlane(v, 3);
        uint32_t res[8] = {NIL, NIL, NIL, NIL, NIL, NIL, NIL, NIL};
        uint32_t path = 0;
        bool dok = false;
        uint32_t dmine = NIL;
        if (dt && np >= 1 && np <= 8) {  // the direct table: one 64-B line, lanes 0..15
            const uint32_t x = lane < 16 ? dt[16ull * (hk >> (32u - dtb)) + lane] : 0u;
            int c = 0;
            dok = ans_old ? dt_answer(x, lane, hk, dtb, (uint32_t)np, dslot, dmine, c)
                          : dt_answer_fast(x, lane, hk, dtb, (uint32_t)np, dmine, c);
            path = dok ? 4u : 0u;
        }
        uint32_t o = dmine;
        if (!dok) {  // (wave-uniform) the compact window or the walks, on lane 0
            if (lane == 0) {
                bool ok = false;
                if (use_compact && np >= 1 && np <= 4) {
                    uint32_t r4[4] = {NIL, NIL, NIL, NIL};
                    int c = 0;
                    ok = svc_compact_window(cv, hk, np, r4, c);
                    path = ok ? 1u : 2u;
                    if (!ok) {
                        c = compact_fix_walk(fv, hk, np, r4);
                        ok = true;
                    }
#pragma unroll
                    for (int q = 0; q < 4; q++) res[q] = r4[q];
                }
                if (!ok) {
                    ring_walk<8>(rv, rv.find(hk), np > 8 ? 8 : np, res);
                    path = 3;
                }
            }
#pragma unroll
            for (uint32_t q = 0; q < 8; q++) {
                const uint32_t x = __shfl(res[q], 0, 64);
                o = lane == q ? x : o;
            }
        }
        if (prof) {  // diag: seq, poll round trip, lookup (ticks), path
            asm volatile("" ::"v"(o));
            const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
            const uint32_t pth = (uint32_t)__shfl(path, 0, 64);
            const uint32_t d[4] = {seq, (uint32_t)(now - tp), (uint32_t)(t1 - now), pth};
            uint32_t dv = 0;
#pragma unroll
            for (int q = 0; q < 4; q++) dv = lane == (uint32_t)q ? d[q] : dv;
            if (lane < 4) __hip_atomic_store(&io->diag[lane], dv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        if (lane < 8)
            __hip_atomic_store(&io->resp2[seq & 7u][lane], (uint64_t)(lane < W ? o : NIL) | ((uint64_t)seq << 32),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        last = seq;
        t_idle = __builtin_amdgcn_s_memrealtime();
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("" ::"v"(acc));
}

// ---- build kernels ----

// tokens[a*R + i] = farmhash32(name(ids[a]) + String(i)); owners likewise = ids[a].
__global__ void k_replica_tokens(const uint8_t* __restrict__ names, const uint64_t* __restrict__ noff,
                                 const uint32_t* __restrict__ ids, uint32_t n_srv, uint32_t R,
                                 uint32_t* __restrict__ tok, uint32_t* __restrict__ own) {
    const uint64_t total = (uint64_t)n_srv * R;
    const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < total; k += gstride) {
        const uint32_t a = (uint32_t)(k / R), i = (uint32_t)(k % R);
        const uint32_t id = ids[a];
        fh::ReplicaSrc s;
        s.name = names + noff[id];
        s.nlen = (uint32_t)(noff[id + 1] - noff[id]);
        const uint32_t nd = fh::decimal(i, s.dig);
        tok[k] = fh::hash32(s, s.nlen + nd);
        own[k] = id;
    }
}

// owners for caller-supplied tokens
__global__ void k_expand_owner(const uint32_t* __restrict__ ids, uint32_t n_srv, uint32_t R,
                               uint32_t* __restrict__ own) {
    const uint64_t total = (uint64_t)n_srv * R;
    const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < total; k += gstride)
        own[k] = ids[k / R];
}

__device__ __forceinline__ uint32_t lower_bound_dev(const uint32_t* a, uint32_t n, uint32_t v) {
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        uint32_t mid = (lo + hi) >> 1;
        if (a[mid] < v) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// keep sorted-new token p iff first of its equal run (stable sort => first inserted) and
// absent from the live ring (insert-if-absent, rbtree.js:112-116).
__global__ void k_mark_new(const uint32_t* __restrict__ ntok, uint32_t K, const uint32_t* __restrict__ tok,
                           uint32_t M, uint32_t* __restrict__ flag) {
    const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < K; p += gstride) {
        const uint32_t t = ntok[p];
        bool keep = (p == 0) || (ntok[p - 1] != t);
        if (keep && M) {
            const uint32_t i = lower_bound_dev(tok, M, t);
            keep = !(i < M && tok[i] == t);
        }
        flag[p] = keep ? 1u : 0u;
    }
}

__global__ void k_compact_pairs(const uint32_t* __restrict__ kin, const uint32_t* __restrict__ vin,
                                const uint32_t* __restrict__ flag, const uint32_t* __restrict__ pos,
                                uint32_t n, uint32_t* __restrict__ kout, uint32_t* __restrict__ vout) {
    const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += gstride)
        if (flag[p]) {
            kout[pos[p]] = kin[p];
            vout[pos[p]] = vin[p];
        }
}

// Merge two sorted, mutually disjoint token arrays (rank = own index + rank in the other).
__global__ void k_merge(const uint32_t* __restrict__ at, const uint32_t* __restrict__ ao, uint32_t na,
                        const uint32_t* __restrict__ bt, const uint32_t* __restrict__ bo, uint32_t nb,
                        uint32_t* __restrict__ ot, uint32_t* __restrict__ oo) {
    const uint64_t total = (uint64_t)na + nb;
    const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < total; p += gstride) {
        if (p < na) {
            const uint32_t t = at[p];
            const uint32_t d = (uint32_t)p + lower_bound_dev(bt, nb, t);
            ot[d] = t;
            oo[d] = ao[p];
        } else {
            const uint32_t q = (uint32_t)(p - na);
            const uint32_t t = bt[q];
            const uint32_t d = q + lower_bound_dev(at, na, t);
            ot[d] = t;
            oo[d] = bo[q];
        }
    }
}

// erase-by-key (rbtree.js:152-232): mark every live token equal to a removal token.
__global__ void k_mark_del(const uint32_t* __restrict__ rtok, uint64_t K, const uint32_t* __restrict__ tok,
                           uint32_t M, uint32_t* __restrict__ keep) {
    const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < K; p += gstride) {
        const uint32_t t = rtok[p];
        const uint32_t i = lower_bound_dev(tok, M, t);
        if (i < M && tok[i] == t) keep[i] = 0u;
    }
}

__global__ void k_fill_u32(uint32_t* p, uint64_t n, uint32_t v) {
    const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gstride) p[i] = v;
}

__global__ void k_bucket_index(const uint32_t* __restrict__ tok, uint32_t M, uint32_t bbits,
                               uint32_t* __restrict__ bstart) {
    const uint64_t nbk = (1ull << bbits);
    const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b <= nbk; b += gstride) {
        if (b == nbk) bstart[b] = M;
        else bstart[b] = lower_bound_dev(tok, M, (uint32_t)(b << (32 - bbits)));
    }
}

__global__ void k_pack(const uint32_t* __restrict__ tok, const uint32_t* __restrict__ own, uint32_t M,
                       uint32_t B, uint32_t* __restrict__ ent) {
    const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < (uint64_t)M + kEntPad; j += gstride)
        ent[j] = j < M ? ((tok[j] << B) | own[j]) : 0xFFFFFFFFu;
}

// compact entries: 3 bytes per token, (fp << ob) | owner; padding entries are all ones
__global__ void k_pack3(const uint32_t* __restrict__ tok, const uint32_t* __restrict__ own, uint32_t M,
                        uint32_t cb, uint32_t ob, uint32_t fsh, uint8_t* __restrict__ ent) {
    const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
    const uint32_t rmask = cb == 0 ? 0xFFFFFFFFu : ((1u << (32u - cb)) - 1u);
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < (uint64_t)M + kEnt3Pad + 6; j += gstride) {
        const uint32_t v = j < M ? ((((tok[j] & rmask) >> fsh) << ob) | own[j]) : 0xFFFFFFu;
        ent[3 * j + 0] = (uint8_t)v;
        ent[3 * j + 1] = (uint8_t)(v >> 8);
        ent[3 * j + 2] = (uint8_t)(v >> 16);
    }
}

// compact index: per group of 8 buckets {first position, 8 x 4-bit counts}; *over is set when a
// bucket holds more than 15 tokens (the layout is then not used)
__global__ void k_cindex(const uint32_t* __restrict__ bst, uint32_t ngroups, uint32_t* __restrict__ idx,
                         uint32_t* __restrict__ over) {
    const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < ngroups; g += gstride) {
        uint32_t nib = 0;
        bool bad = false;
#pragma unroll
        for (int s = 0; s < 8; s++) {
            const uint32_t c = bst[g * 8 + s + 1] - bst[g * 8 + s];
            bad |= c > 15u;
            nib |= (c > 15u ? 15u : c) << (4 * s);
        }
        idx[2 * g] = bst[g * 8];
        idx[2 * g + 1] = nib;
        if (bad) atomicOr(over, 1u);
    }
}

// The hinted index of the lean kernel's lookupN(3) (round 5): per group g of 8 buckets,
// x = (base - pred(g)) & 0x3FFF | hints << 14 and y = the nibble counts (as k_cindex), pred(g) =
// g * M >> (cb - 3). Bucket s's 2-bit hint h moves window 1's start to max(0, fl - 1 + h - 1)
// (fl = the key's 8 top residual bits x count >> 8, the lean kernel's prediction): of the three,
// the start whose window resolves the largest share of the bucket's hash range (a key whose
// position in the bucket is rel resolves at w = 0 when rel <= 2, at w > 0 when rel is w + 1 or
// w + 2). Buckets of more than 10 tokens keep w = 0 (hint 1). over |= 1 when a base delta does
// not fit 14 bits (the lean kernel then runs without hints).
__global__ void k_cindex_hint(const uint32_t* __restrict__ tok, const uint32_t* __restrict__ bst, uint32_t M,
                              uint32_t cb, uint32_t ngroups, uint32_t* __restrict__ idx, uint32_t* __restrict__ over) {
    const uint32_t bsh = 32u - cb;
    const uint32_t qsh = bsh - 8u;  // residual >> qsh = the 8 bits the kernel's prediction reads
    const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < ngroups; g += gstride) {
        const uint32_t base = bst[g * 8];
        const int64_t delta = (int64_t)base - (int64_t)(((uint64_t)g * M) >> (cb - 3));
        if (delta < -8192 || delta > 8191) atomicOr(over, 1u);
        uint32_t nib = 0, hints = 0;
        for (int s = 0; s < 8; s++) {
            const uint32_t lo = bst[g * 8 + s], bc = bst[g * 8 + s + 1] - lo;
            nib |= (bc > 15u ? 15u : bc) << (4 * s);
            uint32_t best = 1;
            if (bc <= 10u) {
                // resolved length of the hash range for each hint, walking the 256 prediction
                // slices and the bucket's token residuals in order
                uint64_t g0 = 0, g1 = 0, g2 = 0;  // resolved lengths for hints 0, 1, 2
                uint32_t j = 0;  // tokens below the slice start
                const uint64_t S = 1ull << qsh;
                for (uint32_t q = 0; q < 256; q++) {
                    const uint32_t fl = (q * bc) >> 8;
                    uint64_t a = (uint64_t)q * S;
                    const uint64_t e = a + S;
                    uint32_t rel = j;
                    while (true) {
                        // [a, nxt) has position rel
                        const uint64_t tn = rel < bc ? (uint64_t)(tok[lo + rel] & ((1u << bsh) - 1u)) + 1ull : e;
                        const uint64_t nxt = tn < e ? tn : e;
                        if (nxt > a) {
                            auto ok = [&](int w0) {
                                const uint32_t w = w0 > 0 ? (uint32_t)w0 : 0u;
                                return w == 0 ? rel <= 2u : (rel == w + 1 || rel == w + 2);
                            };
                            g0 += ok((int)fl - 2) ? nxt - a : 0;
                            g1 += ok((int)fl - 1) ? nxt - a : 0;
                            g2 += ok((int)fl) ? nxt - a : 0;
                            a = nxt;
                        }
                        if (a >= e) break;
                        rel++;
                    }
                    while (j < bc && (uint64_t)(tok[lo + j] & ((1u << bsh) - 1u)) < e) j++;
                }
                best = (g1 >= g0 && g1 >= g2) ? 1u : (g0 >= g2 ? 0u : 2u);
            }
            hints |= best << (2 * s);
        }
        idx[2 * g] = ((uint32_t)delta & 0x3FFFu) | (hints << 14);
        idx[2 * g + 1] = nib;
    }
}

// The LDS-index layout (round 6; k_lookupn_lds). The bucket search structure moves out of L2 into
// every CU's LDS, so a key takes one L2 trip (its window) instead of two (index record, then
// window). NG groups (a power of two, <= 8,192: 128 KB) of 28 buckets, NB = 28 NG buckets over the
// hash space: a hash h is in group g = h >> (32 - lg) and bucket j = floor(28 x / 2^32) of it, with
// x = h << lg, and its fingerprint is the top fb bits of the remainder (28 x) mod 2^32 (monotone in
// h within a bucket). A group record is 16 B: 28 4-bit token counts, then the group's first
// position as an int16 delta from pred(g) = g M / NG. Entries are 3 B, (fp << ob) | owner.
__device__ __forceinline__ uint32_t lds_first_pos(const uint32_t* __restrict__ tok, uint32_t M, uint32_t lg,
                                                  uint32_t g, uint32_t j) {
    // the least h in bucket (g, j): x >= ceil(j 2^32 / 28)
    const uint64_t xm = ((uint64_t)j << 32) / 28u + (((uint64_t)j << 32) % 28u ? 1u : 0u);
    const uint64_t hm = ((uint64_t)g << (32 - lg)) + (xm >> lg) + ((xm & ((1ull << lg) - 1u)) ? 1u : 0u);
    return hm >= (1ull << 32) ? M : lower_bound_dev(tok, M, (uint32_t)hm);
}
__global__ void k_lidx_build(const uint32_t* __restrict__ tok, uint32_t M, uint32_t lg, uint32_t ng,
                             uint4* __restrict__ idx, uint32_t* __restrict__ over) {
    const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < ng; g += gstride) {
        uint32_t w[4] = {0, 0, 0, 0};
        uint32_t p = lds_first_pos(tok, M, lg, (uint32_t)g, 0);
        const uint32_t base = p;
        bool full = false;
        for (uint32_t j = 0; j < 28; j++) {
            const uint32_t q = j == 27 ? (g + 1 == ng ? M : lds_first_pos(tok, M, lg, (uint32_t)g + 1, 0))
                                       : lds_first_pos(tok, M, lg, (uint32_t)g, j + 1);
            const uint32_t c = q - p;
            full |= c > 15u;
            w[j >> 3] |= (c > 15u ? 15u : c) << (4 * (j & 7));
            p = q;
        }
        const int64_t delta = (int64_t)base - (int64_t)(((uint64_t)g * M) >> lg);
        if (delta < -32767 || delta > 32767) atomicOr(over, 1u);
        // a bucket of 16+ tokens: the counts no longer sum to positions, so every key of the group
        // takes the exact path (delta -32768 marks it)
        w[3] |= (full ? 0x8000u : ((uint32_t)delta & 0xFFFFu)) << 16;
        idx[g] = uint4{w[0], w[1], w[2], w[3]};
    }
}
// LDS-index entries: 3 bytes per token, (fp << ob) | owner; padding entries are all ones
__global__ void k_lpack3(const uint32_t* __restrict__ tok, const uint32_t* __restrict__ own, uint32_t M, uint32_t lg,
                         uint32_t fb, uint32_t ob, uint8_t* __restrict__ ent) {
    const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < (uint64_t)M + kEnt3Pad + 6; j += gstride) {
        uint32_t v = 0xFFFFFFu;
        if (j < M) {
            const uint32_t x = tok[j] << lg;
            const uint32_t fp = (uint32_t)((uint64_t)x * 28u) >> (32u - fb);
            v = (fp << ob) | own[j];
        }
        ent[3 * j + 0] = (uint8_t)v;
        ent[3 * j + 1] = (uint8_t)(v >> 8);
        ent[3 * j + 2] = (uint8_t)(v >> 16);
    }
}

// checksum string pieces: len of (name + ';') for in-ring servers in name order.
__global__ void k_ck_len(const uint32_t* __restrict__ sorted_ids, uint32_t n,
                         const uint8_t* __restrict__ in_ring, const uint64_t* __restrict__ noff,
                         uint32_t* __restrict__ len) {
    const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gstride) {
        const uint32_t id = sorted_ids[i];
        len[i] = in_ring[id] ? (uint32_t)(noff[id + 1] - noff[id]) + 1u : 0u;
    }
}

__global__ void k_ck_scatter(const uint32_t* __restrict__ sorted_ids, uint32_t n,
                             const uint8_t* __restrict__ in_ring, const uint8_t* __restrict__ names,
                             const uint64_t* __restrict__ noff, const uint32_t* __restrict__ pos,
                             uint8_t* __restrict__ buf) {
    // one wave per name: lanes copy bytes
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t wid = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t i = wid; i < n; i += nw) {
        const uint32_t id = sorted_ids[i];
        if (!in_ring[id]) continue;
        const uint64_t b = noff[id];
        const uint32_t L = (uint32_t)(noff[id + 1] - b);
        const uint32_t p = pos[i];
        for (uint32_t q = lane; q < L; q += 64) buf[p + q] = names[b + q];
        if (lane == 0) buf[p + L] = ';';
    }
}

__global__ void k_hash_batch(const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off, uint64_t n,
                             uint32_t* __restrict__ out) {
    const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gstride)
        out[k] = fh::hash32(fh::PtrSrc{bytes + off[k]}, (uint32_t)(off[k + 1] - off[k]));
}

__global__ void k_gen_uuid(uint32_t seed, uint64_t k0, uint64_t n, uint32_t* __restrict__ out) {
    const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gstride) {
        uint32_t w[9];
        uuid_key_words(seed, k0 + k, w);
#pragma unroll
        for (int j = 0; j < 9; j++) out[k * 9 + j] = w[j];
    }
}

}  // namespace

// ---------------------------------------------------------------------------------- handle

struct Ring {
    int device = 0;
    hipStream_t st = nullptr;
    uint32_t R = 100;
    // interned names (host mirror of JS `servers` keys + an id table)
    NameTable nt;
    std::vector<uint8_t> in_ring;
    std::vector<uint64_t> stamp;  // insertion stamp -> Object.keys order
    uint64_t next_stamp = 1;
    uint32_t server_count = 0;
    bool has_checksum = false;
    uint32_t checksum = 0;
    // ring arrays
    DevBuf<uint32_t> tok, own, tok2, own2, bstart;
    uint32_t M = 0;
    uint32_t bbits = 8;
    // packed lookup layout (valid while every interned id < 2^16)
    DevBuf<uint32_t> ent, pbstart;
    DevBuf<uint32_t> slow, nslow;  // deferred keys of the probe / compact kernels
    bool packed = false;
    uint32_t pbits = 16;
    // compact lookup layout (the C2 hot path; valid while every interned id < 2^16)
    DevBuf<uint8_t> cent;
    DevBuf<uint32_t> cidx;
    DevBuf<uint32_t> cidxh;  // the hinted index (k_cindex_hint); valid when chint
    bool chint = false;
    bool chint_pending = false;  // the compact layout changed and the hinted index is not built yet
    bool compact = false;
    uint32_t ccb = 0, cob = 0, cfsh = 0;
    // the LDS-index layout (k_lookupn_lds, round 6), built by the first batch lookup after a change
    DevBuf<uint8_t> lent;
    DevBuf<uint4> lidx;
    bool lds = false, lds_pending = false;
    uint32_t lng = 0, llg = 0, lfb = 0;
    // checksum string + value
    DevBuf<uint8_t> d_inring;
    DevBuf<uint8_t> ck_buf;
    DevBuf<uint32_t> ck_out;  // [0] hash, [1] set
    // scratch
    DevBuf<uint32_t> ntok, nown, flag, pos, ids_dev, tmpk;
    DevBuf<uint64_t> tmp64;
    DevBuf<uint32_t> scalar;
    DevBuf<uint32_t> io_a, io_b;
    DevBuf<uint8_t> io_keys, io_cnt;
    // pinned, device-mapped rows / counts of the small host path (k_lookupn_small)
    uint32_t* pin_out = nullptr;
    uint8_t* pin_cnt = nullptr;
    uint32_t* pin_out_dev = nullptr;
    uint8_t* pin_cnt_dev = nullptr;
    DevBuf<uint64_t> io_off;
    // the lookup service (rp_ring_service): its pinned lines, stream, last answered seq
    SvcLines* svc = nullptr;
    SvcLines* svc_dev = nullptr;
    hipStream_t svc_st = nullptr;
    uint32_t svc_idle_ms = 0, svc_seq = 0;
    std::atomic<bool> svc_live{false};  // a wave launched and not yet stopped (counted in g_svc_live)
    std::recursive_mutex svc_mu;         // the service's lines and state (svc_lookup, svc_stop)
    bool svc_v2 = true;  // k_lookup_service3 (RP_RING_SVC=1: the round-4 kernel; read at rp_ring_service)
    DevBuf<uint4> svc_dt;       // the service's direct table (k_dt_build), built at its first launch after a change
    uint32_t svc_dtb = 0;       // its bucket bits; 0: none (ids past 16 bits, M > 2^22, RP_SVC_DT=0)
    bool svc_dt_valid = false;  // false after every ring change
    uint64_t svc_prof[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};  // RP_SVC_PROF: tick sums, path counts, calls
    // group keys by owner (handleOrProxyAll)
    DevBuf<uint32_t> grp_own, grp_key, grp_first, grp_dk, grp_dv, grp_rank;
    Scratch ws;

    RingView view() const {
        return RingView{tok.p, own.p, bstart.p, M, 32u - bbits};
    }
    PackedView pview() const { return PackedView{ent.p, pbstart.p, M, pbits}; }
    CompactView cview() const {
        const char* a = getenv("RP_LOOKUP_ABLATE");
        return CompactView{cent.p, cidx.p, M, ccb, cob, cfsh, cfsh == 0, a ? (uint32_t)atoi(a) : 0u,
                           (uint32_t)(3ull * ((uint64_t)M + kEnt3Pad + 6) + 16), (uint32_t)(8ull << (ccb - 3)),
                           getenv("RP_LOOKUP_WPRED") && !strcmp(getenv("RP_LOOKUP_WPRED"), "0") ? 0u : 1u,
                           chint && !(getenv("RP_LOOKUP_HINT") && !strcmp(getenv("RP_LOOKUP_HINT"), "0")) ? cidxh.p
                                                                                                       : nullptr};
    }
};

static uint32_t ring_intern(Ring& r, const char* s, uint32_t n) {
    const uint32_t id = r.nt.intern(s, n);
    if (id >= r.in_ring.size()) {
        r.in_ring.resize(id + 1, 0);
        r.stamp.resize(id + 1, 0);
    }
    return id;
}

static uint32_t choose_bbits(uint32_t M) {
    // ~4 tokens per bucket: a bounded 2-3 step search inside one or two cache lines.
    uint32_t b = 8;
    while (b < 22 && (1ull << (b + 2)) < M) b++;
    return b;
}

// The compact layout (CompactView): 2^cb buckets with cb = floor(log2 M), owner ids in ob bits,
// fingerprints of 24 - ob bits. Not built for tiny rings, more than 2^16 interned names, or a
// bucket of more than 15 tokens (caller hashFunc values that collide); the packed / wide
// layouts serve those.
static void ring_build_compact(Ring& r) {
    r.compact = false;
    if (r.M < 64) return;
    uint32_t ob = 1;
    while ((1ull << ob) < r.nt.size()) ob++;
    if (ob > 16) return;
    uint32_t cb = 3;
    while (cb < 24 && (2ull << cb) <= r.M) cb++;
    if (const char* d = getenv("RP_COMPACT_CB_DELTA")) {  // A/B knob: bucket density
        const int c = (int)cb + atoi(d);
        cb = (uint32_t)(c < 3 ? 3 : c > 24 ? 24 : c);
    }
    const uint32_t rb = 32 - cb, fb = 24 - ob;
    const uint32_t fsh = fb >= rb ? 0 : rb - fb;
    const uint64_t nbk = 1ull << cb, ngroups = nbk >> 3;
    r.tmpk.reserve(nbk + 1);
    hipLaunchKernelGGL(k_bucket_index, dim3(grid_for(nbk + 1, 256)), dim3(256), 0, r.st, r.tok.p, r.M, cb, r.tmpk.p);
    r.cidx.reserve(2 * ngroups);
    r.scalar.reserve(1);
    RP_HIP(hipMemsetAsync(r.scalar.p, 0, sizeof(uint32_t), r.st));
    hipLaunchKernelGGL(k_cindex, dim3(grid_for(ngroups, 256)), dim3(256), 0, r.st, r.tmpk.p, (uint32_t)ngroups,
                       r.cidx.p, r.scalar.p);
    r.cent.reserve(3ull * ((uint64_t)r.M + kEnt3Pad + 6) + 16);
    hipLaunchKernelGGL(k_pack3, dim3(grid_for((uint64_t)r.M + kEnt3Pad + 6, 256)), dim3(256), 0, r.st, r.tok.p,
                       r.own.p, r.M, cb, ob, fsh, r.cent.p);
    RP_HIP(hipGetLastError());
    if (read_u32(r.scalar.p, r.st) != 0) return;
    // the hinted index of the lean lookupN(3) (needs bucket bits >= 11: 8 prediction bits below)
    // is built by the first batch lookup that reads it (ring_build_hint): ~1 ms at C2, which a
    // per-call mutation (addServer / removeServer) should not pay
    r.chint = false;
    r.chint_pending = 32 - cb >= 8 && r.M < (1u << 30);
    r.lds = false;
    r.lds_pending = ob <= 14;
    r.compact = true;
    r.ccb = cb;
    r.cob = ob;
    r.cfsh = fsh;
}

static void ring_build_hint(Ring& r) {
    r.chint_pending = false;
    r.chint = false;
    const uint32_t cb = r.ccb;
    const uint64_t nbk = 1ull << cb, ngroups = nbk >> 3;
    r.tmpk.reserve(nbk + 1);
    hipLaunchKernelGGL(k_bucket_index, dim3(grid_for(nbk + 1, 256)), dim3(256), 0, r.st, r.tok.p, r.M, cb, r.tmpk.p);
    r.cidxh.reserve(2 * ngroups);
    RP_HIP(hipMemsetAsync(r.scalar.p, 0, sizeof(uint32_t), r.st));
    hipLaunchKernelGGL(k_cindex_hint, dim3(grid_for(ngroups, 256)), dim3(256), 0, r.st, r.tok.p, r.tmpk.p, r.M, cb,
                       (uint32_t)ngroups, r.cidxh.p, r.scalar.p);
    RP_HIP(hipGetLastError());
    r.chint = read_u32(r.scalar.p, r.st) == 0;
}

// The LDS-index layout (LdsView): ng = the power of two nearest M / 126 (about 4.5 tokens a bucket),
// 64..8,192 groups; not built past 5.5 tokens a bucket at 8,192 groups (M > 1.26 M), for owner ids
// past 14 bits (fingerprints under 10 bits), or when a group's base does not fit its int16 delta.
static void ring_build_lds(Ring& r) {
    r.lds_pending = false;
    r.lds = false;
    uint32_t lg = 6;
    while (lg < 13 && (1ull << lg) * 126ull < r.M) lg++;
    const uint64_t ng = 1ull << lg;
    if ((double)r.M / (28.0 * (double)ng) > 5.5 || r.cob > 14) return;
    const uint32_t fb = 24u - r.cob;
    r.lidx.reserve(ng);
    RP_HIP(hipMemsetAsync(r.scalar.p, 0, sizeof(uint32_t), r.st));
    hipLaunchKernelGGL(k_lidx_build, dim3(grid_for(ng, 256)), dim3(256), 0, r.st, r.tok.p, r.M, lg, (uint32_t)ng,
                       r.lidx.p, r.scalar.p);
    r.lent.reserve(3ull * ((uint64_t)r.M + kEnt3Pad + 6) + 16);
    hipLaunchKernelGGL(k_lpack3, dim3(grid_for((uint64_t)r.M + kEnt3Pad + 6, 256)), dim3(256), 0, r.st, r.tok.p,
                       r.own.p, r.M, lg, fb, r.cob, r.lent.p);
    RP_HIP(hipGetLastError());
    if (read_u32(r.scalar.p, r.st) != 0) return;
    r.lng = (uint32_t)ng;
    r.llg = lg;
    r.lfb = fb;
    r.lds = true;
}

static void ring_rebuild_index(Ring& r) {
    r.svc_dt_valid = false;
    r.bbits = choose_bbits(r.M);
    const uint64_t nbk = (1ull << r.bbits) + 1;
    r.bstart.reserve(nbk);
    hipLaunchKernelGGL(k_bucket_index, dim3(grid_for(nbk, 256)), dim3(256), 0, r.st, r.tok.p, r.M, r.bbits,
                       r.bstart.p);
    RP_HIP(hipGetLastError());
    // packed layout: 2^B >= M (about one token per bucket, so the 4 entries at the bucket
    // start usually hold the answer) and every interned id < 2^B; B <= 24 (64 MB index)
    uint32_t B = 8;
    while (B < 24 && ((1ull << B) < r.M || (1ull << B) < r.nt.size())) B++;
    r.packed = (1ull << B) >= r.nt.size();
    if (r.packed) {
        r.pbits = B;
        r.ent.reserve((uint64_t)r.M + kEntPad);
        r.pbstart.reserve((1ull << B) + 1);
        hipLaunchKernelGGL(k_pack, dim3(grid_for((uint64_t)r.M + kEntPad, 256)), dim3(256), 0, r.st, r.tok.p,
                           r.own.p, r.M, B, r.ent.p);
        hipLaunchKernelGGL(k_bucket_index, dim3(grid_for((1ull << B) + 1, 256)), dim3(256), 0, r.st, r.tok.p, r.M,
                           B, r.pbstart.p);
        RP_HIP(hipGetLastError());
    }
    ring_build_compact(r);
}

// Device replica tokens for server ids (or caller tokens), sorted stably by token.
static uint64_t ring_make_tokens(Ring& r, const std::vector<uint32_t>& sel_ids, const std::vector<uint32_t>* custom) {
    const uint64_t K = (uint64_t)sel_ids.size() * r.R;
    RP_REQUIRE(K < (1ull << 31), "too many replica points in one batch");
    r.ntok.reserve(K + 1);
    r.nown.reserve(K + 1);
    r.ids_dev.reserve(sel_ids.size() + 1);
    RP_HIP(hipMemcpyAsync(r.ids_dev.p, sel_ids.data(), sizeof(uint32_t) * sel_ids.size(), hipMemcpyHostToDevice,
                          r.st));
    if (custom) {
        RP_HIP(hipMemcpyAsync(r.ntok.p, custom->data(), sizeof(uint32_t) * K, hipMemcpyHostToDevice, r.st));
        hipLaunchKernelGGL(k_expand_owner, dim3(grid_for(K, 256)), dim3(256), 0, r.st, r.ids_dev.p,
                           (uint32_t)sel_ids.size(), r.R, r.nown.p);
    } else {
        hipLaunchKernelGGL(k_replica_tokens, dim3(grid_for(K, 256)), dim3(256), 0, r.st, r.nt.d_bytes.p, r.nt.d_noff.p,
                           r.ids_dev.p, (uint32_t)sel_ids.size(), r.R, r.ntok.p, r.nown.p);
    }
    RP_HIP(hipGetLastError());
    return K;
}

static void ring_apply_adds(Ring& r, const std::vector<uint32_t>& add_ids, const std::vector<uint32_t>* custom) {
    if (add_ids.empty()) return;
    const uint64_t K = ring_make_tokens(r, add_ids, custom);
    radix_sort_pairs(r.ntok.p, r.nown.p, K, 0, 32, r.st, r.ws);
    r.flag.reserve(K + 1);
    r.pos.reserve(K + 1);
    hipLaunchKernelGGL(k_mark_new, dim3(grid_for(K, 256)), dim3(256), 0, r.st, r.ntok.p, (uint32_t)K, r.tok.p, r.M,
                       r.flag.p);
    RP_HIP(hipGetLastError());
    scan_exclusive_u32(r.flag.p, r.pos.p, K, r.st, r.ws);
    const uint32_t Kp = read_u32(r.pos.p + K, r.st);
    r.tmpk.reserve((uint64_t)Kp + 1);
    r.ws.c.reserve((uint64_t)Kp + 1);
    hipLaunchKernelGGL(k_compact_pairs, dim3(grid_for(K, 256)), dim3(256), 0, r.st, r.ntok.p, r.nown.p, r.flag.p,
                       r.pos.p, (uint32_t)K, r.tmpk.p, r.ws.c.p);
    const uint64_t nM = (uint64_t)r.M + Kp;
    RP_REQUIRE(nM < 0xFFFFFFF0ull, "ring too large");
    r.tok2.reserve(nM + 1);
    r.own2.reserve(nM + 1);
    hipLaunchKernelGGL(k_merge, dim3(grid_for(nM, 256)), dim3(256), 0, r.st, r.tok.p, r.own.p, r.M, r.tmpk.p,
                       r.ws.c.p, Kp, r.tok2.p, r.own2.p);
    RP_HIP(hipGetLastError());
    r.tok.swap(r.tok2);
    r.own.swap(r.own2);
    r.M = (uint32_t)nM;
}

static void ring_apply_removes(Ring& r, const std::vector<uint32_t>& rem_ids, const std::vector<uint32_t>* custom) {
    if (rem_ids.empty() || r.M == 0) return;
    const uint64_t K = ring_make_tokens(r, rem_ids, custom);
    r.flag.reserve((uint64_t)r.M + 1);
    r.pos.reserve((uint64_t)r.M + 1);
    hipLaunchKernelGGL(k_fill_u32, dim3(grid_for(r.M, 256)), dim3(256), 0, r.st, r.flag.p, (uint64_t)r.M, 1u);
    hipLaunchKernelGGL(k_mark_del, dim3(grid_for(K, 256)), dim3(256), 0, r.st, r.ntok.p, K, r.tok.p, r.M, r.flag.p);
    RP_HIP(hipGetLastError());
    scan_exclusive_u32(r.flag.p, r.pos.p, r.M, r.st, r.ws);
    const uint32_t nM = read_u32(r.pos.p + r.M, r.st);
    r.tok2.reserve((uint64_t)nM + 1);
    r.own2.reserve((uint64_t)nM + 1);
    hipLaunchKernelGGL(k_compact_pairs, dim3(grid_for(r.M, 256)), dim3(256), 0, r.st, r.tok.p, r.own.p, r.flag.p,
                       r.pos.p, r.M, r.tok2.p, r.own2.p);
    RP_HIP(hipGetLastError());
    r.tok.swap(r.tok2);
    r.own.swap(r.own2);
    r.M = nM;
}

// HashRing.computeChecksum (lib/ring/index.js:96-105) on the device:
// hash32(Object.keys(servers).sort().join(';')), names in byte order (NameTable::sort).
static void ring_compute_checksum(Ring& r) {
    r.nt.sort(r.st, r.ws);
    const uint32_t n = r.nt.size();
    r.d_inring.reserve((uint64_t)n + 1);
    if (n) RP_HIP(hipMemcpyAsync(r.d_inring.p, r.in_ring.data(), n, hipMemcpyHostToDevice, r.st));
    r.flag.reserve((uint64_t)n + 1);
    r.pos.reserve((uint64_t)n + 1);
    r.ck_buf.reserve(r.nt.h_bytes.size() + n + 16);
    r.ck_out.reserve(2);
    if (n) {
        hipLaunchKernelGGL(k_ck_len, dim3(grid_for(n, 256)), dim3(256), 0, r.st, r.nt.sorted.p, n, r.d_inring.p,
                           r.nt.d_noff.p, r.flag.p);
        scan_exclusive_u32(r.flag.p, r.pos.p, n, r.st, r.ws);
        hipLaunchKernelGGL(k_ck_scatter, dim3(grid_for((uint64_t)n * 64, 256)), dim3(256), 0, r.st, r.nt.sorted.p, n,
                           r.d_inring.p, r.nt.d_bytes.p, r.nt.d_noff.p, r.pos.p, r.ck_buf.p);
        RP_HIP(hipGetLastError());
        hash_long(r.ck_buf.p, 0, r.pos.p + n, nullptr, r.ck_out.p, r.st);
    } else {
        hash_long(r.ck_buf.p, 0, nullptr, nullptr, r.ck_out.p, r.st);  // "" (empty ring)
    }
    uint32_t v[2];
    RP_HIP(hipMemcpyAsync(v, r.ck_out.p, sizeof v, hipMemcpyDeviceToHost, r.st));
    RP_HIP(hipStreamSynchronize(r.st));
    scratch_check(r.ws, r.st);
    r.checksum = v[0];
    r.has_checksum = true;
}

template <class View>
static void launch_lookupn_view(const View& rv, const uint8_t* keys, const uint64_t* off, uint32_t stride,
                                const uint32_t* hashes, uint64_t n, int np, uint32_t W, uint32_t* out,
                                uint8_t* counts, hipStream_t st) {
    const unsigned grid_fixed = grid_for(n, kLkThreads, 256 * 8);
    const bool fixed36 = !hashes && stride == 36 && ((reinterpret_cast<uintptr_t>(keys) & 3) == 0);
    const int need = np <= 0 ? 1 : np;
    const int ablate = getenv("RP_LOOKUP_ABLATE") ? atoi(getenv("RP_LOOKUP_ABLATE")) : 0;
    if (fixed36 && W <= 4 && need <= 4 && need > 1 && ablate == 1) {
        hipLaunchKernelGGL((k_lookupn_fixed<36, 4, View, 1>), dim3(grid_fixed), dim3(kLkThreads), 0, st, keys, n, rv,
                           np, W, out, counts);
    } else if (fixed36 && W <= 4 && need <= 4 && need > 1 && ablate == 2) {
        hipLaunchKernelGGL((k_lookupn_fixed<36, 4, View, 2>), dim3(grid_fixed), dim3(kLkThreads), 0, st, keys, n, rv,
                           np, W, out, counts);
    } else if (fixed36 && W <= 8 && need <= 8) {
        if (need == 1 && W == 1)
            hipLaunchKernelGGL((k_lookupn_fixed<36, 1, View>), dim3(grid_fixed), dim3(kLkThreads), 0, st, keys, n,
                               rv, np, W, out, counts);
        else if (need <= 4 && W <= 4)
            hipLaunchKernelGGL((k_lookupn_fixed<36, 4, View>), dim3(grid_fixed), dim3(kLkThreads), 0, st, keys, n,
                               rv, np, W, out, counts);
        else
            hipLaunchKernelGGL((k_lookupn_fixed<36, 8, View>), dim3(grid_fixed), dim3(kLkThreads), 0, st, keys, n,
                               rv, np, W, out, counts);
    } else {
        const unsigned g = grid_for(n, 256, 256 * 8);
        if (need == 1)
            hipLaunchKernelGGL((k_lookupn_generic<1, View>), dim3(g), dim3(256), 0, st, keys, off, stride, hashes,
                               n, rv, np, W, out, counts);
        else if (need <= 4)
            hipLaunchKernelGGL((k_lookupn_generic<4, View>), dim3(g), dim3(256), 0, st, keys, off, stride, hashes,
                               n, rv, np, W, out, counts);
        else if (need <= 8)
            hipLaunchKernelGGL((k_lookupn_generic<8, View>), dim3(g), dim3(256), 0, st, keys, off, stride, hashes,
                               n, rv, np, W, out, counts);
        else
            hipLaunchKernelGGL((k_lookupn_generic<0, View>), dim3(g), dim3(256), 0, st, keys, off, stride, hashes,
                               n, rv, np, W, out, counts);
    }
    RP_HIP(hipGetLastError());
}

static void launch_lookupn(Ring& r, const uint8_t* keys, const uint64_t* off, uint32_t stride,
                           const uint32_t* hashes, uint64_t n, int np, uint32_t W, uint32_t* out, uint8_t* counts,
                           hipStream_t st) {
    if (n == 0) return;
    // the ring is rebuilt on r.st; make the caller's stream wait for it
    if (st != r.st) RP_HIP(hipStreamSynchronize(r.st));
    const bool fixed36 = !hashes && stride == 36 && ((reinterpret_cast<uintptr_t>(keys) & 3) == 0);
    const int need = np <= 0 ? 1 : np;
    const bool use_packed = r.packed && !getenv_flag("RP_RING_WIDE");
    const char* lay = getenv("RP_RING_LAYOUT");  // A/B: "packed" forces the packed probe kernel
    const bool use_compact = r.compact && !(lay && !strcmp(lay, "packed")) && !getenv_flag("RP_RING_WIDE");
    const bool aligned16 = ((reinterpret_cast<uintptr_t>(keys) & 15) == 0) && ((reinterpret_cast<uintptr_t>(out) & 15) == 0);
    // the LDS-index kernel (round 6; RP_LOOKUP_LDS=0 keeps the lean kernel, 1 forces this one)
    const char* lds_env = getenv("RP_LOOKUP_LDS");
    const bool lds_on = lds_env ? !strcmp(lds_env, "1") : kLdsDefault;
    if (use_compact && lds_on && fixed36 && aligned16 && (uint32_t)need == W && W <= 4 && n >= 64ull * 8 &&
        !getenv("RP_LOOKUP_ABLATE")) {
        if (r.lds_pending) ring_build_lds(r);
        if (r.lds) {
            RP_REQUIRE(n < (1ull << 32), "lookupn: at most 2^32-1 keys per call");
            constexpr int KPL = 8;
            const uint64_t TK = 64ull * KPL, nwt = n / TK, done = nwt * TK;
            r.slow.reserve(nwt * kSlowPerTile + 1);
            r.nslow.reserve(nwt + 1);
            static const int cus = [] {
                int dev = 0, c = 0;
                (void)hipGetDevice(&dev);
                (void)hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev);
                return c > 0 ? c : 256;
            }();
            const unsigned g = (unsigned)std::min<uint64_t>((uint64_t)env_pos("RP_LOOKUP_LDS_GRID", (uint64_t)cus),
                                                            (nwt + kLdsThreads / 64 - 1) / (kLdsThreads / 64));
            const LdsView lv{r.lent.p, r.lidx.p, r.M, r.lng, r.llg, r.lfb, r.cob,
                             (uint32_t)(3ull * ((uint64_t)r.M + kEnt3Pad + 6) + 16)};
            const int stg = (int)env_pos("RP_LOOKUP_LDS_STG", 0) == 1 ? 1 : 0;
            const int abl = getenv("RP_LOOKUP_LDS_ABL") ? atoi(getenv("RP_LOOKUP_LDS_ABL")) : 0;
#define RP_LDSK(N, S, A) \
    hipLaunchKernelGGL((k_lookupn_lds<KPL, N, S, A>), dim3(g), dim3(kLdsThreads), 0, st, keys, nwt, lv, out, counts, r.slow.p, r.nslow.p)
            if (need == 3 && abl) {  // diagnostics: time ablations (results wrong)
                switch (abl) {
                    case 1: RP_LDSK(3, 0, 1); break;
                    case 2: RP_LDSK(3, 0, 2); break;
                    case 3: RP_LDSK(3, 0, 3); break;
                    case 4: RP_LDSK(3, 0, 4); break;
                    default: RP_LDSK(3, 0, 7); break;
                }
            } else if (stg) {
                switch (need) {
                    case 1: RP_LDSK(1, 1, 0); break;
                    case 2: RP_LDSK(2, 1, 0); break;
                    case 3: RP_LDSK(3, 1, 0); break;
                    default: RP_LDSK(4, 1, 0); break;
                }
            } else {
                switch (need) {
                    case 1: RP_LDSK(1, 0, 0); break;
                    case 2: RP_LDSK(2, 0, 0); break;
                    case 3: RP_LDSK(3, 0, 0); break;
                    default: RP_LDSK(4, 0, 0); break;
                }
            }
#undef RP_LDSK
            RP_HIP(hipGetLastError());
            const CompactFixView fv{r.tok.p, r.own.p, r.cidx.p, r.view(), r.M, r.ccb};
            const uint64_t fthreads = nwt * kSlowPerTile;
            hipLaunchKernelGGL((k_lookupn_fix_tiles<CompactFixView>), dim3((unsigned)((fthreads + 255) / 256)), dim3(256),
                               0, st, keys, fv, np, W, out, counts, r.slow.p, r.nslow.p, nwt, (uint32_t)TK);
            RP_HIP(hipGetLastError());
            if (getenv_flag("RP_LOOKUP_DEBUG")) {
                std::vector<uint32_t> c(nwt);
                RP_HIP(hipMemcpyAsync(c.data(), r.nslow.p, 4 * nwt, hipMemcpyDeviceToHost, st));
                RP_HIP(hipStreamSynchronize(st));
                uint64_t tot = 0, over = 0;
                for (uint32_t x : c) {
                    tot += x;
                    over += x > kSlowPerTile;
                }
                fprintf(stderr, "[rp] lds lookupN: %llu keys, %llu deferred, %llu overflowed tiles (ng %u fb %u ob %u)\n",
                        (unsigned long long)done, (unsigned long long)tot, (unsigned long long)over, r.lng, r.lfb, r.cob);
            }
            if (done < n)
                launch_lookupn_view(r.view(), keys + done * 36, nullptr, 36, nullptr, n - done, np, W, out + done * W,
                                    counts ? counts + done : nullptr, st);
            return;
        }
    }
    if (use_compact && fixed36 && aligned16 && (uint32_t)need == W && W <= 4 && n >= (uint64_t)kLkThreads * 4) {
        RP_REQUIRE(n < (1ull << 32), "lookupn: at most 2^32-1 keys per call");
        if (r.chint_pending && need == 3) ring_build_hint(r);
        const CompactView cv = r.cview();
        // the wave-specialised kernel (round 6, A/B): RP_LOOKUP_WS = "NP:NC" producer and consumer
        // waves a workgroup (1:3, 2:6, 1:7, 4:12, 2:2, 1:15, 2:14; "1" = 1:3)
        const char* ws_env = getenv("RP_LOOKUP_WS");
        if (ws_env && strcmp(ws_env, "0") && need == 3 && !getenv("RP_LOOKUP_KPL") && cv.ablate == 0 &&
            n >= 512ull * 4 && n * 12ull < (1ull << 31)) {
            int wnp = 1, wnc = 3;
            if (strchr(ws_env, ':') && sscanf(ws_env, "%d:%d", &wnp, &wnc) != 2) wnp = 0;
            constexpr uint64_t TK = 512;
            const uint64_t nwt = n / TK, done = nwt * TK;
            r.slow.reserve(nwt * kSlowPerTile + 1);
            r.nslow.reserve(nwt + 2);
            uint32_t* err = r.nslow.p + nwt + 1;
            RP_HIP(hipMemsetAsync(err, 0, 4, st));
            static const int cus = [] {
                int dev = 0, c = 0;
                (void)hipGetDevice(&dev);
                (void)hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev);
                return c > 0 ? c : 256;
            }();
            const uint64_t nwg = (nwt + (uint64_t)wnc - 1) / (uint64_t)(wnc > 0 ? wnc : 1);
            // workgroups a CU: 16 waves (<= 128 VGPRs), and the LDS (an 18-KB key tile a producer,
            // kWsSlots 2-KB ring slots and a 768-B list a consumer)
            const uint64_t lds_wg = (uint64_t)wnp * 18432 + (uint64_t)wnc * (kWsSlots * 2048 + 780);
            const uint64_t per_cu = wnp + wnc > 0 ? std::max<uint64_t>(1, std::min<uint64_t>(16 / (uint64_t)(wnp + wnc), 163840 / lds_wg)) : 1;
            const unsigned g = (unsigned)std::min<uint64_t>(nwg, env_pos("RP_LOOKUP_WS_GRID", (uint64_t)cus * per_cu));
            const int wabl = getenv("RP_LOOKUP_WS_ABL") ? atoi(getenv("RP_LOOKUP_WS_ABL")) : 0;  // diagnostics
#define RP_WSK(P, C) \
    hipLaunchKernelGGL((k_lookupn_ws<P, C>), dim3(g), dim3((P + C) * 64), 0, st, keys, nwt, cv, out, (uint32_t)(n * 12ull), counts, r.slow.p, r.nslow.p, err)
            if (wnp == 1 && wnc == 3)
                RP_WSK(1, 3);
            else if (wnp == 2 && wnc == 6)
                RP_WSK(2, 6);
            else if (wnp == 1 && wnc == 7)
                RP_WSK(1, 7);
            else if (wnp == 4 && wnc == 12 && wabl == 1)
                hipLaunchKernelGGL((k_lookupn_ws<4, 12, 1>), dim3(g), dim3(16 * 64), 0, st, keys, nwt, cv, out, (uint32_t)(n * 12ull), counts, r.slow.p, r.nslow.p, err);
            else if (wnp == 4 && wnc == 12 && wabl == 2)
                hipLaunchKernelGGL((k_lookupn_ws<4, 12, 2>), dim3(g), dim3(16 * 64), 0, st, keys, nwt, cv, out, (uint32_t)(n * 12ull), counts, r.slow.p, r.nslow.p, err);
            else if (wnp == 4 && wnc == 12)
                RP_WSK(4, 12);
            else if (wnp == 2 && wnc == 2)
                RP_WSK(2, 2);
            else if (wnp == 1 && wnc == 15)
                RP_WSK(1, 15);
            else if (wnp == 2 && wnc == 14)
                RP_WSK(2, 14);
            else
                RP_REQUIRE(false, "RP_LOOKUP_WS: one of 1:3, 2:6, 1:7, 4:12, 2:2, 1:15, 2:14");
#undef RP_WSK
            RP_HIP(hipGetLastError());
            const CompactFixView fv{r.tok.p, r.own.p, r.cidx.p, r.view(), r.M, r.ccb};
            const uint64_t fthreads = nwt * kSlowPerTile;
            hipLaunchKernelGGL((k_lookupn_fix_tiles<CompactFixView>), dim3((unsigned)((fthreads + 255) / 256)), dim3(256),
                               0, st, keys, fv, np, W, out, counts, r.slow.p, r.nslow.p, nwt, (uint32_t)TK);
            RP_HIP(hipGetLastError());
            if (getenv_flag("RP_LOOKUP_DEBUG")) {
                std::vector<uint32_t> c(nwt + 2);
                RP_HIP(hipMemcpyAsync(c.data(), r.nslow.p, 4 * (nwt + 2), hipMemcpyDeviceToHost, st));
                RP_HIP(hipStreamSynchronize(st));
                uint64_t tot = 0, over = 0;
                for (uint64_t t = 0; t < nwt; t++) {
                    tot += c[t];
                    over += c[t] > kSlowPerTile;
                }
                fprintf(stderr, "[rp] ws lookupN %d:%d: %llu keys, %llu deferred, %llu overflowed wave-tiles, err %u\n", wnp,
                        wnc, (unsigned long long)done, (unsigned long long)tot, (unsigned long long)over, c[nwt + 1]);
            }
            if (done < n)
                launch_lookupn_view(r.view(), keys + done * 36, nullptr, 36, nullptr, n - done, np, W, out + done * W,
                                    counts ? counts + done : nullptr, st);
            return;
        }
        // lookupN(3) (the C2 bench): 8 keys per lane, staged through LDS in four slices (0.925-0.926
        // against 0.962-0.970 ms for 4 keys per lane; two slices 0.926-0.932; 6 keys per lane
        // 0.956-0.959; profiles/r02/ab_lookup_lean.json); the other widths 4 keys per lane.
        // RP_LOOKUP_KPL / RP_LOOKUP_HALF (slices: 2, 4) override (A/B).
        int kpl = getenv("RP_LOOKUP_KPL") ? atoi(getenv("RP_LOOKUP_KPL")) : (need == 3 ? 8 : 4);
        if (kpl != 1 && kpl != 2 && !((kpl == 3 || kpl == 8) && need == 3)) kpl = 4;  // the instantiated tiles
        if (n < (uint64_t)kLkThreads * kpl) kpl = 4;  // at least one whole tile
        const uint64_t TK = (uint64_t)kLkThreads * kpl;
        const uint64_t ntiles = n / TK, done = ntiles * TK;
        r.slow.reserve(ntiles * kSlowPerTile + 1);
        r.nslow.reserve(ntiles + 1);
        const bool lean = !(getenv("RP_LOOKUP_LEAN") && !strcmp(getenv("RP_LOOKUP_LEAN"), "0"));  // A/B: 0 = round-1 kernel
        // workgroups, tiles strided over them: the lean kernel at 4096 (4 rounds of the 1024 that
        // fit, 8 tiles each at C2) ran 0.905-0.911 ms against 0.926-0.930 at 2048 (3072: 0.917;
        // 5120-16384: 0.908-0.914; profiles/r02/ab_lookup_grid.json). RP_LOOKUP_GRID overrides (A/B).
        const unsigned g = grid_for(ntiles, 1, (unsigned)env_pos("RP_LOOKUP_GRID", lean ? 4096u : 2048u));
        const int half = getenv("RP_LOOKUP_HALF") ? atoi(getenv("RP_LOOKUP_HALF")) : (kpl == 8 ? 4 : 0);
        const CompactFixView fv{r.tok.p, r.own.p, r.cidx.p, r.view(), r.M, r.ccb};
        // deferred keys finished by the lean kernel's own workgroups (A/B): only <8, 3, 4>
        const bool fuse = getenv_flag("RP_LOOKUP_FUSEFIX") && lean && half == 4 && kpl == 8 && need == 3 && cv.ablate != 3;
        const bool stg1 = getenv("RP_LOOKUP_STG") && atoi(getenv("RP_LOOKUP_STG")) == 1 && lean && half == 4 && kpl == 8 &&
                          need == 3 && !fuse;
        // RP_LOOKUP_STG=2: asm DMA ring (RP_LOOKUP_STGHS = 4 | 8 key slices; RP_LOOKUP_LH = 1 | 2)
        const bool stg2 = lean && kpl == 8 && need == 3 && !fuse && getenv("RP_LOOKUP_STG") && atoi(getenv("RP_LOOKUP_STG")) == 2;
        const int lh = (lean && (half == 4 || stg2) && kpl == 8 && need == 3 && !fuse)
                           ? (int)env_pos("RP_LOOKUP_LH", stg2 ? 2 : 1) : 1;
        const int stghs = (int)env_pos("RP_LOOKUP_STGHS", 8);
#define RP_COMPACT(KPL, NEED)                                                                                  \
    do {                                                                                                        \
        if (KPL == 8 && NEED == 3 && stg2 && stghs == 8 && lh == 1)                                             \
            hipLaunchKernelGGL((k_lookupn_lean<8, 3, 8, false, 2, 1>), dim3(g), dim3(kLkThreads), 0, st, keys,  \
                               ntiles, cv, out, counts, r.slow.p, r.nslow.p, fv, np);                           \
        else if (KPL == 8 && NEED == 3 && stg2 && stghs == 8)                                                   \
            hipLaunchKernelGGL((k_lookupn_lean<8, 3, 8, false, 2, 2>), dim3(g), dim3(kLkThreads), 0, st, keys,  \
                               ntiles, cv, out, counts, r.slow.p, r.nslow.p, fv, np);                           \
        else if (KPL == 8 && NEED == 3 && stg2)                                                                 \
            hipLaunchKernelGGL((k_lookupn_lean<8, 3, 4, false, 2, 2>), dim3(g), dim3(kLkThreads), 0, st, keys,  \
                               ntiles, cv, out, counts, r.slow.p, r.nslow.p, fv, np);                           \
        else if (KPL == 8 && NEED == 3 && stg1 && lh == 2)                                                      \
            hipLaunchKernelGGL((k_lookupn_lean<8, 3, 4, false, 1, 2>), dim3(g), dim3(kLkThreads), 0, st, keys,  \
                               ntiles, cv, out, counts, r.slow.p, r.nslow.p, fv, np);                           \
        else if (KPL == 8 && NEED == 3 && lh == 2)                                                              \
            hipLaunchKernelGGL((k_lookupn_lean<8, 3, 4, false, 0, 2>), dim3(g), dim3(kLkThreads), 0, st, keys,  \
                               ntiles, cv, out, counts, r.slow.p, r.nslow.p, fv, np);                           \
        else if (KPL == 8 && NEED == 3 && stg1)                                                                 \
            hipLaunchKernelGGL((k_lookupn_lean<8, 3, 4, false, 1>), dim3(g), dim3(kLkThreads), 0, st, keys,     \
                               ntiles, cv, out, counts, r.slow.p, r.nslow.p, fv, np);                           \
        else if (lean && half == 4 && KPL % 4 == 0 && fuse)                                                     \
            hipLaunchKernelGGL((k_lookupn_lean<KPL, NEED, (KPL % 4 == 0 ? 4 : 1), true>), dim3(g), dim3(kLkThreads), \
                               0, st, keys, ntiles, cv, out, counts, r.slow.p, r.nslow.p, fv, np);               \
        else if (lean && half == 4 && KPL % 4 == 0)                                                             \
            hipLaunchKernelGGL((k_lookupn_lean<KPL, NEED, (KPL % 4 == 0 ? 4 : 1)>), dim3(g), dim3(kLkThreads), 0, \
                               st, keys, ntiles, cv, out, counts, r.slow.p, r.nslow.p, fv, np);                  \
        else if (lean && half == 2 && KPL % 2 == 0)                                                             \
            hipLaunchKernelGGL((k_lookupn_lean<KPL, NEED, (KPL % 2 == 0 ? 2 : 1)>), dim3(g), dim3(kLkThreads), 0, \
                               st, keys, ntiles, cv, out, counts, r.slow.p, r.nslow.p, fv, np);                  \
        else if (lean)                                                                                          \
            hipLaunchKernelGGL((k_lookupn_lean<KPL, NEED>), dim3(g), dim3(kLkThreads), 0, st, keys, ntiles, cv,  \
                               out, counts, r.slow.p, r.nslow.p, fv, np);                                       \
        else                                                                                                    \
            hipLaunchKernelGGL((k_lookupn_compact<KPL, NEED>), dim3(g), dim3(kLkThreads), 0, st, keys, ntiles,   \
                               cv, out, counts, r.slow.p, r.nslow.p);                                           \
    } while (0)
#define RP_COMPACT_N(KPL)         \
    switch (need) {               \
        case 1: RP_COMPACT(KPL, 1); break; \
        case 2: RP_COMPACT(KPL, 2); break; \
        case 3: RP_COMPACT(KPL, 3); break; \
        default: RP_COMPACT(KPL, 4); break; \
    }
        if (kpl == 1) {
            RP_COMPACT_N(1);
        } else if (kpl == 2) {
            RP_COMPACT_N(2);
        } else if (kpl == 8 && need == 3) {
            RP_COMPACT(8, 3);
        } else if (kpl == 3 && need == 3) {
            RP_COMPACT(3, 3);


        } else {
            RP_COMPACT_N(4);
        }
#undef RP_COMPACT_N
#undef RP_COMPACT
        const uint64_t fthreads = ntiles * kSlowPerTile;
        if (cv.ablate != 3 && !fuse)
            hipLaunchKernelGGL((k_lookupn_fix_tiles<CompactFixView>), dim3((unsigned)((fthreads + 255) / 256)),
                               dim3(256), 0, st, keys, fv, np, W, out, counts, r.slow.p, r.nslow.p, ntiles,
                               (uint32_t)TK);
        RP_HIP(hipGetLastError());
#ifdef RP_LK_PROF
        if (getenv_flag("RP_LK_PROF_PRINT")) {
            unsigned long long v[10];
            RP_HIP(hipStreamSynchronize(st));
            RP_HIP(hipMemcpyFromSymbol(v, HIP_SYMBOL(g_lk_prof), sizeof v));
            const double nw = (double)(v[6] ? v[6] : 1);
            fprintf(stderr,
                    "[rp] lean phase cycles per wave-tile (%llu): keys-arrive %.0f hash-all %.0f idx %.0f win1+loop %.0f "
                    "finish2 %.0f barrier+store %.0f\n",
                    v[6], v[0] / nw, v[1] / nw, v[2] / nw, v[3] / nw, v[4] / nw, v[5] / nw);
            memset(v, 0, sizeof v);
            RP_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_lk_prof), v, sizeof v));
        }
#endif
        if (getenv_flag("RP_LOOKUP_DEBUG")) {
            std::vector<uint32_t> c(ntiles);
            RP_HIP(hipMemcpyAsync(c.data(), r.nslow.p, 4 * ntiles, hipMemcpyDeviceToHost, st));
            RP_HIP(hipStreamSynchronize(st));
            uint64_t tot = 0, over = 0;
            for (uint32_t x : c) {
                tot += x;
                over += x > kSlowPerTile;
            }
            fprintf(stderr, "[rp] compact lookupN: %llu keys, %llu deferred, %llu overflowed tiles (cb %u ob %u fsh %u)\n",
                    (unsigned long long)done, (unsigned long long)tot, (unsigned long long)over, r.ccb, r.cob, r.cfsh);
        }
        if (done < n)  // the partial last tile
            launch_lookupn_view(r.view(), keys + done * 36, nullptr, 36, nullptr, n - done, np, W, out + done * W,
                                counts ? counts + done : nullptr, st);
        return;
    }
    if (use_packed && fixed36 && W <= 4 && need <= 4 && !getenv_flag("RP_RING_NOWINDOW")) {
        RP_REQUIRE(n < (1ull << 32), "lookupn: at most 2^32-1 keys per call");
        r.slow.reserve(n + 1);
        r.nslow.reserve(1);
        RP_HIP(hipMemsetAsync(r.nslow.p, 0, sizeof(uint32_t), st));
        const int ablate = getenv("RP_LOOKUP_ABLATE") ? atoi(getenv("RP_LOOKUP_ABLATE")) : 0;
        const int kpl = getenv("RP_LOOKUP_KPL") ? atoi(getenv("RP_LOOKUP_KPL")) : kDefaultKPL;
        const PackedView pv = r.pview();
#define RP_PROBE(KPL, MODE)                                                                                     \
    hipLaunchKernelGGL((k_lookupn_probe<36, KPL, MODE>), dim3(grid_for(n, kLkThreads * KPL, 256 * 8)),           \
                       dim3(kLkThreads), 0, st, keys, n, pv, np, W, out, counts, r.slow.p, r.nslow.p);           \
    hipLaunchKernelGGL((k_lookupn_fix<36, MODE>), dim3(256), dim3(256), 0, st, keys, pv, np, W, out, counts,     \
                       r.slow.p, r.nslow.p)
        if (ablate == 1) {
            RP_PROBE(2, 1);
        } else if (ablate == 2) {
            RP_PROBE(2, 2);
        } else if (kpl == 1) {
            RP_PROBE(1, 0);
        } else if (kpl == 4) {
            RP_PROBE(4, 0);
        } else if (kpl == 8) {
            RP_PROBE(8, 0);
        } else {
            RP_PROBE(2, 0);
        }
#undef RP_PROBE
        RP_HIP(hipGetLastError());
        return;
    }
    if (use_packed)
        launch_lookupn_view(r.pview(), keys, off, stride, hashes, n, np, W, out, counts, st);
    else
        launch_lookupn_view(r.view(), keys, off, stride, hashes, n, np, W, out, counts, st);
}

// ------------------------------------------------------------------- group keys by owner
// RingPop.handleOrProxyAll's keysByDest = _.groupBy(keys, this.lookup) (index.js:609-667, :616)
// and RequestProxySend.lookupKeys (lib/request-proxy/send.js:171-179). _.groupBy appends each
// key to its owner's list in input order and Object.keys(keysByDest) lists the owners in
// first-seen order, so: first[s] = min key index owned by s; the owners ranked by first[s];
// a stable sort of the key indices by that rank.

__global__ void k_grp_first(const uint32_t* __restrict__ own, uint64_t n, uint32_t* __restrict__ first) {
    const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gstride) {
        const uint32_t s = own[i];
        // a plain (possibly stale) read first: once an owner's first key is known, later keys
        // skip the atomic
        if ((uint32_t)i < first[s]) atomicMin(first + s, (uint32_t)i);
    }
}

// (first index, owner) pairs to sort; unseen owners sort after every seen one (key n)
__global__ void k_grp_dest_keys(const uint32_t* __restrict__ first, uint32_t S, uint32_t n,
                                uint32_t* __restrict__ dk, uint32_t* __restrict__ dv) {
    const uint32_t gstride = gridDim.x * blockDim.x;
    for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < S; s += gstride) {
        const uint32_t f = first[s];
        dk[s] = f < n ? f : n;
        dv[s] = s;
    }
}

// owners in first-seen order: dests[p], rank[owner] = p, *ndest
__global__ void k_grp_rank(const uint32_t* __restrict__ dk, const uint32_t* __restrict__ dv, uint32_t S, uint32_t n,
                           uint32_t* __restrict__ rank, uint32_t* __restrict__ dests, uint32_t* __restrict__ ndest) {
    const uint32_t gstride = gridDim.x * blockDim.x;
    for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < S; p += gstride) {
        if (dk[p] >= n) continue;
        rank[dv[p]] = p;
        dests[p] = dv[p];
        if (p + 1 == S || dk[p + 1] >= n) *ndest = p + 1;
    }
}

// sort keys: the owner's rank; values: the key index (stable sort keeps input order per group)
__global__ void k_grp_keys(const uint32_t* __restrict__ own, uint64_t n, const uint32_t* __restrict__ rank,
                           uint32_t* __restrict__ gk, uint32_t* __restrict__ perm) {
    const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gstride) {
        gk[i] = rank[own[i]];
        perm[i] = (uint32_t)i;
    }
}

// group_off[g] = first position of rank g in the sorted keys; group_off[ndest] = n
__global__ void k_grp_bounds(const uint32_t* __restrict__ gk, uint64_t n, uint32_t* __restrict__ goff) {
    const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += gstride) {
        const uint32_t g = gk[p];
        if (p == 0 || gk[p - 1] != g) goff[g] = (uint32_t)p;
        if (p + 1 == n) goff[g + 1] = (uint32_t)n;
    }
}

static int bits_for(uint64_t v) {  // radix bits (multiple of 8) that hold every value <= v
    int b = 8;
    while (b < 32 && (v >> b)) b += 8;
    return b;
}

// keys (or caller hashes) -> owners -> groups; buffers as rp_ring_group_keys_dev documents
static void group_keys(Ring& r, const uint8_t* keys, const uint64_t* off, uint32_t stride, const uint32_t* hashes,
                       uint64_t n, uint32_t self_id, uint32_t* dests, uint32_t* goff, uint32_t* perm,
                       uint32_t* ndest, hipStream_t st) {
    RP_REQUIRE(n < 0xFFFFFFFFull, "group_keys: at most 2^32-2 keys per call");
    if (st != r.st) RP_HIP(hipStreamSynchronize(r.st));
    if (n == 0 || r.M == 0) {
        // lookup returns null for every key and RingPop.lookup answers whoami() (index.js:434-451):
        // one group (self) holding every key in order, or no group at all
        const uint32_t h[3] = {self_id, 0u, (uint32_t)n};
        const uint32_t nd = n ? 1u : 0u;
        RP_HIP(hipMemcpyAsync(ndest, &nd, 4, hipMemcpyHostToDevice, st));
        if (n) {
            RP_HIP(hipMemcpyAsync(dests, h, 4, hipMemcpyHostToDevice, st));
            RP_HIP(hipMemcpyAsync(goff, h + 1, 8, hipMemcpyHostToDevice, st));
            iota_u32(perm, n, st);
        } else {
            RP_HIP(hipMemsetAsync(goff, 0, 4, st));
        }
        RP_HIP(hipStreamSynchronize(st));  // h lives on this stack frame
        return;
    }
    const uint32_t S = r.nt.size();
    r.grp_own.reserve(n);
    r.grp_key.reserve(n);
    r.grp_first.reserve(S);
    r.grp_dk.reserve(S);
    r.grp_dv.reserve(S);
    r.grp_rank.reserve(S);
    launch_lookupn(r, keys, off, stride, hashes, n, 1, 1, r.grp_own.p, nullptr, st);
    RP_HIP(hipMemsetAsync(r.grp_first.p, 0xFF, 4ull * S, st));
    hipLaunchKernelGGL(k_grp_first, dim3(grid_for(n, 256, 256 * 16)), dim3(256), 0, st, r.grp_own.p, n, r.grp_first.p);
    hipLaunchKernelGGL(k_grp_dest_keys, dim3(grid_for(S, 256)), dim3(256), 0, st, r.grp_first.p, S, (uint32_t)n,
                       r.grp_dk.p, r.grp_dv.p);
    radix_sort_pairs(r.grp_dk.p, r.grp_dv.p, S, 0, bits_for(n), st, r.ws);
    hipLaunchKernelGGL(k_grp_rank, dim3(grid_for(S, 256)), dim3(256), 0, st, r.grp_dk.p, r.grp_dv.p, S, (uint32_t)n,
                       r.grp_rank.p, dests, ndest);
    hipLaunchKernelGGL(k_grp_keys, dim3(grid_for(n, 256, 256 * 16)), dim3(256), 0, st, r.grp_own.p, n, r.grp_rank.p,
                       r.grp_key.p, perm);
    radix_sort_pairs(r.grp_key.p, perm, n, 0, bits_for(S - 1), st, r.ws);
    hipLaunchKernelGGL(k_grp_bounds, dim3(grid_for(n, 256, 256 * 16)), dim3(256), 0, st, r.grp_key.p, n, goff);
    RP_HIP(hipGetLastError());
}

}  // namespace rp

// ==================================================================================== C ABI

struct rp_ring {
    rp::Ring impl;
};

using rp::guard;
using rp::guard_host;

static rp::Ring& R(rp_ring* r) {
    if (!r) throw rp::Error(rp::RP_EINVAL, "null ring handle");
    RP_HIP(hipSetDevice(r->impl.device));
    return r->impl;
}

extern "C" {

int rp_ring_create(uint32_t replica_points, int device, rp_ring** out) {
    return guard([&] {
        RP_REQUIRE(out, "out is null");
        int nd = 0;
        RP_HIP(hipGetDeviceCount(&nd));
        RP_REQUIRE(device >= 0 && device < nd, "no such HIP device");
        RP_HIP(hipSetDevice(device));
        auto* h = new rp_ring();
        h->impl.device = device;
        h->impl.R = replica_points ? replica_points : 100;
        hipError_t e = hipStreamCreateWithFlags(&h->impl.st, hipStreamNonBlocking);
        if (e != hipSuccess) {
            delete h;
            throw rp::Error(rp::RP_EDEVICE, std::string("hipStreamCreate: ") + hipGetErrorString(e));
        }
        h->impl.tok.reserve(64);
        h->impl.own.reserve(64);
        rp::ring_rebuild_index(h->impl);
        *out = h;
    });
}

// ---- the lookup service (rp_ring_service; k_lookup_service)
// While the service wave is resident (up to idle_ms after a request), any hipFree in the process
// (a device buffer growing or released) synchronizes the device and so waits for the wave to idle
// out, and the wave's stream may share a hardware queue with another handle's. Every device call of
// the library therefore stops every resident service first and keeps new ones from starting while
// it runs (QuietScope, rp_common.h): rings with a service configured are listed
// in a process-wide registry that svc_quiesce walks.
}  // extern "C" (the registry and its counters have C++ linkage)
namespace rp {
std::atomic<int> g_quiet{0}, g_svc_live{0};
}  // namespace rp
static std::mutex g_svc_reg_mu;            // guards g_svc_reg; taken before any ring's svc_mu
static std::vector<rp::Ring*> g_svc_reg;   // rings with a service configured (rp_ring_service)

static void svc_stop(rp::Ring& r) {
    std::lock_guard<std::recursive_mutex> lk(r.svc_mu);
    if (r.svc_prof[8] && getenv("RP_SVC_PROF")) {
        const double n = (double)r.svc_prof[8];
        fprintf(stderr,
                "[rp] service: %llu calls; device us per call: poll round trip %.3f, lookup %.3f; "
                "direct table %llu, window %llu, exact walk %llu, wide walk %llu\n",
                (unsigned long long)r.svc_prof[8], r.svc_prof[0] / n / 100.0, r.svc_prof[1] / n / 100.0,
                (unsigned long long)r.svc_prof[4], (unsigned long long)r.svc_prof[5],
                (unsigned long long)r.svc_prof[6], (unsigned long long)r.svc_prof[7]);
        for (auto& x : r.svc_prof) x = 0;
    }
    if (!r.svc || !r.svc_live.load()) return;
    __atomic_store_n(&r.svc->req[4], 1u, __ATOMIC_RELEASE);
    const hipError_t e = hipStreamSynchronize(r.svc_st);
    r.svc_live.store(false);
    rp::g_svc_live.fetch_sub(1);
    __atomic_store_n(&r.svc->req[4], 0u, __ATOMIC_RELEASE);
    RP_HIP(e);
}

void rp::svc_quiesce(const void* keep) {
    std::lock_guard<std::mutex> g(g_svc_reg_mu);
    for (rp::Ring* r : g_svc_reg)
        if (r != keep && r->svc_live.load()) svc_stop(*r);
}

static void svc_register(rp::Ring& r, bool on) {
    std::lock_guard<std::mutex> g(g_svc_reg_mu);
    auto it = std::find(g_svc_reg.begin(), g_svc_reg.end(), &r);
    if (on && it == g_svc_reg.end()) g_svc_reg.push_back(&r);
    if (!on && it != g_svc_reg.end()) g_svc_reg.erase(it);
}
extern "C" {

static void svc_launch(rp::Ring& r, uint32_t last) {
    using namespace rp;
    const uint64_t idle = (uint64_t)r.svc_idle_ms * 100000ull, maxt = 30ull * 100000000ull;  // 100 MHz ticks
    const CompactFixView fv{r.tok.p, r.own.p, r.cidx.p, r.view(), r.M, r.ccb};
    if (r.svc_v2) {
        const uint32_t warm = (uint32_t)env_pos("RP_SVC_WARM", 0), prof = getenv("RP_SVC_PROF") ? 1u : 0u;
        if (!r.svc_dt_valid) {  // the direct table for this ring (A/B: RP_SVC_DT=0)
            r.svc_dtb = 0;
            uint32_t B = 16;
            while (B < 22 && (1ull << B) < r.M) B++;
            const bool dt_on = !(getenv("RP_SVC_DT") && !strcmp(getenv("RP_SVC_DT"), "0"));
            if (dt_on && r.M > 0 && (1ull << B) >= r.M && r.nt.size() < 0xFFFFu) {
                r.svc_dt.reserve(4ull << B);
                hipLaunchKernelGGL(k_dt_build, dim3(grid_for(1ull << B, 256, 1u << 20)), dim3(256), 0, r.svc_st, r.tok.p,
                                   r.own.p, r.M, B, r.svc_dt.p);
                RP_HIP(hipGetLastError());
                r.svc_dtb = B;
            }
            r.svc_dt_valid = true;
        }
        const uint32_t* dt = r.svc_dtb ? reinterpret_cast<const uint32_t*>(r.svc_dt.p) : nullptr;
        // RP_SVC_WAVES pollers (one workgroup each, so one an XCD up to 8): see k_lookup_service3
        const uint32_t waves = (uint32_t)std::min<uint64_t>(env_pos("RP_SVC_WAVES", kSvcWaves), 16);
        hipLaunchKernelGGL((k_lookup_service3<RingView>), dim3(waves), dim3(64), 0, r.svc_st, r.svc_dev, r.view(), fv,
                           r.cview(), r.compact ? 1u : 0u, last, idle, maxt, warm, prof, dt, r.svc_dtb,
                           waves > 1 ? (uint32_t)env_pos("RP_SVC_PERIOD", kSvcPeriod) : 0u,
                           (getenv("RP_SVC_ANS") && !strcmp(getenv("RP_SVC_ANS"), "0")) ? 1u : 0u);
    } else
        hipLaunchKernelGGL((k_lookup_service<RingView>), dim3(1), dim3(64), 0, r.svc_st, r.svc_dev, r.view(), fv,
                           r.compact ? 1u : 0u, last, idle, maxt);
    RP_HIP(hipGetLastError());
}

int rp_ring_destroy(rp_ring* r) {
    return guard([&] {
        if (!r) return;
        svc_register(r->impl, false);  // no quiesce walks this ring from here on
        (void)hipSetDevice(r->impl.device);
        if (r->impl.st) {
            (void)hipStreamSynchronize(r->impl.st);
            (void)hipStreamDestroy(r->impl.st);
        }
        if (r->impl.svc) {
            try {
                svc_stop(r->impl);
            } catch (...) {
            }
            (void)hipStreamDestroy(r->impl.svc_st);
            (void)hipHostFree(r->impl.svc);
        }
        if (r->impl.pin_out) (void)hipHostFree(r->impl.pin_out);
        if (r->impl.pin_cnt) (void)hipHostFree(r->impl.pin_cnt);
        delete r;
    });
}

int rp_ring_add_remove(rp_ring* h, const char* add_bytes, const uint32_t* add_off, uint32_t n_add,
                       const uint32_t* add_tokens, const char* rem_bytes, const uint32_t* rem_off, uint32_t n_rem,
                       const uint32_t* rem_tokens, int* changed_out) {
    return guard([&] {
        rp::Ring& r = R(h);
        RP_REQUIRE(n_add == 0 || (add_bytes && add_off), "add names missing");
        svc_stop(r);  // the service reads the table this rebuilds
        RP_REQUIRE(n_rem == 0 || (rem_bytes && rem_off), "remove names missing");
        // lib/ring/index.js:69-76 — adds in order, skipping servers already present
        std::vector<uint32_t> add_ids, rem_ids;
        std::vector<uint32_t> add_tok_sel, rem_tok_sel;
        for (uint32_t j = 0; j < n_add; j++) {
            const uint32_t id = rp::ring_intern(r, add_bytes + add_off[j], add_off[j + 1] - add_off[j]);
            if (r.in_ring[id]) continue;
            r.in_ring[id] = 1;
            r.stamp[id] = r.next_stamp++;
            r.server_count++;
            add_ids.push_back(id);
            if (add_tokens)
                add_tok_sel.insert(add_tok_sel.end(), add_tokens + (uint64_t)j * r.R,
                                   add_tokens + (uint64_t)(j + 1) * r.R);
        }
        // :78-85 — then removes in order, skipping absent servers
        for (uint32_t j = 0; j < n_rem; j++) {
            const uint32_t id = r.nt.find(rem_bytes + rem_off[j], rem_off[j + 1] - rem_off[j]);
            if (id == rp::NIL || !r.in_ring[id]) continue;
            r.in_ring[id] = 0;
            r.server_count--;
            rem_ids.push_back(id);
            if (rem_tokens)
                rem_tok_sel.insert(rem_tok_sel.end(), rem_tokens + (uint64_t)j * r.R,
                                   rem_tokens + (uint64_t)(j + 1) * r.R);
        }
        const bool changed = !add_ids.empty() || !rem_ids.empty();
        if (changed) {
            r.nt.sync(r.st);
            rp::ring_apply_adds(r, add_ids, add_tokens ? &add_tok_sel : nullptr);
            rp::ring_apply_removes(r, rem_ids, rem_tokens ? &rem_tok_sel : nullptr);
            rp::ring_rebuild_index(r);
            rp::ring_compute_checksum(r);  // (89-91)
            RP_HIP(hipStreamSynchronize(r.st));
        }
        if (changed_out) *changed_out = changed ? 1 : 0;
    });
}

int rp_ring_checksum(rp_ring* h, uint32_t* out, int* is_set) {
    return guard_host([&] {
        rp::Ring& r = R(h);
        if (out) *out = r.checksum;
        if (is_set) *is_set = r.has_checksum ? 1 : 0;
    });
}

int rp_ring_checksum_string(rp_ring* h, char* buf, uint64_t cap, uint64_t* len) {
    return guard([&] {
        rp::Ring& r = R(h);
        uint64_t L = 0;
        const uint32_t nn = r.nt.size();
        svc_stop(r);
        if (r.has_checksum && nn) {
            uint32_t total = 0;
            RP_HIP(hipMemcpyAsync(&total, r.pos.p + nn, 4, hipMemcpyDeviceToHost, r.st));
            RP_HIP(hipStreamSynchronize(r.st));
            L = total ? total - 1 : 0;
        }
        if (len) *len = L;
        const uint64_t n = std::min<uint64_t>(cap, L);
        if (buf && n) {
            RP_HIP(hipMemcpyAsync(buf, r.ck_buf.p, n, hipMemcpyDeviceToHost, r.st));
            RP_HIP(hipStreamSynchronize(r.st));
        }
    });
}

int rp_ring_server_count(rp_ring* h, uint32_t* out) {
    return guard_host([&] { *out = R(h).server_count; });
}

int rp_ring_token_count(rp_ring* h, uint32_t* out) {
    return guard_host([&] { *out = R(h).M; });
}

int rp_ring_has_server(rp_ring* h, const char* name, uint32_t len, int* out) {
    return guard_host([&] {
        rp::Ring& r = R(h);
        const uint32_t id = r.nt.find(name, len);
        *out = (id != rp::NIL && r.in_ring[id]) ? 1 : 0;
    });
}

int rp_ring_server_id(rp_ring* h, const char* name, uint32_t len, uint32_t* id) {
    return guard_host([&] {
        rp::Ring& r = R(h);
        *id = r.nt.find(name, len);
    });
}

const char* rp_ring_owner_name(rp_ring* h, uint32_t id, uint32_t* len) {
    if (!h || id >= h->impl.nt.size()) {
        if (len) *len = 0;
        return nullptr;
    }
    if (len) *len = (uint32_t)h->impl.nt.names[id].size();
    return h->impl.nt.names[id].data();
}

int rp_ring_servers(rp_ring* h, uint32_t* ids_out, uint32_t cap, uint32_t* n) {
    return guard_host([&] {
        rp::Ring& r = R(h);
        std::vector<uint32_t> v;
        for (uint32_t id = 0; id < r.nt.size(); id++)
            if (r.in_ring[id]) v.push_back(id);
        std::sort(v.begin(), v.end(), [&](uint32_t a, uint32_t b) { return r.stamp[a] < r.stamp[b]; });
        *n = (uint32_t)v.size();
        for (uint32_t i = 0; i < v.size() && i < cap; i++) ids_out[i] = v[i];
    });
}

int rp_ring_dump(rp_ring* h, uint32_t* tokens, uint32_t* owners, uint32_t cap) {
    return guard([&] {
        rp::Ring& r = R(h);
        const uint32_t n = std::min(cap, r.M);
        svc_stop(r);
        if (n) {
            if (tokens) RP_HIP(hipMemcpyAsync(tokens, r.tok.p, sizeof(uint32_t) * n, hipMemcpyDeviceToHost, r.st));
            if (owners) RP_HIP(hipMemcpyAsync(owners, r.own.p, sizeof(uint32_t) * n, hipMemcpyDeviceToHost, r.st));
        }
        RP_HIP(hipStreamSynchronize(r.st));
    });
}

// ---- lookups

static int np_for(rp::Ring& r, int32_t nrep) {
    int64_t n = nrep;
    if (n > (int64_t)r.server_count) n = r.server_count;  // lib/ring/index.js:159-162
    return (int)n;
}

int rp_ring_lookupn_dev(rp_ring* h, const uint8_t* d_keys, const uint64_t* d_off, uint32_t stride, uint64_t n,
                        int32_t nrep, uint32_t* d_owners, uint8_t* d_counts, void* stream) {
    return guard([&] {
        rp::Ring& r = R(h);
        RP_REQUIRE(n == 0 || (d_keys && d_owners && (stride || d_off)), "lookupn_dev: null buffer");
        svc_stop(r);
        const uint32_t W = nrep > 1 ? (uint32_t)nrep : 1u;
        rp::launch_lookupn(r, d_keys, d_off, stride, nullptr, n, np_for(r, nrep), W, d_owners, d_counts,
                           rp::as_stream(stream));
    });
}

int rp_ring_lookup_dev(rp_ring* h, const uint8_t* d_keys, const uint64_t* d_off, uint32_t stride, uint64_t n,
                       uint32_t* d_owners, void* stream) {
    return guard([&] {
        rp::Ring& r = R(h);
        RP_REQUIRE(n == 0 || (d_keys && d_owners && (stride || d_off)), "lookup_dev: null buffer");
        svc_stop(r);
        // lookup (:145-154) == a one-step walk, independent of getServerCount
        rp::launch_lookupn(r, d_keys, d_off, stride, nullptr, n, 1, 1, d_owners, nullptr, rp::as_stream(stream));
    });
}

int rp_ring_lookupn_hashes_dev(rp_ring* h, const uint32_t* d_hashes, uint64_t n, int32_t nrep, uint32_t* d_owners,
                               uint8_t* d_counts, void* stream) {
    return guard([&] {
        rp::Ring& r = R(h);
        RP_REQUIRE(n == 0 || (d_hashes && d_owners), "lookupn_hashes_dev: null buffer");
        svc_stop(r);
        const uint32_t W = nrep > 1 ? (uint32_t)nrep : 1u;
        rp::launch_lookupn(r, nullptr, nullptr, 0, d_hashes, n, np_for(r, nrep), W, d_owners, d_counts,
                           rp::as_stream(stream));
    });
}

// host-buffer forms: stage through the handle's device buffers on its stream
// The small path: at most kSmallKeys keys of kSmallBytes in all, rows of at most kSmallW owners,
// on the wide view (binary search + the reference walk). RP_RING_SMALL=0 turns it off (A/B).
static bool host_lookup_small(rp::Ring& r, const char* keys, const uint64_t* off, uint32_t stride, uint64_t n, int np,
                              uint32_t W, uint32_t* owners, uint8_t* counts) {
    using namespace rp;
    const char* se = getenv("RP_RING_SMALL");
    const bool on = !(se && !strcmp(se, "0"));
    const int need = np <= 0 ? 1 : np;
    if (!on || n > kSmallKeys || W > kSmallW || need > 8 || r.M == 0) return false;
    const uint64_t bytes = stride ? n * stride : off[n] - off[0];
    if (bytes > kSmallBytes) return false;
    SmallKeys sk;
    sk.n = (uint32_t)n;
    for (uint64_t k = 0; k <= n; k++) sk.off[k] = (uint16_t)(stride ? k * stride : off[k] - off[0]);
    memcpy(sk.b, keys + (stride ? 0 : off[0]), bytes);
    if (!r.pin_out) {
        RP_HIP(hipHostMalloc(reinterpret_cast<void**>(&r.pin_out), 4ull * kSmallKeys * kSmallW, hipHostMallocMapped));
        RP_HIP(hipHostMalloc(reinterpret_cast<void**>(&r.pin_cnt), kSmallKeys, hipHostMallocMapped));
        RP_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&r.pin_out_dev), r.pin_out, 0));
        RP_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&r.pin_cnt_dev), r.pin_cnt, 0));
    }
    const auto rv = r.view();
    uint8_t* cd = counts ? r.pin_cnt_dev : nullptr;
    if (need == 1)
        hipLaunchKernelGGL((k_lookupn_small<1, decltype(rv)>), dim3(1), dim3(64), 0, r.st, sk, rv, np, W, r.pin_out_dev, cd);
    else if (need <= 4)
        hipLaunchKernelGGL((k_lookupn_small<4, decltype(rv)>), dim3(1), dim3(64), 0, r.st, sk, rv, np, W, r.pin_out_dev, cd);
    else
        hipLaunchKernelGGL((k_lookupn_small<8, decltype(rv)>), dim3(1), dim3(64), 0, r.st, sk, rv, np, W, r.pin_out_dev, cd);
    RP_HIP(hipGetLastError());
    RP_HIP(hipStreamSynchronize(r.st));
    memcpy(owners, r.pin_out, 4ull * n * W);
    if (counts) memcpy(counts, r.pin_cnt, n);
    return true;
}

// one key (or, with hash non-null, one caller hash) through the service: false when it does not
// apply (off, a wide row; the round-4 kernel: a long key or a caller hash)
static bool svc_lookup(rp::Ring& r, const char* key, uint32_t len, const uint32_t* hash, int np, uint32_t W,
                       uint32_t* owners, uint8_t* counts) {
    using namespace rp;
    const int need = np <= 0 ? 1 : np;
    if (!r.svc_idle_ms || W > 8 || need > 8 || r.M == 0) return false;
    if (!r.svc_v2 && (hash || len > kSvcKeyMax)) return false;
    if (g_quiet.load() > 0) return false;  // another thread's device call is running
    if (g_svc_live.load() > (r.svc_live.load() ? 1 : 0)) rp::svc_quiesce(&r);  // another ring's wave
    std::lock_guard<std::recursive_mutex> lk(r.svc_mu);
    if (!r.svc) {
        RP_HIP(hipHostMalloc(reinterpret_cast<void**>(&r.svc), sizeof(SvcLines), hipHostMallocMapped | hipHostMallocCoherent));
        memset(r.svc, 0, sizeof(SvcLines));
        RP_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&r.svc_dev), r.svc, 0));
        RP_HIP(hipStreamCreateWithFlags(&r.svc_st, hipStreamNonBlocking));
        r.svc_seq = 0;
    }
    SvcLines* io = r.svc;
    // a wave is needed: none launched, or the last one exited (idle or lifetime). Announce it in
    // g_svc_live before reading g_quiet (the QuietScope handshake, rp_common.h); while another
    // thread's device call runs, this lookup takes the launch path instead.
    bool launch = false;
    if (!r.svc_live.load()) {
        r.svc_live.store(true);
        g_svc_live.fetch_add(1);
        if (g_quiet.load() > 0) {
            r.svc_live.store(false);
            g_svc_live.fetch_sub(1);
            return false;
        }
        launch = true;
    } else if (hipStreamQuery(r.svc_st) == hipSuccess) {
        launch = true;
    }
    const uint32_t s = r.svc_seq + 1;
    if (r.svc_v2) {
        // the key's hash, on the host as the reference computes it (lib/ring/index.js:145-154)
        io->req[1] = hash ? *hash : fh::hash32(fh::PtrSrc{reinterpret_cast<const uint8_t*>(key)}, len);
    } else {
        for (uint32_t c = 0; c * 60 < len; c++) {  // each key line's bytes, then its seq
            memcpy(&io->req[16 * (c + 1)], key + 60 * c, std::min<uint32_t>(60, len - 60 * c));
            __atomic_store_n(&io->req[16 * (c + 1) + 15], s, __ATOMIC_RELEASE);
        }
        io->req[1] = len;
    }
    io->req[2] = (uint32_t)np;
    io->req[3] = W;
    __atomic_store_n(&io->req[15], s, __ATOMIC_RELEASE);  // the header's trailing copy of seq
    __atomic_store_n(&io->req[0], s, __ATOMIC_RELEASE);
    if (launch) svc_launch(r, s - 1);
    uint64_t spins = 0;
    const auto t0 = std::chrono::steady_clock::now();
    // v2: the answer line is taken when all 8 of its words carry seq s (no torn line)
    auto answered = [&]() -> bool {
        if (!r.svc_v2) return __atomic_load_n(&io->resp_seq[0], __ATOMIC_ACQUIRE) == s;
        const uint64_t* a = io->resp2[s & 7u];
        if ((uint32_t)(__atomic_load_n(&a[7], __ATOMIC_ACQUIRE) >> 32) != s) return false;
        for (int q = 0; q < 7; q++)
            if ((uint32_t)(__atomic_load_n(&a[q], __ATOMIC_ACQUIRE) >> 32) != s) return false;
        return true;
    };
    while (!answered()) {
        __builtin_ia32_pause();
        if ((++spins & 4095) == 0) {
            if (hipStreamQuery(r.svc_st) == hipSuccess && !answered()) {
                svc_launch(r, s - 1);  // it exited (idle or lifetime) before taking this request
            }
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(5)) {
                svc_stop(r);
                throw Error(RP_EDEVICE, "lookup service: no answer within 5 s");
            }
        }
    }
    r.svc_seq = s;
    if (r.svc_v2 && getenv("RP_SVC_PROF") && __atomic_load_n(&io->diag[0], __ATOMIC_ACQUIRE) == s) {
        r.svc_prof[0] += io->diag[1];
        r.svc_prof[1] += io->diag[2];
        r.svc_prof[4 + (io->diag[3] & 3)]++;
        r.svc_prof[8]++;
    }
    if (r.svc_v2) {
        uint32_t c = 0;
        for (uint32_t q = 0; q < W; q++) {
            owners[q] = (uint32_t)io->resp2[s & 7u][q];
            c += (c == q && owners[q] != NIL) ? 1u : 0u;
        }
        if (counts) counts[0] = (uint8_t)c;
        return true;
    }
    for (uint32_t q = 0; q < W; q++) owners[q] = io->resp[q];
    if (counts) counts[0] = (uint8_t)io->resp[15];
    return true;
}

static void host_lookup(rp::Ring& r, const char* keys, const uint64_t* off, uint32_t stride, const uint32_t* hashes,
                        uint64_t n, int np, uint32_t W, uint32_t* owners, uint8_t* counts) {
    if (n == 0) return;
    if (n == 1 && (hashes ? svc_lookup(r, nullptr, 0, hashes, np, W, owners, counts)
                          : svc_lookup(r, keys + (stride ? 0 : off[0]), (uint32_t)(stride ? stride : off[1] - off[0]),
                                       nullptr, np, W, owners, counts)))
        return;
    rp::QuietScope quiet;  // the launch path: no resident service (this ring's or another's) meanwhile
    svc_stop(r);
    if (!hashes && host_lookup_small(r, keys, off, stride, n, np, W, owners, counts)) return;
    const uint8_t* dk = nullptr;
    const uint64_t* doff = nullptr;
    const uint32_t* dh = nullptr;
    if (hashes) {
        r.io_a.reserve(n);
        RP_HIP(hipMemcpyAsync(r.io_a.p, hashes, n * 4, hipMemcpyHostToDevice, r.st));
        dh = r.io_a.p;
    } else {
        const uint64_t bytes = stride ? n * stride : off[n];
        r.io_keys.reserve(bytes + 16);
        RP_HIP(hipMemcpyAsync(r.io_keys.p, keys, bytes, hipMemcpyHostToDevice, r.st));
        dk = r.io_keys.p;
        if (!stride) {
            r.io_off.reserve(n + 1);
            RP_HIP(hipMemcpyAsync(r.io_off.p, off, (n + 1) * 8, hipMemcpyHostToDevice, r.st));
            doff = r.io_off.p;
        }
    }
    r.io_b.reserve(n * W);
    if (counts) r.io_cnt.reserve(n);
    rp::launch_lookupn(r, dk, doff, stride, dh, n, np, W, r.io_b.p, counts ? r.io_cnt.p : nullptr, r.st);
    RP_HIP(hipMemcpyAsync(owners, r.io_b.p, n * W * 4, hipMemcpyDeviceToHost, r.st));
    if (counts) RP_HIP(hipMemcpyAsync(counts, r.io_cnt.p, n, hipMemcpyDeviceToHost, r.st));
    RP_HIP(hipStreamSynchronize(r.st));
}

int rp_ring_service(rp_ring* h, uint32_t idle_ms) {
    return guard([&] {
        rp::Ring& r = R(h);
        svc_stop(r);
        svc_register(r, idle_ms > 0);
        r.svc_idle_ms = idle_ms;
        r.svc_v2 = !(getenv("RP_RING_SVC") && !strcmp(getenv("RP_RING_SVC"), "1"));
    });
}

int rp_ring_lookup(rp_ring* h, const char* keys, const uint64_t* off, uint32_t stride, uint64_t n, uint32_t* owners) {
    return guard_host([&] {
        rp::Ring& r = R(h);
        RP_REQUIRE(n == 0 || (keys && owners && (stride || off)), "lookup: null buffer");
        host_lookup(r, keys, off, stride, nullptr, n, 1, 1, owners, nullptr);
    });
}

int rp_ring_lookupn(rp_ring* h, const char* keys, const uint64_t* off, uint32_t stride, uint64_t n, int32_t nrep,
                    uint32_t* owners, uint8_t* counts) {
    return guard_host([&] {
        rp::Ring& r = R(h);
        RP_REQUIRE(n == 0 || (keys && owners && (stride || off)), "lookupn: null buffer");
        host_lookup(r, keys, off, stride, nullptr, n, np_for(r, nrep), nrep > 1 ? (uint32_t)nrep : 1u, owners,
                    counts);
    });
}

int rp_ring_lookup_hashes(rp_ring* h, const uint32_t* hashes, uint64_t n, uint32_t* owners) {
    return guard_host([&] {
        rp::Ring& r = R(h);
        RP_REQUIRE(n == 0 || (hashes && owners), "lookup_hashes: null buffer");
        host_lookup(r, nullptr, nullptr, 0, hashes, n, 1, 1, owners, nullptr);
    });
}

int rp_ring_lookupn_hashes(rp_ring* h, const uint32_t* hashes, uint64_t n, int32_t nrep, uint32_t* owners,
                           uint8_t* counts) {
    return guard_host([&] {
        rp::Ring& r = R(h);
        RP_REQUIRE(n == 0 || (hashes && owners), "lookupn_hashes: null buffer");
        host_lookup(r, nullptr, nullptr, 0, hashes, n, np_for(r, nrep), nrep > 1 ? (uint32_t)nrep : 1u, owners,
                    counts);
    });
}

// ---- group keys by owner (handleOrProxyAll / lookupKeys)

int rp_ring_group_keys_dev(rp_ring* h, const uint8_t* d_keys, const uint64_t* d_off, uint32_t stride, uint64_t n,
                           uint32_t self_id, uint32_t* d_dests, uint32_t* d_group_off, uint32_t* d_perm,
                           uint32_t* d_ndest, void* stream) {
    return guard([&] {
        rp::Ring& r = R(h);
        RP_REQUIRE(d_dests && d_group_off && d_perm && d_ndest, "group_keys_dev: null output buffer");
        RP_REQUIRE(n == 0 || (d_keys && (stride || d_off)), "group_keys_dev: null key buffer");
        svc_stop(r);
        rp::group_keys(r, d_keys, d_off, stride, nullptr, n, self_id, d_dests, d_group_off, d_perm, d_ndest,
                       rp::as_stream(stream));
    });
}

// host-buffer forms: keys (or a caller hashFunc's key hashes) in, groups out
static void host_group(rp::Ring& r, const char* keys, const uint64_t* off, uint32_t stride, const uint32_t* hashes,
                       uint64_t n, uint32_t self_id, uint32_t* dests, uint32_t* goff, uint32_t* perm, uint32_t* ndest) {
    RP_REQUIRE(dests && goff && perm && ndest, "group_keys: null output buffer");
    svc_stop(r);
    const uint8_t* dk = nullptr;
    const uint64_t* doff = nullptr;
    const uint32_t* dh = nullptr;
    if (n && hashes) {
        r.io_a.reserve(n);
        RP_HIP(hipMemcpyAsync(r.io_a.p, hashes, n * 4, hipMemcpyHostToDevice, r.st));
        dh = r.io_a.p;
    } else if (n) {
        const uint64_t bytes = stride ? n * stride : off[n];
        r.io_keys.reserve(bytes + 16);
        RP_HIP(hipMemcpyAsync(r.io_keys.p, keys, bytes, hipMemcpyHostToDevice, r.st));
        dk = r.io_keys.p;
        if (!stride) {
            r.io_off.reserve(n + 1);
            RP_HIP(hipMemcpyAsync(r.io_off.p, off, (n + 1) * 8, hipMemcpyHostToDevice, r.st));
            doff = r.io_off.p;
        }
    }
    // io_b = [perm n | group_off n+1 | dests n | ndest 1]
    const uint64_t nn = n ? n : 1;
    r.io_b.reserve(3 * nn + 2);
    uint32_t* dperm = r.io_b.p;
    uint32_t* dgoff = dperm + nn;
    uint32_t* ddest = dgoff + nn + 1;
    uint32_t* dnd = ddest + nn;
    rp::group_keys(r, dk, doff, stride, dh, n, self_id, ddest, dgoff, dperm, dnd, r.st);
    uint32_t nd = 0;
    RP_HIP(hipMemcpyAsync(&nd, dnd, 4, hipMemcpyDeviceToHost, r.st));
    RP_HIP(hipStreamSynchronize(r.st));
    *ndest = nd;
    if (n) RP_HIP(hipMemcpyAsync(perm, dperm, n * 4, hipMemcpyDeviceToHost, r.st));
    if (nd) RP_HIP(hipMemcpyAsync(dests, ddest, 4ull * nd, hipMemcpyDeviceToHost, r.st));
    RP_HIP(hipMemcpyAsync(goff, dgoff, 4ull * (nd + 1), hipMemcpyDeviceToHost, r.st));
    RP_HIP(hipStreamSynchronize(r.st));
}

int rp_ring_group_keys(rp_ring* h, const char* keys, const uint64_t* off, uint32_t stride, uint64_t n,
                       uint32_t self_id, uint32_t* dests, uint32_t* group_off, uint32_t* perm, uint32_t* ndest) {
    return guard([&] {
        rp::Ring& r = R(h);
        RP_REQUIRE(n == 0 || (keys && (stride || off)), "group_keys: null key buffer");
        host_group(r, keys, off, stride, nullptr, n, self_id, dests, group_off, perm, ndest);
    });
}

int rp_ring_group_hashes(rp_ring* h, const uint32_t* hashes, uint64_t n, uint32_t self_id, uint32_t* dests,
                         uint32_t* group_off, uint32_t* perm, uint32_t* ndest) {
    return guard([&] {
        rp::Ring& r = R(h);
        RP_REQUIRE(n == 0 || hashes, "group_hashes: null hash buffer");
        host_group(r, nullptr, nullptr, 0, hashes, n, self_id, dests, group_off, perm, ndest);
    });
}

// ---- farmhash + key generation

uint32_t rp_hash32(const char* s, size_t len) {
    return rp::fh::hash32(rp::fh::PtrSrc{reinterpret_cast<const uint8_t*>(s)}, (uint32_t)len);
}

int rp_hash32_batch_dev(const uint8_t* d_bytes, const uint64_t* d_off, uint64_t n, uint32_t* d_out, void* stream) {
    return guard([&] {
        if (!n) return;
        RP_REQUIRE(d_bytes && d_off && d_out, "hash32_batch_dev: null buffer");
        hipLaunchKernelGGL(rp::k_hash_batch, dim3(rp::grid_for(n, 256)), dim3(256), 0, rp::as_stream(stream), d_bytes,
                           d_off, n, d_out);
        RP_HIP(hipGetLastError());
    });
}

int rp_hash32_long_dev(const uint8_t* d_bytes, uint64_t len, uint32_t* d_out, void* stream) {
    return guard([&] {
        RP_REQUIRE(d_out && (d_bytes || len == 0), "hash32_long_dev: null buffer");
        RP_REQUIRE(len < (1ull << 32), "hash32_long_dev: at most 2^32-1 bytes");
        rp::hash_long(d_bytes, len, nullptr, nullptr, d_out, rp::as_stream(stream));
    });
}

int rp_hash32_long_multi_dev(const uint8_t* d_bytes, uint64_t stride, uint32_t n, uint32_t* d_meta, void* stream) {
    return guard([&] {
        RP_REQUIRE(n == 0 || (d_bytes && d_meta), "hash32_long_multi_dev: null buffer");
        rp::hash_long_multi(d_bytes, stride, n, d_meta, rp::as_stream(stream));
    });
}

int rp_gen_uuid_keys_dev(uint32_t seed, uint64_t k0, uint64_t n, uint8_t* d_out, void* stream) {
    return guard([&] {
        if (!n) return;
        RP_REQUIRE(d_out && (reinterpret_cast<uintptr_t>(d_out) & 3) == 0, "gen_uuid_keys_dev: need 4-byte aligned out");
        hipLaunchKernelGGL(rp::k_gen_uuid, dim3(rp::grid_for(n, 256, 8192)), dim3(256), 0, rp::as_stream(stream), seed,
                           k0, n, reinterpret_cast<uint32_t*>(d_out));
        RP_HIP(hipGetLastError());
    });
}

}  // extern "C"
