// ub_lookup.hip — microbenchmark of the lookup kernel's access pattern (design tool, not product).
//
// Streams 2^26 36-byte keys (16-B nt loads -> LDS), farmhash32 per key, then touches a table of
// T bytes in one of several patterns, and writes 12 B per key (LDS -> 16-B nt stores):
//   none      : no table access (the hash-only floor)
//   r16       : one random 16-B load per key
//   r8r16     : two dependent random loads (8 B, then 16 B) — the current probe kernel's shape
//   line64    : one lane loads a whole random 64-B line (4 x 16 B)
//   line128   : one lane loads a whole random 128-B line (8 x 16 B)
//   coop128   : 8 lanes per key load one random 128-B line (one 16-B load each)
//   lds+r16   : a 15-step binary search in a 64 KB LDS array, then one random 16-B load
// for T in {0.5 .. 8} MB. Prints ms and algorithmic GB/s (48 B per key).
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -o /tmp/ub tools/ub_lookup.hip && /tmp/ub
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../ringpop-node_amd/csrc/rp_farmhash.h"

#define CK(x)                                                                             \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
            exit(1);                                                                      \
        }                                                                                 \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4_a1 __attribute__((ext_vector_type(4), aligned(1)));

constexpr int T = 256, LEN = 36, W4 = 9;

enum { NONE = 0, R16, R8R16, LINE64, COOP64, R16U, R16A2, R8R16U, R16W4, R16W8 };

// per-key table probe; KPL keys are issued together so their loads overlap
template <int MODE, int KPL>
__device__ __forceinline__ void probe(const uint32_t (&h)[KPL], const uint32_t* __restrict__ tab, uint32_t nlines64,
                                      uint32_t (&r)[KPL][3]) {
#pragma unroll
    for (int k = 0; k < KPL; k++) {
        r[k][0] = h[k];
        r[k][1] = h[k] + 1;
        r[k][2] = h[k] + 2;
    }
    if constexpr (MODE == R16) {
        u32x4 v[KPL];
#pragma unroll
        for (int k = 0; k < KPL; k++) {
            const uint32_t l = (uint32_t)(((uint64_t)h[k] * nlines64) >> 32);
            v[k] = *reinterpret_cast<const u32x4*>(tab + l * 16 + (h[k] & 3) * 4);
        }
#pragma unroll
        for (int k = 0; k < KPL; k++) {
            r[k][0] ^= v[k].x + v[k].w;
            r[k][1] ^= v[k].y;
            r[k][2] ^= v[k].z;
        }
    } else if constexpr (MODE == R16W4 || MODE == R16W8) {
        // a 16-B load at a 4-B (R16W4) or 8-B (R16W8) aligned, not 16-B aligned, address
        const uint32_t nent = nlines64 * 64 / 3 - 16;
        u32x4 v[KPL];
#pragma unroll
        for (int k = 0; k < KPL; k++) {
            const uint32_t pos = (uint32_t)(((uint64_t)h[k] * nent) >> 32);
            const uintptr_t a = (uintptr_t)(reinterpret_cast<const uint8_t*>(tab) + 3ull * pos) & (MODE == R16W4 ? ~(uintptr_t)3 : ~(uintptr_t)7);
            v[k] = *reinterpret_cast<const u32x4_a1*>(a);
        }
#pragma unroll
        for (int k = 0; k < KPL; k++) {
            r[k][0] ^= v[k].x + v[k].w;
            r[k][1] ^= v[k].y;
            r[k][2] ^= v[k].z;
        }
    } else if constexpr (MODE == R16U || MODE == R16A2) {
        // a 16-B window of 3-B entries at entry position pos: one unaligned load (R16U), or the
        // two aligned 16-B chunks that cover it (R16A2)
        const uint32_t nent = nlines64 * 64 / 3 - 16;
        u32x4 v[KPL], u[KPL];
#pragma unroll
        for (int k = 0; k < KPL; k++) {
            const uint32_t pos = (uint32_t)(((uint64_t)h[k] * nent) >> 32);
            const uint8_t* p = reinterpret_cast<const uint8_t*>(tab) + 3ull * pos;
            if constexpr (MODE == R16U) {
                v[k] = *reinterpret_cast<const u32x4_a1*>(p);
                u[k] = v[k];
            } else {
                const u32x4* a = reinterpret_cast<const u32x4*>((uintptr_t)p & ~(uintptr_t)15);
                v[k] = a[0];
                u[k] = a[1];
            }
        }
#pragma unroll
        for (int k = 0; k < KPL; k++) {
            r[k][0] ^= v[k].x + u[k].w;
            r[k][1] ^= v[k].y ^ u[k].z;
            r[k][2] ^= v[k].z + u[k].x;
        }
    } else if constexpr (MODE == R8R16U) {
        // the compact kernel's shape: an 8-B index record, then an unaligned 16-B window
        const uint32_t nw = nlines64 * 16;
        u32x2 b[KPL];
#pragma unroll
        for (int k = 0; k < KPL; k++) {
            const uint32_t a = (uint32_t)(((uint64_t)h[k] * (nw / 8 - 1)) >> 32);  // first eighth: 512 KB
            b[k] = *reinterpret_cast<const u32x2*>(tab + 2 * a);
        }
        u32x4 v[KPL];
#pragma unroll
        for (int k = 0; k < KPL; k++) {
            const uint32_t c = (nw * 4 / 8) + ((b[k].x ^ h[k]) % (nw * 4 / 8 * 7 - 64));
            v[k] = *reinterpret_cast<const u32x4_a1*>(reinterpret_cast<const uint8_t*>(tab) + c);
        }
#pragma unroll
        for (int k = 0; k < KPL; k++) {
            r[k][0] ^= v[k].x + b[k].y;
            r[k][1] ^= v[k].y;
            r[k][2] ^= v[k].z + v[k].w;
        }
    } else if constexpr (MODE == R8R16) {
        const uint32_t nw = nlines64 * 16;
        u32x2 b[KPL];
#pragma unroll
        for (int k = 0; k < KPL; k++) {
            const uint32_t a = (uint32_t)(((uint64_t)h[k] * (nw / 4 - 1)) >> 32);  // first quarter
            b[k] = *reinterpret_cast<const u32x2*>(tab + a);
        }
        u32x4 v[KPL];
#pragma unroll
        for (int k = 0; k < KPL; k++) {
            const uint32_t c = (nw / 4) + ((b[k].x ^ h[k]) % (nw / 4 * 3 - 4));
            v[k] = *reinterpret_cast<const u32x4*>(tab + (c & ~3u));
        }
#pragma unroll
        for (int k = 0; k < KPL; k++) {
            r[k][0] ^= v[k].x + b[k].y;
            r[k][1] ^= v[k].y;
            r[k][2] ^= v[k].z + v[k].w;
        }
    } else if constexpr (MODE == LINE64) {
#pragma unroll
        for (int k = 0; k < KPL; k++) {
            const uint32_t l = (uint32_t)(((uint64_t)h[k] * nlines64) >> 32);
            const u32x4* p = reinterpret_cast<const u32x4*>(tab + l * 16);
            uint32_t acc = 0;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const u32x4 v = p[q];
                acc += (v.x < h[k]) + (v.y < h[k]) + (v.z < h[k]) + (v.w < h[k]);
            }
            r[k][0] ^= acc;
        }
    } else if constexpr (MODE == COOP64) {
        const int lane = threadIdx.x & 63, g0 = lane & ~3, sub = lane & 3;
#pragma unroll
        for (int k = 0; k < KPL; k++) {
            uint32_t mine = 0;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const uint32_t hk = __shfl(h[k], g0 + q, 64);
                const uint32_t l = (uint32_t)(((uint64_t)hk * nlines64) >> 32);
                const u32x4 v = *reinterpret_cast<const u32x4*>(tab + l * 16 + sub * 4);
                uint32_t c = (v.x < hk) + (v.y < hk) + (v.z < hk) + (v.w < hk);
                c += __shfl_xor(c, 1, 64);
                c += __shfl_xor(c, 2, 64);
                mine = (sub == q) ? c : mine;
            }
            r[k][0] ^= mine;
        }
    }
}

template <int MODE, int KPL = 1, bool PIPE = false>
__global__ __launch_bounds__(T) void k_ub(const uint8_t* __restrict__ keys, uint64_t n, const uint32_t* __restrict__ tab,
                                          uint32_t nlines64, uint32_t* __restrict__ out) {
    constexpr int TK = T * KPL;
    constexpr int V4 = TK * W4 / 4;
    constexpr int PER = (V4 + T - 1) / T;
    __shared__ __attribute__((aligned(16))) uint32_t sk[TK * W4];
    const int tid = threadIdx.x;
    const uint64_t ntiles = n / TK;
    u32x4 pre[PER];
    auto issue = [&](uint64_t t) {
        const u32x4* s4 = reinterpret_cast<const u32x4*>(keys + t * TK * LEN);
#pragma unroll
        for (int q = 0; q < PER; q++) {
            const int k = tid + q * T;
            if (k < V4) pre[q] = __builtin_nontemporal_load(s4 + k);
        }
    };
    uint64_t t = blockIdx.x;
    if (PIPE && t < ntiles) issue(t);
    for (; t < ntiles; t += gridDim.x) {
        if (!PIPE) issue(t);
#pragma unroll
        for (int q = 0; q < PER; q++) {
            const int k = tid + q * T;
            if (k < V4) reinterpret_cast<u32x4*>(sk)[k] = pre[q];
        }
        __syncthreads();
        if (PIPE && t + gridDim.x < ntiles) issue(t + gridDim.x);
        uint32_t h[KPL];
#pragma unroll
        for (int k = 0; k < KPL; k++) {
            uint32_t w[W4];
#pragma unroll
            for (int j = 0; j < W4; j++) w[j] = sk[(tid + k * T) * W4 + j];
            h[k] = rp::fh::hash32_words<LEN>(w);
        }
        uint32_t r[KPL][3];
        probe<MODE, KPL>(h, tab, nlines64, r);
        __syncthreads();
#pragma unroll
        for (int k = 0; k < KPL; k++) {
#pragma unroll
            for (int q = 0; q < 3; q++) sk[(tid + k * T) * 3 + q] = r[k][q];
        }
        __syncthreads();
        u32x4* d4 = reinterpret_cast<u32x4*>(out + t * TK * 3);
        for (int k = tid; k < TK * 3 / 4; k += T) __builtin_nontemporal_store(reinterpret_cast<const u32x4*>(sk)[k], d4 + k);
        __syncthreads();
    }
}

__global__ void k_fill(uint32_t* p, uint64_t n, uint32_t seed) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        p[i] = rp::fh::fmix((uint32_t)i * 0x9E3779B9u + seed);
}

template <int MODE, int KPL, bool PIPE>
static float run(const uint8_t* keys, uint64_t n, const uint32_t* tab, uint32_t nlines64, uint32_t* out, int grid) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<float> ts;
    for (int rep = 0; rep < 7; rep++) {
        CK(hipEventRecord(a));
        k_ub<MODE, KPL, PIPE><<<grid, T>>>(keys, n, tab, nlines64, out);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    return ts[3];
}

static const double kMB[] = {2, 3, 4, 6, 8};

template <int MODE, int KPL, bool PIPE>
static void row(const char* name, const uint8_t* keys, uint64_t n, const uint32_t* tab, uint32_t* out, int grid) {
    printf("%-8s kpl%d %s", name, KPL, PIPE ? "pipe" : "sync");
    for (double mb : kMB) printf(" %8.3f", run<MODE, KPL, PIPE>(keys, n, tab, (uint32_t)(mb * 16384.0), out, grid));
    printf("\n");
    fflush(stdout);
}

template <int MODE>
static void rows(const char* name, const uint8_t* keys, uint64_t n, const uint32_t* tab, uint32_t* out, int grid) {
    row<MODE, 1, false>(name, keys, n, tab, out, grid);
    row<MODE, 1, true>(name, keys, n, tab, out, grid);
    row<MODE, 2, false>(name, keys, n, tab, out, grid);
    row<MODE, 2, true>(name, keys, n, tab, out, grid);
    row<MODE, 4, false>(name, keys, n, tab, out, grid);
}


// LDS-resident bucket index (the candidate one-global-access layout): a 512-thread workgroup
// holds a 140 KB index in LDS (2^18 4-bit bucket counts + 3-B bases per 64 buckets, emulated
// with random words). Each wave streams its own keys (no workgroup barriers): 64 keys = 144
// 16-B vectors per sub-tile, KPL sub-tiles per round, the next round's vectors prefetched into
// registers while this round hashes; keys pass through a 2.3 KB per-wave LDS buffer. Per key:
// two LDS reads (count word, base) -> position -> NWIN adjacent random 16-B global loads.
constexpr int TL = 512;
constexpr int IDXW = (128 + 12) * 1024 / 4;  // index words in LDS
template <int KPL, int NWIN>
__global__ __launch_bounds__(TL) void k_ub_lds(const uint8_t* __restrict__ keys, uint64_t n,
                                               const uint32_t* __restrict__ tab, uint32_t nlines64,
                                               const uint32_t* __restrict__ gidx, uint32_t* __restrict__ out) {
    constexpr int TW = 64 * KPL;  // keys per wave per round
    __shared__ __attribute__((aligned(16))) uint32_t idx[IDXW];
    __shared__ __attribute__((aligned(16))) uint32_t sk[TL / 64][64 * W4];  // 2304 B per wave
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    for (int i = tid; i < IDXW / 4; i += TL) reinterpret_cast<u32x4*>(idx)[i] = reinterpret_cast<const u32x4*>(gidx)[i];
    __syncthreads();
    uint32_t* const buf = sk[wv];
    const uint64_t nw = n / TW;  // wave-rounds
    const uint64_t wstride = (uint64_t)gridDim.x * (TL / 64);
    const uint32_t nent = nlines64 * 64 / 3 - 16;
    u32x4 pre[KPL][3];
    auto issue = [&](uint64_t r) {
        const u32x4* s4 = reinterpret_cast<const u32x4*>(keys + r * TW * LEN);
#pragma unroll
        for (int k = 0; k < KPL; k++)
#pragma unroll
            for (int q = 0; q < 3; q++) {
                const int v = lane + 64 * q;
                if (v < 144) pre[k][q] = __builtin_nontemporal_load(s4 + k * 144 + v);
            }
    };
    uint64_t t = blockIdx.x * (uint64_t)(TL / 64) + wv;
    if (t < nw) issue(t);
    for (; t < nw; t += wstride) {
        uint32_t h[KPL];
#pragma unroll
        for (int k = 0; k < KPL; k++) {
#pragma unroll
            for (int q = 0; q < 3; q++) {
                const int v = lane + 64 * q;
                if (v < 144) reinterpret_cast<u32x4*>(buf)[v] = pre[k][q];
            }
            uint32_t w[W4];
#pragma unroll
            for (int j = 0; j < W4; j++) w[j] = buf[lane * W4 + j];
            h[k] = rp::fh::hash32_words<LEN>(w);
        }
        if (t + wstride < nw) issue(t + wstride);
        constexpr int NV = NWIN > 0 ? NWIN : 1;
        uint32_t r[KPL][3];
        u32x4 v[KPL][NV];
#pragma unroll
        for (int k = 0; k < KPL; k++) {
            const uint32_t b = h[k] >> 14;                  // 2^18 buckets
            const uint32_t cw = idx[b >> 3];                // 8 nibbles
            const uint32_t base = idx[32768 + (b >> 6)] & 0xFFFFFu;
            const uint32_t s4 = (b & 7) * 4;
            const uint32_t below = cw & ((1u << s4) - 1u);
            const uint32_t x = (below & 0x0F0F0F0Fu) + ((below >> 4) & 0x0F0F0F0Fu);
            const uint32_t pos = (base + ((x * 0x01010101u) >> 24) + (b & 63) * 4) % nent;
            const uint8_t* p = reinterpret_cast<const uint8_t*>(tab) + 3ull * pos;
            if constexpr (NWIN == 0) {
                v[k][0] = u32x4{pos, pos, pos, pos};
            } else {
#pragma unroll
                for (int q = 0; q < NWIN; q++) v[k][q] = *reinterpret_cast<const u32x4_a1*>(p + 16 * q);
            }
        }
#pragma unroll
        for (int k = 0; k < KPL; k++) {
            r[k][0] = h[k] ^ v[k][0].x;
            r[k][1] = v[k][0].y + v[k][NV - 1].z;
            r[k][2] = v[k][0].w ^ v[k][NV - 1].x;
        }
        // 64 keys x 12 B = 768 B per sub-tile out through the wave buffer
        u32x4* d4 = reinterpret_cast<u32x4*>(out + t * TW * 3);
#pragma unroll
        for (int k = 0; k < KPL; k++) {
#pragma unroll
            for (int q = 0; q < 3; q++) buf[lane * 3 + q] = r[k][q];
            if (lane < 48) __builtin_nontemporal_store(reinterpret_cast<const u32x4*>(buf)[lane], d4 + k * 48 + lane);
        }
    }
}

// The same with the table loads software-pipelined against the next round's hashing: round t's
// windows are issued, round t+1 is hashed while they are in flight, then round t is finished.
template <int KPL, int NWIN>
__global__ __launch_bounds__(TL) void k_ub_lds2(const uint8_t* __restrict__ keys, uint64_t n,
                                                const uint32_t* __restrict__ tab, uint32_t nlines64,
                                                const uint32_t* __restrict__ gidx, uint32_t* __restrict__ out) {
    constexpr int TW = 64 * KPL;
    constexpr int NV = NWIN > 0 ? NWIN : 1;
    __shared__ __attribute__((aligned(16))) uint32_t idx[IDXW];
    __shared__ __attribute__((aligned(16))) uint32_t sk[TL / 64][64 * W4];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    for (int i = tid; i < IDXW / 4; i += TL) reinterpret_cast<u32x4*>(idx)[i] = reinterpret_cast<const u32x4*>(gidx)[i];
    __syncthreads();
    uint32_t* const buf = sk[wv];
    const uint64_t nw = n / TW;
    const uint64_t wstride = (uint64_t)gridDim.x * (TL / 64);
    const uint32_t nent = nlines64 * 64 / 3 - 16;
    u32x4 pre[KPL][3];
    auto issue = [&](uint64_t r) {
        const u32x4* s4 = reinterpret_cast<const u32x4*>(keys + r * TW * LEN);
#pragma unroll
        for (int k = 0; k < KPL; k++)
#pragma unroll
            for (int q = 0; q < 3; q++) {
                const int v = lane + 64 * q;
                if (v < 144) pre[k][q] = __builtin_nontemporal_load(s4 + k * 144 + v);
            }
    };
    auto hash_round = [&](uint32_t (&h)[KPL]) {
#pragma unroll
        for (int k = 0; k < KPL; k++) {
#pragma unroll
            for (int q = 0; q < 3; q++) {
                const int v = lane + 64 * q;
                if (v < 144) reinterpret_cast<u32x4*>(buf)[v] = pre[k][q];
            }
            uint32_t w[W4];
#pragma unroll
            for (int j = 0; j < W4; j++) w[j] = buf[lane * W4 + j];
            h[k] = rp::fh::hash32_words<LEN>(w);
        }
    };
    u32x4 v[KPL][NV];
    auto windows = [&](const uint32_t (&h)[KPL]) {
#pragma unroll
        for (int k = 0; k < KPL; k++) {
            const uint32_t b = h[k] >> 14;
            const uint32_t cw = idx[b >> 3];
            const uint32_t base = idx[32768 + (b >> 6)] & 0xFFFFFu;
            const uint32_t s4 = (b & 7) * 4;
            const uint32_t below = cw & ((1u << s4) - 1u);
            const uint32_t x = (below & 0x0F0F0F0Fu) + ((below >> 4) & 0x0F0F0F0Fu);
            const uint32_t pos = (uint32_t)(((uint64_t)(base + ((x * 0x01010101u) >> 24) + (b & 63) * 4) * nent) >> 20);
            const uint8_t* p = reinterpret_cast<const uint8_t*>(tab) + 3ull * (pos % nent);
            if constexpr (NWIN == 0) {
                v[k][0] = u32x4{pos, pos, pos, pos};
            } else {
#pragma unroll
                for (int q = 0; q < NWIN; q++) v[k][q] = *reinterpret_cast<const u32x4_a1*>(p + 16 * q);
            }
        }
    };
    uint64_t t = blockIdx.x * (uint64_t)(TL / 64) + wv;
    if (t >= nw) return;
    issue(t);
    uint32_t hc[KPL];
    hash_round(hc);
    if (t + wstride < nw) issue(t + wstride);
    windows(hc);
    for (; t < nw; t += wstride) {
        uint32_t hn[KPL];
        const bool more = t + wstride < nw;
        if (more) {
            hash_round(hn);
            if (t + 2 * wstride < nw) issue(t + 2 * wstride);
        }
        uint32_t r[KPL][3];
#pragma unroll
        for (int k = 0; k < KPL; k++) {
            r[k][0] = hc[k] ^ v[k][0].x;
            r[k][1] = v[k][0].y + v[k][NV - 1].z;
            r[k][2] = v[k][0].w ^ v[k][NV - 1].x;
        }
        u32x4* d4 = reinterpret_cast<u32x4*>(out + t * TW * 3);
#pragma unroll
        for (int k = 0; k < KPL; k++) {
#pragma unroll
            for (int q = 0; q < 3; q++) buf[lane * 3 + q] = r[k][q];
            if (lane < 48) __builtin_nontemporal_store(reinterpret_cast<const u32x4*>(buf)[lane], d4 + k * 48 + lane);
        }
        if (more) {
#pragma unroll
            for (int k = 0; k < KPL; k++) hc[k] = hn[k];
            windows(hc);
        }
    }
}

template <int KPL, int NWIN, bool PIPE = false>
static void row_lds(const uint8_t* keys, uint64_t n, const uint32_t* tab, const uint32_t* gidx, uint32_t* out, int grid) {
    printf("ldsidx%d kpl%d %s", NWIN, KPL, PIPE ? "pipe" : "    ");
    for (double mb : kMB) {
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        std::vector<float> ts;
        for (int rep = 0; rep < 7; rep++) {
            CK(hipEventRecord(a));
            if (PIPE)
                k_ub_lds2<KPL, NWIN><<<grid, TL>>>(keys, n, tab, (uint32_t)(mb * 16384.0), gidx, out);
            else
                k_ub_lds<KPL, NWIN><<<grid, TL>>>(keys, n, tab, (uint32_t)(mb * 16384.0), gidx, out);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        printf(" %8.3f", ts[3]);
    }
    printf("\n");
    fflush(stdout);
}

int main(int argc, char** argv) {
    const uint64_t n = 1ull << 26;
    int grid = argc > 1 ? atoi(argv[1]) : 256 * 20;
    uint8_t* keys;
    uint32_t *tab, *out;
    CK(hipMalloc(&keys, n * LEN));
    CK(hipMalloc(&tab, 16u << 20));
    CK(hipMalloc(&out, n * 12));
    k_fill<<<4096, 256>>>(reinterpret_cast<uint32_t*>(keys), n * LEN / 4, 1);
    k_fill<<<4096, 256>>>(tab, 4u << 20, 2);
    CK(hipDeviceSynchronize());
    printf("grid %d; ms per 2^26 keys (alg GB/s = 3221 / ms)\nT(MB)            ", grid);
    for (double mb : kMB) printf(" %8.1f", mb);
    printf("\n");
    if (argc > 2 && argv[2][0] == 'q') {  // one launch per variant at 3 MB (PMC runs)
        const uint32_t nl = 3 * 16384;
        k_ub<NONE, 4, false><<<grid, T>>>(keys, n, tab, nl, out);
        k_ub<R16, 4, false><<<grid, T>>>(keys, n, tab, nl, out);
        k_ub<R16U, 4, false><<<grid, T>>>(keys, n, tab, nl, out);
        k_ub<R16A2, 4, false><<<grid, T>>>(keys, n, tab, nl, out);
        k_ub<R16W4, 4, false><<<grid, T>>>(keys, n, tab, nl, out);
        k_ub<R16W8, 4, false><<<grid, T>>>(keys, n, tab, nl, out);
        k_ub<R8R16U, 4, false><<<grid, T>>>(keys, n, tab, nl, out);
        k_ub<COOP64, 4, false><<<grid, T>>>(keys, n, tab, nl, out);
        CK(hipDeviceSynchronize());
        return 0;
    }
    if (argc > 2) {  // LDS-index rows only
        for (int g : {256}) {
            if (argv[2][0] == 'm') break;
            row_lds<4, 0, true>(keys, n, tab, tab, out, g);
            row_lds<4, 1, true>(keys, n, tab, tab, out, g);
            row_lds<4, 2, true>(keys, n, tab, tab, out, g);
            row_lds<8, 1, true>(keys, n, tab, tab, out, g);
            row_lds<8, 2, true>(keys, n, tab, tab, out, g);
            if (argv[2][0] == 'p') break;
            printf("grid %d (one 512-thread workgroup per CU)\n", g);
            row_lds<4, 0>(keys, n, tab, tab, out, g);
            row_lds<4, 1>(keys, n, tab, tab, out, g);
            row_lds<4, 2>(keys, n, tab, tab, out, g);
            row_lds<8, 0>(keys, n, tab, tab, out, g);
            row_lds<8, 1>(keys, n, tab, tab, out, g);
            row_lds<8, 2>(keys, n, tab, tab, out, g);
        }
        row<NONE, 4, false>("none", keys, n, tab, out, grid);
        row<R16, 4, false>("r16", keys, n, tab, out, grid);
        row<R16U, 4, false>("r16u", keys, n, tab, out, grid);
        row<R16A2, 4, false>("r16a2", keys, n, tab, out, grid);
        row<R16W4, 4, false>("r16w4", keys, n, tab, out, grid);
        row<R16W8, 4, false>("r16w8", keys, n, tab, out, grid);
        row<R8R16, 4, false>("r8r16", keys, n, tab, out, grid);
        row<R8R16U, 4, false>("r8r16u", keys, n, tab, out, grid);
        row<COOP64, 4, false>("coop64", keys, n, tab, out, grid);
        return 0;
    }
    rows<NONE>("none", keys, n, tab, out, grid);
    rows<R16>("r16", keys, n, tab, out, grid);
    rows<R8R16>("r8r16", keys, n, tab, out, grid);
    rows<LINE64>("line64", keys, n, tab, out, grid);
    rows<COOP64>("coop64", keys, n, tab, out, grid);
    return 0;
}
