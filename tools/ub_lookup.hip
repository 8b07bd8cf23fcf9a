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

constexpr int T = 256, LEN = 36, W4 = 9;

enum { NONE = 0, R16, R8R16, LINE64, COOP64 };

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
    rows<NONE>("none", keys, n, tab, out, grid);
    rows<R16>("r16", keys, n, tab, out, grid);
    rows<R8R16>("r8r16", keys, n, tab, out, grid);
    rows<LINE64>("line64", keys, n, tab, out, grid);
    rows<COOP64>("coop64", keys, n, tab, out, grid);
    return 0;
}
