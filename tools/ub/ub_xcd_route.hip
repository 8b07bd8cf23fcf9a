// ub_xcd_route.hip — microbenchmark (design tool, not product): can lookups be routed to XCDs by
// hash range, so each XCD's L2 holds only its eighth of a table eight times richer per token?
//
// Same key stream as tools/ub_lookup.hip: 2^26 36-byte keys, farmhash32 each, 12 B written per key
// (48 algorithmic bytes). Shapes, ms per 2^26 keys (median of 7):
//   single/r8r16u  one kernel: stream + hash, an 8-B index record then an unaligned 16-B window in
//                  a 3.5 MB table, rows stored in key order (the lean lookup kernel's shape)
//   single/r16     the same with one aligned random 16-B load in a 4 MB table (the one-access floor)
//   route          K1: stream + hash, (hash, key index) pairs appended per tile to 8 hash-range
//                  partitions (fixed 256-entry segments per tile and partition); K2: block b folds
//                  partition b % 8 (blocks are dealt round-robin over the XCDs), one aligned random
//                  16-B load per key in that partition's 4 MB slice of a 32 MB table, its 12-B row
//                  stored at the key's index (scattered: eight XCDs write into the same lines)
//   route/K1, route/K2  each kernel alone
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -o tools/ub/ub_xcd_route tools/ub/ub_xcd_route.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../ringpop-node_amd/csrc/rp_farmhash.h"

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4_a1 __attribute__((ext_vector_type(4), aligned(1)));

constexpr int T = 256, LEN = 36, W4 = 9, KPL = 4, TK = T * KPL;  // 1,024 keys per tile
constexpr int SEGCAP = 256;                                       // entries per (tile, partition)

// stage a tile's keys through LDS and hash KPL keys per lane
__device__ __forceinline__ void tile_hash(const uint8_t* __restrict__ keys, uint64_t t, uint32_t* sk, uint32_t (&h)[KPL]) {
    constexpr int V4 = TK * W4 / 4, PER = (V4 + T - 1) / T;
    const int tid = threadIdx.x;
    const u32x4* s4 = reinterpret_cast<const u32x4*>(keys + t * TK * LEN);
    u32x4 pre[PER];
#pragma unroll
    for (int q = 0; q < PER; q++) {
        const int k = tid + q * T;
        if (k < V4) pre[q] = __builtin_nontemporal_load(s4 + k);
    }
#pragma unroll
    for (int q = 0; q < PER; q++) {
        const int k = tid + q * T;
        if (k < V4) reinterpret_cast<u32x4*>(sk)[k] = pre[q];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < KPL; k++) {
        uint32_t w[W4];
#pragma unroll
        for (int j = 0; j < W4; j++) w[j] = sk[(tid + k * T) * W4 + j];
        h[k] = rp::fh::hash32_words<LEN>(w);
    }
    __syncthreads();
}

// single-kernel shapes: MODE 0 = r8r16u in 3.5 MB, 1 = r16 in 4 MB
template <int MODE>
__global__ __launch_bounds__(T) void k_single(const uint8_t* __restrict__ keys, uint64_t n, const uint32_t* __restrict__ tab,
                                              uint32_t* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) uint32_t sk[TK * W4];
    const int tid = threadIdx.x;
    for (uint64_t t = blockIdx.x; t < n / TK; t += gridDim.x) {
        uint32_t h[KPL], r[KPL][3];
        tile_hash(keys, t, sk, h);
        if (MODE == 0) {
            constexpr uint32_t nw = 3584u * 1024u / 4u;  // 3.5 MB in words: 0.5 MB index, 3 MB entries
            u32x2 b[KPL];
#pragma unroll
            for (int k = 0; k < KPL; k++) b[k] = *reinterpret_cast<const u32x2*>(tab + 2 * (uint32_t)(((uint64_t)h[k] * (nw / 14)) >> 32));
            u32x4 v[KPL];
#pragma unroll
            for (int k = 0; k < KPL; k++) {
                const uint32_t c = nw / 7 * 4 + ((b[k].x ^ h[k]) % (nw / 7 * 24 - 64));
                v[k] = *reinterpret_cast<const u32x4_a1*>(reinterpret_cast<const uint8_t*>(tab) + c);
            }
#pragma unroll
            for (int k = 0; k < KPL; k++) {
                r[k][0] = h[k] ^ (v[k].x + b[k].y);
                r[k][1] = v[k].y;
                r[k][2] = v[k].z + v[k].w;
            }
        } else {
            constexpr uint32_t nl = 4u * 1024u * 1024u / 16u;
            u32x4 v[KPL];
#pragma unroll
            for (int k = 0; k < KPL; k++) v[k] = *reinterpret_cast<const u32x4*>(tab + 4 * (uint32_t)(((uint64_t)h[k] * nl) >> 32));
#pragma unroll
            for (int k = 0; k < KPL; k++) {
                r[k][0] = h[k] ^ (v[k].x + v[k].w);
                r[k][1] = v[k].y;
                r[k][2] = v[k].z;
            }
        }
#pragma unroll
        for (int k = 0; k < KPL; k++)
#pragma unroll
            for (int q = 0; q < 3; q++) sk[(tid + k * T) * 3 + q] = r[k][q];
        __syncthreads();
        u32x4* d4 = reinterpret_cast<u32x4*>(out + t * TK * 3);
        for (int k = tid; k < TK * 3 / 4; k += T) __builtin_nontemporal_store(reinterpret_cast<const u32x4*>(sk)[k], d4 + k);
        __syncthreads();
    }
}

// K1: hash, then (hash, index) per key into the tile's segment of partition hash >> 29
__global__ __launch_bounds__(T) void k_route(const uint8_t* __restrict__ keys, uint64_t n, u32x2* __restrict__ part,
                                             uint32_t* __restrict__ cnt) {
    __shared__ __attribute__((aligned(16))) uint32_t sk[TK * W4];
    __shared__ uint32_t c8[8];
    const int tid = threadIdx.x;
    const uint64_t ntiles = n / TK;
    for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        if (tid < 8) c8[tid] = 0;
        uint32_t h[KPL];
        tile_hash(keys, t, sk, h);
        uint32_t rk[KPL];
#pragma unroll
        for (int k = 0; k < KPL; k++) rk[k] = atomicAdd(&c8[h[k] >> 29], 1u);
#pragma unroll
        for (int k = 0; k < KPL; k++) {
            const uint32_t x = h[k] >> 29;
            if (rk[k] < SEGCAP)
                part[((uint64_t)x * ntiles + t) * SEGCAP + rk[k]] = u32x2{h[k], (uint32_t)(t * TK) + tid + k * T};
        }
        __syncthreads();
        if (tid < 8) cnt[(uint64_t)tid * ntiles + t] = c8[tid] < SEGCAP ? c8[tid] : SEGCAP;
        __syncthreads();
    }
}

// K2: block b serves partition b % 8; one aligned 16-B load in the partition's 4 MB slice, the
// 12-B row at the key's index
__global__ __launch_bounds__(T) void k_xlookup(const u32x2* __restrict__ part, const uint32_t* __restrict__ cnt,
                                               uint64_t ntiles, const uint32_t* __restrict__ tab, uint32_t* __restrict__ out) {
    const uint32_t x = blockIdx.x & 7u, nb = gridDim.x >> 3;
    constexpr uint32_t nl = 4u * 1024u * 1024u / 16u;  // 16-B records per slice
    const uint32_t* slice = tab + (uint64_t)x * (nl * 4);
    for (uint64_t t = blockIdx.x >> 3; t < ntiles; t += nb) {
        const uint32_t c = cnt[(uint64_t)x * ntiles + t];
        const u32x2* p = part + ((uint64_t)x * ntiles + t) * SEGCAP;
        if (threadIdx.x < c) {
            const u32x2 e = p[threadIdx.x];
            const u32x4 v = *reinterpret_cast<const u32x4*>(slice + 4 * (uint32_t)(((uint64_t)(e.x << 3) * nl) >> 32));
            uint32_t* o = out + (uint64_t)e.y * 3;
            o[0] = e.x ^ (v.x + v.w);
            o[1] = v.y;
            o[2] = v.z;
        }
    }
}

__global__ void k_fill(uint32_t* p, uint64_t n, uint32_t seed) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        p[i] = rp::fh::fmix((uint32_t)i * 0x9E3779B9u + seed);
}

template <class F>
static float timed(F f) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<float> ts;
    for (int rep = 0; rep < 7; rep++) {
        CK(hipEventRecord(a));
        f();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        ts.push_back(ms);
    }
    CK(hipGetLastError());
    std::sort(ts.begin(), ts.end());
    return ts[3];
}

int main(int argc, char** argv) {
    const uint64_t n = 1ull << 26, ntiles = n / TK;
    const int grid = argc > 1 ? atoi(argv[1]) : 4096;
    uint8_t* keys;
    uint32_t *tab, *out, *cnt;
    u32x2* part;
    CK(hipMalloc(&keys, n * LEN));
    CK(hipMalloc(&tab, 32ull << 20));
    CK(hipMalloc(&out, n * 12));
    CK(hipMalloc(&part, 8 * ntiles * SEGCAP * sizeof(u32x2)));
    CK(hipMalloc(&cnt, 8 * ntiles * sizeof(uint32_t)));
    k_fill<<<4096, 256>>>(reinterpret_cast<uint32_t*>(keys), n * LEN / 4, 1);
    k_fill<<<4096, 256>>>(tab, (32ull << 20) / 4, 2);
    CK(hipDeviceSynchronize());
    const float s0 = timed([&] { k_single<0><<<grid, T>>>(keys, n, tab, out); });
    const float s1 = timed([&] { k_single<1><<<grid, T>>>(keys, n, tab, out); });
    const float k1 = timed([&] { k_route<<<grid, T>>>(keys, n, part, cnt); });
    const float k2 = timed([&] { k_xlookup<<<grid, T>>>(part, cnt, ntiles, tab, out); });
    const float rt = timed([&] {
        k_route<<<grid, T>>>(keys, n, part, cnt);
        k_xlookup<<<grid, T>>>(part, cnt, ntiles, tab, out);
    });
    const double gb = 48.0 * n / 1e9;
    printf("{\"keys\": %llu, \"grid\": %d, \"single_r8r16u_ms\": %.4f, \"single_r16_ms\": %.4f, \"route_k1_ms\": %.4f, "
           "\"route_k2_ms\": %.4f, \"route_ms\": %.4f, \"route_frac_of_8TBps\": %.3f, \"single_r8r16u_frac\": %.3f}\n",
           (unsigned long long)n, grid, s0, s1, k1, k2, rt, gb / (rt * 1e-3) / 8000.0, gb / (s0 * 1e-3) / 8000.0);
    return 0;
}
