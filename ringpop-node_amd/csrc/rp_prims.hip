// rp_prims.hip — exclusive scan and stable LSD radix sort for gfx950.
//
// Sort design (wave64-native, no CUDA warp idioms): each 256-thread workgroup owns a
// contiguous 2048-element tile. Pass 1 builds a per-tile 256-bin digit histogram in LDS;
// the [digit][tile] table is scanned; pass 2 re-reads the tile in 8 rounds of 256 and ranks
// each element stably with 8 wave ballots (a 64-lane "match any" on the digit) plus per-wave
// digit counts in LDS, then scatters. Stability is what the ring build relies on: equal
// tokens keep insertion order, so "first insert wins" (rbtree.js:112-116) is the first
// element of each equal run.
#include "rp_prims.h"

namespace rp {

namespace {

constexpr int kThreads = 256;
constexpr int kItems = 8;
constexpr int kTile = kThreads * kItems;  // 2048

__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t* lds, uint32_t* total) {
    // lds: >= kThreads + 1 entries. Hillis-Steele on 256 values via wave shuffles + LDS.
    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    // x = inclusive within wave
    if (lane == 63) lds[wave] = x;
    __syncthreads();
    uint32_t wbase = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < kThreads / 64; w++) {
        uint32_t s = lds[w];
        if (w < wave) wbase += s;
        tot += s;
    }
    __syncthreads();
    *total = tot;
    return wbase + x - v;
}

__global__ __launch_bounds__(kThreads) void k_scan_tiles(const uint32_t* in,
                                                         uint32_t* out, uint64_t n,
                                                         uint32_t* __restrict__ sums) {
    __shared__ uint32_t lds[kThreads + 1];
    const uint64_t base = (uint64_t)blockIdx.x * kTile + (uint64_t)threadIdx.x * kItems;
    uint32_t v[kItems];
    uint32_t s = 0;
#pragma unroll
    for (int j = 0; j < kItems; j++) {
        uint64_t i = base + j;
        v[j] = i < n ? in[i] : 0u;
        s += v[j];
    }
    uint32_t total;
    uint32_t ex = block_exclusive_scan(s, lds, &total);
#pragma unroll
    for (int j = 0; j < kItems; j++) {
        uint64_t i = base + j;
        uint32_t t = v[j];
        if (i < n) out[i] = ex;
        ex += t;
    }
    if (threadIdx.x == 0) sums[blockIdx.x] = total;
}

__global__ void k_scan_add(uint32_t* __restrict__ out, uint64_t n, const uint32_t* __restrict__ sums) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (; i < n; i += stride) out[i] += sums[i / kTile];
}

__global__ void k_set_total(uint32_t* out, uint64_t n, const uint32_t* sums_scanned, uint64_t nb) {
    if (threadIdx.x == 0 && blockIdx.x == 0) out[n] = sums_scanned[nb];
}

__global__ void k_single_total(uint32_t* out, uint64_t n, const uint32_t* sums) {
    if (threadIdx.x == 0 && blockIdx.x == 0) out[n] = sums[0];
}

void scan_level(const uint32_t* in, uint32_t* out, uint64_t n, hipStream_t st, DevBuf<uint32_t>* const* lv,
                int depth) {
    if (depth >= 3) throw Error(RP_EINVAL, "scan too large");
    uint64_t nb = (n + kTile - 1) / kTile;
    if (nb == 0) nb = 1;
    DevBuf<uint32_t>& sums = *lv[depth];
    sums.reserve(nb + 1);
    hipLaunchKernelGGL(k_scan_tiles, dim3((unsigned)nb), dim3(kThreads), 0, st, in, out, n, sums.p);
    RP_HIP(hipGetLastError());
    if (nb == 1) {
        hipLaunchKernelGGL(k_single_total, dim3(1), dim3(64), 0, st, out, n, sums.p);
        return;
    }
    scan_level(sums.p, sums.p, nb, st, lv, depth + 1);  // sums[nb] = total
    hipLaunchKernelGGL(k_scan_add, dim3(grid_for(n, 256)), dim3(256), 0, st, out, n, sums.p);
    hipLaunchKernelGGL(k_set_total, dim3(1), dim3(64), 0, st, out, n, sums.p, nb);
    RP_HIP(hipGetLastError());
}

__global__ __launch_bounds__(kThreads) void k_radix_hist(const uint32_t* __restrict__ keys, uint64_t n,
                                                         int shift, uint32_t* __restrict__ hist,
                                                         uint32_t nb) {
    __shared__ uint32_t h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * kTile;
#pragma unroll
    for (int j = 0; j < kItems; j++) {
        uint64_t i = base + (uint64_t)j * kThreads + threadIdx.x;
        if (i < n) atomicAdd(&h[(keys[i] >> shift) & 255u], 1u);
    }
    __syncthreads();
    hist[(uint64_t)threadIdx.x * nb + blockIdx.x] = h[threadIdx.x];
}

__global__ __launch_bounds__(kThreads) void k_radix_scatter(const uint32_t* __restrict__ kin,
                                                            const uint32_t* __restrict__ vin,
                                                            uint32_t* __restrict__ kout,
                                                            uint32_t* __restrict__ vout, uint64_t n,
                                                            int shift, const uint32_t* __restrict__ offs,
                                                            uint32_t nb) {
    __shared__ uint32_t base_d[256];
    __shared__ uint32_t run[256];
    __shared__ uint32_t wcnt[kThreads / 64][256];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    base_d[tid] = offs[(uint64_t)tid * nb + blockIdx.x];
    run[tid] = 0;
#pragma unroll
    for (int w = 0; w < kThreads / 64; w++) wcnt[w][tid] = 0;
    __syncthreads();
    const uint64_t tbase = (uint64_t)blockIdx.x * kTile;
    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    for (int j = 0; j < kItems; j++) {
        const uint64_t i = tbase + (uint64_t)j * kThreads + tid;
        const bool valid = i < n;
        uint32_t k = valid ? kin[i] : 0u;
        uint32_t v = (valid && vin) ? vin[i] : 0u;
        uint32_t d = (k >> shift) & 255u;
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; b++) {
            const bool bit = (d >> b) & 1u;
            uint64_t m = __ballot(valid && bit);
            peers &= bit ? m : ~m;
        }
        const uint64_t below = peers & lt_mask;
        const uint32_t rank = (uint32_t)__popcll(below);
        if (valid && below == 0) wcnt[wave][d] = (uint32_t)__popcll(peers);
        __syncthreads();
        if (valid) {
            uint32_t pos = run[d] + rank;
            for (int w = 0; w < wave; w++) pos += wcnt[w][d];
            const uint32_t dst = base_d[d] + pos;
            kout[dst] = k;
            if (vin) vout[dst] = v;
        }
        __syncthreads();
        uint32_t add = 0;
#pragma unroll
        for (int w = 0; w < kThreads / 64; w++) {
            add += wcnt[w][tid];
            wcnt[w][tid] = 0;
        }
        run[tid] += add;
        __syncthreads();
    }
}

__global__ void k_iota(uint32_t* out, uint64_t n) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (; i < n; i += stride) out[i] = (uint32_t)i;
}

__global__ void k_gather(const uint32_t* __restrict__ src, const uint32_t* __restrict__ idx,
                         uint32_t* __restrict__ dst, uint64_t n) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (; i < n; i += stride) dst[i] = src[idx[i]];
}

}  // namespace

void scan_exclusive_u32(const uint32_t* in, uint32_t* out, uint64_t n, hipStream_t st, Scratch& ws) {
    DevBuf<uint32_t>* lv[3] = {&ws.s0, &ws.s1, &ws.s2};
    scan_level(in, out, n, st, lv, 0);
}

void radix_sort_pairs(uint32_t* keys, uint32_t* vals, uint64_t n, int begin_bit, int end_bit,
                      hipStream_t st, Scratch& ws) {
    if (n <= 1) return;
    RP_REQUIRE(n < (1ull << 32), "radix_sort_pairs: n must be < 2^32");
    const uint32_t nb = (uint32_t)((n + kTile - 1) / kTile);
    ws.a.reserve(n);
    if (vals) ws.b.reserve(n);
    ws.hist.reserve((uint64_t)256 * nb + 1);
    ws.hscan.reserve((uint64_t)256 * nb + 1);
    uint32_t *kin = keys, *vin = vals, *kout = ws.a.p, *vout = vals ? ws.b.p : nullptr;
    int passes = 0;
    for (int shift = begin_bit; shift < end_bit; shift += 8, passes++) {
        hipLaunchKernelGGL(k_radix_hist, dim3(nb), dim3(kThreads), 0, st, kin, n, shift, ws.hist.p, nb);
        RP_HIP(hipGetLastError());
        scan_exclusive_u32(ws.hist.p, ws.hscan.p, (uint64_t)256 * nb, st, ws);
        hipLaunchKernelGGL(k_radix_scatter, dim3(nb), dim3(kThreads), 0, st, kin, vin, kout, vout, n, shift,
                           ws.hscan.p, nb);
        RP_HIP(hipGetLastError());
        std::swap(kin, kout);
        std::swap(vin, vout);
    }
    if (passes & 1) {
        RP_HIP(hipMemcpyAsync(keys, kin, n * sizeof(uint32_t), hipMemcpyDeviceToDevice, st));
        if (vals) RP_HIP(hipMemcpyAsync(vals, vin, n * sizeof(uint32_t), hipMemcpyDeviceToDevice, st));
    }
}

void iota_u32(uint32_t* out, uint64_t n, hipStream_t st) {
    if (!n) return;
    hipLaunchKernelGGL(k_iota, dim3(grid_for(n, 256)), dim3(256), 0, st, out, n);
    RP_HIP(hipGetLastError());
}

void gather_u32(const uint32_t* src, const uint32_t* idx, uint32_t* dst, uint64_t n, hipStream_t st) {
    if (!n) return;
    hipLaunchKernelGGL(k_gather, dim3(grid_for(n, 256)), dim3(256), 0, st, src, idx, dst, n);
    RP_HIP(hipGetLastError());
}

uint32_t read_u32(const uint32_t* p, hipStream_t st) {
    uint32_t v = 0;
    RP_HIP(hipMemcpyAsync(&v, p, sizeof v, hipMemcpyDeviceToHost, st));
    RP_HIP(hipStreamSynchronize(st));
    return v;
}

}  // namespace rp
