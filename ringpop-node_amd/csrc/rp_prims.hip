// rp_prims.hip — exclusive scan and stable LSD radix sort for gfx950.
//
// Sort design (wave64-native, no CUDA warp idioms): each 256-thread workgroup owns a
// contiguous tile and ranks its elements stably with 8 wave ballots per 64 elements (a 64-lane
// "match any" on the digit) plus per-wave digit counts in LDS. Stability is
// what the ring build relies on: equal tokens keep insertion order, so "first insert wins"
// (rbtree.js:112-116) is the first element of each equal run.
//
// Default (single-pass) path: one launch computes the global histograms of every digit, then
// each digit is one launch in which a tile finds its output offsets by decoupled look-back
// over its predecessors' per-digit counts and writes its elements staged through LDS in digit
// order; the scan is likewise one launch. At the batch sizes of the membership fold (~1e5)
// these primitives are launch-bound, so launches are what they save: a 24-bit sort is 4
// launches instead of 21. The multi-pass path (per-tile histograms -> scan -> scatter per
// digit, multi-level scans) stays selectable for A/B (RP_PRIMS_MULTIPASS=1).
#include "rp_prims.h"

#include <algorithm>
#include <cstdlib>
#include <vector>

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

// ------------------------------------------------------------ single-pass (look-back) kernels
//
// Tiles take a ticket in launch order (so every tile they wait on is already running), publish
// their own aggregate (flag A) at once, sum predecessors' words back to the nearest inclusive
// prefix (flag P), then publish their own P. A look-back word is
// [epoch:30 | flag:2 | value:32]; agent-scope atomics bypass the per-XCD L2s. Words from an
// earlier launch carry another epoch and read as "not ready", so the array is never cleared.
// The exclusive prefix of `tile` for the word column `col` (stride words per tile), by one
// thread: kLbWin predecessor words per step, back to the nearest P.
__device__ uint32_t lookback_thread(const uint64_t* lb, uint32_t tile, uint32_t stride, uint32_t col,
                                    uint64_t tag, uint32_t* err) {
    uint32_t excl = 0;
    int64_t t = (int64_t)tile - 1;
    while (t >= 0) {
        uint64_t v[kLbWin];
        const int m = t + 1 < kLbWin ? (int)(t + 1) : kLbWin;
#pragma unroll
        for (int q = 0; q < kLbWin; q++)
            if (q < m) v[q] = lb_load(lb + (uint64_t)(t - q) * stride + col);
        bool done = false;
        int q = 0;
        for (; q < m; q++) {
            uint32_t spin = 0;
            for (; !lb_ready(v[q], tag) && spin < kLbSpinCap; spin++) {
                __builtin_amdgcn_s_sleep(1);
                v[q] = lb_load(lb + (uint64_t)(t - q) * stride + col);
            }
            if (spin == kLbSpinCap) atomicOr(err, kErrSpin);
            excl += (uint32_t)v[q];
            if (v[q] & kLbP) {
                done = true;
                break;
            }
        }
        if (done) break;
        t -= m;
    }
    return excl;
}

// Global digit histograms of every pass in one read of the keys; the last workgroup to finish
// turns them into digit bases (exclusive scan per pass) and zeroes them for the next sort.
// dig: [0, 1024) histograms, [1024, 2048) bases, [2048] finished-workgroup counter.
__global__ __launch_bounds__(kThreads) void k_os_hist(const uint32_t* __restrict__ keys, uint32_t n, int begin,
                                                      int npass, uint32_t* __restrict__ dig,
                                                      const uint32_t* __restrict__ run_if) {
    if (run_if && *run_if == 0) return;  // (every workgroup: the finish counter is untouched)
    __shared__ uint32_t h[4][256];
    __shared__ uint32_t lds[kThreads + 1];
    __shared__ bool last;
    const int tid = threadIdx.x, lane = tid & 63;
    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
#pragma unroll
    for (int p = 0; p < 4; p++) h[p][tid] = 0;
    __syncthreads();
    const uint32_t stride = gridDim.x * kThreads;
    for (uint32_t i0 = blockIdx.x * kThreads; i0 < n; i0 += stride) {
        const uint32_t i = i0 + tid;
        const bool valid = i < n;
        const uint32_t k = valid ? keys[i] : 0u;
        for (int p = 0; p < npass; p++) {
            // one LDS atomic per distinct digit in the wave (skewed digits do not serialise)
            const uint32_t d = (k >> (begin + 8 * p)) & 255u;
            uint64_t peers = __ballot(valid);
#pragma unroll
            for (int b = 0; b < 8; b++) {
                const bool bit = (d >> b) & 1u;
                const uint64_t m = __ballot(valid && bit);
                peers &= bit ? m : ~m;
            }
            if (valid && (peers & lt_mask) == 0) atomicAdd(&h[p][d], (uint32_t)__popcll(peers));
        }
    }
    __syncthreads();
    for (int p = 0; p < npass; p++)
        if (h[p][tid]) atomicAdd(&dig[p * 256 + tid], h[p][tid]);
    __threadfence();
    __syncthreads();
    if (tid == 0) last = atomicAdd(&dig[2048], 1u) == gridDim.x - 1;
    __syncthreads();
    if (!last) return;
    __threadfence();
    for (int p = 0; p < npass; p++) {
        const uint32_t v = __hip_atomic_load(&dig[p * 256 + tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        uint32_t tot;
        const uint32_t ex = block_exclusive_scan(v, lds, &tot);
        dig[1024 + p * 256 + tid] = ex;
        __hip_atomic_store(&dig[p * 256 + tid], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (tid == 0) __hip_atomic_store(&dig[2048], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One 8-bit digit pass over 4096-element tiles. vin == nullptr && IOTA: the values are the
// element indices; vin == nullptr && !IOTA: keys only. Each wave ranks its own contiguous
// 1024 elements (64 at a time: 8 ballots give the lanes holding the same digit; a per-wave
// digit counter in LDS, which the wave's own in-order LDS traffic keeps consistent without
// barriers), so the ranking needs no barrier.
template <bool IOTA, int kOsItems>
__global__ __launch_bounds__(kThreads) void k_os_scatter(const uint32_t* __restrict__ kin,
                                                         const uint32_t* __restrict__ vin,
                                                         uint32_t* __restrict__ kout, uint32_t* __restrict__ vout,
                                                         uint32_t n, int shift, const uint32_t* __restrict__ dbase,
                                                         uint64_t* __restrict__ lb, unsigned long long* ctr,
                                                         uint32_t ntiles, uint64_t tag, uint32_t* err,
                                                         const uint32_t* __restrict__ run_if) {
    constexpr int kOsTile = kThreads * kOsItems;
    constexpr int kOsWave = kOsTile / (kThreads / 64);
    __shared__ uint32_t wcnt[kThreads / 64][256];
    __shared__ uint32_t lstart[256];
    __shared__ uint32_t gbase[256];
    __shared__ uint32_t lds[kThreads + 1];
    __shared__ uint32_t lk[kOsTile], lv[kOsTile];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const bool has_v = IOTA || vin != nullptr;
#pragma unroll
    for (int w = 0; w < kThreads / 64; w++) wcnt[w][tid] = 0;
    if (run_if && *run_if == 0) return;  // (the whole launch: no tickets taken)
    const uint32_t tile = take_unit(ctr, ntiles, err);  // (syncs)
    if (tile >= ntiles) return;  // a ticket count out of step (reported): never write out of bounds
    const uint32_t t0 = tile * (uint32_t)kOsTile;
    const uint32_t w0 = t0 + (uint32_t)(wave * kOsWave);
    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    uint32_t key[kOsItems], val[kOsItems], rank[kOsItems];
#pragma unroll
    for (int j = 0; j < kOsItems; j++) {
        const uint32_t i = w0 + (uint32_t)(j * 64 + lane);
        const bool valid = i < n;
        key[j] = valid ? kin[i] : 0u;
        val[j] = IOTA ? i : (valid && vin ? vin[i] : 0u);
    }
#pragma unroll
    for (int j = 0; j < kOsItems; j++) {
        const bool valid = w0 + (uint32_t)(j * 64 + lane) < n;
        const uint32_t d = (key[j] >> shift) & 255u;
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; b++) {
            const bool bit = (d >> b) & 1u;
            const uint64_t m = __ballot(valid && bit);
            peers &= bit ? m : ~m;
        }
        const uint64_t below = peers & lt_mask;
        const uint32_t c = wcnt[wave][d];
        rank[j] = valid ? c + (uint32_t)__popcll(below) : 0xFFFFFFFFu;
        if (valid && below == 0) wcnt[wave][d] = c + (uint32_t)__popcll(peers);
    }
    __syncthreads();
    // digit `tid`: the tile's count and each wave's offset inside the digit
    uint32_t cnt = 0;
#pragma unroll
    for (int w = 0; w < kThreads / 64; w++) {
        const uint32_t c = wcnt[w][tid];
        wcnt[w][tid] = cnt;
        cnt += c;
    }
    uint64_t* mine = lb + (uint64_t)tile * 256 + tid;
    lb_store(mine, tag | (tile == 0 ? kLbP : kLbA) | cnt);
    uint32_t tot;
    lstart[tid] = block_exclusive_scan(cnt, lds, &tot);  // (syncs)
    if (tile > 0) {
        const uint32_t excl = lookback_thread(lb, tile, 256, (uint32_t)tid, tag, err);
        lb_store(mine, tag | kLbP | (excl + cnt));
        gbase[tid] = dbase[tid] + excl;
    } else {
        gbase[tid] = dbase[tid];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kOsItems; j++)
        if (rank[j] != 0xFFFFFFFFu) {
            const uint32_t d = (key[j] >> shift) & 255u;
            const uint32_t p = lstart[d] + wcnt[wave][d] + rank[j];
            lk[p] = key[j];
            if (has_v) lv[p] = val[j];
        }
    __syncthreads();
    const uint32_t tn = n - t0 < (uint32_t)kOsTile ? n - t0 : (uint32_t)kOsTile;
    for (uint32_t p = tid; p < tn; p += kThreads) {
        const uint32_t k = lk[p];
        const uint32_t d = (k >> shift) & 255u;
        const uint32_t dst = gbase[d] + p - lstart[d];
        kout[dst] = k;
        if (has_v) vout[dst] = lv[p];
    }
}

// Exclusive scan in one launch: 2048 elements per tile (8 consecutive per thread), tile
// prefixes by a wave-wide look-back (64 predecessor words per step).
__global__ __launch_bounds__(kThreads) void k_os_scan(const uint32_t* in, uint32_t* out, uint32_t n,
                                                      uint64_t* __restrict__ lb, unsigned long long* ctr,
                                                      uint64_t tag, uint32_t ntiles, uint32_t* err) {
    __shared__ uint32_t lds[kThreads + 1];
    __shared__ uint32_t s_excl;
    const int tid = threadIdx.x;
    const uint32_t tile = take_unit(ctr, ntiles, err);
    if (tile >= ntiles) return;  // a ticket count out of step (reported): never write out of bounds
    const uint64_t base = (uint64_t)tile * kTile + (uint64_t)tid * kItems;
    uint32_t v[kItems];
    uint32_t s = 0;
#pragma unroll
    for (int j = 0; j < kItems; j++) {
        const uint64_t i = base + j;
        v[j] = i < n ? in[i] : 0u;
        s += v[j];
    }
    uint32_t total;
    uint32_t ex = block_exclusive_scan(s, lds, &total);
    if (tid == 0) lb_store(lb + tile, tag | (tile == 0 ? kLbP : kLbA) | total);
    if (tid < 64) {
        const uint32_t excl = lookback_wave(lb, tile, tag, err);
        if (tid == 0) {
            if (tile > 0) lb_store(lb + tile, tag | kLbP | (excl + total));
            s_excl = excl;
            if (tile == ntiles - 1) out[n] = excl + total;
        }
    }
    __syncthreads();
    ex += s_excl;
#pragma unroll
    for (int j = 0; j < kItems; j++) {
        const uint64_t i = base + j;
        if (i < n) out[i] = ex;
        ex += v[j];
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

static int g_force_multipass = -1;  // rp_selftest_prims: -1 = environment, 0 = single-pass, 1 = multi-pass

bool prims_multipass() {
    static const bool on = [] {
        const char* e = getenv("RP_PRIMS_MULTIPASS");
        return e && *e && *e != '0';
    }();
    return g_force_multipass >= 0 ? g_force_multipass != 0 : on;
}

namespace {

}  // namespace

// Look-back state for one single-pass launch of `tiles` tiles with `cols` words each: returns
// the launch's epoch tag (the ticket counter is 0 between launches).
uint64_t lb_begin(Scratch& ws, uint64_t tiles, uint32_t cols, hipStream_t st) {
    ws.use_on(st);
    if (!ws.ticket.p) {
        ws.ticket.reserve(1);
        ws.err.reserve(1);
        RP_HIP(hipMemsetAsync(ws.ticket.p, 0, sizeof(unsigned long long), st));
        RP_HIP(hipMemsetAsync(ws.err.p, 0, sizeof(uint32_t), st));
    }
    const uint64_t words = tiles * cols;
    bool zero = false;
    if (ws.lb.cap < words) {
        ws.lb.release();
        ws.lb.reserve(words);
        zero = true;
    }
    if (++ws.epoch >= (1u << 29)) {  // epochs wrap: start over on a cleared array
        ws.epoch = 1;
        zero = true;
    }
    if (zero) RP_HIP(hipMemsetAsync(ws.lb.p, 0, ws.lb.cap * sizeof(uint64_t), st));
    return (uint64_t)ws.epoch << kLbEpochShift;
}

LookBack lookback_prepare(Scratch& ws, uint64_t units, hipStream_t st) {
    LookBack L{};
    RP_REQUIRE(units > 0 && units < (1ull << 32), "lookback_prepare: units");
    L.tag = lb_begin(ws, units, 1, st);
    L.words = ws.lb.p;
    L.ticket = ws.ticket.p;
    L.err = ws.err.p;
    return L;
}

void scratch_check(Scratch& ws, hipStream_t st) {
    if (!ws.err.p) return;
    uint32_t e = 0;
    RP_HIP(hipMemcpyAsync(&e, ws.err.p, sizeof e, hipMemcpyDeviceToHost, st));
    RP_HIP(hipStreamSynchronize(st));
    if (e) {
        RP_HIP(hipMemsetAsync(ws.err.p, 0, sizeof(uint32_t), st));
        RP_HIP(hipStreamSynchronize(st));
        if (e & kErrRange)
            throw Error(RP_EDEVICE, "a member incarnation outside [-2^60, 2^60) or a status past leave (3) reached the "
                                    "member table: results "
                                    "of the last calls on this handle are not valid");
        throw Error(RP_EDEVICE, std::string("device primitive reported a broken ordering (") +
                                    (e & kErrSpin ? "look-back wait gave up" : "") +
                                    (e == (kErrSpin | kErrTicket) ? ", " : "") +
                                    (e & kErrTicket ? "ticket past the launch's tiles" : "") +
                                    "): results of the last calls on this handle are not valid");
    }
}

namespace {

void os_sort(const uint32_t* kin0, const uint32_t* vin0, bool iota, uint32_t* keys, uint32_t* vals, uint64_t n,
             int begin_bit, int end_bit, hipStream_t st, Scratch& ws, const uint32_t* run_if = nullptr) {
    const int npass = (end_bit - begin_bit + 7) / 8;
    RP_REQUIRE(npass >= 1 && npass <= 4, "radix sort: bit range");
    // 16 elements per thread (4096-element tiles) for large sorts; 8 below 2^20 elements, where
    // the sort is latency-bound and more, shorter tiles finish sooner
    static const int items_env = [] {
        const char* e = getenv("RP_OS_ITEMS");
        return e && *e ? atoi(e) : 0;
    }();
    const int items = items_env == 8 || items_env == 16 ? items_env : (n >= (1u << 20) ? 16 : 8);
    const uint32_t tile_n = kThreads * items;
    const uint32_t tiles = (uint32_t)((n + tile_n - 1) / tile_n);
    if (!ws.dig.p) {
        ws.dig.reserve(2048 + 64);
        RP_HIP(hipMemsetAsync(ws.dig.p, 0, ws.dig.cap * sizeof(uint32_t), st));
    }
    const uint32_t hist_blocks = (uint32_t)std::min<uint64_t>((n + 1023) / 1024, 1024);
    hipLaunchKernelGGL(k_os_hist, dim3(hist_blocks), dim3(kThreads), 0, st, kin0, (uint32_t)n, begin_bit, npass,
                       ws.dig.p, run_if);
    RP_HIP(hipGetLastError());
    const bool has_v = iota || vin0 != nullptr;
    ws.a.reserve(n);
    if (has_v) ws.b.reserve(n);
    if (npass == 3) {
        ws.c.reserve(n);
        if (has_v) ws.d.reserve(n);
    }
    // destinations so that the last pass lands in (keys, vals) and no pass writes its input
    //   in place:        1: A (+ copy back)   2: A K   3: A C K   4: A K A K
    //   separate input:  1: K                 2: A K   3: K A K   4: A K A K
    // (K = keys/vals, A = ws.a/ws.b, C = ws.c/ws.d)
    const bool sep = kin0 != keys;
    static const char in_place[4][5] = {"A", "AK", "ACK", "AKAK"};
    static const char separate[4][5] = {"K", "AK", "KAK", "AKAK"};
    const char* plan = sep ? separate[npass - 1] : in_place[npass - 1];
    uint32_t* dk[4];
    uint32_t* dv[4];
    for (int p = 0; p < npass; p++) {
        const char c = plan[p];
        dk[p] = c == 'K' ? keys : c == 'A' ? ws.a.p : ws.c.p;
        dv[p] = !has_v ? nullptr : c == 'K' ? vals : c == 'A' ? ws.b.p : ws.d.p;
    }
    const bool copy_back = npass == 1 && !sep;
    const uint32_t* kin = kin0;
    const uint32_t* vin = vin0;
    for (int p = 0; p < npass; p++) {
        const uint64_t tag = lb_begin(ws, tiles, 256, st);
        RP_REQUIRE(dk[p] != kin, "radix sort: pass writes its input");
        const bool io = p == 0 && iota;
        auto kern = io ? (items == 16 ? k_os_scatter<true, 16> : k_os_scatter<true, 8>)
                       : (items == 16 ? k_os_scatter<false, 16> : k_os_scatter<false, 8>);
        hipLaunchKernelGGL(kern, dim3(tiles), dim3(kThreads), 0, st, kin, io ? nullptr : vin, dk[p], dv[p],
                           (uint32_t)n, begin_bit + 8 * p, ws.dig.p + 1024 + 256 * p, ws.lb.p, ws.ticket.p, tiles, tag,
                           ws.err.p, run_if);
        RP_HIP(hipGetLastError());
        kin = dk[p];
        vin = dv[p];
    }
    if (copy_back) {
        RP_HIP(hipMemcpyAsync(keys, ws.a.p, n * sizeof(uint32_t), hipMemcpyDeviceToDevice, st));
        if (has_v) RP_HIP(hipMemcpyAsync(vals, ws.b.p, n * sizeof(uint32_t), hipMemcpyDeviceToDevice, st));
    }
}

}  // namespace

// Which sort a size takes (measured on MI355X, tests/test_prims_gpu.py and
// profiles/r02/prims_ab.json): the single-pass sort wins where the multi-pass one is
// launch-bound (1e5 keys: 0.068 vs 0.084 ms) and at 4M keys (0.32 vs 0.37 ms), and loses around
// 1M keys (0.21 vs 0.16 ms), where every tile is resident at once and the first tiles' look-back
// chains run the length of the grid.
bool single_pass_sort(uint64_t n) {
    if (prims_multipass()) return false;
    if (g_force_multipass == 0) return true;  // rp_selftest_prims mode 0: every size
    return n < (1u << 19) || n >= (1u << 22);
}

void scan_exclusive_u32(const uint32_t* in, uint32_t* out, uint64_t n, hipStream_t st, Scratch& ws) {
    ws.use_on(st);
    if (prims_multipass() || n == 0) {
        DevBuf<uint32_t>* lv[3] = {&ws.s0, &ws.s1, &ws.s2};
        scan_level(in, out, n, st, lv, 0);
        return;
    }
    RP_REQUIRE(n < (1ull << 32), "scan_exclusive_u32: n must be < 2^32");
    const uint32_t tiles = (uint32_t)((n + kTile - 1) / kTile);
    const uint64_t tag = lb_begin(ws, tiles, 1, st);
    hipLaunchKernelGGL(k_os_scan, dim3(tiles), dim3(kThreads), 0, st, in, out, (uint32_t)n, ws.lb.p, ws.ticket.p,
                       tag, tiles, ws.err.p);
    RP_HIP(hipGetLastError());
}

void radix_sort_index(const uint32_t* keys_in, uint32_t* keys_out, uint32_t* idx_out, uint64_t n, int begin_bit,
                      int end_bit, hipStream_t st, Scratch& ws, const uint32_t* run_if) {
    if (n == 0) return;
    RP_REQUIRE(n < (1ull << 32), "radix_sort_index: n must be < 2^32");
    ws.use_on(st);
    RP_REQUIRE(keys_in != keys_out, "radix_sort_index: keys_in must not be keys_out");
    if (n == 1) {  // (run regardless of run_if: harmless)
        RP_HIP(hipMemcpyAsync(keys_out, keys_in, sizeof(uint32_t), hipMemcpyDeviceToDevice, st));
        iota_u32(idx_out, 1, st);
        return;
    }
    if (!single_pass_sort(n) && !run_if) {  // (a gated sort always takes the single-pass kernels)
        RP_HIP(hipMemcpyAsync(keys_out, keys_in, n * sizeof(uint32_t), hipMemcpyDeviceToDevice, st));
        iota_u32(idx_out, n, st);
        radix_sort_pairs(keys_out, idx_out, n, begin_bit, end_bit, st, ws);
        return;
    }
    os_sort(keys_in, nullptr, true, keys_out, idx_out, n, begin_bit, end_bit, st, ws, run_if);
}

void radix_sort_pairs(uint32_t* keys, uint32_t* vals, uint64_t n, int begin_bit, int end_bit,
                      hipStream_t st, Scratch& ws) {
    if (n <= 1) return;
    RP_REQUIRE(n < (1ull << 32), "radix_sort_pairs: n must be < 2^32");
    ws.use_on(st);
    if (single_pass_sort(n)) {
        os_sort(keys, vals, false, keys, vals, n, begin_bit, end_bit, st, ws);
        return;
    }
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

// ------------------------------------------------------------------ self-test (GPU tests only)
//
// rp_selftest_prims: sorts and scans seeded keys on the device with the single-pass primitives
// (mode 0) or the multi-pass ones (mode 1) and checks them against std::stable_sort / a host
// prefix sum. skew: 0 uniform, 1 all equal, 2 sixteen distinct values, 3 descending. Returns
// the number of mismatching elements over all checks in *bad and the mean device time of the
// pair sort in *sort_ms (reps timed repetitions).
extern "C" int rp_selftest_prims(uint64_t n, uint32_t seed, int bits, int skew, int mode, int reps,
                                 uint64_t* bad, float* sort_ms) {
    using namespace rp;
    return guard([&] {
        RP_REQUIRE(bad && n < (1ull << 31) && bits >= 8 && bits <= 32 && bits % 8 == 0, "selftest: arguments");
        g_force_multipass = mode ? 1 : 0;
        struct Reset {
            ~Reset() { g_force_multipass = -1; }
        } reset;
        std::vector<uint32_t> k(n), v(n);
        uint64_t x = seed * 0x9E3779B97F4A7C15ull + 1;
        for (uint64_t i = 0; i < n; i++) {
            x ^= x << 13;
            x ^= x >> 7;
            x ^= x << 17;
            const uint32_t r = (uint32_t)(x >> 11);
            k[i] = skew == 1 ? 0x5A5A5A5Au : skew == 2 ? (r & 15u) * 0x10101010u : skew == 3 ? (uint32_t)(n - i) : r;
            v[i] = (uint32_t)i;
        }
        const uint32_t mask = bits == 32 ? 0xFFFFFFFFu : ((1u << bits) - 1u);
        std::vector<uint32_t> ord(n);
        for (uint64_t i = 0; i < n; i++) ord[i] = (uint32_t)i;
        std::stable_sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) { return (k[a] & mask) < (k[b] & mask); });
        hipStream_t st;
        RP_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
        Scratch ws;
        DevBuf<uint32_t> dk, dv, dk2, dv2, dscan;
        const uint64_t m = n ? n : 1;
        dk.reserve(m);
        dv.reserve(m);
        dk2.reserve(m);
        dv2.reserve(m);
        dscan.reserve(m + 1);
        std::vector<uint32_t> hk(n), hv(n);
        uint64_t nbad = 0;
        auto check_sorted = [&](const std::vector<uint32_t>& kk, const std::vector<uint32_t>* vv) {
            for (uint64_t i = 0; i < n; i++) {
                const uint32_t want = ord[i];
                if (kk[i] != k[want] || (vv && (*vv)[i] != want)) nbad++;
            }
        };
        auto put = [&]() {
            if (!n) return;
            RP_HIP(hipMemcpyAsync(dk.p, k.data(), n * 4, hipMemcpyHostToDevice, st));
            RP_HIP(hipMemcpyAsync(dv.p, v.data(), n * 4, hipMemcpyHostToDevice, st));
        };
        auto get = [&](const uint32_t* kp, const uint32_t* vp) {
            if (!n) return;
            RP_HIP(hipMemcpyAsync(hk.data(), kp, n * 4, hipMemcpyDeviceToHost, st));
            if (vp) RP_HIP(hipMemcpyAsync(hv.data(), vp, n * 4, hipMemcpyDeviceToHost, st));
            RP_HIP(hipStreamSynchronize(st));
        };
        // pairs, in place
        put();
        radix_sort_pairs(dk.p, dv.p, n, 0, bits, st, ws);
        get(dk.p, dv.p);
        check_sorted(hk, &hv);
        // keys only, in place
        put();
        radix_sort_pairs(dk.p, nullptr, n, 0, bits, st, ws);
        get(dk.p, nullptr);
        check_sorted(hk, nullptr);
        // (key, index) from a separate input
        put();
        radix_sort_index(dk.p, dk2.p, dv2.p, n, 0, bits, st, ws);
        get(dk2.p, dv2.p);
        check_sorted(hk, &hv);
        // exclusive scans of the low byte: separate output, then in place
        std::vector<uint32_t> lo(n), want(n + 1);
        uint32_t acc = 0;
        for (uint64_t i = 0; i < n; i++) {
            lo[i] = k[i] & 255u;
            want[i] = acc;
            acc += lo[i];
        }
        want[n] = acc;
        std::vector<uint32_t> got(n + 1);
        for (int inplace = 0; inplace < 2; inplace++) {
            if (n) RP_HIP(hipMemcpyAsync(dscan.p, lo.data(), n * 4, hipMemcpyHostToDevice, st));
            RP_HIP(hipMemsetAsync(dscan.p + n, 0xFF, 4, st));
            if (inplace) {
                scan_exclusive_u32(dscan.p, dscan.p, n, st, ws);
                RP_HIP(hipMemcpyAsync(got.data(), dscan.p, (n + 1) * 4, hipMemcpyDeviceToHost, st));
            } else {
                if (n) RP_HIP(hipMemcpyAsync(dk2.p, lo.data(), n * 4, hipMemcpyHostToDevice, st));
                DevBuf<uint32_t> o;
                o.reserve(n + 1);
                scan_exclusive_u32(dk2.p, o.p, n, st, ws);
                RP_HIP(hipMemcpyAsync(got.data(), o.p, (n + 1) * 4, hipMemcpyDeviceToHost, st));
                RP_HIP(hipStreamSynchronize(st));
            }
            RP_HIP(hipStreamSynchronize(st));
            for (uint64_t i = 0; i <= n; i++)
                if (got[i] != want[i]) nbad++;
        }
        // timing of the in-place pair sort (events around each sort only)
        float ms = 0.f;
        if (reps > 0 && n) {
            std::vector<hipEvent_t> ev(2 * reps);
            for (auto& e : ev) RP_HIP(hipEventCreate(&e));
            for (int r = 0; r < reps; r++) {
                put();
                RP_HIP(hipEventRecord(ev[2 * r], st));
                radix_sort_pairs(dk.p, dv.p, n, 0, bits, st, ws);
                RP_HIP(hipEventRecord(ev[2 * r + 1], st));
            }
            RP_HIP(hipStreamSynchronize(st));
            for (int r = 0; r < reps; r++) {
                float t = 0.f;
                RP_HIP(hipEventElapsedTime(&t, ev[2 * r], ev[2 * r + 1]));
                if (r > 0 || reps == 1) ms += t;  // the first repetition warms up
            }
            for (auto& e : ev) RP_HIP(hipEventDestroy(e));
            ms /= (float)(reps > 1 ? reps - 1 : 1);
        }
        RP_HIP(hipStreamSynchronize(st));
        RP_HIP(hipStreamDestroy(st));
        *bad = nbad;
        if (sort_ms) *sort_ms = ms;
    });
}
