// rp_hashlong.hip — one long farmhash32 chain on the device.
//
// farmhashmk::Hash32 over a long string is a serial chain across 20-byte chunks, so one
// string runs on one lane. Everything in a chunk that does not depend on the chain state
// (the five words and the three Murmur pre-mixes rotr(x*c1,17)*c2 of d, c and b+e*c1) is
// computed ahead by 128 producer lanes of the workgroup into a double-buffered LDS window;
// the chain lanes then do 5 dependent ops per chunk (the regrouping below). Per-view parallel checksums (the
// simulator) use one lane per view instead.
#include <cstdlib>

#include "rp_farmhash.h"
#include "rp_hashlong.h"

namespace rp {

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4), aligned(4)));  // (a chunk is 20 B: dword-aligned loads)

constexpr int kHlThreads = 256;
constexpr int kWin = 1024;  // chunks per LDS window

__device__ __forceinline__ uint32_t premix(uint32_t x) { return fh::rotr(x * fh::kC1, 17) * fh::kC2; }

__device__ __forceinline__ uint32_t ld32(const uint8_t* p, uint64_t o) {
    return (uint32_t)p[o] | ((uint32_t)p[o + 1] << 8) | ((uint32_t)p[o + 2] << 16) | ((uint32_t)p[o + 3] << 24);
}

// The chain in "pre-added" form. farmhashmk's chunk step (h += a; g += b; f += c; then three
// Murmur rounds; f += g; g += f) is regrouped so that each state word enters a chunk with the
// chunk's addend already folded in (hp = h + a, gp = g + b, fp = f + c), and the combine with
// the next chunk's addends is one precomputed constant per word:
//   r_x = rotr(xp ^ premix_x, 19)                         (x = h, g, f)
//   hp' = 5 r_h + (K + e + a')
//   fp' = 5 (r_f + r_g) + (2K + a + d + c')               (= f + g + c' of the original)
//   gp' = 5 (r_f + 2 r_g) + (3K + 2a + d + b')            (= g + f + b')
// where a', b', c' are the next chunk's words (0 after the last chunk, which leaves plain h, g,
// f). The dependent path per chunk drops from 7 to 5 VALU ops; the six per-chunk words
// {premix(d), premix(c), premix(b + e c1), K + e + a', 2K + a + d + c', 3K + 2a + d + b'} are
// independent of the chain and precomputed by the producer lanes.
constexpr uint32_t kK = 0xe6546b64u;

// (a << sh) + b as one v_lshl_add_u32 (inline asm keeps the compiler from re-associating the
// chain's sums into a longer dependent sequence)
template <int SH>
__device__ __forceinline__ uint32_t lshl_add(uint32_t a, uint32_t b) {
    uint32_t r;
    asm("v_lshl_add_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "i"(SH), "v"(b));
    return r;
}
__device__ __forceinline__ uint32_t mul5_add(uint32_t x, uint32_t c) {  // 5x + c: two dependent ops
    return lshl_add<2>(x, x + c);
}

// The coupled (g, f) pair runs on two lanes of one wave, g on lane 0 and f on lane 1, so one
// instruction advances both. With r = rotr(v ^ premix, 19) per lane and sh = 1 (g) or 0 (f):
//   v' = 5 r_other + (5 (r_self << sh) + c_self)
// (lane 0: 5 (r_f + 2 r_g) + c_g, lane 1: 5 (r_g + r_f) + c_f); the first term is a DPP quad
// permute of 5 r folded into the final add. Six VALU ops per chunk for both words where the
// single-lane form issued eleven, and no DPP wait states (5 r is written two ops before it is
// read across lanes): a lone wave issues about one instruction per four cycles, so the chain's
// rate is its instruction count. h (which never mixes with g and f before the finalisation)
// runs on lane 64.
__device__ __forceinline__ uint32_t lshl_add_v(uint32_t a, uint32_t sh, uint32_t b) {  // (a << sh) + b
    uint32_t r;
    asm("v_lshl_add_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(sh), "v"(b));
    return r;
}
__device__ __forceinline__ uint32_t swap_pair(uint32_t v) {  // lanes 2i <-> 2i+1 (quad_perm 1,0,3,2)
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, true);
}

// One string's chain by the whole workgroup (see the kernels below).
__device__ void hash_long_block(const uint8_t* __restrict__ s, uint64_t len, uint32_t* __restrict__ out) {
    // per window, per chain lane (g, f, h), per chunk: {premix word, next-chunk addend}
    __shared__ __attribute__((aligned(16))) uint2 win[2][3][kWin];
    __shared__ uint32_t s_st[3];
    const int tid = threadIdx.x;
    if (len <= 24) {
        if (tid == 0) {
            out[0] = fh::hash32(fh::PtrSrc{s}, (uint32_t)len);
            out[1] = 1;
        }
        return;
    }
    const bool aligned = (reinterpret_cast<uintptr_t>(s) & 3) == 0;
    const uint64_t iters = (len - 1) / 20;
    auto word = [&](uint64_t o) -> uint32_t {
        return aligned ? *reinterpret_cast<const uint32_t*>(s + o) : ld32(s, o);
    };
    auto fill = [&](int buf, uint64_t c0, int t0, int nt) {
        for (int j = t0; j < kWin; j += nt) {
            const uint64_t c = c0 + j;
            if (c >= iters) break;
            const uint64_t o = c * 20;
            const uint32_t a = word(o), b = word(o + 4), cc = word(o + 8), d = word(o + 12), e = word(o + 16);
            uint32_t a2 = 0, b2 = 0, c2 = 0;
            if (c + 1 < iters) {
                a2 = word(o + 20);
                b2 = word(o + 24);
                c2 = word(o + 28);
            }
            win[buf][0][j] = uint2{premix(cc), 3u * kK + 2u * a + d + b2};
            win[buf][1][j] = uint2{premix(b + e * fh::kC1), 2u * kK + a + d + c2};
            win[buf][2][j] = uint2{premix(d), kK + e + a2};
        }
    };
    if (tid == 0) {  // chain state pre-added with chunk 0's words
        const uint32_t L = (uint32_t)len;
        uint32_t h = L, g = fh::kC1 * L, f = g;
        const uint32_t a0 = premix(ld32(s, len - 4)), a1 = premix(ld32(s, len - 8)), a2 = premix(ld32(s, len - 16)),
                       a3 = premix(ld32(s, len - 12)), a4 = premix(ld32(s, len - 20));
        h ^= a0;
        h = fh::rotr(h, 19) * 5 + kK;
        h ^= a2;
        h = fh::rotr(h, 19) * 5 + kK;
        g ^= a1;
        g = fh::rotr(g, 19) * 5 + kK;
        g ^= a3;
        g = fh::rotr(g, 19) * 5 + kK;
        f += a4;
        f = fh::rotr(f, 19) + 113;
        s_st[0] = g + word(4);
        s_st[1] = f + word(8);
        s_st[2] = h + word(0);
    }
    fill(0, 0, tid, kHlThreads);
    __syncthreads();
    // lane 0: g, lane 1: f (wave 0); lane 64: h (wave 1)
    const int ln = tid < 2 ? tid : 2;
    uint32_t v = (tid < 2 || tid == 64) ? s_st[ln] : 0u;
    const uint32_t sh = tid == 0 ? 1u : 0u, sh2 = sh + 2u;
    const uint64_t nwin = (iters + kWin - 1) / kWin;
#ifdef RP_CK_PROF
    uint64_t t_chain = 0;
    const uint64_t t_start = clock64();
#endif
    auto step_gf = [&](const uint2 x) {
        const uint32_t y = v ^ x.x;
        const uint32_t r = __builtin_amdgcn_alignbit(y, y, 19);
        const uint32_t r5 = (r << 2) + r;
        const uint32_t own = (r << sh2) + ((r << sh) + x.y);
        v = swap_pair(r5) + own;
    };
    auto step_h = [&](const uint2 x) {
        const uint32_t y = v ^ x.x;
        v = mul5_add(__builtin_amdgcn_alignbit(y, y, 19), x.y);
    };
    for (uint64_t w = 0; w < nwin; w++) {
        const int cur = (int)(w & 1);
        if (tid >= 128) {
            if (w + 1 < nwin) fill(cur ^ 1, (w + 1) * kWin, tid - 128, kHlThreads - 128);
        } else if (tid < 2 || tid == 64) {
#ifdef RP_CK_PROF
            const uint64_t tc0 = clock64();
#endif
            const uint64_t c0 = w * kWin;
            const int n = (int)((iters - c0) < (uint64_t)kWin ? (iters - c0) : kWin);
            const uint2* src = win[cur][ln];
            int j = 0;
            if (tid < 2) {
                for (; j + 8 <= n; j += 8) {  // the LDS reads of 8 chunks issued ahead of their steps
                    uint4 x[4];
#pragma unroll
                    for (int q = 0; q < 4; q++) x[q] = *reinterpret_cast<const uint4*>(src + j + 2 * q);
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        step_gf(uint2{x[q].x, x[q].y});
                        step_gf(uint2{x[q].z, x[q].w});
                    }
                }
                for (; j < n; j++) step_gf(src[j]);
            } else {
                for (; j + 8 <= n; j += 8) {
                    uint4 x[4];
#pragma unroll
                    for (int q = 0; q < 4; q++) x[q] = *reinterpret_cast<const uint4*>(src + j + 2 * q);
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        step_h(uint2{x[q].x, x[q].y});
                        step_h(uint2{x[q].z, x[q].w});
                    }
                }
                for (; j < n; j++) step_h(src[j]);
            }
#ifdef RP_CK_PROF
            if (tid == 0) t_chain += clock64() - tc0;
#endif
        }
        __syncthreads();
    }
    if (tid < 2 || tid == 64) s_st[ln] = v;
    __syncthreads();
    if (tid == 0) {
        uint32_t h = s_st[2], g = s_st[0], f = s_st[1];  // the last chunk's next-words were 0
        g = fh::rotr(g, 11) * fh::kC1;
        g = fh::rotr(g, 17) * fh::kC1;
        f = fh::rotr(f, 11) * fh::kC1;
        f = fh::rotr(f, 17) * fh::kC1;
        h = fh::rotr(h + g, 19);
        h = h * 5 + kK;
        h = fh::rotr(h, 17) * fh::kC1;
        h = fh::rotr(h + f, 19);
        h = h * 5 + kK;
        h = fh::rotr(h, 17) * fh::kC1;
        out[0] = h;
        out[1] = 1;
#ifdef RP_CK_PROF
        printf("hlprof iters %llu total %llu chain %llu cycles (%.1f per chunk)\n", (unsigned long long)iters,
               (unsigned long long)(clock64() - t_start), (unsigned long long)t_chain, (double)t_chain / iters);
#endif
    }
}

__global__ __launch_bounds__(kHlThreads) void k_hash_long(const uint8_t* __restrict__ s, uint64_t len_host,
                                                          const uint32_t* __restrict__ d_total,
                                                          const uint32_t* __restrict__ d_gate,
                                                          uint32_t* __restrict__ out) {
    if (d_gate && *d_gate == 0) return;
    uint64_t len = len_host;
    if (d_total) {
        const uint32_t t = *d_total;
        len = t ? t - 1 : 0;
    }
    hash_long_block(s, len, out);
}

// Many strings at once, one workgroup (one serial chain + its producers) per string: string b
// is s + b * stride, meta[4b] = its builder's total (length + 1), meta[4b + 1] = its gate (0:
// skip); the hash goes to meta[4b + 2] (meta[4b + 3] = 1).
__global__ __launch_bounds__(kHlThreads) void k_hash_long_multi(const uint8_t* __restrict__ s, uint64_t stride,
                                                                uint32_t* __restrict__ meta) {
    uint32_t* m = meta + 4ull * blockIdx.x;
    if (m[1] == 0) return;
    const uint32_t t = m[0];
    hash_long_block(s + stride * blockIdx.x, t ? t - 1 : 0, m + 2);
}

// Many strings per workgroup (round 6; the C3 checksum groups). k_hash_long_multi gives each
// string a workgroup: 128 strings take 128 workgroups of four waves whose chain lanes run alone
// on their SIMDs, and a group of 256 took twice as long as one of 128 beside the folds. Here one
// wave runs the (g, f) pairs of kHpStr strings on lane pairs 2q, 2q + 1 (the same instruction
// stream as hash_long_block's lanes 0 and 1: swap_pair is a quad permute) and a second wave the
// h chains on lanes 0..kHpStr-1, so a chain costs what it did but a workgroup carries kHpStr of
// them. Four producer waves fill the next window of every string's pre-added words (two 16-B
// loads per chunk: words 0..3 and 4..7 of [20c, 20c + 32)), with the loads for the window after
// it issued before the barrier, so their latency overlaps a whole window. Strings of a workgroup
// run in lockstep to the shortest one's chunk count, then the rest under per-lane masks.
constexpr int kHpStr = 16;                    // strings per workgroup
constexpr int kHpWin = 64;                    // chunks per window
constexpr int kHpProd = 4;                    // producer waves
constexpr int kHpThreads = 64 * (2 + kHpProd);
constexpr int kHpRow = kHpWin + 2;            // uint2 per (word, string) row: 528 B, a 4-bank shift a row
constexpr int kHpItems = kHpStr * kHpWin / (64 * kHpProd);  // (string, chunk) items per producer lane

__global__ __launch_bounds__(kHpThreads) void k_hash_long_pack(const uint8_t* __restrict__ sbase, uint64_t stride,
                                                               uint32_t n, uint32_t* __restrict__ meta) {
    __shared__ __attribute__((aligned(16))) uint2 win[2][3 * kHpStr][kHpRow];
    __shared__ uint32_t s_it[kHpStr], s_st[3][kHpStr], s_common, s_max;
    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
    const uint32_t q0 = blockIdx.x * kHpStr;
    if (tid < kHpStr) {  // per string: gate, length, chain state pre-added with chunk 0's words
        const uint32_t q = q0 + tid;
        uint32_t it = 0;
        if (q < n && meta[4 * q + 1] != 0) {
            const uint32_t t = meta[4 * q];
            const uint64_t len = t ? t - 1 : 0;
            const uint8_t* str = sbase + stride * q;
            if (len <= 24) {
                meta[4 * q + 2] = fh::hash32(fh::PtrSrc{str}, (uint32_t)len);
                meta[4 * q + 3] = 1;
            } else {
                it = (uint32_t)((len - 1) / 20);
                const uint32_t L = (uint32_t)len;
                uint32_t h = L, g = fh::kC1 * L, f = g;
                const uint32_t a0 = premix(ld32(str, len - 4)), a1 = premix(ld32(str, len - 8)),
                               a2 = premix(ld32(str, len - 16)), a3 = premix(ld32(str, len - 12)),
                               a4 = premix(ld32(str, len - 20));
                h ^= a0;
                h = fh::rotr(h, 19) * 5 + kK;
                h ^= a2;
                h = fh::rotr(h, 19) * 5 + kK;
                g ^= a1;
                g = fh::rotr(g, 19) * 5 + kK;
                g ^= a3;
                g = fh::rotr(g, 19) * 5 + kK;
                f += a4;
                f = fh::rotr(f, 19) + 113;
                const uint32_t* w = reinterpret_cast<const uint32_t*>(str);
                s_st[0][tid] = g + w[1];
                s_st[1][tid] = f + w[2];
                s_st[2][tid] = h + w[0];
            }
        }
        s_it[tid] = it;
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t lo = 0xFFFFFFFFu, hi = 0;
        for (int q = 0; q < kHpStr; q++)
            if (s_it[q]) {
                lo = s_it[q] < lo ? s_it[q] : lo;
                hi = s_it[q] > hi ? s_it[q] : hi;
            }
        s_common = hi ? lo : 0u;
        s_max = hi;
    }
    __syncthreads();
    const uint32_t common = s_common, itmax = s_max;
    if (itmax == 0) return;  // block-uniform: no long string here
    const uint32_t nwin = (itmax + kHpWin - 1) / kHpWin;
    // producers: item i of lane p is (string (p + 256 i) >> 6, chunk (p + 256 i) & 63) of a window
    const int p = tid - 128;
    u32x4 ra[kHpItems], rb[kHpItems];
    auto issue = [&](uint32_t w) {  // the raw words of window w, into registers
#pragma unroll
        for (int i = 0; i < kHpItems; i++) {
            const int item = p + 64 * kHpProd * i, q = item / kHpWin, j = item % kHpWin;
            const uint64_t c = (uint64_t)w * kHpWin + j;
            if (c < s_it[q]) {
                const u32x4* src = reinterpret_cast<const u32x4*>(sbase + stride * (q0 + q) + 20 * c);
                ra[i] = src[0];
                rb[i] = src[1];
            }
        }
    };
    auto fill = [&](int buf, uint32_t w) {  // window w's pre-added words from the registers
#pragma unroll
        for (int i = 0; i < kHpItems; i++) {
            const int item = p + 64 * kHpProd * i, q = item / kHpWin, j = item % kHpWin;
            const uint64_t c = (uint64_t)w * kHpWin + j;
            if (c < s_it[q]) {
                const uint32_t a = ra[i].x, b = ra[i].y, cc = ra[i].z, d = ra[i].w, e = rb[i].x;
                const bool nx = c + 1 < s_it[q];
                const uint32_t a2 = nx ? rb[i].y : 0u, b2 = nx ? rb[i].z : 0u, c2 = nx ? rb[i].w : 0u;
                win[buf][q][j] = uint2{premix(cc), 3u * kK + 2u * a + d + b2};
                win[buf][kHpStr + q][j] = uint2{premix(b + e * fh::kC1), 2u * kK + a + d + c2};
                win[buf][2 * kHpStr + q][j] = uint2{premix(d), kK + e + a2};
            }
        }
    };
    if (tid >= 128) {
        issue(0);
        fill(0, 0);
        if (nwin > 1) issue(1);
    }
    __syncthreads();
    // chain lanes: wave 0 lanes 0..2 kHpStr - 1 run (g, f) of string lane >> 1; wave 1 lanes
    // 0..kHpStr - 1 run h of string lane
    const bool gf = wv == 0, hw = wv == 1;
    const uint32_t cq = gf ? (uint32_t)(lane >> 1) % kHpStr : (uint32_t)lane % kHpStr;
    const uint32_t comp = gf ? (uint32_t)(lane & 1) : 2u;
    const bool live = (gf && lane < 2 * kHpStr) || (hw && lane < kHpStr);
    uint32_t v = live ? s_st[comp][cq] : 0u;
    const uint32_t mine = live ? s_it[cq] : 0u;
    const uint32_t sh = (gf && comp == 0) ? 1u : 0u, sh2 = sh + 2u;
    const int row = (int)(comp * kHpStr + cq);
    auto step_gf = [&](const uint2 x) {
        const uint32_t y = v ^ x.x;
        const uint32_t r = __builtin_amdgcn_alignbit(y, y, 19);
        const uint32_t r5 = (r << 2) + r;
        const uint32_t own = (r << sh2) + ((r << sh) + x.y);
        v = swap_pair(r5) + own;
    };
    auto step_h = [&](const uint2 x) {
        const uint32_t y = v ^ x.x;
        v = mul5_add(__builtin_amdgcn_alignbit(y, y, 19), x.y);
    };
    for (uint32_t w = 0; w < nwin; w++) {
        const int cur = (int)(w & 1);
        if (tid >= 128) {
            if (w + 1 < nwin) {
                fill(cur ^ 1, w + 1);
                if (w + 2 < nwin) issue(w + 2);
            }
        } else {
            const uint32_t c0 = w * kHpWin;
            const int nw = (int)((itmax - c0) < (uint32_t)kHpWin ? (itmax - c0) : (uint32_t)kHpWin);
            const int nc = common > c0 ? (int)((common - c0) < (uint32_t)nw ? (common - c0) : (uint32_t)nw) : 0;
            const uint2* src = &win[cur][row][0];
            int j = 0;
            if (gf) {
                for (; j + 8 <= nc; j += 8) {  // every string still running: no masks
                    uint4 x[4];
#pragma unroll
                    for (int q = 0; q < 4; q++) x[q] = *reinterpret_cast<const uint4*>(src + j + 2 * q);
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        step_gf(uint2{x[q].x, x[q].y});
                        step_gf(uint2{x[q].z, x[q].w});
                    }
                }
                for (; j < nw; j++) {  // past the shortest string: a lane pair stops at its own end
                    const uint32_t keep = v;
                    step_gf(src[j]);
                    v = c0 + (uint32_t)j < mine ? v : keep;
                }
            } else {
                for (; j + 8 <= nc; j += 8) {
                    uint4 x[4];
#pragma unroll
                    for (int q = 0; q < 4; q++) x[q] = *reinterpret_cast<const uint4*>(src + j + 2 * q);
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        step_h(uint2{x[q].x, x[q].y});
                        step_h(uint2{x[q].z, x[q].w});
                    }
                }
                for (; j < nw; j++) {
                    const uint32_t keep = v;
                    step_h(src[j]);
                    v = c0 + (uint32_t)j < mine ? v : keep;
                }
            }
        }
        __syncthreads();
    }
    if (live) s_st[comp][cq] = v;
    __syncthreads();
    if (tid < kHpStr && s_it[tid]) {
        uint32_t h = s_st[2][tid], g = s_st[0][tid], f = s_st[1][tid];  // the last chunk's next-words were 0
        g = fh::rotr(g, 11) * fh::kC1;
        g = fh::rotr(g, 17) * fh::kC1;
        f = fh::rotr(f, 11) * fh::kC1;
        f = fh::rotr(f, 17) * fh::kC1;
        h = fh::rotr(h + g, 19);
        h = h * 5 + kK;
        h = fh::rotr(h, 17) * fh::kC1;
        h = fh::rotr(h + f, 19);
        h = h * 5 + kK;
        h = fh::rotr(h, 17) * fh::kC1;
        uint32_t* m = meta + 4ull * (q0 + tid);
        m[2] = h;
        m[3] = 1;
    }
}

}  // namespace

void hash_long(const uint8_t* d_s, uint64_t len, const uint32_t* d_total, const uint32_t* d_gate, uint32_t* d_out,
               hipStream_t st) {
    hipLaunchKernelGGL(k_hash_long, dim3(1), dim3(kHlThreads), 0, st, d_s, len, d_total, d_gate, d_out);
    RP_HIP(hipGetLastError());
}

void hash_long_multi(const uint8_t* d_s, uint64_t stride, uint32_t n, uint32_t* d_meta, hipStream_t st) {
    if (!n) return;
    // RP_HL_LDS_PAD (A/B): bytes of unused dynamic LDS per chain workgroup, so that fewer chains
    // share a CU (48 KB of windows each: up to three a CU otherwise)
    const char* pe = getenv("RP_HL_LDS_PAD");
    const uint32_t pad = pe && *pe ? (uint32_t)atoi(pe) : 0u;
    // kHpStr strings a workgroup (round 6; RP_HL_PACK=0: one workgroup a string) for 16-B aligned
    // strings at a 16-B multiple stride (the membership slots are 256-B aligned)
    const char* pk = getenv("RP_HL_PACK");
    const bool pack = !(pk && *pk == '0') && ((reinterpret_cast<uintptr_t>(d_s) | stride) & 15) == 0;
    if (pack)
        hipLaunchKernelGGL(k_hash_long_pack, dim3((n + kHpStr - 1) / kHpStr), dim3(kHpThreads), 0, st, d_s, stride, n,
                           d_meta);
    else
        hipLaunchKernelGGL(k_hash_long_multi, dim3(n), dim3(kHlThreads), pad, st, d_s, stride, d_meta);
    RP_HIP(hipGetLastError());
}

}  // namespace rp
