// rp_hashlong.hip — one long farmhash32 chain on the device.
//
// farmhashmk::Hash32 over a long string is a serial chain across 20-byte chunks, so one
// string runs on one lane. Everything in a chunk that does not depend on the chain state
// (the five words and the three Murmur pre-mixes rotr(x*c1,17)*c2 of d, c and b+e*c1) is
// computed ahead by 128 producer lanes of the workgroup into a double-buffered LDS window;
// the chain lanes then do 5 dependent ops per chunk (the regrouping below). Per-view parallel checksums (the
// simulator) use one lane per view instead.
#include "rp_farmhash.h"
#include "rp_hashlong.h"

namespace rp {

namespace {

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

}  // namespace

void hash_long(const uint8_t* d_s, uint64_t len, const uint32_t* d_total, const uint32_t* d_gate, uint32_t* d_out,
               hipStream_t st) {
    hipLaunchKernelGGL(k_hash_long, dim3(1), dim3(kHlThreads), 0, st, d_s, len, d_total, d_gate, d_out);
    RP_HIP(hipGetLastError());
}

void hash_long_multi(const uint8_t* d_s, uint64_t stride, uint32_t n, uint32_t* d_meta, hipStream_t st) {
    if (!n) return;
    hipLaunchKernelGGL(k_hash_long_multi, dim3(n), dim3(kHlThreads), 0, st, d_s, stride, d_meta);
    RP_HIP(hipGetLastError());
}

}  // namespace rp
