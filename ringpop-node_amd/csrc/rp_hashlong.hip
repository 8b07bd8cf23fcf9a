// rp_hashlong.hip — one long farmhash32 chain on the device.
//
// farmhashmk::Hash32 over a long string is a serial chain across 20-byte chunks, so one
// string runs on one lane. Everything in a chunk that does not depend on the chain state
// (the five words and the three Murmur pre-mixes rotr(x*c1,17)*c2 of d, c and b+e*c1) is
// computed ahead by the other 192 lanes of the workgroup into a double-buffered LDS window;
// the chain lane then does ~7 dependent ops per chunk. Per-view parallel checksums (the
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

__global__ __launch_bounds__(kHlThreads) void k_hash_long(const uint8_t* __restrict__ s, uint64_t len_host,
                                                          const uint32_t* __restrict__ d_total,
                                                          const uint32_t* __restrict__ d_gate,
                                                          uint32_t* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) uint32_t win[2][kWin][8];
    if (d_gate && *d_gate == 0) return;
    uint64_t len = len_host;
    if (d_total) {
        const uint32_t t = *d_total;
        len = t ? t - 1 : 0;
    }
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
    auto fill = [&](int buf, uint64_t c0, int t0, int nt) {
        for (int j = t0; j < kWin; j += nt) {
            const uint64_t c = c0 + j;
            if (c >= iters) break;
            const uint64_t o = c * 20;
            uint32_t a, b, cc, d, e;
            if (aligned) {
                const uint32_t* w = reinterpret_cast<const uint32_t*>(s + o);
                a = w[0]; b = w[1]; cc = w[2]; d = w[3]; e = w[4];
            } else {
                a = ld32(s, o); b = ld32(s, o + 4); cc = ld32(s, o + 8); d = ld32(s, o + 12); e = ld32(s, o + 16);
            }
            uint32_t* r = win[buf][j];
            r[0] = a; r[1] = b; r[2] = cc; r[3] = d;
            r[4] = e; r[5] = premix(d); r[6] = premix(cc); r[7] = premix(b + e * fh::kC1);
        }
    };
    // chain state (lane 0 only)
    uint32_t h = 0, g = 0, f = 0;
    if (tid == 0) {
        const uint32_t L = (uint32_t)len;
        h = L;
        g = fh::kC1 * L;
        f = g;
        const uint32_t a0 = premix(ld32(s, len - 4)), a1 = premix(ld32(s, len - 8)), a2 = premix(ld32(s, len - 16)),
                       a3 = premix(ld32(s, len - 12)), a4 = premix(ld32(s, len - 20));
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
    fill(0, 0, tid, kHlThreads);
    __syncthreads();
    const uint64_t nwin = (iters + kWin - 1) / kWin;
    for (uint64_t w = 0; w < nwin; w++) {
        const int cur = (int)(w & 1);
        if (tid >= 64) {
            if (w + 1 < nwin) fill(cur ^ 1, (w + 1) * kWin, tid - 64, kHlThreads - 64);
        } else if (tid == 0) {
            const uint64_t c0 = w * kWin;
            const int n = (int)((iters - c0) < (uint64_t)kWin ? (iters - c0) : kWin);
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
        out[0] = h;
        out[1] = 1;
    }
}

}  // namespace

void hash_long(const uint8_t* d_s, uint64_t len, const uint32_t* d_total, const uint32_t* d_gate, uint32_t* d_out,
               hipStream_t st) {
    hipLaunchKernelGGL(k_hash_long, dim3(1), dim3(kHlThreads), 0, st, d_s, len, d_total, d_gate, d_out);
    RP_HIP(hipGetLastError());
}

}  // namespace rp
