// rp_farmhash.h — farmhash32 (farmhashmk::Hash32) for host C++ and HIP device code.
//
// Replaces the reference's only native component, the npm `farmhash` ^0.2.0 addon
// (reference package.json:34), at every call site: lib/ring/index.js:29,55,102,140,146,166
// and lib/membership/index.js:65. Written against the published FarmHash algorithm; the
// byte-source is a template parameter so one body serves
//   - plain byte buffers (host, and device strings at arbitrary offsets),
//   - "server + decimal(i)" replica strings that are never materialised (ring build),
//   - fixed-length keys already held in registers (the lookup hot loop, hash32_words<LEN>).
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define RP_HD __host__ __device__ __forceinline__
#else
#define RP_HD inline
#endif

namespace rp {
namespace fh {

constexpr uint32_t kC1 = 0xcc9e2d51u;
constexpr uint32_t kC2 = 0x1b873593u;

RP_HD uint32_t rotr(uint32_t v, int s) { return s == 0 ? v : ((v >> s) | (v << (32 - s))); }

RP_HD uint32_t fmix(uint32_t h) {
    h ^= h >> 16;
    h *= 0x85ebca6bu;
    h ^= h >> 13;
    h *= 0xc2b2ae35u;
    h ^= h >> 16;
    return h;
}

RP_HD uint32_t mur(uint32_t a, uint32_t h) {
    a *= kC1;
    a = rotr(a, 17);
    a *= kC2;
    h ^= a;
    h = rotr(h, 19);
    return h * 5 + 0xe6546b64u;
}

// Byte source over memory. w(o) = little-endian 32-bit fetch at byte offset o.
struct PtrSrc {
    const uint8_t* p;
    RP_HD uint32_t w(uint32_t o) const {
        return (uint32_t)p[o] | ((uint32_t)p[o + 1] << 8) | ((uint32_t)p[o + 2] << 16) |
               ((uint32_t)p[o + 3] << 24);
    }
    RP_HD int8_t b(uint32_t o) const { return (int8_t)p[o]; }
};

// The replica string `server + String(i)` (lib/ring/index.js:55,140) without materialising it.
struct ReplicaSrc {
    const uint8_t* name;
    uint32_t nlen;
    uint8_t dig[12];
    RP_HD uint8_t byte(uint32_t o) const { return o < nlen ? name[o] : dig[o - nlen]; }
    RP_HD uint32_t w(uint32_t o) const {
        return (uint32_t)byte(o) | ((uint32_t)byte(o + 1) << 8) | ((uint32_t)byte(o + 2) << 16) |
               ((uint32_t)byte(o + 3) << 24);
    }
    RP_HD int8_t b(uint32_t o) const { return (int8_t)byte(o); }
};

// Writes decimal(i) into dig, returns the digit count.
RP_HD uint32_t decimal(uint32_t i, uint8_t* dig) {
    uint8_t tmp[12];
    uint32_t n = 0;
    do {
        tmp[n++] = (uint8_t)('0' + i % 10);
        i /= 10;
    } while (i);
    for (uint32_t k = 0; k < n; k++) dig[k] = tmp[n - 1 - k];
    return n;
}

template <class S>
RP_HD uint32_t hash32(const S& s, uint32_t len) {
    if (len <= 4) {
        uint32_t b = 0, c = 9;
        for (uint32_t i = 0; i < len; i++) {
            b = b * kC1 + (uint32_t)(int32_t)s.b(i);
            c ^= b;
        }
        return fmix(mur(b, mur(len, c)));
    }
    if (len <= 12) {
        uint32_t a = len, b = len * 5, c = 9, d = b;
        a += s.w(0);
        b += s.w(len - 4);
        c += s.w((len >> 1) & 4);
        return fmix(mur(c, mur(b, mur(a, d))));
    }
    if (len <= 24) {
        uint32_t a = s.w((len >> 1) - 4);
        uint32_t b = s.w(4);
        uint32_t c = s.w(len - 8);
        uint32_t d = s.w(len >> 1);
        uint32_t e = s.w(0);
        uint32_t f = s.w(len - 4);
        uint32_t h = d * kC1 + len;
        a = rotr(a, 12) + f;
        h = mur(c, h) + a;
        a = rotr(a, 3) + c;
        h = mur(e, h) + a;
        a = rotr(a + f, 12) + d;
        h = mur(b, h) + a;
        return fmix(h);
    }
    uint32_t h = len, g = kC1 * len, f = g;
    uint32_t a0 = rotr(s.w(len - 4) * kC1, 17) * kC2;
    uint32_t a1 = rotr(s.w(len - 8) * kC1, 17) * kC2;
    uint32_t a2 = rotr(s.w(len - 16) * kC1, 17) * kC2;
    uint32_t a3 = rotr(s.w(len - 12) * kC1, 17) * kC2;
    uint32_t a4 = rotr(s.w(len - 20) * kC1, 17) * kC2;
    h ^= a0;
    h = rotr(h, 19) * 5 + 0xe6546b64u;
    h ^= a2;
    h = rotr(h, 19) * 5 + 0xe6546b64u;
    g ^= a1;
    g = rotr(g, 19) * 5 + 0xe6546b64u;
    g ^= a3;
    g = rotr(g, 19) * 5 + 0xe6546b64u;
    f += a4;
    f = rotr(f, 19) + 113;
    uint32_t iters = (len - 1) / 20;
    uint32_t o = 0;
    do {
        uint32_t a = s.w(o), b = s.w(o + 4), c = s.w(o + 8), d = s.w(o + 12), e = s.w(o + 16);
        h += a;
        g += b;
        f += c;
        h = mur(d, h) + e;
        g = mur(c, g) + a;
        f = mur(b + e * kC1, f) + d;
        f += g;
        g += f;
        o += 20;
    } while (--iters != 0);
    g = rotr(g, 11) * kC1;
    g = rotr(g, 17) * kC1;
    f = rotr(f, 11) * kC1;
    f = rotr(f, 17) * kC1;
    h = rotr(h + g, 19);
    h = h * 5 + 0xe6546b64u;
    h = rotr(h, 17) * kC1;
    h = rotr(h + f, 19);
    h = h * 5 + 0xe6546b64u;
    h = rotr(h, 17) * kC1;
    return h;
}

// h * 5 + 0xe6546b64 as a shift-add: hipcc otherwise emits v_mad_u64_u32 (a 64-bit
// multiply-add at a fraction of the VALU rate) for the 32-bit result. Device only.
RP_HD uint32_t m5c(uint32_t h) {
#if defined(__HIP_DEVICE_COMPILE__)
    uint32_t r;
    asm volatile("v_lshl_add_u32 %0, %1, 2, %1" : "=v"(r) : "v"(h));
    return r + 0xe6546b64u;
#else
    return h * 5 + 0xe6546b64u;
#endif
}

RP_HD uint32_t mur_w(uint32_t a, uint32_t h) {
    a *= kC1;
    a = rotr(a, 17);
    a *= kC2;
    h ^= a;
    return m5c(rotr(h, 19));
}

// Fixed-length key (LEN % 4 == 0, LEN > 24) held as LEN/4 little-endian words: every fetch
// offset is a compile-time multiple of 4, so the whole hash runs out of registers.
template <uint32_t LEN>
RP_HD uint32_t hash32_words(const uint32_t* w) {
    static_assert(LEN % 4 == 0 && LEN > 24, "hash32_words needs LEN % 4 == 0 and LEN > 24");
    uint32_t h = LEN, g = kC1 * LEN, f = g;
    uint32_t a0 = rotr(w[(LEN - 4) / 4] * kC1, 17) * kC2;
    uint32_t a1 = rotr(w[(LEN - 8) / 4] * kC1, 17) * kC2;
    uint32_t a2 = rotr(w[(LEN - 16) / 4] * kC1, 17) * kC2;
    uint32_t a3 = rotr(w[(LEN - 12) / 4] * kC1, 17) * kC2;
    uint32_t a4 = rotr(w[(LEN - 20) / 4] * kC1, 17) * kC2;
    h ^= a0;
    h = m5c(rotr(h, 19));
    h ^= a2;
    h = m5c(rotr(h, 19));
    g ^= a1;
    g = m5c(rotr(g, 19));
    g ^= a3;
    g = m5c(rotr(g, 19));
    f += a4;
    f = rotr(f, 19) + 113;
    constexpr uint32_t iters = (LEN - 1) / 20;
#if defined(__HIPCC__)
#pragma unroll
#endif
    for (uint32_t it = 0; it < iters; it++) {
        uint32_t a = w[it * 5 + 0], b = w[it * 5 + 1], c = w[it * 5 + 2], d = w[it * 5 + 3],
                 e = w[it * 5 + 4];
        h += a;
        g += b;
        f += c;
        h = mur_w(d, h) + e;
        g = mur_w(c, g) + a;
        f = mur_w(b + e * kC1, f) + d;
        f += g;
        g += f;
    }
    g = rotr(g, 11) * kC1;
    g = rotr(g, 17) * kC1;
    f = rotr(f, 11) * kC1;
    f = rotr(f, 17) * kC1;
    h = m5c(rotr(h + g, 19));
    h = rotr(h, 17) * kC1;
    h = m5c(rotr(h + f, 19));
    h = rotr(h, 17) * kC1;
    return h;
}

}  // namespace fh
}  // namespace rp
