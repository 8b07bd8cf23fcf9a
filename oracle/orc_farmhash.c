/*
 * orc_farmhash.c — CPU restatement of the third-party npm `farmhash` ^0.2.0 hash32
 * (reference package.json:34). TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * npm farmhash 0.2.x wraps Google FarmHash; util::Hash32 built with node-gyp's default
 * x86-64 flags (no SSE4.1/4.2 defines) resolves to farmhashmk::Hash32 (== Fingerprint32).
 * This file restates that published algorithm byte-by-byte (little-endian Fetch32,
 * RIGHT rotations, Murmur3 fmix). Call sites in the reference:
 *   lib/ring/index.js:29,55,102,140,146,166 and lib/membership/index.js:65.
 * Pin: Hash32("") == 0xdc56d17a (published FarmHash/go-farm known answer).
 */
#include "oracle.h"

static const uint32_t C1 = 0xcc9e2d51u;
static const uint32_t C2 = 0x1b873593u;

static uint32_t fetch32(const uint8_t *p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

static uint32_t rot32(uint32_t v, int s) { return s == 0 ? v : ((v >> s) | (v << (32 - s))); }

static uint32_t fmix(uint32_t h) {
    h ^= h >> 16;
    h *= 0x85ebca6bu;
    h ^= h >> 13;
    h *= 0xc2b2ae35u;
    h ^= h >> 16;
    return h;
}

static uint32_t mur(uint32_t a, uint32_t h) {
    a *= C1;
    a = rot32(a, 17);
    a *= C2;
    h ^= a;
    h = rot32(h, 19);
    return h * 5 + 0xe6546b64u;
}

static uint32_t len0to4(const uint8_t *s, size_t len) {
    uint32_t b = 0, c = 9;
    for (size_t i = 0; i < len; i++) {
        signed char v = (signed char)s[i];
        b = b * C1 + (uint32_t)(int32_t)v;
        c ^= b;
    }
    return fmix(mur(b, mur((uint32_t)len, c)));
}

static uint32_t len5to12(const uint8_t *s, size_t len) {
    uint32_t a = (uint32_t)len, b = (uint32_t)len * 5, c = 9, d = b;
    a += fetch32(s);
    b += fetch32(s + len - 4);
    c += fetch32(s + ((len >> 1) & 4));
    return fmix(mur(c, mur(b, mur(a, d))));
}

static uint32_t len13to24(const uint8_t *s, size_t len) {
    uint32_t a = fetch32(s - 4 + (len >> 1));
    uint32_t b = fetch32(s + 4);
    uint32_t c = fetch32(s + len - 8);
    uint32_t d = fetch32(s + (len >> 1));
    uint32_t e = fetch32(s);
    uint32_t f = fetch32(s + len - 4);
    uint32_t h = d * C1 + (uint32_t)len;
    a = rot32(a, 12) + f;
    h = mur(c, h) + a;
    a = rot32(a, 3) + c;
    h = mur(e, h) + a;
    a = rot32(a + f, 12) + d;
    h = mur(b, h) + a;
    return fmix(h);
}

uint32_t orc_hash32(const uint8_t *s, size_t len) {
    if (len <= 24) {
        if (len <= 12) return len <= 4 ? len0to4(s, len) : len5to12(s, len);
        return len13to24(s, len);
    }
    uint32_t h = (uint32_t)len, g = C1 * (uint32_t)len, f = g;
    uint32_t a0 = rot32(fetch32(s + len - 4) * C1, 17) * C2;
    uint32_t a1 = rot32(fetch32(s + len - 8) * C1, 17) * C2;
    uint32_t a2 = rot32(fetch32(s + len - 16) * C1, 17) * C2;
    uint32_t a3 = rot32(fetch32(s + len - 12) * C1, 17) * C2;
    uint32_t a4 = rot32(fetch32(s + len - 20) * C1, 17) * C2;
    h ^= a0;
    h = rot32(h, 19);
    h = h * 5 + 0xe6546b64u;
    h ^= a2;
    h = rot32(h, 19);
    h = h * 5 + 0xe6546b64u;
    g ^= a1;
    g = rot32(g, 19);
    g = g * 5 + 0xe6546b64u;
    g ^= a3;
    g = rot32(g, 19);
    g = g * 5 + 0xe6546b64u;
    f += a4;
    f = rot32(f, 19) + 113;
    size_t iters = (len - 1) / 20;
    do {
        uint32_t a = fetch32(s);
        uint32_t b = fetch32(s + 4);
        uint32_t c = fetch32(s + 8);
        uint32_t d = fetch32(s + 12);
        uint32_t e = fetch32(s + 16);
        h += a;
        g += b;
        f += c;
        h = mur(d, h) + e;
        g = mur(c, g) + a;
        f = mur(b + e * C1, f) + d;
        f += g;
        g += f;
        s += 20;
    } while (--iters != 0);
    g = rot32(g, 11) * C1;
    g = rot32(g, 17) * C1;
    f = rot32(f, 11) * C1;
    f = rot32(f, 17) * C1;
    h = rot32(h + g, 19);
    h = h * 5 + 0xe6546b64u;
    h = rot32(h, 17) * C1;
    h = rot32(h + f, 19);
    h = h * 5 + 0xe6546b64u;
    h = rot32(h, 17) * C1;
    return h;
}
