// rp_philox.h — Philox4x32-10 and the synthetic UUID key format, host + device.
//
// The reference draws ids/keys from uuid.v4 / Math.random (lib/membership/update.js:30,
// lib/membership/index.js:130); the build's deterministic stand-in for every such draw is
// a counter-based Philox4x32-10 stream, so device, oracle and the injected
// reference harness see identical inputs.
#pragma once

#include <stdint.h>

#include "rp_farmhash.h"  // RP_HD

namespace rp {

struct U4 {
    uint32_t x, y, z, w;
};

RP_HD U4 philox4x32_10(U4 c, uint32_t k0, uint32_t k1) {
#if defined(__HIPCC__)
#pragma unroll
#endif
    for (int r = 0; r < 10; r++) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
        U4 n;
        n.x = (uint32_t)(p1 >> 32) ^ c.y ^ k0;
        n.y = (uint32_t)p1;
        n.z = (uint32_t)(p0 >> 32) ^ c.w ^ k1;
        n.w = (uint32_t)p0;
        c = n;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c;
}

constexpr uint32_t kUuidKeyTag = 0x52494e47u;  // 'RING'

// Key k of stream `seed`: 16 Philox bytes, uuid.v4 version/variant bits, 8-4-4-4-12
// lowercase hex. Writes 36 bytes as 9 little-endian words.
RP_HD void uuid_key_words(uint32_t seed, uint64_t k, uint32_t* out9) {
    U4 r = philox4x32_10(U4{(uint32_t)k, (uint32_t)(k >> 32), 0u, 0u}, seed, kUuidKeyTag);
    uint32_t rw[4] = {r.x, r.y, r.z, r.w};
    uint8_t b[16];
    for (int i = 0; i < 16; i++) b[i] = (uint8_t)(rw[i >> 2] >> (8 * (i & 3)));
    b[6] = (uint8_t)((b[6] & 0x0f) | 0x40);
    b[8] = (uint8_t)((b[8] & 0x3f) | 0x80);
    uint8_t s[36];
    int o = 0;
    for (int i = 0; i < 16; i++) {
        if (i == 4 || i == 6 || i == 8 || i == 10) s[o++] = '-';
        uint32_t hi = b[i] >> 4, lo = b[i] & 15;
        s[o++] = (uint8_t)(hi < 10 ? '0' + hi : 'a' + hi - 10);
        s[o++] = (uint8_t)(lo < 10 ? '0' + lo : 'a' + lo - 10);
    }
    for (int i = 0; i < 9; i++)
        out9[i] = (uint32_t)s[4 * i] | ((uint32_t)s[4 * i + 1] << 8) |
                  ((uint32_t)s[4 * i + 2] << 16) | ((uint32_t)s[4 * i + 3] << 24);
}

}  // namespace rp
