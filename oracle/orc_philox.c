/*
 * orc_philox.c — Philox4x32-10 and the synthetic input formats of SURVEY.md §8d.
 * TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * The reference draws keys/ids from Math.random / uuid.v4 (lib/membership/update.js:30);
 * the build replaces every such draw by a counter-based Philox4x32-10 stream so the GPU,
 * this oracle and the injected reference harness see identical inputs.
 * Pin: Random123 known answer philox4x32_10(ctr=0, key=0) = 6627e8d5 e169c58d bc57ac4c 9b00dbd8.
 */
#include <stdio.h>
#include <string.h>

#include "oracle.h"

void orc_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
    uint32_t k0 = key[0], k1 = key[1];
    for (int r = 0; r < 10; r++) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        uint32_t n0 = hi1 ^ c1 ^ k0;
        uint32_t n1 = lo1;
        uint32_t n2 = hi0 ^ c3 ^ k1;
        uint32_t n3 = lo0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* key k -> 16 random bytes (little-endian words of philox(ctr={k_lo,k_hi,0,0},
 * key={seed,0x52494e47 'RING'})), version/variant bits set as uuid.v4 does, formatted
 * 8-4-4-4-12 lowercase hex (node-uuid unparse order). */
void orc_uuid_key(uint32_t seed, uint64_t k, char out[36]) {
    static const char hex[] = "0123456789abcdef";
    uint32_t ctr[4] = {(uint32_t)k, (uint32_t)(k >> 32), 0, 0};
    uint32_t key[2] = {seed, 0x52494e47u};
    uint32_t r[4];
    orc_philox4x32_10(ctr, key, r);
    uint8_t b[16];
    for (int i = 0; i < 4; i++) {
        b[4 * i + 0] = (uint8_t)(r[i]);
        b[4 * i + 1] = (uint8_t)(r[i] >> 8);
        b[4 * i + 2] = (uint8_t)(r[i] >> 16);
        b[4 * i + 3] = (uint8_t)(r[i] >> 24);
    }
    b[6] = (uint8_t)((b[6] & 0x0f) | 0x40);
    b[8] = (uint8_t)((b[8] & 0x3f) | 0x80);
    int o = 0;
    for (int i = 0; i < 16; i++) {
        if (i == 4 || i == 6 || i == 8 || i == 10) out[o++] = '-';
        out[o++] = hex[b[i] >> 4];
        out[o++] = hex[b[i] & 15];
    }
}

void orc_gen_uuid_keys(uint32_t seed, uint64_t k0, uint64_t n, char *out) {
    for (uint64_t i = 0; i < n; i++) orc_uuid_key(seed, k0 + i, out + 36 * i);
}

/* "10." + (i>>16&255) + "." + (i>>8&255) + "." + (i&255) + ":" + (20800+i%36) */
int orc_c2_addr(uint32_t i, char *out) {
    char buf[64];
    int n = snprintf(buf, sizeof buf, "10.%u.%u.%u:%u", (i >> 16) & 255u, (i >> 8) & 255u, i & 255u,
                     20800u + i % 36u);
    memcpy(out, buf, (size_t)n);
    return n;
}
