// rp_swim.h — SWIM membership rules as device/host functions, shared by the membership merge
// and the gossip simulator.
#pragma once

#include <stdint.h>

#include "rp_farmhash.h"  // RP_HD

namespace rp {

// Member.Status (lib/membership/member.js:204-209), encoded by precedence of the checksum
// strings' spelling: the numeric order carries no meaning for the rules below.
enum : uint8_t { ST_ALIVE = 0, ST_SUSPECT = 1, ST_FAULTY = 2, ST_LEAVE = 3 };

RP_HD uint32_t status_len(uint8_t s) { return s == ST_ALIVE ? 5u : s == ST_SUSPECT ? 7u : s == ST_FAULTY ? 6u : 5u; }

RP_HD uint8_t status_char(uint8_t s, uint32_t i) {
    // "alive" "suspect" "faulty" "leave"
    const char* const t = s == ST_ALIVE ? "alive" : s == ST_SUSPECT ? "suspect" : s == ST_FAULTY ? "faulty" : "leave";
    return (uint8_t)t[i];
}

// Member._isOtherOverride (member.js:171-202): may update (st, inc) replace (cur, cur_inc)?
RP_HD bool other_override(uint8_t cur, int64_t cur_inc, uint8_t st, int64_t inc) {
    switch (st) {
    case ST_ALIVE:  // isAliveOverride: any known status, strictly newer incarnation
        return inc > cur_inc;
    case ST_SUSPECT:  // isSuspectOverride
        return (cur == ST_SUSPECT && inc > cur_inc) || (cur == ST_FAULTY && inc > cur_inc) ||
               (cur == ST_ALIVE && inc >= cur_inc);
    case ST_FAULTY:  // isFaultyOverride
        return (cur == ST_SUSPECT && inc >= cur_inc) || (cur == ST_FAULTY && inc > cur_inc) ||
               (cur == ST_ALIVE && inc >= cur_inc);
    case ST_LEAVE:  // isLeaveOverride
        return cur != ST_LEAVE && inc >= cur_inc;
    }
    return false;
}

// Member.evaluateUpdate (member.js:71-122) for an existing member. Returns true if applied;
// (st, inc) are rewritten by the local override (suspect/faulty about the local member ->
// alive at Date.now(), member.js:76-81,155-169).
RP_HD bool evaluate_update(uint8_t cur, int64_t cur_inc, bool is_local_member, uint8_t& st, int64_t& inc,
                           int64_t now_ms) {
    if (is_local_member && (st == ST_SUSPECT || st == ST_FAULTY)) {
        st = ST_ALIVE;
        inc = now_ms;
        return true;
    }
    return other_override(cur, cur_inc, st, inc);
}

// Decimal digits of an int64 as JS prints an integral Number (|x| < 2^53 in practice).
// Comparisons against powers of ten: no 64-bit division on the device.
RP_HD uint32_t dec_len(int64_t v) {
    const uint64_t u = v < 0 ? (uint64_t)(-(v + 1)) + 1 : (uint64_t)v;
    uint32_t n = 1;
    uint64_t p = 10;
    while (n < 20 && u >= p) {
        n++;
        if (n < 20) p *= 10;
    }
    return n + (v < 0 ? 1u : 0u);
}

// Writes the n characters of dec_len(v). 64-bit divisions only while the value exceeds 32 bits.
RP_HD void dec_write(int64_t v, uint8_t* out, uint32_t n) {
    uint64_t u = v < 0 ? (uint64_t)(-(v + 1)) + 1 : (uint64_t)v;
    const uint32_t lo = v < 0 ? 1u : 0u;
    if (v < 0) out[0] = '-';
    uint32_t i = n;
    while (u > 0xFFFFFFFFull && i > lo) {
        const uint64_t q = u / 10;
        out[--i] = (uint8_t)('0' + (uint32_t)(u - q * 10));
        u = q;
    }
    uint32_t w = (uint32_t)u;
    while (i > lo) {
        const uint32_t q = w / 10;
        out[--i] = (uint8_t)('0' + (w - q * 10));
        w = q;
    }
}

}  // namespace rp
