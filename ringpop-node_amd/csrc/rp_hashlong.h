// rp_hashlong.h — farmhash32 of ONE long device string (the ring / membership checksums).
#pragma once

#include "rp_common.h"

namespace rp {

// Hashes d_s[0 .. L) where L = (*d_total ? *d_total - 1 : 0) (a ';'-joined string whose
// builder counted one separator per piece) or L = len when d_total is null. If d_gate is
// non-null and *d_gate == 0 nothing is written. On completion d_out[0] = hash, d_out[1] = 1.
void hash_long(const uint8_t* d_s, uint64_t len, const uint32_t* d_total, const uint32_t* d_gate, uint32_t* d_out,
               hipStream_t st);

// n strings d_s + b * stride (b < n) hashed side by side, one workgroup each. d_meta[4b] = the
// builder's total (length + 1), d_meta[4b + 1] = gate (0: skip); hash -> d_meta[4b + 2],
// d_meta[4b + 3] = 1.
void hash_long_multi(const uint8_t* d_s, uint64_t stride, uint32_t n, uint32_t* d_meta, hipStream_t st);

}  // namespace rp
