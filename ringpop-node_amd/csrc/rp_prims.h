// rp_prims.h — device primitives shared by the ring, membership and simulator paths:
// exclusive scan and a stable LSD radix sort of (uint32 key, uint32 value) pairs, both
// hand-written for gfx950 (wave64 ballots, LDS histograms).
#pragma once

#include "rp_common.h"

namespace rp {

struct Scratch {
    DevBuf<uint32_t> a, b, c, d;  // sort ping-pong keys/vals
    DevBuf<uint32_t> hist, hscan;  // radix histograms
    DevBuf<uint32_t> s0, s1, s2;   // scan block sums (3 levels)
};

// out[0..n) = exclusive prefix sum of in[0..n); out[n] = total. out may alias in.
// Supports n < 2048^3.
void scan_exclusive_u32(const uint32_t* in, uint32_t* out, uint64_t n, hipStream_t st, Scratch& ws);

// Stable sort of (keys, vals) by key bits [begin_bit, end_bit) (multiples of 8).
// vals may be null. Result is left in keys/vals.
void radix_sort_pairs(uint32_t* keys, uint32_t* vals, uint64_t n, int begin_bit, int end_bit,
                      hipStream_t st, Scratch& ws);

// out[i] = i for i < n
void iota_u32(uint32_t* out, uint64_t n, hipStream_t st);

// dst[i] = src[idx[i]] for i < n
void gather_u32(const uint32_t* src, const uint32_t* idx, uint32_t* dst, uint64_t n, hipStream_t st);

// Read one uint32 from device memory (synchronizes the stream).
uint32_t read_u32(const uint32_t* p, hipStream_t st);

}  // namespace rp
