// rp_prims.h — device primitives shared by the ring, membership and simulator paths:
// exclusive scan and a stable LSD radix sort of (uint32 key, uint32 value) pairs, both
// hand-written for gfx950 (wave64 ballots, LDS histograms).
#pragma once

#include "rp_common.h"

namespace rp {

struct Scratch {
    DevBuf<uint32_t> a, b, c, d;  // sort ping-pong keys/vals
    DevBuf<uint32_t> hist, hscan;  // radix histograms (multi-pass path)
    DevBuf<uint32_t> s0, s1, s2;   // scan block sums (3 levels, multi-pass path)
    // single-pass (decoupled look-back) sort and scan: per-tile look-back words tagged with the
    // launch's epoch (never cleared between launches), the global digit histograms + their
    // bases, and a tile ticket counter that only ever grows (host mirror in `tickets`)
    DevBuf<uint64_t> lb;
    DevBuf<uint32_t> dig;
    DevBuf<unsigned long long> ticket;
    uint64_t tickets = 0;
    uint32_t epoch = 0;
};

// out[0..n) = exclusive prefix sum of in[0..n); out[n] = total. out may alias in.
// One launch (decoupled look-back across 2048-element tiles); n < 2^32.
void scan_exclusive_u32(const uint32_t* in, uint32_t* out, uint64_t n, hipStream_t st, Scratch& ws);

// Stable sort of (keys, vals) by key bits [begin_bit, end_bit) (multiples of 8).
// vals may be null. Result is left in keys/vals. One histogram launch for all digits, then one
// launch per 8-bit digit (ranks within a tile by wave ballots, tile offsets by decoupled
// look-back, writes staged through LDS in digit order).
void radix_sort_pairs(uint32_t* keys, uint32_t* vals, uint64_t n, int begin_bit, int end_bit,
                      hipStream_t st, Scratch& ws);

// Stable sort of the pairs (keys_in[i], i): sorted keys to keys_out, original indices to
// idx_out (keys_in is not modified; no copy of it or iota is made). run_if (device word, may be
// null): the launches do nothing unless *run_if != 0 when they run; only with
// single_pass_sort(n).
void radix_sort_index(const uint32_t* keys_in, uint32_t* keys_out, uint32_t* idx_out, uint64_t n, int begin_bit,
                      int end_bit, hipStream_t st, Scratch& ws, const uint32_t* run_if = nullptr);

// Whether radix sorts of n elements take the single-pass path.
bool single_pass_sort(uint64_t n);

// RP_PRIMS_MULTIPASS=1 selects the earlier multi-launch scan and sort (A/B and cross-checks).
bool prims_multipass();

// out[i] = i for i < n
void iota_u32(uint32_t* out, uint64_t n, hipStream_t st);

// dst[i] = src[idx[i]] for i < n
void gather_u32(const uint32_t* src, const uint32_t* idx, uint32_t* dst, uint64_t n, hipStream_t st);

// Read one uint32 from device memory (synchronizes the stream).
uint32_t read_u32(const uint32_t* p, hipStream_t st);

}  // namespace rp
