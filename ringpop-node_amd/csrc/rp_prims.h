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
    // bases, and a tile ticket counter that is 0 between launches (the launch's last ticket
    // resets it on the device, so no host count can drift from it)
    DevBuf<uint64_t> lb;
    DevBuf<uint32_t> dig;
    DevBuf<unsigned long long> ticket;
    // device error word: kErrSpin (a look-back wait gave up) | kErrTicket (a ticket past the
    // launch's units); read and cleared by scratch_check at the host's next sync point
    DevBuf<uint32_t> err;
    // the wire decoder's record stash and slow-path flags (grow-only: a 640 MB decode keeps
    // ~750 MB here rather than allocating and freeing it per call)
    DevBuf<uint8_t> wire_stash, wire_slow;
    DevBuf<uint32_t> wire_retry;  // messages the decoder's first pass left to its second
    uint32_t epoch = 0;
    // the stream that last used this scratch: a launch on another stream first waits for it
    // (use_on), so two streams never interleave tickets or look-back words
    hipStream_t last_st = nullptr;
    hipEvent_t ev = nullptr;
    bool used = false;
    Scratch() = default;
    Scratch(const Scratch&) = delete;
    Scratch& operator=(const Scratch&) = delete;
    ~Scratch() {
        if (ev) (void)hipEventDestroy(ev);
    }
    // order this scratch's next use on `st` after everything queued on the stream that used it
    // last
    void use_on(hipStream_t st) {
        if (used && st != last_st) {
            if (!ev) RP_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
            RP_HIP(hipEventRecord(ev, last_st));
            RP_HIP(hipStreamWaitEvent(st, ev, 0));
        }
        last_st = st;
        used = true;
    }
};

constexpr uint32_t kErrSpin = 1u, kErrTicket = 2u, kErrRange = 4u;  // kErrRange: a member incarnation past +-2^60 or status > 3

// Throws (RP_EDEVICE) if a single-pass launch on this scratch reported a broken ordering since
// the last check; synchronizes `st`.
void scratch_check(Scratch& ws, hipStream_t st);

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
// null): the launches do nothing unless *run_if != 0 when they run; a gated sort takes the
// single-pass kernels at every size.
void radix_sort_index(const uint32_t* keys_in, uint32_t* keys_out, uint32_t* idx_out, uint64_t n, int begin_bit,
                      int end_bit, hipStream_t st, Scratch& ws, const uint32_t* run_if = nullptr);

// Whether radix sorts of n elements take the single-pass path.
bool single_pass_sort(uint64_t n);

// RP_PRIMS_MULTIPASS=1 selects the earlier multi-launch scan and sort (A/B and cross-checks).
bool prims_multipass();

// ---- decoupled look-back (shared by the single-pass scan / sort and other one-launch
// prefix computations). Units (tiles, messages) take tickets in launch order, so every unit a
// unit waits on is already running; a unit publishes its own count (flag A) at once, sums its
// predecessors' words back to the nearest inclusive prefix (flag P), then publishes its P. A
// word is [epoch:30 | flag:2 | value:32]; agent-scope atomics bypass the per-XCD L2s; words of
// an earlier launch carry another epoch and read as "not ready", so nothing is cleared.
constexpr uint64_t kLbA = 1ull << 32, kLbP = 2ull << 32, kLbFlags = 3ull << 32;
constexpr int kLbEpochShift = 34;
constexpr int kLbWin = 16;  // predecessor words in flight per per-thread look-back step
// A waiting unit gives up after this many polls (seconds) and reports kErrSpin: a broken ordering
// then shows up as an error at the next host sync instead of a hung device.
constexpr uint32_t kLbSpinCap = 1u << 24;

struct LookBack {
    uint64_t* words;  // one per unit
    unsigned long long* ticket;
    uint64_t tag;
    uint32_t* err;
};
// State for one launch over `units` (> 0) units with one word each (uses ws.lb / ws.ticket).
// Every unit of the launch takes exactly one ticket (take_unit), or none of them does (a launch
// gated off as a whole): the last ticket resets the counter for the next launch.
LookBack lookback_prepare(Scratch& ws, uint64_t units, hipStream_t st);

// The calling workgroup's unit: tickets in launch order (so every unit a unit waits on is
// already running). The ticket `units - 1` resets the counter to 0. A ticket past the units
// (only if two launches shared the counter) reports kErrTicket and returns `units`: the caller
// must then return without writing. Syncs the workgroup.
__device__ __forceinline__ uint32_t take_unit(unsigned long long* ctr, uint32_t units, uint32_t* err) {
    __shared__ uint32_t s_unit;
    if (threadIdx.x == 0) {
        const unsigned long long t = atomicAdd(ctr, 1ull);
        if (t == (unsigned long long)units - 1ull)
            __hip_atomic_store(ctr, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (t >= units) atomicOr(err, kErrTicket);
        s_unit = t < units ? (uint32_t)t : units;
    }
    __syncthreads();
    return s_unit;
}

__device__ __forceinline__ uint64_t lb_load(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void lb_store(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool lb_ready(uint64_t v, uint64_t tag) {
    return (v >> kLbEpochShift) == (tag >> kLbEpochShift) && (v & kLbFlags) != 0;
}

// The exclusive prefix of unit `u` over one word per unit, by all 64 lanes of one wave: 64
// predecessor words per step, back to the nearest P.
__device__ __forceinline__ uint32_t lookback_wave(const uint64_t* lb, uint32_t u, uint64_t tag, uint32_t* err) {
    const int lane = threadIdx.x & 63;
    uint32_t excl = 0;
    int64_t t = (int64_t)u - 1 - lane;
    while (u > 0) {
        uint64_t w = t >= 0 ? lb_load(lb + t) : (tag | kLbP);
        uint32_t spin = 0;
        for (; !__all(lb_ready(w, tag)) && spin < kLbSpinCap; spin++) {
            __builtin_amdgcn_s_sleep(1);
            if (!lb_ready(w, tag)) w = lb_load(lb + t);
        }
        if (spin == kLbSpinCap && lane == 0) atomicOr(err, kErrSpin);
        const uint64_t pm = __ballot((w & kLbP) != 0);
        uint32_t x = (uint32_t)w;
        if (pm && lane > __ffsll((long long)pm) - 1) x = 0;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o, 64);
        excl += x;
        if (pm) break;
        t -= 64;
    }
    return excl;
}

// out[i] = i for i < n
void iota_u32(uint32_t* out, uint64_t n, hipStream_t st);

// dst[i] = src[idx[i]] for i < n
void gather_u32(const uint32_t* src, const uint32_t* idx, uint32_t* dst, uint64_t n, hipStream_t st);

// Read one uint32 from device memory (synchronizes the stream).
uint32_t read_u32(const uint32_t* p, hipStream_t st);

}  // namespace rp
