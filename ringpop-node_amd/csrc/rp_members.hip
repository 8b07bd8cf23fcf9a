// rp_members.hip — the membership view on MI355X: batched SWIM merge + membership checksum.
//
// Replaces the hot loop of lib/membership/index.js Membership.update (249-324: a sequential
// fold of Member.evaluateUpdate, member.js:71-202) and computeChecksum /
// generateChecksumString (48-75, 100-123). The fold is order-sensitive only among changes to
// the same address, so the batch is stably sorted by member id (keeping arrival order inside
// each id), and one lane folds each id's segment in arrival order while all segments run in
// parallel. The member table is SoA in HBM (exists u8, status u8, incarnation i64 per id).
// The checksum string is rebuilt on the device in address order (lengths -> scan -> scatter)
// and hashed by the long-chain farmhash kernel; every step is gated on "anything applied" read
// from device memory, so a batch never syncs with the host.
#include <algorithm>
#include <cstring>
#include <cstdlib>
#include <string>
#include <vector>

#include "../../include/ringpop_amd.h"
#include "rp_damp.h"
#include "rp_hashlong.h"
#include "rp_names.h"
#include "rp_swim.h"

namespace rp {

namespace {

// Damp-scoring state by member id (Member.dampScore / lastUpdateDampScore /
// lastUpdateTimestamp, member.js:35-39) and the per-change outputs of the batch being folded.
// score == nullptr: not tracked (rp_members_damp_configure never called).
struct DampArgs {
    damp::Config c;
    double* score;
    double* last;
    int64_t* ts;    // 0 stands for a null lastUpdateTimestamp (JS `now - null` = now)
    double* out;    // per change: the member's dampScore after it
    uint8_t* exc;   // per change: 'suppressLimitExceeded' emitted (member.js:141-152)
};

// One member row in HBM, 8 B since round 5 (16 B before, with the grouped fold's change counter,
// which now has its own array): incarnation << 3 | exists << 2 | status, the incarnation a
// signed 61-bit integer (a JS Number is exact to 2^53, a wire number has at most 18 digits;
// kMemberIncMax bounds what a row can hold and the fold reports anything past it). One dwordx2
// load / store per row; the 2^22 bucket fold moves half the row bytes it did.
struct alignas(8) MRow {
    uint64_t v;
};
static_assert(sizeof(MRow) == 8, "MRow is one 8-byte load");
constexpr int64_t kMemberIncMax = (1ll << 60) - 1, kMemberIncMin = -(1ll << 60);
struct MRowV {  // a row as loaded
    int64_t inc;
    uint8_t status;
    uint8_t exists;
};
__host__ __device__ __forceinline__ MRowV row_unpack(uint64_t v) {
    return MRowV{(int64_t)v >> 3, (uint8_t)(v & 3u), (uint8_t)((v >> 2) & 1u)};
}
__host__ __device__ __forceinline__ uint64_t row_pack(int64_t inc, uint8_t status, uint8_t exists) {
    return ((uint64_t)inc << 3) | ((uint64_t)(exists ? 1u : 0u) << 2) | (uint64_t)(status & 3u);
}
__device__ __forceinline__ MRowV row_load(const MRow* p) { return row_unpack(*reinterpret_cast<const uint64_t*>(p)); }
// err (nullable): kErrRange when the incarnation or the status does not fit the row (the row then
// holds garbage; the call reports RP_EDEVICE at the handle's next sync)
__device__ __forceinline__ void row_store(MRow* p, int64_t inc, uint8_t status, uint8_t exists,
                                          uint32_t* err = nullptr) {
    if (err && (inc > kMemberIncMax || inc < kMemberIncMin || status > 3u)) atomicOr(err, kErrRange);
    *reinterpret_cast<uint64_t*>(p) = row_pack(inc, status, exists);
}

// The batch and table operands of one Membership.update fold.
struct FoldArgs {
    const uint8_t* ch_status;
    const int64_t* ch_inc;
    MRow* rows;
    uint32_t* cnt;  // per member: the grouped fold's change counter (0 between batches) / kOvfMark
    uint32_t* err;  // the handle's device error word (kErrRange)
    uint32_t local_id;
    int64_t now_ms;
    uint8_t* applied;
    uint8_t* new_status;
    int64_t* new_inc;
    uint32_t* n_applied;
    DampArgs da;
};

// The sequential fold of Membership.update restricted to one address (lib/membership/
// index.js:272-304) over its changes in arrival order: change(q) for q < c is the batch index
// of the address's q-th change. applied: 0 = not applied, 1 = applied to an existing member,
// 2 = created a new member. With damp tracking on, an applied update to another member takes
// _applyUpdatePenalty (member.js:98-107, 133-153) and every applied update stamps
// lastUpdateTimestamp (:115-118). `row` is the member's row as loaded; it is written back once
// with its change counter set to cnt_after (cleared, except by the overflow fold).
// Returns the number of changes applied (the caller sums them per wave: one atomic per wave,
// not per address, on the batch's applied counter).
template <class Change>
__device__ __forceinline__ uint32_t fold_address(const FoldArgs& A, uint32_t id, MRowV row, uint32_t c, Change change,
                                                 uint32_t cnt_after = 0) {
    const DampArgs& da = A.da;
    bool ex = row.exists != 0;
    uint8_t st = row.status;
    int64_t in = row.inc;
    double sc = 0.0, ls = 0.0;
    int64_t lt = 0;
    if (da.score) {
        sc = da.score[id];
        ls = da.last[id];
        lt = da.ts[id];
    }
    uint32_t napp = 0;
    for (uint32_t q = 0; q < c; q++) {
        const uint32_t j = change(q);
        uint8_t us = A.ch_status[j];
        int64_t ui = A.ch_inc[j];
        if (us > 3u && A.err) atomicOr(A.err, kErrRange);  // a status past leave (no rule takes it)
        uint8_t a;
        bool exc = false;
        if (!ex) {  // _createMember verbatim (index.js:277-291): a fresh Member (member.js:28-41)
            ex = true;
            a = 2;
            sc = ls = da.c.initial;
            lt = 0;
        } else {
            a = evaluate_update(st, in, id == A.local_id, us, ui, A.now_ms) ? 1 : 0;
        }
        if (a) {
            st = us;
            in = ui;
            napp++;
        }
        if (a == 1 && da.score) {
            if (da.c.enabled && id != A.local_id) {
                sc = damp::penalized(da.c, ls, lt, A.now_ms, &exc);
                ls = sc;
            }
            lt = A.now_ms;
        }
        if (A.applied) A.applied[j] = a;
        if (A.new_status) A.new_status[j] = us;
        if (A.new_inc) A.new_inc[j] = ui;
        if (da.out) {
            da.out[j] = sc;
            da.exc[j] = exc ? 1 : 0;
        }
    }
    row_store(A.rows + id, in, st, ex ? 1 : 0, A.err);
    A.cnt[id] = cnt_after;
    if (da.score) {
        da.score[id] = sc;
        da.last[id] = ls;
        da.ts[id] = lt;
    }
    return napp;
}

// The sum of every thread's v over the workgroup (256 threads), valid in thread 0; called by
// all threads. (One atomic per wave on a single counter serialises: MI355X retires about 88
// same-address atomics per µs, so 1,563 waves of a C3 batch cost 18 µs and 65,536 waves of a
// 2^22 batch 0.75 ms. The fold kernels reduce per workgroup instead.)
__device__ __forceinline__ uint32_t block_sum256(uint32_t v) {
    __shared__ uint32_t s_w[4];
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = v;
    __syncthreads();
    return s_w[0] + s_w[1] + s_w[2] + s_w[3];
}

// The last workgroup of a launch to get here (done: a counter that is 0 before the launch and is
// left 0 after it) publishes the batch's applied count to *out and, when reset is non-null,
// clears *reset (the gate word this launch ran under). Called by every thread of every
// workgroup after its atomics. Every workgroup pays an agent-scope release fence here (an L2
// write-back on gfx950), so only the rare sorted fold uses it; the grouped path hands the
// count on through the next launch instead (k_fold gated off).
__device__ __forceinline__ void last_block_publish(uint32_t* done, const uint32_t* napplied, uint32_t* out,
                                                   uint32_t* reset) {
    __shared__ bool s_last;
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) s_last = atomicAdd(done, 1u) == gridDim.x - 1;
    __syncthreads();
    if (!s_last || threadIdx.x != 0) return;
    __threadfence();
    if (out) *out = __hip_atomic_load(napplied, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (reset) __hip_atomic_store(reset, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Sorted path: one lane per id segment of the (id, arrival)-sorted batch. run_if (may be null):
// skip unless *run_if != 0; the last workgroup then clears *run_if. done / out: see
// last_block_publish (out may be null). Every id of the batch gets its row written (counter
// cleared), so a grouped attempt that overflowed leaves no counts behind. Gated off, the
// grouped fold ran before it in the stream: workgroup 0 sums that fold's per-workgroup applied
// counts (part[0..nparts)) into *A.n_applied (the checksum gate) and *out.
__global__ __launch_bounds__(256) void k_fold(const uint32_t* __restrict__ sk, const uint32_t* __restrict__ sv,
                                              uint32_t k, FoldArgs A, uint32_t* __restrict__ run_if,
                                              uint32_t* __restrict__ done, uint32_t* __restrict__ out,
                                              const uint32_t* __restrict__ part, uint32_t nparts) {
    if (run_if && *run_if == 0) {
        if (blockIdx.x != 0) return;
        uint32_t v = 0;
        for (uint32_t b = threadIdx.x; b < nparts; b += 256) v += part[b];
        v = block_sum256(v);
        if (threadIdx.x == 0) {
            *A.n_applied = v;
            if (out) *out = v;
        }
        return;
    }
    const uint32_t gstride = gridDim.x * blockDim.x;
    uint32_t napp = 0;
    for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < k; p += gstride) {
        const uint32_t id = sk[p];
        if (p > 0 && sk[p - 1] == id) continue;  // not a segment head
        uint32_t c = 1;
        while (p + c < k && sk[p + c] == id) c++;
        napp += fold_address(A, id, row_load(A.rows + id), c, [&](uint32_t q) { return sv[p + q]; });
    }
    napp = block_sum256(napp);
    if (threadIdx.x == 0 && napp) atomicAdd(A.n_applied, napp);
    last_block_publish(done, A.n_applied, out, run_if);
}

// Grouped path (no sort, round 3): two launches per batch.
//   k_link: every change takes its rank among its address's changes from an atomic on the
//   address's row counter (arbitrary order), keeps it (rk), and a change of rank 1..kSlots
//   writes its batch index into the address's inline slot array. Rank kSlots + 1 (an address
//   with more than kSlots + 1 changes) sets *ovf.
//   k_fold_fast: the rank-0 change of every address loads the row (count included) and, for a
//   repeated address, its slots (contiguous, no dependent list walk), puts the indices in
//   arrival order in registers and folds them. An address with more changes is marked
//   (counter = kOvfMark) and left to k_fold_ovf, one gated launch after it.
// Each address costs one atomic on its counter, one 8-B row load and one 8-B row store (and its
// counter reset); the batch's applied counter is cleared by k_link, so the batch needs no memset.
constexpr uint32_t kSlots = 15;  // changes per address on the grouped path: kSlots + 1
constexpr uint32_t kOvfMark = 0xFFFFFFFFu;  // row counter of an address left to k_fold_ovf
constexpr uint32_t kDoneWords = 4;  // [0] k_link_fold barrier count, [1] k_fold, [2] k_ovf_len's ticket, [3] barrier generation

__device__ __forceinline__ void link_one(uint32_t i, const uint32_t* __restrict__ ids, uint32_t k,
                                         uint32_t* __restrict__ cnt, uint32_t* __restrict__ slots,
                                         uint8_t* __restrict__ rk, uint32_t* __restrict__ ovf,
                                         uint32_t* __restrict__ napplied) {
    if (i == 0) *napplied = 0;
    if (i >= k) return;
    const uint32_t id = ids[i];
    const uint32_t r = atomicAdd(&cnt[id], 1u);
    rk[i] = r < 255u ? (uint8_t)r : (uint8_t)255;
    if (r >= 1u && r <= kSlots) slots[(uint64_t)id * kSlots + (r - 1u)] = i;
    if (r == kSlots + 1u) *ovf = 1u;
}

__global__ void k_link(const uint32_t* __restrict__ ids, uint32_t k, uint32_t* __restrict__ cnt,
                       uint32_t* __restrict__ slots, uint8_t* __restrict__ rk, uint32_t* __restrict__ ovf,
                       uint32_t* __restrict__ napplied) {
    link_one(blockIdx.x * blockDim.x + threadIdx.x, ids, k, cnt, slots, rk, ovf, napplied);
}

// The workgroup's applied count goes to part[blockIdx.x] (summed by k_ovf_len or k_fold_ovf).
__device__ __forceinline__ void fold_fast_block(const uint32_t* __restrict__ ids, uint32_t k,
                                                const uint8_t* __restrict__ rk, const uint32_t* __restrict__ slots,
                                                const FoldArgs& A, uint32_t* __restrict__ part, uint32_t blk,
                                                uint32_t nblk) {
    const uint32_t i = blk * blockDim.x + threadIdx.x;
    uint32_t napp = 0;
    if (i < k && rk[i] == 0) {
        const uint32_t id = ids[i];
        const MRowV row = row_load(A.rows + id);
        const uint32_t c = A.cnt[id];
        if (c > kSlots + 1) {  // more changes than slots: marked for k_fold_ovf
            A.cnt[id] = kOvfMark;
        } else if (c <= 1) {
            napp = fold_address(A, id, row, 1, [&](uint32_t) { return i; });
        } else {
            uint32_t idx[kSlots + 1];
            idx[0] = i;
            const uint32_t* sl = slots + (uint64_t)id * kSlots;
            for (uint32_t q = 1; q < c; q++) {
                const uint32_t x = sl[q - 1];
                uint32_t r = q;
                while (r > 0 && idx[r - 1] > x) {
                    idx[r] = idx[r - 1];
                    r--;
                }
                idx[r] = x;
            }
            napp = fold_address(A, id, row, c, [&](uint32_t q) { return idx[q]; });
        }
    }
    napp = block_sum256(napp);
    if (threadIdx.x == 0) part[blk] = napp;
    if (threadIdx.x == 0 && blk == 0) part[nblk] = 0;  // the overflow fold's count (k_ovf_len)
}

__global__ __launch_bounds__(256) void k_fold_fast(const uint32_t* __restrict__ ids, uint32_t k,
                                                   const uint8_t* __restrict__ rk, const uint32_t* __restrict__ slots,
                                                   FoldArgs A, uint32_t* __restrict__ part) {
    fold_fast_block(ids, k, rk, slots, A, part, blockIdx.x, gridDim.x);
}

// Every workgroup of the launch waits here until all have arrived (count / generation words,
// zero between launches; the last to arrive resets the count and bumps the generation). Only
// for grids that are resident at once (the caller checks the occupancy); a wait that outlasts
// kLbSpinCap polls gives up and reports kErrSpin, so no launch can hang.
__device__ __forceinline__ void grid_sync(uint32_t* cnt, uint32_t* gen, uint32_t* err) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // this thread's writes, before the arrival
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t g = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t arrived = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) + 1u;
        if (arrived == gridDim.x) {
            __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(gen, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            uint32_t spin = 0;
            while (__hip_atomic_load(gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == g) {
                if (++spin == kLbSpinCap) {
                    atomicOr(err, kErrSpin);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
    }
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
}

// k_link and k_fold_fast in one launch, a grid barrier between them (round 4): one launch fewer
// per batch on the grouped path (C3).
__global__ __launch_bounds__(256) void k_link_fold(const uint32_t* __restrict__ ids, uint32_t k,
                                                   uint32_t* __restrict__ slots, uint8_t* __restrict__ rk,
                                                   uint32_t* __restrict__ ovf, uint32_t* __restrict__ napplied,
                                                   FoldArgs A, uint32_t* __restrict__ part, uint32_t* __restrict__ err) {
    link_one(blockIdx.x * blockDim.x + threadIdx.x, ids, k, A.cnt, slots, rk, ovf, napplied);
    grid_sync(napplied + 2, napplied + 5, err);
    fold_fast_block(ids, k, rk, slots, A, part, blockIdx.x, gridDim.x);
}

// The grouped path's overflow fold: the addresses k_fold_fast marked (more than kSlots + 1
// changes in the batch), folded by one workgroup of NT threads over the batch in NT-change
// chunks in arrival order: a chunk's marked changes are compacted, sorted by (address,
// arrival) in LDS and folded one lane per address segment, the rows keeping the mark until the
// last chunk; then the marks are cleared. An address's changes are applied in arrival order, as
// the sequential fold does. Returns this thread's applied count.
template <int NT>
__device__ uint32_t ovf_fold(const uint32_t* __restrict__ ids, uint32_t k, const FoldArgs& A) {
    __shared__ uint64_t s_key[NT];
    __shared__ uint32_t s_cnt[NT / 64];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    uint32_t napp = 0;
    for (uint32_t c0 = 0; c0 < k; c0 += NT) {
        const uint32_t i = c0 + tid;
        uint32_t id = 0;
        bool f = false;
        if (i < k) {
            id = ids[i];
            f = __hip_atomic_load(&A.cnt[id], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == kOvfMark;
        }
        const uint64_t bal = __ballot(f);
        if (lane == 0) s_cnt[wv] = (uint32_t)__popcll(bal);
        __syncthreads();
        uint32_t base = 0, m = 0;
        for (uint32_t w = 0; w < NT / 64; w++) {
            base += w < wv ? s_cnt[w] : 0u;
            m += s_cnt[w];
        }
        if (m == 0) {  // uniform
            __syncthreads();
            continue;
        }
        const uint32_t pos = base + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull));
        if (f) s_key[pos] = ((uint64_t)id << 32) | i;
        uint32_t np = 1;
        while (np < m) np <<= 1;
        if (tid >= m && tid < np) s_key[tid] = ~0ull;
        __syncthreads();
        for (uint32_t k2 = 2; k2 <= np; k2 <<= 1)
            for (uint32_t j = k2 >> 1; j > 0; j >>= 1) {
                const uint32_t x = tid ^ j;
                if (tid < np && x > tid) {
                    const uint64_t a = s_key[tid], b = s_key[x];
                    if ((a > b) == ((tid & k2) == 0)) {
                        s_key[tid] = b;
                        s_key[x] = a;
                    }
                }
                __syncthreads();
            }
        if (tid < m) {
            const uint32_t sid = (uint32_t)(s_key[tid] >> 32);
            if (tid == 0 || (uint32_t)(s_key[tid - 1] >> 32) != sid) {
                uint32_t c = 1;
                while (tid + c < m && (uint32_t)(s_key[tid + c] >> 32) == sid) c++;
                napp += fold_address(A, sid, row_load(A.rows + sid), c,
                                     [&](uint32_t q) { return (uint32_t)s_key[tid + q]; }, kOvfMark);
            }
        }
        __syncthreads();
    }
    for (uint32_t i = tid; i < k; i += NT) {
        const uint32_t id = ids[i];
        if (A.cnt[id] == kOvfMark) A.cnt[id] = 0;
    }
    return napp;
}

// The grouped path's third launch when the batch's checksum string is not built (deferred, or
// another replica's batch): gated off (*ovf == 0, the normal case) it only sums the fold's
// per-workgroup applied counts into *A.n_applied (the checksum gate) and *out; gated on, it
// runs the overflow fold first and resets *ovf.
__global__ __launch_bounds__(1024) void k_fold_ovf(const uint32_t* __restrict__ ids, uint32_t k,
                                                   uint32_t* __restrict__ ovf, FoldArgs A,
                                                   const uint32_t* __restrict__ part, uint32_t nparts,
                                                   uint32_t* __restrict__ out) {
    __shared__ uint32_t s_on, s_w[16];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    uint32_t v = 0;  // the counts are loaded beside the gate word (the overflow fold leaves part alone)
    for (uint32_t b = tid; b < nparts; b += 1024) v += part[b];
    if (tid == 0) s_on = *ovf;
    __syncthreads();
    if (s_on) v += ovf_fold<1024>(ids, k, A);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) s_w[wv] = v;
    __syncthreads();
    if (tid == 0) {
        uint32_t t = 0;
        for (int w = 0; w < 16; w++) t += s_w[w];
        *A.n_applied = t;
        if (out) *out = t;
        if (s_on) *ovf = 0;
    }
}

// Bucket path (large batches, round 3): the batch is partitioned by id into buckets of kBk ids
// (a stable-per-id order is not needed: an address's changes are put back in arrival order by
// their batch index), then one workgroup folds one bucket with the bucket's 32 KB of rows
// resident in its XCD's L2, so the row accesses and the rank counters stop being random HBM /
// memory-side atomics (k_link's one atomic per change was half of a 2^22 batch). Two launches
// and the gated overflow fold:
//   k_bk_scatter a 4,096-change tile sorts its records (8 B with a tile incarnation base, else
//                12 B: {bucket-local id, tile-relative index, status; incarnation}) by bucket in
//                LDS and stores them as one contiguous run at recs + tile * kBkTile (whole
//                lines); seg[bucket][tile] = the bucket's segment of that run (start << 16 |
//                length). No global count pass or scan: the fold walks a bucket's segments of
//                every tile.
//   k_bk_fold    a workgroup per bucket: reads the bucket's segments once, in order, keeping
//                per id the first change (batch index, status, incarnation) in LDS and flagging
//                repeated ids; then the bucket's ids in id order (rows as whole lines): a single
//                change folds from LDS, an address's repeated changes are sorted by batch index
//                in LDS and folded by one lane; a bucket whose repeated changes overflow the LDS
//                list marks them for the overflow fold (k_fold_ovf / k_ovf_len, as on the grouped
//                path). Applied flags go straight to applied[batch index] (DIRECT), or (A/B) to a
//                2-bit per-id map res2 / resj[batch index] that
//   k_bk_gather  turns back into batch order, from res2[ids[j]] (1 MB, L2-resident), four
//                changes per lane. The new status / incarnation outputs are copied from the
//                input by k_bk_scatter (unless they alias it); the fold rewrites local overrides.
#ifndef RP_BK_BITS
#define RP_BK_BITS 12
#endif
#ifndef RP_BK_FT
#define RP_BK_FT 512
#endif
constexpr uint32_t kBkBits = RP_BK_BITS, kBk = 1u << kBkBits;  // ids per bucket (4,096: 64 KB of rows)
#ifndef RP_BK_TILE
#define RP_BK_TILE 4096
#endif
constexpr uint32_t kBkTile = RP_BK_TILE;                       // changes per scatter tile
constexpr uint32_t kBkST = 1024;                               // threads per scatter tile
constexpr uint32_t kBkFT = RP_BK_FT;                           // threads per fold workgroup
#ifndef RP_BK_DUP
#define RP_BK_DUP 256
#endif
constexpr uint32_t kBkDup = RP_BK_DUP;  // repeated-address changes a bucket sorts in LDS (1 % repeats: ~80)
static_assert(kBkDup <= kBkFT && kBkDup <= 1024, "k_bk_fold: one repeated change per thread, 10-bit entry in the key");
static_assert(kBk % kBkFT == 0 && kBkFT % 64 == 0, "k_bk_fold: whole ids per lane");
constexpr uint32_t kBkMaxBuckets = 2048;               // (LDS of the scatter tiles): 8M ids
constexpr uint8_t kResLocal = 4;                       // result: the local override rewrote (status, inc)
constexpr uint8_t kResRep = 8;                         // repeated changes, results in resj
static_assert(RP_BK_BITS + (RP_BK_TILE > 4096 ? 13 : 12) <= 30, "bucket-local id + tile-relative index + status in 32 bits");
static_assert(RP_BK_TILE == 4096 || RP_BK_TILE == 8192, "scatter tiles of 4,096 or 8,192 changes");
// the per-id result the gather reads, 2 bits (16 ids per word): 0 / 1 / 2 = applied, 3 = repeated
// changes (the results are in resj)
constexpr uint32_t kRes2Rep = 3;

// seg layout: groups of 16 buckets, then tile, then bucket (one 64-B line per (group, tile)), so
// a scatter tile writes whole lines and the 16 buckets that share a line fold on one XCD
__host__ __device__ __forceinline__ uint64_t seg_at(uint32_t b, uint32_t t, uint32_t ntiles) {
    return ((uint64_t)(b >> 4) * ntiles + t) * 16 + (b & 15u);
}

// A staged change in the wide form, 12 B: {bucket-local id | tile-relative batch index << kBkBits |
// status << 30, incarnation lo, hi} (the compact form keeps x and the incarnation - tile base). The tile is the run it sits in (the fold knows it from the segment), so
// the batch index is tile * kBkTile + the relative index: no 16-B record with a full id and index.
struct BRec {
    uint32_t x;
    uint32_t lo, hi;
};
static_assert(sizeof(BRec) == 12, "12-byte records");
constexpr uint32_t kBkRelBits = kBkTile > 4096 ? 13 : 12;
static_assert((1u << kBkRelBits) >= kBkTile, "tile-relative batch index");
__device__ __forceinline__ uint32_t brec_x(uint32_t il, uint32_t rel, uint32_t st) {
    return il | (rel << kBkBits) | (st << 30);
}

// Compact records (round 5): a tile whose incarnations span less than 2^32 (ms timestamps of one
// batch always do) stores 8-B records {x, incarnation - tile base} and its base in tb[tile];
// otherwise 12-B records and tb[tile] = kBkWide. The fold reads a tile's base beside its segment.
constexpr int64_t kBkWide = INT64_MIN;
constexpr uint32_t kBkNone = 0xFFFFFFFFu, kBkRep = 1u << 29;  // k_bk_fold's fjs: no change / repeated
__device__ __forceinline__ void bk_minmax(int64_t& mn, int64_t& mx) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const int64_t a = __shfl_xor(mn, o, 64), b = __shfl_xor(mx, o, 64);
        mn = a < mn ? a : mn;
        mx = b > mx ? b : mx;
    }
}

template <bool LOOP>
__global__ __launch_bounds__(kBkST) void k_bk_scatter(const uint32_t* __restrict__ ids, const uint8_t* __restrict__ chs,
                                                    const int64_t* __restrict__ chi, uint32_t k, uint32_t nb,
                                                    uint32_t ntiles, BRec* __restrict__ recs,
                                                    uint32_t* __restrict__ seg, int64_t* __restrict__ tb,
                                                    uint8_t* __restrict__ nst, int64_t* __restrict__ ninc,
                                                    uint32_t* __restrict__ err, uint32_t b_lo, uint32_t b_hi) {
    __shared__ __attribute__((aligned(16))) uint32_t stage[kBkTile * 3];
    __shared__ uint32_t h[kBkMaxBuckets], s_w[kBkST / 64];
    __shared__ int64_t s_mn[kBkST / 64], s_mx[kBkST / 64];
    __shared__ uint16_t ls[kBkMaxBuckets];  // <= 4,096 (60 KB in all: two tiles per CU)
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    constexpr uint32_t PER = kBkTile / kBkST;
    uint32_t rk[PER], idv[PER];
    uint8_t stv[PER];
    int64_t incv[PER];
    auto load = [&](uint32_t tt) {  // every load of a tile in flight at once
        const uint32_t bs = tt * kBkTile, nn = k - bs < kBkTile ? k - bs : kBkTile;
#pragma unroll
        for (uint32_t q = 0; q < PER; q++) {
            const uint32_t i = tid + q * kBkST;
            idv[q] = i < nn ? ids[bs + i] : 0u;
            stv[q] = i < nn ? chs[bs + i] : (uint8_t)0;
            incv[q] = i < nn ? chi[bs + i] : 0;
        }
    };
    // the outputs start as copies; the fold rewrites local overrides. Outputs that alias the
    // inputs (the reference rewrites its update objects in place) need no copy.
    const bool cst = nst && nst != chs, cinc = ninc && ninc != chi;
    // LOOP (A/B, RP_BK_SGRID): a workgroup takes tiles blockIdx.x, + gridDim.x, ...: the next
    // tile's inputs are loaded while this tile's records are stored. The default grid covers every
    // tile once and is compiled without that loop: the prefetched inputs cost 36 VGPRs (94 against
    // 58), which left one 1,024-thread tile a CU instead of two (2^22 fold 0.089 -> 0.077 ms, r05an)
    uint32_t t = blockIdx.x;
    if (t < ntiles) load(t);
    for (; t < ntiles; t = LOOP ? t + gridDim.x : ntiles) {
        const uint32_t base = t * kBkTile;
        const uint32_t n = k - base < kBkTile ? k - base : kBkTile;
        for (uint32_t b = tid; b < nb; b += kBkST) h[b] = 0;
        __syncthreads();
        bool bad = false;  // a status past leave: the record keeps 2 bits (row_store's kErrRange)
#pragma unroll
        for (uint32_t q = 0; q < PER; q++) {
            const uint32_t i = tid + q * kBkST;
            if (i < n) {
                const uint32_t bq = idv[q] >> kBkBits;
                if (bq >= b_lo && bq < b_hi) {  // (a range update: only its own buckets' outputs)
                    if (cst) nst[base + i] = stv[q];
                    if (cinc) ninc[base + i] = incv[q];
                }
                bad |= stv[q] > 3u;
            }
        }
        if (bad) atomicOr(err, kErrRange);
        int64_t mn = INT64_MAX, mx = INT64_MIN;
#pragma unroll
        for (uint32_t q = 0; q < PER; q++)
            if (tid + q * kBkST < n) {
                mn = incv[q] < mn ? incv[q] : mn;
                mx = incv[q] > mx ? incv[q] : mx;
            }
        bk_minmax(mn, mx);
        if (lane == 0) {
            s_mn[wv] = mn;
            s_mx[wv] = mx;
        }
#pragma unroll
        for (uint32_t q = 0; q < PER; q++) rk[q] = tid + q * kBkST < n ? atomicAdd(&h[idv[q] >> kBkBits], 1u) : 0u;
        __syncthreads();
        for (uint32_t w = 0; w < kBkST / 64; w++) {
            mn = s_mn[w] < mn ? s_mn[w] : mn;
            mx = s_mx[w] > mx ? s_mx[w] : mx;
        }
        const bool c8 = tb != nullptr && mn != kBkWide && (uint64_t)(mx - mn) <= 0xFFFFFFFFull;  // block-uniform
        if (tid == 0 && tb) tb[t] = c8 ? mn : kBkWide;
        // exclusive scan of h over the buckets (contiguous runs per thread, then across threads)
        const uint32_t per = (nb + kBkST - 1) / kBkST, b0 = min(nb, tid * per), b1 = min(nb, b0 + per);
        uint32_t run = 0;
        for (uint32_t b = b0; b < b1; b++) run += h[b];
        uint32_t inc = run;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t x = __shfl_up(inc, o, 64);
            if (lane >= (uint32_t)o) inc += x;
        }
        if (lane == 63) s_w[wv] = inc;
        __syncthreads();
        uint32_t ex = inc - run;
        for (uint32_t w = 0; w < wv; w++) ex += s_w[w];
        for (uint32_t b = b0; b < b1; b++) {
            ls[b] = ex;
            seg[seg_at(b, t, ntiles)] = (ex << 16) | h[b];  // start <= 4,096, length <= 4,096
            ex += h[b];
        }
        __syncthreads();
        const uint32_t rw = c8 ? 2u : 3u;  // record words
#pragma unroll
        for (uint32_t q = 0; q < PER; q++) {
            const uint32_t i = tid + q * kBkST;
            if (i < n) {
                const uint32_t b = idv[q] >> kBkBits, e = rw * (ls[b] + rk[q]);
                const int64_t inc8 = incv[q];
                stage[e] = brec_x(idv[q] & (kBk - 1u), i, stv[q] & 3u);
                if (c8) {
                    stage[e + 1] = (uint32_t)(uint64_t)(inc8 - mn);
                } else {
                    stage[e + 1] = (uint32_t)(uint64_t)inc8;
                    stage[e + 2] = (uint32_t)((uint64_t)inc8 >> 32);
                }
            }
        }
        if (LOOP && t + gridDim.x < ntiles) load(t + gridDim.x);  // in flight under the stores below
        __syncthreads();
        // the tile's run: n records of 8 or 12 B at recs + tile * kBkTile (16-B stores; the tile's
        // run starts 16-B aligned, and its padded tail is never read). A range update stores only
        // the part of the run its buckets [b_lo, b_hi) hold (records sorted by bucket: one stretch)
        uint4* d4 = reinterpret_cast<uint4*>(recs + (uint64_t)t * kBkTile);
        const uint4* s4 = reinterpret_cast<const uint4*>(stage);
        const uint32_t r0 = b_lo < nb ? ls[b_lo] : n, r1 = b_hi < nb ? ls[b_hi] : n;
        for (uint32_t q = (rw * r0) / 4u + tid; q < (rw * r1 + 3u) / 4u; q += kBkST) d4[q] = s4[q];
    }
}

// One change on a member row (the step of fold_address without damp scoring): returns applied
// (0, 1 existing, 2 created) | kResLocal when the local override rewrote the change.
__device__ __forceinline__ uint8_t bk_step(const FoldArgs& A, uint32_t id, bool& ex, uint8_t& st, int64_t& in,
                                          uint8_t us, int64_t ui) {
    uint8_t a, loc = 0;
    if (!ex) {
        ex = true;
        a = 2;
    } else {
        const uint8_t us0 = us;
        const int64_t ui0 = ui;
        a = evaluate_update(st, in, id == A.local_id, us, ui, A.now_ms) ? 1 : 0;
        loc = (us != us0 || ui != ui0) ? kResLocal : 0;
    }
    if (a) {
        st = us;
        in = ui;
    }
    return a | loc;
}

// A change about the local member that the override rewrote (suspect / faulty: alive at now):
// its outputs, copied from the input by k_bk_scatter
__device__ __forceinline__ void bk_local(const FoldArgs& A, uint32_t j) {
    if (A.new_status) A.new_status[j] = ST_ALIVE;
    if (A.new_inc) A.new_inc[j] = A.now_ms;
}

// A workgroup per bucket (52 KB of LDS since round 5: three per CU): per id the first change
// (an LDS CAS; a later change flags the id as repeated), read from the bucket's segments in
// record order; then the bucket's ids in id order, so the rows move as whole lines: a single
// change folds at once, repeated changes go to the sorted LDS list (one lane per address, in
// batch order), a bucket whose repeated changes overflow the list to the overflow fold.
// DIRECT (round 5): each change's applied flag is stored straight to applied[batch index] (a
// scattered byte; the batch index is in the record, fjs / the repeated list) and k_bk_gather with
// its 2-bit map does not run. A/B: RP_BK_DIRECT=0 keeps the map and the gather.
// Phase cycle counters of k_bk_fold (diagnostics only: -DRP_BK_PROF; the product build has none):
// thread 0 of every workgroup stamps s_memtime after each phase's barrier; the sums over the
// workgroups land in g_bk_prof (printed by the launcher under RP_BK_PROF_PRINT).
#ifdef RP_BK_PROF
__device__ unsigned long long g_bk_prof[8];
__device__ unsigned long long g_bk_wg[2 * kBkMaxBuckets];  // per bucket: start, end (s_memrealtime, 100 MHz)
#define BK_T(var)   \
    uint64_t var;   \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(var))
#else
#define BK_T(var)
#endif
template <bool DIRECT>
__global__ __launch_bounds__(kBkFT) void k_bk_fold(const BRec* __restrict__ recs, const uint32_t* __restrict__ seg,
                                                  const int64_t* __restrict__ tb, uint32_t ntiles, uint32_t nb,
                                                  uint32_t b_lo, uint32_t b_hi, FoldArgs A,
                                                  uint32_t* __restrict__ res2, uint8_t* __restrict__ resj,
                                                  uint32_t* __restrict__ ovf, uint32_t* __restrict__ part) {
    // fjs: per id the first change's {batch index | status << 30} (kBkNone: none; kBkRep set when
    // the address has repeated changes; a batch index is below 2^29), first by an LDS CAS
    __shared__ uint32_t fjs[kBk];
    __shared__ uint8_t rcode[DIRECT ? 16 : kBk];  // (map path) 2-bit result codes, packed 16 to a word
    __shared__ int64_t finc[kBk];
    // repeated changes: key (address << 40 | batch index << 10 | entry), the entry's status and
    // incarnation beside it, so the per-address fold reads only LDS
    __shared__ uint64_t dk[kBkDup];
    __shared__ int64_t dinc[kBkDup];
    __shared__ uint8_t dst[kBkDup];
    __shared__ uint32_t s_nd, s_w[kBkFT / 64];
    // XCD-aware: blocks are dealt round-robin over the 8 XCDs, so block i's XCD folds the
    // contiguous bucket range (i % 8) * per ...: neighbouring buckets, whose segments share record
    // lines in every tile run, fold at the same time in one L2
    // (a range update folds buckets [b_lo, b_hi) only; the whole table: 0, nb)
    const uint32_t per = (b_hi - b_lo + 7) / 8, b = b_lo + (blockIdx.x & 7u) * per + (blockIdx.x >> 3);
    if (b >= b_hi) return;
    const uint32_t tid = threadIdx.x, id0 = b << kBkBits;
#ifdef RP_BK_PROF
    if (tid == 0) g_bk_wg[2 * b] = __builtin_amdgcn_s_memrealtime();
#endif
    auto dput = [&](uint32_t d, uint32_t il, uint32_t js, int64_t in) {
        dk[d] = ((uint64_t)il << 40) | ((uint64_t)(js & 0x3FFFFFFFu) << 10) | d;
        dst[d] = (uint8_t)(js >> 30);
        dinc[d] = in;
    };
    for (uint32_t q = tid; q < kBk; q += kBkFT) fjs[q] = kBkNone;
    if (tid == 0) s_nd = 0;
    __syncthreads();
    BK_T(t0);
    // a lane per tile segment, up to 8 records in flight; a change that finds its address
    // already counted goes straight to the repeated list (the first change is added below)
    auto take = [&](uint32_t x, uint32_t jt, int64_t in) {
        const uint32_t il = x & (kBk - 1u);
        const uint32_t js = (jt + ((x >> kBkBits) & (kBkTile - 1u))) | (x & 0xC0000000u);
        const uint32_t old = atomicCAS(&fjs[il], kBkNone, js);
        if (old == kBkNone) {
            finc[il] = in;
        } else {
            if (!(old & kBkRep)) atomicOr(&fjs[il], kBkRep);
            const uint32_t d = atomicAdd(&s_nd, 1u);
            if (d < kBkDup) dput(d, il, js, in);
        }
    };
    for (uint32_t t = tid; t < ntiles; t += kBkFT) {
        const uint32_t e = seg[seg_at(b, t, ntiles)], n = e & 0xFFFFu;
        const int64_t base = tb ? tb[t] : kBkWide;
        const uint32_t jt = t * kBkTile;  // the tile's first batch index
        if (base != kBkWide) {  // 8-B records
            const uint2* r = reinterpret_cast<const uint2*>(recs + (uint64_t)t * kBkTile) + (e >> 16);
            for (uint32_t i0 = 0; i0 < n; i0 += 8) {
                uint2 v[8];
#pragma unroll
                for (uint32_t q = 0; q < 8; q++) v[q] = i0 + q < n ? r[i0 + q] : uint2{0, 0};
#pragma unroll
                for (uint32_t q = 0; q < 8; q++)
                    if (i0 + q < n) take(v[q].x, jt, base + (int64_t)v[q].y);
            }
        } else {
            const BRec* r = recs + (uint64_t)t * kBkTile + (e >> 16);
            for (uint32_t i0 = 0; i0 < n; i0 += 8) {
                BRec v[8];
#pragma unroll
                for (uint32_t q = 0; q < 8; q++) v[q] = i0 + q < n ? r[i0 + q] : BRec{0, 0, 0};
#pragma unroll
                for (uint32_t q = 0; q < 8; q++)
                    if (i0 + q < n) take(v[q].x, jt, (int64_t)(((uint64_t)v[q].hi << 32) | v[q].lo));
            }
        }
    }
    __syncthreads();
    BK_T(t1);
    // + the first change of every repeated address
    for (uint32_t q = tid; q < kBk; q += kBkFT) {
        const uint32_t v = fjs[q];
        if (v != kBkNone && (v & kBkRep)) {
            const uint32_t d = atomicAdd(&s_nd, 1u);
            if (d < kBkDup) dput(d, q, v & ~kBkRep, finc[q]);
        }
    }
    __syncthreads();
    BK_T(t2);
    const uint32_t nd = s_nd;
    const bool listed = nd <= kBkDup;  // block-uniform
    uint32_t napp = 0;
    constexpr uint32_t PI = kBk / kBkFT;  // ids per lane
    uint64_t wv4[PI];
#pragma unroll
    for (uint32_t u = 0; u < PI; u++) {  // each lane's rows in flight together
        const uint32_t q = tid + u * kBkFT, v = fjs[q];
        if (v != kBkNone) wv4[u] = *reinterpret_cast<const uint64_t*>(A.rows + id0 + q);
    }
#pragma unroll
    for (uint32_t u = 0; u < PI; u++) {  // ids in order: coalesced rows and results
        const uint32_t q = tid + u * kBkFT;
        const uint32_t v = fjs[q], id = id0 + q;
        uint8_t r = 0;
        if (v != kBkNone && !(v & kBkRep)) {
            const MRowV rw = row_unpack(wv4[u]);
            bool ex = rw.exists != 0;
            uint8_t st = rw.status;
            int64_t in = rw.inc;
            r = bk_step(A, id, ex, st, in, (uint8_t)(v >> 30), finc[q]);
            row_store(A.rows + id, in, st, 1, A.err);
            if (DIRECT && A.applied) A.applied[v & 0x1FFFFFFFu] = r & 3u;
            if (r & kResLocal) bk_local(A, v & 0x1FFFFFFFu);
            napp += (r & 3u) ? 1u : 0u;
        } else if (v != kBkNone) {
            r = kResRep;
            if (!listed) {  // the overflow fold takes the address
                A.cnt[id] = kOvfMark;
                *ovf = 1u;
            } else {  // its row, for the repeated fold below (finc of a repeated id is free by now)
                finc[q] = (int64_t)wv4[u];
            }
        }
        if (!DIRECT) rcode[q] = r == kResRep ? (uint8_t)kRes2Rep : (uint8_t)(r & 3u);
    }
    __syncthreads();
    BK_T(t3);
    if (!DIRECT && tid < kBk / 16) {  // 16 codes to a word: the gather's map is 1 MB at 2^22 ids, not 4 MB
        const uint4 c4 = reinterpret_cast<const uint4*>(rcode)[tid];
        const uint32_t c[4] = {c4.x, c4.y, c4.z, c4.w};
        uint32_t w = 0;
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int bb = 0; bb < 4; bb++) w |= ((c[i] >> (8 * bb)) & 3u) << (2 * (4 * i + bb));
        res2[(id0 >> 4) + tid] = w;
    }
    if (listed && nd) {  // repeated addresses: sort by (address, batch index), fold per address
        // rank sort (nd <= kBkDup <= kBkFT: one key per thread; the wave reads each key as a broadcast)
        const uint64_t my = tid < nd ? dk[tid] : 0;
        uint32_t rk = 0;
        if (tid < nd)
            for (uint32_t f = 0; f < nd; f++) rk += dk[f] < my ? 1u : 0u;
        __syncthreads();
        if (tid < nd) dk[rk] = my;
        __syncthreads();
        for (uint32_t q = tid; q < nd; q += kBkFT) {
            const uint32_t il = (uint32_t)(dk[q] >> 40);
            if (q > 0 && (uint32_t)(dk[q - 1] >> 40) == il) continue;  // not a segment head
            const uint32_t id = id0 + il;
            const MRowV row = row_unpack((uint64_t)finc[il]);  // loaded with the bucket's rows
            bool ex = row.exists != 0;
            uint8_t st = row.status;
            int64_t in = row.inc;
            for (uint32_t e = q; e < nd && (uint32_t)(dk[e] >> 40) == il; e++) {
                const uint64_t key = dk[e];
                const uint32_t j = (uint32_t)(key >> 10) & 0x3FFFFFFFu, x = (uint32_t)key & 1023u;
                const uint8_t r = bk_step(A, id, ex, st, in, dst[x] & 3u, dinc[x]);
                if (!DIRECT) resj[j] = r;
                else if (A.applied) A.applied[j] = r & 3u;
                if (r & kResLocal) bk_local(A, j);
                napp += (r & 3u) ? 1u : 0u;
            }
            row_store(A.rows + id, in, st, ex ? 1 : 0, A.err);
        }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) napp += __shfl_xor(napp, o, 64);
    if ((tid & 63) == 0) s_w[tid >> 6] = napp;
    __syncthreads();
    BK_T(t4);
#ifdef RP_BK_PROF
    if (tid == 0) {
        atomicAdd(&g_bk_prof[0], (unsigned long long)(t1 - t0));
        atomicAdd(&g_bk_prof[1], (unsigned long long)(t2 - t1));
        atomicAdd(&g_bk_prof[2], (unsigned long long)(t3 - t2));
        atomicAdd(&g_bk_prof[3], (unsigned long long)(t4 - t3));
        atomicAdd(&g_bk_prof[4], 1ull);
        g_bk_wg[2 * b + 1] = __builtin_amdgcn_s_memrealtime();
    }
#endif
    if (tid == 0) {
        uint32_t t = 0;
        for (int w = 0; w < (int)(kBkFT / 64); w++) t += s_w[w];
        part[b] = t;
        if (b == 0) part[nb] = 0;  // the overflow fold's count (k_ovf_len)
    }
}

// applied per change in batch order from the 2-bit map res2 (1 MB at 2^22 ids, L2-resident) or
// resj[j]. V = 4: four consecutive changes per lane (16-B id loads, 4-B stores; the host checks
// the alignment).
template <uint32_t V>
__global__ __launch_bounds__(256) void k_bk_gather(const uint32_t* __restrict__ ids, const uint32_t* __restrict__ res2,
                                                   const uint8_t* __restrict__ resj, uint32_t k,
                                                   uint8_t* __restrict__ applied) {
    const uint32_t j0 = (blockIdx.x * blockDim.x + threadIdx.x) * V;
    if (j0 >= k) return;
    auto one = [&](uint32_t j, uint32_t id) -> uint32_t {
        const uint32_t r = (res2[id >> 4] >> (2u * (id & 15u))) & 3u;
        return r == kRes2Rep ? resj[j] & 3u : r;
    };
    if (V == 4 && j0 + 4 <= k) {
        const uint4 iv = *reinterpret_cast<const uint4*>(ids + j0);
        *reinterpret_cast<uint32_t*>(applied + j0) =
            one(j0, iv.x) | (one(j0 + 1, iv.y) << 8) | (one(j0 + 2, iv.z) << 16) | (one(j0 + 3, iv.w) << 24);
        return;
    }
    for (uint32_t j = j0; j < j0 + V && j < k; j++) applied[j] = (uint8_t)one(j, ids[j]);
}

// Membership._decayMembersDampScore (index.js:374-383): decayDampScore on every member
// (member.js:45-66). Reads 17 B and writes 8 B per id.
__global__ void k_damp_decay(const MRow* __restrict__ rows, uint32_t n, double* __restrict__ score,
                             const double* __restrict__ last, const int64_t* __restrict__ ts, damp::Config c,
                             int64_t now_ms) {
    const uint32_t gstride = gridDim.x * blockDim.x;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gstride)
        if (row_load(rows + i).exists) score[i] = damp::decayed(c, last[i], ts[i], now_ms);
}

template <class T>
__global__ void k_copy_fill(const T* __restrict__ a, uint32_t na, T* __restrict__ b, uint32_t nb, T fill) {
    const uint32_t gstride = gridDim.x * blockDim.x;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nb; i += gstride) b[i] = i < na ? a[i] : fill;
}

// mergeMembershipChangesets (lib/membership/merge.js:22-51) over the (id, arrival)-sorted
// stash: one lane per id segment skips the local member, keeps the change with the strictly
// greatest incarnation (the first one on ties) and marks it at the segment's first arrival
// index, so that compacting the marks in index order gives first-seen address order.
__global__ void k_merge_pick(const uint32_t* __restrict__ sk, const uint32_t* __restrict__ sv, uint32_t k,
                             const int64_t* __restrict__ ch_inc, uint32_t local_id, uint32_t* __restrict__ mark) {
    const uint32_t gstride = gridDim.x * blockDim.x;
    for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < k; p += gstride) {
        const uint32_t id = sk[p];
        if ((p > 0 && sk[p - 1] == id) || id == local_id) continue;
        const uint32_t first = sv[p];
        uint32_t best = first;
        int64_t bi = ch_inc[first];
        for (uint32_t q = p + 1; q < k && sk[q] == id; q++) {
            const uint32_t j = sv[q];
            if (ch_inc[j] > bi) {
                bi = ch_inc[j];
                best = j;
            }
        }
        mark[first] = best + 1u;
    }
}

__global__ void k_flag_nonzero(const uint32_t* __restrict__ mark, uint32_t k, uint32_t* __restrict__ flag) {
    const uint32_t gstride = gridDim.x * blockDim.x;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < k; i += gstride) flag[i] = mark[i] ? 1u : 0u;
}

// Membership.set (index.js:208-247) for the picked changes, in first-seen order: an existing
// member takes the change's status and incarnation verbatim, an unknown address is created.
// Each picked change makes a new Member (index.js:237-241), so its damp state restarts.
__global__ void k_set_apply(const uint32_t* __restrict__ mark, const uint32_t* __restrict__ pos, uint32_t k,
                            const uint32_t* __restrict__ ids, const uint8_t* __restrict__ chs,
                            const int64_t* __restrict__ chi, MRow* __restrict__ rows, uint32_t* __restrict__ pick,
                            uint32_t* __restrict__ npick, DampArgs da, uint32_t* __restrict__ err) {
    const uint32_t gstride = gridDim.x * blockDim.x;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < k; i += gstride) {
        if (i == 0 && npick) *npick = pos[k];
        const uint32_t m = mark[i];
        if (!m) continue;
        const uint32_t j = m - 1u, id = ids[j];
        row_store(rows + id, chi[j], chs[j], 1, err);
        if (da.score) {
            da.score[id] = da.last[id] = da.c.initial;
            da.ts[id] = 0;
        }
        if (pick) pick[pos[i]] = j;
    }
}

// generateChecksumString pieces (index.js:115-120): address + status + incarnation + ';' per
// member in address order, in two launches after the fold (round 3; round 2's single launch
// found each tile's offset by decoupled look-back behind a ticket counter, and its 391
// same-address ticket atomics plus the look-back chain cost more than a second launch):
//   k_ovf_len: the grouped fold's third step (the overflow fold when *ovf is set, and the
//   batch's applied count into the checksum gate) and, per tile of 256 members, the sum of the
//   pieces' lengths into tile_tot (always: it reflects the table after the fold).
//   k_mck_write: each tile sums the totals of the tiles before it (a few hundred words read in
//   parallel), scans its own lengths, assembles its pieces in LDS and stores them as aligned
//   16-byte words; the last tile records the slot's meta. Gated off (*gate == 0), tile 0 only
//   records the meta.

static bool getenv_on(const char* name) {
    const char* v = getenv(name);
    return v && *v && *v != '0';
}
constexpr uint32_t kMckStage = 24576;  // LDS bytes a tile's pieces are assembled in

// One member's piece: row, length and (for names of at most 28 bytes plus alignment) the
// name's aligned dwords, loaded together before the tile's scan so their latency overlaps it.
// Names come by rank from the table's address-ordered copy (NameTable::sort_bytes: soff / sbytes),
// so a tile's names are one contiguous run; only the row is a random access.
struct MckItem {
    uint32_t id, len, nlen, sh;
    MRowV row;
    uint64_t noff;
    uint32_t w[8];
};
// snap (nullable): the rows in rank order, as k_ovf_len copied them (the side-stream build reads
// the copy, coalesced, while the next batch folds the table)
__device__ __forceinline__ void mck_load(uint32_t i, const uint32_t* __restrict__ order, uint32_t n,
                                         const MRow* __restrict__ rows, const uint32_t* __restrict__ soff,
                                         MckItem& t, const uint64_t* __restrict__ snap = nullptr) {
    t.id = snap ? 0u : (i < n ? order[i] : 0u);
    t.row = snap ? row_unpack(i < n ? snap[i] : 0ull) : row_load(rows + t.id);
    t.noff = i < n ? soff[i] : 0u;
    t.nlen = i < n ? soff[i + 1] - (uint32_t)t.noff : 0u;
    t.len = (i < n && t.row.exists) ? t.nlen + status_len(t.row.status) + dec_len(t.row.inc) + 1u : 0u;
}
__device__ __forceinline__ void mck_load_name(const uint8_t* __restrict__ names, MckItem& t) {
    const uint8_t* src = names + t.noff;
    t.sh = (uint32_t)(reinterpret_cast<uintptr_t>(src) & 3u);
    const uint32_t* a4 = reinterpret_cast<const uint32_t*>(src - t.sh);
    const uint32_t nw = t.len && t.sh + t.nlen <= 32u ? (t.sh + t.nlen + 3u) >> 2 : 0u;
#pragma unroll
    for (int k = 0; k < 8; k++) t.w[k] = (uint32_t)k < nw ? a4[k] : 0u;
}
// address + status + incarnation + ';' at o (global or LDS)
__device__ __forceinline__ void mck_emit(uint8_t* o, const uint8_t* __restrict__ names, const MckItem& t) {
    const uint32_t L = t.nlen;
    if (t.sh + L <= 32u) {
#pragma unroll
        for (int k = 0; k < 8; k++)
#pragma unroll
            for (int bb = 0; bb < 4; bb++) {
                const int q = 4 * k + bb - (int)t.sh;
                if (q >= 0 && q < (int)L) o[q] = (uint8_t)(t.w[k] >> (8 * bb));
            }
    } else {
        const uint8_t* src = names + t.noff;
        for (uint32_t q = 0; q < L; q++) o[q] = src[q];
    }
    o += L;
    const uint8_t stc = t.row.status;
    const uint32_t sl = status_len(stc);
    for (uint32_t q = 0; q < sl; q++) o[q] = status_char(stc, q);
    o += sl;
    const uint32_t dl = dec_len(t.row.inc);
    dec_write(t.row.inc, o, dl);
    o[dl] = ';';
}

// Grid: one workgroup per tile. When *ovf is set, the first workgroup to take a ticket runs the
// overflow fold (its applied count to part[nparts]) and clears *ovf; the others wait for that
// before reading rows (the ticket holder is running, so the wait ends). A workgroup that takes
// ticket 0 after the fold finds *ovf clear and skips it; every ticket-0 holder resets the
// counter when done, so it is 0 again after the launch. Workgroup 0 then sums the applied
// counts into *A.n_applied and *out.
__global__ __launch_bounds__(256) void k_ovf_len(const uint32_t* __restrict__ order, uint32_t n,
                                                 const uint32_t* __restrict__ soff, uint32_t* __restrict__ tile_tot,
                                                 const uint32_t* __restrict__ ids, uint32_t k, uint32_t* ovf, FoldArgs A,
                                                 uint32_t* part, uint32_t nparts, uint32_t* __restrict__ out,
                                                 uint32_t* tick, uint32_t* err, uint64_t* __restrict__ snap,
                                                 uint32_t* __restrict__ gate_copy) {
    __shared__ uint32_t s_on, s_t, s_w[4];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    if (tid == 0) s_on = __hip_atomic_load(ovf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (s_on) {  // rare: uniform per workgroup
        if (tid == 0) s_t = atomicAdd(tick, 1u);
        __syncthreads();
        if (s_t == 0) {
            if (tid == 0) s_on = __hip_atomic_load(ovf, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
            __syncthreads();
            if (s_on) {
                const uint32_t v = block_sum256(ovf_fold<256>(ids, k, A));
                if (tid == 0) {
                    part[nparts] = v;
                    __hip_atomic_store(ovf, 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
            if (tid == 0) __hip_atomic_store(tick, 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        } else if (tid == 0) {
            uint32_t spin = 0;
            while (__hip_atomic_load(ovf, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) != 0) {
                if (++spin == kLbSpinCap) {
                    atomicOr(err, kErrSpin);
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
        }
        __syncthreads();
    }
    MckItem t;
    mck_load(blockIdx.x * 256u + tid, order, n, A.rows, soff, t);
    if (snap && blockIdx.x * 256u + tid < n) snap[blockIdx.x * 256u + tid] = row_pack(t.row.inc, t.row.status, t.row.exists);
    const uint32_t total = block_sum256(t.len);
    if (tid == 0) tile_tot[blockIdx.x] = total;
    if (blockIdx.x == 0) {
        uint32_t v = 0;
        for (uint32_t b = tid; b <= nparts; b += 256) v += part[b];
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
        __syncthreads();
        if (lane == 0) s_w[wv] = v;
        __syncthreads();
        if (tid == 0) {
            const uint32_t a = s_w[0] + s_w[1] + s_w[2] + s_w[3];
            *A.n_applied = a;
            if (out) *out = a;
            if (gate_copy) *gate_copy = a;
        }
    }
}

// The sorted path and Membership.set: the tile lengths alone (ungated; the gate is already set).
__global__ __launch_bounds__(256) void k_mck_len(const uint32_t* __restrict__ order, uint32_t n,
                                                 const MRow* __restrict__ rows, const uint32_t* __restrict__ soff,
                                                 uint32_t* __restrict__ tile_tot) {
    MckItem t;
    mck_load(blockIdx.x * 256u + threadIdx.x, order, n, rows, soff, t);
    const uint32_t total = block_sum256(t.len);
    if (threadIdx.x == 0) tile_tot[blockIdx.x] = total;
}

// One tile of the checksum string (tile `tile` of `ntiles`); see k_mck_write.
struct MckArgs {
    const uint32_t* order;
    uint32_t n;
    const MRow* rows;
    const uint8_t* names;
    const uint32_t* soff;
    const uint32_t* gate;
    const uint32_t* tile_tot;
    uint8_t* buf;
    uint32_t* meta;
    const uint64_t* snap;
};
__device__ __forceinline__ void mck_write_block(const MckArgs& a, uint32_t tile, uint32_t ntiles) {
    const uint32_t* __restrict__ order = a.order;
    const uint32_t n = a.n;
    const MRow* __restrict__ rows = a.rows;
    const uint8_t* __restrict__ names = a.names;
    const uint32_t* __restrict__ soff = a.soff;
    const uint32_t* __restrict__ gate = a.gate;
    const uint32_t* __restrict__ tile_tot = a.tile_tot;
    uint8_t* __restrict__ buf = a.buf;
    uint32_t* __restrict__ meta = a.meta;
    const uint64_t* __restrict__ snap = a.snap;
    __shared__ uint32_t s_wsum[4], s_pre[4];
    __shared__ uint32_t s_stage[kMckStage / 4 + 4];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    if (gate && *gate == 0) {
        if (tile == 0 && tid == 0) {
            meta[0] = 0;
            meta[1] = 0;
            meta[3] = 0;
        }
        return;
    }
    uint32_t pre = 0;  // this thread's share of the earlier tiles' totals
    for (uint32_t q = tid; q < tile; q += 256) pre += tile_tot[q];
    MckItem t;
    mck_load(tile * 256u + tid, order, n, rows, soff, t, snap);
    mck_load_name(names, t);
    // inclusive scan of the lengths within each wave; wave totals and prefix shares
    uint32_t x = t.len;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if ((int)lane >= o) x += y;
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) pre += __shfl_xor(pre, o, 64);
    if (lane == 63) s_wsum[wv] = x;
    if (lane == 0) s_pre[wv] = pre;
    __syncthreads();
    uint32_t wbase = 0, total = 0;
#pragma unroll
    for (uint32_t w = 0; w < 4; w++) {
        wbase += w < wv ? s_wsum[w] : 0u;
        total += s_wsum[w];
    }
    const uint32_t g0 = s_pre[0] + s_pre[1] + s_pre[2] + s_pre[3];
    if (tid == 0 && tile == ntiles - 1) {
        meta[0] = g0 + total;
        meta[1] = 1;
        meta[3] = 0;
    }
    const uint32_t pos = wbase + x - t.len;  // this thread's first byte, tile-relative
    if (total > kMckStage) {  // a tile of long names: each thread writes its piece straight out
        if (t.len) mck_emit(buf + g0 + pos, names, t);
        return;
    }
    // Staged: the pieces are assembled in LDS (byte writes there are cheap), then the tile leaves
    // as aligned 16-byte stores; the tile's first and last partial 16 bytes, which it shares
    // with its neighbours, are written bytewise.
    uint8_t* const st = reinterpret_cast<uint8_t*>(s_stage);
    if (t.len) mck_emit(st + pos, names, t);
    __syncthreads();
    const uint32_t a0 = g0 & ~15u, nch = (g0 + total - a0 + 15u) >> 4;
    for (uint32_t c = tid; c < nch; c += 256) {
        const uint32_t a = a0 + 16u * c;
        if (a >= g0 && a + 16u <= g0 + total) {
            const uint32_t l = a - g0, d = l >> 2, r = (l & 3u) * 8u;
            uint32_t w[5];
#pragma unroll
            for (int q = 0; q < 5; q++) w[q] = s_stage[d + q];
            uint4 o;
            o.x = r ? __builtin_amdgcn_alignbit(w[1], w[0], r) : w[0];
            o.y = r ? __builtin_amdgcn_alignbit(w[2], w[1], r) : w[1];
            o.z = r ? __builtin_amdgcn_alignbit(w[3], w[2], r) : w[2];
            o.w = r ? __builtin_amdgcn_alignbit(w[4], w[3], r) : w[3];
            *reinterpret_cast<uint4*>(buf + a) = o;
        } else {
            const uint32_t lo = a > g0 ? a : g0, hi = a + 16u < g0 + total ? a + 16u : g0 + total;
            for (uint32_t q = lo; q < hi; q++) buf[q] = st[q - g0];
        }
    }
}


__global__ __launch_bounds__(256) void k_mck_write(MckArgs a) { mck_write_block(a, blockIdx.x, gridDim.x); }

// The grouped fold of batch b + 1 and the checksum string of batch b in one launch (round 6,
// deferred string write): blocks [0, nfold) fold, the rest write the string from the row snapshot
// k_ovf_len took of batch b, which the fold does not touch. Both are latency-bound, so their
// blocks overlap; the string costs no launch, stream or event of its own.
__global__ __launch_bounds__(256) void k_fold_fast_mck(const uint32_t* __restrict__ ids, uint32_t k,
                                                       const uint8_t* __restrict__ rk,
                                                       const uint32_t* __restrict__ slots, FoldArgs A,
                                                       uint32_t* __restrict__ part, uint32_t nfold, MckArgs m) {
    if (blockIdx.x < nfold)
        fold_fast_block(ids, k, rk, slots, A, part, blockIdx.x, nfold);
    else
        mck_write_block(m, blockIdx.x - nfold, gridDim.x - nfold);
}

// the per-batch history (rp_members_checksum_shard): the group's update-batch slots (bit j of
// mask) append {hash, gate} in slot order
struct SlotMask {
    uint64_t w[1024 / 64];
};
__global__ void k_ck_hist(const uint32_t* __restrict__ meta, uint32_t n, SlotMask mask, uint32_t* __restrict__ hist) {
    uint32_t c = 0;
    for (uint32_t j = 0; j < n; j++) {
        if (!((mask.w[j >> 6] >> (j & 63)) & 1u)) continue;
        hist[2 * c] = meta[4 * j + 1] ? meta[4 * j + 2] : 0u;
        hist[2 * c + 1] = meta[4 * j + 1];
        c++;
    }
}

// the group's results in batch order: the membership checksum is the last gated batch's hash
__global__ void k_ck_commit(const uint32_t* __restrict__ meta, uint32_t n, uint32_t* __restrict__ ck) {
    for (uint32_t b = 0; b < n; b++)
        if (meta[4 * b + 1] && meta[4 * b + 3]) {
            ck[0] = meta[4 * b + 2];
            ck[1] = 1;
        }
}

// the table's rows as the host API returns them (rp_members_dump): exists, status, incarnation
__global__ void k_rows_split(const MRow* __restrict__ rows, uint32_t n, uint8_t* __restrict__ ex,
                             uint8_t* __restrict__ st, int64_t* __restrict__ inc) {
    const uint32_t gstride = gridDim.x * blockDim.x;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gstride) {
        const MRowV r = row_load(rows + i);
        ex[i] = r.exists;
        st[i] = r.status;
        inc[i] = r.inc;
    }
}

}  // namespace

struct Members {
    int device = 0;
    hipStream_t st = nullptr;
    NameTable nt;
    uint32_t local_id = 0xFFFFFFFFu;
    uint32_t cap = 0;
    bool defer_ck = false;  // rp_members_defer_checksum
    DevBuf<MRow> rows;          // the member table, one 8-B row per id
    DevBuf<uint32_t> rcnt;      // per id: the grouped fold's change counter / overflow mark
    DevBuf<uint32_t> ck;        // [0] checksum, [1] is_set
    // [0] per-batch applied count (the checksum gate), [1] the grouped path overflowed (cleared
    // by the sorted fold that then runs), [2..) the launches' last-workgroup counters
    DevBuf<uint32_t> napplied;
    // Checksum strings wait in slots until read or until a group of slots is pending, then one
    // launch hashes the group side by side: a batched caller pays one chain's latency per group
    // instead of per batch. The slots form ngroups groups of group_slots; a full group is hashed on
    // a side stream (ck_st) while the next batches fold and build their strings into the next
    // group, so up to ngroups - 1 groups of chains overlap the folds. Reads flush and wait. The
    // slot count is what fits RP_MEMBERS_CK_BYTES (default 6 GiB of HBM), at most kMaxSlots.
    // Groups of 512 (round 6; RP_MEMBERS_GROUP_SLOTS overrides): the packed chain kernel
    // (k_hash_long_pack, 16 strings a workgroup) hashes 16 to 512 strings of 3.6 MB in the same
    // ~4 ms, so the chains of a 512-batch group cost no more than a 128-batch one did (rounds 2-5:
    // a workgroup a string, groups of 128, 2 GiB; 1.00-1.07 G updates/s against 0.86 with groups
    // of 64 then).
    static constexpr uint32_t kMaxSlots = 1024, kGroupSlots = 512, kMaxGroups = 4;
    uint32_t nslots = 1, group_slots = 1, ngroups = 1;
    DevBuf<uint8_t> ck_buf;   // nslots strings of slot_bytes
    uint64_t slot_bytes = 0;
    DevBuf<uint32_t> ck_meta;  // [kMaxSlots][4]: total, gate, hash, done
    DevBuf<uint32_t> ck_tiles;  // the string build's per-tile byte totals
    uint32_t npending = 0;     // pending strings in the current group
    // Batch-strided checksums over replicas (rp_members_checksum_shard): every replica folds every
    // batch; this one builds and hashes the strings of update batches b with b % ck_nsh == ck_sh
    // only, and records each one's {hash, gate} in ck_hist (hist_cap entries, hist_n used).
    uint32_t ck_nsh = 1, ck_sh = 0;
    uint64_t batch_no = 0;  // update batches (k > 0) seen
    DevBuf<uint32_t> ck_hist;
    uint32_t hist_cap = 0, hist_n = 0;
    static_assert(kMaxSlots <= sizeof(SlotMask) * 8, "one mask bit per slot");
    SlotMask pend_mask = {};  // pending slots that are update batches (history)
    uint32_t cur_group = 0;
    hipStream_t pend_st = nullptr;  // the stream the pending strings were built on
    hipStream_t ck_st = nullptr;    // the side stream the chains run on
    hipEvent_t ev_built = nullptr, ev_hashed[kMaxGroups] = {};
    bool group_busy[kMaxGroups] = {};  // this group's last hash may still be running
    uint32_t slot_index(uint32_t j) const { return cur_group * group_slots + j; }
    DevBuf<uint32_t> ck_len, ck_pos;
    DevBuf<uint32_t> sk, sv;
    // the grouped (sort-free) fold: per id inline slots for repeated addresses, per change its
    // rank among its address's changes (RP_MEMBERS_SORTED_FOLD=1 always sorts)
    bool grouped_fold = !getenv_on("RP_MEMBERS_SORTED_FOLD");
    DevBuf<uint32_t> g_slots;
    DevBuf<uint8_t> g_rk;
    DevBuf<uint32_t> g_part;  // per-workgroup applied counts of k_fold_fast (per bucket: k_bk_fold)
    // the bucket path (batches of kBkMin changes or more without damp scoring; RP_MEMBERS_BUCKET_FOLD
    // = 0 | 1 overrides the size rule)
    DevBuf<uint32_t> bk_seg;
    DevBuf<BRec> bk_recs;
    DevBuf<int64_t> bk_tb;  // per scatter tile: the compact records' incarnation base, or kBkWide
    DevBuf<uint32_t> bk_res2;  // the bucket fold's 2-bit per-id results (k_bk_gather)
    DevBuf<uint8_t> bk_resj;
    static constexpr uint32_t kBkMin = 1u << 19;
    // RP_MEMBERS_FUSE=1 (A/B, off by default): k_link_fold for a grid that is resident at once
    // with half the machine to spare (its grid barrier needs every workgroup running). Measured
    // slower: the C3 fold 0.098-0.102 ms against 0.021 for the two launches, the batch 115-119
    // against 39 us (profiles/r04/r04s): the barrier's agent-scope release / acquire (an L2
    // write-back and invalidate per wave, since the XCDs' L2s are not coherent) costs far more
    // than the launch it saves.
    int fuse_cap = -1;
    bool fuse_fold(uint32_t g1, hipStream_t s) {
        const char* e = getenv("RP_MEMBERS_FUSE");
        if (!e || *e != '1') return false;
        if (fuse_cap < 0) {
            int dev = 0, cus = 0, nbl = 0;
            RP_HIP(hipGetDevice(&dev));
            RP_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
            RP_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nbl, reinterpret_cast<const void*>(k_link_fold), 256, 0));
            fuse_cap = cus * nbl / 2;
        }
        if ((int)g1 > fuse_cap) return false;
        if (!ws.err.p) {
            ws.err.reserve(1);
            RP_HIP(hipMemsetAsync(ws.err.p, 0, sizeof(uint32_t), s));
        }
        return true;
    }
    bool use_bucket_fold(uint32_t k, uint32_t nb) const {
        if (damp_on || nb > kBkMaxBuckets || k >= (1u << 29) || !grouped_fold) return false;
        const char* e = getenv("RP_MEMBERS_BUCKET_FOLD");
        if (e && *e) return *e != '0';
        return k >= kBkMin;
    }
    DevBuf<uint32_t> mk, mpos;  // set: merge marks and their positions
    // host-buffer staging
    DevBuf<uint32_t> io_ids, io_pick;
    DevBuf<uint8_t> io_st, io_app, io_nst;
    DevBuf<int64_t> io_inc, io_ninc;
    Scratch ws;
    // damp scoring (rp_members_damp_configure): per id score / last score / last timestamp, and
    // the per-change score + suppress flag of the last update batch
    bool damp_on = false;
    damp::Config dcfg{};
    DevBuf<double> d_score, d_last, d_out;
    DevBuf<int64_t> d_ts;
    DevBuf<uint8_t> d_exc;
    uint32_t d_out_k = 0;

    DampArgs damp_args(bool outputs) {
        DampArgs a{};
        a.c = dcfg;
        if (damp_on) {
            a.score = d_score.p;
            a.last = d_last.p;
            a.ts = d_ts.p;
            if (outputs) {
                a.out = d_out.p;
                a.exc = d_exc.p;
            }
        }
        return a;
    }

    template <class T>
    void grow_one(DevBuf<T>& b, uint32_t old_n, uint32_t new_n, T fill) {
        DevBuf<T> b2;
        b2.reserve(new_n);
        hipLaunchKernelGGL(k_copy_fill<T>, dim3(grid_for(new_n, 256)), dim3(256), 0, st, b.p, old_n, b2.p, new_n,
                           fill);
        RP_HIP(hipGetLastError());
        RP_HIP(hipStreamSynchronize(st));
        b.swap(b2);
    }

    void grow(uint32_t need) {
        if (need <= cap) return;
        uint32_t nc = std::max<uint32_t>(need, cap ? cap * 2 : 1024);
        grow_one<MRow>(rows, cap, nc, MRow{0});
        grow_one<uint32_t>(rcnt, cap, nc, 0u);
        if (damp_on) {
            grow_one<double>(d_score, cap, nc, dcfg.initial);
            grow_one<double>(d_last, cap, nc, dcfg.initial);
            grow_one<int64_t>(d_ts, cap, nc, 0);
        }
        cap = nc;
    }

    // rp_members_damp_configure: every member (present or not yet created) starts as a fresh
    // Member would (member.js:35-39)
    void damp_configure(const damp::Config& c) {
        dcfg = c;
        if (!damp_on) {
            damp_on = true;
            d_score.release();
            d_last.release();
            d_ts.release();
            grow_one<double>(d_score, 0, cap, c.initial);
            grow_one<double>(d_last, 0, cap, c.initial);
            grow_one<int64_t>(d_ts, 0, cap, 0);
        }
    }

    // Everything below is stream-ordered on `s` and never syncs with the host.
    // Grouped path (every batch size): k_link + k_fold_fast + k_fold_ovf (gated on the overflow
    // word on the device: it folds only addresses with more than kSlots + 1 changes, and sums
    // the applied count into n_applied_out). RP_MEMBERS_SORTED_FOLD=1: radix sort + k_fold.
    // ranged (rp_members_update_range_dev): only the changes whose id lies in [id_lo, id_hi), whole
    // buckets of kBk ids, through the bucket path; no checksum (the rows outside are not this
    // handle's to keep current).
    void update_dev(const uint32_t* ids, const uint8_t* chs, const int64_t* chi, uint32_t k, int64_t now_ms,
                    uint8_t* applied, uint8_t* nst, int64_t* ninc, uint32_t* n_applied_out, hipStream_t s,
                    bool ranged = false, uint32_t id_lo = 0, uint32_t id_hi = 0) {
        if (ranged) {
            RP_REQUIRE(id_lo % kBk == 0 && (id_hi % kBk == 0 || id_hi >= cap) && id_lo <= id_hi,
                       "update_range: the range must be whole buckets of 4,096 ids");
            RP_REQUIRE(!damp_on && grouped_fold && (cap + kBk - 1) / kBk <= kBkMaxBuckets && k < (1u << 29),
                       "update_range: needs the bucket fold (no damp scoring, at most 8M ids)");
        }
        if (s != st) RP_HIP(hipStreamSynchronize(st));
        if (!k) {
            RP_HIP(hipMemsetAsync(napplied.p, 0, sizeof(uint32_t), s));
            if (n_applied_out) RP_HIP(hipMemsetAsync(n_applied_out, 0, sizeof(uint32_t), s));
            return;
        }
        if (pw.on && (ranged || pw.st != s || use_bucket_fold(k, (cap + kBk - 1) / kBk) || !grouped_fold ||
                      getenv_on("RP_MEMBERS_FUSE")))
            drain_write();  // only the grouped fold's launch carries a deferred string
        if (damp_on) {
            d_out.reserve(k);
            d_exc.reserve(k);
            d_out_k = k;
        }
        if (!ws.err.p) {
            ws.err.reserve(1);
            RP_HIP(hipMemsetAsync(ws.err.p, 0, sizeof(uint32_t), s));
        }
        const FoldArgs A{chs, chi, rows.p, rcnt.p, ws.err.p, local_id, now_ms, applied, nst, ninc, napplied.p,
                         damp_args(true)};
        int bits = 8;
        while (bits < 32 && (1ull << bits) < nt.size()) bits += 8;
        sk.reserve(k);
        sv.reserve(k);
        uint32_t* ovf = napplied.p + 1;
        uint32_t* done = napplied.p + 2;
        const unsigned g = grid_for(k, 256);
        const bool mine = ck_nsh <= 1 || batch_no % ck_nsh == ck_sh;
        const bool build = !defer_ck && mine && !ranged;
        if (build && hist_cap && nt.size()) {  // refuse before anything is applied
            uint32_t pend = 0;
            for (uint64_t w : pend_mask.w) pend += (uint32_t)__builtin_popcountll(w);
            if (hist_n + pend + 1 > hist_cap)
                throw Error(RP_ESTATE, "checksum history full (history_cap of rp_members_checksum_shard): read and "
                                       "drain it with rp_members_checksum_history_drain");
        }
        batch_no++;
        const uint32_t nb = (cap + kBk - 1) / kBk;
        const uint32_t b_lo = ranged ? std::min(nb, id_lo / kBk) : 0u;
        const uint32_t b_hi = ranged ? (uint32_t)std::min<uint64_t>(nb, ((uint64_t)id_hi + kBk - 1) / kBk) : nb;
        if (ranged && b_lo >= b_hi) {  // a range past the table (a rank with no ids yet): nothing to fold
            RP_HIP(hipMemsetAsync(napplied.p, 0, sizeof(uint32_t), s));
            if (n_applied_out) RP_HIP(hipMemsetAsync(n_applied_out, 0, sizeof(uint32_t), s));
            return;
        }
        if (ranged || use_bucket_fold(k, nb)) {
            const uint32_t ntiles = (k + kBkTile - 1) / kBkTile;
            bk_seg.reserve((uint64_t)((nb + 15) / 16) * 16 * ntiles);
            bk_recs.reserve((uint64_t)ntiles * kBkTile);
            bk_res2.reserve((uint64_t)nb * kBk / 16);
            bk_resj.reserve(k);
            g_part.reserve(nb + 1);
            bk_tb.reserve(ntiles);
            const bool rec8 = !(getenv("RP_BK_REC8") && !strcmp(getenv("RP_BK_REC8"), "0"));  // A/B: 0 = 12-B always
            // workgroups of the scatter (A/B: RP_BK_SGRID; 0 or >= ntiles: one tile each)
            const uint32_t sg = (uint32_t)env_pos("RP_BK_SGRID", 0);
            if (sg && sg < ntiles)
                hipLaunchKernelGGL(k_bk_scatter<true>, dim3(sg), dim3(kBkST), 0, s, ids, chs, chi, k, nb, ntiles,
                                   bk_recs.p, bk_seg.p, rec8 ? bk_tb.p : nullptr, nst, ninc, ws.err.p, b_lo, b_hi);
            else
                hipLaunchKernelGGL(k_bk_scatter<false>, dim3(ntiles), dim3(kBkST), 0, s, ids, chs, chi, k, nb, ntiles,
                                   bk_recs.p, bk_seg.p, rec8 ? bk_tb.p : nullptr, nst, ninc, ws.err.p, b_lo, b_hi);
            const bool direct = ranged || !(getenv("RP_BK_DIRECT") && !strcmp(getenv("RP_BK_DIRECT"), "0"));
            if (ranged) RP_HIP(hipMemsetAsync(g_part.p, 0, sizeof(uint32_t) * (nb + 1), s));  // other ranks' buckets
            const dim3 fg((b_hi - b_lo + 7) / 8 * 8);
            if (direct)
                hipLaunchKernelGGL(k_bk_fold<true>, fg, dim3(kBkFT), 0, s, bk_recs.p, bk_seg.p, rec8 ? bk_tb.p : nullptr,
                                   ntiles, nb, b_lo, b_hi, A, bk_res2.p, bk_resj.p, ovf, g_part.p);
            else
                hipLaunchKernelGGL(k_bk_fold<false>, fg, dim3(kBkFT), 0, s, bk_recs.p, bk_seg.p, rec8 ? bk_tb.p : nullptr,
                                   ntiles, nb, b_lo, b_hi, A, bk_res2.p, bk_resj.p, ovf, g_part.p);
#ifdef RP_BK_PROF
            if (getenv("RP_BK_PROF_PRINT")) {
                unsigned long long v[8];
                RP_HIP(hipStreamSynchronize(s));
                RP_HIP(hipMemcpyFromSymbol(v, HIP_SYMBOL(g_bk_prof), sizeof v));
                const double nw = (double)(v[4] ? v[4] : 1);
                fprintf(stderr, "[rp] k_bk_fold cycles per workgroup (%llu): records %.0f dup-heads %.0f rows+map %.0f dups+count %.0f\n",
                        v[4], v[0] / nw, v[1] / nw, v[2] / nw, v[3] / nw);
                memset(v, 0, sizeof v);
                RP_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_bk_prof), v, sizeof v));
                // per-workgroup timeline (the grid's quantization): starts and ends in us
                // from the first start; how many workgroups run at each tenth of the span
                std::vector<unsigned long long> wg(2 * kBkMaxBuckets);
                RP_HIP(hipMemcpyFromSymbol(wg.data(), HIP_SYMBOL(g_bk_wg), sizeof(unsigned long long) * 2 * nb));
                unsigned long long t0 = ~0ull, t1 = 0;
                std::vector<double> st(nb), du(nb);
                for (uint32_t i = 0; i < nb; i++) {
                    t0 = std::min(t0, wg[2 * i]);
                    t1 = std::max(t1, wg[2 * i + 1]);
                }
                for (uint32_t i = 0; i < nb; i++) {
                    st[i] = (wg[2 * i] - t0) / 100.0;
                    du[i] = (wg[2 * i + 1] - wg[2 * i]) / 100.0;
                }
                std::vector<double> ss = st, dd = du;
                std::sort(ss.begin(), ss.end());
                std::sort(dd.begin(), dd.end());
                const double span = (t1 - t0) / 100.0;
                fprintf(stderr, "[rp] k_bk_fold workgroups %u: span %.1f us; starts p50 %.1f p75 %.1f p90 %.1f last %.1f; "
                                "durations min %.1f p50 %.1f p90 %.1f max %.1f; running at tenths:",
                        nb, span, ss[nb / 2], ss[nb * 3 / 4], ss[nb * 9 / 10], ss[nb - 1], dd[0], dd[nb / 2], dd[nb * 9 / 10],
                        dd[nb - 1]);
                for (int q = 0; q < 10; q++) {
                    const double t = span * (q + 0.5) / 10.0;
                    int c = 0;
                    for (uint32_t i = 0; i < nb; i++) c += (st[i] <= t && st[i] + du[i] > t) ? 1 : 0;
                    fprintf(stderr, " %d", c);
                }
                fprintf(stderr, "\n");
            }
#endif
            if (applied && !direct) {
                const bool v4 = ((uintptr_t)ids & 15) == 0 && ((uintptr_t)applied & 3) == 0;
                if (v4)
                    hipLaunchKernelGGL(k_bk_gather<4>, dim3(grid_for((k + 3) / 4, 256, 1u << 30)), dim3(256), 0, s,
                                       ids, bk_res2.p, bk_resj.p, k, applied);
                else
                    hipLaunchKernelGGL(k_bk_gather<1>, dim3(grid_for(k, 256, 1u << 30)), dim3(256), 0, s, ids,
                                       bk_res2.p, bk_resj.p, k, applied);
            }
            RP_HIP(hipGetLastError());
            if (build && nt.size()) {
                const OvfArgs ov{ids, k, ovf, A, g_part.p, nb, n_applied_out};
                checksum_dev(s, napplied.p, true, &ov);
                return;
            }
            hipLaunchKernelGGL(k_fold_ovf, dim3(1), dim3(1024), 0, s, ids, k, ovf, A, g_part.p, nb, n_applied_out);
        } else if (grouped_fold) {
            g_slots.reserve((uint64_t)cap * kSlots);
            g_rk.reserve(k);
            const unsigned g1 = (unsigned)((k + 255) / 256);
            g_part.reserve(g1 + 1);
            if (fuse_fold(g1, s)) {
                hipLaunchKernelGGL(k_link_fold, dim3(g1), dim3(256), 0, s, ids, k, g_slots.p, g_rk.p, ovf, napplied.p, A,
                                   g_part.p, ws.err.p);
            } else {
                hipLaunchKernelGGL(k_link, dim3(g1), dim3(256), 0, s, ids, k, rcnt.p, g_slots.p, g_rk.p, ovf,
                                   napplied.p);
                if (pw.on && pw.st == s) {  // the previous batch's string rides on this fold's launch
                    pw.on = false;
                    hipLaunchKernelGGL(k_fold_fast_mck, dim3(g1 + pw.ntl), dim3(256), 0, s, ids, k, g_rk.p, g_slots.p, A,
                                       g_part.p, g1, pw.a);
                } else {
                    hipLaunchKernelGGL(k_fold_fast, dim3(g1), dim3(256), 0, s, ids, k, g_rk.p, g_slots.p, A, g_part.p);
                }
            }
            RP_HIP(hipGetLastError());
            if (build && nt.size()) {  // the overflow fold rides on the string build's length launch
                const OvfArgs ov{ids, k, ovf, A, g_part.p, g1, n_applied_out};
                checksum_dev(s, napplied.p, true, &ov);
                return;
            }
            hipLaunchKernelGGL(k_fold_ovf, dim3(1), dim3(1024), 0, s, ids, k, ovf, A, g_part.p, g1, n_applied_out);
        } else {
            RP_HIP(hipMemsetAsync(napplied.p, 0, sizeof(uint32_t), s));
            radix_sort_index(ids, sk.p, sv.p, k, 0, bits, s, ws);
            hipLaunchKernelGGL(k_fold, dim3(g), dim3(256), 0, s, sk.p, sv.p, k, A, nullptr, done + 1, n_applied_out,
                               nullptr, 0u);
        }
        RP_HIP(hipGetLastError());
        if (build) checksum_dev(s, napplied.p, true);
    }

    // Membership.set over a stash of k changes (arrival order): merge, set, checksum once.
    void set_dev(const uint32_t* ids, const uint8_t* chs, const int64_t* chi, uint32_t k, uint32_t* pick,
                 uint32_t* npick, hipStream_t s) {
        if (s != st) RP_HIP(hipStreamSynchronize(st));
        if (!k) {
            if (npick) RP_HIP(hipMemsetAsync(npick, 0, sizeof(uint32_t), s));
            return;
        }
        if (!ws.err.p) {
            ws.err.reserve(1);
            RP_HIP(hipMemsetAsync(ws.err.p, 0, sizeof(uint32_t), s));
        }
        sk.reserve(k);
        sv.reserve(k);
        mk.reserve(k);
        mpos.reserve(k + 1);
        int bits = 8;
        while (bits < 32 && (1ull << bits) < nt.size()) bits += 8;
        radix_sort_index(ids, sk.p, sv.p, k, 0, bits, s, ws);
        RP_HIP(hipMemsetAsync(mk.p, 0, 4ull * k, s));
        hipLaunchKernelGGL(k_merge_pick, dim3(grid_for(k, 256)), dim3(256), 0, s, sk.p, sv.p, k, chi, local_id, mk.p);
        hipLaunchKernelGGL(k_flag_nonzero, dim3(grid_for(k, 256)), dim3(256), 0, s, mk.p, k, mpos.p);
        scan_exclusive_u32(mpos.p, mpos.p, k, s, ws);
        hipLaunchKernelGGL(k_set_apply, dim3(grid_for(k, 256)), dim3(256), 0, s, mk.p, mpos.p, k, ids, chs, chi,
                           rows.p, pick, npick, damp_args(false), ws.err.p);
        RP_HIP(hipGetLastError());
        checksum_dev(s, nullptr);
    }

    // Membership.computeChecksum (index.js:48-75) gated on *gate != 0 (null = always): the
    // string is built now (it reflects the table after this batch) into the next slot; its hash
    // lands in ck when the group is flushed.
    // ov: the grouped fold's overflow step, run by the length launch (k_ovf_len).
    struct OvfArgs {
        const uint32_t* ids;
        uint32_t k;
        uint32_t* ovf;
        FoldArgs A;
        uint32_t* part;
        uint32_t nparts;
        uint32_t* out;
    };
    // Where an update batch's checksum string is written (round 6; RP_MEMBERS_SIDE_BUILD selects,
    // for A/B). For an update batch the length launch (k_ovf_len) also copies every member's row
    // in rank order and the batch's applied count into a snapshot, so the writer no longer needs
    // the table as it was after this batch:
    //   2 (default) deferred: the string of batch b is written by the blocks that k_fold_fast_mck
    //     appends to batch b + 1's fold launch (any other call first writes it with its own launch,
    //     drain_write); one snapshot suffices, since batch b + 1's lengths follow that launch;
    //   1 build stream: k_mck_write runs on a second stream from one of two snapshots, ordered by
    //     events (0.0410 -> 0.0369 ms per C3 batch, r06e; the events cost the host ~9 us a batch);
    //   0 inline: k_mck_write right after k_ovf_len on the caller's stream, from the table.
    hipStream_t bs = nullptr;                     // the build stream (mode 1)
    hipEvent_t ev_len = nullptr, ev_snap[2] = {};  // lengths + snapshot ready; snapshot p free again
    bool snap_busy[2] = {false, false};
    uint32_t snap_p = 0;
    DevBuf<uint64_t> snap_rows[2];
    DevBuf<uint32_t> snap_tiles[2], snap_gate;
    hipStream_t pend_main = nullptr;  // the caller's stream of the pending group
    struct PendingWrite {  // mode 2: the string k_fold_fast_mck (or drain_write) still has to write
        bool on = false;
        uint32_t ntl = 0;
        hipStream_t st = nullptr;
        MckArgs a{};
    } pw;
    int string_mode() const {
        const char* e = getenv("RP_MEMBERS_SIDE_BUILD");
        return e && (*e == '0' || *e == '1') ? *e - '0' : 2;
    }
    // write a deferred string now (its own launch, on the stream it was deferred on)
    void drain_write() {
        if (!pw.on) return;
        pw.on = false;
        hipLaunchKernelGGL(k_mck_write, dim3(pw.ntl), dim3(256), 0, pw.st, pw.a);
        RP_HIP(hipGetLastError());
    }
    // the writer reads the names' rank order and bytes (nt.sorted / soff / sbytes): a call that
    // may rewrite them (interning, the wire codec's name index) has it written first
    void settle_build() {
        if (pw.on) {
            const hipStream_t w = pw.st;
            drain_write();
            RP_HIP(hipStreamSynchronize(w));
        }
        if (bs) RP_HIP(hipStreamSynchronize(bs));
    }
    void checksum_dev(hipStream_t s, const uint32_t* gate, bool is_batch = false, const OvfArgs* ov = nullptr) {
        const uint32_t n = nt.size();
        if (!n) return;
        drain_write();
        ck_len.reserve(n + 1);
        ck_pos.reserve(n + 1);
        const int mode = ov ? string_mode() : 0;
        if (mode == 1 && !bs) {
            RP_HIP(hipStreamCreateWithFlags(&bs, hipStreamNonBlocking));
            RP_HIP(hipEventCreateWithFlags(&ev_len, hipEventDisableTiming));
            for (auto& e : ev_snap) RP_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        }
        const hipStream_t bst = mode == 1 ? bs : s;  // where this string is written
        // worst-case string: names + ';' + "suspect" + 20 digits per member
        const uint64_t need = (nt.h_bytes.size() + (uint64_t)n * 29 + 16 + 255) & ~255ull;
        if (npending && (s != pend_main || bst != pend_st || need > slot_bytes)) {  // keep the group on one stream
            flush_checksums();
            RP_HIP(hipStreamSynchronize(pend_st));
        }
        if (!ck_st) {
            RP_HIP(hipStreamCreateWithFlags(&ck_st, hipStreamNonBlocking));
            RP_HIP(hipEventCreateWithFlags(&ev_built, hipEventDisableTiming));
            for (auto& e : ev_hashed) RP_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        }
        if (need > slot_bytes) {
            RP_HIP(hipStreamSynchronize(ck_st));  // no chain still reads the old pool
            if (bs) RP_HIP(hipStreamSynchronize(bs));  // no writer still writes it
            for (auto& b : group_busy) b = false;
            cur_group = 0;
            ck_buf.release();
            // 6 GiB of HBM: at C3's 4.7 MB slots, 2 groups of 512 (round 6: the packed chain kernel
            // hashes 16 to 512 strings in the same ~4 ms, so a group of 512 costs what one of 128
            // did: 0.0384 -> 0.0311 ms per C3 batch, profiles/r06/r06j/); rounds 2-5 kept 2 GiB and
            // groups of 128 (1 GiB / 2 groups: 51.4 against 45.2 us per batch, profiles/r04/r04e/)
            const uint64_t budget = env_pos("RP_MEMBERS_CK_BYTES", 6ull << 30);
            nslots = (uint32_t)std::min<uint64_t>(kMaxSlots, std::max<uint64_t>(1, budget / need));
            const uint32_t gmax = (uint32_t)env_pos("RP_MEMBERS_GROUP_SLOTS", kGroupSlots);  // A/B: chains per launch
            group_slots = std::max<uint32_t>(1, std::min<uint32_t>(gmax, nslots / 2));
            ngroups = std::max<uint32_t>(1, std::min<uint32_t>(kMaxGroups, nslots / group_slots));
            ck_buf.reserve(need * (uint64_t)group_slots * ngroups);
            slot_bytes = need;
        }
        if (npending == group_slots) flush_checksums();
        if (npending == 0 && group_busy[cur_group]) {  // this group's previous strings must be hashed
            RP_HIP(hipStreamWaitEvent(bst, ev_hashed[cur_group], 0));
            group_busy[cur_group] = false;
        }
        pend_st = bst;
        pend_main = s;
        ck_meta.reserve(4 * kMaxSlots);
        uint8_t* buf = ck_buf.p + slot_bytes * slot_index(npending);
        {
            const uint32_t ntl = (n + 255) / 256;
            uint32_t* meta = ck_meta.p + 4ull * slot_index(npending);
            if (ov) {
                if (!ws.err.p) {
                    ws.err.reserve(1);
                    RP_HIP(hipMemsetAsync(ws.err.p, 0, sizeof(uint32_t), s));
                }
                uint64_t* snap = nullptr;
                uint32_t* tiles = nullptr;
                uint32_t* gcopy = nullptr;
                const uint32_t p = mode == 1 ? snap_p : 0u;
                if (mode >= 1) {
                    if (mode == 1 && snap_busy[p]) RP_HIP(hipStreamWaitEvent(s, ev_snap[p], 0));  // its writer has read it
                    if (snap_rows[p].cap < n) {
                        if (bs) RP_HIP(hipStreamSynchronize(bs));
                        snap_rows[p].reserve(n);
                    }
                    snap_tiles[p].reserve(ntl);
                    snap_gate.reserve(2);
                    snap = snap_rows[p].p;
                    tiles = snap_tiles[p].p;
                    gcopy = snap_gate.p + p;
                } else {
                    ck_tiles.reserve(ntl);
                    tiles = ck_tiles.p;
                }
                hipLaunchKernelGGL(k_ovf_len, dim3(ntl), dim3(256), 0, s, nt.sorted.p, n, nt.soff.p, tiles,
                                   ov->ids, ov->k, ov->ovf, ov->A, ov->part, ov->nparts, ov->out,
                                   napplied.p + 2 + 2, ws.err.p, snap, gcopy);
                const MckArgs ma{nt.sorted.p, n, rows.p, nt.sbytes.p, nt.soff.p, mode >= 1 ? gcopy : gate, tiles, buf,
                                 meta, snap};
                if (mode == 2) {
                    pw.on = true;
                    pw.ntl = ntl;
                    pw.st = s;
                    pw.a = ma;
                } else if (mode == 1) {
                    RP_HIP(hipEventRecord(ev_len, s));
                    RP_HIP(hipStreamWaitEvent(bs, ev_len, 0));
                    hipLaunchKernelGGL(k_mck_write, dim3(ntl), dim3(256), 0, bs, ma);
                    RP_HIP(hipEventRecord(ev_snap[p], bs));
                    snap_busy[p] = true;
                    snap_p ^= 1u;
                } else {
                    hipLaunchKernelGGL(k_mck_write, dim3(ntl), dim3(256), 0, s, ma);
                }
            } else {
                ck_tiles.reserve(ntl);
                hipLaunchKernelGGL(k_mck_len, dim3(ntl), dim3(256), 0, s, nt.sorted.p, n, rows.p, nt.soff.p,
                                   ck_tiles.p);
                const MckArgs ma{nt.sorted.p, n, rows.p, nt.sbytes.p, nt.soff.p, gate, ck_tiles.p, buf, meta, nullptr};
                hipLaunchKernelGGL(k_mck_write, dim3(ntl), dim3(256), 0, s, ma);
            }
        }
        RP_HIP(hipGetLastError());
        if (is_batch && hist_cap) pend_mask.w[npending >> 6] |= 1ull << (npending & 63);
        npending++;
    }

    // hash the current group's pending strings (side by side) on the side stream once they are
    // built, then commit the last gated one to ck (groups commit in batch order: one stream)
    void flush_checksums() {
        if (!npending) return;
        drain_write();  // the group's last string, if its batch's successor has not written it
        RP_HIP(hipEventRecord(ev_built, pend_st));
        RP_HIP(hipStreamWaitEvent(ck_st, ev_built, 0));
        const uint64_t first = slot_index(0);
        hash_long_multi(ck_buf.p + slot_bytes * first, slot_bytes, npending, ck_meta.p + 4 * first, ck_st);
        hipLaunchKernelGGL(k_ck_commit, dim3(1), dim3(1), 0, ck_st, ck_meta.p + 4 * first, npending, ck.p);
        RP_HIP(hipGetLastError());
        uint32_t nb = 0;
        for (uint64_t w : pend_mask.w) nb += (uint32_t)__builtin_popcountll(w);
        // update_dev refuses a batch the history cannot take before it launches anything, so the
        // nb entries always fit here and this path never throws with the group half-flushed
        if (nb) {
            hipLaunchKernelGGL(k_ck_hist, dim3(1), dim3(1), 0, ck_st, ck_meta.p + 4 * first, npending, pend_mask,
                               ck_hist.p + 2ull * hist_n);
            hist_n += nb;
        }
        pend_mask = {};
        RP_HIP(hipEventRecord(ev_hashed[cur_group], ck_st));
        group_busy[cur_group] = true;
        cur_group = (cur_group + 1) % ngroups;
        npending = 0;
        RP_HIP(hipGetLastError());
    }
    // flush and wait, before a host read of the checksum
    void settle_checksums() {
        flush_checksums();
        if (ck_st) RP_HIP(hipStreamSynchronize(ck_st));
        for (auto& b : group_busy) b = false;
    }
    void release_streams() {
        if (bs) {
            (void)hipStreamSynchronize(bs);
            (void)hipStreamDestroy(bs);
            (void)hipEventDestroy(ev_len);
            for (auto& e : ev_snap) (void)hipEventDestroy(e);
            bs = nullptr;
        }
        if (ck_st) {
            (void)hipStreamSynchronize(ck_st);
            (void)hipStreamDestroy(ck_st);
            (void)hipEventDestroy(ev_built);
            for (auto& e : ev_hashed) (void)hipEventDestroy(e);
            ck_st = nullptr;
        }
    }
};

}  // namespace rp

// ==================================================================================== C ABI

struct rp_members {
    rp::Members impl;
};

using rp::guard;

static rp::Members& MB(rp_members* m);

namespace rp {
// The interned addresses the wire codec (rp_wire.hip) reads and resolves against.
NameTable& members_names(rp_members* h, hipStream_t* st, Scratch** ws) {
    Members& m = MB(h);
    m.settle_build();
    *st = m.st;
    *ws = &m.ws;
    return m.nt;
}
}  // namespace rp

static rp::Members& MB(rp_members* m) {
    if (!m) throw rp::Error(rp::RP_EINVAL, "null members handle");
    RP_HIP(hipSetDevice(m->impl.device));
    return m->impl;
}

extern "C" {

int rp_members_create(uint32_t capacity, int device, rp_members** out) {
    return guard([&] {
        RP_REQUIRE(out, "out is null");
        int nd = 0;
        RP_HIP(hipGetDeviceCount(&nd));
        RP_REQUIRE(device >= 0 && device < nd, "no such HIP device");
        RP_HIP(hipSetDevice(device));
        auto* h = new rp_members();
        rp::Members& m = h->impl;
        m.device = device;
        hipError_t e = hipStreamCreateWithFlags(&m.st, hipStreamNonBlocking);
        if (e != hipSuccess) {
            delete h;
            throw rp::Error(rp::RP_EDEVICE, std::string("hipStreamCreate: ") + hipGetErrorString(e));
        }
        m.ck.reserve(2);
        m.napplied.reserve(2 + rp::kDoneWords);
        RP_HIP(hipMemsetAsync(m.ck.p, 0, 2 * sizeof(uint32_t), m.st));
        RP_HIP(hipMemsetAsync(m.napplied.p, 0, (2 + rp::kDoneWords) * sizeof(uint32_t), m.st));
        m.grow(capacity ? capacity : 1024);
        RP_HIP(hipStreamSynchronize(m.st));
        *out = h;
    });
}

int rp_members_destroy(rp_members* m) {
    return guard([&] {
        if (!m) return;
        (void)hipSetDevice(m->impl.device);
        if (m->impl.st) {
            (void)hipStreamSynchronize(m->impl.st);
            (void)hipStreamDestroy(m->impl.st);
        }
        m->impl.release_streams();
        delete m;
    });
}

int rp_members_intern(rp_members* h, const char* bytes, const uint32_t* off, uint32_t n, uint32_t* ids_out) {
    return guard([&] {
        rp::Members& m = MB(h);
        RP_REQUIRE(n == 0 || (bytes && off), "intern: null names");
        m.settle_build();
        for (uint32_t i = 0; i < n; i++) {
            const uint32_t id = m.nt.intern(bytes + off[i], off[i + 1] - off[i]);
            if (ids_out) ids_out[i] = id;
        }
        m.grow(m.nt.size());
        m.nt.sort_bytes(m.st, m.ws);  // address order for checksums (also uploads the names)
        RP_HIP(hipStreamSynchronize(m.st));
    });
}

int rp_members_set_local(rp_members* h, uint32_t local_id) {
    return guard([&] { MB(h).local_id = local_id; });
}

int rp_members_update_dev(rp_members* h, const uint32_t* d_ids, const uint8_t* d_status, const int64_t* d_inc,
                          uint32_t k, int64_t now_ms, uint8_t* d_applied, uint8_t* d_new_status, int64_t* d_new_inc,
                          uint32_t* d_n_applied, void* stream) {
    return guard([&] {
        rp::Members& m = MB(h);
        RP_REQUIRE(k == 0 || (d_ids && d_status && d_inc), "update_dev: null change buffers");
        m.update_dev(d_ids, d_status, d_inc, k, now_ms, d_applied, d_new_status, d_new_inc, d_n_applied,
                     rp::as_stream(stream));
    });
}

int rp_members_update_range_dev(rp_members* h, const uint32_t* d_ids, const uint8_t* d_status, const int64_t* d_inc,
                                uint32_t k, int64_t now_ms, uint32_t id_lo, uint32_t id_hi, uint8_t* d_applied,
                                uint8_t* d_new_status, int64_t* d_new_inc, uint32_t* d_n_applied, void* stream) {
    return guard([&] {
        rp::Members& m = MB(h);
        RP_REQUIRE(k == 0 || (d_ids && d_status && d_inc), "update_range_dev: null change buffers");
        m.update_dev(d_ids, d_status, d_inc, k, now_ms, d_applied, d_new_status, d_new_inc, d_n_applied,
                     rp::as_stream(stream), true, id_lo, id_hi);
    });
}

int rp_members_rows_copy(rp_members* h, void* d_buf, uint32_t id_lo, uint32_t id_hi, int into_table, void* stream) {
    return guard([&] {
        rp::Members& m = MB(h);
        RP_REQUIRE(id_lo <= id_hi && id_hi <= m.cap, "rows_copy: range outside the table's capacity");
        RP_REQUIRE(id_lo == id_hi || d_buf, "rows_copy: null buffer");
        if (id_lo == id_hi) return;
        m.settle_build();  // a deferred string write still reads the rows' snapshot, not the rows
        const hipStream_t s = rp::as_stream(stream);
        if (s != m.st) RP_HIP(hipStreamSynchronize(m.st));
        const uint64_t bytes = sizeof(rp::MRow) * (uint64_t)(id_hi - id_lo);
        if (into_table)
            RP_HIP(hipMemcpyAsync(m.rows.p + id_lo, d_buf, bytes, hipMemcpyDeviceToDevice, s));
        else
            RP_HIP(hipMemcpyAsync(d_buf, m.rows.p + id_lo, bytes, hipMemcpyDeviceToDevice, s));
        if (s != m.st && into_table) RP_HIP(hipStreamSynchronize(s));  // the handle's own stream reads them next
    });
}

int rp_members_update(rp_members* h, const uint32_t* ids, const uint8_t* status, const int64_t* inc, uint32_t k,
                      int64_t now_ms, uint8_t* applied, uint8_t* new_status, int64_t* new_inc, uint32_t* n_applied) {
    return guard([&] {
        rp::Members& m = MB(h);
        RP_REQUIRE(k == 0 || (ids && status && inc), "update: null change buffers");
        for (uint32_t i = 0; i < k; i++) {
            RP_REQUIRE(ids[i] < m.nt.size(), "update: id was never interned");
            // a member row holds a 61-bit incarnation and a 2-bit status (MRow)
            RP_REQUIRE(inc[i] >= rp::kMemberIncMin && inc[i] <= rp::kMemberIncMax && status[i] < 4,
                       "update: incarnation outside [-2^60, 2^60) or status past leave");
        }
        const uint32_t kk = k ? k : 1;
        m.io_ids.reserve(kk);
        m.io_st.reserve(kk);
        m.io_inc.reserve(kk);
        m.io_app.reserve(kk);
        m.io_nst.reserve(kk);
        m.io_ninc.reserve(kk);
        if (k) {
            RP_HIP(hipMemcpyAsync(m.io_ids.p, ids, 4ull * k, hipMemcpyHostToDevice, m.st));
            RP_HIP(hipMemcpyAsync(m.io_st.p, status, k, hipMemcpyHostToDevice, m.st));
            RP_HIP(hipMemcpyAsync(m.io_inc.p, inc, 8ull * k, hipMemcpyHostToDevice, m.st));
        }
        m.update_dev(m.io_ids.p, m.io_st.p, m.io_inc.p, k, now_ms, m.io_app.p, m.io_nst.p, m.io_ninc.p, nullptr, m.st);
        if (k) {
            if (applied) RP_HIP(hipMemcpyAsync(applied, m.io_app.p, k, hipMemcpyDeviceToHost, m.st));
            if (new_status) RP_HIP(hipMemcpyAsync(new_status, m.io_nst.p, k, hipMemcpyDeviceToHost, m.st));
            if (new_inc) RP_HIP(hipMemcpyAsync(new_inc, m.io_ninc.p, 8ull * k, hipMemcpyDeviceToHost, m.st));
        }
        uint32_t na = 0;
        RP_HIP(hipMemcpyAsync(&na, m.napplied.p, 4, hipMemcpyDeviceToHost, m.st));
        RP_HIP(hipStreamSynchronize(m.st));
        rp::scratch_check(m.ws, m.st);
        if (n_applied) *n_applied = na;
    });
}

int rp_members_set_dev(rp_members* h, const uint32_t* d_ids, const uint8_t* d_status, const int64_t* d_inc,
                       uint32_t k, uint32_t* d_pick, uint32_t* d_npick, void* stream) {
    return guard([&] {
        rp::Members& m = MB(h);
        RP_REQUIRE(k == 0 || (d_ids && d_status && d_inc), "set_dev: null change buffers");
        m.set_dev(d_ids, d_status, d_inc, k, d_pick, d_npick, rp::as_stream(stream));
    });
}

int rp_members_set(rp_members* h, const uint32_t* ids, const uint8_t* status, const int64_t* inc, uint32_t k,
                   uint32_t* pick, uint32_t* npick) {
    return guard([&] {
        rp::Members& m = MB(h);
        RP_REQUIRE(k == 0 || (ids && status && inc), "set: null change buffers");
        for (uint32_t i = 0; i < k; i++) {
            RP_REQUIRE(ids[i] < m.nt.size(), "set: id was never interned");
            RP_REQUIRE(inc[i] >= rp::kMemberIncMin && inc[i] <= rp::kMemberIncMax && status[i] < 4,
                       "set: incarnation outside [-2^60, 2^60) or status past leave");
        }
        const uint32_t kk = k ? k : 1;
        m.io_ids.reserve(kk + 1);
        m.io_st.reserve(kk);
        m.io_inc.reserve(kk);
        m.io_pick.reserve(kk + 1);
        if (k) {
            RP_HIP(hipMemcpyAsync(m.io_ids.p, ids, 4ull * k, hipMemcpyHostToDevice, m.st));
            RP_HIP(hipMemcpyAsync(m.io_st.p, status, k, hipMemcpyHostToDevice, m.st));
            RP_HIP(hipMemcpyAsync(m.io_inc.p, inc, 8ull * k, hipMemcpyHostToDevice, m.st));
        }
        m.set_dev(m.io_ids.p, m.io_st.p, m.io_inc.p, k, m.io_pick.p, m.io_pick.p + kk, m.st);
        uint32_t np = 0;
        RP_HIP(hipMemcpyAsync(&np, m.io_pick.p + kk, 4, hipMemcpyDeviceToHost, m.st));
        RP_HIP(hipStreamSynchronize(m.st));
        rp::scratch_check(m.ws, m.st);
        if (pick && np) RP_HIP(hipMemcpy(pick, m.io_pick.p, 4ull * np, hipMemcpyDeviceToHost));
        if (npick) *npick = np;
    });
}

int rp_members_checksum(rp_members* h, uint32_t* out, int* is_set) {
    return guard([&] {
        rp::Members& m = MB(h);
        m.settle_checksums();
        uint32_t v[2];
        RP_HIP(hipMemcpyAsync(v, m.ck.p, sizeof v, hipMemcpyDeviceToHost, m.st));
        RP_HIP(hipStreamSynchronize(m.st));
        rp::scratch_check(m.ws, m.st);
        if (out) *out = v[0];
        if (is_set) *is_set = v[1] ? 1 : 0;
    });
}

int rp_members_defer_checksum(rp_members* h, int defer) {
    return guard([&] {
        rp::Members& m = MB(h);
        // a deferred batch records no history entry, which would misalign the per-batch record
        RP_REQUIRE(!(defer && m.hist_cap), "defer_checksum: not with a checksum history (checksum_shard)");
        m.defer_ck = defer != 0;
    });
}

int rp_members_checksum_shard(rp_members* h, uint32_t nshards, uint32_t shard, uint32_t history_cap) {
    return guard([&] {
        rp::Members& m = MB(h);
        RP_REQUIRE(nshards >= 1 && shard < nshards, "checksum_shard: shard must be < nshards");
        RP_REQUIRE(!(history_cap && m.defer_ck), "checksum_shard: a history needs per-batch checksums (defer is on)");
        m.settle_checksums();  // pending strings keep the old numbering
        m.ck_nsh = nshards;
        m.ck_sh = shard;
        m.batch_no = 0;
        m.hist_n = 0;
        m.hist_cap = history_cap;
        if (history_cap) m.ck_hist.reserve(2ull * history_cap);
    });
}

int rp_members_checksum_history(rp_members* h, uint32_t* hash, uint8_t* applied, uint32_t cap, uint32_t* n) {
    return guard([&] {
        rp::Members& m = MB(h);
        m.settle_checksums();
        const uint32_t c = std::min(cap, m.hist_n);
        if (c && (hash || applied)) {
            std::vector<uint32_t> v(2ull * c);
            RP_HIP(hipMemcpy(v.data(), m.ck_hist.p, 8ull * c, hipMemcpyDeviceToHost));
            for (uint32_t i = 0; i < c; i++) {
                if (hash) hash[i] = v[2 * i];
                if (applied) applied[i] = v[2 * i + 1] ? 1 : 0;
            }
        }
        if (n) *n = m.hist_n;
    });
}

int rp_members_checksum_history_drain(rp_members* h, uint32_t count) {
    return guard([&] {
        rp::Members& m = MB(h);
        m.settle_checksums();
        RP_REQUIRE(count <= m.hist_n, "checksum_history_drain: count exceeds the recorded entries");
        if (count && count < m.hist_n) {  // keep the entries after the drained ones, in order
            std::vector<uint32_t> v(2ull * (m.hist_n - count));  // (the ranges may overlap)
            RP_HIP(hipMemcpy(v.data(), m.ck_hist.p + 2ull * count, 4ull * v.size(), hipMemcpyDeviceToHost));
            RP_HIP(hipMemcpy(m.ck_hist.p, v.data(), 4ull * v.size(), hipMemcpyHostToDevice));
        }
        m.hist_n -= count;
    });
}

int rp_members_compute_checksum(rp_members* h) {
    return guard([&] {
        rp::Members& m = MB(h);
        m.checksum_dev(m.st, nullptr);
        m.settle_checksums();
    });
}

int rp_members_checksum_string(rp_members* h, char* buf, uint64_t cap, uint64_t* len) {
    return guard([&] {
        rp::Members& m = MB(h);
        const uint32_t n = m.nt.size();
        uint32_t total = 0;
        const uint8_t* str = nullptr;
        if (n) {
            m.checksum_dev(m.st, nullptr);
            str = m.ck_buf.p + m.slot_bytes * m.slot_index(m.npending - 1);
            RP_HIP(hipMemcpyAsync(&total, m.ck_meta.p + 4ull * m.slot_index(m.npending - 1), 4,
                                  hipMemcpyDeviceToHost, m.st));
            RP_HIP(hipStreamSynchronize(m.st));
        }
        const uint64_t L = total ? total - 1 : 0;
        if (len) *len = L;
        const uint64_t c = std::min<uint64_t>(cap, L);
        if (buf && c) {
            RP_HIP(hipMemcpyAsync(buf, str, c, hipMemcpyDeviceToHost, m.st));
            RP_HIP(hipStreamSynchronize(m.st));
        }
        m.settle_checksums();
    });
}

int rp_members_dump(rp_members* h, uint8_t* exists, uint8_t* status, int64_t* inc, uint32_t cap) {
    return guard([&] {
        rp::Members& m = MB(h);
        const uint32_t n = std::min(cap, m.nt.size());
        if (n) {
            rp::DevBuf<uint8_t> de, ds;
            rp::DevBuf<int64_t> di;
            de.reserve(n);
            ds.reserve(n);
            di.reserve(n);
            hipLaunchKernelGGL(rp::k_rows_split, dim3(rp::grid_for(n, 256)), dim3(256), 0, m.st, m.rows.p, n, de.p,
                               ds.p, di.p);
            RP_HIP(hipGetLastError());
            if (exists) RP_HIP(hipMemcpyAsync(exists, de.p, n, hipMemcpyDeviceToHost, m.st));
            if (status) RP_HIP(hipMemcpyAsync(status, ds.p, n, hipMemcpyDeviceToHost, m.st));
            if (inc) RP_HIP(hipMemcpyAsync(inc, di.p, 8ull * n, hipMemcpyDeviceToHost, m.st));
            RP_HIP(hipStreamSynchronize(m.st));
        }
        RP_HIP(hipStreamSynchronize(m.st));
    });
}

int rp_members_count(rp_members* h, uint32_t* n_names) {
    return guard([&] { *n_names = MB(h).nt.size(); });
}

int rp_members_damp_configure(rp_members* h, const rp_damp_config* cfg) {
    return guard([&] {
        rp::Members& m = MB(h);
        RP_REQUIRE(cfg, "damp_configure: null config");
        RP_REQUIRE(cfg->half_life > 0.0, "damp_configure: half_life must be > 0");
        rp::damp::Config c{cfg->enabled, cfg->initial, cfg->min, cfg->max, cfg->penalty, cfg->suppress_limit,
                           cfg->half_life};
        m.damp_configure(c);
    });
}

int rp_members_damp_last(rp_members* h, double* score, uint8_t* exceeded, uint32_t k) {
    return guard([&] {
        rp::Members& m = MB(h);
        RP_REQUIRE(m.damp_on, "damp_last: damp scoring is not configured");
        RP_REQUIRE(k <= m.d_out_k, "damp_last: more changes asked for than the last batch had");
        if (k && score) RP_HIP(hipMemcpyAsync(score, m.d_out.p, 8ull * k, hipMemcpyDeviceToHost, m.st));
        if (k && exceeded) RP_HIP(hipMemcpyAsync(exceeded, m.d_exc.p, k, hipMemcpyDeviceToHost, m.st));
        RP_HIP(hipStreamSynchronize(m.st));
    });
}

int rp_members_damp_decay_dev(rp_members* h, int64_t now_ms, void* stream) {
    return guard([&] {
        rp::Members& m = MB(h);
        RP_REQUIRE(m.damp_on, "damp_decay: damp scoring is not configured");
        hipStream_t s = rp::as_stream(stream);
        if (s != m.st) RP_HIP(hipStreamSynchronize(m.st));
        const uint32_t n = m.nt.size();
        if (n)
            hipLaunchKernelGGL(rp::k_damp_decay, dim3(rp::grid_for(n, 256)), dim3(256), 0, s, m.rows.p, n,
                               m.d_score.p, m.d_last.p, m.d_ts.p, m.dcfg, now_ms);
        RP_HIP(hipGetLastError());
    });
}

int rp_members_damp_decay(rp_members* h, int64_t now_ms) {
    // on the handle's own stream: it is non-blocking, so a launch on the null stream would not
    // be ordered before the reads (damp_dump, the next fold) that run on it
    hipStream_t st = nullptr;
    int rc = guard([&] { st = MB(h).st; });
    if (rc) return rc;
    rc = rp_members_damp_decay_dev(h, now_ms, st);
    if (rc) return rc;
    return guard([&] { RP_HIP(hipStreamSynchronize(MB(h).st)); });
}

int rp_members_damp_dump(rp_members* h, double* score, double* last_score, int64_t* last_ts, uint32_t cap) {
    return guard([&] {
        rp::Members& m = MB(h);
        RP_REQUIRE(m.damp_on, "damp_dump: damp scoring is not configured");
        const uint32_t n = std::min(cap, m.nt.size());
        if (n) {
            if (score) RP_HIP(hipMemcpyAsync(score, m.d_score.p, 8ull * n, hipMemcpyDeviceToHost, m.st));
            if (last_score) RP_HIP(hipMemcpyAsync(last_score, m.d_last.p, 8ull * n, hipMemcpyDeviceToHost, m.st));
            if (last_ts) RP_HIP(hipMemcpyAsync(last_ts, m.d_ts.p, 8ull * n, hipMemcpyDeviceToHost, m.st));
        }
        RP_HIP(hipStreamSynchronize(m.st));
    });
}

}  // extern "C"
