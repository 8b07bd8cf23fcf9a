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

// The batch and table operands of one Membership.update fold.
struct FoldArgs {
    const uint8_t* ch_status;
    const int64_t* ch_inc;
    uint8_t* exists;
    uint8_t* status;
    int64_t* inc;
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
// lastUpdateTimestamp (:115-118).
// Returns the number of changes applied (the caller sums them per wave: one atomic per wave,
// not per address, on the batch's applied counter).
template <class Change>
__device__ __forceinline__ uint32_t fold_address(const FoldArgs& A, uint32_t id, uint32_t c, Change change) {
    const DampArgs& da = A.da;
    bool ex = A.exists[id] != 0;
    uint8_t st = A.status[id];
    int64_t in = A.inc[id];
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
    A.exists[id] = ex ? 1 : 0;
    A.status[id] = st;
    A.inc[id] = in;
    if (da.score) {
        da.score[id] = sc;
        da.last[id] = ls;
        da.ts[id] = lt;
    }
    return napp;
}

// Adds every lane's v to *p with one atomic per wave; called by all lanes of the wave.
__device__ __forceinline__ void wave_atomic_add(uint32_t* p, uint32_t v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(p, v);
}

// Sorted path: one lane per id segment of the (id, arrival)-sorted batch. run_if (may be null):
// skip unless *run_if != 0.
// g_cnt / g_head (non-null after a grouped attempt that overflowed): every id of the batch gets
// its grouped-path entries reset here as well (they are only read by the grouped path), which
// saves the batch a launch.
__global__ void k_fold(const uint32_t* __restrict__ sk, const uint32_t* __restrict__ sv, uint32_t k, FoldArgs A,
                       const uint32_t* __restrict__ run_if, uint32_t* __restrict__ g_cnt = nullptr,
                       uint32_t* __restrict__ g_head = nullptr) {
    if (run_if && *run_if == 0) return;
    const uint32_t gstride = gridDim.x * blockDim.x;
    uint32_t napp = 0;
    for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < k; p += gstride) {
        const uint32_t id = sk[p];
        if (g_cnt) {
            g_cnt[id] = 0;
            g_head[id] = 0xFFFFFFFFu;
        }
        if (p > 0 && sk[p - 1] == id) continue;  // not a segment head
        uint32_t c = 1;
        while (p + c < k && sk[p + c] == id) c++;
        napp += fold_address(A, id, c, [&](uint32_t q) { return sv[p + q]; });
    }
    wave_atomic_add(A.n_applied, napp);
}

// Grouped path (no sort): every change links itself into its address's list (arbitrary order)
// and counts it; an address with more than kGroupMax changes in the batch sets *overflow and
// the batch takes the sorted path instead. cnt / head are all-zero / all-EMPTY between batches
// (each fold resets the entries it used).
constexpr uint32_t kGroupMax = 16;
// Batches up to here take the grouped fold: below it the sorted fold is launch-bound (1e5
// changes: 0.054 vs 0.096 ms per batch); above it the grouped fold's scattered per-address
// atomics and table accesses cost more than the sort saves (4M changes: 1.03 vs 0.68 ms).
constexpr uint32_t kGroupedMaxBatch = 1u << 19;
constexpr uint32_t kGroupEmpty = 0xFFFFFFFFu;

__global__ void k_group_link(const uint32_t* __restrict__ ids, uint32_t k, uint32_t* __restrict__ cnt,
                             uint32_t* __restrict__ head, uint32_t* __restrict__ nxt, uint32_t* __restrict__ overflow) {
    const uint32_t gstride = gridDim.x * blockDim.x;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < k; i += gstride) {
        const uint32_t id = ids[i];
        const uint32_t c = atomicAdd(&cnt[id], 1u);
        nxt[i] = atomicExch(&head[id], i);
        if (c == kGroupMax) *overflow = 1u;
    }
}

// One lane per address: the lane of the address's last-linked change (head) gathers the list,
// puts it in arrival order (insertion sort of at most kGroupMax indices) and folds it; a
// single change folds directly. Then the address's cnt / head entries are reset.
__global__ void k_fold_grouped(const uint32_t* __restrict__ ids, uint32_t k, uint32_t* __restrict__ cnt,
                               uint32_t* __restrict__ head, const uint32_t* __restrict__ nxt,
                               const uint32_t* __restrict__ overflow, FoldArgs A) {
    if (*overflow) return;
    const uint32_t gstride = gridDim.x * blockDim.x;
    uint32_t napp = 0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < k; i += gstride) {
        const uint32_t id = ids[i];
        const uint32_t c = cnt[id];
        if (c == 1) {
            napp += fold_address(A, id, 1, [&](uint32_t) { return i; });
            cnt[id] = 0;
            head[id] = kGroupEmpty;
            continue;
        }
        if (c == 0 || head[id] != i) continue;  // another lane owns this address
        uint32_t idx[kGroupMax];
        uint32_t j = i;
        for (uint32_t q = 0; q < c; q++) {
            uint32_t x = j, r = q;
            while (r > 0 && idx[r - 1] > x) {
                idx[r] = idx[r - 1];
                r--;
            }
            idx[r] = x;
            j = nxt[j];
        }
        napp += fold_address(A, id, c, [&](uint32_t q) { return idx[q]; });
        cnt[id] = 0;
        head[id] = kGroupEmpty;
    }
    wave_atomic_add(A.n_applied, napp);
}

// Membership._decayMembersDampScore (index.js:374-383): decayDampScore on every member
// (member.js:45-66). Reads 17 B and writes 8 B per id.
__global__ void k_damp_decay(const uint8_t* __restrict__ exists, uint32_t n, double* __restrict__ score,
                             const double* __restrict__ last, const int64_t* __restrict__ ts, damp::Config c,
                             int64_t now_ms) {
    const uint32_t gstride = gridDim.x * blockDim.x;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gstride)
        if (exists[i]) score[i] = damp::decayed(c, last[i], ts[i], now_ms);
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
                            const int64_t* __restrict__ chi, uint8_t* __restrict__ exists,
                            uint8_t* __restrict__ status, int64_t* __restrict__ inc, uint32_t* __restrict__ pick,
                            uint32_t* __restrict__ npick, DampArgs da) {
    const uint32_t gstride = gridDim.x * blockDim.x;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < k; i += gstride) {
        if (i == 0 && npick) *npick = pos[k];
        const uint32_t m = mark[i];
        if (!m) continue;
        const uint32_t j = m - 1u, id = ids[j];
        exists[id] = 1;
        status[id] = chs[j];
        inc[id] = chi[j];
        if (da.score) {
            da.score[id] = da.last[id] = da.c.initial;
            da.ts[id] = 0;
        }
        if (pick) pick[pos[i]] = j;
    }
}

// generateChecksumString pieces (index.js:115-120): address + status + incarnation + ';'
__global__ void k_mck_len(const uint32_t* __restrict__ order, uint32_t n, const uint8_t* __restrict__ exists,
                          const uint8_t* __restrict__ status, const int64_t* __restrict__ inc,
                          const uint64_t* __restrict__ noff, const uint32_t* __restrict__ gate,
                          uint32_t* __restrict__ len) {
    if (gate && *gate == 0) return;
    const uint32_t gstride = gridDim.x * blockDim.x;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gstride) {
        const uint32_t id = order[i];
        len[i] = exists[id] ? (uint32_t)(noff[id + 1] - noff[id]) + status_len(status[id]) + dec_len(inc[id]) + 1u : 0u;
    }
}

__global__ void k_mck_write(const uint32_t* __restrict__ order, uint32_t n, const uint8_t* __restrict__ exists,
                            const uint8_t* __restrict__ status, const int64_t* __restrict__ inc,
                            const uint8_t* __restrict__ names, const uint64_t* __restrict__ noff,
                            const uint32_t* __restrict__ pos, const uint32_t* __restrict__ gate,
                            uint8_t* __restrict__ buf) {
    if (gate && *gate == 0) return;
    const uint32_t gstride = gridDim.x * blockDim.x;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gstride) {
        const uint32_t id = order[i];
        if (!exists[id]) continue;
        uint8_t* o = buf + pos[i];
        const uint64_t b = noff[id];
        const uint32_t L = (uint32_t)(noff[id + 1] - b);
        for (uint32_t q = 0; q < L; q++) *o++ = names[b + q];
        const uint8_t st = status[id];
        const uint32_t sl = status_len(st);
        for (uint32_t q = 0; q < sl; q++) *o++ = status_char(st, q);
        const uint32_t dl = dec_len(inc[id]);
        dec_write(inc[id], o, dl);
        o[dl] = ';';
    }
}

// The checksum string in one launch (round 2): a tile of 256 x kMckItems members in address
// order computes its pieces' lengths, finds its byte offset by decoupled look-back over the
// tiles (rp_prims.h), and writes its pieces; the last tile records the slot's meta. This
// replaces k_mck_len + the scan + k_mck_write + k_slot_meta (four launches per checksummed
// batch). Gated off (*gate == 0), every workgroup still takes its ticket and tile 0 records
// the meta.

static bool getenv_on(const char* name) {
    const char* v = getenv(name);
    return v && *v && *v != '0';
}
template <int kMckItems>
__global__ __launch_bounds__(256) void k_mck_build(const uint32_t* __restrict__ order, uint32_t n,
                                                   const uint8_t* __restrict__ exists, const uint8_t* __restrict__ status,
                                                   const int64_t* __restrict__ inc, const uint8_t* __restrict__ names,
                                                   const uint64_t* __restrict__ noff, const uint32_t* __restrict__ gate,
                                                   uint8_t* __restrict__ buf, uint32_t* __restrict__ meta, uint64_t* lb,
                                                   unsigned long long* ctr, unsigned long long tbase, uint64_t tag,
                                                   uint32_t ntiles) {
    __shared__ uint32_t s_tile, s_gate, s_excl;
    __shared__ uint32_t s_wsum[4];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    if (tid == 0) {
        s_tile = (uint32_t)(atomicAdd(ctr, 1ull) - tbase);
        s_gate = gate ? *gate : 1u;
    }
    __syncthreads();
    const uint32_t tile = s_tile;
    if (tile >= ntiles) return;  // a ticket count out of step: never write out of bounds
    if (!s_gate) {
        if (tile == 0 && tid == 0) {
            meta[0] = 0;
            meta[1] = 0;
            meta[3] = 0;
        }
        return;
    }
    const uint32_t i0 = tile * (256u * kMckItems) + (uint32_t)tid * kMckItems;
    uint32_t ids[kMckItems], len[kMckItems];
    uint32_t sum = 0;
#pragma unroll
    for (int j = 0; j < kMckItems; j++) {
        const uint32_t i = i0 + j;
        ids[j] = i < n ? order[i] : 0u;
        len[j] = (i < n && exists[ids[j]])
                     ? (uint32_t)(noff[ids[j] + 1] - noff[ids[j]]) + status_len(status[ids[j]]) + dec_len(inc[ids[j]]) + 1u
                     : 0u;
        sum += len[j];
    }
    // exclusive scan of the threads' sums
    uint32_t x = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) s_wsum[wv] = x;
    __syncthreads();
    uint32_t wbase = 0, total = 0;
#pragma unroll
    for (int w = 0; w < 4; w++) {
        wbase += w < wv ? s_wsum[w] : 0u;
        total += s_wsum[w];
    }
    if (tid == 0) lb_store(lb + tile, tag | (tile == 0 ? kLbP : kLbA) | total);
    if (tid < 64) {
        const uint32_t excl = lookback_wave(lb, tile, tag);
        if (tid == 0) {
            if (tile > 0) lb_store(lb + tile, tag | kLbP | (excl + total));
            s_excl = excl;
            if (tile == ntiles - 1) {
                meta[0] = excl + total;
                meta[1] = 1;
                meta[3] = 0;
            }
        }
    }
    __syncthreads();
    uint32_t pos = s_excl + wbase + x - sum;
#pragma unroll
    for (int j = 0; j < kMckItems; j++) {
        if (len[j]) {
            const uint32_t id = ids[j];
            uint8_t* o = buf + pos;
            const uint64_t b = noff[id];
            const uint32_t L = (uint32_t)(noff[id + 1] - b);
            for (uint32_t q = 0; q < L; q++) *o++ = names[b + q];
            const uint8_t st = status[id];
            const uint32_t sl = status_len(st);
            for (uint32_t q = 0; q < sl; q++) *o++ = status_char(st, q);
            const uint32_t dl = dec_len(inc[id]);
            dec_write(inc[id], o, dl);
            o[dl] = ';';
        }
        pos += len[j];
    }
}

// a pending checksum slot's total (string length + 1) and gate value, captured at build time
__global__ void k_slot_meta(const uint32_t* __restrict__ total, const uint32_t* __restrict__ gate,
                            uint32_t* __restrict__ meta) {
    const uint32_t g = gate ? *gate : 1u;
    meta[0] = g ? *total : 0u;
    meta[1] = g;
    meta[3] = 0;
}

// the group's results in batch order: the membership checksum is the last gated batch's hash
__global__ void k_ck_commit(const uint32_t* __restrict__ meta, uint32_t n, uint32_t* __restrict__ ck) {
    for (uint32_t b = 0; b < n; b++)
        if (meta[4 * b + 1] && meta[4 * b + 3]) {
            ck[0] = meta[4 * b + 2];
            ck[1] = 1;
        }
}

__global__ void k_copy_grow(const uint8_t* __restrict__ a, const uint8_t* __restrict__ b,
                            const int64_t* __restrict__ c, uint32_t n, uint8_t* __restrict__ a2,
                            uint8_t* __restrict__ b2, int64_t* __restrict__ c2, uint32_t n2) {
    const uint32_t gstride = gridDim.x * blockDim.x;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += gstride) {
        a2[i] = i < n ? a[i] : 0;
        b2[i] = i < n ? b[i] : 0;
        c2[i] = i < n ? c[i] : 0;
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
    DevBuf<uint8_t> exists, status;
    DevBuf<int64_t> inc;
    DevBuf<uint32_t> ck;        // [0] checksum, [1] is_set
    DevBuf<uint32_t> napplied;  // per-batch applied count (the checksum gate)
    // Checksum strings wait in slots until read or until a group of slots is pending, then one
    // launch hashes the group side by side (one serial chain per workgroup): a batched caller
    // pays one chain's latency per group instead of per batch. The slots form ngroups groups
    // of group_slots; a full group is hashed on a side stream (ck_st) while the next batches
    // fold and build their strings into the next group, so up to ngroups - 1 groups of chains
    // overlap the folds. Reads flush and wait. The slot count is what fits
    // RP_MEMBERS_CK_BYTES (default 1 GiB of HBM), at most kMaxSlots. Groups of 128: a launch of
    // 128 chains (one workgroup each) takes about as long as one of 64, and the folds and string
    // builds of the next 128 batches take about as long (C3: 1.00-1.07 G updates/s against 0.86
    // with groups of 64, 0.44 with 32; RP_MEMBERS_GROUP_SLOTS overrides).
    static constexpr uint32_t kMaxSlots = 256, kGroupSlots = 128, kMaxGroups = 4;
    uint32_t nslots = 1, group_slots = 1, ngroups = 1;
    DevBuf<uint8_t> ck_buf;   // nslots strings of slot_bytes
    uint64_t slot_bytes = 0;
    DevBuf<uint32_t> ck_meta;  // [kMaxSlots][4]: total, gate, hash, done
    uint32_t npending = 0;     // pending strings in the current group
    uint32_t cur_group = 0;
    hipStream_t pend_st = nullptr;  // the stream the pending strings were built on
    hipStream_t ck_st = nullptr;    // the side stream the chains run on
    hipEvent_t ev_built = nullptr, ev_hashed[kMaxGroups] = {};
    bool group_busy[kMaxGroups] = {};  // this group's last hash may still be running
    uint32_t slot_index(uint32_t j) const { return cur_group * group_slots + j; }
    DevBuf<uint32_t> ck_len, ck_pos;
    DevBuf<uint32_t> sk, sv;
    // the grouped (sort-free) fold: per id change count and list head, per change list link
    // (RP_MEMBERS_SORTED_FOLD=1 always sorts)
    bool grouped_fold = [] {
        const char* e = getenv("RP_MEMBERS_SORTED_FOLD");
        return !(e && *e && *e != '0');
    }();
    DevBuf<uint32_t> g_cnt, g_head, g_nxt;
    uint32_t g_cap = 0;
    uint32_t grouped_max = [] {  // RP_MEMBERS_GROUPED_MAX overrides kGroupedMaxBatch (A/B)
        const char* e = getenv("RP_MEMBERS_GROUPED_MAX");
        return e && *e ? (uint32_t)strtoul(e, nullptr, 10) : kGroupedMaxBatch;
    }();
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
        DevBuf<uint8_t> e2, s2;
        DevBuf<int64_t> i2;
        e2.reserve(nc);
        s2.reserve(nc);
        i2.reserve(nc);
        hipLaunchKernelGGL(k_copy_grow, dim3(grid_for(nc, 256)), dim3(256), 0, st, exists.p, status.p, inc.p, cap,
                           e2.p, s2.p, i2.p, nc);
        RP_HIP(hipGetLastError());
        RP_HIP(hipStreamSynchronize(st));
        exists.swap(e2);
        status.swap(s2);
        inc.swap(i2);
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
    void update_dev(const uint32_t* ids, const uint8_t* chs, const int64_t* chi, uint32_t k, int64_t now_ms,
                    uint8_t* applied, uint8_t* nst, int64_t* ninc, uint32_t* n_applied_out, hipStream_t s) {
        if (s != st) RP_HIP(hipStreamSynchronize(st));
        // napplied[0]: applied count (the checksum gate); [1]: the grouped path overflowed
        RP_HIP(hipMemsetAsync(napplied.p, 0, 2 * sizeof(uint32_t), s));
        if (k) {
            if (damp_on) {
                d_out.reserve(k);
                d_exc.reserve(k);
                d_out_k = k;
            }
            const FoldArgs A{chs, chi, exists.p, status.p, inc.p, local_id, now_ms, applied, nst, ninc, napplied.p,
                             damp_args(true)};
            int bits = 8;
            while (bits < 32 && (1ull << bits) < nt.size()) bits += 8;
            sk.reserve(k);
            sv.reserve(k);
            const unsigned g = grid_for(k, 256);
            if (grouped_fold && k < grouped_max && single_pass_sort(k)) {
                // no sort unless some address has more than kGroupMax changes in the batch; then
                // the sorted path runs instead (its launches are gated on the overflow word)
                if (g_cap < cap) {
                    g_cnt.release();
                    g_head.release();
                    g_cnt.reserve(cap);
                    g_head.reserve(cap);
                    RP_HIP(hipMemsetAsync(g_cnt.p, 0, 4ull * cap, s));
                    RP_HIP(hipMemsetAsync(g_head.p, 0xFF, 4ull * cap, s));
                    g_cap = cap;
                }
                g_nxt.reserve(k);
                uint32_t* ovf = napplied.p + 1;
                hipLaunchKernelGGL(k_group_link, dim3(g), dim3(256), 0, s, ids, k, g_cnt.p, g_head.p, g_nxt.p, ovf);
                hipLaunchKernelGGL(k_fold_grouped, dim3(g), dim3(256), 0, s, ids, k, g_cnt.p, g_head.p, g_nxt.p, ovf,
                                   A);
                RP_HIP(hipGetLastError());
                radix_sort_index(ids, sk.p, sv.p, k, 0, bits, s, ws, ovf);
                hipLaunchKernelGGL(k_fold, dim3(g), dim3(256), 0, s, sk.p, sv.p, k, A, ovf, g_cnt.p, g_head.p);
            } else {
                radix_sort_index(ids, sk.p, sv.p, k, 0, bits, s, ws);
                hipLaunchKernelGGL(k_fold, dim3(g), dim3(256), 0, s, sk.p, sv.p, k, A, nullptr);
            }
            RP_HIP(hipGetLastError());
            if (!defer_ck) checksum_dev(s, napplied.p);
        }
        if (n_applied_out)
            RP_HIP(hipMemcpyAsync(n_applied_out, napplied.p, sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
    }

    // Membership.set over a stash of k changes (arrival order): merge, set, checksum once.
    void set_dev(const uint32_t* ids, const uint8_t* chs, const int64_t* chi, uint32_t k, uint32_t* pick,
                 uint32_t* npick, hipStream_t s) {
        if (s != st) RP_HIP(hipStreamSynchronize(st));
        if (!k) {
            if (npick) RP_HIP(hipMemsetAsync(npick, 0, sizeof(uint32_t), s));
            return;
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
                           exists.p, status.p, inc.p, pick, npick, damp_args(false));
        RP_HIP(hipGetLastError());
        checksum_dev(s, nullptr);
    }

    // Membership.computeChecksum (index.js:48-75) gated on *gate != 0 (null = always): the
    // string is built now (it reflects the table after this batch) into the next slot; its hash
    // lands in ck when the group is flushed.
    void checksum_dev(hipStream_t s, const uint32_t* gate) {
        const uint32_t n = nt.size();
        if (!n) return;
        ck_len.reserve(n + 1);
        ck_pos.reserve(n + 1);
        // worst-case string: names + ';' + "suspect" + 20 digits per member
        const uint64_t need = (nt.h_bytes.size() + (uint64_t)n * 29 + 16 + 255) & ~255ull;
        if (npending && (s != pend_st || need > slot_bytes)) {  // keep the group on one stream
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
            for (auto& b : group_busy) b = false;
            cur_group = 0;
            ck_buf.release();
            const char* e = getenv("RP_MEMBERS_CK_BYTES");
            const uint64_t budget = e && *e ? strtoull(e, nullptr, 10) : (1ull << 30);
            nslots = (uint32_t)std::min<uint64_t>(kMaxSlots, std::max<uint64_t>(1, budget / need));
            const char* gs = getenv("RP_MEMBERS_GROUP_SLOTS");  // A/B: chains per group launch
            const uint32_t gmax = gs && *gs ? (uint32_t)strtoul(gs, nullptr, 10) : kGroupSlots;
            group_slots = std::max<uint32_t>(1, std::min<uint32_t>(gmax, nslots / 2));
            ngroups = std::max<uint32_t>(1, std::min<uint32_t>(kMaxGroups, nslots / group_slots));
            ck_buf.reserve(need * (uint64_t)group_slots * ngroups);
            slot_bytes = need;
        }
        if (npending == group_slots) flush_checksums();
        if (npending == 0 && group_busy[cur_group]) {  // this group's previous strings must be hashed
            RP_HIP(hipStreamWaitEvent(s, ev_hashed[cur_group], 0));
            group_busy[cur_group] = false;
        }
        pend_st = s;
        ck_meta.reserve(4 * kMaxSlots);
        uint8_t* buf = ck_buf.p + slot_bytes * slot_index(npending);
        if (getenv_on("RP_MEMBERS_CK3")) {  // A/B: the three-launch build (lengths, scan, write)
            hipLaunchKernelGGL(k_mck_len, dim3(grid_for(n, 256)), dim3(256), 0, s, nt.sorted.p, n, exists.p,
                               status.p, inc.p, nt.d_noff.p, gate, ck_len.p);
            RP_HIP(hipGetLastError());
            scan_exclusive_u32(ck_len.p, ck_pos.p, n, s, ws);
            hipLaunchKernelGGL(k_mck_write, dim3(grid_for(n, 256)), dim3(256), 0, s, nt.sorted.p, n, exists.p,
                               status.p, inc.p, nt.d_bytes.p, nt.d_noff.p, ck_pos.p, gate, buf);
            hipLaunchKernelGGL(k_slot_meta, dim3(1), dim3(1), 0, s, ck_pos.p + n, gate,
                               ck_meta.p + 4ull * slot_index(npending));
        } else {
            const char* it = getenv("RP_MEMBERS_CK_ITEMS");  // A/B: members per thread
            const int items = it && *it ? atoi(it) : 1;
            const uint32_t per = 256u * (items == 2 ? 2u : items == 4 ? 4u : 1u);
            const uint32_t ntl = (uint32_t)((n + per - 1) / per);
            const LookBack L = lookback_prepare(ws, ntl, 0, s);
#define RP_MCK(I)                                                                                               \
    hipLaunchKernelGGL((k_mck_build<I>), dim3(ntl), dim3(256), 0, s, nt.sorted.p, n, exists.p, status.p, inc.p, \
                       nt.d_bytes.p, nt.d_noff.p, gate, buf, ck_meta.p + 4ull * slot_index(npending), L.words,   \
                       L.ticket, L.tbase, L.tag, ntl)
            if (items == 2)
                RP_MCK(2);
            else if (items == 4)
                RP_MCK(4);
            else
                RP_MCK(1);
#undef RP_MCK
        }
        RP_HIP(hipGetLastError());
        npending++;
    }

    // hash the current group's pending strings (side by side) on the side stream once they are
    // built, then commit the last gated one to ck (groups commit in batch order: one stream)
    void flush_checksums() {
        if (!npending) return;
        RP_HIP(hipEventRecord(ev_built, pend_st));
        RP_HIP(hipStreamWaitEvent(ck_st, ev_built, 0));
        const uint64_t first = slot_index(0);
        hash_long_multi(ck_buf.p + slot_bytes * first, slot_bytes, npending, ck_meta.p + 4 * first, ck_st);
        hipLaunchKernelGGL(k_ck_commit, dim3(1), dim3(1), 0, ck_st, ck_meta.p + 4 * first, npending, ck.p);
        RP_HIP(hipGetLastError());
        RP_HIP(hipEventRecord(ev_hashed[cur_group], ck_st));
        group_busy[cur_group] = true;
        cur_group = (cur_group + 1) % ngroups;
        npending = 0;
    }
    // flush and wait, before a host read of the checksum
    void settle_checksums() {
        flush_checksums();
        if (ck_st) RP_HIP(hipStreamSynchronize(ck_st));
        for (auto& b : group_busy) b = false;
    }
    void release_streams() {
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
        m.napplied.reserve(2);
        RP_HIP(hipMemsetAsync(m.ck.p, 0, 2 * sizeof(uint32_t), m.st));
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
        for (uint32_t i = 0; i < n; i++) {
            const uint32_t id = m.nt.intern(bytes + off[i], off[i + 1] - off[i]);
            if (ids_out) ids_out[i] = id;
        }
        m.grow(m.nt.size());
        m.nt.sort(m.st, m.ws);  // address order for checksums (also uploads the names)
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

int rp_members_update(rp_members* h, const uint32_t* ids, const uint8_t* status, const int64_t* inc, uint32_t k,
                      int64_t now_ms, uint8_t* applied, uint8_t* new_status, int64_t* new_inc, uint32_t* n_applied) {
    return guard([&] {
        rp::Members& m = MB(h);
        RP_REQUIRE(k == 0 || (ids && status && inc), "update: null change buffers");
        for (uint32_t i = 0; i < k; i++) RP_REQUIRE(ids[i] < m.nt.size(), "update: id was never interned");
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
        for (uint32_t i = 0; i < k; i++) RP_REQUIRE(ids[i] < m.nt.size(), "set: id was never interned");
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
        if (out) *out = v[0];
        if (is_set) *is_set = v[1] ? 1 : 0;
    });
}

int rp_members_defer_checksum(rp_members* h, int defer) {
    return guard([&] { MB(h).defer_ck = defer != 0; });
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
            if (exists) RP_HIP(hipMemcpyAsync(exists, m.exists.p, n, hipMemcpyDeviceToHost, m.st));
            if (status) RP_HIP(hipMemcpyAsync(status, m.status.p, n, hipMemcpyDeviceToHost, m.st));
            if (inc) RP_HIP(hipMemcpyAsync(inc, m.inc.p, 8ull * n, hipMemcpyDeviceToHost, m.st));
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
            hipLaunchKernelGGL(rp::k_damp_decay, dim3(rp::grid_for(n, 256)), dim3(256), 0, s, m.exists.p, n,
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
