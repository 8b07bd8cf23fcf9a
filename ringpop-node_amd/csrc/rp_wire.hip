// rp_wire.hip — gossip wire bodies on the device: dissemination change records as JSON.
//
// Encoder: one message = one list of change records, written as the bytes JSON.stringify
// produces for
//   issueAs records      {id, source, sourceIncarnationNumber, address, status, incarnationNumber}
//                        (lib/gossip/dissemination.js:163-170; JSON.stringify drops an undefined
//                        member: per record, an id row starting with NUL, a source of NULL_ID or a
//                        sourceIncarnationNumber of INT64_MIN is left out)
//   fullSync records     {source, address, status, incarnationNumber} (dissemination.js:64-73)
// wrapped as a body (RP_WIRE_BODY_*): a bare array; a ping request {checksum, changes, source,
// sourceIncarnationNumber} (lib/gossip/ping-sender.js:71-76); a ping response {changes}
// (server/protocol/ping.js:45-48); a ping-req request {checksum, changes, source,
// sourceIncarnationNumber, target} (lib/gossip/ping-req-sender.js:75-81); a ping-req response
// {changes, pingStatus, target} (server/protocol/ping-req.js:61-65); a join response {app,
// coordinator, membership, membershipChecksum} (server/protocol/join.js:128-133; membership =
// fullSync records). Ids and offsets are validated on the device before anything is written.
// Three passes over thread-per-record / thread-per-message grids: record lengths -> scans ->
// records written at their final offsets (the same emit routine measures and writes, so
// lengths and bytes cannot disagree).
//
// Decoder: one thread per message parses a changes array, or a body object whose `changes` (or a
// join response's `membership`) member is that array (other members skipped; checksum /
// membershipChecksum, source / coordinator, sourceIncarnationNumber, target, pingStatus
// captured), into per-record columns with addresses interned against the members' name table
// by binary search over its byte-ordered ids. Strings with escapes are rejected (addresses and
// uuids never hold one), numbers must be integral. Count pass -> scan -> fill pass.
#include <climits>
#include <type_traits>

#include "rp_names.h"
#include "rp_swim.h"
#include "../../include/ringpop_amd.h"

namespace rp {
NameTable& members_names(rp_members* m, hipStream_t* st, Scratch** ws);
}

namespace rp {
namespace {

constexpr uint32_t NULL_ID = 0xFFFFFFFFu;

struct Names {
    const uint8_t* bytes;
    const uint64_t* off;
    const uint32_t* sorted;
    uint32_t n;
    const uint32_t* hslot;  // NameTable::hslot (hash index of the names, 8 words a slot)
    uint32_t hmask;
};

// ------------------------------------------------------------------ encoder
struct Sink {
    uint8_t* out;  // null: measure only
    uint32_t n = 0;
    __device__ void lit(const char* s) {
        for (; *s; s++) {
            if (out) out[n] = (uint8_t)*s;
            n++;
        }
    }
    __device__ void bytes(const uint8_t* s, uint32_t len) {
        if (out)
            for (uint32_t i = 0; i < len; i++) out[n + i] = s[i];
        n += len;
    }
    __device__ void name(const Names& nm, uint32_t id) {
        const uint64_t a = nm.off[id], b = nm.off[id + 1];
        bytes(nm.bytes + a, (uint32_t)(b - a));
    }
    __device__ void num(int64_t v) {
        const uint32_t k = dec_len(v);
        if (out) dec_write(v, out + n, k);
        n += k;
    }
    __device__ void status(uint8_t s) {
        const uint32_t k = status_len(s);
        if (out)
            for (uint32_t i = 0; i < k; i++) out[n + i] = status_char(s, i);
        n += k;
    }
    __device__ void str(const Names& nm, uint32_t id) {  // "name"
        lit("\"");
        name(nm, id);
        lit("\"");
    }
};

struct Recs {
    const uint32_t* addr;
    const uint32_t* src;
    const uint8_t* status;
    const int64_t* inc;
    const int64_t* src_inc;
    const uint8_t* ids;  // 36 B per record or null
    int form;            // 0 issueAs, 1 fullSync
};

__device__ void emit_record(Sink& s, const Names& nm, const Recs& R, uint64_t r) {
    s.lit("{");
    if (R.form == 0) {
        if (R.ids && R.ids[r * 36] != 0) {
            s.lit("\"id\":\"");
            s.bytes(R.ids + r * 36, 36);
            s.lit("\",");
        }
        if (R.src[r] != NULL_ID) {
            s.lit("\"source\":");
            s.str(nm, R.src[r]);
            s.lit(",");
        }
        if (R.src_inc && R.src_inc[r] != LLONG_MIN) {
            s.lit("\"sourceIncarnationNumber\":");
            s.num(R.src_inc[r]);
            s.lit(",");
        }
    } else if (R.src[r] != NULL_ID) {
        s.lit("\"source\":");
        s.str(nm, R.src[r]);
        s.lit(",");
    }
    s.lit("\"address\":\"");
    s.name(nm, R.addr[r]);
    s.lit("\",\"status\":\"");
    s.status(R.status[r]);
    s.lit("\",\"incarnationNumber\":");
    s.num(R.inc[r]);
    s.lit("}");
}

enum Body : int { B_ARRAY = 0, B_PING = 1, B_PING_RESP = 2, B_PINGREQ = 3, B_PINGREQ_RESP = 4, B_JOIN_RESP = 5 };

struct Msgs {
    const uint32_t* rec_off;  // n+1
    const uint32_t* checksum;     // ping, ping-req: checksum; join response: membershipChecksum
    const uint32_t* source;       // ping, ping-req: source; join response: coordinator
    const int64_t* source_inc;    // ping, ping-req: sourceIncarnationNumber
    const uint32_t* target;       // ping-req request / response: target
    const uint8_t* ping_status;   // ping-req response: pingStatus
    const uint8_t* app;           // join response: the app name (one for the batch)
    uint32_t app_len;
    int body;
};

__device__ void emit_head(Sink& s, const Names& nm, const Msgs& M, uint32_t m) {
    switch (M.body) {
    case B_PING:
    case B_PINGREQ:
        s.lit("{\"checksum\":");
        s.num((int64_t)M.checksum[m]);
        s.lit(",\"changes\":[");
        break;
    case B_PING_RESP:
    case B_PINGREQ_RESP:
        s.lit("{\"changes\":[");
        break;
    case B_JOIN_RESP:
        s.lit("{\"app\":\"");
        s.bytes(M.app, M.app_len);
        s.lit("\",\"coordinator\":");
        s.str(nm, M.source[m]);
        s.lit(",\"membership\":[");
        break;
    default:
        s.lit("[");
    }
}

__device__ void emit_tail(Sink& s, const Names& nm, const Msgs& M, uint32_t m) {
    switch (M.body) {
    case B_PING:
    case B_PINGREQ:
        s.lit("],\"source\":");
        s.str(nm, M.source[m]);
        s.lit(",\"sourceIncarnationNumber\":");
        s.num(M.source_inc[m]);
        if (M.body == B_PINGREQ) {
            s.lit(",\"target\":");
            s.str(nm, M.target[m]);
        }
        s.lit("}");
        break;
    case B_PING_RESP:
        s.lit("]}");
        break;
    case B_PINGREQ_RESP:
        s.lit("],\"pingStatus\":");
        s.lit(M.ping_status[m] ? "true" : "false");
        s.lit(",\"target\":");
        s.str(nm, M.target[m]);
        s.lit("}");
        break;
    case B_JOIN_RESP:
        s.lit("],\"membershipChecksum\":");
        s.num((int64_t)M.checksum[m]);
        s.lit("}");
        break;
    default:
        s.lit("]");
    }
}

// Everything the encoder indexes with, checked before it writes: *bad = 1 + the first failing
// kind (1 offsets, 2 record address, 3 record source, 4 status, 5 message source / coordinator,
// 6 target).
__global__ void k_validate(Names nm, Recs R, Msgs M, uint32_t n_msgs, uint64_t n_rec, uint32_t* bad) {
    const uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x, gs = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t m = g; m <= n_msgs; m += gs) {
        const bool ok = m == 0 ? M.rec_off[0] == 0
                               : M.rec_off[m] >= M.rec_off[m - 1] && (m < n_msgs || M.rec_off[m] == n_rec);
        if (!ok) atomicMin(bad, 2u);
        if (m == n_msgs) continue;
        const bool src_used = M.body == B_PING || M.body == B_PINGREQ || M.body == B_JOIN_RESP;
        if (src_used && M.source[m] >= nm.n) atomicMin(bad, 6u);
        if ((M.body == B_PINGREQ || M.body == B_PINGREQ_RESP) && M.target[m] >= nm.n) atomicMin(bad, 7u);
    }
    for (uint64_t r = g; r < n_rec; r += gs) {
        if (R.addr[r] >= nm.n) atomicMin(bad, 3u);
        if (R.src[r] >= nm.n && R.src[r] != NULL_ID) atomicMin(bad, 4u);
        if (R.status[r] > 3) atomicMin(bad, 5u);
    }
}

__device__ uint32_t msg_of(const uint32_t* rec_off, uint32_t n_msgs, uint64_t r) {
    // last m with rec_off[m] <= r (empty messages share offsets: pick the one that holds r)
    uint32_t lo = 0, hi = n_msgs;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (rec_off[mid] <= r) lo = mid; else hi = mid;
    }
    return lo;
}

__global__ void k_rec_len(Names nm, Recs R, Msgs M, uint32_t n_msgs, uint64_t n_rec, uint32_t* len) {
    for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < n_rec; r += (uint64_t)gridDim.x * blockDim.x) {
        Sink s{nullptr};
        emit_record(s, nm, R, r);
        const uint32_t m = msg_of(M.rec_off, n_msgs, r);
        len[r] = s.n + (r + 1 < M.rec_off[m + 1] ? 1u : 0u);  // the comma after it
    }
}

__global__ void k_msg_len(Names nm, Msgs M, uint32_t n_msgs, const uint32_t* rec_scan, uint32_t* mlen) {
    for (uint32_t m = blockIdx.x * blockDim.x + threadIdx.x; m < n_msgs; m += gridDim.x * blockDim.x) {
        Sink s{nullptr};
        emit_head(s, nm, M, m);
        emit_tail(s, nm, M, m);
        mlen[m] = s.n + rec_scan[M.rec_off[m + 1]] - rec_scan[M.rec_off[m]];
    }
}

__global__ void k_msg_write(Names nm, Msgs M, uint32_t n_msgs, const uint32_t* moff, const uint32_t* rec_scan,
                            uint8_t* out, uint64_t* out_off) {
    for (uint32_t m = blockIdx.x * blockDim.x + threadIdx.x; m <= n_msgs; m += gridDim.x * blockDim.x) {
        out_off[m] = moff[m];
        if (m == n_msgs || !out) continue;
        Sink h{out + moff[m]};
        emit_head(h, nm, M, m);
        Sink t{out + moff[m] + h.n + rec_scan[M.rec_off[m + 1]] - rec_scan[M.rec_off[m]]};
        emit_tail(t, nm, M, m);
    }
}

__global__ void k_rec_write(Names nm, Recs R, Msgs M, uint32_t n_msgs, uint64_t n_rec, const uint32_t* moff,
                            const uint32_t* rec_scan, uint8_t* out) {
    for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < n_rec; r += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t m = msg_of(M.rec_off, n_msgs, r);
        Sink h{nullptr};
        emit_head(h, nm, M, m);
        uint8_t* p = out + moff[m] + h.n + (rec_scan[r] - rec_scan[M.rec_off[m]]);
        Sink s{p};
        emit_record(s, nm, R, r);
        if (r + 1 < M.rec_off[m + 1]) p[s.n] = ',';
    }
}

// Same records staged through LDS: each thread assembles its record in its own slot (65-dword
// stride, so the 64 lanes' byte writes fall in distinct banks), then the wave stores the 64
// records one after another with consecutive lanes on consecutive bytes — coalesced HBM
// writes instead of 64 scattered byte streams. Records longer than a slot go direct.
constexpr uint32_t kSlot = 260;
constexpr uint32_t kWrThreads = 256;

__global__ __launch_bounds__(kWrThreads) void k_rec_write_lds(Names nm, Recs R, Msgs M, uint32_t n_msgs,
                                                              uint64_t n_rec, const uint32_t* moff,
                                                              const uint32_t* rec_scan, uint8_t* out) {
    __shared__ uint8_t buf[kWrThreads * kSlot];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint8_t* mine = buf + threadIdx.x * kSlot;
    for (uint64_t base = blockIdx.x * (uint64_t)kWrThreads; base < n_rec; base += (uint64_t)gridDim.x * kWrThreads) {
        const uint64_t r = base + threadIdx.x;
        uint32_t len = 0;
        uint64_t dst = 0;
        if (r < n_rec) {
            const uint32_t m = msg_of(M.rec_off, n_msgs, r);
            Sink h{nullptr};
            emit_head(h, nm, M, m);
            dst = moff[m] + h.n + (rec_scan[r] - rec_scan[M.rec_off[m]]);
            const uint32_t full = rec_scan[r + 1] - rec_scan[r];
            const bool comma = r + 1 < M.rec_off[m + 1];
            Sink s{full <= kSlot ? mine : out + dst};
            emit_record(s, nm, R, r);
            if (comma) s.out[s.n] = ',';
            len = full <= kSlot ? full : 0;
        }
        __syncthreads();
        const uint8_t* wbuf = buf + wv * 64 * kSlot;
        for (int j = 0; j < 64; j++) {
            const uint32_t lj = __shfl(len, j);
            const uint64_t dj = ((uint64_t)(uint32_t)__shfl((uint32_t)(dst >> 32), j) << 32) |
                                (uint32_t)__shfl((uint32_t)dst, j);
            const uint8_t* src = wbuf + j * kSlot;
            for (uint32_t b = lane; b < lj; b += 64) out[dj + b] = src[b];
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------ decoder
struct In {
    const uint8_t* buf;
    const uint64_t* msg_off;
};

struct Out {
    uint32_t* cnt;  // count pass: records per message
    const uint32_t* rec_off;
    uint32_t rec_cap;
    uint32_t* addr;
    uint32_t* src;
    uint8_t* status;
    int64_t* inc;
    int64_t* src_inc;
    uint64_t* id_off;
    uint64_t* addr_off;
    uint32_t* addr_len;
    uint64_t* err;  // per message: 0 ok, else 1 + byte offset of the failure
    uint32_t* m_checksum;
    uint32_t* m_source;
    int64_t* m_source_inc;
    uint32_t* m_target;
    uint8_t* m_ping_status;  // 0 false, 1 true, 0xFF absent
};

// name id's bytes == s[0..len): 16 bytes per step, all loads of a step issued together
__device__ bool name_eq(const Names& nm, const uint8_t* s, uint32_t len, uint32_t id) {
    const uint64_t a = nm.off[id];
    if (nm.off[id + 1] - a != len) return false;
    for (uint32_t i = 0; i < len; i += 16) {
        uint32_t d = 0;
#pragma unroll
        for (uint32_t j = 0; j < 16; j++) {
            const uint32_t k = min(i + j, len - 1);
            d |= (uint32_t)(s[k] ^ nm.bytes[a + k]);
        }
        if (d) return false;
    }
    return true;
}

// the interned id of the bytes s[0..len), or NULL_ID: one farmhash32 and, expected, about one
// probe of the names' hash index
__device__ uint32_t name_find(const Names& nm, const uint8_t* s, uint32_t len) {
    uint32_t slot = fh::hash32(fh::PtrSrc{s}, len) & nm.hmask;
    while (true) {
        const uint32_t* w = nm.hslot + (uint64_t)NameTable::kSlotWords * slot;
        const uint32_t id = w[0];
        if (id == NULL_ID || (w[1] == len && name_eq(nm, s, len, id))) return id;
        slot = (slot + 1) & nm.hmask;
    }
}

// s[0..N-1) == k, every byte compared (no early exit), so the loads issue together
template <int N>
__device__ __forceinline__ bool key_eq(const uint8_t* s, const char (&k)[N]) {
    uint32_t d = 0;
#pragma unroll
    for (int i = 0; i < N - 1; i++) d |= (uint32_t)(s[i] ^ (uint8_t)k[i]);
    return d == 0;
}

template <int N>
__device__ bool key_is(const uint8_t* s, uint32_t len, const char (&k)[N]) {
    return len == N - 1 && key_eq(s, k);
}

struct Parser {
    const uint8_t* p;
    uint64_t i, end;
    bool bad = false;
    uint64_t bad_at = 0;

    __device__ void fail() {
        if (!bad) {
            bad = true;
            bad_at = i;
        }
        i = end;
    }
    __device__ void ws() {
        while (i < end && (p[i] == ' ' || p[i] == '\t' || p[i] == '\n' || p[i] == '\r')) i++;
    }
    __device__ bool peek(uint8_t c) {
        ws();
        return i < end && p[i] == c;
    }
    __device__ void expect(uint8_t c) {
        ws();
        if (i < end && p[i] == c) i++; else fail();
    }
    // string without escapes: returns its span
    __device__ void str(uint64_t& s0, uint32_t& len) {
        ws();
        if (i >= end || p[i] != '"') { fail(); s0 = 0; len = 0; return; }
        s0 = ++i;
        while (i < end && p[i] != '"') {
            if (p[i] == '\\' || p[i] < 0x20) { fail(); len = 0; return; }
            i++;
        }
        if (i >= end) { fail(); len = 0; return; }
        len = (uint32_t)(i - s0);
        i++;
    }
    // true / false (1 / 0)
    __device__ uint8_t boolean() {
        ws();
        if (i + 4 <= end && p[i] == 't' && p[i + 1] == 'r' && p[i + 2] == 'u' && p[i + 3] == 'e') {
            i += 4;
            return 1;
        }
        if (i + 5 <= end && p[i] == 'f' && p[i + 1] == 'a' && p[i + 2] == 'l' && p[i + 3] == 's' && p[i + 4] == 'e') {
            i += 5;
            return 0;
        }
        fail();
        return 0;
    }
    __device__ int64_t integer() {
        ws();
        bool neg = false;
        if (i < end && p[i] == '-') { neg = true; i++; }
        uint64_t v = 0;
        int nd = 0;
        while (i < end && p[i] >= '0' && p[i] <= '9') {
            v = v * 10 + (p[i] - '0');
            i++;
            if (++nd > 18) { fail(); return 0; }
        }
        if (nd == 0 || (i < end && (p[i] == '.' || p[i] == 'e' || p[i] == 'E'))) { fail(); return 0; }
        return neg ? -(int64_t)v : (int64_t)v;
    }
    // skip any JSON value (strings without escapes)
    __device__ void skip_value() {
        ws();
        if (i >= end) { fail(); return; }
        const uint8_t c = p[i];
        if (c == '"') {
            uint64_t a; uint32_t l;
            str(a, l);
        } else if (c == '{' || c == '[') {
            int depth = 0;
            while (i < end) {
                const uint8_t d = p[i];
                if (d == '"') {
                    uint64_t a; uint32_t l;
                    str(a, l);
                    continue;
                }
                if (d == '{' || d == '[') depth++;
                else if (d == '}' || d == ']') {
                    if (--depth == 0) { i++; return; }
                }
                i++;
            }
            fail();
        } else {
            while (i < end && p[i] != ',' && p[i] != '}' && p[i] != ']' && p[i] != ' ' && p[i] != '\n' &&
                   p[i] != '\r' && p[i] != '\t')
                i++;
        }
    }
};

__device__ uint8_t status_code(const uint8_t* s, uint32_t len) {
    if (len == 5) return key_eq(s, "alive") ? ST_ALIVE : key_eq(s, "leave") ? ST_LEAVE : 0xFF;
    if (len == 7) return key_eq(s, "suspect") ? ST_SUSPECT : 0xFF;
    if (len == 6) return key_eq(s, "faulty") ? ST_FAULTY : 0xFF;
    return 0xFF;
}

// One change record object; FILL writes column k.
template <bool FILL>
__device__ void parse_record(Parser& P, const Names& nm, const Out& O, uint64_t k, uint64_t kend) {
    P.expect('{');
    uint32_t addr = NULL_ID, src = NULL_ID, alen = 0;
    uint64_t aoff = 0, idoff = ~0ull;
    uint8_t st = 0xFF;
    int64_t inc = 0, sinc = LLONG_MIN;
    bool has_inc = false;
    if (P.peek('}')) {
        P.i++;
    } else {
        while (true) {
            uint64_t ks; uint32_t kl;
            P.str(ks, kl);
            P.expect(':');
            if (P.bad) return;
            const uint8_t* key = P.p + ks;
            if (key_is(key, kl, "address")) {
                P.str(aoff, alen);
                if (FILL && !P.bad) addr = name_find(nm, P.p + aoff, alen);
            } else if (key_is(key, kl, "source")) {
                uint64_t so; uint32_t sl;
                P.str(so, sl);
                if (FILL && !P.bad) src = name_find(nm, P.p + so, sl);
            } else if (key_is(key, kl, "status")) {
                uint64_t so; uint32_t sl;
                P.str(so, sl);
                if (!P.bad) st = status_code(P.p + so, sl);
                if (st == 0xFF) P.fail();
            } else if (key_is(key, kl, "incarnationNumber")) {
                inc = P.integer();
                has_inc = true;
            } else if (key_is(key, kl, "sourceIncarnationNumber")) {
                sinc = P.integer();
            } else if (key_is(key, kl, "id")) {
                uint64_t so; uint32_t sl;
                P.str(so, sl);
                idoff = so;
            } else {
                P.skip_value();
            }
            if (P.bad) return;
            if (P.peek(',')) { P.i++; continue; }
            P.expect('}');
            break;
        }
    }
    if (P.bad) return;
    if (alen == 0 || st == 0xFF || !has_inc) { P.fail(); return; }
    // kend: the count pass's total for this message (0 when it failed there)
    if (FILL && k < kend && k < O.rec_cap) {
        O.addr[k] = addr;
        O.status[k] = st;
        O.inc[k] = inc;
        if (O.src) O.src[k] = src;
        if (O.src_inc) O.src_inc[k] = sinc;
        if (O.id_off) O.id_off[k] = idoff;
        if (O.addr_off) O.addr_off[k] = aoff;
        if (O.addr_len) O.addr_len[k] = alen;
    }
}

template <bool FILL>
__device__ uint32_t parse_changes(Parser& P, const Names& nm, const Out& O, uint64_t k0, uint64_t kend) {
    P.expect('[');
    uint32_t n = 0;
    if (P.peek(']')) { P.i++; return 0; }
    while (!P.bad) {
        parse_record<FILL>(P, nm, O, k0 + n, kend);
        n++;
        if (P.peek(',')) { P.i++; continue; }
        P.expect(']');
        break;
    }
    return n;
}

// The thread parser over message m. !FILL: returns its record count (0 when it does not
// parse) and writes nothing; FILL: writes its records k0.. (below kend, the count it had) and
// the message's error and header outputs.
template <bool FILL>
__device__ uint32_t thread_parse(const In& I, const Names& nm, const Out& O, uint32_t m, uint64_t k0, uint64_t kend) {
    Parser P{I.buf, I.msg_off[m], I.msg_off[m + 1]};
    uint32_t n = 0;
    bool seen = false;
    uint32_t ck = 0, msrc = NULL_ID, mtgt = NULL_ID;
    int64_t msinc = LLONG_MIN;
    uint8_t pst = 0xFF;
    if (P.peek('[')) {
        n = parse_changes<FILL>(P, nm, O, k0, kend);
        seen = true;
    } else {
        P.expect('{');
        if (P.peek('}')) P.i++;
        else
            while (!P.bad) {
                uint64_t ks; uint32_t kl;
                P.str(ks, kl);
                P.expect(':');
                if (P.bad) break;
                const uint8_t* key = P.p + ks;
                if (key_is(key, kl, "changes") || key_is(key, kl, "membership")) {
                    n = parse_changes<FILL>(P, nm, O, k0, kend);
                    seen = true;
                } else if (key_is(key, kl, "checksum") || key_is(key, kl, "membershipChecksum")) {
                    ck = (uint32_t)P.integer();
                } else if (key_is(key, kl, "source") || key_is(key, kl, "coordinator")) {
                    uint64_t so; uint32_t sl;
                    P.str(so, sl);
                    if (FILL && !P.bad) msrc = name_find(nm, P.p + so, sl);
                } else if (key_is(key, kl, "sourceIncarnationNumber")) {
                    msinc = P.integer();
                } else if (key_is(key, kl, "target")) {
                    uint64_t so; uint32_t sl;
                    P.str(so, sl);
                    if (FILL && !P.bad) mtgt = name_find(nm, P.p + so, sl);
                } else if (key_is(key, kl, "pingStatus")) {
                    pst = P.boolean();
                } else {
                    P.skip_value();
                }
                if (P.peek(',')) { P.i++; continue; }
                P.expect('}');
                break;
            }
    }
    P.ws();
    if (!P.bad && P.i != P.end) P.fail();
    if (!P.bad && !seen) P.fail();
    if (P.bad) n = 0;
    if (FILL) {
        O.err[m] = P.bad ? P.bad_at - I.msg_off[m] + 1 : 0;
        if (O.m_checksum) O.m_checksum[m] = ck;
        if (O.m_source) O.m_source[m] = msrc;
        if (O.m_source_inc) O.m_source_inc[m] = msinc;
        if (O.m_target) O.m_target[m] = mtgt;
        if (O.m_ping_status) O.m_ping_status[m] = pst;
    }
    return n;
}

// slow != null: only the messages the wave kernel left (slow[m] != 0)
template <bool FILL>
__global__ void k_decode(In I, Names nm, Out O, uint32_t n_msgs, const uint8_t* __restrict__ slow) {
    for (uint32_t m = blockIdx.x * blockDim.x + threadIdx.x; m < n_msgs; m += gridDim.x * blockDim.x) {
        if (slow && !slow[m]) continue;
        const uint64_t k0 = FILL ? O.rec_off[m] : 0;
        const uint64_t kend = FILL ? O.rec_off[m + 1] : 0;
        const uint32_t n = thread_parse<FILL>(I, nm, O, m, k0, kend);
        if (!FILL) O.cnt[m] = n;
    }
}

// ---- the wave-per-message decoder
//
// One wave stages a message in LDS with coalesced loads, then classifies its bytes 64 at a
// time: a ballot of quotes gives, by a prefix parity, which bytes lie inside strings (the
// grammar has no escapes: any backslash or control byte sends the message to the thread
// parser); the quotes and the structural characters outside strings become a compacted token
// list, and a second ballot pass gives each token's nesting depth. The body object's keys are
// walked wave-uniformly, the records of the changes array are found as the '{' tokens one
// level inside it and parsed one lane per record. Anything the wave parser does not accept
// exactly as the thread parser would (k_decode: its grammar and its error offsets) is left to
// the thread parser: the wave kernel marks it in `slow` and k_decode picks only those up.
constexpr uint32_t kWBuf = 8192;  // message bytes staged per wave (longer: the thread parser)
// Two LDS layouts. The first pass holds up to 1,280 tokens and 512 level tokens in 15.6 KB a
// wave, so ten waves fit a CU (2.30 ms per 640 MB against 2.63 with the full layout's eight:
// profiles/r04/r04m); a message past either bound is left (slow = 2) for a second pass with the
// full layout (2,048 tokens, 1,024 level tokens, 19.7 KB a wave), which hands anything else it
// cannot take to the thread parser as the first pass does.
constexpr uint32_t kWTok = 2048, kWLvl = 1024;   // the full layout
constexpr uint32_t kWTokS = 1280, kWLvlS = 512;  // the first pass
#ifndef RP_WIRE_WAVES_S
#define RP_WIRE_WAVES_S 2
#endif
constexpr int kDecWaves = 4, kDecWavesS = RP_WIRE_WAVES_S;     // waves a workgroup
#ifndef RP_WIRE_MEMBERS
#define RP_WIRE_MEMBERS 0
#endif
#ifndef RP_WIRE_NAME_SPLIT
#define RP_WIRE_NAME_SPLIT 1
#endif
constexpr bool kWaveNameSplit = RP_WIRE_NAME_SPLIT != 0;  // records' names looked up together (3.36 vs 3.58 ms; 0: A/B)
constexpr bool kWaveMembers = RP_WIRE_MEMBERS != 0;  // records parsed a lane per member (-DRP_WIRE_MEMBERS=1; A/B)
#ifndef RP_WIRE_CLS16
#define RP_WIRE_CLS16 1
#endif
constexpr bool kWaveCls16 = RP_WIRE_CLS16 != 0;  // classifier: 16 bytes per lane a step (0: 4 bytes; A/B)
#ifndef RP_WIRE_NIBBLE
#define RP_WIRE_NIBBLE 1
#endif
constexpr bool kWaveNibbleCls = RP_WIRE_NIBBLE != 0;  // byte classes by nibble tables (0: SWAR compares; A/B)
#ifndef RP_WIRE_TOKLOOP
#define RP_WIRE_TOKLOOP 1
#endif
#ifndef RP_WIRE_FUSED_LVL
#define RP_WIRE_FUSED_LVL 1
#endif
constexpr bool kWaveFusedLvl = RP_WIRE_FUSED_LVL != 0;  // level list from the depth pass (0: its own scan; A/B)
#ifndef RP_WIRE_DEPTH4
#define RP_WIRE_DEPTH4 1
#endif
constexpr bool kWaveDepth4 = RP_WIRE_DEPTH4 != 0;  // depth pass: four tokens per lane a step (0: one; A/B)
constexpr bool kWaveTokLoop = RP_WIRE_TOKLOOP != 0;  // token writes: a loop over set bits (0: 16 predicated; A/B)
#ifndef RP_WIRE_ABL
#define RP_WIRE_ABL 0  // timing ablations (results wrong): 1 no body name lookups, 2 no record name lookups
#endif
#ifndef RP_WIRE_BODY_LANES
#define RP_WIRE_BODY_LANES 1
#endif
constexpr bool kWaveBodyLanes = RP_WIRE_BODY_LANES != 0;  // body members a lane each (0: the serial walk; A/B)

// BUF: message bytes staged (a longer message goes to the next pass); HASTC: the tokens'
// characters kept (else read back through pos from the staged bytes)
template <uint32_t TOK, uint32_t LVL, uint32_t BUF = kWBuf, bool HASTC = true>
struct alignas(16) WaveLdsT {
    static constexpr uint32_t kTok = TOK, kLvl = LVL, kBuf = BUF;
    static constexpr bool kHasTc = HASTC;
    alignas(16) uint32_t buf[BUF / 4 + 2];
    uint16_t pos[TOK];   // token byte offset in the message
    int8_t dep[TOK];     // depth before the token ({ [ open, } ] close)
    uint8_t tc[HASTC ? TOK : 4];  // the token's character
    alignas(16) uint16_t lvl[LVL];  // the changes array's level tokens (the classifier's scratch before)
    uint64_t scal[BUF / 64 + 16];  // buffer bytes outside strings that are neither tokens nor
                                    // whitespace (bit sh + i: message byte i)
    uint16_t op1[32], cl2[32];      // openers at depth 1 / closers at depth 2, in order: the k-th pair
    uint16_t sep1[64];              // the body's member separators (',' at depth 1), in order
    alignas(16) uint32_t hprobe[16];  // the body's source / target first probe slots (LDS DMA)
};
using WaveLds = WaveLdsT<kWTok, kWLvl>;
#ifndef RP_WIRE_SMALL2
#define RP_WIRE_SMALL2 1
#endif
// RP_WIRE_SMALL2 (round 4): the first pass with 7 KB of message bytes, 256 level tokens and no
// token characters (12.9 KB a wave: 12 waves a CU) instead of 8 KB / 512 / characters kept
// (15.8 KB: 10 waves a CU)
using WaveLdsS = std::conditional_t<RP_WIRE_SMALL2 != 0, WaveLdsT<kWTokS, 256, 7168, false>, WaveLdsT<kWTokS, kWLvlS>>;

// SWAR over the four bytes of a dword: bit 7 of byte j set where byte j == c
__device__ __forceinline__ uint32_t swar_eq(uint32_t x, uint8_t c) {
    const uint32_t t = x ^ (0x01010101u * c);
    return ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t) & 0x80808080u;
}
// The classifier's byte classes from two nibble-table lookups (v_perm_b32 per 8 entries), for
// the four bytes of x at once: class = LO[x & 15] & HI[x >> 4] with bits 0 '"', 1 ',', 2 ':',
// 3 { } [ ], 4 backslash, 5 space, 6 tab / LF / CR, 7 any byte below 0x20. A byte of no class
// (including every byte >= 0x80) is 0.
__device__ __forceinline__ uint32_t byte_class(uint32_t x) {
    const uint32_t lo = x & 0x0F0F0F0Fu, hi = (x >> 4) & 0x0F0F0F0Fu;
    // LO: 0 A0, 1 80, 2 81, 3-8 80, 9 C0, A C4, B 88, C 92, D C8, E-F 80
    const uint32_t l0 = __builtin_amdgcn_perm(0x80808080u, 0x808180A0u, lo & 0x07070707u);
    const uint32_t l1 = __builtin_amdgcn_perm(0x8080C892u, 0x88C4C080u, lo & 0x07070707u);
    const uint32_t ml = ((lo >> 3) & 0x01010101u) * 0xFFu;
    // HI: 0 C0, 1 80, 2 23, 3 04, 4 00, 5 18, 6 00, 7 08, 8-F 00
    const uint32_t h0 = __builtin_amdgcn_perm(0x08001800u, 0x042380C0u, hi & 0x07070707u);
    const uint32_t mh = ((hi >> 3) & 0x01010101u) * 0xFFu;
    return ((l1 & ml) | (l0 & ~ml)) & (h0 & ~mh);
}
// bit 7 of bytes 0..3 → bits 0..3
__device__ __forceinline__ uint32_t swar_bits(uint32_t m) {
    return ((m >> 7) & 1u) | ((m >> 14) & 2u) | ((m >> 21) & 4u) | ((m >> 28) & 8u);
}
__device__ __forceinline__ bool wave_isws(uint8_t c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }
__device__ __forceinline__ bool wave_isopen(uint8_t c) { return c == '{' || c == '['; }
__device__ __forceinline__ bool wave_isclose(uint8_t c) { return c == '}' || c == ']'; }

// k's bytes as little-endian dwords against w (bytes past k's length ignored): the wave
// decoder reads keys and values as aligned LDS dwords funnel-shifted into place, not bytewise
template <int N>
__device__ __forceinline__ bool words_eq(const uint32_t* w, const char (&k)[N]) {
    uint32_t d = 0;
#pragma unroll
    for (int i = 0; i < (N + 2) / 4; i++) {
        uint32_t kw = 0, m = 0;
#pragma unroll
        for (int j = 0; j < 4; j++)
            if (4 * i + j < N - 1) {
                kw |= (uint32_t)(uint8_t)k[4 * i + j] << (8 * j);
                m |= 0xFFu << (8 * j);
            }
        d |= (w[i] ^ kw) & m;
    }
    return d == 0;
}

// farmhash's byte source over the staged message: byte ib + o of the LDS dwords d
struct LdsSrc {
    const uint32_t* d;
    uint32_t ib;
    __device__ uint32_t w(uint32_t o) const {
        const uint32_t x = ib + o;
        return __builtin_amdgcn_alignbyte(d[(x >> 2) + 1], d[x >> 2], x & 3u);
    }
    __device__ int8_t b(uint32_t o) const {
        const uint32_t x = ib + o;
        return (int8_t)(d[x >> 2] >> (8u * (x & 3u)));
    }
};

// len bytes of a name at g (global, read as the dwords holding them) against the staged bytes
// from ib (LDS dwords), 16 bytes a step
__device__ bool bytes_eq_lds(const uint8_t* gp, const uint32_t* d, uint32_t ib, uint32_t len) {
    const uintptr_t ga = reinterpret_cast<uintptr_t>(gp);
    const uint32_t* g = reinterpret_cast<const uint32_t*>(ga & ~(uintptr_t)3);
    const uint32_t gs = (uint32_t)(ga & 3u), ls = ib & 3u;
    const uint32_t ng = (gs + len + 3) / 4;
    const uint32_t* l = d + (ib >> 2);
    for (uint32_t i = 0; i < len; i += 16) {
        const uint32_t k = i / 4;
        uint32_t G[5], L[5];
#pragma unroll
        for (uint32_t j = 0; j < 5; j++) {
            G[j] = k + j < ng ? g[k + j] : 0u;
            L[j] = l[k + j];
        }
        uint32_t dd = 0;
#pragma unroll
        for (uint32_t j = 0; j < 4; j++) {
            const uint32_t o = i + 4 * j;
            const uint32_t m = o >= len ? 0u : len - o >= 4 ? ~0u : (1u << (8 * (len - o))) - 1u;
            dd |= (__builtin_amdgcn_alignbyte(G[j + 1], G[j], gs) ^ __builtin_amdgcn_alignbyte(L[j + 1], L[j], ls)) & m;
        }
        if (dd) return false;
    }
    return true;
}

// name_find over the staged bytes: the string's first kNameInline bytes are compared with the
// slot's copy (one 32-byte read a probe); only a longer name reads the rest of its bytes.
// name_probe: the probe sequence from a slot whose 32 bytes (a, b) are already loaded; the
// first slot is compared inline, a collision's further probes (rare at load factor <= 1/2) out
// of line.
__device__ __forceinline__ bool name_slot_eq(const Names& nm, const uint32_t* d, uint32_t ib, uint32_t len, uint4 a,
                                             uint4 b) {
    constexpr uint32_t kIn = NameTable::kNameInline;
    const uint32_t* l = d + (ib >> 2);
    uint32_t L[kIn / 4 + 1];
#pragma unroll
    for (uint32_t j = 0; j <= kIn / 4; j++) L[j] = l[j];
    const uint32_t bw[kIn / 4] = {a.w, b.x, b.y, b.z, b.w};
    uint32_t dd = 0;
#pragma unroll
    for (uint32_t j = 0; j < kIn / 4; j++) {
        const uint32_t o = 4 * j;
        const uint32_t m = o >= len ? 0u : len - o >= 4 ? ~0u : (1u << (8 * (len - o))) - 1u;
        dd |= (__builtin_amdgcn_alignbyte(L[j + 1], L[j], ib & 3u) & m) ^ bw[j];
    }
    return a.y == len && dd == 0 && (len <= kIn || bytes_eq_lds(nm.bytes + a.z + kIn, d, ib + kIn, len - kIn));
}

__device__ uint32_t name_probe_more(const Names& nm, const uint32_t* d, uint32_t ib, uint32_t len,
                                                 uint32_t slot) {
    while (true) {
        slot = (slot + 1) & nm.hmask;
        const uint4* w = reinterpret_cast<const uint4*>(nm.hslot + (uint64_t)NameTable::kSlotWords * slot);
        const uint4 a = w[0], b = w[1];
        if (a.x == NULL_ID) return NULL_ID;
        if (name_slot_eq(nm, d, ib, len, a, b)) return a.x;
    }
}

__device__ __forceinline__ uint32_t name_probe(const Names& nm, const uint32_t* d, uint32_t ib, uint32_t len,
                                               uint32_t slot, uint4 a, uint4 b) {
    if (a.x == NULL_ID) return NULL_ID;
    if (name_slot_eq(nm, d, ib, len, a, b)) return a.x;
    return name_probe_more(nm, d, ib, len, slot);
}

__device__ __forceinline__ uint32_t name_slot(const Names& nm, const uint32_t* d, uint32_t ib, uint32_t len) {
    return fh::hash32(LdsSrc{d, ib}, len) & nm.hmask;
}

__device__ uint32_t name_find_lds(const Names& nm, const uint32_t* d, uint32_t ib, uint32_t len) {
    const uint32_t slot = name_slot(nm, d, ib, len);
    const uint4* w = reinterpret_cast<const uint4*>(nm.hslot + (uint64_t)NameTable::kSlotWords * slot);
    return name_probe(nm, d, ib, len, slot, w[0], w[1]);
}

template <class WL>
struct WaveMsg {
    const WL* W;
    const uint8_t* b;  // message byte 0 in LDS
    uint32_t len, ntok;
    uint32_t sh;       // byte 0's offset in the staged dwords
    __device__ uint8_t at(uint32_t i) const { return b[i]; }
    __device__ uint8_t tch(uint32_t t) const {
        if constexpr (WL::kHasTc)
            return W->tc[t];
        else
            return b[W->pos[t]];
    }
    // no scalar byte strictly between byte offsets lo and hi
    __device__ bool clean(uint32_t lo, uint32_t hi) const {
        for (uint32_t i = lo + 1; i < hi;) {
            const uint32_t ib = i + sh;
            const uint64_t w = W->scal[ib >> 6] >> (ib & 63);
            if (w == 0) {
                i += 64u - (ib & 63u);
                continue;
            }
            return (uint32_t)__builtin_ctzll(w) + i >= hi;
        }
        return true;
    }
    // the scalar strictly between tokens t and t + 1: [s, e) without surrounding whitespace;
    // false when it is empty or holds whitespace inside
    __device__ bool scalar(uint32_t t, uint32_t& s, uint32_t& e) const {
        uint32_t lo = W->pos[t] + 1, hi = t + 1 < ntok ? W->pos[t + 1] : len;
        while (lo < hi && wave_isws(at(lo))) lo++;
        while (hi > lo && wave_isws(at(hi - 1))) hi--;
        if (lo == hi) return false;
        for (uint32_t i = lo; i < hi; i++)
            if (wave_isws(at(i))) return false;
        s = lo;
        e = hi;
        return true;
    }
    // Parser::integer over [s, e): -?[0-9]{1,18}
    __device__ bool integer(uint32_t s, uint32_t e, int64_t& v) const {
        bool neg = false;
        if (s < e && at(s) == '-') {
            neg = true;
            s++;
        }
        if (s == e || e - s > 18) return false;
        uint64_t x = 0;
        for (uint32_t i = s; i < e; i++) {
            const uint8_t c = at(i);
            if (c < '0' || c > '9') return false;
            x = x * 10 + (c - '0');
        }
        v = neg ? -(int64_t)x : (int64_t)x;
        return true;
    }
    // The integer strictly between tokens t and t + 1 (Parser::integer after the scalar's
    // whitespace trim). JSON.stringify's form (no whitespace at either end) is read with all
    // its bytes loaded at once; anything else takes scalar() + integer().
    __device__ bool int_tok(uint32_t t, int64_t& v) const {
        const uint32_t lo = W->pos[t] + 1, hi = t + 1 < ntok ? W->pos[t + 1] : len;
        if (hi <= lo || hi - lo > 19 || wave_isws(at(lo)) || wave_isws(at(hi - 1))) {
            uint32_t s, e;
            return scalar(t, s, e) && integer(s, e, v);
        }
        uint32_t w[5];  // up to 23 bytes past the buffer's end stay inside this wave's WaveLds
        words<5>(lo, w);
        uint8_t c[19];
#pragma unroll
        for (int i = 0; i < 19; i++) c[i] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
        const uint32_t n = hi - lo;
        const bool neg = c[0] == '-';
        if (n - (neg ? 1u : 0u) == 0 || n - (neg ? 1u : 0u) > 18) return false;
        uint64_t x = 0;
        bool ok = true;
#pragma unroll
        for (uint32_t i = 0; i < 19; i++) {
            const uint32_t d = (uint32_t)c[i] - '0';
            const bool in = i < n && !(i == 0 && neg);
            ok &= !in || d <= 9;
            x = in ? x * 10 + d : x;
        }
        v = neg ? -(int64_t)x : (int64_t)x;
        return ok;
    }
    // the 4N message bytes from byte o as dwords (aligned LDS reads, funnel-shifted)
    template <int N>
    __device__ __forceinline__ void words(uint32_t o, uint32_t (&w)[N]) const {
        const uint32_t x = sh + o;
        const uint32_t* d = W->buf + (x >> 2);
        uint32_t L[N + 1];
#pragma unroll
        for (int i = 0; i <= N; i++) L[i] = d[i];
#pragma unroll
        for (int i = 0; i < N; i++) w[i] = __builtin_amdgcn_alignbyte(L[i + 1], L[i], x & 3u);
    }
    // a record member's key at byte o, kl bytes: 1 address, 2 source, 3 status, 4 id,
    // 5 incarnationNumber, 6 sourceIncarnationNumber, 0 any other
    __device__ int rec_kind(uint32_t o, uint32_t kl) const {
        uint32_t w[6];
        words<6>(o, w);
        return kl == 7 ? (words_eq(w, "address") ? 1 : 0)
             : kl == 6 ? (words_eq(w, "source") ? 2 : words_eq(w, "status") ? 3 : 0)
             : kl == 2 ? (words_eq(w, "id") ? 4 : 0)
             : kl == 17 ? (words_eq(w, "incarnationNumber") ? 5 : 0)
             : kl == 23 ? (words_eq(w, "sourceIncarnationNumber") ? 6 : 0) : 0;
    }
    // a body member's key (top_kind's codes)
    __device__ int top_kind_w(uint32_t o, uint32_t kl) const {
        uint32_t w[6];
        words<6>(o, w);
        switch (kl) {
            case 7: return words_eq(w, "changes") ? 1 : 0;
            case 10: return words_eq(w, "membership") ? 1 : words_eq(w, "pingStatus") ? 4 : 0;
            case 8: return words_eq(w, "checksum") ? 2 : 0;
            case 18: return words_eq(w, "membershipChecksum") ? 2 : 0;
            case 23: return words_eq(w, "sourceIncarnationNumber") ? 3 : 0;
            case 6: return words_eq(w, "source") ? 5 : words_eq(w, "target") ? 6 : 0;
            case 11: return words_eq(w, "coordinator") ? 5 : 0;
            default: return 0;
        }
    }
    // status_code of the string at byte o
    __device__ uint8_t status(uint32_t o, uint32_t len) const {
        uint32_t w[2];
        words<2>(o, w);
        if (len == 5) return words_eq(w, "alive") ? ST_ALIVE : words_eq(w, "leave") ? ST_LEAVE : 0xFF;
        if (len == 7) return words_eq(w, "suspect") ? ST_SUSPECT : 0xFF;
        if (len == 6) return words_eq(w, "faulty") ? ST_FAULTY : 0xFF;
        return 0xFF;
    }
    // name_find of the string at byte o
    __device__ uint32_t find(const Names& nm, uint32_t o, uint32_t len) const {
        return name_find_lds(nm, W->buf, sh + o, len);
    }
    // the token closing the nested value opened at token t (same depth after it)
    __device__ uint32_t match(uint32_t t) const {
        const int32_t d = W->dep[t];
        for (uint32_t u = t + 1; u < ntok; u++)
            if (W->dep[u] == d + 1 && wave_isclose(tch(u))) return u;
        return ntok;
    }
    // a value starting at token t (after ':' at token t - 1): returns the token after it, or
    // ntok on anything the thread parser would not skip the same way
    __device__ uint32_t skip(uint32_t t) const {
        if (t >= ntok) return ntok;
        const uint8_t c = tch(t);
        if (c == '"') return clean(W->pos[t - 1], W->pos[t]) ? t + 2 : ntok;
        if (wave_isopen(c)) {
            if (!clean(W->pos[t - 1], W->pos[t])) return ntok;
            const uint32_t u = match(t);
            return u < ntok ? u + 1 : ntok;
        }
        uint32_t s, e;
        return scalar(t - 1, s, e) ? t : ntok;  // t is the ',' / '}' after the scalar
    }
};

// A body member's key: 1 changes / membership, 2 checksum / membershipChecksum,
// 3 sourceIncarnationNumber, 4 pingStatus, 5 source / coordinator, 6 target, 0 any other
__device__ int top_kind(const uint8_t* kp, uint32_t kl) {
    switch (kl) {
        case 7: return key_eq(kp, "changes") ? 1 : 0;
        case 10: return key_eq(kp, "membership") ? 1 : key_eq(kp, "pingStatus") ? 4 : 0;
        case 8: return key_eq(kp, "checksum") ? 2 : 0;
        case 18: return key_eq(kp, "membershipChecksum") ? 2 : 0;
        case 23: return key_eq(kp, "sourceIncarnationNumber") ? 3 : 0;
        case 6: return key_eq(kp, "source") ? 5 : key_eq(kp, "target") ? 6 : 0;
        case 11: return key_eq(kp, "coordinator") ? 5 : 0;
        default: return 0;
    }
}

// One record's fields as parsed.
struct RecF {
    uint32_t addr, src, alen;
    uint64_t aoff, idoff;
    uint8_t st;
    int64_t inc, sinc;
};

// One record object, tokens [t0 = '{', t1 = its '}'], parsed by one lane (addresses resolved).
// false: leave the message to the thread parser. Each member's tokens (key, ':', value and
// the separator after it) are read from LDS together, so a member costs about three dependent
// LDS trips: its tokens, then its key's and value's bytes, then the name lookups.
// DEFER: the address is not looked up (the caller looks up every record's address and source
// at once, a name per lane) and the source's byte offset | length << 16 is left in sref.
template <bool DEFER, class WL>
__device__ bool wave_record(const WaveMsg<WL>& M, const Names& nm, uint64_t base, uint32_t t0, uint32_t t1, RecF& f,
                            uint32_t& sref) {
    f.addr = NULL_ID;
    f.src = NULL_ID;
    f.alen = 0;
    f.aoff = 0;
    f.idoff = ~0ull;
    f.st = 0xFF;
    f.inc = 0;
    f.sinc = LLONG_MIN;
    bool has_inc = false;
    const uint16_t* P = M.W->pos;
    uint32_t t = t0 + 1;
    if (t >= t1) return false;  // {} : no address
    while (true) {
        // "key" : value (,|}) — tokens t .. t + 5 (indices past t1 are read but not used:
        // they stay inside this wave's WaveLds)
        if (t + 2 >= t1) return false;
        const uint32_t pm = P[t - 1], p0 = P[t], p1 = P[t + 1], p2 = P[t + 2], p3 = P[t + 3], p4 = P[t + 4],
                       p5 = P[t + 5];
        const uint8_t c0 = M.tch(t), c1 = M.tch(t + 1), c2 = M.tch(t + 2), c3 = M.tch(t + 3), c4 = M.tch(t + 4),
                      c5 = M.tch(t + 5);
        if (!((c0 == '"') & (c1 == '"') & (c2 == ':')) || !M.clean(pm, p0) || !M.clean(p1, p2)) return false;
        // 1 address, 2 source, 3 status, 4 id, 5 incarnationNumber, 6 sourceIncarnationNumber
        const int kind = M.rec_kind(p0 + 1, p1 - p0 - 1);
        uint32_t nx;
        uint8_t cn, cb;  // the separator token's character and the one before it
        uint32_t pb, pn;  // their positions
        if (kind >= 1 && kind <= 4) {
            // a string value: tokens t + 3, t + 4; the separator t + 5
            if (t + 4 >= t1 || c3 != '"' || !M.clean(p2, p3)) return false;
            const uint32_t so = p3 + 1, sl = p4 - so;
            if (kind == 1) {
                f.aoff = base + so;
                f.alen = sl;
                if (!DEFER) f.addr = M.find(nm, so, sl);
            } else if (kind == 2) {
                if (DEFER)
                    sref = so | (sl << 16);
                else
                    f.src = M.find(nm, so, sl);
            } else if (kind == 3) {
                f.st = M.status(so, sl);
                if (f.st == 0xFF) return false;
            } else {
                f.idoff = base + so;
            }
            nx = t + 5;
            cn = c5;
            cb = c4;
            pb = p4;
            pn = p5;
        } else if (kind >= 5) {
            // an integer between tokens t + 2 and t + 3 (the separator)
            int64_t x;
            if (!M.int_tok(t + 2, x)) return false;
            if (kind == 5) {
                f.inc = x;
                has_inc = true;
            } else {
                f.sinc = x;
            }
            nx = t + 3;
            cn = c3;
            cb = c2;
            pb = p2;
            pn = p3;
        } else {
            nx = M.skip(t + 3);
            if (nx > t1) return false;
            cn = M.tch(nx);
            cb = M.tch(nx - 1);
            pb = P[nx - 1];
            pn = P[nx];
        }
        // , or }
        if (nx > t1) return false;
        if (cb != ':' && !M.clean(pb, pn)) return false;
        if (nx == t1) {
            if (cn != '}') return false;
            break;
        }
        if (cn != ',') return false;
        t = nx + 1;
    }
    return f.alen != 0 && f.st != 0xFF && has_inc;
}

// The records of the changes array [arr, arr_end] (nrec <= 64, record depth d + 1) parsed member
// by member, a lane per member (round 4): a message's ~6 members x 32 records run on all 64 lanes
// in about three passes instead of one lane walking each record's members one after another, and
// the address / source name lookups then run one per lane. true: all nrec records parsed into
// out[]. false: the caller runs wave_record per record instead (which accepts or hands the message
// to the thread parser) — on anything it would take a different route for: a nested member value,
// a repeated known key (last one wins), more boundary tokens than fit, any record it would reject.
// LDS: the caller's level-list scan leaves the nb boundary tokens (record opens, member
// separators, record closes) at the top of W.lvl, below nothing of the level list (W.lvl[0,
// 2 nrec - 1), which wave_record needs); the per-record fields go over the W.dep bytes, the array
// being known to hold no nested value (wave_record reads W.dep only for those).
template <class WL>
__device__ bool wave_records_mp(const WaveMsg<WL>& M, WL& W, const Names& nm, uint64_t base, uint32_t nb,
                                uint32_t nrec, RecF* __restrict__ out, uint32_t lane) {
    const uint64_t lt = (1ull << lane) - 1ull;
    static_assert(WL::kTok >= 2048, "the record fields take 1,984 B over W.dep");
    const uint16_t* BT = W.lvl + WL::kLvl - 1;  // boundary i at BT[-i]
    if (nb > WL::kLvl || nb < 2) return false;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    // per-record fields over the W.dep bytes (1,984 of its 2,048)
    uint8_t* R = reinterpret_cast<uint8_t*>(W.dep);
    int64_t* r_inc = reinterpret_cast<int64_t*>(R);
    int64_t* r_sinc = reinterpret_cast<int64_t*>(R + 512);
    uint32_t* r_aref = reinterpret_cast<uint32_t*>(R + 1024);  // address offset | length << 16
    uint32_t* r_sref = reinterpret_cast<uint32_t*>(R + 1280);  // source offset | length << 16, then its id
    uint16_t* r_id = reinterpret_cast<uint16_t*>(R + 1536);
    uint8_t* r_st = R + 1664;
    uint32_t* r_fl = reinterpret_cast<uint32_t*>(R + 1728);  // bit k: known key k seen
    if (lane < nrec) {
        r_fl[lane] = 0;
        r_st[lane] = 0xFF;
        r_aref[lane] = 0;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    // members: boundary i that is a '{' or ',' starts one; its value ends at boundary i + 1
    const uint16_t* P = W.pos;
    uint32_t recbase = 0;
    bool bad = false;
    for (uint32_t i0 = 0; i0 < nb; i0 += 64) {
        const uint32_t i = i0 + lane;
        const bool in = i < nb;
        const uint32_t bt = in ? BT[-(int32_t)i] : 0u;
        const uint8_t bc = in ? M.tch(bt) : (uint8_t)'}';
        const uint64_t mo = __ballot(in && bc == '{');
        const int32_t rec = (int32_t)(recbase + (uint32_t)__popcll(mo & lt)) + ((in && bc == '{') ? 0 : -1);
        recbase += (uint32_t)__popcll(mo);
        if (!in || bc == '}') continue;
        if (i + 1 >= nb || rec < 0 || (uint32_t)rec >= nrec) {
            bad = true;
            continue;
        }
        const uint32_t t = bt + 1, sep = BT[-(int32_t)i - 1];
        if (t + 2 >= sep) {  // {} , {,} ...: no key
            bad = true;
            continue;
        }
        const uint32_t pm = P[t - 1], p0 = P[t], p1 = P[t + 1], p2 = P[t + 2], p3 = P[t + 3], p4 = P[t + 4];
        const uint8_t c0 = M.tch(t), c1 = M.tch(t + 1), c2 = M.tch(t + 2), c3 = M.tch(t + 3);
        if (!((c0 == '"') & (c1 == '"') & (c2 == ':')) || !M.clean(pm, p0) || !M.clean(p1, p2)) {
            bad = true;
            continue;
        }
        const int kind = M.rec_kind(p0 + 1, p1 - p0 - 1);
        uint32_t nx;
        uint32_t vs = 0, vl = 0;  // a string value's offset and length
        int64_t x = 0;
        if (kind >= 1 && kind <= 4) {
            if (c3 != '"' || !M.clean(p2, p3)) {
                bad = true;
                continue;
            }
            vs = p3 + 1;
            vl = p4 - vs;
            nx = t + 5;
        } else if (kind >= 5) {
            if (!M.int_tok(t + 2, x)) {
                bad = true;
                continue;
            }
            nx = t + 3;
        } else {
            nx = M.skip(t + 3);  // a string or a scalar (nested values were refused above)
        }
        if (nx != sep || (M.tch(nx - 1) != ':' && !M.clean(P[nx - 1], P[nx]))) {
            bad = true;
            continue;
        }
        if (kind) {
            const uint32_t old = atomicOr(&r_fl[rec], 1u << kind);
            if (old & (1u << kind)) {  // a repeated key: the thread parser keeps the last one
                bad = true;
                continue;
            }
        }
        if (kind == 1) {
            r_aref[rec] = vs | (vl << 16);
        } else if (kind == 2) {
            r_sref[rec] = vs | (vl << 16);
        } else if (kind == 3) {
            const uint8_t st = M.status(vs, vl);
            if (st == 0xFF) {
                bad = true;
                continue;
            }
            r_st[rec] = st;
        } else if (kind == 4) {
            r_id[rec] = (uint16_t)vs;
        } else if (kind == 5) {
            r_inc[rec] = x;
        } else if (kind == 6) {
            r_sinc[rec] = x;
        }
    }
    if (__ballot(bad) != 0 || recbase != nrec) return false;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    // the source names on lanes nrec .. 2 nrec - 1 when they fit, beside the addresses
    const bool split = 2 * nrec <= 64;
    if (split && lane >= nrec && lane < 2 * nrec) {
        const uint32_t r = lane - nrec;
        if (r_fl[r] & (1u << 2)) {
            const uint32_t sr = r_sref[r];
            r_sref[r] = M.find(nm, sr & 0xFFFFu, sr >> 16);
        }
    }
    uint32_t addr = NULL_ID;
    uint32_t fl = 0, ar = 0;
    if (lane < nrec) {
        fl = r_fl[lane];
        ar = r_aref[lane];
        if (ar >> 16) addr = M.find(nm, ar & 0xFFFFu, ar >> 16);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    bool rok = true;
    if (lane < nrec) {
        RecF f;
        f.addr = addr;
        f.alen = ar >> 16;
        f.aoff = base + (ar & 0xFFFFu);
        f.st = r_st[lane];
        f.inc = (fl & (1u << 5)) ? r_inc[lane] : 0;
        f.sinc = (fl & (1u << 6)) ? r_sinc[lane] : LLONG_MIN;
        f.idoff = (fl & (1u << 4)) ? base + r_id[lane] : ~0ull;
        f.src = NULL_ID;
        if (fl & (1u << 2)) {
            const uint32_t sr = r_sref[lane];
            f.src = split ? sr : M.find(nm, sr & 0xFFFFu, sr >> 16);
        }
        if (!(fl & (1u << 1))) f.aoff = 0;  // as wave_record leaves it with no address member
        rok = f.alen != 0 && f.st != 0xFF && (fl & (1u << 5));
        out[lane] = f;
    }
    return __ballot(!rok) == 0;
}

// Stash slots of message m: [stash_slot(m), stash_slot(m + 1)). An accepted record is at least
// kMinRec bytes ({"address":"x","status":"alive","incarnationNumber":0} is 55), so a message of
// L bytes holds at most L / kMinRec records and floor(off / kMinRec) + m leaves room for them.
constexpr uint64_t kMinRec = 48;
__device__ __forceinline__ uint64_t stash_slot(const In& I, uint32_t m) {
    return (I.msg_off[m] - I.msg_off[0]) / kMinRec + m;
}

__device__ __forceinline__ void rec_write(const Out& O, uint64_t k, uint64_t kend, const RecF& f) {
    if (k < kend && k < O.rec_cap) {
        O.addr[k] = f.addr;
        O.status[k] = f.st;
        O.inc[k] = f.inc;
        if (O.src) O.src[k] = f.src;
        if (O.src_inc) O.src_inc[k] = f.sinc;
        if (O.id_off) O.id_off[k] = f.idoff;
        if (O.addr_off) O.addr_off[k] = f.aoff;
        if (O.addr_len) O.addr_len[k] = f.alen;
    }
}

#ifdef RP_WIRE_PROF
__device__ unsigned long long g_wprof[8];
#define WPROF(k)                                                   \
    do {                                                           \
        const uint64_t t_ = clock64();                             \
        if (lane == 0) atomicAdd(&g_wprof[k], t_ - tprof);         \
        tprof = t_;                                                \
    } while (0)
#else
#define WPROF(k) \
    do {         \
    } while (0)
#endif

// One parse per message: a wave parses a message, resolves its addresses and leaves its
// records in the message's stash slots (slots are laid out from the message byte offsets, so no
// count is needed first) and its count; a scan of the counts gives the record offsets and
// k_decode_place moves the records to them. A message the wave parser does not accept is
// counted by the wave's lane 0 with the thread parser and marked slow; k_decode fills those.
// PASS 0: the only pass; 1: the first of two (a message past the layout's token or level bound
// is marked slow = 2, nothing else done for it); 2: the second (only the messages marked 2)
template <class WL, int WAVES, int PASS>
__global__ __launch_bounds__(64 * WAVES) __attribute__((amdgpu_waves_per_eu(WL::kTok < 2048 ? 3 : 1))) void k_decode_wave(In I, Names nm, Out O, uint32_t n_msgs, uint64_t vb,
                                                            uint64_t ve, RecF* __restrict__ stash,
                                                            uint8_t* __restrict__ slow,
                                                            uint32_t* __restrict__ n_by_waves,
                                                            uint32_t* __restrict__ n_retry) {
    if (PASS == 2 && __builtin_nontemporal_load(n_retry) == 0) return;  // nothing left by the first pass
    __shared__ WL lds[WAVES];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    WL& W = lds[wv];
    const uint64_t lt = (1ull << lane) - 1ull;
    uint32_t nwave = 0;  // messages this wave parsed itself (RP_WIRE_DEBUG)
    uint32_t nmp = 0;    // of them, records parsed a lane per member
    uint32_t nretry = 0;  // PASS 1: messages left to the second pass
    const uint32_t nwaves = gridDim.x * WAVES;
    for (uint32_t m = blockIdx.x * WAVES + wv; m < n_msgs; m += nwaves) {
        if (PASS == 2 && slow[m] != 2) continue;  // wave-uniform
        bool retry = false;  // PASS 1: past this layout's bounds
#ifdef RP_WIRE_PROF
        uint64_t tprof = clock64();
#endif
        const uint64_t b0 = I.msg_off[m], b1 = I.msg_off[m + 1];
        const uint64_t len64 = b1 - b0;
        bool ok = len64 > 0 && len64 <= WL::kBuf;
        retry = PASS == 1 && len64 > WL::kBuf && len64 <= kWBuf;  // the next pass stages up to kWBuf
        const uintptr_t p0 = reinterpret_cast<uintptr_t>(I.buf) + b0;
        const uint32_t sh = (uint32_t)(p0 & 3u);
        const uint32_t len = ok ? (uint32_t)len64 : 0u;
        // stage: dwords wholly inside the batch's bytes [vb, ve) go global -> LDS directly
        // (global_load_lds: no registers held per load, so every load of the message is in
        // flight at once), the few at the batch's edges bytewise through registers
        if (ok) {
            const uintptr_t a0 = p0 - sh;
            const uint32_t nd = (sh + len + 3) / 4;
            uint32_t edge = 0, edge_d = ~0u;
            const int nq = (int)((nd + 63) / 64);
            for (int q = 0; q < nq; q++) {  // not unrolled: no per-q address kept live
                const uint32_t d = lane + 64u * q;
                const uintptr_t a = a0 + 4ull * d;
                if (d < nd) {
                    if (a >= vb && a + 4 <= ve) {
                        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(a), &W.buf[64u * q], 4, 0, 0);
                    } else {  // at most two dwords of the whole batch (its first and last)
                        uint32_t x = 0;
                        for (uint32_t j = 0; j < 4; j++)
                            if (a + j >= p0 && a + j < p0 + len)
                                x |= (uint32_t)(*reinterpret_cast<const uint8_t*>(a + j)) << (8 * j);
                        if (edge_d == ~0u) {
                            edge_d = d;
                            edge = x;
                        } else {
                            W.buf[d] = x;
                        }
                    }
                }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (edge_d != ~0u) W.buf[edge_d] = edge;
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        WPROF(0);
        const uint8_t* B = reinterpret_cast<const uint8_t*>(W.buf) + sh;
        // classify 256 bytes per step, a staged dword per lane, in buffer coordinates (buffer
        // byte sh + i is message byte i): a quote's string parity from the lane's own quotes and
        // a ballot of the lanes with an odd count; the tokens (quotes and structural characters
        // outside strings) compacted by a prefix of the lanes' token counts (three ballots); the
        // scalar bitmap packed from the lanes' nibbles through LDS
        uint32_t ntok = 0, quotes = 0;
        bool bad = false;
        const uint32_t nbd = (sh + len + 3) / 4;
        if (kWaveCls16) {
            // 1 KB per step, 16 staged bytes (four dwords) per lane: one prefix of the lanes'
            // quote parities and one of their token counts (five ballots) per step, and the
            // lane's 16 scalar bits stored straight into the bitmap as a u16
            for (uint32_t d0 = 0; ok && d0 < nbd; d0 += 256) {
                const uint32_t dw0 = d0 + 4u * lane;
                uint4 v = make_uint4(0x20202020u, 0x20202020u, 0x20202020u, 0x20202020u);
                if (dw0 < nbd) v = *reinterpret_cast<const uint4*>(&W.buf[dw0]);  // past nbd: masked below
                uint32_t x[4] = {v.x, v.y, v.z, v.w};
                uint32_t p[4], Qd[4];
                uint32_t par = 0;
                if (4 * dw0 < sh || 4 * dw0 + 16 > sh + len) {  // the message's first / last bytes only
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        const uint32_t dw = dw0 + k;
                        const int lo = min(max((int)sh - (int)(4 * dw), 0), 4);
                        const int hi = min(max((int)(sh + len) - (int)(4 * dw), 0), 4);
                        const uint32_t m_in =
                            (uint32_t)((0x80808080ull << (8 * lo)) & (0x80808080ull >> (8 * (4 - hi))));
                        const uint32_t bm = (m_in >> 7) * 0xFFu;
                        x[k] = (x[k] & bm) | (0x20202020u & ~bm);
                    }
                }
                uint32_t cls[4];
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    cls[k] = kWaveNibbleCls ? byte_class(x[k]) : 0u;
                    const uint32_t Q = kWaveNibbleCls ? (cls[k] << 7) & 0x80808080u : swar_eq(x[k], '"');
                    uint32_t pp = Q ^ (Q << 8);
                    pp ^= pp << 16;
                    p[k] = pp ^ (par ? 0x80808080u : 0u);  // parity of the lane's quotes up to each byte
                    par ^= (pp >> 31) & 1u;
                    Qd[k] = Q;
                }
                const uint64_t Po = __ballot(par);
                const uint32_t pre = (quotes + (uint32_t)__popcll(Po & lt)) & 1u;
                uint32_t tm = 0, sm = 0;
                bool ctrl = false;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const uint32_t Q = Qd[k], xk = x[k], c = cls[k];
                    const uint32_t instr = p[k] ^ (pre ? 0x80808080u : 0u);
                    uint32_t st_any, ws, lt20, bsl;
                    if (kWaveNibbleCls) {  // the class bits (byte_class) as bit 7 of each byte
                        st_any = ((c & 0x0E0E0E0Eu) + 0x7F7F7F7Fu) & 0x80808080u;
                        ws = ((c & 0x60606060u) + 0x7F7F7F7Fu) & 0x80808080u;
                        lt20 = c & 0x80808080u;
                        bsl = (c << 3) & 0x80808080u;
                    } else {
                        const uint32_t xd = xk & 0xDFDFDFDFu;
                        st_any = swar_eq(xd, 0x5B) | swar_eq(xd, 0x5D) | swar_eq(xk, ':') | swar_eq(xk, ',');
                        ws = swar_eq(xk, ' ') | swar_eq(xk, '\t') | swar_eq(xk, '\n') | swar_eq(xk, '\r');
                        lt20 = ~(((xk & 0x7F7F7F7Fu) + 0x60606060u) | xk) & 0x80808080u;
                        bsl = swar_eq(xk, '\\');
                    }
                    const uint32_t structural = st_any & ~instr & ~Q;
                    const uint32_t tokb = Q | structural;
                    const uint32_t str_body = instr & ~Q;
                    ctrl |= ((lt20 & ~(ws & ~str_body)) | bsl) != 0;
                    const uint32_t sb = ~instr & ~tokb & ~ws & 0x80808080u;
                    tm |= swar_bits(tokb) << (4 * k);
                    sm |= swar_bits(sb) << (4 * k);
                }
                bad |= __ballot(ctrl) != 0;
                const uint32_t kc = (uint32_t)__builtin_popcount(tm);
                const uint64_t K0 = __ballot(kc & 1u), K1 = __ballot(kc & 2u), K2 = __ballot(kc & 4u),
                               K3 = __ballot(kc & 8u), K4 = __ballot(kc & 16u);
                uint32_t idx = ntok + (uint32_t)__popcll(K0 & lt) + 2u * (uint32_t)__popcll(K1 & lt) +
                               4u * (uint32_t)__popcll(K2 & lt) + 8u * (uint32_t)__popcll(K3 & lt) +
                               16u * (uint32_t)__popcll(K4 & lt);
                if (kWaveTokLoop) {
                    // a lane's tokens one per iteration (as many iterations as the densest lane has)
                    for (uint32_t mm = tm; mm; mm &= mm - 1u) {
                        const uint32_t j = (uint32_t)__builtin_ctz(mm);
                        const uint32_t w = j < 8 ? (j < 4 ? x[0] : x[1]) : (j < 12 ? x[2] : x[3]);
                        if (idx < WL::kTok) {
                            W.pos[idx] = (uint16_t)(4 * dw0 + j - sh);
                            if constexpr (WL::kHasTc) W.tc[idx] = (uint8_t)(w >> (8 * (j & 3u)));
                        }
                        idx++;
                    }
                } else {
#pragma unroll
                    for (int j = 0; j < 16; j++)
                        if ((tm >> j) & 1u) {
                            if (idx < WL::kTok) {
                                W.pos[idx] = (uint16_t)(4 * dw0 + j - sh);
                                if constexpr (WL::kHasTc) W.tc[idx] = (uint8_t)(x[j >> 2] >> (8 * (j & 3)));
                            }
                            idx++;
                        }
                }
                reinterpret_cast<uint16_t*>(W.scal)[(d0 >> 2) + lane] = (uint16_t)sm;
                ntok += (uint32_t)__popcll(K0) + 2u * (uint32_t)__popcll(K1) + 4u * (uint32_t)__popcll(K2) +
                        8u * (uint32_t)__popcll(K3) + 16u * (uint32_t)__popcll(K4);
                quotes += (uint32_t)__popcll(Po);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
        } else {
            uint8_t* nib = reinterpret_cast<uint8_t*>(W.lvl);
            for (uint32_t d0 = 0; ok && d0 < nbd; d0 += 64) {
                const uint32_t dw = d0 + lane;
                uint32_t x = dw < nbd ? W.buf[dw] : 0x20202020u;
                // the message's bytes of this dword (a neighbour's bytes at either end read as blanks)
                const int lo = min(max((int)sh - (int)(4 * dw), 0), 4);
                const int hi = min(max((int)(sh + len) - (int)(4 * dw), 0), 4);
                const uint32_t m_in = (uint32_t)((0x80808080ull << (8 * lo)) & (0x80808080ull >> (8 * (4 - hi))));
                const uint32_t bm = (m_in >> 7) * 0xFFu;
                x = (x & bm) | (0x20202020u & ~bm);
                // bytes as bit 7 of each byte lane (SWAR)
                const uint32_t Q = swar_eq(x, '"');
                uint32_t p = Q ^ (Q << 8);
                p ^= p << 16;  // bit 7 of byte j: odd number of the lane's quotes up to byte j
                const uint64_t Po = __ballot((p >> 31) & 1u);
                const uint32_t pre = (quotes + (uint32_t)__popcll(Po & lt)) & 1u;
                const uint32_t instr = p ^ (pre ? 0x80808080u : 0u);  // opening quote + body
                const uint32_t xd = x & 0xDFDFDFDFu;                  // { [ → 0x5B, } ] → 0x5D
                const uint32_t structural = (swar_eq(xd, 0x5B) | swar_eq(xd, 0x5D) | swar_eq(x, ':') | swar_eq(x, ',')) &
                                            ~instr & ~Q;
                const uint32_t tokb = Q | structural;
                const uint32_t ws = swar_eq(x, ' ') | swar_eq(x, '\t') | swar_eq(x, '\n') | swar_eq(x, '\r');
                const uint32_t lt20 = ~(((x & 0x7F7F7F7Fu) + 0x60606060u) | x) & 0x80808080u;
                const uint32_t str_body = instr & ~Q;
                const uint32_t ctrlb = (lt20 & ~(ws & ~str_body)) | swar_eq(x, '\\');
                const uint32_t sb = ~instr & ~tokb & ~ws & 0x80808080u;
                const uint32_t tm = swar_bits(tokb), sm = swar_bits(sb);
                const bool ctrl = ctrlb != 0;
                bad |= __ballot(ctrl) != 0;
                const uint32_t k = (uint32_t)__builtin_popcount(tm);
                const uint64_t K0 = __ballot(k & 1u), K1 = __ballot(k & 2u), K2 = __ballot(k & 4u);
                uint32_t idx = ntok + (uint32_t)__popcll(K0 & lt) + 2u * (uint32_t)__popcll(K1 & lt) +
                               4u * (uint32_t)__popcll(K2 & lt);
    #pragma unroll
                for (int j = 0; j < 4; j++)
                    if ((tm >> j) & 1u) {
                        if (idx < WL::kTok) {
                            W.pos[idx] = (uint16_t)(4 * dw + j - sh);
                            if constexpr (WL::kHasTc) W.tc[idx] = (uint8_t)(x >> (8 * j));
                        }
                        idx++;
                    }
                nib[lane] = (uint8_t)sm;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                if (lane < 4) {  // 16 lanes' nibbles → the bitmap word of 64 buffer bytes
                    const uint4 v = *reinterpret_cast<const uint4*>(nib + 16 * lane);
                    uint64_t a = (uint64_t)v.x | ((uint64_t)v.y << 32), c = (uint64_t)v.z | ((uint64_t)v.w << 32);
                    a = (a | (a >> 4)) & 0x00FF00FF00FF00FFull;
                    a = (a | (a >> 8)) & 0x0000FFFF0000FFFFull;
                    a = (a | (a >> 16)) & 0xFFFFFFFFull;
                    c = (c | (c >> 4)) & 0x00FF00FF00FF00FFull;
                    c = (c | (c >> 8)) & 0x0000FFFF0000FFFFull;
                    c = (c | (c >> 16)) & 0xFFFFFFFFull;
                    W.scal[d0 / 16 + lane] = a | (c << 32);
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                ntok += (uint32_t)__popcll(K0) + 2u * (uint32_t)__popcll(K1) + 4u * (uint32_t)__popcll(K2);
                quotes += (uint32_t)__popcll(Po);
            }
        }
        retry = retry || (ok && !bad && ntok > WL::kTok);
        ok = ok && !bad && ntok <= WL::kTok && (quotes & 1u) == 0 && ntok > 0;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        WPROF(1);
        WaveMsg<WL> M{&W, B, len, ntok, sh};
        // depth before every token
        int32_t depth = 0;
        bool neg = false;
        uint32_t nop1 = 0, ncl2 = 0, nsep1 = 0, nlv2 = 0;
        // 256 tokens a step, four per lane (their characters in one LDS read, their depths in one
        // write): the lanes' depth changes (-4..4) prefixed by four ballots; the level / opener /
        // closer / separator lists compacted from per-lane counts (three ballots each, the rare
        // three only in steps that hold one)
        for (uint32_t t0 = 0; kWaveDepth4 && ok && t0 < ntok; t0 += 256) {
            const uint32_t tb = t0 + 4u * lane;
            uint32_t cw = 0x20202020u;
            if constexpr (WL::kHasTc) {
                if (tb < ntok) cw = *reinterpret_cast<const uint32_t*>(&W.tc[tb]);
            } else {
#pragma unroll
                for (int k = 0; k < 4; k++)
                    if (tb + k < ntok) cw = (cw & ~(0xFFu << (8 * k))) | ((uint32_t)M.tch(tb + k) << (8 * k));
            }
            uint32_t op = 0, cl = 0;  // bit k: token tb + k opens / closes
            int32_t pk[4];
            int32_t run = 0;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint8_t c = tb + k < ntok ? (uint8_t)(cw >> (8 * k)) : (uint8_t)' ';
                const bool o = wave_isopen(c), x = wave_isclose(c);
                op |= (o ? 1u : 0u) << k;
                cl |= (x ? 1u : 0u) << k;
                pk[k] = run;
                run += (o ? 1 : 0) - (x ? 1 : 0);
            }
            const uint32_t u = (uint32_t)(run + 4);
            const uint64_t B0 = __ballot(u & 1u), B1 = __ballot(u & 2u), B2 = __ballot(u & 4u), B3 = __ballot(u & 8u);
            const int32_t excl = (int32_t)((uint32_t)__popcll(B0 & lt) + 2u * (uint32_t)__popcll(B1 & lt) +
                                           4u * (uint32_t)__popcll(B2 & lt) + 8u * (uint32_t)__popcll(B3 & lt)) -
                                 4 * (int32_t)lane;
            const int32_t tot = (int32_t)((uint32_t)__popcll(B0) + 2u * (uint32_t)__popcll(B1) +
                                          4u * (uint32_t)__popcll(B2) + 8u * (uint32_t)__popcll(B3)) -
                                4 * 64;
            uint32_t dw = 0, l2 = 0, o1 = 0, c2 = 0, s1 = 0;
            bool bad_d = false;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int32_t d = depth + excl + pk[k];
                const bool v = tb + k < ntok;
                const uint8_t c = (uint8_t)(cw >> (8 * k));
                dw |= (uint32_t)(uint8_t)(int8_t)d << (8 * k);
                const bool x = (cl >> k) & 1u, o = (op >> k) & 1u;
                bad_d |= v && (d < 0 || d > 120 || (x && d < 1));
                l2 |= (v && d == 2 && (c == '{' || c == ',') ? 1u : 0u) << k;
                o1 |= (v && o && d == 1 ? 1u : 0u) << k;
                c2 |= (v && x && d == 2 ? 1u : 0u) << k;
                s1 |= (v && c == ',' && d == 1 ? 1u : 0u) << k;
            }
            if (tb < ntok) *reinterpret_cast<uint32_t*>(&W.dep[tb]) = dw;
            neg |= __ballot(bad_d) != 0;
            // a list's entries of this step: lane counts 0..4 prefixed by three ballots
            auto compact = [&](uint32_t bits, uint32_t& n, uint16_t* list, uint32_t cap) {
                const uint32_t cnt = (uint32_t)__builtin_popcount(bits);
                const uint64_t C0 = __ballot(cnt & 1u), C1 = __ballot(cnt & 2u), C2b = __ballot(cnt & 4u);
                uint32_t i = n + (uint32_t)__popcll(C0 & lt) + 2u * (uint32_t)__popcll(C1 & lt) +
                             4u * (uint32_t)__popcll(C2b & lt);
#pragma unroll
                for (int k = 0; k < 4; k++)
                    if ((bits >> k) & 1u) {
                        if (i < cap) list[i] = (uint16_t)(tb + k);
                        i++;
                    }
                n += (uint32_t)__popcll(C0) + 2u * (uint32_t)__popcll(C1) + 4u * (uint32_t)__popcll(C2b);
            };
            if (kWaveFusedLvl) compact(l2, nlv2, W.lvl, WL::kLvl);
            if (__ballot((o1 | c2 | s1) != 0) != 0) {
                compact(o1, nop1, W.op1, 32);
                compact(c2, ncl2, W.cl2, 32);
                compact(s1, nsep1, W.sep1, 64);
            }
            depth += tot;
        }
        for (uint32_t t0 = 0; !kWaveDepth4 && ok && t0 < ntok; t0 += 64) {
            const uint32_t t = t0 + lane;
            const uint8_t ch = t < ntok ? M.tch(t) : (uint8_t)' ';
            const uint64_t Op = __ballot(t < ntok && wave_isopen(ch));
            const uint64_t Cl = __ballot(t < ntok && wave_isclose(ch));
            const int32_t d = depth + __popcll(Op & lt) - __popcll(Cl & lt);
            if (t < ntok) W.dep[t] = (int8_t)d;
            neg |= __ballot(t < ntok && (d < 0 || d > 120 || (wave_isclose(ch) && d < 1))) != 0;
            const uint64_t O1 = __ballot(t < ntok && wave_isopen(ch) && d == 1);
            const uint64_t C2 = __ballot(t < ntok && wave_isclose(ch) && d == 2);
            const uint32_t io = nop1 + (uint32_t)__popcll(O1 & lt), ic = ncl2 + (uint32_t)__popcll(C2 & lt);
            if (((O1 >> lane) & 1ull) && io < 32) W.op1[io] = (uint16_t)t;
            if (((C2 >> lane) & 1ull) && ic < 32) W.cl2[ic] = (uint16_t)t;
            if (kWaveFusedLvl) {  // the level tokens of a body's depth-1 array, in case it is the changes
                const uint64_t L2 = __ballot(t < ntok && d == 2 && (ch == '{' || ch == ','));
                const uint32_t il = nlv2 + (uint32_t)__popcll(L2 & lt);
                if (((L2 >> lane) & 1ull) && il < WL::kLvl) W.lvl[il] = (uint16_t)t;
                nlv2 += (uint32_t)__popcll(L2);
            }
            const uint64_t S1 = __ballot(t < ntok && ch == ',' && d == 1);
            const uint32_t is = nsep1 + (uint32_t)__popcll(S1 & lt);
            if (((S1 >> lane) & 1ull) && is < 64) W.sep1[is] = (uint16_t)t;
            nsep1 += (uint32_t)__popcll(S1);
            nop1 += (uint32_t)__popcll(O1);
            ncl2 += (uint32_t)__popcll(C2);
            depth += __popcll(Op) - __popcll(Cl);
        }
        ok = ok && !neg && depth == 0 && nop1 <= 32 && nop1 == ncl2;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        WPROF(2);
        // the top level, wave-uniformly: [records] or {key: value, ...}
        uint32_t arr = ntok, arr_end = ntok;  // the changes array's '[' and ']'
        uint32_t ck = 0, msrc = NULL_ID, mtgt = NULL_ID;
        uint32_t href5 = ~0u, href6 = ~0u;  // the body's source / target (offset | length << 16), to look up
        uint32_t hslot = 0;                 // lanes 0 / 1: their name's first slot (DMA'd to W.hprobe)
        auto body_names = [&]() {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the probes' DMA
            uint32_t id = NULL_ID;
            const uint32_t r = lane == 0 ? href5 : lane == 1 ? href6 : ~0u;
            if (r != ~0u) {
                const uint4 a = *reinterpret_cast<const uint4*>(&W.hprobe[4 * lane]);
                const uint4 b = *reinterpret_cast<const uint4*>(&W.hprobe[8 + 4 * lane]);
                id = name_probe(nm, W.buf, sh + (r & 0xFFFFu), r >> 16, hslot, a, b);
            }
            const uint32_t h5 = __shfl(id, 0, 64), h6 = __shfl(id, 1, 64);
            if (href5 != ~0u) msrc = h5;
            if (href6 != ~0u) mtgt = h6;
            href5 = href6 = ~0u;
        };
        int64_t msinc = LLONG_MIN;
        uint8_t pst = 0xFF;
        if (ok) {
            const uint8_t c = M.tch(0);
            ok = M.clean(0xFFFFFFFFu, W.pos[0]);  // only whitespace before the first token
            const uint32_t last = ntok - 1;
            ok = ok && M.clean(W.pos[last], len) && wave_isclose(M.tch(last)) && W.dep[last] == 1;
            if (ok && c == '[') {
                ok = M.tch(last) == ']';
                arr = 0;
                arr_end = last;
            } else if (ok && c == '{' && kWaveBodyLanes && nsep1 < 64) {
                // a lane per body member (member j: after separator j - 1 up to separator j, the
                // last one up to the closing '}'), with the serial walk's checks and its results:
                // the last of a repeated key wins, a repeated or missing changes array fails
                ok = M.tch(last) == '}';
                const uint32_t ns = nsep1;
                const bool act = ok && lane <= ns;
                bool okl = act, isopen = false;
                int kind = -1;
                uint32_t t = 1, e = last, nx = ntok, sref = ~0u, a0 = ntok, a1 = ntok;
                int64_t x = 0;
                uint8_t ps = 0xFF;
                if (act) {
                    t = lane == 0 ? 1u : (uint32_t)W.sep1[lane - 1] + 1u;
                    e = lane < ns ? (uint32_t)W.sep1[lane] : last;
                    const uint8_t c0 = M.tch(t), c1 = M.tch(t + 1), c2 = M.tch(t + 2);
                    okl = t + 2 < e && (c0 == '"') & (c1 == '"') & (c2 == ':') && M.clean(W.pos[t - 1], W.pos[t]) &&
                          M.clean(W.pos[t + 1], W.pos[t + 2]);
                    if (okl) {
                        kind = M.top_kind_w(W.pos[t] + 1, (uint32_t)(W.pos[t + 1] - W.pos[t] - 1));
                        isopen = t + 3 < last && wave_isopen(M.tch(t + 3));
                    }
                }
                // the k-th nested value of a changes / unknown member is the k-th depth-1 opener
                const uint64_t Mo = __ballot(okl && isopen && (kind == 1 || kind == 0));
                if (okl) {
                    const uint32_t v = t + 3;
                    const uint32_t k = (uint32_t)__popcll(Mo & lt);
                    if (kind == 1) {
                        okl = isopen && M.tch(v) == '[' && M.clean(W.pos[v - 1], W.pos[v]) && k < nop1 && W.op1[k] == v;
                        a0 = v;
                        a1 = okl ? (uint32_t)W.cl2[k] : ntok;
                        okl = okl && a1 < last && M.tch(a1) == ']';
                        nx = a1 + 1;
                    } else if (kind == 2 || kind == 3) {
                        okl = M.int_tok(t + 2, x);
                        nx = v;
                    } else if (kind == 4) {
                        uint32_t s0, e0;
                        okl = M.scalar(t + 2, s0, e0);
                        if (okl && e0 - s0 == 4 && B[s0] == 't' && B[s0 + 1] == 'r' && B[s0 + 2] == 'u' && B[s0 + 3] == 'e')
                            ps = 1;
                        else if (okl && e0 - s0 == 5 && B[s0] == 'f' && B[s0 + 1] == 'a' && B[s0 + 2] == 'l' &&
                                 B[s0 + 3] == 's' && B[s0 + 4] == 'e')
                            ps = 0;
                        else
                            okl = false;
                        nx = v;
                    } else if (kind == 5 || kind == 6) {
                        okl = v + 1 < last && M.tch(v) == '"' && M.clean(W.pos[v - 1], W.pos[v]);
                        if (okl) sref = (uint32_t)(W.pos[v] + 1) | ((uint32_t)(W.pos[v + 1] - W.pos[v] - 1) << 16);
                        nx = v + 2;
                    } else if (isopen) {
                        okl = k < nop1 && W.op1[k] == v && M.clean(W.pos[v - 1], W.pos[v]);
                        nx = okl ? (uint32_t)W.cl2[k] + 1u : ntok;
                    } else {
                        nx = M.skip(v);
                    }
                    okl = okl && nx == e && (M.clean(W.pos[nx - 1], W.pos[nx]) || M.tch(nx - 1) == ':');
                }
                const uint64_t K1 = __ballot(okl && kind == 1);
                ok = ok && __ballot(act && !okl) == 0 && __popcll(K1) == 1;
                if (ok) {
                    const int l1 = __builtin_ctzll(K1);
                    arr = __shfl(a0, l1, 64);
                    arr_end = __shfl(a1, l1, 64);
                    const uint64_t K2 = __ballot(kind == 2), K3 = __ballot(kind == 3), K4 = __ballot(kind == 4),
                                   K5 = __ballot(kind == 5), K6 = __ballot(kind == 6);
                    const int w2 = 63 - __builtin_clzll(K2 | 1ull), w3 = 63 - __builtin_clzll(K3 | 1ull),
                              w4 = 63 - __builtin_clzll(K4 | 1ull), w5 = 63 - __builtin_clzll(K5 | 1ull),
                              w6 = 63 - __builtin_clzll(K6 | 1ull);
                    const int64_t x2 = __shfl(x, w2, 64), x3 = __shfl(x, w3, 64);
                    const uint32_t p4 = __shfl((uint32_t)ps, w4, 64);
                    if (K2) ck = (uint32_t)x2;
                    if (K3) msinc = x3;
                    if (K4) pst = (uint8_t)p4;
                    // the source and target names: looked up with the records' names
                    const uint32_t r5 = __shfl(sref, w5, 64), r6 = __shfl(sref, w6, 64);
                    href5 = K5 && !(RP_WIRE_ABL & 1) ? r5 : ~0u;
                    href6 = K6 && !(RP_WIRE_ABL & 1) ? r6 : ~0u;
                    if (href5 != ~0u || href6 != ~0u) {
                        // lanes 0 / 1 hash the source / target and start their first probes' 32-B
                        // slot reads as LDS DMA (no VGPR destination, nothing waits on them until
                        // body_names(), after the records' walk): [a0 a1 b0 b1] in W.hprobe.
                        // Both lanes issue (a dummy slot for a missing name), so the DMA's lane
                        // layout does not depend on the exec mask.
                        const uint32_t la = __builtin_amdgcn_readfirstlane(
                            (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t*)W.hprobe);
                        if (lane < 2) {
                            const uint32_t r = lane == 0 ? href5 : href6;
                            hslot = r != ~0u ? name_slot(nm, W.buf, sh + (r & 0xFFFFu), r >> 16) : 0u;
                            const uint32_t* g = nm.hslot + (uint64_t)NameTable::kSlotWords * hslot;
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
                            asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
                                         :
                                         : "v"(g), "s"(la)
                                         : "memory", "m0");
                            asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
                                         :
                                         : "v"(g + 4), "s"(la + 32u)
                                         : "memory", "m0");
#pragma clang diagnostic pop
                        }
                    }
                }
            } else if (ok && c == '{') {
                ok = M.tch(last) == '}';
                uint32_t t = 1, kop = 0;  // kop: the next depth-1 opener, in walk order
                bool seen = false, closed = false;
                while (ok) {
                    const uint8_t c0 = M.tch(t), c1 = M.tch(t + 1), c2 = M.tch(t + 2);
                    if (t + 2 >= last || !((c0 == '"') & (c1 == '"') & (c2 == ':')) ||
                        !M.clean(W.pos[t - 1], W.pos[t]) || !M.clean(W.pos[t + 1], W.pos[t + 2])) {
                        ok = false;
                        break;
                    }
                    const uint32_t v = t + 3;
                    uint32_t nx = ntok;
                    const int kind = M.top_kind_w(W.pos[t] + 1, (uint32_t)(W.pos[t + 1] - W.pos[t] - 1));
                    if (kind == 1) {
                        if (seen || v >= last || M.tch(v) != '[' || !M.clean(W.pos[v - 1], W.pos[v])) {
                            ok = false;
                            break;
                        }
                        seen = true;
                        arr = v;
                        ok = kop < nop1 && W.op1[kop] == v;  // its ']' is the matching depth-2 closer
                        arr_end = ok ? W.cl2[kop++] : ntok;
                        ok = ok && arr_end < last && M.tch(arr_end) == ']';
                        nx = arr_end + 1;
                    } else if (kind == 2 || kind == 3) {
                        int64_t x;
                        ok = M.int_tok(t + 2, x);
                        if (kind == 3)
                            msinc = x;
                        else
                            ck = (uint32_t)x;
                        nx = v;
                    } else if (kind == 4) {
                        uint32_t s0, e0;
                        ok = M.scalar(t + 2, s0, e0);
                        if (ok && e0 - s0 == 4 && B[s0] == 't' && B[s0 + 1] == 'r' && B[s0 + 2] == 'u' && B[s0 + 3] == 'e')
                            pst = 1;
                        else if (ok && e0 - s0 == 5 && B[s0] == 'f' && B[s0 + 1] == 'a' && B[s0 + 2] == 'l' &&
                                 B[s0 + 3] == 's' && B[s0 + 4] == 'e')
                            pst = 0;
                        else
                            ok = false;
                        nx = v;
                    } else if (kind == 5 || kind == 6) {
                        ok = v + 1 < last && M.tch(v) == '"' && M.clean(W.pos[v - 1], W.pos[v]);
                        if (ok) {
                            const uint32_t so = W.pos[v] + 1, sl = W.pos[v + 1] - so;
                            const uint32_t id = lane == 0 ? M.find(nm, so, sl) : 0u;
                            const uint32_t idb = __shfl(id, 0, 64);
                            if (kind == 6)
                                mtgt = idb;
                            else
                                msrc = idb;
                        }
                        nx = v + 2;
                    } else if (v < last && wave_isopen(M.tch(v))) {  // an unknown member's nested value
                        ok = kop < nop1 && W.op1[kop] == v && M.clean(W.pos[v - 1], W.pos[v]);
                        nx = ok ? W.cl2[kop++] + 1u : ntok;
                    } else {
                        nx = M.skip(v);
                    }
                    if (!ok || nx > last) {
                        ok = false;
                        break;
                    }
                    if (!M.clean(W.pos[nx - 1], W.pos[nx]) && M.tch(nx - 1) != ':') {
                        ok = false;
                        break;
                    }
                    if (nx == last) {
                        closed = true;
                        break;
                    }
                    if (M.tch(nx) != ',') {
                        ok = false;
                        break;
                    }
                    t = nx + 1;
                }
                ok = ok && seen && closed;
            } else {
                ok = false;
            }
        }
        WPROF(3);
        // the changes array: its level tokens are { , { , ... {
        uint32_t nrec = 0;
        uint32_t nb = 0;  // member boundaries (~0: a nested member value)
        uint32_t lv0 = 0;  // the level list is W.lvl[lv0, lv0 + nl)
        if (ok) {
            const int32_t d = W.dep[arr];
            uint32_t nl = 0;
            bool deep = false;
            const bool fused = kWaveFusedLvl && !kWaveMembers && d == 1 && nlv2 <= WL::kLvl;
            if (fused) {
                // the depth pass listed every depth-2 '{' / ',': the changes array's are the run
                // of them between its brackets (counted by two ballot passes over the list)
                uint32_t a0 = 0, a1 = 0;
                for (uint32_t j0 = 0; j0 < nlv2; j0 += 64) {
                    const uint32_t j = j0 + lane;
                    const uint32_t t = j < nlv2 ? (uint32_t)W.lvl[j] : 0xFFFFFFFFu;
                    a0 += (uint32_t)__popcll(__ballot(t <= arr));
                    a1 += (uint32_t)__popcll(__ballot(t < arr_end));
                }
                lv0 = __builtin_amdgcn_readfirstlane(a0);
                nl = __builtin_amdgcn_readfirstlane(a1 - a0);
            }
            for (uint32_t t0 = arr + 1; !fused && t0 < arr_end; t0 += 64) {
                const uint32_t t = t0 + lane;
                const bool in = t < arr_end;
                const int32_t dt = in ? (int32_t)W.dep[t] : 0;
                const bool lv = in && dt == d + 1;
                const uint64_t L = __ballot(lv);
                const uint32_t idx = nl + (uint32_t)__popcll(L & lt);
                if (lv && idx < WL::kLvl) W.lvl[idx] = (uint16_t)t;
                nl += (uint32_t)__popcll(L);
                if (kWaveMembers) {
                    // the member boundaries too: record opens (level d + 1), member separators and
                    // record closes (d + 2), from the top of W.lvl down (never over a level token)
                    const uint8_t c = in ? M.tch(t) : (uint8_t)' ';
                    const bool b = (lv && c == '{') || (in && dt == d + 2 && (c == ',' || c == '}'));
                    deep |= in && dt > d + 2;
                    const uint64_t mb = __ballot(b);
                    const uint32_t ib = nb + (uint32_t)__popcll(mb & lt);
                    if (b && ib + nl < WL::kLvl) W.lvl[WL::kLvl - 1 - ib] = (uint16_t)t;
                    nb += (uint32_t)__popcll(mb);
                }
            }
            nb = (__ballot(deep) != 0 || nl + nb > WL::kLvl) ? ~0u : nb;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            // n records give 2n - 1 level tokens; an empty array none
            if (nl == 0)
                ok = arr_end == arr + 1 && M.clean(W.pos[arr], W.pos[arr_end]);
            else
                ok = nl < WL::kLvl && (nl & 1u) == 1u;
            retry = retry || nl >= WL::kLvl;
            bool pat = true;
            for (uint32_t j = lane; ok && j < nl; j += 64) {
                const uint32_t t = W.lvl[lv0 + j];
                const uint8_t c = M.tch(t);
                pat &= (j & 1u) ? c == ',' : c == '{';
                // a record's last token is its '}', right before the next level token
                if (!(j & 1u)) {
                    const uint32_t nxt = j + 1 < nl ? W.lvl[lv0 + j + 1] : arr_end;
                    pat &= M.tch(nxt - 1) == '}' && W.dep[nxt - 1] == d + 2 && M.clean(W.pos[nxt - 1], W.pos[nxt]);
                    const uint32_t prv = j == 0 ? arr : W.lvl[lv0 + j - 1];
                    // the fused list holds only '{' and ',': no other token may sit between a
                    // record's opener and the '[' or ',' before it
                    pat &= M.clean(W.pos[prv], W.pos[t]) && (!fused || t == prv + 1);
                }
            }
            ok = ok && __ballot(!pat) == 0;
            nrec = ok ? (nl + 1) / 2 : 0;
        }
        WPROF(4);
        // the records, one lane each, parsed into this message's stash slots (its byte range
        // bounds its record count: an accepted record is at least kMinRec bytes)
        const uint64_t s0 = stash_slot(I, m), s1 = stash_slot(I, m + 1);
        ok = ok && nrec <= s1 - s0;
        bool rok = true;
        bool mp = false;
        if constexpr (kWaveMembers && WL::kTok >= 2048) {
            if (ok && nrec > 0 && nrec <= 64)  // a lane per member (wave-uniform)
                mp = wave_records_mp(M, W, nm, b0, nb, nrec, stash + s0, lane);
        }
        nmp += mp ? 1u : 0u;
        if (!mp && kWaveNameSplit && nrec <= 32) {
            // a lane per record, then its address and source names looked up together: lanes
            // [0, nrec) the addresses, [nrec, 2 nrec) the sources
            RecF f;
            uint32_t sref = ~0u;
            if (ok && lane < nrec) {
                const uint32_t t0 = W.lvl[lv0 + 2 * lane];
                const uint32_t t1 = (2 * lane + 1 < (nrec * 2 - 1) ? W.lvl[lv0 + 2 * lane + 1] : arr_end) - 1;
                rok = wave_record<true>(M, nm, b0, t0, t1, f, sref);
            }
            if (href5 != ~0u || href6 != ~0u) body_names();  // their probes landed during the walk
            const uint32_t sx = __shfl(sref, (int)((lane - nrec) & 63u), 64);
            const uint32_t aref = lane < nrec && f.alen ? (uint32_t)(f.aoff - b0) | (f.alen << 16) : ~0u;
            const uint32_t ref = lane < nrec ? aref : lane < 2 * nrec ? sx : ~0u;
            const uint32_t id = ok && ref != ~0u && !(RP_WIRE_ABL & 2) ? M.find(nm, ref & 0xFFFFu, ref >> 16) : NULL_ID;
            const uint32_t sid = __shfl(id, (int)((lane + nrec) & 63u), 64);
            if (ok && lane < nrec) {
                f.addr = id;
                f.src = sref != ~0u ? sid : NULL_ID;
                stash[s0 + lane] = f;
            }
        } else if (!mp) {
            for (uint32_t r = lane; ok && r < nrec; r += 64) {
                const uint32_t t0 = W.lvl[lv0 + 2 * r];
                const uint32_t t1 = (2 * r + 1 < (nrec * 2 - 1) ? W.lvl[lv0 + 2 * r + 1] : arr_end) - 1;
                RecF f;
                uint32_t sref;
                rok &= wave_record<false>(M, nm, b0, t0, t1, f, sref);
                stash[s0 + r] = f;
            }
        }
        ok = ok && __ballot(!rok) == 0;
        if (href5 != ~0u || href6 != ~0u) body_names();  // not taken inside the records' pass
        WPROF(5);
        nwave += ok ? 1u : 0u;
        retry = PASS == 1 && !ok && retry;
        nretry += retry ? 1u : 0u;
        if (lane == 0) {
            slow[m] = ok ? 0 : retry ? 2 : 1;
            // the record count (the thread parser's, 0 when the message does not parse)
            O.cnt[m] = ok ? nrec : retry ? 0u : thread_parse<false>(I, nm, O, m, 0, 0);
            if (ok) {
                O.err[m] = 0;
                if (O.m_checksum) O.m_checksum[m] = ck;
                if (O.m_source) O.m_source[m] = msrc;
                if (O.m_source_inc) O.m_source_inc[m] = msinc;
                if (O.m_target) O.m_target[m] = mtgt;
                if (O.m_ping_status) O.m_ping_status[m] = pst;
            }
        }
        WPROF(6);
        __builtin_amdgcn_wave_barrier();
    }
    if (PASS == 1 && lane == 0 && nretry) atomicAdd(n_retry, nretry);
    if (n_by_waves && lane == 0 && nwave) atomicAdd(n_by_waves, nwave);
    if (n_by_waves && lane == 0 && nmp) atomicAdd(n_by_waves + 1, nmp);
}

// After the scan of the counts: the wave-parsed messages' records from their stash slots to
// their places (a wave per message, a lane per record); the thread parser fills the rest.
__global__ void k_decode_place(In I, Out O, uint32_t n_msgs, const RecF* __restrict__ stash,
                               const uint8_t* __restrict__ slow) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t nw = (gridDim.x * blockDim.x) >> 6;
    for (uint32_t m = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; m < n_msgs; m += nw) {
        if (slow[m]) continue;
        const uint64_t k0 = O.rec_off[m], kend = O.rec_off[m + 1];
        const uint64_t s0 = stash_slot(I, m);
        for (uint64_t r = lane; k0 + r < kend; r += 64) rec_write(O, k0 + r, kend, stash[s0 + r]);
    }
}

__global__ void k_zero_tail(uint32_t* p, uint32_t n) {
    if (threadIdx.x == 0 && blockIdx.x == 0) p[n] = 0;
}

Names names_of(NameTable& nt, hipStream_t st, Scratch& ws) {
    nt.sort(st, ws);
    nt.hash_index(st);
    return Names{nt.d_bytes.p, nt.d_noff.p, nt.sorted.p, nt.size(), nt.hslot.p, (1u << nt.hbits) - 1u};
}

}  // namespace
}  // namespace rp

using rp::guard;

namespace {
const char* const kBad[] = {"", "message record offsets must start at 0, not decrease and end at n_rec",
                            "a record's address is not an interned id", "a record's source is not an interned id",
                            "a record's status is not 0..3", "a message's source / coordinator is not an interned id",
                            "a message's target is not an interned id"};
}  // namespace

extern "C" {

int rp_wire_encode_dev(rp_members* m, uint32_t n_msgs, const uint32_t* d_msg_rec_off, uint64_t n_rec,
                       const rp_wire_records* recs, int form, int body, const rp_wire_headers* hdr, uint8_t* d_out,
                       uint64_t* d_out_off, void* stream) {
    return guard([&] {
        RP_REQUIRE(m, "null members handle");
        RP_REQUIRE(form == 0 || form == 1, "form must be 0 (issueAs) or 1 (fullSync)");
        RP_REQUIRE(body >= RP_WIRE_BODY_ARRAY && body <= RP_WIRE_BODY_JOIN_RESPONSE, "unknown body");
        RP_REQUIRE(d_msg_rec_off && d_out_off, "null offsets");
        const rp_wire_records R0 = recs ? *recs : rp_wire_records{};
        const rp_wire_headers H0 = hdr ? *hdr : rp_wire_headers{};
        RP_REQUIRE(n_rec == 0 || (R0.addr && R0.src && R0.status && R0.inc), "null record column");
        const bool need_src = body == RP_WIRE_BODY_PING || body == RP_WIRE_BODY_PINGREQ ||
                              body == RP_WIRE_BODY_JOIN_RESPONSE;
        RP_REQUIRE(n_msgs == 0 || !need_src || (H0.source && H0.checksum), "this body needs source and checksum columns");
        RP_REQUIRE(n_msgs == 0 || !(body == RP_WIRE_BODY_PING || body == RP_WIRE_BODY_PINGREQ) || H0.source_inc,
                   "this body needs the sourceIncarnationNumber column");
        RP_REQUIRE(n_msgs == 0 || !(body == RP_WIRE_BODY_PINGREQ || body == RP_WIRE_BODY_PINGREQ_RESPONSE) || H0.target,
                   "this body needs the target column");
        RP_REQUIRE(n_msgs == 0 || body != RP_WIRE_BODY_PINGREQ_RESPONSE || H0.ping_status,
                   "the ping-req response needs the pingStatus column");
        RP_REQUIRE(body != RP_WIRE_BODY_JOIN_RESPONSE || H0.app || H0.app_len == 0, "null app");
        hipStream_t hst;
        rp::Scratch* ws;
        rp::NameTable& nt = rp::members_names(m, &hst, &ws);
        hipStream_t st = stream ? rp::as_stream(stream) : hst;
        // every byte offset fits u32: bound the worst case on the host
        const uint64_t rec_max = 180 + 2ull * nt.max_len;
        RP_REQUIRE(n_rec * rec_max + (uint64_t)n_msgs * (120 + 2ull * nt.max_len + H0.app_len) < 0xFFFFFFFFull,
                   "encoded batch may exceed 4 GiB: split it");
        rp::Names nm = rp::names_of(nt, st, *ws);
        rp::DevBuf<uint8_t> app;
        app.reserve(H0.app_len + 1);
        if (H0.app_len) RP_HIP(hipMemcpyAsync(app.p, H0.app, H0.app_len, hipMemcpyHostToDevice, st));
        rp::Recs R{R0.addr, R0.src, R0.status, R0.inc, R0.src_inc, R0.ids, form};
        rp::Msgs M{d_msg_rec_off, H0.checksum, H0.source, H0.source_inc, H0.target, H0.ping_status, app.p,
                   H0.app_len, body};
        rp::DevBuf<uint32_t> rscan, mscan, bad;
        bad.reserve(1);
        RP_HIP(hipMemsetAsync(bad.p, 0xFF, 4, st));
        hipLaunchKernelGGL(rp::k_validate, dim3(rp::grid_for(std::max<uint64_t>(n_rec, (uint64_t)n_msgs + 1), 256, 4096)),
                           dim3(256), 0, st, nm, R, M, n_msgs, n_rec, bad.p);
        RP_HIP(hipGetLastError());
        uint32_t b = 0;
        RP_HIP(hipMemcpyAsync(&b, bad.p, 4, hipMemcpyDeviceToHost, st));
        RP_HIP(hipStreamSynchronize(st));
        if (b != 0xFFFFFFFFu) throw rp::Error(rp::RP_EINVAL, std::string("wire encode: ") + kBad[b - 1]);
        rscan.reserve(n_rec + 1);
        mscan.reserve((uint64_t)n_msgs + 1);
        if (n_rec) {
            hipLaunchKernelGGL(rp::k_rec_len, dim3(rp::grid_for(n_rec, 256)), dim3(256), 0, st, nm, R, M, n_msgs,
                               n_rec, rscan.p);
            RP_HIP(hipGetLastError());
        }
        rp::scan_exclusive_u32(rscan.p, rscan.p, n_rec, st, *ws);
        if (n_msgs) {
            hipLaunchKernelGGL(rp::k_msg_len, dim3(rp::grid_for(n_msgs, 256)), dim3(256), 0, st, nm, M, n_msgs,
                               rscan.p, mscan.p);
            RP_HIP(hipGetLastError());
        }
        rp::scan_exclusive_u32(mscan.p, mscan.p, n_msgs, st, *ws);
        hipLaunchKernelGGL(rp::k_msg_write, dim3(rp::grid_for((uint64_t)n_msgs + 1, 256)), dim3(256), 0, st, nm, M,
                           n_msgs, mscan.p, rscan.p, d_out, d_out_off);
        RP_HIP(hipGetLastError());
        if (d_out && n_rec) {
            hipLaunchKernelGGL(rp::k_rec_write_lds,
                               dim3(rp::grid_for(n_rec, rp::kWrThreads,
                                                 (unsigned)rp::env_pos("RP_WIRE_WGRID", 4096u))),
                               dim3(rp::kWrThreads), 0, st, nm, R, M, n_msgs, n_rec, mscan.p, rscan.p, d_out);
            RP_HIP(hipGetLastError());
        }
        RP_HIP(hipStreamSynchronize(st));  // scratch buffers are local
    });
}

int rp_wire_decode_dev(rp_members* m, const uint8_t* d_buf, const uint64_t* d_msg_off, uint32_t n_msgs,
                       uint32_t* d_msg_rec_off, uint32_t rec_cap, const rp_wire_records_out* recs,
                       const rp_wire_headers_out* hdr, uint64_t* d_err, void* stream) {
    return guard([&] {
        RP_REQUIRE(m, "null members handle");
        RP_REQUIRE(d_msg_off && d_msg_rec_off && d_err, "null message offsets / errors");
        const rp_wire_records_out R = recs ? *recs : rp_wire_records_out{};
        const rp_wire_headers_out H = hdr ? *hdr : rp_wire_headers_out{};
        RP_REQUIRE(rec_cap == 0 || (R.addr && R.status && R.inc), "null record column");
        hipStream_t hst;
        rp::Scratch* ws;
        rp::NameTable& nt = rp::members_names(m, &hst, &ws);
        hipStream_t st = stream ? rp::as_stream(stream) : hst;
        rp::Names nm = rp::names_of(nt, st, *ws);
        rp::In I{d_buf, d_msg_off};
        rp::Out O{d_msg_rec_off, d_msg_rec_off, rec_cap, R.addr, R.src, R.status, R.inc, R.src_inc, R.id_off,
                  R.addr_off, R.addr_len, d_err, H.checksum, H.source, H.source_inc, H.target, H.ping_status};
        // a wave per message (k_decode_wave: one launch, the thread parser inside it for the
        // messages the wave parser leaves); RP_WIRE_THREAD=1: the thread parser for every message
        const bool wave = !getenv("RP_WIRE_THREAD");
        if (n_msgs && wave) {
            uint64_t vb = 0, ve = 0;
            RP_HIP(hipMemcpyAsync(&vb, d_msg_off, 8, hipMemcpyDeviceToHost, st));
            RP_HIP(hipMemcpyAsync(&ve, d_msg_off + n_msgs, 8, hipMemcpyDeviceToHost, st));
            RP_HIP(hipStreamSynchronize(st));
            vb += reinterpret_cast<uint64_t>(d_buf);
            ve += reinterpret_cast<uint64_t>(d_buf);
            // a wave per message (3.73 ms at 100 k messages against 3.75-3.86 with 512-8192
            // workgroups striding; tools/wire_grid.sh); RP_WIRE_GRID caps it (A/B).
            // RP_WIRE_ONEPASS=1: the full layout alone (A/B)
            const bool onepass = getenv("RP_WIRE_ONEPASS") != nullptr;
            const unsigned gcap = (unsigned)rp::env_pos("RP_WIRE_GRID", 1u << 20);
            const unsigned g = rp::grid_for(n_msgs, onepass ? rp::kDecWaves : rp::kDecWavesS, gcap);
            const uint64_t nslots = (ve - vb) / rp::kMinRec + n_msgs + 1;
            ws->wire_stash.reserve(nslots * sizeof(rp::RecF));
            ws->wire_slow.reserve(n_msgs);
            rp::RecF* stash = reinterpret_cast<rp::RecF*>(ws->wire_stash.p);
            uint8_t* slow = ws->wire_slow.p;
            ws->wire_retry.reserve(1);
            RP_HIP(hipMemsetAsync(ws->wire_retry.p, 0, 4, st));
            const bool dbg = getenv("RP_WIRE_DEBUG") != nullptr;
            rp::DevBuf<uint32_t> nbw;
            if (dbg) {
                nbw.reserve(2);
                RP_HIP(hipMemsetAsync(nbw.p, 0, 8, st));
            }
            if (onepass) {
                hipLaunchKernelGGL((rp::k_decode_wave<rp::WaveLds, rp::kDecWaves, 0>), dim3(g),
                                   dim3(64 * rp::kDecWaves), 0, st, I, nm, O, n_msgs, vb, ve, stash, slow,
                                   dbg ? nbw.p : nullptr, ws->wire_retry.p);
            } else {
                hipLaunchKernelGGL((rp::k_decode_wave<rp::WaveLdsS, rp::kDecWavesS, 1>), dim3(g),
                                   dim3(64 * rp::kDecWavesS), 0, st, I, nm, O, n_msgs, vb, ve, stash, slow,
                                   dbg ? nbw.p : nullptr, ws->wire_retry.p);
                // the messages past the first layout's bounds: 1,024 workgroups striding the flags
                hipLaunchKernelGGL((rp::k_decode_wave<rp::WaveLds, rp::kDecWaves, 2>),
                                   dim3(rp::grid_for(n_msgs, rp::kDecWaves, std::min(gcap, 1024u))),
                                   dim3(64 * rp::kDecWaves), 0, st, I, nm, O, n_msgs, vb, ve, stash, slow,
                                   dbg ? nbw.p : nullptr, ws->wire_retry.p);
            }
            RP_HIP(hipGetLastError());
            rp::scan_exclusive_u32(d_msg_rec_off, d_msg_rec_off, n_msgs, st, *ws);
            hipLaunchKernelGGL(rp::k_decode_place, dim3(rp::grid_for((uint64_t)n_msgs * 64, 256, 8192)), dim3(256), 0,
                               st, I, O, n_msgs, stash, slow);
            hipLaunchKernelGGL(rp::k_decode<true>, dim3(rp::grid_for(n_msgs, 64)), dim3(64), 0, st, I, nm, O, n_msgs,
                               slow);
            RP_HIP(hipGetLastError());
            RP_HIP(hipStreamSynchronize(st));  // the stash is reused by the next call
            rp::scratch_check(*ws, st);
            if (dbg) {
                uint32_t h[2] = {0, 0};
                RP_HIP(hipMemcpy(h, nbw.p, 8, hipMemcpyDeviceToHost));
                fprintf(stderr, "[rp] wire decode: %u of %u messages by waves (records a lane per member: %u)\n", h[0],
                        n_msgs, h[1]);
            }
#ifdef RP_WIRE_PROF
            {
                RP_HIP(hipStreamSynchronize(st));
                unsigned long long h[8];
                RP_HIP(hipMemcpyFromSymbol(h, HIP_SYMBOL(rp::g_wprof), sizeof h));
                fprintf(stderr, "[rp] wire wave cycles (sum over waves): stage %llu classify %llu depth %llu top %llu "
                        "level %llu records %llu publish+fill %llu\n", h[0], h[1], h[2], h[3], h[4], h[5], h[6]);
            }
#endif
        } else {
            if (n_msgs) {
                hipLaunchKernelGGL(rp::k_decode<false>, dim3(rp::grid_for(n_msgs, 64)), dim3(64), 0, st, I, nm, O,
                                   n_msgs, nullptr);
                RP_HIP(hipGetLastError());
            } else {
                hipLaunchKernelGGL(rp::k_zero_tail, dim3(1), dim3(64), 0, st, d_msg_rec_off, 0u);
            }
            rp::scan_exclusive_u32(d_msg_rec_off, d_msg_rec_off, n_msgs, st, *ws);
            if (n_msgs) {
                hipLaunchKernelGGL(rp::k_decode<true>, dim3(rp::grid_for(n_msgs, 64)), dim3(64), 0, st, I, nm, O,
                                   n_msgs, nullptr);
                RP_HIP(hipGetLastError());
            }
        }
        if (!stream) RP_HIP(hipStreamSynchronize(st));
    });
}

// The first-round entry points, as thin forms of the two above.
int rp_wire_encode_changes_dev(rp_members* m, uint32_t n_msgs, const uint32_t* d_msg_rec_off, uint64_t n_rec,
                               const uint32_t* d_addr, const uint32_t* d_src, const uint8_t* d_status,
                               const int64_t* d_inc, const int64_t* d_src_inc, const uint8_t* d_ids, int form,
                               int body, const uint32_t* d_msg_checksum, const uint32_t* d_msg_source,
                               const int64_t* d_msg_source_inc, uint8_t* d_out, uint64_t* d_out_off, void* stream) {
    if (body < 0 || body > 2) {
        rp::set_error("rp_wire_encode_changes_dev: body must be 0..2 (rp_wire_encode_dev takes every body)");
        return rp::RP_EINVAL;
    }
    const rp_wire_records R{d_addr, d_src, d_status, d_inc, d_src_inc, d_ids};
    const rp_wire_headers H{d_msg_checksum, d_msg_source, d_msg_source_inc, nullptr, nullptr, nullptr, 0};
    return rp_wire_encode_dev(m, n_msgs, d_msg_rec_off, n_rec, &R, form, body, &H, d_out, d_out_off, stream);
}

int rp_wire_decode_changes_dev(rp_members* m, const uint8_t* d_buf, const uint64_t* d_msg_off, uint32_t n_msgs,
                               uint32_t* d_msg_rec_off, uint32_t rec_cap, uint32_t* d_addr, uint32_t* d_src,
                               uint8_t* d_status, int64_t* d_inc, int64_t* d_src_inc, uint64_t* d_id_off,
                               uint64_t* d_addr_off, uint32_t* d_addr_len, uint64_t* d_err,
                               uint32_t* d_msg_checksum, uint32_t* d_msg_source, int64_t* d_msg_source_inc,
                               void* stream) {
    const rp_wire_records_out R{d_addr, d_src, d_status, d_inc, d_src_inc, d_id_off, d_addr_off, d_addr_len};
    const rp_wire_headers_out H{d_msg_checksum, d_msg_source, d_msg_source_inc, nullptr, nullptr};
    return rp_wire_decode_dev(m, d_buf, d_msg_off, n_msgs, d_msg_rec_off, rec_cap, &R, &H, d_err, stream);
}

}  // extern "C"

// ------------------------------------------------------------------ host-buffer forms
// For callers holding host memory (the N-API addon, ctypes): stage through the handle's
// device, run the device form on the handle's stream, copy back. PCIe-bound.
namespace {
template <class T>
T* stage(rp::DevBuf<T>& d, const T* h, uint64_t n, hipStream_t st) {
    if (!h) return nullptr;
    d.reserve(n ? n : 1);
    if (n) RP_HIP(hipMemcpyAsync(d.p, h, sizeof(T) * n, hipMemcpyHostToDevice, st));
    return d.p;
}
template <class T>
void fetch(T* h, const rp::DevBuf<T>& d, uint64_t n) {
    if (h && n) RP_HIP(hipMemcpy(h, d.p, sizeof(T) * n, hipMemcpyDeviceToHost));
}
}  // namespace

extern "C" {

int rp_wire_encode(rp_members* m, uint32_t n_msgs, const uint32_t* msg_rec_off, const rp_wire_records* recs, int form,
                   int body, const rp_wire_headers* hdr, uint8_t* out, uint64_t cap, uint64_t* out_off) {
    return guard([&] {
        RP_REQUIRE(m && msg_rec_off && out_off, "null handle / offsets");
        RP_REQUIRE(msg_rec_off[0] == 0, "message record offsets must start at 0");
        for (uint32_t j = 0; j < n_msgs; j++)
            RP_REQUIRE(msg_rec_off[j + 1] >= msg_rec_off[j], "message record offsets must not decrease");
        hipStream_t st;
        rp::Scratch* ws;
        rp::NameTable& nt = rp::members_names(m, &st, &ws);
        const uint64_t n_rec = msg_rec_off[n_msgs];
        const rp_wire_records R = recs ? *recs : rp_wire_records{};
        const rp_wire_headers H = hdr ? *hdr : rp_wire_headers{};
        RP_REQUIRE(n_rec == 0 || (R.addr && R.src && R.status && R.inc), "null record column");
        const uint32_t nn = nt.size();
        for (uint64_t r = 0; r < n_rec; r++) {  // the ids index the name table: check them here
            RP_REQUIRE(R.addr[r] < nn, "wire encode: a record's address is not an interned id");
            RP_REQUIRE(R.src[r] < nn || R.src[r] == RP_NULL_ID, "wire encode: a record's source is not an interned id");
        }
        rp::DevBuf<uint32_t> d_ro, d_a, d_s, d_ck, d_ms, d_tg;
        rp::DevBuf<uint8_t> d_st, d_ids, d_out, d_ps;
        rp::DevBuf<int64_t> d_i, d_si, d_msi;
        rp::DevBuf<uint64_t> d_oo;
        stage(d_ro, msg_rec_off, (uint64_t)n_msgs + 1, st);
        const rp_wire_records DR{stage(d_a, R.addr, n_rec, st), stage(d_s, R.src, n_rec, st),
                                 stage(d_st, R.status, n_rec, st), stage(d_i, R.inc, n_rec, st),
                                 stage(d_si, R.src_inc, n_rec, st), stage(d_ids, R.ids, n_rec * 36, st)};
        const rp_wire_headers DH{stage(d_ck, H.checksum, n_msgs, st), stage(d_ms, H.source, n_msgs, st),
                                 stage(d_msi, H.source_inc, n_msgs, st), stage(d_tg, H.target, n_msgs, st),
                                 stage(d_ps, H.ping_status, n_msgs, st), H.app, H.app_len};
        d_oo.reserve((uint64_t)n_msgs + 1);
        auto run = [&](uint8_t* o) {
            const int rc = rp_wire_encode_dev(m, n_msgs, d_ro.p, n_rec, &DR, form, body, &DH, o, d_oo.p, st);
            if (rc) throw rp::Error(rc, rp_last_error());
        };
        run(nullptr);
        RP_HIP(hipMemcpy(out_off, d_oo.p, sizeof(uint64_t) * (n_msgs + 1), hipMemcpyDeviceToHost));
        const uint64_t total = out_off[n_msgs];
        if (!out) return;  // size query
        RP_REQUIRE(cap >= total, "encode: output buffer too small (query the size with out = NULL)");
        d_out.reserve(total ? total : 1);
        run(d_out.p);
        if (total) RP_HIP(hipMemcpy(out, d_out.p, total, hipMemcpyDeviceToHost));
    });
}

int rp_wire_decode(rp_members* m, const char* buf, const uint64_t* msg_off, uint32_t n_msgs, uint32_t* msg_rec_off,
                   uint32_t rec_cap, const rp_wire_records_out* recs, const rp_wire_headers_out* hdr, uint64_t* err) {
    return guard([&] {
        RP_REQUIRE(m && msg_off && msg_rec_off && err, "null handle / offsets / errors");
        const uint64_t nb = msg_off[n_msgs];
        RP_REQUIRE(buf || nb == 0, "null buffer with message bytes");
        for (uint32_t j = 0; j < n_msgs; j++) RP_REQUIRE(msg_off[j + 1] >= msg_off[j], "message offsets must not decrease");
        hipStream_t st;
        rp::Scratch* ws;
        rp::members_names(m, &st, &ws);
        const rp_wire_records_out R = recs ? *recs : rp_wire_records_out{};
        const rp_wire_headers_out H = hdr ? *hdr : rp_wire_headers_out{};
        rp::DevBuf<uint8_t> d_buf, d_st, d_ps;
        rp::DevBuf<uint64_t> d_off, d_err, d_id, d_ao;
        rp::DevBuf<uint32_t> d_ro, d_a, d_s, d_al, d_ck, d_ms, d_tg;
        rp::DevBuf<int64_t> d_i, d_si, d_msi;
        stage(d_buf, reinterpret_cast<const uint8_t*>(buf), nb, st);
        if (!buf) d_buf.reserve(1);
        stage(d_off, msg_off, (uint64_t)n_msgs + 1, st);
        d_ro.reserve((uint64_t)n_msgs + 1);
        const uint64_t nm1 = n_msgs ? n_msgs : 1;
        d_err.reserve(nm1);
        const uint64_t c = rec_cap ? rec_cap : 1;
        d_a.reserve(c); d_st.reserve(c); d_i.reserve(c);
        auto opt = [&](auto& d, const void* want, uint64_t n) { if (want) d.reserve(n); return want ? d.p : nullptr; };
        const rp_wire_records_out DR{d_a.p, opt(d_s, R.src, c), d_st.p, d_i.p, opt(d_si, R.src_inc, c),
                                     opt(d_id, R.id_off, c), opt(d_ao, R.addr_off, c), opt(d_al, R.addr_len, c)};
        const rp_wire_headers_out DH{opt(d_ck, H.checksum, nm1), opt(d_ms, H.source, nm1),
                                     opt(d_msi, H.source_inc, nm1), opt(d_tg, H.target, nm1),
                                     opt(d_ps, H.ping_status, nm1)};
        const int rc = rp_wire_decode_dev(m, d_buf.p, d_off.p, n_msgs, d_ro.p, rec_cap, &DR, &DH, d_err.p, st);
        if (rc) throw rp::Error(rc, rp_last_error());
        RP_HIP(hipStreamSynchronize(st));
        RP_HIP(hipMemcpy(msg_rec_off, d_ro.p, sizeof(uint32_t) * (n_msgs + 1), hipMemcpyDeviceToHost));
        fetch(err, d_err, n_msgs);
        fetch(H.checksum, d_ck, n_msgs);
        fetch(H.source, d_ms, n_msgs);
        fetch(H.source_inc, d_msi, n_msgs);
        fetch(H.target, d_tg, n_msgs);
        fetch(H.ping_status, d_ps, n_msgs);
        const uint64_t k = std::min<uint64_t>(msg_rec_off[n_msgs], rec_cap);
        fetch(R.addr, d_a, k);
        fetch(R.src, d_s, k);
        fetch(R.status, d_st, k);
        fetch(R.inc, d_i, k);
        fetch(R.src_inc, d_si, k);
        fetch(R.id_off, d_id, k);
        fetch(R.addr_off, d_ao, k);
        fetch(R.addr_len, d_al, k);
    });
}

int rp_wire_encode_changes(rp_members* m, uint32_t n_msgs, const uint32_t* msg_rec_off, const uint32_t* addr,
                           const uint32_t* src, const uint8_t* status, const int64_t* inc, const int64_t* src_inc,
                           const uint8_t* ids, int form, int body, const uint32_t* msg_checksum,
                           const uint32_t* msg_source, const int64_t* msg_source_inc, uint8_t* out, uint64_t cap,
                           uint64_t* out_off) {
    if (body < 0 || body > 2) {
        rp::set_error("rp_wire_encode_changes: body must be 0..2 (rp_wire_encode takes every body)");
        return rp::RP_EINVAL;
    }
    const rp_wire_records R{addr, src, status, inc, src_inc, ids};
    const rp_wire_headers H{msg_checksum, msg_source, msg_source_inc, nullptr, nullptr, nullptr, 0};
    return rp_wire_encode(m, n_msgs, msg_rec_off, &R, form, body, &H, out, cap, out_off);
}

int rp_wire_decode_changes(rp_members* m, const char* buf, const uint64_t* msg_off, uint32_t n_msgs,
                           uint32_t* msg_rec_off, uint32_t rec_cap, uint32_t* addr, uint32_t* src, uint8_t* status,
                           int64_t* inc, int64_t* src_inc, uint64_t* err) {
    const rp_wire_records_out R{addr, src, status, inc, src_inc, nullptr, nullptr, nullptr};
    return rp_wire_decode(m, buf, msg_off, n_msgs, msg_rec_off, rec_cap, &R, nullptr, err);
}

}  // extern "C"
