// rp_wire.hip — gossip wire bodies on the device: dissemination change records as JSON.
//
// Encoder: one message = one list of change records, written as the bytes JSON.stringify
// produces for
//   issueAs records      {id, source, sourceIncarnationNumber, address, status, incarnationNumber}
//                        (lib/gossip/dissemination.js:163-170; `id` dropped when absent, as
//                        JSON.stringify drops an undefined member)
//   fullSync records     {source, address, status, incarnationNumber} (dissemination.js:64-73)
// wrapped as a bare array, a ping request body {checksum, changes, source, sourceIncarnationNumber}
// (lib/gossip/ping-sender.js:71-76) or a ping response body {changes} (server/protocol/ping.js:45-48).
// Three passes over thread-per-record / thread-per-message grids: record lengths -> scans ->
// records written at their final offsets (the same emit routine measures and writes, so
// lengths and bytes cannot disagree).
//
// Decoder: one thread per message parses a changes array, or a body object whose `changes`
// member is that array (other members skipped; checksum / source / sourceIncarnationNumber
// captured), into per-record columns with addresses interned against the members' name table
// by binary search over its byte-ordered ids. Strings with escapes are rejected (addresses and
// uuids never hold one), numbers must be integral. Count pass -> scan -> fill pass.
#include <climits>

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
    if (R.form == 0) {
        if (R.ids) {
            s.lit("{\"id\":\"");
            s.bytes(R.ids + r * 36, 36);
            s.lit("\",\"source\":\"");
        } else {
            s.lit("{\"source\":\"");
        }
        s.name(nm, R.src[r]);
        s.lit("\",\"sourceIncarnationNumber\":");
        s.num(R.src_inc[r]);
        s.lit(",\"address\":\"");
    } else {
        s.lit("{\"source\":\"");
        s.name(nm, R.src[r]);
        s.lit("\",\"address\":\"");
    }
    s.name(nm, R.addr[r]);
    s.lit("\",\"status\":\"");
    s.status(R.status[r]);
    s.lit("\",\"incarnationNumber\":");
    s.num(R.inc[r]);
    s.lit("}");
}

struct Msgs {
    const uint32_t* rec_off;  // n+1
    const uint32_t* checksum;
    const uint32_t* source;
    const int64_t* source_inc;
    int body;  // 0 array, 1 ping request, 2 ping response
};

__device__ void emit_head(Sink& s, const Msgs& M, uint32_t m) {
    if (M.body == 1) {
        s.lit("{\"checksum\":");
        s.num((int64_t)M.checksum[m]);
        s.lit(",\"changes\":[");
    } else if (M.body == 2) {
        s.lit("{\"changes\":[");
    } else {
        s.lit("[");
    }
}

__device__ void emit_tail(Sink& s, const Names& nm, const Msgs& M, uint32_t m) {
    if (M.body == 1) {
        s.lit("],\"source\":\"");
        s.name(nm, M.source[m]);
        s.lit("\",\"sourceIncarnationNumber\":");
        s.num(M.source_inc[m]);
        s.lit("}");
    } else if (M.body == 2) {
        s.lit("]}");
    } else {
        s.lit("]");
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
        emit_head(s, M, m);
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
        emit_head(h, M, m);
        Sink t{out + moff[m] + h.n + rec_scan[M.rec_off[m + 1]] - rec_scan[M.rec_off[m]]};
        emit_tail(t, nm, M, m);
    }
}

__global__ void k_rec_write(Names nm, Recs R, Msgs M, uint32_t n_msgs, uint64_t n_rec, const uint32_t* moff,
                            const uint32_t* rec_scan, uint8_t* out) {
    for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < n_rec; r += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t m = msg_of(M.rec_off, n_msgs, r);
        Sink h{nullptr};
        emit_head(h, M, m);
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
            emit_head(h, M, m);
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
};

__device__ int name_cmp(const Names& nm, const uint8_t* s, uint32_t len, uint32_t id) {
    const uint64_t a = nm.off[id], b = nm.off[id + 1];
    const uint32_t l2 = (uint32_t)(b - a);
    const uint32_t k = len < l2 ? len : l2;
    for (uint32_t i = 0; i < k; i++) {
        const uint8_t x = s[i], y = nm.bytes[a + i];
        if (x != y) return x < y ? -1 : 1;
    }
    return len == l2 ? 0 : (len < l2 ? -1 : 1);
}

__device__ uint32_t name_find(const Names& nm, const uint8_t* s, uint32_t len) {
    uint32_t lo = 0, hi = nm.n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        const int c = name_cmp(nm, s, len, nm.sorted[mid]);
        if (c == 0) return nm.sorted[mid];
        if (c < 0) hi = mid; else lo = mid + 1;
    }
    return NULL_ID;
}

template <int N>
__device__ bool key_is(const uint8_t* s, uint32_t len, const char (&k)[N]) {
    if (len != N - 1) return false;
    for (int i = 0; i < N - 1; i++)
        if (s[i] != (uint8_t)k[i]) return false;
    return true;
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
    if (key_is(s, len, "alive")) return ST_ALIVE;
    if (key_is(s, len, "suspect")) return ST_SUSPECT;
    if (key_is(s, len, "faulty")) return ST_FAULTY;
    if (key_is(s, len, "leave")) return ST_LEAVE;
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

template <bool FILL>
__global__ void k_decode(In I, Names nm, Out O, uint32_t n_msgs) {
    for (uint32_t m = blockIdx.x * blockDim.x + threadIdx.x; m < n_msgs; m += gridDim.x * blockDim.x) {
        Parser P{I.buf, I.msg_off[m], I.msg_off[m + 1]};
        const uint64_t k0 = FILL ? O.rec_off[m] : 0;
        const uint64_t kend = FILL ? O.rec_off[m + 1] : 0;
        uint32_t n = 0;
        bool seen = false;
        uint32_t ck = 0, msrc = NULL_ID;
        int64_t msinc = LLONG_MIN;
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
                    if (key_is(key, kl, "changes")) {
                        n = parse_changes<FILL>(P, nm, O, k0, kend);
                        seen = true;
                    } else if (key_is(key, kl, "checksum")) {
                        ck = (uint32_t)P.integer();
                    } else if (key_is(key, kl, "source")) {
                        uint64_t so; uint32_t sl;
                        P.str(so, sl);
                        if (FILL && !P.bad) msrc = name_find(nm, P.p + so, sl);
                    } else if (key_is(key, kl, "sourceIncarnationNumber")) {
                        msinc = P.integer();
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
        if (!FILL) {
            O.cnt[m] = n;
        } else {
            O.err[m] = P.bad ? P.bad_at - I.msg_off[m] + 1 : 0;
            if (O.m_checksum) O.m_checksum[m] = ck;
            if (O.m_source) O.m_source[m] = msrc;
            if (O.m_source_inc) O.m_source_inc[m] = msinc;
        }
    }
}

__global__ void k_zero_tail(uint32_t* p, uint32_t n) {
    if (threadIdx.x == 0 && blockIdx.x == 0) p[n] = 0;
}

Names names_of(NameTable& nt, hipStream_t st, Scratch& ws) {
    nt.sort(st, ws);
    return Names{nt.d_bytes.p, nt.d_noff.p, nt.sorted.p, nt.size()};
}

}  // namespace
}  // namespace rp

using rp::guard;

extern "C" {

int rp_wire_encode_changes_dev(rp_members* m, uint32_t n_msgs, const uint32_t* d_msg_rec_off, uint64_t n_rec,
                               const uint32_t* d_addr, const uint32_t* d_src, const uint8_t* d_status,
                               const int64_t* d_inc, const int64_t* d_src_inc, const uint8_t* d_ids, int form,
                               int body, const uint32_t* d_msg_checksum, const uint32_t* d_msg_source,
                               const int64_t* d_msg_source_inc, uint8_t* d_out, uint64_t* d_out_off, void* stream) {
    return guard([&] {
        RP_REQUIRE(m, "null members handle");
        RP_REQUIRE(form == 0 || form == 1, "form must be 0 (issueAs) or 1 (fullSync)");
        RP_REQUIRE(body >= 0 && body <= 2, "body must be 0 (array), 1 (ping request) or 2 (ping response)");
        RP_REQUIRE(d_msg_rec_off && d_out_off, "null offsets");
        RP_REQUIRE(n_rec == 0 || (d_addr && d_src && d_status && d_inc), "null record column");
        RP_REQUIRE(n_rec == 0 || form == 1 || d_src_inc, "issueAs records need sourceIncarnationNumber");
        RP_REQUIRE(body != 1 || (d_msg_checksum && d_msg_source && d_msg_source_inc), "ping body needs header columns");
        hipStream_t hst;
        rp::Scratch* ws;
        rp::NameTable& nt = rp::members_names(m, &hst, &ws);
        hipStream_t st = stream ? rp::as_stream(stream) : hst;
        // every byte offset fits u32: bound the worst case on the host
        const uint64_t rec_max = 180 + 2ull * nt.max_len;
        RP_REQUIRE(n_rec * rec_max + (uint64_t)n_msgs * (80 + nt.max_len) < 0xFFFFFFFFull,
                   "encoded batch may exceed 4 GiB: split it");
        rp::Names nm = rp::names_of(nt, st, *ws);
        rp::Recs R{d_addr, d_src, d_status, d_inc, d_src_inc, d_ids, form};
        rp::Msgs M{d_msg_rec_off, d_msg_checksum, d_msg_source, d_msg_source_inc, body};
        rp::DevBuf<uint32_t> rscan, mscan;
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
            hipLaunchKernelGGL(rp::k_rec_write_lds, dim3(rp::grid_for(n_rec, rp::kWrThreads, 4096)),
                               dim3(rp::kWrThreads), 0, st, nm, R, M, n_msgs, n_rec, mscan.p, rscan.p, d_out);
            RP_HIP(hipGetLastError());
        }
        RP_HIP(hipStreamSynchronize(st));  // scratch buffers are local
    });
}

int rp_wire_decode_changes_dev(rp_members* m, const uint8_t* d_buf, const uint64_t* d_msg_off, uint32_t n_msgs,
                               uint32_t* d_msg_rec_off, uint32_t rec_cap, uint32_t* d_addr, uint32_t* d_src,
                               uint8_t* d_status, int64_t* d_inc, int64_t* d_src_inc, uint64_t* d_id_off,
                               uint64_t* d_addr_off, uint32_t* d_addr_len, uint64_t* d_err,
                               uint32_t* d_msg_checksum, uint32_t* d_msg_source, int64_t* d_msg_source_inc,
                               void* stream) {
    return guard([&] {
        RP_REQUIRE(m, "null members handle");
        RP_REQUIRE(d_msg_off && d_msg_rec_off && d_err, "null message offsets / errors");
        RP_REQUIRE(rec_cap == 0 || (d_addr && d_status && d_inc), "null record column");
        hipStream_t hst;
        rp::Scratch* ws;
        rp::NameTable& nt = rp::members_names(m, &hst, &ws);
        hipStream_t st = stream ? rp::as_stream(stream) : hst;
        rp::Names nm = rp::names_of(nt, st, *ws);
        rp::In I{d_buf, d_msg_off};
        rp::Out O{d_msg_rec_off, d_msg_rec_off, rec_cap, d_addr, d_src, d_status, d_inc, d_src_inc, d_id_off,
                  d_addr_off, d_addr_len, d_err, d_msg_checksum, d_msg_source, d_msg_source_inc};
        if (n_msgs) {
            hipLaunchKernelGGL(rp::k_decode<false>, dim3(rp::grid_for(n_msgs, 64)), dim3(64), 0, st, I, nm, O,
                               n_msgs);
            RP_HIP(hipGetLastError());
        } else {
            hipLaunchKernelGGL(rp::k_zero_tail, dim3(1), dim3(64), 0, st, d_msg_rec_off, 0u);
        }
        rp::scan_exclusive_u32(d_msg_rec_off, d_msg_rec_off, n_msgs, st, *ws);
        if (n_msgs) {
            hipLaunchKernelGGL(rp::k_decode<true>, dim3(rp::grid_for(n_msgs, 64)), dim3(64), 0, st, I, nm, O,
                               n_msgs);
            RP_HIP(hipGetLastError());
        }
        if (!stream) RP_HIP(hipStreamSynchronize(st));
    });
}

}  // extern "C"

// ------------------------------------------------------------------ host-buffer forms
// For callers holding host memory (the N-API addon, ctypes): stage through the handle's
// device, run the _dev form on the handle's stream, copy back. PCIe-bound.
namespace {
template <class T>
T* stage(rp::DevBuf<T>& d, const T* h, uint64_t n, hipStream_t st) {
    if (!h) return nullptr;
    d.reserve(n ? n : 1);
    if (n) RP_HIP(hipMemcpyAsync(d.p, h, sizeof(T) * n, hipMemcpyHostToDevice, st));
    return d.p;
}
}  // namespace

extern "C" {

int rp_wire_encode_changes(rp_members* m, uint32_t n_msgs, const uint32_t* msg_rec_off, const uint32_t* addr,
                           const uint32_t* src, const uint8_t* status, const int64_t* inc, const int64_t* src_inc,
                           const uint8_t* ids, int form, int body, const uint32_t* msg_checksum,
                           const uint32_t* msg_source, const int64_t* msg_source_inc, uint8_t* out, uint64_t cap,
                           uint64_t* out_off) {
    return guard([&] {
        RP_REQUIRE(m && msg_rec_off && out_off, "null handle / offsets");
        hipStream_t st;
        rp::Scratch* ws;
        rp::members_names(m, &st, &ws);
        const uint64_t n_rec = msg_rec_off[n_msgs];
        rp::DevBuf<uint32_t> d_ro, d_a, d_s, d_ck, d_ms;
        rp::DevBuf<uint8_t> d_st, d_ids, d_out;
        rp::DevBuf<int64_t> d_i, d_si, d_msi;
        rp::DevBuf<uint64_t> d_oo;
        stage(d_ro, msg_rec_off, (uint64_t)n_msgs + 1, st);
        const bool ping = body == 1;
        d_oo.reserve((uint64_t)n_msgs + 1);
        auto run = [&](uint8_t* o) {
            const int rc = rp_wire_encode_changes_dev(
                m, n_msgs, d_ro.p, n_rec, stage(d_a, addr, n_rec, st), stage(d_s, src, n_rec, st),
                stage(d_st, status, n_rec, st), stage(d_i, inc, n_rec, st), stage(d_si, src_inc, n_rec, st),
                stage(d_ids, ids, n_rec * 36, st), form, body, ping ? stage(d_ck, msg_checksum, n_msgs, st) : nullptr,
                ping ? stage(d_ms, msg_source, n_msgs, st) : nullptr,
                ping ? stage(d_msi, msg_source_inc, n_msgs, st) : nullptr, o, d_oo.p, st);
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

int rp_wire_decode_changes(rp_members* m, const char* buf, const uint64_t* msg_off, uint32_t n_msgs,
                           uint32_t* msg_rec_off, uint32_t rec_cap, uint32_t* addr, uint32_t* src, uint8_t* status,
                           int64_t* inc, int64_t* src_inc, uint64_t* err) {
    return guard([&] {
        RP_REQUIRE(m && msg_off && msg_rec_off && err, "null handle / offsets / errors");
        hipStream_t st;
        rp::Scratch* ws;
        rp::members_names(m, &st, &ws);
        const uint64_t nb = msg_off[n_msgs];
        rp::DevBuf<uint8_t> d_buf, d_st;
        rp::DevBuf<uint64_t> d_off, d_err;
        rp::DevBuf<uint32_t> d_ro, d_a, d_s;
        rp::DevBuf<int64_t> d_i, d_si;
        stage(d_buf, reinterpret_cast<const uint8_t*>(buf), nb, st);
        if (!buf) d_buf.reserve(1);
        stage(d_off, msg_off, (uint64_t)n_msgs + 1, st);
        d_ro.reserve((uint64_t)n_msgs + 1);
        d_err.reserve(n_msgs ? n_msgs : 1);
        const uint64_t c = rec_cap ? rec_cap : 1;
        d_a.reserve(c); d_s.reserve(c); d_st.reserve(c); d_i.reserve(c); d_si.reserve(c);
        const int rc = rp_wire_decode_changes_dev(m, d_buf.p, d_off.p, n_msgs, d_ro.p, rec_cap, d_a.p, d_s.p, d_st.p,
                                                  d_i.p, d_si.p, nullptr, nullptr, nullptr, d_err.p, nullptr, nullptr,
                                                  nullptr, st);
        if (rc) throw rp::Error(rc, rp_last_error());
        RP_HIP(hipStreamSynchronize(st));
        RP_HIP(hipMemcpy(msg_rec_off, d_ro.p, sizeof(uint32_t) * (n_msgs + 1), hipMemcpyDeviceToHost));
        if (n_msgs) RP_HIP(hipMemcpy(err, d_err.p, sizeof(uint64_t) * n_msgs, hipMemcpyDeviceToHost));
        const uint64_t k = std::min<uint64_t>(msg_rec_off[n_msgs], rec_cap);
        if (k) {
            if (addr) RP_HIP(hipMemcpy(addr, d_a.p, 4 * k, hipMemcpyDeviceToHost));
            if (src) RP_HIP(hipMemcpy(src, d_s.p, 4 * k, hipMemcpyDeviceToHost));
            if (status) RP_HIP(hipMemcpy(status, d_st.p, k, hipMemcpyDeviceToHost));
            if (inc) RP_HIP(hipMemcpy(inc, d_i.p, 8 * k, hipMemcpyDeviceToHost));
            if (src_inc) RP_HIP(hipMemcpy(src_inc, d_si.p, 8 * k, hipMemcpyDeviceToHost));
        }
    });
}

}  // extern "C"
