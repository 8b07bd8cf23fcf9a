// rp_common.h — shared plumbing for the librpamd C-ABI: error slot, HIP checks, sizes.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <atomic>
#include <stdexcept>
#include <string>

namespace rp {

// Thread-local last-error string behind rp_last_error() (SURVEY §8b "Errors").
void set_error(const std::string& msg);
const char* last_error();

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

enum : int {
    RP_OK = 0,
    RP_EINVAL = -1,
    RP_EDEVICE = -2,
    RP_ENOMEM = -3,
    RP_ESTATE = -4,
};

#define RP_HIP(expr)                                                                          \
    do {                                                                                      \
        hipError_t rp_e_ = (expr);                                                            \
        if (rp_e_ != hipSuccess)                                                              \
            throw ::rp::Error(::rp::RP_EDEVICE, std::string(#expr) + ": " +                   \
                                                    hipGetErrorString(rp_e_));                \
    } while (0)

#define RP_REQUIRE(cond, msg)                                                                 \
    do {                                                                                      \
        if (!(cond)) throw ::rp::Error(::rp::RP_EINVAL, (msg));                               \
    } while (0)

// Resident lookup services (rp_ring_service, rp_ring.hip) against every other device call.
// While a service wave is resident, hipFree (a buffer growing or released) synchronizes the
// device and waits for it, and the service's stream may share a hardware queue with any other
// stream of the process (GPU_MAX_HW_QUEUES). So every C-ABI call that may touch the device holds
// a QuietScope: it stops every resident service before its body runs, and a service lookup that
// arrives meanwhile (another thread) takes the launch path instead of starting a wave, until the
// scope ends. The pair of counters is a Dekker handshake: a scope raises g_quiet, then reads
// g_svc_live; a service raises g_svc_live, then reads g_quiet (both sequentially consistent), so
// at least one of them sees the other.
extern std::atomic<int> g_quiet;     // QuietScopes open in the process
extern std::atomic<int> g_svc_live;  // services launched and not yet stopped
void svc_quiesce(const void* keep);  // stop every resident service but `keep`'s ring's

struct QuietScope {
    QuietScope() {
        g_quiet.fetch_add(1);
        try {
            if (g_svc_live.load() > 0) svc_quiesce(nullptr);
        } catch (...) {  // (the destructor does not run when the constructor throws)
            g_quiet.fetch_sub(1);
            throw;
        }
    }
    ~QuietScope() { g_quiet.fetch_sub(1); }
    QuietScope(const QuietScope&) = delete;
    QuietScope& operator=(const QuietScope&) = delete;
};

// Run a C-ABI body; convert exceptions into an int status + rp_last_error(). guard_host is for
// entry points that touch no device state (or, the ring's lookups, manage the service themselves).
template <class F>
int guard_host(F&& f) {
    try {
        f();
        return RP_OK;
    } catch (const Error& e) {
        set_error(e.what());
        return e.code;
    } catch (const std::bad_alloc&) {
        set_error("host out of memory");
        return RP_ENOMEM;
    } catch (const std::exception& e) {
        set_error(e.what());
        return RP_EINVAL;
    }
}

template <class F>
int guard(F&& f) {
    return guard_host([&] {
        QuietScope quiet;
        f();
    });
}

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// A positive integer from the environment (A/B knobs: grid caps, group sizes); `dflt` when the
// variable is unset, empty, not a number, or not positive, so no knob can ask for a 0-workgroup
// launch.
inline uint64_t env_pos(const char* name, uint64_t dflt) {
    const char* e = getenv(name);
    if (!e || !*e) return dflt;
    char* end = nullptr;
    const unsigned long long v = strtoull(e, &end, 10);
    return (end && *end == 0 && v > 0) ? (uint64_t)v : dflt;
}

inline unsigned grid_for(uint64_t items, unsigned per_block, unsigned cap = 2048) {
    uint64_t g = (items + per_block - 1) / per_block;
    if (g == 0) g = 1;
    return (unsigned)(g > cap ? cap : g);
}

// Device buffer with explicit capacity (owned by a handle; freed in its destructor).
template <class T>
struct DevBuf {
    T* p = nullptr;
    uint64_t cap = 0;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    ~DevBuf() { release(); }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    void reserve(uint64_t n) {  // discards contents
        if (n <= cap) return;
        release();
        uint64_t c = n < 64 ? 64 : n;
        if (hipMalloc(&p, c * sizeof(T)) != hipSuccess) {
            p = nullptr;
            throw Error(RP_ENOMEM, "hipMalloc failed (" + std::to_string(c * sizeof(T)) + " bytes)");
        }
        cap = c;
    }
    void swap(DevBuf& o) {
        std::swap(p, o.p);
        std::swap(cap, o.cap);
    }
};

}  // namespace rp
