// rp_capi.hip — library-wide C-ABI entry points (errors, version, devices).
#include <string>

#include "../../include/ringpop_amd.h"
#include "rp_common.h"

namespace rp {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }
const char* last_error() { return g_last_error.c_str(); }

}  // namespace rp

extern "C" {

const char* rp_last_error(void) { return rp::last_error(); }

uint32_t rp_version(void) { return (1u << 16) | 0u; }

int rp_device_count(int* n) {
    return rp::guard([&] {
        int c = 0;
        if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
        *n = c;
    });
}

int rp_copy(void* dst, const void* src, uint64_t bytes, void* stream) {
    return rp::guard([&] {
        if (!bytes) return;
        RP_REQUIRE(dst && src, "copy: null pointer");
        RP_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, rp::as_stream(stream)));
        if (!stream) RP_HIP(hipStreamSynchronize(nullptr));
    });
}

}  // extern "C"
