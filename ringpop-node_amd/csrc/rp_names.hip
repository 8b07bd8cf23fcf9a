// rp_names.hip — interned address table: host map + device mirror + device byte-order sort.
#include <algorithm>

#include "rp_farmhash.h"
#include "rp_names.h"

namespace rp {

namespace {

// big-endian 4-byte chunk c of name(ids[i]) (0-padded): the LSD radix key for byte order.
__global__ void k_name_chunk(const uint8_t* __restrict__ names, const uint64_t* __restrict__ noff,
                             const uint32_t* __restrict__ ids, uint32_t n, uint32_t c, uint32_t* __restrict__ key) {
    const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gstride) {
        const uint32_t id = ids[i];
        const uint64_t b = noff[id];
        const uint32_t L = (uint32_t)(noff[id + 1] - b);
        uint32_t k = 0;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t o = c * 4 + q;
            k = (k << 8) | (o < L ? names[b + o] : 0u);
        }
        key[i] = k;
    }
}

__global__ void k_name_hash_insert(const uint8_t* __restrict__ names, const uint64_t* __restrict__ noff, uint32_t n,
                                   uint32_t* __restrict__ hs, uint32_t mask) {
    const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gstride) {
        const uint64_t b = noff[i];
        const uint32_t L = (uint32_t)(noff[i + 1] - b);
        uint32_t slot = fh::hash32(fh::PtrSrc{names + b}, L) & mask;
        while (atomicCAS(&hs[NameTable::kSlotWords * slot], 0xFFFFFFFFu, (uint32_t)i) != 0xFFFFFFFFu)
            slot = (slot + 1) & mask;
        uint32_t* w = hs + NameTable::kSlotWords * slot;
        w[1] = L;
        w[2] = (uint32_t)b;
#pragma unroll
        for (uint32_t q = 0; q < NameTable::kNameInline / 4; q++) {
            uint32_t x = 0;
#pragma unroll
            for (uint32_t j = 0; j < 4; j++) {
                const uint32_t o = 4 * q + j;
                x |= (o < L ? (uint32_t)names[b + o] : 0u) << (8 * j);
            }
            w[3 + q] = x;
        }
    }
}

// soff[i] = the length of the i-th name in byte order (soff[n] = 0, for the exclusive scan)
__global__ void k_name_sorted_len(const uint64_t* __restrict__ noff, const uint32_t* __restrict__ sorted, uint32_t n,
                                  uint32_t* __restrict__ len) {
    const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= n; i += gstride)
        len[i] = i < n ? (uint32_t)(noff[sorted[i] + 1] - noff[sorted[i]]) : 0u;
}

__global__ void k_name_sorted_copy(const uint8_t* __restrict__ names, const uint64_t* __restrict__ noff,
                                   const uint32_t* __restrict__ sorted, const uint32_t* __restrict__ soff, uint32_t n,
                                   uint8_t* __restrict__ sbytes) {
    const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gstride) {
        const uint8_t* src = names + noff[sorted[i]];
        uint8_t* dst = sbytes + soff[i];
        const uint32_t L = soff[i + 1] - soff[i];
        for (uint32_t q = 0; q < L; q++) dst[q] = src[q];
    }
}

}  // namespace

void NameTable::sort_bytes(hipStream_t st, Scratch& ws) {
    sort(st, ws);
    const uint32_t n = (uint32_t)names.size();
    if (sbytes_n == n && soff.p) return;
    if (h_bytes.size() > 0xFFFFFF00ull) throw Error(RP_EINVAL, "names past 4 GB of bytes (32-bit sorted offsets)");
    soff.reserve((uint64_t)n + 1);
    sbytes.reserve(h_bytes.size() + 32);
    RP_HIP(hipMemsetAsync(sbytes.p, 0, h_bytes.size() + 32, st));
    hipLaunchKernelGGL(k_name_sorted_len, dim3(grid_for((uint64_t)n + 1, 256)), dim3(256), 0, st, d_noff.p, sorted.p, n,
                       soff.p);
    RP_HIP(hipGetLastError());
    scan_exclusive_u32(soff.p, soff.p, (uint64_t)n + 1, st, ws);
    if (n)
        hipLaunchKernelGGL(k_name_sorted_copy, dim3(grid_for(n, 256)), dim3(256), 0, st, d_bytes.p, d_noff.p,
                           sorted.p, soff.p, n, sbytes.p);
    RP_HIP(hipGetLastError());
    sbytes_n = n;
}

void NameTable::hash_index(hipStream_t st) {
    const uint32_t n = (uint32_t)names.size();
    if (htab_n == n && hslot.p) return;
    sync(st);
    uint32_t b = 4;
    while ((1ull << b) < 2ull * n) b++;  // load factor <= 1/2
    if (h_bytes.size() > 0xFFFFFF00ull) throw Error(RP_EINVAL, "names past 4 GB of bytes (32-bit offsets in the index)");
    hslot.reserve((uint64_t)kSlotWords << b);
    RP_HIP(hipMemsetAsync(hslot.p, 0xFF, (4ull * kSlotWords) << b, st));
    if (n)
        hipLaunchKernelGGL(k_name_hash_insert, dim3(grid_for(n, 256)), dim3(256), 0, st, d_bytes.p, d_noff.p, n,
                           hslot.p, (1u << b) - 1u);
    RP_HIP(hipGetLastError());
    hbits = b;
    htab_n = n;
}

uint32_t NameTable::find(const char* s, uint32_t n) const {
    auto it = ids.find(std::string(s, n));
    return it == ids.end() ? 0xFFFFFFFFu : it->second;
}

uint32_t NameTable::intern(const char* s, uint32_t n) {
    std::string key(s, n);
    auto it = ids.find(key);
    if (it != ids.end()) return it->second;
    const uint32_t id = (uint32_t)names.size();
    ids.emplace(key, id);
    names.push_back(key);
    h_bytes.insert(h_bytes.end(), key.begin(), key.end());
    h_noff.push_back(h_bytes.size());
    max_len = std::max(max_len, n);
    return id;
}

void NameTable::sync(hipStream_t st) {
    if (dev_n == names.size()) return;
    const uint32_t nn = (uint32_t)names.size();
    d_bytes.reserve(h_bytes.size() + 16);
    d_noff.reserve((uint64_t)nn + 1);
    if (!h_bytes.empty())
        RP_HIP(hipMemcpyAsync(d_bytes.p, h_bytes.data(), h_bytes.size(), hipMemcpyHostToDevice, st));
    RP_HIP(hipMemcpyAsync(d_noff.p, h_noff.data(), sizeof(uint64_t) * (nn + 1), hipMemcpyHostToDevice, st));
    // the async copies read host vectors that may grow later: finish them now
    RP_HIP(hipStreamSynchronize(st));
    dev_n = nn;
}

void NameTable::sort(hipStream_t st, Scratch& ws) {
    const uint32_t n = (uint32_t)names.size();
    if (sorted_n == n) return;
    sync(st);
    sorted.reserve((uint64_t)n + 1);
    tmp.reserve((uint64_t)n + 1);
    iota_u32(sorted.p, n, st);
    const uint32_t nchunks = (max_len + 3) / 4;
    for (int c = (int)nchunks - 1; c >= 0; c--) {
        hipLaunchKernelGGL(k_name_chunk, dim3(grid_for(n, 256)), dim3(256), 0, st, d_bytes.p, d_noff.p, sorted.p, n,
                           (uint32_t)c, tmp.p);
        RP_HIP(hipGetLastError());
        radix_sort_pairs(tmp.p, sorted.p, n, 0, 32, st, ws);
    }
    sorted_n = n;
}

}  // namespace rp
