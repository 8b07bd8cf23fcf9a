// rp_names.h — interned address table shared by the ring and the membership view.
//
// Host side keeps the id <-> string map (the JS caller owns strings anyway); the device keeps
// a mirror of the bytes + offsets and the ids sorted in byte order (== JS default string sort
// for ASCII addresses: lib/ring/index.js:100, lib/membership/index.js:102-110), which every
// checksum string is built in.
#pragma once

#include <string>
#include <unordered_map>
#include <vector>

#include "rp_prims.h"

namespace rp {

struct NameTable {
    std::vector<std::string> names;
    std::unordered_map<std::string, uint32_t> ids;
    std::vector<uint64_t> h_noff{0};
    std::vector<uint8_t> h_bytes;
    uint32_t max_len = 0;
    // device mirror
    DevBuf<uint8_t> d_bytes;
    DevBuf<uint64_t> d_noff;
    uint32_t dev_n = 0;
    // ids in byte order of their names
    DevBuf<uint32_t> sorted;
    uint32_t sorted_n = 0;
    DevBuf<uint32_t> tmp;
    // the names concatenated in byte order (sbytes, padded by 32 bytes) and their offsets by
    // rank (soff[n] = the total): the membership checksum string reads its names in order
    DevBuf<uint8_t> sbytes;
    DevBuf<uint32_t> soff;
    uint32_t sbytes_n = 0;
    // open-addressing index over the device names (the wire decoder's interning): 2^hbits slots
    // of 32 B, keyed by farmhash32 of the name, linear probing. A slot holds the id (0xFFFFFFFF
    // empty), the name's length, its byte offset and its first kNameInline bytes (zero padded),
    // so a probe of a name that short is one 32-byte read, not id -> offsets -> bytes.
    static constexpr uint32_t kSlotWords = 8, kNameInline = 20;
    DevBuf<uint32_t> hslot;
    uint32_t htab_n = 0, hbits = 0;

    uint32_t size() const { return (uint32_t)names.size(); }
    uint32_t find(const char* s, uint32_t n) const;
    uint32_t intern(const char* s, uint32_t n);
    // upload new names (stream-ordered)
    void sync(hipStream_t st);
    // (re)sort ids by name on the device if names were added
    void sort(hipStream_t st, Scratch& ws);
    // sort(), then (re)build sbytes / soff if names were added
    void sort_bytes(hipStream_t st, Scratch& ws);
    // (re)build htab if names were added
    void hash_index(hipStream_t st);
};

}  // namespace rp
