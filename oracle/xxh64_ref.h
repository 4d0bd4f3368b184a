// XXH64 (the published algorithm, Yann Collet) for the oracle's C++
// restatements -- TEST INFRASTRUCTURE ONLY, written independently of the
// product's kcp_amd/csrc/xxh64.h.  Pinned by tests/test_oracle_cpp.py against
// the Python xxhash 3.8.1 package.
#pragma once
#include <stdint.h>
#include <string.h>

namespace oracle {

static inline uint64_t x64_rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }

static inline uint64_t xxh64_ref(const void* data, size_t len, uint64_t seed) {
    static const uint64_t P1 = 11400714785074694791ULL, P2 = 14029467366897019727ULL,
                          P3 = 1609587929392839161ULL, P4 = 9650029242287828579ULL, P5 = 2870177450012600261ULL;
    const uint8_t* p = (const uint8_t*)data;
    const uint8_t* const end = p + len;
    auto r64 = [](const uint8_t* q) { uint64_t v; memcpy(&v, q, 8); return v; };
    auto r32 = [](const uint8_t* q) { uint32_t v; memcpy(&v, q, 4); return (uint64_t)v; };
    auto round = [&](uint64_t acc, uint64_t in) { return x64_rotl(acc + in * P2, 31) * P1; };
    uint64_t h;
    if (len >= 32) {
        uint64_t v[4] = {seed + P1 + P2, seed + P2, seed, seed - P1};
        for (; p + 32 <= end; p += 32)
            for (int k = 0; k < 4; k++) v[k] = round(v[k], r64(p + 8 * k));
        h = x64_rotl(v[0], 1) + x64_rotl(v[1], 7) + x64_rotl(v[2], 12) + x64_rotl(v[3], 18);
        for (int k = 0; k < 4; k++) h = (h ^ round(0, v[k])) * P1 + P4;
    } else {
        h = seed + P5;
    }
    h += (uint64_t)len;
    for (; p + 8 <= end; p += 8) h = x64_rotl(h ^ round(0, r64(p)), 27) * P1 + P4;
    if (p + 4 <= end) {
        h = x64_rotl(h ^ (r32(p) * P1), 23) * P2 + P3;
        p += 4;
    }
    for (; p < end; p++) h = x64_rotl(h ^ (*p * P5), 11) * P1;
    h ^= h >> 33;
    h *= P2;
    h ^= h >> 29;
    h *= P3;
    h ^= h >> 32;
    return h;
}

}  // namespace oracle
