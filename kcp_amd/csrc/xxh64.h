// XXH64 (published algorithm, Yann Collet), shared by the host encoder (path
// hashes) and K0's path hashes (tokdev.h).  Known answers pinned in
// tests/test_oracle_kat.py against the Python xxhash 3.8.1 package.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

namespace gd {

constexpr uint64_t XP1 = 0x9E3779B185EBCA87ULL;
constexpr uint64_t XP2 = 0xC2B2AE3D27D4EB4FULL;
constexpr uint64_t XP3 = 0x165667B19E3779F9ULL;
constexpr uint64_t XP4 = 0x85EBCA77C2B2AE63ULL;
constexpr uint64_t XP5 = 0x27D4EB2F165667C5ULL;

__host__ __device__ inline uint64_t xrotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
__host__ __device__ inline uint64_t xround(uint64_t acc, uint64_t in) {
    acc += in * XP2;
    acc = xrotl(acc, 31);
    return acc * XP1;
}
__host__ __device__ inline uint64_t xmerge(uint64_t acc, uint64_t v) {
    acc ^= xround(0, v);
    return acc * XP1 + XP4;
}
__host__ __device__ inline uint64_t xavalanche(uint64_t h) {
    h ^= h >> 33;
    h *= XP2;
    h ^= h >> 29;
    h *= XP3;
    h ^= h >> 32;
    return h;
}

// Host: arbitrary alignment.
inline uint64_t xxh64_host(const void* data, size_t len, uint64_t seed) {
    const uint8_t* p = (const uint8_t*)data;
    const uint8_t* end = p + len;
    uint64_t h;
    auto rd64 = [](const uint8_t* q) { uint64_t v; memcpy(&v, q, 8); return v; };
    auto rd32 = [](const uint8_t* q) { uint32_t v; memcpy(&v, q, 4); return v; };
    if (len >= 32) {
        uint64_t v1 = seed + XP1 + XP2, v2 = seed + XP2, v3 = seed, v4 = seed - XP1;
        const uint8_t* lim = end - 32;
        do {
            v1 = xround(v1, rd64(p));
            v2 = xround(v2, rd64(p + 8));
            v3 = xround(v3, rd64(p + 16));
            v4 = xround(v4, rd64(p + 24));
            p += 32;
        } while (p <= lim);
        h = xrotl(v1, 1) + xrotl(v2, 7) + xrotl(v3, 12) + xrotl(v4, 18);
        h = xmerge(h, v1);
        h = xmerge(h, v2);
        h = xmerge(h, v3);
        h = xmerge(h, v4);
    } else {
        h = seed + XP5;
    }
    h += (uint64_t)len;
    while (p + 8 <= end) {
        h ^= xround(0, rd64(p));
        h = xrotl(h, 27) * XP1 + XP4;
        p += 8;
    }
    if (p + 4 <= end) {
        h ^= (uint64_t)rd32(p) * XP1;
        h = xrotl(h, 23) * XP2 + XP3;
        p += 4;
    }
    while (p < end) {
        h ^= (uint64_t)(*p) * XP5;
        h = xrotl(h, 11) * XP1;
        p++;
    }
    return xavalanche(h);
}

// Tail of XXH64 over the last (len % 32) bytes held as little-endian words.
__host__ __device__ inline uint64_t xxh64_tail(uint64_t h, const uint64_t* w, uint32_t rem) {
    // w[0..3] hold up to 32 bytes; consume rem bytes
    uint32_t i = 0;
    for (; i + 8 <= rem; i += 8) {
        h ^= xround(0, w[i >> 3]);
        h = xrotl(h, 27) * XP1 + XP4;
    }
    if (i + 4 <= rem) {
        uint32_t v = (uint32_t)(w[i >> 3] >> ((i & 7) * 8));
        h ^= (uint64_t)v * XP1;
        h = xrotl(h, 23) * XP2 + XP3;
        i += 4;
    }
    for (; i < rem; i++) {
        uint64_t b = (w[i >> 3] >> ((i & 7) * 8)) & 0xFF;
        h ^= b * XP5;
        h = xrotl(h, 11) * XP1;
    }
    return h;
}

}  // namespace gd
