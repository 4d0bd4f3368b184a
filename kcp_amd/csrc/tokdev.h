// Device helpers shared by K0 (tokenize.hip) and K10 (marshal.hip): wave
// primitives, Go string/number decoding, XXH64 over virtual word streams.
// Internal; each including TU gets its own copy (anonymous namespace).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gpudiff.h"
#include "decfloat.h"
#include "ryu_tables.h"
#include "tokenize.h"
#include "xxh64.h"

namespace gd {

namespace {

constexpr uint32_t TK_CLOSEQ = 0x01u;     // token code of a closing quote
constexpr uint32_t TK_OPENQ_SLOW = 0x02u; // opening quote of a string that needs decoding
// opening quotes of the exact strings "metadata", "status", "labels", "annotations"
constexpr uint32_t TK_KEY_META = 0x03u, TK_KEY_STATUS = 0x04u, TK_KEY_LABELS = 0x05u, TK_KEY_ANNOT = 0x06u;
constexpr uint32_t POS_MASK = 0xFFFFFFu;

// node info word
constexpr uint32_t NI_TAG = 7u;
constexpr uint32_t NI_LEAF = 1u << 3;
constexpr uint32_t NI_ATOM = 1u << 4;
constexpr uint32_t NI_SLOW = 1u << 5;
constexpr uint32_t NI_STR = 1u << 6;
constexpr uint32_t NI_REG_SHIFT = 8;
constexpr uint32_t NI_DEPTH_SHIFT = 16;
constexpr uint32_t KEYBIT = 0x80000000u;
constexpr uint32_t NONE = 0xFFFFFFFFu;

enum : uint32_t { R_NONE = 0, R_SPEC = 1, R_META = 2, R_LABELS = 3, R_ANNOT = 4, R_STATUS = 5 };
enum : uint32_t { E_ROOT, E_KEY, E_KEYCLOSE, E_COLON, E_VALUE, E_STRCLOSE, E_NEXT, E_END };

constexpr uint32_t kMaxDepth = 255;
#ifndef K0_WPB
#define K0_WPB 1  // one document a workgroup (profiles/r05e: 2.04 ms vs 2.30 with 2 and 2.55 with 4 per 65,536 documents)
#endif
constexpr uint32_t kWavesPerBlock = K0_WPB;  // waves (documents) per K0 workgroup
constexpr uint32_t kLdsPerWave = 5120;
constexpr uint32_t kLdsSort = 384;  // node keys sorted in LDS up to this many (12 B each)
constexpr uint32_t kLdsOrder = 768;  // phase 3b's depth order in LDS up to this many nodes (4 B each, behind 2 KiB)
constexpr uint32_t kLdsHash = 256;   // ... and up to this many nodes their hashes too (order 1 KiB + hashes 2 KiB)
constexpr uint32_t kRank = 256;      // phase 4 ranks up to this many node keys in LDS (no sort arrays)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }
__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }
__device__ __forceinline__ uint32_t popc64(uint64_t m) { return (uint32_t)__popcll(m); }
__device__ __forceinline__ uint64_t mask_lt(uint32_t n) { return n >= 64 ? ~0ULL : ((1ULL << n) - 1ULL); }
__device__ __forceinline__ uint32_t rdlane(uint32_t v, uint32_t l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l);
}
__device__ __forceinline__ uint64_t rdlane64(uint64_t v, uint32_t l) {
    return ((uint64_t)rdlane((uint32_t)(v >> 32), l) << 32) | rdlane((uint32_t)v, l);
}
__device__ __forceinline__ uint32_t shfl32(uint32_t v, uint32_t src) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)v);
}
// inclusive wave scans in six DPP steps (row_shr 1, 2, 4, 8 within each 16-lane row, then row_bcast 15 / 31 carry
// rows 0 and 0-1 into the rows after them): register-to-register, where the ds_bpermute form paid six LDS round
// trips and their waits. A lane whose DPP source does not exist, or whose row the row mask leaves out, keeps `id`
template <class Op>
__device__ __forceinline__ uint32_t dpp_incl_scan(uint32_t x, uint32_t id, Op op) {
    x = op(x, (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)x, 0x111, 0xF, 0xF, false));  // row_shr:1
    x = op(x, (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)x, 0x112, 0xF, 0xF, false));  // row_shr:2
    x = op(x, (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)x, 0x114, 0xF, 0xF, false));  // row_shr:4
    x = op(x, (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)x, 0x118, 0xF, 0xF, false));  // row_shr:8
    x = op(x, (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)x, 0x142, 0xA, 0xF, false));  // row_bcast:15
    x = op(x, (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)x, 0x143, 0xC, 0xF, false));  // row_bcast:31
    return x;
}
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    return dpp_incl_scan(v, 0u, [](uint32_t a, uint32_t b) { return a + b; });
}
// wave reductions: the scan's last lane, read into a scalar the compiler knows to be uniform (loop bounds and
// branches on it stay scalar instead of becoming exec-mask loops). Every lane must be active
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
    return rdlane(wave_incl_scan(v), 63);
}
__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
    return rdlane(dpp_incl_scan(v, 0u, [](uint32_t a, uint32_t b) { return a > b ? a : b; }), 63);
}
// the same reductions left in vector registers (K10 / K11 / K13's phases: their register allocation was tuned so)
__device__ __forceinline__ uint32_t wave_sum_v(uint32_t v) {
#pragma unroll
    for (uint32_t d = 32; d >= 1; d >>= 1) v += (uint32_t)__shfl_xor((int)v, (int)d);
    return v;
}
__device__ __forceinline__ uint32_t wave_max_v(uint32_t v) {
#pragma unroll
    for (uint32_t d = 32; d >= 1; d >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, (int)d));
    return v;
}
// the wave's own global writes become visible to its other lanes
__device__ __forceinline__ void wave_sync() { __threadfence_block(); }
// set bits of m in the lanes below this one
__device__ __forceinline__ uint32_t mbcnt64(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
// whole-wave lane shifts (DPP wave_shr:1 / wave_shl:1): lane i gets v of lane
// i - 1 (i + 1); the lane without a source gets `fill`
__device__ __forceinline__ uint32_t wave_shr1(uint32_t v, uint32_t fill) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)fill, (int)v, 0x138, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t wave_shl1(uint32_t v, uint32_t fill) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)fill, (int)v, 0x130, 0xF, 0xF, false);
}
// LDS written by this wave's lanes is read by its other lanes: LDS executes a
// wave's operations in order, so only the compiler must not reorder
__device__ __forceinline__ void lds_order() { __asm__ volatile("" ::: "memory"); }

// unaligned 8-byte read; up to 15 bytes past p must be readable
__device__ __forceinline__ uint64_t ld8u(const uint8_t* p) {
    const uintptr_t a = (uintptr_t)p;
    const uint64_t* q = (const uint64_t*)(a & ~(uintptr_t)7);
    const uint32_t sh = (uint32_t)(a & 7u) * 8u;
    const uint64_t lo = q[0], hi = q[1];  // both words always (a branch around the second cost a mask switch)
    return (lo >> sh) | ((hi << 1) << (63u - sh));  // = hi << (64 - sh), and 0 when sh = 0, without a select
}

// XXH64 over a virtual byte stream given as 8-byte little-endian words
template <class F>
__device__ __forceinline__ uint64_t xxh64_words(uint64_t seed, uint32_t len, F word) {
    uint64_t h;
    const uint32_t stripes = len >> 5;
    if (stripes) {
        uint64_t v1 = seed + XP1 + XP2, v2 = seed + XP2, v3 = seed, v4 = seed - XP1;
#pragma unroll 2
        for (uint32_t s = 0; s < stripes; s++) {
            v1 = xround(v1, word(4 * s));
            v2 = xround(v2, word(4 * s + 1));
            v3 = xround(v3, word(4 * s + 2));
            v4 = xround(v4, word(4 * s + 3));
        }
        h = xrotl(v1, 1) + xrotl(v2, 7) + xrotl(v3, 12) + xrotl(v4, 18);
        h = xmerge(h, v1);
        h = xmerge(h, v2);
        h = xmerge(h, v3);
        h = xmerge(h, v4);
    } else {
        h = seed + XP5;
    }
    h += len;
    const uint32_t rem = len & 31u;
    uint64_t w[4] = {0, 0, 0, 0};
#pragma unroll
    for (uint32_t j = 0; j < 4; j++)
        if (8 * j < rem) w[j] = word(4 * stripes + j);
    h = xxh64_tail(h, w, rem);
    return xavalanche(h);
}

// path component hashes: 0x01 u32le(len) key | 0x02 u32le(index)
__device__ __forceinline__ uint64_t hash_key(uint64_t seed, const uint8_t* k, uint32_t klen) {
    return xxh64_words(seed, klen + 5u, [&](uint32_t i) -> uint64_t {
        if (i == 0) return 0x01ull | ((uint64_t)klen << 8) | (ld8u(k) << 40);
        return ld8u(k + 8u * i - 5u);
    });
}
// XXH64 of a stream of at most 32 bytes held in four registers (W0..W3: its 8-byte little-endian words), straight
// code without loops or arrays: the same value as xxh64_words over those words
__device__ __forceinline__ uint64_t xxh64_small(uint64_t seed, uint32_t L, uint64_t W0, uint64_t W1, uint64_t W2,
                                                uint64_t W3) {
    uint64_t h;
    if (L >= 32u) {  // exactly one stripe
        const uint64_t v1 = xround(seed + XP1 + XP2, W0), v2 = xround(seed + XP2, W1), v3 = xround(seed, W2),
                       v4 = xround(seed - XP1, W3);
        h = xrotl(v1, 1) + xrotl(v2, 7) + xrotl(v3, 12) + xrotl(v4, 18);
        h = xmerge(xmerge(xmerge(xmerge(h, v1), v2), v3), v4);
    } else {
        h = seed + XP5;
    }
    h += L;
    const uint32_t rem = L & 31u, n8 = rem >> 3;
    uint64_t hn = xrotl(h ^ xround(0, W0), 27) * XP1 + XP4;
    h = n8 > 0u ? hn : h;
    hn = xrotl(h ^ xround(0, W1), 27) * XP1 + XP4;
    h = n8 > 1u ? hn : h;
    hn = xrotl(h ^ xround(0, W2), 27) * XP1 + XP4;
    h = n8 > 2u ? hn : h;
    uint64_t wr = n8 == 0u ? W0 : n8 == 1u ? W1 : n8 == 2u ? W2 : W3;
    uint32_t r = rem & 7u;
    const uint64_t h4 = xrotl(h ^ ((uint64_t)(uint32_t)wr * XP1), 23) * XP2 + XP3;
    const bool four = r >= 4u;
    h = four ? h4 : h;
    wr = four ? wr >> 32 : wr;
    r = four ? r - 4u : r;
#pragma unroll
    for (uint32_t k = 0; k < 3u; k++) {
        const uint64_t hk = xrotl(h ^ (((wr >> (8u * k)) & 0xFFu) * XP5), 11) * XP1;
        h = k < r ? hk : h;  // a select, not a branch
    }
    return xavalanche(h);
}
// hash_key over a key of at most 27 bytes held in registers: w0..w3 = the 32 bytes at the key (ld32u); word i >= 1
// of the component holds key bytes [8i - 5, 8i + 3), the high five bytes of w[i - 1] and the low three of w[i]
__device__ __forceinline__ uint64_t hash_key_w(uint64_t seed, uint32_t klen, uint64_t w0, uint64_t w1, uint64_t w2,
                                               uint64_t w3) {
    return xxh64_small(seed, klen + 5u, 0x01ull | ((uint64_t)klen << 8) | (w0 << 40), (w0 >> 24) | (w1 << 40),
                       (w1 >> 24) | (w2 << 40), (w2 >> 24) | (w3 << 40));
}
__device__ __forceinline__ uint64_t hash_index_w(uint64_t seed, uint32_t idx) {
    return xxh64_small(seed, 5u, 0x02ull | ((uint64_t)idx << 8), 0ull, 0ull, 0ull);
}
__device__ __forceinline__ uint64_t hash_index(uint64_t seed, uint32_t idx) {
    return xxh64_words(seed, 5u, [&](uint32_t) -> uint64_t { return 0x02ull | ((uint64_t)idx << 8); });
}
__device__ __forceinline__ uint64_t hash_bytes(const uint8_t* p, uint32_t len) {
    return xxh64_words(0, len, [&](uint32_t i) -> uint64_t { return ld8u(p + 8u * i); });
}

__device__ __forceinline__ uint64_t seg_bytes(uint32_t l, uint32_t arena) { return (uint64_t)l * 16u + arena; }
__device__ __forceinline__ uint32_t meta_arena(uint32_t m) {
    // long strings: the tail past the first 8 bytes, at a 4-byte aligned arena offset (include/gpudiff_format.h)
    return ((m & 7u) == GPUDIFF_TAG_STR && (m >> 3) > GPUDIFF_INLINE_MAX) ? (((m >> 3) - GPUDIFF_INLINE_MAX + 3u) & ~3u)
                                                                         : 0u;
}

__device__ __forceinline__ bool is_ws(uint32_t c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }
__device__ __forceinline__ bool is_delim(uint32_t c) {
    return is_ws(c) || c == ',' || c == '}' || c == ']' || c == ':' || c == '"' || c == '{' || c == '[';
}
__device__ __forceinline__ bool is_digit(uint32_t c) { return c - '0' < 10u; }

// utf8.DecodeRune validity (json.cpp go_rune_len): sequence size, 0 if invalid
__device__ int rune_len(const uint8_t* p, const uint8_t* end) {
    const uint32_t c0 = p[0];
    int size;
    uint32_t lo = 0x80, hi = 0xBF;
    if (c0 < 0x80) return 1;
    if (c0 >= 0xC2 && c0 <= 0xDF) size = 2;
    else if (c0 == 0xE0) { size = 3; lo = 0xA0; }
    else if ((c0 >= 0xE1 && c0 <= 0xEC) || c0 == 0xEE || c0 == 0xEF) size = 3;
    else if (c0 == 0xED) { size = 3; hi = 0x9F; }
    else if (c0 == 0xF0) { size = 4; lo = 0x90; }
    else if (c0 >= 0xF1 && c0 <= 0xF3) size = 4;
    else if (c0 == 0xF4) { size = 4; hi = 0x8F; }
    else return 0;
    if (end - p < size) return 0;
    if (p[1] < lo || p[1] > hi) return 0;
    for (int k = 2; k < size; k++)
        if (p[k] < 0x80 || p[k] > 0xBF) return 0;
    return size;
}
__device__ __forceinline__ int hexv(uint32_t c) {
    if (c - '0' < 10u) return (int)(c - '0');
    if (c - 'a' < 6u) return (int)(c - 'a' + 10);
    if (c - 'A' < 6u) return (int)(c - 'A' + 10);
    return -1;
}
__device__ int getu4(const uint8_t* p, const uint8_t* end) {
    if (end - p < 6 || p[0] != '\\' || p[1] != 'u') return -1;
    int v = 0;
    for (int k = 2; k < 6; k++) {
        const int h = hexv(p[k]);
        if (h < 0) return -1;
        v = (v << 4) | h;
    }
    return v;
}
__device__ __forceinline__ uint8_t* put_utf8(uint8_t* o, uint32_t r) {
    if (r < 0x80) {
        *o++ = (uint8_t)r;
    } else if (r < 0x800) {
        *o++ = (uint8_t)(0xC0 | (r >> 6));
        *o++ = (uint8_t)(0x80 | (r & 0x3F));
    } else if (r < 0x10000) {
        *o++ = (uint8_t)(0xE0 | (r >> 12));
        *o++ = (uint8_t)(0x80 | ((r >> 6) & 0x3F));
        *o++ = (uint8_t)(0x80 | (r & 0x3F));
    } else {
        *o++ = (uint8_t)(0xF0 | (r >> 18));
        *o++ = (uint8_t)(0x80 | ((r >> 12) & 0x3F));
        *o++ = (uint8_t)(0x80 | ((r >> 6) & 0x3F));
        *o++ = (uint8_t)(0x80 | (r & 0x3F));
    }
    return o;
}

// Go string decoding (encoding/json unquote, json.cpp JsonParser::string):
// raw bytes [p, q) between the quotes -> dst (never longer than the raw
// bytes); returns the decoded length, or -1 for the host to decide (invalid
// escape or control character: a Go error; invalid UTF-8: U+FFFD repair)
__device__ int decode_string(const uint8_t* p, const uint8_t* q, const uint8_t* end, uint8_t* dst) {
    uint8_t* o = dst;
    while (p < q) {
        const uint32_t c = *p;
        if (c == '\\') {
            if (end - p < 2) return -1;
            const uint32_t e = p[1];
            uint32_t b = 0;
            switch (e) {
                case '"': b = '"'; break;
                case '\\': b = '\\'; break;
                case '/': b = '/'; break;
                case 'b': b = '\b'; break;
                case 'f': b = '\f'; break;
                case 'n': b = '\n'; break;
                case 'r': b = '\r'; break;
                case 't': b = '\t'; break;
                case 'u': {
                    int rr = getu4(p, end);
                    if (rr < 0) return -1;
                    p += 6;
                    if (rr >= 0xD800 && rr < 0xE000) {
                        const int rr1 = getu4(p, end);
                        if (rr < 0xDC00 && rr1 >= 0xDC00 && rr1 < 0xE000) {
                            const uint32_t dec = (((uint32_t)(rr - 0xD800) << 10) | (uint32_t)(rr1 - 0xDC00)) + 0x10000u;
                            o = put_utf8(o, dec);
                            p += 6;
                            continue;
                        }
                        rr = 0xFFFD;
                    }
                    o = put_utf8(o, (uint32_t)rr);
                    continue;
                }
                default: return -1;
            }
            *o++ = (uint8_t)b;
            p += 2;
            continue;
        }
        if (c < 0x20) return -1;
        if (c < 0x80) {
            *o++ = (uint8_t)c;
            p++;
            continue;
        }
        const int l = rune_len(p, end);
        if (l == 0) return -1;  // U+FFFD repair would outgrow the in-place area: host encoder
        for (int k = 0; k < l; k++) *o++ = p[k];
        p += l;
    }
    return (int)(o - dst);
}
// decode_string(p, p + raw, end, dst) by the whole wave (every lane gets the answer): a lane per byte over coalesced
// loads instead of one lane's dependent byte-by-byte loop.  Bytes are paired with escapes as decode_string pairs them
// (a backslash not itself escaped escapes the next byte; a \u's four digits hold no backslash, or the string is
// invalid anyway), so it fails exactly on a control byte, an invalid escape or a \u without four hex digits (the
// closing quote, never a digit, bounds them).  WRITE (K10): the decoded bytes go to dst -- an escaped byte maps to
// its character, its backslash emits nothing -- and the length is returned; a string with a \u escape or a
// non-ASCII byte is decoded by lane 0's decode_string instead.  !WRITE (K11 / K13): only the verdict (>= 0 or -1);
// lane 0's decode_string decides only the UTF-8 validity of a string with a non-ASCII byte.
template <bool WRITE>
__device__ int wave_decode_string(const uint8_t* p, uint32_t raw, const uint8_t* end, uint8_t* dst, uint32_t lane) {
    bool bad = false, hard = false;
    uint64_t carry = 0;
    uint32_t outn = 0;
    for (uint32_t o = 0; o < raw; o += 64u) {
        const uint32_t k = o + lane;
        const bool in = k < raw;
        const uint32_t c = in ? p[k] : 0x20u;
        const uint64_t bs = ballot(in & (c == '\\'));
        uint64_t esc = carry;  // byte 0 of this chunk escaped by the previous chunk's last byte
        carry = 0;
        for (uint64_t m = bs; m; m &= m - 1) {
            const uint32_t b = (uint32_t)__builtin_ctzll(m);
            if ((esc >> b) & 1ull) continue;  // an escaped backslash escapes nothing
            if (b == 63u) carry = 1;
            else esc |= 1ull << (b + 1u);
        }
        const bool e = in & (((esc >> lane) & 1ull) != 0ull);
        const bool ok_e = (c == '"') | (c == '\\') | (c == '/') | (c == 'b') | (c == 'f') | (c == 'n') | (c == 'r') |
                          (c == 't') | (c == 'u');
        bool ubad = false;
        if (e & (c == 'u'))
            ubad = (hexv(p[k + 1]) | hexv(p[k + 2]) | hexv(p[k + 3]) | hexv(p[k + 4])) < 0;
        bad |= in & ((c < 0x20u) | (e & !ok_e) | ubad);
        hard |= in & ((c >= 0x80u) | (WRITE & e & (c == 'u')));
        if constexpr (WRITE) {
            if (ballot(hard)) break;  // lane 0's decode_string decides the whole string (its errors included)
            const bool emit = in & !((c == '\\') & !e);
            const uint32_t mc = c == 'b' ? 8u : c == 'f' ? 12u : c == 'n' ? 10u : c == 'r' ? 13u : c == 't' ? 9u : c;
            const uint64_t em = ballot(emit);
            if (emit) dst[outn + mbcnt64(em)] = (uint8_t)(e ? mc : c);
            outn += popc64(em);
        }
    }
    if (ballot(bad)) return -1;
    if (!ballot(hard)) return (int)outn;
    const int dl = lane == 0 ? decode_string(p, p + raw, end, dst) : 0;
    return (int)rdlane((uint32_t)dl, 0);
}
__device__ __forceinline__ bool wave_string_ok(const uint8_t* p, uint32_t raw, const uint8_t* end, uint8_t* dst,
                                               uint32_t lane) {
    return wave_decode_string<false>(p, raw, end, dst, lane) >= 0;
}

// literal / number (json.cpp value + number): tag + canonical 8 bytes, or a GPUDIFF_TOK_* error.  at(k) is the
// atom's k-th byte, read only for k < left (the bytes to the document's end)
template <class At>
__device__ __forceinline__ uint32_t parse_atom_core(At at, uint64_t left, uint32_t* tag, uint64_t* val) {
    const uint32_t c = at(0);
    *val = 0;
    if (c == 't' || c == 'f' || c == 'n') {
        const uint32_t n = c == 'f' ? 5u : 4u;
        if (left < n) return GPUDIFF_TOK_SYNTAX;
        uint64_t w = 0;
        for (uint32_t k = 0; k < n; k++) w |= (uint64_t)at(k) << (8u * k);
        const uint64_t want = c == 't' ? 0x65757274ull : c == 'f' ? 0x65736c6166ull : 0x6c6c756eull;
        if (w != want) return GPUDIFF_TOK_SYNTAX;
        if (n < left && !is_delim(at(n))) return GPUDIFF_TOK_SYNTAX;
        *tag = c == 't' ? GPUDIFF_TAG_TRUE : c == 'f' ? GPUDIFF_TAG_FALSE : GPUDIFF_TAG_NULL;
        return GPUDIFF_TOK_OK;
    }
    // number grammar: -? (0 | [1-9][0-9]*) (. [0-9]+)? ([eE] [+-]? [0-9]+)?
    uint64_t q = 0;
    const bool neg = c == '-';
    if (neg) q++;
    if (q >= left) return GPUDIFF_TOK_SYNTAX;
    if (at(q) == '0') {
        q++;
    } else if (at(q) >= '1' && at(q) <= '9') {
        while (q < left && is_digit(at(q))) q++;
    } else {
        return GPUDIFF_TOK_SYNTAX;
    }
    const uint64_t d0 = neg ? 1u : 0u;
    const uint64_t int_end = q;
    uint64_t frac_beg = q, frac_end = q;
    bool is_int = true;
    if (q < left && at(q) == '.') {
        is_int = false;
        q++;
        frac_beg = q;
        if (q >= left || !is_digit(at(q))) return GPUDIFF_TOK_SYNTAX;
        while (q < left && is_digit(at(q))) q++;
        frac_end = q;
    }
    int64_t ex = 0;
    if (q < left && (at(q) == 'e' || at(q) == 'E')) {
        is_int = false;
        q++;
        bool eneg = false;
        if (q < left && (at(q) == '+' || at(q) == '-')) {
            eneg = at(q) == '-';
            q++;
        }
        if (q >= left || !is_digit(at(q))) return GPUDIFF_TOK_SYNTAX;
        while (q < left && is_digit(at(q))) {
            if (ex < 100000) ex = ex * 10 + (at(q) - '0');
            q++;
        }
        if (eneg) ex = -ex;
    }
    if (q < left && !is_delim(at(q))) return GPUDIFF_TOK_SYNTAX;
    if (is_int) {  // strconv.ParseInt(s, 10, 64)
        const uint64_t lim = neg ? (1ull << 63) : ((1ull << 63) - 1ull);
        uint64_t v = 0;
        bool ovf = false;
        for (uint64_t k = d0; k < int_end; k++) {
            const uint64_t dig = (uint64_t)(at(k) - '0');
            if (v > (lim - dig) / 10) {
                ovf = true;
                break;
            }
            v = v * 10 + dig;
        }
        if (!ovf) {
            *tag = GPUDIFF_TAG_INT;
            *val = neg ? (0ull - v) : v;
            return GPUDIFF_TOK_OK;
        }
        // beyond int64: convertNumber falls back to float64
    }
    // strconv.ParseFloat on the significant digits (first to last nonzero),
    // <= 19 of them: decfloat.h (Clinger's exact path, else Eisel-Lemire)
    const uint32_t n_int = (uint32_t)(int_end - d0), n_frac = (uint32_t)(frac_end - frac_beg);
    const uint32_t n_all = n_int + n_frac;
    auto digit = [&](uint32_t k) -> uint32_t { return at(k < n_int ? d0 + k : frac_beg + (k - n_int)) - '0'; };
    uint32_t first = n_all, last = 0;
    for (uint32_t k = 0; k < n_all; k++)
        if (digit(k)) {
            if (first == n_all) first = k;
            last = k;
        }
    *tag = GPUDIFF_TAG_FLOAT;
    if (first == n_all) {
        *val = 0;  // +-0.0 -> +0.0 (Go ==)
        return GPUDIFF_TOK_OK;
    }
    if (last - first + 1 > 19) return GPUDIFF_TOK_NUMBER;
    uint64_t w = 0;
    for (uint32_t k = first; k <= last; k++) w = w * 10 + digit(k);
    const int64_t e10 = ex - (int64_t)n_frac + (int64_t)(n_all - 1 - last);
    uint64_t bits;
    if (!decimal_to_double(w, e10, neg, &bits)) return GPUDIFF_TOK_NUMBER;
    *val = bits;
    return GPUDIFF_TOK_OK;
}
// byte by byte from memory (K10 / K11 / K13: their larger kernels keep no window)
__device__ uint32_t parse_atom_mem(const uint8_t* p, const uint8_t* end, uint32_t* tag, uint64_t* val) {
    return parse_atom_core([&](uint64_t k) -> uint32_t { return p[k]; }, (uint64_t)(end - p), tag, val);
}

// the bytes at p in two / four registers (aligned-word loads issued together; p + 23 must be readable)
__device__ __forceinline__ void ld16u(const uint8_t* p, uint64_t* w0, uint64_t* w1) {
    const uintptr_t a = (uintptr_t)p;
    const uint64_t* q = (const uint64_t*)(a & ~(uintptr_t)7);
    const uint32_t sh = (uint32_t)(a & 7u) * 8u;
    const uint64_t x0 = q[0], x1 = q[1], x2 = q[2];
    *w0 = (x0 >> sh) | ((x1 << 1) << (63u - sh));
    *w1 = (x1 >> sh) | ((x2 << 1) << (63u - sh));
}
// (ld32u: only the words wholly before lim are read, the others are zero -- a document is readable to kTokSlack = 32
// bytes past its end, and a 32-byte window at its last bytes reaches up to 40)
__device__ __forceinline__ void ld32u(const uint8_t* p, const uint8_t* lim, uint64_t& w0, uint64_t& w1, uint64_t& w2,
                                      uint64_t& w3) {
    const uintptr_t a = (uintptr_t)p;
    const uint64_t* q = (const uint64_t*)(a & ~(uintptr_t)7);
    const uint32_t sh = (uint32_t)(a & 7u) * 8u;
    const uint64_t* ql = (const uint64_t*)lim;
    // the words past lim read as zero: their loads go to q[0] instead (a select of addresses, not a branch)
    const bool r3 = q + 4 <= ql, r4 = q + 5 <= ql;
    const uint64_t y3 = *(r3 ? q + 3 : q), y4 = *(r4 ? q + 4 : q);
    const uint64_t x0 = q[0], x1 = q[1], x2 = q[2], x3 = r3 ? y3 : 0ull, x4 = r4 ? y4 : 0ull;
    w0 = (x0 >> sh) | ((x1 << 1) << (63u - sh));
    w1 = (x1 >> sh) | ((x2 << 1) << (63u - sh));
    w2 = (x2 >> sh) | ((x3 << 1) << (63u - sh));
    w3 = (x3 >> sh) | ((x4 << 1) << (63u - sh));
}
// byte k of a 16-byte window: a select by mask (a ternary became a private array and scratch loads)
__device__ __forceinline__ uint32_t win16_at(uint64_t w0, uint64_t w1, uint32_t k) {
    const uint64_t m = 0ull - (uint64_t)((k >> 3) & 1u);
    return (uint32_t)((((w0 & ~m) | (w1 & m)) >> (8u * (k & 7u))) & 0xFFu);
}
// K0's sort of up to kRank node keys: keys[j] & mask (j < ns) are node j + 1's key, in LDS (phase 3b's hashes).
// Lane k ranks keys k, k + 64, ... by counting the keys below each -- all ns read two at a time by broadcast -- and
// writes its nodes' ids to their ranks in ids. Ranks are a permutation when the keys are distinct; an equal pair (a
// duplicate or a collision under the seed) or a key equal to the root's hash sets GPUDIFF_TOK_HASH instead, as the
// bitonic path's check does
template <int NK>
__device__ __forceinline__ void rank_sort_n(const uint64_t* keys, uint64_t mask, uint16_t* ids, uint32_t ns,
                                            uint32_t lane, uint64_t root, uint32_t& status) {
    uint64_t k[NK];
    uint32_t r[NK], e[NK];
#pragma unroll
    for (int q = 0; q < NK; q++) {
        k[q] = lane + 64u * q < ns ? keys[lane + 64u * q] & mask : 0ull;
        r[q] = 0u;
        e[q] = 0u;
    }
    const uint32_t np = ns & ~1u;
    for (uint32_t j = 0; j < np; j += 2) {
        const uint64_t a = keys[j] & mask, b = keys[j + 1] & mask;
#pragma unroll
        for (int q = 0; q < NK; q++) {
            r[q] += (uint32_t)(a < k[q]) + (uint32_t)(b < k[q]);
            e[q] += (uint32_t)(a == k[q]) + (uint32_t)(b == k[q]);
        }
    }
    if (np < ns) {
        const uint64_t a = keys[np] & mask;
#pragma unroll
        for (int q = 0; q < NK; q++) {
            r[q] += (uint32_t)(a < k[q]);
            e[q] += (uint32_t)(a == k[q]);
        }
    }
    bool dup = false;
#pragma unroll
    for (int q = 0; q < NK; q++)
        if (lane + 64u * q < ns && (e[q] > 1u || k[q] == root)) dup = true;
    if (__builtin_amdgcn_ballot_w64(dup)) {
        status = GPUDIFF_TOK_HASH;
        return;
    }
#pragma unroll
    for (int q = 0; q < NK; q++)
        if (lane + 64u * q < ns) ids[r[q]] = (uint16_t)(lane + 64u * q + 1u);
    __asm__ volatile("" ::: "memory");
}
__device__ __forceinline__ void rank_sort(const uint64_t* keys, uint64_t mask, uint16_t* ids, uint32_t ns,
                                          uint32_t lane, uint64_t root, uint32_t& status) {
    if (ns <= 64u) rank_sort_n<1>(keys, mask, ids, ns, lane, root, status);
    else if (ns <= 128u) rank_sort_n<2>(keys, mask, ids, ns, lane, root, status);
    else rank_sort_n<4>(keys, mask, ids, ns, lane, root, status);
}

// K0's values pass: the common atoms -- true, false, null and integers of at most 15 digits ending in a delimiter or
// the document's end -- from the 16-byte register window w0, w1 at the atom (left: bytes to the document's end).
// 0: decided (tag, val); 1: not decided here -- floats, exponents, longer numbers, any syntax doubt go to
// parse_atom_win (K0's slow-atom pass), whose answers are parse_atom_mem's, so results are by construction.
__device__ __forceinline__ uint32_t parse_atom_fast(uint64_t w0, uint64_t w1, uint64_t left, uint32_t* tag,
                                                    uint64_t* val) {
    const uint32_t avail = left < 16u ? (uint32_t)left : 16u;
    const uint32_t c = (uint32_t)(w0 & 0xFFu);
    if (c == 't' || c == 'f' || c == 'n') {
        const uint32_t n = c == 'f' ? 5u : 4u;
        const uint64_t want = c == 't' ? 0x65757274ull : c == 'f' ? 0x65736c6166ull : 0x6c6c756eull;
        if (avail >= n && (w0 & ((1ull << (8 * n)) - 1ull)) == want &&
            (avail == n ? left == n : is_delim(win16_at(w0, w1, n)))) {
            *val = 0;
            *tag = c == 't' ? GPUDIFF_TAG_TRUE : c == 'f' ? GPUDIFF_TAG_FALSE : GPUDIFF_TAG_NULL;
            return 0u;
        }
        return 1u;
    }
    const uint32_t d0 = c == '-' ? 1u : 0u;
    uint32_t k = d0;
    uint64_t v = 0;
    bool run = true;
    // the digit run, 16 predicated steps (a loop with a per-lane trip count switched the exec mask every step)
#pragma unroll
    for (uint32_t s = 0; s < 16u; s++) {
        const uint32_t cs = (uint32_t)(((s < 8u ? w0 : w1) >> (8u * (s & 7u))) & 0xFFu);
        const bool dig = run & (s >= d0) & (s < avail) & is_digit(cs);
        v = dig ? v * 10u + (cs - '0') : v;
        k = dig ? s + 1u : k;
        run = run & ((s < d0) | dig);
    }
    const uint32_t nd = k - d0;
    // accepted: 1..15 digits, no leading zero unless alone, then the document's end or a delimiter that is not
    // the start of a fraction or an exponent ('.', 'e', 'E' are no delimiters)
    const bool at_end = k == avail && left == avail;
    if (nd == 0 || nd > 15 || (win16_at(w0, w1, d0) == '0' && nd > 1) ||
        !(at_end || (k < avail && is_delim(win16_at(w0, w1, k)))))
        return 1u;
    *tag = GPUDIFF_TAG_INT;
    *val = d0 ? 0ull - v : v;
    return 0u;
}
// K11 / K13: parse_atom_mem's answer, from a 16-byte window when parse_atom_fast decides the atom (the common
// literals and short integers: two word loads instead of a dependent load per byte); p + 23 must be readable, as a
// document is to kTokSlack bytes past its end
__device__ __forceinline__ uint32_t parse_atom_quick(const uint8_t* p, const uint8_t* end, uint32_t* tag, uint64_t* val) {
    uint64_t w0, w1;
    ld16u(p, &w0, &w1);
    if (parse_atom_fast(w0, w1, (uint64_t)(end - p), tag, val) == 0u) return GPUDIFF_TOK_OK;
    return parse_atom_mem(p, end, tag, val);
}
// any atom from the 32-byte register window w at p (ld32u); one that runs past the window is parsed from memory
__device__ __forceinline__ uint32_t parse_atom_win(const uint8_t* p, const uint8_t* end, uint64_t w0, uint64_t w1,
                                                   uint64_t w2, uint64_t w3, uint32_t* tag, uint64_t* val) {
    bool spill = false;
    const uint32_t e = parse_atom_core(
        [&](uint64_t j) -> uint32_t {
            // past the window: 0xFF, neither a digit, a sign, '.', 'e' nor a delimiter -- the parse stops there and
            // the atom is parsed again from memory (selects, no branch)
            const bool past = j >= 32u;
            spill |= past;
            const uint32_t k = (uint32_t)j & 31u;  // selects by mask, as win16_at
            const uint64_t m8 = 0ull - (uint64_t)((k >> 3) & 1u), m16 = 0ull - (uint64_t)((k >> 4) & 1u);
            const uint64_t lo = (w0 & ~m8) | (w1 & m8), hi = (w2 & ~m8) | (w3 & m8);
            return past ? 0xFFu : (uint32_t)((((lo & ~m16) | (hi & m16)) >> (8u * (k & 7u))) & 0xFFu);
        },
        (uint64_t)(end - p), tag, val);
    return spill ? parse_atom_mem(p, end, tag, val) : e;
}

// ---- K10 (write path) helpers: Go 1.16 encodeState.string(s, escapeHTML=true)
// over decoded (valid UTF-8) bytes; strconv.AppendInt
__device__ __forceinline__ uint32_t go_esc_len(const uint8_t* s, uint32_t n) {
    uint32_t out = 0;
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t c = s[i];
        if (c < 0x80u) {
            if (c == '"' || c == '\\' || c == '\n' || c == '\r' || c == '\t') out += 2;
            else if (c < 0x20u || c == '<' || c == '>' || c == '&') out += 6;
            else out += 1;
        } else if (c == 0xE2u && i + 2 < n && s[i + 1] == 0x80u && (s[i + 2] == 0xA8u || s[i + 2] == 0xA9u)) {
            out += 6;  // U+2028 / U+2029
            i += 2;
        } else {
            out += 1;
        }
    }
    return out;
}
__device__ __forceinline__ uint8_t* go_esc_put(uint8_t* o, const uint8_t* s, uint32_t n) {
    const char* hx = "0123456789abcdef";
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t c = s[i];
        if (c < 0x80u) {
            if (c == '"' || c == '\\') {
                *o++ = '\\';
                *o++ = (uint8_t)c;
            } else if (c == '\n' || c == '\r' || c == '\t') {
                *o++ = '\\';
                *o++ = c == '\n' ? 'n' : c == '\r' ? 'r' : 't';
            } else if (c < 0x20u || c == '<' || c == '>' || c == '&') {
                *o++ = '\\';
                *o++ = 'u';
                *o++ = '0';
                *o++ = '0';
                *o++ = (uint8_t)hx[c >> 4];
                *o++ = (uint8_t)hx[c & 15u];
            } else {
                *o++ = (uint8_t)c;
            }
        } else if (c == 0xE2u && i + 2 < n && s[i + 1] == 0x80u && (s[i + 2] == 0xA8u || s[i + 2] == 0xA9u)) {
            *o++ = '\\';
            *o++ = 'u';
            *o++ = '2';
            *o++ = '0';
            *o++ = '2';
            *o++ = s[i + 2] == 0xA8u ? '8' : '9';
            i += 2;
        } else {
            *o++ = (uint8_t)c;
        }
    }
    return o;
}
// wave-cooperative escaping of long strings: the output length of byte i
// (1, 2 or 6; the three bytes of U+2028 / U+2029 give 6, 0, 0 -- E2 is a lead
// byte, so a 0x80 / 0xA8 after it is that sequence's continuation)
__device__ __forceinline__ uint32_t esc_unit(const uint8_t* s, uint32_t n, uint32_t i) {
    const uint32_t c = s[i];
    if (c < 0x80u) {
        if (c == '"' || c == '\\' || c == '\n' || c == '\r' || c == '\t') return 2;
        return (c < 0x20u || c == '<' || c == '>' || c == '&') ? 6u : 1u;
    }
    if (c == 0xE2u) return (i + 2 < n && s[i + 1] == 0x80u && (s[i + 2] == 0xA8u || s[i + 2] == 0xA9u)) ? 6u : 1u;
    if (c == 0x80u) return (i >= 1 && s[i - 1] == 0xE2u && i + 1 < n && (s[i + 1] == 0xA8u || s[i + 1] == 0xA9u)) ? 0u : 1u;
    if (c == 0xA8u || c == 0xA9u) return (i >= 2 && s[i - 1] == 0x80u && s[i - 2] == 0xE2u) ? 0u : 1u;
    return 1u;
}
__device__ __forceinline__ uint32_t wave_esc_len(const uint8_t* s, uint32_t n) {
    uint32_t acc = 0;
    for (uint32_t b = 0; b < n; b += 64) {
        const uint32_t i = b + __lane_id();
        acc += i < n ? esc_unit(s, n, i) : 0u;
    }
    return wave_sum(acc);
}
// writes the escaped bytes of s[0, n) at o (the whole wave)
__device__ __forceinline__ void wave_esc_put(uint8_t* o, const uint8_t* s, uint32_t n) {
    const char* hx = "0123456789abcdef";
    uint32_t run = 0;
    for (uint32_t b = 0; b < n; b += 64) {
        const uint32_t i = b + __lane_id();
        const uint32_t u = i < n ? esc_unit(s, n, i) : 0u;
        const uint32_t inc = wave_incl_scan(u);
        uint8_t* q = o + run + inc - u;
        if (u == 1) {
            q[0] = s[i];
        } else if (u == 2) {
            const uint32_t c = s[i];
            q[0] = '\\';
            q[1] = c == '\n' ? 'n' : c == '\r' ? 'r' : c == '\t' ? 't' : (uint8_t)c;
        } else if (u == 6) {
            const uint32_t c = s[i];
            q[0] = '\\';
            q[1] = 'u';
            if (c == 0xE2u) {
                q[2] = '2';
                q[3] = '0';
                q[4] = '2';
                q[5] = s[i + 2] == 0xA8u ? '8' : '9';
            } else {
                q[2] = '0';
                q[3] = '0';
                q[4] = (uint8_t)hx[c >> 4];
                q[5] = (uint8_t)hx[c & 15u];
            }
        }
        run += __builtin_amdgcn_readlane((int)inc, 63);
    }
}
constexpr uint32_t kLongString = 16;

// ---- flattened string passes (K10, K0's keys): every lane's string (at most one per lane) is cut into 8-byte
// units (4-byte ones for wave_copy_dwords0) laid end to end; each pass the wave takes 64 consecutive units, a unit's owner lane found by a
// binary search over the inclusive unit prefix (as K2 does over 16-B chunks), so a window's strings of
// any length cost sum(len) / 256 passes instead of one pass per long string plus the longest short one.
// Unit loads read up to 15 bytes past a string (ld8u): the JSON and decoded-string buffers keep that slack.
__device__ __forceinline__ uint64_t shfl64(uint64_t v, uint32_t src) {
    return ((uint64_t)shfl32((uint32_t)(v >> 32), src) << 32) | shfl32((uint32_t)v, src);
}
struct FlatUnits {
    uint32_t incl, total;
};
__device__ __forceinline__ FlatUnits flat_units(bool has, uint32_t n) {
    const uint32_t units = has ? (n + 3u) >> 2 : 0u;
    const uint32_t incl = wave_incl_scan(units);
    return FlatUnits{incl, rdlane(incl, 63)};
}
// 8-byte units (wave_esc_extra, wave_copy_flat: half the passes of 4-byte ones, each still one ld8u per lane)
__device__ __forceinline__ FlatUnits flat_units8(bool has, uint32_t n) {
    const uint32_t units = has ? (n + 7u) >> 3 : 0u;
    const uint32_t incl = wave_incl_scan(units);
    return FlatUnits{incl, rdlane(incl, 63)};
}
// any byte of x that Go's HTML-safe string encoder does not write as itself: < 0x20, >= 0x80, '"', '\\', '<', '>',
// '&' (SWAR: exact as to "any", which is all the caller asks before its per-byte pass)
__device__ __forceinline__ bool swar_has_esc(uint64_t x) {
    constexpr uint64_t L = 0x0101010101010101ull, H = 0x8080808080808080ull;
    auto has0 = [&](uint64_t v) -> uint64_t { return (v - L) & ~v & H; };
    const uint64_t lt20 = (x - 0x20u * L) & ~x & H;
    return ((x & H) | lt20 | has0(x ^ ('"' * L)) | has0(x ^ ('\\' * L)) | has0(x ^ ('<' * L)) | has0(x ^ ('>' * L)) |
            has0(x ^ ('&' * L))) != 0ull;
}
// owner lane of unit g (the first lane whose inclusive prefix exceeds g; 63 past the end)
__device__ __forceinline__ uint32_t flat_owner(const FlatUnits& f, uint32_t g) {
    uint32_t o = 0;
#pragma unroll
    for (uint32_t st = 32; st >= 1; st >>= 1)
        if (shfl32(f.incl, o + st - 1u) <= g) o += st;
    return min(o, 63u);
}
// extra output bytes of this lane's string s[0, n) under Go's HTML-safe escaping (escaped length - n);
// 0 iff every byte is written as it is
__device__ uint32_t wave_esc_extra(bool has, const uint8_t* s, uint32_t n) {
    const uint32_t lane = __lane_id();
    const FlatUnits f = flat_units8(has, n);
    const uint32_t units = has ? (n + 7u) >> 3 : 0u;
    const uint64_t sp = (uint64_t)(uintptr_t)s;
    int32_t acc = 0;
    for (uint32_t b = 0; b < f.total; b += 64) {
        const uint32_t g = b + lane;
        const uint32_t o = flat_owner(f, g);
        const uint32_t first = shfl32(f.incl - units, o), on = shfl32(n, o);
        const uint64_t op = shfl64(sp, o);
        int32_t extra = 0;
        if (g < f.total) {
            const uint32_t k = 8u * (g - first);
            const uint8_t* p = (const uint8_t*)(uintptr_t)op;
            const uint64_t w = ld8u(p + k);
            const uint32_t nb = min(8u, on - k);
            // the bytes past the string read as 'a' (plain)
            const uint64_t keep = nb >= 8u ? ~0ull : (1ull << (8u * nb)) - 1ull;
            if (swar_has_esc((w & keep) | (0x6161616161616161ull & ~keep))) {  // rare: the bytes one by one
                for (uint32_t j = 0; j < nb; j++) {
                    const uint32_t c = (uint32_t)(w >> (8u * j)) & 0xFFu;
                    const bool plain = c >= 0x20u && c < 0x80u && c != '"' && c != '\\' && c != '<' && c != '>' && c != '&';
                    if (!plain) extra += (int32_t)esc_unit(p, on, k + j) - 1;
                }
            }
        }
        for (uint64_t m = __ballot(extra != 0); m; m &= m - 1) {  // escapes are rare
            const uint32_t j = (uint32_t)__builtin_ctzll(m);
            const int32_t e = (int32_t)rdlane((uint32_t)extra, j);
            if (lane == rdlane(o, j)) acc += e;
        }
    }
    return (uint32_t)acc;
}
// copies this lane's string s[0, n) to o[0, n) (strings that need no escaping)
__device__ void wave_copy_flat(bool has, const uint8_t* s, uint32_t n, uint8_t* o) {
    const uint32_t lane = __lane_id();
    const FlatUnits f = flat_units8(has, n);
    const uint32_t units = has ? (n + 7u) >> 3 : 0u;
    const uint64_t sp = (uint64_t)(uintptr_t)s, dp = (uint64_t)(uintptr_t)o;
    for (uint32_t b = 0; b < f.total; b += 64) {
        const uint32_t g = b + lane;
        const uint32_t ow = flat_owner(f, g);
        const uint32_t first = shfl32(f.incl - units, ow), on = shfl32(n, ow);
        const uint64_t op = shfl64(sp, ow), od = shfl64(dp, ow);
        if (g < f.total) {
            const uint32_t k = 8u * (g - first);
            const uint64_t w = ld8u((const uint8_t*)(uintptr_t)op + k);
            uint8_t* q = (uint8_t*)(uintptr_t)od + k;
            const uint32_t nb = min(8u, on - k);
            q[0] = (uint8_t)w;
#pragma unroll
            for (uint32_t j = 1; j < 8; j++)
                if (nb > j) q[j] = (uint8_t)(w >> (8u * j));
        }
    }
}

// copies this lane's n bytes at s into 4-byte aligned o as whole dwords, the last one zero past n (K0's arena
// tails), flattened over the wave like wave_copy_flat
__device__ void wave_copy_dwords0(bool has, const uint8_t* s, uint32_t n, uint32_t* o) {
    const uint32_t lane = __lane_id();
    const FlatUnits f = flat_units(has, n);
    const uint32_t units = has ? (n + 3u) >> 2 : 0u;
    const uint64_t sp = (uint64_t)(uintptr_t)s, dp = (uint64_t)(uintptr_t)o;
    for (uint32_t b = 0; b < f.total; b += 64) {
        const uint32_t g = b + lane;
        const uint32_t ow = flat_owner(f, g);
        const uint32_t first = shfl32(f.incl - units, ow), on = shfl32(n, ow);
        const uint64_t op = shfl64(sp, ow), od = shfl64(dp, ow);
        if (g < f.total) {
            const uint32_t u = g - first;
            uint32_t w = (uint32_t)ld8u((const uint8_t*)(uintptr_t)op + 4u * u);
            const uint32_t rem = on - 4u * u;
            if (rem < 4u) w &= (1u << (8u * rem)) - 1u;
            ((uint32_t*)(uintptr_t)od)[u] = w;
        }
    }
}

// ---- float64 -> Go text (floatEncoder(64): strconv.AppendFloat(f, 'f'|'e', -1, 64)
// with the 1e-6 / 1e21 switch and the e-09 -> e-9 clean-up).  The shortest,
// closest (ties to even) digit string is Ryu's (Adams, PLDI 2018): this is
// tools/gen_ryu_table.py d2d_model restated over the same 125-bit tables.
__device__ __forceinline__ uint32_t ryu_pow5bits(int32_t e) { return (uint32_t)(((uint32_t)e * 1217359u) >> 19) + 1u; }
__device__ __forceinline__ uint64_t ryu_mulshift(uint64_t m, const uint64_t* mul, int32_t j) {
    // (m * mul) >> j over the 192-bit product; j >= 64
    const uint64_t b0_hi = __umul64hi(m, mul[0]);
    const uint64_t b2_lo = m * mul[1], b2_hi = __umul64hi(m, mul[1]);
    const uint64_t s_lo = b2_lo + b0_hi, s_hi = b2_hi + (s_lo < b2_lo ? 1ull : 0ull);
    const int32_t sh = j - 64;
    if (sh == 0) return s_lo;
    if (sh >= 64) return s_hi >> (sh - 64);
    return (s_lo >> sh) | (s_hi << (64 - sh));
}
__device__ __forceinline__ bool ryu_pow5_multiple(uint64_t v, int32_t p) {
    int32_t c = 0;
    while (v % 5u == 0u) {
        v /= 5u;
        if (++c >= p) return true;
    }
    return c >= p;
}
// finite nonzero double -> (digits, decimal exponent of the last digit)
__device__ inline void ryu_d2d(uint64_t bits, uint64_t* digits, int32_t* exp10) {
    const uint64_t ieee_m = bits & ((1ull << 52) - 1ull);
    const uint32_t ieee_e = (uint32_t)((bits >> 52) & 0x7FFu);
    int32_t e2;
    uint64_t m2;
    if (ieee_e == 0) {
        e2 = 1 - 1023 - 52 - 2;
        m2 = ieee_m;
    } else {
        e2 = (int32_t)ieee_e - 1023 - 52 - 2;
        m2 = (1ull << 52) | ieee_m;
    }
    const bool accept = (m2 & 1u) == 0;
    const uint64_t mv = 4u * m2;
    const uint32_t mm_shift = (ieee_m != 0 || ieee_e <= 1) ? 1u : 0u;
    bool vm_tz = false, vr_tz = false;
    uint64_t vr, vp, vm;
    int32_t e10;
    if (e2 >= 0) {
        const int32_t q = (int32_t)(((uint32_t)e2 * 78913u) >> 18) - (e2 > 3 ? 1 : 0);
        e10 = q;
        const int32_t k = kRyuPow5InvBits + (int32_t)ryu_pow5bits(q) - 1;
        const int32_t i = -e2 + q + k;
        const uint64_t* mul = kRyuPow5InvSplit[q];
        vr = ryu_mulshift(4u * m2, mul, i);
        vp = ryu_mulshift(4u * m2 + 2u, mul, i);
        vm = ryu_mulshift(4u * m2 - 1u - mm_shift, mul, i);
        if (q <= 21) {
            if (mv % 5u == 0u) vr_tz = ryu_pow5_multiple(mv, q);
            else if (accept) vm_tz = ryu_pow5_multiple(mv - 1u - mm_shift, q);
            else vp -= ryu_pow5_multiple(mv + 2u, q) ? 1u : 0u;
        }
    } else {
        const int32_t q = (int32_t)(((uint32_t)(-e2) * 732923u) >> 20) - (-e2 > 1 ? 1 : 0);
        e10 = q + e2;
        const int32_t i = -e2 - q;
        const int32_t k = (int32_t)ryu_pow5bits(i) - kRyuPow5Bits;
        const int32_t j = q - k;
        const uint64_t* mul = kRyuPow5Split[i];
        vr = ryu_mulshift(4u * m2, mul, j);
        vp = ryu_mulshift(4u * m2 + 2u, mul, j);
        vm = ryu_mulshift(4u * m2 - 1u - mm_shift, mul, j);
        if (q <= 1) {
            vr_tz = true;
            if (accept) vm_tz = mm_shift == 1;
            else vp--;
        } else if (q < 63) {
            vr_tz = (mv & ((1ull << q) - 1ull)) == 0;
        }
    }
    int32_t removed = 0;
    uint64_t out;
    if (vm_tz || vr_tz) {
        uint32_t last = 0;
        while (vp / 10u > vm / 10u) {
            vm_tz = vm_tz && vm % 10u == 0;
            vr_tz = vr_tz && last == 0;
            last = (uint32_t)(vr % 10u);
            vr /= 10u;
            vp /= 10u;
            vm /= 10u;
            removed++;
        }
        if (vm_tz) {
            while (vm % 10u == 0) {
                vr_tz = vr_tz && last == 0;
                last = (uint32_t)(vr % 10u);
                vr /= 10u;
                vp /= 10u;
                vm /= 10u;
                removed++;
            }
        }
        if (vr_tz && last == 5 && vr % 2u == 0) last = 4;
        out = vr + (((vr == vm && (!accept || !vm_tz)) || last >= 5) ? 1u : 0u);
    } else {
        bool round_up = false;
        if (vp / 100u > vm / 100u) {
            round_up = vr % 100u >= 50u;
            vr /= 100u;
            vp /= 100u;
            vm /= 100u;
            removed += 2;
        }
        while (vp / 10u > vm / 10u) {
            round_up = vr % 10u >= 5u;
            vr /= 10u;
            vp /= 10u;
            vm /= 10u;
            removed++;
        }
        out = vr + ((vr == vm || round_up) ? 1u : 0u);
    }
    *digits = out;
    *exp10 = e10 + removed;
}
// Go's text of a decoded float64 (bits; neg_zero: the literal was a negative
// zero, which the canonical value does not keep); o == nullptr: length only
__device__ inline uint32_t go_float_put(uint64_t bits, bool neg_zero, uint8_t* o) {
    uint32_t n = 0;
    auto put = [&](uint32_t c) {
        if (o) o[n] = (uint8_t)c;
        n++;
    };
    if ((bits & ~(1ull << 63)) == 0) {
        if (neg_zero || (bits >> 63)) put('-');
        put('0');
        return n;
    }
    if (bits >> 63) put('-');
    uint64_t dg;
    int32_t e;
    ryu_d2d(bits, &dg, &e);
    char buf[20];
    uint32_t nd = 0;
    for (uint64_t t = dg; t; t /= 10u) buf[nd++] = (char)('0' + t % 10u);  // reversed
    const int32_t x = e + (int32_t)nd - 1;  // exponent of the first digit
    const double a = __longlong_as_double((long long)(bits & ~(1ull << 63)));
    if (a < 1e-6 || a >= 1e21) {
        put(buf[nd - 1]);
        if (nd > 1) {
            put('.');
            for (int32_t k = (int32_t)nd - 2; k >= 0; k--) put(buf[k]);
        }
        put('e');
        put(x < 0 ? '-' : '+');
        uint32_t ax = (uint32_t)(x < 0 ? -x : x);
        if (x >= 0 && ax < 10) put('0');
        if (ax >= 100) put('0' + ax / 100u);
        if (ax >= 10) put('0' + (ax / 10u) % 10u);
        put('0' + ax % 10u);
    } else if (x >= (int32_t)nd - 1) {
        for (int32_t k = (int32_t)nd - 1; k >= 0; k--) put(buf[k]);
        for (int32_t k = 0; k < x - ((int32_t)nd - 1); k++) put('0');
    } else if (x >= 0) {
        for (int32_t k = (int32_t)nd - 1, c = 0; k >= 0; k--, c++) {
            if (c == x + 1) put('.');
            put(buf[k]);
        }
    } else {
        put('0');
        put('.');
        for (int32_t k = 0; k < -x - 1; k++) put('0');
        for (int32_t k = (int32_t)nd - 1; k >= 0; k--) put(buf[k]);
    }
    return n;
}  // strings longer than this are escaped by the whole wave

__device__ __forceinline__ uint32_t i64_len(int64_t v) {
    uint64_t u = v < 0 ? 0ull - (uint64_t)v : (uint64_t)v;
    uint32_t n = v < 0 ? 2u : 1u;
    while (u >= 10u) {
        u /= 10u;
        n++;
    }
    return n;
}
__device__ __forceinline__ void i64_put(uint8_t* o, int64_t v, uint32_t n) {
    uint64_t u = v < 0 ? 0ull - (uint64_t)v : (uint64_t)v;
    for (uint32_t k = n; k-- > (v < 0 ? 1u : 0u);) {
        o[k] = (uint8_t)('0' + u % 10u);
        u /= 10u;
    }
    if (v < 0) o[0] = '-';
}
template <class T>
__device__ __forceinline__ bool bytes_eq(const uint8_t* a, uint32_t al, const T* b, uint32_t bl) {
    if (al != bl) return false;
    for (uint32_t i = 0; i < al; i++)
        if (a[i] != (uint8_t)b[i]) return false;
    return true;
}
// Go string order (bytes, then length)
__device__ __forceinline__ int bytes_cmp(const uint8_t* a, uint32_t al, const uint8_t* b, uint32_t bl) {
    const uint32_t n = al < bl ? al : bl;
    uint32_t i = 0;
    for (; i + 8 <= n; i += 8) {
        const uint64_t x = __builtin_bswap64(ld8u(a + i)), y = __builtin_bswap64(ld8u(b + i));
        if (x != y) return x < y ? -1 : 1;
    }
    for (; i < n; i++)
        if (a[i] != b[i]) return a[i] < b[i] ? -1 : 1;
    return al < bl ? -1 : al > bl ? 1 : 0;
}
__device__ __forceinline__ uint32_t wave_min_v(uint32_t v) {
#pragma unroll
    for (uint32_t d = 32; d >= 1; d >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, (int)d));
    return v;
}
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
    return rdlane(dpp_incl_scan(v, ~0u, [](uint32_t a, uint32_t b) { return a < b ? a : b; }), 63);
}
constexpr uint32_t MF_HIDDEN = 1u, MF_CUSTOM = 2u, MF_HASVIS = 4u, MF_VIS = 8u, MF_FLOAT = 16u;
constexpr uint32_t MF_VCLEAN = 32u, MF_KCLEAN = 64u;  // string value / key written as its own bytes
constexpr uint32_t kMarshalMaxMembers = 2048;
constexpr int kModeEncode = 0, kModeMarshal = 1, kModeRollup = 2, kModeNegotiate = 3;

// K11 (roll-up mode): Go's struct field lookup for an ASCII key -- 0 no
// match, 1 exact, 2 equal only under ASCII case folding (encoding/json
// fold.go; the device never sees non-ASCII keys: they are slow strings)
//
// The key's first 32 bytes are loaded once as four words (KeyWin, ld32u) and every name is compared from registers
// (a byte loop paid a dependent load per matching byte, per name).  A byte matches when it is equal, or differs by
// 0x20 at a letter of the name (then both are the same letter: the byte loop's (a ^ b) == 0x20 && (a | 0x20) is a
// letter).  Names are <= 32 bytes, constants after inlining.
struct KeyWin {
    uint64_t w[4];
    uint32_t kl;
};
__device__ __forceinline__ KeyWin key_window(const uint8_t* kp, uint32_t kl, const uint8_t* lim) {
    KeyWin K;
    ld32u(kp, lim, K.w[0], K.w[1], K.w[2], K.w[3]);
    K.kl = kl;
    return K;
}
__device__ __forceinline__ uint32_t field_fold(const KeyWin& K, const char* name, uint32_t nl) {
    if (K.kl != nl) return 0u;
    uint64_t diff = 0, nonfold = 0;
#pragma unroll
    for (uint32_t j = 0; j < 4; j++) {
        if (8u * j >= nl) break;
        uint64_t nw = 0, lm = 0;
#pragma unroll
        for (uint32_t b = 0; b < 8; b++) {
            if (8u * j + b >= nl) break;
            const uint32_t c = (uint8_t)name[8u * j + b];
            nw |= (uint64_t)c << (8u * b);
            if ((c | 0x20u) - 'a' <= 25u) lm |= 0x20ull << (8u * b);
        }
        const uint64_t valid = nl >= 8u * j + 8u ? ~0ull : (1ull << (8u * (nl - 8u * j))) - 1ull;
        const uint64_t x = (K.w[j] ^ nw) & valid;
        diff |= x;
        nonfold |= x & ~lm;
    }
    return diff == 0ull ? 1u : nonfold == 0ull ? 2u : 0u;
}
// appsv1.DeploymentStatus counters summed by deployment.go:79-85, in RollOut.v order
__device__ __forceinline__ const char* roll_field(uint32_t k) {
    return k == 0 ? "replicas" : k == 1 ? "updatedReplicas" : k == 2 ? "readyReplicas"
         : k == 3 ? "availableReplicas" : "unavailableReplicas";
}
__device__ __forceinline__ uint32_t roll_field_len(uint32_t k) {
    return k == 0 ? 8u : k == 1 ? 15u : k == 2 ? 13u : k == 3 ? 17u : 19u;
}

// K13 (negotiation mode): metav1.Time's time.Parse(time.RFC3339, s) for the
// strict shape "YYYY-MM-DDTHH:MM:SS[.f{1,9}](Z|+hh:mm|-hh:mm)" (2-digit hour);
// false = not certain (other shapes Go may accept, range errors): the host decides
__device__ __forceinline__ int64_t neg_days_from_civil(int64_t y, uint32_t m, uint32_t d) {
    y -= m <= 2u;
    const int64_t era = (y >= 0 ? y : y - 399) / 400;
    const int64_t yoe = y - era * 400;
    const int64_t doy = (153 * (int64_t)(m + (m > 2u ? -3 : 9)) + 2) / 5 + (int64_t)d - 1;
    const int64_t doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
    return era * 146097 + doe - 719468;
}
// The bytes come from a 40-byte register window (six aligned word loads issued together; a byte loop's early exits
// made each load wait for the last): the strict shape is at most 35 bytes (nine fraction digits and an offset), so a
// longer string is never it, and a document is readable to kTokSlack bytes past its end.
__device__ __forceinline__ bool neg_parse_time(const uint8_t* s, uint32_t l, int64_t* sec, int32_t* nsec) {
    if (l < 20u || l > 35u) return false;
    const uintptr_t a = (uintptr_t)s;
    const uint64_t* q = (const uint64_t*)(a & ~(uintptr_t)7);
    const uint32_t sh = (uint32_t)(a & 7u) * 8u;
    const uint64_t x0 = q[0], x1 = q[1], x2 = q[2], x3 = q[3], x4 = q[4], x5 = q[5];
    auto fw = [&](uint64_t lo, uint64_t hi) -> uint64_t { return (lo >> sh) | ((hi << 1) << (63u - sh)); };
    const uint64_t w0 = fw(x0, x1), w1 = fw(x1, x2), w2 = fw(x2, x3), w3 = fw(x3, x4), w4 = fw(x4, x5);
    auto at = [&](uint32_t i) -> uint32_t {  // i < 40: selects, no private array
        const uint32_t k = i >> 3;
        const uint64_t v = k == 0u ? w0 : k == 1u ? w1 : k == 2u ? w2 : k == 3u ? w3 : w4;
        return (uint32_t)(v >> (8u * (i & 7u))) & 0xFFu;
    };
    auto dg = [&](uint32_t i) -> uint32_t { return at(i) - '0'; };
    const uint32_t dpos[14] = {0, 1, 2, 3, 5, 6, 8, 9, 11, 12, 14, 15, 17, 18};
#pragma unroll
    for (uint32_t k = 0; k < 14; k++)
        if (dg(dpos[k]) > 9u) return false;
    if (at(4) != '-' || at(7) != '-' || at(10) != 'T' || at(13) != ':' || at(16) != ':') return false;
    const uint32_t year = dg(0) * 1000u + dg(1) * 100u + dg(2) * 10u + dg(3);
    const uint32_t mon = dg(5) * 10u + dg(6), day = dg(8) * 10u + dg(9);
    const uint32_t hh = dg(11) * 10u + dg(12), mi = dg(14) * 10u + dg(15), ss = dg(17) * 10u + dg(18);
    if (mon < 1u || mon > 12u || hh >= 24u || mi >= 60u || ss >= 60u || day < 1u) return false;
    const bool leap = (year % 4u == 0u) && (year % 100u != 0u || year % 400u == 0u);
    const uint32_t dim = mon == 2u ? (leap ? 29u : 28u) : (mon == 4u || mon == 6u || mon == 9u || mon == 11u) ? 30u : 31u;
    if (day > dim) return false;
    uint32_t p = 19u;
    int32_t ns = 0;
    if (at(p) == '.' && p + 1u < l && dg(p + 1u) <= 9u) {
        uint32_t n = 0;
        p++;
        while (p < l && dg(p) <= 9u) {
            if (++n > 9u) return false;
            ns = ns * 10 + (int32_t)dg(p);
            p++;
        }
        for (uint32_t k = n; k < 9u; k++) ns *= 10;
    }
    int64_t off = 0;
    if (p < l && at(p) == 'Z') {
        p++;
    } else {
        if (p + 6u != l || (at(p) != '+' && at(p) != '-') || at(p + 3u) != ':' || dg(p + 1u) > 9u || dg(p + 2u) > 9u ||
            dg(p + 4u) > 9u || dg(p + 5u) > 9u)
            return false;
        off = ((int64_t)(dg(p + 1u) * 10u + dg(p + 2u)) * 60 + (int64_t)(dg(p + 4u) * 10u + dg(p + 5u))) * 60;
        if (at(p) == '-') off = -off;
        p += 6u;
    }
    if (p != l) return false;
    *sec = neg_days_from_civil((int64_t)year, mon, day) * 86400 + (int64_t)(hh * 3600u + mi * 60u + ss) - off;
    *nsec = ns;
    return true;
}
__device__ __forceinline__ const char* neg_meta_field(uint32_t k) {
    return k == 0 ? "resourceVersion" : k == 1 ? "generation" : k == 2 ? "labels" : "annotations";
}
__device__ __forceinline__ uint32_t neg_meta_field_len(uint32_t k) { return k == 0 ? 15u : k == 1 ? 10u : k == 2 ? 6u : 11u; }
// APIResourceImportCondition / NegotiatedAPIResourceCondition json names, NegCond order + time last
__device__ __forceinline__ const char* neg_cond_field(uint32_t k) {
    return k == 0 ? "type" : k == 1 ? "status" : k == 2 ? "reason" : k == 3 ? "message" : "lastTransitionTime";
}
__device__ __forceinline__ uint32_t neg_cond_field_len(uint32_t k) {
    return k == 0 ? 4u : k == 1 ? 6u : k == 2 ? 6u : k == 3 ? 7u : 18u;
}
// apiextensions/v1 CustomResourceDefinitionNames json names, struct order
__device__ __forceinline__ const char* neg_crd_names_field(uint32_t k) {
    return k == 0 ? "plural" : k == 1 ? "singular" : k == 2 ? "shortNames" : k == 3 ? "kind" : k == 4 ? "listKind"
                                                                                                       : "categories";
}
__device__ __forceinline__ uint32_t neg_crd_names_field_len(uint32_t k) {
    return k == 0 ? 6u : k == 1 ? 8u : k == 2 ? 10u : k == 3 ? 4u : k == 4 ? 8u : 10u;
}

struct Scratch {
    uint32_t* tok;
    uint4* rec;
    uint64_t *h, *val, *skey;
    uint32_t *meta, *order, *sidx;
    uint8_t* str;
};

}  // namespace

}  // namespace gd
