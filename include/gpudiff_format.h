/*
 * gpudiff_format.h -- canonical encoding shared by the host encoder and the
 * HIP kernels (DESIGN.md "Canonical encoding").  Plain C layout, no HIP types.
 *
 * One object = one 16-byte aligned blob in a pool:
 *
 *   [ spec segment ][ status segment ]
 *
 *   segment(L, arena) = keys[L] u64 | vals[L] u64 | metas[L] u32 | pad to 16
 *                       | arena (each long string value padded to 16 bytes)
 *
 *   keys   = pathHash = XXH64(path bytes, pair seed), ascending, unique
 *   vals   = inline value bytes (<= 8, zero padded) or, for strings longer
 *            than 8 bytes, XXH64(value bytes, 0) filled by kernel K1
 *   metas  = (len << 3) | tag
 *
 * Two objects' compared regions are equal under the reference predicates
 * (pkg/syncer/specsyncer.go:17-41, statussyncer.go:15-27) iff their segments
 * are byte-identical, because the encoding is a deterministic function of the
 * leaf set and the path hash is verified injective over each pair's path
 * union by the encoder (it re-seeds the pair on a collision).
 */
#ifndef GPUDIFF_FORMAT_H
#define GPUDIFF_FORMAT_H

#include <stdint.h>

#define GPUDIFF_TAG_NULL 0u
#define GPUDIFF_TAG_FALSE 1u
#define GPUDIFF_TAG_TRUE 2u
#define GPUDIFF_TAG_INT 3u
#define GPUDIFF_TAG_FLOAT 4u
#define GPUDIFF_TAG_STR 5u
#define GPUDIFF_TAG_EOBJ 6u
#define GPUDIFF_TAG_EARR 7u

#define GPUDIFF_INLINE_MAX 8u

/* object flags (PairRow.flags_a / flags_b) */
#define GPUDIFF_OBJ_HAS_STATUS 0x1u   /* top-level "status" key present (even null) */
#define GPUDIFF_OBJ_DECODE_ERR 0x2u   /* JSON failed the Go decode rules */
#define GPUDIFF_OBJ_FRESH 0x4u        /* object store: blob uploaded with this batch (K1 hashes
                                         its long values; resident blobs were hashed on arrival) */
/* object store: root of the fingerprint chain, an independent second path hash
 * (fp(p + c) = XXH64(enc(c), fp(p))) kept after a resident blob's segments */
#define GPUDIFF_FP_ROOT 0x9FB21C651E98DF25ull

/* bits 8..15 of flags_a: per-pair path-hash seed */
#define GPUDIFF_OBJ_SEED_SHIFT 8u

#ifdef __cplusplus
extern "C" {
#endif

/* One pair descriptor, 64 bytes, device resident.  Offsets are byte offsets
 * into the pool the row lives with. */
typedef struct gpudiff_pair_row {
    uint64_t off_a;          /* blob of A (old / upstream) */
    uint64_t off_b;          /* blob of B (new / downstream) */
    uint32_t spec_l_a, spec_l_b;       /* spec-region leaves */
    uint32_t spec_ar_a, spec_ar_b;     /* spec arena bytes (multiple of 16) */
    uint32_t stat_l_a, stat_l_b;       /* status-region leaves */
    uint32_t stat_ar_a, stat_ar_b;     /* status arena bytes (multiple of 16) */
    uint32_t flags_a, flags_b;
    uint32_t pair_id, cluster_id;
} gpudiff_pair_row;

static inline uint64_t gpudiff_seg_bytes(uint32_t l, uint32_t arena) {
    return ((((uint64_t)l * 20u) + 15u) & ~(uint64_t)15u) + (uint64_t)arena;
}

static inline uint32_t gpudiff_meta(uint32_t tag, uint32_t len) { return (len << 3) | tag; }
static inline uint32_t gpudiff_meta_tag(uint32_t m) { return m & 7u; }
static inline uint32_t gpudiff_meta_len(uint32_t m) { return m >> 3; }
static inline int gpudiff_meta_is_long(uint32_t m) {
    return gpudiff_meta_tag(m) == GPUDIFF_TAG_STR && gpudiff_meta_len(m) > GPUDIFF_INLINE_MAX;
}
static inline uint32_t gpudiff_meta_arena(uint32_t m) {
    return gpudiff_meta_is_long(m) ? ((gpudiff_meta_len(m) + 15u) & ~15u) : 0u;
}

#ifdef __cplusplus
}
#endif
#endif
