/*
 * gpudiff_format.h -- canonical encoding shared by the host encoder and the
 * HIP kernels (DESIGN.md "Canonical encoding").  Plain C layout, no HIP types.
 *
 * One object = one blob in a pool, its start and its segments' end aligned to
 * GPUDIFF_BLOB_ALIGN (128 B, the HBM line) with zeros:
 *
 *   [ spec segment ][ status segment ][ zero pad to 128 ]
 *
 * The decision kernel streams whole lines: a stream that starts or ends inside
 * a line costs a partial-line request per blob edge (measured on MI355X: 16-B
 * aligned blobs of ~3.2 KB read at 6.1 TB/s, line-aligned ones at 6.8 TB/s).
 *
 *   segment(L, arena) = vals[L] u64 | keys[L] u32 | metas[L] u32
 *                       | arena: the tails of the long string values in key
 *                         order, each at a 4-byte aligned offset (zero padded
 *                         to 4), the whole zero padded to a multiple of 16
 *
 *   keys   = pathHash: the chained XXH64 path hash under the pair seed, cut
 *            to GPUDIFF_PATH_HASH_BITS (32) bits, ascending, unique
 *   vals   = the value's first 8 bytes: the whole value when it fits (inline:
 *            <= 8 bytes, zero padded), else the head of a long string, whose
 *            remaining len - 8 bytes (its tail) sit in the arena
 *   metas  = (len << 3) | tag
 *
 * Every byte of a value is stored exactly once: the leaf record carries the
 * first 8, the arena the rest.  (Until ABI 4 a long string's vals slot held an
 * XXH64 digest and the arena the whole value: the decision kernel compares
 * arena bytes anyway, so the digest was 8 redundant bytes per long value in
 * every pass -- 9.6% of config3's compared bytes.)
 *
 * Two objects' compared regions are equal under the reference predicates
 * (pkg/syncer/specsyncer.go:17-41, statussyncer.go:15-27) iff their segments
 * are byte-identical, because the encoding is a deterministic function of the
 * leaf set and the path hash is verified injective over each pair's path
 * union: by the encoder over both path sets (it re-seeds the pair on a
 * collision), or, in the object store, against the resident version's path
 * table (below).
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
/* width of the path hashes kept in segments and reported in changed-path
 * lists: 32 bits (16 B per leaf record).  Exactness never rests on the width:
 * the hash is verified injective over each pair's path union (re-seeded on a
 * collision) and the object store's path tables agree at any width. */
#define GPUDIFF_PATH_HASH_BITS 32u

/* object flags (PairRow.flags_a / flags_b) */
#define GPUDIFF_OBJ_HAS_STATUS 0x1u   /* top-level "status" key present (even null) */
#define GPUDIFF_OBJ_DECODE_ERR 0x2u   /* JSON failed the Go decode rules */
#define GPUDIFF_OBJ_FRESH 0x4u        /* object store: blob uploaded with this batch (informational) */
/* object store: the path table kept after a resident blob's segments (the
 * "trailer"), which makes the store's old-vs-new path check exact.  Its n
 * entries are the region leaves and all their ancestors except the root,
 * ascending by (masked) path hash:
 *
 *   hs[n] u64 | phs[n] u64 | cs[n] u64 | key bytes | pad (the whole a multiple of 128),
 *   at the blob's body end (gpudiff_blob_body)
 *
 *   hs    = the node's path hash; unique, and none equals the root's (the seed)
 *   phs   = its parent's path hash (depth-1 nodes: the seed)
 *   cs    = its last component: GPUDIFF_TAB_INDEX | index, or
 *           (key length << 32) | offset of the key bytes in the key area
 *
 * Two tables agree when every hash both hold has the same parent hash and the
 * same component in each.  By induction on depth (the root is the same in
 * both; a node's parent hash names exactly one node of each table), agreeing
 * tables give every shared hash the same path in both objects: an equal key in
 * two segments is then an equal path, whatever the hash width. */
#define GPUDIFF_TAB_INDEX 0x8000000000000000ull
/* entry count of a blob stored without a valid table (its node hashes are not
 * unique under the pair's seed): nothing agrees with it, so the next event on
 * its slot is re-encoded from old_json */
#define GPUDIFF_TAB_NONE 0xFFFFFFFFu
static inline uint64_t gpudiff_tab_bytes(uint32_t n, uint64_t key_bytes) {
    return (24ull * n + key_bytes + 127u) & ~(uint64_t)127u;  /* blobs stay GPUDIFF_BLOB_ALIGN multiples */
}

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

/* segment bytes: 16 B per leaf record (a multiple of 16) + the arena */
static inline uint64_t gpudiff_seg_bytes(uint32_t l, uint32_t arena) { return (uint64_t)l * 16u + (uint64_t)arena; }

#define GPUDIFF_BLOB_ALIGN 128u
/* a blob's body: both segments, zero padded to GPUDIFF_BLOB_ALIGN -- the span the
 * decision kernel reads; a device-store blob's path table starts here */
static inline uint64_t gpudiff_blob_body(uint32_t sl, uint32_t sar, uint32_t tl, uint32_t tar) {
    return (gpudiff_seg_bytes(sl, sar) + gpudiff_seg_bytes(tl, tar) + (GPUDIFF_BLOB_ALIGN - 1u)) &
           ~(uint64_t)(GPUDIFF_BLOB_ALIGN - 1u);
}

/* B_pair: the bytes the decision kernel (K2) reads for one pair -- the 64-B row, the flag byte and, per
 * object, the compared 16-B chunks: the whole body (segments + zero pad) when both regions' sizes match
 * and B has status; the spec segment when only the spec sizes match (padded to the line too when neither
 * side has status leaves); the status segment when only the status sizes match; nothing else (a size
 * mismatch decides the region without reading it).  The roofline's format bytes and the shard weight. */
static inline uint64_t gpudiff_pair_compare_bytes(const gpudiff_pair_row* r) {
    const uint64_t al = GPUDIFF_BLOB_ALIGN - 1u;
    uint64_t per = 0;
    if ((r->flags_a | r->flags_b) & GPUDIFF_OBJ_DECODE_ERR) return sizeof(gpudiff_pair_row) + 1u;
    {
        const int spec_sz = r->spec_l_a == r->spec_l_b && r->spec_ar_a == r->spec_ar_b;
        const int stat_sz = (r->flags_b & GPUDIFF_OBJ_HAS_STATUS) && r->stat_l_a == r->stat_l_b &&
                            r->stat_ar_a == r->stat_ar_b;
        const uint64_t seg_s = gpudiff_seg_bytes(r->spec_l_a, r->spec_ar_a);
        const uint64_t seg_t = gpudiff_seg_bytes(r->stat_l_a, r->stat_ar_a);
        if (spec_sz && stat_sz) per = (seg_s + seg_t + al) & ~al;
        else if (spec_sz) per = (r->stat_l_a | r->stat_l_b | r->stat_ar_a | r->stat_ar_b) ? seg_s : (seg_s + al) & ~al;
        else if (stat_sz) per = seg_t;
    }
    return sizeof(gpudiff_pair_row) + 1u + 2u * per;
}

static inline uint32_t gpudiff_meta(uint32_t tag, uint32_t len) { return (len << 3) | tag; }
static inline uint32_t gpudiff_meta_tag(uint32_t m) { return m & 7u; }
static inline uint32_t gpudiff_meta_len(uint32_t m) { return m >> 3; }
static inline int gpudiff_meta_is_long(uint32_t m) {
    return gpudiff_meta_tag(m) == GPUDIFF_TAG_STR && gpudiff_meta_len(m) > GPUDIFF_INLINE_MAX;
}
/* arena bytes of one leaf's value (long strings: the tail past the 8 bytes in
 * vals, its length rounded up to 4) */
static inline uint32_t gpudiff_meta_arena(uint32_t m) {
    return gpudiff_meta_is_long(m) ? ((gpudiff_meta_len(m) - GPUDIFF_INLINE_MAX + 3u) & ~3u) : 0u;
}
/* a segment's arena size (the row's *_ar fields): the sum of its leaves'
 * gpudiff_meta_arena, rounded up to 16 */
static inline uint32_t gpudiff_arena_bytes(uint32_t sum) { return (sum + 15u) & ~15u; }

#ifdef __cplusplus
}
#endif
#endif
