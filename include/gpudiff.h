/*
 * gpudiff.h -- C ABI of the MI355X batched reconciliation-diff engine.
 *
 * Drop-in boundary for kcp's syncer change detection.  Each entry point names
 * the reference interface (paths relative to the sttts/kcp tree) it replaces;
 * INTEGRATION.md shows the cgo binding a maintainer adds to pkg/syncer.
 *
 *   reference seam                                   replaced by
 *   ------------------------------------------------ ---------------------------
 *   deepEqualApartFromStatus  specsyncer.go:17-41    gpudiff_spec_equal (1 pair),
 *                                                    spec bits of gpudiff_wait
 *   deepEqualStatus           statussyncer.go:15-27  gpudiff_status_equal (1 pair),
 *                                                    status bits of gpudiff_wait
 *   UpdateFunc gates          specsyncer.go:47-51,   gpudiff_submit/gpudiff_wait:
 *                             statussyncer.go:32-36  dirty IDs -> AddToQueue
 *   Controller.AddToQueue     syncer.go:222-224      consumer of dirty_ids
 *
 * Conventions: 0 = OK, negative = error (gpudiff_strerror).  No exceptions or
 * longjmp cross the ABI.  The caller owns inputs until the call that reads
 * them returns (gpudiff_encode_pairs copies everything it needs).  The library
 * owns result buffers until gpudiff_result_release.  A context is not
 * reentrant: one submitting thread per context (the Go shim's batcher
 * goroutine).  Errors are conservative, as in the reference
 * (specsyncer.go:20-22): a pair that cannot be decoded is reported dirty in
 * both regions with GPUDIFF_DECODE_ERROR set, never "equal".
 *
 * There is no CPU fallback for the diff: device entry points on a context
 * without a GPU return GPUDIFF_E_NODEVICE.
 */
#ifndef GPUDIFF_H
#define GPUDIFF_H

#include <stddef.h>
#include <stdint.h>

#include "gpudiff_format.h"

#ifdef __cplusplus
extern "C" {
#endif

#define GPUDIFF_ABI_VERSION 6  /* 6: bit 0x100 (the K2 timeline build) retired: gpudiff_k2_profile selects that build;
                                   5: the tuning option bits removed (GPUDIFF_OPT_KNOWN); result slots own their counts */

enum {
    GPUDIFF_OK = 0,
    GPUDIFF_E_INVAL = -1,     /* bad argument */
    GPUDIFF_E_NOMEM = -2,     /* host allocation failed */
    GPUDIFF_E_DEVICE = -3,    /* HIP runtime error */
    GPUDIFF_E_NODEVICE = -4,  /* context has no GPU */
    GPUDIFF_E_CAPACITY = -5,  /* device batch capacity exceeded */
    GPUDIFF_E_STATE = -6,     /* call order violated (e.g. wait on unknown ticket) */
    GPUDIFF_E_DECODE = -7,    /* single-pair helpers: an input failed to decode */
    GPUDIFF_E_NOTFOUND = -8,  /* gpudiff_resolve_path: hash not in either object */
};

/* per-pair result flags */
#define GPUDIFF_SPEC_DIRTY 0x1u
#define GPUDIFF_STATUS_DIRTY 0x2u
#define GPUDIFF_DECODE_ERROR 0x4u
/* write-path hints, set only on dirty pairs: the write the
 * syncer issues for the decision would not change what the predicate compares, so the API call can
 * be skipped.  GPUDIFF_SPEC_NOOP: every changed spec leaf is an int64 v on one side and a float64
 * == v (|v| <= 2^53) on the other -- Go's json.Marshal writes both as the same digits and the API
 * server decodes them back to int64 v, so the two documents' bodies agree on the wire in that
 * region (gpudiff_write_plan_get_ex says what that means for informer and for (A, B) pairs).
 * GPUDIFF_STATUS_NOOP: the same for the status leaves, and when B has no status key, A has none
 * either (UpdateStatus would write nothing). */
#define GPUDIFF_SPEC_NOOP 0x8u
#define GPUDIFF_STATUS_NOOP 0x10u

/* device encoder (K0) per-object status: 0 = encoded on the device; otherwise
 * the reason the object was handed to the host encoder (the Go-exact path) */
#define GPUDIFF_TOK_OK 0
#define GPUDIFF_TOK_SYNTAX 1  /* not in the device's JSON subset: the host decides (usually a Go decode error) */
#define GPUDIFF_TOK_NUMBER 2  /* number outside the exact fast path (float needing full strtod, int64 overflow) */
#define GPUDIFF_TOK_KEY 3     /* object key that needs unescaping or UTF-8 repair */
#define GPUDIFF_TOK_STRING 4  /* control character or invalid escape in a string */
#define GPUDIFF_TOK_HASH 5    /* equal path hashes: duplicate key, or a collision under the seed */
#define GPUDIFF_TOK_DEPTH 6   /* nesting deeper than 255 */
#define GPUDIFF_TOK_SIZE 7    /* document larger than 16 MiB */
#define GPUDIFF_TOK_SPACE 8   /* output space exhausted */
#define GPUDIFF_TOK_FLOAT 9   /* K10 (write path): a float64 value (Go's shortest formatting is done on the host) */
#define GPUDIFF_TOK_WIDE 10   /* K10: an object with more than 2048 members (quadratic key ranking) */
#define GPUDIFF_TOK_FIELD 11  /* K11 (roll-up): a field the typed decode must judge on the host (duplicate,
                                 case-folded key, type mismatch, counter not an int32 literal, escaped label) */
#define GPUDIFF_TOK_LIST 12   /* K0: a top-level key the informer decoder's list probe matches ("items" under
                                 Go's case folding): the host decides (the object is an UnstructuredList, the
                                 pair is dirty -- specsyncer.go:18-22) */

/* changed-path kinds (low 2 bits); bit 7 = status region */
#define GPUDIFF_PATH_CHANGED 0u        /* present in both, value differs */
#define GPUDIFF_PATH_ADDED 1u          /* only in new (B) */
#define GPUDIFF_PATH_REMOVED 2u        /* only in old (A) */
#define GPUDIFF_PATH_STATUS_ABSENT 3u  /* new has no "status" key (statussyncer.go:22-26) */
#define GPUDIFF_PATH_REGION_STATUS 0x80u

/* context option flags (any other bit: gpudiff_open returns GPUDIFF_E_INVAL).  Round 5 removed the A/B tuning
 * bits of earlier rounds whose measurements rejected them (DESIGN.md §5-§6 keep the numbers):
 * 0x2 two upload streams, 0x4 index-order final round, 0x8 pipelined K4 join, 0x10-0x80 tail shapes, bits 9-20
 * kernel variants / blocks per CU / segmented passes, bits 26-31 K0 occupancy, items per wave, deep-join bounds.
 * ABI 6 retired 0x100 (ABI 5's K2 timeline bit, ABI 4's K2 variant bit): refused like the rest, so no caller of
 * either meaning gets the other; the timeline build is selected by gpudiff_k2_profile. */
#define GPUDIFF_OPT_TIMING 0x1u          /* record per-kernel HIP event times (gpudiff_last_timings) */
#define GPUDIFF_OPT_ARENA_SHIFT 21u      /* 4 bits, test hook: shrink the per-wave path arena 2^k-fold (forces
                                            pairs through the deferred K4 path) */
#define GPUDIFF_OPT_DEVICE_ENCODE 0x2000000u /* gpudiff_submit / single-pair helpers: raw JSON up, kernel K0
                                                encodes (as GPUDIFF_STORE_DEVICE_ENCODE does for the store) */
#define GPUDIFF_OPT_KNOWN (GPUDIFF_OPT_TIMING | (0xFu << GPUDIFF_OPT_ARENA_SHIFT) | GPUDIFF_OPT_DEVICE_ENCODE)

#define GPUDIFF_DEVICE_CURRENT (-1)
#define GPUDIFF_DEVICE_NONE (-2)   /* host-only context: encoding only */

typedef struct gpudiff_opts {
    int32_t device;          /* HIP ordinal, GPUDIFF_DEVICE_CURRENT or GPUDIFF_DEVICE_NONE */
    uint32_t encode_threads; /* 0 = all host cores */
    void* stream;            /* hipStream_t to launch on; NULL = context-owned stream */
    uint32_t flags;          /* GPUDIFF_OPT_* */
    uint32_t path_hash_bits; /* 0 (or >= 32): GPUDIFF_PATH_HASH_BITS = 32; 8..31 only to force collisions in tests */
} gpudiff_opts;

typedef struct gpudiff_json_pair {
    const uint8_t* old_json;  /* A: upstream (kcp) copy / old version */
    size_t old_len;
    const uint8_t* new_json;  /* B: downstream copy / new version */
    size_t new_len;
    uint32_t pair_id;         /* echoed in results */
    uint32_t cluster_id;      /* logical cluster (shard key, syncer.go:106-108) */
} gpudiff_json_pair;

typedef struct gpudiff_ctx gpudiff_ctx;
typedef struct gpudiff_hbatch gpudiff_hbatch;  /* encoded pairs in host memory */
typedef struct gpudiff_dbatch gpudiff_dbatch;  /* encoded pairs resident in HBM */
typedef uint64_t gpudiff_ticket;

typedef struct gpudiff_hbatch_info {
    size_t n_pairs;
    const gpudiff_pair_row* rows;   /* offsets relative to pool */
    const uint8_t* pool;
    uint64_t pool_bytes;
    uint64_t total_leaves;          /* over both objects of every pair */
    uint64_t n_decode_errors;
    uint64_t n_reseeded;            /* pairs whose path hash needed seed > 0 */
} gpudiff_hbatch_info;

typedef struct gpudiff_result {
    size_t n_pairs;
    const uint8_t* pair_flags;          /* [n_pairs], batch order, GPUDIFF_*_DIRTY */
    size_t n_spec_dirty;
    const uint32_t* spec_dirty_ids;     /* pair_id, batch order */
    size_t n_status_dirty;
    const uint32_t* status_dirty_ids;
    size_t n_dirty;                     /* spec or status dirty */
    const uint32_t* dirty_ids;
    const uint32_t* path_offsets;       /* [n_dirty + 1] into the path arrays */
    size_t n_paths;
    const uint64_t* path_hashes;        /* per dirty pair: spec asc, status asc, sentinel */
    const uint8_t* path_kinds;
    void* internal_;
} gpudiff_result;

/* device-side view of a diffed batch (for RCCL gathers; pointers are HBM).  The pointers belong to the batch's
 * current result slot: after gpudiff_dbatch_result_slot switches slots, fetch the view again (counts included --
 * a slot owns its counts since ABI 5). */
typedef struct gpudiff_device_view {
    const uint8_t* pair_flags;
    const uint32_t* spec_dirty_ids;
    const uint32_t* status_dirty_ids;
    const uint32_t* dirty_ids;
    const uint32_t* counts;   /* [0]=n_spec [1]=n_status [2]=n_dirty [3]=n_paths [4]=overflow */
} gpudiff_device_view;

typedef struct gpudiff_batch_stats {
    uint64_t n_pairs;
    uint64_t pool_bytes;       /* bytes of object blobs resident */
    uint64_t total_leaves;
    uint64_t compare_bytes;    /* format bytes one diff pass reads */
    uint64_t value_bytes;      /* canonical bytes of the long (non-inline) string values of every object:
                                  V of SURVEY.md §8(d)'s B_pair = sum over A, B of (24 L + V + 8) + O */
} gpudiff_batch_stats;

typedef struct gpudiff_timings {
    float compare_ms;     /* K2: all k2_launches launches of a pass (back to back on the stream) */
    float compact_ms;     /* K3 (scan + compaction); 0 when overlapped with K2 (segmented pass) */
    float join_ms;        /* K4 merge-join; segmented pass: the part not hidden behind K2 */
    float emit_ms;        /* K5 + K6 path scan and copy */
    float total_ms;       /* first to last event of gpudiff_diff */
    uint32_t n_passes;    /* diff passes averaged (since gpudiff_timing_reset) */
    uint32_t k2_launches; /* K2 launches per pass (batch segments) */
} gpudiff_timings;

/* ---- library ---- */
const char* gpudiff_strerror(int err);
int gpudiff_abi_version(void);
/* 16 hex digits: SHA-256 over the contents of every source, header, map and build script the library was
 * compiled from (kcp_amd/buildinfo.py).  A binding that ships the sources recomputes it and refuses a
 * library built from anything else; the bench line carries it as `build_id`. */
const char* gpudiff_build_id(void);
int gpudiff_device_count(int* n);

/* ---- context ---- */
int gpudiff_open(const gpudiff_opts* opts, gpudiff_ctx** out);
void gpudiff_close(gpudiff_ctx* ctx);

/* ---- host encoding (canonical CSR, no GPU needed) ---- */
int gpudiff_encode_pairs(gpudiff_ctx* ctx, const gpudiff_json_pair* pairs, size_t n,
                         gpudiff_hbatch** out);
int gpudiff_hbatch_info_get(const gpudiff_hbatch* hb, gpudiff_hbatch_info* info);
/* empty host batch (pinned on a GPU context) for pairs encoded elsewhere in the
 * canonical format (pre-encoded replays, synthetic populations); the caller
 * fills *pool and *rows (row offsets relative to *pool) before appending */
int gpudiff_hbatch_create(gpudiff_ctx* ctx, uint64_t pool_bytes, size_t n_pairs, uint64_t total_leaves,
                          gpudiff_hbatch** out, uint8_t** pool, gpudiff_pair_row** rows);
/* reuses a host batch (staging ring): waits for its last H2D copy, grows the
 * buffers only when needed, and returns them for refilling */
int gpudiff_hbatch_resize(gpudiff_ctx* ctx, gpudiff_hbatch* hb, uint64_t pool_bytes, size_t n_pairs,
                          uint64_t total_leaves, uint8_t** pool, gpudiff_pair_row** rows);
void gpudiff_hbatch_free(gpudiff_ctx* ctx, gpudiff_hbatch* hb);

/* ---- device batches ---- */
int gpudiff_dbatch_create(gpudiff_ctx* ctx, uint64_t pool_bytes, uint64_t max_pairs,
                          gpudiff_dbatch** out);
/* A view of `base`: a batch with its own per-pass outputs (flags, lists, path arenas, scratch, counts) over
 * base's resident pairs (pool, rows and pair IDs are base's; appends to base are seen by later diffs of
 * the view; append / reset on a view are GPUDIFF_E_INVAL).  With a second context (its own stream) it lets
 * two diff passes over one population be in flight at once -- pass s + 1's decision kernel fills the CUs
 * pass s's tail frees, and pass s's compaction, joins and collective run beside it.  Same device as base;
 * the caller orders base's appends before the view's diffs (e.g. gpudiff_sync on base's context).  Free
 * views before their base. */
int gpudiff_dbatch_create_view(gpudiff_ctx* ctx, const gpudiff_dbatch* base, gpudiff_dbatch** out);
/* async H2D of hb into the batch (rows rebased onto the batch's pool) */
int gpudiff_dbatch_append(gpudiff_ctx* ctx, gpudiff_dbatch* db, const gpudiff_hbatch* hb);
int gpudiff_dbatch_reset(gpudiff_ctx* ctx, gpudiff_dbatch* db);
int gpudiff_dbatch_stats_get(const gpudiff_dbatch* db, gpudiff_batch_stats* st);
int gpudiff_dbatch_device_view(const gpudiff_dbatch* db, gpudiff_device_view* v);
/* async device-to-device copy of a diffed batch's results into caller memory
 * (e.g. a tensor handed to an RCCL all-gather), ordered on the context
 * stream; copies min(count, max_elems) elements of `what` */
#define GPUDIFF_EXPORT_COUNTS 0u      /* 8 x u32: n_spec, n_status, n_dirty, K4 scratch entries (saturating),
                                         overflow, n_paths, any join deferred to K3/K4, 0 */
#define GPUDIFF_EXPORT_SPEC_IDS 1u    /* u32 */
#define GPUDIFF_EXPORT_STATUS_IDS 2u  /* u32 */
#define GPUDIFF_EXPORT_DIRTY_IDS 3u   /* u32 */
#define GPUDIFF_EXPORT_FLAGS 4u       /* u8 per pair */
int gpudiff_dbatch_export(gpudiff_ctx* ctx, const gpudiff_dbatch* db, uint32_t what, void* dst_device,
                          uint64_t max_elems, uint64_t known_count);
/* Gather binding: while bound, every diff of this batch also writes -- from its K3 compaction, no extra
 * launch or copy -- the buffer a per-step all-gather sends (kcp_amd/shard.py DirtyGather): u32
 * [8 counts | cap_spec spec-dirty IDs | cap_status status-dirty IDs], counts = (n_spec, n_status, n_dirty,
 * K4 scratch entries, 0, 0, 0, 0).  The counts are the batch totals even past a capacity; IDs past it are
 * not written (the caller grows its buffers and exports them with gpudiff_dbatch_export, whose lists are
 * always complete).  Words 4..7 are zeroed here, on the context stream, when the buffer differs from the
 * one bound (rebinding the same buffer is free).  send_dev = NULL unbinds. */
int gpudiff_dbatch_bind_gather(gpudiff_ctx* ctx, gpudiff_dbatch* db, void* send_dev, uint32_t cap_spec,
                               uint32_t cap_status);
/* Result slots: the spec / status dirty-ID lists and the counts (GPUDIFF_EXPORT_COUNTS) come in two slots
 * (0 by default; slot 1 allocated on first use).  Later diffs write, and exports / gpudiff_wait read, the
 * selected slot; the other keeps the lists and counts of the last diff made under it.  A per-step collective that checks step s's gathered counts only after
 * step s + 1's diff is enqueued alternates slots by step, so a capacity regrow can still export step s's
 * complete lists (kcp_amd/shard.py DirtyGather, lookahead).  Host-only state: ordered like every call. */
int gpudiff_dbatch_result_slot(gpudiff_ctx* ctx, gpudiff_dbatch* db, uint32_t slot);
/* synchronous D2H copy of resident pool bytes (inspection / tests) */
int gpudiff_dbatch_read_pool(gpudiff_ctx* ctx, const gpudiff_dbatch* db, uint64_t off, void* dst,
                             uint64_t bytes);
void gpudiff_dbatch_free(gpudiff_ctx* ctx, gpudiff_dbatch* db);

/* ---- sharding by logical cluster ----
 * The reference runs one syncer per logical cluster (pkg/reconciler/cluster/cluster.go:125-138), so a
 * node shards pairs by whole cluster with no data-path exchange.  A rank's step time is its decision
 * kernel's byte stream, so clusters are balanced by Σ B_pair, not by pair count (object sizes differ by
 * tenant).  Host-only; no GPU needed.
 * gpudiff_cluster_bytes adds each row's B_pair -- the bytes K2 streams for it: the 64-B row, the flag
 * and both objects' compared 16-B chunks (gpudiff_pair_compare_bytes, gpudiff_format.h) -- into
 * out[row.cluster_id] (out has n_clusters entries; a row with cluster_id >= n_clusters is
 * GPUDIFF_E_INVAL).  Weights can come from the previous step's encoded rows of each cluster.
 * gpudiff_shard_lpt: greedy LPT -- clusters by descending weight (ties: lower cluster id) each onto the
 * least-loaded rank (ties: lower rank); owner[c] = its rank.  The heaviest rank's load is at most
 * 4/3 of the optimum (Graham's bound) and within one cluster's weight of the mean. */
int gpudiff_cluster_bytes(const gpudiff_pair_row* rows, size_t n, uint32_t n_clusters, uint64_t* out);
int gpudiff_shard_lpt(const uint64_t* weights, uint32_t n_clusters, uint32_t world, int32_t* owner);

/* ---- diff (the hot path) ---- */
/* enqueue K2..K6 on the context stream; returns immediately */
int gpudiff_diff(gpudiff_ctx* ctx, gpudiff_dbatch* db, gpudiff_ticket* ticket);
/* block until the ticket's diff finished and copy results to host */
int gpudiff_wait(gpudiff_ctx* ctx, gpudiff_ticket ticket, gpudiff_result* res);
void gpudiff_result_release(gpudiff_ctx* ctx, gpudiff_result* res);
/* mean per-kernel times over the passes recorded since the last reset
 * (GPUDIFF_OPT_TIMING); synchronizes the context stream */
int gpudiff_last_timings(gpudiff_ctx* ctx, gpudiff_timings* t);
int gpudiff_timing_reset(gpudiff_ctx* ctx);
int gpudiff_sync(gpudiff_ctx* ctx);

/* encode + upload into a context-owned batch + diff (the syncer batcher's call) */
int gpudiff_submit(gpudiff_ctx* ctx, const gpudiff_json_pair* pairs, size_t n,
                   gpudiff_ticket* ticket);

/* ---- device-resident object store (watch replay) ----
 * The informer cache's "old" objects stay resident in HBM, one per caller
 * slot (the shim maps (cluster, gvr, namespace, name) to a slot, as the
 * indexer at pkg/syncer/syncer.go:318 keys its cache).  An Update event
 * uploads only its new version: the engine diffs it against the slot's
 * resident version -- UpdateFunc(old, new), specsyncer.go:47-51 and
 * statussyncer.go:32-36 -- and the new version becomes the resident one.
 * Events of one batch apply in order, so two events on one slot chain.
 * Exactness: every resident blob carries a path table (one entry per region
 * leaf and ancestor: its hash, its parent's hash, its last component;
 * include/gpudiff_format.h); a new version's table must agree
 * with the resident one, which makes every shared path hash name the same path
 * in both.  A disagreement (a path-hash collision between versions, or within
 * the new one) re-encodes the pair with the smallest valid seed from old_json
 * (dirty with GPUDIFF_DECODE_ERROR when old_json is absent).  Blobs are
 * appended to the current space and the live ones are packed into the other
 * space (K7 k_move_blobs) when it fills. */
typedef struct gpudiff_store gpudiff_store;

typedef struct gpudiff_event {
    uint32_t slot;            /* < max_slots */
    uint32_t pair_id;         /* echoed in the result id lists */
    uint32_t cluster_id;      /* logical cluster */
    uint32_t reserved;        /* 0 */
    const uint8_t* new_json;  /* the event's object (required) */
    size_t new_len;
    /* optional: the informer's old object, read only when the slot is empty
     * (a first sighting diffs against it) or a collision forces a re-seed.
     * An empty slot without old_json diffs against the empty object {};
     * a collision without old_json reports the event dirty with
     * GPUDIFF_DECODE_ERROR (conservative) and stores the new version. */
    const uint8_t* old_json;
    size_t old_len;
} gpudiff_event;

typedef struct gpudiff_store_stats {
    uint64_t max_slots, live_slots;
    uint64_t space_bytes;      /* per space (two are allocated) */
    uint64_t used_bytes;       /* appended to the current space */
    uint64_t live_bytes;       /* resident blobs */
    uint64_t compactions;
    uint64_t events, old_encoded, reseeded, collisions_unresolved;
    uint64_t last_batch_bytes; /* bytes uploaded by the last submit (blobs; device-encode: JSON) */
    uint64_t deferred;         /* device-encode: events K0 handed to the host encoder */
    /* device-encode with GPUDIFF_OPT_TIMING: per-batch means (ms) of the host side of submit,
     * the H2D copy, K0 and K0c+K0x */
    float host_submit_ms, h2d_ms, encode_ms, link_ms;
    /* the host side of submit split: waiting for the ring slot's previous upload,
     * the document / slot-chain tables, the JSON copy into pinned staging, the
     * enqueue of copies and kernels; and the store's part of gpudiff_wait */
    float submit_wait_ms, submit_docs_ms, submit_copy_ms, submit_enqueue_ms, finish_ms;
    uint32_t timing_batches; /* batches the means are over */
    uint32_t zero_copy_batches; /* batches uploaded straight from a gpudiff_host_alloc buffer (gpudiff_submit's
                                    device-encode pairs, or this store's device-encode events) */
    uint64_t space_conservative; /* device-encode: deferred events reported dirty (GPUDIFF_DECODE_ERROR, slot
                                    emptied) because the space could not take their re-encoded blobs */
} gpudiff_store_stats;

int gpudiff_store_create(gpudiff_ctx* ctx, uint32_t max_slots, uint64_t space_bytes, uint32_t max_events,
                         gpudiff_store** out);
/* GPUDIFF_STORE_DEVICE_ENCODE: events go up as raw JSON; kernel K0 encodes
 * them in HBM, K0c checks collisions against the resident versions, K0x
 * chains events per slot, and the host encoder only re-does the events K0
 * defers (GPUDIFF_TOK_*), inside gpudiff_wait, with identical results.  In
 * this mode event buffers must stay valid until gpudiff_wait on the ticket
 * returns, and tickets are waited in submit order (at most two in flight). */
#define GPUDIFF_STORE_DEVICE_ENCODE 0x1u
int gpudiff_store_create_ex(gpudiff_ctx* ctx, uint32_t max_slots, uint64_t space_bytes, uint32_t max_events,
                            uint32_t flags, gpudiff_store** out);
/* encode (host threads), H2D into the current space,
 * K2..K6 over the batch's (resident, new) pairs; results via gpudiff_wait.
 * Two submits may be in flight (the next batch encodes while the GPU diffs
 * the previous one); wait on a ticket before its slot in the ring is reused. */
int gpudiff_store_submit(gpudiff_ctx* ctx, gpudiff_store* st, const gpudiff_event* events, size_t n,
                         gpudiff_ticket* ticket);
/* Delete event: the slot is empty again */
int gpudiff_store_forget(gpudiff_ctx* ctx, gpudiff_store* st, uint32_t slot);
int gpudiff_store_stats_get(const gpudiff_store* st, gpudiff_store_stats* out);
/* The same statistics for gpudiff_submit's device-encode path (GPUDIFF_OPT_DEVICE_ENCODE: the context's
 * pair-mode store), e.g. the per-phase times of JSON-in with GPUDIFF_OPT_TIMING; GPUDIFF_E_STATE before the
 * context's first device-encoded submit. */
int gpudiff_submit_stats_get(gpudiff_ctx* ctx, gpudiff_store_stats* out);
void gpudiff_store_free(gpudiff_ctx* ctx, gpudiff_store* st);
/* Pinned host memory for gpudiff_submit's JSON on a device-encode context (no reference counterpart: the syncer
 * batcher renders each flush's objects into it).  A batch whose documents all lie in ONE such
 * buffer, in pair order (old_0, new_0, old_1, new_1, ...), each at a 16-B aligned address and followed by at
 * least its staged span -- len + 32 bytes rounded up to 16 -- before the next document (the last one's span and
 * 32 more bytes inside the buffer) is uploaded straight from it: no staging copy.  The engine zeroes each
 * document's padding up to that span (those bytes are its to write).  The same holds for gpudiff_store_submit on
 * a GPUDIFF_STORE_DEVICE_ENCODE store (the watch stream's events rendered straight into engine-pinned memory):
 * the documents the store encodes -- per event, in submit order, its old object when the slot is seen for the
 * first time, then its new object -- lie in ONE such buffer in that order, 16-B aligned, each followed by its
 * staged span before the next (gaps allowed; old objects the store does not encode may lie anywhere).  Any
 * other layout takes the staging copy; results are identical either way
 * (gpudiff_store_stats.zero_copy_batches counts the zero-copy ones).  The buffer must stay untouched until
 * gpudiff_wait on the ticket returns; gpudiff_close frees what is left. */
int gpudiff_host_alloc(gpudiff_ctx* ctx, size_t bytes, void** out);
int gpudiff_host_free(gpudiff_ctx* ctx, void* p);

/* ---- object encoding in the device-store format (inspection / parity) ----
 * An object's blob followed by its path table (gpudiff_format.h: the node
 * hashes, parent hashes and last components of the region leaves and their
 * ancestors, which the store checks old-vs-new paths with exactly).
 * gpudiff_encode_objects
 * runs kernel K0 (the device JSON tokenizer + encoder) over n documents;
 * gpudiff_encode_object_host runs the host encoder (the Go-exact path) over
 * one.  Where K0 reports GPUDIFF_TOK_OK the two are byte-identical. */
typedef struct gpudiff_obj_info {
    int32_t status;          /* GPUDIFF_TOK_*: 0 = encoded */
    uint32_t oflags;         /* GPUDIFF_OBJ_HAS_STATUS */
    uint32_t spec_l, spec_ar, stat_l, stat_ar;
    uint64_t off;            /* blob offset in out */
    uint64_t bytes;          /* blob + path-table bytes */
    uint32_t n_tab;          /* path-table entries */
    uint32_t reserved;
} gpudiff_obj_info;

int gpudiff_encode_objects(gpudiff_ctx* ctx, const uint8_t* const* docs, const size_t* lens, const uint32_t* seeds,
                           size_t n, uint8_t* out, uint64_t out_cap, gpudiff_obj_info* info);
int gpudiff_encode_object_host(const uint8_t* doc, size_t len, uint32_t seed, uint32_t path_hash_bits, uint8_t* out,
                               uint64_t out_cap, gpudiff_obj_info* info);
/* profiling hook: K0 per-phase wall-clock ticks (100 MHz, summed over waves) since the
 * previous call (scan, tree, values, hashes, sort, blob, -, -); enable != 0
 * keeps recording */
int gpudiff_k0_profile(gpudiff_ctx* ctx, int enable, uint64_t* ticks8);
/* profiling hook: the decision kernel's per-wave timeline.  While a buffer is installed (dev_buf != NULL) this
 * context's passes run the timeline build of the decision kernel (the same kernel plus timestamps), writing 12
 * u64 per wave (start, end of the first
 * item, items, start of the last item, end, streaming ticks, join ticks, hardware CU id, then ticks
 * spent per item on its rows, between its rows and its first pass, after its joins, and from one
 * item's end to the next one's start; 100 MHz) into device memory dev_buf of cap_waves records;
 * dev_buf NULL stops recording and returns the context to the default build */
int gpudiff_k2_profile(gpudiff_ctx* ctx, uint64_t* dev_buf, uint32_t cap_waves);

/* ---- write path: the request body for a dirty object ----
 * GPUDIFF_UPSERT_SPEC: what upsertIntoDownstream hands to client.Create
 *   (pkg/syncer/specsyncer.go:86-110): the object with metadata.uid and
 *   metadata.resourceVersion removed and every owner reference whose name equals
 *   the kcp.dev/owned-by label dropped (the rest normalized as
 *   Unstructured.SetOwnerReferences writes them; the field removed when none
 *   remain).
 * GPUDIFF_UPSERT_STATUS: updateStatusInUpstream's object (statussyncer.go:41-48)
 *   before the live resourceVersion is set: uid and resourceVersion removed.
 * Bytes are exactly json.NewEncoder(w).Encode(obj.Object) of Go 1.16 -- what the
 * dynamic client sends (UnstructuredJSONScheme): keys sorted, HTML-safe string
 * escaping, shortest floats, trailing newline.  Kernel K10 emits the bodies in
 * HBM; documents outside its subset (floats, duplicate keys, undecodable input,
 * ...) are marshalled by the host path, with identical bytes. */
#define GPUDIFF_UPSERT_SPEC 0u
#define GPUDIFF_UPSERT_STATUS 1u

typedef struct gpudiff_bodies {
    size_t n;
    const uint64_t* offsets;  /* n + 1: body i = bytes[offsets[i], offsets[i + 1]) */
    const uint8_t* bytes;
    const int32_t* status;    /* 0 = body; GPUDIFF_E_DECODE = Go could not decode the object (empty body) */
    const uint8_t* source;    /* GPUDIFF_BODY_DEVICE / GPUDIFF_BODY_HOST per document */
    const int32_t* k10_status; /* K10's GPUDIFF_TOK_* per document (why the host took it over) */
    size_t n_host;            /* documents the host marshalled */
    void* internal;
} gpudiff_bodies;
#define GPUDIFF_BODY_DEVICE 0u
#define GPUDIFF_BODY_HOST 1u

/* n documents (JSON objects) -> n bodies; synchronous.  Release with
 * gpudiff_bodies_release. */
int gpudiff_upsert_bodies(gpudiff_ctx* ctx, const uint8_t* const* docs, const size_t* lens, size_t n, uint32_t mode,
                          gpudiff_bodies* out);
void gpudiff_bodies_release(gpudiff_ctx* ctx, gpudiff_bodies* b);

/* Gate -> write on the device.  For a
 * batch submitted with GPUDIFF_OPT_DEVICE_ENCODE and waited (gpudiff_wait), the
 * writes the syncer issues for its decisions, rendered by K10 from the pairs'
 * JSON still staged in HBM -- no re-upload.  Which document a write renders
 * depends on what the submitted pairs are (`mode` of gpudiff_write_plan_get_ex):
 *   GPUDIFF_PLAN_INFORMER (default): each pair is an informer Update event
 *     (old, new).  UpdateFunc enqueues newObj (specsyncer.go:47-50,
 *     statussyncer.go:32-35) and the worker writes that object, so both kinds
 *     render the NEW document: a spec-dirty pair gets upsertIntoDownstream's
 *     body of new (GPUDIFF_UPSERT_SPEC, specsyncer.go:86-132), a status-dirty
 *     pair updateStatusInUpstream's body of new (GPUDIFF_UPSERT_STATUS,
 *     statussyncer.go:41-63).
 *   GPUDIFF_PLAN_UPSTREAM_DOWNSTREAM: each pair is (A = upstream/kcp copy,
 *     B = downstream copy): a spec-dirty pair gets the spec body
 *     of A (written over B), a status-dirty pair the status body of B (written
 *     into A).
 * GPUDIFF_PLAN_SPEC / GPUDIFF_PLAN_STATUS select which kinds are listed (an
 * upstream informer's batch wants spec writes only, a downstream informer's
 * status writes only); neither bit = both.
 * A write whose pair carries GPUDIFF_SPEC_NOOP / GPUDIFF_STATUS_NOOP is listed
 * with noop = 1 and no body: what the write carries in that region is, on the
 * wire, exactly what the write of the other document of the pair carries (Go
 * marshals int64 v and float64 v the same way).  For informer pairs that means
 * the call repeats the write already issued for `old`; for (A, B) pairs it
 * leaves B's compared content as it is.  Call after gpudiff_wait on the ticket
 * and before the submit after the next one (the staging is reused then);
 * GPUDIFF_E_STATE otherwise, or for a batch the context encoded on the host.
 * Release with gpudiff_write_plan_release. */
#define GPUDIFF_PLAN_INFORMER 0x0u
#define GPUDIFF_PLAN_SPEC 0x1u
#define GPUDIFF_PLAN_STATUS 0x2u
#define GPUDIFF_PLAN_UPSTREAM_DOWNSTREAM 0x4u
typedef struct gpudiff_write_plan {
    size_t n;                    /* writes: the spec-dirty pairs (ascending index), then the status-dirty ones */
    const uint32_t* pair_index;  /* the pair's index in the submitted batch */
    const uint8_t* kind;         /* GPUDIFF_UPSERT_SPEC / GPUDIFF_UPSERT_STATUS */
    const uint8_t* noop;         /* 1 = skip the call (no body) */
    gpudiff_bodies bodies;       /* n bodies (empty for no-op writes; status GPUDIFF_E_DECODE = undecodable) */
    void* internal;
} gpudiff_write_plan;
/* gpudiff_write_plan_get = _ex(..., GPUDIFF_PLAN_INFORMER, ...).  ABI 3 rendered a spec write from the
 * pair's FIRST document (the upstream/downstream reading); since ABI 4 the default is the informer
 * reading (the NEW document).  Bindings must check gpudiff_abi_version() == GPUDIFF_ABI_VERSION at load
 * (the Go binding and kcp_amd/gpudiff.py refuse a mismatched library) and pass
 * GPUDIFF_PLAN_UPSTREAM_DOWNSTREAM to _ex for (A, B) pairs. */
int gpudiff_write_plan_get(gpudiff_ctx* ctx, gpudiff_ticket ticket, gpudiff_write_plan* out);
int gpudiff_write_plan_get_ex(gpudiff_ctx* ctx, gpudiff_ticket ticket, uint32_t mode, gpudiff_write_plan* out);
void gpudiff_write_plan_release(gpudiff_ctx* ctx, gpudiff_write_plan* p);

/* The staged form: documents uploaded once into HBM (gpudiff_wbatch_create),
 * K10 launched on the context's stream (gpudiff_wbatch_run, asynchronous; with
 * GPUDIFF_OPT_TIMING each launch is bracketed by HIP events and
 * gpudiff_wbatch_stats.k10_ms is the mean), bodies read back and host-completed
 * (gpudiff_wbatch_fetch). */
typedef struct gpudiff_wbatch gpudiff_wbatch;
typedef struct gpudiff_wbatch_stats {
    uint64_t n_docs, json_bytes, body_bytes;  /* body_bytes: K10's output (valid after a fetch) */
    uint64_t scratch_bytes, out_cap_bytes;
    double k10_ms;                            /* mean K10 duration over the timed runs */
    uint64_t runs;                            /* timed runs (GPUDIFF_OPT_TIMING) */
} gpudiff_wbatch_stats;
int gpudiff_wbatch_create(gpudiff_ctx* ctx, const uint8_t* const* docs, const size_t* lens, size_t n, uint32_t mode,
                          gpudiff_wbatch** out);
int gpudiff_wbatch_run(gpudiff_ctx* ctx, gpudiff_wbatch* wb);
int gpudiff_wbatch_fetch(gpudiff_ctx* ctx, gpudiff_wbatch* wb, gpudiff_bodies* out);
int gpudiff_wbatch_stats_get(const gpudiff_wbatch* wb, gpudiff_wbatch_stats* st);
void gpudiff_wbatch_free(gpudiff_ctx* ctx, gpudiff_wbatch* wb);

/* The host path (Go-exact restatement; also what completes K10's deferrals):
 * one body into out[0, cap).  *out_len = the body length (also when it does not
 * fit: then GPUDIFF_E_CAPACITY).  GPUDIFF_E_DECODE if Go cannot decode doc. */
int gpudiff_upsert_body_host(const uint8_t* doc, size_t len, uint32_t mode, uint8_t* out, size_t cap,
                             size_t* out_len);

/* ---- Deployment splitter status roll-up ----
 * pkg/reconciler/deployment/deployment.go:41-91: when a leaf Deployment
 * changes, the splitter lists every cached Deployment labelled
 * kcp.dev/owned-by=<root> (:44-51; all namespaces, all logical clusters), sums
 * their status.{replicas, updatedReplicas, readyReplicas, availableReplicas,
 * unavailableReplicas} into the root's status (:74-85, int32: Go wrap-around)
 * and copies others[0].status.conditions (:89-91).  Batch form: n cached
 * Deployments (JSON) -> one group per distinct owned-by value, ordered by first
 * appearance; others[0] is the member with the lowest index (the lister's order
 * is unspecified).  The objects are typed appsv1.Deployments: Go 1.16
 * encoding/json rules apply to the fields read (case-insensitive field names,
 * repeated keys merge, null is a no-op, counters must be int32 literals); a
 * document Go cannot decode gets GPUDIFF_ROLLUP_DECODE.  Kernel K11 extracts
 * the fields (roll-up mode of k_encode_docs), K12 groups by label on the device;
 * documents outside K11's subset (GPUDIFF_TOK_*) are decided by the host path
 * (gpudiff_rollup_doc_host), which then regroups the batch with identical
 * results. */
typedef struct gpudiff_rollup_group {
    uint32_t first_doc;  /* others[0]: its status.conditions become the root's */
    uint32_t n_members;
    int32_t sums[5];     /* replicas, updatedReplicas, readyReplicas, availableReplicas, unavailableReplicas */
    uint32_t reserved;
} gpudiff_rollup_group;
#define GPUDIFF_ROLLUP_NONE (-1)    /* no kcp.dev/owned-by label: not a leaf */
#define GPUDIFF_ROLLUP_DECODE (-2)  /* Go cannot decode the document into an appsv1.Deployment */

typedef struct gpudiff_rollup {
    size_t n_docs;
    const int32_t* doc_group;              /* [n_docs]: group index or GPUDIFF_ROLLUP_* */
    size_t n_groups;
    const gpudiff_rollup_group* groups;    /* ascending first_doc */
    const int32_t* k11_status;             /* [n_docs]: K11's GPUDIFF_TOK_* (why the host took it) */
    size_t n_host;                         /* documents the host path decided */
    uint32_t host_grouped;                 /* 1: the host regrouped (deferrals or a label-hash collision) */
    void* internal;
} gpudiff_rollup;

typedef struct gpudiff_rbatch gpudiff_rbatch;
typedef struct gpudiff_rbatch_stats {
    uint64_t n_docs, json_bytes, scratch_bytes;
    double k11_ms, k12_ms;  /* mean durations over the timed runs (GPUDIFF_OPT_TIMING) */
    uint64_t runs;
} gpudiff_rbatch_stats;
/* documents uploaded once into HBM; run = K11 + K12 on the context stream
 * (asynchronous); fetch = results to the host, host path for deferrals.  The
 * caller's document buffers must stay valid until gpudiff_rbatch_free (the
 * host path and regrouping read them). */
int gpudiff_rbatch_create(gpudiff_ctx* ctx, const uint8_t* const* docs, const size_t* lens, size_t n,
                          gpudiff_rbatch** out);
int gpudiff_rbatch_run(gpudiff_ctx* ctx, gpudiff_rbatch* rb);
int gpudiff_rbatch_fetch(gpudiff_ctx* ctx, gpudiff_rbatch* rb, gpudiff_rollup* out);
int gpudiff_rbatch_stats_get(const gpudiff_rbatch* rb, gpudiff_rbatch_stats* st);
void gpudiff_rbatch_free(gpudiff_ctx* ctx, gpudiff_rbatch* rb);
/* create + run + fetch + free */
int gpudiff_rollup_status(gpudiff_ctx* ctx, const uint8_t* const* docs, const size_t* lens, size_t n,
                          gpudiff_rollup* out);
void gpudiff_rollup_release(gpudiff_ctx* ctx, gpudiff_rollup* r);
/* the host path for one document (Go-exact typed decode of the fields read):
 * counters into v[5]; the owned-by value into label[0, cap) with *label_len
 * its length, or SIZE_MAX when the label is absent (GPUDIFF_E_CAPACITY when it
 * does not fit); GPUDIFF_E_DECODE when Go rejects the document. */
int gpudiff_rollup_doc_host(const uint8_t* doc, size_t len, int32_t* v, uint8_t* label, size_t cap,
                            size_t* label_len);

/* ---- API-negotiation update classifier (second half) ----
 * Replaces the "Update" branch of Controller.enqueue,
 * pkg/reconciler/apiresource/controller.go:253-283, for the three kinds its
 * toQueueElementType (:185-236) types: APIResourceImport and
 * NegotiatedAPIResource (GPUDIFF_NEG_KIND_API; both have status {conditions:
 * [{type, status, lastTransitionTime, reason, message}]}) and
 * CustomResourceDefinition (GPUDIFF_NEG_KIND_CRD, :186-199; apiextensions/v1
 * status {conditions (same five fields), acceptedNames {plural, singular,
 * shortNames[], kind, listKind, categories[]}, storedVersions[]}).  Per
 * (old, new) pair: no old object
 * -> CREATED; equal resourceVersion -> IGNORE; different generation -> SPEC;
 * status not Semantic.DeepEqual (nil == empty, metav1.Time by instant) ->
 * STATUS; annotations differ OR labels EQUAL (the reference's missing `!` at
 * :278, reproduced) -> META; else IGNORE.  Objects are decoded with Go 1.16
 * encoding/json typed rules; DECODE when a side is not valid JSON, is not an
 * object, or a field the classifier reads (metadata.resourceVersion /
 * generation / labels / annotations, the typed status's fields and their
 * elements) fails Go's typed decode.  Type errors in fields the classifier does not read
 * (spec, metadata.name, ...) are not checked: such an object cannot reach the
 * reference's informer at all, so no reference outcome exists for it.
 * Kernel K13 (negotiation mode of k_encode_docs) extracts each document's
 * fields, K14 classifies each pair on the device; pairs with a document outside
 * K13's subset are classified by the host path (gpudiff_negotiate_pair_host). */
#define GPUDIFF_NEG_IGNORE 0
#define GPUDIFF_NEG_SPEC 1     /* SpecChanged */
#define GPUDIFF_NEG_STATUS 2   /* StatusOnlyChanged */
#define GPUDIFF_NEG_META 3     /* AnnotationOrLabelsOnlyChanged */
#define GPUDIFF_NEG_CREATED 4  /* no old object */
#define GPUDIFF_NEG_DECODE (-1)
#define GPUDIFF_NEG_KIND_API 0 /* APIResourceImport / NegotiatedAPIResource */
#define GPUDIFF_NEG_KIND_CRD 1 /* CustomResourceDefinition */

typedef struct gpudiff_nbatch gpudiff_nbatch;
typedef struct gpudiff_nbatch_stats {
    uint64_t n_pairs, json_bytes, scratch_bytes, n_host;
    double k13_ms, k14_ms;  /* mean durations over the timed runs (GPUDIFF_OPT_TIMING) */
    uint64_t runs;
} gpudiff_nbatch_stats;
/* olds[i] == NULL: no old object.  The documents are uploaded once into HBM;
 * run = K13 + K14 on the context stream (asynchronous); fetch = actions[n] to
 * the host, host path for the deferred pairs (GPUDIFF_E_STATE before the first
 * run).  The caller's buffers must stay
 * valid until gpudiff_nbatch_free. */
int gpudiff_nbatch_create(gpudiff_ctx* ctx, const uint8_t* const* olds, const size_t* old_lens,
                          const uint8_t* const* news, const size_t* new_lens, size_t n, gpudiff_nbatch** out);
/* kinds[i]: GPUDIFF_NEG_KIND_* of pair i (NULL: all GPUDIFF_NEG_KIND_API --
 * what the *_kinds-less entry points use); other values: GPUDIFF_E_INVAL */
int gpudiff_nbatch_create_kinds(gpudiff_ctx* ctx, const uint8_t* kinds, const uint8_t* const* olds,
                                const size_t* old_lens, const uint8_t* const* news, const size_t* new_lens, size_t n,
                                gpudiff_nbatch** out);
int gpudiff_nbatch_run(gpudiff_ctx* ctx, gpudiff_nbatch* nb);
int gpudiff_nbatch_fetch(gpudiff_ctx* ctx, gpudiff_nbatch* nb, int32_t* actions);
int gpudiff_nbatch_stats_get(const gpudiff_nbatch* nb, gpudiff_nbatch_stats* st);
void gpudiff_nbatch_free(gpudiff_ctx* ctx, gpudiff_nbatch* nb);
/* The host path (Go-exact typed decode + classification) over n pairs on
 * `threads` host threads -- no device needed; what the batch falls back to for
 * K13's deferrals, exposed for CPU baselines and callers without a GPU. */
int gpudiff_classify_updates_host(const uint8_t* const* olds, const size_t* old_lens, const uint8_t* const* news,
                                  const size_t* new_lens, size_t n, uint32_t threads, int32_t* actions);
int gpudiff_classify_updates_host_kinds(const uint8_t* kinds, const uint8_t* const* olds, const size_t* old_lens,
                                        const uint8_t* const* news, const size_t* new_lens, size_t n, uint32_t threads,
                                        int32_t* actions);
/* create + run + fetch + free */
int gpudiff_classify_updates(gpudiff_ctx* ctx, const uint8_t* const* olds, const size_t* old_lens,
                             const uint8_t* const* news, const size_t* new_lens, size_t n, int32_t* actions);
int gpudiff_classify_updates_kinds(gpudiff_ctx* ctx, const uint8_t* kinds, const uint8_t* const* olds,
                                   const size_t* old_lens, const uint8_t* const* news, const size_t* new_lens, size_t n,
                                   int32_t* actions);
/* the host path for one pair (old == NULL: no old object) */
int gpudiff_negotiate_pair_host(const uint8_t* old_json, size_t old_len, const uint8_t* new_json, size_t new_len,
                                int32_t* action);
int gpudiff_negotiate_pair_host_kind(uint32_t kind, const uint8_t* old_json, size_t old_len, const uint8_t* new_json,
                                     size_t new_len, int32_t* action);

/* ---- single-pair drop-ins (same semantics as the Go predicates) ---- */
int gpudiff_spec_equal(gpudiff_ctx* ctx, const uint8_t* old_json, size_t old_len,
                       const uint8_t* new_json, size_t new_len, int* equal);
int gpudiff_status_equal(gpudiff_ctx* ctx, const uint8_t* old_json, size_t old_len,
                         const uint8_t* new_json, size_t new_len, int* equal);

/* ---- host helper: render a changed path ("spec.containers[0].image") ----
 * path_kind is the kind byte reported with the hash (selects the region). */
int gpudiff_resolve_path(const uint8_t* old_json, size_t old_len, const uint8_t* new_json,
                         size_t new_len, uint64_t path_hash, uint8_t path_kind,
                         uint32_t path_hash_bits, char* buf, size_t cap, size_t* out_len);

#ifdef __cplusplus
}
#endif
#endif
