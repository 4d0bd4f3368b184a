// K0: device JSON tokenizer + canonical encoder (tokenize.hip) and the
// device object-store kernels around it.  Internal, not part of the ABI.
//
// One wave turns one raw JSON object (an informer event body) into the same
// blob the host encoder writes (include/gpudiff_format.h), followed by the
// path table the object store checks old-vs-new paths with:
//
//   blob = [spec segment][status segment][hs u64[n] | phs u64[n] | cs u64[n] | key bytes | pad]
//
// Anything outside the device's exact subset -- a Go decode error of any kind,
// a float literal beyond the exact fast path, a key that needs unescaping, a
// duplicate key or path-hash collision, nesting deeper than 255 -- is not
// guessed at: the object is reported with a nonzero status and the host
// encoder (json.cpp + encoder.cpp, the Go-exact path) takes it over.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gpudiff_format.h"

namespace gd {

struct TokDoc {
    uint64_t json_off;     // document bytes in the staged JSON buffer (16-B aligned, kTokSlack readable after)
    uint64_t scratch_off;  // per-document working area (tok_scratch_bytes(json_len) bytes)
    uint32_t json_len;
    uint32_t seed;         // path-hash seed (the slot's)
    uint32_t pad[2];
};

struct TokOut {
    uint64_t off;          // blob offset in the output space
    uint32_t bytes;        // blob bytes incl. the path table (multiple of 16)
    uint32_t spec_l, spec_ar, stat_l, stat_ar;
    uint32_t oflags;       // GPUDIFF_OBJ_HAS_STATUS
    uint32_t status;       // GPUDIFF_TOK_*
    uint32_t n_nodes;
    uint32_t n_tab;        // path-table entries
};
static_assert(sizeof(TokDoc) == 32, "TokDoc");
static_assert(sizeof(TokOut) == 48, "TokOut");

__host__ __device__ inline uint64_t tok_align(uint64_t x) { return (x + 255u) & ~(uint64_t)255u; }
__host__ __device__ inline uint32_t tok_cap(uint32_t len) { return len + 2u; }
__host__ __device__ inline uint32_t node_cap(uint32_t len) { return len / 2u + 2u; }

// Per-document working area: tokens, node records, hashes, values, sort keys,
// decoded strings.  Bounded by the JSON length (a node needs >= 2 bytes).
struct TokLayout {
    uint64_t tok, rec, h, val, skey, meta, order, sidx, str, total;
};
__host__ __device__ inline TokLayout tok_layout(uint32_t len) {
    TokLayout L;
    const uint64_t nc = node_cap(len);
    L.tok = 0;
    L.rec = tok_align(4ull * tok_cap(len));
    L.h = L.rec + tok_align(16ull * nc);
    L.val = L.h + tok_align(8ull * nc);
    L.skey = L.val + tok_align(8ull * nc);
    L.meta = L.skey + tok_align(8ull * nc);
    L.order = L.meta + tok_align(4ull * nc);
    L.sidx = L.order + tok_align(4ull * nc);
    L.str = L.sidx + tok_align(4ull * nc);
    L.total = L.str + tok_align((uint64_t)len + 32u);
    return L;
}
__host__ __device__ inline uint64_t tok_scratch_bytes(uint32_t len) { return tok_layout(len).total; }
// upper bound of a document's blob: a node takes >= 2 JSON bytes and <= 20 B
// of segment + 16 B of long-value pad + 24 B of path table; key bytes <= len
__host__ __device__ inline uint64_t tok_blob_bound(uint32_t len) { return 31ull * len + 96u; }

// K10 (k_encode_docs in marshal mode, the write path): per-document working
// area.  tok/rec/str are laid out as phases 1-2 of K0 expect; the rest holds
// one word per node (own text size, key size, subtree size, flags, child
// count, child-list base, child list, sibling prefix sums, rank, value start,
// depth order) and the decoded int64 / string location.
struct MarshalLayout {
    uint64_t tok, rec, str, val, vsz, ksz, sz, fl, nch, base, kids, pre, rank, vst, order, total;
};
__host__ __device__ inline MarshalLayout marshal_layout(uint32_t len) {
    MarshalLayout L;
    const uint64_t nc = node_cap(len);
    L.tok = 0;
    L.rec = tok_align(4ull * tok_cap(len));
    L.str = L.rec + tok_align(16ull * nc);
    L.val = L.str + tok_align((uint64_t)len + 32u);
    L.vsz = L.val + tok_align(8ull * nc);
    L.ksz = L.vsz + tok_align(4ull * nc);
    L.sz = L.ksz + tok_align(4ull * nc);
    L.fl = L.sz + tok_align(4ull * nc);
    L.nch = L.fl + tok_align(4ull * nc);
    L.base = L.nch + tok_align(4ull * nc);
    L.kids = L.base + tok_align(4ull * nc);
    L.pre = L.kids + tok_align(4ull * nc);
    L.rank = L.pre + tok_align(4ull * nc);
    L.vst = L.rank + tok_align(4ull * nc);
    L.order = L.vst + tok_align(4ull * nc);
    L.total = L.order + tok_align(4ull * nc);
    return L;
}
__host__ __device__ inline uint64_t marshal_scratch_bytes(uint32_t len) { return marshal_layout(len).total; }
// output room per document: a body longer than this is left to the host
// (escaping can grow a string 6-fold, owner references gain their fixed keys)
__host__ __device__ inline uint64_t marshal_out_cap(uint32_t len) { return ((2ull * len + 512u) + 15u) & ~15ull; }

// K11 (k_encode_docs in roll-up mode, the Deployment splitter's status
// aggregation): per document, the five status counters and the owned-by label
// span; a nonzero status leaves the document to the host path.
struct RollOut {
    int32_t v[5];        // replicas, updatedReplicas, readyReplicas, availableReplicas, unavailableReplicas
    uint32_t label_off;  // kcp.dev/owned-by value bytes in the document (no escapes)
    uint32_t label_len;
    uint16_t status;     // GPUDIFF_TOK_*
    uint16_t flags;      // kRollHasLabel
};
static_assert(sizeof(RollOut) == 32, "RollOut");
constexpr uint16_t kRollHasLabel = 1u;
// phases 1-2 only: tokens, node records, decoded-string room
__host__ __device__ inline uint64_t rollup_scratch_bytes(uint32_t len) {
    return tok_align(4ull * tok_cap(len)) + tok_align(16ull * node_cap(len)) + tok_align((uint64_t)len + 32u);
}

// K13 (k_encode_docs in negotiation mode, the API-negotiation update
// classifier): per document, the fields controller.go:253-283 reads, as spans
// into the document (no escapes) and parsed values; a nonzero status leaves
// every pair holding the document to the host path.
constexpr uint32_t kNegMaxMembers = 16;  // labels / annotations entries on the device
constexpr uint32_t kNegMaxConds = 8;     // status.conditions elements on the device
struct NegMember {
    uint32_t koff, klen, voff, vlen;
};
struct NegCond {
    uint32_t off[4], len[4];  // type, status, reason, message
    int64_t sec;              // lastTransitionTime: unix seconds (zero Time: -62135596800)
    int32_t nsec;
    uint32_t pad;
};
constexpr uint32_t kNegMaxList = 8;      // CRD []string elements on the device (each list)
struct NegSpan {
    uint32_t off, len;
};
struct NegOut {
    uint32_t status;          // GPUDIFF_TOK_*
    uint32_t n_lab, n_ann, n_cond;
    uint32_t rv_off, rv_len, pad0, pad1;
    int64_t gen;
    int64_t pad2;
    NegMember lab[kNegMaxMembers], ann[kNegMaxMembers];
    NegCond cond[kNegMaxConds];
    // GPUDIFF_NEG_KIND_CRD only (TokDoc.pad[0]): status.acceptedNames {plural,
    // singular, kind, listKind} (absent / null: empty spans), shortNames,
    // categories, storedVersions (nil and empty: 0 elements)
    NegSpan names[4];
    uint32_t n_short, n_cat, n_stored, pad3;
    NegSpan shortn[kNegMaxList], cat[kNegMaxList], stored[kNegMaxList];
};
static_assert(sizeof(NegCond) == 48 && sizeof(NegOut) == 1184, "NegOut");
constexpr int64_t kZeroTimeSec = -62135596800ll;

constexpr uint32_t kTokMaxLen = (1u << 24) - 64u;  // token words hold 24-bit positions
constexpr uint32_t kTokSlack = 32u;                 // readable bytes K0 needs after each staged document

// ------------------------------------------------------------ device object store
// One slot per informer-cache object: its resident blob (K0 format, with the
// path table) in the current space.
struct DSlot {
    uint64_t off;
    uint32_t spec_l, spec_ar, stat_l, stat_ar;
    uint32_t bytes;   // blob + path table
    uint32_t flags;   // DS_* | seed << 8
    uint32_t pend;    // last batch that deferred an event of this slot to the host
    uint32_t n_tab;   // path-table entries
};
static_assert(sizeof(DSlot) == 40, "DSlot");
constexpr uint32_t DS_LIVE = 1u, DS_HAS_STATUS = 2u, DS_PENDING = 4u;

// Per staged document of a store batch: its slot chain inside the batch.
struct DocLink {
    uint32_t slot;
    int32_t prev;       // previous document of the slot in this batch, -1
    int32_t next;       // next one, -1
    uint32_t row;       // result row (event index); kNoRow for an old_json first-sighting document
    uint32_t pair_id, cluster_id;
    uint32_t pad[2];
};
static_assert(sizeof(DocLink) == 32, "DocLink");
constexpr uint32_t kNoRow = 0xFFFFFFFFu;

// counters[] of a store (device): 1 live slots, 2-3 live bytes (u64)
constexpr uint32_t kCtrLive = 1, kCtrLiveBytes = 2;

// host-resolved state of one slot (kernel k_place applies it)
struct SlotUpdate {
    DSlot entry;        // off tagged with kRelTag = relative to the placed bytes
    uint32_t slot;
    uint32_t batch;     // the batch whose deferred events produced it
};
constexpr uint64_t kRelTag = 1ull << 63;   // offset relative to the placed bytes
constexpr uint64_t kSlotTag = 1ull << 62;  // the resident blob of slot (off & 0xFFFFFFFF)

// tuning: per-phase wall-clock ticks (100 MHz) of K0 summed over waves since the
// last call; enable = record from now on
hipError_t k0_profile(int enable, uint64_t* out8);

// K0 over docs [0, n): blobs appended to space at atomic offsets (*used).
// slots/links (optional): the seed is the slot's (DSlot.flags >> 8).
hipError_t launch_encode_docs(hipStream_t s, const TokDoc* docs, uint32_t n, const uint8_t* json, uint8_t* scratch,
                              uint8_t* space, uint64_t space_cap, unsigned long long* used, uint64_t mask,
                              TokOut* out, const DSlot* slots = nullptr, const DocLink* links = nullptr);
// K10: the write path's request bodies (GPUDIFF_UPSERT_*): docs[i].pad holds
// the body's u64 offset in `bodies` (room: marshal_out_cap(json_len)); out[i]
// gets {off, bytes, status}.  A nonzero status leaves the document to the host.
hipError_t launch_marshal_docs(hipStream_t s, const TokDoc* docs, uint32_t n, const uint8_t* json, uint8_t* scratch,
                               uint8_t* bodies, uint32_t mode, TokOut* out);
// K11: roll-up fields per document into outs (RollOut[n]); scratch per document at docs[i].scratch_off
hipError_t launch_rollup_docs(hipStream_t s, const TokDoc* docs, uint32_t n, const uint8_t* json, uint8_t* scratch,
                              RollOut* outs);
// K13: negotiation fields per document into outs (NegOut[n]); scratch as K11's
hipError_t launch_negotiate_docs(hipStream_t s, const TokDoc* docs, uint32_t n, const uint8_t* json, uint8_t* scratch,
                                 NegOut* outs);
// K14: one action per pair (old doc 2i, new doc 2i+1; absent[i]: no old object);
// kNegDefer = the host decides the pair
constexpr int32_t kNegDefer = -2;
hipError_t launch_negotiate_pairs(hipStream_t s, const NegOut* outs, const uint8_t* absent, const TokDoc* docs,
                                  const uint8_t* json, uint32_t n_pairs, int32_t* actions);
// K12: group the documents by owned-by label (xxh64 radix sort + byte check),
// int32 sums per group; see rollup.hip
// K0c: per event, a path-hash collision with its old side (the two path tables disagree)
hipError_t launch_collide(hipStream_t s, const DocLink* links, const TokOut* outs, const DSlot* slots, uint32_t n,
                          const uint8_t* space, uint8_t* coll);
// K0x: walk each slot's chain: rows for K2, deferrals, the slot's new resident blob
hipError_t launch_link(hipStream_t s, const uint32_t* heads, uint32_t n_heads, const DocLink* links,
                       const TokOut* outs, const uint8_t* coll, DSlot* slots, gpudiff_pair_row* rows,
                       uint32_t* pair_ids, uint8_t* deferred, uint32_t batch, uint32_t* n_deferred,
                       uint32_t* counters);
// compaction: pack every live slot's blob into dst, rewrite the offsets, *used = total
hipError_t launch_compact_store(hipStream_t s, DSlot* slots, uint32_t n, const uint8_t* src, uint8_t* dst,
                                uint64_t* sizes, uint64_t* block_sums, unsigned long long* used);
// place host-resolved blobs, rows and slot states
hipError_t launch_place(hipStream_t s, const uint8_t* stage, uint64_t bytes, uint8_t* space,
                        unsigned long long* used, uint64_t cap, gpudiff_pair_row* rows, uint32_t* pair_ids,
                        uint32_t n_rows, const SlotUpdate* ups, uint32_t n_ups, DSlot* slots, uint32_t* counters,
                        uint32_t* err);
hipError_t launch_forget(hipStream_t s, DSlot* slots, uint32_t slot, uint32_t* counters);

}  // namespace gd
