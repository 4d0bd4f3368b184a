// Internal engine state shared by the C-ABI translation units (api.cpp,
// store.cpp).  Not part of the ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <functional>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/gpudiff.h"
#include "encoder.h"
#include "pool.h"
#include "kernels.h"

using gd::PairEncoder;
using gd::EncodeConfig;

namespace gd {
extern thread_local std::string g_last_hip_error;
}

#define HIPCHK(x)                                             \
    do {                                                      \
        hipError_t e_ = (x);                                  \
        if (e_ != hipSuccess) {                               \
            gd::g_last_hip_error = hipGetErrorString(e_);     \
            return GPUDIFF_E_DEVICE;                          \
        }                                                     \
    } while (0)

namespace gd {
struct Part {
    std::vector<uint8_t> pool;
    std::vector<gpudiff_pair_row> rows;
    uint64_t leaves = 0, errors = 0, reseeded = 0;
};
}  // namespace gd

// changed-path arena entries per K2 wave (a pair whose worst case does not
// fit the wave's remaining arena is deferred to K4)
inline constexpr uint32_t kArenaPerWave = 16384;

struct gpudiff_hbatch {
    uint8_t* pool = nullptr;
    gpudiff_pair_row* rows = nullptr;
    size_t n = 0;
    uint64_t pool_bytes = 0;
    uint64_t leaves = 0, errors = 0, reseeded = 0;
    uint64_t pool_cap = 0;
    size_t rows_cap = 0;
    bool pinned = false;
    hipEvent_t used = nullptr;  // last async copy that reads this batch
};

struct gpudiff_dbatch {
    uint64_t pool_cap = 0, pool_used = 0;
    uint64_t max_pairs = 0, n_pairs = 0;
    uint64_t leaves = 0, compare_bytes = 0, value_bytes = 0;
    // K0-encoded batches (the device-encode store / submit): the rows are built on the device, so
    // compare_bytes is unknown on the host; this is the batch's JSON bytes per pair side x 2 (config3
    // objects: 0.85 compare bytes per JSON byte), the size class K2's item split goes by (k2_sub_shift)
    uint64_t size_hint_bytes = 0;
    uint8_t* pool = nullptr;
    bool pool_borrowed = false;  // pool owned by a gpudiff_store (its current space)
    gpudiff_pair_row* rows = nullptr;
    uint32_t* pair_ids = nullptr;
    uint8_t* flags = nullptr;
    uint32_t* caps = nullptr;
    void* chunk_counts = nullptr;
    uint32_t* summary = nullptr;
    uint32_t* spec_ids = nullptr;
    uint32_t* status_ids = nullptr;
    uint32_t* dirty_ids = nullptr;
    uint32_t* dirty_idx = nullptr;
    uint32_t* scratch_off = nullptr;
    uint32_t* path_count = nullptr;
    uint32_t* path_off = nullptr;
    uint32_t* tile_sums = nullptr;
    uint32_t* path_src = nullptr;
    uint32_t* path_cnt = nullptr;
    uint8_t* nbits = nullptr;   // per pair: no-op bits of K2's joins
    uint8_t* noop_d = nullptr;  // per dirty pair: no-op bits
    uint64_t arena_cap = 0;
    uint64_t* arena_h = nullptr;
    uint8_t* arena_k = nullptr;
    uint64_t scratch_cap = 0;
    uint64_t* scratch_h = nullptr;
    uint8_t* scratch_k = nullptr;
    uint32_t* slot_owner = nullptr;  // K4 slices (kernels.h DiffBuffers)
    uint32_t* slice_cnt = nullptr;
    uint8_t* slice_weq = nullptr;
    uint64_t* out_h = nullptr;
    uint8_t* out_k = nullptr;
    hipEvent_t done = nullptr;
    gpudiff_ticket ticket = 0;
    uint32_t* gather_send = nullptr;  // gpudiff_dbatch_bind_gather
    uint32_t gather_cap_spec = 0, gather_cap_status = 0;
    // gpudiff_dbatch_result_slot: the spec / status lists and the summary (counts) of the other slot
    // (spec_ids / status_ids / summary are always the current slot's; switching swaps them), allocated on
    // first use -- all three or none
    uint32_t* ids_alt[2] = {nullptr, nullptr};
    uint32_t* summary_alt = nullptr;
    uint32_t res_slot = 0;
    // gpudiff_dbatch_create_view: this batch diffs `base`'s resident pairs (pool, rows, pair IDs borrowed,
    // refreshed at every diff) into its own outputs, so two passes over one population can be in flight
    const gpudiff_dbatch* base = nullptr;
    // a base's live views (gpudiff_dbatch_create_view registers, gpudiff_dbatch_free removes): the passes of one
    // population that can be in flight together -- K2 launches half its grid while another of them is running
    mutable std::vector<gpudiff_dbatch*> views;
    int device = -1;
    uint32_t* tail_perm = nullptr;  // K2's largest-first final round (kernels.h DiffBuffers)
    gd::TailPermKey tail_perm_key;
    uint64_t rows_gen = 0;  // bumped whenever the rows change (appends, resets, store batches): K2's cached order
};

struct DStore;

struct ResultStore {
    std::vector<uint8_t> flags;
    std::vector<uint32_t> spec, status, dirty, off;
    std::vector<uint64_t> hashes;
    std::vector<uint8_t> kinds;
};

struct gpudiff_ctx {
    int device = GPUDIFF_DEVICE_NONE;
    bool has_device = false;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    uint32_t threads = 1;
    uint32_t flags = 0;
    bool k2_timeline = false;  // gpudiff_k2_profile installed a buffer: the timeline build of K2 runs
    EncodeConfig ecfg;
    uint64_t hash_mask = ~0ULL;
    std::vector<std::unique_ptr<PairEncoder>> encoders;
    std::vector<gd::Part> parts;
    gpudiff_ticket next_ticket = 1;
    std::unordered_map<gpudiff_ticket, gpudiff_dbatch*> tickets;
    std::vector<std::array<hipEvent_t, 5>> pass_ev;
    size_t n_pass = 0;
    hipStream_t rb = nullptr;     // result readback (never behind work queued after the batch)
    // per-ticket completion hooks run by gpudiff_wait before results are
    // published (the device-encode store resolves its host-deferred events)
    std::unordered_map<gpudiff_ticket, std::function<int(ResultStore&)>> finishers;
    // GPUDIFF_OPT_DEVICE_ENCODE: gpudiff_submit's pairs go through K0 (dstore.cpp, pair mode)
    DStore* pair_store = nullptr;
    // submit ring
    gpudiff_dbatch* ring[2] = {nullptr, nullptr};
    gpudiff_hbatch* ring_hb[2] = {nullptr, nullptr};
    uint32_t ring_next = 0;
    // persistent host workers (c->threads of them, the calling thread included), made on first use
    std::unique_ptr<gd::WorkerPool> pool;
};

// ------------------------------------------------------------------ helpers
inline gd::WorkerPool& workers(gpudiff_ctx* c) {
    if (!c->pool) c->pool.reset(new gd::WorkerPool(c->threads));
    return *c->pool;
}

inline int set_device(gpudiff_ctx* c) {
    if (!c->has_device) return GPUDIFF_E_NODEVICE;
    HIPCHK(hipSetDevice(c->device));
    return GPUDIFF_OK;
}

template <class T>
inline int dalloc(T** p, uint64_t count) {
    *p = nullptr;
    size_t bytes = (size_t)std::max<uint64_t>(count, 1) * sizeof(T);
    HIPCHK(hipMalloc((void**)p, bytes));
    return GPUDIFF_OK;
}

inline void dfree_all(gpudiff_dbatch* d) {
    if (d->pool && !d->pool_borrowed) (void)hipFree(d->pool);
    if (d->base) d->rows = nullptr, d->pair_ids = nullptr;  // a view's inputs are its base's
    void* ps[] = {d->rows, d->pair_ids, d->flags, d->caps, d->chunk_counts, d->summary, d->spec_ids,
                  d->status_ids, d->dirty_ids, d->dirty_idx, d->scratch_off, d->path_count, d->path_off,
                  d->tile_sums, d->path_src, d->path_cnt, d->arena_h, d->arena_k,
                  d->scratch_h, d->scratch_k, d->out_h, d->out_k, d->nbits, d->noop_d, d->slot_owner,
                  d->slice_cnt, d->slice_weq, d->ids_alt[0], d->ids_alt[1], d->summary_alt, d->tail_perm};
    for (void* p : ps)
        if (p) (void)hipFree(p);
    if (d->done) (void)hipEventDestroy(d->done);
}

// copies a finished diff pass's results to host memory (gpudiff_wait's body)
int collect_results(gpudiff_ctx* c, gpudiff_dbatch* d, ResultStore& rs);

// canonical bytes of one object's long string values (V of SURVEY §8(d)); blob at pool + off
inline uint64_t blob_value_bytes(const uint8_t* blob, uint32_t spec_l, uint32_t spec_ar, uint32_t stat_l) {
    uint64_t v = 0;
    const uint32_t* m = (const uint32_t*)(blob + 12ull * spec_l);
    for (uint32_t i = 0; i < spec_l; i++)
        if (gpudiff_meta_is_long(m[i])) v += gpudiff_meta_len(m[i]);
    m = (const uint32_t*)(blob + gpudiff_seg_bytes(spec_l, spec_ar) + 12ull * stat_l);
    for (uint32_t i = 0; i < stat_l; i++)
        if (gpudiff_meta_is_long(m[i])) v += gpudiff_meta_len(m[i]);
    return v;
}

// bytes the decision kernel must read for this pair (DESIGN.md "Roofline"; the same rule as
// k_compare_flat's streamed chunks): gpudiff_format.h gpudiff_pair_compare_bytes
inline uint64_t pair_compare_bytes(const gpudiff_pair_row& r) { return gpudiff_pair_compare_bytes(&r); }
