// C-ABI of the gpudiff engine (include/gpudiff.h): contexts, host encoding,
// device batches, the diff pipeline and result retrieval.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/gpudiff.h"
#include "encoder.h"
#include "dstore.h"
#include "engine.h"
#include "kernels.h"
#include "xxh64.h"

using namespace gd;

namespace gd {
thread_local std::string g_last_hip_error;
}
using gd::g_last_hip_error;

// Changed-path buffers: the K2 wave arenas (arena entries), the K4 scratch for
// deferred pairs (scratch entries) and the compacted output, which can never
// hold more than both together.
static int ensure_paths(gpudiff_dbatch* d, uint64_t arena, uint64_t scratch) {
    const bool ok_a = arena <= d->arena_cap && d->arena_h;
    const bool ok_s = scratch <= d->scratch_cap && d->scratch_h;
    if (ok_a && ok_s) return GPUDIFF_OK;
    // Only the short buffers are replaced: the overflow re-run of the join grows
    // the scratch while the wave arenas still hold the paths K2 joined in place.
    auto drop = [](auto*& p) {
        if (p) (void)hipFree(p);
        p = nullptr;
    };
    drop(d->out_h);
    drop(d->out_k);
    int rc;
    if (!ok_a) {
        drop(d->arena_h);
        drop(d->arena_k);
        d->arena_cap = 0;
        if ((rc = dalloc(&d->arena_h, arena)) || (rc = dalloc(&d->arena_k, arena))) return rc;
        d->arena_cap = arena;
    }
    if (!ok_s) {
        // scratch offsets share a u32 with the arena bit (scratch_off): at most 2^31 entries
        if (scratch > kMaxScratchEntries) return GPUDIFF_E_CAPACITY;
        scratch = std::min<uint64_t>(std::max<uint64_t>({scratch + scratch / 8, d->scratch_cap, 1u << 16}),
                                     kMaxScratchEntries);
        scratch = (scratch + kJoinSliceHost - 1) / kJoinSliceHost * kJoinSliceHost;  // whole K4 slice slots
        drop(d->scratch_h);
        drop(d->scratch_k);
        drop(d->slot_owner);
        drop(d->slice_cnt);
        drop(d->slice_weq);
        d->scratch_cap = 0;
        const uint64_t slots = scratch / kJoinSliceHost;
        if ((rc = dalloc(&d->scratch_h, scratch)) || (rc = dalloc(&d->scratch_k, scratch)) ||
            (rc = dalloc(&d->slot_owner, slots)) || (rc = dalloc(&d->slice_cnt, slots)) ||
            (rc = dalloc(&d->slice_weq, slots)))
            return rc;
        d->scratch_cap = scratch;
    }
    const uint64_t out = d->arena_cap + d->scratch_cap;
    if ((rc = dalloc(&d->out_h, out)) || (rc = dalloc(&d->out_k, out))) return rc;
    return GPUDIFF_OK;
}

static DiffBuffers buffers_of(gpudiff_ctx* c, gpudiff_dbatch* d) {
    DiffBuffers b;
    b.rows = d->rows;
    b.pool = d->pool;
    b.pair_ids = d->pair_ids;
    b.n_pairs = (uint32_t)d->n_pairs;
    b.flags = d->flags;
    b.caps = d->caps;
    b.chunk_counts = d->chunk_counts;
    b.summary = d->summary;
    b.spec_ids = d->spec_ids;
    b.status_ids = d->status_ids;
    b.dirty_ids = d->dirty_ids;
    b.dirty_idx = d->dirty_idx;
    b.scratch_off = d->scratch_off;
    b.path_count = d->path_count;
    b.path_off = d->path_off;
    b.tile_sums = d->tile_sums;
    b.path_src = d->path_src;
    b.path_cnt = d->path_cnt;
    b.nbits = d->nbits;
    b.noop_d = d->noop_d;
    b.arena_h = d->arena_h;
    b.arena_k = d->arena_k;
    b.arena_per_wave = kArenaPerWave >> ((c->flags >> GPUDIFF_OPT_ARENA_SHIFT) & 0xFu);
    b.scratch_h = d->scratch_h;
    b.scratch_k = d->scratch_k;
    b.scratch_cap = d->scratch_cap;
    b.out_h = d->out_h;
    b.out_k = d->out_k;
    b.slot_owner = d->slot_owner;
    b.slice_cnt = d->slice_cnt;
    b.slice_weq = d->slice_weq;
    b.hash_mask = c->hash_mask;
    b.k2_timeline = c->k2_timeline ? 1u : 0u;
    b.k2_shared = 0u;
    b.tail_perm = d->tail_perm;
    b.tail_perm_key = &d->tail_perm_key;
    b.rows_gen = d->rows_gen;
    b.gather_send = d->gather_send;
    b.gather_cap_spec = d->gather_cap_spec;
    b.gather_cap_status = d->gather_cap_status;
    b.avg_pair_bytes = d->n_pairs ? (d->compare_bytes ? d->compare_bytes : d->size_hint_bytes) / d->n_pairs : 0;
    return b;
}


// ------------------------------------------------------------------ library
extern "C" {

const char* gpudiff_strerror(int err) {
    switch (err) {
        case GPUDIFF_OK: return "ok";
        case GPUDIFF_E_INVAL: return "invalid argument";
        case GPUDIFF_E_NOMEM: return "out of host memory";
        case GPUDIFF_E_DEVICE: return g_last_hip_error.empty() ? "HIP runtime error" : g_last_hip_error.c_str();
        case GPUDIFF_E_NODEVICE: return "no GPU in this context (there is no CPU fallback)";
        case GPUDIFF_E_CAPACITY: return "device batch capacity exceeded";
        case GPUDIFF_E_STATE: return "invalid call order / unknown ticket";
        case GPUDIFF_E_DECODE: return "input failed to decode as a JSON object";
        case GPUDIFF_E_NOTFOUND: return "path hash not found";
        default: return "unknown error";
    }
}

int gpudiff_abi_version(void) { return GPUDIFF_ABI_VERSION; }

int gpudiff_device_count(int* n) {
    if (!n) return GPUDIFF_E_INVAL;
    *n = 0;
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) return GPUDIFF_OK;
    *n = c;
    return GPUDIFF_OK;
}

int gpudiff_open(const gpudiff_opts* opts, gpudiff_ctx** out) {
    if (!out) return GPUDIFF_E_INVAL;
    *out = nullptr;
    gpudiff_opts o{};
    o.device = GPUDIFF_DEVICE_CURRENT;
    if (opts) o = *opts;
    if (o.flags & ~GPUDIFF_OPT_KNOWN) return GPUDIFF_E_INVAL;  // a removed tuning bit, or a typo
    std::unique_ptr<gpudiff_ctx> c(new (std::nothrow) gpudiff_ctx());
    if (!c) return GPUDIFF_E_NOMEM;
    uint32_t hw = std::max(1u, std::thread::hardware_concurrency());
    c->threads = o.encode_threads ? o.encode_threads : std::min(hw, 16u);
    c->flags = o.flags;
    c->ecfg.hash_bits = (o.path_hash_bits == 0 || o.path_hash_bits >= GPUDIFF_PATH_HASH_BITS) ? GPUDIFF_PATH_HASH_BITS
                                                                                            : o.path_hash_bits;
    if (c->ecfg.hash_bits < 8) return GPUDIFF_E_INVAL;
    c->hash_mask = c->ecfg.hash_bits >= 64 ? ~0ULL : ((1ULL << c->ecfg.hash_bits) - 1);
    if (o.device != GPUDIFF_DEVICE_NONE) {
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return GPUDIFF_E_NODEVICE;
        int dev = o.device;
        if (dev == GPUDIFF_DEVICE_CURRENT) HIPCHK(hipGetDevice(&dev));
        if (dev < 0 || dev >= n) return GPUDIFF_E_INVAL;
        c->device = dev;
        c->has_device = true;
        HIPCHK(hipSetDevice(dev));
        if (o.stream) {
            c->stream = (hipStream_t)o.stream;
        } else {
            HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
            c->own_stream = true;
        }
        HIPCHK(hipStreamCreateWithFlags(&c->rb, hipStreamNonBlocking));
    }
    *out = c.release();
    return GPUDIFF_OK;
}

void gpudiff_close(gpudiff_ctx* c) {
    if (!c) return;
    if (c->has_device) {
        (void)hipSetDevice(c->device);
        (void)hipStreamSynchronize(c->stream);
        if (c->pair_store) dstore_free(c, c->pair_store);
        dstore_host_bufs_release(c);  // gpudiff_host_alloc buffers the caller did not free
        for (int i = 0; i < 2; i++) {
            if (c->ring[i]) gpudiff_dbatch_free(c, c->ring[i]);
            if (c->ring_hb[i]) gpudiff_hbatch_free(c, c->ring_hb[i]);
        }
        for (auto& a : c->pass_ev)
            for (auto& e : a) (void)hipEventDestroy(e);
        if (c->rb) {
            (void)hipStreamSynchronize(c->rb);
            (void)hipStreamDestroy(c->rb);
        }
        if (c->own_stream) (void)hipStreamDestroy(c->stream);
    }
    delete c;
}

// ------------------------------------------------------------------ encoding
int gpudiff_encode_pairs(gpudiff_ctx* c, const gpudiff_json_pair* pairs, size_t n, gpudiff_hbatch** out) {
    if (!c || !out || (n && !pairs)) return GPUDIFF_E_INVAL;
    if (n > 0xFFFFFFFFull) return GPUDIFF_E_INVAL;
    *out = nullptr;
    uint32_t T = (uint32_t)std::min<size_t>(c->threads, std::max<size_t>(1, n / 256));
    while (c->encoders.size() < T) c->encoders.emplace_back(new PairEncoder(c->ecfg));
    if (c->parts.size() < T) c->parts.resize(T);
    try {
        auto work = [&](uint32_t t) {
            Part& part = c->parts[t];
            part.pool.clear();
            part.rows.clear();
            PairEncoder& enc = *c->encoders[t];
            enc.leaves_written = enc.reseeded = enc.decode_errors = 0;
            size_t b = n * t / T, e = n * (t + 1) / T;
            part.rows.resize(e - b);
            for (size_t i = b; i < e; i++) {
                const gpudiff_json_pair& p = pairs[i];
                enc.encode_json(p.old_json, p.old_len, p.new_json, p.new_len, p.pair_id, p.cluster_id, part.pool,
                                part.rows[i - b]);
            }
            size_t pad = (part.pool.size() + GPUDIFF_BLOB_ALIGN - 1) & ~(size_t)(GPUDIFF_BLOB_ALIGN - 1);
            part.pool.resize(pad, 0);
            part.leaves = enc.leaves_written;
            part.errors = enc.decode_errors;
            part.reseeded = enc.reseeded;
        };
        workers(c).run(T, work);
    } catch (const std::bad_alloc&) {
        return GPUDIFF_E_NOMEM;
    }
    uint64_t total = 0;
    for (uint32_t t = 0; t < T; t++) total += c->parts[t].pool.size();
    gpudiff_hbatch* raw = nullptr;
    uint8_t* pool_p = nullptr;
    gpudiff_pair_row* rows_p = nullptr;
    int rc = gpudiff_hbatch_create(c, total, n, 0, &raw, &pool_p, &rows_p);
    if (rc) return rc;
    std::unique_ptr<gpudiff_hbatch> hb(raw);
    uint64_t base = 0;
    size_t r0 = 0;
    for (uint32_t t = 0; t < T; t++) {
        Part& part = c->parts[t];
        if (!part.pool.empty()) memcpy(hb->pool + base, part.pool.data(), part.pool.size());
        for (size_t i = 0; i < part.rows.size(); i++) {
            gpudiff_pair_row r = part.rows[i];
            r.off_a += base;
            r.off_b += base;
            hb->rows[r0 + i] = r;
        }
        r0 += part.rows.size();
        base += part.pool.size();
        hb->leaves += part.leaves;
        hb->errors += part.errors;
        hb->reseeded += part.reseeded;
    }
    *out = hb.release();
    return GPUDIFF_OK;
}

static void hb_release_buffers(gpudiff_hbatch* hb) {
    if (hb->pinned) {
        if (hb->pool) (void)hipHostFree(hb->pool);
        if (hb->rows) (void)hipHostFree(hb->rows);
    } else {
        free(hb->pool);
        free(hb->rows);
    }
    hb->pool = nullptr;
    hb->rows = nullptr;
    hb->pool_cap = hb->rows_cap = 0;
}

// (re)allocates hb's buffers for at least pool_bytes / n rows; pinned on GPU contexts
static int hb_reserve(gpudiff_ctx* c, gpudiff_hbatch* hb, uint64_t pool_bytes, size_t n) {
    if (hb->used) HIPCHK(hipEventSynchronize(hb->used));  // an in-flight H2D may still read it
    if (pool_bytes <= hb->pool_cap && n <= hb->rows_cap && hb->pool) return GPUDIFF_OK;
    hb_release_buffers(hb);
    size_t pool_alloc = (size_t)std::max<uint64_t>((pool_bytes + 63) & ~63ull, 64);
    size_t rows_alloc = std::max<size_t>(n, 1) * sizeof(gpudiff_pair_row);
    if (c->has_device) {
        HIPCHK(hipSetDevice(c->device));
        if (hipHostMalloc((void**)&hb->pool, pool_alloc, hipHostMallocDefault) != hipSuccess ||
            hipHostMalloc((void**)&hb->rows, rows_alloc, hipHostMallocDefault) != hipSuccess) {
            hb_release_buffers(hb);
            return GPUDIFF_E_NOMEM;
        }
        hb->pinned = true;
        if (!hb->used) HIPCHK(hipEventCreateWithFlags(&hb->used, hipEventDisableTiming));
    } else {
        hb->pool = (uint8_t*)aligned_alloc(64, pool_alloc);
        hb->rows = (gpudiff_pair_row*)aligned_alloc(64, (rows_alloc + 63) & ~(size_t)63);
        if (!hb->pool || !hb->rows) {
            hb_release_buffers(hb);
            return GPUDIFF_E_NOMEM;
        }
        hb->pinned = false;
    }
    hb->pool_cap = pool_alloc;
    hb->rows_cap = std::max<size_t>(n, 1);
    return GPUDIFF_OK;
}

int gpudiff_hbatch_create(gpudiff_ctx* c, uint64_t pool_bytes, size_t n, uint64_t total_leaves, gpudiff_hbatch** out,
                          uint8_t** pool, gpudiff_pair_row** rows) {
    if (!c || !out || !pool || !rows || (pool_bytes & 15)) return GPUDIFF_E_INVAL;
    *out = nullptr;
    std::unique_ptr<gpudiff_hbatch> hb(new (std::nothrow) gpudiff_hbatch());
    if (!hb) return GPUDIFF_E_NOMEM;
    int rc = hb_reserve(c, hb.get(), pool_bytes, n);
    if (rc) return rc;
    hb->n = n;
    hb->pool_bytes = pool_bytes;
    hb->leaves = total_leaves;
    *pool = hb->pool;
    *rows = hb->rows;
    *out = hb.release();
    return GPUDIFF_OK;
}

int gpudiff_hbatch_resize(gpudiff_ctx* c, gpudiff_hbatch* hb, uint64_t pool_bytes, size_t n, uint64_t total_leaves,
                          uint8_t** pool, gpudiff_pair_row** rows) {
    if (!c || !hb || !pool || !rows || (pool_bytes & 15)) return GPUDIFF_E_INVAL;
    int rc = hb_reserve(c, hb, pool_bytes, n);
    if (rc) return rc;
    hb->n = n;
    hb->pool_bytes = pool_bytes;
    hb->leaves = total_leaves;
    hb->errors = hb->reseeded = 0;
    *pool = hb->pool;
    *rows = hb->rows;
    return GPUDIFF_OK;
}

int gpudiff_hbatch_info_get(const gpudiff_hbatch* hb, gpudiff_hbatch_info* info) {
    if (!hb || !info) return GPUDIFF_E_INVAL;
    info->n_pairs = hb->n;
    info->rows = hb->rows;
    info->pool = hb->pool;
    info->pool_bytes = hb->pool_bytes;
    info->total_leaves = hb->leaves;
    info->n_decode_errors = hb->errors;
    info->n_reseeded = hb->reseeded;
    return GPUDIFF_OK;
}

void gpudiff_hbatch_free(gpudiff_ctx* c, gpudiff_hbatch* hb) {
    if (!hb) return;
    if (c && c->has_device) (void)hipSetDevice(c->device);
    if (hb->used) {
        (void)hipEventSynchronize(hb->used);
        (void)hipEventDestroy(hb->used);
    }
    hb_release_buffers(hb);
    delete hb;
}

// ------------------------------------------------------------------ device batches
static int alloc_outputs(gpudiff_dbatch* d);

int gpudiff_dbatch_create(gpudiff_ctx* c, uint64_t pool_bytes, uint64_t max_pairs, gpudiff_dbatch** out) {
    if (!c || !out) return GPUDIFF_E_INVAL;
    *out = nullptr;
    int rc = set_device(c);
    if (rc) return rc;
    if (max_pairs > 0xFFFFFFF0ull) return GPUDIFF_E_INVAL;
    std::unique_ptr<gpudiff_dbatch> d(new (std::nothrow) gpudiff_dbatch());
    if (!d) return GPUDIFF_E_NOMEM;
    d->pool_cap = (pool_bytes + 15) & ~15ull;
    d->max_pairs = max_pairs;
    d->device = c->device;
    const uint64_t np = std::max<uint64_t>(max_pairs, 1);
    if ((rc = dalloc(&d->pool, d->pool_cap)) || (rc = dalloc(&d->rows, np)) || (rc = dalloc(&d->pair_ids, np)) ||
        (rc = alloc_outputs(d.get()))) {
        dfree_all(d.get());
        return rc;
    }
    *out = d.release();
    return GPUDIFF_OK;
}

int gpudiff_dbatch_create_view(gpudiff_ctx* c, const gpudiff_dbatch* base, gpudiff_dbatch** out) {
    if (!c || !base || !out || base->base) return GPUDIFF_E_INVAL;
    *out = nullptr;
    int rc = set_device(c);
    if (rc) return rc;
    if (base->device != c->device) return GPUDIFF_E_INVAL;
    std::unique_ptr<gpudiff_dbatch> d(new (std::nothrow) gpudiff_dbatch());
    if (!d) return GPUDIFF_E_NOMEM;
    d->base = base;
    d->pool_borrowed = true;
    d->max_pairs = base->max_pairs;
    d->device = c->device;
    if ((rc = alloc_outputs(d.get()))) {
        dfree_all(d.get());
        return rc;
    }
    base->views.push_back(d.get());
    *out = d.release();
    return GPUDIFF_OK;
}

// a view sees its base's resident pairs as of this call (appends made since are ordered by the caller:
// they run on the base's context stream)
static void view_sync(gpudiff_dbatch* d) {
    if (!d->base) return;
    const gpudiff_dbatch* b = d->base;
    d->pool = b->pool;
    d->pool_cap = b->pool_cap;
    d->pool_used = b->pool_used;
    d->rows = b->rows;
    d->pair_ids = b->pair_ids;
    d->n_pairs = b->n_pairs;
    d->leaves = b->leaves;
    d->compare_bytes = b->compare_bytes;
    d->value_bytes = b->value_bytes;
    d->size_hint_bytes = b->size_hint_bytes;
    d->rows_gen = b->rows_gen;
}

// every per-pass output of a batch (a view has only these)
static int alloc_outputs(gpudiff_dbatch* d) {
    int rc;
    const uint64_t np = std::max<uint64_t>(d->max_pairs, 1);
    const uint64_t nchunks = (np + 63) / 64;
    const uint64_t ntiles = 4 * (np / 4096 + 2);  // scan tile sums (4 x u32 for the chunk scan)
    uint4* cc = nullptr;
    if ((rc = dalloc(&d->flags, np)) || (rc = dalloc(&d->caps, np)) || (rc = dalloc(&cc, nchunks)) ||
        (rc = dalloc(&d->summary, kSummaryWords)) || (rc = dalloc(&d->spec_ids, np)) || (rc = dalloc(&d->status_ids, np)) ||
        (rc = dalloc(&d->dirty_ids, np)) || (rc = dalloc(&d->dirty_idx, np)) || (rc = dalloc(&d->scratch_off, np)) ||
        (rc = dalloc(&d->path_count, np)) || (rc = dalloc(&d->path_off, np + 1)) ||
        (rc = dalloc(&d->path_src, np)) || (rc = dalloc(&d->path_cnt, np)) || (rc = dalloc(&d->nbits, np)) ||
        (rc = dalloc(&d->noop_d, np)) ||
        (rc = dalloc(&d->tile_sums, ntiles)) ||
        (rc = dalloc(&d->tail_perm, 16384))) {
        d->chunk_counts = cc;
        return rc;
    }
    d->chunk_counts = cc;
    if (hipEventCreateWithFlags(&d->done, hipEventDisableTiming) != hipSuccess) return GPUDIFF_E_DEVICE;
    return GPUDIFF_OK;
}

int gpudiff_dbatch_append(gpudiff_ctx* c, gpudiff_dbatch* d, const gpudiff_hbatch* hb) {
    if (!c || !d || !hb || d->base) return GPUDIFF_E_INVAL;
    int rc = set_device(c);
    if (rc) return rc;
    if (d->pool_used + hb->pool_bytes > d->pool_cap || d->n_pairs + hb->n > d->max_pairs) return GPUDIFF_E_CAPACITY;
    if (hb->n == 0) return GPUDIFF_OK;
    const uint64_t base = d->pool_used;
    const uint32_t begin = (uint32_t)d->n_pairs, end = (uint32_t)(d->n_pairs + hb->n);
    if (hb->pool_bytes)
        HIPCHK(hipMemcpyAsync(d->pool + base, hb->pool, hb->pool_bytes, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(d->rows + begin, hb->rows, hb->n * sizeof(gpudiff_pair_row), hipMemcpyHostToDevice,
                          c->stream));
    if (hb->used) HIPCHK(hipEventRecord(hb->used, c->stream));
    HIPCHK(launch_rebase(c->stream, d->rows, begin, end, base, d->pair_ids));
    uint64_t cb = 0, vb = 0;
    for (size_t i = 0; i < hb->n; i++) {
        const gpudiff_pair_row& r = hb->rows[i];
        cb += pair_compare_bytes(r);
        if ((r.flags_a | r.flags_b) & GPUDIFF_OBJ_DECODE_ERR) continue;
        vb += blob_value_bytes(hb->pool + r.off_a, r.spec_l_a, r.spec_ar_a, r.stat_l_a) +
              blob_value_bytes(hb->pool + r.off_b, r.spec_l_b, r.spec_ar_b, r.stat_l_b);
    }
    d->compare_bytes += cb;
    d->value_bytes += vb;
    d->pool_used += hb->pool_bytes;
    d->n_pairs = end;
    d->rows_gen++;
    d->leaves += hb->leaves;
    return GPUDIFF_OK;
}

int gpudiff_dbatch_reset(gpudiff_ctx* c, gpudiff_dbatch* d) {
    if (!c || !d || d->base) return GPUDIFF_E_INVAL;
    int rc = set_device(c);
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(c->stream));
    d->pool_used = d->n_pairs = d->leaves = d->compare_bytes = d->value_bytes = d->size_hint_bytes = 0;
    d->ticket = 0;
    d->rows_gen++;
    return GPUDIFF_OK;
}

int gpudiff_dbatch_stats_get(const gpudiff_dbatch* d, gpudiff_batch_stats* st) {
    if (!d || !st) return GPUDIFF_E_INVAL;
    if (d->base) d = d->base;
    st->n_pairs = d->n_pairs;
    st->pool_bytes = d->pool_used;
    st->total_leaves = d->leaves;
    st->compare_bytes = d->compare_bytes;
    st->value_bytes = d->value_bytes;
    return GPUDIFF_OK;
}

int gpudiff_dbatch_device_view(const gpudiff_dbatch* d, gpudiff_device_view* v) {
    if (!d || !v) return GPUDIFF_E_INVAL;
    v->pair_flags = d->flags;
    v->spec_dirty_ids = d->spec_ids;
    v->status_dirty_ids = d->status_ids;
    v->dirty_ids = d->dirty_ids;
    v->counts = d->summary;
    return GPUDIFF_OK;
}

int gpudiff_dbatch_export(gpudiff_ctx* c, const gpudiff_dbatch* d, uint32_t what, void* dst, uint64_t max_elems,
                          uint64_t known_count) {
    if (!c || !d || (!dst && max_elems)) return GPUDIFF_E_INVAL;
    int rc = set_device(c);
    if (rc) return rc;
    const void* src;
    size_t esz = 4;
    uint64_t n = std::min<uint64_t>(max_elems, known_count);
    switch (what) {
        case GPUDIFF_EXPORT_COUNTS: src = d->summary; n = std::min<uint64_t>(max_elems, 8); break;
        case GPUDIFF_EXPORT_SPEC_IDS: src = d->spec_ids; break;
        case GPUDIFF_EXPORT_STATUS_IDS: src = d->status_ids; break;
        case GPUDIFF_EXPORT_DIRTY_IDS: src = d->dirty_ids; break;
        case GPUDIFF_EXPORT_FLAGS: src = d->flags; esz = 1; break;
        default: return GPUDIFF_E_INVAL;
    }
    if (what != GPUDIFF_EXPORT_COUNTS && n > d->n_pairs) n = d->n_pairs;
    if (n) HIPCHK(hipMemcpyAsync(dst, src, n * esz, hipMemcpyDeviceToDevice, c->stream));
    return GPUDIFF_OK;
}

int gpudiff_dbatch_bind_gather(gpudiff_ctx* c, gpudiff_dbatch* d, void* send_dev, uint32_t cap_spec,
                               uint32_t cap_status) {
    if (!c || !d) return GPUDIFF_E_INVAL;
    int rc = set_device(c);
    if (rc) return rc;
    const bool fresh = send_dev && send_dev != (void*)d->gather_send;
    d->gather_send = (uint32_t*)send_dev;
    d->gather_cap_spec = send_dev ? cap_spec : 0;
    d->gather_cap_status = send_dev ? cap_status : 0;
    // a rebinding of the same buffer (every step of a per-step collective) costs nothing on the stream
    if (fresh) HIPCHK(hipMemsetAsync((uint32_t*)send_dev + 4, 0, 4 * sizeof(uint32_t), c->stream));
    return GPUDIFF_OK;
}

int gpudiff_dbatch_result_slot(gpudiff_ctx* c, gpudiff_dbatch* d, uint32_t slot) {
    if (!c || !d || slot > 1) return GPUDIFF_E_INVAL;
    int rc = set_device(c);
    if (rc) return rc;
    if (slot == d->res_slot) return GPUDIFF_OK;
    if (!d->summary_alt) {  // all three buffers or none (a half-allocated slot would swap in a null list)
        const uint64_t np = std::max<uint64_t>(d->max_pairs, 1);
        uint32_t *a = nullptr, *b = nullptr, *sm = nullptr;
        if ((rc = dalloc(&a, np)) || (rc = dalloc(&b, np)) || (rc = dalloc(&sm, kSummaryWords))) {
            for (uint32_t* p : {a, b, sm})
                if (p) (void)hipFree(p);
            return rc;
        }
        if (hipMemset(sm, 0, kSummaryWords * sizeof(uint32_t)) != hipSuccess) {
            for (uint32_t* p : {a, b, sm}) (void)hipFree(p);
            return GPUDIFF_E_DEVICE;
        }
        d->ids_alt[0] = a, d->ids_alt[1] = b, d->summary_alt = sm;
    }
    // the counts are per slot too: a lookahead regrow re-exports step s's counts after step s + 1 ran
    // (one shared summary paired step s + 1's counts with step s's lists)
    std::swap(d->spec_ids, d->ids_alt[0]);
    std::swap(d->status_ids, d->ids_alt[1]);
    std::swap(d->summary, d->summary_alt);
    d->res_slot = slot;
    return GPUDIFF_OK;
}

int gpudiff_dbatch_read_pool(gpudiff_ctx* c, const gpudiff_dbatch* d, uint64_t off, void* dst, uint64_t bytes) {
    if (!c || !d || (!dst && bytes)) return GPUDIFF_E_INVAL;
    if (d->base) d = d->base;
    int rc = set_device(c);
    if (rc) return rc;
    if (off > d->pool_used || bytes > d->pool_used - off) return GPUDIFF_E_INVAL;
    HIPCHK(hipStreamSynchronize(c->stream));
    if (bytes) HIPCHK(hipMemcpy(dst, d->pool + off, bytes, hipMemcpyDeviceToHost));
    return GPUDIFF_OK;
}

// ------------------------------------------------------------------ sharding
int gpudiff_cluster_bytes(const gpudiff_pair_row* rows, size_t n, uint32_t n_clusters, uint64_t* out) {
    if ((n && !rows) || (n_clusters && !out)) return GPUDIFF_E_INVAL;
    for (size_t i = 0; i < n; i++)
        if (rows[i].cluster_id >= n_clusters) return GPUDIFF_E_INVAL;
    for (size_t i = 0; i < n; i++) out[rows[i].cluster_id] += gpudiff_pair_compare_bytes(&rows[i]);
    return GPUDIFF_OK;
}

int gpudiff_shard_lpt(const uint64_t* weights, uint32_t n_clusters, uint32_t world, int32_t* owner) {
    if (world == 0 || world > 0x7FFFFFFFu || (n_clusters && (!weights || !owner))) return GPUDIFF_E_INVAL;
    try {
        std::vector<uint32_t> order(n_clusters);
        for (uint32_t c = 0; c < n_clusters; c++) order[c] = c;
        std::sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) {
            return weights[x] != weights[y] ? weights[x] > weights[y] : x < y;
        });
        // least-loaded rank first, ties to the lower rank: a min-heap of (load, rank)
        std::vector<std::pair<uint64_t, uint32_t>> heap;
        heap.reserve(world);
        for (uint32_t r = 0; r < world; r++) heap.emplace_back(0, r);
        auto gt = [](const std::pair<uint64_t, uint32_t>& a, const std::pair<uint64_t, uint32_t>& b) { return a > b; };
        std::make_heap(heap.begin(), heap.end(), gt);
        for (uint32_t c : order) {
            std::pop_heap(heap.begin(), heap.end(), gt);
            auto& top = heap.back();
            owner[c] = (int32_t)top.second;
            top.first += weights[c];
            std::push_heap(heap.begin(), heap.end(), gt);
        }
    } catch (const std::bad_alloc&) {
        return GPUDIFF_E_NOMEM;
    }
    return GPUDIFF_OK;
}

void gpudiff_dbatch_free(gpudiff_ctx* c, gpudiff_dbatch* d) {
    if (!d) return;
    if (d->base) {
        auto& v = d->base->views;
        v.erase(std::remove(v.begin(), v.end(), d), v.end());
    }
    if (c && c->has_device) {
        (void)hipSetDevice(c->device);
        (void)hipStreamSynchronize(c->stream);
        if (d->ticket) c->tickets.erase(d->ticket);
    }
    dfree_all(d);
    delete d;
}

// ------------------------------------------------------------------ diff
// Timing: one set of 5 events per recorded pass ([0] before K2, [1] after K2,
// [2] after K3, [3] after K4, [4] after K5/K6); gpudiff_last_timings averages
// every pass recorded since gpudiff_timing_reset.
static hipEvent_t* pass_events(gpudiff_ctx* c) {
    if (c->n_pass >= c->pass_ev.size()) {
        std::array<hipEvent_t, 5> a{};
        for (auto& e : a)
            if (hipEventCreate(&e) != hipSuccess) return nullptr;
        c->pass_ev.push_back(a);
    }
    return c->pass_ev[c->n_pass].data();
}

// K4 over every dirty pair + K5/K6 on the main stream (overflow re-run)
static int enqueue_join_emit(gpudiff_ctx* c, gpudiff_dbatch* d) {
    DiffBuffers b = buffers_of(c, d);
    const uint32_t nchunks = (uint32_t)((d->n_pairs + 63) / 64);
    HIPCHK(launch_slot_owners(c->stream, b));
    HIPCHK(launch_join(c->stream, b, 0, nchunks, nullptr, (const uint4*)d->summary));
    HIPCHK(launch_emit(c->stream, b));
    return GPUDIFF_OK;
}

int gpudiff_diff(gpudiff_ctx* c, gpudiff_dbatch* d, gpudiff_ticket* ticket) {
    if (!c || !d) return GPUDIFF_E_INVAL;
    int rc = set_device(c);
    if (rc) return rc;
    if (d->base && d->base->device != c->device) return GPUDIFF_E_INVAL;
    view_sync(d);
    // scratch for changed paths: sized from the batch, grown on overflow
    {
        const uint32_t nch = (uint32_t)((d->n_pairs + 63) / 64);
        DiffBuffers b0 = buffers_of(c, d);
        const uint64_t arena = (uint64_t)k2_grid_waves(b0, std::max(nch, 1u)) * kArenaPerWave;
        if ((rc = ensure_paths(d, arena, std::max<uint64_t>(d->n_pairs / 64, 1u << 16)))) return rc;
    }
    hipEvent_t* ev = nullptr;
    if ((c->flags & GPUDIFF_OPT_TIMING) && d->n_pairs) {
        ev = pass_events(c);
        if (!ev) return GPUDIFF_E_DEVICE;
    }
    hipStream_t ms = c->stream;
    DiffBuffers b = buffers_of(c, d);
    // Two passes in flight (a view and its base diffed by two contexts): while another pass over the population is
    // still running, this pass's K2 launches half its resident grid.  A full-occupancy K2 grid holds every CU slot
    // until its drain, so the other pass's K2 could not start before this one ended -- the two passes ran back to
    // back (rocprofv3 trace, profiles/r06z); with half grids both stream at once and each fills the other's drain.
    // An isolated pass (the other one done) launches the full grid, and so does a large pass, whose drain is a
    // small part of it: two-in-flight step -5% on config2 (1M pairs, 5.2 GB a pass) and -4.5% on the N = 8 share of
    // config3 (1.25M pairs, 6.4 GB), +1% on config3 at 10M (51 GB) -- profiles/r06aa.
    constexpr uint64_t kHalfGridMaxBytes = 16ull << 30;
    if (d->compare_bytes && d->compare_bytes <= kHalfGridMaxBytes) {
        const gpudiff_dbatch* fam = d->base ? d->base : d;
        auto busy = [&](const gpudiff_dbatch* m) {
            return m != d && m->done && m->ticket && hipEventQuery(m->done) == hipErrorNotReady;
        };
        bool shared = busy(fam);
        for (const gpudiff_dbatch* v : fam->views) shared = shared || busy(v);
        b.k2_shared = shared ? 1u : 0u;
    }
    uint4* total = (uint4*)d->summary;  // summary[0..3]: n_spec, n_status, n_dirty, scratch cap
    if (ev) HIPCHK(hipEventRecord(ev[0], ms));
    if (d->n_pairs == 0) {
        HIPCHK(hipMemsetAsync(d->summary, 0, kSummaryWords * sizeof(uint32_t), ms));
        HIPCHK(hipMemsetAsync(d->path_off, 0, sizeof(uint32_t), ms));
    } else {
        const uint32_t nchunks = (uint32_t)((d->n_pairs + 63) / 64);
        HIPCHK(launch_compare(ms, b));  // zeroes the summary (+ K2's item counters) first
        if (ev) HIPCHK(hipEventRecord(ev[1], ms));
        HIPCHK(launch_compact(ms, b, 0, nchunks, nullptr, total));
        if (ev) HIPCHK(hipEventRecord(ev[2], ms));
        HIPCHK(launch_join(ms, b, 0, nchunks, nullptr, total));
        if (ev) HIPCHK(hipEventRecord(ev[3], ms));
        HIPCHK(launch_emit(ms, b));
        if (ev) HIPCHK(hipEventRecord(ev[4], ms));
    }
    if (ev) c->n_pass++;
    HIPCHK(hipEventRecord(d->done, c->stream));
    if (d->ticket) c->tickets.erase(d->ticket);
    d->ticket = c->next_ticket++;
    c->tickets[d->ticket] = d;
    if (ticket) *ticket = d->ticket;
    return GPUDIFF_OK;
}

int gpudiff_sync(gpudiff_ctx* c) {
    if (!c) return GPUDIFF_E_INVAL;
    int rc = set_device(c);
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(c->stream));
    return GPUDIFF_OK;
}

int gpudiff_timing_reset(gpudiff_ctx* c) {
    if (!c) return GPUDIFF_E_INVAL;
    int rc = set_device(c);
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(c->stream));
    c->n_pass = 0;
    if (c->pair_store) dstore_timing_reset(c->pair_store);
    return GPUDIFF_OK;
}

int gpudiff_last_timings(gpudiff_ctx* c, gpudiff_timings* t) {
    if (!c || !t) return GPUDIFF_E_INVAL;
    memset(t, 0, sizeof(*t));
    if (!c->has_device) return GPUDIFF_E_NODEVICE;
    if (!(c->flags & GPUDIFF_OPT_TIMING)) return GPUDIFF_E_STATE;
    HIPCHK(hipStreamSynchronize(c->stream));
    t->n_passes = (uint32_t)c->n_pass;
    t->k2_launches = 1;
    if (!c->n_pass) return GPUDIFF_OK;
    double s[5] = {0, 0, 0, 0, 0};
    for (size_t i = 0; i < c->n_pass; i++) {
        hipEvent_t* e = c->pass_ev[i].data();
        float x;
        HIPCHK(hipEventElapsedTime(&x, e[0], e[1])); s[0] += x;
        HIPCHK(hipEventElapsedTime(&x, e[1], e[2])); s[1] += x;
        HIPCHK(hipEventElapsedTime(&x, e[2], e[3])); s[2] += x;
        HIPCHK(hipEventElapsedTime(&x, e[3], e[4])); s[3] += x;
        HIPCHK(hipEventElapsedTime(&x, e[0], e[4])); s[4] += x;
    }
    const double n = (double)c->n_pass;
    t->compare_ms = (float)(s[0] / n);
    t->compact_ms = (float)(s[1] / n);
    t->join_ms = (float)(s[2] / n);
    t->emit_ms = (float)(s[3] / n);
    t->total_ms = (float)(s[4] / n);
    return GPUDIFF_OK;
}

int gpudiff_wait(gpudiff_ctx* c, gpudiff_ticket ticket, gpudiff_result* res) {
    if (!c || !res) return GPUDIFF_E_INVAL;
    memset(res, 0, sizeof(*res));
    int rc = set_device(c);
    if (rc) return rc;
    auto it = c->tickets.find(ticket);
    if (it == c->tickets.end()) return GPUDIFF_E_STATE;
    gpudiff_dbatch* d = it->second;
    std::unique_ptr<ResultStore> rs(new (std::nothrow) ResultStore());
    if (!rs) return GPUDIFF_E_NOMEM;
    if ((rc = collect_results(c, d, *rs))) return rc;
    auto fin = c->finishers.find(ticket);
    if (fin != c->finishers.end()) {
        auto fn = std::move(fin->second);
        c->finishers.erase(fin);
        if ((rc = fn(*rs))) return rc;
    }
    res->n_pairs = rs->flags.size();
    res->pair_flags = rs->flags.data();
    res->n_spec_dirty = rs->spec.size();
    res->spec_dirty_ids = rs->spec.data();
    res->n_status_dirty = rs->status.size();
    res->status_dirty_ids = rs->status.data();
    res->n_dirty = rs->dirty.size();
    res->dirty_ids = rs->dirty.data();
    res->path_offsets = rs->off.data();
    res->n_paths = rs->hashes.size();
    res->path_hashes = rs->hashes.data();
    res->path_kinds = rs->kinds.data();
    res->internal_ = rs.release();
    return GPUDIFF_OK;
}

}  // extern "C"

int collect_results(gpudiff_ctx* c, gpudiff_dbatch* d, ResultStore& rsr) {
    ResultStore* rs = &rsr;
    int rc;
    HIPCHK(hipEventSynchronize(d->done));
    // read back on the context's readback stream: a synchronous hipMemcpy would also wait for the
    // work queued behind this batch (the next batch's K0 / diff pass), serialising the pipeline
    hipStream_t rb = c->rb;
    uint32_t sum[8];
    HIPCHK(hipMemcpyAsync(sum, d->summary, sizeof(sum), hipMemcpyDeviceToHost, rb));
    HIPCHK(hipStreamSynchronize(rb));
    if (sum[4]) {  // path scratch overflow: grow to the exact need and redo the join
        if ((rc = ensure_paths(d, d->arena_cap, sum[3]))) return rc;
        uint32_t zero = 0;
        HIPCHK(hipMemcpyAsync(d->summary + 4, &zero, sizeof(zero), hipMemcpyHostToDevice, c->stream));
        if ((rc = enqueue_join_emit(c, d))) return rc;
        HIPCHK(hipStreamSynchronize(c->stream));
        HIPCHK(hipMemcpyAsync(sum, d->summary, sizeof(sum), hipMemcpyDeviceToHost, rb));
        HIPCHK(hipStreamSynchronize(rb));
        if (sum[4]) return GPUDIFF_E_CAPACITY;
    }
    std::vector<uint32_t> idx;
    std::vector<uint8_t> nb;
    try {
        rs->flags.resize(d->n_pairs);
        rs->spec.resize(sum[0]);
        rs->status.resize(sum[1]);
        rs->dirty.resize(sum[2]);
        rs->off.resize((size_t)sum[2] + 1);
        rs->hashes.resize(sum[5]);
        rs->kinds.resize(sum[5]);
        idx.resize(sum[2]);
        nb.resize(sum[2]);
    } catch (const std::bad_alloc&) {
        return GPUDIFF_E_NOMEM;
    }
    auto d2h = [&](void* dst, const void* src, uint64_t bytes) -> hipError_t {
        return bytes ? hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, rb) : hipSuccess;
    };
    HIPCHK(d2h(rs->flags.data(), d->flags, d->n_pairs));
    HIPCHK(d2h(idx.data(), d->dirty_idx, sum[2] * 4ull));
    HIPCHK(d2h(nb.data(), d->noop_d, sum[2]));
    HIPCHK(d2h(rs->spec.data(), d->spec_ids, sum[0] * 4ull));
    HIPCHK(d2h(rs->status.data(), d->status_ids, sum[1] * 4ull));
    HIPCHK(d2h(rs->dirty.data(), d->dirty_ids, sum[2] * 4ull));
    HIPCHK(d2h(rs->off.data(), d->path_off, (sum[2] + 1ull) * 4ull));
    HIPCHK(d2h(rs->hashes.data(), d->out_h, sum[5] * 8ull));
    HIPCHK(d2h(rs->kinds.data(), d->out_k, sum[5]));
    HIPCHK(hipStreamSynchronize(rb));
    for (uint8_t& f : rs->flags) f &= (uint8_t)(GPUDIFF_SPEC_DIRTY | GPUDIFF_STATUS_DIRTY | GPUDIFF_DECODE_ERROR);
    for (uint32_t k = 0; k < sum[2]; k++) {  // the write-path no-op bits of the dirty pairs (K2 / K4 via K3)
        uint8_t& f = rs->flags[idx[k]];
        if (f & GPUDIFF_DECODE_ERROR) continue;
        if ((nb[k] & 1u) && (f & GPUDIFF_SPEC_DIRTY)) f |= GPUDIFF_SPEC_NOOP;
        if ((nb[k] & 2u) && (f & GPUDIFF_STATUS_DIRTY)) f |= GPUDIFF_STATUS_NOOP;
    }
    return GPUDIFF_OK;
}

extern "C" {

void gpudiff_result_release(gpudiff_ctx* c, gpudiff_result* res) {
    (void)c;
    if (!res) return;
    delete (ResultStore*)res->internal_;
    memset(res, 0, sizeof(*res));
}

int gpudiff_submit(gpudiff_ctx* c, const gpudiff_json_pair* pairs, size_t n, gpudiff_ticket* ticket) {
    if (!c || (n && !pairs)) return GPUDIFF_E_INVAL;
    int rc = set_device(c);
    if (rc) return rc;
    if ((c->flags & GPUDIFF_OPT_DEVICE_ENCODE) && n) {
        rc = dstore_submit_pairs(c, pairs, n, ticket);
        if (rc != GPUDIFF_E_CAPACITY) return rc;
    }
    gpudiff_hbatch* hb = nullptr;
    if ((rc = gpudiff_encode_pairs(c, pairs, n, &hb))) return rc;
    const uint32_t slot = c->ring_next;
    c->ring_next ^= 1u;
    gpudiff_dbatch*& d = c->ring[slot];
    if (d) HIPCHK(hipEventSynchronize(d->done));
    if (c->ring_hb[slot]) {
        gpudiff_hbatch_free(c, c->ring_hb[slot]);
        c->ring_hb[slot] = nullptr;
    }
    if (d && (d->pool_cap < hb->pool_bytes || d->max_pairs < n)) {
        gpudiff_dbatch_free(c, d);
        d = nullptr;
    }
    if (!d) {
        uint64_t pool = std::max<uint64_t>(hb->pool_bytes * 2, 1u << 20);
        uint64_t np = std::max<uint64_t>(n * 2, 1024);
        if ((rc = gpudiff_dbatch_create(c, pool, np, &d))) {
            gpudiff_hbatch_free(c, hb);
            return rc;
        }
    }
    d->pool_used = d->n_pairs = d->leaves = d->compare_bytes = d->value_bytes = d->size_hint_bytes = 0;
    if ((rc = gpudiff_dbatch_append(c, d, hb)) || (rc = gpudiff_diff(c, d, ticket))) {
        gpudiff_hbatch_free(c, hb);
        return rc;
    }
    c->ring_hb[slot] = hb;  // freed when the slot is reused (after its copy completed)
    return GPUDIFF_OK;
}

static int single_pair(gpudiff_ctx* c, const uint8_t* a, size_t al, const uint8_t* b, size_t bl, uint32_t bit,
                       int* equal) {
    if (!c || !equal || !a || !b) return GPUDIFF_E_INVAL;
    gpudiff_json_pair p{a, al, b, bl, 0, 0};
    gpudiff_ticket t = 0;
    int rc = gpudiff_submit(c, &p, 1, &t);
    if (rc) return rc;
    gpudiff_result r;
    if ((rc = gpudiff_wait(c, t, &r))) return rc;
    const uint8_t f = r.pair_flags[0];
    gpudiff_result_release(c, &r);
    *equal = (f & bit) ? 0 : 1;
    return (f & GPUDIFF_DECODE_ERROR) ? GPUDIFF_E_DECODE : GPUDIFF_OK;
}

int gpudiff_spec_equal(gpudiff_ctx* c, const uint8_t* a, size_t al, const uint8_t* b, size_t bl, int* equal) {
    return single_pair(c, a, al, b, bl, GPUDIFF_SPEC_DIRTY, equal);
}

int gpudiff_status_equal(gpudiff_ctx* c, const uint8_t* a, size_t al, const uint8_t* b, size_t bl, int* equal) {
    return single_pair(c, a, al, b, bl, GPUDIFF_STATUS_DIRTY, equal);
}

int gpudiff_resolve_path(const uint8_t* a, size_t al, const uint8_t* b, size_t bl, uint64_t h, uint8_t kind,
                         uint32_t bits, char* buf, size_t cap, size_t* out_len) {
    if (!a || !b) return GPUDIFF_E_INVAL;
    EncodeConfig cfg;
    cfg.hash_bits = (bits == 0 || bits >= GPUDIFF_PATH_HASH_BITS) ? GPUDIFF_PATH_HASH_BITS : bits;
    PairEncoder enc(cfg);
    std::vector<uint8_t> pool;
    gpudiff_pair_row row;
    enc.encode_json(a, al, b, bl, 0, 0, pool, row);
    if (row.flags_a & GPUDIFF_OBJ_DECODE_ERR) return GPUDIFF_E_DECODE;
    // encode_json left both flattened objects (with seed-assigned hashes) in place
    std::string s;
    bool found = false;
    const bool status = (kind & GPUDIFF_PATH_REGION_STATUS) != 0;
    if ((kind & 3u) != GPUDIFF_PATH_STATUS_ABSENT) {
        for (const FlatObject* o : {&enc.flat_a, &enc.flat_b}) {
            const std::vector<LeafRec>& v = status ? o->stat : o->spec;
            auto it = std::lower_bound(v.begin(), v.end(), h, [](const LeafRec& r, uint64_t x) { return r.h < x; });
            if (it != v.end() && it->h == h) {
                s = render_path(o->paths.data() + it->path_off, it->path_len);
                found = true;
                break;
            }
        }
    } else {
        const uint64_t mask = cfg.hash_bits >= 64 ? ~0ULL : ((1ULL << cfg.hash_bits) - 1);
        const uint32_t seed = (row.flags_a >> GPUDIFF_OBJ_SEED_SHIFT) & 0xFF;
        const std::string& sp = status_path_bytes();
        if ((chain_hash(sp.data(), sp.size(), seed) & mask) == h) {
            s = "status";
            found = true;
        }
    }
    if (!found) return GPUDIFF_E_NOTFOUND;
    if (out_len) *out_len = s.size();
    if (buf && cap) {
        size_t k = std::min(cap - 1, s.size());
        memcpy(buf, s.data(), k);
        buf[k] = 0;
    }
    return GPUDIFF_OK;
}

}  // extern "C"
