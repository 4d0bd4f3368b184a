// Device-resident object store (include/gpudiff.h "device-resident object
// store"): the informer cache's old objects stay in HBM, each Update event
// uploads only its new version, which is diffed against the slot's resident
// version and then replaces it.
//
// Host side per submit:
//   1. events are split by slot over the encode threads (slot % T), so the
//      events of one slot are encoded in order by one thread and chain;
//   2. each new object is parsed, flattened, hashed with the slot's seed and
//      its path table checked against the resident version's (exact: a hash
//      both hold must have the same parent hash and last component in each,
//      include/gpudiff_format.h); a disagreement is a collision and the pair is
//      re-encoded from old_json with a fresh seed (PairEncoder::pair_seed, the
//      same seed the batch path would pick when b's table allows it);
//   3. blobs go to per-thread parts with batch-local offsets; after the
//      threads join, the current space is compacted into the other one if
//      the batch does not fit (K7 k_move_blobs packs every live blob and every
//      blob this batch still reads), offsets are finalised, and one H2D copies
//      the batch's blobs behind the space's append point;
//   4. the ordinary diff pass (K2..K6, gpudiff_diff) runs over the batch's
//      (resident, new) rows.
#include <string.h>

#include <algorithm>
#include <memory>
#include <new>
#include <thread>
#include <unordered_map>
#include <vector>

#include "dstore.h"
#include "engine.h"
#include "xxh64.h"

using namespace gd;

namespace {

constexpr uint64_t kLocal = 1ull << 63;  // offset tag: batch-local (part << 48 | offset in part)
constexpr int kLocalPartShift = 48;

struct Slot {
    bool live = false;
    uint32_t seed = 0;
    uint64_t off = 0;  // absolute offset in the current space, or a kLocal tag
    uint32_t bytes = 0, spec_l = 0, spec_ar = 0, stat_l = 0, stat_ar = 0;
    uint32_t oflags = 0;   // GPUDIFF_OBJ_HAS_STATUS
    uint64_t epoch = 0;    // last batch that touched the slot
    PathTable tab;         // the resident version's path table (host RAM)
};

struct Blob {
    uint64_t off;
    uint32_t bytes, spec_l, spec_ar, stat_l, stat_ar, oflags;
    bool fresh;
};

struct Worker {
    std::unique_ptr<PairEncoder> enc;
    Arena arena_old, arena_new;
    FlatObject fo, fn;
    std::vector<uint8_t> pool;
    std::vector<uint32_t> touched;                         // slots set to batch-local offsets
    std::vector<std::pair<uint64_t, uint32_t>> pre;        // batch-start resident blobs of touched slots
    uint64_t old_encoded = 0, reseeded = 0, unresolved = 0, leaves = 0;
    int64_t live_delta = 0, bytes_delta = 0;  // resident slot count / bytes changes of this batch
};

inline uint64_t local_tag(uint32_t part, uint64_t off) { return kLocal | ((uint64_t)part << kLocalPartShift) | off; }

uint32_t blob_bytes(uint32_t sl, uint32_t sar, uint32_t tl, uint32_t tar) {
    return (uint32_t)gpudiff_blob_body(sl, sar, tl, tar);
}

}  // namespace

struct gpudiff_store {
    DStore* dev = nullptr;  // device-encode mode (dstore.cpp)
    uint32_t max_slots = 0, max_events = 0;
    uint64_t space_bytes = 0;
    uint8_t* space[2] = {nullptr, nullptr};
    uint32_t cur = 0;
    uint64_t used = 0;  // append point in space[cur]
    std::vector<Slot> slots;
    uint64_t epoch = 0;
    bool broken = false;
    std::vector<std::unique_ptr<Worker>> workers;
    gpudiff_dbatch* ring[2] = {nullptr, nullptr};
    gpudiff_hbatch* staging[2] = {nullptr, nullptr};
    uint32_t ring_next = 0;
    BlobMove* moves_dev = nullptr;
    uint64_t moves_cap = 0;
    gpudiff_store_stats st{};
};

static int store_grow_moves(gpudiff_store* s, uint64_t n) {
    if (n <= s->moves_cap) return GPUDIFF_OK;
    if (s->moves_dev) (void)hipFree(s->moves_dev);
    s->moves_dev = nullptr;
    s->moves_cap = 0;
    int rc = dalloc(&s->moves_dev, n + n / 4);
    if (rc) return rc;
    s->moves_cap = n + n / 4;
    return GPUDIFF_OK;
}

// Packs every live resident blob plus the batch-start blobs this batch still
// reads into the other space; remaps their offsets (rows + slots).
static int store_compact(gpudiff_ctx* c, gpudiff_store* s, std::vector<gpudiff_pair_row>& rows) {
    std::vector<BlobMove> mv;
    std::unordered_map<uint64_t, uint64_t> remap;
    uint64_t dst = 0;
    auto add = [&](uint64_t off, uint32_t bytes) -> uint64_t {
        auto it = remap.find(off);
        if (it != remap.end()) return it->second;
        const uint64_t d = dst;
        if (bytes) mv.push_back(BlobMove{off, d, bytes});
        dst += bytes;
        remap.emplace(off, d);
        return d;
    };
    for (Slot& sl : s->slots)
        if (sl.live && !(sl.off & kLocal)) sl.off = add(sl.off, sl.bytes);
    for (auto& w : s->workers)
        for (auto& p : w->pre) add(p.first, p.second);
    for (gpudiff_pair_row& r : rows)
        if (!(r.off_a & kLocal)) {
            auto it = remap.find(r.off_a);
            r.off_a = it != remap.end() ? it->second : 0;  // 0-byte blobs (empty object, decode errors)
        }
    int rc = store_grow_moves(s, std::max<uint64_t>(mv.size(), 1));
    if (rc) return rc;
    if (!mv.empty()) {
        HIPCHK(hipMemcpyAsync(s->moves_dev, mv.data(), mv.size() * sizeof(BlobMove), hipMemcpyHostToDevice,
                              c->stream));
        HIPCHK(launch_move_blobs(c->stream, s->space[s->cur], s->space[1 - s->cur], s->moves_dev,
                                 (uint32_t)mv.size()));
        HIPCHK(hipStreamSynchronize(c->stream));  // mv is pageable host memory
    }
    s->cur = 1 - s->cur;
    s->used = dst;
    s->st.compactions++;
    return GPUDIFF_OK;
}

// Encodes the events whose slot % T == t, in batch order.
static void store_encode_part(gpudiff_ctx* c, gpudiff_store* s, const gpudiff_event* ev, size_t n, uint32_t t,
                              uint32_t T, gpudiff_pair_row* rows) {
    Worker& w = *s->workers[t];
    PairEncoder& enc = *w.enc;
    const uint64_t epoch = s->epoch;
    for (size_t i = 0; i < n; i++) {
        const gpudiff_event& e = ev[i];
        if (e.slot % T != t) continue;
        Slot& S = s->slots[e.slot];
        if (S.epoch != epoch) {  // first touch in this batch: its resident blob may be read, keep it
            S.epoch = epoch;
            if (S.live && !(S.off & kLocal)) w.pre.emplace_back(S.off, S.bytes);
        }
        if (S.live) {  // its contribution is re-added below if it stays resident
            w.live_delta--;
            w.bytes_delta -= S.bytes;
        }
        gpudiff_pair_row& r = rows[i];
        memset(&r, 0, sizeof(r));
        r.pair_id = e.pair_id;
        r.cluster_id = e.cluster_id;
        auto conservative = [&]() {  // reported dirty in both regions, no paths (specsyncer.go:20-22)
            r.flags_a = r.flags_b = GPUDIFF_OBJ_DECODE_ERR;
            r.off_a = r.off_b = 0;
        };
        if (!enc.flatten_json(e.new_json, e.new_len, w.arena_new, w.fn)) {
            conservative();
            S.live = false;
            S.tab.clear();
            continue;
        }
        Blob A{0, 0, 0, 0, 0, 0, 0, false};
        uint32_t seed = 0;
        bool ok = false, pair_error = false;
        if (S.live && S.seed == 0 && enc.hash_single(w.fn, 0) && tab_agree(tab_view(S.tab), tab_view(w.fn.tab))) {
            ok = true;  // the common case: the resident version is the old side as it stands
            A = Blob{S.off, S.bytes, S.spec_l, S.spec_ar, S.stat_l, S.stat_ar, S.oflags, false};
        } else if (e.old_json) {
            // first sighting, a re-seeded slot, or a collision: encode the pair from old_json
            if (enc.flatten_json(e.old_json, e.old_len, w.arena_old, w.fo) && enc.pair_seed(w.fo, w.fn, &seed)) {
                uint64_t off;
                A.fresh = true;
                enc.write_object(w.fo, w.pool, &off, &A.spec_l, &A.spec_ar, &A.stat_l, &A.stat_ar);
                A.off = local_tag(t, off);
                A.bytes = blob_bytes(A.spec_l, A.spec_ar, A.stat_l, A.stat_ar);
                A.oflags = w.fo.flags;
                w.leaves += w.fo.spec.size() + w.fo.stat.size();
                w.old_encoded++;
                if (S.live) w.reseeded++;
                ok = true;
            } else {
                pair_error = true;  // undecodable old object or no valid seed: as gpudiff_encode_pairs
            }
        } else if (S.live && S.seed && enc.hash_single(w.fn, S.seed) &&
                   tab_agree(tab_view(S.tab), tab_view(w.fn.tab))) {
            ok = true;  // slot re-seeded earlier and no old object to re-encode: keep its seed
            seed = S.seed;
            A = Blob{S.off, S.bytes, S.spec_l, S.spec_ar, S.stat_l, S.stat_ar, S.oflags, false};
        } else if (!S.live) {
            // first sighting without an old object: diff against the empty object {}
            ok = enc.first_seed(w.fn, &seed);
            pair_error = !ok;
        } else {
            pair_error = true;
            w.unresolved++;
        }
        // store the new version (self-consistent seed if the pair failed)
        if (pair_error) {
            conservative();
            if (!enc.store_seed(w.fn, &seed)) {
                S.live = false;
                S.tab.clear();
                continue;
            }
        }
        uint64_t off;
        uint32_t sl, sar, tl, tar;
        enc.write_object(w.fn, w.pool, &off, &sl, &sar, &tl, &tar);
        w.leaves += w.fn.spec.size() + w.fn.stat.size();
        if (!pair_error) {
            r.off_a = A.bytes ? A.off : local_tag(t, off);  // a 0-byte blob is never read
            r.spec_l_a = A.spec_l;
            r.spec_ar_a = A.spec_ar;
            r.stat_l_a = A.stat_l;
            r.stat_ar_a = A.stat_ar;
            r.flags_a = A.oflags | (seed << GPUDIFF_OBJ_SEED_SHIFT) | (A.fresh ? GPUDIFF_OBJ_FRESH : 0u);
            r.off_b = local_tag(t, off);
            r.spec_l_b = sl;
            r.spec_ar_b = sar;
            r.stat_l_b = tl;
            r.stat_ar_b = tar;
            r.flags_b = w.fn.flags | (seed << GPUDIFF_OBJ_SEED_SHIFT) | GPUDIFF_OBJ_FRESH;
        } else {
            // the conservative row reads nothing (decode error): it still names the stored blob,
            // on its own side only (flags_b FRESH with zero-length A)
            r.off_b = local_tag(t, off);
            r.spec_l_b = sl;
            r.spec_ar_b = sar;
            r.stat_l_b = tl;
            r.stat_ar_b = tar;
            r.flags_b = GPUDIFF_OBJ_DECODE_ERR | GPUDIFF_OBJ_FRESH;
        }
        S.live = true;
        S.seed = seed;
        S.off = local_tag(t, off);
        S.bytes = blob_bytes(sl, sar, tl, tar);
        S.spec_l = sl;
        S.spec_ar = sar;
        S.stat_l = tl;
        S.stat_ar = tar;
        S.oflags = w.fn.flags & GPUDIFF_OBJ_HAS_STATUS;
        w.live_delta++;
        w.bytes_delta += S.bytes;
        std::swap(S.tab, w.fn.tab);
        w.touched.push_back(e.slot);
    }
    size_t pad = (w.pool.size() + GPUDIFF_BLOB_ALIGN - 1) & ~(size_t)(GPUDIFF_BLOB_ALIGN - 1);
    w.pool.resize(pad, 0);
}

extern "C" {

int gpudiff_store_create(gpudiff_ctx* c, uint32_t max_slots, uint64_t space_bytes, uint32_t max_events,
                         gpudiff_store** out) {
    return gpudiff_store_create_ex(c, max_slots, space_bytes, max_events, 0, out);
}

int gpudiff_store_create_ex(gpudiff_ctx* c, uint32_t max_slots, uint64_t space_bytes, uint32_t max_events,
                            uint32_t flags, gpudiff_store** out) {
    if (!c || !out || !max_slots || !max_events || space_bytes < 4096) return GPUDIFF_E_INVAL;
    if (flags & ~GPUDIFF_STORE_DEVICE_ENCODE) return GPUDIFF_E_INVAL;
    *out = nullptr;
    int rc = set_device(c);
    if (rc) return rc;
    if (flags & GPUDIFF_STORE_DEVICE_ENCODE) {
        std::unique_ptr<gpudiff_store> s(new (std::nothrow) gpudiff_store());
        if (!s) return GPUDIFF_E_NOMEM;
        s->dev = dstore_create(c, max_slots, space_bytes, max_events, &rc);
        if (!s->dev) return rc;
        *out = s.release();
        return GPUDIFF_OK;
    }
    std::unique_ptr<gpudiff_store> s(new (std::nothrow) gpudiff_store());
    if (!s) return GPUDIFF_E_NOMEM;
    try {
        s->slots.resize(max_slots);
    } catch (const std::bad_alloc&) {
        return GPUDIFF_E_NOMEM;
    }
    s->max_slots = max_slots;
    s->max_events = max_events;
    s->space_bytes = (space_bytes + 15) & ~15ull;
    auto fail = [&](int e) {
        gpudiff_store_free(c, s.release());
        return e;
    };
    for (auto& sp : s->space)
        if ((rc = dalloc(&sp, s->space_bytes))) return fail(rc);
    for (auto& d : s->ring) {
        if ((rc = gpudiff_dbatch_create(c, 16, max_events, &d))) return fail(rc);
        (void)hipFree(d->pool);  // the batch reads the store's current space
        d->pool = nullptr;
        d->pool_borrowed = true;
    }
    for (uint32_t t = 0; t < std::max(1u, c->threads); t++) {
        std::unique_ptr<Worker> w(new (std::nothrow) Worker());
        if (!w) return fail(GPUDIFF_E_NOMEM);
        w->enc.reset(new (std::nothrow) PairEncoder(c->ecfg));
        if (!w->enc) return fail(GPUDIFF_E_NOMEM);
        s->workers.push_back(std::move(w));
    }
    s->st.max_slots = max_slots;
    s->st.space_bytes = s->space_bytes;
    *out = s.release();
    return GPUDIFF_OK;
}

int gpudiff_store_submit(gpudiff_ctx* c, gpudiff_store* s, const gpudiff_event* ev, size_t n, gpudiff_ticket* ticket) {
    if (!c || !s || (n && !ev)) return GPUDIFF_E_INVAL;
    int rc = set_device(c);
    if (rc) return rc;
    if (s->dev) return dstore_submit(c, s->dev, ev, n, ticket);
    if (n > s->max_events) return GPUDIFF_E_INVAL;
    if (s->broken) return GPUDIFF_E_STATE;
    for (size_t i = 0; i < n; i++)
        if (ev[i].slot >= s->max_slots || !ev[i].new_json) return GPUDIFF_E_INVAL;
    const uint32_t slot_ring = s->ring_next;
    s->ring_next ^= 1u;
    gpudiff_dbatch* d = s->ring[slot_ring];
    HIPCHK(hipEventSynchronize(d->done));  // its previous pass is finished (results are read by wait)

    // 1-2: encode, split by slot over the threads
    s->epoch++;
    const uint32_t T = (uint32_t)std::min<size_t>(s->workers.size(), std::max<size_t>(1, n / 128));
    std::vector<gpudiff_pair_row> rows;
    try {
        rows.resize(n);
        for (auto& w : s->workers) {
            w->pool.clear();
            w->touched.clear();
            w->pre.clear();
        }
        workers(c).run(T, [&](uint32_t t) { store_encode_part(c, s, ev, n, t, T, rows.data()); });
    } catch (const std::bad_alloc&) {
        s->broken = true;
        return GPUDIFF_E_NOMEM;
    }
    uint64_t total = 0;
    std::vector<uint64_t> part_base(T);
    for (uint32_t t = 0; t < T; t++) {
        part_base[t] = total;
        total += s->workers[t]->pool.size();
    }
    // 3: space management, then final offsets
    if (s->used + total > s->space_bytes) {
        if ((rc = store_compact(c, s, rows))) {
            s->broken = true;
            return rc;
        }
        if (s->used + total > s->space_bytes) {
            s->broken = true;  // live set + batch exceed a space: recreate the store larger
            return GPUDIFF_E_CAPACITY;
        }
    }
    const uint64_t base = s->used;
    auto fix = [&](uint64_t off) -> uint64_t {
        if (!(off & kLocal)) return off;
        const uint32_t part = (uint32_t)((off >> kLocalPartShift) & 0x7FFF);
        return base + part_base[part] + (off & ((1ull << kLocalPartShift) - 1));
    };
    uint64_t cb = 0;
    for (gpudiff_pair_row& r : rows) {
        r.off_a = fix(r.off_a);
        r.off_b = fix(r.off_b);
        cb += pair_compare_bytes(r);
    }
    uint64_t leaves = 0;
    for (uint32_t t = 0; t < T; t++) {
        Worker& w = *s->workers[t];
        for (uint32_t sl : w.touched) {
            Slot& S = s->slots[sl];
            if (S.live && (S.off & kLocal)) S.off = fix(S.off);
        }
        leaves += w.leaves;
        w.leaves = 0;
        s->st.live_slots += w.live_delta;
        s->st.live_bytes += w.bytes_delta;
        w.live_delta = w.bytes_delta = 0;
        s->st.old_encoded += w.old_encoded;
        s->st.reseeded += w.reseeded;
        s->st.collisions_unresolved += w.unresolved;
        w.old_encoded = w.reseeded = w.unresolved = 0;
    }
    // 4: stage (pinned), H2D, diff
    gpudiff_hbatch*& hb = s->staging[slot_ring];
    uint8_t* hp = nullptr;
    gpudiff_pair_row* hr = nullptr;
    if (!hb) rc = gpudiff_hbatch_create(c, (total + 15) & ~15ull, n, leaves, &hb, &hp, &hr);
    else rc = gpudiff_hbatch_resize(c, hb, (total + 15) & ~15ull, n, leaves, &hp, &hr);
    if (rc) {
        s->broken = true;
        return rc;
    }
    for (uint32_t t = 0; t < T; t++)
        if (!s->workers[t]->pool.empty())
            memcpy(hp + part_base[t], s->workers[t]->pool.data(), s->workers[t]->pool.size());
    if (n) memcpy(hr, rows.data(), n * sizeof(gpudiff_pair_row));
    uint8_t* space = s->space[s->cur];
    if (total) HIPCHK(hipMemcpyAsync(space + base, hp, total, hipMemcpyHostToDevice, c->stream));
    if (n) HIPCHK(hipMemcpyAsync(d->rows, hr, n * sizeof(gpudiff_pair_row), hipMemcpyHostToDevice, c->stream));
    if (hb->used) HIPCHK(hipEventRecord(hb->used, c->stream));
    if (n) {
        HIPCHK(launch_rebase(c->stream, d->rows, 0, (uint32_t)n, 0, d->pair_ids));  // pair_ids SoA copy
    }
    s->used += total;
    d->pool = space;
    d->pool_cap = s->space_bytes;
    d->pool_used = s->used;
    d->n_pairs = n;
    d->rows_gen++;
    d->leaves = leaves;
    d->compare_bytes = cb;
    d->value_bytes = 0;
    if ((rc = gpudiff_diff(c, d, ticket))) {
        s->broken = true;
        return rc;
    }
    s->st.events += n;
    s->st.last_batch_bytes = total;
    return GPUDIFF_OK;
}

int gpudiff_store_forget(gpudiff_ctx* c, gpudiff_store* s, uint32_t slot) {
    if (!c || !s) return GPUDIFF_E_INVAL;
    if (s->dev) {
        int rc = set_device(c);
        if (rc) return rc;
        return dstore_forget(c, s->dev, slot);
    }
    if (slot >= s->max_slots) return GPUDIFF_E_INVAL;
    Slot& S = s->slots[slot];
    if (S.live) {
        s->st.live_slots--;
        s->st.live_bytes -= S.bytes;
    }
    S.live = false;
    S.seed = 0;
    S.tab = PathTable();
    return GPUDIFF_OK;
}

int gpudiff_store_stats_get(const gpudiff_store* s, gpudiff_store_stats* out) {
    if (!s || !out) return GPUDIFF_E_INVAL;
    if (s->dev) return dstore_stats(s->dev, out);
    *out = s->st;
    out->used_bytes = s->used;
    return GPUDIFF_OK;
}

void gpudiff_store_free(gpudiff_ctx* c, gpudiff_store* s) {
    if (!s) return;
    if (s->dev) {
        dstore_free(c, s->dev);
        delete s;
        return;
    }
    if (c && c->has_device) {
        (void)hipSetDevice(c->device);
        (void)hipStreamSynchronize(c->stream);
    }
    for (auto& d : s->ring)
        if (d) gpudiff_dbatch_free(c, d);
    for (auto& hb : s->staging)
        if (hb) gpudiff_hbatch_free(c, hb);
    for (auto& sp : s->space)
        if (sp) (void)hipFree(sp);
    if (s->moves_dev) (void)hipFree(s->moves_dev);
    delete s;
}

}  // extern "C"
