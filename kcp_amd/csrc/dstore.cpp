// Device-encode mode of the object store (gpudiff_store_create_ex with
// GPUDIFF_STORE_DEVICE_ENCODE; include/gpudiff.h): the informer's events go
// up as raw JSON and the GPU does the rest.
//
// submit (host work is a memcpy into pinned staging plus O(1) per event):
//   1. documents: each event's new object, plus its old object when the slot
//      has never been seen (the first sighting diffs against it); per slot a
//      chain of the batch's documents (prev/next) so events on one slot apply
//      in order;
//   2. one H2D of the JSON and the document table;
//   3. K0 (tokenize.hip) encodes every document into the current space; K0c
//      checks each event against its old side for path-hash collisions; K0x
//      walks the chains, writes the (old, new) rows and the slots' new resident
//      blobs; then the ordinary diff pass (K2..K6).
// Everything K0 does not take (a Go decode error, a float beyond its exact
// conversion, an escaped key, a duplicate key or a collision, ...) is
// deferred: its row is conservative in the device pass, the slot is marked
// pending, and gpudiff_wait re-does those events on the host with the
// Go-exact encoder (the same decisions store.cpp makes), places the blobs,
// diffs them and patches the results -- so every result equals the host
// store's, and later batches defer events of pending slots until then.
//
// Contract of this mode: event buffers stay valid until gpudiff_wait on the
// ticket returns (deferred events are re-read), and batches are waited in
// submit order, at most two in flight.
#include "dstore.h"

#include <emmintrin.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <mutex>
#include <new>
#include <thread>
#include <unordered_map>
#include <vector>

#include "tokenize.h"

using namespace gd;

namespace {

constexpr uint64_t kScratchCap = 2ull << 30;  // K0 working area, reused across launches
// a device-encoded batch's JSON is staged, uploaded and encoded in up to kMaxUpChunks chunks of at least
// kUpChunkBytes (whole documents): the smaller the chunks, the sooner the first upload starts and the shorter
// the last chunk's K0 after the copy stream is done.  GPUDIFF_H2D_CHUNK_MIB / GPUDIFF_H2D_MAX_CHUNKS (read once
// per store, A/B tuning only) override them; round 3 used 4 chunks of >= 16 MiB.
constexpr uint32_t kMaxUpChunks = 16;
constexpr uint64_t kUpChunkBytes = 16ull << 20;
// ... and of at least kMinChunkDocs documents: each chunk's K0 launch (a wave per document) should fill the
// chip's ~8k resident waves twice over (r04m: 12 chunks of 5.4k documents made config5's K0 6.4 ms, from 4.1)
constexpr uint64_t kMinChunkDocs = 16384;
// store mode: the K0 stage on the kernel stream.  The decoupled form (K0 stage on its own stream; compaction,
// Delete and the host resolution's placement ordered against it) measured within box noise on config 5
// (profiles/r04zs) and stays compiled out until a measurement shows a gain
constexpr bool kDecoupleStore = false;

struct Ring {
    gpudiff_dbatch* d = nullptr;  // rows, pair_ids, results; pool = the store's current space
    uint8_t* hjson = nullptr;     // pinned staging
    uint64_t hjson_cap = 0;
    uint8_t* hmeta = nullptr;     // pinned: TokDoc[] | DocLink[] | heads[]
    uint64_t hmeta_cap = 0;
    uint8_t* djson = nullptr;
    uint64_t djson_cap = 0;
    uint8_t* dmeta = nullptr;
    uint64_t dmeta_cap = 0;
    TokOut* douts = nullptr;
    uint8_t* dcoll = nullptr;
    uint8_t* ddef = nullptr;
    uint64_t docs_cap = 0, coll_cap = 0, def_cap = 0;
    uint32_t* dcnt = nullptr;     // deferred events of the batch
    hipEvent_t staged = nullptr;  // its H2D copies finished (pinned buffers reusable)
    hipEvent_t k0_done = nullptr;  // its K0..K0x finished reading the device JSON / document table
    bool k0_recorded = false;
    hipEvent_t pass_done = nullptr;  // pair mode: its diff pass finished reading its space (K0 may refill it)
    bool pass_recorded = false;
    hipEvent_t t_ev[5] = {};      // GPUDIFF_OPT_TIMING: H2D begin/end (copy stream), K0 begin/end, K0c+K0x end
    hipEvent_t chunk_ev[kMaxUpChunks] = {};  // each JSON chunk's H2D done: its K0 launches may start
    std::vector<gpudiff_event> events;
    std::vector<uint8_t> final_flags;  // the waited batch's result flags (deferred events resolved)
    bool waited = false;
    uint32_t batch = 0, nev = 0;
    uint64_t bound = 0;
    gpudiff_ticket ticket = 0;
    bool outstanding = false;
};

// gpudiff_host_alloc's pinned buffers: a gpudiff_submit batch laid out in one of them (gpudiff.h) is uploaded
// straight from it, without the staging copy
struct HostBuf {
    gpudiff_ctx* c;
    uint8_t* p;
    uint64_t n;
};
std::mutex g_hb_mu;
std::vector<HostBuf> g_hb;

bool find_host_buf(gpudiff_ctx* c, const void* q, uint8_t** base, uint64_t* size) {
    std::lock_guard<std::mutex> lk(g_hb_mu);
    for (const HostBuf& h : g_hb)
        if (h.c == c && (const uint8_t*)q >= h.p && (const uint8_t*)q < h.p + h.n) {
            *base = h.p;
            *size = h.n;
            return true;
        }
    return false;
}

}  // namespace

struct DStore {
    gpudiff_ctx* c = nullptr;
    uint32_t max_slots = 0, max_events = 0;
    uint64_t space_bytes = 0;
    uint8_t* space[2] = {nullptr, nullptr};
    uint32_t cur = 0;
    unsigned long long* used_dev = nullptr;  // the current space's append point (one of used_base[0..1])
    unsigned long long* used_base = nullptr;
    uint64_t used_ub = 0;  // host upper bound of *used_dev
    // gpudiff_submit's pair mode: ring slot r's batches own space[r] and used_base[r] (each batch starts it
    // empty: the batch two submits back is dropped), so neither a compaction nor its host sync is ever needed
    DSlot* slots = nullptr;
    uint32_t* ctr = nullptr;  // kCtrLive, kCtrLiveBytes
    hipStream_t cs = nullptr;  // H2D of the next batch overlaps K0 of the current one
    // K0 of odd chunks runs on a second stream (its own half of the scratch), so one chunk's launch tail
    // overlaps the next chunk's start instead of idling the CUs between back-to-back launches on one stream
    // (interleaved A/B, profiles/r04ze: one K0 stream 7.44-7.51M pairs/s vs 7.90-8.37M)
    hipStream_t ks = nullptr;
    hipEvent_t ks_ev = nullptr;
    // pair mode with two K0 streams: the whole K0 stage (slot reset, K0 of even chunks, K0c, K0x) runs on ks0 and
    // waits only for what it reuses -- the previous batch's K0x (the shared slot table) and this ring slot's
    // previous diff pass (its space) -- so a batch's K0 overlaps the previous batch's diff pass on the kernel stream
    hipStream_t ks0 = nullptr;
    int last_ring = -1;  // the ring slot of the previous submit
    // store mode with kDecoupleStore (off): the K0 stage on ks0 there too; whatever the kernel stream
    // does to the slot table or the space between submits (compaction, Delete, the host resolution's placement)
    // first waits for the last K0 stage and sets st_slot_ops, and the next K0 stage then waits for the kernel stream
    bool dec_store = false;
    bool st_slot_ops = false;
    hipEvent_t st_ev = nullptr;
    uint64_t* sizes = nullptr;
    uint64_t* tile_sums = nullptr;
    uint8_t* scratch = nullptr;
    uint64_t scratch_cap = 0;
    Ring ring[2];
    uint32_t ring_next = 0;
    uint32_t batch_seq = 0;
    uint32_t next_wait = 1;  // batches are waited in submit order
    // per slot, one cache line fetch per event: the batch that last staged a document of the slot,
    // that document, and whether the slot was submitted before (its resident version may exist)
    struct SlotState {
        uint32_t stamp;
        int32_t last;
    };
    std::vector<SlotState> sstate;
    std::vector<uint8_t> seen;
    std::unordered_map<uint32_t, uint32_t> forgotten;  // slot -> batch_seq at forget
    // resolution
    std::unique_ptr<PairEncoder> enc;
    gpudiff_dbatch* res_d = nullptr;
    uint8_t* res_stage = nullptr;
    uint64_t res_stage_cap = 0;
    SlotUpdate* res_ups = nullptr;
    uint64_t res_ups_cap = 0;
    uint32_t* res_err = nullptr;
    bool broken = false;
    bool pair_mode = false;  // gpudiff_submit with GPUDIFF_OPT_DEVICE_ENCODE: slot i = pair i, no state kept
    gpudiff_store_stats st{};
    uint64_t deferred_total = 0;
    // GPUDIFF_OPT_TIMING: per-batch sums (ms) of host submit, H2D, K0, K0c+K0x
    double t_sum[4] = {0, 0, 0, 0};
    double t_sub[5] = {0, 0, 0, 0, 0};  // submit: slot wait, tables, copy, enqueue; finisher
    uint64_t t_n = 0;
};

namespace {

// one staged document: its bytes, then zeros up to `span` (a multiple of 16; dst 16-B aligned), with
// non-temporal 16-B stores -- the pinned staging is only read by the DMA engine, so the stores skip
// the read-for-ownership and do not evict the workers' caches
void stream_doc(uint8_t* dst, const uint8_t* src, size_t len, size_t span) {
    size_t i = 0;
    for (; i + 16 <= len; i += 16)
        _mm_stream_si128((__m128i*)(dst + i), _mm_loadu_si128((const __m128i*)(src + i)));
    if (i < len) {
        alignas(16) uint8_t t[16] = {0};
        memcpy(t, src + i, len - i);
        _mm_stream_si128((__m128i*)(dst + i), _mm_load_si128((const __m128i*)t));
        i += 16;
    }
    const __m128i z = _mm_setzero_si128();
    for (; i < span; i += 16) _mm_stream_si128((__m128i*)(dst + i), z);
}

int grow_pinned(uint8_t** p, uint64_t* cap, uint64_t need) {
    if (need <= *cap) return GPUDIFF_OK;
    if (*p) (void)hipHostFree(*p);
    *p = nullptr;
    *cap = 0;
    const uint64_t n = std::max<uint64_t>(need + need / 4, 1 << 16);
    HIPCHK(hipHostMalloc((void**)p, n, hipHostMallocDefault));
    *cap = n;
    return GPUDIFF_OK;
}

template <class T>
int grow_dev(T** p, uint64_t* cap, uint64_t need) {
    if (need <= *cap) return GPUDIFF_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    const uint64_t n = std::max<uint64_t>(need + need / 4, 256);
    int rc = dalloc(p, n);
    if (rc) return rc;
    *cap = n;
    return GPUDIFF_OK;
}

// a kernel-stream operation on the slot table or the space (store mode with the K0 stage on its own stream):
// after the last K0 stage, and the next K0 stage waits for it
int before_st_slot_op(DStore* s) {
    if (!s->dec_store) return GPUDIFF_OK;
    if (s->last_ring >= 0 && s->ring[s->last_ring].k0_recorded)
        HIPCHK(hipStreamWaitEvent(s->c->stream, s->ring[s->last_ring].k0_done, 0));
    s->st_slot_ops = true;
    return GPUDIFF_OK;
}

// packs the live blobs into the other space (stream-ordered), then reads the
// exact append point back
int compact(DStore* s) {
    gpudiff_ctx* c = s->c;
    if (int rc = before_st_slot_op(s)) return rc;
    HIPCHK(launch_compact_store(c->stream, s->slots, s->max_slots, s->space[s->cur], s->space[1 - s->cur], s->sizes,
                                s->tile_sums, s->used_dev));
    s->cur = 1 - s->cur;
    uint64_t used = 0;
    HIPCHK(hipMemcpyAsync(&used, s->used_dev, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    s->used_ub = used;
    s->st.compactions++;
    return GPUDIFF_OK;
}

// compacts when `want` bytes may not fit; fails only when not even `need` bytes fit after it
int ensure_space(DStore* s, uint64_t want, uint64_t need) {
    if (s->used_ub + want <= s->space_bytes) return GPUDIFF_OK;
    if (s->pair_mode)  // the other space is the other ring slot's batch: no compaction into it
        return s->used_ub + need <= s->space_bytes ? GPUDIFF_OK : GPUDIFF_E_CAPACITY;
    int rc = compact(s);
    if (rc) return rc;
    return s->used_ub + need <= s->space_bytes ? GPUDIFF_OK : GPUDIFF_E_CAPACITY;
}

// ------------------------------------------------------------------ host resolution
struct HostSlot {
    bool fetched = false;
    bool live = false, has_status = false;
    uint32_t seed = 0;
    uint64_t off = 0;  // absolute, or kRelTag | offset in the resolution pool
    uint32_t sl = 0, sar = 0, tl = 0, tar = 0, bytes = 0, n_tab = 0;
    bool tab_loaded = false;
    PathTable tab;
};

int fetch_slot(DStore* s, uint32_t slot, HostSlot& H) {
    DSlot d;
    HIPCHK(hipMemcpy(&d, s->slots + slot, sizeof(DSlot), hipMemcpyDeviceToHost));
    H.fetched = true;
    H.live = d.flags & DS_LIVE;
    H.has_status = d.flags & DS_HAS_STATUS;
    H.seed = (d.flags >> 8) & 0xFF;
    H.off = d.off;
    H.sl = d.spec_l;
    H.sar = d.spec_ar;
    H.tl = d.stat_l;
    H.tar = d.stat_ar;
    H.bytes = d.bytes;
    H.n_tab = d.n_tab;
    H.tab_loaded = false;
    return GPUDIFF_OK;
}

// the path table of a device-resident blob: its trailer
int load_tab(DStore* s, HostSlot& H) {
    if (H.tab_loaded) return GPUDIFF_OK;
    const uint64_t segs = gpudiff_blob_body(H.sl, H.sar, H.tl, H.tar);  // the table follows the body
    H.tab.n = H.n_tab;
    H.tab.data.resize(H.bytes - segs);
    if (!H.tab.data.empty())
        HIPCHK(hipMemcpy(H.tab.data.data(), s->space[s->cur] + H.off + segs, H.tab.data.size(), hipMemcpyDeviceToHost));
    H.tab_loaded = true;
    return GPUDIFF_OK;
}

void set_tab(HostSlot& H, const FlatObject& o) {
    H.tab = o.tab;
    H.n_tab = o.tab.n;
    H.tab_loaded = true;
}

// Re-does the batch's deferred events on the host (store.cpp's decisions),
// diffs them on the device and patches rs.
int resolve(DStore* s, Ring& R, ResultStore& rs) {
    gpudiff_ctx* c = s->c;
    HIPCHK(hipStreamSynchronize(c->stream));
    if (s->dec_store) {  // the slot reads below see every K0 stage submitted so far, and the placement follows them
        HIPCHK(hipStreamSynchronize(s->ks0));
        s->st_slot_ops = true;
    }
    std::vector<uint8_t> def(R.nev);
    if (R.nev) HIPCHK(hipMemcpy(def.data(), R.ddef, R.nev, hipMemcpyDeviceToHost));
    std::vector<uint32_t> drows;
    for (uint32_t i = 0; i < R.nev; i++)
        if (def[i]) drows.push_back(i);
    if (drows.empty()) return GPUDIFF_OK;
    s->deferred_total += drows.size();
    int rc;
    PairEncoder& enc = *s->enc;
    Arena arena_new, arena_old;
    FlatObject fn, fo;
    std::vector<uint8_t> pool;
    std::vector<gpudiff_pair_row> rows(drows.size());
    std::unordered_map<uint32_t, HostSlot> hs;
    std::vector<uint32_t> touched;
    for (size_t k = 0; k < drows.size(); k++) {
        const gpudiff_event& e = R.events[drows[k]];
        if (s->pair_mode) {  // gpudiff_encode_pairs' decisions on (old_json, new_json)
            gpudiff_pair_row& r = rows[k];
            memset(&r, 0, sizeof(r));
            r.pair_id = e.pair_id;
            r.cluster_id = e.cluster_id;
            uint32_t seed = 0;
            if (e.old_json && enc.flatten_json(e.old_json, e.old_len, arena_old, fo) &&
                enc.flatten_json(e.new_json, e.new_len, arena_new, fn) && enc.pair_seed(fo, fn, &seed)) {
                uint64_t oa, ob;
                enc.write_object(fo, pool, &oa, &r.spec_l_a, &r.spec_ar_a, &r.stat_l_a, &r.stat_ar_a);
                enc.write_object(fn, pool, &ob, &r.spec_l_b, &r.spec_ar_b, &r.stat_l_b, &r.stat_ar_b);
                r.off_a = kRelTag | oa;
                r.off_b = kRelTag | ob;
                r.flags_a = (fo.flags & GPUDIFF_OBJ_HAS_STATUS) | (seed << GPUDIFF_OBJ_SEED_SHIFT);
                r.flags_b = (fn.flags & GPUDIFF_OBJ_HAS_STATUS) | (seed << GPUDIFF_OBJ_SEED_SHIFT);
            } else {
                r.flags_a = r.flags_b = GPUDIFF_OBJ_DECODE_ERR;
            }
            continue;
        }
        HostSlot& S = hs[e.slot];
        if (!S.fetched) {
            if ((rc = fetch_slot(s, e.slot, S))) return rc;
            touched.push_back(e.slot);
        }
        gpudiff_pair_row& r = rows[k];
        memset(&r, 0, sizeof(r));
        r.pair_id = e.pair_id;
        r.cluster_id = e.cluster_id;
        auto conservative = [&]() { r.flags_a = r.flags_b = GPUDIFF_OBJ_DECODE_ERR; };
        if (!enc.flatten_json(e.new_json, e.new_len, arena_new, fn)) {
            conservative();
            S.live = false;
            S.tab_loaded = false;
            continue;
        }
        bool ok = false, pair_error = false, a_live = false;
        uint32_t seed = 0;
        uint64_t a_off = 0;
        uint32_t a_sl = 0, a_sar = 0, a_tl = 0, a_tar = 0, a_of = 0;
        auto a_is_slot = [&]() {
            a_live = true;
            // the slot's blob as it is when k_place runs (a compaction may move it)
            a_off = (S.off & kRelTag) ? S.off : (kSlotTag | e.slot);
            a_sl = S.sl;
            a_sar = S.sar;
            a_tl = S.tl;
            a_tar = S.tar;
            a_of = S.has_status ? GPUDIFF_OBJ_HAS_STATUS : 0u;
        };
        if (S.live && S.seed == 0) {
            if ((rc = load_tab(s, S))) return rc;
            if (enc.hash_single(fn, 0) && tab_agree(tab_view(S.tab), tab_view(fn.tab))) {
                ok = true;
                a_is_slot();
            }
        }
        if (!ok && e.old_json) {
            if (enc.flatten_json(e.old_json, e.old_len, arena_old, fo) && enc.pair_seed(fo, fn, &seed)) {
                uint64_t off;
                enc.write_object(fo, pool, &off, &a_sl, &a_sar, &a_tl, &a_tar);
                a_live = true;
                a_off = kRelTag | off;
                a_of = fo.flags & GPUDIFF_OBJ_HAS_STATUS;
                s->st.old_encoded++;
                if (S.live) s->st.reseeded++;
                ok = true;
            } else {
                pair_error = true;
            }
        } else if (!ok && S.live && S.seed) {
            if ((rc = load_tab(s, S))) return rc;
            if (enc.hash_single(fn, S.seed) && tab_agree(tab_view(S.tab), tab_view(fn.tab))) {
                ok = true;
                seed = S.seed;
                a_is_slot();
            } else {
                pair_error = true;
                s->st.collisions_unresolved++;
            }
        } else if (!ok && !S.live) {
            ok = enc.first_seed(fn, &seed);
            pair_error = !ok;
        } else if (!ok) {
            pair_error = true;
            s->st.collisions_unresolved++;
        }
        if (pair_error) {
            conservative();
            if (!enc.store_seed(fn, &seed)) {
                S.live = false;
                S.tab_loaded = false;
                continue;
            }
        }
        uint64_t off;
        uint32_t sl, sar, tl, tar, bytes;
        enc.write_object_tab(fn, pool, &off, &sl, &sar, &tl, &tar, &bytes);
        if (!pair_error) {
            r.off_a = a_live ? a_off : 0;
            r.spec_l_a = a_sl;
            r.spec_ar_a = a_sar;
            r.stat_l_a = a_tl;
            r.stat_ar_a = a_tar;
            r.flags_a = a_of | (seed << GPUDIFF_OBJ_SEED_SHIFT);
            r.off_b = kRelTag | off;
            r.spec_l_b = sl;
            r.spec_ar_b = sar;
            r.stat_l_b = tl;
            r.stat_ar_b = tar;
            r.flags_b = (fn.flags & GPUDIFF_OBJ_HAS_STATUS) | (seed << GPUDIFF_OBJ_SEED_SHIFT);
        }
        S.live = true;
        S.seed = seed;
        S.has_status = fn.flags & GPUDIFF_OBJ_HAS_STATUS;
        S.off = kRelTag | off;
        S.sl = sl;
        S.sar = sar;
        S.tl = tl;
        S.tar = tar;
        S.bytes = bytes;
        set_tab(S, fn);
    }
    // slot states (forgotten-since slots keep their forget)
    std::vector<SlotUpdate> ups;
    for (uint32_t slot : touched) {
        auto f = s->forgotten.find(slot);
        if (f != s->forgotten.end() && f->second >= R.batch) continue;
        const HostSlot& S = hs[slot];
        SlotUpdate u{};
        u.slot = slot;
        u.batch = R.batch;
        if (S.live) {
            u.entry.off = S.off;
            u.entry.spec_l = S.sl;
            u.entry.spec_ar = S.sar;
            u.entry.stat_l = S.tl;
            u.entry.stat_ar = S.tar;
            u.entry.bytes = S.bytes;
            u.entry.n_tab = S.n_tab;
            u.entry.flags = DS_LIVE | (S.has_status ? DS_HAS_STATUS : 0u) | (S.seed << 8);
        } else {
            s->seen[slot] = 0;  // the next event stages its old object again
        }
        ups.push_back(u);
    }
    // place: blobs behind the append point, rows, slot states
    const uint64_t pbytes = (pool.size() + GPUDIFF_BLOB_ALIGN - 1) & ~(uint64_t)(GPUDIFF_BLOB_ALIGN - 1);
    pool.resize(pbytes, 0);
    if ((rc = ensure_space(s, pbytes, pbytes))) {
        if (rc != GPUDIFF_E_CAPACITY) return rc;
        // The space cannot take the re-encoded blobs even after a compaction (K0 deferred these
        // events for lack of space, and the host's blobs do not fit either).  The store stays
        // usable: the events are reported dirty with GPUDIFF_DECODE_ERROR (the reference's
        // conservative rule, specsyncer.go:20-22: never "equal") and their slots are emptied, so
        // each slot's next event stages its old object again.
        for (SlotUpdate& u : ups) {
            memset(&u.entry, 0, sizeof(u.entry));
            s->seen[u.slot] = 0;
        }
        if ((rc = grow_dev(&s->res_ups, &s->res_ups_cap, std::max<size_t>(ups.size(), 1)))) return rc;
        if (!ups.empty()) HIPCHK(hipMemcpy(s->res_ups, ups.data(), ups.size() * sizeof(SlotUpdate), hipMemcpyHostToDevice));
        HIPCHK(hipMemsetAsync(s->res_err, 0, 4, c->stream));
        HIPCHK(launch_place(c->stream, nullptr, 0, s->space[s->cur], s->used_dev, s->space_bytes, nullptr, nullptr, 0,
                            s->res_ups, (uint32_t)ups.size(), s->slots, s->ctr, s->res_err));
        HIPCHK(hipStreamSynchronize(c->stream));
        s->st.space_conservative += drows.size();
        ResultStore out;
        out.flags.resize(R.nev);
        out.off.push_back(0);
        size_t jr = 0;
        for (uint32_t i = 0; i < R.nev; i++) {
            uint8_t f = rs.flags[i];
            uint32_t lo = 0, hi = 0;
            if (f & (GPUDIFF_SPEC_DIRTY | GPUDIFF_STATUS_DIRTY)) {
                lo = rs.off[jr];
                hi = rs.off[jr + 1];
                jr++;
            }
            if (def[i]) {
                f = GPUDIFF_SPEC_DIRTY | GPUDIFF_STATUS_DIRTY | GPUDIFF_DECODE_ERROR;
                lo = hi = 0;
            }
            out.flags[i] = f;
            const uint32_t pid = R.events[i].pair_id;
            if (f & GPUDIFF_SPEC_DIRTY) out.spec.push_back(pid);
            if (f & GPUDIFF_STATUS_DIRTY) out.status.push_back(pid);
            if (f & (GPUDIFF_SPEC_DIRTY | GPUDIFF_STATUS_DIRTY)) {
                out.dirty.push_back(pid);
                for (uint32_t q = lo; q < hi; q++) {
                    out.hashes.push_back(rs.hashes[q]);
                    out.kinds.push_back(rs.kinds[q]);
                }
                out.off.push_back((uint32_t)out.hashes.size());
            }
        }
        rs = std::move(out);
        return GPUDIFF_OK;
    }
    if ((rc = grow_dev(&s->res_stage, &s->res_stage_cap, std::max<uint64_t>(pbytes, 16)))) return rc;
    if ((rc = grow_dev(&s->res_ups, &s->res_ups_cap, std::max<size_t>(ups.size(), 1)))) return rc;
    gpudiff_dbatch* d = s->res_d;
    if (d->max_pairs < rows.size()) {
        gpudiff_dbatch_free(c, d);
        s->res_d = nullptr;
        if ((rc = gpudiff_dbatch_create(c, 16, rows.size() + rows.size() / 2, &s->res_d))) return rc;
        d = s->res_d;
        (void)hipFree(d->pool);
        d->pool = nullptr;
        d->pool_borrowed = true;
    }
    if (pbytes) HIPCHK(hipMemcpy(s->res_stage, pool.data(), pbytes, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(d->rows, rows.data(), rows.size() * sizeof(gpudiff_pair_row), hipMemcpyHostToDevice));
    if (!ups.empty()) HIPCHK(hipMemcpy(s->res_ups, ups.data(), ups.size() * sizeof(SlotUpdate), hipMemcpyHostToDevice));
    HIPCHK(hipMemsetAsync(s->res_err, 0, 4, c->stream));
    HIPCHK(launch_place(c->stream, s->res_stage, pbytes, s->space[s->cur], s->used_dev, s->space_bytes, d->rows,
                        d->pair_ids, (uint32_t)rows.size(), s->res_ups, (uint32_t)ups.size(), s->slots, s->ctr,
                        s->res_err));
    s->used_ub += pbytes;
    d->pool = s->space[s->cur];
    d->pool_cap = s->space_bytes;
    d->n_pairs = rows.size();
    d->rows_gen++;
    gpudiff_ticket t2;
    if ((rc = gpudiff_diff(c, d, &t2))) return rc;
    ResultStore r2;
    if ((rc = collect_results(c, d, r2))) return rc;
    c->tickets.erase(t2);
    d->ticket = 0;
    uint32_t err = 0;
    HIPCHK(hipMemcpy(&err, s->res_err, 4, hipMemcpyDeviceToHost));
    if (err) return GPUDIFF_E_CAPACITY;

    // patch: deferred rows take r2's results, the rest keep rs's
    ResultStore out;
    out.flags.resize(R.nev);
    out.off.push_back(0);
    size_t jr = 0, j2 = 0, k = 0;
    for (uint32_t i = 0; i < R.nev; i++) {
        const bool d_in = (rs.flags[i] & (GPUDIFF_SPEC_DIRTY | GPUDIFF_STATUS_DIRTY)) != 0;
        uint32_t lo = 0, hi = 0;
        const ResultStore* src = &rs;
        if (d_in) {
            lo = rs.off[jr];
            hi = rs.off[jr + 1];
            jr++;
        }
        uint8_t f = rs.flags[i];
        if (def[i]) {
            f = r2.flags[k++];
            src = &r2;
            lo = hi = 0;
            if (f & (GPUDIFF_SPEC_DIRTY | GPUDIFF_STATUS_DIRTY)) {
                lo = r2.off[j2];
                hi = r2.off[j2 + 1];
                j2++;
            }
        }
        out.flags[i] = f;
        const uint32_t pid = R.events[i].pair_id;
        if (f & GPUDIFF_SPEC_DIRTY) out.spec.push_back(pid);
        if (f & GPUDIFF_STATUS_DIRTY) out.status.push_back(pid);
        if (f & (GPUDIFF_SPEC_DIRTY | GPUDIFF_STATUS_DIRTY)) {
            out.dirty.push_back(pid);
            for (uint32_t q = lo; q < hi; q++) {
                out.hashes.push_back(src->hashes[q]);
                out.kinds.push_back(src->kinds[q]);
            }
            out.off.push_back((uint32_t)out.hashes.size());
        }
    }
    rs = std::move(out);
    return GPUDIFF_OK;
}

}  // namespace

// ------------------------------------------------------------------ API
DStore* dstore_create(gpudiff_ctx* c, uint32_t max_slots, uint64_t space_bytes, uint32_t max_events, int* rc_out) {
    std::unique_ptr<DStore> s(new (std::nothrow) DStore());
    int rc = GPUDIFF_E_NOMEM;
    if (!s) {
        *rc_out = rc;
        return nullptr;
    }
    s->c = c;
    s->max_slots = max_slots;
    s->max_events = max_events;
    s->space_bytes = (space_bytes + 15) & ~15ull;
    auto fail = [&](int e) {
        dstore_free(c, s.release());
        *rc_out = e;
        return (DStore*)nullptr;
    };
    try {
        s->sstate.assign(max_slots, DStore::SlotState{0u, -1});
        s->seen.assign(max_slots, 0);
    } catch (const std::bad_alloc&) {
        return fail(GPUDIFF_E_NOMEM);
    }
    EncodeConfig cfg = c->ecfg;
    s->enc.reset(new (std::nothrow) PairEncoder(cfg));
    if (!s->enc) return fail(GPUDIFF_E_NOMEM);
    for (auto& sp : s->space)
        if ((rc = dalloc(&sp, s->space_bytes))) return fail(rc);
    if ((rc = dalloc(&s->used_base, 2)) || (rc = dalloc(&s->slots, max_slots)) || (rc = dalloc(&s->ctr, 4)) ||
        (rc = dalloc(&s->sizes, max_slots)) || (rc = dalloc(&s->tile_sums, (max_slots + 1023) / 1024 + 1)) ||
        (rc = dalloc(&s->res_err, 1)))
        return fail(rc);
    s->used_dev = s->used_base;
    if (hipMemset(s->used_base, 0, 16) != hipSuccess || hipMemset(s->slots, 0, sizeof(DSlot) * (size_t)max_slots) ||
        hipMemset(s->ctr, 0, 16) != hipSuccess)
        return fail(GPUDIFF_E_DEVICE);
    for (Ring& R : s->ring) {
        if ((rc = gpudiff_dbatch_create(c, 16, max_events, &R.d))) return fail(rc);
        (void)hipFree(R.d->pool);
        R.d->pool = nullptr;
        R.d->pool_borrowed = true;
        if ((rc = dalloc(&R.dcnt, 1))) return fail(rc);
        if (hipEventCreateWithFlags(&R.staged, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&R.k0_done, hipEventDisableTiming) != hipSuccess)
            return fail(GPUDIFF_E_DEVICE);
    }
    if (hipStreamCreateWithFlags(&s->cs, hipStreamNonBlocking) != hipSuccess) return fail(GPUDIFF_E_DEVICE);
    // the pair-mode K0 stage on its own stream (interleaved A/B, profiles/r04zf: on the kernel stream 7.71-7.79M
    // pairs/s staged vs 7.90-8.37M)
    if (hipStreamCreateWithFlags(&s->ks, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&s->ks_ev, hipEventDisableTiming) != hipSuccess ||
        hipStreamCreateWithFlags(&s->ks0, hipStreamNonBlocking) != hipSuccess)
        return fail(GPUDIFF_E_DEVICE);
    for (Ring& R : s->ring)
        if (hipEventCreateWithFlags(&R.pass_done, hipEventDisableTiming) != hipSuccess) return fail(GPUDIFF_E_DEVICE);
    if (kDecoupleStore) {
        if (hipEventCreateWithFlags(&s->st_ev, hipEventDisableTiming) != hipSuccess) return fail(GPUDIFF_E_DEVICE);
        s->dec_store = true;
    }
    if ((rc = gpudiff_dbatch_create(c, 16, 1024, &s->res_d))) return fail(rc);
    (void)hipFree(s->res_d->pool);
    s->res_d->pool = nullptr;
    s->res_d->pool_borrowed = true;
    s->st.max_slots = max_slots;
    s->st.space_bytes = s->space_bytes;
    *rc_out = GPUDIFF_OK;
    return s.release();
}

int dstore_submit(gpudiff_ctx* c, DStore* s, const gpudiff_event* ev, size_t n, gpudiff_ticket* ticket) {
    if (s->broken) return GPUDIFF_E_STATE;
    if (n > s->max_events) return GPUDIFF_E_INVAL;
    const auto t_host0 = std::chrono::steady_clock::now();
    const bool timing = (c->flags & GPUDIFF_OPT_TIMING) != 0;
    Ring& R = s->ring[s->ring_next];
    if (R.outstanding) {
        if (!s->pair_mode) return GPUDIFF_E_STATE;  // wait on the batch two submits back first
        // pair mode keeps gpudiff_submit's ring rule: the ticket two submits back is dropped
        c->finishers.erase(R.ticket);
        R.outstanding = false;
    }
    int rc;
    if (R.staged) HIPCHK(hipEventSynchronize(R.staged));
    // pair mode with the K0 stage on its own streams (ks0 / ks): decoupled from the kernel stream
    const bool dec = (s->pair_mode || s->dec_store) && s->ks0;
    if (s->pair_mode) {  // this ring slot's space, emptied behind its previous batch (stream order)
        s->cur = s->ring_next;
        s->used_dev = s->used_base + s->ring_next;
        s->used_ub = 0;
        if (!dec) HIPCHK(hipMemsetAsync(s->used_dev, 0, 8, c->stream));  // (dec: on ks0, below)
    }
    auto lap = [&, t = std::chrono::steady_clock::now()](int k) mutable {
        if (!timing) return;
        const auto now = std::chrono::steady_clock::now();
        s->t_sub[k] += std::chrono::duration<double, std::milli>(now - t).count();
        t = now;
    };
    lap(0);
    const uint32_t batch = ++s->batch_seq;

    // 1. documents and slot chains
    const uint64_t max_docs = 2 * (uint64_t)n;
    const uint64_t meta_bytes = max_docs * (sizeof(TokDoc) + sizeof(DocLink)) + 4 * (uint64_t)n + 64;
    if ((rc = grow_pinned(&R.hmeta, &R.hmeta_cap, meta_bytes))) return rc;
    TokDoc* docs = (TokDoc*)R.hmeta;
    DocLink* links = (DocLink*)(R.hmeta + max_docs * sizeof(TokDoc));
    uint32_t* heads = (uint32_t*)(R.hmeta + max_docs * (sizeof(TokDoc) + sizeof(DocLink)));
    std::vector<const uint8_t*> src;
    src.reserve(max_docs);
    const uint8_t* zsrc = nullptr;  // zero copy: the caller's pinned buffer holds the staged layout (offset 0 here)
    uint32_t nd = 0, nh = 0;
    uint64_t jbytes = 0, bound = 0, floor = 0, new_json_bytes = 0;
    auto add_doc = [&](const uint8_t* p, size_t len, uint32_t slot, uint32_t row, const gpudiff_event& e) {
        TokDoc& D = docs[nd];
        memset(&D, 0, sizeof(D));
        D.json_off = jbytes;
        D.json_len = (uint32_t)len;
        jbytes = (jbytes + len + kTokSlack + 15) & ~15ull;
        // blob + path table: typically < 2.5x the JSON (the append estimate that triggers compaction);
        // K0 defers a document that does not fit (SPACE) to the host
        bound += (5 * (uint64_t)len) / 2 + 384;  // + the body's and the table's pads to 128 B
        floor += len;
        DocLink& L = links[nd];
        memset(&L, 0, sizeof(L));
        L.slot = slot;
        L.row = row;
        L.pair_id = e.pair_id;
        L.cluster_id = e.cluster_id;
        L.next = -1;
        DStore::SlotState& ss = s->sstate[slot];
        if (ss.stamp == batch) {
            L.prev = ss.last;
            links[L.prev].next = (int32_t)nd;
        } else {
            L.prev = -1;
            ss.stamp = batch;
            heads[nh++] = nd;
        }
        ss.last = (int32_t)nd;
        src.push_back(p);
        nd++;
    };
    if (s->pair_mode) {
        // gpudiff_submit's pairs: event i is slot i with documents 2i (old) and 2i + 1 (new), so the tables
        // are filled by the workers -- a per-thread byte sum, then each thread writes its range from its
        // offset.  Same tables as add_doc builds (it is the order-dependent path for store events).
        static const uint8_t kNone[1] = {0};
        const uint32_t T = (uint32_t)std::min<size_t>(std::max(1u, c->threads), std::max<size_t>(1, n / 4096));
        std::vector<uint64_t> part(4 * (size_t)T + 4, 0);  // per thread: JSON bytes, bound, floor, new bytes
        std::atomic<int> bad{0};
        src.resize(2 * n);
        auto step = [](size_t len) -> uint64_t { return (len + kTokSlack + 15) & ~15ull; };
        // Zero copy: every document in one gpudiff_host_alloc buffer, 16-B aligned, in pair order, each followed
        // by its staged span (step) before the next -- then the buffer's range is the staged layout itself
        uint8_t* zb = nullptr;
        uint64_t zn = 0;
        bool zc = ev[0].old_json && find_host_buf(c, ev[0].old_json, &zb, &zn);
        std::atomic<int> zc_bad{0};
        const uint8_t* zend = zb + zn - kTokSlack;  // the upload runs kTokSlack past the last document's span
        workers(c).run(T, [&](uint32_t t) {
            uint64_t jb = 0, bd = 0, fl = 0, nj = 0;
            for (size_t i = n * t / T, i1 = n * (t + 1) / T; i < i1; i++) {
                const gpudiff_event& e = ev[i];
                if (e.slot != i || e.slot >= s->max_slots || !e.new_json || e.new_len > kTokMaxLen ||
                    e.old_len > kTokMaxLen)
                    bad.store(1, std::memory_order_relaxed);
                if (zc) {
                    const uint8_t* next = i + 1 < n ? ev[i + 1].old_json : zend;
                    if (!e.old_json || e.old_json < zb || (((uintptr_t)e.old_json | (uintptr_t)e.new_json) & 15u) ||
                        e.new_json < e.old_json + step(e.old_len) || !next || next < e.new_json + step(e.new_len) ||
                        next > zend)
                        zc_bad.store(1, std::memory_order_relaxed);
                }
                const size_t lo = e.old_json ? e.old_len : 0;
                jb += step(lo) + step(e.new_len);
                bd += (5 * (uint64_t)lo) / 2 + (5 * (uint64_t)e.new_len) / 2 + 768;
                fl += lo + e.new_len;
                nj += e.new_len;
            }
            uint64_t* q = &part[4 * (size_t)(t + 1)];
            q[0] = jb, q[1] = bd, q[2] = fl, q[3] = nj;
        });
        if (bad.load()) return GPUDIFF_E_INVAL;
        zc = zc && !zc_bad.load();
        const uint8_t* zlo = ev[0].old_json;
        for (uint32_t t = 1; t <= T; t++)
            for (int k = 0; k < 4; k++) part[4 * (size_t)t + k] += part[4 * (size_t)(t - 1) + k];
        workers(c).run(T, [&](uint32_t t) {
            uint64_t off = part[4 * (size_t)t];
            for (size_t i = n * t / T, i1 = n * (t + 1) / T; i < i1; i++) {
                const gpudiff_event& e = ev[i];
                const uint8_t* pj[2] = {e.old_json ? e.old_json : kNone, e.new_json};
                const size_t len[2] = {e.old_json ? e.old_len : 0, e.new_len};
                for (uint32_t h = 0; h < 2; h++) {
                    const size_t k = 2 * i + h;
                    TokDoc& D = docs[k];
                    memset(&D, 0, sizeof(D));
                    D.json_off = zc ? (uint64_t)(pj[h] - zlo) : off;
                    D.json_len = (uint32_t)len[h];
                    off += step(len[h]);
                    if (zc)  // the staged span's padding, as the staging copy writes it (gpudiff.h: engine-owned)
                        memset((uint8_t*)pj[h] + len[h], 0, step(len[h]) - len[h]);
                    DocLink& L = links[k];
                    memset(&L, 0, sizeof(L));
                    L.slot = e.slot;
                    L.row = h ? (uint32_t)i : kNoRow;
                    L.pair_id = e.pair_id;
                    L.cluster_id = e.cluster_id;
                    L.prev = h ? (int32_t)(2 * i) : -1;
                    L.next = h ? -1 : (int32_t)(2 * i + 1);
                    src[k] = pj[h];
                }
                heads[i] = (uint32_t)(2 * i);
                s->sstate[e.slot] = DStore::SlotState{batch, (int32_t)(2 * i + 1)};
            }
        });
        const uint64_t* tot = &part[4 * (size_t)T];
        nd = (uint32_t)(2 * n);
        nh = (uint32_t)n;
        jbytes = tot[0], bound = tot[1], floor = tot[2], new_json_bytes = tot[3];
        if (zc) {
            zsrc = zlo;
            jbytes = (uint64_t)(ev[n - 1].new_json + step(ev[n - 1].new_len) - zlo);
            s->st.zero_copy_batches++;
        }
    }
    for (size_t i = 0; i < n && !s->pair_mode; i++) {
        const gpudiff_event& e = ev[i];
        if (i + 16 < n && ev[i + 16].slot < s->max_slots) {  // the slot state 16 events ahead
            __builtin_prefetch(&s->sstate[ev[i + 16].slot], 1);
            if (!s->pair_mode) __builtin_prefetch(&s->seen[ev[i + 16].slot], 1);
        }
        if (e.slot >= s->max_slots || !e.new_json || e.new_len > kTokMaxLen || e.old_len > kTokMaxLen)
            return GPUDIFF_E_INVAL;
        if (s->pair_mode) {  // every pair: its old object, then its new one (an absent old object: decode error)
            static const uint8_t kNone[1] = {0};
            add_doc(e.old_json ? e.old_json : kNone, e.old_json ? e.old_len : 0, e.slot, kNoRow, e);
        } else {
            if (!s->seen[e.slot] && e.old_json) {  // first sighting: its old object is the old side
                add_doc(e.old_json, e.old_len, e.slot, kNoRow, e);
                s->st.old_encoded++;
            }
            s->seen[e.slot] = 1;
        }
        add_doc(e.new_json, e.new_len, e.slot, (uint32_t)i, e);
        new_json_bytes += e.new_len;
    }
    if (!s->pair_mode && nd) {
        // Store-mode zero copy: the documents this submit encodes -- per event, its old object on a
        // slot's first sighting, then its new one -- lie in one gpudiff_host_alloc buffer in that order, each 16-B
        // aligned and followed by its staged span, so the buffer's range is the staged layout (gaps between the
        // documents, e.g. old objects the store does not encode, are uploaded but never read).  No staging copy.
        auto step = [](size_t len) -> uint64_t { return (len + kTokSlack + 15) & ~15ull; };
        uint8_t* zb = nullptr;
        uint64_t zn = 0;
        if (find_host_buf(c, src[0], &zb, &zn) && zn > kTokSlack) {
            const uint8_t* zend = zb + zn - kTokSlack;  // the upload runs kTokSlack past the last document's span
            const uint8_t* at = src[0];
            bool ok = true;
            for (uint32_t k = 0; k < nd && ok; k++) {
                const uint8_t* p = src[k];
                ok = p >= at && !((uintptr_t)p & 15u) && p + step(docs[k].json_len) <= zend;
                at = p + step(docs[k].json_len);
            }
            if (ok) {
                zsrc = src[0];
                for (uint32_t k = 0; k < nd; k++) {
                    docs[k].json_off = (uint64_t)(src[k] - zsrc);
                    // the staged span's padding, as the staging copy writes it (gpudiff.h: engine-owned)
                    memset((uint8_t*)src[k] + docs[k].json_len, 0, step(docs[k].json_len) - docs[k].json_len);
                }
                jbytes = (uint64_t)(at - zsrc);
                s->st.zero_copy_batches++;
            }
        }
    }
    jbytes += kTokSlack;
    if (!zsrc && (rc = grow_pinned(&R.hjson, &R.hjson_cap, jbytes))) return rc;
    const uint8_t* hsrc = zsrc ? zsrc : R.hjson;
    lap(1);
    // Chunks of the batch's JSON (by bytes, whole documents): the host copies chunk c into pinned
    // staging while chunk c - 1 is uploading, and K0 starts on a chunk as soon as it has landed, so
    // copy, upload and encode of one batch overlap instead of running back to back.
    auto first_doc = [&](uint64_t b) -> uint32_t {  // first document starting at or after byte b
        uint32_t lo = 0, hi = nd;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) / 2;
            if (docs[mid].json_off < b) lo = mid + 1;
            else hi = mid;
        }
        return lo;
    };
    const uint32_t C = (uint32_t)std::min<uint64_t>(
        std::min<uint64_t>(kMaxUpChunks, std::max<uint64_t>(1, nd / kMinChunkDocs)),
        std::max<uint64_t>(1, jbytes / kUpChunkBytes));
    uint32_t cdoc[kMaxUpChunks + 1];
    for (uint32_t q = 0; q <= C; q++) cdoc[q] = q == C ? nd : first_doc(jbytes * q / C);
    auto cbyte = [&](uint32_t q) -> uint64_t { return q == C || cdoc[q] >= nd ? jbytes : docs[cdoc[q]].json_off; };
    // K0 scratch: per-document areas within launches of at most kScratchCap, never across a chunk
    std::vector<std::pair<uint32_t, uint32_t>> launches;
    std::vector<uint32_t> chunk_of_launch;
    uint64_t max_sb = 0;  // the largest launch's scratch: one such area per K0 stream
    for (uint32_t q = 0; q < C; q++) {
        uint64_t sb = 0;
        uint32_t first = cdoc[q];
        for (uint32_t k = cdoc[q]; k < cdoc[q + 1]; k++) {
            const uint64_t need = tok_scratch_bytes(docs[k].json_len);
            if (sb && sb + need > std::max(kScratchCap, need)) {
                launches.emplace_back(first, k);
                chunk_of_launch.push_back(q);
                first = k;
                sb = 0;
            }
            docs[k].scratch_off = sb;
            sb += need;
            max_sb = std::max(max_sb, sb);
        }
        if (cdoc[q + 1] > first) {
            launches.emplace_back(first, cdoc[q + 1]);
            chunk_of_launch.push_back(q);
        }
    }
    const uint64_t scratch_half = (max_sb + 255u) & ~255ull;
    if ((rc = grow_dev(&s->scratch, &s->scratch_cap, s->ks ? 2 * scratch_half : scratch_half))) return rc;
    // 2. capacity (compaction is stream-ordered after every earlier batch)
    if ((rc = ensure_space(s, bound, floor))) return rc;
    // 3. upload + kernels
    if ((rc = grow_dev(&R.djson, &R.djson_cap, jbytes)) ||
        (rc = grow_dev(&R.dmeta, &R.dmeta_cap, meta_bytes)) || (rc = grow_dev(&R.douts, &R.docs_cap, nd + 1)))
        return rc;
    if ((rc = grow_dev(&R.dcoll, &R.coll_cap, nd + 1)) || (rc = grow_dev(&R.ddef, &R.def_cap, n + 1))) return rc;
    hipStream_t st = c->stream, cs = s->cs;
    hipStream_t k0s = dec ? s->ks0 : st;  // the K0 stage's stream (even chunks, K0c, K0x)
    if (timing && !R.t_ev[0])
        for (auto& e : R.t_ev) HIPCHK(hipEventCreate(&e));
    if (!R.chunk_ev[0])
        for (auto& e : R.chunk_ev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    // the upload runs on the copy stream, behind this ring slot's previous K0 (which read the
    // same device buffers), so it overlaps the other batch's K0 / diff pass
    if (R.k0_recorded) HIPCHK(hipStreamWaitEvent(cs, R.k0_done, 0));
    if (timing) HIPCHK(hipEventRecord(R.t_ev[0], cs));
    // the tables' used parts only (their device offsets are sized for 2n documents)
    HIPCHK(hipMemcpyAsync(R.dmeta, R.hmeta, (uint64_t)nd * sizeof(TokDoc), hipMemcpyHostToDevice, cs));
    HIPCHK(hipMemcpyAsync(R.dmeta + max_docs * sizeof(TokDoc), R.hmeta + max_docs * sizeof(TokDoc),
                          (uint64_t)nd * sizeof(DocLink), hipMemcpyHostToDevice, cs));
    HIPCHK(hipMemcpyAsync(R.dmeta + max_docs * (sizeof(TokDoc) + sizeof(DocLink)),
                          R.hmeta + max_docs * (sizeof(TokDoc) + sizeof(DocLink)), 4ull * nh + 4,
                          hipMemcpyHostToDevice, cs));
    // One run of the workers over all chunks: worker t copies its share of chunk 0, then of chunk
    // 1, ... and counts each chunk done; the calling thread (worker 0) enqueues a chunk's upload as
    // soon as every worker has counted it, then goes on with its own share of the next chunk.
    const uint32_t T = (uint32_t)std::min<uint64_t>(std::max(1u, c->threads), std::max<uint64_t>(1, jbytes >> 20));
    std::atomic<uint32_t> chunk_done[kMaxUpChunks];
    for (auto& x : chunk_done) x.store(0, std::memory_order_relaxed);
    std::atomic<int> up_err{0};
    uint32_t uploaded = 0;
    if (dec) {  // what this batch's K0 stage reuses: the slot table (the previous batch's K0x read it) and this
                // ring slot's space, douts and rows (its previous batch's diff pass read them)
        if (s->last_ring >= 0 && s->ring[s->last_ring].k0_recorded)
            HIPCHK(hipStreamWaitEvent(k0s, s->ring[s->last_ring].k0_done, 0));
        if (R.pass_recorded) HIPCHK(hipStreamWaitEvent(k0s, R.pass_done, 0));
        if (s->pair_mode) HIPCHK(hipMemsetAsync(s->used_dev, 0, 8, k0s));
        if (s->st_slot_ops) {  // store mode: a compaction, Delete or placement since the last K0 stage
            HIPCHK(hipEventRecord(s->st_ev, st));
            HIPCHK(hipStreamWaitEvent(k0s, s->st_ev, 0));
            s->st_slot_ops = false;
        }
    }
    if (s->pair_mode) HIPCHK(hipMemsetAsync(s->slots, 0, sizeof(DSlot) * n, k0s));  // every pair starts empty
    if (s->ks) {  // the second K0 stream starts behind everything before this batch's K0 on the K0 stage's stream
        HIPCHK(hipEventRecord(s->ks_ev, k0s));
        HIPCHK(hipStreamWaitEvent(s->ks, s->ks_ev, 0));
    }
    const TokDoc* ddocs = (const TokDoc*)R.dmeta;
    const DocLink* dlinks = (const DocLink*)(R.dmeta + max_docs * sizeof(TokDoc));
    const uint32_t* dheads = (const uint32_t*)(R.dmeta + max_docs * (sizeof(TokDoc) + sizeof(DocLink)));
    uint8_t* space = s->space[s->cur];
    size_t li = 0;  // next K0 launch
    // chunk q's K0 launches go on the kernel stream as soon as its upload is enqueued (behind its copy
    // event), so K0 of chunk q runs while chunk q + 1 is on the link -- not after the host has staged them all
    auto upload = [&](uint32_t q) {
        const uint64_t b0 = cbyte(q), b1 = cbyte(q + 1);
        if (!zsrc && q + 1 == C && cdoc[q] >= nd) memset(R.hjson + b0, 0, b1 - b0);  // no documents: the slack only
        hipStream_t qs = cs;  // one DMA queue saturates the link (two measured slower, profiles/r04z)
        const bool odd = (q & 1u) != 0u;
        hipStream_t kq = odd ? s->ks : k0s;  // this chunk's K0 stream, and its half of the scratch
        uint8_t* scr = s->scratch + (odd ? scratch_half : 0);
        if (hipMemcpyAsync(R.djson + b0, hsrc + b0, b1 - b0, hipMemcpyHostToDevice, qs) != hipSuccess ||
            hipEventRecord(R.chunk_ev[q], qs) != hipSuccess || hipStreamWaitEvent(kq, R.chunk_ev[q], 0) != hipSuccess ||
            (q == 0 && timing && hipEventRecord(R.t_ev[2], k0s) != hipSuccess)) {
            up_err.store(1);
            return;
        }
        for (; li < launches.size() && chunk_of_launch[li] == q; li++) {
            const auto& L = launches[li];
            if (launch_encode_docs(kq, ddocs + L.first, L.second - L.first, R.djson, scr, space, s->space_bytes,
                                   s->used_dev, c->hash_mask, R.douts + L.first, s->slots, dlinks + L.first) !=
                hipSuccess) {
                up_err.store(1);
                return;
            }
        }
    };
    if (zsrc)  // nothing to stage: every chunk's upload (and its K0 launches) goes out at once
        while (uploaded < C) upload(uploaded++);
    else
    workers(c).run(T, [&](uint32_t t) {
        for (uint32_t q = 0; q < C; q++) {
            const uint64_t b0 = cbyte(q), b1 = cbyte(q + 1);
            const uint32_t k0 = std::max(cdoc[q], first_doc(b0 + (b1 - b0) * t / T));
            const uint32_t k1 = std::min(cdoc[q + 1], first_doc(b0 + (b1 - b0) * (t + 1) / T));
            for (uint32_t k = k0; k < k1; k++) {
                const uint64_t o = docs[k].json_off;
                const uint64_t end = k + 1 < nd ? docs[k + 1].json_off : jbytes;
                stream_doc(R.hjson + o, src[k], docs[k].json_len, end - o);
            }
            _mm_sfence();  // the streaming stores are visible before the chunk counts as done
            chunk_done[q].fetch_add(1, std::memory_order_release);
            if (t == 0)  // upload every chunk all workers have finished, in order, without waiting
                while (uploaded <= q && chunk_done[uploaded].load(std::memory_order_acquire) >= T) upload(uploaded++);
        }
        if (t == 0)
            while (uploaded < C) {
                if (chunk_done[uploaded].load(std::memory_order_acquire) < T) {
                    std::this_thread::yield();
                    continue;
                }
                upload(uploaded++);
            }
    });
    if (up_err.load()) return GPUDIFF_E_DEVICE;
    lap(2);
    HIPCHK(hipEventRecord(R.staged, cs));
    if (timing) HIPCHK(hipEventRecord(R.t_ev[1], cs));
    if (li != launches.size()) return GPUDIFF_E_STATE;  // every launch belongs to an uploaded chunk
    if (s->ks) {  // K0c waits for the odd chunks' K0 too
        HIPCHK(hipEventRecord(s->ks_ev, s->ks));
        HIPCHK(hipStreamWaitEvent(k0s, s->ks_ev, 0));
    }
    HIPCHK(hipStreamWaitEvent(k0s, R.staged, 0));  // every chunk (and the tables) landed
    if (timing) HIPCHK(hipEventRecord(R.t_ev[3], k0s));
    HIPCHK(launch_collide(k0s, dlinks, R.douts, s->slots, nd, space, R.dcoll));
    HIPCHK(hipMemsetAsync(R.dcnt, 0, 4, k0s));
    gpudiff_dbatch* d = R.d;
    HIPCHK(launch_link(k0s, dheads, nh, dlinks, R.douts, R.dcoll, s->slots, d->rows, d->pair_ids, R.ddef, batch,
                       R.dcnt, s->ctr));
    HIPCHK(hipEventRecord(R.k0_done, k0s));
    R.k0_recorded = true;
    if (timing) HIPCHK(hipEventRecord(R.t_ev[4], k0s));
    if (dec) HIPCHK(hipStreamWaitEvent(st, R.k0_done, 0));  // the diff pass reads the rows K0x wrote
    s->used_ub += bound;
    // 4. the diff pass over the batch's rows
    d->pool = space;
    d->pool_cap = s->space_bytes;
    d->pool_used = s->used_ub;
    d->n_pairs = n;
    d->rows_gen++;
    d->leaves = 0;
    d->compare_bytes = d->value_bytes = 0;
    d->size_hint_bytes = 2 * new_json_bytes;  // k2_sub_shift's size class (engine.h)
    if ((rc = gpudiff_diff(c, d, ticket))) {
        s->broken = true;
        return rc;
    }
    if (dec) {  // this ring slot's next K0 stage may refill its space once this pass has read it
        HIPCHK(hipEventRecord(R.pass_done, st));
        R.pass_recorded = true;
    }
    s->last_ring = (int)(&R - s->ring);
    R.events.assign(ev, ev + n);
    R.waited = false;
    R.batch = batch;
    R.nev = (uint32_t)n;
    R.bound = bound;
    R.ticket = *ticket;
    R.outstanding = true;
    Ring* Rp = &R;
    c->finishers[*ticket] = [s, Rp](ResultStore& rs) -> int {
        const auto t_fin0 = std::chrono::steady_clock::now();
        Ring& RR = *Rp;
        RR.outstanding = false;
        if (!s->pair_mode) {
            if (RR.batch != s->next_wait) return GPUDIFF_E_STATE;  // waits follow submit order
            s->next_wait++;
        }
        uint32_t ndef = 0;
        uint64_t used = 0;
        if (s->pair_mode) {  // resolution appends to this batch's own space
            s->cur = (uint32_t)(Rp - s->ring);
            s->used_dev = s->used_base + s->cur;
        }
        HIPCHK(hipMemcpyAsync(&ndef, RR.dcnt, 4, hipMemcpyDeviceToHost, s->c->rb));  // behind K0x: d->done waited
        HIPCHK(hipMemcpyAsync(&used, s->used_dev, 8, hipMemcpyDeviceToHost, s->c->rb));
        HIPCHK(hipStreamSynchronize(s->c->rb));
        // exact append point + what the other batch in flight may still add
        const Ring& other = s->ring[(Rp - s->ring) ^ 1];
        s->used_ub = s->pair_mode ? used : std::max<uint64_t>(used, used + (other.outstanding ? other.bound : 0));
        if (RR.t_ev[0] && (s->c->flags & GPUDIFF_OPT_TIMING)) {
            float ms[3];
            HIPCHK(hipEventElapsedTime(&ms[0], RR.t_ev[0], RR.t_ev[1]));  // H2D
            HIPCHK(hipEventElapsedTime(&ms[1], RR.t_ev[2], RR.t_ev[3]));  // K0
            HIPCHK(hipEventElapsedTime(&ms[2], RR.t_ev[3], RR.t_ev[4]));  // K0c + K0x
            for (int k = 0; k < 3; k++) s->t_sum[1 + k] += ms[k];
            s->t_n++;
        }
        int r2 = ndef ? resolve(s, RR, rs) : GPUDIFF_OK;
        if (r2) s->broken = true;
        if (!r2 && s->pair_mode) {  // kept for gpudiff_write_plan_get
            RR.final_flags.assign(rs.flags.begin(), rs.flags.end());
            RR.waited = true;
        }
        // forgets older than every outstanding batch are settled
        for (auto it = s->forgotten.begin(); it != s->forgotten.end();)
            it = it->second < s->next_wait ? s->forgotten.erase(it) : std::next(it);
        s->t_sub[4] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_fin0).count();
        return r2;
    };
    s->ring_next ^= 1u;
    lap(3);
    if (timing)
        s->t_sum[0] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_host0).count();
    s->st.events += n;
    s->st.last_batch_bytes = jbytes;
    return GPUDIFF_OK;
}

int dstore_submit_pairs(gpudiff_ctx* c, const gpudiff_json_pair* pairs, size_t n, gpudiff_ticket* ticket) {
    DStore*& s = c->pair_store;
    uint64_t json = 0;
    for (size_t i = 0; i < n; i++) json += pairs[i].old_len + pairs[i].new_len;
    // one space per ring slot, each taking a whole batch: dstore_submit's bound (5/2 of the JSON + 384 B a
    // document), with half again as headroom so a growing batch does not recreate the store every time
    const uint64_t need = (5 * json) / 2 + 768 * (uint64_t)n + (1ull << 20);
    const uint64_t space = std::max<uint64_t>(512ull << 20, need + need / 2);
    if (!s || s->max_events < n || s->space_bytes < need) {
        if (s && (s->ring[0].outstanding || s->ring[1].outstanding))
            return GPUDIFF_E_CAPACITY;  // grows only between batches: gpudiff_submit encodes this one on the host
        if (s) dstore_free(c, s);
        s = nullptr;
        const uint32_t cap = (uint32_t)std::max<size_t>(65536, n + n / 2);
        int rc;
        s = dstore_create(c, cap, space, cap, &rc);
        if (!s) return rc;
        s->pair_mode = true;
    }
    std::vector<gpudiff_event> ev(n);
    for (size_t i = 0; i < n; i++) {
        const gpudiff_json_pair& p = pairs[i];
        ev[i] = gpudiff_event{(uint32_t)i, p.pair_id, p.cluster_id, 0, p.new_json, p.new_len, p.old_json, p.old_len};
        if (!p.new_json) {  // as gpudiff_encode_pairs: an absent object is a decode error
            static const uint8_t kNone[1] = {0};
            ev[i].new_json = kNone;
            ev[i].new_len = 0;
        }
    }
    return dstore_submit(c, s, ev.data(), n, ticket);
}

void dstore_timing_reset(DStore* s) {
    for (double& x : s->t_sum) x = 0;
    for (double& x : s->t_sub) x = 0;
    s->t_n = 0;
}

extern "C" int gpudiff_submit_stats_get(gpudiff_ctx* c, gpudiff_store_stats* out) {
    if (!c || !out) return GPUDIFF_E_INVAL;
    if (!c->pair_store) return GPUDIFF_E_STATE;
    return dstore_stats(c->pair_store, out);
}

extern "C" int gpudiff_host_alloc(gpudiff_ctx* c, size_t bytes, void** out) {
    if (!c || !out || !bytes) return GPUDIFF_E_INVAL;
    if (!c->has_device) return GPUDIFF_E_NODEVICE;
    HIPCHK(hipSetDevice(c->device));
    uint8_t* p = nullptr;
    if (hipHostMalloc((void**)&p, bytes, hipHostMallocDefault) != hipSuccess) return GPUDIFF_E_NOMEM;
    {
        std::lock_guard<std::mutex> lk(g_hb_mu);
        g_hb.push_back(HostBuf{c, p, (uint64_t)bytes});
    }
    *out = p;
    return GPUDIFF_OK;
}

extern "C" int gpudiff_host_free(gpudiff_ctx* c, void* p) {
    if (!c || !p) return GPUDIFF_E_INVAL;
    {
        std::lock_guard<std::mutex> lk(g_hb_mu);
        auto it = std::find_if(g_hb.begin(), g_hb.end(), [&](const HostBuf& h) { return h.c == c && h.p == p; });
        if (it == g_hb.end()) return GPUDIFF_E_INVAL;
        g_hb.erase(it);
    }
    if (c->has_device) (void)hipSetDevice(c->device);
    return hipHostFree(p) == hipSuccess ? GPUDIFF_OK : GPUDIFF_E_DEVICE;
}

void dstore_host_bufs_release(gpudiff_ctx* c) {
    std::lock_guard<std::mutex> lk(g_hb_mu);
    for (auto it = g_hb.begin(); it != g_hb.end();)
        if (it->c == c) {
            (void)hipHostFree(it->p);
            it = g_hb.erase(it);
        } else {
            ++it;
        }
}

int dstore_forget(gpudiff_ctx* c, DStore* s, uint32_t slot) {
    if (int rc = before_st_slot_op(s)) return rc;
    HIPCHK(launch_forget(c->stream, s->slots, slot, s->ctr));
    s->seen[slot] = 0;
    s->forgotten[slot] = s->batch_seq;
    return GPUDIFF_OK;
}

int dstore_stats(const DStore* s, gpudiff_store_stats* out) {
    *out = s->st;
    uint32_t ctr[4] = {0, 0, 0, 0};
    uint64_t used = 0;
    HIPCHK(hipSetDevice(s->c->device));
    HIPCHK(hipStreamSynchronize(s->c->stream));
    HIPCHK(hipMemcpy(ctr, s->ctr, 16, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(&used, s->used_dev, 8, hipMemcpyDeviceToHost));
    out->live_slots = ctr[kCtrLive];
    uint64_t lb;
    memcpy(&lb, ctr + kCtrLiveBytes, 8);
    out->live_bytes = lb;
    out->used_bytes = used;
    out->deferred = s->deferred_total;
    if (s->t_n) {
        out->host_submit_ms = (float)(s->t_sum[0] / s->t_n);
        out->h2d_ms = (float)(s->t_sum[1] / s->t_n);
        out->encode_ms = (float)(s->t_sum[2] / s->t_n);
        out->link_ms = (float)(s->t_sum[3] / s->t_n);
        float* sub[5] = {&out->submit_wait_ms, &out->submit_docs_ms, &out->submit_copy_ms, &out->submit_enqueue_ms,
                         &out->finish_ms};
        for (int k = 0; k < 5; k++) *sub[k] = (float)(s->t_sub[k] / s->t_n);
        out->timing_batches = (uint32_t)s->t_n;
    }
    return GPUDIFF_OK;
}

void dstore_free(gpudiff_ctx* c, DStore* s) {
    if (!s) return;
    if (c && c->has_device) {
        (void)hipSetDevice(c->device);
        (void)hipStreamSynchronize(c->stream);
        if (s->cs) (void)hipStreamSynchronize(s->cs);
    }
    for (Ring& R : s->ring) {
        if (R.d) gpudiff_dbatch_free(c, R.d);
        if (R.ticket) c->finishers.erase(R.ticket);
        for (void* p : {(void*)R.djson, (void*)R.dmeta, (void*)R.douts, (void*)R.dcoll, (void*)R.ddef, (void*)R.dcnt})
            if (p) (void)hipFree(p);
        for (void* p : {(void*)R.hjson, (void*)R.hmeta})
            if (p) (void)hipHostFree(p);
        if (R.staged) (void)hipEventDestroy(R.staged);
        if (R.k0_done) (void)hipEventDestroy(R.k0_done);
        for (auto& e : R.t_ev)
            if (e) (void)hipEventDestroy(e);
        for (auto& e : R.chunk_ev)
            if (e) (void)hipEventDestroy(e);
    }
    if (s->res_d) gpudiff_dbatch_free(c, s->res_d);
    for (hipStream_t* k : {&s->ks, &s->ks0})
        if (*k) {
            (void)hipStreamSynchronize(*k);
            (void)hipStreamDestroy(*k);
        }
    for (Ring& R : s->ring)
        if (R.pass_done) (void)hipEventDestroy(R.pass_done);
    if (s->st_ev) (void)hipEventDestroy(s->st_ev);
    if (s->ks_ev) (void)hipEventDestroy(s->ks_ev);
    if (s->cs) {
        (void)hipStreamSynchronize(s->cs);
        (void)hipStreamDestroy(s->cs);
    }
    for (void* p : {(void*)s->space[0], (void*)s->space[1], (void*)s->used_base, (void*)s->slots, (void*)s->ctr,
                    (void*)s->sizes, (void*)s->tile_sums, (void*)s->scratch, (void*)s->res_stage, (void*)s->res_ups,
                    (void*)s->res_err})
        if (p) (void)hipFree(p);
    delete s;
}

int dstore_staged_pairs(gpudiff_ctx* c, gpudiff_ticket t, StagedPairs* out) {
    DStore* s = c->pair_store;
    if (!s || !t) return GPUDIFF_E_STATE;
    for (Ring& R : s->ring) {
        if (R.ticket != t) continue;
        if (!R.waited || R.outstanding) return GPUDIFF_E_STATE;  // gpudiff_wait first
        const uint64_t max_docs = 2 * (uint64_t)R.nev;
        (void)max_docs;
        out->hdocs = (const TokDoc*)R.hmeta;
        out->djson = R.djson;
        out->n = R.nev;
        out->flags = &R.final_flags;
        out->events = &R.events;
        return GPUDIFF_OK;
    }
    return GPUDIFF_E_STATE;  // not a device-encoded batch, or its staging was reused
}

int dstore_staged_mark_read(gpudiff_ctx* c, gpudiff_ticket t) {
    DStore* s = c->pair_store;
    if (!s) return GPUDIFF_E_STATE;
    for (Ring& R : s->ring)
        if (R.ticket == t) {
            HIPCHK(hipEventRecord(R.k0_done, c->stream));
            R.k0_recorded = true;
            return GPUDIFF_OK;
        }
    return GPUDIFF_E_STATE;
}
