// Device-encode mode of the object store (dstore.cpp); internal.
#pragma once
#include "engine.h"
#include "tokenize.h"

struct DStore;

DStore* dstore_create(gpudiff_ctx* c, uint32_t max_slots, uint64_t space_bytes, uint32_t max_events, int* rc);
int dstore_submit(gpudiff_ctx* c, DStore* s, const gpudiff_event* ev, size_t n, gpudiff_ticket* ticket);
int dstore_forget(gpudiff_ctx* c, DStore* s, uint32_t slot);
// gpudiff_submit with GPUDIFF_OPT_DEVICE_ENCODE: pairs through K0 (c->pair_store);
// GPUDIFF_E_CAPACITY = take the host-encode path for this batch
int dstore_submit_pairs(gpudiff_ctx* c, const gpudiff_json_pair* pairs, size_t n, gpudiff_ticket* ticket);
int dstore_stats(const DStore* s, gpudiff_store_stats* out);
void dstore_timing_reset(DStore* s);  // gpudiff_timing_reset: the submit path's phase sums too
void dstore_free(gpudiff_ctx* c, DStore* s);
void dstore_host_bufs_release(gpudiff_ctx* c);  // gpudiff_close: the context's remaining gpudiff_host_alloc buffers

// The staged JSON of a waited pair-mode batch (gpudiff_submit with GPUDIFF_OPT_DEVICE_ENCODE): pair i's
// old object is document 2i, its new one 2i + 1; hdocs[] holds their offsets into djson (HBM); flags = the
// batch's final result flags (host-deferred pairs resolved).  Valid until the ring slot is reused by the
// submit after the next one.  There is no host copy to offer: a zero-copy batch was uploaded from the
// caller's buffer (reusable once gpudiff_wait returned), so host work on a staged document reads it back
// from djson.
struct StagedPairs {
    const gd::TokDoc* hdocs = nullptr;
    const uint8_t* djson = nullptr;
    uint32_t n = 0;
    const std::vector<uint8_t>* flags = nullptr;
    const std::vector<gpudiff_event>* events = nullptr;
};
int dstore_staged_pairs(gpudiff_ctx* c, gpudiff_ticket t, StagedPairs* out);
// work launched on the context stream now reads the batch's device JSON: the ring slot's next upload waits
int dstore_staged_mark_read(gpudiff_ctx* c, gpudiff_ticket t);
