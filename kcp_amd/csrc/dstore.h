// Device-encode mode of the object store (dstore.cpp); internal.
#pragma once
#include "engine.h"

struct DStore;

DStore* dstore_create(gpudiff_ctx* c, uint32_t max_slots, uint64_t space_bytes, uint32_t max_events, int* rc);
int dstore_submit(gpudiff_ctx* c, DStore* s, const gpudiff_event* ev, size_t n, gpudiff_ticket* ticket);
int dstore_forget(gpudiff_ctx* c, DStore* s, uint32_t slot);
// gpudiff_submit with GPUDIFF_OPT_DEVICE_ENCODE: pairs through K0 (c->pair_store);
// GPUDIFF_E_CAPACITY = take the host-encode path for this batch
int dstore_submit_pairs(gpudiff_ctx* c, const gpudiff_json_pair* pairs, size_t n, gpudiff_ticket* ticket);
int dstore_stats(const DStore* s, gpudiff_store_stats* out);
void dstore_free(gpudiff_ctx* c, DStore* s);
