// Device-encode mode of the object store (dstore.cpp); internal.
#pragma once
#include "engine.h"

struct DStore;

DStore* dstore_create(gpudiff_ctx* c, uint32_t max_slots, uint64_t space_bytes, uint32_t max_events, int* rc);
int dstore_submit(gpudiff_ctx* c, DStore* s, const gpudiff_event* ev, size_t n, gpudiff_ticket* ticket);
int dstore_forget(gpudiff_ctx* c, DStore* s, uint32_t slot);
int dstore_stats(const DStore* s, gpudiff_store_stats* out);
void dstore_free(gpudiff_ctx* c, DStore* s);
