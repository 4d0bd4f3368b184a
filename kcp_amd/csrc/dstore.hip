// Device object store kernels (gfx950, wave64): the device-encode mode of
// gpudiff_store (include/gpudiff.h), where raw JSON goes up and everything
// else -- encoding (K0, tokenize.hip), collision checks, slot chains,
// compaction -- stays in HBM.
//
//   K0c k_collide        wave per event: every path-table node of the new blob
//                        is looked up in its old side's table (the previous
//                        document of the slot in this batch, else the slot's
//                        resident blob) by a lane-parallel binary search; an
//                        equal hash whose parent hash or component (key bytes,
//                        index) differs is a path-hash collision (host re-seeds)
//   K0x k_link           lane per slot chain: walks the slot's documents in
//                        batch order, writes each event's (old, new) row for the
//                        diff pass or defers the rest of the chain to the host,
//                        and makes the last encoded version resident
//   K8  k_slot_sizes / k_scan_* / k_pack_slots   compaction of the live blobs
//                        into the other space
//   K9  k_place          host-resolved blobs, rows and slot states
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gpudiff.h"
#include "tokenize.h"

namespace gd {

namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }
__device__ __forceinline__ uint64_t seg_bytes(uint32_t l, uint32_t arena) { return (uint64_t)l * 16u + arena; }

struct BlobRef {
    uint64_t off;
    uint32_t sl, sar, tl, tar;
    uint32_t oflags;  // GPUDIFF_OBJ_HAS_STATUS
    uint32_t ntab;    // path-table entries
};

__device__ __forceinline__ BlobRef ref_of(const TokOut& o) {
    return BlobRef{o.off, o.spec_l, o.spec_ar, o.stat_l, o.stat_ar, o.oflags, o.n_tab};
}
__device__ __forceinline__ BlobRef ref_of(const DSlot& s) {
    return BlobRef{s.off, s.spec_l, s.spec_ar, s.stat_l, s.stat_ar,
                   (s.flags & DS_HAS_STATUS) ? GPUDIFF_OBJ_HAS_STATUS : 0u, s.n_tab};
}

}  // namespace

// ---------------------------------------------------------------- K0c
__global__ __launch_bounds__(256) void k_collide(const DocLink* __restrict__ links, const TokOut* __restrict__ outs,
                                                 const DSlot* __restrict__ slots, uint32_t n,
                                                 const uint8_t* __restrict__ space, uint8_t* __restrict__ coll) {
    const uint32_t lane = lane_id();
    const uint32_t e = __builtin_amdgcn_readfirstlane((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    if (e >= n) return;
    const DocLink L = links[e];
    const TokOut B = outs[e];
    bool have_a = false;
    BlobRef A{};
    if (L.row != kNoRow && B.status == GPUDIFF_TOK_OK) {
        if (L.prev >= 0) {
            const TokOut P = outs[L.prev];
            if (P.status == GPUDIFF_TOK_OK) {
                A = ref_of(P);
                have_a = true;
            }
        } else {
            const DSlot S = slots[L.slot];
            if ((S.flags & DS_LIVE) && !(S.flags & DS_PENDING)) {
                A = ref_of(S);
                have_a = true;
            }
        }
    }
    bool bad = have_a && A.ntab == GPUDIFF_TAB_NONE;  // stored without a valid table: old_json decides
    if (have_a && !bad && B.n_tab && A.ntab) {
        // the path tables (include/gpudiff_format.h): a hash both hold must have the same parent
        // hash and the same last component in each
        const uint32_t na = A.ntab, nb = B.n_tab;
        // each table at its blob's body end (gpudiff_blob_body: the segments rounded up to 128 B)
        const uint64_t* ha = (const uint64_t*)(space + A.off + ((seg_bytes(A.sl, A.sar) + seg_bytes(A.tl, A.tar) + 127u) & ~127ull));
        const uint64_t* hb = (const uint64_t*)(space + B.off + ((seg_bytes(B.spec_l, B.spec_ar) +
                                                                 seg_bytes(B.stat_l, B.stat_ar) + 127u) & ~127ull));
        const uint8_t* ka = (const uint8_t*)(ha + 3ull * na);
        const uint8_t* kb = (const uint8_t*)(hb + 3ull * nb);
        for (uint32_t i = lane; i < nb; i += 64) {
            const uint64_t k = hb[i];
            uint32_t lo = 0, hi = na;
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (ha[mid] < k) lo = mid + 1;
                else hi = mid;
            }
            if (lo < na && ha[lo] == k) {
                const uint64_t ca = ha[2ull * na + lo], cb = hb[2ull * nb + i];
                const bool ia = (ca & GPUDIFF_TAB_INDEX) != 0, ib = (cb & GPUDIFF_TAB_INDEX) != 0;
                if (ha[na + lo] != hb[nb + i] || ia != ib || (ia && ca != cb)) {
                    bad = true;
                } else if (!ia) {
                    const uint32_t l = (uint32_t)(ca >> 32);
                    if (l != (uint32_t)(cb >> 32)) {
                        bad = true;
                    } else {
                        const uint8_t* x = ka + (uint32_t)ca;
                        const uint8_t* y = kb + (uint32_t)cb;
                        for (uint32_t q = 0; q < l; q++)
                            if (x[q] != y[q]) bad = true;
                    }
                }
            }
        }
    }
    const bool any = __ballot(bad) != 0ull;
    if (lane == 0) coll[e] = any ? 1 : 0;
}

// ---------------------------------------------------------------- K0x
__global__ __launch_bounds__(256) void k_link(const uint32_t* __restrict__ heads, uint32_t n_heads,
                                              const DocLink* __restrict__ links, const TokOut* __restrict__ outs,
                                              const uint8_t* __restrict__ coll, DSlot* __restrict__ slots,
                                              gpudiff_pair_row* __restrict__ rows, uint32_t* __restrict__ pair_ids,
                                              uint8_t* __restrict__ deferred, uint32_t batch,
                                              uint32_t* __restrict__ n_deferred, uint32_t* __restrict__ counters) {
    const uint32_t h = blockIdx.x * blockDim.x + threadIdx.x;
    if (h >= n_heads) return;
    int32_t doc = (int32_t)heads[h];
    const uint32_t slot = links[doc].slot;
    const DSlot S0 = slots[slot];
    const bool was_live = S0.flags & DS_LIVE;
    bool defer = (S0.flags & DS_PENDING) != 0;
    const uint32_t seed = (S0.flags >> 8) & 0xFFu;
    bool have_a = was_live && !defer;
    BlobRef A = have_a ? ref_of(S0) : BlobRef{0, 0, 0, 0, 0, 0, 0};
    uint32_t a_bytes = S0.bytes;
    bool changed = false;
    uint32_t n_def = 0;
    for (; doc >= 0; doc = links[doc].next) {
        const DocLink L = links[doc];
        const TokOut o = outs[doc];
        if (L.row == kNoRow) {  // first sighting's old object: the old side of the next event
            if (!defer && o.status == GPUDIFF_TOK_OK) {
                A = ref_of(o);
                a_bytes = o.bytes;
                have_a = true;
            } else {
                defer = true;
            }
            continue;
        }
        if (!defer && (o.status != GPUDIFF_TOK_OK || coll[doc])) defer = true;
        gpudiff_pair_row r{};
        r.pair_id = L.pair_id;
        r.cluster_id = L.cluster_id;
        pair_ids[L.row] = L.pair_id;
        if (defer) {  // conservative until the host resolves it (gpudiff_wait)
            r.flags_a = r.flags_b = GPUDIFF_OBJ_DECODE_ERR;
            rows[L.row] = r;
            deferred[L.row] = 1;
            n_def++;
            continue;
        }
        deferred[L.row] = 0;
        r.off_a = have_a ? A.off : 0;
        r.spec_l_a = have_a ? A.sl : 0;
        r.spec_ar_a = have_a ? A.sar : 0;
        r.stat_l_a = have_a ? A.tl : 0;
        r.stat_ar_a = have_a ? A.tar : 0;
        r.flags_a = (have_a ? A.oflags : 0u) | (seed << GPUDIFF_OBJ_SEED_SHIFT);
        r.off_b = o.off;
        r.spec_l_b = o.spec_l;
        r.spec_ar_b = o.spec_ar;
        r.stat_l_b = o.stat_l;
        r.stat_ar_b = o.stat_ar;
        r.flags_b = o.oflags | (seed << GPUDIFF_OBJ_SEED_SHIFT);
        rows[L.row] = r;
        A = ref_of(o);
        a_bytes = o.bytes;
        have_a = true;
        changed = true;
    }
    if (changed) {
        DSlot N{};
        N.off = A.off;
        N.spec_l = A.sl;
        N.spec_ar = A.sar;
        N.stat_l = A.tl;
        N.stat_ar = A.tar;
        N.bytes = a_bytes;
        N.n_tab = A.ntab;
        N.flags = DS_LIVE | ((A.oflags & GPUDIFF_OBJ_HAS_STATUS) ? DS_HAS_STATUS : 0u) | (seed << 8) |
                  (defer ? DS_PENDING : 0u);
        N.pend = defer ? batch : S0.pend;
        slots[slot] = N;
        atomicAdd(&counters[kCtrLive], was_live ? 0u : 1u);
        atomicAdd((unsigned long long*)(counters + kCtrLiveBytes),
                  (unsigned long long)((uint64_t)a_bytes - (was_live ? (uint64_t)S0.bytes : 0ull)));
    } else if (defer) {
        slots[slot].flags = S0.flags | DS_PENDING;
        slots[slot].pend = batch;
    }
    if (n_def) atomicAdd(n_deferred, n_def);
}

// ---------------------------------------------------------------- K8: compaction
__global__ __launch_bounds__(256) void k_slot_sizes(const DSlot* __restrict__ slots, uint32_t n,
                                                    uint64_t* __restrict__ sizes) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) sizes[i] = (slots[i].flags & DS_LIVE) ? slots[i].bytes : 0ull;
}

// exclusive scan of u64 in tiles of 1024 (256 threads x 4): tile sums, then
// a one-block scan of the tile sums, then each tile rescans with its base
constexpr uint32_t kTile = 1024;

__device__ uint64_t block_excl_scan(uint64_t v, uint64_t* tmp, uint64_t* total) {
    const uint32_t t = threadIdx.x;
    tmp[t] = v;
    __syncthreads();
    for (uint32_t d = 1; d < blockDim.x; d <<= 1) {
        const uint64_t o = t >= d ? tmp[t - d] : 0ull;
        __syncthreads();
        tmp[t] += o;
        __syncthreads();
    }
    const uint64_t incl = tmp[t];
    *total = tmp[blockDim.x - 1];
    __syncthreads();
    return incl - v;
}

__global__ __launch_bounds__(256) void k_scan_tiles_u64(const uint64_t* __restrict__ in, uint32_t n,
                                                        uint64_t* __restrict__ tile_sums) {
    __shared__ uint64_t tmp[256];
    const uint32_t base = blockIdx.x * kTile + threadIdx.x * 4;
    uint64_t s = 0;
    for (uint32_t k = 0; k < 4; k++)
        if (base + k < n) s += in[base + k];
    uint64_t total;
    (void)block_excl_scan(s, tmp, &total);
    if (threadIdx.x == 0) tile_sums[blockIdx.x] = total;
}

__global__ __launch_bounds__(256) void k_scan_top_u64(uint64_t* __restrict__ tile_sums, uint32_t n_tiles,
                                                      unsigned long long* __restrict__ used) {
    __shared__ uint64_t tmp[256];
    uint64_t run = 0;
    for (uint32_t b = 0; b < n_tiles; b += 256) {
        const uint32_t i = b + threadIdx.x;
        const uint64_t v = i < n_tiles ? tile_sums[i] : 0ull;
        uint64_t total;
        const uint64_t ex = block_excl_scan(v, tmp, &total);
        if (i < n_tiles) tile_sums[i] = run + ex;
        run += total;
    }
    if (threadIdx.x == 0) *used = run;
}

__global__ __launch_bounds__(256) void k_pack_slots(DSlot* __restrict__ slots, uint32_t n,
                                                    const uint64_t* __restrict__ sizes,
                                                    const uint64_t* __restrict__ tile_base,
                                                    const uint8_t* __restrict__ src, uint8_t* __restrict__ dst) {
    __shared__ uint64_t tmp[256];
    __shared__ uint64_t offs[kTile];
    const uint32_t tile0 = blockIdx.x * kTile;
    const uint32_t base = tile0 + threadIdx.x * 4;
    uint64_t v[4], s = 0;
    for (uint32_t k = 0; k < 4; k++) {
        v[k] = base + k < n ? sizes[base + k] : 0ull;
        s += v[k];
    }
    uint64_t total;
    uint64_t ex = block_excl_scan(s, tmp, &total) + tile_base[blockIdx.x];
    for (uint32_t k = 0; k < 4; k++) {
        offs[threadIdx.x * 4 + k] = ex;
        ex += v[k];
    }
    __syncthreads();
    // wave per live blob: 16-B copies
    const uint32_t lane = lane_id(), wave = threadIdx.x >> 6;
    for (uint32_t j = wave; j < kTile; j += blockDim.x >> 6) {
        const uint32_t i = tile0 + j;
        if (i >= n) break;
        const DSlot S = slots[i];
        if (!(S.flags & DS_LIVE)) continue;
        const u32x4* s4 = (const u32x4*)(src + S.off);
        u32x4* d4 = (u32x4*)(dst + offs[j]);
        for (uint32_t k = lane; k < (S.bytes >> 4); k += 64) d4[k] = __builtin_nontemporal_load(s4 + k);
        if (lane == 0) slots[i].off = offs[j];
    }
}

// ---------------------------------------------------------------- K9: host-resolved state
__global__ __launch_bounds__(256) void k_place(const uint8_t* __restrict__ stage, uint64_t bytes,
                                               uint8_t* __restrict__ space, unsigned long long* __restrict__ used,
                                               uint64_t cap, gpudiff_pair_row* __restrict__ rows,
                                               uint32_t* __restrict__ pair_ids, uint32_t n_rows,
                                               const SlotUpdate* __restrict__ ups, uint32_t n_ups,
                                               DSlot* __restrict__ slots, uint32_t* __restrict__ counters,
                                               uint32_t* __restrict__ err) {
    __shared__ uint64_t base;
    if (threadIdx.x == 0) {
        base = bytes ? atomicAdd(used, (unsigned long long)bytes) : 0ull;
        if (base + bytes > cap) *err = 1u;
    }
    __syncthreads();
    if (base + bytes > cap) return;
    const uint4* s4 = (const uint4*)stage;
    uint4* d4 = (uint4*)(space + base);
    for (uint64_t k = threadIdx.x; k < (bytes >> 4); k += blockDim.x) d4[k] = s4[k];
    auto fix = [&](uint64_t off) -> uint64_t {
        if (off & kRelTag) return base + (off & ~kRelTag);
        if (off & kSlotTag) return slots[(uint32_t)off].off;
        return off;
    };
    for (uint32_t i = threadIdx.x; i < n_rows; i += blockDim.x) {
        rows[i].off_a = fix(rows[i].off_a);
        rows[i].off_b = fix(rows[i].off_b);
        pair_ids[i] = rows[i].pair_id;
    }
    __syncthreads();  // rows read the slots as they were before the updates below
    if (threadIdx.x == 0) {  // in order: a slot may be updated more than once
        for (uint32_t u = 0; u < n_ups; u++) {
            const SlotUpdate U = ups[u];
            const DSlot old = slots[U.slot];
            DSlot N = U.entry;
            N.off = fix(N.off);
            // a later batch deferred on this slot too: it stays pending for that batch
            const bool later = (old.flags & DS_PENDING) && old.pend != U.batch;
            if (later) {
                N.flags |= DS_PENDING;
                N.pend = old.pend;
            } else {
                N.flags &= ~DS_PENDING;
                N.pend = old.pend;
            }
            slots[U.slot] = N;
            const bool wl = old.flags & DS_LIVE, nl = N.flags & DS_LIVE;
            counters[kCtrLive] += (uint32_t)((int32_t)nl - (int32_t)wl);
            *(unsigned long long*)(counters + kCtrLiveBytes) +=
                (unsigned long long)((nl ? (uint64_t)N.bytes : 0ull) - (wl ? (uint64_t)old.bytes : 0ull));
        }
    }
}

__global__ void k_forget(DSlot* __restrict__ slots, uint32_t slot, uint32_t* __restrict__ counters) {
    const DSlot old = slots[slot];
    if (old.flags & DS_LIVE) {
        counters[kCtrLive] -= 1u;
        *(unsigned long long*)(counters + kCtrLiveBytes) -= (unsigned long long)old.bytes;
    }
    DSlot z{};
    slots[slot] = z;
}

// ---------------------------------------------------------------- launchers
hipError_t launch_collide(hipStream_t s, const DocLink* links, const TokOut* outs, const DSlot* slots, uint32_t n,
                          const uint8_t* space, uint8_t* coll) {
    if (!n) return hipSuccess;
    k_collide<<<(n + 3) / 4, 256, 0, s>>>(links, outs, slots, n, space, coll);
    return hipGetLastError();
}

hipError_t launch_link(hipStream_t s, const uint32_t* heads, uint32_t n_heads, const DocLink* links,
                       const TokOut* outs, const uint8_t* coll, DSlot* slots, gpudiff_pair_row* rows,
                       uint32_t* pair_ids, uint8_t* deferred, uint32_t batch, uint32_t* n_deferred,
                       uint32_t* counters) {
    if (!n_heads) return hipSuccess;
    k_link<<<(n_heads + 255) / 256, 256, 0, s>>>(heads, n_heads, links, outs, coll, slots, rows, pair_ids, deferred,
                                                  batch, n_deferred, counters);
    return hipGetLastError();
}

hipError_t launch_compact_store(hipStream_t s, DSlot* slots, uint32_t n, const uint8_t* src, uint8_t* dst,
                                uint64_t* sizes, uint64_t* block_sums, unsigned long long* used) {
    const uint32_t tiles = (n + kTile - 1) / kTile;
    k_slot_sizes<<<(n + 255) / 256, 256, 0, s>>>(slots, n, sizes);
    k_scan_tiles_u64<<<tiles, 256, 0, s>>>(sizes, n, block_sums);
    k_scan_top_u64<<<1, 256, 0, s>>>(block_sums, tiles, used);
    k_pack_slots<<<tiles, 256, 0, s>>>(slots, n, sizes, block_sums, src, dst);
    return hipGetLastError();
}

hipError_t launch_place(hipStream_t s, const uint8_t* stage, uint64_t bytes, uint8_t* space,
                        unsigned long long* used, uint64_t cap, gpudiff_pair_row* rows, uint32_t* pair_ids,
                        uint32_t n_rows, const SlotUpdate* ups, uint32_t n_ups, DSlot* slots, uint32_t* counters,
                        uint32_t* err) {
    k_place<<<1, 256, 0, s>>>(stage, bytes, space, used, cap, rows, pair_ids, n_rows, ups, n_ups, slots, counters,
                              err);
    return hipGetLastError();
}

hipError_t launch_forget(hipStream_t s, DSlot* slots, uint32_t slot, uint32_t* counters) {
    k_forget<<<1, 1, 0, s>>>(slots, slot, counters);
    return hipGetLastError();
}

}  // namespace gd
