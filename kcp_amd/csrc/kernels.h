// Launchers of the gpudiff HIP kernels (kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gpudiff_format.h"

namespace gd {

// K4 slices: a sliced deferral's scratch is a whole number of kJoinSlice-entry slots
constexpr uint32_t kJoinSliceHost = 1024;  // = kJoinSlice in kernels.hip
// the K4 scratch's limit: a deferred pair's offset shares a u32 with the arena bit (scratch_off); a batch
// whose deferred joins need more (summary[3] saturates at 2^32 - 1 past u32) fails with GPUDIFF_E_CAPACITY
constexpr uint64_t kMaxScratchEntries = 1ull << 31;

// Device buffers of one diff pass.  summary[]: 0 n_spec, 1 n_status,
// 2 n_dirty, 3 K4 scratch entries (saturating), 4 overflow, 5 n_paths, 6 any pair deferred to K4, 7 -.
struct DiffBuffers {
    const gpudiff_pair_row* rows;
    const uint8_t* pool;
    const uint32_t* pair_ids;
    uint32_t n_pairs;
    uint8_t* flags;
    uint32_t* caps;
    uint32_t* path_src;   // per pair: arena index of the paths K2 wrote
    uint32_t* path_cnt;   // per pair: number of those paths
    uint8_t* nbits;       // per pair: write-path no-op bits K2 computed (NOOP_SPEC | NOOP_STATUS)
    uint8_t* noop_d;      // per dirty pair (dirty order): the no-op bits (K3 copies K2's, K4 writes its own)
    void* chunk_counts;   // uint4 per 64 pairs
    uint32_t* summary;
    uint32_t* spec_ids;
    uint32_t* status_ids;
    uint32_t* dirty_ids;
    uint32_t* dirty_idx;
    uint32_t* scratch_off;  // per dirty pair: K4 scratch slot, or ARENA_BIT | arena index
    uint32_t* path_count;
    uint32_t* path_off;     // n_dirty + 1
    uint32_t* tile_sums;
    uint64_t* arena_h;      // K2 wave arenas (arena_per_wave entries per K2 wave)
    uint8_t* arena_k;
    uint32_t arena_per_wave;
    uint64_t* scratch_h;    // K4 scratch for deferred pairs
    uint8_t* scratch_k;
    uint64_t scratch_cap;
    uint32_t* slot_owner;   // per K4 slice slot of the scratch (kJoinSlice entries): its dirty pair, or
                            // ~0 inside a whole deferral's entries (K3)
    uint32_t* slice_cnt;    // per slot: paths its slice wrote (K4a)
    uint8_t* slice_weq;     // per slot: every path a wire-equal number change (K4a)
    uint64_t* out_h;
    uint8_t* out_k;
    uint64_t hash_mask;
    uint32_t k2_timeline;       // gpudiff_k2_profile installed a buffer: the per-wave timeline build of K2
    uint32_t k2_shared;         // another pass over the same population is in flight: K2 takes half the chip
    uint32_t* tail_perm;        // K2's largest-first final round: its order (device, kK2LptMax u32)
    struct TailPermKey* tail_perm_key;  // (host) the rows and launch shape tail_perm was computed for
    uint64_t rows_gen;          // bumped whenever the batch's rows change (appends, resets, store batches)
    uint64_t avg_pair_bytes;    // format bytes K2 reads per pair, averaged over the batch (0: unknown)
    uint32_t* gather_send;      // gpudiff_dbatch_bind_gather: K3 also writes counts + IDs here (nullptr: unbound)
    uint32_t gather_cap_spec, gather_cap_status;
};

// the exact launch a cached largest-first order was computed for (kernels.hip launch_compare)
struct TailPermKey {
    const void* rows = nullptr;
    uint64_t rows_gen = ~0ull;
    uint32_t n_pairs = 0, lpt = 0, sub = 0, r2 = 0;
    bool operator==(const TailPermKey& o) const {
        return rows == o.rows && rows_gen == o.rows_gen && n_pairs == o.n_pairs && lpt == o.lpt && sub == o.sub &&
               r2 == o.r2;
    }
};

// summary[8]: K2's main item counter; summary[8 + kK2TailCounters]: its tail item counter (zeroed with the pass)
constexpr uint32_t kK2TailCounters = 8, kSummaryWords = 8 + 2 * kK2TailCounters;
// default tail: half a chunk per resident wave, in items of half a main item (in-process A/B on MI355X,
// profiles/r02zj-r02zm: 8-pair tail items cost more than the imbalance they remove; with no tail at all
// the main items' tickets are fetched late in the last two rounds instead)
constexpr uint32_t kK2TailQuarters = 2;

// waves of a K2 launch over nchunks 64-pair chunks (sizes the wave arenas)
uint32_t k2_grid_waves(const DiffBuffers& b, uint32_t nchunks);

hipError_t launch_rebase(hipStream_t s, gpudiff_pair_row* rows, uint32_t begin, uint32_t end, uint64_t base,
                         uint32_t* pair_ids);
// object-store compaction: blob copies between the two spaces
struct BlobMove {
    uint64_t src, dst, bytes;
};
hipError_t launch_move_blobs(hipStream_t s, const uint8_t* src, uint8_t* dst, const BlobMove* moves, uint32_t n);
// K2 (+ fused join) over the whole batch; zeroes the pass's summary first
hipError_t launch_compare(hipStream_t s, const DiffBuffers& b);
// K3 over chunks [c0, c1): running (n_spec, n_status, n_dirty, cap) totals before -> after
hipError_t launch_compact(hipStream_t s, const DiffBuffers& b, uint32_t c0, uint32_t c1, const uint4* before,
                          uint4* after);
// K4 over the deferred dirty pairs the segment added (before.z .. after.z)
// K4's slot owners again (the scratch-overflow re-run of K4-K6)
hipError_t launch_slot_owners(hipStream_t s, const DiffBuffers& b);
hipError_t launch_join(hipStream_t s, const DiffBuffers& b, uint32_t c0, uint32_t c1, const uint4* before,
                       const uint4* after);
hipError_t launch_emit(hipStream_t s, const DiffBuffers& b);
// profiling hook: the timeline build (gpudiff_k2_profile) of K2 writes 12 u64 per wave (start, first item end, items,
// last item start, end, streaming ticks, join ticks, hw id, rows, pre, post, ticket ticks) into dev_buf
// (cap_waves waves); nullptr disables
hipError_t k2_profile(uint64_t* dev_buf, uint32_t cap_waves);

}  // namespace gd
