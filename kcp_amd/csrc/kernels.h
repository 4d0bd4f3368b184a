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
    uint32_t k2_variant;        // tuning: 0 = by batch shape (k2_variant_of: 8 or 16 x 16-B chunks in flight per lane per object)
    uint32_t k2_items_per_wave; // tuning: 0 = default; 64-pair chunks split until each resident wave has this many items
    uint32_t k2_blocks_per_cu;  // tuning: 0 = the variant's occupancy (4 resident 256-thread blocks per CU)
    uint32_t k2_tail_quarters;  // tuning: a tail of (this - 1) / 4 x the launch's waves chunks; 0 = default
    uint32_t k2_tail8;          // tuning: tail items of 8 pairs instead of half a main item
    uint32_t* tail_perm;        // K2's largest-first final round: its order (device, kK2LptMax u32)
    uint64_t* tail_perm_key;    // (host) the launch shape tail_perm was computed for
    uint32_t k2_no_lpt;         // tuning (GPUDIFF_OPT_K2_NO_LPT): the final round in index order
    uint64_t avg_pair_bytes;    // format bytes K2 reads per pair, averaged over the batch (0: unknown)
    uint32_t k4_pipelined;      // tuning (GPUDIFF_OPT_K4_PIPELINED_JOIN): K4's slices with join_region_pl
    uint32_t* gather_send;      // gpudiff_dbatch_bind_gather: K3 also writes counts + IDs here (nullptr: unbound)
    uint32_t gather_cap_spec, gather_cap_status;
    uint32_t k2_deep_mode;      // tuning (GPUDIFF_OPT_K2_DEEP_SHIFT): 0 defer joins over 2048 keys to K4's
                                // slices, 1 keep every join in K2, 2 / 3 defer over 4096 / 8192
};

// summary[8 + seg]: K2's main item counter of segment seg; summary[8 + kK2TailCounters + seg]: its tail
// item counter (zeroed with the pass)
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
// K2 (+ fused join) over the 64-pair chunks [c0, c1), batch segment seg of nsegs
hipError_t launch_compare(hipStream_t s, const DiffBuffers& b, uint32_t c0, uint32_t c1, uint32_t seg,
                          uint32_t nsegs, bool reset_summary);
// K3 over chunks [c0, c1): running (n_spec, n_status, n_dirty, cap) totals before -> after
hipError_t launch_compact(hipStream_t s, const DiffBuffers& b, uint32_t c0, uint32_t c1, const uint4* before,
                          uint4* after);
// K4 over the deferred dirty pairs the segment added (before.z .. after.z)
// K4's slot owners again (the scratch-overflow re-run of K4-K6)
hipError_t launch_slot_owners(hipStream_t s, const DiffBuffers& b);
hipError_t launch_join(hipStream_t s, const DiffBuffers& b, uint32_t c0, uint32_t c1, const uint4* before,
                       const uint4* after);
hipError_t launch_emit(hipStream_t s, const DiffBuffers& b);
// tuning: K2 variant 14 writes 8 u64 per wave (start, first item end, items, last item start, end,
// streaming ticks, join ticks, hw id) into dev_buf (cap_waves waves); nullptr disables
hipError_t k2_profile(uint64_t* dev_buf, uint32_t cap_waves);

}  // namespace gd
