// K11/K12: the Deployment splitter's status roll-up.
// Internal, not part of the ABI (gpudiff_rollup_* in include/gpudiff.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gpudiff.h"
#include "tokenize.h"

namespace gd {

// one group = the Deployments sharing one kcp.dev/owned-by value (the
// selector of deployment.go:44-51); layout of gpudiff_rollup_group
struct RollGroup {
    uint32_t first;    // lowest member document (others[0])
    uint32_t count;
    int32_t sums[5];   // int32 wrap-around sums of RollOut.v
    uint32_t pad;
};
static_assert(sizeof(RollGroup) == sizeof(gpudiff_rollup_group), "RollGroup");

constexpr uint32_t kRollFlagSentinel = 1u;   // a label hashed to the sort sentinel ~0
constexpr uint32_t kRollFlagCollision = 2u;  // equal hashes, different labels
constexpr int32_t kRollDeferred = -3;        // doc_group of a document K11 left to the host

struct RollGroupBufs {
    uint64_t *keys, *keys_alt;
    uint32_t *vals, *vals_alt, *head, *gid, *mark, *rank, *remap, *doc_tmp;
    RollGroup *groups_tmp, *groups;
    int32_t* doc_group;
    uint32_t* counts;  // [0] groups, [1] kRollFlag* bits
    void* temp;
    uint64_t temp_bytes;
    uint64_t total;
};

uint64_t rollup_group_scratch_bytes(uint32_t n);
// carve the grouping buffers out of base (nullptr: sizes only, .total)
RollGroupBufs rollup_group_layout(uint8_t* base, uint32_t n);
// K12 over the K11 outputs ro[0, n)
hipError_t launch_rollup_group(hipStream_t s, const RollOut* ro, const TokDoc* docs, const uint8_t* json, uint32_t n,
                               const RollGroupBufs& B);

}  // namespace gd
