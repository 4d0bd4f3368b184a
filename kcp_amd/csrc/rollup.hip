// K12: the Deployment splitter's roll-up groups.
//
// pkg/reconciler/deployment/deployment.go:44-91: for a root named R, every
// cached Deployment whose kcp.dev/owned-by label equals R (the lister's
// selector, all namespaces and logical clusters) is summed into R's status
// (int32 additions: Go wrap-around), and others[0]'s conditions are copied.
// The batch form groups a whole population at once, after K11 extracted each
// document's counters and label span:
//
//   k_roll_keys   lane per document: XXH64 of the owned-by value (documents
//                 without one, or left to the host, sort last under ~0)
//   radix sort    (hash, document) pairs, hipCUB
//   k_roll_heads  lane per sorted position: a group starts where the hash
//                 changes; equal hashes must have byte-equal labels (a
//                 collision flags the batch for the host's exact grouping)
//   scan          inclusive sum of the heads -> group ids
//   k_roll_accum  lane per member: u32 atomics on its group's sums (two's
//                 complement adds = Go's int32 wrap-around), atomicMin of the
//                 first document, member count
//   k_roll_mark / scan / k_roll_place / k_roll_docs: groups renumbered by
//                 their first document (first-appearance order), per-document
//                 group ids
//
// All of it is latency/atomic work over 40-70 bytes per document; the HBM
// traffic is the K11 pass over the JSON.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>

#include <algorithm>

#include "../../include/gpudiff.h"
#include "rollup.h"
#include "tokenize.h"
#include "xxh64.h"

#include "tokdev.h"

namespace gd {

namespace {

constexpr uint32_t kTpb = 256;
inline uint32_t nblk(uint64_t n) { return (uint32_t)((n + kTpb - 1) / kTpb); }

__device__ __forceinline__ const uint8_t* label_ptr(const RollOut& r, const TokDoc* docs, const uint8_t* json,
                                                     uint32_t d) {
    return json + docs[d].json_off + r.label_off;
}

__global__ void k_roll_keys(const RollOut* __restrict__ ro, const TokDoc* __restrict__ docs,
                            const uint8_t* __restrict__ json, uint32_t n, uint64_t* __restrict__ keys,
                            uint32_t* __restrict__ vals, uint32_t* __restrict__ flags) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const RollOut r = ro[i];
    uint64_t key = ~0ull;
    if (r.status == 0 && (r.flags & kRollHasLabel)) {
        key = hash_bytes(label_ptr(r, docs, json, i), r.label_len);
        if (key == ~0ull) atomicOr(flags, kRollFlagSentinel);  // a real label on the sentinel: host groups
    }
    keys[i] = key;
    vals[i] = i;
}

__global__ void k_roll_heads(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ vals,
                             const RollOut* __restrict__ ro, const TokDoc* __restrict__ docs,
                             const uint8_t* __restrict__ json, uint32_t n, uint32_t* __restrict__ head,
                             uint32_t* __restrict__ flags) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const uint64_t k = keys[p];
    uint32_t h = 0;
    if (k != ~0ull) {
        h = (p == 0 || keys[p - 1] != k) ? 1u : 0u;
        if (!h) {  // same hash as the previous member: the label bytes must agree
            const uint32_t a = vals[p], b = vals[p - 1];
            const RollOut ra = ro[a], rb = ro[b];
            if (!bytes_eq(label_ptr(ra, docs, json, a), ra.label_len, label_ptr(rb, docs, json, b), rb.label_len))
                atomicOr(flags, kRollFlagCollision);
        }
    }
    head[p] = h;
}

__global__ void k_roll_init(RollGroup* __restrict__ g, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    RollGroup z{};
    z.first = 0xFFFFFFFFu;
    g[i] = z;
}

__global__ void k_roll_accum(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ vals,
                             const uint32_t* __restrict__ gid, const RollOut* __restrict__ ro, uint32_t n,
                             RollGroup* __restrict__ groups, uint32_t* __restrict__ doc_tmp) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n || keys[p] == ~0ull) return;
    const uint32_t d = vals[p], g = gid[p] - 1u;
    const RollOut r = ro[d];
    RollGroup* G = groups + g;
    atomicAdd(&G->count, 1u);
    atomicMin(&G->first, d);
#pragma unroll
    for (int f = 0; f < 5; f++) atomicAdd((uint32_t*)&G->sums[f], (uint32_t)r.v[f]);
    doc_tmp[d] = g;
}

__global__ void k_roll_mark(const RollGroup* __restrict__ groups, const uint32_t* __restrict__ gid, uint32_t n,
                            uint32_t* __restrict__ mark) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t ng = gid[n - 1];
    if (g >= ng) return;
    mark[groups[g].first] = 1u;
}

__global__ void k_roll_place(const RollGroup* __restrict__ groups, const uint32_t* __restrict__ gid,
                             const uint32_t* __restrict__ rank, uint32_t n, RollGroup* __restrict__ out,
                             uint32_t* __restrict__ remap, uint32_t* __restrict__ counts) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t ng = gid[n - 1];
    if (g == 0) counts[0] = ng;
    if (g >= ng) return;
    const RollGroup G = groups[g];
    const uint32_t r = rank[G.first];
    out[r] = G;
    remap[g] = r;
}

__global__ void k_roll_docs(const RollOut* __restrict__ ro, const uint32_t* __restrict__ doc_tmp,
                            const uint32_t* __restrict__ remap, uint32_t n, int32_t* __restrict__ doc_group) {
    const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= n) return;
    const RollOut r = ro[d];
    int32_t g;
    if (r.status != 0) g = kRollDeferred;
    else if (!(r.flags & kRollHasLabel)) g = GPUDIFF_ROLLUP_NONE;
    else g = (int32_t)remap[doc_tmp[d]];
    doc_group[d] = g;
}

}  // namespace

uint64_t rollup_group_scratch_bytes(uint32_t n) {
    size_t a = 0, b = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, a, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                             (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)n);
    (void)hipcub::DeviceScan::InclusiveSum(nullptr, b, (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)n);
    return std::max<uint64_t>(a, b) + 256;
}

RollGroupBufs rollup_group_layout(uint8_t* base, uint32_t n) {
    RollGroupBufs B;
    uint64_t o = 0;
    auto take = [&](uint64_t bytes) {
        uint8_t* p = base ? base + o : nullptr;
        o += (bytes + 255) & ~255ull;
        return p;
    };
    const uint64_t m = n ? n : 1;
    B.keys = (uint64_t*)take(8 * m);
    B.keys_alt = (uint64_t*)take(8 * m);
    B.vals = (uint32_t*)take(4 * m);
    B.vals_alt = (uint32_t*)take(4 * m);
    B.head = (uint32_t*)take(4 * m);
    B.gid = (uint32_t*)take(4 * m);
    B.mark = (uint32_t*)take(4 * m);
    B.rank = (uint32_t*)take(4 * m);
    B.remap = (uint32_t*)take(4 * m);
    B.doc_tmp = (uint32_t*)take(4 * m);
    B.groups_tmp = (RollGroup*)take(sizeof(RollGroup) * m);
    B.groups = (RollGroup*)take(sizeof(RollGroup) * m);
    B.doc_group = (int32_t*)take(4 * m);
    B.counts = (uint32_t*)take(64);
    B.temp_bytes = rollup_group_scratch_bytes(n);
    B.temp = take(B.temp_bytes);
    B.total = o;
    return B;
}

hipError_t launch_rollup_group(hipStream_t s, const RollOut* ro, const TokDoc* docs, const uint8_t* json, uint32_t n,
                               const RollGroupBufs& B) {
    hipError_t e;
    if ((e = hipMemsetAsync(B.counts, 0, 64, s)) != hipSuccess) return e;
    if (!n) return hipSuccess;
    k_roll_keys<<<nblk(n), kTpb, 0, s>>>(ro, docs, json, n, B.keys, B.vals, B.counts + 1);
    size_t tb = B.temp_bytes;
    if ((e = hipcub::DeviceRadixSort::SortPairs(B.temp, tb, B.keys, B.keys_alt, B.vals, B.vals_alt, (int)n, 0, 64,
                                                s)) != hipSuccess)
        return e;
    k_roll_heads<<<nblk(n), kTpb, 0, s>>>(B.keys_alt, B.vals_alt, ro, docs, json, n, B.head, B.counts + 1);
    tb = B.temp_bytes;
    if ((e = hipcub::DeviceScan::InclusiveSum(B.temp, tb, B.head, B.gid, (int)n, s)) != hipSuccess) return e;
    k_roll_init<<<nblk(n), kTpb, 0, s>>>(B.groups_tmp, n);
    k_roll_accum<<<nblk(n), kTpb, 0, s>>>(B.keys_alt, B.vals_alt, B.gid, ro, n, B.groups_tmp, B.doc_tmp);
    if ((e = hipMemsetAsync(B.mark, 0, 4ull * n, s)) != hipSuccess) return e;
    k_roll_mark<<<nblk(n), kTpb, 0, s>>>(B.groups_tmp, B.gid, n, B.mark);
    tb = B.temp_bytes;
    if ((e = hipcub::DeviceScan::ExclusiveSum(B.temp, tb, B.mark, B.rank, (int)n, s)) != hipSuccess) return e;
    k_roll_place<<<nblk(n), kTpb, 0, s>>>(B.groups_tmp, B.gid, B.rank, n, B.groups, B.remap, B.counts);
    k_roll_docs<<<nblk(n), kTpb, 0, s>>>(ro, B.doc_tmp, B.remap, n, B.doc_group);
    return hipGetLastError();
}

}  // namespace gd
