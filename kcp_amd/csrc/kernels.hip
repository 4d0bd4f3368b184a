// HIP kernels of the gpudiff engine, written for gfx950 (CDNA4, wave64).
//
//   K2 k_compare_flat spec/status decision per pair: the item's compared
//                     segments flattened into one stream of 16-B chunks,
//                     streamed by the whole wave (non-temporal 16-B loads),
//                     mismatches marked by ballot; a dirty pair's changed
//                     paths merge-joined on the spot (join_pair) into the
//                     wave's path arena
//   K3 k_scan_*<V4>   reduce-then-scan of the per-chunk counts
//      k_compact      ballot/prefix compaction of dirty pair IDs + scratch
//                     slots for the deferred joins
//   K4 k_join         merge-join of the pairs K2 deferred: sorted leaf keys in
//                     64-key windows held in registers (cross-lane binary
//                     search with ds_bpermute), byte-exact confirmation of
//                     long values whose first 8 bytes agree
//   K5 k_scan_*<u32>  exclusive scan of per-pair path counts
//   K6 k_copy_paths   compaction of the path arenas / scratch into the CSR
//
// Semantics: DESIGN.md "Kernels"; reference predicates
// pkg/syncer/specsyncer.go:17-41 and pkg/syncer/statussyncer.go:15-27.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gpudiff.h"
#include "kernels.h"
#include "xxh64.h"

namespace gd {

// per-pair flag byte written by K2: bits 0-2 are the public GPUDIFF_* result
// bits; bits 3-6 are internal hints for K4/K6 (masked off on the host)
constexpr uint32_t F_SPEC = 1u, F_STATUS = 2u, F_ERR = 4u;
constexpr uint32_t F_SENT = 8u;    // status-absent-in-new sentinel path
constexpr uint32_t F_JSPEC = 16u;  // spec region needs the merge-join
constexpr uint32_t F_JSTAT = 32u;  // status region needs the merge-join
constexpr uint32_t F_SEED = 64u;   // pair path-hash seed != 0
constexpr uint32_t F_DEFER = 128u; // paths not produced by K2 (wave arena full): K4 joins it
constexpr uint32_t ARENA_BIT = 0x80000000u;  // scratch_off[d]: paths live in the K2 wave arenas

// K4 merge-path slices (k_join_slices below)
constexpr uint32_t kJoinSlice = 1024;  // merged keys per slice (<= 16 windows of 64 + 64)
constexpr uint32_t kDeepJoin = 2048;   // K2 defers a dirty pair whose join covers more keys
constexpr uint32_t kTailJoinMax = 1024;  // K2's largest-first rounds: joins over this many keys go to K4's slices

// Scratch entries of a deferred pair.  need = the merged keys of each joined region + the status-absent
// sentinel (when the pair has one) bounds its paths.  A pair with need <= kJoinSlice -- one K2 deferred
// only because its wave arena was full -- is a *whole* deferral: exactly need entries, joined by one
// wave in K3 (k_compact).  A larger one is *sliced*: each region's merged keys in kJoinSlice-key slices,
// every slice writing at its own kJoinSlice-entry offset, so the cap is a whole number of slices (and at
// least need, for the sentinel after the packed paths); a sliced cap is therefore >= 2 * kJoinSlice and
// cap <= kJoinSlice tells the two kinds apart.
constexpr uint32_t kNoOwner = 0xFFFFFFFFu;  // slot_owner of a slot inside a whole deferral's entries
__device__ __forceinline__ uint32_t defer_cap(uint32_t spec_l_a, uint32_t spec_l_b, uint32_t stat_l_a,
                                              uint32_t stat_l_b, uint32_t f) {
    const uint32_t Ls = (f & F_JSPEC) ? spec_l_a + spec_l_b : 0u;
    const uint32_t Lt = (f & F_JSTAT) ? stat_l_a + stat_l_b : 0u;
    const uint32_t need = Ls + Lt + ((f & F_SENT) ? 1u : 0u);
    if (need <= kJoinSlice) return need;
    const uint32_t slices = (Ls + kJoinSlice - 1u) / kJoinSlice + (Lt + kJoinSlice - 1u) / kJoinSlice;
    return max(slices, (need + kJoinSlice - 1u) / kJoinSlice) * kJoinSlice;
}
__device__ __forceinline__ uint32_t sat_add(uint32_t a, uint32_t b) {
    const uint32_t s = a + b;
    return s < a ? 0xFFFFFFFFu : s;
}


// ---------------------------------------------------------------- wave helpers
__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

__device__ __forceinline__ uint32_t shfl32(uint32_t v, uint32_t src) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)v);
}
__device__ __forceinline__ uint64_t shfl64(uint64_t v, uint32_t src) {
    uint32_t lo = shfl32((uint32_t)v, src), hi = shfl32((uint32_t)(v >> 32), src);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }
__device__ __forceinline__ uint32_t popc64(uint64_t m) { return (uint32_t)__popcll(m); }
__device__ __forceinline__ uint64_t mask_lt(uint32_t n) { return n >= 64 ? ~0ULL : ((1ULL << n) - 1ULL); }

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    const uint32_t lane = lane_id();
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
        uint32_t o = shfl32(v, lane >= d ? lane - d : lane);
        if (lane >= d) v += o;
    }
    return v;
}
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
    for (uint32_t d = 32; d >= 1; d >>= 1) v += (uint32_t)__shfl_xor((int)v, (int)d);
    return v;
}
__device__ __forceinline__ uint32_t wave_min(uint32_t v) {
#pragma unroll
    for (uint32_t d = 32; d >= 1; d >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, (int)d));
    return v;
}
__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
#pragma unroll
    for (uint32_t d = 32; d >= 1; d >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, (int)d));
    return v;
}
__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

__device__ __forceinline__ uint64_t seg_bytes(uint32_t l, uint32_t arena) { return (uint64_t)l * 16u + arena; }
__device__ __forceinline__ bool meta_long(uint32_t m) { return (m & 7u) == GPUDIFF_TAG_STR && (m >> 3) > 8u; }
// arena bytes of a leaf's value: a long string's tail past its first 8 bytes (which sit in vals), at a
// 4-byte aligned offset (include/gpudiff_format.h)
__device__ __forceinline__ uint32_t meta_arena(uint32_t m) { return meta_long(m) ? (((m >> 3) - 8u + 3u) & ~3u) : 0u; }

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ bool neq16(const u32x4& a, const u32x4& b) {
    const u32x4 x = a ^ b;
    return (x.x | x.y | x.z | x.w) != 0u;
}

// ---------------------------------------------------------------- scans
// Reduce-then-scan over u32 or 4 x u32 elements in tiles of 4096 (256 threads
// x 16), two launches: tile sums -> per-tile exclusive scan, each workgroup
// summing the tile sums before its own tile (a few thousand at most, L2-
// resident) instead of a third, one-workgroup launch scanning them.  The
// element count comes from the host (n_host) or from device memory (n_dev,
// e.g. the dirty count).
constexpr uint32_t SCAN_TILE = 4096;

struct V4 {
    uint32_t x, y, z, w;
};
__device__ __forceinline__ uint32_t vadd(uint32_t a, uint32_t b) { return a + b; }
// w (the deferred pairs' scratch entries) saturates at 2^32 - 1 -- saturating addition is associative --
// so a batch whose deferred joins would need more scratch than u32 offsets address is reported
// (GPUDIFF_E_CAPACITY) instead of wrapping into overlapping scratch
__device__ __forceinline__ V4 vadd(const V4& a, const V4& b) {
    return V4{a.x + b.x, a.y + b.y, a.z + b.z, sat_add(a.w, b.w)};
}
template <class V> __device__ __forceinline__ V vzero() { return V{}; }
__device__ __forceinline__ uint32_t vshfl(uint32_t v, uint32_t src) { return shfl32(v, src); }
__device__ __forceinline__ V4 vshfl(const V4& v, uint32_t src) {
    return V4{shfl32(v.x, src), shfl32(v.y, src), shfl32(v.z, src), shfl32(v.w, src)};
}
template <class V>
__device__ __forceinline__ V wave_incl_scan_v(V v) {
    const uint32_t lane = lane_id();
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
        V o = vshfl(v, lane >= d ? lane - d : lane);
        if (lane >= d) v = vadd(v, o);
    }
    return v;
}

__device__ __forceinline__ uint32_t scan_n(const uint32_t* n_dev, uint32_t n_host) { return n_dev ? *n_dev : n_host; }

template <class V>
__global__ __launch_bounds__(256) void k_scan_tiles(const V* __restrict__ in, const uint32_t* __restrict__ n_dev,
                                                    uint32_t n_host, V* __restrict__ tile_sums) {
    __shared__ V red[4];
    const uint32_t n = scan_n(n_dev, n_host);
    const uint32_t base = blockIdx.x * SCAN_TILE;
    if (base >= n) return;
    V s = vzero<V>();
    for (uint32_t i = threadIdx.x; i < SCAN_TILE; i += 256)
        if (base + i < n) s = vadd(s, in[base + i]);
    s = vshfl(wave_incl_scan_v(s), 63);
    if (lane_id() == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) tile_sums[blockIdx.x] = vadd(vadd(red[0], red[1]), vadd(red[2], red[3]));
}

__device__ __forceinline__ void mirror_store(uint32_t* m, const V4& v) {
    m[0] = v.x;
    m[1] = v.y;
    m[2] = v.z;
    m[3] = v.w;
}
__device__ __forceinline__ void mirror_store(uint32_t* m, uint32_t v) { m[0] = v; }

// out[i] = *base_in (nullptr = 0) + exclusive prefix of in (out may alias in).  The workgroup holding the
// last element (workgroup 0 when n == 0) writes *total = base + sum -- total must not alias base_in -- and,
// if write_terminal, out[n] = the same, and, if mirror, the total's words there too (the bound gather
// buffer's counts).  Launch at least (n ? (n - 1) / SCAN_TILE + 1 : 1) workgroups.
template <class V>
__global__ __launch_bounds__(256) void k_scan_apply(const V* in, const uint32_t* __restrict__ n_dev, uint32_t n_host,
                                                    const V* __restrict__ tile_sums, const V* base_in, V* total,
                                                    V* out, bool write_terminal, uint32_t* __restrict__ mirror) {
    __shared__ V wsum[4];
    __shared__ V wpre[4];
    const uint32_t n = scan_n(n_dev, n_host);
    const uint32_t last = n ? (n - 1) / SCAN_TILE : 0;
    if (blockIdx.x > last) return;
    const uint32_t base = blockIdx.x * SCAN_TILE;
    const uint32_t t = threadIdx.x;
    V p = vzero<V>();
    for (uint32_t i = t; i < blockIdx.x; i += 256) p = vadd(p, tile_sums[i]);
    p = vshfl(wave_incl_scan_v(p), 63);
    if (lane_id() == 0) wpre[t >> 6] = p;
    V v[16];
    V s = vzero<V>();
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const uint32_t i = base + t * 16 + k;
        v[k] = i < n ? in[i] : vzero<V>();
        s = vadd(s, v[k]);
    }
    const V incl = wave_incl_scan_v(s);
    if (lane_id() == 63) wsum[t >> 6] = incl;
    __syncthreads();
    V run = vadd(vadd(wpre[0], wpre[1]), vadd(wpre[2], wpre[3]));
    if (base_in) run = vadd(run, *base_in);
    for (uint32_t w = 0; w < (t >> 6); w++) run = vadd(run, wsum[w]);
    const V excl_thread = vshfl(incl, lane_id() ? lane_id() - 1 : 0);
    if (lane_id()) run = vadd(run, excl_thread);
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const uint32_t i = base + t * 16 + k;
        if (i < n) out[i] = run;
        run = vadd(run, v[k]);
    }
    if (blockIdx.x == last && t == 255) {  // run = base + every element of the tile (zero past n)
        *total = run;
        if (write_terminal) out[n] = run;
        if (mirror) mirror_store(mirror, run);
    }
}

// ---------------------------------------------------------------- K4
struct RegionView {
    const uint32_t* keys;
    const uint64_t* vals;
    const uint32_t* metas;
    const uint8_t* arena;
    uint32_t L;
};

__device__ __forceinline__ RegionView region_view(const uint8_t* pool, uint64_t off, uint32_t sl, uint32_t sar,
                                                  bool status, uint32_t L) {
    const uint8_t* seg = pool + off + (status ? seg_bytes(sl, sar) : 0);
    RegionView v;
    v.vals = (const uint64_t*)seg;  // vals u64 | keys u32 | metas u32 | arena (include/gpudiff_format.h)
    v.keys = (const uint32_t*)(seg + 8ull * L);
    v.metas = (const uint32_t*)(seg + 12ull * L);
    v.arena = seg + 16ull * L;
    v.L = L;
    return v;
}

// number of tile keys (lanes < nt, ascending) strictly less than x
__device__ __forceinline__ uint32_t tile_lower_bound(uint32_t x, uint32_t tile, uint32_t nt) {
    uint32_t j = 0;
#pragma unroll
    for (uint32_t s = 64; s >= 1; s >>= 1) {
        const uint32_t cand = j + s;
        const uint32_t t = shfl32(tile, min(cand, 64u) - 1u);
        if (cand <= nt && t < x) j = cand;
    }
    return j;
}

// Byte-exact confirmation of every lane's pending long value at once (same
// length, same first 8 bytes): the tails of len bytes in the two arenas.  The
// lanes' tails are flattened into one index space of dwords (prefix sum of
// dword counts: tails sit at 4-byte aligned arena offsets, zero padded to 4, so
// two equal-length tails are equal iff their padded dwords are); each pass the
// wave compares 64 x CV_U dwords (consecutive dwords of a tail are consecutive
// addresses), finding a dword's owner lane by a cross-lane binary search over
// the prefix sums.  No load reaches past a tail's padded end.  Returns true in
// the lanes whose tail differs.
__device__ bool confirm_values(bool need, const uint8_t* arena_a, uint32_t off_a, const uint8_t* arena_b,
                               uint32_t off_b, uint32_t len, uint32_t lane) {
    const uint32_t n4 = need ? (len + 3u) >> 2 : 0u;
    const uint32_t incl = wave_incl_scan(n4);
    const uint32_t total = shfl32(incl, 63);
    uint64_t bad = 0;  // lanes whose value differs (wave-uniform)
    constexpr int CV_U = 4;  // dword pairs in flight per lane
    for (uint32_t base = 0; base < total; base += 64 * CV_U) {
        uint32_t xa[CV_U], xb[CV_U];
        uint32_t own[CV_U];
        bool act[CV_U];
#pragma unroll
        for (int u = 0; u < CV_U; u++) {
            const uint32_t g = base + u * 64 + lane;
            act[u] = g < total;
            // owner = number of lanes whose inclusive dword prefix is <= g
            uint32_t o = 0;
#pragma unroll
            for (uint32_t s = 64; s >= 1; s >>= 1) {
                const uint32_t cand = o + s;
                const uint32_t t = shfl32(incl, min(cand, 64u) - 1u);
                if (cand <= 64u && t <= g) o = cand;
            }
            own[u] = min(o, 63u);
            const uint32_t oa = shfl32(off_a, own[u]), ob = shfl32(off_b, own[u]);
            const uint32_t first = shfl32(incl - n4, own[u]);
            if (act[u]) {
                const uint32_t k = g - first;
                xa[u] = *(const uint32_t*)(arena_a + oa + 4u * k);
                xb[u] = *(const uint32_t*)(arena_b + ob + 4u * k);
            }
        }
#pragma unroll
        for (int u = 0; u < CV_U; u++) {
            uint64_t m = ballot(act[u] && xa[u] != xb[u]);
            while (m) {  // values that differ only past their first 8 bytes
                const uint32_t j = (uint32_t)__builtin_ctzll(m);
                m &= m - 1;
                bad |= 1ull << shfl32(own[u], j);
            }
        }
    }
    return (bad >> lane) & 1ull;
}

// A changed leaf whose two values Go's json.Marshal writes as the same text
// and the API server decodes back to the same int64 (the write-path no-op rule,
// DESIGN.md §4g): an int64 v on one side, a float64 f == v on the other,
// |v| <= 2^53 (canonical values: int64 / float64 bits, -0.0 stored as +0.0).
__device__ __forceinline__ bool wire_equal_number(uint32_t ma, uint64_t xa, uint32_t mb, uint64_t xb) {
    const uint32_t ta = ma & 7u, tb = mb & 7u;
    if (!((ta == GPUDIFF_TAG_INT && tb == GPUDIFF_TAG_FLOAT) || (ta == GPUDIFF_TAG_FLOAT && tb == GPUDIFF_TAG_INT)))
        return false;
    const int64_t v = (int64_t)(ta == GPUDIFF_TAG_INT ? xa : xb);
    const double f = __longlong_as_double((long long)(ta == GPUDIFF_TAG_INT ? xb : xa));
    const int64_t lim = 1ll << 53;
    return v >= -lim && v <= lim && (double)v == f;
}

// Merge-join of one region; returns the number of paths emitted.  Emission
// order = ascending key (the union of both sorted key lists).  *weq_all: every
// emitted path is a CHANGED leaf with wire_equal_number values (wave-uniform).
template <bool EMIT>
__device__ uint32_t join_region(const RegionView& A, const RegionView& B, uint8_t region_bit,
                                uint64_t* __restrict__ out_h, uint8_t* __restrict__ out_k, uint32_t out_base,
                                uint32_t lane, bool* weq_all) {
    uint32_t ia = 0, ib = 0, arA = 0, arB = 0, outpos = 0;
    bool weq = true;
    const uint64_t lt = mask_lt(lane);
    while (ia < A.L || ib < B.L) {
        const uint32_t na = min(64u, A.L - ia), nb = min(64u, B.L - ib);
        const bool va = lane < na, vb = lane < nb;
        const uint32_t ka = va ? A.keys[ia + lane] : 0u;
        const uint32_t kb = vb ? B.keys[ib + lane] : 0u;
        const uint32_t ma = va ? A.metas[ia + lane] : 0u;
        const uint32_t mb = vb ? B.metas[ib + lane] : 0u;
        const uint64_t xa = va ? A.vals[ia + lane] : 0ull;
        const uint64_t xb = vb ? B.vals[ib + lane] : 0ull;
        const bool endA = ia + na == A.L, endB = ib + nb == B.L;
        const uint32_t lastA = na ? shfl32(ka, na - 1) : 0u;
        const uint32_t lastB = nb ? shfl32(kb, nb - 1) : 0u;
        // everything <= bound is resolvable in this window
        bool inf = true;
        uint32_t bound = 0;
        if (!endA) { bound = lastA; inf = false; }
        if (!endB) { bound = inf ? lastB : min(bound, lastB); inf = false; }
        const bool inA = va && (inf || ka <= bound);
        const bool inB = vb && (inf || kb <= bound);
        // arena offsets of this window's long values
        const uint32_t asA = meta_arena(ma), asB = meta_arena(mb);
        const uint32_t incA = wave_incl_scan(asA), incB = wave_incl_scan(asB);
        const uint32_t offA = arA + incA - asA, offB = arB + incB - asB;
        // resolve A keys against the B window
        const uint32_t jA = tile_lower_bound(ka, kb, nb);
        const uint32_t kbj = shfl32(kb, min(jA, 63u));
        const uint32_t mbj = shfl32(mb, min(jA, 63u));
        const uint64_t xbj = shfl64(xb, min(jA, 63u));
        const uint32_t obj = shfl32(offB, min(jA, 63u));
        const bool matchA = inA && jA < nb && kbj == ka;
        bool differ = matchA && (ma != mbj || xa != xbj);
        // equal head (the first 8 bytes, in vals) and length: confirm the tails in the arenas
        differ |= confirm_values(matchA && !differ && meta_long(ma), A.arena, offA, B.arena, obj, (ma >> 3) - 8u, lane);
        // resolve B keys against the A window
        const uint32_t iB = tile_lower_bound(kb, ka, na);
        const uint32_t kai = shfl32(ka, min(iB, 63u));
        const bool matchB = inB && iB < na && kai == kb;
        const bool emitA = inA && (!matchA || differ);
        const bool emitB = inB && !matchB;
        const uint64_t balA = ballot(emitA), balB = ballot(emitB);
        if (ballot((emitA && !(matchA && wire_equal_number(ma, xa, mbj, xbj))) || emitB)) weq = false;
        if (EMIT) {
            if (emitA) {
                const uint32_t pos = popc64(balA & lt) + popc64(balB & mask_lt(jA));
                out_h[out_base + outpos + pos] = ka;
                out_k[out_base + outpos + pos] = region_bit | (matchA ? GPUDIFF_PATH_CHANGED : GPUDIFF_PATH_REMOVED);
            }
            if (emitB) {
                const uint32_t pos = popc64(balB & lt) + popc64(balA & mask_lt(iB));
                out_h[out_base + outpos + pos] = kb;
                out_k[out_base + outpos + pos] = region_bit | GPUDIFF_PATH_ADDED;
            }
        }
        outpos += popc64(balA) + popc64(balB);
        const uint32_t ca = popc64(ballot(inA)), cb = popc64(ballot(inB));
        arA += ca ? shfl32(incA, ca - 1) : 0u;
        arB += cb ? shfl32(incB, cb - 1) : 0u;
        ia += ca;
        ib += cb;
    }
    *weq_all = weq;
    return outpos;
}

__device__ uint64_t status_sentinel_hash(uint32_t seed, uint64_t mask) {
    // XXH64 of the 11 path bytes 01 06 00 00 00 's' 't' 'a' 't' 'u' 's'
    // bytes: [0]=01 [1]=06 [2..4]=00 [5]='s' [6]='t' [7]='a' | [8]='t' [9]='u' [10]='s'
    uint64_t w[4] = {0, 0, 0, 0};
    w[0] = 0x01ull | (0x06ull << 8) | ((uint64_t)'s' << 40) | ((uint64_t)'t' << 48) | ((uint64_t)'a' << 56);
    w[1] = (uint64_t)'t' | ((uint64_t)'u' << 8) | ((uint64_t)'s' << 16);
    uint64_t h = (uint64_t)seed + XP5 + 11u;
    h = xxh64_tail(h, w, 11);
    return xavalanche(h) & mask;
}

// The write-path no-op bits of a dirty pair: bit 0 = the spec
// write (A's body over B) changes nothing deepEqualApartFromStatus compares
// (every changed spec leaf is a wire_equal_number change); bit 1 = the status
// write (B's status into A) changes nothing (every changed status leaf is one,
// and when B has no status key, A has none either).
constexpr uint32_t NOOP_SPEC = 1u, NOOP_STATUS = 2u;
__device__ __forceinline__ uint32_t sentinel_noop_bits(uint32_t flags_a) {
    return (flags_a & GPUDIFF_OBJ_HAS_STATUS) ? 0u : NOOP_STATUS;
}

template <bool EMIT>
__device__ uint32_t join_pair(const gpudiff_pair_row& r, uint32_t f, const uint8_t* pool, uint64_t mask,
                              uint64_t* out_h, uint8_t* out_k, uint32_t base, uint32_t lane, uint32_t* noop) {
    uint32_t n = 0;
    bool spec_weq = true, stat_weq = true;
    if (f & F_JSPEC) {
        RegionView A = region_view(pool, r.off_a, r.spec_l_a, r.spec_ar_a, false, r.spec_l_a);
        RegionView B = region_view(pool, r.off_b, r.spec_l_b, r.spec_ar_b, false, r.spec_l_b);
        n += join_region<EMIT>(A, B, 0, out_h, out_k, base + n, lane, &spec_weq);
    }
    if (f & F_JSTAT) {
        RegionView A = region_view(pool, r.off_a, r.spec_l_a, r.spec_ar_a, true, r.stat_l_a);
        RegionView B = region_view(pool, r.off_b, r.spec_l_b, r.spec_ar_b, true, r.stat_l_b);
        n += join_region<EMIT>(A, B, GPUDIFF_PATH_REGION_STATUS, out_h, out_k, base + n, lane, &stat_weq);
    }
    const bool stat_ok = stat_weq && (!(f & F_SENT) || !(r.flags_a & GPUDIFF_OBJ_HAS_STATUS));
    *noop = (((f & F_SPEC) && spec_weq) ? NOOP_SPEC : 0u) | (((f & F_STATUS) && stat_ok) ? NOOP_STATUS : 0u);
    if (f & F_SENT) {
        if (EMIT && lane == 0) {
            out_h[base + n] = status_sentinel_hash((r.flags_a >> GPUDIFF_OBJ_SEED_SHIFT) & 0xFFu, mask);
            out_k[base + n] = GPUDIFF_PATH_REGION_STATUS | GPUDIFF_PATH_STATUS_ABSENT;
        }
        n += 1;
    }
    return n;
}

// ---------------------------------------------------------------- K3 compaction
// A deferred pair's scratch entries [so, so + cap): a sliced deferral owns every kJoinSlice-aligned slot
// that starts inside them (exactly cap / kJoinSlice slots: its cap is a multiple of kJoinSlice), and its
// slice i is the i-th of those; a whole deferral's entries hold at most one slot start, marked kNoOwner.
// The slots of [before, after) are therefore exactly those starting in it, each written once.  Returns
// whether the entries fit the scratch (else K4 reports the overflow and the host re-runs K4-K6).
__device__ __forceinline__ bool place_deferred(uint32_t d, uint64_t so, uint32_t cap, uint64_t scratch_cap,
                                               uint32_t* __restrict__ slot_owner) {
    if (so > scratch_cap || cap > scratch_cap - so) return false;
    const uint32_t b0 = (uint32_t)((so + kJoinSlice - 1u) / kJoinSlice);
    const uint32_t b1 = (uint32_t)((so + cap + kJoinSlice - 1u) / kJoinSlice);  // slots starting before the end
    if (cap > kJoinSlice) {
        for (uint32_t q = b0; q < b1; q++) slot_owner[q] = d;
    } else if (b0 < b1) {
        slot_owner[b0] = kNoOwner;
    }
    return true;
}

// The whole deferrals among the wave's lanes (bit k: lane k's pair), one at a time: join_pair straight
// into the pair's exact scratch entries, path count and no-op bits written here (K4 skips them).
__device__ __forceinline__ void join_whole(uint64_t wm, uint32_t p, uint32_t d, uint32_t so, uint32_t f,
                                           const gpudiff_pair_row* __restrict__ rows, const uint8_t* __restrict__ pool,
                                           uint64_t mask, uint64_t* __restrict__ sh, uint8_t* __restrict__ sk,
                                           uint32_t* __restrict__ path_count, uint8_t* __restrict__ noop_d,
                                           uint32_t lane) {
    for (; wm; wm &= wm - 1) {
        const uint32_t k = (uint32_t)__builtin_ctzll(wm);
        const uint32_t pk = (uint32_t)__builtin_amdgcn_readlane((int)p, (int)k);
        const uint32_t dk = (uint32_t)__builtin_amdgcn_readlane((int)d, (int)k);
        const uint32_t sok = (uint32_t)__builtin_amdgcn_readlane((int)so, (int)k);
        const uint32_t fk = (uint32_t)__builtin_amdgcn_readlane((int)f, (int)k);
        const gpudiff_pair_row r = rows[pk];
        uint32_t nb = 0;
        const uint32_t cnt = join_pair<true>(r, fk, pool, mask, sh, sk, sok, lane, &nb);
        if (lane == 0) {
            path_count[dk] = cnt;
            noop_d[dk] = (uint8_t)nb;
        }
    }
}

// One wave per chunk: ballot + prefix compaction into the ID lists; scratch entries and K4 slots of the
// deferred pairs (place_deferred), and the whole deferrals joined on the spot.
__global__ __launch_bounds__(256) void k_compact(const uint8_t* __restrict__ flags, const uint32_t* __restrict__ caps,
                                                 const uint32_t* __restrict__ pair_ids, uint32_t n,
                                                 const uint4* __restrict__ cbase, uint32_t* __restrict__ spec_ids,
                                                 uint32_t* __restrict__ status_ids, uint32_t* __restrict__ dirty_ids,
                                                 uint32_t* __restrict__ dirty_idx, uint32_t* __restrict__ scratch_off,
                                                 uint32_t c_begin, uint32_t c_end, const uint32_t* __restrict__ path_src,
                                                 const uint32_t* __restrict__ path_cnt,
                                                 uint32_t* __restrict__ path_count, const uint8_t* __restrict__ nbits,
                                                 uint8_t* __restrict__ noop_d, uint32_t* __restrict__ slot_owner,
                                                 uint64_t scratch_cap, const gpudiff_pair_row* __restrict__ rows,
                                                 const uint8_t* __restrict__ pool, uint64_t mask,
                                                 uint64_t* __restrict__ sh, uint8_t* __restrict__ sk,
                                                 uint32_t* __restrict__ gsend, uint32_t gcap_s, uint32_t gcap_t) {
    const uint32_t lane = lane_id();
    const uint32_t wave = uni((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
    const uint64_t lt = mask_lt(lane);
    for (uint32_t c = c_begin + wave; c < c_end; c += nwaves) {
        const uint32_t p = (c << 6) + lane;
        const bool valid = p < n;
        const uint32_t f = valid ? flags[p] : 0u;
        const uint64_t bs = ballot(f & F_SPEC), bt = ballot(f & F_STATUS), bd = ballot(f & (F_SPEC | F_STATUS));
        if (bd == 0) continue;
        const uint4 base = cbase[c];
        const bool dirty = (f & (F_SPEC | F_STATUS)) != 0u;
        const uint32_t id = dirty ? pair_ids[p] : 0u;
        const uint32_t cap = dirty ? caps[p] : 0u;
        const uint32_t cincl = wave_incl_scan(cap);
        // the dirty lists, and (gpudiff_dbatch_bind_gather) the same IDs straight into the collective's send
        // buffer [8 counts | gcap_s spec IDs | gcap_t status IDs]: no export copies per step
        if (f & F_SPEC) {
            const uint32_t q = base.x + popc64(bs & lt);
            spec_ids[q] = id;
            if (gsend && q < gcap_s) gsend[8u + q] = id;
        }
        if (f & F_STATUS) {
            const uint32_t q = base.y + popc64(bt & lt);
            status_ids[q] = id;
            if (gsend && q < gcap_t) gsend[8u + gcap_s + q] = id;
        }
        uint32_t d = 0, so = 0;
        bool whole = false;
        if (dirty) {
            d = base.z + popc64(bd & lt);
            dirty_ids[d] = id;
            dirty_idx[d] = p;
            if (f & F_DEFER) {  // K4 (or, whole, this wave) joins it into its scratch entries
                // base.w saturates (a batch past u32 scratch offsets): then nothing fits and K4 reports it
                const uint64_t so64 = base.w == 0xFFFFFFFFu ? ~0ull : (uint64_t)base.w + (cincl - cap);
                so = (uint32_t)min(so64, (uint64_t)0xFFFFFFFFu);
                scratch_off[d] = so;
                whole = place_deferred(d, so64, cap, scratch_cap, slot_owner) && cap <= kJoinSlice;
            } else {            // K2 already wrote its paths into a wave arena (and the no-op bits)
                scratch_off[d] = path_src[p] | ARENA_BIT;
                path_count[d] = path_cnt[p];
                noop_d[d] = nbits[p];
            }
        }
        join_whole(ballot(whole), p, d, so, f, rows, pool, mask, sh, sk, path_count, noop_d, lane);
    }
}

// The overflow re-run after the scratch grew (K3 placed nothing past the old scratch): every deferred
// pair placed again and its whole deferrals joined.  Wave per 64 dirty pairs.
__global__ __launch_bounds__(256) void k_slot_owners(const uint8_t* __restrict__ flags, const uint32_t* __restrict__ caps,
                                                     const uint32_t* __restrict__ dirty_idx,
                                                     const uint32_t* __restrict__ scratch_off,
                                                     const uint32_t* __restrict__ summary, uint64_t scratch_cap,
                                                     uint32_t* __restrict__ slot_owner,
                                                     const gpudiff_pair_row* __restrict__ rows,
                                                     const uint8_t* __restrict__ pool, uint64_t mask,
                                                     uint64_t* __restrict__ sh, uint8_t* __restrict__ sk,
                                                     uint32_t* __restrict__ path_count, uint8_t* __restrict__ noop_d) {
    const uint32_t lane = lane_id();
    const uint32_t wave = uni((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
    const uint32_t ndirty = summary[2];
    if (summary[6] == 0u) return;
    for (uint32_t c = wave; c < (ndirty + 63u) >> 6; c += nwaves) {
        const uint32_t d = (c << 6) + lane;
        const uint32_t p = d < ndirty ? dirty_idx[d] : 0u;
        const uint32_t f = d < ndirty ? flags[p] : 0u;
        bool whole = false;
        uint32_t so = 0;
        if (f & F_DEFER) {
            so = scratch_off[d];
            const uint32_t cap = caps[p];
            whole = place_deferred(d, so, cap, scratch_cap, slot_owner) && cap <= kJoinSlice;
        }
        join_whole(ballot(whole), p, d, so, f, rows, pool, mask, sh, sk, path_count, noop_d, lane);
    }
}

// ---------------------------------------------------------------- K4: merge-path slices
// A deferred pair's join -- one K2 could not hold in its wave arena, or one over kDeepJoin keys that
// would keep a single K2 wave busy long after the others finish (config4's list shifts: thousands of
// changed paths) -- is cut along its merge path: each region's two sorted key
// lists, merged (A before B on equal keys), are split into slices of kJoinSlice merged keys, and every
// slice is joined by its own wave, all slices of all deferred pairs spread over the whole grid.  The
// scratch a deferred pair gets (its K2 cap, rounded by defer_cap) holds one kJoinSlice-entry slot per
// slice, so a slice writes its paths at its slot with no coordination; K4b (k_join_gather) then packs
// each pair's slices in order and adds the status-absent sentinel.  K3 maps every slot to its pair.
// merge-path split of two sorted unique key lists (A before B on equal keys): the number of A keys
// among the first dg merged keys.  64-ary search: each step the lanes probe 64 evenly spaced
// candidates of the remaining range at once.
__device__ uint32_t merge_split(const uint32_t* __restrict__ ka, uint32_t La, const uint32_t* __restrict__ kb,
                                uint32_t Lb, uint32_t dg, uint32_t lane) {
    uint32_t lo = dg > Lb ? dg - Lb : 0u, hi = min(dg, La);  // the answer is in [lo, hi]
    while (lo < hi) {
        // candidate ia = lo + step * (lane + 1) - 1 ... : "A[ia] belongs to the first dg" <=> A[ia] <= B[dg-ia-1]
        const uint32_t span = hi - lo;
        const uint32_t step = (span + 63u) / 64u;
        const uint32_t ia = lo + lane * step;
        bool inc = false;  // A[ia] is among the first dg merged keys
        if (ia < hi) inc = ka[ia] <= kb[dg - ia - 1u];
        const uint64_t b = ballot(ia < hi && !inc);
        // the predicate is monotone (true then false): the first false lane bounds the answer
        if (!b) {
            const uint32_t last = min(63u, (span - 1u) / step);  // last probing lane
            lo = lo + last * step + 1u;
            if (step == 1u) break;
            hi = min(hi, lo + step - 1u);
        } else {
            const uint32_t f = (uint32_t)__builtin_ctzll(b);
            const uint32_t nhi = lo + f * step;            // A[nhi] is not included: answer <= nhi
            lo = f ? lo + (f - 1u) * step + 1u : lo;       // A[lo + (f-1) step] is included
            hi = nhi;
        }
    }
    return lo;
}

// first scratch slot starting at or after entry e
__device__ __forceinline__ uint32_t slot_ceil(uint32_t e) { return (uint32_t)(((uint64_t)e + kJoinSlice - 1u) / kJoinSlice); }

// arena bytes of entries [0, n) of a region (long values' tails before entry n).  Every slice of a pair
// sums the metas before its start, so a region of L keys costs O(L^2 / kJoinSlice) meta reads over its
// slices; they are L2-resident re-reads, and this loop keeps 8 x 16 B (32 metas) per lane in
// flight -- 2048 metas per wave step, 8x the former 4-byte loop -- so even a 100k-key list (the k8s
// object size limit) takes ~50 steps per slice, about the slice's own join time.  The metas array starts
// 4-B aligned (12 L bytes into a 16-B aligned segment): a dword head reaches 16-B alignment first.
__device__ uint32_t arena_prefix(const uint32_t* __restrict__ metas, uint32_t n, uint32_t lane) {
    const uint32_t head = min(n, (uint32_t)((16u - ((uintptr_t)metas & 15u)) & 15u) >> 2);
    uint32_t acc = lane < head ? meta_arena(metas[lane]) : 0u;
    const u32x4* m4 = (const u32x4*)(metas + head);
    const uint32_t n4 = (n - head) >> 2, rest = (n - head) & 3u;
    constexpr uint32_t PU = 8;
    for (uint32_t i = 0; i < n4; i += 64u * PU) {
        u32x4 v[PU];
#pragma unroll
        for (uint32_t u = 0; u < PU; u++) {
            const uint32_t j = i + u * 64u + lane;
            v[u] = j < n4 ? m4[j] : u32x4{0u, 0u, 0u, 0u};
        }
#pragma unroll
        for (uint32_t u = 0; u < PU; u++)
            acc += meta_arena(v[u].x) + meta_arena(v[u].y) + meta_arena(v[u].z) + meta_arena(v[u].w);
    }
    if (lane < rest) acc += meta_arena(metas[head + 4u * n4 + lane]);
    return wave_sum(acc);
}

// one slice [dg0, dg1) of a region's merge path, joined into out[base ...]; returns the paths written
__device__ uint32_t join_slice(const RegionView& A, const RegionView& B, uint32_t dg0, uint32_t dg1,
                               uint8_t region_bit, uint64_t* __restrict__ out_h, uint8_t* __restrict__ out_k,
                               uint32_t base, uint32_t lane, bool* weq) {
    uint32_t ia0 = merge_split(A.keys, A.L, B.keys, B.L, dg0, lane), ib0 = dg0 - ia0;
    uint32_t ia1 = merge_split(A.keys, A.L, B.keys, B.L, dg1, lane), ib1 = dg1 - ia1;
    // an equal key straddling a split (A[ia - 1] last before it, B[ib] first after it) belongs to the
    // slice holding its A side
    if (ia0 > 0u && ib0 < B.L && A.keys[ia0 - 1u] == B.keys[ib0]) ib0++;
    if (ia1 > 0u && ib1 < B.L && A.keys[ia1 - 1u] == B.keys[ib1]) ib1++;
    RegionView As = A, Bs = B;
    As.keys += ia0;
    As.vals += ia0;
    As.metas += ia0;
    As.arena += arena_prefix(A.metas, ia0, lane);
    As.L = ia1 - ia0;
    Bs.keys += ib0;
    Bs.vals += ib0;
    Bs.metas += ib0;
    Bs.arena += arena_prefix(B.metas, ib0, lane);
    Bs.L = ib1 > ib0 ? ib1 - ib0 : 0u;
    return join_region<true>(As, Bs, region_bit, out_h, out_k, base, lane, weq);
}

// K4a: wave per scratch slot starting in [before.w, after.w) (this segment's deferred pairs: place_deferred);
// writes each slice's path count and whether all its paths are wire-equal number changes
__global__ __launch_bounds__(256) void k_join_slices(const gpudiff_pair_row* __restrict__ rows,
                                                     const uint8_t* __restrict__ pool, const uint8_t* __restrict__ flags,
                                                     const uint32_t* __restrict__ dirty_idx,
                                                     const uint32_t* __restrict__ scratch_off,
                                                     const uint32_t* __restrict__ slot_owner,
                                                     uint32_t* __restrict__ summary, const uint4* __restrict__ tot_before,
                                                     const uint4* __restrict__ tot_after, uint64_t scratch_cap,
                                                     uint64_t* __restrict__ sh, uint8_t* __restrict__ sk,
                                                     uint32_t* __restrict__ slice_cnt, uint8_t* __restrict__ slice_weq) {
    const uint32_t lane = lane_id();
    const uint32_t wave = uni((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
    if (summary[6] == 0u) return;  // K2 produced every pair's paths (no F_DEFER)
    const uint4 after = *tot_after;
    if ((uint64_t)after.w > scratch_cap) {  // the host grows the scratch and re-runs K4-K6
        if (blockIdx.x == 0 && threadIdx.x == 0) summary[4] = 1u;
        return;
    }
    const uint32_t s0 = slot_ceil(tot_before ? tot_before->w : 0u), s1 = slot_ceil(after.w);
    for (uint32_t s = s0 + wave; s < s1; s += nwaves) {
        const uint32_t d = uni(slot_owner[s]);
        if (d == kNoOwner) continue;  // inside a whole deferral (K3 joined it)
        const uint32_t so = uni(scratch_off[d]);
        const uint32_t i = s - slot_ceil(so);  // slice of this pair
        const uint32_t p = uni(dirty_idx[d]);
        const uint32_t f = uni((uint32_t)flags[p]);
        const gpudiff_pair_row r = rows[p];
        const uint32_t Ls = (f & F_JSPEC) ? r.spec_l_a + r.spec_l_b : 0u;
        const uint32_t Lt = (f & F_JSTAT) ? r.stat_l_a + r.stat_l_b : 0u;
        const uint32_t nsl = (Ls + kJoinSlice - 1u) / kJoinSlice, ntl = (Lt + kJoinSlice - 1u) / kJoinSlice;
        uint32_t cnt = 0;
        bool weq = true;
        if (i < nsl) {
            const RegionView A = region_view(pool, r.off_a, r.spec_l_a, r.spec_ar_a, false, r.spec_l_a);
            const RegionView B = region_view(pool, r.off_b, r.spec_l_b, r.spec_ar_b, false, r.spec_l_b);
            const uint32_t dg0 = i * kJoinSlice;
            cnt = join_slice(A, B, dg0, min(dg0 + kJoinSlice, Ls), 0, sh, sk, so + i * kJoinSlice, lane, &weq);
        } else if (i - nsl < ntl) {
            const RegionView A = region_view(pool, r.off_a, r.spec_l_a, r.spec_ar_a, true, r.stat_l_a);
            const RegionView B = region_view(pool, r.off_b, r.spec_l_b, r.spec_ar_b, true, r.stat_l_b);
            const uint32_t dg0 = (i - nsl) * kJoinSlice;
            cnt = join_slice(A, B, dg0, min(dg0 + kJoinSlice, Lt), GPUDIFF_PATH_REGION_STATUS, sh, sk,
                             so + i * kJoinSlice, lane, &weq);
        }
        if (lane == 0) {
            slice_cnt[s] = cnt;
            slice_weq[s] = weq ? 1u : 0u;
        }
    }
}

// K4b: wave per deferred pair of this segment, found as the first slot of its scratch (so the grid walks
// only deferred pairs, in parallel: one wave per 64 dirty pairs, walking the deferred ones in turn, took
// 53 us on config4, profiles/r03o); each deferred pair's slices are packed in order at the
// start of its scratch slot (moving left, 64 entries at a time: every entry is read before any write
// can reach it), the sentinel appended, its path count and no-op bits written
__global__ __launch_bounds__(256) void k_join_gather(const gpudiff_pair_row* __restrict__ rows,
                                                     const uint8_t* __restrict__ flags,
                                                     const uint32_t* __restrict__ dirty_idx,
                                                     const uint32_t* __restrict__ scratch_off,
                                                     const uint32_t* __restrict__ slot_owner,
                                                     const uint32_t* __restrict__ summary,
                                                     const uint4* __restrict__ tot_before,
                                                     const uint4* __restrict__ tot_after, uint64_t mask,
                                                     uint64_t* __restrict__ sh, uint8_t* __restrict__ sk,
                                                     const uint32_t* __restrict__ slice_cnt,
                                                     const uint8_t* __restrict__ slice_weq,
                                                     uint32_t* __restrict__ path_count, uint8_t* __restrict__ noop_d) {
    const uint32_t lane = lane_id();
    const uint32_t wave = uni((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
    if (summary[6] == 0u || summary[4] != 0u) return;
    const uint32_t s0 = slot_ceil(tot_before ? tot_before->w : 0u), s1 = slot_ceil(tot_after->w);
    for (uint32_t s = s0 + wave; s < s1; s += nwaves) {
        const uint32_t dk = uni(slot_owner[s]);
        if (dk == kNoOwner) continue;  // inside a whole deferral
        const uint32_t so = uni(scratch_off[dk]);
        if (s != slot_ceil(so)) continue;  // not its pair's first slot
        const uint32_t pk = uni(dirty_idx[dk]);
        const uint32_t fk = uni((uint32_t)flags[pk]);
        const gpudiff_pair_row r = rows[pk];
        const uint32_t Ls = (fk & F_JSPEC) ? r.spec_l_a + r.spec_l_b : 0u;
        const uint32_t Lt = (fk & F_JSTAT) ? r.stat_l_a + r.stat_l_b : 0u;
        const uint32_t nsl = (Ls + kJoinSlice - 1u) / kJoinSlice, ntl = (Lt + kJoinSlice - 1u) / kJoinSlice;
        const uint32_t s_first = s;  // = slot_ceil(so): the pair's first slot
        uint32_t n = 0;
        bool spec_weq = true, stat_weq = true;
        for (uint32_t i = 0; i < nsl + ntl; i++) {
            const uint32_t cnt = uni(slice_cnt[s_first + i]);
            const bool w = uni((uint32_t)slice_weq[s_first + i]) != 0u;
            if (i < nsl) spec_weq &= w;
            else stat_weq &= w;
            const uint32_t src = so + i * kJoinSlice, dst = so + n;
            if (src != dst)
                for (uint32_t q = 0; q < cnt; q += 64u) {
                    const bool act = q + lane < cnt;
                    uint64_t h = 0;
                    uint8_t kk = 0;
                    if (act) {
                        h = sh[src + q + lane];
                        kk = sk[src + q + lane];
                    }
                    __builtin_amdgcn_wave_barrier();
                    if (act) {
                        sh[dst + q + lane] = h;
                        sk[dst + q + lane] = kk;
                    }
                }
            n += cnt;
        }
        if (fk & F_SENT) {
            if (lane == 0) {
                sh[so + n] = status_sentinel_hash((r.flags_a >> GPUDIFF_OBJ_SEED_SHIFT) & 0xFFu, mask);
                sk[so + n] = GPUDIFF_PATH_REGION_STATUS | GPUDIFF_PATH_STATUS_ABSENT;
            }
            n += 1;
        }
        const bool stat_ok = stat_weq && (!(fk & F_SENT) || !(r.flags_a & GPUDIFF_OBJ_HAS_STATUS));
        if (lane == 0) {
            path_count[dk] = n;
            noop_d[dk] = (uint8_t)((((fk & F_SPEC) && spec_weq) ? NOOP_SPEC : 0u) |
                                   (((fk & F_STATUS) && stat_ok) ? NOOP_STATUS : 0u));
        }
    }
}

// ---------------------------------------------------------------- K2, flattened stream
// the chunks at the end of a launch handed out as smaller items (half a main item, at least 8 pairs), unless
// the whole launch is split already: a tail of q quarters of the launch's wave count, in 64-pair chunks
// items of the largest-first final round: one per resident wave, at most half the launch's main items
__host__ __device__ inline uint32_t k2_lpt_round(uint32_t n_full, uint32_t nwaves, uint32_t rounds) {
    const uint32_t want = rounds * nwaves;
    const uint32_t r = want < n_full / 2u ? want : n_full / 2u;
    return r < 2u ? 0u : r;
}
__host__ __device__ inline uint32_t k2_item_round(uint32_t n_main, uint32_t nwaves) {
    return n_main >= 3u * nwaves ? nwaves : 0u;  // one item per resident wave, when the bulk keeps two rounds
}
__host__ __device__ inline uint32_t k2_tail_chunks(uint32_t nch, uint32_t nwaves, uint32_t sub_shift, uint32_t q) {
    return sub_shift >= 3u ? 0u : min(nch, nwaves / 4u * q);
}
// One wave per work item of P = 64 >> sub_shift consecutive pairs.  Lane k
// loads pair k's 64-B row with four coalesced 16-B loads (one 4 KiB read per
// item instead of a scalar row load per pair).  The item's compared segments
// form one flattened index space of 16-B chunks (a wave prefix sum of the
// per-pair chunk counts); each pass the wave issues U x 64 chunk loads of A
// and of B with non-temporal 16-B loads, a chunk's owner pair found by a
// cross-lane binary search over the prefix sums.  So the HBM stream never
// waits at a pair boundary and no lane idles on a small pair (config3's pairs
// average ~200 chunks a side: a wave-per-pair pass leaves 1/5 of its loads
// unused and pays a row + data latency per pair).  A mismatching chunk marks
// its pair (spec or status region); then the wave merge-joins its dirty pairs
// one at a time into its arena (flags, caps, arena order and the F_DEFER rule:
// DESIGN.md §5).
// After its first item a wave takes the next one from a per-launch counter
// (summary[8], zeroed with the pass), fetched while it streams the
// current item, so the launch ends when the work does, not when the wave with
// the heaviest static share of items does; the last k2_tail_chunks() chunks are
// handed out as 8-pair items, so the final round of items is short too.
// K2 per-wave timeline (PROF: the timeline build only, selected by gpudiff_k2_profile, tools/k2_wave_profile.py): 12 u64 per wave --
// start, end of the first item, items, start of the last item, end, streaming ticks, join ticks,
// hardware id (wall clock: 100 MHz)
__device__ uint64_t* g_k2_prof;
__device__ uint32_t g_k2_prof_cap;

// HELP (the deep-pair kernel): the four waves of a workgroup share their current items through LDS.  An owner
// publishes its item (first pair, pairs, chunks) and claims its passes from the item's chunk cursor; a wave that
// finds no ticket left streams passes of a sibling's item from the same cursor and ORs its mismatch bits into the
// item's masks; the owner decides once every helper has left.  So the launch's last items -- single deep pairs
// streaming at a few GB/s each under full load -- end up to 4x sooner instead of holding the launch open while
// the other waves of their workgroups idle (profiles/r05a/wave_c4.json: 32% of the waves still running 20 us
// after the first ones ran out of work).  Waves only help after their own work is done, so the bulk is unchanged.
struct HelpSlot {
    uint32_t gen;      // odd while the owner (re)publishes
    uint32_t cursor;   // next unclaimed chunk of the item
    uint32_t total;    // chunks of the item
    uint32_t helpers;  // waves attached to the item
    uint32_t p0, cnt;  // its pairs
    uint64_t mis_s, mis_t;
};
// The slot protocol's ordering is stated in the memory model, not left to LDS executing a wave's
// operations in order: the owner's field stores are ordered before its closing gen store by release, and a helper's
// gen loads are acquires, so a helper that reads the same even gen before and after the fields (g1 == g2 == g, read
// AFTER its helpers increment) read the fields of that publication; the owner cannot republish while helpers != 0
// (it waits for 0 with acquire loads), so the fields stay put while the helper streams.  Mismatch bits go in with
// release ORs before the helper's release decrement, and the owner reads them after its acquire load of helpers == 0.
// All workgroup scope: LDS only, no cache maintenance.
__device__ __forceinline__ uint32_t lds_ld(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ uint64_t lds_ld64(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_st(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_or64(uint64_t* p, uint64_t v) {
    __hip_atomic_fetch_or(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ uint32_t lds_add(uint32_t* p, uint32_t v) {
    return __hip_atomic_fetch_add(p, v, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
}

template <int U, int MINB, bool PROF = false, bool HELP = false>
__global__ __launch_bounds__(256, MINB) void k_compare_flat(const gpudiff_pair_row* __restrict__ rows,
                                                      const uint8_t* __restrict__ pool, uint32_t n,
                                                      uint8_t* __restrict__ flags, uint32_t* __restrict__ caps,
                                                      uint4* __restrict__ chunk_counts, uint32_t c_begin,
                                                      uint32_t c_end, uint64_t* __restrict__ ah,
                                                      uint8_t* __restrict__ ak, uint32_t arena_off,
                                                      uint32_t arena_per_wave, uint32_t arena_stride,
                                                      uint32_t* __restrict__ path_src, uint32_t* __restrict__ path_cnt,
                                                      uint8_t* __restrict__ nbits, uint64_t mask,
                                                      uint32_t* __restrict__ summary, uint32_t sub_arg,
                                                      const uint32_t* __restrict__ tail_perm) {
    const uint32_t lane = lane_id();
    const uint32_t wave = uni((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
    // (launch_compare packs: sub_shift | tail quarters << 8 | largest-first rounds << 20 | item round << 22)
    const uint32_t sub_shift = sub_arg & 0xFFu, tail_q = (sub_arg >> 8) & 0xFFu;
    const uint32_t tail_ish = min(sub_shift + 1u, 3u);  // tail items: half a main item, at least 8 pairs
    const uint32_t wbase = arena_off + wave * arena_stride;
    uint32_t used = 0;  // entries of this wave's arena in use (wave-uniform)
    bool deferred = false;
    const uint64_t sent0 = status_sentinel_hash(0, mask);
    __shared__ HelpSlot help_slots[HELP ? 4 : 1];
    [[maybe_unused]] HelpSlot* const my = &help_slots[HELP ? (threadIdx.x >> 6) : 0];
    if constexpr (HELP) {
        if (lane == 0) {
            my->gen = my->cursor = my->total = my->helpers = my->p0 = my->cnt = 0u;
            my->mis_s = my->mis_t = 0ull;
        }
        __syncthreads();  // every slot initialised before a sibling reads it
    }
    // one pass of a wave over chunks [base, base + 64 U) of an item's flattened stream (lane k's registers: pair k's
    // inclusive chunk prefix, first chunk, spec chunks, arena adjustments and blob offsets); mismatching chunks mark
    // their pairs in mis_s / mis_t
    auto stream_pass = [&](uint32_t base, uint32_t total, uint32_t incl, uint32_t first, uint32_t n1, uint32_t adj_a,
                           uint32_t adj_b, uint64_t off_a, uint64_t off_b, uint64_t& mis_s, uint64_t& mis_t) {
        u32x4 va[U], vb[U];
        uint32_t own[U];
        bool st[U], act[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t g = base + (uint32_t)u * 64u + lane;
            act[u] = g < total;
            uint32_t o = 0;  // owner = number of lanes whose inclusive prefix is <= g
#pragma unroll
            for (uint32_t s = 32; s >= 1; s >>= 1)
                if (shfl32(incl, o + s - 1u) <= g) o += s;
            const uint32_t k = g - shfl32(first, o);
            st[u] = k >= shfl32(n1, o);
            const uint32_t xa = shfl32(adj_a, o), xb = shfl32(adj_b, o);
            const uint64_t oa = shfl64(off_a, o), ob = shfl64(off_b, o);
            own[u] = o;
            const uint64_t rel = 16ull * k;
            if (act[u]) {
                va[u] = __builtin_nontemporal_load((const u32x4*)(pool + oa + rel + (st[u] ? xa : 0u)));
                vb[u] = __builtin_nontemporal_load((const u32x4*)(pool + ob + rel + (st[u] ? xb : 0u)));
            }
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            uint64_t m = ballot(act[u] && neq16(va[u], vb[u]));
            while (m) {  // differing chunks: only in dirty pairs
                const uint32_t j = (uint32_t)__builtin_ctzll(m);
                m &= m - 1;
                const uint64_t bit = 1ull << (uint32_t)__builtin_amdgcn_readlane((int)own[u], (int)j);
                if (__builtin_amdgcn_readlane((int)(st[u] ? 1 : 0), (int)j)) mis_t |= bit;
                else mis_s |= bit;
            }
        }
    };
    [[maybe_unused]] uint64_t tp_start = 0, tp_first = 0, tp_last = 0, tp_stream = 0, tp_join = 0, tp_items = 0;
    [[maybe_unused]] uint64_t tp_rows = 0, tp_pre = 0, tp_post = 0, tp_adv = 0, tp_e = 0, tp_r = 0, tp_je = 0;
    if constexpr (PROF) tp_start = wall_clock64();
    const uint32_t nch = c_end - c_begin;
    const uint32_t tail_c = k2_tail_chunks(nch, nwaves, sub_shift, tail_q);
    const uint32_t n_full = (nch - tail_c) << sub_shift;  // items of 64 >> sub_shift pairs, then 8-pair items
    // largest-first final round (k2_lpt_round; large pairs): the pairs of the last lpt_r main items are handed
    // out one pair an item by the tail counter in tail_perm's order -- by descending bytes -- so the launch ends
    // with its smallest pairs; the bulk stays in index order (neighbouring waves stream neighbouring pool bytes)
    const uint32_t lpt_rounds = (sub_arg >> 20) & 3u;  // launch_compare: 0 when the round is off
    const uint32_t lpt_r = (tail_perm && tail_c == 0u && lpt_rounds) ? k2_lpt_round(n_full, nwaves, lpt_rounds) : 0u;
    const uint32_t n_main = n_full - lpt_r;
    // ... and the round before it in whole items, also largest first (sub_arg bit 22): its biggest items then start
    // a round earlier instead of running past the pair round's end
    const uint32_t r2 = (lpt_r && ((sub_arg >> 22) & 1u)) ? k2_item_round(n_main, nwaves) : 0u;
    const uint32_t n_main2 = n_main - r2;
    const uint32_t lpt_pairs = lpt_r << (6u - sub_shift);
    const uint32_t lpt_p0 = ((c_begin + (n_main >> sub_shift)) << 6) + (n_main & ((1u << sub_shift) - 1u)) * (64u >> sub_shift);
    const uint32_t nitems = lpt_r ? n_main + (lpt_r << (6u - sub_shift)) : n_full + (tail_c << tail_ish);
    // Two ticket counters per segment: main items are taken with a prefetch (the next main ticket as an
    // item starts, waited for only at its end); tail items from their own counter only when a wave is
    // free. With one counter a prefetch made as a long main item started could reserve a tail item,
    // which then waited behind that item (and its joins) while every other wave had run out of work
    // (the last ~0.13 ms of a 10M-pair pass, tools/k2_wave_profile.py).
    uint32_t* const ctr = summary + 8u + (arena_per_wave ? arena_off / arena_per_wave : 0u);
    uint32_t* const ctr_tail = ctr + kK2TailCounters;
    const uint32_t tail0 = max(n_main, nwaves);  // the first item the tail counter hands out
    auto advance = [&](uint32_t cur, uint32_t tk) -> uint32_t {
        if (cur < n_main) {
            const uint32_t nx = uni(__builtin_amdgcn_readlane(tk, 0)) + nwaves;
            if (nx < n_main) return nx;
        }
        uint32_t tt = 0;
        if (lane == 0) tt = atomicAdd(ctr_tail, 1u);
        return tail0 + uni(__builtin_amdgcn_readlane(tt, 0));
    };
    // The default kernel takes its next main ticket once the item's first pass is in flight (round 6): issued at the
    // item's start, the atomic's queue-loaded round trip was waited for together with the item's rows (vmcnt counts
    // in order).  Prefetching the next item's rows as well cut the per-item latency from 6.3 to 2.5 us in the
    // timeline but measured neutral (profiles/r06j): the saved time went into slower streaming -- the pass is
    // bandwidth-bound, not latency-bound.
    for (uint32_t it = wave, tk = 0; it < nitems; it = advance(it, tk)) {
        // the item this ticket stands for: in the largest-first round, one pair (the permuted order)
        const bool lpt = lpt_r && it >= n_main;
        // the largest-first rounds' dirty pairs join only up to kTailJoinMax keys here (bigger ones go to K4's
        // slices, spread over the whole grid): a deep join late in the launch would run past everyone's end
        const bool tail_round = lpt_r && it >= n_main2;
        const uint32_t im = lpt ? 0u : (r2 && it >= n_main2) ? n_main2 + tail_perm[lpt_pairs + (it - n_main2)] : it;
        const bool tail = !lpt && im >= n_full;
        // the next main ticket: fetched while this item streams
        if (HELP && it < n_main && lane == 0) tk = atomicAdd(ctr, 1u);
        [[maybe_unused]] uint64_t tp_i = 0;
        if constexpr (PROF) {
            tp_i = wall_clock64();
            if (tp_e) tp_adv += tp_i - tp_e;  // the previous item's end to this one's start (ticket)
            tp_last = tp_i;
            tp_items++;
        }
        const uint32_t ish = lpt ? 6u : tail ? tail_ish : sub_shift;
        const uint32_t j = tail ? im - n_full : im;
        const uint32_t lp = lpt ? lpt_p0 + tail_perm[it - n_main] : 0u;
        const uint32_t c = lpt ? lp >> 6 : c_begin + (tail ? nch - tail_c : 0u) + (j >> ish);
        const uint32_t per = 64u >> ish;
        const uint32_t p0 = lpt ? lp : (c << 6) + (j & ((1u << ish) - 1u)) * per;
        if (p0 >= n) {  // an item past the batch's end: still take the next ticket (advance() reads it)
            if (!HELP && it < n_main && lane == 0) tk = atomicAdd(ctr, 1u);
            continue;
        }
        const uint32_t cnt = min(per, n - p0);
        const bool valid = lane < cnt;
        // ---- rows: lane k holds pair p0 + k
        u32x4 v0 = {0, 0, 0, 0}, v1 = v0, v2 = v0, v3 = v0;
        if (valid) {
            const u32x4* rp = (const u32x4*)(rows + p0 + lane);
            v0 = rp[0];  // off_a, off_b
            v1 = rp[1];  // spec_l_a, spec_l_b, spec_ar_a, spec_ar_b
            v2 = rp[2];  // stat_l_a, stat_l_b, stat_ar_a, stat_ar_b
            v3 = rp[3];  // flags_a, flags_b, pair_id, cluster_id
        }
        if constexpr (PROF) {
            tp_r = wall_clock64();
            tp_rows += tp_r - tp_i;
        }
        const uint64_t off_a = ((uint64_t)v0.y << 32) | v0.x, off_b = ((uint64_t)v0.w << 32) | v0.z;
        const bool err = valid && ((v3.x | v3.y) & GPUDIFF_OBJ_DECODE_ERR) != 0u;
        const bool ok = valid && !err;
        const bool spec_sz = v1.x == v1.y && v1.z == v1.w;
        const bool has_st_b = (v3.y & GPUDIFF_OBJ_HAS_STATUS) != 0u;
        const bool stat_sz = has_st_b && v2.x == v2.y && v2.z == v2.w;
        const uint32_t seg_a = (uint32_t)seg_bytes(v1.x, v1.z), seg_b = (uint32_t)seg_bytes(v1.y, v1.w);
        const uint32_t seg_t = (uint32_t)seg_bytes(v2.x, v2.z);
        // whole 128-B lines wherever both sides' spans are equal: with both regions compared the stream
        // runs to the body's end (segments + zero pad, gpudiff_blob_body), with spec only and no status
        // leaves on either side the spec span is padded the same way; a stream that ends inside a line
        // costs a partial-line request per object (engine.h pair_compare_bytes counts the same chunks)
        const uint32_t r128 = ((seg_a + seg_t + 127u) & ~127u);
        const bool no_stat = (v2.x | v2.y | v2.z | v2.w) == 0u;
        const uint32_t n1 = (ok && spec_sz) ? ((!stat_sz && no_stat) ? ((seg_a + 127u) & ~127u) : seg_a) >> 4 : 0u;
        const uint32_t n2 = (ok && stat_sz) ? (spec_sz ? r128 - seg_a : seg_t) >> 4 : 0u;
        const uint32_t tot = n1 + n2;
        const uint32_t incl = wave_incl_scan(tot);
        const uint32_t total = uni(shfl32(incl, 63));
        const uint32_t first = incl - tot;
        // chunk k of a pair: spec chunk at off + 16k (k < n1), status chunk at off + seg + 16 (k - n1)
        const uint32_t adj_a = seg_a - 16u * n1, adj_b = seg_b - 16u * n1;
        uint64_t mis_s = 0, mis_t = 0;  // pairs with a differing spec / status chunk (wave-uniform)
        [[maybe_unused]] uint64_t tp_s0 = 0;
        if constexpr (PROF) {
            tp_s0 = wall_clock64();
            tp_pre += tp_s0 - tp_r;
        }
        if constexpr (HELP) {
            // publish the item (gen odd while the fields change; helpers of the previous item have left), then
            // claim passes from its cursor -- the first one up front, each next one while the current one streams
            if (lane == 0) lds_st(&my->gen, lds_ld(&my->gen) + 1u);
            while (uni(lds_ld(&my->helpers)) != 0u) __builtin_amdgcn_s_sleep(1);
            if (lane == 0) {
                lds_st(&my->p0, p0);
                lds_st(&my->cnt, cnt);
                lds_st(&my->total, total);
                __hip_atomic_store(&my->mis_s, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                __hip_atomic_store(&my->mis_t, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                lds_st(&my->cursor, 64u * U);
                lds_st(&my->gen, lds_ld(&my->gen) + 1u);
            }
            for (uint32_t base = 0; base < total;) {
                uint32_t nb = 0;
                if (lane == 0) nb = lds_add(&my->cursor, 64u * U);
                stream_pass(base, total, incl, first, n1, adj_a, adj_b, off_a, off_b, mis_s, mis_t);
                base = uni(__builtin_amdgcn_readlane(nb, 0));
            }
            if (lane == 0) {
                lds_or64(&my->mis_s, mis_s);
                lds_or64(&my->mis_t, mis_t);
            }
            while (uni(lds_ld(&my->helpers)) != 0u) __builtin_amdgcn_s_sleep(1);
            const uint64_t ms = lds_ld64(&my->mis_s), mt = lds_ld64(&my->mis_t);
            mis_s = ((uint64_t)uni((uint32_t)(ms >> 32)) << 32) | uni((uint32_t)ms);
            mis_t = ((uint64_t)uni((uint32_t)(mt >> 32)) << 32) | uni((uint32_t)mt);
        } else {
            uint32_t pass = 0;
            for (uint32_t base = 0; base < total; base += 64u * U, pass++) {
                stream_pass(base, total, incl, first, n1, adj_a, adj_b, off_a, off_b, mis_s, mis_t);
                if (pass == 0 && it < n_main && lane == 0) tk = atomicAdd(ctr, 1u);  // back by the next pass
            }
            if (pass == 0 && it < n_main && lane == 0) tk = atomicAdd(ctr, 1u);  // an item with nothing to stream
        }
        [[maybe_unused]] uint64_t tp_s1 = 0;
        if constexpr (PROF) {
            tp_s1 = wall_clock64();
            tp_stream += tp_s1 - tp_s0;
        }
        // ---- decisions (compare_pair's rules)
        uint32_t myflag = 0, mycap = 0, mysrc = 0, mycnt = 0, mynoop = 0;
        if (err) {
            myflag = F_SPEC | F_STATUS | F_ERR;
        } else if (valid) {
            const bool spec_dirty = !spec_sz || ((mis_s >> lane) & 1ull);
            const bool stat_dirty = !stat_sz || ((mis_t >> lane) & 1ull);
            const bool stat_join = stat_dirty && (v2.x + v2.y) != 0u;
            myflag = (spec_dirty ? F_SPEC | F_JSPEC : 0u) | (stat_dirty ? F_STATUS : 0u) | (stat_join ? F_JSTAT : 0u) |
                     (stat_dirty && !has_st_b ? F_SENT : 0u) | (((v3.x >> GPUDIFF_OBJ_SEED_SHIFT) & 0xFFu) ? F_SEED : 0u);
            mycap = (spec_dirty ? v1.x + v1.y : 0u) + (stat_dirty ? v2.x + v2.y + (has_st_b ? 0u : 1u) : 0u);
        }
        // ---- changed paths of the dirty pairs into this wave's arena.  First every pair whose only path is the
        // status-absent sentinel (every ConfigMap/Secret update: all of config2), one entry a lane, in one step
        const bool sent_only = valid && !err && (myflag & F_SENT) && !(myflag & (F_JSPEC | F_JSTAT));
        const uint64_t sm = ballot(sent_only);
        uint64_t done = 0;
        if (sm && used + popc64(sm) <= arena_per_wave) {
            if (sent_only) {
                const uint32_t src = wbase + used + popc64(sm & mask_lt(lane));
                ah[src] = (myflag & F_SEED) ? status_sentinel_hash((v3.x >> GPUDIFF_OBJ_SEED_SHIFT) & 0xFFu, mask) : sent0;
                ak[src] = GPUDIFF_PATH_REGION_STATUS | GPUDIFF_PATH_STATUS_ABSENT;
                mycap = 0;  // no K4 scratch slot needed
                mysrc = src;
                mycnt = 1;
                mynoop = sentinel_noop_bits(v3.x);
            }
            used += popc64(sm);
            done = sm;
        }
        // ... then the others one at a time, in pair order
        for (uint64_t dm = ballot((myflag & (F_SPEC | F_STATUS)) != 0u) & ~done; dm; dm &= dm - 1) {
            const uint32_t k = (uint32_t)__builtin_ctzll(dm);
            const uint32_t fk = (uint32_t)__builtin_amdgcn_readlane((int)myflag, (int)k);
            const uint32_t ck = (uint32_t)__builtin_amdgcn_readlane((int)mycap, (int)k);
            uint32_t src = 0, pc = 0, nb = 0;
            bool defer = false;
            if (used + ck <= arena_per_wave && ck <= (tail_round ? kTailJoinMax : kDeepJoin)) {
                src = wbase + used;
                if (fk & (F_JSPEC | F_JSTAT)) {
                    // the row again, as a scalar load (just read: an L2 hit), so the row registers are
                    // dead during the join
                    // (joining small pairs from a copy staged in LDS by direct-to-LDS loads cut config2's join time
                    // per item 32 -> 15 us but raised K2 to 137 VGPRs, 3 waves/SIMD: config3 at 10M lost 3.5%,
                    // profiles/r06m, r06n; staging K3's whole deferrals cost K3 4.5 us a pass in LDS occupancy)
                    const gpudiff_pair_row r = rows[p0 + k];
                    pc = join_pair<true>(r, fk, pool, mask, ah, ak, src, lane, &nb);
                } else if (fk & F_SENT) {  // status-absent only (every ConfigMap/Secret update)
                    const uint32_t fa = (uint32_t)__builtin_amdgcn_readlane((int)v3.x, (int)k);
                    nb = sentinel_noop_bits(fa);
                    if (lane == 0) {
                        ah[src] = (fk & F_SEED) ? status_sentinel_hash((fa >> GPUDIFF_OBJ_SEED_SHIFT) & 0xFFu, mask)
                                                : sent0;
                        ak[src] = GPUDIFF_PATH_REGION_STATUS | GPUDIFF_PATH_STATUS_ABSENT;
                    }
                    pc = 1;
                }
                used += pc;
            } else {
                defer = true;
                deferred = true;
            }
            if (lane == k) {
                if (defer) {
                    myflag |= F_DEFER;
                    mycap = defer_cap(v1.x, v1.y, v2.x, v2.y, myflag);  // whole K4 slices
                } else {
                    mycap = 0;  // no K4 scratch slot needed
                    mysrc = src;
                    mycnt = pc;
                    mynoop = nb;
                }
            }
        }
        if constexpr (PROF) {
            const uint64_t t = wall_clock64();
            tp_join += t - tp_s1;
            if (tp_items == 1) tp_first = t;
            tp_je = t;  // the item's end section starts here
        }
        const bool dirty = (myflag & (F_SPEC | F_STATUS)) != 0u;
        const uint32_t ns = popc64(ballot(myflag & F_SPEC));
        const uint32_t nt = popc64(ballot(myflag & F_STATUS));
        const uint32_t nd = popc64(ballot(dirty));
        const uint32_t cs = wave_sum(dirty ? mycap : 0u);
        if (valid) {
            flags[p0 + lane] = (uint8_t)myflag;
            if (dirty) {
                caps[p0 + lane] = mycap;
                path_src[p0 + lane] = mysrc;
                path_cnt[p0 + lane] = mycnt;
                nbits[p0 + lane] = (uint8_t)mynoop;
            }
        }
        if (lane == 0) {
            if (!ish) {
                chunk_counts[c] = make_uint4(ns, nt, nd, cs);
            } else if (ns | nt | nd | cs) {
                uint32_t* cc = (uint32_t*)(chunk_counts + c);
                atomicAdd(cc + 0, ns);
                atomicAdd(cc + 1, nt);
                atomicAdd(cc + 2, nd);
                atomicAdd(cc + 3, cs);
            }
        }
        if constexpr (PROF) {
            tp_e = wall_clock64();
            tp_post += tp_e - tp_je;
        }
    }
    if constexpr (HELP) {
        // no ticket left: stream passes of the siblings' items until none has an unclaimed chunk
        const uint32_t wib = threadIdx.x >> 6;
        for (bool any = true; any;) {
            any = false;
            for (uint32_t q = 1; q < 4; q++) {
                HelpSlot* const h = &help_slots[(wib + q) & 3u];
                const uint32_t g = uni(lds_ld(&h->gen));
                if ((g & 1u) || uni(lds_ld(&h->cursor)) >= uni(lds_ld(&h->total))) continue;
                any = true;
                if (lane == 0) lds_add(&h->helpers, 1u);
                const uint32_t g1 = uni(lds_ld(&h->gen));  // after the increment: the owner cannot republish now
                const uint32_t hp0 = uni(lds_ld(&h->p0)), hcnt = uni(lds_ld(&h->cnt)), htot = uni(lds_ld(&h->total));
                const uint32_t g2 = uni(lds_ld(&h->gen));
                if (g1 == g && g2 == g) {  // the item published at gen g: its geometry from its rows
                    u32x4 v0 = {0, 0, 0, 0}, v1 = v0, v2 = v0, v3 = v0;
                    const bool valid = lane < hcnt;
                    if (valid) {
                        const u32x4* rp = (const u32x4*)(rows + hp0 + lane);
                        v0 = rp[0];
                        v1 = rp[1];
                        v2 = rp[2];
                        v3 = rp[3];
                    }
                    const uint64_t off_a = ((uint64_t)v0.y << 32) | v0.x, off_b = ((uint64_t)v0.w << 32) | v0.z;
                    const bool ok = valid && ((v3.x | v3.y) & GPUDIFF_OBJ_DECODE_ERR) == 0u;
                    const bool spec_sz = v1.x == v1.y && v1.z == v1.w;
                    const bool stat_sz = (v3.y & GPUDIFF_OBJ_HAS_STATUS) != 0u && v2.x == v2.y && v2.z == v2.w;
                    const uint32_t seg_a = (uint32_t)seg_bytes(v1.x, v1.z), seg_b = (uint32_t)seg_bytes(v1.y, v1.w);
                    const uint32_t seg_t = (uint32_t)seg_bytes(v2.x, v2.z);
                    const uint32_t r128 = ((seg_a + seg_t + 127u) & ~127u);
                    const bool no_stat = (v2.x | v2.y | v2.z | v2.w) == 0u;
                    const uint32_t n1 =
                        (ok && spec_sz) ? ((!stat_sz && no_stat) ? ((seg_a + 127u) & ~127u) : seg_a) >> 4 : 0u;
                    const uint32_t n2 = (ok && stat_sz) ? (spec_sz ? r128 - seg_a : seg_t) >> 4 : 0u;
                    const uint32_t tot = n1 + n2;
                    const uint32_t incl = wave_incl_scan(tot);
                    const uint32_t first = incl - tot;
                    const uint32_t adj_a = seg_a - 16u * n1, adj_b = seg_b - 16u * n1;
                    uint64_t ms = 0, mt = 0;
                    for (;;) {
                        uint32_t nb = 0;
                        if (lane == 0) nb = lds_add(&h->cursor, 64u * U);
                        nb = uni(__builtin_amdgcn_readlane(nb, 0));
                        if (nb >= htot) break;
                        stream_pass(nb, htot, incl, first, n1, adj_a, adj_b, off_a, off_b, ms, mt);
                    }
                    if (lane == 0) {
                        if (ms) lds_or64(&h->mis_s, ms);
                        if (mt) lds_or64(&h->mis_t, mt);
                    }
                }
                if (lane == 0) __hip_atomic_fetch_sub(&h->helpers, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
    }
    if (deferred && lane == 0) summary[6] = 1u;
    if constexpr (PROF) {
        const uint64_t t_end = wall_clock64();
        if (lane == 0 && g_k2_prof && wave < g_k2_prof_cap) {
            uint64_t* r = g_k2_prof + 12ull * wave;
            r[0] = tp_start;
            r[1] = tp_first;
            r[2] = tp_items;
            r[3] = tp_last;
            r[4] = t_end;
            r[5] = tp_stream;
            r[6] = tp_join;
            r[7] = (uint64_t)__smid();
            r[8] = tp_rows;
            r[9] = tp_pre;
            r[10] = tp_post;
            r[11] = tp_adv;
        }
    }
}


hipError_t k2_profile(uint64_t* dev_buf, uint32_t cap_waves) {
    hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_k2_prof), &dev_buf, sizeof(dev_buf));
    if (e != hipSuccess) return e;
    return hipMemcpyToSymbol(HIP_SYMBOL(g_k2_prof_cap), &cap_waves, sizeof(cap_waves));
}

// ---------------------------------------------------------------- K6
// Lane per dirty pair (most pairs have 1-3 paths); pairs with many paths
// (list shifts in deep objects) are copied by the whole wave.
__global__ __launch_bounds__(256) void k_copy_paths(const uint32_t* __restrict__ summary,
                                                    const uint32_t* __restrict__ scratch_off,
                                                    const uint32_t* __restrict__ path_off,
                                                    const uint32_t* __restrict__ path_count,
                                                    const uint64_t* __restrict__ sh, const uint8_t* __restrict__ sk,
                                                    const uint64_t* __restrict__ ah, const uint8_t* __restrict__ ak,
                                                    uint64_t* __restrict__ oh, uint8_t* __restrict__ ok) {
    const uint32_t lane = lane_id();
    const uint32_t wave = uni((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
    const uint32_t ndirty = summary[2];
    if (summary[4]) return;  // scratch overflow: the host grows the slot pool and re-runs K4-K6
    const uint32_t nchunks = (ndirty + 63u) >> 6;
    for (uint32_t c = wave; c < nchunks; c += nwaves) {
        const uint32_t d = (c << 6) + lane;
        const bool valid = d < ndirty;
        const uint32_t sraw = valid ? scratch_off[d] : 0u;
        const bool arena = (sraw & ARENA_BIT) != 0u;  // written by K2 (else K4's scratch)
        const uint32_t so = sraw & ~ARENA_BIT;
        const uint32_t po = valid ? path_off[d] : 0u;
        const uint32_t cnt = valid ? path_count[d] : 0u;
        const uint64_t* srch = arena ? ah : sh;
        const uint8_t* srck = arena ? ak : sk;
        const bool big = cnt > 16u;
        if (!big)
            for (uint32_t i = 0; i < cnt; i++) {
                oh[po + i] = srch[so + i];
                ok[po + i] = srck[so + i];
            }
        uint64_t m = ballot(big);
        while (m) {
            const uint32_t k = (uint32_t)__builtin_ctzll(m);
            m &= m - 1;
            const uint32_t sok = uni(shfl32(so, k)), pok = uni(shfl32(po, k)), ck = uni(shfl32(cnt, k));
            const bool ak_ = uni(shfl32(arena ? 1u : 0u, k)) != 0u;
            const uint64_t* bh = ak_ ? ah : sh;
            const uint8_t* bk = ak_ ? ak : sk;
            for (uint32_t i = lane; i < ck; i += 64) {
                oh[pok + i] = bh[sok + i];
                ok[pok + i] = bk[sok + i];
            }
        }
    }
}

// ---------------------------------------------------------------- object store compaction
// Wave per live blob: copies it from the old space to its packed offset in
// the new one with 16-B loads/stores (blobs are 16-B aligned and sized).
__global__ __launch_bounds__(256) void k_move_blobs(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                    const BlobMove* __restrict__ moves, uint32_t n) {
    const uint32_t lane = lane_id();
    const uint32_t wave = uni((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
    for (uint32_t i = wave; i < n; i += nwaves) {
        const BlobMove m = moves[i];
        const u32x4* s4 = (const u32x4*)(src + m.src);
        u32x4* d4 = (u32x4*)(dst + m.dst);
        const uint64_t n16 = m.bytes >> 4;
        for (uint64_t k = lane; k < n16; k += 64) d4[k] = __builtin_nontemporal_load(s4 + k);
    }
}

// ---------------------------------------------------------------- ingest helper
__global__ __launch_bounds__(256) void k_rebase_rows(gpudiff_pair_row* __restrict__ rows, uint32_t begin, uint32_t end,
                                                     uint64_t base, uint32_t* __restrict__ pair_ids) {
    const uint32_t i = begin + blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= end) return;
    rows[i].off_a += base;
    rows[i].off_b += base;
    pair_ids[i] = rows[i].pair_id;
}

// ---------------------------------------------------------------- launchers
static inline uint32_t grid_for(uint64_t waves_wanted, uint32_t cap_blocks) {
    uint64_t blocks = (waves_wanted + 3) / 4;
    if (blocks < 1) blocks = 1;
    return (uint32_t)(blocks < cap_blocks ? blocks : cap_blocks);
}

// 256 CUs x 8 resident 256-thread workgroups
static constexpr uint32_t kPersistBlocks = 256 * 8;

hipError_t launch_rebase(hipStream_t s, gpudiff_pair_row* rows, uint32_t begin, uint32_t end, uint64_t base,
                         uint32_t* pair_ids) {
    if (end <= begin) return hipSuccess;
    k_rebase_rows<<<(end - begin + 255) / 256, 256, 0, s>>>(rows, begin, end, base, pair_ids);
    return hipGetLastError();
}



hipError_t launch_move_blobs(hipStream_t s, const uint8_t* src, uint8_t* dst, const BlobMove* moves, uint32_t n) {
    if (!n) return hipSuccess;
    k_move_blobs<<<grid_for(n, kPersistBlocks), 256, 0, s>>>(src, dst, moves, n);
    return hipGetLastError();
}

// The decision kernels: 8 x 16-B chunks a side in flight per lane at 4 waves/SIMD (123 VGPRs, round 6) by default, 16 at
// 2 waves/SIMD for deep pairs (>= kK2BigPairBytes a pair on average), each also as the per-wave timeline build
// (gpudiff_k2_profile, tools/k2_wave_profile.py).  In-process A/B (profiles/r04p): 8 in flight beat round
// 3's 4 at 4 waves on every shape -- config3 10M K2 8.21 vs 8.28 ms, the N = 8 share 1.147 vs 1.164, config4 1.080
// vs 1.091 -- and 16 wins only on deep pairs (config4 1.043 ms, but config3 8.44 and the share 1.195): when the
// items are 16-256 KiB the last round's waves stream alone and their own loads in flight set the tail's rate.
// Rejected and removed in round 5 (measurements in DESIGN.md §5, §6): a wave per pair (k_compare),
// 2 / 4 / 12 chunks in flight, plain loads, rows prefetched into LDS, static striding.
typedef void (*K2Fn)(const gpudiff_pair_row*, const uint8_t*, uint32_t, uint8_t*, uint32_t*, uint4*, uint32_t, uint32_t,
                     uint64_t*, uint8_t*, uint32_t, uint32_t, uint32_t, uint32_t*, uint32_t*, uint8_t*, uint64_t,
                     uint32_t*, uint32_t, const uint32_t*);
constexpr uint32_t kK2Kernels = 4;
static K2Fn k2_kernel(uint32_t k) {
    switch (k) {
        case 1: return k_compare_flat<16, 1, false, true>;
        case 2: return k_compare_flat<8, 1, true>;
        case 3: return k_compare_flat<16, 1, true, true>;
        default: return k_compare_flat<8, 1>;
    }
}

constexpr uint64_t kK2BigPairBytes = 16384;
static uint32_t k2_variant_of(const DiffBuffers& b) {
    return (b.avg_pair_bytes >= kK2BigPairBytes ? 1u : 0u) | (b.k2_timeline ? 2u : 0u);
}

constexpr uint32_t kK2LptMax = 16384;  // largest-first rounds: at most this many pairs (one block sorts them in LDS)
// largest-first rounds for deep pairs: one round of single pairs (two scatter the stream further: config4 K2
// 1.093 ms vs 1.060 with one and 1.070 in index order, profiles/r04w), after one round of whole items sorted the
// same way (-0.4%, profiles/r04zk); in both, joins over kTailJoinMax keys are deferred to K4
constexpr uint32_t kK2LptRounds = 1;
constexpr uint32_t kK2MaxSubShift = 3;  // items of >= 64 >> 3 = 8 pairs
// 64-pair chunks are split into 2^k items until every resident K2 wave has at least this many
constexpr uint32_t kK2ItemsPerWave = 6;  // >= 6 items per resident wave: config3 at the N = 8 share (19.5k chunks) and config2 (15.6k) both split to 32-pair items, the best of 4 / 8 on each (profiles/r02zz3)

static uint32_t k2_cap_blocks(const DiffBuffers& b) {
    // one resident 256-thread block per CU per wave slot a SIMD offers the
    // kernel (its measured occupancy, hipOccupancyMaxActiveBlocksPerMultiprocessor):
    // a larger grid would leave blocks waiting for a free slot, i.e. a tail
    static int occ[kK2Kernels] = {0};
    const uint32_t v = k2_variant_of(b);
    if (!occ[v]) {
        int n = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, reinterpret_cast<const void*>(k2_kernel(v)), 256, 0) !=
                hipSuccess || n <= 0)
            n = 4;
        occ[v] = n;
    }
    // another pass over the population in flight (DiffBuffers::k2_shared): half the resident grid, so both fit --
    // the default kernel only: the deep-pair kernel's 2 waves/SIMD halved lost 7% of config4's two-in-flight step
    // (profiles/r06ac)
    return 256u * (uint32_t)((b.k2_shared && !(v & 1u)) ? std::max(1, occ[v] / 2) : occ[v]);
}

// Deep pairs (>= 16 KiB of compared bytes on average: config4's 8-64 KiB objects) are split below
// 8-pair items, until >= 8 items per resident wave: with 8-pair items a config4 wave had 2-5 items of
// ~0.5 MB each and the pass ended ~0.5 ms after the median wave (tools/k2_wave_profile.py,
// profiles/r03e/wave_c4.json: 68% of the span busy); in-process A/B on config4 (profiles/r03h,
// r03i ab_c4.json): 1-pair items 1.56 ms, 2-pair 1.21, 4-pair 1.26-1.28 -- 8 per wave gives 2-pair
constexpr uint32_t kK2ItemsPerWaveBig = 8, kK2MaxSubShiftBig = 6;

// 64-pair chunks split into 2^k items until there are >= kK2ItemsPerWave items per resident wave
// (config3's 156k chunks: k = 0; deep pairs: see above)
static uint32_t k2_sub_shift(const DiffBuffers& b, uint32_t nchunks) {
    const bool big = b.avg_pair_bytes >= kK2BigPairBytes;
    const uint64_t want = (uint64_t)(big ? kK2ItemsPerWaveBig : kK2ItemsPerWave) * 4u * k2_cap_blocks(b);
    const uint32_t max_shift = big ? kK2MaxSubShiftBig : kK2MaxSubShift;
    // items of at least 8 pairs: a small batch (a watch-replay batch of 64k events: 1k chunks) split
    // further than that pays a row load, a prefix sum and a ticket per 2-4 pairs (config5: K2 0.42 ms
    // at 2-pair items vs 0.26 at 4 -- profiles/r02zy)
    uint32_t k = 0;
    while (k < max_shift && (uint64_t)nchunks << k < want) k++;
    return k;
}

uint32_t k2_grid_waves(const DiffBuffers& b, uint32_t nchunks) {
    const uint64_t items = (uint64_t)nchunks << k2_sub_shift(b, nchunks);
    return grid_for(items, k2_cap_blocks(b)) * 4u;
}

// A pass's zeroing in one launch (hipMemsetAsync is a fill kernel each): the summary words (when the pass
// starts with this K2 launch) and the chunk counts that split chunks accumulate with atomics
__global__ __launch_bounds__(256) void k_pass_reset(uint32_t* __restrict__ summary, uint32_t nwords,
                                                    uint4* __restrict__ cc, uint32_t ncc) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (summary && i < nwords) summary[i] = 0u;
    for (uint32_t j = i; j < ncc; j += gridDim.x * 256u) cc[j] = make_uint4(0u, 0u, 0u, 0u);
}

// bytes K2 streams for a pair (the rule of its n1 / n2 chunk counts; gpudiff_pair_compare_bytes on the host)
__device__ __forceinline__ uint64_t pair_stream_bytes(const gpudiff_pair_row& r) {
    if ((r.flags_a | r.flags_b) & GPUDIFF_OBJ_DECODE_ERR) return 65u;
    const bool spec_sz = r.spec_l_a == r.spec_l_b && r.spec_ar_a == r.spec_ar_b;
    const bool stat_sz = (r.flags_b & GPUDIFF_OBJ_HAS_STATUS) && r.stat_l_a == r.stat_l_b && r.stat_ar_a == r.stat_ar_b;
    const uint64_t seg_s = seg_bytes(r.spec_l_a, r.spec_ar_a), seg_t = seg_bytes(r.stat_l_a, r.stat_ar_a);
    uint64_t per = 0;
    if (spec_sz && stat_sz) per = (seg_s + seg_t + 127u) & ~127ull;
    else if (spec_sz) per = (r.stat_l_a | r.stat_l_b | r.stat_ar_a | r.stat_ar_b) ? seg_s : (seg_s + 127u) & ~127ull;
    else if (stat_sz) per = seg_t;
    return 65u + 2u * per;
}

// The largest-first final round's order (large pairs): one block sorts the pairs of the last round's main items
// by their compared bytes, descending (ties by index), into perm (offsets from the round's first pair).
// Cached per batch by the host (launch_compare): the order depends only on the rows and the launch shape, and
// any permutation is correct -- a stale one only orders the round less well.
// one block: sorts key[0, r) ascending (bitonic, padded to a power of two with ~0)
__device__ void block_sort_u32(uint32_t* key, uint32_t r) {
    uint32_t m2 = 1;
    while (m2 < r) m2 <<= 1;
    for (uint32_t t = r + threadIdx.x; t < m2; t += blockDim.x) key[t] = ~0u;
    __syncthreads();
    for (uint32_t k = 2; k <= m2; k <<= 1)
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t i = threadIdx.x; i < m2; i += blockDim.x) {
                const uint32_t l = i ^ j;
                if (l > i) {
                    const uint32_t a = key[i], bb = key[l];
                    if (((i & k) == 0) == (a > bb)) {
                        key[i] = bb;
                        key[l] = a;
                    }
                }
            }
            __syncthreads();
        }
}

__global__ __launch_bounds__(1024) void k_tail_order(const gpudiff_pair_row* __restrict__ rows, uint32_t n,
                                                     uint32_t p_first, uint32_t r, uint32_t c_begin, uint32_t n_main2,
                                                     uint32_t r2, uint32_t sub_shift, uint32_t* __restrict__ perm) {
    __shared__ uint32_t key[kK2LptMax];  // 64 KiB
    // the last round's pairs: descending bytes (in 16-B units, saturating at 1 MiB), ascending index -- sort
    // ascending on (~bytes16, t); padding sorts last
    for (uint32_t t = threadIdx.x; t < r; t += blockDim.x) {
        const uint32_t p = p_first + t;
        const uint64_t bytes = p < n ? pair_stream_bytes(rows[p]) : 0u;
        const uint32_t b16 = (uint32_t)min(bytes >> 4, (uint64_t)0xFFFFu);
        key[t] = ((0xFFFFu - b16) << 16) | t;
    }
    block_sort_u32(key, r);
    for (uint32_t t = threadIdx.x; t < r; t += blockDim.x) perm[t] = key[t] & 0xFFFFu;
    __syncthreads();
    // the round before, in whole items of 64 >> sub_shift pairs (32-B units, saturating at 2 MiB)
    const uint32_t per = 64u >> sub_shift;
    for (uint32_t t = threadIdx.x; t < r2; t += blockDim.x) {
        const uint32_t m = n_main2 + t;
        const uint32_t p0 = ((c_begin + (m >> sub_shift)) << 6) + (m & ((1u << sub_shift) - 1u)) * per;
        uint64_t bytes = 0;
        for (uint32_t p = p0; p < min(p0 + per, n); p++) bytes += pair_stream_bytes(rows[p]);
        const uint32_t b32 = (uint32_t)min(bytes >> 5, (uint64_t)0xFFFFu);
        key[t] = ((0xFFFFu - b32) << 16) | t;
    }
    if (r2) {
        block_sort_u32(key, r2);
        for (uint32_t t = threadIdx.x; t < r2; t += blockDim.x) perm[r + t] = key[t] & 0xFFFFu;
    }
}

// the launch's largest-first round (0 = none): large pairs only, no pair-split tail (k2_tail_chunks() == 0: the
// items of large pairs are split to 1-2 pairs already)
static uint32_t k2_lpt_items(const DiffBuffers& b, uint32_t nch, uint32_t nwaves, uint32_t sub, uint32_t tail) {
    if (!b.tail_perm || tail || b.avg_pair_bytes < kK2BigPairBytes) return 0;
    const uint32_t r = k2_lpt_round(nch << sub, nwaves, kK2LptRounds);
    // the round's pairs and the item round before it are sorted in one block's LDS / kept in tail_perm
    return (r << (6u - sub)) + k2_item_round((nch << sub) - r, nwaves) <= kK2LptMax ? r : 0;
}

hipError_t launch_compare(hipStream_t s, const DiffBuffers& b) {
    const uint32_t nch = (b.n_pairs + 63u) / 64u;
    const dim3 grid(k2_grid_waves(b, nch) / 4u);
    uint4* cc = (uint4*)b.chunk_counts;
    const uint32_t sub = k2_sub_shift(b, nch);
    const uint32_t v = k2_variant_of(b);
    const uint32_t tq = kK2TailQuarters;
    const uint32_t tail = k2_tail_chunks(nch, grid.x * 4u, sub, tq);
    const uint32_t lpt = k2_lpt_items(b, nch, grid.x * 4u, sub, tail);
    const uint32_t* perm = nullptr;
    if (lpt) {
        const uint32_t n_main = (nch << sub) - lpt;
        const uint32_t p_first = ((n_main >> sub) << 6) + (n_main & ((1u << sub) - 1u)) * (64u >> sub);
        const uint32_t r2 = k2_item_round(n_main, grid.x * 4u);
        // the order depends on the rows and the launch shape: cached under the exact tuple (a permutation made
        // for another round size would visit pairs outside the round, or one twice -- ADVICE r4)
        const TailPermKey key{b.rows, b.rows_gen, b.n_pairs, lpt, sub, r2};
        if (!(*b.tail_perm_key == key)) {
            k_tail_order<<<1, 1024, 0, s>>>(b.rows, b.n_pairs, p_first, lpt << (6u - sub), 0u, n_main - r2, r2, sub,
                                            b.tail_perm);
            *b.tail_perm_key = key;
        }
        perm = b.tail_perm;
    }
    {  // one launch zeroes the summary and the chunk counts split items accumulate with atomics
        const uint32_t z0 = sub ? 0u : lpt ? (((nch << sub) - lpt) >> sub) : nch - tail;
        const uint32_t ncc = nch - z0;
        k_pass_reset<<<std::max(1u, std::min(1024u, (ncc + 255u) / 256u)), 256, 0, s>>>(b.summary, kSummaryWords,
                                                                                        cc + z0, ncc);
    }
    // sub_arg: sub_shift | tail quarters << 8 | largest-first rounds << 20 | item round << 22
    const uint32_t sub_arg = sub | (tq << 8) | (lpt ? kK2LptRounds << 20 | 1u << 22 : 0u);
    k2_kernel(v)<<<grid, 256, 0, s>>>(b.rows, b.pool, b.n_pairs, b.flags, b.caps, cc, 0u, nch, b.arena_h, b.arena_k, 0u,
                                      b.arena_per_wave, b.arena_per_wave, b.path_src, b.path_cnt, b.nbits, b.hash_mask,
                                      b.summary, sub_arg, perm);
    return hipGetLastError();
}

// k_compact's grid: one resident block per CU per slot its occupancy allows (it carries the whole-deferral
// join, so it holds more VGPRs than a plain compaction; a larger grid would only queue blocks)
static uint32_t compact_cap_blocks() {
    static int occ = 0;
    if (!occ) {
        int n = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, reinterpret_cast<const void*>(k_compact), 256, 0) !=
                hipSuccess || n <= 0)
            n = 4;
        occ = n;
    }
    return std::min<uint32_t>(kPersistBlocks, 256u * (uint32_t)occ);
}

// K3 over the chunks [c0, c1) of one segment: running totals before -> after
hipError_t launch_compact(hipStream_t s, const DiffBuffers& b, uint32_t c0, uint32_t c1, const uint4* before,
                          uint4* after) {
    const uint32_t n = c1 - c0;
    const uint32_t ntiles = (n + SCAN_TILE - 1) / SCAN_TILE;
    V4* cc = (V4*)b.chunk_counts + c0;
    V4* ts = (V4*)b.tile_sums;
    if (ntiles) k_scan_tiles<V4><<<ntiles, 256, 0, s>>>(cc, nullptr, n, ts);
    // the bound gather buffer's counts: the batch totals, written with the last segment's (the total's) scan
    uint32_t* mirror = (b.gather_send && (const void*)after == (const void*)b.summary) ? b.gather_send : nullptr;
    k_scan_apply<V4><<<std::max(ntiles, 1u), 256, 0, s>>>(cc, nullptr, n, ts, (const V4*)before, (V4*)after, cc,
                                                          false, mirror);
    k_compact<<<grid_for(n, compact_cap_blocks()), 256, 0, s>>>(
        b.flags, b.caps, b.pair_ids, b.n_pairs, (const uint4*)b.chunk_counts, b.spec_ids, b.status_ids, b.dirty_ids,
        b.dirty_idx, b.scratch_off, c0, c1, b.path_src, b.path_cnt, b.path_count, b.nbits, b.noop_d, b.slot_owner,
        b.scratch_cap, b.rows, b.pool, b.hash_mask, b.scratch_h, b.scratch_k, b.gather_send, b.gather_cap_spec,
        b.gather_cap_status);
    return hipGetLastError();
}

hipError_t launch_join(hipStream_t s, const DiffBuffers& b, uint32_t c0, uint32_t c1, const uint4* before,
                       const uint4* after) {
    // K4a: a resident grid walks the segment's slices (their number is on the device); exits at once
    // when K2 deferred nothing.  The slices can never outnumber the scratch's slots (a larger need is the
    // overflow re-run, after the scratch grew), so the grid is at most one wave per slot: an empty K4
    // over the default 64k-entry scratch costs a 16-block launch, not 2048 blocks (~4 us each)
    const uint32_t k4_blocks = (uint32_t)std::min<uint64_t>(kPersistBlocks,
                                                            (b.scratch_cap / kJoinSlice + 3u) / 4u + 1u);
    (void)c0;
    (void)c1;
    k_join_slices<<<k4_blocks, 256, 0, s>>>(b.rows, b.pool, b.flags, b.dirty_idx, b.scratch_off, b.slot_owner,
                                                 b.summary, before, after, b.scratch_cap, b.scratch_h, b.scratch_k,
                                                 b.slice_cnt, b.slice_weq);
    k_join_gather<<<k4_blocks, 256, 0, s>>>(b.rows, b.flags, b.dirty_idx, b.scratch_off, b.slot_owner,
                                                                     b.summary, before, after, b.hash_mask,
                                                                     b.scratch_h, b.scratch_k, b.slice_cnt,
                                                                     b.slice_weq, b.path_count, b.noop_d);
    return hipGetLastError();
}

hipError_t launch_slot_owners(hipStream_t s, const DiffBuffers& b) {
    k_slot_owners<<<compact_cap_blocks(), 256, 0, s>>>(b.flags, b.caps, b.dirty_idx, b.scratch_off, b.summary,
                                                       b.scratch_cap, b.slot_owner, b.rows, b.pool, b.hash_mask,
                                                       b.scratch_h, b.scratch_k, b.path_count, b.noop_d);
    return hipGetLastError();
}

hipError_t launch_emit(hipStream_t s, const DiffBuffers& b) {
    const uint32_t ntiles = b.n_pairs / SCAN_TILE + 1;  // >= (n_dirty - 1) / SCAN_TILE + 1 workgroups
    const uint32_t* nd = b.summary + 2;
    k_scan_tiles<uint32_t><<<ntiles, 256, 0, s>>>(b.path_count, nd, 0, b.tile_sums);
    k_scan_apply<uint32_t><<<ntiles, 256, 0, s>>>(b.path_count, nd, 0, b.tile_sums, nullptr, b.summary + 5,
                                                  b.path_off, true, nullptr);
    k_copy_paths<<<grid_for((b.n_pairs + 63) / 64, kPersistBlocks), 256, 0, s>>>(
        b.summary, b.scratch_off, b.path_off, b.path_count, b.scratch_h, b.scratch_k, b.arena_h, b.arena_k, b.out_h,
        b.out_k);
    return hipGetLastError();
}

}  // namespace gd
