// CPU merge over the canonical CSR encoding -- the "cpu-csr" line of
// BASELINE.md §2 (TEST INFRASTRUCTURE / CPU BASELINE ONLY: never linked into
// the product).
//
// Restates on the host what the device diff pass computes from the same
// blobs (include/gpudiff_format.h): per pair the spec decision
// of deepEqualApartFromStatus (pkg/syncer/specsyncer.go:17-41) as "the two
// spec segments are byte-identical", the status decision of deepEqualStatus
// (pkg/syncer/statussyncer.go:15-27) as "B has a status key and the status
// segments are byte-identical", and for a dirty pair the build-defined
// field-path diff as a merge-join of the two sorted
// key arrays: equal keys whose (meta, value) differ are CHANGED, keys only in
// A REMOVED, only in B ADDED; a long string is its first 8 bytes in the value
// slot plus its tail in the arena, and both are compared.  Written from the format definition, not
// from the kernels' code; parity with the device is checked by the bench's
// three-way sample check and tests/test_oracle_cpp.py.
#include <stdint.h>
#include <string.h>

#include <chrono>
#include <thread>
#include <vector>

#include "../include/gpudiff.h"
#include "../include/gpudiff_format.h"
#include "timed_threads.h"
#include "xxh64_ref.h"

namespace {

struct Seg {
    const uint8_t* p;
    uint32_t l, ar;
    const uint64_t* vals() const { return (const uint64_t*)p; }
    const uint32_t* keys() const { return (const uint32_t*)(p + 8ull * l); }
    const uint32_t* metas() const { return (const uint32_t*)(p + 12ull * l); }
    const uint8_t* arena() const { return p + 16ull * l; }
    uint64_t bytes() const { return gpudiff_seg_bytes(l, ar); }
};

bool seg_equal(const Seg& a, const Seg& b) {
    return a.l == b.l && a.ar == b.ar && memcmp(a.p, b.p, a.bytes()) == 0;
}

// merge-join of two segments: (hash, kind | region) in ascending hash order
template <class Emit>
void join(const Seg& a, const Seg& b, uint8_t region, Emit&& emit) {
    uint32_t i = 0, j = 0;
    uint64_t oa = 0, ob = 0;  // arena offsets of the next long value
    const uint32_t *ka = a.keys(), *kb = b.keys();
    const uint64_t *va = a.vals(), *vb = b.vals();
    const uint32_t *ma = a.metas(), *mb = b.metas();
    while (i < a.l || j < b.l) {
        if (j >= b.l || (i < a.l && ka[i] < kb[j])) {
            emit(ka[i], (uint8_t)(GPUDIFF_PATH_REMOVED | region));
            oa += gpudiff_meta_arena(ma[i]);
            i++;
        } else if (i >= a.l || kb[j] < ka[i]) {
            emit(kb[j], (uint8_t)(GPUDIFF_PATH_ADDED | region));
            ob += gpudiff_meta_arena(mb[j]);
            j++;
        } else {
            bool same = ma[i] == mb[j] && va[i] == vb[j];
            if (same && gpudiff_meta_is_long(ma[i]))
                same = memcmp(a.arena() + oa, b.arena() + ob, gpudiff_meta_len(ma[i]) - GPUDIFF_INLINE_MAX) == 0;
            if (!same) emit(ka[i], (uint8_t)(GPUDIFF_PATH_CHANGED | region));
            oa += gpudiff_meta_arena(ma[i]);
            ob += gpudiff_meta_arena(mb[j]);
            i++;
            j++;
        }
    }
}

uint64_t status_sentinel(uint32_t seed) {
    uint8_t comp[11] = {0x01, 6, 0, 0, 0, 's', 't', 'a', 't', 'u', 's'};
    return oracle::xxh64_ref(comp, sizeof comp, seed) & ((1ull << GPUDIFF_PATH_HASH_BITS) - 1);  // the build's width
}

// one pair: flags (bit0 spec, bit1 status, bit2 decode error); paths via emit
template <class Emit>
uint8_t diff_pair(const uint8_t* pool, const gpudiff_pair_row& r, Emit&& emit) {
    if ((r.flags_a | r.flags_b) & GPUDIFF_OBJ_DECODE_ERR) return 7;
    const Seg sa{pool + r.off_a, r.spec_l_a, r.spec_ar_a}, sb{pool + r.off_b, r.spec_l_b, r.spec_ar_b};
    const Seg ta{pool + r.off_a + sa.bytes(), r.stat_l_a, r.stat_ar_a},
        tb{pool + r.off_b + sb.bytes(), r.stat_l_b, r.stat_ar_b};
    const bool b_status = (r.flags_b & GPUDIFF_OBJ_HAS_STATUS) != 0;
    const bool sd = !seg_equal(sa, sb);
    const bool td = !b_status || !seg_equal(ta, tb);
    if (sd) join(sa, sb, 0, emit);
    if (td) {
        join(ta, tb, GPUDIFF_PATH_REGION_STATUS, emit);
        if (!b_status)
            emit(status_sentinel((r.flags_a >> GPUDIFF_OBJ_SEED_SHIFT) & 0xFFu),
                 (uint8_t)(GPUDIFF_PATH_STATUS_ABSENT | GPUDIFF_PATH_REGION_STATUS));
    }
    return (uint8_t)((sd ? 1 : 0) | (td ? 2 : 0));
}

}  // namespace

extern "C" {

// Timed: decisions + changed paths of every pair (paths counted, not kept),
// threads repeating their slices until min_seconds; returns sweeps
// (fractional), *seconds = wall time, *n_paths = paths per sweep.
double oracle_csr_run(const uint8_t* pool, const gpudiff_pair_row* rows, size_t n, int threads, double min_seconds,
                      uint8_t* flags, double* seconds, uint64_t* n_paths) {
    if (threads < 1) threads = 1;
    std::vector<uint64_t> per(threads, 0), sink(threads, 0);
    const double sw = oracle::timed_sweeps(n, threads, min_seconds, seconds, [&](int t, size_t b, size_t e) {
        uint64_t cnt = 0, x = 0;
        auto emit = [&](uint64_t h, uint8_t k) {
            cnt++;
            x ^= h + k;
        };
        for (size_t i = b; i < e; i++) flags[i] = diff_pair(pool, rows[i], emit);
        per[t] = cnt;
        sink[t] ^= x;  // keeps the emitted paths live
    });
    uint64_t tot = 0, xs = 0;
    for (int t = 0; t < threads; t++) {
        tot += per[t];
        xs ^= sink[t];
    }
    static volatile uint64_t g_sink;
    g_sink = xs;
    if (n_paths) *n_paths = tot;
    return sw;
}

// Checker: the changed-path CSR of the dirty pairs (gpudiff_result layout:
// offsets[n_dirty + 1], hashes, kinds).  Returns the number of paths, or -1
// if cap is too small.
long oracle_csr_paths(const uint8_t* pool, const gpudiff_pair_row* rows, size_t n, uint8_t* flags, uint32_t* offsets,
                      uint64_t* hashes, uint8_t* kinds, size_t cap) {
    size_t total = 0, k = 0;
    bool over = false;
    offsets[0] = 0;
    for (size_t i = 0; i < n; i++) {
        auto emit = [&](uint64_t h, uint8_t kd) {
            if (total < cap) {
                hashes[total] = h;
                kinds[total] = kd;
            } else {
                over = true;
            }
            total++;
        };
        flags[i] = diff_pair(pool, rows[i], emit);
        if (flags[i] & 3) offsets[++k] = (uint32_t)total;
    }
    return over ? -1 : (long)total;
}

}  // extern "C"
