// K14: the API-negotiation update classifier over K13's per-document fields
// (pkg/reconciler/apiresource/controller.go:253-283).
// One lane per (old, new) pair: documents 2i (old) and 2i+1 (new) of the batch.
// The work per pair is a handful of short span compares on 2 x 1184-byte NegOut
// records; like K12 it is latency-bound and tiny next to K13.
#include <hip/hip_runtime.h>

#include "../../include/gpudiff.h"
#include "tokenize.h"

namespace gd {

namespace {

// unaligned 8-byte read (two aligned words); up to 15 bytes past p are read: a document's JSON is readable to
// kTokSlack = 32 bytes past its end, and every span lies inside its document
__device__ __forceinline__ uint64_t ld8(const uint8_t* p) {
    const uintptr_t a = (uintptr_t)p;
    const uint64_t* q = (const uint64_t*)(a & ~(uintptr_t)7);
    const uint32_t sh = (uint32_t)(a & 7u) * 8u;
    return (q[0] >> sh) | ((q[1] << 1) << (63u - sh));
}

// spans compared 8 bytes a step (a byte loop paid a dependent load per equal byte: condition messages, names)
__device__ __forceinline__ bool span_eq(const uint8_t* a, uint32_t al, const uint8_t* b, uint32_t bl) {
    if (al != bl) return false;
    for (uint32_t i = 0; i < al; i += 8) {
        const uint32_t r = al - i;
        const uint64_t m = r >= 8u ? ~0ull : (1ull << (8u * r)) - 1ull;
        if ((ld8(a + i) ^ ld8(b + i)) & m) return false;
    }
    return true;
}

// Semantic.DeepEqual of two map[string]string (nil == empty; K13 left no repeated keys)
__device__ bool map_eq(const NegMember* a, uint32_t na, const uint8_t* da, const NegMember* b, uint32_t nb,
                       const uint8_t* db) {
    if (na != nb) return false;
    for (uint32_t i = 0; i < na; i++) {
        const NegMember x = a[i];
        bool found = false;
        for (uint32_t j = 0; j < nb && !found; j++) {
            const NegMember y = b[j];
            if (span_eq(da + x.koff, x.klen, db + y.koff, y.klen)) {
                if (!span_eq(da + x.voff, x.vlen, db + y.voff, y.vlen)) return false;
                found = true;
            }
        }
        if (!found) return false;
    }
    return true;
}

// Semantic.DeepEqual of the two statuses: conditions element-wise (nil == empty),
// strings by bytes, metav1.Time by instant (a.UTC() == b.UTC())
__device__ bool status_eq(const NegOut& A, const uint8_t* da, const NegOut& B, const uint8_t* db) {
    if (A.n_cond != B.n_cond) return false;
    for (uint32_t c = 0; c < A.n_cond; c++) {
        const NegCond& x = A.cond[c];
        const NegCond& y = B.cond[c];
        if (x.sec != y.sec || x.nsec != y.nsec) return false;
        for (uint32_t f = 0; f < 4; f++)
            if (!span_eq(da + x.off[f], x.len[f], db + y.off[f], y.len[f])) return false;
    }
    return true;
}

// []string element-wise (nil == empty)
__device__ bool list_eq(const NegSpan* a, uint32_t na, const uint8_t* da, const NegSpan* b, uint32_t nb,
                        const uint8_t* db) {
    if (na != nb) return false;
    for (uint32_t i = 0; i < na; i++)
        if (!span_eq(da + a[i].off, a[i].len, db + b[i].off, b[i].len)) return false;
    return true;
}

// the rest of CustomResourceDefinitionStatus: acceptedNames (a struct: its four
// strings and two lists), storedVersions
__device__ bool crd_status_eq(const NegOut& A, const uint8_t* da, const NegOut& B, const uint8_t* db) {
    for (uint32_t f = 0; f < 4; f++)
        if (!span_eq(da + A.names[f].off, A.names[f].len, db + B.names[f].off, B.names[f].len)) return false;
    return list_eq(A.shortn, A.n_short, da, B.shortn, B.n_short, db) && list_eq(A.cat, A.n_cat, da, B.cat, B.n_cat, db) &&
           list_eq(A.stored, A.n_stored, da, B.stored, B.n_stored, db);
}

__global__ __launch_bounds__(256) void k_negotiate_pairs(const NegOut* __restrict__ outs, const uint8_t* __restrict__ absent,
                                                         const TokDoc* __restrict__ docs, const uint8_t* __restrict__ json,
                                                         uint32_t n, int32_t* __restrict__ actions) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const NegOut& B = outs[2u * i + 1u];
    int32_t act;
    if (B.status != GPUDIFF_TOK_OK) {
        act = kNegDefer;
    } else if (absent[i]) {
        act = GPUDIFF_NEG_CREATED;  // controller.go:258-261
    } else {
        const NegOut& A = outs[2u * i];
        const uint8_t* da = json + docs[2u * i].json_off;
        const uint8_t* db = json + docs[2u * i + 1u].json_off;
        if (A.status != GPUDIFF_TOK_OK) act = kNegDefer;
        else if (span_eq(da + A.rv_off, A.rv_len, db + B.rv_off, B.rv_len)) act = GPUDIFF_NEG_IGNORE;  // :263-265
        else if (A.gen != B.gen) act = GPUDIFF_NEG_SPEC;                                                 // :267-270
        else if (!status_eq(A, da, B, db) ||
                 (docs[2u * i + 1u].pad[0] == GPUDIFF_NEG_KIND_CRD && !crd_status_eq(A, da, B, db)))
            act = GPUDIFF_NEG_STATUS;  // :272-275
        else if (!map_eq(A.ann, A.n_ann, da, B.ann, B.n_ann, db) || map_eq(A.lab, A.n_lab, da, B.lab, B.n_lab, db))
            act = GPUDIFF_NEG_META;  // :277-281, the missing `!` before the labels term kept
        else
            act = GPUDIFF_NEG_IGNORE;  // :282-283
    }
    actions[i] = act;
}

}  // namespace

hipError_t launch_negotiate_pairs(hipStream_t s, const NegOut* outs, const uint8_t* absent, const TokDoc* docs,
                                  const uint8_t* json, uint32_t n_pairs, int32_t* actions) {
    if (!n_pairs) return hipSuccess;
    k_negotiate_pairs<<<(n_pairs + 255u) / 256u, 256, 0, s>>>(outs, absent, docs, json, n_pairs, actions);
    return hipGetLastError();
}

}  // namespace gd
