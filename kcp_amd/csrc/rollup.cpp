// Deployment splitter status roll-up: host side.
//
// The reference (pkg/reconciler/deployment/deployment.go:41-91) reconciles one
// leaf at a time: List(owned-by=<root>), sum five int32 counters, copy
// others[0]'s conditions, UpdateStatus.  The batch form here answers that for
// a whole population: K11 (roll-up mode of k_encode_docs) extracts every
// document's counters and owned-by label in HBM, K12 (rollup.hip) groups by
// label and sums on the device.  Documents outside K11's exact subset are
// decided by the host path below, and the batch is then regrouped on the host
// with the same rules, so results never depend on who decided a document.
//
// The host path is the Go-exact restatement of the typed decode the splitter's
// informer does (appsv1.Deployment via Go 1.16 encoding/json), restricted to
// the fields the roll-up reads: a streaming scanner over the JSON (Go's
// scanner rules: grammar, escapes, control characters, nesting depth 10000)
// that applies struct field lookup (exact, else case-insensitive with Go's
// fold rules), merges repeated keys into the same field as Go does, treats
// null as a no-op (a nil map for labels), and accepts a counter only as a
// number literal strconv.ParseInt takes that fits int32.
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "engine.h"
#include "goscan.h"
#include "rollup.h"
#include "tokenize.h"

using namespace gd;

struct gpudiff_rbatch {
    uint32_t n = 0;
    std::vector<TokDoc> docs;
    std::vector<const uint8_t*> src;
    std::vector<size_t> lens;
    uint64_t json_bytes = 0, scratch_bytes = 0;
    void *d_json = nullptr, *d_scratch = nullptr, *d_docs = nullptr, *d_ro = nullptr, *d_grp = nullptr;
    RollGroupBufs B{};
    hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
    bool pending_timing = false;
    double k11_ms_sum = 0, k12_ms_sum = 0;
    uint64_t runs = 0;
};

namespace {

// ------------------------------------------------------------------ host path
struct Fields {
    int32_t v[5] = {0, 0, 0, 0, 0};
    bool labels_nil = true;
    bool has_owned = false;
    std::string owned;
};

const char* const kFieldNames[5] = {"replicas", "updatedReplicas", "readyReplicas", "availableReplicas",
                                    "unavailableReplicas"};

using namespace goscan;

class RollScanner : public goscan::Scanner {
   public:
    using goscan::Scanner::Scanner;

    bool run(Fields& f) {
        ws();
        if (p_ >= e_ || *p_ != '{') return false;
        bool ok = members(1, [&](const std::string& k) -> bool {
            if (field_match("metadata", k)) return metadata(f);
            if (field_match("status", k)) return status(f);
            return skip(1);
        });
        if (!ok) return false;
        ws();
        return p_ == e_;
    }

   private:
    // metadata: ObjectMeta, only labels read
    bool metadata(Fields& f) {
        if (peek_null()) return lit("null");  // null into a struct: no-op
        if (p_ >= e_ || *p_ != '{') return false;  // a type error: Go rejects the object
        return members(2, [&](const std::string& k) -> bool {
            if (!field_match("labels", k)) return skip(2);
            if (peek_null()) {  // null into a map: nil
                f.labels_nil = true;
                f.has_owned = false;
                f.owned.clear();
                return lit("null");
            }
            if (p_ >= e_ || *p_ != '{') return false;
            f.labels_nil = false;  // decoding into the existing map: entries merge
            return members(3, [&](const std::string& lk) -> bool {
                // map[string]string: a string, or null (the element keeps its zero value "")
                const bool own = lk == "kcp.dev/owned-by";
                if (peek_null()) {
                    if (own) {
                        f.has_owned = true;
                        f.owned.clear();
                    }
                    return lit("null");
                }
                if (p_ >= e_ || *p_ != '"') return false;  // a type error
                if (own) f.has_owned = true;
                return str(own ? &f.owned : nullptr);
            });
        });
    }
    // status: DeploymentStatus, the five counters read
    bool status(Fields& f) {
        if (peek_null()) return lit("null");
        if (p_ >= e_ || *p_ != '{') return false;
        return members(2, [&](const std::string& k) -> bool {
            int fi = -1;
            for (int i = 0; i < 5 && fi < 0; i++)
                if (field_match(kFieldNames[i], k)) fi = i;
            if (fi < 0) return skip(2);
            if (peek_null()) return lit("null");  // null into an int32: no-op
            const uint8_t c = p_ < e_ ? *p_ : 0;
            if (c != '-' && (c < '0' || c > '9')) return false;  // not a number: UnmarshalTypeError
            const uint8_t* s;
            bool is_int;
            if (!number(&s, &is_int) || !is_int) return false;
            // strconv.ParseInt(s, 10, 64), then the int32 overflow check
            const bool neg = *s == '-';
            int64_t v = 0;
            for (const uint8_t* q = s + (neg ? 1 : 0); q < p_; q++) {
                v = v * 10 + (*q - '0');
                if (v > (int64_t)1 << 31) return false;
            }
            if (neg) v = -v;
            if (v < INT32_MIN || v > INT32_MAX) return false;
            f.v[fi] = (int32_t)v;
            return true;
        });
    }
};

// the fields of one document; false = Go cannot decode it
bool host_fields(const uint8_t* doc, size_t len, Fields& f) {
    RollScanner sc(doc, len);
    return sc.run(f);
}

struct RollupStore {
    std::vector<int32_t> doc_group, k11;
    std::vector<gpudiff_rollup_group> groups;
};

void publish(RollupStore* rs, gpudiff_rollup* out, size_t n, size_t n_host, uint32_t host_grouped) {
    out->n_docs = n;
    out->doc_group = rs->doc_group.data();
    out->n_groups = rs->groups.size();
    out->groups = rs->groups.data();
    out->k11_status = rs->k11.data();
    out->n_host = n_host;
    out->host_grouped = host_grouped;
    out->internal = rs;
}

inline int32_t wrap_add(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }

void free_rbatch(gpudiff_rbatch* rb) {
    if (!rb) return;
    void* ptrs[] = {rb->d_json, rb->d_scratch, rb->d_docs, rb->d_ro, rb->d_grp};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    for (hipEvent_t& e : rb->ev)
        if (e) (void)hipEventDestroy(e);
    delete rb;
}

void fold_timing(gpudiff_rbatch* rb) {
    float a = 0, b = 0;
    if (hipEventElapsedTime(&a, rb->ev[0], rb->ev[1]) == hipSuccess &&
        hipEventElapsedTime(&b, rb->ev[1], rb->ev[2]) == hipSuccess) {
        rb->k11_ms_sum += a;
        rb->k12_ms_sum += b;
        rb->runs++;
    }
    rb->pending_timing = false;
}

}  // namespace

extern "C" {

int gpudiff_rollup_doc_host(const uint8_t* doc, size_t len, int32_t* v, uint8_t* label, size_t cap,
                            size_t* label_len) {
    if ((!doc && len) || !v || !label_len) return GPUDIFF_E_INVAL;
    Fields f;
    if (!host_fields(doc ? doc : (const uint8_t*)"", len, f)) {
        *label_len = SIZE_MAX;
        return GPUDIFF_E_DECODE;
    }
    memcpy(v, f.v, sizeof(f.v));
    if (!f.has_owned) {
        *label_len = SIZE_MAX;
        return GPUDIFF_OK;
    }
    *label_len = f.owned.size();
    if (f.owned.size() > cap || (!label && f.owned.size())) return GPUDIFF_E_CAPACITY;
    if (f.owned.size()) memcpy(label, f.owned.data(), f.owned.size());
    return GPUDIFF_OK;
}

int gpudiff_rbatch_create(gpudiff_ctx* c, const uint8_t* const* docs, const size_t* lens, size_t n,
                          gpudiff_rbatch** out) {
    if (!c || !out || (n && (!docs || !lens)) || n > 0x7FFFFFFFu) return GPUDIFF_E_INVAL;
    *out = nullptr;
    int rc = set_device(c);
    if (rc) return rc;
    gpudiff_rbatch* rb = new (std::nothrow) gpudiff_rbatch();
    if (!rb) return GPUDIFF_E_NOMEM;
    rb->n = (uint32_t)n;
    rb->docs.resize(n);
    rb->src.assign(docs, docs + n);
    rb->lens.assign(lens, lens + n);
    uint64_t jb = 0, sb = 0;
    for (size_t i = 0; i < n; i++) {
        // documents beyond the size limit still get a TokDoc: K11 reports GPUDIFF_TOK_SIZE
        const uint32_t l = lens[i] > kTokMaxLen ? kTokMaxLen + 1 : (uint32_t)lens[i];
        TokDoc& t = rb->docs[i];
        memset(&t, 0, sizeof(t));
        t.json_off = jb;
        t.json_len = l;
        t.scratch_off = sb;
        if (l <= kTokMaxLen) {
            jb = (jb + l + kTokSlack + 15) & ~15ull;
            sb += rollup_scratch_bytes(l);
        }
    }
    jb += kTokSlack;
    rb->json_bytes = jb;
    rb->scratch_bytes = sb;
    const RollGroupBufs L = rollup_group_layout(nullptr, rb->n);
    auto fail = [&](hipError_t e) {
        free_rbatch(rb);
        return e == hipErrorOutOfMemory ? GPUDIFF_E_CAPACITY : GPUDIFF_E_DEVICE;
    };
    hipError_t e;
    if ((e = hipMalloc(&rb->d_json, jb)) != hipSuccess) return fail(e);
    if ((e = hipMalloc(&rb->d_scratch, std::max<uint64_t>(sb, 256))) != hipSuccess) return fail(e);
    if ((e = hipMalloc(&rb->d_docs, std::max<size_t>(n, 1) * sizeof(TokDoc))) != hipSuccess) return fail(e);
    if ((e = hipMalloc(&rb->d_ro, std::max<size_t>(n, 1) * sizeof(RollOut))) != hipSuccess) return fail(e);
    if ((e = hipMalloc(&rb->d_grp, L.total)) != hipSuccess) return fail(e);
    rb->B = rollup_group_layout((uint8_t*)rb->d_grp, rb->n);
    void* stage = nullptr;
    if ((e = hipHostMalloc(&stage, jb, hipHostMallocDefault)) != hipSuccess) return fail(e);
    memset(stage, 0, jb);
    for (size_t i = 0; i < n; i++)
        if (rb->docs[i].json_len <= kTokMaxLen && lens[i]) memcpy((uint8_t*)stage + rb->docs[i].json_off, docs[i], lens[i]);
    e = hipMemcpyAsync(rb->d_json, stage, jb, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess && n)
        e = hipMemcpyAsync(rb->d_docs, rb->docs.data(), n * sizeof(TokDoc), hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    (void)hipHostFree(stage);
    if (e != hipSuccess) return fail(e);
    if (c->flags & GPUDIFF_OPT_TIMING)
        for (hipEvent_t& ev : rb->ev)
            if ((e = hipEventCreate(&ev)) != hipSuccess) return fail(e);
    *out = rb;
    return GPUDIFF_OK;
}

int gpudiff_rbatch_run(gpudiff_ctx* c, gpudiff_rbatch* rb) {
    if (!c || !rb) return GPUDIFF_E_INVAL;
    int rc = set_device(c);
    if (rc) return rc;
    if (rb->pending_timing) {
        HIPCHK(hipEventSynchronize(rb->ev[2]));
        fold_timing(rb);
    }
    if (rb->ev[0]) HIPCHK(hipEventRecord(rb->ev[0], c->stream));
    HIPCHK(launch_rollup_docs(c->stream, (const TokDoc*)rb->d_docs, rb->n, (const uint8_t*)rb->d_json,
                              (uint8_t*)rb->d_scratch, (RollOut*)rb->d_ro));
    if (rb->ev[1]) HIPCHK(hipEventRecord(rb->ev[1], c->stream));
    HIPCHK(launch_rollup_group(c->stream, (const RollOut*)rb->d_ro, (const TokDoc*)rb->d_docs,
                               (const uint8_t*)rb->d_json, rb->n, rb->B));
    if (rb->ev[2]) {
        HIPCHK(hipEventRecord(rb->ev[2], c->stream));
        rb->pending_timing = true;
    }
    return GPUDIFF_OK;
}

int gpudiff_rbatch_fetch(gpudiff_ctx* c, gpudiff_rbatch* rb, gpudiff_rollup* out) {
    if (!c || !rb || !out) return GPUDIFF_E_INVAL;
    memset(out, 0, sizeof(*out));
    int rc = set_device(c);
    if (rc) return rc;
    const size_t n = rb->n;
    std::vector<RollOut> ro(n);
    uint32_t counts[2] = {0, 0};
    RollupStore* rs = new (std::nothrow) RollupStore();
    if (!rs) return GPUDIFF_E_NOMEM;
    rs->doc_group.resize(n);
    auto bail = [&](hipError_t) {
        delete rs;
        return GPUDIFF_E_DEVICE;
    };
    hipError_t e = hipSuccess;
    if (n) e = hipMemcpyAsync(ro.data(), rb->d_ro, n * sizeof(RollOut), hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess && n)
        e = hipMemcpyAsync(rs->doc_group.data(), rb->B.doc_group, n * 4, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(counts, rb->B.counts, 8, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return bail(e);
    if (rb->pending_timing) fold_timing(rb);
    rs->k11.resize(n);
    std::vector<uint32_t> def;
    for (size_t i = 0; i < n; i++) {
        rs->k11[i] = ro[i].status;
        if (ro[i].status != GPUDIFF_TOK_OK) def.push_back((uint32_t)i);
    }
    const bool regroup = !def.empty() || counts[1] != 0;
    if (!regroup) {
        rs->groups.resize(counts[0]);
        if (counts[0])
            e = hipMemcpy(rs->groups.data(), rb->B.groups, counts[0] * sizeof(gpudiff_rollup_group),
                          hipMemcpyDeviceToHost);
        if (e != hipSuccess) return bail(e);
        publish(rs, out, n, 0, 0);
        return GPUDIFF_OK;
    }
    // the host path for the deferred documents, on the context's encode threads
    std::vector<Fields> hf(def.size());
    std::vector<uint8_t> hok(def.size(), 0);
    const uint32_t T = std::max<uint32_t>(1, std::min<uint32_t>(c->threads, (uint32_t)((def.size() + 63) / 64)));
    auto work = [&](uint32_t t) {
        for (size_t k = t; k < def.size(); k += T) hok[k] = host_fields(rb->src[def[k]], rb->lens[def[k]], hf[k]);
    };
    workers(c).run(T, work);
    // exact regrouping in document order (first appearance = ascending first_doc)
    std::unordered_map<std::string, int32_t> index;
    index.reserve(counts[0] + def.size());
    size_t k = 0;
    for (size_t i = 0; i < n; i++) {
        const int32_t* v;
        std::string label;
        bool has = false;
        if (ro[i].status == GPUDIFF_TOK_OK) {
            v = ro[i].v;
            has = ro[i].flags & kRollHasLabel;
            if (has) label.assign((const char*)rb->src[i] + ro[i].label_off, ro[i].label_len);
        } else {
            const size_t kk = k++;
            if (!hok[kk]) {
                rs->doc_group[i] = GPUDIFF_ROLLUP_DECODE;
                continue;
            }
            v = hf[kk].v;
            has = hf[kk].has_owned;
            if (has) label = std::move(hf[kk].owned);
        }
        if (!has) {
            rs->doc_group[i] = GPUDIFF_ROLLUP_NONE;
            continue;
        }
        auto it = index.emplace(std::move(label), (int32_t)rs->groups.size());
        if (it.second) {
            gpudiff_rollup_group g{};
            g.first_doc = (uint32_t)i;
            rs->groups.push_back(g);
        }
        gpudiff_rollup_group& g = rs->groups[it.first->second];
        g.n_members++;
        for (int f = 0; f < 5; f++) g.sums[f] = wrap_add(g.sums[f], v[f]);
        rs->doc_group[i] = it.first->second;
    }
    publish(rs, out, n, def.size(), 1);
    return GPUDIFF_OK;
}

int gpudiff_rbatch_stats_get(const gpudiff_rbatch* rb, gpudiff_rbatch_stats* st) {
    if (!rb || !st) return GPUDIFF_E_INVAL;
    memset(st, 0, sizeof(*st));
    st->n_docs = rb->n;
    for (size_t l : rb->lens) st->json_bytes += l;
    st->scratch_bytes = rb->scratch_bytes + rb->B.total;
    st->runs = rb->runs;
    st->k11_ms = rb->runs ? rb->k11_ms_sum / (double)rb->runs : 0.0;
    st->k12_ms = rb->runs ? rb->k12_ms_sum / (double)rb->runs : 0.0;
    return GPUDIFF_OK;
}

void gpudiff_rbatch_free(gpudiff_ctx* c, gpudiff_rbatch* rb) {
    if (!rb) return;
    if (c && c->has_device) {
        (void)hipSetDevice(c->device);
        (void)hipStreamSynchronize(c->stream);
    }
    free_rbatch(rb);
}

int gpudiff_rollup_status(gpudiff_ctx* c, const uint8_t* const* docs, const size_t* lens, size_t n,
                          gpudiff_rollup* out) {
    if (!out) return GPUDIFF_E_INVAL;
    memset(out, 0, sizeof(*out));
    gpudiff_rbatch* rb = nullptr;
    int rc = gpudiff_rbatch_create(c, docs, lens, n, &rb);
    if (rc) return rc;
    rc = gpudiff_rbatch_run(c, rb);
    if (!rc) rc = gpudiff_rbatch_fetch(c, rb, out);
    gpudiff_rbatch_free(c, rb);
    return rc;
}

void gpudiff_rollup_release(gpudiff_ctx*, gpudiff_rollup* r) {
    if (!r) return;
    delete (RollupStore*)r->internal;
    memset(r, 0, sizeof(*r));
}

}  // extern "C"
