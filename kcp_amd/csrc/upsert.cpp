// Write path: the request body the syncer sends for a
// dirty object, on the device (kernel K10, marshal mode of k_encode_docs) with
// the host completing the documents K10 leaves (floats, duplicate keys, Go
// decode errors, ...).
//
// The host path here is the Go-exact restatement:
//   * decode with the informer's rules (json.cpp: k8s util/json over Go
//     1.16 encoding/json, duplicate keys last-wins, U+FFFD repair);
//   * transform as upsertIntoDownstream (pkg/syncer/specsyncer.go:94-108:
//     SetUID(""), SetResourceVersion(""), owner references named by the
//     kcp.dev/owned-by label dropped, SetOwnerReferences) or
//     updateStatusInUpstream (pkg/syncer/statussyncer.go:44-48: SetUID(""),
//     SetResourceVersion(""));
//   * marshal as the dynamic client's body, json.NewEncoder(w).Encode(obj):
//     map keys sorted by bytes, encodeState.string with escapeHTML, floats via
//     strconv.AppendFloat(f, 'f' | 'e', -1, 64) with the 1e-6 / 1e21 switch and
//     the e-09 -> e-9 clean-up, trailing '\n'.
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <charconv>
#include <string>
#include <thread>
#include <vector>

#include "dstore.h"
#include "engine.h"
#include "json.h"
#include "tokenize.h"

using namespace gd;

namespace {

const char kHex[] = "0123456789abcdef";

void put_str(std::string& o, const char* s, size_t n) {
    o.push_back('"');
    for (size_t i = 0; i < n; i++) {
        const uint8_t c = (uint8_t)s[i];
        if (c < 0x80) {
            if (c == '"' || c == '\\') {
                o.push_back('\\');
                o.push_back((char)c);
            } else if (c == '\n') {
                o += "\\n";
            } else if (c == '\r') {
                o += "\\r";
            } else if (c == '\t') {
                o += "\\t";
            } else if (c < 0x20 || c == '<' || c == '>' || c == '&') {
                o += "\\u00";
                o.push_back(kHex[c >> 4]);
                o.push_back(kHex[c & 15]);
            } else {
                o.push_back((char)c);
            }
        } else if (c == 0xE2 && i + 2 < n && (uint8_t)s[i + 1] == 0x80 &&
                   ((uint8_t)s[i + 2] == 0xA8 || (uint8_t)s[i + 2] == 0xA9)) {
            o += "\\u202";
            o.push_back((uint8_t)s[i + 2] == 0xA8 ? '8' : '9');
            i += 2;
        } else {
            o.push_back((char)c);  // decoded strings are valid UTF-8 (json.cpp repairs)
        }
    }
    o.push_back('"');
}

// floatEncoder(64): strconv.AppendFloat(f, 'f' | 'e', -1, 64).  Go formats the
// shortest round-trip digit string (closest on ties) in the chosen layout, so
// 'f' pads with zeros (2^63 -> "9223372036854776000"); std::to_chars' fixed
// form would print the exact integer instead, so the digits come from its
// scientific form and are laid out here.
void put_float(std::string& o, double f) {
    char b[64];
    auto r = std::to_chars(b, b + sizeof(b) - 1, f, std::chars_format::scientific);
    size_t n = (size_t)(r.ptr - b);
    b[n] = 0;
    const double a = f < 0 ? -f : f;
    if (a != 0 && (a < 1e-6 || a >= 1e21)) {
        if (n >= 4 && b[n - 4] == 'e' && b[n - 3] == '-' && b[n - 2] == '0') {  // e-07 -> e-7
            b[n - 2] = b[n - 1];
            n--;
        }
        o.append(b, n);
        return;
    }
    size_t i = 0;
    if (b[0] == '-') {
        o.push_back('-');
        i = 1;
    }
    std::string dig;
    for (; i < n && b[i] != 'e'; i++)
        if (b[i] != '.') dig.push_back(b[i]);
    const int x = atoi(b + i + 1);  // decimal exponent of the first digit
    const int nd = (int)dig.size();
    if (x >= nd - 1) {
        o += dig;
        o.append((size_t)(x - (nd - 1)), '0');
    } else if (x >= 0) {
        o.append(dig, 0, (size_t)x + 1);
        o.push_back('.');
        o.append(dig, (size_t)x + 1, std::string::npos);
    } else {
        o += "0.";
        o.append((size_t)(-x - 1), '0');
        o += dig;
    }
}

const Member* find(const Node& obj, const char* k) {
    const size_t kl = strlen(k);
    for (uint32_t i = 0; i < obj.n; i++)
        if (obj.u.mem[i].klen == kl && memcmp(obj.u.mem[i].k, k, kl) == 0) return &obj.u.mem[i];
    return nullptr;
}

std::vector<const Member*> sorted_members(const Node& obj) {
    std::vector<const Member*> m(obj.n);
    for (uint32_t i = 0; i < obj.n; i++) m[i] = &obj.u.mem[i];
    std::sort(m.begin(), m.end(), [](const Member* a, const Member* b) {
        const int c = memcmp(a->k, b->k, std::min(a->klen, b->klen));
        return c != 0 ? c < 0 : a->klen < b->klen;
    });
    return m;
}

void put_value(std::string& o, const Node& v);

void put_object(std::string& o, const Node& v) {
    o.push_back('{');
    bool first = true;
    for (const Member* m : sorted_members(v)) {
        if (!first) o.push_back(',');
        first = false;
        put_str(o, m->k, m->klen);
        o.push_back(':');
        put_value(o, m->v);
    }
    o.push_back('}');
}

void put_value(std::string& o, const Node& v) {
    switch (v.t) {
        case J_NULL: o += "null"; break;
        case J_FALSE: o += "false"; break;
        case J_TRUE: o += "true"; break;
        case J_INT: {
            char b[24];
            auto r = std::to_chars(b, b + sizeof(b), (long long)v.u.i);
            o.append(b, (size_t)(r.ptr - b));
            break;
        }
        case J_FLOAT: put_float(o, v.u.d); break;
        case J_STR: put_str(o, v.u.s, v.n); break;
        case J_ARR:
            o.push_back('[');
            for (uint32_t i = 0; i < v.n; i++) {
                if (i) o.push_back(',');
                put_value(o, v.u.items[i]);
            }
            o.push_back(']');
            break;
        default: put_object(o, v); break;
    }
}

// Unstructured.GetOwnerReferences -> filter -> SetOwnerReferences, written as
// ToUnstructured(&OwnerReference) maps (apiVersion, blockOwnerDeletion?,
// controller?, kind, name, uid).  Returns false when the field is removed
// (no reference kept: the Go slice stays nil, specsyncer.go:101-108).
bool put_owner_refs(std::string& o, const Node& refs, const char* owned, size_t owned_len) {
    if (refs.t != J_ARR || refs.n == 0) return false;
    for (uint32_t i = 0; i < refs.n; i++)
        if (refs.u.items[i].t != J_OBJ) return false;  // GetOwnerReferences: nil
    size_t kept = 0;
    std::string tmp;
    for (uint32_t i = 0; i < refs.n; i++) {
        const Node& e = refs.u.items[i];
        auto sval = [&](const char* k, const char** p, size_t* n) {
            const Member* m = find(e, k);
            if (m && m->v.t == J_STR) {
                *p = m->v.u.s;
                *n = m->v.n;
            } else {
                *p = "";
                *n = 0;
            }
        };
        const char* np;
        size_t nl;
        sval("name", &np, &nl);
        if (nl == owned_len && memcmp(np, owned, nl) == 0) continue;  // reference.Name == ownedByLabel
        if (kept++) tmp.push_back(',');
        const char* p;
        size_t n;
        tmp += "{\"apiVersion\":";
        sval("apiVersion", &p, &n);
        put_str(tmp, p, n);
        const Member* b = find(e, "blockOwnerDeletion");
        if (b && (b->v.t == J_TRUE || b->v.t == J_FALSE)) tmp += b->v.t == J_TRUE ? ",\"blockOwnerDeletion\":true" : ",\"blockOwnerDeletion\":false";
        const Member* c = find(e, "controller");
        if (c && (c->v.t == J_TRUE || c->v.t == J_FALSE)) tmp += c->v.t == J_TRUE ? ",\"controller\":true" : ",\"controller\":false";
        tmp += ",\"kind\":";
        sval("kind", &p, &n);
        put_str(tmp, p, n);
        tmp += ",\"name\":";
        put_str(tmp, np, nl);
        tmp += ",\"uid\":";
        sval("uid", &p, &n);
        put_str(tmp, p, n);
        tmp.push_back('}');
    }
    if (!kept) return false;
    o.push_back('[');
    o += tmp;
    o.push_back(']');
    return true;
}

}  // namespace

namespace gd {

// The body for one decoded object (root: a J_OBJ).
void upsert_body(const Node& root, uint32_t mode, std::string& o) {
    o.clear();
    const Member* md = find(root, "metadata");
    if (!md || md->v.t != J_OBJ) {
        put_object(o, root);  // RemoveNestedField / SetNestedField: no-ops without a metadata map
        o.push_back('\n');
        return;
    }
    // owned-by: GetLabels() is NestedStringMap (nil unless every value is a string)
    const char* owned = "";
    size_t owned_len = 0;
    if (mode == GPUDIFF_UPSERT_SPEC) {
        const Member* lb = find(md->v, "labels");
        if (lb && lb->v.t == J_OBJ) {
            bool all_str = true;
            for (uint32_t i = 0; i < lb->v.n; i++)
                if (lb->v.u.mem[i].v.t != J_STR) all_str = false;
            const Member* ob = all_str ? find(lb->v, "kcp.dev/owned-by") : nullptr;
            if (ob) {
                owned = ob->v.u.s;
                owned_len = ob->v.n;
            }
        }
    }
    o.push_back('{');
    bool first = true;
    for (const Member* m : sorted_members(root)) {
        if (!first) o.push_back(',');
        first = false;
        put_str(o, m->k, m->klen);
        o.push_back(':');
        if (m != md) {
            put_value(o, m->v);
            continue;
        }
        o.push_back('{');
        bool f2 = true;
        for (const Member* x : sorted_members(md->v)) {
            auto is = [&](const char* k) { return x->klen == strlen(k) && memcmp(x->k, k, x->klen) == 0; };
            if (is("uid") || is("resourceVersion")) continue;
            std::string item;
            if (!f2) item.push_back(',');
            put_str(item, x->k, x->klen);
            item.push_back(':');
            if (mode == GPUDIFF_UPSERT_SPEC && is("ownerReferences")) {
                if (!put_owner_refs(item, x->v, owned, owned_len)) continue;
            } else {
                put_value(item, x->v);
            }
            o += item;
            f2 = false;
        }
        o.push_back('}');
    }
    o.push_back('}');
    o.push_back('\n');
}

}  // namespace gd

// ------------------------------------------------------------------ C-ABI
struct gpudiff_wbatch {
    uint32_t n = 0, mode = 0;
    std::vector<TokDoc> docs;
    std::vector<const uint8_t*> src;
    std::vector<size_t> lens;
    uint64_t json_bytes = 0, scratch_bytes = 0, out_bytes = 0;
    void *d_json = nullptr, *d_scratch = nullptr, *d_out = nullptr, *d_docs = nullptr, *d_res = nullptr;
    hipEvent_t ev[2] = {nullptr, nullptr};
    bool pending_timing = false;
    double k10_ms_sum = 0;
    uint64_t runs = 0, body_bytes = 0;
};

namespace {

struct BodiesStore {
    std::vector<uint64_t> offsets;
    std::vector<uint8_t> bytes;
    std::vector<int32_t> status, k10;
    std::vector<uint8_t> source;
};

void publish(BodiesStore* bs, gpudiff_bodies* out, size_t n, size_t n_host) {
    out->n = n;
    out->offsets = bs->offsets.data();
    out->bytes = bs->bytes.data();
    out->status = bs->status.data();
    out->source = bs->source.data();
    out->k10_status = bs->k10.data();
    out->n_host = n_host;
    out->internal = bs;
}

void free_wbatch(gpudiff_wbatch* wb) {
    for (void* p : {wb->d_json, wb->d_scratch, wb->d_out, wb->d_docs, wb->d_res})
        if (p) (void)hipFree(p);
    for (hipEvent_t e : wb->ev)
        if (e) (void)hipEventDestroy(e);
    delete wb;
}

// host marshal of one document into o; false = Go decode error
bool host_body(const uint8_t* doc, size_t len, uint32_t mode, std::string& o) {
    JsonParser jp;
    Arena arena;
    Node root;
    if (!jp.parse_object(doc, len, arena, &root)) return false;
    upsert_body(root, mode, o);
    return true;
}

}  // namespace

extern "C" {

int gpudiff_upsert_body_host(const uint8_t* doc, size_t len, uint32_t mode, uint8_t* out, size_t cap,
                             size_t* out_len) {
    if ((!doc && len) || !out_len || mode > GPUDIFF_UPSERT_STATUS) return GPUDIFF_E_INVAL;
    std::string o;
    if (!host_body(doc ? doc : (const uint8_t*)"", len, mode, o)) {
        *out_len = 0;
        return GPUDIFF_E_DECODE;
    }
    *out_len = o.size();
    if (o.size() > cap || (!out && o.size())) return GPUDIFF_E_CAPACITY;
    if (o.size()) memcpy(out, o.data(), o.size());
    return GPUDIFF_OK;
}

int gpudiff_wbatch_create(gpudiff_ctx* c, const uint8_t* const* docs, const size_t* lens, size_t n, uint32_t mode,
                          gpudiff_wbatch** out) {
    if (!c || !out || (n && (!docs || !lens)) || n > 0xFFFFFFFFu || mode > GPUDIFF_UPSERT_STATUS)
        return GPUDIFF_E_INVAL;
    *out = nullptr;
    int rc = set_device(c);
    if (rc) return rc;
    gpudiff_wbatch* wb = new (std::nothrow) gpudiff_wbatch();
    if (!wb) return GPUDIFF_E_NOMEM;
    wb->n = (uint32_t)n;
    wb->mode = mode;
    wb->docs.resize(n);
    wb->src.assign(docs, docs + n);
    wb->lens.assign(lens, lens + n);
    uint64_t jb = 0, sb = 0, ob = 0;
    for (size_t i = 0; i < n; i++) {
        // documents beyond K10's size limit still get a TokDoc: the kernel reports GPUDIFF_TOK_SIZE
        const uint32_t l = lens[i] > kTokMaxLen ? kTokMaxLen + 1 : (uint32_t)lens[i];
        TokDoc& t = wb->docs[i];
        memset(&t, 0, sizeof(t));
        t.json_off = jb;
        t.json_len = l;
        t.scratch_off = sb;
        t.pad[0] = (uint32_t)ob;
        t.pad[1] = (uint32_t)(ob >> 32);
        if (l <= kTokMaxLen) {
            jb = (jb + l + kTokSlack + 15) & ~15ull;
            sb += marshal_scratch_bytes(l);
            ob += marshal_out_cap(l);
        }
    }
    jb += kTokSlack;
    wb->json_bytes = jb;
    wb->scratch_bytes = sb;
    wb->out_bytes = ob;
    auto fail = [&](hipError_t e) {
        free_wbatch(wb);
        return e == hipErrorOutOfMemory ? GPUDIFF_E_CAPACITY : GPUDIFF_E_DEVICE;
    };
    hipError_t e;
    if ((e = hipMalloc(&wb->d_json, jb)) != hipSuccess) return fail(e);
    if ((e = hipMalloc(&wb->d_scratch, std::max<uint64_t>(sb, 256))) != hipSuccess) return fail(e);
    if ((e = hipMalloc(&wb->d_out, std::max<uint64_t>(ob, 256))) != hipSuccess) return fail(e);
    if ((e = hipMalloc(&wb->d_docs, std::max<size_t>(n, 1) * sizeof(TokDoc))) != hipSuccess) return fail(e);
    if ((e = hipMalloc(&wb->d_res, std::max<size_t>(n, 1) * sizeof(TokOut))) != hipSuccess) return fail(e);
    // JSON up through one pinned staging buffer
    void* stage = nullptr;
    if ((e = hipHostMalloc(&stage, jb, hipHostMallocDefault)) != hipSuccess) return fail(e);
    memset(stage, 0, jb);
    for (size_t i = 0; i < n; i++)
        if (wb->docs[i].json_len <= kTokMaxLen && lens[i]) memcpy((uint8_t*)stage + wb->docs[i].json_off, docs[i], lens[i]);
    e = hipMemcpyAsync(wb->d_json, stage, jb, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess && n)
        e = hipMemcpyAsync(wb->d_docs, wb->docs.data(), n * sizeof(TokDoc), hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    (void)hipHostFree(stage);
    if (e != hipSuccess) return fail(e);
    if (c->flags & GPUDIFF_OPT_TIMING) {
        if ((e = hipEventCreate(&wb->ev[0])) != hipSuccess) return fail(e);
        if ((e = hipEventCreate(&wb->ev[1])) != hipSuccess) return fail(e);
    }
    *out = wb;
    return GPUDIFF_OK;
}

int gpudiff_wbatch_run(gpudiff_ctx* c, gpudiff_wbatch* wb) {
    if (!c || !wb) return GPUDIFF_E_INVAL;
    int rc = set_device(c);
    if (rc) return rc;
    if (wb->pending_timing) {  // fold the previous run's duration in
        float ms = 0;
        HIPCHK(hipEventSynchronize(wb->ev[1]));
        HIPCHK(hipEventElapsedTime(&ms, wb->ev[0], wb->ev[1]));
        wb->k10_ms_sum += ms;
        wb->runs++;
        wb->pending_timing = false;
    }
    if (wb->ev[0]) HIPCHK(hipEventRecord(wb->ev[0], c->stream));
    HIPCHK(launch_marshal_docs(c->stream, (const TokDoc*)wb->d_docs, wb->n, (const uint8_t*)wb->d_json,
                               (uint8_t*)wb->d_scratch, (uint8_t*)wb->d_out, wb->mode, (TokOut*)wb->d_res));
    if (wb->ev[1]) {
        HIPCHK(hipEventRecord(wb->ev[1], c->stream));
        wb->pending_timing = true;
    }
    return GPUDIFF_OK;
}

int gpudiff_wbatch_fetch(gpudiff_ctx* c, gpudiff_wbatch* wb, gpudiff_bodies* out) {
    if (!c || !wb || !out) return GPUDIFF_E_INVAL;
    memset(out, 0, sizeof(*out));
    int rc = set_device(c);
    if (rc) return rc;
    const size_t n = wb->n;
    std::vector<TokOut> to(n);
    std::vector<uint8_t> raw(wb->out_bytes);
    if (n) HIPCHK(hipMemcpyAsync(to.data(), wb->d_res, n * sizeof(TokOut), hipMemcpyDeviceToHost, c->stream));
    if (wb->out_bytes) HIPCHK(hipMemcpyAsync(raw.data(), wb->d_out, wb->out_bytes, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (wb->pending_timing) {
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, wb->ev[0], wb->ev[1]));
        wb->k10_ms_sum += ms;
        wb->runs++;
        wb->pending_timing = false;
    }
    BodiesStore* bs = new (std::nothrow) BodiesStore();
    if (!bs) return GPUDIFF_E_NOMEM;
    bs->offsets.resize(n + 1);
    bs->status.assign(n, 0);
    bs->k10.resize(n);
    bs->source.assign(n, GPUDIFF_BODY_DEVICE);
    // documents K10 left: the host path, on the context's encode threads
    std::vector<uint32_t> def;
    for (size_t i = 0; i < n; i++)
        if (to[i].status != GPUDIFF_TOK_OK) def.push_back((uint32_t)i);
    std::vector<std::string> hb(def.size());
    std::vector<uint8_t> hok(def.size(), 0);
    const uint32_t T = std::max<uint32_t>(1, std::min<uint32_t>(c->threads, (uint32_t)((def.size() + 63) / 64)));
    auto work = [&](uint32_t t) {
        for (size_t k = t; k < def.size(); k += T)
            hok[k] = host_body(wb->src[def[k]], wb->lens[def[k]], wb->mode, hb[k]) ? 1 : 0;
    };
    workers(c).run(T, work);
    const size_t n_host = def.size();
    uint64_t dev_bytes = 0;
    size_t k = 0;
    for (size_t i = 0; i < n; i++) {
        bs->offsets[i] = bs->bytes.size();
        bs->k10[i] = (int32_t)to[i].status;
        if (to[i].status == GPUDIFF_TOK_OK) {
            const uint8_t* p = raw.data() + to[i].off;
            bs->bytes.insert(bs->bytes.end(), p, p + to[i].bytes);
            dev_bytes += to[i].bytes;
        } else {
            bs->source[i] = GPUDIFF_BODY_HOST;
            if (hok[k]) bs->bytes.insert(bs->bytes.end(), hb[k].begin(), hb[k].end());
            else bs->status[i] = GPUDIFF_E_DECODE;
            k++;
        }
    }
    bs->offsets[n] = bs->bytes.size();
    wb->body_bytes = dev_bytes;
    publish(bs, out, n, n_host);
    return GPUDIFF_OK;
}

int gpudiff_wbatch_stats_get(const gpudiff_wbatch* wb, gpudiff_wbatch_stats* st) {
    if (!wb || !st) return GPUDIFF_E_INVAL;
    memset(st, 0, sizeof(*st));
    st->n_docs = wb->n;
    for (size_t l : wb->lens) st->json_bytes += l;
    st->body_bytes = wb->body_bytes;
    st->scratch_bytes = wb->scratch_bytes;
    st->out_cap_bytes = wb->out_bytes;
    st->runs = wb->runs;
    st->k10_ms = wb->runs ? wb->k10_ms_sum / (double)wb->runs : 0.0;
    return GPUDIFF_OK;
}

void gpudiff_wbatch_free(gpudiff_ctx* c, gpudiff_wbatch* wb) {
    if (!wb) return;
    if (c && c->has_device) {
        (void)hipSetDevice(c->device);
        (void)hipStreamSynchronize(c->stream);
    }
    free_wbatch(wb);
}

int gpudiff_upsert_bodies(gpudiff_ctx* c, const uint8_t* const* docs, const size_t* lens, size_t n, uint32_t mode,
                          gpudiff_bodies* out) {
    if (!out) return GPUDIFF_E_INVAL;
    memset(out, 0, sizeof(*out));
    gpudiff_wbatch* wb = nullptr;
    int rc = gpudiff_wbatch_create(c, docs, lens, n, mode, &wb);
    if (rc) return rc;
    rc = gpudiff_wbatch_run(c, wb);
    if (!rc) rc = gpudiff_wbatch_fetch(c, wb, out);
    gpudiff_wbatch_free(c, wb);
    return rc;
}

void gpudiff_bodies_release(gpudiff_ctx*, gpudiff_bodies* b) {
    if (!b) return;
    delete (BodiesStore*)b->internal;
    memset(b, 0, sizeof(*b));
}

// ------------------------------------------------------------------ gate -> write on the device
struct PlanStore {
    std::vector<uint32_t> pair_index;
    std::vector<uint8_t> kind, noop;
};

int gpudiff_write_plan_get(gpudiff_ctx* c, gpudiff_ticket ticket, gpudiff_write_plan* out) {
    return gpudiff_write_plan_get_ex(c, ticket, GPUDIFF_PLAN_INFORMER, out);
}

int gpudiff_write_plan_get_ex(gpudiff_ctx* c, gpudiff_ticket ticket, uint32_t mode, gpudiff_write_plan* out) {
    if (!c || !out) return GPUDIFF_E_INVAL;
    if (mode & ~(GPUDIFF_PLAN_SPEC | GPUDIFF_PLAN_STATUS | GPUDIFF_PLAN_UPSTREAM_DOWNSTREAM)) return GPUDIFF_E_INVAL;
    const uint32_t kinds = (mode & (GPUDIFF_PLAN_SPEC | GPUDIFF_PLAN_STATUS)) ? mode : (GPUDIFF_PLAN_SPEC | GPUDIFF_PLAN_STATUS);
    // informer pairs (old, new): UpdateFunc enqueues newObj and the worker writes it (specsyncer.go:47-50 ->
    // :86-132, statussyncer.go:32-35 -> :41-63), so both kinds render document 2i+1; (A, B) pairs: the spec
    // write is A's (2i), the status write B's (2i+1)
    const uint32_t spec_side = (mode & GPUDIFF_PLAN_UPSTREAM_DOWNSTREAM) ? 0u : 1u;
    memset(out, 0, sizeof(*out));
    int rc = set_device(c);
    if (rc) return rc;
    StagedPairs sp;
    if ((rc = dstore_staged_pairs(c, ticket, &sp))) return rc;
    const std::vector<uint8_t>& fl = *sp.flags;
    std::unique_ptr<PlanStore> ps(new (std::nothrow) PlanStore());
    if (!ps) return GPUDIFF_E_NOMEM;
    // the writes: spec-dirty pairs, then status-dirty pairs
    for (uint32_t kind = GPUDIFF_UPSERT_SPEC; kind <= GPUDIFF_UPSERT_STATUS; kind++) {
        if (!(kinds & (kind == GPUDIFF_UPSERT_SPEC ? GPUDIFF_PLAN_SPEC : GPUDIFF_PLAN_STATUS))) continue;
        const uint8_t dirty = kind == GPUDIFF_UPSERT_SPEC ? GPUDIFF_SPEC_DIRTY : GPUDIFF_STATUS_DIRTY;
        const uint8_t noop = kind == GPUDIFF_UPSERT_SPEC ? GPUDIFF_SPEC_NOOP : GPUDIFF_STATUS_NOOP;
        for (uint32_t p = 0; p < sp.n; p++)
            if (fl[p] & dirty) {
                ps->pair_index.push_back(p);
                ps->kind.push_back((uint8_t)kind);
                ps->noop.push_back((fl[p] & noop) ? 1 : 0);
            }
    }
    const size_t nw = ps->pair_index.size();
    // K10 documents: the staged document of every write that is not a no-op, read where K0 read it (HBM)
    std::vector<TokDoc> docs;
    std::vector<uint32_t> wdoc(nw, UINT32_MAX);
    uint32_t n_spec_docs = 0;
    uint64_t sb = 0, ob = 0;
    for (size_t w = 0; w < nw; w++) {
        if (ps->noop[w]) continue;
        const uint32_t di = 2 * ps->pair_index[w] + (ps->kind[w] == GPUDIFF_UPSERT_SPEC ? spec_side : 1u);
        TokDoc t = sp.hdocs[di];
        t.seed = 0;
        t.scratch_off = sb;
        t.pad[0] = (uint32_t)ob;
        t.pad[1] = (uint32_t)(ob >> 32);
        sb += marshal_scratch_bytes(t.json_len);
        ob += marshal_out_cap(t.json_len);
        wdoc[w] = (uint32_t)docs.size();
        docs.push_back(t);
        if (ps->kind[w] == GPUDIFF_UPSERT_SPEC) n_spec_docs++;
    }
    const size_t nd = docs.size();
    void *d_docs = nullptr, *d_scratch = nullptr, *d_out = nullptr, *d_res = nullptr;
    auto cleanup = [&]() {
        for (void* p : {d_docs, d_scratch, d_out, d_res})
            if (p) (void)hipFree(p);
    };
    std::vector<TokOut> to(nd);
    std::vector<uint8_t> raw(ob);
    if (nd) {
        hipError_t e;
        if ((e = hipMalloc(&d_docs, nd * sizeof(TokDoc))) != hipSuccess ||
            (e = hipMalloc(&d_scratch, std::max<uint64_t>(sb, 256))) != hipSuccess ||
            (e = hipMalloc(&d_out, std::max<uint64_t>(ob, 256))) != hipSuccess ||
            (e = hipMalloc(&d_res, nd * sizeof(TokOut))) != hipSuccess) {
            cleanup();
            return e == hipErrorOutOfMemory ? GPUDIFF_E_CAPACITY : GPUDIFF_E_DEVICE;
        }
        hipError_t le = hipMemcpyAsync(d_docs, docs.data(), nd * sizeof(TokDoc), hipMemcpyHostToDevice, c->stream);
        if (le == hipSuccess && n_spec_docs)
            le = launch_marshal_docs(c->stream, (const TokDoc*)d_docs, n_spec_docs, sp.djson, (uint8_t*)d_scratch,
                                     (uint8_t*)d_out, GPUDIFF_UPSERT_SPEC, (TokOut*)d_res);
        if (le == hipSuccess && nd > n_spec_docs)
            le = launch_marshal_docs(c->stream, (const TokDoc*)d_docs + n_spec_docs, (uint32_t)(nd - n_spec_docs),
                                     sp.djson, (uint8_t*)d_scratch, (uint8_t*)d_out, GPUDIFF_UPSERT_STATUS,
                                     (TokOut*)d_res + n_spec_docs);
        if (le == hipSuccess && (rc = dstore_staged_mark_read(c, ticket))) le = hipErrorUnknown;
        if (le == hipSuccess) le = hipMemcpyAsync(to.data(), d_res, nd * sizeof(TokOut), hipMemcpyDeviceToHost, c->stream);
        if (le == hipSuccess) le = hipMemcpyAsync(raw.data(), d_out, ob, hipMemcpyDeviceToHost, c->stream);
        if (le == hipSuccess) le = hipStreamSynchronize(c->stream);
        cleanup();
        if (le != hipSuccess) {
            gd::g_last_hip_error = hipGetErrorString(le);
            return GPUDIFF_E_DEVICE;
        }
    }
    // K10's deferrals: the host path over the same staged JSON, read back from HBM (the batch may have been
    // uploaded zero-copy from a caller's buffer that is reusable since gpudiff_wait returned, and a staging
    // copy in the ring slot may belong to another batch)
    std::vector<uint32_t> def;
    for (size_t k = 0; k < nd; k++)
        if (to[k].status != GPUDIFF_TOK_OK) def.push_back((uint32_t)k);
    std::vector<uint64_t> hoff(def.size() + 1, 0);
    for (size_t k = 0; k < def.size(); k++) hoff[k + 1] = hoff[k] + docs[def[k]].json_len;
    std::vector<uint8_t> hjson;
    if (!def.empty()) {
        // one gather on the device (K7's 16-B copies: staged documents start 16-B aligned and their spans run at
        // least 16 bytes past their ends), then ONE copy back -- not a pageable round trip per document
        std::vector<BlobMove> mv(def.size());
        uint64_t gb = 0;
        for (size_t k = 0; k < def.size(); k++) {
            const TokDoc& d = docs[def[k]];
            mv[k] = BlobMove{d.json_off, gb, ((uint64_t)d.json_len + 15u) & ~15ull};
            hoff[k] = gb;
            gb += mv[k].bytes;
        }
        hjson.resize(gb);
        void *d_mv = nullptr, *d_gather = nullptr;
        hipError_t e = hipMalloc(&d_mv, mv.size() * sizeof(BlobMove));
        if (e == hipSuccess) e = hipMalloc(&d_gather, std::max<uint64_t>(gb, 16));
        if (e == hipSuccess)
            e = hipMemcpyAsync(d_mv, mv.data(), mv.size() * sizeof(BlobMove), hipMemcpyHostToDevice, c->stream);
        if (e == hipSuccess)
            e = launch_move_blobs(c->stream, sp.djson, (uint8_t*)d_gather, (const BlobMove*)d_mv, (uint32_t)mv.size());
        // the staged JSON's read marker again, behind the last read of it (k0_done covers every read)
        if (e == hipSuccess && dstore_staged_mark_read(c, ticket)) e = hipErrorUnknown;
        if (e == hipSuccess) e = hipMemcpyAsync(hjson.data(), d_gather, gb, hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        for (void* q : {d_mv, d_gather})
            if (q) (void)hipFree(q);
        if (e != hipSuccess) {
            gd::g_last_hip_error = hipGetErrorString(e);
            return GPUDIFF_E_DEVICE;
        }
    }
    std::vector<std::string> hb(def.size());
    std::vector<uint8_t> hok(def.size(), 0);
    const uint32_t mode_split = n_spec_docs;
    {
        const uint32_t T = std::max<uint32_t>(1, std::min<uint32_t>(c->threads, (uint32_t)((def.size() + 63) / 64)));
        auto work = [&](uint32_t t) {
            for (size_t k = t; k < def.size(); k += T) {
                const TokDoc& d = docs[def[k]];
                hok[k] = host_body(hjson.data() + hoff[k], d.json_len,
                                   def[k] < mode_split ? GPUDIFF_UPSERT_SPEC : GPUDIFF_UPSERT_STATUS, hb[k])
                             ? 1
                             : 0;
            }
        };
        workers(c).run(T, work);
    }
    std::vector<int32_t> hidx(nd, -1);
    for (size_t k = 0; k < def.size(); k++) hidx[def[k]] = (int32_t)k;
    BodiesStore* bs = new (std::nothrow) BodiesStore();
    if (!bs) return GPUDIFF_E_NOMEM;
    bs->offsets.resize(nw + 1);
    bs->status.assign(nw, 0);
    bs->k10.assign(nw, GPUDIFF_TOK_OK);
    bs->source.assign(nw, GPUDIFF_BODY_DEVICE);
    for (size_t w = 0; w < nw; w++) {
        bs->offsets[w] = bs->bytes.size();
        if (wdoc[w] == UINT32_MAX) continue;  // no-op write: no body
        const uint32_t k = wdoc[w];
        bs->k10[w] = (int32_t)to[k].status;
        if (to[k].status == GPUDIFF_TOK_OK) {
            const uint8_t* p = raw.data() + to[k].off;
            bs->bytes.insert(bs->bytes.end(), p, p + to[k].bytes);
        } else {
            bs->source[w] = GPUDIFF_BODY_HOST;
            const int32_t h = hidx[k];
            if (hok[h]) bs->bytes.insert(bs->bytes.end(), hb[h].begin(), hb[h].end());
            else bs->status[w] = GPUDIFF_E_DECODE;
        }
    }
    bs->offsets[nw] = bs->bytes.size();
    publish(bs, &out->bodies, nw, def.size());
    out->n = nw;
    out->pair_index = ps->pair_index.data();
    out->kind = ps->kind.data();
    out->noop = ps->noop.data();
    out->internal = ps.release();
    return GPUDIFF_OK;
}

void gpudiff_write_plan_release(gpudiff_ctx* c, gpudiff_write_plan* p) {
    if (!p) return;
    gpudiff_bodies_release(c, &p->bodies);
    delete (PlanStore*)p->internal;
    memset(p, 0, sizeof(*p));
}

}  // extern "C"
