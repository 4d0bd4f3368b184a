// CPU restatement of the kcp syncer change-detection predicates
// (TEST INFRASTRUCTURE / CPU BASELINE ONLY -- never linked into the product).
//
// Follows, line by line:
//   deepEqualApartFromStatus  pkg/syncer/specsyncer.go:17-41
//   deepEqualStatus           pkg/syncer/statussyncer.go:15-27
// over decoded unstructured trees with the value semantics of
// equality.Semantic.DeepEqual (apimachinery third_party/forked/golang/reflect,
// module pinned at go.mod:33), Unstructured.GetLabels/GetAnnotations
// (NestedStringMap: fresh map per call, nil on any non-string value) and the
// k8s util/json decode rules (int64 if ParseInt accepts the literal else
// float64; duplicate keys last-wins; Go string unescaping).  Maps are hash maps
// and every GetLabels/GetAnnotations/StringKeySet/Union call allocates, as the
// Go code does, so the timing reflects the reference algorithm's structure.
//
// This is the "port" CPU baseline of bench.py and the large-sample checker of
// the bench (decision bits only).  Parity of this restatement is pinned by
// tests/test_oracle_cpp.py against the Python oracle and the Appendix A.4 KATs;
// against the Go reference itself it is unpinned (no Go toolchain).
#include <errno.h>
#include <locale.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <charconv>
#include <chrono>
#include <memory>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../include/gpudiff_format.h"
#include "timed_threads.h"
#include "xxh64_ref.h"

namespace oracle {

struct Value;
using Map = std::unordered_map<std::string, Value>;
using Arr = std::vector<Value>;

struct Value {
    enum Kind : uint8_t { NIL, BOOL, INT, FLOAT, STR, MAP, ARR } k = NIL;
    bool b = false;
    int64_t i = 0;
    double f = 0;
    std::string s;
    std::shared_ptr<Map> m;
    std::shared_ptr<Arr> a;
};

// ------------------------------------------------------------ decoder
struct Dec {
    const unsigned char* p;
    const unsigned char* e;
    bool ok = true;
    int depth = 0;

    void ws() {
        while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) p++;
    }
    static void utf8(std::string& o, uint32_t r) {
        if (r < 0x80) o += (char)r;
        else if (r < 0x800) { o += (char)(0xC0 | (r >> 6)); o += (char)(0x80 | (r & 63)); }
        else if (r < 0x10000) { o += (char)(0xE0 | (r >> 12)); o += (char)(0x80 | ((r >> 6) & 63)); o += (char)(0x80 | (r & 63)); }
        else { o += (char)(0xF0 | (r >> 18)); o += (char)(0x80 | ((r >> 12) & 63)); o += (char)(0x80 | ((r >> 6) & 63)); o += (char)(0x80 | (r & 63)); }
    }
    // Go utf8.DecodeRune: length of a valid rune at q, or 0
    int rune(const unsigned char* q) {
        unsigned c = q[0];
        int n;
        unsigned lo = 0x80, hi = 0xBF;
        if (c < 0x80) return 1;
        if (c >= 0xC2 && c <= 0xDF) n = 2;
        else if (c == 0xE0) { n = 3; lo = 0xA0; }
        else if (c >= 0xE1 && c <= 0xEF && c != 0xED) n = 3;
        else if (c == 0xED) { n = 3; hi = 0x9F; }
        else if (c == 0xF0) { n = 4; lo = 0x90; }
        else if (c >= 0xF1 && c <= 0xF3) n = 4;
        else if (c == 0xF4) { n = 4; hi = 0x8F; }
        else return 0;
        if (e - q < n || q[1] < lo || q[1] > hi) return 0;
        for (int j = 2; j < n; j++)
            if (q[j] < 0x80 || q[j] > 0xBF) return 0;
        return n;
    }
    int u4(const unsigned char* q) {
        if (e - q < 6 || q[0] != '\\' || q[1] != 'u') return -1;
        int v = 0;
        for (int j = 2; j < 6; j++) {
            int c = q[j], h;
            if (c >= '0' && c <= '9') h = c - '0';
            else if (c >= 'a' && c <= 'f') h = c - 'a' + 10;
            else if (c >= 'A' && c <= 'F') h = c - 'A' + 10;
            else return -1;
            v = v * 16 + h;
        }
        return v;
    }
    bool str(std::string& o) {
        p++;
        for (;;) {
            if (p >= e) return false;
            unsigned c = *p;
            if (c == '"') { p++; return true; }
            if (c == '\\') {
                if (e - p < 2) return false;
                unsigned x = p[1];
                const char* simple = "\"\\/bfnrt";
                const char* rep = "\"\\/\b\f\n\r\t";
                const char* f = x ? strchr(simple, (int)x) : nullptr;
                if (f) { o += rep[f - simple]; p += 2; continue; }
                if (x != 'u') return false;
                int r = u4(p);
                if (r < 0) return false;
                p += 6;
                if (r >= 0xD800 && r < 0xE000) {
                    int r2 = u4(p);
                    if (r < 0xDC00 && r2 >= 0xDC00 && r2 < 0xE000) {
                        utf8(o, 0x10000 + (((uint32_t)r - 0xD800) << 10) + ((uint32_t)r2 - 0xDC00));
                        p += 6;
                        continue;
                    }
                    r = 0xFFFD;
                }
                utf8(o, (uint32_t)r);
                continue;
            }
            if (c < 0x20) return false;
            int n = rune(p);
            if (n == 0) { o += "\xEF\xBF\xBD"; p++; }
            else { o.append((const char*)p, n); p += n; }
        }
    }
    bool num(Value& v) {
        const unsigned char* s = p;
        if (*p == '-') p++;
        if (p >= e) return false;
        if (*p == '0') p++;
        else if (*p >= '1' && *p <= '9') { while (p < e && *p >= '0' && *p <= '9') p++; }
        else return false;
        bool integer = true;
        if (p < e && *p == '.') {
            integer = false;
            p++;
            if (p >= e || *p < '0' || *p > '9') return false;
            while (p < e && *p >= '0' && *p <= '9') p++;
        }
        if (p < e && (*p == 'e' || *p == 'E')) {
            integer = false;
            p++;
            if (p < e && (*p == '+' || *p == '-')) p++;
            if (p >= e || *p < '0' || *p > '9') return false;
            while (p < e && *p >= '0' && *p <= '9') p++;
        }
        std::string t((const char*)s, (size_t)(p - s));
        if (integer) {  // strconv.ParseInt(t, 10, 64)
            errno = 0;
            char* end = nullptr;
            long long x = strtoll(t.c_str(), &end, 10);
            if (errno == 0 && end && *end == 0) {
                v.k = Value::INT;
                v.i = x;
                return true;
            }
        }
        static locale_t cl = newlocale(LC_ALL_MASK, "C", (locale_t)0);
        double d = strtod_l(t.c_str(), nullptr, cl);  // strconv.ParseFloat
        if (isinf(d)) return false;
        v.k = Value::FLOAT;
        v.f = d;
        return true;
    }
    bool val(Value& v) {
        ws();
        if (p >= e) return false;
        unsigned c = *p;
        if (c == '{') {
            if (++depth > 10000) return false;
            p++;
            v.k = Value::MAP;
            v.m = std::make_shared<Map>();
            ws();
            if (p < e && *p == '}') { p++; depth--; return true; }
            for (;;) {
                ws();
                if (p >= e || *p != '"') return false;
                std::string key;
                if (!str(key)) return false;
                ws();
                if (p >= e || *p != ':') return false;
                p++;
                Value x;
                if (!val(x)) return false;
                (*v.m)[key] = std::move(x);  // last one wins
                ws();
                if (p >= e) return false;
                c = *p++;
                if (c == ',') continue;
                if (c == '}') { depth--; return true; }
                return false;
            }
        }
        if (c == '[') {
            if (++depth > 10000) return false;
            p++;
            v.k = Value::ARR;
            v.a = std::make_shared<Arr>();
            ws();
            if (p < e && *p == ']') { p++; depth--; return true; }
            for (;;) {
                Value x;
                if (!val(x)) return false;
                v.a->push_back(std::move(x));
                ws();
                if (p >= e) return false;
                c = *p++;
                if (c == ',') continue;
                if (c == ']') { depth--; return true; }
                return false;
            }
        }
        if (c == '"') { v.k = Value::STR; return str(v.s); }
        if (e - p >= 4 && !memcmp(p, "true", 4)) { p += 4; v.k = Value::BOOL; v.b = true; return true; }
        if (e - p >= 5 && !memcmp(p, "false", 5)) { p += 5; v.k = Value::BOOL; v.b = false; return true; }
        if (e - p >= 4 && !memcmp(p, "null", 4)) { p += 4; v.k = Value::NIL; return true; }
        if (c == '-' || (c >= '0' && c <= '9')) return num(v);
        return false;
    }
};

bool decode(const char* data, size_t n, Value& out) {
    Dec d{(const unsigned char*)data, (const unsigned char*)data + n};
    d.ws();
    if (d.p >= d.e || *d.p != '{') return false;
    if (!d.val(out)) return false;
    d.ws();
    return d.p == d.e;
}

// ------------------------------------------------------------ DeepEqual
bool deep_equal(const Value& x, const Value& y) {
    if (x.k == Value::NIL || y.k == Value::NIL) return x.k == Value::NIL && y.k == Value::NIL;
    if (x.k != y.k) return false;
    switch (x.k) {
        case Value::BOOL: return x.b == y.b;
        case Value::INT: return x.i == y.i;
        case Value::FLOAT: return x.f == y.f;
        case Value::STR: return x.s == y.s;
        case Value::MAP: {
            if (x.m->empty() || y.m->empty()) return x.m->empty() && y.m->empty();
            if (x.m->size() != y.m->size()) return false;
            for (const auto& kv : *x.m) {
                auto it = y.m->find(kv.first);
                if (it == y.m->end()) return false;
                if (!deep_equal(kv.second, it->second)) return false;
            }
            return true;
        }
        case Value::ARR: {
            if (x.a->empty() || y.a->empty()) return x.a->empty() && y.a->empty();
            if (x.a->size() != y.a->size()) return false;
            for (size_t i = 0; i < x.a->size(); i++)
                if (!deep_equal((*x.a)[i], (*y.a)[i])) return false;
            return true;
        }
        default: return true;
    }
}

using StrMap = std::unordered_map<std::string, std::string>;

// unstructured.NestedStringMap(obj, "metadata", field): a fresh map, or nil
std::unique_ptr<StrMap> nested_string_map(const Value& obj, const char* field) {
    auto md = obj.m->find("metadata");
    if (md == obj.m->end() || md->second.k != Value::MAP) return nullptr;
    auto f = md->second.m->find(field);
    if (f == md->second.m->end() || f->second.k != Value::MAP) return nullptr;
    std::unique_ptr<StrMap> out(new StrMap());
    out->reserve(f->second.m->size());
    for (const auto& kv : *f->second.m) {
        if (kv.second.k != Value::STR) return nullptr;
        (*out)[kv.first] = kv.second.s;
    }
    return out;
}

bool de_string_map(const StrMap* a, const StrMap* b) {
    const bool ea = !a || a->empty(), eb = !b || b->empty();
    if (ea || eb) return ea && eb;
    if (a->size() != b->size()) return false;
    for (const auto& kv : *a) {
        auto it = b->find(kv.first);
        if (it == b->end() || it->second != kv.second) return false;
    }
    return true;
}

static const Value kNil;

// specsyncer.go:17-41
bool deep_equal_apart_from_status(const Value& o, const Value& n) {
    {
        auto a = nested_string_map(o, "annotations"), b = nested_string_map(n, "annotations");  // :23
        if (!de_string_map(a.get(), b.get())) return false;
    }
    {
        auto a = nested_string_map(o, "labels"), b = nested_string_map(n, "labels");  // :26
        if (!de_string_map(a.get(), b.get())) return false;
    }
    std::unordered_set<std::string> ok, nk;  // sets.StringKeySet x2 (:30-31)
    for (const auto& kv : *o.m) ok.insert(kv.first);
    for (const auto& kv : *n.m) nk.insert(kv.first);
    std::unordered_set<std::string> uni(ok);  // Union (:32)
    uni.insert(nk.begin(), nk.end());
    std::vector<std::string> keys(uni.begin(), uni.end());  // UnsortedList
    for (const std::string& key : keys) {
        if (key == "metadata" || key == "status") continue;  // :33-35
        auto x = o.m->find(key), y = n.m->find(key);
        const Value& vx = x == o.m->end() ? kNil : x->second;
        const Value& vy = y == n.m->end() ? kNil : y->second;
        if (!deep_equal(vx, vy)) return false;  // :36
    }
    return true;
}

// statussyncer.go:15-27
bool deep_equal_status(const Value& o, const Value& n) {
    auto ns = n.m->find("status");
    if (ns != n.m->end()) {  // :22
        auto os = o.m->find("status");
        return deep_equal(os == o.m->end() ? kNil : os->second, ns->second);  // :23-24
    }
    return false;  // :26
}

// apimachinery unstructuredJSONScheme.decode [3P] probes the bytes with
// encoding/json into struct{ Items json.RawMessage } first: a top-level key
// equal to "Items" under fold.go's equalFoldRight (ASCII case folding, U+017F
// for s) decodes as an UnstructuredList, and the predicates' type assertions
// (specsyncer.go:18-22, statussyncer.go:16-20) fail
static bool list_probe(const Value& root) {
    for (const auto& kv : *root.m) {
        const std::string& k = kv.first;
        const char* name = "Items";
        size_t i = 0;
        bool ok = true;
        for (const char* s = name; *s && ok; s++) {
            if (i >= k.size()) { ok = false; break; }
            const unsigned char t = (unsigned char)k[i];
            if (t < 0x80) {
                ok = (unsigned char)(*s | 0x20) == (t | 0x20) && ((t | 0x20) >= 'a' && (t | 0x20) <= 'z');
                i++;
            } else if ((*s == 's' || *s == 'S') && t == 0xC5 && i + 1 < k.size() && (unsigned char)k[i + 1] == 0xBF) {
                i += 2;
            } else {
                ok = false;
            }
        }
        if (ok && i == k.size()) return true;
    }
    return false;
}

// ------------------------------------------------------------ field-path diff (build-defined)
// The same definition as the Python oracle (oracle/gpudiff_oracle.py spec_leaves /
// status_leaves / _region_diff), over the decoded trees: leaves keyed by their encoded
// path (0x01 u32le(len) key | 0x02 u32le(index)), chained path hash under the pair's seed.
struct Leaf {
    uint8_t tag;
    std::string bytes;
    bool operator==(const Leaf& o) const { return tag == o.tag && bytes == o.bytes; }
};
using LeafMap = std::unordered_map<std::string, std::pair<uint64_t, Leaf>>;  // path bytes -> (hash, leaf)

static void put_comp(std::string& p, uint8_t kind, const void* data, uint32_t n) {
    p.push_back((char)kind);
    if (kind == 0x01) {
        p.append((const char*)&n, 4);
        p.append((const char*)data, n);
    } else {
        p.append((const char*)data, 4);
    }
}

// reported path hashes are cut to the build's width (include/gpudiff_format.h)
static const uint64_t kPathMask = (1ull << GPUDIFF_PATH_HASH_BITS) - 1;

static void flatten(const Value& v, std::string& path, uint64_t h, LeafMap& out) {
    if (v.k == Value::MAP && !v.m->empty()) {
        for (const auto& kv : *v.m) {
            const size_t mark = path.size();
            put_comp(path, 0x01, kv.first.data(), (uint32_t)kv.first.size());
            flatten(kv.second, path, xxh64_ref(path.data() + mark, path.size() - mark, h), out);
            path.resize(mark);
        }
        return;
    }
    if (v.k == Value::ARR && !v.a->empty()) {
        for (uint32_t i = 0; i < v.a->size(); i++) {
            const size_t mark = path.size();
            put_comp(path, 0x02, &i, 4);
            flatten((*v.a)[i], path, xxh64_ref(path.data() + mark, path.size() - mark, h), out);
            path.resize(mark);
        }
        return;
    }
    Leaf l;
    switch (v.k) {
        case Value::NIL: l.tag = 0; break;
        case Value::BOOL: l.tag = v.b ? 2 : 1; break;
        case Value::INT: l.tag = 3; l.bytes.assign((const char*)&v.i, 8); break;
        case Value::FLOAT: {
            const double d = v.f == 0.0 ? 0.0 : v.f;
            l.tag = 4;
            l.bytes.assign((const char*)&d, 8);
            break;
        }
        case Value::STR: l.tag = 5; l.bytes = v.s; break;
        case Value::MAP: l.tag = 6; break;
        default: l.tag = 7; break;
    }
    out[path] = {h, std::move(l)};
}

static uint64_t key_hash(uint64_t h, const char* k, std::string& path) {
    const size_t mark = path.size();
    put_comp(path, 0x01, k, (uint32_t)strlen(k));
    return xxh64_ref(path.data() + mark, path.size() - mark, h);
}

static void spec_leaves(const Value& o, uint64_t seed, LeafMap& out) {
    for (const auto& kv : *o.m) {
        if (kv.first == "metadata" || kv.first == "status" || kv.second.k == Value::NIL) continue;
        std::string path;
        put_comp(path, 0x01, kv.first.data(), (uint32_t)kv.first.size());
        flatten(kv.second, path, xxh64_ref(path.data(), path.size(), seed), out);
    }
    for (const char* field : {"labels", "annotations"}) {
        auto m = nested_string_map(o, field);
        if (!m || m->empty()) continue;
        std::string path;
        uint64_t h = key_hash(seed, "metadata", path);
        h = key_hash(h, field, path);
        for (const auto& kv : *m) {
            const size_t mark = path.size();
            put_comp(path, 0x01, kv.first.data(), (uint32_t)kv.first.size());
            out[path] = {xxh64_ref(path.data() + mark, path.size() - mark, h), Leaf{5, kv.second}};
            path.resize(mark);
        }
    }
}

static void status_leaves(const Value& o, uint64_t seed, LeafMap& out) {
    auto s = o.m->find("status");
    if (s == o.m->end() || s->second.k == Value::NIL) return;
    std::string path;
    const uint64_t h = key_hash(seed, "status", path);
    flatten(s->second, path, h, out);
}

// entries (hash, kind | region bit) of one region, ascending hash
static void region_diff(const LeafMap& a, const LeafMap& b, uint8_t region_bit,
                        std::vector<std::pair<uint64_t, uint8_t>>& out) {
    const size_t base = out.size();
    for (const auto& kv : a) {
        auto it = b.find(kv.first);
        if (it == b.end()) out.push_back({kv.second.first, (uint8_t)(2 | region_bit)});  // removed
        else if (!(it->second.second == kv.second.second)) out.push_back({kv.second.first, (uint8_t)(0 | region_bit)});
    }
    for (const auto& kv : b)
        if (!a.count(kv.first)) out.push_back({kv.second.first, (uint8_t)(1 | region_bit)});  // added
    for (size_t i = base; i < out.size(); i++) out[i].first &= kPathMask;  // the build's width
    std::sort(out.begin() + base, out.end());
}

struct Pairs {
    std::vector<Value> a, b;
    std::vector<uint8_t> err;
};

}  // namespace oracle

using namespace oracle;

extern "C" {

// decode n pairs (untimed); returns a handle
void* oracle_load(const char* const* a, const size_t* alen, const char* const* b, const size_t* blen, size_t n) {
    Pairs* p = new Pairs();
    p->a.resize(n);
    p->b.resize(n);
    p->err.assign(n, 0);
    for (size_t i = 0; i < n; i++) {
        if (!decode(a[i], alen[i], p->a[i]) || !decode(b[i], blen[i], p->b[i]) || list_probe(p->a[i]) ||
            list_probe(p->b[i]))
            p->err[i] = 1;
    }
    return p;
}

// changed paths of every pair (checker, untimed): pair i under path-hash seed
// seeds[i]; for each dirty pair, offsets[k] .. offsets[k+1] of (hashes, kinds)
// in output order -- spec entries by ascending hash, then (status dirty only)
// status entries, then the status-absent sentinel.  Returns the number of
// entries, or -1 if cap is too small.
long oracle_tree_paths(void* h, const uint8_t* seeds, uint32_t* offsets, uint64_t* hashes, uint8_t* kinds,
                       size_t cap) {
    Pairs* p = (Pairs*)h;
    size_t k = 0, total = 0;
    offsets[0] = 0;
    std::vector<std::pair<uint64_t, uint8_t>> ent;
    for (size_t i = 0; i < p->a.size(); i++) {
        if (p->err[i]) {
            offsets[++k] = (uint32_t)total;  // decode error: dirty, no paths
            continue;
        }
        const bool sd = !deep_equal_apart_from_status(p->a[i], p->b[i]);
        const bool td = !deep_equal_status(p->a[i], p->b[i]);
        if (!sd && !td) continue;
        ent.clear();
        LeafMap la, lb;
        spec_leaves(p->a[i], seeds[i], la);
        spec_leaves(p->b[i], seeds[i], lb);
        region_diff(la, lb, 0, ent);
        if (td) {
            LeafMap ta, tb;
            status_leaves(p->a[i], seeds[i], ta);
            status_leaves(p->b[i], seeds[i], tb);
            region_diff(ta, tb, 0x80, ent);
            if (!p->b[i].m->count("status")) {
                std::string path;
                ent.push_back({key_hash(seeds[i], "status", path) & kPathMask, (uint8_t)(3 | 0x80)});
            }
        }
        if (total + ent.size() > cap) return -1;
        for (const auto& e : ent) {
            hashes[total] = e.first;
            kinds[total] = e.second;
            total++;
        }
        offsets[++k] = (uint32_t)total;
    }
    return (long)total;
}

void oracle_free(void* h) { delete (Pairs*)h; }

// The full-size checker (tools/full_tree_check.py; TEST INFRASTRUCTURE): n pairs as JSON text, pair i's A
// at buf[offs[2i], offs[2i+1]) and B at buf[offs[2i+1], offs[2i+2]), decoded by this file's own decoder
// and decided + path-diffed by the tree walk (what oracle_load + oracle_decide + oracle_tree_paths do), on
// `threads` threads over contiguous slices, nothing kept between pairs.  flags[i] as oracle_decide; for the
// dirty pairs in order, offsets[k] .. offsets[k+1] of (hashes, kinds) as oracle_tree_paths.  Returns the
// entries written, or -1 if cap is too small.
long oracle_tree_check(const uint8_t* buf, const uint64_t* offs, size_t n, const uint8_t* seeds, int threads,
                       uint8_t* flags, uint32_t* offsets, uint64_t* hashes, uint8_t* kinds, size_t cap) {
    if (threads < 1) threads = 1;
    struct Part {
        std::vector<uint32_t> cnt;  // per dirty pair of the slice
        std::vector<std::pair<uint64_t, uint8_t>> ent;
    };
    std::vector<Part> parts(threads);
    auto work = [&](int t) {
        const size_t b = n * t / threads, e = n * (t + 1) / threads;
        Part& P = parts[t];
        std::vector<std::pair<uint64_t, uint8_t>> ent;
        for (size_t i = b; i < e; i++) {
            Value va, vb;
            const char* pa = (const char*)buf + offs[2 * i];
            const char* pb = (const char*)buf + offs[2 * i + 1];
            if (!decode(pa, offs[2 * i + 1] - offs[2 * i], va) || !decode(pb, offs[2 * i + 2] - offs[2 * i + 1], vb) ||
                list_probe(va) || list_probe(vb)) {
                flags[i] = 7;
                P.cnt.push_back(0);
                continue;
            }
            const bool sd = !deep_equal_apart_from_status(va, vb);
            const bool td = !deep_equal_status(va, vb);
            flags[i] = (sd ? 1 : 0) | (td ? 2 : 0);
            if (!sd && !td) continue;
            ent.clear();
            LeafMap la, lb;
            spec_leaves(va, seeds[i], la);
            spec_leaves(vb, seeds[i], lb);
            region_diff(la, lb, 0, ent);
            if (td) {
                LeafMap ta, tb;
                status_leaves(va, seeds[i], ta);
                status_leaves(vb, seeds[i], tb);
                region_diff(ta, tb, 0x80, ent);
                if (!vb.m->count("status")) {
                    std::string path;
                    ent.push_back({key_hash(seeds[i], "status", path) & kPathMask, (uint8_t)(3 | 0x80)});
                }
            }
            P.cnt.push_back((uint32_t)ent.size());
            P.ent.insert(P.ent.end(), ent.begin(), ent.end());
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < threads; t++) th.emplace_back(work, t);
    work(0);
    for (auto& x : th) x.join();
    size_t total = 0, k = 0;
    offsets[0] = 0;
    for (const Part& P : parts) {
        if (total + P.ent.size() > cap) return -1;
        size_t j = 0;
        for (uint32_t c : P.cnt) {
            for (uint32_t q = 0; q < c; q++, j++) {
                hashes[total] = P.ent[j].first;
                kinds[total] = P.ent[j].second;
                total++;
            }
            offsets[++k] = (uint32_t)total;
        }
    }
    return (long)total;
}

// runs both predicates over every pair; flags bit0 spec dirty, bit1 status
// dirty, bit2 decode error.  Threads repeat their slices until min_seconds
// elapsed; returns the sweeps done (fractional) and the wall seconds.
double oracle_decide(void* h, uint8_t* flags, int threads, double min_seconds, double* seconds) {
    Pairs* p = (Pairs*)h;
    return timed_sweeps(p->a.size(), threads, min_seconds, seconds, [&](int, size_t b, size_t e) {
        for (size_t i = b; i < e; i++) {
            uint8_t f;
            if (p->err[i]) f = 7;
            else f = (deep_equal_apart_from_status(p->a[i], p->b[i]) ? 0 : 1) |
                     (deep_equal_status(p->a[i], p->b[i]) ? 0 : 2);
            flags[i] = f;
        }
    });
}

}  // extern "C"

// ------------------------------------------------------------ write path
// upsertIntoDownstream (pkg/syncer/specsyncer.go:94-110): unstrob.DeepCopy(),
// SetUID(""), SetResourceVersion(""), owner references whose Name equals the
// kcp.dev/owned-by label (GetLabels: NestedStringMap) dropped, the rest written
// back as ToUnstructured(&OwnerReference) maps; the field removed when none are
// kept.  updateStatusInUpstream (statussyncer.go:44-48): DeepCopy, SetUID(""),
// SetResourceVersion("").  Then the dynamic client's body,
// json.NewEncoder(w).Encode(obj.Object) (Go 1.16): sorted keys, HTML-safe
// escaping, shortest floats, trailing newline.  Like the Go code, the
// transform works on a deep copy of the decoded (cached) object.
namespace oracle {

Value deep_copy(const Value& v) {
    Value o;
    o.k = v.k;
    o.b = v.b;
    o.i = v.i;
    o.f = v.f;
    o.s = v.s;
    if (v.k == Value::MAP) {
        o.m = std::make_shared<Map>();
        o.m->reserve(v.m->size());
        for (const auto& kv : *v.m) (*o.m)[kv.first] = deep_copy(kv.second);
    } else if (v.k == Value::ARR) {
        o.a = std::make_shared<Arr>();
        o.a->reserve(v.a->size());
        for (const auto& x : *v.a) o.a->push_back(deep_copy(x));
    }
    return o;
}

static Value str_value(const std::string& s) {
    Value v;
    v.k = Value::STR;
    v.s = s;
    return v;
}

void transform(Value& obj, int mode) {
    auto md = obj.m->find("metadata");
    if (md == obj.m->end() || md->second.k != Value::MAP) return;  // RemoveNestedField: no-op
    Map& m = *md->second.m;
    m.erase("uid");
    m.erase("resourceVersion");
    if (mode != 0) return;
    auto labels = nested_string_map(obj, "labels");
    std::string owned;
    if (labels) {
        auto it = labels->find("kcp.dev/owned-by");
        if (it != labels->end()) owned = it->second;
    }
    // GetOwnerReferences: nil unless a list of maps
    std::vector<Value> kept;
    auto refs = m.find("ownerReferences");
    if (refs != m.end() && refs->second.k == Value::ARR) {
        bool all_maps = true;
        for (const auto& e : *refs->second.a)
            if (e.k != Value::MAP) all_maps = false;
        if (all_maps) {
            for (const auto& e : *refs->second.a) {
                auto gs = [&](const char* k) {
                    auto it = e.m->find(k);
                    return it != e.m->end() && it->second.k == Value::STR ? it->second.s : std::string();
                };
                if (gs("name") == owned) continue;
                Value r;
                r.k = Value::MAP;
                r.m = std::make_shared<Map>();
                (*r.m)["apiVersion"] = str_value(gs("apiVersion"));
                (*r.m)["kind"] = str_value(gs("kind"));
                (*r.m)["name"] = str_value(gs("name"));
                (*r.m)["uid"] = str_value(gs("uid"));
                for (const char* k : {"controller", "blockOwnerDeletion"}) {
                    auto it = e.m->find(k);
                    if (it != e.m->end() && it->second.k == Value::BOOL) (*r.m)[k] = it->second;
                }
                kept.push_back(std::move(r));
            }
        }
    }
    if (kept.empty()) {
        m.erase("ownerReferences");
    } else {
        Value l;
        l.k = Value::ARR;
        l.a = std::make_shared<Arr>(std::move(kept));
        m["ownerReferences"] = std::move(l);
    }
}

static void m_str(std::string& o, const std::string& s) {
    static const char hx[] = "0123456789abcdef";
    o.push_back('"');
    for (size_t i = 0; i < s.size(); i++) {
        const unsigned char c = (unsigned char)s[i];
        if (c == '"' || c == '\\') { o.push_back('\\'); o.push_back((char)c); }
        else if (c == '\n') o += "\\n";
        else if (c == '\r') o += "\\r";
        else if (c == '\t') o += "\\t";
        else if (c < 0x20 || c == '<' || c == '>' || c == '&') { o += "\\u00"; o.push_back(hx[c >> 4]); o.push_back(hx[c & 15]); }
        else if (c == 0xE2 && i + 2 < s.size() && (unsigned char)s[i + 1] == 0x80 &&
                 ((unsigned char)s[i + 2] == 0xA8 || (unsigned char)s[i + 2] == 0xA9)) {
            o += (unsigned char)s[i + 2] == 0xA8 ? "\\u2028" : "\\u2029";
            i += 2;
        } else o.push_back((char)c);
    }
    o.push_back('"');
}

// strconv.AppendFloat(f, 'f'|'e', -1, 64): the shortest digits laid out
static void m_float(std::string& o, double f) {
    char b[64];
    auto r = std::to_chars(b, b + 63, f, std::chars_format::scientific);
    *r.ptr = 0;
    std::string s(b);
    const double a = fabs(f);
    if (a != 0 && (a < 1e-6 || a >= 1e21)) {
        const size_t n = s.size();
        if (n >= 4 && s[n - 4] == 'e' && s[n - 3] == '-' && s[n - 2] == '0') s.erase(n - 2, 1);
        o += s;
        return;
    }
    const size_t e = s.find('e');
    std::string mant = s.substr(0, e);
    const int x = atoi(s.c_str() + e + 1);
    bool neg = mant[0] == '-';
    std::string dig;
    for (char c : mant) if (c >= '0' && c <= '9') dig.push_back(c);
    const int nd = (int)dig.size();
    if (neg) o.push_back('-');
    if (x >= nd - 1) o += dig + std::string((size_t)(x - nd + 1), '0');
    else if (x >= 0) o += dig.substr(0, (size_t)x + 1) + "." + dig.substr((size_t)x + 1);
    else o += "0." + std::string((size_t)(-x - 1), '0') + dig;
}

void marshal(std::string& o, const Value& v) {
    switch (v.k) {
        case Value::NIL: o += "null"; break;
        case Value::BOOL: o += v.b ? "true" : "false"; break;
        case Value::INT: o += std::to_string(v.i); break;
        case Value::FLOAT: m_float(o, v.f); break;
        case Value::STR: m_str(o, v.s); break;
        case Value::ARR:
            o.push_back('[');
            for (size_t i = 0; i < v.a->size(); i++) {
                if (i) o.push_back(',');
                marshal(o, (*v.a)[i]);
            }
            o.push_back(']');
            break;
        case Value::MAP: {
            std::vector<const std::pair<const std::string, Value>*> kv;  // encoding/json sorts map keys
            kv.reserve(v.m->size());
            for (const auto& x : *v.m) kv.push_back(&x);
            std::sort(kv.begin(), kv.end(), [](auto* a, auto* b) { return a->first < b->first; });
            o.push_back('{');
            for (size_t i = 0; i < kv.size(); i++) {
                if (i) o.push_back(',');
                m_str(o, kv[i]->first);
                o.push_back(':');
                marshal(o, kv[i]->second);
            }
            o.push_back('}');
            break;
        }
    }
}

struct Docs {
    std::vector<Value> v;
    std::vector<uint8_t> err;
};

}  // namespace oracle

extern "C" {

void* oracle_docs_load(const char* const* d, const size_t* len, size_t n) {
    Docs* p = new Docs();
    p->v.resize(n);
    p->err.assign(n, 0);
    for (size_t i = 0; i < n; i++)
        if (!decode(d[i], len[i], p->v[i])) p->err[i] = 1;
    return p;
}

void oracle_docs_free(void* h) { delete (Docs*)h; }

// body of doc i (DeepCopy + transform + marshal); returns its length, -1 on a
// decode error; writes min(len, cap) bytes
long oracle_upsert_body(void* h, size_t i, int mode, char* out, size_t cap) {
    Docs* p = (Docs*)h;
    if (p->err[i]) return -1;
    Value c = deep_copy(p->v[i]);
    transform(c, mode);
    std::string o;
    marshal(o, c);
    o.push_back('\n');
    memcpy(out, o.data(), std::min(cap, o.size()));
    return (long)o.size();
}

// the timed CPU baseline: every document's body, threads repeating their
// slices until min_seconds; returns sweeps (fractional), *bytes = body bytes of
// one sweep
double oracle_upsert_run(void* h, int mode, int threads, double min_seconds, double* seconds, uint64_t* bytes) {
    Docs* p = (Docs*)h;
    if (threads < 1) threads = 1;
    std::vector<uint64_t> tb(threads, 0);
    const double sw = timed_sweeps(p->v.size(), threads, min_seconds, seconds, [&](int t, size_t b, size_t e) {
        uint64_t acc = 0;
        std::string o;
        for (size_t i = b; i < e; i++) {
            if (p->err[i]) continue;
            Value c = deep_copy(p->v[i]);
            transform(c, mode);
            o.clear();
            marshal(o, c);
            o.push_back('\n');
            acc += o.size();
        }
        tb[t] = acc;
    });
    if (bytes) {
        *bytes = 0;
        for (auto x : tb) *bytes += x;
    }
    return sw;
}

}  // extern "C"
