// CPU restatement of the Deployment splitter's status roll-up -- TEST
// INFRASTRUCTURE ONLY (checker and CPU baseline; the product never links it).
//
// Follows oracle/rollup_oracle.py step for step, in C++ for timing:
//   * decode each cached Deployment's JSON into a DOM that keeps every object
//     member in document order (repeated keys included), numbers as literal
//     text -- Go 1.16 encoding/json's scanner rules (grammar, escapes, U+FFFD
//     repair, control characters, depth 10000);
//   * typed-decode restatement of the fields the splitter reads
//     (pkg/reconciler/deployment/deployment.go:42-85): struct field lookup
//     exact-or-fold, repeated keys merging into the same field, null as a
//     no-op (nil for the labels map, "" for a map element), int32 counters
//     from strconv.ParseInt-accepted literals only;
//   * the reconcile loop's aggregation for every root at once: group by the
//     kcp.dev/owned-by value (the lister selector, :44-51), int32 wrap-around
//     sums (:79-85), others[0] = lowest document index (:89-91).
#include <stdint.h>
#include <string.h>

#include <chrono>
#include <memory>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace {

struct V {
    enum T : uint8_t { NUL, BOOL, NUM, STR, OBJ, ARR } t = NUL;
    std::string s;                                  // STR: decoded bytes; NUM: literal
    std::vector<std::pair<std::string, V>> mem;     // OBJ, document order
    std::vector<V> arr;
};

struct P {
    const uint8_t* p;
    const uint8_t* e;
    void ws() {
        while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) p++;
    }
    static int rlen(const uint8_t* q, const uint8_t* e) {
        const uint8_t c = q[0];
        int n;
        uint8_t lo = 0x80, hi = 0xBF;
        if (c < 0x80) return 1;
        if (c >= 0xC2 && c <= 0xDF) n = 2;
        else if (c == 0xE0) n = 3, lo = 0xA0;
        else if ((c >= 0xE1 && c <= 0xEC) || c == 0xEE || c == 0xEF) n = 3;
        else if (c == 0xED) n = 3, hi = 0x9F;
        else if (c == 0xF0) n = 4, lo = 0x90;
        else if (c >= 0xF1 && c <= 0xF3) n = 4;
        else if (c == 0xF4) n = 4, hi = 0x8F;
        else return 0;
        if (e - q < n || q[1] < lo || q[1] > hi) return 0;
        for (int k = 2; k < n; k++)
            if (q[k] < 0x80 || q[k] > 0xBF) return 0;
        return n;
    }
    static void utf8(std::string& o, uint32_t r) {
        if (r < 0x80) {
            o += (char)r;
        } else if (r < 0x800) {
            o += (char)(0xC0 | (r >> 6));
            o += (char)(0x80 | (r & 63));
        } else if (r < 0x10000) {
            o += (char)(0xE0 | (r >> 12));
            o += (char)(0x80 | ((r >> 6) & 63));
            o += (char)(0x80 | (r & 63));
        } else {
            o += (char)(0xF0 | (r >> 18));
            o += (char)(0x80 | ((r >> 12) & 63));
            o += (char)(0x80 | ((r >> 6) & 63));
            o += (char)(0x80 | (r & 63));
        }
    }
    int hex4(const uint8_t* q) {
        if (e - q < 6 || q[0] != '\\' || q[1] != 'u') return -1;
        int v = 0;
        for (int k = 2; k < 6; k++) {
            const uint8_t c = q[k];
            const int h = c >= '0' && c <= '9' ? c - '0' : c >= 'a' && c <= 'f' ? c - 'a' + 10
                        : c >= 'A' && c <= 'F' ? c - 'A' + 10 : -1;
            if (h < 0) return -1;
            v = v * 16 + h;
        }
        return v;
    }
    bool str(std::string& o) {
        p++;
        while (true) {
            if (p >= e) return false;
            const uint8_t c = *p;
            if (c == '"') {
                p++;
                return true;
            }
            if (c == '\\') {
                if (e - p < 2) return false;
                const uint8_t x = p[1];
                const char* m = strchr("\"\\/bfnrt", x);
                if (x && m) {
                    o += "\"\\/\b\f\n\r\t"[m - "\"\\/bfnrt"];
                    p += 2;
                    continue;
                }
                int r = hex4(p);
                if (r < 0) return false;
                p += 6;
                if (r >= 0xD800 && r < 0xE000) {
                    const int r2 = hex4(p);
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
            const int n = rlen(p, e);
            if (!n) {
                o += "\xEF\xBF\xBD";
                p++;
            } else {
                o.append((const char*)p, n);
                p += n;
            }
        }
    }
    bool digits() {
        if (p >= e || *p < '0' || *p > '9') return false;
        while (p < e && *p >= '0' && *p <= '9') p++;
        return true;
    }
    bool value(V& v, int depth) {
        ws();
        if (p >= e) return false;
        const uint8_t c = *p;
        if (c == '{' || c == '[') {
            if (depth + 1 > 10000) return false;
            const bool ob = c == '{';
            v.t = ob ? V::OBJ : V::ARR;
            p++;
            ws();
            if (p < e && *p == (ob ? '}' : ']')) {
                p++;
                return true;
            }
            while (true) {
                ws();
                if (ob) {
                    if (p >= e || *p != '"') return false;
                    v.mem.emplace_back();
                    if (!str(v.mem.back().first)) return false;
                    ws();
                    if (p >= e || *p != ':') return false;
                    p++;
                    if (!value(v.mem.back().second, depth + 1)) return false;
                } else {
                    v.arr.emplace_back();
                    if (!value(v.arr.back(), depth + 1)) return false;
                }
                ws();
                if (p >= e) return false;
                const uint8_t x = *p++;
                if (x == ',') continue;
                return x == (ob ? '}' : ']');
            }
        }
        if (c == '"') {
            v.t = V::STR;
            return str(v.s);
        }
        auto word = [&](const char* w, V::T t) {
            const size_t n = strlen(w);
            if ((size_t)(e - p) < n || memcmp(p, w, n)) return false;
            p += n;
            v.t = t;
            return true;
        };
        if (c == 't') return word("true", V::BOOL);
        if (c == 'f') return word("false", V::BOOL);
        if (c == 'n') return word("null", V::NUL);
        const uint8_t* s = p;
        if (*p == '-') p++;
        if (p < e && *p == '0') p++;
        else if (!digits()) return false;
        if (p < e && *p == '.') {
            p++;
            if (!digits()) return false;
        }
        if (p < e && (*p == 'e' || *p == 'E')) {
            p++;
            if (p < e && (*p == '+' || *p == '-')) p++;
            if (!digits()) return false;
        }
        v.t = V::NUM;
        v.s.assign((const char*)s, p - s);
        return true;
    }
};

// encoding/json field lookup: ASCII case folding; U+017F folds to s, U+212A to k
bool fold(const char* name, const std::string& key) {
    size_t i = 0;
    for (; *name; name++) {
        if (i >= key.size()) return false;
        const uint8_t c = (uint8_t)key[i], n = (uint8_t)*name;
        if (c < 0x80) {
            const uint8_t lc = c >= 'A' && c <= 'Z' ? c + 32 : c, ln = n >= 'A' && n <= 'Z' ? n + 32 : n;
            if (lc != ln) return false;
            i++;
        } else if ((n | 32) == 's' && key.compare(i, 2, "\xC5\xBF") == 0) {
            i += 2;
        } else if ((n | 32) == 'k' && key.compare(i, 3, "\xE2\x84\xAA") == 0) {
            i += 3;
        } else {
            return false;
        }
    }
    return i == key.size();
}

const char* kF[5] = {"replicas", "updatedReplicas", "readyReplicas", "availableReplicas", "unavailableReplicas"};

struct Doc {
    bool ok = false, has = false;
    int32_t v[5] = {0, 0, 0, 0, 0};
    std::string owned;
};

bool to_i32(const V& x, int32_t* out) {
    if (x.t == V::NUL) return true;
    if (x.t != V::NUM) return false;
    const std::string& s = x.s;
    size_t i = s[0] == '-' ? 1 : 0;
    long long v = 0;
    for (; i < s.size(); i++) {
        if (s[i] < '0' || s[i] > '9') return false;
        v = v * 10 + (s[i] - '0');
        if (v > (1ll << 31)) return false;
    }
    if (s[0] == '-') v = -v;
    if (v < -(1ll << 31) || v > (1ll << 31) - 1) return false;
    *out = (int32_t)v;
    return true;
}

void extract(const uint8_t* d, size_t n, Doc& out) {
    out = Doc();
    P p{d, d + n};
    V root;
    p.ws();
    if (p.p >= p.e || *p.p != '{' || !p.value(root, 0)) return;
    p.ws();
    if (p.p != p.e) return;
    bool labels_nil = true;
    std::unordered_map<std::string, std::string> labels;
    for (auto& m : root.mem) {
        const bool is_md = fold("metadata", m.first), is_st = !is_md && fold("status", m.first);
        if (!is_md && !is_st) continue;
        const V& v = m.second;
        if (v.t == V::NUL) continue;
        if (v.t != V::OBJ) return;
        for (auto& f : v.mem) {
            if (is_md) {
                if (!fold("labels", f.first)) continue;
                if (f.second.t == V::NUL) {
                    labels_nil = true;
                    labels.clear();
                    continue;
                }
                if (f.second.t != V::OBJ) return;
                labels_nil = false;
                for (auto& l : f.second.mem) {
                    if (l.second.t == V::NUL) labels[l.first] = "";
                    else if (l.second.t == V::STR) labels[l.first] = l.second.s;
                    else return;
                }
            } else {
                for (int k = 0; k < 5; k++)
                    if (fold(kF[k], f.first)) {
                        if (!to_i32(f.second, &out.v[k])) return;
                        break;
                    }
            }
        }
    }
    if (!labels_nil) {
        auto it = labels.find("kcp.dev/owned-by");
        if (it != labels.end()) {
            out.has = true;
            out.owned = it->second;
        }
    }
    out.ok = true;
}

struct Docs {
    std::vector<std::string> src;
};

struct Result {
    std::vector<int32_t> doc_group;
    std::vector<uint32_t> first, count;
    std::vector<int32_t> sums;
};

void run_once(const Docs& D, int threads, Result& R) {
    const size_t n = D.src.size();
    std::vector<Doc> ds(n);
    std::vector<std::thread> th;
    for (int t = 0; t < threads; t++)
        th.emplace_back([&, t] {
            for (size_t i = t; i < n; i += threads) extract((const uint8_t*)D.src[i].data(), D.src[i].size(), ds[i]);
        });
    for (auto& x : th) x.join();
    R.doc_group.assign(n, -1);
    R.first.clear();
    R.count.clear();
    R.sums.clear();
    std::unordered_map<std::string, int32_t> idx;
    idx.reserve(n);
    for (size_t i = 0; i < n; i++) {
        if (!ds[i].ok) {
            R.doc_group[i] = -2;
            continue;
        }
        if (!ds[i].has) continue;
        auto it = idx.emplace(ds[i].owned, (int32_t)R.first.size());
        if (it.second) {
            R.first.push_back((uint32_t)i);
            R.count.push_back(0);
            for (int k = 0; k < 5; k++) R.sums.push_back(0);
        }
        const int32_t g = it.first->second;
        R.count[g]++;
        for (int k = 0; k < 5; k++) R.sums[5 * g + k] = (int32_t)((uint32_t)R.sums[5 * g + k] + (uint32_t)ds[i].v[k]);
        R.doc_group[i] = g;
    }
}

}  // namespace

extern "C" {

void* oracle_rollup_load(const char** docs, const size_t* lens, size_t n) {
    Docs* D = new Docs();
    D->src.reserve(n);
    for (size_t i = 0; i < n; i++) D->src.emplace_back(docs[i], lens[i]);
    return D;
}

void oracle_rollup_free(void* h) { delete (Docs*)h; }

// decode + group, repeated until min_seconds; returns sweeps, *secs = elapsed;
// the last sweep's result into the out arrays (doc_group[n]; first/count[n],
// sums[5n] for up to n groups), *n_groups
int oracle_rollup_run(void* h, int threads, double min_seconds, double* secs, int32_t* doc_group, uint32_t* first,
                      uint32_t* count, int32_t* sums, size_t* n_groups) {
    const Docs& D = *(const Docs*)h;
    Result R;
    int sweeps = 0;
    const auto t0 = std::chrono::steady_clock::now();
    double el = 0;
    do {
        run_once(D, threads < 1 ? 1 : threads, R);
        sweeps++;
        el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    } while (el < min_seconds);
    *secs = el;
    const size_t n = D.src.size();
    if (doc_group) memcpy(doc_group, R.doc_group.data(), 4 * n);
    if (first) memcpy(first, R.first.data(), 4 * R.first.size());
    if (count) memcpy(count, R.count.data(), 4 * R.count.size());
    if (sums) memcpy(sums, R.sums.data(), 4 * R.sums.size());
    *n_groups = R.first.size();
    return sweeps;
}

}  // extern "C"
