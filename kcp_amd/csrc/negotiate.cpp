// API-negotiation update classifier (second half): host side.
//
// The reference (pkg/reconciler/apiresource/controller.go:238-295) classifies
// one informer Update at a time on the handler goroutine.  The batch form here
// classifies n (old, new) pairs: K13 (negotiation mode of k_encode_docs)
// extracts every document's resourceVersion, generation, labels, annotations and
// status conditions in HBM, K14 (negotiate.hip) classifies each pair on the
// device.  Pairs holding a document outside K13's exact subset are classified
// by the host path below, so results never depend on who decided a pair.
//
// The host path restates Go 1.16 encoding/json's typed decode of the fields
// read (goscan.h: scanner grammar, escapes, field lookup with case folding;
// repeated keys decode again into the same field -- maps merge, structs merge,
// slices are re-decoded element by element into the existing backing array),
// metav1.Time's UnmarshalJSON (null -> zero Time, else time.Parse(RFC3339)),
// and Semantic.DeepEqual (nil == empty maps and slices, times by instant).
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <string>
#include <thread>
#include <vector>

#include "engine.h"
#include "goscan.h"
#include "tokenize.h"

using namespace gd;

struct gpudiff_nbatch {
    uint32_t n = 0;
    std::vector<TokDoc> docs;  // 2 per pair: old, new
    std::vector<const uint8_t*> olds, news;
    std::vector<size_t> old_lens, new_lens;
    std::vector<uint8_t> kinds;  // GPUDIFF_NEG_KIND_* per pair
    uint64_t json_bytes = 0, scratch_bytes = 0, n_host = 0;
    bool ran = false;  // a run was issued (fetch before any run: GPUDIFF_E_STATE)
    void *d_json = nullptr, *d_scratch = nullptr, *d_docs = nullptr, *d_no = nullptr, *d_absent = nullptr,
         *d_act = nullptr;
    hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
    bool pending_timing = false;
    double k13_ms_sum = 0, k14_ms_sum = 0;
    uint64_t runs = 0;
};

namespace {

using namespace goscan;

struct Cond {
    std::string f[4];  // type, status, reason, message
    int64_t sec = kZeroTimeSec;
    int64_t nsec = 0;
    bool operator==(const Cond& o) const {
        return sec == o.sec && nsec == o.nsec && f[0] == o.f[0] && f[1] == o.f[1] && f[2] == o.f[2] && f[3] == o.f[3];
    }
};

// a Go slice over its backing array: backing.size() == cap, len elements in use
template <class T>
struct GoSlice {
    std::vector<T> backing;
    size_t len = 0;
    bool operator==(const GoSlice& o) const {  // Semantic.DeepEqual: nil == empty
        if (len != o.len) return false;
        for (size_t i = 0; i < len; i++)
            if (!(backing[i] == o.backing[i])) return false;
        return true;
    }
};

// apiextensions/v1 CustomResourceDefinitionNames
struct CrdNames {
    std::string s[4];  // plural, singular, kind, listKind
    GoSlice<std::string> shortn, cat;
    bool operator==(const CrdNames& o) const {
        return s[0] == o.s[0] && s[1] == o.s[1] && s[2] == o.s[2] && s[3] == o.s[3] && shortn == o.shortn &&
               cat == o.cat;
    }
};

struct NegFields {
    std::string rv;
    int64_t gen = 0;
    std::map<std::string, std::string> lab, ann;  // nil and empty compare equal: no flag needed
    GoSlice<Cond> conds;
    // kind GPUDIFF_NEG_KIND_CRD: the rest of CustomResourceDefinitionStatus
    CrdNames names;
    GoSlice<std::string> stored;
};

// ---------------------------------------------------------------- time.Parse(time.RFC3339, s), Go 1.16
int64_t days_from_civil(int64_t y, int64_t m, int64_t d) {
    y -= m <= 2;
    const int64_t era = (y >= 0 ? y : y - 399) / 400;
    const int64_t yoe = y - era * 400;
    const int64_t doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
    const int64_t doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
    return era * 146097 + doe - 719468;
}
bool isdig(const std::string& s, size_t i) { return i < s.size() && s[i] >= '0' && s[i] <= '9'; }
// time.getnum
bool getnum(const std::string& s, size_t& p, bool fixed, int64_t* v) {
    if (!isdig(s, p)) return false;
    if (!isdig(s, p + 1)) {
        if (fixed) return false;
        *v = s[p] - '0';
        p += 1;
        return true;
    }
    *v = (s[p] - '0') * 10 + (s[p + 1] - '0');
    p += 2;
    return true;
}
// time.atoi: optional sign, leadingInt over the rest (all digits, no int64 overflow)
bool go_atoi(const std::string& s, int64_t* v) {
    size_t i = 0;
    bool neg = false;
    if (!s.empty() && (s[0] == '-' || s[0] == '+')) {
        neg = s[0] == '-';
        i = 1;
    }
    uint64_t x = 0;
    for (; i < s.size() && s[i] >= '0' && s[i] <= '9'; i++) {
        if (x > (1ull << 63) / 10) return false;
        x = x * 10 + (uint64_t)(s[i] - '0');
        if (x >= (1ull << 63)) return false;
    }
    if (i != s.size()) return false;
    *v = neg ? -(int64_t)x : (int64_t)x;
    return true;
}
bool parse_rfc3339(const std::string& s, int64_t* sec, int64_t* nsec) {
    if (s.size() < 4 || !isdig(s, 0)) return false;
    int64_t year, month, day, hour, minute, second, ns = 0, off = 0;
    if (!go_atoi(s.substr(0, 4), &year)) return false;
    size_t p = 4;
    if (p >= s.size() || s[p] != '-') return false;
    p++;
    if (!getnum(s, p, true, &month) || month < 1 || month > 12) return false;
    if (p >= s.size() || s[p] != '-') return false;
    p++;
    if (!getnum(s, p, true, &day)) return false;
    if (p >= s.size() || s[p] != 'T') return false;
    p++;
    if (!getnum(s, p, false, &hour) || hour >= 24) return false;
    if (p >= s.size() || s[p] != ':') return false;
    p++;
    if (!getnum(s, p, true, &minute) || minute >= 60) return false;
    if (p >= s.size() || s[p] != ':') return false;
    p++;
    if (!getnum(s, p, true, &second) || second >= 60) return false;
    if (s.size() - p >= 2 && s[p] == '.' && isdig(s, p + 1)) {
        size_t n = 2;
        while (isdig(s, p + n)) n++;
        if (!go_atoi(s.substr(p + 1, n - 1), &ns) || ns < 0 || ns >= 1000000000) return false;
        for (size_t k = n; k < 10; k++) ns *= 10;
        p += n;
    }
    if (p < s.size() && s[p] == 'Z') {
        p++;
    } else {
        if (s.size() - p < 6 || s[p + 3] != ':') return false;
        int64_t hh, mm;
        if (!go_atoi(s.substr(p + 1, 2), &hh) || !go_atoi(s.substr(p + 4, 2), &mm)) return false;
        off = (hh * 60 + mm) * 60;
        if (s[p] == '-') off = -off;
        else if (s[p] != '+') return false;
        p += 6;
    }
    if (p != s.size()) return false;
    const bool leap = year % 4 == 0 && (year % 100 != 0 || year % 400 == 0);
    const int64_t dim = month == 2 ? (leap ? 29 : 28) : (month == 4 || month == 6 || month == 9 || month == 11) ? 30 : 31;
    if (day < 1 || day > dim) return false;
    *sec = days_from_civil(year, month, day) * 86400 + hour * 3600 + minute * 60 + second - off;
    *nsec = ns;
    return true;
}

const char* const kMetaNames[4] = {"resourceVersion", "generation", "labels", "annotations"};
const char* const kCondNames[5] = {"type", "status", "lastTransitionTime", "reason", "message"};
const char* const kCrdStatusNames[3] = {"conditions", "acceptedNames", "storedVersions"};
const char* const kCrdNamesNames[6] = {"plural", "singular", "shortNames", "kind", "listKind", "categories"};

// encoding/json object(): the first exact match among the struct's fields, else the first fold match
int lookup(const char* const* names, int n, const std::string& k) {
    for (int i = 0; i < n; i++)
        if (k == names[i]) return i;
    for (int i = 0; i < n; i++)
        if (field_match(names[i], k)) return i;
    return -1;
}

class NegScanner : public goscan::Scanner {
   public:
    NegScanner(const uint8_t* p, size_t n, uint32_t kind) : goscan::Scanner(p, n), kind_(kind) {}

    bool run(NegFields& f) {
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
    uint32_t kind_;

    bool string_into(std::string& out) {  // null: no-op; else a JSON string
        if (peek_null()) return lit("null");
        if (p_ >= e_ || *p_ != '"') return false;
        return str(&out);
    }
    bool string_map(std::map<std::string, std::string>& m) {
        if (peek_null()) {
            m.clear();  // nil
            return lit("null");
        }
        if (p_ >= e_ || *p_ != '{') return false;
        return members(3, [&](const std::string& k) -> bool {
            if (peek_null()) {
                m[k] = std::string();
                return lit("null");
            }
            if (p_ >= e_ || *p_ != '"') return false;
            return str(&m[k]);
        });
    }
    // encoding/json array(): element i decoded INTO backing[i]; reflect growth
    // (cap + cap/2, at least 4, the first len elements copied); the length
    // becomes the array's; an empty array is an empty non-nil slice, null nil
    template <class T, class F>
    bool slice(GoSlice<T>& sl, F&& elem_into) {
        if (peek_null()) {
            sl.backing.clear();
            sl.len = 0;
            return lit("null");
        }
        if (p_ >= e_ || *p_ != '[') return false;
        p_++;
        ws();
        size_t i = 0;
        if (p_ < e_ && *p_ == ']') {
            p_++;
        } else {
            while (true) {
                if (i >= sl.backing.size()) {
                    const size_t cap = std::max<size_t>(4, sl.backing.size() + sl.backing.size() / 2);
                    std::vector<T> nb(cap);
                    for (size_t q = 0; q < sl.len; q++) nb[q] = sl.backing[q];
                    sl.backing.swap(nb);
                }
                if (i >= sl.len) sl.len = i + 1;
                ws();
                if (!elem_into(sl.backing[i])) return false;
                i++;
                ws();
                if (p_ >= e_) return false;
                const uint8_t x = *p_++;
                if (x == ',') continue;
                if (x == ']') break;
                return false;
            }
        }
        if (i < sl.len) sl.len = i;
        if (i == 0) {
            sl.backing.clear();
            sl.len = 0;
        }
        return true;
    }
    bool strings(GoSlice<std::string>& sl) {
        return slice(sl, [&](std::string& e) { return string_into(e); });
    }
    bool metadata(NegFields& f) {
        if (peek_null()) return lit("null");
        if (p_ >= e_ || *p_ != '{') return false;
        return members(2, [&](const std::string& k) -> bool {
            switch (lookup(kMetaNames, 4, k)) {
                case 0:
                    return string_into(f.rv);
                case 1: {
                    if (peek_null()) return lit("null");
                    const uint8_t c = p_ < e_ ? *p_ : 0;
                    if (c != '-' && (c < '0' || c > '9')) return false;
                    const uint8_t* s;
                    bool is_int;
                    if (!number(&s, &is_int) || !is_int) return false;
                    // strconv.ParseInt(s, 10, 64)
                    const bool neg = *s == '-';
                    uint64_t v = 0;
                    for (const uint8_t* q = s + (neg ? 1 : 0); q < p_; q++) {
                        if (v > (1ull << 63) / 10) return false;
                        v = v * 10 + (uint64_t)(*q - '0');
                        if (v > (1ull << 63)) return false;
                    }
                    if (!neg && v > (uint64_t)INT64_MAX) return false;
                    f.gen = neg ? (int64_t)(0 - v) : (int64_t)v;
                    return true;
                }
                case 2:
                    return string_map(f.lab);
                case 3:
                    return string_map(f.ann);
                default:
                    return skip(2);
            }
        });
    }
    bool cond_into(Cond& c) {
        if (peek_null()) return lit("null");
        if (p_ >= e_ || *p_ != '{') return false;
        return members(4, [&](const std::string& k) -> bool {
            const int fi = lookup(kCondNames, 5, k);
            if (fi < 0) return skip(4);
            if (fi == 2) {  // metav1.Time.UnmarshalJSON
                if (peek_null()) {
                    c.sec = kZeroTimeSec;
                    c.nsec = 0;
                    return lit("null");
                }
                if (p_ >= e_ || *p_ != '"') {
                    skip(4);
                    return false;
                }
                std::string t;
                if (!str(&t)) return false;
                return parse_rfc3339(t, &c.sec, &c.nsec);
            }
            return string_into(c.f[fi == 0 ? 0 : fi == 1 ? 1 : fi == 3 ? 2 : 3]);
        });
    }
    bool conditions(NegFields& f) {
        return slice(f.conds, [&](Cond& c) { return cond_into(c); });
    }
    // CustomResourceDefinitionNames: a struct (null: no-op; a repeated key merges)
    bool names_into(CrdNames& n) {
        if (peek_null()) return lit("null");
        if (p_ >= e_ || *p_ != '{') return false;
        return members(3, [&](const std::string& k) -> bool {
            switch (lookup(kCrdNamesNames, 6, k)) {
                case 0:
                    return string_into(n.s[0]);
                case 1:
                    return string_into(n.s[1]);
                case 2:
                    return strings(n.shortn);
                case 3:
                    return string_into(n.s[2]);
                case 4:
                    return string_into(n.s[3]);
                case 5:
                    return strings(n.cat);
                default:
                    return skip(3);
            }
        });
    }
    bool status(NegFields& f) {
        if (peek_null()) return lit("null");
        if (p_ >= e_ || *p_ != '{') return false;
        if (kind_ == GPUDIFF_NEG_KIND_CRD)
            return members(2, [&](const std::string& k) -> bool {
                switch (lookup(kCrdStatusNames, 3, k)) {
                    case 0:
                        return conditions(f);
                    case 1:
                        return names_into(f.names);
                    case 2:
                        return strings(f.stored);
                    default:
                        return skip(2);
                }
            });
        return members(2, [&](const std::string& k) -> bool {
            if (!field_match("conditions", k)) return skip(2);
            return conditions(f);
        });
    }
};

bool host_fields(const uint8_t* doc, size_t len, uint32_t kind, NegFields& f) {
    NegScanner sc(doc ? doc : (const uint8_t*)"", len, kind);
    return sc.run(f);
}

int32_t classify_host(const uint8_t* a, size_t al, const uint8_t* b, size_t bl, uint32_t kind) {
    NegFields B, A;
    if (!host_fields(b, bl, kind, B)) return GPUDIFF_NEG_DECODE;
    if (!a) return GPUDIFF_NEG_CREATED;
    if (!host_fields(a, al, kind, A)) return GPUDIFF_NEG_DECODE;
    if (A.rv == B.rv) return GPUDIFF_NEG_IGNORE;
    if (A.gen != B.gen) return GPUDIFF_NEG_SPEC;
    if (!(A.conds == B.conds) || !(A.names == B.names) || !(A.stored == B.stored)) return GPUDIFF_NEG_STATUS;
    if (A.ann != B.ann || A.lab == B.lab) return GPUDIFF_NEG_META;
    return GPUDIFF_NEG_IGNORE;
}

void free_nbatch(gpudiff_nbatch* nb) {
    if (!nb) return;
    void* ptrs[] = {nb->d_json, nb->d_scratch, nb->d_docs, nb->d_no, nb->d_absent, nb->d_act};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    for (hipEvent_t& e : nb->ev)
        if (e) (void)hipEventDestroy(e);
    delete nb;
}

void fold_timing(gpudiff_nbatch* nb) {
    float a = 0, b = 0;
    if (hipEventElapsedTime(&a, nb->ev[0], nb->ev[1]) == hipSuccess &&
        hipEventElapsedTime(&b, nb->ev[1], nb->ev[2]) == hipSuccess) {
        nb->k13_ms_sum += a;
        nb->k14_ms_sum += b;
        nb->runs++;
    }
    nb->pending_timing = false;
}

}  // namespace

extern "C" {

int gpudiff_negotiate_pair_host_kind(uint32_t kind, const uint8_t* old_json, size_t old_len, const uint8_t* new_json,
                                     size_t new_len, int32_t* action) {
    if (!action || (!new_json && new_len) || kind > GPUDIFF_NEG_KIND_CRD) return GPUDIFF_E_INVAL;
    *action = classify_host(old_json, old_len, new_json, new_len, kind);
    return GPUDIFF_OK;
}

int gpudiff_negotiate_pair_host(const uint8_t* old_json, size_t old_len, const uint8_t* new_json, size_t new_len,
                                int32_t* action) {
    return gpudiff_negotiate_pair_host_kind(GPUDIFF_NEG_KIND_API, old_json, old_len, new_json, new_len, action);
}

int gpudiff_classify_updates_host_kinds(const uint8_t* kinds, const uint8_t* const* olds, const size_t* old_lens,
                                        const uint8_t* const* news, const size_t* new_lens, size_t n, uint32_t threads,
                                        int32_t* actions) {
    if (n && (!olds || !old_lens || !news || !new_lens || !actions)) return GPUDIFF_E_INVAL;
    for (size_t i = 0; i < n; i++)
        if ((!news[i] && new_lens[i]) || (kinds && kinds[i] > GPUDIFF_NEG_KIND_CRD)) return GPUDIFF_E_INVAL;
    const uint32_t T = (uint32_t)std::max<size_t>(1, std::min<size_t>(threads ? threads : 1, n ? n : 1));
    auto work = [&](uint32_t t) {
        for (size_t i = n * t / T, e = n * (t + 1) / T; i < e; i++)
            actions[i] = classify_host(olds[i], olds[i] ? old_lens[i] : 0, news[i], new_lens[i], kinds ? kinds[i] : 0);
    };
    std::vector<std::thread> th;  // no context here: the caller's thread count, spawned per call
    for (uint32_t t = 1; t < T; t++) th.emplace_back(work, t);
    work(0);
    for (auto& x : th) x.join();
    return GPUDIFF_OK;
}

int gpudiff_classify_updates_host(const uint8_t* const* olds, const size_t* old_lens, const uint8_t* const* news,
                                  const size_t* new_lens, size_t n, uint32_t threads, int32_t* actions) {
    return gpudiff_classify_updates_host_kinds(nullptr, olds, old_lens, news, new_lens, n, threads, actions);
}

int gpudiff_nbatch_create_kinds(gpudiff_ctx* c, const uint8_t* kinds, const uint8_t* const* olds,
                                const size_t* old_lens, const uint8_t* const* news, const size_t* new_lens, size_t n,
                                gpudiff_nbatch** out) {
    if (!c || !out || (n && (!olds || !old_lens || !news || !new_lens)) || n > 0x3FFFFFFFu) return GPUDIFF_E_INVAL;
    *out = nullptr;
    for (size_t i = 0; i < n; i++)
        if ((!news[i] && new_lens[i]) || (kinds && kinds[i] > GPUDIFF_NEG_KIND_CRD)) return GPUDIFF_E_INVAL;
    int rc = set_device(c);
    if (rc) return rc;
    gpudiff_nbatch* nb = new (std::nothrow) gpudiff_nbatch();
    if (!nb) return GPUDIFF_E_NOMEM;
    nb->n = (uint32_t)n;
    nb->olds.assign(olds, olds + n);
    nb->news.assign(news, news + n);
    nb->old_lens.assign(old_lens, old_lens + n);
    nb->new_lens.assign(new_lens, new_lens + n);
    if (kinds) nb->kinds.assign(kinds, kinds + n);
    else nb->kinds.assign(n, (uint8_t)GPUDIFF_NEG_KIND_API);
    nb->docs.resize(2 * n);
    std::vector<uint8_t> absent(n, 0);
    uint64_t jb = 0, sb = 0;
    for (size_t i = 0; i < 2 * n; i++) {
        const size_t p = i / 2;
        const bool is_old = (i & 1) == 0;
        if (is_old && !olds[p]) absent[p] = 1;
        const size_t raw = is_old ? (olds[p] ? old_lens[p] : 0) : new_lens[p];
        const uint32_t l = raw > kTokMaxLen ? kTokMaxLen + 1 : (uint32_t)raw;
        TokDoc& t = nb->docs[i];
        memset(&t, 0, sizeof(t));
        t.json_off = jb;
        t.json_len = l;
        t.scratch_off = sb;
        t.pad[0] = nb->kinds[p];  // K13: which typed status to read
        if (l <= kTokMaxLen) {
            jb = (jb + l + kTokSlack + 15) & ~15ull;
            sb += rollup_scratch_bytes(l);
        }
    }
    jb += kTokSlack;
    nb->json_bytes = jb;
    nb->scratch_bytes = sb;
    auto fail = [&](hipError_t e) {
        free_nbatch(nb);
        return e == hipErrorOutOfMemory ? GPUDIFF_E_CAPACITY : GPUDIFF_E_DEVICE;
    };
    hipError_t e;
    const size_t nd = std::max<size_t>(2 * n, 1);
    if ((e = hipMalloc(&nb->d_json, jb)) != hipSuccess) return fail(e);
    if ((e = hipMalloc(&nb->d_scratch, std::max<uint64_t>(sb, 256))) != hipSuccess) return fail(e);
    if ((e = hipMalloc(&nb->d_docs, nd * sizeof(TokDoc))) != hipSuccess) return fail(e);
    if ((e = hipMalloc(&nb->d_no, nd * sizeof(NegOut))) != hipSuccess) return fail(e);
    if ((e = hipMalloc(&nb->d_absent, std::max<size_t>(n, 1))) != hipSuccess) return fail(e);
    if ((e = hipMalloc(&nb->d_act, std::max<size_t>(n, 1) * 4)) != hipSuccess) return fail(e);
    void* stage = nullptr;
    if ((e = hipHostMalloc(&stage, jb, hipHostMallocDefault)) != hipSuccess) return fail(e);
    memset(stage, 0, jb);
    for (size_t i = 0; i < 2 * n; i++) {
        const size_t p = i / 2;
        const uint8_t* src = (i & 1) ? news[p] : olds[p];
        const TokDoc& t = nb->docs[i];
        if (src && t.json_len && t.json_len <= kTokMaxLen) memcpy((uint8_t*)stage + t.json_off, src, t.json_len);
    }
    e = hipMemcpyAsync(nb->d_json, stage, jb, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess && n)
        e = hipMemcpyAsync(nb->d_docs, nb->docs.data(), 2 * n * sizeof(TokDoc), hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess && n) e = hipMemcpyAsync(nb->d_absent, absent.data(), n, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    (void)hipHostFree(stage);
    if (e != hipSuccess) return fail(e);
    if (c->flags & GPUDIFF_OPT_TIMING)
        for (hipEvent_t& ev : nb->ev)
            if ((e = hipEventCreate(&ev)) != hipSuccess) return fail(e);
    *out = nb;
    return GPUDIFF_OK;
}

int gpudiff_nbatch_run(gpudiff_ctx* c, gpudiff_nbatch* nb) {
    if (!c || !nb) return GPUDIFF_E_INVAL;
    int rc = set_device(c);
    if (rc) return rc;
    if (nb->pending_timing) {
        HIPCHK(hipEventSynchronize(nb->ev[2]));
        fold_timing(nb);
    }
    if (nb->ev[0]) HIPCHK(hipEventRecord(nb->ev[0], c->stream));
    HIPCHK(launch_negotiate_docs(c->stream, (const TokDoc*)nb->d_docs, 2 * nb->n, (const uint8_t*)nb->d_json,
                                 (uint8_t*)nb->d_scratch, (NegOut*)nb->d_no));
    if (nb->ev[1]) HIPCHK(hipEventRecord(nb->ev[1], c->stream));
    HIPCHK(launch_negotiate_pairs(c->stream, (const NegOut*)nb->d_no, (const uint8_t*)nb->d_absent,
                                  (const TokDoc*)nb->d_docs, (const uint8_t*)nb->d_json, nb->n, (int32_t*)nb->d_act));
    if (nb->ev[2]) {
        HIPCHK(hipEventRecord(nb->ev[2], c->stream));
        nb->pending_timing = true;
    }
    nb->ran = true;
    return GPUDIFF_OK;
}

int gpudiff_nbatch_fetch(gpudiff_ctx* c, gpudiff_nbatch* nb, int32_t* actions) {
    if (!c || !nb || (nb->n && !actions)) return GPUDIFF_E_INVAL;
    if (!nb->ran) return GPUDIFF_E_STATE;  // nothing classified yet: d_act holds no actions
    int rc = set_device(c);
    if (rc) return rc;
    const size_t n = nb->n;
    if (n) HIPCHK(hipMemcpyAsync(actions, nb->d_act, n * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (nb->pending_timing) fold_timing(nb);
    std::vector<uint32_t> def;
    for (size_t i = 0; i < n; i++)
        if (actions[i] == kNegDefer) def.push_back((uint32_t)i);
    nb->n_host = def.size();
    if (def.empty()) return GPUDIFF_OK;
    // the host path for the deferred pairs, on the context's encode threads
    const uint32_t T = std::max<uint32_t>(1, std::min<uint32_t>(c->threads, (uint32_t)((def.size() + 63) / 64)));
    auto work = [&](uint32_t t) {
        for (size_t k = t; k < def.size(); k += T) {
            const uint32_t i = def[k];
            actions[i] = classify_host(nb->olds[i], nb->old_lens[i], nb->news[i], nb->new_lens[i], nb->kinds[i]);
        }
    };
    workers(c).run(T, work);
    return GPUDIFF_OK;
}

int gpudiff_nbatch_stats_get(const gpudiff_nbatch* nb, gpudiff_nbatch_stats* st) {
    if (!nb || !st) return GPUDIFF_E_INVAL;
    memset(st, 0, sizeof(*st));
    st->n_pairs = nb->n;
    for (size_t i = 0; i < nb->n; i++) st->json_bytes += (nb->olds[i] ? nb->old_lens[i] : 0) + nb->new_lens[i];
    st->scratch_bytes = nb->scratch_bytes + 2ull * nb->n * sizeof(NegOut);
    st->n_host = nb->n_host;
    st->runs = nb->runs;
    st->k13_ms = nb->runs ? nb->k13_ms_sum / (double)nb->runs : 0.0;
    st->k14_ms = nb->runs ? nb->k14_ms_sum / (double)nb->runs : 0.0;
    return GPUDIFF_OK;
}

void gpudiff_nbatch_free(gpudiff_ctx* c, gpudiff_nbatch* nb) {
    if (!nb) return;
    if (c && c->has_device) {
        (void)hipSetDevice(c->device);
        (void)hipStreamSynchronize(c->stream);
    }
    free_nbatch(nb);
}

int gpudiff_nbatch_create(gpudiff_ctx* c, const uint8_t* const* olds, const size_t* old_lens,
                          const uint8_t* const* news, const size_t* new_lens, size_t n, gpudiff_nbatch** out) {
    return gpudiff_nbatch_create_kinds(c, nullptr, olds, old_lens, news, new_lens, n, out);
}

int gpudiff_classify_updates_kinds(gpudiff_ctx* c, const uint8_t* kinds, const uint8_t* const* olds,
                                   const size_t* old_lens, const uint8_t* const* news, const size_t* new_lens, size_t n,
                                   int32_t* actions) {
    gpudiff_nbatch* nb = nullptr;
    int rc = gpudiff_nbatch_create_kinds(c, kinds, olds, old_lens, news, new_lens, n, &nb);
    if (rc) return rc;
    rc = gpudiff_nbatch_run(c, nb);
    if (!rc) rc = gpudiff_nbatch_fetch(c, nb, actions);
    gpudiff_nbatch_free(c, nb);
    return rc;
}

int gpudiff_classify_updates(gpudiff_ctx* c, const uint8_t* const* olds, const size_t* old_lens,
                             const uint8_t* const* news, const size_t* new_lens, size_t n, int32_t* actions) {
    return gpudiff_classify_updates_kinds(c, nullptr, olds, old_lens, news, new_lens, n, actions);
}

}  // extern "C"
