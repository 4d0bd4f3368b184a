// Go-compatible JSON decoder (see json.h for the rules it reproduces).
#include "json.h"

#include <locale.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <new>

namespace gd {

static constexpr int kMaxDepth = 10000;  // encoding/json scanner maxNestingDepth

// ---------------------------------------------------------------- Arena
Arena::~Arena() {
    for (auto& b : blocks_) free(b.p);
}

void* Arena::alloc(size_t bytes, size_t align) {
    for (;;) {
        if (cur_ < blocks_.size()) {
            Block& b = blocks_[cur_];
            size_t off = (used_ + align - 1) & ~(align - 1);
            if (off + bytes <= b.cap) {
                used_ = off + bytes;
                return b.p + off;
            }
            cur_++;
            used_ = 0;
            continue;
        }
        size_t cap = std::max<size_t>(bytes + align, blocks_.empty() ? (64u << 10) : blocks_.back().cap * 2);
        char* p = (char*)malloc(cap);
        if (!p) throw std::bad_alloc();
        blocks_.push_back({p, cap});
        cur_ = blocks_.size() - 1;
        used_ = 0;
    }
}

void Arena::reset() {
    cur_ = 0;
    used_ = 0;
}

// ---------------------------------------------------------------- helpers
static inline bool is_ws(uint8_t c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }

// utf8.DecodeRune: returns size of a valid sequence, 0 if invalid (Go then
// consumes exactly one byte and emits U+FFFD).
static inline int go_rune_len(const uint8_t* p, const uint8_t* end) {
    uint8_t c0 = p[0];
    int size;
    uint8_t lo = 0x80, hi = 0xBF;
    if (c0 < 0x80) return 1;
    if (c0 >= 0xC2 && c0 <= 0xDF) size = 2;
    else if (c0 == 0xE0) { size = 3; lo = 0xA0; }
    else if ((c0 >= 0xE1 && c0 <= 0xEC) || c0 == 0xEE || c0 == 0xEF) size = 3;
    else if (c0 == 0xED) { size = 3; hi = 0x9F; }
    else if (c0 == 0xF0) { size = 4; lo = 0x90; }
    else if (c0 >= 0xF1 && c0 <= 0xF3) size = 4;
    else if (c0 == 0xF4) { size = 4; hi = 0x8F; }
    else return 0;
    if (end - p < size) return 0;
    if (p[1] < lo || p[1] > hi) return 0;
    for (int k = 2; k < size; k++)
        if (p[k] < 0x80 || p[k] > 0xBF) return 0;
    return size;
}

static inline int hexv(uint8_t c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
}

// getu4: "\uXXXX" at p -> code unit, or -1
static inline int getu4(const uint8_t* p, const uint8_t* end) {
    if (end - p < 6 || p[0] != '\\' || p[1] != 'u') return -1;
    int v = 0;
    for (int k = 2; k < 6; k++) {
        int h = hexv(p[k]);
        if (h < 0) return -1;
        v = (v << 4) | h;
    }
    return v;
}

static inline void put_utf8(std::string& o, uint32_t r) {
    if (r < 0x80) {
        o.push_back((char)r);
    } else if (r < 0x800) {
        o.push_back((char)(0xC0 | (r >> 6)));
        o.push_back((char)(0x80 | (r & 0x3F)));
    } else if (r < 0x10000) {
        o.push_back((char)(0xE0 | (r >> 12)));
        o.push_back((char)(0x80 | ((r >> 6) & 0x3F)));
        o.push_back((char)(0x80 | (r & 0x3F)));
    } else {
        o.push_back((char)(0xF0 | (r >> 18)));
        o.push_back((char)(0x80 | ((r >> 12) & 0x3F)));
        o.push_back((char)(0x80 | ((r >> 6) & 0x3F)));
        o.push_back((char)(0x80 | (r & 0x3F)));
    }
}

// ---------------------------------------------------------------- parser
void JsonParser::ws() {
    while (p_ < end_ && is_ws(*p_)) p_++;
}

bool JsonParser::parse_object(const uint8_t* data, size_t len, Arena& arena, Node* out) {
    p_ = data;
    end_ = data + len;
    arena_ = &arena;
    mstack_.clear();
    istack_.clear();
    ws();
    if (p_ >= end_ || *p_ != '{') return false;
    if (!value(out, 0)) return false;
    ws();
    return p_ == end_;  // trailing data is rejected (conservative)
}

bool JsonParser::value(Node* out, int depth) {
    ws();
    if (p_ >= end_) return false;
    uint8_t c = *p_;
    switch (c) {
        case '{': return object(out, depth + 1);
        case '[': return array(out, depth + 1);
        case '"': {
            out->t = J_STR;
            return string(&out->u.s, &out->n);
        }
        case 't':
            if (end_ - p_ >= 4 && memcmp(p_, "true", 4) == 0) { p_ += 4; out->t = J_TRUE; return true; }
            return false;
        case 'f':
            if (end_ - p_ >= 5 && memcmp(p_, "false", 5) == 0) { p_ += 5; out->t = J_FALSE; return true; }
            return false;
        case 'n':
            if (end_ - p_ >= 4 && memcmp(p_, "null", 4) == 0) { p_ += 4; out->t = J_NULL; return true; }
            return false;
        default:
            if (c == '-' || (c >= '0' && c <= '9')) return number(out);
            return false;
    }
}

bool JsonParser::string(const char** s, uint32_t* n) {
    const uint8_t* q = p_ + 1;
    // fast scan: plain bytes that need no rewriting
    const uint8_t* r = q;
    while (r < end_) {
        uint8_t c = *r;
        if (c == '"' || c == '\\' || c < 0x20) break;
        if (c < 0x80) { r++; continue; }
        int l = go_rune_len(r, end_);
        if (l == 0) break;
        r += l;
    }
    if (r < end_ && *r == '"') {  // zero-copy
        *s = (const char*)q;
        *n = (uint32_t)(r - q);
        p_ = r + 1;
        return true;
    }
    // slow path: decode into tmp_
    tmp_.assign((const char*)q, (size_t)(r - q));
    while (true) {
        if (r >= end_) return false;
        uint8_t c = *r;
        if (c == '"') { r++; break; }
        if (c == '\\') {
            if (end_ - r < 2) return false;
            uint8_t e = r[1];
            switch (e) {
                case '"': tmp_.push_back('"'); r += 2; continue;
                case '\\': tmp_.push_back('\\'); r += 2; continue;
                case '/': tmp_.push_back('/'); r += 2; continue;
                case 'b': tmp_.push_back('\b'); r += 2; continue;
                case 'f': tmp_.push_back('\f'); r += 2; continue;
                case 'n': tmp_.push_back('\n'); r += 2; continue;
                case 'r': tmp_.push_back('\r'); r += 2; continue;
                case 't': tmp_.push_back('\t'); r += 2; continue;
                case 'u': {
                    int rr = getu4(r, end_);
                    if (rr < 0) return false;
                    r += 6;
                    if (rr >= 0xD800 && rr < 0xE000) {
                        int rr1 = getu4(r, end_);
                        if (rr < 0xDC00 && rr1 >= 0xDC00 && rr1 < 0xE000) {
                            uint32_t dec = (((uint32_t)(rr - 0xD800) << 10) | (uint32_t)(rr1 - 0xDC00)) + 0x10000;
                            put_utf8(tmp_, dec);
                            r += 6;
                            continue;
                        }
                        rr = 0xFFFD;
                    }
                    put_utf8(tmp_, (uint32_t)rr);
                    continue;
                }
                default: return false;
            }
        }
        if (c < 0x20) return false;
        if (c < 0x80) { tmp_.push_back((char)c); r++; continue; }
        int l = go_rune_len(r, end_);
        if (l == 0) {
            tmp_.append("\xEF\xBF\xBD", 3);
            r++;
        } else {
            tmp_.append((const char*)r, l);
            r += l;
        }
    }
    char* dst = (char*)arena_->alloc(tmp_.size() ? tmp_.size() : 1, 1);
    memcpy(dst, tmp_.data(), tmp_.size());
    *s = dst;
    *n = (uint32_t)tmp_.size();
    p_ = r;
    return true;
}

bool JsonParser::number(Node* out) {
    const uint8_t* s = p_;
    const uint8_t* q = p_;
    bool neg = false;
    if (*q == '-') { neg = true; q++; }
    if (q >= end_) return false;
    if (*q == '0') {
        q++;
    } else if (*q >= '1' && *q <= '9') {
        while (q < end_ && *q >= '0' && *q <= '9') q++;
    } else {
        return false;
    }
    bool is_int = true;
    if (q < end_ && *q == '.') {
        is_int = false;
        q++;
        if (q >= end_ || *q < '0' || *q > '9') return false;
        while (q < end_ && *q >= '0' && *q <= '9') q++;
    }
    if (q < end_ && (*q == 'e' || *q == 'E')) {
        is_int = false;
        q++;
        if (q < end_ && (*q == '+' || *q == '-')) q++;
        if (q >= end_ || *q < '0' || *q > '9') return false;
        while (q < end_ && *q >= '0' && *q <= '9') q++;
    }
    p_ = q;
    if (is_int) {  // strconv.ParseInt(s, 10, 64)
        const uint8_t* d = s + (neg ? 1 : 0);
        uint64_t lim = neg ? (uint64_t)1 << 63 : ((uint64_t)1 << 63) - 1;
        uint64_t v = 0;
        bool ovf = false;
        for (; d < q; d++) {
            uint64_t dig = (uint64_t)(*d - '0');
            if (v > (lim - dig) / 10) { ovf = true; break; }
            v = v * 10 + dig;
        }
        if (!ovf) {
            out->t = J_INT;
            out->u.i = neg ? (int64_t)(0 - v) : (int64_t)v;
            return true;
        }
    }
    // strconv.ParseFloat(s, 64): correctly rounded; overflow -> error
    static locale_t cloc = newlocale(LC_ALL_MASK, "C", (locale_t)0);
    size_t len = (size_t)(q - s);
    char buf[96];
    double d;
    if (len < sizeof(buf)) {
        memcpy(buf, s, len);
        buf[len] = 0;
        d = strtod_l(buf, nullptr, cloc);
    } else {
        std::string t((const char*)s, len);
        d = strtod_l(t.c_str(), nullptr, cloc);
    }
    if (isinf(d)) return false;
    out->t = J_FLOAT;
    out->u.d = d;
    return true;
}

static inline bool key_eq(const Member& a, const Member& b) {
    return a.klen == b.klen && memcmp(a.k, b.k, a.klen) == 0;
}

bool JsonParser::object(Node* out, int depth) {
    if (depth > kMaxDepth) return false;
    p_++;  // '{'
    size_t base = mstack_.size();
    ws();
    if (p_ < end_ && *p_ == '}') {
        p_++;
        out->t = J_OBJ;
        out->n = 0;
        out->u.mem = nullptr;
        return true;
    }
    while (true) {
        ws();
        if (p_ >= end_ || *p_ != '"') return false;
        Member m;
        if (!string(&m.k, &m.klen)) return false;
        ws();
        if (p_ >= end_ || *p_ != ':') return false;
        p_++;
        if (!value(&m.v, depth)) return false;
        mstack_.push_back(m);
        ws();
        if (p_ >= end_) return false;
        uint8_t c = *p_++;
        if (c == ',') continue;
        if (c == '}') break;
        return false;
    }
    size_t cnt = mstack_.size() - base;
    Member* ms = &mstack_[base];
    // duplicate keys: last one wins
    idx_.clear();
    if (cnt <= 16) {
        for (size_t i = 0; i < cnt; i++) {
            bool dup = false;
            for (size_t j = i + 1; j < cnt; j++)
                if (key_eq(ms[i], ms[j])) { dup = true; break; }
            if (!dup) idx_.push_back((uint32_t)i);
        }
    } else {
        std::vector<uint32_t> ord(cnt);
        for (size_t i = 0; i < cnt; i++) ord[i] = (uint32_t)i;
        std::sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) {
            const Member& x = ms[a];
            const Member& y = ms[b];
            uint32_t l = std::min(x.klen, y.klen);
            int c = memcmp(x.k, y.k, l);
            if (c != 0) return c < 0;
            if (x.klen != y.klen) return x.klen < y.klen;
            return a < b;
        });
        std::vector<uint8_t> keep(cnt, 0);
        for (size_t i = 0; i < cnt; i++) {
            if (i + 1 < cnt && key_eq(ms[ord[i]], ms[ord[i + 1]])) continue;
            keep[ord[i]] = 1;
        }
        for (size_t i = 0; i < cnt; i++)
            if (keep[i]) idx_.push_back((uint32_t)i);
    }
    Member* dst = (Member*)arena_->alloc(sizeof(Member) * idx_.size(), alignof(Member));
    for (size_t i = 0; i < idx_.size(); i++) dst[i] = ms[idx_[i]];
    out->t = J_OBJ;
    out->n = (uint32_t)idx_.size();
    out->u.mem = dst;
    mstack_.resize(base);
    return true;
}

bool JsonParser::array(Node* out, int depth) {
    if (depth > kMaxDepth) return false;
    p_++;  // '['
    size_t base = istack_.size();
    ws();
    if (p_ < end_ && *p_ == ']') {
        p_++;
        out->t = J_ARR;
        out->n = 0;
        out->u.items = nullptr;
        return true;
    }
    while (true) {
        Node v;
        if (!value(&v, depth)) return false;
        istack_.push_back(v);
        ws();
        if (p_ >= end_) return false;
        uint8_t c = *p_++;
        if (c == ',') continue;
        if (c == ']') break;
        return false;
    }
    size_t cnt = istack_.size() - base;
    Node* dst = (Node*)arena_->alloc(sizeof(Node) * cnt, alignof(Node));
    memcpy((void*)dst, (const void*)&istack_[base], sizeof(Node) * cnt);
    out->t = J_ARR;
    out->n = (uint32_t)cnt;
    out->u.items = dst;
    istack_.resize(base);
    return true;
}

}  // namespace gd

namespace gd {

// encoding/json fold.go equalFoldRight (Go 1.16) for an ASCII field name
// against a decoded (valid UTF-8) key: ASCII case folding, plus U+017F (long
// s) for s/S and U+212A (Kelvin sign) for k/K
static bool go_equal_fold_right(const char* name, const char* k, size_t klen) {
    size_t i = 0;
    for (const char* s = name; *s; s++) {
        const uint8_t sb = (uint8_t)*s;
        if (i >= klen) return false;
        const uint8_t tb = (uint8_t)k[i];
        if (tb < 0x80) {
            if (sb != tb) {
                const uint8_t up = sb & 0xDF;
                if (up < 'A' || up > 'Z' || up != (tb & 0xDF)) return false;
            }
            i++;
            continue;
        }
        if ((sb == 's' || sb == 'S') && i + 1 < klen && tb == 0xC5 && (uint8_t)k[i + 1] == 0xBF) {
            i += 2;
        } else if ((sb == 'k' || sb == 'K') && i + 2 < klen && tb == 0xE2 && (uint8_t)k[i + 1] == 0x84 &&
                   (uint8_t)k[i + 2] == 0xAA) {
            i += 3;
        } else {
            return false;
        }
    }
    return i == klen;
}

bool decodes_as_list(const Node& root) {
    if (root.t != J_OBJ) return false;
    for (uint32_t m = 0; m < root.n; m++)
        if (go_equal_fold_right("Items", root.u.mem[m].k, root.u.mem[m].klen)) return true;
    return false;
}

}  // namespace gd
