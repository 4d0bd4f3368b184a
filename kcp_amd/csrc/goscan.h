// Go 1.16 encoding/json scanning primitives shared by the host paths that
// restate a typed decode (rollup.cpp, negotiate.cpp): the scanner grammar,
// escapes (invalid UTF-8 -> U+FFFD), control characters, nesting depth 10000,
// and struct field lookup (exact, else case-insensitive with Go's fold rules).
#pragma once
#include <stdint.h>
#include <string.h>

#include <string>

namespace gd {
namespace goscan {

constexpr int kMaxDepth = 10000;  // encoding/json scanner maxNestingDepth

inline int rune_len(const uint8_t* p, const uint8_t* end) {  // utf8.DecodeRune size, 0 = invalid
    const uint8_t c0 = p[0];
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
    if (end - p < size || p[1] < lo || p[1] > hi) return 0;
    for (int k = 2; k < size; k++)
        if (p[k] < 0x80 || p[k] > 0xBF) return 0;
    return size;
}

inline int hexv(uint8_t c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
}

inline void put_utf8(std::string& o, uint32_t r) {
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

// encoding/json fold.go for an ASCII-letter field name: ASCII case folding;
// where the name holds s/S or k/K (equalFoldRight) a key rune U+017F / U+212A
// matches it too
inline bool field_match(const char* name, const std::string& key) {
    const uint8_t* t = (const uint8_t*)key.data();
    const uint8_t* te = t + key.size();
    for (const char* s = name; *s; s++) {
        if (t == te) return false;
        const uint8_t sb = (uint8_t)*s;
        if (*t < 0x80) {
            if (*t != sb && ((*t ^ sb) != 0x20 || (uint8_t)((sb | 0x20) - 'a') > 25)) return false;
            t++;
            continue;
        }
        if ((sb | 0x20) == 's' && te - t >= 2 && t[0] == 0xC5 && t[1] == 0xBF) {
            t += 2;
        } else if ((sb | 0x20) == 'k' && te - t >= 3 && t[0] == 0xE2 && t[1] == 0x84 && t[2] == 0xAA) {
            t += 3;
        } else {
            return false;
        }
    }
    return t == te;
}

class Scanner {
   public:
    Scanner(const uint8_t* p, size_t n) : p_(p), e_(p + n) {}

   protected:
    const uint8_t* p_;
    const uint8_t* e_;
    std::string key_;

    void ws() {
        while (p_ < e_ && (*p_ == ' ' || *p_ == '\t' || *p_ == '\n' || *p_ == '\r')) p_++;
    }
    bool lit(const char* w) {
        const size_t l = strlen(w);
        if ((size_t)(e_ - p_) < l || memcmp(p_, w, l) != 0) return false;
        p_ += l;
        return true;
    }
    bool peek_null() {
        ws();
        return e_ - p_ >= 4 && memcmp(p_, "null", 4) == 0;
    }
    // a string at p_ (Go unescaping, invalid UTF-8 -> U+FFFD); out may be null
    bool str(std::string* out) {
        if (p_ >= e_ || *p_ != '"') return false;
        p_++;
        if (out) out->clear();
        while (true) {
            if (p_ >= e_) return false;
            const uint8_t c = *p_;
            if (c == '"') {
                p_++;
                return true;
            }
            if (c == '\\') {
                if (e_ - p_ < 2) return false;
                const uint8_t x = p_[1];
                const char* simple = x == '"' ? "\"" : x == '\\' ? "\\" : x == '/' ? "/" : x == 'b' ? "\b"
                                   : x == 'f' ? "\f" : x == 'n' ? "\n" : x == 'r' ? "\r" : x == 't' ? "\t" : nullptr;
                if (simple) {
                    if (out) out->push_back(*simple);
                    p_ += 2;
                    continue;
                }
                if (x != 'u') return false;
                int r = u4(p_);
                if (r < 0) return false;
                p_ += 6;
                if (r >= 0xD800 && r < 0xE000) {
                    const int r1 = (e_ - p_ >= 6 && p_[0] == '\\' && p_[1] == 'u') ? u4(p_) : -1;
                    if (r < 0xDC00 && r1 >= 0xDC00 && r1 < 0xE000) {
                        if (out) put_utf8(*out, (((uint32_t)(r - 0xD800) << 10) | (uint32_t)(r1 - 0xDC00)) + 0x10000);
                        p_ += 6;
                        continue;
                    }
                    r = 0xFFFD;
                }
                if (out) put_utf8(*out, (uint32_t)r);
                continue;
            }
            if (c < 0x20) return false;
            if (c < 0x80) {
                if (out) out->push_back((char)c);
                p_++;
                continue;
            }
            const int l = rune_len(p_, e_);
            if (!l) {
                if (out) out->append("\xEF\xBF\xBD", 3);
                p_++;
            } else {
                if (out) out->append((const char*)p_, l);
                p_ += l;
            }
        }
    }
    int u4(const uint8_t* q) {
        if (e_ - q < 6) return -1;
        int v = 0;
        for (int k = 2; k < 6; k++) {
            const int h = hexv(q[k]);
            if (h < 0) return -1;
            v = (v << 4) | h;
        }
        return v;
    }
    // number literal (Go's grammar) -> [s, p_)
    bool number(const uint8_t** s, bool* is_int) {
        *s = p_;
        *is_int = true;
        if (p_ < e_ && *p_ == '-') p_++;
        if (p_ >= e_) return false;
        if (*p_ == '0') {
            p_++;
        } else if (*p_ >= '1' && *p_ <= '9') {
            while (p_ < e_ && *p_ >= '0' && *p_ <= '9') p_++;
        } else {
            return false;
        }
        if (p_ < e_ && *p_ == '.') {
            *is_int = false;
            p_++;
            if (p_ >= e_ || *p_ < '0' || *p_ > '9') return false;
            while (p_ < e_ && *p_ >= '0' && *p_ <= '9') p_++;
        }
        if (p_ < e_ && (*p_ == 'e' || *p_ == 'E')) {
            *is_int = false;
            p_++;
            if (p_ < e_ && (*p_ == '+' || *p_ == '-')) p_++;
            if (p_ >= e_ || *p_ < '0' || *p_ > '9') return false;
            while (p_ < e_ && *p_ >= '0' && *p_ <= '9') p_++;
        }
        return true;
    }
    // members of the object at p_ ('{'); on_member(key) consumes the value
    template <class F>
    bool members(int depth, F on_member) {
        if (depth > kMaxDepth) return false;
        p_++;
        ws();
        if (p_ < e_ && *p_ == '}') {
            p_++;
            return true;
        }
        while (true) {
            ws();
            std::string k;
            if (!str(&k)) return false;
            ws();
            if (p_ >= e_ || *p_ != ':') return false;
            p_++;
            ws();
            if (!on_member(k)) return false;
            ws();
            if (p_ >= e_) return false;
            const uint8_t c = *p_++;
            if (c == ',') continue;
            if (c == '}') return true;
            return false;
        }
    }
    // any value (syntax only); depth = nesting of the value's container
    bool skip(int depth) {
        ws();
        if (p_ >= e_) return false;
        const uint8_t c = *p_;
        if (c == '{') return members(depth + 1, [&](const std::string&) { return skip(depth + 1); });
        if (c == '[') {
            if (depth + 1 > kMaxDepth) return false;
            p_++;
            ws();
            if (p_ < e_ && *p_ == ']') {
                p_++;
                return true;
            }
            while (true) {
                if (!skip(depth + 1)) return false;
                ws();
                if (p_ >= e_) return false;
                const uint8_t x = *p_++;
                if (x == ',') continue;
                if (x == ']') return true;
                return false;
            }
        }
        if (c == '"') return str(nullptr);
        if (c == 't') return lit("true");
        if (c == 'f') return lit("false");
        if (c == 'n') return lit("null");
        const uint8_t* s;
        bool is_int;
        return number(&s, &is_int);
    }
};

}  // namespace goscan
}  // namespace gd
