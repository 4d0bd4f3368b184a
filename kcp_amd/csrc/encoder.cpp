// Host canonical encoder (see encoder.h and include/gpudiff_format.h).
#include "encoder.h"

#include <string.h>

#include <algorithm>

#include "xxh64.h"

namespace gd {

static const Node* find_member(const Node& obj, const char* key, uint32_t klen) {
    if (obj.t != J_OBJ) return nullptr;
    for (uint32_t i = 0; i < obj.n; i++) {
        const Member& m = obj.u.mem[i];
        if (m.klen == klen && memcmp(m.k, key, klen) == 0) return &m.v;
    }
    return nullptr;
}

static inline void push_key(std::string& p, const char* k, uint32_t n) {
    char hdr[5];
    hdr[0] = 0x01;
    memcpy(hdr + 1, &n, 4);
    p.append(hdr, 5);
    p.append(k, n);
}

static inline void push_idx(std::string& p, uint32_t i) {
    char hdr[5];
    hdr[0] = 0x02;
    memcpy(hdr + 1, &i, 4);
    p.append(hdr, 5);
}

uint64_t chain_hash(const char* p, size_t n, uint64_t seed) {
    uint64_t h = seed;
    size_t i = 0;
    while (i + 5 <= n) {
        uint32_t len = 5;
        if (p[i] == 0x01) {
            uint32_t k;
            memcpy(&k, p + i + 1, 4);
            len += k;
        }
        h = xxh64_host(p + i, len, h);
        i += len;
    }
    return h;
}

const std::string& status_path_bytes() {
    static const std::string s = [] {
        std::string p;
        push_key(p, "status", 6);
        return p;
    }();
    return s;
}

namespace {
struct Flattener {
    FlatObject& o;
    std::string path;
    std::vector<LeafRec>* cur = nullptr;

    explicit Flattener(FlatObject& out) : o(out) {}

    void leaf(const Node& n) {
        LeafRec r;
        r.h = 0;
        r.val = 0;
        r.vptr = nullptr;
        r.vlen = 0;
        uint32_t tag = n.t, len = 0;
        switch (n.t) {
            case J_INT:
                len = 8;
                r.val = (uint64_t)n.u.i;
                break;
            case J_FLOAT: {
                len = 8;
                double d = n.u.d == 0.0 ? 0.0 : n.u.d;  // -0.0 == 0.0 under Go ==
                memcpy(&r.val, &d, 8);
                break;
            }
            case J_STR:
                len = n.n;
                r.vptr = n.u.s;
                r.vlen = n.n;
                if (n.n <= GPUDIFF_INLINE_MAX) memcpy(&r.val, n.u.s, n.n);
                break;
            default:
                break;  // null, bools, empty {} / []: tag only
        }
        r.meta = (len << 3) | tag;
        r.path_off = (uint32_t)o.paths.size();
        r.path_len = (uint32_t)path.size();
        o.paths.append(path);
        cur->push_back(r);
    }

    void walk(const Node& n) {
        if (n.t == J_OBJ && n.n) {
            size_t l = path.size();
            for (uint32_t i = 0; i < n.n; i++) {
                const Member& m = n.u.mem[i];
                push_key(path, m.k, m.klen);
                walk(m.v);
                path.resize(l);
            }
        } else if (n.t == J_ARR && n.n) {
            size_t l = path.size();
            for (uint32_t i = 0; i < n.n; i++) {
                push_idx(path, i);
                walk(n.u.items[i]);
                path.resize(l);
            }
        } else {
            leaf(n);
        }
    }

    // GetLabels / GetAnnotations (NestedStringMap): nil unless metadata.<field>
    // is a map whose values are all strings; nil and empty compare equal, so an
    // empty map contributes no leaves either.
    void string_map(const Node& root, const char* field, uint32_t flen) {
        const Node* md = find_member(root, "metadata", 8);
        if (!md || md->t != J_OBJ) return;
        const Node* m = find_member(*md, field, flen);
        if (!m || m->t != J_OBJ || m->n == 0) return;
        for (uint32_t i = 0; i < m->n; i++)
            if (m->u.mem[i].v.t != J_STR) return;
        path.clear();
        push_key(path, "metadata", 8);
        push_key(path, field, flen);
        size_t l = path.size();
        for (uint32_t i = 0; i < m->n; i++) {
            push_key(path, m->u.mem[i].k, m->u.mem[i].klen);
            leaf(m->u.mem[i].v);
            path.resize(l);
        }
    }
};
}  // namespace

void flatten_object(const Node& root, FlatObject& o) {
    o.clear();
    Flattener f(o);
    // spec region S (specsyncer.go:30-39)
    f.cur = &o.spec;
    for (uint32_t i = 0; i < root.n; i++) {
        const Member& m = root.u.mem[i];
        if ((m.klen == 8 && memcmp(m.k, "metadata", 8) == 0) || (m.klen == 6 && memcmp(m.k, "status", 6) == 0))
            continue;
        if (m.v.t == J_NULL) continue;  // top-level null == missing key
        f.path.clear();
        push_key(f.path, m.k, m.klen);
        f.walk(m.v);
    }
    // regions L and N (specsyncer.go:23,26)
    f.string_map(root, "labels", 6);
    f.string_map(root, "annotations", 11);
    // status region T (statussyncer.go:22-24)
    const Node* st = find_member(root, "status", 6);
    if (st) {
        o.flags |= GPUDIFF_OBJ_HAS_STATUS;
        if (st->t != J_NULL) {
            f.cur = &o.stat;
            f.path = status_path_bytes();
            f.walk(*st);
        }
    }
}

static inline bool path_eq(const FlatObject& a, const LeafRec& x, const FlatObject& b, const LeafRec& y) {
    return x.path_len == y.path_len && memcmp(a.paths.data() + x.path_off, b.paths.data() + y.path_off, x.path_len) == 0;
}

static bool merge_check(const FlatObject& a, const std::vector<LeafRec>& va, const FlatObject& b,
                        const std::vector<LeafRec>& vb) {
    size_t i = 0, j = 0;
    while (i < va.size() && j < vb.size()) {
        if (va[i].h < vb[j].h) i++;
        else if (va[i].h > vb[j].h) j++;
        else {
            if (!path_eq(a, va[i], b, vb[j])) return false;
            i++;
            j++;
        }
    }
    return true;
}

static bool sentinel_check(const FlatObject& o, const std::vector<LeafRec>& v, uint64_t hs) {
    auto it = std::lower_bound(v.begin(), v.end(), hs, [](const LeafRec& r, uint64_t h) { return r.h < h; });
    if (it == v.end() || it->h != hs) return true;
    const std::string& sp = status_path_bytes();
    return it->path_len == sp.size() && memcmp(o.paths.data() + it->path_off, sp.data(), sp.size()) == 0;
}

bool PairEncoder::pair_valid(FlatObject& a, FlatObject& b, uint32_t seed) {
    const uint64_t mask = cfg_.hash_bits >= 64 ? ~0ULL : ((1ULL << cfg_.hash_bits) - 1);
    auto by_h = [](const LeafRec& x, const LeafRec& y) { return x.h < y.h; };
    for (FlatObject* o : {&a, &b})
        for (std::vector<LeafRec>* v : {&o->spec, &o->stat}) {
            for (LeafRec& r : *v) r.h = chain_hash(o->paths.data() + r.path_off, r.path_len, seed) & mask;
            std::sort(v->begin(), v->end(), by_h);
        }
    for (FlatObject* o : {&a, &b})
        for (std::vector<LeafRec>* v : {&o->spec, &o->stat})
            for (size_t i = 1; i < v->size(); i++)
                if ((*v)[i].h == (*v)[i - 1].h) return false;  // paths are unique within an object
    if (!merge_check(a, a.spec, b, b.spec) || !merge_check(a, a.stat, b, b.stat)) return false;
    const std::string& sp = status_path_bytes();
    const uint64_t hs = chain_hash(sp.data(), sp.size(), seed) & mask;
    return sentinel_check(a, a.stat, hs) && sentinel_check(b, b.stat, hs);
}

bool PairEncoder::assign_seed(FlatObject& a, FlatObject& b, uint32_t* seed_out) {
    for (uint32_t seed = 0; seed <= 255; seed++)
        if (pair_valid(a, b, seed)) {
            *seed_out = seed;
            return true;
        }
    return false;
}

static inline void pool_align(std::vector<uint8_t>& pool) {
    size_t n = (pool.size() + GPUDIFF_BLOB_ALIGN - 1) & ~(size_t)(GPUDIFF_BLOB_ALIGN - 1);
    pool.resize(n, 0);
}

void PairEncoder::write_blob(const FlatObject& o, std::vector<uint8_t>& pool, uint64_t* off, uint32_t* sl,
                             uint32_t* sar, uint32_t* tl, uint32_t* tar) {
    pool_align(pool);
    *off = pool.size();
    auto seg = [&](const std::vector<LeafRec>& v, uint32_t* L, uint32_t* AR) {
        const size_t n = v.size();
        uint32_t arena = 0;
        for (const LeafRec& r : v)
            arena += gpudiff_meta_arena(r.meta);
        arena = gpudiff_arena_bytes(arena);
        const size_t head = n * 16;  // vals u64 | keys u32 | metas u32
        const size_t base = pool.size();
        pool.resize(base + head + arena, 0);
        uint8_t* p = pool.data() + base;
        uint8_t* vals = p;
        uint8_t* keys = p + 8 * n;
        uint8_t* metas = p + 12 * n;
        uint8_t* ar = p + head;
        uint32_t aoff = 0;
        for (size_t i = 0; i < n; i++) {
            const LeafRec& r = v[i];
            uint64_t val = r.val;
            if (gpudiff_meta_is_long(r.meta)) {  // head in the record, tail in the arena
                memcpy(&val, r.vptr, GPUDIFF_INLINE_MAX);
                memcpy(ar + aoff, r.vptr + GPUDIFF_INLINE_MAX, r.vlen - GPUDIFF_INLINE_MAX);
                aoff += gpudiff_meta_arena(r.meta);
            }
            const uint32_t k32 = (uint32_t)r.h;  // hashes are masked to <= 32 bits
            memcpy(keys + 4 * i, &k32, 4);
            memcpy(vals + 8 * i, &val, 8);
            memcpy(metas + 4 * i, &r.meta, 4);
        }
        *L = (uint32_t)n;
        *AR = arena;
        leaves_written += n;
    };
    seg(o.spec, sl, sar);
    seg(o.stat, tl, tar);
    pool_align(pool);  // the body's zero pad (gpudiff_blob_body)
}

void PairEncoder::encode_flat(FlatObject* fa, FlatObject* fb, uint32_t pair_id, uint32_t cluster_id,
                              std::vector<uint8_t>& pool, gpudiff_pair_row& row) {
    memset(&row, 0, sizeof(row));
    row.pair_id = pair_id;
    row.cluster_id = cluster_id;
    uint32_t seed = 0;
    if (!fa || !fb || !assign_seed(*fa, *fb, &seed)) {
        decode_errors++;
        pool_align(pool);
        row.off_a = row.off_b = pool.size();
        row.flags_a = row.flags_b = GPUDIFF_OBJ_DECODE_ERR;
        return;
    }
    if (seed) reseeded++;
    write_blob(*fa, pool, &row.off_a, &row.spec_l_a, &row.spec_ar_a, &row.stat_l_a, &row.stat_ar_a);
    write_blob(*fb, pool, &row.off_b, &row.spec_l_b, &row.spec_ar_b, &row.stat_l_b, &row.stat_ar_b);
    row.flags_a = fa->flags | (seed << GPUDIFF_OBJ_SEED_SHIFT);
    row.flags_b = fb->flags | (seed << GPUDIFF_OBJ_SEED_SHIFT);
}

void PairEncoder::encode_nodes(const Node* a, const Node* b, uint32_t pair_id, uint32_t cluster_id,
                               std::vector<uint8_t>& pool, gpudiff_pair_row& row) {
    FlatObject* fa = nullptr;
    FlatObject* fb = nullptr;
    if (a && b) {
        flatten_object(*a, flat_a);
        flatten_object(*b, flat_b);
        fa = &flat_a;
        fb = &flat_b;
    }
    encode_flat(fa, fb, pair_id, cluster_id, pool, row);
}

void PairEncoder::encode_json(const uint8_t* a, size_t alen, const uint8_t* b, size_t blen, uint32_t pair_id,
                              uint32_t cluster_id, std::vector<uint8_t>& pool, gpudiff_pair_row& row) {
    arena_a.reset();
    arena_b.reset();
    Node na, nb;
    bool oka = a && parser.parse_object(a, alen, arena_a, &na) && !decodes_as_list(na);
    bool okb = oka && b && parser.parse_object(b, blen, arena_b, &nb) && !decodes_as_list(nb);
    encode_nodes(oka ? &na : nullptr, okb ? &nb : nullptr, pair_id, cluster_id, pool, row);
}

// ------------------------------------------------------------------ object store helpers

bool PairEncoder::flatten_json(const uint8_t* json, size_t len, Arena& arena, FlatObject& o) {
    arena.reset();
    Node n;
    if (!json || !parser.parse_object(json, len, arena, &n) || decodes_as_list(n)) return false;
    flatten_object(n, o);
    return true;
}

bool PairEncoder::path_table(FlatObject& o, uint32_t seed) {
    // every non-root prefix of every region leaf's path: (hash, parent hash,
    // component, the prefix itself to tell a shared node from a collision)
    // (prefix = paths[poff, pend); key bytes at paths[koff, koff + klen))
    using PN = TabNode;
    const uint64_t mask = cfg_.hash_bits >= 64 ? ~0ULL : ((1ULL << cfg_.hash_bits) - 1);
    const uint64_t root = (uint64_t)seed & mask;
    std::vector<PN>& v = tab_scratch_;
    v.clear();
    const char* P = o.paths.data();
    for (const std::vector<LeafRec>* lv : {&o.spec, &o.stat})
        for (const LeafRec& r : *lv) {
            uint64_t hp = seed;
            uint32_t i = 0;
            while (i + 5 <= r.path_len) {
                const char* c = P + r.path_off + i;
                uint32_t x;
                memcpy(&x, c + 1, 4);
                const bool key = c[0] == 0x01;
                const uint32_t len = key ? 5u + x : 5u;
                const uint64_t h = xxh64_host(c, len, hp);
                PN n;
                n.h = h & mask;
                n.ph = hp & mask;
                n.c = key ? ((uint64_t)x << 32) : (GPUDIFF_TAB_INDEX | x);
                n.poff = r.path_off;
                n.pend = r.path_off + i + len;
                n.koff = r.path_off + i + 5;
                if (n.h == root) {
                    o.tab.n = GPUDIFF_TAB_NONE;
                    o.tab.data.clear();
                    return false;
                }
                v.push_back(n);
                hp = h;
                i += len;
            }
        }
    std::sort(v.begin(), v.end(), [](const PN& a, const PN& b) { return a.h < b.h; });
    size_t u = 0, kb = 0;
    for (size_t i = 0; i < v.size(); i++) {
        if (u && v[u - 1].h == v[i].h) {
            const PN& a = v[u - 1];
            const PN& b = v[i];
            if (a.pend - a.poff != b.pend - b.poff || memcmp(P + a.poff, P + b.poff, a.pend - a.poff) != 0) {
                o.tab.n = GPUDIFF_TAB_NONE;  // two nodes, one hash
                o.tab.data.clear();
                return false;
            }
            continue;
        }
        v[u++] = v[i];
        if (!(v[i].c & GPUDIFF_TAB_INDEX)) kb += v[i].c >> 32;
    }
    v.resize(u);
    const uint32_t n = (uint32_t)u;
    PathTable& t = o.tab;
    t.n = n;
    t.data.assign(gpudiff_tab_bytes(n, kb), 0);
    uint64_t* hs = (uint64_t*)t.data.data();
    uint64_t* phs = hs + n;
    uint64_t* cs = phs + n;
    uint8_t* keys = t.data.data() + 24ull * n;
    uint32_t ko = 0;
    for (uint32_t i = 0; i < n; i++) {
        hs[i] = v[i].h;
        phs[i] = v[i].ph;
        if (v[i].c & GPUDIFF_TAB_INDEX) {
            cs[i] = v[i].c;
        } else {
            const uint32_t kl = (uint32_t)(v[i].c >> 32);
            cs[i] = ((uint64_t)kl << 32) | ko;
            memcpy(keys + ko, P + v[i].koff, kl);
            ko += kl;
        }
    }
    return true;
}

bool tab_agree(const TabView& a, const TabView& b) {
    if (a.n == GPUDIFF_TAB_NONE || b.n == GPUDIFF_TAB_NONE) return false;
    uint32_t i = 0, j = 0;
    while (i < a.n && j < b.n) {
        if (a.hs[i] < b.hs[j]) {
            i++;
        } else if (a.hs[i] > b.hs[j]) {
            j++;
        } else {
            if (a.phs[i] != b.phs[j]) return false;
            const uint64_t ca = a.cs[i], cb = b.cs[j];
            if ((ca & GPUDIFF_TAB_INDEX) || (cb & GPUDIFF_TAB_INDEX)) {
                if (ca != cb) return false;
            } else {
                const uint32_t l = (uint32_t)(ca >> 32);
                if (l != (uint32_t)(cb >> 32) || memcmp(a.keys + (uint32_t)ca, b.keys + (uint32_t)cb, l) != 0)
                    return false;
            }
            i++;
            j++;
        }
    }
    return true;
}

bool PairEncoder::hash_single(FlatObject& o, uint32_t seed) {
    return hash_leaves(o, seed) && path_table(o, seed);
}

bool PairEncoder::first_seed(FlatObject& o, uint32_t* seed) {
    for (uint32_t s = 0; s <= 255; s++)
        if (hash_leaves(o, s)) {
            *seed = s;
            (void)path_table(o, s);
            return true;
        }
    return false;
}

bool PairEncoder::store_seed(FlatObject& o, uint32_t* seed) {
    for (uint32_t s = 0; s <= 255; s++)
        if (hash_single(o, s)) {
            *seed = s;
            return true;
        }
    return first_seed(o, seed);
}

bool PairEncoder::hash_leaves(FlatObject& o, uint32_t seed) {
    const uint64_t mask = cfg_.hash_bits >= 64 ? ~0ULL : ((1ULL << cfg_.hash_bits) - 1);
    auto by_h = [](const LeafRec& x, const LeafRec& y) { return x.h < y.h; };
    for (std::vector<LeafRec>* v : {&o.spec, &o.stat}) {
        for (LeafRec& r : *v) r.h = chain_hash(o.paths.data() + r.path_off, r.path_len, seed) & mask;
        std::sort(v->begin(), v->end(), by_h);
        for (size_t i = 1; i < v->size(); i++)
            if ((*v)[i].h == (*v)[i - 1].h) return false;
    }
    const std::string& sp = status_path_bytes();
    return sentinel_check(o, o.stat, chain_hash(sp.data(), sp.size(), seed) & mask);
}

bool PairEncoder::pair_seed(FlatObject& a, FlatObject& b, uint32_t* seed) {
    if (!assign_seed(a, b, seed)) return false;
    (void)path_table(b, *seed);  // b.tab: valid, or GPUDIFF_TAB_NONE (its slot then goes through old_json)
    return true;
}

void PairEncoder::write_object(const FlatObject& o, std::vector<uint8_t>& pool, uint64_t* off, uint32_t* sl,
                               uint32_t* sar, uint32_t* tl, uint32_t* tar) {
    write_blob(o, pool, off, sl, sar, tl, tar);
}

void PairEncoder::write_object_tab(const FlatObject& o, std::vector<uint8_t>& pool, uint64_t* off, uint32_t* sl,
                                   uint32_t* sar, uint32_t* tl, uint32_t* tar, uint32_t* bytes) {
    write_blob(o, pool, off, sl, sar, tl, tar);
    pool.insert(pool.end(), o.tab.data.begin(), o.tab.data.end());
    *bytes = (uint32_t)(pool.size() - *off);
}

std::string render_path(const char* p, size_t n) {
    std::string s;
    size_t i = 0;
    while (i + 5 <= n) {
        uint8_t k = (uint8_t)p[i];
        uint32_t v;
        memcpy(&v, p + i + 1, 4);
        i += 5;
        if (k == 0x01) {
            if (!s.empty()) s.push_back('.');
            s.append(p + i, v);
            i += v;
        } else {
            s += "[" + std::to_string(v) + "]";
        }
    }
    return s;
}

}  // namespace gd
