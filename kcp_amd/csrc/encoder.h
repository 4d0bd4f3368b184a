// Host canonical encoder: decoded unstructured object -> sorted CSR leaf
// segments (include/gpudiff_format.h).
//
// The leaf set it extracts is exactly what the reference predicates compare:
//   spec region   = top-level keys except metadata/status with top-level
//                   nulls dropped (specsyncer.go:30-39; a missing key reads as
//                   nil, so `k: null` == absent), plus canonical labels and
//                   annotations (GetLabels/GetAnnotations at specsyncer.go:23,26:
//                   NestedStringMap, nil unless every value is a string)
//   status region = the "status" subtree (statussyncer.go:22-24), a top-level
//                   `status: null` contributes no leaves but sets HAS_STATUS.
// Leaves are scalars and empty containers; paths are encoded component by
// component (0x01 u32le(len) key | 0x02 u32le(index)) and hashed with the
// chained XXH64 below.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/gpudiff.h"
#include "json.h"

namespace gd {

struct LeafRec {
    uint64_t h;
    uint64_t val;
    uint32_t meta;
    uint32_t path_off;
    uint32_t path_len;
    uint32_t vlen;
    const char* vptr;
};

// Object store: a blob's path table (include/gpudiff_format.h), serialized as
// the device trailer: hs[n] | phs[n] | cs[n] | key bytes | pad to a multiple of 16.
struct PathTable {
    std::vector<uint8_t> data;
    uint32_t n = 0;  // GPUDIFF_TAB_NONE: no valid table (data empty)
    void clear() {
        data.clear();
        n = 0;
    }
};

// read-only view of a table (host memory: a PathTable or a trailer copied back)
struct TabView {
    const uint64_t* hs = nullptr;
    const uint64_t* phs = nullptr;
    const uint64_t* cs = nullptr;
    const uint8_t* keys = nullptr;
    uint32_t n = 0;
};
inline TabView tab_view(const uint8_t* trailer, uint32_t n) {
    TabView v;
    if (n == GPUDIFF_TAB_NONE) {
        v.n = n;
        return v;
    }
    v.hs = (const uint64_t*)trailer;
    v.phs = v.hs + n;
    v.cs = v.phs + n;
    v.keys = trailer + 24ull * n;
    v.n = n;
    return v;
}
inline TabView tab_view(const PathTable& t) { return tab_view(t.data.data(), t.n); }
// true iff both tables are valid and every path hash both hold has the same
// parent hash and the same last component in each (then the shared hashes
// name the same paths)
bool tab_agree(const TabView& old, const TabView& nw);

struct FlatObject {
    std::vector<LeafRec> spec, stat;
    std::string paths;   // concatenated path bytes
    uint32_t flags = 0;  // GPUDIFF_OBJ_*
    PathTable tab;       // object store: built by hash_single / pair_seed
    void clear() {
        spec.clear();
        stat.clear();
        paths.clear();
        tab.clear();
        flags = 0;
    }
};

struct EncodeConfig {
    uint32_t hash_bits = GPUDIFF_PATH_HASH_BITS;  // <= 32: segments keep 32-bit keys
};

// Flattens a decoded top-level object into its spec/status leaves.
void flatten_object(const Node& root, FlatObject& out);

class PairEncoder {
   public:
    explicit PairEncoder(const EncodeConfig& cfg) : cfg_(cfg) {}
    // Encodes one pair from JSON bytes; appends blob A then blob B to pool.
    void encode_json(const uint8_t* a, size_t alen, const uint8_t* b, size_t blen, uint32_t pair_id,
                     uint32_t cluster_id, std::vector<uint8_t>& pool, gpudiff_pair_row& row);
    // Encodes one pair from decoded trees (nullptr = decode error).
    void encode_nodes(const Node* a, const Node* b, uint32_t pair_id, uint32_t cluster_id,
                      std::vector<uint8_t>& pool, gpudiff_pair_row& row);
    // Assigns the pair seed, sorts, and writes both blobs.
    void encode_flat(FlatObject* fa, FlatObject* fb, uint32_t pair_id, uint32_t cluster_id,
                     std::vector<uint8_t>& pool, gpudiff_pair_row& row);
    // ---- object store (single objects against a resident version)
    // Parses and flattens one object into `o` (false on a decode error).
    bool flatten_json(const uint8_t* json, size_t len, Arena& arena, FlatObject& o);
    // Path hashes under `seed` (sorted) plus the path table; true iff the
    // hashes are unique within the object, the status sentinel is unambiguous
    // and the table is valid (its node hashes unique and none the root's).
    bool hash_single(FlatObject& o, uint32_t seed);
    // The leaf part of hash_single (the seed the pair ({}, o) takes); o.tab
    // is left alone.
    bool hash_leaves(FlatObject& o, uint32_t seed);
    // Smallest seed for o diffed against the empty object (as encode_json
    // picks it), with o.tab built (GPUDIFF_TAB_NONE if not valid there).
    bool first_seed(FlatObject& o, uint32_t* seed);
    // Seed o is stored with when its event is reported conservatively: the
    // smallest with a valid table, else the smallest leaf-valid one.
    bool store_seed(FlatObject& o, uint32_t* seed);
    // Smallest seed valid for the pair (a, b) as encode_json would pick it;
    // fills b.tab (GPUDIFF_TAB_NONE if b's table is not valid under that
    // seed).  False if no seed <= 255 works.
    bool pair_seed(FlatObject& a, FlatObject& b, uint32_t* seed);
    // o.tab for the region leaves' paths under `seed` (false, and n =
    // GPUDIFF_TAB_NONE: not valid)
    bool path_table(FlatObject& o, uint32_t seed);
    // Appends o's blob (16-B aligned) and reports its layout.
    void write_object(const FlatObject& o, std::vector<uint8_t>& pool, uint64_t* off, uint32_t* sl, uint32_t* sar,
                      uint32_t* tl, uint32_t* tar);
    // Device object store format: the blob followed by its path table (o.tab)
    // -- the bytes kernel K0 writes for the same object.
    void write_object_tab(const FlatObject& o, std::vector<uint8_t>& pool, uint64_t* off, uint32_t* sl,
                          uint32_t* sar, uint32_t* tl, uint32_t* tar, uint32_t* bytes);

    uint64_t leaves_written = 0;
    uint64_t reseeded = 0;
    uint64_t decode_errors = 0;

    JsonParser parser;
    Arena arena_a, arena_b;
    FlatObject flat_a, flat_b;

   private:
    bool assign_seed(FlatObject& a, FlatObject& b, uint32_t* seed);
    bool pair_valid(FlatObject& a, FlatObject& b, uint32_t seed);
    void write_blob(const FlatObject& o, std::vector<uint8_t>& pool, uint64_t* off, uint32_t* sl,
                    uint32_t* sar, uint32_t* tl, uint32_t* tar);
    EncodeConfig cfg_;
    struct TabNode {  // path_table's working set: one per path prefix
        uint64_t h, ph, c;
        uint32_t pend, koff, poff;
    };
    std::vector<TabNode> tab_scratch_;
};

// Chained path hash over encoded path bytes: h(empty) = seed,
// h(p + c) = XXH64(enc(c), seed = h(p)).  A child's hash depends only on its
// parent's hash and its own component, so the device tokenizer hashes a tree
// level by level (kernels K0*).  Masking to hash_bits happens on the result.
uint64_t chain_hash(const char* p, size_t n, uint64_t seed);

// Status-region sentinel path bytes: [Key "status"]
const std::string& status_path_bytes();

// Renders encoded path bytes as "a.b[3].c".
std::string render_path(const char* p, size_t n);

}  // namespace gd
