// Go-compatible JSON decoder for unstructured Kubernetes objects.
//
// Reproduces the value domain the informer hands to the syncer predicates
// (SURVEY.md §8(a) a5, Appendix A.2): encoding/json with UseNumber followed by
// k8s.io/apimachinery/pkg/util/json's convertNumber (int64 if strconv.ParseInt
// accepts the literal, else float64; float overflow is an error), duplicate
// object keys last-wins, strings unescaped with Go's surrogate and invalid
// UTF-8 -> U+FFFD rules, nesting depth limit 10000.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <string>
#include <vector>

namespace gd {

enum JType : uint8_t {
    J_NULL = 0, J_FALSE = 1, J_TRUE = 2, J_INT = 3, J_FLOAT = 4, J_STR = 5,
    J_OBJ = 6,  // object (possibly empty)
    J_ARR = 7,  // array (possibly empty)
};

struct Member;

struct Node {
    uint8_t t = J_NULL;
    uint32_t n = 0;  // string bytes / members / items
    union {
        int64_t i;
        double d;
        const char* s;
        Node* items;
        Member* mem;
    } u{};
};

struct Member {
    const char* k;
    uint32_t klen;
    Node v;
};

// Bump allocator; memory is reused across objects after reset().
class Arena {
   public:
    Arena() = default;
    Arena(const Arena&) = delete;
    Arena& operator=(const Arena&) = delete;
    ~Arena();
    void* alloc(size_t bytes, size_t align = 8);
    void reset();

   private:
    struct Block {
        char* p;
        size_t cap;
    };
    std::vector<Block> blocks_;
    size_t cur_ = 0;   // block index
    size_t used_ = 0;  // bytes used in current block
};

// Parser with reusable scratch; one per thread.
class JsonParser {
   public:
    // Parses one top-level JSON object.  Strings may point into `data`, which
    // must outlive the returned tree.  Returns false on any decode error.
    bool parse_object(const uint8_t* data, size_t len, Arena& arena, Node* out);

   private:
    bool value(Node* out, int depth);
    bool object(Node* out, int depth);
    bool array(Node* out, int depth);
    bool string(const char** s, uint32_t* n);
    bool number(Node* out);
    void ws();

    const uint8_t* p_ = nullptr;
    const uint8_t* end_ = nullptr;
    Arena* arena_ = nullptr;
    std::vector<Member> mstack_;
    std::vector<Node> istack_;
    std::vector<uint32_t> idx_;
    std::string tmp_;
};

// The list probe of apimachinery's unstructuredJSONScheme.decode [3P]: the
// informer's decoder first unmarshals the bytes into struct{ Items
// json.RawMessage }; a top-level key equal to "Items" under encoding/json's
// case folding (any value, null included) makes the object an
// UnstructuredList.  The predicates' type assertions then fail
// (specsyncer.go:18-22, statussyncer.go:16-20): the pair is dirty, like a
// decode error.
bool decodes_as_list(const Node& root);

}  // namespace gd
