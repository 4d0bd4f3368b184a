// Seeded synthetic populations for bench.py / tests (include/gpudiff_synth.h).
// Builds decoded trees directly (no JSON text on the hot generation path) and
// encodes them with the product encoder; JSON text is produced on demand for
// the CPU-baseline / parity samples.
#include "../../include/gpudiff_synth.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <memory>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "encoder.h"
#include "json.h"

using namespace gd;

namespace {

enum Kind : uint32_t { K_CM = 0, K_SECRET = 1, K_DEPLOY = 2, K_CRD = 3, K_DEEP = 4 };

inline uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

struct Rng {
    uint64_t s;
    explicit Rng(uint64_t seed) : s(seed) {}
    uint64_t next() {
        s += 0x9E3779B97F4A7C15ULL;
        uint64_t z = s;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
        return z ^ (z >> 31);
    }
    uint32_t range(uint32_t lo, uint32_t hi) { return lo + (uint32_t)(next() % (uint64_t)(hi - lo + 1)); }
    double unit() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
};

const char kAlnum[] = "abcdefghijklmnopqrstuvwxyz0123456789";
const char kText[] = "abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789 _-./:";
const char kB64[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";

// Mutation directive applied while generating B.
struct Directive {
    enum Op : uint32_t { NONE = 0, LEAF_EDIT, LIST_INSERT, LIST_DELETE, LABEL_EDIT, ANNOT_EDIT, KEY_ADD, KEY_DEL,
                         COND_REVERSE, INT_RETYPE };
    Op op = NONE;
    bool status = false;    // target region
    uint64_t target = 0;    // index among the counted targets of that kind/region
};

// Tree builder over an Arena; counts editable leaves / lists per region so a
// directive can address "the k-th leaf of the spec region".
struct Gen {
    Arena& ar;
    Rng rng;
    Directive dir;
    bool in_status = false;
    bool no_count = false;  // metadata lists are not mutation targets
    uint64_t leaf_ctr[2] = {0, 0}, list_ctr[2] = {0, 0};
    bool applied = false;
    std::vector<Member> mtmp;
    std::vector<Node> itmp;

    Gen(Arena& a, uint64_t seed, const Directive& d) : ar(a), rng(seed), dir(d) {}

    Node str(const char* s, uint32_t n) {
        Node x;
        x.t = J_STR;
        char* p = (char*)ar.alloc(n ? n : 1, 1);
        memcpy(p, s, n);
        x.u.s = p;
        x.n = n;
        return x;
    }
    Node cstr(const char* s) { return str(s, (uint32_t)strlen(s)); }
    Node rstr(uint32_t lo, uint32_t hi, const char* alpha, uint32_t alen) {
        uint32_t n = rng.range(lo, hi);
        Node x;
        x.t = J_STR;
        char* p = (char*)ar.alloc(n + 1, 1);  // +1: room for an edit suffix
        for (uint32_t i = 0; i < n; i++) p[i] = alpha[rng.next() % alen];
        x.u.s = p;
        x.n = n;
        return x;
    }
    Node i64(int64_t v) {
        Node x;
        x.t = J_INT;
        x.u.i = v;
        return x;
    }
    Node f64(double v) {
        Node x;
        x.t = J_FLOAT;
        x.u.d = v;
        return x;
    }
    Node boolean(bool b) {
        Node x;
        x.t = b ? J_TRUE : J_FALSE;
        return x;
    }
    Node null() { return Node(); }

    // editable leaf: applies LEAF_EDIT / INT_RETYPE when addressed
    Node leaf(Node v) {
        const int r = in_status ? 1 : 0;
        const uint64_t k = leaf_ctr[r]++;
        if (dir.op == Directive::LEAF_EDIT && dir.status == in_status && dir.target == k) {
            applied = true;
            switch (v.t) {
                case J_STR: {
                    char* p = (char*)ar.alloc(v.n + 1, 1);
                    memcpy(p, v.u.s, v.n);
                    p[v.n] = '~';
                    v.u.s = p;
                    v.n += 1;
                    break;
                }
                case J_INT: v.t = J_FLOAT; v.u.d = (double)v.u.i + 0.5; break;
                case J_FLOAT: v.u.d += 1.0; break;
                case J_TRUE: v.t = J_FALSE; break;
                case J_FALSE: v.t = J_TRUE; break;
                default: v = cstr("changed"); break;
            }
        }
        return v;
    }

    struct ObjB {
        Gen& g;
        size_t base;
        explicit ObjB(Gen& gg) : g(gg), base(gg.mtmp.size()) {}
        void add(const char* k, Node v) {
            Member m;
            uint32_t n = (uint32_t)strlen(k);
            char* p = (char*)g.ar.alloc(n ? n : 1, 1);
            memcpy(p, k, n);
            m.k = p;
            m.klen = n;
            m.v = v;
            g.mtmp.push_back(m);
        }
        void addk(Node key, Node v) {
            for (size_t i = base; i < g.mtmp.size(); i++)  // random keys: keep them unique
                if (g.mtmp[i].klen == key.n && memcmp(g.mtmp[i].k, key.u.s, key.n) == 0) return;
            Member m;
            m.k = key.u.s;
            m.klen = key.n;
            m.v = v;
            g.mtmp.push_back(m);
        }
        Node done() {
            size_t cnt = g.mtmp.size() - base;
            Node x;
            x.t = J_OBJ;
            x.n = (uint32_t)cnt;
            Member* d = (Member*)g.ar.alloc(sizeof(Member) * (cnt ? cnt : 1), alignof(Member));
            for (size_t i = 0; i < cnt; i++) d[i] = g.mtmp[base + i];
            x.u.mem = d;
            g.mtmp.resize(base);
            return x;
        }
    };
    struct ArrB {
        Gen& g;
        size_t base;
        uint64_t list_id;
        explicit ArrB(Gen& gg) : g(gg), base(gg.itmp.size()) {
            list_id = gg.no_count ? ~0ULL : gg.list_ctr[gg.in_status ? 1 : 0]++;
        }
        void add(Node v) { g.itmp.push_back(v); }
        Node done() {
            size_t cnt = g.itmp.size() - base;
            const Directive& d = g.dir;
            if (d.status == g.in_status && d.target == list_id && cnt >= 2) {
                if (d.op == Directive::LIST_INSERT) {
                    g.itmp.insert(g.itmp.begin() + base + cnt / 2, g.cstr("inserted"));
                    cnt++;
                    g.applied = true;
                } else if (d.op == Directive::LIST_DELETE) {
                    g.itmp.erase(g.itmp.begin() + base + cnt / 2);
                    cnt--;
                    g.applied = true;
                }
            }
            Node x;
            x.t = J_ARR;
            x.n = (uint32_t)cnt;
            Node* p = (Node*)g.ar.alloc(sizeof(Node) * (cnt ? cnt : 1), alignof(Node));
            for (size_t i = 0; i < cnt; i++) p[i] = g.itmp[base + i];
            x.u.items = p;
            g.itmp.resize(base);
            return x;
        }
    };
};

struct PairSpec {
    uint64_t g;        // global index
    uint32_t cluster;
    uint32_t kind;
    bool mutated;
};

// ------------------------------------------------------------------ object shapes
void hexstr(char* out, uint64_t v, int n) {
    static const char hx[] = "0123456789abcdef";
    for (int i = n - 1; i >= 0; i--) {
        out[i] = hx[v & 15];
        v >>= 4;
    }
}

Node metadata(Gen& G, const PairSpec& ps, bool is_b, uint32_t nlabels, uint32_t nann) {
    G.no_count = true;
    Gen::ObjB m(G);
    char buf[96];
    snprintf(buf, sizeof(buf), "obj-%llu", (unsigned long long)ps.g);
    m.add("name", G.cstr(buf));
    snprintf(buf, sizeof(buf), "ns-%llu", (unsigned long long)(ps.g % 97));
    m.add("namespace", G.cstr(buf));
    // ignored metadata: differs between A and B
    uint64_t h = mix64(ps.g * 2 + (is_b ? 1 : 0));
    char uid[37] = "00000000-0000-4000-8000-000000000000";
    hexstr(uid, h >> 32, 8);
    hexstr(uid + 24, h & 0xFFFFFFFFFFFFULL, 12);
    m.add("uid", G.cstr(uid));
    snprintf(buf, sizeof(buf), "%llu", (unsigned long long)(h % 10000000));
    m.add("resourceVersion", G.cstr(buf));
    m.add("creationTimestamp", G.cstr("2021-10-04T15:09:37Z"));
    snprintf(buf, sizeof(buf), "lc-%05u", ps.cluster);
    Node lc = G.cstr(buf);
    m.add("clusterName", lc);
    if (is_b) {
        Gen::ArrB mf(G);
        Gen::ObjB e(G);
        e.add("manager", G.cstr("syncer"));
        e.add("operation", G.cstr("Update"));
        mf.add(e.done());
        m.add("managedFields", mf.done());
    }
    // labels / annotations (canonical regions L and N)
    {
        Gen::ObjB l(G);
        l.add("kcp.dev/cluster", lc);
        static const char* keys[] = {"app", "tier", "team", "env", "track"};
        for (uint32_t i = 0; i + 1 < nlabels; i++) {
            Node v = G.rstr(3, 12, kAlnum, 36);
            if (G.dir.op == Directive::LABEL_EDIT && i == G.dir.target % (nlabels - 1)) {
                G.applied = true;
                if (G.dir.target & 1) continue;  // label removed
                v = G.cstr("MUTATED");           // label changed (not in the label alphabet)
            }
            l.add(keys[i % 5], v);
        }
        if (G.dir.op == Directive::LABEL_EDIT && nlabels <= 1) {
            l.add("added", G.cstr("1"));
            G.applied = true;
        }
        m.add("labels", l.done());
    }
    if (nann) {
        Gen::ObjB a(G);
        static const char* keys[] = {"kcp.dev/owned-by", "note", "revision"};
        for (uint32_t i = 0; i < nann; i++) {
            Node v = G.rstr(8, 40, kText, sizeof(kText) - 1);
            if (G.dir.op == Directive::ANNOT_EDIT && i == 0) {
                char* p = (char*)G.ar.alloc(v.n + 1, 1);
                memcpy(p, v.u.s, v.n);
                p[v.n] = '!';
                v.u.s = p;
                v.n++;
                G.applied = true;
            }
            a.add(keys[i % 3], v);
        }
        m.add("annotations", a.done());
    }
    G.no_count = false;
    return m.done();
}

Node gen_configmap(Gen& G, const PairSpec& ps, bool is_b, bool secret) {
    Gen::ObjB o(G);
    o.add("apiVersion", G.cstr("v1"));
    o.add("kind", G.cstr(secret ? "Secret" : "ConfigMap"));
    o.add("metadata", metadata(G, ps, is_b, 4, 2));
    Gen::ObjB d(G);
    const uint32_t nkeys = 8;
    const uint32_t del = (G.dir.op == Directive::KEY_DEL) ? (uint32_t)(G.dir.target % nkeys) : ~0u;
    for (uint32_t i = 0; i < nkeys; i++) {
        Node k = G.rstr(8, 24, kAlnum, 36);
        Node v = secret ? G.rstr(64, 512, kB64, 64) : G.rstr(64, 512, kText, sizeof(kText) - 1);
        if (secret) v.n &= ~3u;  // base64 text length
        if (i == del) {
            G.applied = true;
            continue;
        }
        d.addk(k, G.leaf(v));
    }
    if (G.dir.op == Directive::KEY_ADD) {
        d.add("zz-added-key", G.cstr("1"));
        G.applied = true;
    }
    o.add("data", d.done());
    if (secret) o.add("type", G.cstr("Opaque"));
    return o.done();
}

Node condition(Gen& G, const char* type, const char* st, const char* reason, const char* msg) {
    Gen::ObjB c(G);
    c.add("type", G.leaf(G.cstr(type)));
    c.add("status", G.leaf(G.cstr(st)));
    c.add("reason", G.leaf(G.cstr(reason)));
    c.add("message", G.leaf(G.cstr(msg)));
    c.add("lastUpdateTime", G.leaf(G.cstr("2021-10-04T15:10:00Z")));
    c.add("lastTransitionTime", G.leaf(G.cstr("2021-10-04T15:09:37Z")));
    return c.done();
}

Node gen_deployment(Gen& G, const PairSpec& ps, bool is_b) {
    Gen::ObjB o(G);
    o.add("apiVersion", G.leaf(G.cstr("apps/v1")));
    o.add("kind", G.leaf(G.cstr("Deployment")));
    o.add("metadata", metadata(G, ps, is_b, 2, 1));
    char buf[64];
    Gen::ObjB spec(G);
    int64_t replicas = G.rng.range(1, 10);
    if (G.dir.op == Directive::INT_RETYPE && !G.dir.status) {
        spec.add("replicas", G.f64((double)replicas));  // int64 -> float64 retype (KAT #7)
        G.applied = true;
        G.leaf_ctr[0]++;
    } else {
        spec.add("replicas", G.leaf(G.i64(replicas)));
    }
    {
        Gen::ObjB sel(G), ml(G);
        ml.add("app", G.leaf(G.cstr("nginx")));
        sel.add("matchLabels", ml.done());
        spec.add("selector", sel.done());
    }
    {
        Gen::ObjB tpl(G), tmd(G), tl(G), ps2(G);
        tl.add("app", G.leaf(G.cstr("nginx")));
        tmd.add("labels", tl.done());
        tmd.add("creationTimestamp", G.null());
        tpl.add("metadata", tmd.done());
        Gen::ArrB cs(G);
        Gen::ObjB c(G);
        c.add("name", G.leaf(G.cstr("busybox")));
        snprintf(buf, sizeof(buf), "busybox:1.%u", G.rng.range(20, 36));
        c.add("image", G.leaf(G.cstr(buf)));
        Gen::ArrB cmd(G);
        cmd.add(G.leaf(G.cstr("/bin/sh")));
        cmd.add(G.leaf(G.cstr("-ec")));
        cmd.add(G.leaf(G.cstr("echo \"Going to sleep\"\ntail -f /dev/null\n")));
        c.add("command", cmd.done());
        Gen::ObjB res(G);
        c.add("resources", G.leaf(res.done()));
        c.add("terminationMessagePath", G.leaf(G.cstr("/dev/termination-log")));
        c.add("terminationMessagePolicy", G.leaf(G.cstr("File")));
        c.add("imagePullPolicy", G.leaf(G.cstr("IfNotPresent")));
        cs.add(c.done());
        ps2.add("containers", cs.done());
        ps2.add("restartPolicy", G.leaf(G.cstr("Always")));
        ps2.add("terminationGracePeriodSeconds", G.leaf(G.i64(30)));
        ps2.add("dnsPolicy", G.leaf(G.cstr("ClusterFirst")));
        Gen::ObjB sc(G);
        ps2.add("securityContext", G.leaf(sc.done()));
        ps2.add("schedulerName", G.leaf(G.cstr("default-scheduler")));
        tpl.add("spec", ps2.done());
        spec.add("template", tpl.done());
    }
    {
        Gen::ObjB st(G), ru(G);
        st.add("type", G.leaf(G.cstr("RollingUpdate")));
        ru.add("maxUnavailable", G.leaf(G.cstr("25%")));
        ru.add("maxSurge", G.leaf(G.cstr("25%")));
        st.add("rollingUpdate", ru.done());
        spec.add("strategy", st.done());
    }
    spec.add("revisionHistoryLimit", G.leaf(G.i64(10)));
    spec.add("progressDeadlineSeconds", G.leaf(G.i64(600)));
    o.add("spec", spec.done());
    G.in_status = true;
    Gen::ObjB status(G);
    status.add("observedGeneration", G.leaf(G.i64(1)));
    status.add("replicas", G.leaf(G.i64(replicas)));
    status.add("updatedReplicas", G.leaf(G.i64(replicas)));
    status.add("readyReplicas", G.leaf(G.i64(replicas)));
    status.add("availableReplicas", G.leaf(G.i64(replicas)));
    Gen::ArrB conds(G);
    Node c1 = condition(G, "Available", "True", "MinimumReplicasAvailable", "Deployment has minimum availability.");
    snprintf(buf, sizeof(buf), "ReplicaSet \"example-%08x\" has successfully progressed.", G.rng.range(0, 0x7fffffff));
    Node c2 = condition(G, "Progressing", "True", "NewReplicaSetAvailable", buf);
    if (G.dir.op == Directive::COND_REVERSE) {
        std::swap(c1, c2);
        G.applied = true;
    }
    conds.add(c1);
    conds.add(c2);
    status.add("conditions", conds.done());
    o.add("status", status.done());
    G.in_status = false;
    return o.done();
}

// random nested subtree with a leaf budget
Node rtree(Gen& G, int depth, int& budget, uint32_t vlo, uint32_t vhi) {
    if (depth <= 0 || budget <= 1 || G.rng.unit() < 0.3) {
        budget--;
        double c = G.rng.unit();
        if (c < 0.25) return G.leaf(G.i64((int64_t)G.rng.range(0, 1000000) - 1000));
        if (c < 0.32) return G.leaf(G.f64(G.rng.unit() * 100.0));
        if (c < 0.40) return G.leaf(G.boolean(G.rng.next() & 1));
        if (c < 0.43) return G.leaf(G.null());
        return G.leaf(G.rstr(vlo, vhi, kText, sizeof(kText) - 1));
    }
    if (G.rng.unit() < 0.45) {
        Gen::ArrB a(G);
        uint32_t n = G.rng.range(2, 6);
        for (uint32_t i = 0; i < n && budget > 0; i++) a.add(rtree(G, depth - 1, budget, vlo, vhi));
        return a.done();
    }
    Gen::ObjB o(G);
    uint32_t n = G.rng.range(1, 6);
    for (uint32_t i = 0; i < n && budget > 0; i++) {
        Node k = G.rstr(3, 12, kAlnum, 36);
        o.addk(k, rtree(G, depth - 1, budget, vlo, vhi));
    }
    return o.done();
}

Node gen_crd(Gen& G, const PairSpec& ps, bool is_b, bool deep, uint32_t crd_leaves) {
    Gen::ObjB o(G);
    o.add("apiVersion", G.leaf(G.cstr(deep ? "deep.kcp.dev/v1" : "example.kcp.dev/v1")));
    o.add("kind", G.leaf(G.cstr(deep ? "DeepWidget" : "Widget")));
    o.add("metadata", metadata(G, ps, is_b, 4, 2));
    int leaves, depth;
    uint32_t vlo, vhi, nitems;
    if (deep) {  // 300..3000 leaves log-uniform, depth up to 31
        leaves = (int)(300.0 * pow(10.0, G.rng.unit()));
        depth = (int)G.rng.range(8, 31);
        vlo = 4;
        vhi = 40;
        nitems = (uint32_t)(64.0 * pow(16.0, G.rng.unit()));  // 64..1024 status items
    } else {
        leaves = (int)crd_leaves;
        depth = 6;
        vlo = 8;
        vhi = 48;
        nitems = 5;
    }
    Gen::ObjB spec(G);
    int budget = leaves - (int)(deep ? nitems * 3 : 30);
    if (budget < 10) budget = 10;
    // one guaranteed list so list mutations always have a target
    {
        Gen::ArrB items(G);
        for (int i = 0; i < 6; i++) items.add(G.leaf(G.rstr(vlo, vhi, kText, sizeof(kText) - 1)));
        spec.add("items", items.done());
    }
    while (budget > 0) {
        Node k = G.rstr(3, 12, kAlnum, 36);
        spec.addk(k, rtree(G, depth, budget, vlo, vhi));
    }
    o.add("spec", spec.done());
    G.in_status = true;
    Gen::ObjB status(G);
    status.add("phase", G.leaf(G.cstr("Ready")));
    status.add("observedGeneration", G.leaf(G.i64(G.rng.range(1, 100))));
    Gen::ArrB conds(G);
    for (uint32_t i = 0; i < nitems; i++) {
        Gen::ObjB c(G);
        char buf[32];
        snprintf(buf, sizeof(buf), "C%u", i);
        c.add("type", G.leaf(G.cstr(buf)));
        c.add("status", G.leaf(G.cstr((G.rng.next() & 1) ? "True" : "False")));
        c.add("reason", G.leaf(G.rstr(5, 20, kAlnum, 36)));
        conds.add(c.done());
    }
    status.add("conditions", conds.done());
    o.add("status", status.done());
    G.in_status = false;
    return o.done();
}

Node gen_object(Gen& G, const PairSpec& ps, bool is_b, uint32_t crd_leaves) {
    switch (ps.kind) {
        case K_CM: return gen_configmap(G, ps, is_b, false);
        case K_SECRET: return gen_configmap(G, ps, is_b, true);
        case K_DEPLOY: return gen_deployment(G, ps, is_b);
        case K_CRD: return gen_crd(G, ps, is_b, false, crd_leaves);
        default: return gen_crd(G, ps, is_b, true, crd_leaves);
    }
}

// Picks the mutation for a pair (needs A's leaf / list counts).
Directive pick_mutation(const PairSpec& ps, const Gen& ga, uint32_t* truth) {
    Rng r(mix64(ps.g ^ 0xA5A5A5A5DEADBEEFULL));
    double c = r.unit();
    Directive d;
    if (ps.kind == K_CM || ps.kind == K_SECRET) {
        if (c < 0.70) { d.op = Directive::LEAF_EDIT; d.target = r.next() % ga.leaf_ctr[0]; }
        else if (c < 0.85) { d.op = Directive::LABEL_EDIT; d.target = r.next() % 1000; }
        else if (c < 0.95) { d.op = Directive::ANNOT_EDIT; }
        else if (c < 0.975) { d.op = Directive::KEY_ADD; }
        else { d.op = Directive::KEY_DEL; d.target = r.next() % 8; }
        *truth |= GPUDIFF_SYNTH_SPEC_MUT;
    } else if (ps.kind == K_DEPLOY) {
        if (c < 0.4) { d.op = Directive::LEAF_EDIT; d.target = r.next() % ga.leaf_ctr[0]; *truth |= GPUDIFF_SYNTH_SPEC_MUT; }
        else if (c < 0.5) { d.op = Directive::INT_RETYPE; *truth |= GPUDIFF_SYNTH_SPEC_MUT; }
        else if (c < 0.6) { d.op = Directive::LABEL_EDIT; d.target = r.next() % 1000; *truth |= GPUDIFF_SYNTH_SPEC_MUT; }
        else if (c < 0.85) { d.op = Directive::LEAF_EDIT; d.status = true; d.target = r.next() % ga.leaf_ctr[1]; *truth |= GPUDIFF_SYNTH_STATUS_MUT; }
        else { d.op = Directive::COND_REVERSE; *truth |= GPUDIFF_SYNTH_STATUS_MUT; }
    } else {
        if (c < 0.3 && ga.list_ctr[0]) {
            d.op = (r.next() & 1) ? Directive::LIST_INSERT : Directive::LIST_DELETE;
            d.target = 0;  // the guaranteed "items" list (>= 2 elements)
            *truth |= GPUDIFF_SYNTH_SPEC_MUT;
        } else if (c < 0.55) {
            d.op = Directive::LEAF_EDIT; d.status = true; d.target = r.next() % ga.leaf_ctr[1];
            *truth |= GPUDIFF_SYNTH_STATUS_MUT;
        } else if (c < 0.65) {
            d.op = (r.next() & 1) ? Directive::LIST_INSERT : Directive::LIST_DELETE; d.status = true; d.target = 0;
            *truth |= GPUDIFF_SYNTH_STATUS_MUT;
        } else {
            d.op = Directive::LEAF_EDIT; d.target = r.next() % ga.leaf_ctr[0];
            *truth |= GPUDIFF_SYNTH_SPEC_MUT;
        }
    }
    return d;
}

// ------------------------------------------------------------------ JSON text
void json_str(std::string& o, const char* s, uint32_t n) {
    o.push_back('"');
    for (uint32_t i = 0; i < n; i++) {
        unsigned char c = (unsigned char)s[i];
        if (c == '"') o += "\\\"";
        else if (c == '\\') o += "\\\\";
        else if (c == '\n') o += "\\n";
        else if (c < 0x20) {
            char b[8];
            snprintf(b, sizeof(b), "\\u%04x", c);
            o += b;
        } else o.push_back((char)c);
    }
    o.push_back('"');
}

void to_json(std::string& o, const Node& n) {
    switch (n.t) {
        case J_NULL: o += "null"; break;
        case J_FALSE: o += "false"; break;
        case J_TRUE: o += "true"; break;
        case J_INT: o += std::to_string(n.u.i); break;
        case J_FLOAT: {
            char b[40];
            snprintf(b, sizeof(b), "%.17g", n.u.d);
            std::string s(b);
            if (s.find_first_of(".eEn") == std::string::npos) s += ".0";  // keep float64 on decode
            o += s;
            break;
        }
        case J_STR: json_str(o, n.u.s, n.n); break;
        case J_OBJ:
            o.push_back('{');
            for (uint32_t i = 0; i < n.n; i++) {
                if (i) o.push_back(',');
                json_str(o, n.u.mem[i].k, n.u.mem[i].klen);
                o.push_back(':');
                to_json(o, n.u.mem[i].v);
            }
            o.push_back('}');
            break;
        case J_ARR:
            o.push_back('[');
            for (uint32_t i = 0; i < n.n; i++) {
                if (i) o.push_back(',');
                to_json(o, n.u.items[i]);
            }
            o.push_back(']');
            break;
    }
}

struct Worker {
    EncodeConfig cfg;
    PairEncoder enc{cfg};
    Arena ar_a, ar_b;
    FlatObject fa, fb;
    std::vector<uint8_t> pool;
    std::vector<gpudiff_pair_row> rows;
    std::vector<uint8_t> truth;
    uint64_t leaves = 0;
};

}  // namespace

struct ClusterRange {
    uint64_t gstart, count, lstart;
    uint32_t cluster;
};

struct gpudiff_synth {
    gpudiff_synth_cfg cfg;
    std::vector<ClusterRange> local;  // ascending cluster id
    uint64_t n_local = 0;
    double cum[5];
    std::vector<std::unique_ptr<Worker>> workers;
    uint32_t last_threads = 0;
    uint64_t last_n = 0;

    PairSpec spec_of(uint64_t i) const {
        auto it = std::upper_bound(local.begin(), local.end(), i,
                                   [](uint64_t x, const ClusterRange& r) { return x < r.lstart; });
        --it;
        PairSpec ps;
        ps.g = it->gstart + (i - it->lstart);
        ps.cluster = it->cluster;
        const uint64_t h = mix64(cfg.seed * 0x100000001B3ULL + ps.g);
        const double u = (double)(h >> 11) * (1.0 / 9007199254740992.0);
        uint32_t k = 0;
        while (k < 4 && u >= cum[k]) k++;
        ps.kind = k;
        const double v = (double)(mix64(h ^ 0x5bd1e995) >> 11) * (1.0 / 9007199254740992.0);
        ps.mutated = v < cfg.mutate_frac;
        return ps;
    }

    // builds A and, when mutated or requested, B; returns ground truth bits
    uint32_t build(Worker& w, const PairSpec& ps, Node* a, Node* b, bool* same, bool want_b) {
        const uint64_t seed = mix64(cfg.seed ^ (ps.g * 0x9E3779B97F4A7C15ULL));
        w.ar_a.reset();
        w.ar_b.reset();
        Gen ga(w.ar_a, seed, Directive());
        *a = gen_object(ga, ps, false, cfg.crd_leaves);
        uint32_t truth = 0;
        *same = true;
        Directive d;
        if (ps.mutated) {
            d = pick_mutation(ps, ga, &truth);
            *same = false;
        }
        if (ps.mutated || want_b) {
            Gen gb(w.ar_b, seed, d);
            *b = gen_object(gb, ps, true, cfg.crd_leaves);
            if (ps.mutated && !gb.applied) truth = 0;  // directive found no target
        }
        if (ps.kind == K_DEPLOY || ps.kind == K_CRD || ps.kind == K_DEEP) truth |= GPUDIFF_SYNTH_B_HAS_STATUS;
        return truth;
    }
};

// cluster sizes: rank-frequency Zipf(1.1) with offset 10 over a seeded permutation
static std::vector<uint64_t> cluster_sizes(const gpudiff_synth_cfg* cfg) {
    const uint32_t C = cfg->n_clusters;
    std::vector<uint32_t> perm(C);
    for (uint32_t i = 0; i < C; i++) perm[i] = i;
    Rng r(mix64(cfg->seed ^ 0xC1u));
    for (uint32_t i = C - 1; i > 0; i--) std::swap(perm[i], perm[r.next() % (i + 1)]);
    std::vector<double> wt(C);
    double ws = 0;
    for (uint32_t c = 0; c < C; c++) {
        wt[c] = pow((double)perm[c] + 10.0, -1.1);
        ws += wt[c];
    }
    std::vector<uint64_t> size(C);
    uint64_t assigned = 0;
    for (uint32_t c = 0; c < C; c++) {
        size[c] = (uint64_t)floor((double)cfg->n_pairs * wt[c] / ws);
        assigned += size[c];
    }
    for (uint64_t k = 0; assigned < cfg->n_pairs; k++, assigned++) size[k % C]++;
    return size;
}

// a population whose local clusters are those with mine(c)
template <class Mine>
static int synth_plan(const gpudiff_synth_cfg* cfg, Mine mine, gpudiff_synth** out) {
    std::unique_ptr<gpudiff_synth> s(new (std::nothrow) gpudiff_synth());
    if (!s) return -2;
    s->cfg = *cfg;
    if (s->cfg.crd_leaves == 0) s->cfg.crd_leaves = 200;
    double w[5] = {cfg->w_configmap, cfg->w_secret, cfg->w_deployment, cfg->w_crd, cfg->w_deep};
    double tot = 0;
    for (double x : w) tot += x;
    if (tot <= 0) return -1;
    double acc = 0;
    for (int k = 0; k < 5; k++) {
        acc += w[k] / tot;
        s->cum[k] = acc;
    }
    const std::vector<uint64_t> size = cluster_sizes(cfg);
    uint64_t g = 0, l = 0;
    for (uint32_t c = 0; c < cfg->n_clusters; c++) {
        if (mine(c) && size[c]) {
            s->local.push_back({g, size[c], l, c});
            l += size[c];
        }
        g += size[c];
    }
    s->n_local = l;
    *out = s.release();
    return 0;
}

extern "C" {

int gpudiff_synth_open_ex(const gpudiff_synth_cfg* cfg, int world, int rank, const uint64_t* cluster_weight,
                          gpudiff_synth** out) {
    if (!cfg || !out || world < 1 || rank < 0 || rank >= world || cfg->n_clusters == 0) return -1;
    // LPT of clusters onto ranks: by the given weights (sum of B_pair,
    // gpudiff_synth_cluster_bytes), else by pair count; the rule of gpudiff_shard_lpt / shard.lpt_assign
    const uint32_t C = cfg->n_clusters;
    const std::vector<uint64_t> size = cluster_sizes(cfg);
    const uint64_t* wt = cluster_weight ? cluster_weight : size.data();
    std::vector<uint32_t> order(C);
    for (uint32_t i = 0; i < C; i++) order[i] = i;
    std::sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) { return wt[x] != wt[y] ? wt[x] > wt[y] : x < y; });
    std::vector<uint64_t> load(world, 0);
    std::vector<int> owner(C);
    for (uint32_t c : order) {
        int best = 0;
        for (int k = 1; k < world; k++)
            if (load[k] < load[best]) best = k;
        owner[c] = best;
        load[best] += wt[c];
    }
    return synth_plan(cfg, [&](uint32_t c) { return owner[c] == rank; }, out);
}

int gpudiff_synth_open(const gpudiff_synth_cfg* cfg, int world, int rank, gpudiff_synth** out) {
    return gpudiff_synth_open_ex(cfg, world, rank, nullptr, out);
}

int gpudiff_synth_cluster_sizes(const gpudiff_synth_cfg* cfg, uint64_t* out) {
    if (!cfg || !out || cfg->n_clusters == 0) return -1;
    const std::vector<uint64_t> size = cluster_sizes(cfg);
    memcpy(out, size.data(), size.size() * sizeof(uint64_t));
    return 0;
}

void gpudiff_synth_close(gpudiff_synth* s) { delete s; }
uint64_t gpudiff_synth_local_pairs(const gpudiff_synth* s) { return s ? s->n_local : 0; }
uint64_t gpudiff_synth_local_clusters(const gpudiff_synth* s) { return s ? s->local.size() : 0; }
uint64_t gpudiff_synth_global_index(const gpudiff_synth* s, uint64_t i) { return s->spec_of(i).g; }
int gpudiff_synth_local_ids(const gpudiff_synth* s, uint32_t* out) {
    if (!s || !out) return -1;
    for (const ClusterRange& r : s->local)
        for (uint64_t k = 0; k < r.count; k++) out[r.lstart + k] = (uint32_t)(r.gstart + k);
    return 0;
}

int gpudiff_synth_encode(gpudiff_synth* s, uint64_t first, uint64_t n, uint32_t threads, uint64_t* pool_bytes,
                         uint64_t* total_leaves) {
    if (!s || first + n > s->n_local) return -1;
    uint32_t T = std::max<uint32_t>(1, std::min<uint64_t>(threads ? threads : 1, std::max<uint64_t>(1, n / 64)));
    while (s->workers.size() < T) s->workers.emplace_back(new Worker());
    auto work = [&](uint32_t t) {
        Worker& w = *s->workers[t];
        w.pool.clear();
        w.rows.clear();
        w.truth.clear();
        w.enc.leaves_written = 0;
        const uint64_t b = first + n * t / T, e = first + n * (t + 1) / T;
        w.rows.resize(e - b);
        w.truth.resize(e - b);
        for (uint64_t i = b; i < e; i++) {
            const PairSpec ps = s->spec_of(i);
            Node a, bn;
            bool same;
            const uint32_t truth = s->build(w, ps, &a, &bn, &same, false);
            flatten_object(a, w.fa);
            if (same) {
                w.enc.encode_flat(&w.fa, &w.fa, (uint32_t)ps.g, ps.cluster, w.pool, w.rows[i - b]);
            } else {
                flatten_object(bn, w.fb);
                w.enc.encode_flat(&w.fa, &w.fb, (uint32_t)ps.g, ps.cluster, w.pool, w.rows[i - b]);
            }
            w.truth[i - b] = (uint8_t)truth;
        }
        w.pool.resize((w.pool.size() + GPUDIFF_BLOB_ALIGN - 1) & ~(size_t)(GPUDIFF_BLOB_ALIGN - 1), 0);
        w.leaves = w.enc.leaves_written;
    };
    std::vector<std::thread> th;
    for (uint32_t t = 1; t < T; t++) th.emplace_back(work, t);
    work(0);
    for (auto& x : th) x.join();
    uint64_t pb = 0, lv = 0;
    for (uint32_t t = 0; t < T; t++) {
        pb += s->workers[t]->pool.size();
        lv += s->workers[t]->leaves;
    }
    s->last_threads = T;
    s->last_n = n;
    if (pool_bytes) *pool_bytes = pb;
    if (total_leaves) *total_leaves = lv;
    return 0;
}

int gpudiff_synth_cluster_bytes(const gpudiff_synth_cfg* cfg, uint32_t stride, uint32_t offset, uint32_t threads,
                                uint64_t* out) {
    if (!cfg || !out || stride == 0 || offset >= stride || cfg->n_clusters == 0) return -1;
    gpudiff_synth* raw = nullptr;
    int rc = synth_plan(cfg, [&](uint32_t c) { return c % stride == offset; }, &raw);
    if (rc) return rc;
    std::unique_ptr<gpudiff_synth> s(raw);
    for (uint32_t c = offset; c < cfg->n_clusters; c += stride) out[c] = 0;
    const uint64_t step = 1ull << 17;
    for (uint64_t first = 0; first < s->n_local; first += step) {
        const uint64_t n = std::min(step, s->n_local - first);
        if ((rc = gpudiff_synth_encode(s.get(), first, n, threads, nullptr, nullptr))) return rc;
        for (uint32_t t = 0; t < s->last_threads; t++)
            for (const gpudiff_pair_row& r : s->workers[t]->rows) out[r.cluster_id] += gpudiff_pair_compare_bytes(&r);
    }
    return 0;
}

int gpudiff_synth_copy_out(gpudiff_synth* s, uint8_t* pool, gpudiff_pair_row* rows, uint8_t* truth) {
    if (!s) return -1;
    uint64_t base = 0, r0 = 0;
    for (uint32_t t = 0; t < s->last_threads; t++) {
        Worker& w = *s->workers[t];
        if (pool && !w.pool.empty()) memcpy(pool + base, w.pool.data(), w.pool.size());
        for (size_t i = 0; i < w.rows.size(); i++) {
            gpudiff_pair_row r = w.rows[i];
            r.off_a += base;
            r.off_b += base;
            if (rows) rows[r0 + i] = r;
            if (truth) truth[r0 + i] = w.truth[i];
        }
        r0 += w.rows.size();
        base += w.pool.size();
    }
    return 0;
}

int gpudiff_synth_json(gpudiff_synth* s, uint64_t i, char* a, size_t acap, size_t* alen, char* b, size_t bcap,
                       size_t* blen) {
    if (!s || i >= s->n_local) return -1;
    if (s->workers.empty()) s->workers.emplace_back(new Worker());
    Worker& w = *s->workers[0];
    const PairSpec ps = s->spec_of(i);
    Node na, nb;
    bool same;
    s->build(w, ps, &na, &nb, &same, true);
    std::string ja, jb;
    to_json(ja, na);
    to_json(jb, nb);
    if (alen) *alen = ja.size();
    if (blen) *blen = jb.size();
    if (a && acap >= ja.size()) memcpy(a, ja.data(), ja.size());
    if (b && bcap >= jb.size()) memcpy(b, jb.data(), jb.size());
    return (acap >= ja.size() && bcap >= jb.size()) ? 0 : 1;
}

// JSON of pairs [first, first+n): A_i then B_i for every pair, concatenated
// into one buffer (watch-replay inputs); offs[2n+1] are byte offsets.
int gpudiff_synth_json_range(gpudiff_synth* s, uint64_t first, uint64_t n, uint32_t threads, uint8_t** buf,
                             uint64_t* offs, uint8_t* truth) {
    if (!s || !buf || !offs || first + n > s->n_local) return -1;
    *buf = nullptr;
    const uint32_t T = std::max<uint32_t>(1, std::min<uint64_t>(threads ? threads : 1, std::max<uint64_t>(1, n / 64)));
    while (s->workers.size() < T) s->workers.emplace_back(new Worker());
    std::vector<std::string> parts(T);
    std::vector<std::vector<uint64_t>> lens(T);
    auto work = [&](uint32_t t) {
        Worker& w = *s->workers[t];
        const uint64_t b = first + n * t / T, e = first + n * (t + 1) / T;
        std::string ja, jb;
        for (uint64_t i = b; i < e; i++) {
            const PairSpec ps = s->spec_of(i);
            Node na, nb;
            bool same;
            const uint32_t tr = s->build(w, ps, &na, &nb, &same, true);
            if (truth) truth[i - first] = (uint8_t)tr;
            ja.clear();
            jb.clear();
            to_json(ja, na);
            to_json(jb, nb);
            parts[t] += ja;
            parts[t] += jb;
            lens[t].push_back(ja.size());
            lens[t].push_back(jb.size());
        }
    };
    std::vector<std::thread> th;
    for (uint32_t t = 1; t < T; t++) th.emplace_back(work, t);
    work(0);
    for (auto& x : th) x.join();
    uint64_t total = 0;
    for (auto& p : parts) total += p.size();
    uint8_t* out = (uint8_t*)malloc(std::max<uint64_t>(total, 1));
    if (!out) return -2;
    uint64_t pos = 0, k = 0;
    offs[0] = 0;
    for (uint32_t t = 0; t < T; t++) {
        memcpy(out + pos, parts[t].data(), parts[t].size());
        pos += parts[t].size();
        for (uint64_t l : lens[t]) {
            offs[k + 1] = offs[k] + l;
            k++;
        }
    }
    *buf = out;
    return 0;
}

void gpudiff_synth_free_buf(uint8_t* buf) { free(buf); }

}  // extern "C"
