// Object encoding in the device-store format: kernel K0 (device JSON
// tokenizer + encoder) over a set of documents, and the host encoder over one
// document, for inspection and the K0 parity tests (include/gpudiff.h).
#include <string.h>

#include <vector>

#include "engine.h"
#include "tokenize.h"

using namespace gd;

namespace {

struct DevBuf {
    void* p = nullptr;
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
};

}  // namespace

extern "C" {

int gpudiff_encode_object_host(const uint8_t* doc, size_t len, uint32_t seed, uint32_t bits, uint8_t* out,
                               uint64_t out_cap, gpudiff_obj_info* info) {
    if (!doc || !info || seed > 255) return GPUDIFF_E_INVAL;
    memset(info, 0, sizeof(*info));
    EncodeConfig cfg;
    cfg.hash_bits = (bits == 0 || bits >= GPUDIFF_PATH_HASH_BITS) ? GPUDIFF_PATH_HASH_BITS : bits;
    PairEncoder enc(cfg);
    Arena arena;
    FlatObject o;
    if (!enc.flatten_json(doc, len, arena, o)) {
        info->status = GPUDIFF_TOK_SYNTAX;
        return GPUDIFF_OK;
    }
    info->oflags = o.flags & GPUDIFF_OBJ_HAS_STATUS;
    if (!enc.hash_single(o, seed)) {
        info->status = GPUDIFF_TOK_HASH;
        return GPUDIFF_OK;
    }
    std::vector<uint8_t> pool;
    uint64_t off;
    uint32_t bytes;
    enc.write_object_tab(o, pool, &off, &info->spec_l, &info->spec_ar, &info->stat_l, &info->stat_ar, &bytes);
    info->n_tab = o.tab.n;
    info->off = 0;
    info->bytes = bytes;
    if (out) {
        if (bytes > out_cap) return GPUDIFF_E_CAPACITY;
        memcpy(out, pool.data() + off, bytes);
    }
    return GPUDIFF_OK;
}

int gpudiff_encode_objects(gpudiff_ctx* c, const uint8_t* const* docs, const size_t* lens, const uint32_t* seeds,
                           size_t n, uint8_t* out, uint64_t out_cap, gpudiff_obj_info* info) {
    if (!c || (n && (!docs || !lens || !info)) || n > 0xFFFFFFFFu) return GPUDIFF_E_INVAL;
    int rc = set_device(c);
    if (rc) return rc;
    if (!n) return GPUDIFF_OK;
    std::vector<TokDoc> td(n);
    uint64_t jbytes = 0, sbytes = 0;
    for (size_t i = 0; i < n; i++) {
        if (lens[i] > 0xFFFFFFFFull) return GPUDIFF_E_INVAL;
        memset(&td[i], 0, sizeof(TokDoc));
        td[i].json_off = jbytes;
        td[i].json_len = (uint32_t)lens[i];
        td[i].scratch_off = sbytes;
        td[i].seed = seeds ? seeds[i] : 0u;
        jbytes = (jbytes + lens[i] + kTokSlack + 15) & ~15ull;
        sbytes += tok_scratch_bytes(td[i].json_len);
    }
    jbytes += kTokSlack;
    std::vector<uint8_t> jb(jbytes, 0);
    for (size_t i = 0; i < n; i++)
        if (lens[i]) memcpy(jb.data() + td[i].json_off, docs[i], lens[i]);
    const uint64_t cap = out_cap ? out_cap : 16;
    DevBuf dj, ds, dsp, du, dd, dout;
    HIPCHK(hipMalloc(&dj.p, jbytes));
    HIPCHK(hipMalloc(&ds.p, std::max<uint64_t>(sbytes, 256)));
    HIPCHK(hipMalloc(&dsp.p, cap));
    HIPCHK(hipMalloc(&du.p, 8));
    HIPCHK(hipMalloc(&dd.p, n * sizeof(TokDoc)));
    HIPCHK(hipMalloc(&dout.p, n * sizeof(TokOut)));
    HIPCHK(hipMemcpyAsync(dj.p, jb.data(), jbytes, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(dd.p, td.data(), n * sizeof(TokDoc), hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemsetAsync(du.p, 0, 8, c->stream));
    HIPCHK(hipMemsetAsync(dsp.p, 0xA5, cap, c->stream));  // poison: every blob byte must be written by K0
    HIPCHK(launch_encode_docs(c->stream, (const TokDoc*)dd.p, (uint32_t)n, (const uint8_t*)dj.p, (uint8_t*)ds.p,
                              (uint8_t*)dsp.p, cap, (unsigned long long*)du.p, c->hash_mask, (TokOut*)dout.p,
                              nullptr, nullptr));
    std::vector<TokOut> to(n);
    uint64_t used = 0;
    HIPCHK(hipMemcpyAsync(to.data(), dout.p, n * sizeof(TokOut), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(&used, du.p, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (out && out_cap) HIPCHK(hipMemcpy(out, dsp.p, std::min(used, out_cap), hipMemcpyDeviceToHost));
    for (size_t i = 0; i < n; i++) {
        gpudiff_obj_info& f = info[i];
        f.status = (int32_t)to[i].status;
        f.oflags = to[i].oflags;
        f.spec_l = to[i].spec_l;
        f.spec_ar = to[i].spec_ar;
        f.stat_l = to[i].stat_l;
        f.stat_ar = to[i].stat_ar;
        f.off = to[i].off;
        f.bytes = to[i].bytes;
        f.n_tab = to[i].n_tab;
    }
    return GPUDIFF_OK;
}

int gpudiff_k2_profile(gpudiff_ctx* c, uint64_t* dev_buf, uint32_t cap_waves) {
    if (!c) return GPUDIFF_E_INVAL;
    int rc = set_device(c);
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(c->stream));
    HIPCHK(k2_profile(dev_buf, cap_waves));
    c->k2_timeline = dev_buf != nullptr;
    return GPUDIFF_OK;
}

int gpudiff_k0_profile(gpudiff_ctx* c, int enable, uint64_t* ticks8) {
    if (!c) return GPUDIFF_E_INVAL;
    int rc = set_device(c);
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(c->stream));
    HIPCHK(k0_profile(enable, ticks8));
    return GPUDIFF_OK;
}

}  // extern "C"
