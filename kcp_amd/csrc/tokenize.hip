// K0 k_encode_docs: device JSON tokenizer + canonical encoder (gfx950, wave64).
//
// One wave per document (a raw informer event body).  The output is the blob
// the host encoder writes for the same object (encoder.cpp write_blob) plus
// the path-table trailer of the object store:
// byte-identical, so the diff kernels cannot tell the two producers apart.
//
// Phases (all inside one wave, working set in a per-document scratch area):
//   1 structural scan, 64 bytes per step: ballots give 64-bit masks of
//     backslashes, quotes, structural characters and whitespace; escapes and
//     in-string state are resolved on the masks (prefix-xor of the unescaped
//     quotes), and every token start (structural, open/close quote, atom
//     start) is appended with its position in one coalesced store per step
//   2 tree building: the wave walks the token list (64 tokens per vector
//     load, readlane per token) as a uniform state machine that checks the
//     JSON grammar, creates one node per value (parent, key token or array
//     index) and assigns the reference's regions -- S (top-level keys except
//     metadata/status, top-level null dropped), L/N (metadata.labels /
//     metadata.annotations children, kept only if every value is a string),
//     T (status subtree) -- specsyncer.go:17-41, statussyncer.go:15-27
//   3 per node, lane-parallel: chained path hash level by level
//     (h(child) = XXH64(component, h(parent))), value decoding (Go escapes /
//     UTF-8 repair, int64 or exact-fast-path float64, literals)
//   4 bitonic sort of the node keys; equal neighbours (a duplicate key or a
//     collision) or a node hash equal to the root's hand the document to the
//     host
//   5 ballot/prefix compaction of the spec / status leaves in key order into
//     the blob, and of the path-table nodes (region leaves and their
//     ancestors) behind it, allocated with one atomic on the space's append
//     point
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gpudiff.h"
#include "decfloat.h"
#include "tokenize.h"
#include "xxh64.h"

#include "tokdev.h"

namespace gd {

// tuning hook (gpudiff_k0_profile): per-phase wall-clock ticks summed over waves
__device__ unsigned long long g_k0_prof[8];
__device__ int g_k0_prof_on;

template <int MINW, int MODE = kModeEncode>
__global__ __launch_bounds__(256, MINW) void k_encode_docs(const TokDoc* __restrict__ docs, uint32_t n_docs,
                                                     const uint8_t* __restrict__ json, uint8_t* __restrict__ scratch,
                                                     uint8_t* __restrict__ space, uint64_t space_cap,
                                                     unsigned long long* __restrict__ used, uint64_t mask,
                                                     TokOut* __restrict__ out, const DSlot* __restrict__ slots,
                                                     const DocLink* __restrict__ links) {
    // per wave, one LDS area reused phase by phase (5 KiB -> 8 workgroups of 4 waves per CU):
    //   phase 1: [0, 2048) byte ring; phase 2: [2048, 4096) container stack;
    //   phases 3a-3b, small documents (<= kLdsHash nodes, depth < 32): [0, 256) depth histogram + cursors,
    //   [256, 2304) the nodes' hash inputs, [2304, 2816) depth order (u16), [3072, 5120) hashes; phase 3a's decoded
    //   strings staged at [2304, 5120) after its loop;
    //   phase 3b, other documents: [0, 2048) depth histogram + cursors, [2048, ..) depth order (<= kLdsOrder nodes);
    //   phase 4: [0, 4608) sort (ns <= kLdsSort)
    __shared__ __attribute__((aligned(16))) uint8_t s_lds[kWavesPerBlock][kLdsPerWave];

    const uint32_t lane = lane_id();
    const uint32_t wib = threadIdx.x >> 6;
    const uint32_t doc_i = __builtin_amdgcn_readfirstlane(blockIdx.x * kWavesPerBlock + wib);
    if (doc_i >= n_docs) return;
    uint8_t* lds = s_lds[wib];
    uint32_t* hist = (uint32_t*)lds;
    uint32_t* cur = (uint32_t*)(lds + 1024);

    const TokDoc D = docs[doc_i];
    const uint8_t* d = json + D.json_off;
    const uint32_t len = D.json_len;
    TokOut o{};
    if (len > kTokMaxLen) {
        if (lane == 0) {
            if constexpr (MODE == kModeRollup) {
                RollOut R{};
                R.status = GPUDIFF_TOK_SIZE;
                ((RollOut*)space)[doc_i] = R;
            } else if constexpr (MODE == kModeNegotiate) {
                ((NegOut*)space)[doc_i].status = GPUDIFF_TOK_SIZE;
            } else {
                o.status = GPUDIFF_TOK_SIZE;
                out[doc_i] = o;
            }
        }
        return;
    }
    uint8_t* base = scratch + D.scratch_off;
    Scratch S;
    if constexpr (MODE == kModeRollup || MODE == kModeNegotiate) {
        S = Scratch{};
        S.tok = (uint32_t*)base;
        S.rec = (uint4*)(base + tok_align(4ull * tok_cap(len)));
        S.str = base + tok_align(4ull * tok_cap(len)) + tok_align(16ull * node_cap(len));
    } else if constexpr (MODE == kModeMarshal) {
        const MarshalLayout ML = marshal_layout(len);
        S = Scratch{};
        S.tok = (uint32_t*)(base + ML.tok);
        S.rec = (uint4*)(base + ML.rec);
        S.str = base + ML.str;
    } else {
        const TokLayout LY = tok_layout(len);
        S.tok = (uint32_t*)(base + LY.tok);
        S.rec = (uint4*)(base + LY.rec);
        S.h = (uint64_t*)(base + LY.h);
        S.val = (uint64_t*)(base + LY.val);
        S.skey = (uint64_t*)(base + LY.skey);
        S.meta = (uint32_t*)(base + LY.meta);
        S.order = (uint32_t*)(base + LY.order);
        S.sidx = (uint32_t*)(base + LY.sidx);
        S.str = base + LY.str;
    }
    const uint32_t ncap = node_cap(len);
    uint32_t status = GPUDIFF_TOK_OK;

    const bool prof = g_k0_prof_on != 0;
    uint64_t t_prev = prof ? wall_clock64() : 0;
    auto mark = [&](int ph) {
        if (prof) {
            const uint64_t t = wall_clock64();
            if (lane == 0) atomicAdd(&g_k0_prof[ph], (unsigned long long)(t - t_prev));
            t_prev = t;
        }
    };
    // ------------------------------------------------------------ phase 1: structural scan
    // One byte per lane per 64-byte step.  Byte classes are VALU compares (their
    // ballots are the step's masks), the in-string state is the parity of an
    // mbcnt of unescaped quotes, token codes are chosen per lane without
    // branches.  The document sits in a 4 x 1 KiB LDS ring: up to 4 KiB is
    // staged in one go; past that, chunk ch + 1 (the lookahead of chunk ch) is
    // written from registers loaded one chunk earlier, so no step waits on HBM.
    uint8_t* ring = lds;
    uint32_t ntok = 0;
    uint64_t esc_carry = 0, atom_carry = 0;
    uint32_t str_par = 0;
    uint32_t last_open_idx = NONE, last_open_pos = 0, last_marked = NONE;
    bool ctl_in_string = false;
    const uint32_t nchunks = (len + 1023u) >> 10;
    auto ld_chunk = [&](uint32_t ch) -> u32x4 {
        const uint32_t o = (ch << 10) + lane * 16u;
        u32x4 v = {0x20202020u, 0x20202020u, 0x20202020u, 0x20202020u};
        if (o < len) v = *(const u32x4*)(d + o);  // d is 16-B aligned, kTokSlack readable past len
        return v;
    };
    auto put_chunk = [&](uint32_t ch, u32x4 v) { *(u32x4*)(ring + ((ch & 3u) << 10) + lane * 16u) = v; };
    {
        u32x4 v[4];
#pragma unroll
        for (uint32_t j = 0; j < 4; j++)
            if (j < nchunks) v[j] = ld_chunk(j);
#pragma unroll
        for (uint32_t j = 0; j < 4; j++)
            if (j < nchunks) put_chunk(j, v[j]);
    }
    u32x4 pre = {0u, 0u, 0u, 0u};
    if (nchunks > 4) pre = ld_chunk(4);
    lds_order();
    auto ring32 = [&](uint32_t p) -> uint32_t { return *(const uint32_t*)(ring + (p & 4095u)); };
    // the token code of an opening quote at pos: a region keyword when the exact string follows (the 16 bytes
    // after the quote, from five LDS words; bytes past the document cannot fake a match: a string that closes
    // inside the document puts its quote inside the compared span), else the quote itself
    auto keyword = [&](uint32_t pos) -> uint32_t {
        const uint32_t a = (pos + 1u) & ~3u, sh = (pos + 1u) & 3u;
        const uint32_t w0 = ring32(a), w1 = ring32(a + 4u), w2 = ring32(a + 8u), w3 = ring32(a + 12u);
        const uint32_t x0 = __builtin_amdgcn_alignbyte(w1, w0, sh), x1 = __builtin_amdgcn_alignbyte(w2, w1, sh);
        const uint32_t x2 = __builtin_amdgcn_alignbyte(w3, w2, sh);
        uint32_t kw = '"';
        kw = (x0 == 0x6174656du && x1 == 0x61746164u && (x2 & 0xFFu) == 0x22u) ? TK_KEY_META : kw;  // metadata"
        kw = (x0 == 0x74617473u && (x1 & 0xFFFFFFu) == 0x227375u) ? TK_KEY_STATUS : kw;          // status"
        kw = (x0 == 0x6562616cu && (x1 & 0xFFFFFFu) == 0x22736cu) ? TK_KEY_LABELS : kw;          // labels"
        kw = (x0 == 0x6f6e6e61u && x1 == 0x69746174u && x2 == 0x22736e6fu) ? TK_KEY_ANNOT : kw;  // annotations"
        return kw;
    };
    // 256 bytes in one step, 4 per lane, when the block holds no backslash and no byte >= 0x80 (and no escape
    // carries into it): no escapes, so the unescaped quotes are the quotes; a lane's in-string state is the parity
    // of the quotes in the lanes below it (one ballot + mbcnt) and its own prefix parity; tokens are compacted with
    // a 3-ballot prefix of the per-lane counts.  The same tokens, codes and state as four 64-byte steps (below).
    // Returns false (nothing done) otherwise.
    auto fast_block = [&](uint32_t b) -> bool {
        const uint32_t p4 = b + 4u * lane;
        uint32_t x = *(const uint32_t*)(ring + (p4 & 4095u));
        if (p4 + 4u > len) {  // bytes past the document read as spaces
            const uint32_t nv = p4 >= len ? 0u : len - p4;
            const uint32_t keep = (1u << (8u * nv)) - 1u;
            x = (x & keep) | (0x20202020u & ~keep);
        }
        // byte classes of the lane's four bytes at once (SWAR): a class is a mask with bit 8j + 7 set for byte j.
        // nz7(v) has bit 8j + 7 set iff byte j of v is nonzero (no carry crosses a byte); x ^ c for each class byte
        // c, the classes' nz7 ANDed, the complement's high bits = the bytes equal to one of them (half the VALU and a
        // third of the scalar work of per-byte compares, whose lane masks the scalar unit combined)
        constexpr uint32_t K8 = 0x80808080u;
        auto nz7 = [](uint32_t v) -> uint32_t { return ((v & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | v; };
        const uint32_t xb = x & 0xDFDFDFDFu;  // '[' ']' and '{' '}' fold together
        const uint32_t Qn = K8 & ~nz7(x ^ 0x22222222u);
        const uint32_t Sn = K8 & ~(nz7(xb ^ 0x5B5B5B5Bu) & nz7(xb ^ 0x5D5D5D5Du) & nz7(x ^ 0x3A3A3A3Au) & nz7(x ^ 0x2C2C2C2Cu));
        const uint32_t Wn = K8 & ~(nz7(x ^ 0x20202020u) & nz7(x ^ 0x0A0A0A0Au) & nz7(x ^ 0x0D0D0D0Du) & nz7(x ^ 0x09090909u));
        const uint32_t Cn = K8 & ~nz7(x & 0xE0E0E0E0u);                      // < 0x20
        const uint32_t Mn = (K8 & ~nz7(x ^ 0x5C5C5C5Cu)) | (x & K8);         // '\\' or >= 0x80
        if (esc_carry || ballot(Mn != 0u)) return false;
        const uint64_t odd = ballot(__builtin_popcount(Qn) & 1u);
        const uint32_t P = (str_par + mbcnt64(odd)) & 1u;  // parity of the quotes before this lane
        uint32_t px = Qn ^ (Qn << 8);
        px = px ^ (px << 16);                               // inclusive prefix parity within the lane
        const uint32_t In = px ^ (P ? K8 : 0u);             // in a string (opening quote in, closing out)
        str_par = (str_par + popc64(odd)) & 1u;
        const uint32_t opens = Qn & In, closes = Qn & ~In;
        const uint32_t atom = K8 & ~In & ~Qn & ~Sn & ~Wn;
        const uint32_t prev = wave_shr1(atom >> 31, (uint32_t)atom_carry);  // byte 3 of the lane below
        const uint32_t astart = atom & ~((atom << 8) | (prev << 7));
        atom_carry = rdlane(atom >> 31, 63);
        if (ballot((Cn & In & ~opens) != 0u)) ctl_in_string = true;
        const uint32_t Tn = (Sn & ~In) | Qn | astart;
        const uint32_t tc = __builtin_popcount(Tn);
        const uint64_t c0 = ballot(tc & 1u), c1 = ballot(tc & 2u), c2 = ballot(tc & 4u);
        const uint32_t pre = mbcnt64(c0) + 2u * mbcnt64(c1) + 4u * mbcnt64(c2);
        const uint32_t j1 = opens ? (uint32_t)__builtin_ctz(opens) >> 3 : 4u;  // most lanes hold at most one opening
        // (every lane reads its keyword window -- LDS reads and compares, no branch; the result is used only at an
        // opening quote)
        const uint32_t kw1 = keyword(p4 + j1);
        const uint32_t op2 = opens & (opens - 1u);
        uint32_t kw2 = 0u;
        if (ballot(op2 != 0u)) kw2 = keyword(p4 + (op2 ? (uint32_t)__builtin_ctz(op2) >> 3 : 0u));  // uniform test
        // every lane stores four words: a byte that starts no token writes slot len + 1, which no token uses (a
        // document of len bytes has at most len tokens, tok_cap = len + 2) -- stores without a branch each
        uint32_t k = ntok + pre;
#pragma unroll
        for (uint32_t j = 0; j < 4; j++) {
            const bool tj = (Tn >> (8u * j + 7u)) & 1u;
            const uint32_t code = ((closes >> (8u * j + 7u)) & 1u) ? TK_CLOSEQ
                                  : ((opens >> (8u * j + 7u)) & 1u) ? (j == j1 ? kw1 : kw2) : (x >> (8u * j)) & 0xFFu;
            S.tok[tj ? k : len + 1u] = (code << 24) | (p4 + j);
            k += tj ? 1u : 0u;
        }
        const uint64_t om = ballot(opens != 0u);
        if (om) {  // the last opening quote of the block (a later step may mark its string slow)
            const uint32_t L = 63u - (uint32_t)__builtin_clzll(om);
            const uint32_t jl = opens ? (31u - (uint32_t)__builtin_clz(opens)) >> 3 : 0u;
            last_open_idx = rdlane(ntok + pre + __builtin_popcount(Tn & ((1u << (8u * jl)) - 1u)), L);
            last_open_pos = b + 4u * L + rdlane(jl, L);
        }
        ntok += popc64(c0) + 2u * popc64(c1) + 4u * popc64(c2);
        return true;
    };
    for (uint32_t ch = 0; ch < nchunks; ch++) {
        if (ch >= 3 && ch + 1 < nchunks) {  // the lookahead chunk, loaded during chunk ch - 1
            put_chunk(ch + 1, pre);
            if (ch + 2 < nchunks) pre = ld_chunk(ch + 2);
            lds_order();
        }
        const uint32_t bend = min(len, (ch + 1) << 10);
        for (uint32_t b4 = ch << 10; b4 < bend; b4 += 256) {
          if (fast_block(b4)) continue;
          for (uint32_t b = b4; b < min(bend, b4 + 256u); b += 64) {  // the block holds an escape or a
                                                                        // non-ASCII byte: 64 bytes a step
            const uint32_t pos = b + lane;
            const uint32_t c = pos < len ? (uint32_t)ring[pos & 4095u] : 0x20u;
            const uint64_t bs = ballot(c == '\\');
            const uint64_t qt = ballot(c == '"');
            const uint32_t cb = c & 0xDFu;  // '[' ']' and '{' '}' fold together
            const uint64_t st = ballot((cb == '[') | (cb == ']') | (c == ':') | (c == ','));
            const uint64_t wsm = ballot((c == ' ') | (c == '\n') | (c == '\r') | (c == '\t'));
            const uint64_t ctl = ballot(c < 0x20u);  // inside a string every control byte is an error
            const uint64_t hi = ballot(c >= 0x80u);
            // escaped characters: an unescaped backslash escapes the next byte
            uint64_t esc = esc_carry;
            esc_carry = 0;
            for (uint64_t m = bs; m;) {
                const uint32_t i = (uint32_t)__builtin_ctzll(m);
                m &= m - 1;
                if ((esc >> i) & 1ull) continue;
                if (i == 63) esc_carry = 1;
                else esc |= 1ull << (i + 1);
            }
            const uint64_t q = qt & ~esc;
            // inside a string (its opening quote included, its closing quote not):
            // the parity of the unescaped quotes up to and including this byte
            const uint32_t par = (mbcnt64(q) + (uint32_t)(c == '"' && !((esc >> lane) & 1ull)) + str_par) & 1u;
            const uint64_t instr = ballot(par != 0u);
            str_par = (uint32_t)(instr >> 63);
            const uint64_t valid = mask_lt(len - b);
            const uint64_t opens = q & instr, closes = q & ~instr;
            const uint64_t structural = st & ~instr & valid;
            const uint64_t atom = ~instr & ~q & ~st & ~wsm & valid;
            const uint64_t astart = atom & ~((atom << 1) | atom_carry);
            atom_carry = atom >> 63;
            if (ctl & valid & instr & ~opens) ctl_in_string = true;
            const uint64_t tokens = structural | opens | closes | astart;
            // strings that need decoding (a backslash or a non-ASCII byte inside)
            uint64_t slow_opens = 0;
            for (uint64_t marks = (bs | hi) & instr & ~opens; marks;) {
                const uint32_t mb = (uint32_t)__builtin_ctzll(marks);
                const uint64_t ob = opens & mask_lt(mb);
                if (ob) {
                    slow_opens |= 1ull << (63 - __builtin_clzll(ob));
                } else if (last_open_idx != NONE && last_open_idx != last_marked) {
                    // the string opened in an earlier step: rewrite its token
                    wave_sync();
                    if (lane == 0) S.tok[last_open_idx] = (TK_OPENQ_SLOW << 24) | last_open_pos;
                    last_marked = last_open_idx;
                }
                const uint64_t nx = opens & ~mask_lt(mb + 1);
                marks = nx ? (marks & ~mask_lt((uint32_t)__builtin_ctzll(nx))) : 0ull;
            }
            if ((tokens >> lane) & 1ull) {
                // region keywords (an exact string: its closing quote follows the word):
                // the 16 bytes after the byte, from five LDS words.  Bytes past the
                // document cannot fake a match: a string that closes inside the
                // document puts its quote inside the compared span.
                const uint32_t a = (pos + 1u) & ~3u, sh = (pos + 1u) & 3u;
                const uint32_t w0 = ring32(a), w1 = ring32(a + 4u), w2 = ring32(a + 8u), w3 = ring32(a + 12u);
                const uint32_t w4 = ring32(a + 16u);
                const uint32_t x0 = __builtin_amdgcn_alignbyte(w1, w0, sh), x1 = __builtin_amdgcn_alignbyte(w2, w1, sh);
                const uint32_t x2 = __builtin_amdgcn_alignbyte(w3, w2, sh), x3 = __builtin_amdgcn_alignbyte(w4, w3, sh);
                (void)x3;
                uint32_t kw = c;
                kw = (x0 == 0x6174656du && x1 == 0x61746164u && (x2 & 0xFFu) == 0x22u) ? TK_KEY_META : kw;  // metadata"
                kw = (x0 == 0x74617473u && (x1 & 0xFFFFFFu) == 0x227375u) ? TK_KEY_STATUS : kw;          // status"
                kw = (x0 == 0x6562616cu && (x1 & 0xFFFFFFu) == 0x22736cu) ? TK_KEY_LABELS : kw;          // labels"
                kw = (x0 == 0x6f6e6e61u && x1 == 0x69746174u && x2 == 0x22736e6fu) ? TK_KEY_ANNOT : kw;  // annotations"
                const bool is_close = (closes >> lane) & 1ull, is_slow = (slow_opens >> lane) & 1ull;
                const bool is_open = (opens >> lane) & 1ull;
                const uint32_t code = is_close ? TK_CLOSEQ : is_slow ? TK_OPENQ_SLOW : is_open ? kw : c;
                S.tok[ntok + mbcnt64(tokens)] = (code << 24) | pos;
            }
            if (opens) {
                const uint32_t ob = 63u - (uint32_t)__builtin_clzll(opens);
                last_open_idx = ntok + popc64(tokens & mask_lt(ob));
                last_open_pos = b + ob;
                if ((slow_opens >> ob) & 1ull) last_marked = last_open_idx;
            }
            ntok += popc64(tokens);
          }
        }
    }
    if (str_par) status = GPUDIFF_TOK_SYNTAX;  // unterminated string
    if (ctl_in_string && status == GPUDIFF_TOK_OK) status = GPUDIFF_TOK_STRING;
    wave_sync();

    mark(0);
    // ------------------------------------------------------------ phase 2: tree building
    // Lane per token, 64 tokens per batch.  A token's level (containers open
    // before it) is an mbcnt of opens minus closes; its enclosing container is
    // the last open one level up before it: found with a ballot per level
    // present in the batch, or carried from earlier batches in a per-level LDS
    // table.  A quote is a key when the token two after it is ':' (lookahead),
    // so node ids are a ballot prefix count and every lane checks its token
    // against its predecessor on its own (the first failing token decides the
    // status, as the sequential grammar would stop there).
    struct LvlEnt {
        uint32_t id, info, base, cnt1;  // last open at this level: node id, kind/region/flags, level+1 nodes
                                        // before it; level+1 nodes so far
    };
    LvlEnt* const lvt = (LvlEnt*)lds;  // kMaxDepth entries (4080 B; the ring is free now)
    constexpr uint32_t LF_ARR = 1u, LF_META = 16u, LF_LAB = 32u, LF_ANN = 64u;  // info: is_arr | reg << 1 | flags
    uint32_t nn = 0;
    uint32_t meta_node = NONE, labels_node = NONE, annot_node = NONE;
    bool labels_ok = true, annot_ok = true, has_status = false;
    uint32_t max_depth = 0;
    if (status == GPUDIFF_TOK_OK) {
        for (uint32_t q = lane; q < kMaxDepth; q += 64) lvt[q] = LvlEnt{0u, 0u, 0u, 0u};
        lds_order();
        int32_t lvl_c = 0;                   // level at the batch start
        uint32_t pc1 = 0, pc2 = 0, pc3 = 0;  // codes of the three tokens before the batch (0: none)
        uint32_t pp1 = 0, pp2 = 0, pp3 = 0;  // ... and their positions
        // tokens two batches deep in registers: a batch needs the next one's first two (lookahead), and the load of
        // the batch after that is issued a whole batch before it is used
        uint32_t t_cur = lane < ntok ? S.tok[lane] : 0u;
        uint32_t t_nxt = 64u + lane < ntok ? S.tok[64u + lane] : 0u;
        for (uint32_t tb = 0; tb < ntok; tb += 64) {
            const bool live = tb + lane < ntok;
            const uint32_t t = t_cur;
            const uint32_t t_far = tb + 128u + lane < ntok ? S.tok[tb + 128u + lane] : 0u;
            const uint32_t code = t >> 24;
            const uint32_t tn0 = rdlane(t_nxt, 0), nx0 = tn0 >> 24, nx1 = rdlane(t_nxt, 1) >> 24;
            t_cur = t_nxt;
            t_nxt = t_far;
            const uint32_t cp1 = wave_shr1(code, pc1), cp2 = wave_shr1(cp1, pc2), cp3 = wave_shr1(cp2, pc3);
            const uint32_t cn1 = wave_shl1(code, nx0), cn2 = wave_shl1(cn1, nx1);
            // positions of the key's quotes (two and three tokens back) and of a string's closing quote (next token)
            const uint32_t pos = t & POS_MASK;
            const uint32_t pm1 = wave_shr1(pos, pp1), pm2 = wave_shr1(pm1, pp2), pm3 = wave_shr1(pm2, pp3);
            const uint32_t pn1 = wave_shl1(pos, tn0 & POS_MASK);
            const bool is_o = live && (code == '{' || code == '[');
            const bool is_c = live && (code == '}' || code == ']');
            const bool is_qo = live && (code == '"' || (code >= TK_OPENQ_SLOW && code <= TK_KEY_ANNOT));
            const bool is_key = is_qo && cn2 == ':';
            const bool is_at = live && !is_o && !is_c && !is_qo && code != TK_CLOSEQ && code != ':' && code != ',';
            const bool is_node = is_o || is_at || (is_qo && !is_key);
            const uint64_t m_o = ballot(is_o), m_c = ballot(is_c), m_node = ballot(is_node);
            const int32_t lvl = lvl_c + (int32_t)mbcnt64(m_o) - (int32_t)mbcnt64(m_c);
            const uint32_t id = nn + mbcnt64(m_node);
            const bool empty = is_o && cn1 == (code == '{' ? (uint32_t)'}' : (uint32_t)']');
            // per-lane results of the level loop
            uint32_t e_id = NONE, e_info = 0u, my_info = code == '[' ? LF_ARR : 0u, my_base = 0u, comp = 0u, reg = R_NONE;
            // (flags carried across the level loop as 0/1 words: a loop-carried bool became a lane mask merged with
            // exec by three scalar instructions an iteration)
            uint32_t bad_lab = 0u, bad_ann = 0u;
            const int32_t lmin = (int32_t)wave_min_u32(live ? (uint32_t)(lvl + 0x40000000) : 0x7FFFFFFFu) - 0x40000000;
            const int32_t lmax = (int32_t)wave_max(live ? (uint32_t)(lvl + 0x40000000) : 0u) - 0x40000000;
            // levels of enclosing containers (lmin - 1 ..) and of this batch's opens (.. lmax)
            const int32_t lo = max(lmin - 1, 0), hi = min(lmax, (int32_t)kMaxDepth - 1);
            const uint64_t m_live = ballot(live);
            for (int32_t L = lo; L <= hi; L++) {
                const bool at_l = is_o && lvl == L;
                const bool at1 = live && lvl == L + 1;
                // the level masks as compare masks ANDed on the scalar unit (a ballot of a combined predicate
                // re-materialised it in a VGPR and compared it again: two vector instructions a ballot)
                const uint64_t eq0 = __builtin_amdgcn_uicmp((uint32_t)lvl, (uint32_t)L, 32);       // ICMP_EQ
                const uint64_t eq1 = __builtin_amdgcn_uicmp((uint32_t)lvl, (uint32_t)(L + 1), 32);
                const uint64_t m_ol = m_o & eq0, m_ch = m_node & eq1;
                if (!m_ol && !(m_live & eq1)) continue;
                LvlEnt st = lvt[L];
                const uint32_t nb = st.cnt1 + mbcnt64(m_ch);  // level-(L+1) nodes before this token
                if (at_l) my_base = nb;
                const uint64_t below = m_ol & mask_lt(lane);
                const uint32_t e = below ? 63u - (uint32_t)__builtin_clzll(below) : lane;
                const uint32_t x_id = shfl32(id, e), x_info = shfl32(my_info, e), x_base = shfl32(my_base, e);
                // the parent of this level's tokens (selects; the depth tests are uniform: L is a scalar)
                const uint32_t p_id = below ? x_id : st.id, p_info = below ? x_info : st.info;
                const uint32_t p_base = below ? x_base : st.base;
                e_id = at1 ? p_id : e_id;
                e_info = at1 ? p_info : e_info;
                {
                    const bool nd = at1 & is_node;
                    const bool p_arr = (p_info & LF_ARR) != 0u;
                    const uint32_t preg = (p_info >> 1) & 7u;
                    const uint32_t depth = (uint32_t)L + 1u;
                    const uint32_t comp_n = p_arr ? nb - p_base : ((tb + lane - 3u) | KEYBIT);
                    uint32_t reg_n, fl = 0u;
                    bool bl = false, ba = false;
                    if (depth == 1u) {
                        const bool km = cp3 == TK_KEY_META;
                        reg_n = km ? R_META : code == 'n' ? R_NONE : cp3 == TK_KEY_STATUS ? R_STATUS : R_SPEC;
                        fl = (km & (code == '{')) ? LF_META : 0u;
                    } else {
                        // metadata's members (labels / annotations objects), their members, anything below them
                        const bool c2 = (depth == 2u) & !p_arr & ((p_info & LF_META) != 0u);
                        const bool c3l = !c2 & (depth == 3u) & ((p_info & LF_LAB) != 0u);
                        const bool c3a = !c2 & !c3l & (depth == 3u) & ((p_info & LF_ANN) != 0u);
                        const uint32_t f2 = cp3 == TK_KEY_LABELS ? LF_LAB : cp3 == TK_KEY_ANNOT ? LF_ANN : 0u;
                        fl = (c2 & (code == '{')) ? f2 : 0u;
                        const bool below_meta = (preg == R_LABELS) | (preg == R_ANNOT);
                        reg_n = c2 ? preg : c3l ? R_LABELS : c3a ? R_ANNOT : below_meta ? R_META : preg;
                        bl = c3l & !is_qo;
                        ba = c3a & !is_qo;
                    }
                    comp = nd ? comp_n : comp;
                    reg = nd ? reg_n : reg;
                    bad_lab = nd ? (uint32_t)bl : bad_lab;
                    bad_ann = nd ? (uint32_t)ba : bad_ann;
                    my_info = nd ? ((code == '[' ? LF_ARR : 0u) | (reg_n << 1) | fl) : my_info;
                }
                // the table entry for level L
                if (m_ol) {
                    const uint32_t last = 63u - (uint32_t)__builtin_clzll(m_ol);
                    st.id = rdlane(id, last);
                    st.info = rdlane(my_info, last);
                    st.base = rdlane(my_base, last);
                }
                st.cnt1 += popc64(m_ch);
                if (m_ch) max_depth = max(max_depth, (uint32_t)L + 1u);
                lvt[L] = st;  // every lane: the same 16 bytes to one address (no exec-mask branch)
                lds_order();
            }
            // grammar: each token against its predecessor (cp1; 0 before the first token)
            const bool earr = e_info & LF_ARR;
            const bool p_qo = (cp1 == '"') | ((cp1 >= TK_OPENQ_SLOW) & (cp1 <= TK_KEY_ANNOT));
            const bool p_end = (cp1 == TK_CLOSEQ) | (cp1 == '}') | (cp1 == ']') |
                               ((cp1 != 0u) & !p_qo & (cp1 != '{') & (cp1 != '[') & (cp1 != ':') & (cp1 != ','));
            // the first failing check per token class, as selects (the grammar of a sequential parser)
            const bool first_tok = tb + lane == 0u;
            const uint32_t e_key = !((cp1 == '{') | ((cp1 == ',') & !earr)) ? GPUDIFF_TOK_SYNTAX
                                   : code == TK_OPENQ_SLOW                  ? GPUDIFF_TOK_KEY
                                                                            : 0u;
            const uint32_t e_node = !((cp1 == ':') | (cp1 == '[') | ((cp1 == ',') & earr)) ? GPUDIFF_TOK_SYNTAX
                                    : (is_o & !empty & (lvl >= (int32_t)kMaxDepth))          ? GPUDIFF_TOK_DEPTH
                                    : id + 3u > ncap                                        ? GPUDIFF_TOK_SIZE
                                                                                            : 0u;
            const bool bad_p = code == ':'   ? cp1 != TK_CLOSEQ
                               : code == ',' ? !p_end
                               : code == '}' ? !((cp1 == '{') | (p_end & !earr))
                               : code == ']' ? !((cp1 == '[') | (p_end & earr))
                                             : false;
            const uint32_t err = !live      ? 0u
                                 : first_tok ? (code != '{' ? GPUDIFF_TOK_SYNTAX : 0u)
                                 : lvl <= 0  ? GPUDIFF_TOK_SYNTAX  // after the root closed
                                 : is_key    ? e_key
                                 : is_node   ? e_node
                                 : bad_p     ? GPUDIFF_TOK_SYNTAX
                                             : 0u;
            const uint64_t m_err = ballot(err != 0u);
            const uint64_t upto = m_err ? mask_lt((uint32_t)__builtin_ctzll(m_err)) : ~0ull;
            // node records (the root: no parent, no key, never a leaf)
            {
                // every lane stores: a token that makes no node here writes slot ncap - 1, which no node uses
                const bool wr = is_node & (((upto >> lane) & 1ull) != 0ull) & (id < ncap);
                const uint32_t wid = wr ? id : ncap - 1u;
                const uint32_t leaf = (is_o & empty) ? NI_LEAF | (code == '{' ? GPUDIFF_TAG_EOBJ : GPUDIFF_TAG_EARR)
                                      : is_qo ? NI_LEAF | NI_STR | GPUDIFF_TAG_STR | (code == TK_OPENQ_SLOW ? NI_SLOW : 0u)
                                      : is_at ? NI_LEAF | NI_ATOM
                                              : 0u;
                const uint32_t info = tb + lane == 0u ? R_NONE << NI_REG_SHIFT
                                                      : (reg << NI_REG_SHIFT) | leaf | ((uint32_t)lvl << NI_DEPTH_SHIFT);
                S.rec[wid] = make_uint4(tb + lane == 0u ? NONE : e_id, comp, tb + lane, info);
                if constexpr (MODE == kModeEncode) {
                    // for phase 3a: a member's key span, a leaf's value positions (its slot until 3a fills it)
                    S.skey[(comp & KEYBIT) ? wid : ncap - 1u] = ((uint64_t)(pm2 - pm3 - 1u) << 32) | (pm3 + 1u);
                    S.val[wid] = ((uint64_t)pn1 << 32) | pos;
                }
            }
            const uint64_t ok_node = m_node & upto;
            const uint64_t m_meta = ballot(is_node & (lvl == 1) & (cp3 == TK_KEY_META) & (code == '{')) & upto;
            const uint64_t m_lab = ballot(is_node & ((my_info & LF_LAB) != 0u)) & upto;
            const uint64_t m_ann = ballot(is_node & ((my_info & LF_ANN) != 0u)) & upto;
            if (m_meta) meta_node = rdlane(id, 63u - (uint32_t)__builtin_clzll(m_meta));
            if (m_lab) labels_node = rdlane(id, 63u - (uint32_t)__builtin_clzll(m_lab));
            if (m_ann) annot_node = rdlane(id, 63u - (uint32_t)__builtin_clzll(m_ann));
            if (ballot(is_node & (lvl == 1) & (cp3 == TK_KEY_STATUS)) & upto) has_status = true;
            if (ballot(bad_lab != 0u) & upto) labels_ok = false;
            if (ballot(bad_ann != 0u) & upto) annot_ok = false;
            nn += popc64(ok_node);
            if (m_err) {
                status = rdlane(err, (uint32_t)__builtin_ctzll(m_err));
                break;
            }
            lvl_c += (int32_t)popc64(m_o) - (int32_t)popc64(m_c);
            const uint32_t kend = min(64u, ntok - tb);
            const uint32_t o1 = pc1, o2 = pc2, q1 = pp1, q2 = pp2;
            pc1 = rdlane(code, kend - 1u);
            pc2 = kend >= 2u ? rdlane(code, kend - 2u) : o1;
            pc3 = kend >= 3u ? rdlane(code, kend - 3u) : kend == 2u ? o1 : o2;
            pp1 = rdlane(pos, kend - 1u);
            pp2 = kend >= 2u ? rdlane(pos, kend - 2u) : q1;
            pp3 = kend >= 3u ? rdlane(pos, kend - 3u) : kend == 2u ? q1 : q2;
        }
        if (status == GPUDIFF_TOK_OK && (ntok == 0u || lvl_c != 0)) status = GPUDIFF_TOK_SYNTAX;
    }
    wave_sync();

    if constexpr (MODE == kModeMarshal) {
#include "marshal_phases.inc"
    }
    if constexpr (MODE == kModeRollup) {
#include "rollup_phases.inc"
    }
    if constexpr (MODE == kModeNegotiate) {
#include "negotiate_phases.inc"
    }

    const uint64_t seed = slots ? ((slots[links[doc_i].slot].flags >> 8) & 0xFFu) : D.seed;
    mark(1);
    // which leaves the blob encodes, and which nodes its path table lists (phases 3a and 5)
    auto region_of = [&](uint32_t w) -> uint32_t {  // 1 spec, 2 status, 0 not encoded (selects, no branches)
        const uint32_t reg = (w >> NI_REG_SHIFT) & 7u;
        const bool sp = (reg == R_SPEC) | ((reg == R_LABELS) & labels_ok) | ((reg == R_ANNOT) & annot_ok);
        const uint32_t r = sp ? 1u : reg == R_STATUS ? 2u : 0u;
        return (w & NI_LEAF) ? r : 0u;
    };
    // path-table nodes: the region leaves and their ancestors but the root -- every container of the spec / status
    // subtrees, and metadata, metadata.labels and metadata.annotations when label / annotation leaves are encoded
    const bool lab_in = status == GPUDIFF_TOK_OK && labels_node != NONE && labels_ok && !(S.rec[labels_node].w & NI_LEAF);
    const bool ann_in = status == GPUDIFF_TOK_OK && annot_node != NONE && annot_ok && !(S.rec[annot_node].w & NI_LEAF);
    const bool meta_in = lab_in || ann_in;
    auto in_tab = [&](uint32_t i, uint32_t w) -> bool {
        const uint32_t reg = (w >> NI_REG_SHIFT) & 7u;
        return (region_of(w) != 0u) | (!(w & NI_LEAF) & ((reg == R_SPEC) | (reg == R_STATUS))) |
               ((i == meta_node) & meta_in) | ((i == labels_node) & lab_in) | ((i == annot_node) & ann_in);
    };
    // phase 5's sizes: spec / status leaves, their arena bytes, path-table nodes and their key bytes
    uint32_t n_ls = 0, n_lt = 0, n_as = 0, n_at = 0, n_nt = 0, n_kb = 0;
    // small documents: phase 3a also counts the nodes per depth and leaves each node's hash inputs in LDS (key bytes'
    // offset or array index; parent, depth, key length), so phase 3b orders and hashes them without reloading records
    bool small = nn <= kLdsHash && max_depth < 32u;
    uint32_t* const h32 = (uint32_t*)lds;           // nodes per depth
    uint32_t* const c32 = (uint32_t*)(lds + 128);   // depth cursors
    // hin: x = key offset or index; y = parent | depth << 8 | key << 13 | region << 14 | klen << 16 | path-table
    // node << 21 | string << 22 | decoded string << 23
    uint2* const hin = (uint2*)(lds + 256);
    uint16_t* const ord16 = (uint16_t*)(lds + 2304);
    constexpr uint32_t kStage = 2304;               // phase 3a's decoded strings are staged from here
    if (small && lane < 32u) h32[lane] = 0u;
    lds_order();
    // ------------------------------------------------------------ phase 3a: values (lane per node)
    if (status == GPUDIFF_TOK_OK) {
        uint32_t err = GPUDIFF_TOK_OK, nslow = 0, natom = 0;
        // two dependent rounds of loads per 64 nodes, each issued for every lane before any is waited for: the
        // record with the key span and value positions the tree phase left beside it; 16 bytes at the value and 8
        // at a root key.
        // Strings that need decoding (an escape, a non-ASCII byte) are decoded after the batch, one at a time by
        // the whole wave: their raw bytes staged into LDS with coalesced loads, then unescaped from there by lane 0 (a
        // lane's byte-by-byte loop over global memory paid a dependent round trip per byte -- config3's
        // Deployments carry one such 50-byte command string each, profiles/r05f)
        for (uint32_t i0 = 1; i0 < nn; i0 += 64) {
            const uint32_t i = i0 + lane;
            const bool live = i < nn;
            // no per-lane branches in this loop: every lane loads (a lane past the nodes reads node 0's words) and
            // every lane stores (what a lane keeps nothing of goes to node 0's slots, the root's, which no later
            // phase reads; list entries past the lists go to slot ncap - 1, never a node)
            const uint32_t ii = live ? i : 0u;
            const uint4 r0 = S.rec[ii];
            const uint64_t ks = S.skey[ii], pv = S.val[ii];  // the tree phase's key span and value positions
            const uint4 r = live ? r0 : make_uint4(0u, 0u, 0u, 0u);
            const uint32_t rg = live ? region_of(r.w) : 0u;
            const bool tb = live & in_tab(i, r.w);
            const bool key = live & ((r.y & KEYBIT) != 0u), leaf = live & ((r.w & NI_LEAF) != 0u);
            const bool str = leaf & ((r.w & NI_STR) != 0u), atom = leaf & ((r.w & NI_ATOM) != 0u);
            const bool slow = str & ((r.w & NI_SLOW) != 0u);
            const uint32_t kop = key ? (uint32_t)ks - 1u : 0u;
            const uint32_t kcp = key ? kop + 1u + (uint32_t)(ks >> 32) : 0u;
            const uint32_t vop = (str | atom) ? (uint32_t)pv : 0u, vcp = (str | atom) ? (uint32_t)(pv >> 32) : 0u;
            uint64_t w0, w1;
            ld16u(d + vop + (str ? 1u : 0u), &w0, &w1);
            const uint64_t kw = ld8u(d + kop + 1u);
            // the list probe of the informer's decoder (json.cpp decodes_as_list): a root key equal to "items" under
            // ASCII case folding (a non-ASCII key is a slow key: TOK_KEY)
            const bool items = key & (r.x == 0u) & (kcp - kop - 1u == 5u) & ((kw & 0xDFDFDFDFDFull) == 0x534D455449ull);
            err = items ? GPUDIFF_TOK_LIST : err;
            uint32_t atag = r.w & NI_TAG;
            uint64_t av = 0;
            const bool aslow = parse_atom_fast(w0, w1, len - vop, &atag, &av) != 0u;
            const bool store0 = leaf & !slow & !items;
            const bool slow_atom = store0 & atom & aslow;  // parsed after the loop
            const bool store = store0 & !slow_atom;
            const uint32_t sl = vcp - vop - 1u;
            // the value's first 8 bytes (a long string's tail goes to the arena in phase 5)
            const uint64_t sv = sl >= GPUDIFF_INLINE_MAX ? w0 : sl ? (w0 & (~0ull >> (64u - 8u * sl))) : 0ull;
            const uint32_t tag = atom ? atag : r.w & NI_TAG;
            const uint32_t mlen = str ? sl : ((tag == GPUDIFF_TAG_INT) | (tag == GPUDIFF_TAG_FLOAT)) ? 8u : 0u;
            const uint64_t v = str ? sv : atom ? av : 0ull;
            S.val[store ? i : 0u] = v;
            S.meta[store ? i : 0u] = (mlen << 3) | tag;
            if (small) {
                const uint32_t dep = (r.w >> NI_DEPTH_SHIFT) & 0xFFu, kl = kcp - kop - 1u;
                atomicAdd(&h32[live ? dep : 31u], live ? 1u : 0u);
                hin[ii] = make_uint2(key ? kop + 1 : r.y, r.x | (dep << 8) | (key ? (1u << 13) | ((kl & 31u) << 16) : 0u) |
                                                              (rg << 14) | (tb ? 1u << 21 : 0u) | (str ? 1u << 22 : 0u) |
                                                              (slow ? 1u << 23 : 0u));
                // for phase 5 (the sort area is free up to kLdsSort)
                S.sidx[(str & (nn <= kRank + 1u)) ? i : 0u] = vop;
            }
            if (ballot(key && kcp - kop - 1 > 27u)) small = false;  // keys hashed from registers: <= 27 bytes
            // the blob's sizes (phase 5), counted here where every operand is in registers (wave totals, scalar)
            const uint32_t a = store ? meta_arena((mlen << 3) | tag) : 0u;
            n_ls += popc64(ballot(rg == 1u));
            n_lt += popc64(ballot(rg == 2u));
            n_nt += popc64(ballot(tb));
            n_as += wave_sum(rg == 1u ? a : 0u);
            n_at += wave_sum(rg == 2u ? a : 0u);
            n_kb += wave_sum(tb && key ? kcp - kop - 1 : 0u);
            // strings that need decoding and atoms the window did not decide: listed for after the loop, the strings
            // from the front of the depth-order area, the atoms from its back, each with its value's token positions
            // in the hash area (both free until phase 3b)
            const uint64_t sm = ballot(slow), am = ballot(slow_atom);
            const uint32_t qs = nslow + mbcnt64(sm), qa = nn - 1u - (natom + mbcnt64(am));
            const uint32_t q = slow ? qs : slow_atom ? qa : ncap - 1u;
            S.order[q] = i;
            S.h[q] = slow ? ((uint64_t)rg << 56) | ((uint64_t)vcp << 32) | vop : (uint64_t)vop;  // positions < 2^24
            nslow += popc64(sm);
            natom += popc64(am);
        }
        if (nslow | natom) wave_sync();
        // atoms: a lane each, from a 32-byte window
        for (uint32_t j0 = 0; j0 < natom; j0 += 64) {
            const uint32_t j = j0 + lane;
            if (j < natom) {
                const uint32_t q = nn - 1u - j;
                const uint32_t i = S.order[q], aop = (uint32_t)S.h[q];
                uint64_t w0, w1, w2, w3;
                ld32u(d + aop, d + len + kTokSlack, w0, w1, w2, w3);
                uint32_t tag = GPUDIFF_TAG_NULL;
                uint64_t v = 0;
                const uint32_t e = parse_atom_win(d + aop, d + len, w0, w1, w2, w3, &tag, &v);
                if (e) {
                    err = e;
                } else {
                    S.val[i] = v;
                    S.meta[i] = (((tag == GPUDIFF_TAG_INT || tag == GPUDIFF_TAG_FLOAT) ? 8u : 0u) << 3) | tag;
                }
            }
        }
        // strings: one at a time by the wave (the next entry's loads issued while this one decodes)
        uint32_t ni = nslow ? S.order[0] : 0u;
        uint64_t npos = nslow ? S.h[0] : 0ull;
        for (uint32_t j = 0; j < nslow; j++) {
            const uint32_t i = rdlane(ni, 0), sop = rdlane((uint32_t)npos, 0), hi = rdlane((uint32_t)(npos >> 32), 0);
            const uint32_t scp = hi & 0xFFFFFFu, rg = hi >> 24;
            if (j + 1u < nslow) {
                ni = S.order[j + 1u];
                npos = S.h[j + 1u];
            }
            const uint32_t raw = scp - sop - 1;  // bytes between the quotes
            uint8_t* const dst = S.str + sop + 1;
            const uint32_t ob = (raw + 16u) & ~15u;  // the decoded bytes' offset in the staging area (<= raw of them)
            int dl;
            uint64_t h8 = 0;
            if (ob + raw + 16u <= kLdsPerWave - kStage) {
                // the raw bytes and the closing quote into LDS (16 B a lane, up to 1 KiB a step; a \u escape never
                // reads past the quote: its fourth digit position holds it), unescaped there by lane 0, then the
                // decoded bytes copied out by the wave
                uint8_t* const st = lds + kStage;
                const uint8_t* const sp = d + sop + 1;
                for (uint32_t o = 16u * lane; o < raw + 1u; o += 1024u) {
                    const uint64_t a0 = ld8u(sp + o), a1 = ld8u(sp + o + 8u);
                    *(uint64_t*)(st + o) = a0;
                    *(uint64_t*)(st + o + 8u) = a1;
                }
                lds_order();
                // the common case by the whole wave, a lane per byte: only ASCII bytes and the escapes \" \\ \/ \b \f
                // \n \r \t -- an escaped byte maps to its character, its backslash emits nothing. Anything else (a \u
                // escape, a non-ASCII byte, an invalid escape) is left to lane 0's decode_string, which also decides
                // its errors (lane 0 alone paid ~14 scalar instructions a byte on the CU's one scalar unit)
                bool simple = true;
                uint32_t outn = 0, carry = 0;
                for (uint32_t o = 0; o < raw; o += 64u) {
                    const uint32_t p = o + lane;
                    const bool in = p < raw;
                    const uint32_t c = in ? st[p] : 0x20u;
                    const uint64_t bs = ballot(in & (c == '\\'));
                    uint64_t esc = carry;  // byte 0 of this chunk escaped by the previous chunk's last byte
                    carry = 0;
                    for (uint64_t m = bs; m; m &= m - 1) {
                        const uint32_t b = (uint32_t)__builtin_ctzll(m);
                        if ((esc >> b) & 1ull) continue;  // an escaped backslash escapes nothing
                        if (b == 63u) carry = 1;
                        else esc |= 1ull << (b + 1u);
                    }
                    const bool e = (esc >> lane) & 1ull;
                    const bool ok_e = (c == '"') | (c == '\\') | (c == '/') | (c == 'b') | (c == 'f') | (c == 'n') |
                                      (c == 'r') | (c == 't');
                    if (ballot(in & ((c >= 0x80u) | (e & !ok_e)))) {
                        simple = false;
                        break;
                    }
                    const bool emit = in & !((c == '\\') & !e);
                    const uint32_t mc = c == 'b' ? 8u : c == 'f' ? 12u : c == 'n' ? 10u : c == 'r' ? 13u : c == 't' ? 9u : c;
                    const uint64_t em = ballot(emit);
                    if (emit) st[ob + outn + mbcnt64(em)] = (uint8_t)(e ? mc : c);
                    outn += popc64(em);
                }
                lds_order();
                dl = (int)outn;
                if (!simple) {
                    dl = lane == 0 ? decode_string(st, st + raw, st + raw + 1u, st + ob) : 0;
                    lds_order();
                    dl = (int)rdlane((uint32_t)dl, 0);
                }
                if (dl > 0) {
                    for (uint32_t o = lane; o < (uint32_t)dl; o += 64u) dst[o] = st[ob + o];
                    h8 = *(const uint64_t*)(st + ob);
                }
                lds_order();
            } else {
                dl = lane == 0 ? decode_string(d + sop + 1, d + scp, d + len, dst) : 0;
                dl = (int)rdlane((uint32_t)dl, 0);
                if (dl > 0 && lane == 0) h8 = ld8u(dst);
            }
            if (dl < 0) {
                err = GPUDIFF_TOK_STRING;
            } else if (lane == 0) {
                const uint32_t sl = (uint32_t)dl;
                S.val[i] = sl >= GPUDIFF_INLINE_MAX ? h8 : sl ? (h8 & (~0ull >> (64u - 8u * sl))) : 0ull;
                S.meta[i] = (sl << 3) | GPUDIFF_TAG_STR;
            }
            if (dl > 0) {
                const uint32_t sa = meta_arena(((uint32_t)dl << 3) | GPUDIFF_TAG_STR);
                if (rg == 1u) n_as += sa;
                if (rg == 2u) n_at += sa;
            }
        }
        const uint32_t e = wave_max(err);  // any error: SYNTAX < NUMBER < ... all nonzero
        if (e) status = e;
    }

    mark(2);
    // ------------------------------------------------------------ phase 3b: path hashes by depth
    // nodes counting-sorted by depth (the order in LDS up to kLdsOrder nodes), then level by level a lane per
    // node: its record and key span (phase 3a) in one round trip, its parent's hash and its key bytes in the next
    // Up to kLdsHash nodes their hashes stay in LDS too (behind the order): a level reads its parents' hashes there,
    // with no fence on the global stores between levels
    const bool h_in_lds = nn <= kLdsHash;
    uint64_t* const hl = (uint64_t*)(lds + 2048 + 4 * kLdsHash);
    if (status == GPUDIFF_TOK_OK && nn > 1 && small) {
        // small documents: everything but the key bytes is in LDS -- the depth order from phase 3a's counts, then
        // level by level a lane per node: its inputs and its parent's hash from LDS, its key bytes from the JSON
        const uint32_t cnt = lane <= max_depth ? h32[lane] : 0u;
        const uint32_t inc = wave_incl_scan(cnt);
        if (lane <= max_depth) c32[lane] = inc - cnt;
        lds_order();
        for (uint32_t i0 = 1; i0 < nn; i0 += 64) {
            const uint32_t i = i0 + lane;
            if (i < nn) {
                const uint32_t p = atomicAdd(&c32[(hin[i].y >> 8) & 31u], 1u);
                ord16[p] = (uint16_t)i;
            }
        }
        lds_order();
        // level by level, 64 nodes of a level at a time, a lane per node: its inputs and its parent's hash from LDS,
        // its key bytes in registers -- loaded one step ahead (the next step's nodes are known from the order alone,
        // so their key loads fly while this step hashes)
        uint32_t dep = 1, j0 = 0, beg = 0;  // the step being hashed: depth, offset in its level, level start (depth 1
                                            // holds the root's members: never empty)
        auto next_step = [&](uint32_t& d_, uint32_t& j_, uint32_t& b_) {
            j_ += 64u;
            while (d_ <= max_depth && j_ >= rdlane(cnt, d_)) {
                b_ += rdlane(cnt, d_);
                d_++;
                j_ = 0;
            }
        };
        uint32_t ci = 0, cy = 0, cx = 0;
        uint64_t c0w = 0, c1w = 0, c2w = 0, c3w = 0;
        uint32_t clive = 0u;  // (0/1, not a loop-carried bool: see the tree phase)
        auto load_step = [&](uint32_t d_, uint32_t j_, uint32_t b_, uint32_t& i_, uint32_t& y_, uint32_t& x_,
                             uint64_t& w0_, uint64_t& w1_, uint64_t& w2_, uint64_t& w3_, uint32_t& live_) {
            // every lane loads (a lane past the step reads entry 0 and the document's first bytes): no branch
            live_ = ((d_ <= max_depth) & (j_ + lane < rdlane(cnt, min(d_, 31u)))) ? 1u : 0u;
            i_ = ord16[live_ ? b_ + j_ + lane : 0u];
            const uint2 in = hin[i_];
            y_ = live_ ? in.y : 0u;
            x_ = in.x;
            ld32u(d + ((in.y & (1u << 13)) ? in.x : 0u), d + len + kTokSlack, w0_, w1_, w2_, w3_);
        };
        load_step(dep, j0, beg, ci, cy, cx, c0w, c1w, c2w, c3w, clive);
        while (dep <= max_depth) {
            uint32_t nd = dep, nj = j0, nb = beg;
            next_step(nd, nj, nb);
            uint32_t ni, ny, nx;
            uint64_t n0w, n1w, n2w, n3w;
            uint32_t nlive;
            load_step(nd, nj, nb, ni, ny, nx, n0w, n1w, n2w, n3w, nlive);
            {
                // every lane hashes; a lane past the step writes slot 0 (the root's, read by nothing after this)
                const uint32_t par = cy & 0xFFu;
                const uint64_t hp = hl[par];
                const uint64_t ph = par == 0u ? seed : hp;
                // one XXH64 over the component's words, selected: 0x01 u32le(klen) key bytes | 0x02 u32le(index)
                // (hash_key_w / hash_index_w, tokdev.h)
                const bool isk = (cy & (1u << 13)) != 0u;
                const uint32_t kl = (cy >> 16) & 31u;
                const uint64_t W0 = isk ? 0x01ull | ((uint64_t)kl << 8) | (c0w << 40) : 0x02ull | ((uint64_t)cx << 8);
                const uint64_t W1 = isk ? (c0w >> 24) | (c1w << 40) : 0ull, W2 = isk ? (c1w >> 24) | (c2w << 40) : 0ull;
                const uint64_t W3 = isk ? (c2w >> 24) | (c3w << 40) : 0ull;
                const uint64_t hh = xxh64_small(ph, isk ? kl + 5u : 5u, W0, W1, W2, W3);
                // (LDS only: a small document's later phases read its hashes from hl -- phase 4 ranks them there,
                // phase 5's tiny path reads them there -- so they are not stored to the scratch's hash area too)
                static_assert(kRank + 1u >= kLdsHash, "a small document's phases 4-5 take the LDS (tiny) paths");
                const uint32_t wi = clive ? ci : 0u;
                hl[wi] = hh;
            }
            lds_order();  // the next level reads these hashes
            dep = nd;
            j0 = nj;
            beg = nb;
            ci = ni;
            cy = ny;
            cx = nx;
            c0w = n0w;
            c1w = n1w;
            c2w = n2w;
            c3w = n3w;
            clive = nlive;
        }
        wave_sync();  // phases 4-5 read S.h
    } else if (status == GPUDIFF_TOK_OK && nn > 1) {
        uint32_t* order = nn - 1 <= kLdsOrder ? (uint32_t*)(lds + 2048) : S.order;
        // counting sort of nodes by depth
        for (uint32_t i = lane; i <= kMaxDepth; i += 64) hist[i] = 0;
        wave_sync();
        for (uint32_t i0 = 1; i0 < nn; i0 += 64) {
            const uint32_t i = i0 + lane;
            if (i < nn) atomicAdd(&hist[(S.rec[i].w >> NI_DEPTH_SHIFT) & 0xFFu], 1u);
        }
        wave_sync();
        uint32_t run = 0;
        for (uint32_t d0 = 0; d0 <= kMaxDepth; d0 += 64) {
            const uint32_t dd = d0 + lane;
            const uint32_t cnt = dd <= kMaxDepth ? hist[dd] : 0u;
            const uint32_t inc = wave_incl_scan(cnt);
            if (dd <= kMaxDepth) cur[dd] = run + inc - cnt;
            run += rdlane(inc, 63);
        }
        wave_sync();
        for (uint32_t i0 = 1; i0 < nn; i0 += 64) {
            const uint32_t i = i0 + lane;
            if (i < nn) {
                const uint32_t dep = (S.rec[i].w >> NI_DEPTH_SHIFT) & 0xFFu;
                const uint32_t p = atomicAdd(&cur[dep], 1u);
                order[p] = i;  // nodes 1 .. nn - 1 (the root is not sorted): depths >= 1
            }
        }
        wave_sync();
        uint32_t beg = 0;
        for (uint32_t dep = 1; dep <= max_depth; dep++) {
            const uint32_t cnt = (uint32_t)__builtin_amdgcn_readfirstlane((int)hist[dep]);  // uniform: a scalar loop
            for (uint32_t j0 = 0; j0 < cnt; j0 += 64) {
                if (j0 + lane < cnt) {
                    const uint32_t i = order[beg + j0 + lane];
                    const uint4 r = S.rec[i];
                    const uint64_t ks = S.skey[i];
                    const uint64_t ph = r.x == 0 ? seed : h_in_lds ? hl[r.x] : S.h[r.x];
                    const uint64_t hh = (r.y & KEYBIT) ? hash_key(ph, d + (uint32_t)ks, (uint32_t)(ks >> 32))
                                                       : hash_index(ph, r.y);
                    S.h[i] = hh;
                    if (h_in_lds) hl[i] = hh;
                }
            }
            beg += cnt;
            if (h_in_lds) lds_order();  // the next level reads these hashes from LDS (in order within the wave)
            else wave_sync();
        }
        wave_sync();  // phases 4-5 read S.h
    }

    mark(3);
    // ------------------------------------------------------------ phase 4: sort keys, uniqueness
    const uint32_t ns = nn > 1 ? nn - 1 : 0;  // every node but the root
    uint64_t* skey = ns <= kLdsSort ? (uint64_t*)lds : S.skey;
    uint32_t* sidx = ns <= kLdsSort ? (uint32_t*)(lds + 8 * kLdsSort) : S.sidx;
    // up to kRank nodes: ranked straight from phase 3b's hashes in LDS into a u16 node order (the node records and
    // hash inputs stay in LDS for phase 5); more: the keys sorted with their node ids
    const bool rk = ns <= kRank && h_in_lds;  // (the hashes must be in LDS: nn <= kLdsHash)
    uint16_t* const ids16 = (uint16_t*)(lds + 2304);
    if (status == GPUDIFF_TOK_OK && ns) {
        const uint64_t root = seed & mask;
        if (rk) {
            // rank sort: a lane ranks its keys (up to two) against all ns keys, read by broadcast from LDS -- no
            // barrier, no divergent exchange; an equal key (a duplicate or a collision under the seed) or the root's
            // hash hands the document to the host, as below
            rank_sort(hl + 1, mask, ids16, ns, lane, root, status);
        } else {
            // (from LDS when phase 3b kept the hashes there: batch b reads hl[64b + 1 ..] before it writes sidx over
            // hl entries below 32 (b + 1), all read by earlier batches)
            for (uint32_t j = lane; j < ns; j += 64) {
                const uint64_t hj = h_in_lds ? hl[j + 1] : S.h[j + 1];
                lds_order();
                skey[j] = hj & mask;
                sidx[j] = j + 1;
            }
            wave_sync();
            // bitonic sort, all comparators ascending (flip + half-cleaners):
            // indices >= ns act as +inf and never move
            for (uint32_t kk = 2; (kk >> 1) < ns; kk <<= 1) {
                for (uint32_t dd = kk; dd >= 2; dd >>= 1) {
                    const bool flip = dd == kk;
#pragma unroll 1
                    for (uint32_t i = lane; i < ns; i += 64) {
                        const uint32_t j = flip ? (i ^ (kk - 1u)) : (i ^ (dd >> 1));
                        if (j > i && j < ns) {
                            const uint64_t a = skey[i], b = skey[j];
                            if (a > b) {
                                const uint32_t ia = sidx[i], ib = sidx[j];
                                skey[i] = b;
                                skey[j] = a;
                                sidx[i] = ib;
                                sidx[j] = ia;
                            }
                        }
                    }
                    wave_sync();
                }
            }
            // unique node hashes, none the root's: a parent hash in the path table
            // then names exactly one node (include/gpudiff_format.h)
            bool dup = false;
            for (uint32_t j = lane; j < ns; j += 64)
                if ((j && skey[j] == skey[j - 1]) || skey[j] == root) dup = true;
            if (ballot(dup)) status = GPUDIFF_TOK_HASH;
        }
    }

    mark(4);
    // ------------------------------------------------------------ phase 5: blob + path table
    o.n_nodes = nn;
    o.oflags = has_status ? GPUDIFF_OBJ_HAS_STATUS : 0u;
    if (status == GPUDIFF_TOK_OK) {
        // the sizes counted in phase 3a (sums over the nodes: the sort order does not change them)
        const uint32_t Ls = n_ls, Lt = n_lt, Nt = n_nt, KB = n_kb;
        const uint32_t ARs = (n_as + 15u) & ~15u;  // gpudiff_arena_bytes: each arena a multiple of 16
        const uint32_t ARt = (n_at + 15u) & ~15u;
        const uint64_t seg_s = seg_bytes(Ls, ARs), seg_t = seg_bytes(Lt, ARt);
        const uint64_t body = (seg_s + seg_t + 127u) & ~127ull;  // gpudiff_blob_body: 128-B line multiples
        const uint64_t tab = (24ull * Nt + KB + 127u) & ~127ull; // gpudiff_tab_bytes
        const uint64_t bytes = body + tab;
        uint64_t off = 0;
        if (lane == 0) off = atomicAdd(used, (unsigned long long)bytes);
        off = rdlane64(off, 0);
        if (off + bytes > space_cap) {
            status = GPUDIFF_TOK_SPACE;
        } else {
            uint8_t* blob = space + off;
            uint8_t* segp[2] = {blob, blob + seg_s};
            const uint32_t Lr[2] = {Ls, Lt};
            uint64_t* hs = (uint64_t*)(blob + body);
            uint64_t* phs = hs + Nt;
            uint64_t* cs = phs + Nt;
            uint8_t* keys = (uint8_t*)(cs + Nt);
            // zero the key area's pad (a segment's leaf records are 16 B each: no pad before the arena)
            for (uint32_t q = lane; q < tab - 24ull * Nt - KB; q += 64) keys[KB + q] = 0;
            if (lane < (body - seg_s - seg_t) / 16u) ((u32x4*)(blob + seg_s + seg_t))[lane] = u32x4{0u, 0u, 0u, 0u};
            const uint64_t root = seed & mask;
            const bool tiny = small && rk;  // phases 3a-4 left every input of this pass in LDS
            uint32_t rank[2] = {0, 0}, aoff[2] = {0, 0}, trank = 0, tko = 0;
            for (uint32_t j0 = 0; j0 < ns; j0 += 64) {
                const uint32_t j = j0 + lane;
                uint32_t rg = 0, i = 0, m = 0, ar = 0, kl = 0, kop = 0, idx = 0;
                bool t = false, isk = false, dec = false;
                uint64_t val = 0, ph = root, key = 0;
                uint32_t vop = 0;
                if (tiny) {
                    // a small document: the node's inputs, its hash and its parent's from LDS; its value, metadata
                    // and string position in one round of loads -- every lane loads (a lane past the order reads
                    // node 0's words and keeps nothing), so no branch
                    const bool jl = j < ns;
                    i = ids16[jl ? j : 0u];
                    const uint2 in = hin[i];
                    const uint32_t y = jl ? in.y : 0u;
                    rg = (y >> 14) & 3u;
                    t = (y >> 21) & 1u;
                    isk = (y >> 13) & 1u;
                    dec = (y >> 23) & 1u;
                    kop = in.x;
                    idx = in.x;
                    kl = t && isk ? (y >> 16) & 31u : 0u;  // key bytes only for path-table entries
                    const uint64_t hi_ = hl[i], hp = hl[y & 0xFFu];
                    key = hi_ & mask;
                    ph = (t && (y & 0xFFu)) ? hp & mask : root;
                    const uint32_t m_ = S.meta[i];
                    const uint64_t v_ = S.val[i];
                    const uint32_t p_ = S.sidx[i];
                    m = rg ? m_ : 0u;
                    val = rg ? v_ : 0ull;
                    vop = (rg && ((y >> 22) & 1u)) ? p_ : 0u;
                    ar = meta_arena(m);
                } else if (j < ns) {
                    i = rk ? ids16[j] : sidx[j];
                    const uint4 r = S.rec[i];
                    rg = region_of(r.w);
                    t = in_tab(i, r.w);
                    isk = (r.y & KEYBIT) != 0u;
                    dec = (r.w & NI_SLOW) != 0u;
                    idx = r.y;
                    key = rk ? (h_in_lds ? hl[i] : S.h[i]) & mask : skey[j];
                    // one round of loads for everything this node needs: its value, its parent's hash, its key span
                    // (the tree phase's, still in the sort-key area when the sort ran in LDS) and its string's position
                    uint64_t ks = 0;
                    if (rg) {
                        m = S.meta[i];
                        val = S.val[i];
                    }
                    if (t && r.x != 0) ph = S.h[r.x] & mask;
                    if (t && isk) {
                        if (ns <= kLdsSort) {
                            ks = S.skey[i];
                        } else {
                            const uint32_t kt = r.y & ~KEYBIT;
                            const uint32_t kp = S.tok[kt] & POS_MASK, kq = S.tok[kt + 1] & POS_MASK;
                            ks = ((uint64_t)(kq - kp - 1) << 32) | (kp + 1);
                        }
                    }
                    if (rg && (r.w & NI_STR)) vop = S.tok[r.z] & POS_MASK;
                    ar = meta_arena(m);
                    kop = (uint32_t)ks;
                    kl = (uint32_t)(ks >> 32);
                }
                uint32_t my_rank = 0, my_aoff = 0;
                for (uint32_t g = 0; g < 2; g++) {
                    const uint64_t bal = ballot(rg == g + 1);
                    const uint32_t inc = wave_incl_scan(rg == g + 1 ? ar : 0u);
                    my_rank = rg == g + 1 ? rank[g] + mbcnt64(bal) : my_rank;
                    my_aoff = rg == g + 1 ? aoff[g] + inc - ar : my_aoff;
                    rank[g] += popc64(bal);
                    aoff[g] += rdlane(inc, 63);
                }
                if (rg) {
                    const uint32_t g = rg - 1;
                    const uint32_t L = Lr[g];
                    uint8_t* sp8 = segp[g];
                    // vals u64 | keys u32 | metas u32 (include/gpudiff_format.h); keys masked to <= 32 bits
                    ((uint64_t*)sp8)[my_rank] = val;
                    ((uint32_t*)(sp8 + 8ull * L))[my_rank] = (uint32_t)key;
                    ((uint32_t*)(sp8 + 12ull * L))[my_rank] = m;
                }
                // the path-table entry: hash, parent hash, component (+ key bytes)
                const uint64_t tbal = ballot(t);
                const uint32_t kinc = wave_incl_scan(kl);
                const uint32_t ko = tko + kinc - kl;  // this entry's key bytes
                if (t) {
                    const uint32_t tr = trank + popc64(tbal & mask_lt(lane));
                    hs[tr] = key;
                    phs[tr] = ph;
                    cs[tr] = isk ? (((uint64_t)kl << 32) | ko) : (GPUDIFF_TAB_INDEX | idx);
                }
                trank += popc64(tbal);
                tko += rdlane(kinc, 63);
                // key bytes of the path-table entries and the long strings' tails (the bytes after the first 8,
                // which sit in the leaf record; 4-byte aligned arena offsets, the last dword zero past the value):
                // wave-cooperative flattened copies over every lane's span at once (one copy loop per string,
                // each a chain of dependent loads, cost this phase a quarter of K0's time, profiles/r05a)
                wave_copy_flat(t && kl, d + kop, kl, keys + ko);
                const bool tail = ar != 0u;
                const uint8_t* tsrc = nullptr;
                uint32_t* tdst = nullptr;
                uint32_t tlen = 0;
                if (tail) {
                    tsrc = (dec ? (S.str + vop + 1) : (d + vop + 1)) + GPUDIFF_INLINE_MAX;
                    tlen = (m >> 3) - GPUDIFF_INLINE_MAX;
                    tdst = (uint32_t*)(segp[rg - 1u] + 16ull * Lr[rg - 1u] + my_aoff);
                }
                wave_copy_dwords0(tail, tsrc, tlen, tdst);
            }
            // zero each arena's tail pad (its values end 4-byte aligned; the arena is a multiple of 16)
            for (uint32_t g = 0; g < 2; g++) {
                const uint32_t ARg = g ? ARt : ARs;
                uint32_t* tail = (uint32_t*)(segp[g] + 16ull * Lr[g] + aoff[g]);
                if (lane < (ARg - aoff[g]) / 4u) tail[lane] = 0u;
            }
            o.off = off;
            o.bytes = (uint32_t)bytes;
            o.spec_l = Ls;
            o.spec_ar = ARs;
            o.stat_l = Lt;
            o.stat_ar = ARt;
            o.n_tab = Nt;
        }
    }
#if defined(K0_PROBE_VALU) || defined(K0_PROBE_SALU)
    // timing-only builds (tools/sessions: the marginal cost of a vector / scalar instruction per document): 1024
    // extra instructions of one kind per document, 8 per iteration of a scalar loop
    {
        uint32_t pa = lane ^ status, pb = nn;
        uint32_t sa = __builtin_amdgcn_readfirstlane(pa), sb = __builtin_amdgcn_readfirstlane(pb);
        (void)sb;
        for (uint32_t q = 0; q < 128u + (nn >> 30); q++) {
#if defined(K0_PROBE_VALU)
            __asm__ volatile("v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n"
                             "v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1"
                             : "+v"(pa) : "v"(pb));
#else
            __asm__ volatile("s_mov_b32 %0, %1\n s_mov_b32 %0, %1\n s_mov_b32 %0, %1\n s_mov_b32 %0, %1\n"
                             "s_mov_b32 %0, %1\n s_mov_b32 %0, %1\n s_mov_b32 %0, %1\n s_mov_b32 %0, %1"
                             : "+s"(sa) : "s"(sb));
#endif
        }
        if ((pa ^ sa) == 0x9E3779B9u) o.n_nodes ^= 0x80000000u;  // never taken in practice: keeps the chains live
    }
#endif
    o.status = status;
    if (lane == 0) out[doc_i] = o;
    mark(5);
}

hipError_t k0_profile(int enable, uint64_t* out8) {
    if (out8) {
        hipError_t e = hipMemcpyFromSymbol(out8, HIP_SYMBOL(g_k0_prof), 8 * sizeof(unsigned long long));
        if (e != hipSuccess) return e;
    }
    unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_k0_prof), z, sizeof(z));
    if (e != hipSuccess) return e;
    return hipMemcpyToSymbol(HIP_SYMBOL(g_k0_prof_on), &enable, sizeof(int));
}

hipError_t launch_encode_docs(hipStream_t s, const TokDoc* docs, uint32_t n, const uint8_t* json, uint8_t* scratch,
                              uint8_t* space, uint64_t space_cap, unsigned long long* used, uint64_t mask,
                              TokOut* out, const DSlot* slots, const DocLink* links) {
    if (!n) return hipSuccess;
    const uint32_t blocks = (n + kWavesPerBlock - 1) / kWavesPerBlock;
    // 8 waves/SIMD (<= 64 VGPRs): unconstrained occupancy measured slower (round 2)
    k_encode_docs<8><<<blocks, 64 * kWavesPerBlock, 0, s>>>(docs, n, json, scratch, space, space_cap, used, mask, out,
                                                            slots, links);
    return hipGetLastError();
}

hipError_t launch_marshal_docs(hipStream_t s, const TokDoc* docs, uint32_t n, const uint8_t* json, uint8_t* scratch,
                               uint8_t* bodies, uint32_t mode, TokOut* out) {
    if (!n) return hipSuccess;
    const uint32_t blocks = (n + kWavesPerBlock - 1) / kWavesPerBlock;
    // 8 waves/SIMD (<= 64 VGPRs, a few spills): faster than 4, 5 or 6 waves on config3 documents (round 2 A/B)
    k_encode_docs<8, kModeMarshal><<<blocks, 64 * kWavesPerBlock, 0, s>>>(docs, n, json, scratch, bodies, 0, nullptr,
                                                                          (uint64_t)mode, out, nullptr, nullptr);
    return hipGetLastError();
}

hipError_t launch_rollup_docs(hipStream_t s, const TokDoc* docs, uint32_t n, const uint8_t* json, uint8_t* scratch,
                              RollOut* outs) {
    if (!n) return hipSuccess;
    const uint32_t blocks = (n + kWavesPerBlock - 1) / kWavesPerBlock;
    k_encode_docs<8, kModeRollup><<<blocks, 64 * kWavesPerBlock, 0, s>>>(docs, n, json, scratch, (uint8_t*)outs, 0,
                                                                        nullptr, 0, nullptr, nullptr, nullptr);
    return hipGetLastError();
}

hipError_t launch_negotiate_docs(hipStream_t s, const TokDoc* docs, uint32_t n, const uint8_t* json, uint8_t* scratch,
                                 NegOut* outs) {
    if (!n) return hipSuccess;
    const uint32_t blocks = (n + kWavesPerBlock - 1) / kWavesPerBlock;
    k_encode_docs<8, kModeNegotiate><<<blocks, 64 * kWavesPerBlock, 0, s>>>(docs, n, json, scratch, (uint8_t*)outs, 0,
                                                                           nullptr, 0, nullptr, nullptr, nullptr);
    return hipGetLastError();
}

}  // namespace gd
