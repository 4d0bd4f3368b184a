/*
 * gpudiff_synth.h -- seeded synthetic object populations for bench.py and
 * the GPU tests (NOT part of the drop-in boundary; libgpudiff_synth.so).
 *
 * Shapes follow SURVEY.md §8(d): ConfigMaps/Secrets (8 data keys, 64-512 B
 * values, 4 labels, 2 annotations, no status), Deployments
 * (contrib/examples/deployment.yaml of the reference plus server defaults and a
 * two-condition status), medium CRDs (~200 leaves, nested lists) and deep
 * list-heavy CRDs (300-3000 leaves, status lists of 64-1024 items).  Pairs are
 * keyed by logical cluster (rank-frequency Zipf 1.1, offset 10); B = A with
 * the metadata the predicates ignore rewritten and, for a seeded fraction, one
 * semantic mutation whose effect (spec / status) the generator records as
 * ground truth.  Every pair is a pure function of (seed, global pair index),
 * independent of rank count, chunking and threads.
 */
#ifndef GPUDIFF_SYNTH_H
#define GPUDIFF_SYNTH_H

#include <stddef.h>
#include <stdint.h>

#include "gpudiff_format.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct gpudiff_synth_cfg {
    uint64_t seed;
    uint64_t n_pairs;        /* whole population */
    uint32_t n_clusters;     /* logical clusters */
    float mutate_frac;
    float w_configmap, w_secret, w_deployment, w_crd, w_deep;  /* kind mix */
    uint32_t crd_leaves;     /* medium CRD target leaves (default 200) */
} gpudiff_synth_cfg;

/* ground truth bits per pair */
#define GPUDIFF_SYNTH_SPEC_MUT 0x1u
#define GPUDIFF_SYNTH_STATUS_MUT 0x2u
#define GPUDIFF_SYNTH_B_HAS_STATUS 0x4u

typedef struct gpudiff_synth gpudiff_synth;

/* plans the population and the LPT shard of `rank` among `world` ranks (clusters by pair count) */
/* the build ID of this library (the same content hash as gpudiff_build_id, kcp_amd/buildinfo.py) */
const char* gpudiff_synth_build_id(void);
int gpudiff_synth_open(const gpudiff_synth_cfg* cfg, int world, int rank, gpudiff_synth** out);
/* the same with the clusters LPT-packed by cluster_weight[n_clusters] (NULL = pair count), the rule of
 * gpudiff_shard_lpt: SURVEY.md §8(e) balances ranks by Σ B_pair (gpudiff_synth_cluster_bytes) */
int gpudiff_synth_open_ex(const gpudiff_synth_cfg* cfg, int world, int rank, const uint64_t* cluster_weight,
                          gpudiff_synth** out);
/* pairs per cluster (out[n_clusters]) */
int gpudiff_synth_cluster_sizes(const gpudiff_synth_cfg* cfg, uint64_t* out);
/* exact Σ B_pair (gpudiff_pair_compare_bytes of the encoded pair) of every cluster c with
 * c % stride == offset into out[c] (others untouched): encodes those clusters' pairs with `threads` host
 * threads (ranks split the work by stride = world, offset = rank, then sum the vectors) */
int gpudiff_synth_cluster_bytes(const gpudiff_synth_cfg* cfg, uint32_t stride, uint32_t offset, uint32_t threads,
                                uint64_t* out);
void gpudiff_synth_close(gpudiff_synth* s);
uint64_t gpudiff_synth_local_pairs(const gpudiff_synth* s);
uint64_t gpudiff_synth_local_clusters(const gpudiff_synth* s);
/* global pair index of local pair i */
uint64_t gpudiff_synth_global_index(const gpudiff_synth* s, uint64_t i);
/* the global pair index (= the encoded pair_id, u32) of every local pair, out[local_pairs] */
int gpudiff_synth_local_ids(const gpudiff_synth* s, uint32_t* out);

/* encodes local pairs [first, first+n) with `threads` host threads into
 * internal buffers; reports the pool bytes and leaves needed */
int gpudiff_synth_encode(gpudiff_synth* s, uint64_t first, uint64_t n, uint32_t threads, uint64_t* pool_bytes,
                         uint64_t* total_leaves);
/* copies the last encoded range out (row offsets relative to `pool`) and the
 * ground truth bits per pair */
int gpudiff_synth_copy_out(gpudiff_synth* s, uint8_t* pool, gpudiff_pair_row* rows, uint8_t* truth);
/* JSON text of local pair i (A then B); returns required sizes */
/* JSON of local pairs [first, first+n): A_i, B_i concatenated into one malloc'ed
 * buffer (free with gpudiff_synth_free_buf); offs[2n+1] byte offsets; truth[n]
 * optional ground-truth bits */
int gpudiff_synth_json_range(gpudiff_synth* s, uint64_t first, uint64_t n, uint32_t threads, uint8_t** buf,
                             uint64_t* offs, uint8_t* truth);
void gpudiff_synth_free_buf(uint8_t* buf);
int gpudiff_synth_json(gpudiff_synth* s, uint64_t i, char* a, size_t acap, size_t* alen, char* b, size_t bcap,
                       size_t* blen);

#ifdef __cplusplus
}
#endif
#endif
