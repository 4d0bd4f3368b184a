#!/usr/bin/env python3
"""Deployment splitter status roll-up benchmark:
cached Deployments aggregated per second by kernels K11 (roll-up mode of
k_encode_docs: typed-decode fields from the raw JSON) + K12 (grouping by the
kcp.dev/owned-by label, int32 sums, first-appearance order).

The population is what the splitter's informer caches after createLeafs
(pkg/reconciler/deployment/deployment.go:127-160): per root Deployment,
`--leaves` leaf Deployments labelled kcp.dev/cluster / kcp.dev/owned-by, every
object API-server JSON (~1.6 KB, the contrib/examples/deployment.yaml shape
with a 2-condition status), shuffled (the cache has no order).  The documents
are uploaded once (gpudiff_rbatch_create); a step is one K11 + K12 pass over
all of them, resident in HBM: the answer of the reconcile loop (:41-91) for
every root at once.

Reported: documents/s (value), K11's HBM GB/s (JSON read + 32 B per document
written) against the roofline, K12 time, checks (full size vs the C++
restatement, a sample vs the Python oracle), CPU baseline: the C++ restatement
(decode + group, decode timed) on a bounded sample.

usage: python bench.py --config rollup [--roots N] [--leaves L] [--steps K]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0


def log(*a):
    print("[rollup]", *a, file=sys.stderr, flush=True)


def run(args):
    import torch

    from kcp_amd import gpudiff as G
    from kcp_amd import synth as S

    torch.cuda.set_device(0)
    from bench import cpu_threads, host_cores
    ncpu = cpu_threads(*host_cores()[::2])  # affinity capped by the cgroup quota: the cores it can run at once
    threads = args.threads or max(1, min(16, ncpu))
    t0 = time.time()
    docs, roots = S.rollup_population(args.roots, args.leaves)
    N = len(docs)
    json_bytes = sum(len(d) for d in docs)
    log("%d Deployments (%d roots x (1 + %d leaves)), %.2f GB of JSON, generated in %.1f s" % (
        N, args.roots, args.leaves, json_bytes / 1e9, time.time() - t0))
    eng = G.Engine(device=0, timing=True)
    rb = eng.rbatch(docs)
    st0 = rb.stats()
    log("resident: scratch %.2f GB" % (st0.scratch_bytes / 1e9))

    # ---- warmup + correctness
    rb.run()
    res = rb.fetch()
    got = res.as_dict()
    from oracle import cpu_ref
    from oracle import rollup_oracle as R
    rd = cpu_ref.RollupDocs(docs)
    _, t_ref, want = rd.run(threads=threads)
    rd.close()
    full = dict(docs=N, groups=len(got["groups"]), device_docs=int((res.k11_status == 0).sum()),
                host_docs=int(res.n_host), host_grouped=bool(res.host_grouped),
                equal_to_cpp_restatement=got == want)
    log("full check:", json.dumps(full))
    # sample vs the Python oracle: the first 2000 documents as their own batch
    sdocs = docs[:2000]
    sres = eng.rollup_status(sdocs).as_dict()
    sw = R.rollup(sdocs)
    sample_ok = sres["doc_group"] == sw["doc_group"] and [g["sums"] for g in sres["groups"]] == \
        [g["sums"] for g in sw["groups"]] and [g["first_doc"] for g in sres["groups"]] == \
        [g["first_doc"] for g in sw["groups"]]
    log("sample vs oracle:", sample_ok)

    for _ in range(max(0, args.warmup - 1)):
        rb.run()
    eng.sync()
    rb.fetch()
    s_before = rb.stats()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        rb.run()
    eng.sync()
    dt = time.perf_counter() - t0
    rb.fetch()
    s_after = rb.stats()
    runs = s_after.runs - s_before.runs
    k11_ms = (s_after.k11_ms * s_after.runs - s_before.k11_ms * s_before.runs) / max(1, runs)
    k12_ms = (s_after.k12_ms * s_after.runs - s_before.k12_ms * s_before.runs) / max(1, runs)
    alg = json_bytes + 32 * N
    achieved = alg / (k11_ms * 1e-3) / 1e9
    value = N * args.steps / dt

    cpu = None
    if not args.no_cpu_baseline:
        n_s = min(args.cpu_sample, N)
        sdocs = docs[:n_s]
        rd = cpu_ref.RollupDocs(sdocs)
        sw_, sec, _ = rd.run(threads=ncpu, min_seconds=args.cpu_seconds)
        sw1, sec1, _ = rd.run(threads=1, min_seconds=args.cpu_seconds / 2)
        rd.close()
        cpu = dict(value=n_s * sw_ / sec, unit="docs/s", cores=ncpu, kind="port",
                   sample="first %d documents of this population (decode + group-by + int32 sums, decode timed), "
                          "%d sweeps in %.1f s; 1-core: %.0f docs/s; full population on %d threads: %.2f s" % (
                              n_s, sw_, sec, n_s * sw1 / sec1, threads, t_ref))
        log("cpu baseline:", json.dumps(cpu))

    line = {
        "metric": "Deployment status roll-up: cached Deployments aggregated/sec (K11+K12, SURVEY 8f row 4) "
                  "+ achieved HBM GB/s",
        "value": value, "unit": "docs/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "u8", "data": "synthetic (Deployments after createLeafs, API-server JSON, seeded counters)",
        "config": {"workload": "rollup: %d cached Deployments (%d roots x %d leaves + roots, %.2f GB JSON) resident "
                               "in HBM, one K11+K12 pass per step" % (N, args.roots, args.leaves, json_bytes / 1e9),
                   "groups": len(got["groups"])},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBPS, "traffic": None, "kernel": "k_encode_docs<rollup> (K11)",
                     "bytes_per_launch": alg, "avg_launch_ms": k11_ms, "launches_per_step": 1,
                     "limiter": "issue/latency: a wave per document walks ~15 dependent lane-per-node phases (DESIGN.md 6d); the HBM fraction is informational, not the bound"},
        "kernels_ms": {"k11": k11_ms, "k12_group": k12_ms},
        "cpu_baseline": cpu,
        "checks": {"full_size": full, "sample": dict(docs=len(sdocs), bit_exact_vs_oracle=sample_ok)},
    }
    rb.close()
    eng.close()
    from kcp_amd import gpudiff as _G
    line["build_id"] = _G.BUILD_ID  # the loaded library's source hash (kcp_amd/buildinfo.py)
    print(json.dumps(line), flush=True)
