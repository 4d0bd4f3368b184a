#!/usr/bin/env python3
"""API-negotiation update classifier benchmark (second
half): Update events classified per second by kernels K13 (negotiation mode of
k_encode_docs: typed-decode fields of both sides from the raw JSON) + K14 (the
controller.go:253-283 decision per pair).

The population is `--pairs` (old, new) Update events of APIResourceImport /
NegotiatedAPIResource objects, API-server JSON (~1.2 KB each; kcp.dev labels, a
CommonAPIResourceSpec with column definitions, 1-3 status conditions), with the
event mix of kcp_amd.synth.negotiate_population.  The documents are uploaded
once (gpudiff_nbatch_create); a step is one K13 + K14 pass over all of them,
resident in HBM.

Reported: pairs/s (value), K13's HBM GB/s (JSON read + 944 B per document
written) against the roofline, K14 time, checks (every action vs the
generator's designed outcome, a sample vs the Python oracle), CPU baseline: the
Python oracle (one core) on a bounded sample.

usage: python bench.py --config negotiate [--pairs N] [--steps K]
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
    print("[negotiate]", *a, file=sys.stderr, flush=True)


_POOL_PAIRS = None


def _pool_work(k_T):
    from oracle import negotiate_oracle as NO
    k, T, n = k_T
    return [NO.classify(a, b) for a, b in _POOL_PAIRS[k:n:T]]


def _pool_baseline(pairs, n):
    """The oracle on every host thread (min(16, affinity) forked processes), wall-clock over n pairs."""
    import multiprocessing as mp
    global _POOL_PAIRS
    _POOL_PAIRS = pairs
    T = max(1, min(16, len(os.sched_getaffinity(0))))
    with mp.get_context("fork").Pool(T) as pool:
        pool.map(_pool_work, [(k, T, k + 1) for k in range(T)])  # workers up, oracle imported
        t = time.perf_counter()
        pool.map(_pool_work, [(k, T, n) for k in range(T)])
        dt = time.perf_counter() - t
    return n / dt, T, n


def run(args):
    import torch

    from kcp_amd import gpudiff as G
    from kcp_amd import synth as S

    t0 = time.time()
    pairs, want = S.negotiate_population(args.pairs)
    N = len(pairs)
    json_bytes = sum(len(a) + len(b) for a, b in pairs)
    log("%d Update pairs, %.2f GB of JSON, generated in %.1f s" % (N, json_bytes / 1e9, time.time() - t0))
    # CPU baseline on all host threads first: forked workers share the population, and the fork happens
    # before this process touches the GPU
    pool_cpu = None
    if not args.no_cpu_baseline:
        pool_cpu = _pool_baseline(pairs, min(N, 16 * args.cpu_sample))
        log("cpu baseline (pool): %.0f pairs/s on %d processes over %d pairs" % pool_cpu)
    torch.cuda.set_device(0)
    eng = G.Engine(device=0, timing=True)
    nb = eng.nbatch(pairs)
    st0 = nb.stats()
    log("resident: scratch %.2f GB" % (st0.scratch_bytes / 1e9))

    # ---- warmup + correctness
    nb.run()
    got = nb.fetch()
    n_host = int(nb.stats().n_host)
    full = dict(pairs=N, mismatches_vs_design=int((got != want).sum()), host_pairs=n_host,
                actions=np.bincount(got + 1, minlength=6).tolist())
    log("full check:", json.dumps(full))
    from oracle import negotiate_oracle as NO
    n_s = min(args.cpu_sample, N)
    t1 = time.perf_counter()
    sw = [NO.classify(a, b) for a, b in pairs[:n_s]]
    t_or = time.perf_counter() - t1
    sample_ok = sw == got[:n_s].tolist()
    log("sample vs oracle:", sample_ok)

    for _ in range(max(0, args.warmup - 1)):
        nb.run()
    eng.sync()
    nb.fetch()
    s_before = nb.stats()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        nb.run()
    eng.sync()
    dt = time.perf_counter() - t0
    nb.fetch()
    s_after = nb.stats()
    runs = s_after.runs - s_before.runs
    k13_ms = (s_after.k13_ms * s_after.runs - s_before.k13_ms * s_before.runs) / max(1, runs)
    k14_ms = (s_after.k14_ms * s_after.runs - s_before.k14_ms * s_before.runs) / max(1, runs)
    alg = json_bytes + 944 * 2 * N
    achieved = alg / (k13_ms * 1e-3) / 1e9
    value = N * args.steps / dt

    cpu = None
    if not args.no_cpu_baseline:
        v, T, n_p = pool_cpu
        cpu = dict(value=v, unit="pairs/s", cores=T, kind="port",
                   sample="first %d pairs of this population through oracle/negotiate_oracle.py (typed decode of "
                          "both sides + classification, decode timed) on %d forked processes, wall clock; "
                          "1-core: %.0f pairs/s over the first %d pairs" % (n_p, T, n_s / t_or, n_s))
        log("cpu baseline:", json.dumps(cpu))

    line = {
        "metric": "API-negotiation update classification: Update events classified/sec (K13+K14, SURVEY 8f row 4) "
                  "+ achieved HBM GB/s",
        "value": value, "unit": "pairs/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "u8", "data": "synthetic (APIResourceImport / NegotiatedAPIResource Update pairs, seeded event mix)",
        "config": {"workload": "negotiate: %d Update pairs (%.2f GB JSON) resident in HBM, one K13+K14 pass per step"
                               % (N, json_bytes / 1e9)},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBPS, "traffic": None, "kernel": "k_encode_docs<negotiate> (K13)",
                     "bytes_per_launch": alg, "avg_launch_ms": k13_ms, "launches_per_step": 1},
        "kernels_ms": {"k13": k13_ms, "k14_classify": k14_ms},
        "cpu_baseline": cpu,
        "checks": {"full_size": full, "sample": dict(pairs=n_s, bit_exact_vs_oracle=sample_ok)},
    }
    nb.close()
    eng.close()
    print(json.dumps(line), flush=True)
