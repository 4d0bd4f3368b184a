#!/usr/bin/env python3
"""API-negotiation update classifier benchmark (second
half): Update events classified per second by kernels K13 (negotiation mode of
k_encode_docs: typed-decode fields of both sides from the raw JSON) + K14 (the
controller.go:253-283 decision per pair).

The population is `--pairs` (old, new) Update events of APIResourceImport /
NegotiatedAPIResource objects (`--kind api`, the default), API-server JSON
(~1.2 KB each; kcp.dev labels, a CommonAPIResourceSpec with column
definitions, 1-3 status conditions), with the event mix of
kcp_amd.synth.negotiate_population; `--kind crd`: CustomResourceDefinition
events (~2.4 KB: an openAPIV3Schema, status conditions + acceptedNames +
storedVersions; kcp_amd.synth.crd_population); `--kind mixed`: both,
interleaved in one batch.  The documents are uploaded
once (gpudiff_nbatch_create); a step is one K13 + K14 pass over all of them,
resident in HBM.

Reported: pairs/s (value: a step = K13 + K14 + the actions' copy-back + the
host path for K13's deferrals, i.e. every pair classified inside the timed
step), the device-only rate beside it, K13's HBM GB/s (JSON read + 1184 B
(NegOut) per document written) against the roofline, K14 time, checks (every action vs the
generator's designed outcome, a sample vs the Python oracle), and the CPU
baseline: the product's Go-exact C++ host path (gpudiff_classify_updates_host,
typed decode of both sides + classification, decode timed) on every host CPU.

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


def run(args):
    import torch

    from kcp_amd import gpudiff as G
    from kcp_amd import synth as S

    t0 = time.time()
    kind = getattr(args, "kind", "api")
    if kind == "api":
        pairs, want = S.negotiate_population(args.pairs)
        kinds = [G.NEG_KIND_API] * len(pairs)
    elif kind == "crd":
        pairs, want = S.crd_population(args.pairs)
        kinds = [G.NEG_KIND_CRD] * len(pairs)
    else:
        pa, wa = S.negotiate_population(args.pairs // 2)
        pc, wc = S.crd_population(args.pairs - args.pairs // 2)
        pairs = [p for ab in zip(pa, pc) for p in ab] + pc[len(pa):]
        want = np.asarray([w for ab in zip(wa.tolist(), wc.tolist()) for w in ab] + wc.tolist()[len(pa):], np.int32)
        kinds = [k for _ in range(len(pa)) for k in (G.NEG_KIND_API, G.NEG_KIND_CRD)] + \
            [G.NEG_KIND_CRD] * (len(pc) - len(pa))
    N = len(pairs)
    json_bytes = sum(len(a) + len(b) for a, b in pairs)
    log("%d Update pairs, %.2f GB of JSON, generated in %.1f s" % (N, json_bytes / 1e9, time.time() - t0))
    torch.cuda.set_device(0)
    eng = G.Engine(device=0, timing=True)
    nb = eng.nbatch(pairs, kinds)
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
    sw = [NO.classify(a, b, k) for (a, b), k in zip(pairs[:n_s], kinds[:n_s])]
    t_or = time.perf_counter() - t1
    sample_ok = sw == got[:n_s].tolist()
    log("sample vs oracle:", sample_ok)

    for _ in range(max(0, args.warmup - 1)):
        nb.run()
        nb.fetch()
    s_before = nb.stats()
    torch.cuda.synchronize()
    # end to end: every step classifies every pair (K13 + K14, actions to the host, host path for deferrals)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        nb.run()
        acts = nb.fetch()
    dt = time.perf_counter() - t0
    steps_ok = bool(np.array_equal(acts, got))
    # device only: K13 + K14 back to back (deferred pairs left to a later fetch)
    t1 = time.perf_counter()
    for _ in range(args.steps):
        nb.run()
    eng.sync()
    dt_dev = time.perf_counter() - t1
    nb.fetch()
    s_after = nb.stats()
    runs = s_after.runs - s_before.runs
    k13_ms = (s_after.k13_ms * s_after.runs - s_before.k13_ms * s_before.runs) / max(1, runs)
    k14_ms = (s_after.k14_ms * s_after.runs - s_before.k14_ms * s_before.runs) / max(1, runs)
    alg = json_bytes + G.NEGOUT_BYTES * 2 * N
    achieved = alg / (k13_ms * 1e-3) / 1e9
    value = N * args.steps / dt

    cpu = None
    if not args.no_cpu_baseline:
        from bench import cpu_threads, host_cores
        T = cpu_threads(*host_cores()[::2])  # affinity capped by the cgroup quota
        n_c = min(N, 20 * args.cpu_sample)
        hp = G.HostPairs(pairs[:n_c], kinds[:n_c])
        hp.classify(threads=T)  # warm
        reps, t_c = 0, time.perf_counter()
        while True:
            ha = hp.classify(threads=T)
            reps += 1
            el = time.perf_counter() - t_c
            if el >= args.cpu_seconds:
                break
        reps1, t_c = 0, time.perf_counter()
        while True:
            hp.classify(threads=1)
            reps1 += 1
            el1 = time.perf_counter() - t_c
            if el1 >= args.cpu_seconds / 3:
                break
        cpu = dict(value=n_c * reps / el, unit="pairs/s", cores=T, kind="port",
                   sample="first %d pairs of this population through the product's Go-exact host path "
                          "(gpudiff_classify_updates_host: typed decode of both sides + classification, decode "
                          "timed), %d sweeps in %.1f s; agrees with the device: %s" % (
                              n_c, reps, el, bool(np.array_equal(ha, got[:n_c]))),
                   one_core=n_c * reps1 / el1, nproc=os.cpu_count(),
                   python_oracle_one_core=n_s / t_or)
        log("cpu baseline:", json.dumps(cpu))

    line = {
        "metric": "API-negotiation update classification: Update events classified/sec (K13+K14, SURVEY 8f row 4) "
                  "+ achieved HBM GB/s",
        "value": value, "unit": "pairs/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "u8", "data": "synthetic (%s Update pairs, seeded event mix)" % {
            "api": "APIResourceImport / NegotiatedAPIResource", "crd": "CustomResourceDefinition",
            "mixed": "APIResourceImport / NegotiatedAPIResource and CustomResourceDefinition"}[kind],
        "config": {"workload": "negotiate (kind %s): %d Update pairs (%.2f GB JSON) resident in HBM, one K13+K14 "
                               "pass per step" % (kind, N, json_bytes / 1e9)},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBPS, "traffic": None, "kernel": "k_encode_docs<negotiate> (K13)",
                     "bytes_per_launch": alg, "avg_launch_ms": k13_ms, "launches_per_step": 1,
                     "limiter": "issue/latency: a wave per document walks ~15 dependent lane-per-node phases (DESIGN.md 6e); the HBM fraction is informational, not the bound"},
        "kernels_ms": {"k13": k13_ms, "k14_classify": k14_ms},
        "device_only": {"pairs_per_s": N * args.steps / dt_dev, "ms_per_step": dt_dev / args.steps * 1e3,
                        "what": "K13 + K14 only; the deferred pairs' host path is outside this rate"},
        "n_host": int(s_after.n_host),
        "cpu_baseline": cpu,
        "checks": {"full_size": full, "sample": dict(pairs=n_s, bit_exact_vs_oracle=sample_ok),
                   "timed_steps_equal_first_run": steps_ok},
    }
    nb.close()
    eng.close()
    from kcp_amd import gpudiff as _G
    line["build_id"] = _G.BUILD_ID  # the loaded library's source hash (kcp_amd/buildinfo.py)
    print(json.dumps(line), flush=True)
