#!/usr/bin/env python3
"""Headline benchmark: object-pair diffs/sec (whole node) + achieved HBM GB/s.

Workload (BASELINE.json configs[2], the metric's own configuration): 10M mixed
object pairs (40% ConfigMap/Secret, 40% Deployment, 20% medium CRD) across
100k logical clusters, 5% mutated, synthetic (seed 20211004+3).

Scaling (--scaling, default weak): pairs are independent and shard by logical
cluster with no data-path exchange, so per-GPU work is fixed -- at N GPUs the
node-wide population is N x the config (N x 10M pairs over N x 100k logical
clusters, same seed and mix) and each rank holds the LPT shard of whole
logical clusters assigned to it (~10M pairs, one config3-sized population per
GPU).  --scaling strong keeps the population fixed at the config's size and
splits it N ways instead.  Either way the pairs are encoded on the host with
the product encoder and are resident in HBM before timing.

A step = one diff pass of the hot path (K2 compare, K3 compaction, K4
changed-path merge-join, K5/K6 path emit) over the rank's resident pairs, plus
(N > 1) the RCCL all-gather of per-rank dirty counts and dirty pair IDs.

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 under
torch.distributed.run (one process per GPU).  Rank 0 prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md "Chip-level parameters")


def log(*a):
    print("[bench r%s]" % os.environ.get("RANK", "0"), *a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="config3", choices=["config1", "config2", "config3", "config4", "config5", "upsert", "rollup", "negotiate"],
                    help="config5 = watch replay through the device-resident object store (bench_replay.py); "
                         "upsert = the write path's request bodies, kernel K10 (bench_upsert.py); "
                         "rollup = the Deployment splitter's status roll-up, K11 + K12 (bench_rollup.py); "
                         "negotiate = the API-negotiation update classifier, K13 + K14 (bench_negotiate.py)")
    ap.add_argument("--docs", type=int, default=131072, help="upsert: documents resident in HBM")
    ap.add_argument("--roots", type=int, default=250000, help="rollup: root Deployments")
    ap.add_argument("--leaves", type=int, default=4, help="rollup: leaf Deployments per root")
    ap.add_argument("--batch", type=int, default=65536, help="config5: events per batch")
    ap.add_argument("--batches", type=int, default=40, help="config5: timed batches")
    ap.add_argument("--warmup-batches", type=int, default=4, help="config5: untimed batches")
    ap.add_argument("--encode", default="device", choices=["device", "host"],
                    help="config5: encode events on the GPU (K0, raw JSON up) or on the host")
    ap.add_argument("--pairs", type=int, default=0, help="override population size (default: the config's)")
    ap.add_argument("--clusters", type=int, default=0)
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="weak: per-GPU work fixed (node population = N x the config); "
                         "strong: the config's population split N ways")
    ap.add_argument("--chunk", type=int, default=262144)
    ap.add_argument("--threads", type=int, default=0, help="host encode threads (default min(16, cpus))")
    ap.add_argument("--sample", type=int, default=600, help="pairs checked bit-exact vs the oracle (JSON path)")
    ap.add_argument("--cpu-sample", type=int, default=20000, help="pairs in the CPU-baseline sample")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic-json", default="latest",
                    help="PMC traffic summary to attach as roofline.traffic (default: the newest committed "
                         "profiles/r*_pmc_summary.json, used only if it was measured on this same workload; "
                         "'none' to skip)")
    args = ap.parse_args()

    if args.config == "upsert":
        import bench_upsert
        args.sample = min(args.sample, 300)
        return bench_upsert.run(args)

    if args.config == "rollup":
        import bench_rollup

        return bench_rollup.run(args)
    if args.config == "negotiate":
        import bench_negotiate
        args.pairs = args.pairs or 500000
        args.cpu_sample = min(args.cpu_sample, 10000)
        return bench_negotiate.run(args)
    if args.config == "config5":
        import bench_replay
        args.sample = min(args.sample, 300)
        return bench_replay.run(args)

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log("note: --gpus %d but WORLD_SIZE %d; using WORLD_SIZE" % (args.gpus, world))

    import torch
    import torch.distributed as dist

    from kcp_amd import gpudiff as G
    from kcp_amd import synth as S

    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    stream = torch.cuda.current_stream(dev)
    ncpu = len(os.sched_getaffinity(0))
    threads = args.threads or max(1, min(16, ncpu))

    eng = G.Engine(device=local_rank, encode_threads=threads, stream=stream.cuda_stream, timing=True)
    base = S.make_cfg(args.config, n_pairs=args.pairs, n_clusters=args.clusters)
    mult = world if args.scaling == "weak" else 1
    cfg = S.make_cfg(args.config, n_pairs=base.n_pairs * mult, n_clusters=base.n_clusters * mult)
    pop = S.Population(cfg, world, rank)
    n = pop.n
    log("config %s: %d pairs / %d clusters total; this rank %d pairs / %d clusters; %d host threads" % (
        args.config, cfg.n_pairs, cfg.n_clusters, n, pop.n_clusters, threads))

    # ---------------- ingest: synthesize + encode on the host, stage, H2D, K1
    t_gen = time.time()
    first = pop.chunk(eng, 0, min(args.chunk, n), threads)
    per_pair = first.pool_bytes / max(1, min(args.chunk, n))
    margin = 1.15 if args.config != "config4" else 1.4
    pool_cap = int(per_pair * n * margin) + (64 << 20)
    db = eng.device_batch(pool_cap, n)
    truth = np.zeros(n, dtype=np.uint8)
    stage = [first.hb, None]
    truth[:first.truth.size] = first.truth
    db.append(first.hb)
    pos = first.truth.size
    leaves = first.leaves
    k = 1
    last_log = time.time()
    while pos < n:
        m = min(args.chunk, n - pos)
        ch = pop.chunk(eng, pos, m, threads, reuse=stage[k & 1])
        stage[k & 1] = ch.hb
        db.append(ch.hb)
        truth[pos:pos + m] = ch.truth
        pos += m
        leaves += ch.leaves
        k += 1
        if time.time() - last_log > 20:
            log("ingest %d/%d pairs (%.0f s)" % (pos, n, time.time() - t_gen))
            last_log = time.time()
    eng.sync()
    t_gen = time.time() - t_gen
    st = db.stats()
    k1_ms = eng.timings().value_hash_ms
    log("ingest done in %.1f s: %.2f GB resident, %.1f leaves/pair, %.2f GB compared per pass" % (
        t_gen, st.pool_bytes / 1e9, st.total_leaves / max(1, n), st.compare_bytes / 1e9))

    # ---------------- warmup + full-size correctness (size-independent properties)
    ticket = eng.diff(db)
    res = eng.wait(ticket)
    exp_flags = pop.expected_flags(truth)
    got = res.pair_flags & (G.SPEC_DIRTY | G.STATUS_DIRTY)
    n_bad = int((got != exp_flags).sum())
    offs = res.path_offsets.astype(np.int64)
    every_dirty_has_path = bool((np.diff(offs) >= 1).all()) if res.dirty_ids.size else True
    ids_ok = (res.spec_dirty_ids.size == int((got & G.SPEC_DIRTY).astype(bool).sum()) and
              res.status_dirty_ids.size == int((got & G.STATUS_DIRTY).astype(bool).sum()))
    full_check = dict(pairs=n, flag_mismatches=n_bad, every_dirty_pair_has_paths=every_dirty_has_path,
                      id_lists_consistent=ids_ok, spec_dirty=int(res.spec_dirty_ids.size),
                      status_dirty=int(res.status_dirty_ids.size), paths=int(res.path_hashes.size))
    log("full-size check:", json.dumps(full_check))
    if n_bad or not every_dirty_has_path or not ids_ok:
        log("FULL-SIZE CHECK FAILED")
    pop_flags = res.pair_flags.copy()
    del res

    sample_check = None

    for _ in range(max(0, args.warmup - 1)):
        eng.diff(db)
    eng.sync()

    # ---------------- timed region
    from kcp_amd import shard

    def fill_from_hbm(col, buf, n):
        db.export(G.EXPORT_SPEC_IDS if col == 0 else G.EXPORT_STATUS_IDS, buf.data_ptr(), buf.numel(), n)

    def gather_step():
        counts = torch.empty(8, dtype=torch.int32, device=dev)
        db.export(G.EXPORT_COUNTS, counts.data_ptr(), 8)
        return shard.gather_dirty(counts, fill_from_hbm, rank, world, dist, dev, trim=False)

    eng.timing_reset()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.diff(db)
        if world > 1:
            gather_step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    tm = eng.timings()
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        tot = torch.tensor([n], dtype=torch.int64, device=dev)
        dist.all_reduce(tot)
        total_pairs = int(tot.item())
    else:
        total_pairs = n

    value = total_pairs * args.steps / dt
    # K2 runs as k2_launches back-to-back launches per pass (pipelined batch
    # segments); per launch: bytes = compare_bytes / launches, time = span / launches
    launches = max(1, tm.k2_launches)
    k2_ms = tm.compare_ms / launches
    bytes_per_launch = st.compare_bytes / launches
    achieved = bytes_per_launch / (k2_ms * 1e-3) / 1e9 if k2_ms > 0 else 0.0
    traffic, traffic_src = None, None
    tj = args.traffic_json
    if tj == "latest":
        import glob
        found = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_summary.json")))
        tj = found[-1] if found else ""
    if tj and tj != "none" and os.path.exists(tj):
        with open(tj) as f:
            pmc = json.load(f)
        # per-launch bytes are only comparable on the same workload and launch split
        if pmc.get("algorithmic_bytes_per_launch") == bytes_per_launch:
            traffic, traffic_src = pmc.get("hbm_bytes_per_launch"), os.path.relpath(tj, ROOT)

    # ---------------- CPU baseline leg (rank 0, N=1 only): the oracle's C++ port
    # timed on the host, and -- the oracle as checker -- a bit-exact sample
    # through the JSON -> encoder -> GPU path vs the Python oracle
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        if args.sample:
            from tests.parity import assert_matches, oracle_batch
            idx = np.unique(np.linspace(0, n - 1, min(args.sample, n)).astype(np.int64))
            pairs = [pop.json_pair(int(i)) for i in idx]
            exp = oracle_batch(pairs)
            r = eng.diff_pairs(pairs)
            ok = True
            try:
                assert_matches(r, pairs, exp=exp)
            except AssertionError as e:
                ok = False
                log("SAMPLE PARITY FAILED:", str(e)[:500])
            same = bool((r.pair_flags == pop_flags[idx]).all())
            sample_check = dict(pairs=int(idx.size), bit_exact_vs_oracle=ok, matches_population_flags=same)
            log("sample check:", json.dumps(sample_check))
        from oracle import cpu_ref
        idx = np.unique(np.linspace(0, n - 1, min(args.cpu_sample, n)).astype(np.int64))
        pairs = [pop.json_pair(int(i)) for i in idx]
        dp = cpu_ref.DecodedPairs(pairs)
        cflags, sweeps, sec = dp.decide(threads=threads, min_seconds=args.cpu_seconds)
        agree = bool((cflags & 3 == pop_flags[idx] & 3).all())
        _, sweeps1, sec1 = dp.decide(threads=1, min_seconds=args.cpu_seconds / 2)
        dp.close()
        cpu = dict(value=len(idx) * sweeps / sec, unit="pairs/s", cores=threads, kind="port",
                   sample="%d pairs (every %dth of this workload, JSON decoded untimed), %d sweeps in %.1f s; "
                          "decisions agree with GPU: %s; 1-core: %.0f pairs/s" % (
                              len(idx), max(1, n // len(idx)), sweeps, sec, agree, len(idx) * sweeps1 / sec1))
        log("cpu baseline:", json.dumps(cpu))

    if rank == 0:
        line = {
            "metric": "object-pair diffs/sec (whole node) + achieved HBM GB/s, 10M objs/100k clusters",
            "value": value,
            "unit": "pairs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (seeded object populations, SURVEY.md 8d; no real cluster data)",
            "config": {
                "workload": "%s: %d pairs / %d logical clusters node-wide%s, %.0f%% mutated (%s)" % (
                    args.config, cfg.n_pairs, cfg.n_clusters,
                    " (%d x %d pairs / %d clusters, one per GPU)" % (world, base.n_pairs, base.n_clusters)
                    if mult > 1 else "", cfg.mutate_frac * 100,
                    "40% ConfigMap/Secret, 40% Deployment, 20% CRD" if args.config == "config3" else args.config),
                "pairs_per_rank": n, "resident_gb_per_rank": st.pool_bytes / 1e9,
                "parallelism": "shard-by-logical-cluster x%d (LPT)%s" % (
                    world, ", RCCL all-gather of dirty counts+IDs per step" if world > 1 else ""),
            },
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBPS, "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": "k_compare (K2)", "bytes_per_launch": bytes_per_launch,
                         "avg_launch_ms": k2_ms, "launches_per_step": launches},
            "kernels_ms": {"compare_all_launches": tm.compare_ms, "compact": tm.compact_ms,
                           "join_exposed": tm.join_ms, "emit": tm.emit_ms, "diff_pass": tm.total_ms,
                           "passes": tm.n_passes, "value_hash_last_chunk": k1_ms},
            "cpu_baseline": cpu,
            "checks": {"full_size": full_check, "sample": sample_check},
            "ingest_s": t_gen,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
