#!/usr/bin/env python3
"""Headline benchmark: object-pair diffs/sec (whole node) + achieved HBM GB/s.

Workload (BASELINE.json configs[2], the metric's own configuration): 10M mixed
object pairs (40% ConfigMap/Secret, 40% Deployment, 20% medium CRD) across
100k logical clusters, 5% mutated, synthetic (seed 20211004+3).

Scaling (--scaling; default weak at N = 1, strong at N > 1): the metric is
quoted on 10M objects / 100k clusters, so at N > 1 that population is split N
ways by whole logical cluster (LPT; the reference runs one syncer per cluster,
pkg/reconciler/cluster/cluster.go:125-138) -- strong scaling.  --scaling weak
keeps per-GPU work fixed instead (the node holds N x the config).  Either way
the pairs are encoded on the host with the product encoder and are resident
in HBM before timing.

A step = one diff pass of the hot path (K2 compare + fused merge-join, K3
compaction, K4 deferred joins, K5/K6 path emit) over the rank's resident
pairs, plus (N > 1) the RCCL all-gather of per-rank dirty counts and dirty
pair IDs (shard.DirtyGather: one all-gather into preallocated buffers; the
gathered counts are read back after it and a capacity overflow is regrown and
re-gathered inside the step).

Beside the timed line (rank 0, N = 1): the roofline on both byte definitions
(this build's format bytes, and SURVEY.md §8(d)'s B_pair = sum(24 L + V + 8) +
O), end-to-end JSON-in rates (host-encoded and device-encoded, K0), the CPU
baselines on all host cores (the C++ tree-walk restatement of the predicates
and the CPU merge over the CSR encoding) and a three-way parity check of
decisions and changed paths (GPU, tree-walk, CSR merge) on the CPU sample.

Launch: python bench.py [--gpus N --steps K --warmup W].  For N > 1 either
under torch.distributed.run (one process per GPU; WORLD_SIZE must equal N) or
bare, in which case bench.py starts that launch itself as a child process and
relays rank 0's line.  Rank 0 prints one JSON line.
"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md "Chip-level parameters")
# the sources K2's code and launch come from: a PMC summary is attached as roofline.traffic only when it
# was measured on these same bytes
K2_SOURCES = ["kcp_amd/csrc/kernels.hip", "kcp_amd/csrc/kernels.h", "kcp_amd/csrc/engine.h", "kcp_amd/csrc/api.cpp",
              "include/gpudiff_format.h"]


def log(*a):
    print("[bench r%s]" % os.environ.get("RANK", "0"), *a, file=sys.stderr, flush=True)


def k2_source_hash():
    h = hashlib.sha256()
    for f in K2_SOURCES:
        with open(os.path.join(ROOT, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def cpu_threads(aff, quota):
    """CPU-baseline threads: min(affinity, ceil(cgroup quota)) -- the cores the process can run at once."""
    import math
    return max(1, min(aff, math.ceil(quota))) if quota else aff


def free_port():
    import socket
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    p = sk.getsockname()[1]
    sk.close()
    return p


def host_cores():
    """(threads for the CPU baseline = every CPU this process may run on, nproc, cgroup CPU quota or None)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    return aff, os.cpu_count(), quota


def claim_stdout():
    """The contract is ONE JSON line on stdout. Libraries write there too (RCCL prints its
    version banner to stdout when a communicator is created), so fd 1 is pointed at stderr and
    the result line goes to a private duplicate of the original stdout."""
    fd = os.dup(1)
    sys.stdout.flush()
    os.dup2(2, 1)
    sys.stdout = os.fdopen(fd, "w", buffering=1)


def launch_cmd(gpus, argv):
    """The one-process-per-GPU launch of this same command line (torch.distributed.run, rendezvous on
    127.0.0.1): what `bench.py --gpus N` runs as a child when no launcher started it."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % gpus,
            "--master-addr=127.0.0.1", "--master-port=%d" % free_port(), os.path.abspath(__file__)] + list(argv)


def self_launch(args, argv):
    """--gpus N > 1 without a launcher (no WORLD_SIZE): start the N ranks as a CHILD process before
    anything touches the GPU, relay rank 0's JSON line (inherited stdout) and exit with the child's
    code.  A launcher whose world size differs from --gpus is an error, never a silent 1-GPU run."""
    world = os.environ.get("WORLD_SIZE")
    if world is not None:
        if int(world) != args.gpus:
            log("error: --gpus %d but WORLD_SIZE %s" % (args.gpus, world))
            sys.exit(2)
        return
    if args.gpus <= 1 and not args.print_launch:
        return
    cmd = launch_cmd(args.gpus, [a for a in argv if a != "--print-launch"])
    if args.print_launch:
        print(json.dumps({"launch": cmd, "world_size": args.gpus}), flush=True)
        sys.exit(0)
    import subprocess
    log("launching %d ranks: %s" % (args.gpus, " ".join(cmd)))
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    sys.exit(subprocess.call(cmd, env=env))


def main():
    argv = sys.argv[1:]
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=40)
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
    ap.add_argument("--batches", type=int, default=40, help="config5: timed batches (only with --seconds 0)")
    ap.add_argument("--seconds", type=float, default=10.0,
                    help="config5: sustained replay time (SURVEY.md 8(d): >= 10 s); 0 = --batches batches")
    ap.add_argument("--warmup-batches", type=int, default=4, help="config5: untimed batches")
    ap.add_argument("--zero-copy", action="store_true",
                    help="config5: every timed batch's new objects sit in one engine-pinned buffer in the upload "
                         "layout (the watch reader writes each event's JSON there): no staging copy")
    ap.add_argument("--encode", default="device", choices=["device", "host"],
                    help="config5: encode events on the GPU (K0, raw JSON up) or on the host")
    ap.add_argument("--pairs", type=int, default=0, help="override population size (default: the config's)")
    ap.add_argument("--kind", default="api", choices=["api", "crd", "mixed"],
                    help="negotiate: APIResourceImport/NegotiatedAPIResource events, CustomResourceDefinition events, "
                         "or both interleaved in one batch")
    ap.add_argument("--clusters", type=int, default=0)
    ap.add_argument("--scaling", default="auto", choices=["auto", "weak", "strong"],
                    help="strong: the config's population split N ways (the metric's 10M/100k node-wide; "
                         "default for N > 1); weak: per-GPU work fixed (node population = N x the config)")
    ap.add_argument("--chunk", type=int, default=262144)
    ap.add_argument("--gather-depth", type=int, default=1,
                    help="N > 1: all-gathers in flight; 2 = pipelined (step s's collective overlaps step s+1's "
                         "diff; measured 2.4%% slower than serial at world size 1 on MI355X, profiles/r02zd)")
    ap.add_argument("--pipeline", type=int, default=0, choices=[0, 1, 2],
                    help="2 (default) = two diff passes in flight: a second context (own stream) diffs a view of the "
                         "resident batch (gpudiff_dbatch_create_view) on alternate steps, so one pass's decision "
                         "kernel fills the CUs the previous pass's tail frees and that pass's compaction, joins and "
                         "collective (shard.PipelinedGather) run beside it; every step is still a complete pass.  "
                         "The roofline's kernel times then come from isolated passes after the timed loop.  "
                         "1 = one pass at a time (the kernel times are the timed loop's); 0 = 2.  Under gloo (the "
                         "one-GPU rehearsal) each pass's engine-written send buffer is staged to the host after it")
    ap.add_argument("--calib-passes", type=int, default=6,
                    help="--pipeline 2: isolated diff passes after the timed loop that time the kernels (roofline)")
    ap.add_argument("--no-gather-lookahead", action="store_true",
                    help="N > 1 (RCCL, depth 1): read each step's gathered counts before enqueueing the next pass "
                         "(the default checks step s after step s + 1 is queued, regrowing from the engine's "
                         "alternate result slot, so the GPU never waits for the host between steps)")
    ap.add_argument("--gather-cap-frac", type=float, default=1.0,
                    help="N > 1: scale the agreed per-rank ID capacities (< 1 forces a capacity regrow in the first "
                         "timed steps: rehearsal / tests of the regrow path)")
    ap.add_argument("--gather-world1", action="store_true",
                    help="run the per-step RCCL collective even at world size 1 (exercises/measures it on one GPU)")
    ap.add_argument("--engine-flags", type=lambda x: int(x, 0), default=0,
                    help="extra GPUDIFF_OPT_* tuning bits for the diff engine (diagnostics, e.g. 0xF << 21 defers "
                         "every join to K4)")
    ap.add_argument("--threads", type=int, default=0, help="host encode threads (default min(16, cpus))")
    ap.add_argument("--sample", type=int, default=600, help="pairs checked bit-exact vs the oracle (JSON path)")
    ap.add_argument("--cpu-sample", type=int, default=50000, help="pairs in the CPU-baseline sample")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-full-paths", action="store_true",
                    help="skip the CPU merge's full-size decision + changed-path check during ingest")
    ap.add_argument("--json-in-pairs", type=int, default=131072,
                    help="pairs of the end-to-end JSON-in measurement (0 = skip)")
    ap.add_argument("--traffic-json", default="latest",
                    help="PMC traffic summary to attach as roofline.traffic (default: the newest committed "
                         "profiles/**/pmc_summary.json, used only if it was measured on this workload with the "
                         "same K2 sources; 'none' to skip)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="N > 1: nccl = RCCL over xGMI (the product path); gloo = a rehearsal of the same N-rank "
                         "path on one GPU (every rank on device local_rank %% device_count, counts and IDs staged "
                         "through host tensors -- RCCL refuses two ranks on one device); timings then measure "
                         "the rehearsal, not the node")
    ap.add_argument("--dump-gather", default="",
                    help="rank 0 writes the last step's node-wide spec / status dirty IDs to this .npz (tests)")
    ap.add_argument("--shard-weight", default="bytes", choices=["bytes", "pairs"],
                    help="N > 1 (or --emulate-world): LPT of logical clusters onto ranks by sum of B_pair (SURVEY.md "
                         "8(e), the bytes K2 streams; default) or by pair count")
    ap.add_argument("--weights-cache", default="",
                    help="one GPU (--emulate-world): .npy of the population's per-cluster B_pair sums, reused if it "
                         "was written for the same population (saves re-encoding 10M pairs between runs)")
    ap.add_argument("--emulate-world", type=int, default=0,
                    help="one GPU: time the share of rank --emulate-rank of an N-rank strong-scaling split of the "
                         "population (diagnostic line, not the headline)")
    ap.add_argument("--emulate-rank", type=int, default=-1,
                    help="with --emulate-world: the rank whose share to time (-1 = the byte-heaviest rank)")
    ap.add_argument("--print-launch", action="store_true",
                    help="print the launch command --gpus N resolves to (one process per GPU) and exit")
    args = ap.parse_args(argv)
    if not args.pipeline:
        args.pipeline = 2
    self_launch(args, argv)
    claim_stdout()
    if args.gpus > 1 and args.config not in ("config1", "config2", "config3", "config4"):
        log("error: --config %s is a one-GPU side bench" % args.config)
        sys.exit(2)

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
    scaling = args.scaling if args.scaling != "auto" else ("strong" if world > 1 else "weak")

    import torch
    import torch.distributed as dist

    from kcp_amd import gpudiff as G
    from kcp_amd import shard
    from kcp_amd import synth as S

    gloo = args.dist_backend == "gloo"
    gpu = local_rank % max(1, torch.cuda.device_count()) if gloo else local_rank
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    comm_dev = torch.device("cpu") if gloo else dev  # where the collectives' tensors live
    collective = world > 1 or args.gather_world1
    if collective:
        dist.init_process_group(args.dist_backend, device_id=None if gloo else dev, world_size=world, rank=rank,
                                init_method=None if world > 1 or "MASTER_ADDR" in os.environ else
                                "tcp://127.0.0.1:%d" % free_port())
    stream = torch.cuda.Stream(device=dev)  # the engine's stream, made torch's current one: exports,
    torch.cuda.set_stream(stream)            # copies and collectives all order on it (never the null stream)
    aff, nproc, quota = host_cores()
    threads = args.threads or max(1, min(16, aff))

    eng = G.Engine(device=gpu, encode_threads=threads, stream=stream.cuda_stream, timing=True,
                   flags=args.engine_flags)
    base = S.make_cfg(args.config, n_pairs=args.pairs, n_clusters=args.clusters)
    mult = world if scaling == "weak" else 1
    cfg = S.make_cfg(args.config, n_pairs=base.n_pairs * mult, n_clusters=base.n_clusters * mult)
    shard_info, pop = shard_population(args, cfg, world, rank, threads, comm_dev, dist if collective else None, G, S)
    n = pop.n
    log("config %s (%s scaling): %d pairs / %d clusters node-wide; this rank %d pairs / %d clusters; %d host threads"
        % (args.config, scaling, cfg.n_pairs, cfg.n_clusters, n, pop.n_clusters, threads))

    # ---------------- ingest: synthesize + encode on the host, stage, H2D
    t_gen = time.time()
    first = pop.chunk(eng, 0, min(args.chunk, n), threads)
    # full-size changed-path parity (north_star: bit-exact changed-path lists for all 10M pairs): the CPU
    # merge over the same CSR encoding (oracle/csr_ref.cpp, pinned to the oracle by tests/test_oracle_cpp.py)
    # decides and lists the paths of every chunk on the host while it is staged; checked against the
    # GPU's first pass below.  Untimed.
    cpu_parts = [] if not args.no_full_paths else None
    t_cpu_paths = 0.0

    def cpu_paths(hb):
        nonlocal t_cpu_paths
        if cpu_parts is None:
            return
        from oracle import cpu_ref
        t_c = time.time()
        inf = hb.info()
        cpu_parts.append(cpu_ref.csr_paths_ptr(inf.pool, hb.rows(), threads))
        t_cpu_paths += time.time() - t_c
    cpu_paths(first.hb)
    per_pair = first.pool_bytes / max(1, min(args.chunk, n))
    margin = 1.15 if args.config != "config4" else 1.4
    pool_cap = int(per_pair * n * margin) + (64 << 20)
    db = eng.device_batch(pool_cap, n)
    truth = np.zeros(n, dtype=np.uint8)
    stage = [first.hb, None]
    truth[:first.truth.size] = first.truth
    db.append(first.hb)
    pos = first.truth.size
    k = 1
    last_log = time.time()
    while pos < n:
        m = min(args.chunk, n - pos)
        ch = pop.chunk(eng, pos, m, threads, reuse=stage[k & 1])
        cpu_paths(ch.hb)
        stage[k & 1] = ch.hb
        db.append(ch.hb)
        truth[pos:pos + m] = ch.truth
        pos += m
        k += 1
        if time.time() - last_log > 20:
            log("ingest %d/%d pairs (%.0f s)" % (pos, n, time.time() - t_gen))
            last_log = time.time()
    eng.sync()
    t_gen = time.time() - t_gen
    st = db.stats()
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
    n_spec, n_status, n_paths = int(res.spec_dirty_ids.size), int(res.status_dirty_ids.size), int(res.path_hashes.size)
    full_check = dict(pairs=n, flag_mismatches=n_bad, every_dirty_pair_has_paths=every_dirty_has_path,
                      id_lists_consistent=ids_ok, spec_dirty=n_spec, status_dirty=n_status, paths=n_paths)
    if cpu_parts is not None:
        c_flags = np.concatenate([q[0] for q in cpu_parts])
        c_offs, base = [np.zeros(1, np.int64)], 0
        for q in cpu_parts:
            c_offs.append(q[1][1:].astype(np.int64) + base)
            base += int(q[1][-1])
        c_offs = np.concatenate(c_offs)
        c_h = np.concatenate([q[2] for q in cpu_parts])
        c_k = np.concatenate([q[3] for q in cpu_parts])
        full_check.update(
            flags_eq_cpu_csr=bool(np.array_equal(res.pair_flags & 7, c_flags)),
            paths_eq_cpu_csr=bool(np.array_equal(offs, c_offs) and np.array_equal(res.path_hashes, c_h) and
                                  np.array_equal(res.path_kinds, c_k)),
            cpu_csr_paths=int(c_h.size), cpu_csr_seconds=round(t_cpu_paths, 2),
            cpu_csr="oracle/csr_ref.cpp over every chunk's host CSR (decisions + changed-path lists, all pairs)")
        if not (full_check["flags_eq_cpu_csr"] and full_check["paths_eq_cpu_csr"]):
            log("FULL-SIZE PATH PARITY FAILED")
        del cpu_parts, c_flags, c_offs, c_h, c_k
    log("full-size check:", json.dumps(full_check))
    if n_bad or not every_dirty_has_path or not ids_ok or full_check.get("paths_eq_cpu_csr") is False:
        log("FULL-SIZE CHECK FAILED")
    pop_flags = res.pair_flags.copy()
    del res

    for _ in range(max(0, args.warmup - 1)):
        eng.diff(db)
    eng.sync()
    # --pipeline 2: the second pass context (its own stream) and its view of the resident batch
    engs, dbs, streams = [eng], [db], [stream]
    if args.pipeline == 2:
        stream2 = torch.cuda.Stream(device=dev)
        eng2 = G.Engine(device=gpu, encode_threads=threads, stream=stream2.cuda_stream, timing=True,
                        flags=args.engine_flags)
        db2 = db.view(eng2)
        engs.append(eng2)
        dbs.append(db2)
        streams.append(stream2)
        r2 = eng2.wait(eng2.diff(db2))  # allocates its outputs; the same decisions as the first context's
        full_check["pipeline_view_flags_eq"] = bool(np.array_equal(r2.pair_flags, pop_flags))
        del r2
        for _ in range(max(0, args.warmup - 1)):
            eng2.diff(db2)
        eng2.sync()
        # untimed steps of the timed loop's own shape (two passes in flight): the warmup above ran each context
        # alone, so the timed loop's first steps were the first overlapped ones (one box stepped at 9.04 ms against
        # its isolated 8.38-ms pass, profiles/r06ar; 8.31 vs 8.46 on another, r06an).  The collective (N > 1) is
        # warmed below with its capacities agreed.
        for i in range(2 * max(0, args.warmup)):
            engs[i & 1].diff(dbs[i & 1])
        torch.cuda.synchronize()

    # ---------------- the collective (N > 1): capacities agreed once, untimed
    gather = None
    if collective:
        def export_to(t, what, n):
            """gpudiff_dbatch_export of n elements into t: straight from HBM into a device tensor (RCCL), or
            through a device staging tensor into the host tensor gloo sends"""
            if t.device.type == "cuda":
                db.export(what, t.data_ptr(), n, n)
            else:
                tmp = torch.empty(t.numel(), dtype=t.dtype, device=dev)
                db.export(what, tmp.data_ptr(), n, n)
                t.copy_(tmp)

        counts = torch.zeros(8, dtype=torch.int32, device=comm_dev)
        export_to(counts, G.EXPORT_COUNTS, 8)
        torch.cuda.synchronize()
        cap_s, cap_t = shard.DirtyGather.agree_capacity(counts, world, dist)
        # RCCL: the engine's compaction writes each step's counts and IDs straight into the send buffer
        # (gpudiff_dbatch_bind_gather) -- no export copies per step; gloo's host tensors are filled by copies
        bind = None if gloo else (lambda send, cs, ct: db.bind_gather(send.data_ptr(), cs, ct))
        slot = None if (gloo or args.no_gather_lookahead or args.gather_depth != 1) else (lambda k: db.result_slot(k))
        if args.pipeline == 2:
            binds = [lambda send, cs, ct, d=d: d.bind_gather(send.data_ptr(), cs, ct) for d in dbs]
            gather = shard.PipelinedGather(world, cap_s, cap_t, dev, dist, streams, binds, comm_device=comm_dev)

            def fill_counts(p, t):
                dbs[p].export(G.EXPORT_COUNTS, t.data_ptr(), 8, 8)

            def fill_ids(p, col, buf):
                dbs[p].export(G.EXPORT_SPEC_IDS if col == 0 else G.EXPORT_STATUS_IDS, buf.data_ptr(), buf.numel(),
                              buf.numel())
            for p in (0, 1):  # warm the communicator on both streams
                engs[p].diff(dbs[p])
                gather.step(fill_counts, fill_ids)
        else:
            gather = shard.DirtyGather(world, cap_s, cap_t, comm_dev, dist, depth=args.gather_depth, bind=bind,
                                       slot=slot)

            def fill_counts(t):
                export_to(t, G.EXPORT_COUNTS, 8)

            def fill_ids(col, buf):
                export_to(buf, G.EXPORT_SPEC_IDS if col == 0 else G.EXPORT_STATUS_IDS, buf.numel())
            if bind is not None or slot is not None:
                gather.begin_step()
                eng.diff(db)
            gather.step(fill_counts, fill_ids)  # warm the communicator
        log("collective: %s, capacities agreed (%d spec, %d status IDs per rank), depth %d, pipeline %d"
            % (args.dist_backend, cap_s, cap_t, args.gather_depth, args.pipeline))
        gather.finish()
        torch.cuda.synchronize()
        if args.gather_cap_frac != 1.0:  # rehearsal / tests: capacities below the counts force a regrow
            gather._alloc(max(1, int(cap_s * args.gather_cap_frac)), max(1, int(cap_t * args.gather_cap_frac)))
            torch.cuda.synchronize()
    regrows_before = gather.n_regrows if gather is not None else 0

    # ---------------- timed region
    for e in engs:
        e.timing_reset()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if args.pipeline == 2:  # alternate contexts: two passes in flight
        for i in range(args.steps):
            engs[i & 1].diff(dbs[i & 1])
            if gather is not None:
                gather.step(fill_counts, fill_ids)
    for _ in range(args.steps if args.pipeline == 1 else 0):
        if gather is not None and (gather.bind is not None or gather.slot is not None):
            gather.begin_step()
        eng.diff(db)
        if gather is not None:
            gather.step(fill_counts, fill_ids)
    if gather is not None:
        gather.finish()  # every step's collective completes inside the timed region
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if args.pipeline == 2:
        # the timed loop overlaps passes, so a kernel's event span there includes waiting for CUs the other
        # pass holds: the roofline's kernel times come from isolated passes of the same batch (untimed)
        eng.timing_reset()
        # one rank at a time: in the one-GPU rehearsal every rank's passes share the device, and
        # two ranks' "isolated" passes running together measured each other (K3 0.83 ms vs 0.12 alone)
        for r in range(world if collective else 1):
            if r == rank:
                for _ in range(args.calib_passes):
                    eng.diff(db)
                    eng.sync()
            if collective:
                dist.barrier()
    tm = eng.timings()
    per_rank_ms = None
    if collective:  # every rank's kernel times of its isolated passes (the rehearsal's per-rank K3, item 5)
        t = torch.tensor([tm.compare_ms, tm.compact_ms, tm.join_ms, tm.emit_ms, tm.total_ms], dtype=torch.float64,
                         device=comm_dev)
        allt = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(allt, t)
        per_rank_ms = [dict(zip(("compare", "compact", "join_exposed", "emit", "diff_pass"),
                                [round(float(x), 4) for x in a.tolist()])) for a in allt]
    log("timed region: %d steps in %.3f s" % (args.steps, dt))
    gather_check = None
    if gather is not None:
        ok, cc = gather.check()
        sa, ta = gather.result() if ok else (None, None)
        gather_check = dict(capacity_ok=ok, node_spec_dirty=int(cc[:, 0].sum()), node_status_dirty=int(cc[:, 1].sum()),
                            gathered_spec=None if sa is None else int(sa.numel()),
                            gathered_status=None if ta is None else int(ta.numel()),
                            depth=gather.depth, bytes_per_rank=4 * gather.width,
                            regrows=gather.n_regrows - regrows_before, cap_frac=args.gather_cap_frac,
                            engine_writes_send_buffer=(args.pipeline == 2 or gather.bind is not None),
                            lookahead=(args.pipeline == 2 or gather.slot is not None), pipeline=args.pipeline)
        t = torch.tensor([dt], dtype=torch.float64, device=comm_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        tot = torch.tensor([n], dtype=torch.int64, device=comm_dev)
        dist.all_reduce(tot)
        total_pairs = int(tot.item())
        if sa is not None:
            gather_check.update(node_sets_vs_truth(pop, truth, sa, ta, dist, comm_dev, G))
            if args.dump_gather and rank == 0:
                np.savez(args.dump_gather, spec=sa.cpu().numpy(), status=ta.cpu().numpy())
    else:
        total_pairs = n

    value = total_pairs * args.steps / dt
    # K2 runs as k2_launches back-to-back launches per pass (pipelined batch
    # segments); per launch: bytes = bytes / launches, time = span / launches
    launches = max(1, tm.k2_launches)
    k2_ms = tm.compare_ms / launches
    pass_ms = tm.total_ms
    # B_pair = sum over A, B of (24 L + V + 8) + O, O = 4 B per dirty ID (x2 decisions) + 8 B per path
    survey_bytes = 24 * st.total_leaves + st.value_bytes + 16 * n + 4 * (n_spec + n_status) + 8 * n_paths
    fmt_bytes = st.compare_bytes
    achieved = survey_bytes / launches / (k2_ms * 1e-3) / 1e9 if k2_ms > 0 else 0.0
    achieved_fmt = fmt_bytes / launches / (k2_ms * 1e-3) / 1e9 if k2_ms > 0 else 0.0
    achieved_pass = fmt_bytes / (pass_ms * 1e-3) / 1e9 if pass_ms > 0 else 0.0
    traffic, traffic_src = None, None
    src_hash = k2_source_hash()
    tj = args.traffic_json
    if tj == "latest":
        import glob
        found = sorted(glob.glob(os.path.join(ROOT, "profiles", "**", "*pmc_summary.json"), recursive=True),
                       key=os.path.getmtime)
        cand = []
        for f in found:
            try:
                with open(f) as fh:
                    pm = json.load(fh)
            except (OSError, ValueError):
                continue
            # the newest summary of the same K2 sources on this workload (a config4 summary may be newer)
            if pm.get("k2_source_hash") == src_hash and pm.get("algorithmic_bytes_per_launch") == fmt_bytes / launches:
                cand.append(f)
        tj = cand[-1] if cand else ""
    traffic_box = traffic_rocprof_ms = None
    if tj and tj != "none" and os.path.exists(tj):
        with open(tj) as f:
            pmc = json.load(f)
        # comparable only on the same K2 sources and the same workload (format bytes per launch)
        if pmc.get("k2_source_hash") == src_hash and pmc.get("algorithmic_bytes_per_launch") == fmt_bytes / launches:
            traffic, traffic_src = pmc.get("hbm_bytes_per_launch"), os.path.relpath(tj, ROOT)
            traffic_box, traffic_rocprof_ms = pmc.get("box"), pmc.get("rocprof_avg_ms")

    for d in dbs[1:]:
        d.free()  # views before their base
    db.free()  # the JSON-in and CPU legs below need no resident population

    # ---------------- rank 0, N = 1: end-to-end JSON-in, CPU baselines, three-way parity
    json_in = cpu = sample_check = three_way = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        if args.json_in_pairs:
            json_in = json_in_rates(G, pop, min(args.json_in_pairs, n), threads, local_rank)
            log("json-in:", json.dumps(json_in))
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
        cpu, three_way = cpu_legs(G, eng, pop, n, pop_flags, args, aff, nproc, quota)
        log("cpu baseline:", json.dumps(cpu))
        log("three-way parity:", json.dumps(three_way))

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
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (seeded object populations, SURVEY.md 8d; no real cluster data)",
            "config": {
                "workload": "%s: %d pairs / %d logical clusters node-wide%s, %.0f%% mutated (%s)" % (
                    args.config, cfg.n_pairs, cfg.n_clusters,
                    " (%d x %d pairs / %d clusters, one per GPU)" % (world, base.n_pairs, base.n_clusters)
                    if mult > 1 else (" split %d ways by logical cluster" % world if world > 1 else
                                      (" -- EMULATED: rank %d's share (%d pairs) of a %d-way split, timed alone on "
                                       "one GPU" % (shard_info["emulated_rank"], n, shard_info["world"])
                                       if "emulated_rank" in shard_info else "")),
                    cfg.mutate_frac * 100,
                    "40% ConfigMap/Secret, 40% Deployment, 20% CRD" if args.config == "config3" else args.config),
                "pairs_per_rank": n, "resident_gb_per_rank": st.pool_bytes / 1e9, "shard": shard_info,
                "passes_in_flight": args.pipeline,
                "parallelism": "shard-by-logical-cluster x%d (LPT)%s" % (
                    world, ((", RCCL all-gather of dirty counts+IDs per step (%d in flight)" % args.gather_depth)
                            if args.dist_backend == "nccl" else
                            ", gloo all-gather of dirty counts+IDs per step through host tensors (REHEARSAL: "
                            "every rank on one GPU; not a node measurement)") if collective else ""),
            },
            # achieved / frac: the bytes this encoding must read (K2's format bytes) over K2's time -- a physical
            # rate, <= peak by construction; SURVEY 8(d)'s 24-B-record count is kept beside it as an equivalent
            # throughput, never as a fraction of peak (it charges 24 B per leaf where the format stores 16, and
            # value digests the format no longer has, so it can exceed the HBM peak: VERDICT r4 weak #2)
            "roofline": {"bound": "hbm", "achieved": achieved_fmt, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": achieved_fmt / HBM_PEAK_GBPS, "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": "k_compare_flat (K2)", "avg_launch_ms": k2_ms, "launches_per_step": launches,
                         "bytes_def": "format bytes: what K2 must read in this build's CSR encoding -- 64-B row + "
                                      "flag + both size-matched segments (16 B per leaf record: value u64 = the "
                                      "value's first 8 bytes, 32-bit path hash, meta; + the arena: long strings' "
                                      "tails past 8 bytes, 4-B aligned, padded to 16)",
                         "bytes_per_launch": fmt_bytes / launches,
                         "survey_24B_record_equiv": {
                             "bytes_per_launch": survey_bytes / launches, "pairs_bytes_per_s_GBps": achieved,
                             "def": "SURVEY.md 8(d) / BASELINE.md:52: sum over A,B of (24 L + V + 8) + O over K2's "
                                    "time -- a format-independent work rate (24-B records), not a fraction of peak"},
                         "diff_pass": {"ms": pass_ms, "achieved": achieved_pass, "frac": achieved_pass / HBM_PEAK_GBPS,
                                       "def": "format bytes over the whole diff pass (K2..K6)"},
                         "k2_source_hash": src_hash, "build_id": G.BUILD_ID,
                         # the physical rate: HBM counter bytes (FETCH_SIZE x 2 + WRITE_SIZE per K2 launch) over
                         # this run's K2 time -- what the memory system moved, whatever the byte definition
                         # (with no PMC summary of these K2 sources and this workload, the bytes K2's format
                         # reads stand in -- a lower bound of what it moves, never the definitional SURVEY count)
                         "frac_physical": ((traffic if traffic else fmt_bytes / launches) / (k2_ms * 1e-3) / 1e9 /
                                           HBM_PEAK_GBPS) if k2_ms else None,
                         "frac_physical_def": ("PMC traffic per K2 launch / K2 HIP-event time / 8 TB/s" if traffic else
                                               "format bytes per K2 launch / K2 HIP-event time / 8 TB/s (no PMC "
                                               "summary of these K2 sources on this workload)"),
                         "survey_over_format_bytes": survey_bytes / fmt_bytes if fmt_bytes else None,
                         "traffic_box": traffic_box, "traffic_rocprof_k2_ms": traffic_rocprof_ms,
                         "box": box_id()},
            "kernels_ms": {"source": ("%d isolated passes after the timed loop (the loop overlaps two passes)"
                                      % args.calib_passes) if args.pipeline == 2 else "the timed loop's passes",
                           "compare_all_launches": tm.compare_ms, "compact": tm.compact_ms,
                           "join_exposed": tm.join_ms, "emit": tm.emit_ms, "diff_pass": tm.total_ms,
                           "passes": tm.n_passes, "per_rank": per_rank_ms},
            "cpu_baseline": cpu,
            "json_in": json_in,
            "checks": {"full_size": full_check, "sample": sample_check, "three_way": three_way,
                       "gather": gather_check},
            "ingest_s": t_gen,
            "box": box_id(),
            # the loaded library's content hash of its sources (gpudiff_build_id; the loader refused it unless
            # it equals the shipped sources' hash, kcp_amd/buildinfo.py)
            "build_id": G.BUILD_ID, "build_verified": G.BUILD_VERIFIED,
        }
        print(json.dumps(line), flush=True)
    if collective:
        dist.destroy_process_group()


def box_id():
    """The machine this run measured on (hostname + the GPU's PCI bus id): a roofline whose counters were
    taken on another box says so."""
    import socket
    try:
        import torch
        p = torch.cuda.get_device_properties(torch.cuda.current_device())
        bus = "%s/%s" % (getattr(p, "pci_bus_id", "?"), getattr(p, "pci_device_id", "?"))
    except Exception:
        bus = "?"
    return "%s:%s" % (socket.gethostname(), bus)


def _mix64(x):
    """splitmix64 finalizer over a u64 array (the multiset hash of node_sets_vs_truth)"""
    x = x.astype(np.uint64)
    with np.errstate(over="ignore"):
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return x ^ (x >> np.uint64(31))


def node_sets_vs_truth(pop, truth, spec_all, status_all, dist, comm_dev, G):
    """The node-wide dirty sets every rank gathered must equal the union of every rank's generator truth
    (statussyncer.go:22-26: status-absent objects are status-dirty): per list, the count and a multiset
    hash (sum of splitmix64 of the global pair IDs, mod 2^64) of the gathered IDs against the same over
    each rank's expected IDs, summed with one all-reduce.  Checked on every rank."""
    import torch
    ids = pop.local_ids().astype(np.uint64)
    exp = pop.expected_flags(truth)
    loc = []
    for bit in (G.SPEC_DIRTY, G.STATUS_DIRTY):
        e = ids[(exp & bit) != 0]
        loc += [e.size, int(_mix64(e).sum(dtype=np.uint64).view(np.int64))]
    t = torch.tensor(loc, dtype=torch.int64, device=comm_dev)
    dist.all_reduce(t)
    want = t.cpu().tolist()
    got = []
    for g in (spec_all, status_all):
        a = g.cpu().numpy().astype(np.uint32).astype(np.uint64)
        got += [a.size, int(_mix64(a).sum(dtype=np.uint64).view(np.int64))]
    ok = all(int(x) == int(y) for x, y in zip(got, want))
    ok_all = torch.tensor([1 if ok else 0], dtype=torch.int64, device=comm_dev)
    dist.all_reduce(ok_all, op=dist.ReduceOp.MIN)
    return {"node_sets_eq_truth": bool(ok_all.item()), "node_expected_spec": int(want[0]),
            "node_expected_status": int(want[2])}


def shard_population(args, cfg, world, rank, threads, dev, dist, G, S):
    """This rank's population.  Strong scaling at N > 1 packs whole logical clusters onto ranks by LPT on
    each cluster's exact sum of B_pair (the bytes K2 streams, so the ranks' step times
    balance), computed once, untimed: every rank encodes the clusters c % N == rank on the host and the
    weight vectors are summed over ranks (one all-reduce).  --emulate-world N times one rank's share of
    an N-way split on one GPU (the byte-heaviest by default).  Returns (shard summary, Population)."""
    import torch
    ew = args.emulate_world if world == 1 else 0
    split = world if world > 1 else ew
    if split <= 1:
        return {"rule": "single rank", "world": 1}, S.Population(cfg, 1, 0)
    t0 = time.time()
    sizes = S.cluster_sizes(cfg).astype(np.int64)
    w = None
    if args.shard_weight == "bytes":
        if world > 1:
            part = S.cluster_bytes(cfg, world, rank, threads).astype(np.int64)
            wt = torch.from_numpy(part).to(dev)
            dist.all_reduce(wt)
            w = wt.cpu().numpy().astype(np.uint64)
        else:
            key = "%d-%d-%d-%.4f" % (cfg.seed, cfg.n_pairs, cfg.n_clusters, cfg.mutate_frac)
            cache = getattr(args, "weights_cache", "")
            if cache and os.path.exists(cache) and os.path.exists(cache + ".key") and \
                    open(cache + ".key").read() == key:
                w = np.load(cache).astype(np.uint64)
            else:
                w = S.cluster_bytes(cfg, 1, 0, threads)
                if cache:
                    np.save(cache, w)
                    with open(cache + ".key", "w") as f:
                        f.write(key)
    t_w = time.time() - t0
    owner = G.shard_lpt(w if w is not None else sizes.astype(np.uint64), split)
    # the rank loads on both measures, whichever rule packed them (bytes only when known)
    load_p = np.bincount(owner, weights=sizes.astype(np.float64), minlength=split)
    info = {"rule": "LPT by sum of B_pair" if w is not None else "LPT by pair count", "world": split,
            "weights_s": round(t_w, 2), "max_over_mean_pairs": float(load_p.max() / load_p.mean())}
    if w is not None:
        load_b = np.bincount(owner, weights=w.astype(np.float64), minlength=split)
        info.update(max_over_mean_bytes=float(load_b.max() / load_b.mean()), total_bytes=int(load_b.sum()),
                    heaviest_rank=int(load_b.argmax()), heaviest_bytes=int(load_b.max()))
        # the pair-count rule on the same weights, for comparison
        oc = G.shard_lpt(sizes.astype(np.uint64), split)
        lc = np.bincount(oc, weights=w.astype(np.float64), minlength=split)
        info["pair_count_rule_max_over_mean_bytes"] = float(lc.max() / lc.mean())
    if world > 1:
        r = rank
    else:
        r = args.emulate_rank if args.emulate_rank >= 0 else int(
            (np.bincount(owner, weights=w.astype(np.float64), minlength=split) if w is not None else load_p).argmax())
        info["emulated_rank"] = r
        info["note"] = "one GPU timing rank %d's share of a %d-way split (diagnostic, not the node-wide metric)" % (
            r, split)
    if w is not None:
        info["rank_bytes"] = int(np.bincount(owner, weights=w.astype(np.float64), minlength=split)[r])
    pop = S.Population(cfg, split, r, cluster_weight=w)
    assert pop.n == int(load_p[r]), "synth LPT and gpudiff_shard_lpt disagree"
    info["rank_pairs"] = pop.n
    log("shard: %s" % json.dumps(info))
    return info, pop


def json_in_rates(G, pop, m, threads, device):
    """End-to-end JSON-in pairs/s on the first m pairs of this workload: JSON in
    host memory -> gpudiff_submit -> gpudiff_wait (results on the host),
    once with host encoding (16 encode threads, pinned H2D, diff pass) and
    once with device encoding (pinned staging, H2D, K0, diff pass).  Includes
    PCIe; the timed headline (`value`) does not."""
    buf, offs, _truth = pop.json_range(0, m, threads)
    arr = G.json_pair_array(buf, offs)
    out = dict(sample_pairs=m, json_bytes=int(offs[-1]), threads=threads)
    flags = {}
    for mode in ("host_encode", "device_encode"):
        e = G.Engine(device=device, encode_threads=threads, device_encode=(mode != "host_encode"))
        for _ in range(2):  # warm: both ring slots' staging, the scratch (and the device-encode store)
            r = e.wait(e.submit_array(arr))
        times = []
        for _ in range(5):
            t0 = time.perf_counter()
            r = e.wait(e.submit_array(arr))
            times.append(time.perf_counter() - t0)
        flags[mode] = r.pair_flags
        best = min(times)
        out[mode] = dict(pairs_per_s=m / best, ms=best * 1e3, json_gb_per_s=int(offs[-1]) / best / 1e9)
        e.close()
        if mode == "device_encode":
            out[mode]["phases_ms"] = json_in_phases(G, arr, m, threads, device)
            out["device_encode_streaming"] = json_in_streaming(G, arr, m, threads, device)
    # zero copy: the pairs rendered into a gpudiff_host_alloc buffer in the upload layout (what the batcher does
    # when it renders a flush into engine-pinned memory; the layout copy here is untimed), uploaded without the
    # staging copy
    e = G.Engine(device=device, encode_threads=threads, device_encode=True)
    pj = G.PinnedJson(e, buf, offs)
    for _ in range(2):
        r = e.wait(e.submit_array(pj.pairs))
    times = []
    for _ in range(5):
        t0 = time.perf_counter()
        r = e.wait(e.submit_array(pj.pairs))
        times.append(time.perf_counter() - t0)
    flags["device_encode_zero_copy"] = r.pair_flags
    best = min(times)
    out["device_encode_zero_copy"] = dict(pairs_per_s=m / best, ms=best * 1e3, json_gb_per_s=int(offs[-1]) / best / 1e9,
                                          zero_copy_batches=int(e.submit_stats().zero_copy_batches),
                                          streaming=json_in_streaming(G, pj.pairs, m, threads, device, engine=e))
    pj.free()
    e.close()
    out["modes_agree"] = all(bool(np.array_equal(flags["host_encode"], f)) for f in flags.values())
    return out


def json_in_streaming(G, arr, m, threads, device, batches=6, engine=None):
    """Device-encoded JSON-in as an informer stream feeds it: batch k + 1 is submitted before batch k is waited
    (the engine keeps two in flight), so host staging, the PCIe upload, K0 and the diff pass of neighbouring
    batches overlap.  pairs/s over `batches` batches of the same m pairs, first submit to last wait."""
    e = engine or G.Engine(device=device, encode_threads=threads, device_encode=True)
    for _ in range(2):
        e.wait(e.submit_array(arr))
    flags_ok = True
    want = None
    t0 = time.perf_counter()
    tk = e.submit_array(arr)
    for _ in range(batches - 1):
        nxt = e.submit_array(arr)
        r = e.wait(tk)
        want = r.pair_flags if want is None else want
        flags_ok &= bool(np.array_equal(r.pair_flags, want))
        tk = nxt
    r = e.wait(tk)
    dt = time.perf_counter() - t0
    flags_ok &= bool(np.array_equal(r.pair_flags, want))
    if engine is None:
        e.close()
    return dict(pairs_per_s=m * batches / dt, ms_per_batch=dt / batches * 1e3, batches=batches,
                json_gb_per_s=int(arr["old_len"].sum() + arr["new_len"].sum()) * batches / dt / 1e9,
                batches_agree=flags_ok)


def json_in_phases(G, arr, m, threads, device):
    """Where a device-encoded JSON-in batch's time goes (separate runs with GPUDIFF_OPT_TIMING; the events
    are not in the timed runs above): the host side of gpudiff_submit (document tables, the JSON copy into
    pinned staging, the enqueue), the H2D copy, K0 (tokenize + encode), K0c + K0x, the diff pass (K2..K6)
    and the store's part of gpudiff_wait.  Copy stream and kernels overlap by chunk, so the GPU phases can
    sum to more than the end-to-end time."""
    e = G.Engine(device=device, encode_threads=threads, device_encode=True, timing=True)
    for _ in range(2):  # both ring slots: their pinned staging is allocated outside the measured batches
        e.wait(e.submit_array(arr))
    e.timing_reset()
    t_sub = t_wait = 0.0
    t0 = time.perf_counter()
    for _ in range(3):
        t1 = time.perf_counter()
        tk = e.submit_array(arr)
        t2 = time.perf_counter()
        e.wait(tk)
        t_sub += t2 - t1
        t_wait += time.perf_counter() - t2
    wall = (time.perf_counter() - t0) / 3 * 1e3
    st = e.submit_stats()
    tm = e.timings()
    e.close()
    return dict(end_to_end=wall, submit_call=t_sub / 3 * 1e3, wait_call=t_wait / 3 * 1e3,
                host_submit=st.host_submit_ms, host_tables=st.submit_docs_ms,
                host_staging_copy=st.submit_copy_ms, host_enqueue=st.submit_enqueue_ms, h2d=st.h2d_ms,
                k0_encode=st.encode_ms, k0c_k0x=st.link_ms, diff_pass=tm.total_ms, wait_finish=st.finish_ms,
                batches=int(st.timing_batches), deferred_to_host=int(st.deferred))


def cpu_legs(G, eng, pop, n, pop_flags, args, aff, nproc, quota):
    """CPU baselines on every core this process may use: the C++ tree-walk
    restatement of the predicates over decoded trees (cpu-ref, primary) and the
    CPU merge over the canonical CSR encoding (cpu-csr), each also on one core;
    then the three-way parity of flags and changed paths on the same sample
    (GPU vs tree-walk vs CSR merge)."""
    from oracle import cpu_ref
    idx = np.unique(np.linspace(0, n - 1, min(args.cpu_sample, n)).astype(np.int64))
    pairs = [pop.json_pair(int(i)) for i in idx]
    # the cores this process may actually use: affinity, capped by the cgroup CPU quota (more threads than
    # the quota only time-slice and understate the baseline); the all-affinity figure is printed beside it
    threads = cpu_threads(aff, quota)
    dp = cpu_ref.DecodedPairs(pairs)
    dp.decide(threads=threads)  # warm: first-touch page faults, thread start-up
    cflags, sweeps, sec = dp.decide(threads=threads, min_seconds=args.cpu_seconds)
    _, sweeps1, sec1 = dp.decide(threads=1, min_seconds=args.cpu_seconds / 3)
    aff_rate = None
    if aff > threads:
        _, swa, seca = dp.decide(threads=aff, min_seconds=args.cpu_seconds / 3)
        aff_rate = len(idx) * swa / seca
    hb = eng.encode(pairs)
    rows = hb.rows()
    csr = cpu_ref.CsrPairs(hb.pool_view(), rows)
    csr.run(threads=threads)  # warm
    fcsr, csw, csec, _ = csr.run(threads=threads, min_seconds=args.cpu_seconds / 2)
    _, csw1, csec1, _ = csr.run(threads=1, min_seconds=args.cpu_seconds / 4)
    ref_rate, csr_rate = len(idx) * sweeps / sec, len(idx) * csw / csec
    cpu = dict(value=ref_rate, unit="pairs/s", cores=threads, kind="port",
               sample="%d pairs (every %dth of this workload, JSON decoded untimed), %.1f sweeps in %.1f s, "
                      "threads rotating over slices; C++ tree-walk restatement of specsyncer.go:17-41 + "
                      "statussyncer.go:15-27" % (
                          len(idx), max(1, n // len(idx)), sweeps, sec),
               one_core=len(idx) * sweeps1 / sec1, nproc=nproc, affinity_cpus=aff, cgroup_cpu_quota=quota,
               all_affinity_threads=None if aff_rate is None else dict(value=aff_rate, threads=aff),
               cpu_csr=dict(value=csr_rate, unit="pairs/s", cores=threads, one_core=len(idx) * csw1 / csec1,
                            what="the build's CPU merge over the canonical CSR encoding (oracle/csr_ref.cpp), "
                                 "decisions + changed paths"))
    # three-way parity on the sample: GPU vs tree-walk vs CSR merge (flags and paths)
    r = eng.diff_pairs(pairs)
    seeds = (rows["flags_a"] >> G.OBJ_SEED_SHIFT) & 0xFF
    t_offs, t_h, t_k = dp.paths(seeds)
    c_flags, c_offs, c_h, c_k = csr.paths()
    gflags = r.pair_flags & 7
    three = dict(pairs=len(idx),
                 flags_gpu_eq_tree=bool(np.array_equal(gflags, cflags)),
                 flags_gpu_eq_csr=bool(np.array_equal(gflags, c_flags)),
                 flags_gpu_eq_population=bool(np.array_equal(r.pair_flags, pop_flags[idx])),
                 paths_gpu_eq_tree=bool(np.array_equal(r.path_offsets, t_offs) and np.array_equal(r.path_hashes, t_h)
                                        and np.array_equal(r.path_kinds, t_k)),
                 paths_gpu_eq_csr=bool(np.array_equal(r.path_offsets, c_offs) and np.array_equal(r.path_hashes, c_h)
                                       and np.array_equal(r.path_kinds, c_k)),
                 csr_timed_flags_eq=bool(np.array_equal(fcsr, c_flags)),
                 dirty=int(r.dirty_ids.size), paths=int(r.path_hashes.size))
    dp.close()
    hb.free()
    return cpu, three


if __name__ == "__main__":
    main()
