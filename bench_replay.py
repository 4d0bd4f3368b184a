#!/usr/bin/env python3
"""Watch-replay benchmark: sustained Update
events/s through the device-resident object store, with end-to-end batch
latency.

M objects (config3 mix: ConfigMap/Secret/Deployment/CRD, synthetic, seed
20211004+3) are loaded into a gpudiff_store (initial list, untimed).  Each
timed event is the next version of one resident object -- the population's
(A, B) versions of that object alternate, so every event is a real Update with
the same 5% spec/status mutation rate as the headline workload -- delivered as
JSON bytes together with the informer's old object (read only on a collision).
Per event the host encodes only the new version; H2D, K1 (fresh blobs only) and
the diff pass run on the GPU while the host encodes the next batch (two
batches in flight).  The timed region therefore includes host encoding and the
PCIe upload: streaming is the point of this configuration.

Reported: events/s over the timed batches, per-batch latency p50/p99 (submit
call -> results on the host), H2D GB/s, the GPU time per batch, and checks:
every timed event's decisions against the generator's ground truth and a
sample bit-exact against the oracle (flags and changed paths).

With --encode device (the default) the events go up as raw JSON and kernel K0
encodes them in HBM; --encode host is the host-encoder mode.

usage: python bench.py --config config5 [--pairs M] [--batch B] [--encode device|host]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

EVENT_DTYPE = np.dtype([("slot", "<u4"), ("pair_id", "<u4"), ("cluster_id", "<u4"), ("reserved", "<u4"),
                        ("new_json", "<u8"), ("new_len", "<u8"), ("old_json", "<u8"), ("old_len", "<u8")])
assert EVENT_DTYPE.itemsize == 48


def log(*a):
    print("[replay]", *a, file=sys.stderr, flush=True)


def run(args):
    import ctypes as C

    import torch

    from kcp_amd import gpudiff as G
    from kcp_amd import synth as S

    assert G.Event.__sizeof__ is not None and C.sizeof(G.Event) == EVENT_DTYPE.itemsize
    torch.cuda.set_device(0)
    from bench import cpu_threads, host_cores
    aff, nproc, quota = host_cores()
    ncpu = cpu_threads(aff, quota)  # the cores this process may run at once (affinity capped by the cgroup quota)
    threads = args.threads or max(1, min(16, ncpu))
    M = args.pairs or (1 << 20)  # 16 batches of 65,536 per epoch
    B = args.batch
    cfg = S.make_cfg("config3", n_pairs=M, n_clusters=args.clusters or max(1, M // 100))
    pop = S.Population(cfg)
    t0 = time.time()
    buf, offs, truth = pop.json_range(0, M, threads)
    log("generated %d objects x 2 versions: %.2f GB JSON in %.1f s" % (M, buf.size / 1e9, time.time() - t0))
    base = buf.ctypes.data
    starts = offs[:-1].astype(np.uint64) + np.uint64(base)
    lens = np.diff(offs).astype(np.uint64)
    a_ptr, b_ptr = starts[0::2], starts[1::2]
    a_len, b_len = lens[0::2], lens[1::2]
    exp_ab = pop.expected_flags(truth)  # decisions of A -> B (and, by symmetry, of B -> A)
    cluster = np.arange(M, dtype=np.uint32) % np.uint32(cfg.n_clusters)

    eng = G.Engine(device=0, encode_threads=threads, timing=True, flags=args.engine_flags)
    per_obj = float(lens.mean()) * 2.2 + 256  # blob + path table ~= 2x the JSON
    space = int(per_obj * M * 2.5) + (B * int(per_obj) * 4) + (256 << 20)
    dev_enc = args.encode == "device"
    st = eng.object_store(M, space, B, device_encode=dev_enc)
    log("store: %d slots, 2 x %.2f GB spaces, batches of %d events, %d host threads, %s encoding" % (
        M, space / 1e9, B, threads, args.encode))

    def events(slots, new_is_b, with_old=True):
        ev = np.zeros(slots.size, dtype=EVENT_DTYPE)
        ev["slot"] = slots
        ev["pair_id"] = np.arange(slots.size, dtype=np.uint32)
        ev["cluster_id"] = cluster[slots]
        ev["new_json"] = np.where(new_is_b, b_ptr[slots], a_ptr[slots])
        ev["new_len"] = np.where(new_is_b, b_len[slots], a_len[slots])
        if with_old:
            ev["old_json"] = np.where(new_is_b, a_ptr[slots], b_ptr[slots])
            ev["old_len"] = np.where(new_is_b, a_len[slots], b_len[slots])
        return ev

    def submit(ev):
        arr = (G.Event * ev.size).from_buffer(ev)
        return st.submit_raw(arr, ev.size, ev)

    # ---- initial list: every object's A version (diffed against {}; untimed)
    t0 = time.time()
    pend = None
    for s0 in range(0, M, B):
        sl = np.arange(s0, min(M, s0 + B), dtype=np.uint32)
        t = submit(events(sl, np.zeros(sl.size, bool), with_old=False))
        if pend is not None:
            eng.wait(pend)
        pend = t
    eng.wait(pend)
    t_load = time.time() - t0
    ss = st.stats()
    log("initial list: %d objects in %.1f s (%.0f objects/s), %.2f GB resident" % (
        M, t_load, M / t_load, ss.live_bytes / 1e9))

    # ---- timed replay (>= 10 s sustained).  The batches come from a cycle built before the
    # clock: two epochs, each a permutation of every resident object cut into batches of B distinct objects; the
    # first epoch advances each object A -> B, the second B -> A, so the cycle can repeat for as long as the run
    # lasts and every event is a real Update of the object's current version (same 5% mutation rate as config3)
    rng = np.random.default_rng(20211004 + 5)
    cycle = []
    zc = getattr(args, "zero_copy", False) and dev_enc
    pinned = []  # --zero-copy: each cycle batch's new objects rendered into an engine-pinned buffer (untimed)
    t_pin = time.time()
    for epoch in range(2):
        perm = rng.permutation(M).astype(np.uint32)
        for s0 in range(0, M, B):
            sl = perm[s0:s0 + B]
            new_is_b = np.full(sl.size, epoch == 0)
            ev = events(sl, new_is_b)
            if zc:
                # the watch reader writes each event's JSON into the engine's pinned memory in the upload layout;
                # the old objects stay where the informer cache holds them (read only on a collision)
                nstart = np.where(new_is_b, offs[2 * sl.astype(np.int64) + 1], offs[2 * sl.astype(np.int64)])
                pd = G.PinnedDocs.of_ranges(eng, buf, nstart, ev["new_len"])
                ev["new_json"] = pd.ptrs
                pinned.append(pd)
            cycle.append((sl, new_is_b, ev))
    if zc:
        log("zero copy: %d batches rendered into pinned buffers (%.2f GB) in %.1f s" % (
            len(pinned), sum(p.nbytes for p in pinned) / 1e9, time.time() - t_pin))
    up_bytes = [int(c[2]["new_len"].sum()) for c in cycle]
    min_batches = args.batches if args.seconds <= 0 else 0
    lat, bytes_up = [], 0
    results = []  # (pair flags, cycle index) of every timed batch: checked after the clock stops
    t_sub, t_wait = [], []  # host time inside submit / wait per timed batch
    done_at = []  # completion time of every timed batch (the throughput series)
    ss0 = None
    mism = 0
    checked = 0
    sample_ok = None
    first_res = None
    inflight = []  # (ticket, t_submit, cycle index, timed)
    eng.timing_reset()
    t_start = None
    k = 0
    n_timed = ev_total = 0
    while True:
        if k == args.warmup_batches:
            # drain the warmup batches, then start the clock
            while inflight:
                eng.wait(inflight.pop(0)[0])
            eng.timing_reset()
            ss0 = st.stats()
            t_start = time.time()
        timed = k >= args.warmup_batches
        if timed:
            el = time.time() - t_start
            if (args.seconds > 0 and el >= args.seconds) or (args.seconds <= 0 and n_timed >= min_batches):
                break
        ci = k % len(cycle)
        ts = time.time()
        tk = submit(cycle[ci][2])
        if timed:
            t_sub.append(time.time() - ts)
            # device encoding uploads the events' JSON; host encoding the encoded blobs
            bytes_up += up_bytes[ci] if dev_enc else st.stats().last_batch_bytes
            n_timed += 1
            ev_total += cycle[ci][0].size
        inflight.append((tk, ts, ci, timed))
        if len(inflight) == 2:
            tk0, ts0, c0, tm0 = inflight.pop(0)
            tw = time.time()
            r = eng.wait(tk0)
            if tm0:
                now = time.time()
                t_wait.append(now - tw)
                lat.append(now - ts0)
                done_at.append(now - t_start)
                results.append((r.pair_flags, c0))
                if first_res is None:
                    first_res = (r, cycle[c0])
        k += 1
    while inflight:
        tk0, ts0, c0, tm0 = inflight.pop(0)
        tw = time.time()
        r = eng.wait(tk0)
        now = time.time()
        t_wait.append(now - tw)
        lat.append(now - ts0)
        done_at.append(now - t_start)
        results.append((r.pair_flags, c0))
        if first_res is None:  # a run whose every timed batch is waited here
            first_res = (r, cycle[c0])
    t_end = time.time()
    el = t_end - t_start
    n_batches = n_timed
    for f, c0 in results:  # every timed decision against the generator's ground truth
        f = f & 3
        mism += int((f != (exp_ab[cycle[c0][0]] & 3)).sum())
        checked += f.size
    # sustained rate per whole second of the run (batches completed in each 1-s window x B)
    done_at = np.array(done_at)
    per_s = [int(((done_at >= w) & (done_at < w + 1)).sum()) * B for w in range(int(el))]
    batches = cycle
    tm = eng.timings()
    ss = st.stats()

    def window(f):  # the mean of a per-batch store timing over the timed batches only
        n1, n0 = ss.timing_batches, ss0.timing_batches
        return (getattr(ss, f) * n1 - getattr(ss0, f) * n0) / max(1, n1 - n0)
    lat_ms = np.array(lat) * 1e3

    # ---- CPU baseline leg: the oracle's C++ port on a sample of the timed events
    # (decoded trees; JSON decode untimed) and, as checker, the Python oracle on
    # the first timed batch (flags + changed paths bit-exact)
    cpu = None
    if not args.no_cpu_baseline and first_res is not None:
        if args.sample and first_res is not None:
            sample_ok = _sample_check(first_res[0], first_res[1], buf, offs, args.sample)
            log("sample bit-exact vs oracle:", sample_ok)
        from oracle import cpu_ref
        sl, new_is_b, _ = first_res[1]
        m = min(args.cpu_sample, sl.size)
        pairs = []
        for i in range(m):
            s_ = int(sl[i])
            a = bytes(buf[offs[2 * s_]:offs[2 * s_ + 1]])
            b = bytes(buf[offs[2 * s_ + 1]:offs[2 * s_ + 2]])
            pairs.append((a, b) if new_is_b[i] else (b, a))
        dp = cpu_ref.DecodedPairs(pairs)
        cflags, sweeps, sec = dp.decide(threads=ncpu, min_seconds=args.cpu_seconds)
        dp.close()
        agree = bool(((cflags & 3) == (first_res[0].pair_flags[:m] & 3)).all()) if first_res else None
        cpu = dict(value=m * sweeps / sec, unit="events/s", cores=ncpu, kind="port",
                   sample="%d events of the first timed batch, old+new JSON decoded untimed (the informer "
                          "decodes them), predicates only, %d sweeps in %.1f s; decisions agree with GPU: %s" % (
                              m, sweeps, sec, agree))
        log("cpu baseline:", json.dumps(cpu))
    line = {
        "metric": "watch-replay Update events/s (device-resident old objects, JSON in, decisions + changed paths out)",
        "value": ev_total / el,
        "unit": "events/s",
        "n_gpus": 1,
        "steps": n_batches,
        "warmup": args.warmup_batches,
        "ms_per_step": el / n_batches * 1e3,
        "higher_is_better": True,
        "scaling": "replicas only",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (config3 object mix; each event alternates an object's two seeded versions)",
        "config": {"workload": "config5: %d resident objects, batches of %d events, 2 in flight, %s%s" % (
            M, B, ("time-based: >= %.0f s sustained" % args.seconds) if args.seconds > 0 else "%d batches" % n_batches,
            ", zero-copy upload (events' JSON in engine-pinned memory)" if zc else ""),
                   "zero_copy": zc, "zero_copy_batches": int(ss.zero_copy_batches - ss0.zero_copy_batches),
                   "encode": "device (K0 JSON tokenizer/encoder in HBM)" if dev_enc else "host (%d threads)" % threads,
                   "host_threads": threads},
        "duration_s": el,
        "latency_ms": {"p50": float(np.percentile(lat_ms, 50)), "p99": float(np.percentile(lat_ms, 99)),
                       "max": float(lat_ms.max()), "def": "submit call -> results on the host, per batch of %d" % B},
        "events_per_second_window": {"series": per_s, "min": min(per_s) if per_s else None,
                                     "max": max(per_s) if per_s else None,
                                     "def": "events of the batches completed in each whole second of the run"},
        "h2d_gbps": bytes_up / el / 1e9,
        "gpu_ms_per_batch": {"diff_pass": tm.total_ms, "k2": tm.compare_ms},
        "store": {"resident_gb": ss.live_bytes / 1e9, "compactions": ss.compactions, "reseeded": ss.reseeded,
                  "old_objects_encoded": ss.old_encoded, "deferred_to_host": ss.deferred},
        "batch_ms": {"host_submit": window("host_submit_ms"), "h2d": window("h2d_ms"),
                     "k0_encode": window("encode_ms"), "k0c_k0x_link": window("link_ms"), "diff_pass": tm.total_ms,
                     "submit_split": {f: window(f) for f in ("submit_wait_ms", "submit_docs_ms", "submit_copy_ms",
                                                             "submit_enqueue_ms")},
                     "store_finish": window("finish_ms"),
                     "submit_call": float(np.mean(t_sub) * 1e3), "wait_call": float(np.mean(t_wait) * 1e3),
                     "share_of_step": {"k0_encode": window("encode_ms") / (el / n_batches * 1e3),
                                       "host_staging_copy": window("submit_copy_ms") / (el / n_batches * 1e3),
                                       "h2d": window("h2d_ms") / (el / n_batches * 1e3),
                                       "def": "per-batch phase time / the sustained time per batch (phases of "
                                              "neighbouring batches overlap, so shares can sum past 1)"}}
        if dev_enc else None,
        "initial_list_objects_per_s": M / t_load,
        "checks": {"events_checked": checked, "decision_mismatches_vs_ground_truth": mism,
                   "sample_bit_exact_vs_oracle": sample_ok},
        "cpu_baseline": cpu,
    }
    from kcp_amd import gpudiff as _G
    line["build_id"] = _G.BUILD_ID  # the loaded library's source hash (kcp_amd/buildinfo.py)
    print(json.dumps(line), flush=True)
    st.free()
    for pd in pinned:
        pd.free()
    eng.close()


def _sample_check(r, batch, buf, offs, n):
    """First n events of a batch: flags + changed paths bit-exact vs the oracle."""
    from oracle import gpudiff_oracle as O
    from tests.parity import expected_flags, expected_paths

    sl, new_is_b, _ = batch
    n = min(n, sl.size)
    pos = {int(d): k for k, d in enumerate(r.dirty_ids.tolist())}
    for i in range(n):
        s = int(sl[i])
        a = bytes(buf[offs[2 * s]:offs[2 * s + 1]])
        b = bytes(buf[offs[2 * s + 1]:offs[2 * s + 2]])
        old, new = (a, b) if new_is_b[i] else (b, a)
        e = O.diff_pair(old, new)
        if int(r.pair_flags[i]) != expected_flags(e):
            return False
        if i in pos:
            if r.paths_of(pos[i]) != expected_paths(e):
                return False
        elif e["paths"]:
            return False
    return True
