"""World-size-2 coverage of the multi-GPU path on CPU (gloo): logical-cluster
sharding (LPT, clusters never split, all pairs covered exactly once) and the
all-gather of dirty counts and IDs, checked against a single-rank view."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from kcp_amd import shard
from kcp_amd import synth as S


def test_lpt_assign_balanced():
    w = [100, 60, 50, 40, 30, 20, 10, 10]
    owner = shard.lpt_assign(w, 2)
    loads = [sum(x for x, o in zip(w, owner) if o == r) for r in range(2)]
    assert abs(loads[0] - loads[1]) <= 10


@pytest.mark.parametrize("world", [2, 3, 8])
def test_synth_shards_partition_population(world):
    cfg = S.make_cfg("config2", n_pairs=20000, n_clusters=300)
    seen = []
    sizes = []
    for r in range(world):
        p = S.Population(cfg, world, r)
        sizes.append(p.n)
        seen.append(np.array([p.global_index(i) for i in range(p.n)], dtype=np.int64))
        p.close()
    allg = np.concatenate(seen)
    assert allg.size == cfg.n_pairs and np.unique(allg).size == cfg.n_pairs
    assert max(sizes) - min(sizes) <= max(sizes) * 0.2  # LPT keeps ranks within a few %


@pytest.mark.parametrize("world", [2, 8])
def test_weak_scaling_shards_are_one_config_each(world):
    """bench.py --scaling weak: the node population is world x config3 and the
    LPT shard every rank holds is one config3-sized population (per-GPU work
    fixed as N grows)."""
    base = S.make_cfg("config3")
    cfg = S.make_cfg("config3", n_pairs=base.n_pairs * world, n_clusters=base.n_clusters * world)
    sizes, clusters = [], []
    for r in range(world):
        p = S.Population(cfg, world, r)
        sizes.append(p.n)
        clusters.append(p.n_clusters)
        p.close()
    assert sum(sizes) == base.n_pairs * world and sum(clusters) <= base.n_clusters * world
    assert max(abs(x - base.n_pairs) for x in sizes) <= base.n_pairs * 0.001


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, flags_all, owners, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mine = np.nonzero(owners == rank)[0]
    f = flags_all[mine]
    spec = torch.tensor(mine[(f & 1) != 0], dtype=torch.int32)
    stat = torch.tensor(mine[(f & 2) != 0], dtype=torch.int32)
    counts = torch.zeros(8, dtype=torch.int32)
    counts[0], counts[1] = spec.numel(), stat.numel()
    sa, ta = shard.gather_dirty(counts, shard.tensor_fill(spec, stat), rank, world, dist)
    q.put((rank, sorted(sa.tolist()), sorted(ta.tolist())))
    dist.destroy_process_group()


def test_gather_dirty_gloo_world2():
    rnd = np.random.default_rng(3)
    n = 5000
    clusters = rnd.integers(0, 97, n)
    flags = rnd.integers(0, 4, n).astype(np.uint8)
    parts = shard.shard_pairs(clusters, 2)
    owners = np.zeros(n, dtype=np.int32)
    for r, idx in enumerate(parts):
        owners[idx] = r
    # a cluster never spans ranks
    for c in np.unique(clusters):
        assert np.unique(owners[clusters == c]).size == 1
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, flags, owners, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want_s = sorted(np.nonzero(flags & 1)[0].tolist())
    want_t = sorted(np.nonzero(flags & 2)[0].tolist())
    for rank, s, t in res:
        assert s == want_s and t == want_t


@pytest.mark.parametrize("world", [2, 8])
def test_strong_scaling_shards_split_one_config(world):
    """bench.py default for N > 1 (--scaling strong): the metric's population
    (config3: 10M pairs / 100k logical clusters) split N ways by whole logical
    cluster (pkg/reconciler/cluster/cluster.go:125-138: one syncer per cluster)."""
    cfg = S.make_cfg("config3")
    sizes, clusters = [], []
    for r in range(world):
        p = S.Population(cfg, world, r)
        sizes.append(p.n)
        clusters.append(p.n_clusters)
        p.close()
    assert sum(sizes) == cfg.n_pairs and sum(clusters) == cfg.n_clusters
    assert max(sizes) - min(sizes) <= cfg.n_pairs // world * 0.002


def _worker_fixed(rank, world, port, flags_all, owners, shrink, q, depth=1):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mine = np.nonzero(owners == rank)[0]
    f = flags_all[mine]
    spec = torch.tensor(mine[(f & 1) != 0], dtype=torch.int32)
    stat = torch.tensor(mine[(f & 2) != 0], dtype=torch.int32)
    counts = torch.zeros(8, dtype=torch.int32)
    counts[0], counts[1] = spec.numel(), stat.numel()
    cs, ct = shard.DirtyGather.agree_capacity(counts, world, dist)
    g = shard.DirtyGather(world, cs - shrink, ct, "cpu", dist, depth=depth)

    def fill_counts(t):
        t.copy_(counts)

    def fill_ids(col, buf):
        src = spec if col == 0 else stat
        k = min(buf.numel(), src.numel())
        buf[:k] = src[:k]
    for _ in range(3):  # repeated steps reuse the buffers (pipelined: round-robin over depth buffers)
        g.step(fill_counts, fill_ids)
    g.finish()
    ok, _ = g.check()
    if ok:
        sa, ta = g.result()
        q.put((rank, True, sorted(sa.tolist()), sorted(ta.tolist()), g.n_regrows))
    else:
        q.put((rank, False, None, None, g.n_regrows))
    dist.destroy_process_group()


def _worker_growing(rank, world, port, flags_all, owners, q):
    """A stream whose dirty count grows step by step past the agreed capacity (depth 1): every step's
    node-wide sets must be exact, the buffers regrown inside the step."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mine = np.nonzero(owners == rank)[0]
    f = flags_all[mine]
    g = None
    out = []
    for step in range(4):
        keep = (len(mine) * (step + 1)) // 4  # this step's results: a growing prefix of the rank's pairs
        spec = torch.tensor(mine[:keep][(f[:keep] & 1) != 0], dtype=torch.int32)
        stat = torch.tensor(mine[:keep][(f[:keep] & 2) != 0], dtype=torch.int32)
        counts = torch.zeros(8, dtype=torch.int32)
        counts[0], counts[1] = spec.numel(), stat.numel()
        if g is None:
            cs, ct = shard.DirtyGather.agree_capacity(counts, world, dist)
            g = shard.DirtyGather(world, cs, ct, "cpu", dist)

        def fill_counts(t):
            t.copy_(counts)

        def fill_ids(col, buf):
            src = spec if col == 0 else stat
            k = min(buf.numel(), src.numel())
            buf[:k] = src[:k]
        g.step(fill_counts, fill_ids)
        sa, ta = g.result()
        out.append((sorted(sa.tolist()), sorted(ta.tolist())))
    q.put((rank, out, g.n_regrows))
    dist.destroy_process_group()


def test_dirty_gather_regrows_inside_the_step_gloo_world2():
    rnd = np.random.default_rng(5)
    n = 4000
    clusters = rnd.integers(0, 61, n)
    flags = rnd.integers(0, 4, n).astype(np.uint8)
    owners = np.zeros(n, dtype=np.int32)
    for r, idx in enumerate(shard.shard_pairs(clusters, 2)):
        owners[idx] = r
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_growing, args=(r, 2, port, flags, owners, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, out, regrows in res:
        assert regrows >= 1
        for step, (s, t) in enumerate(out):
            sel = np.zeros(n, dtype=bool)
            for r in range(2):
                mine = np.nonzero(owners == r)[0]
                sel[mine[:(len(mine) * (step + 1)) // 4]] = True
            assert s == sorted(np.nonzero(sel & ((flags & 1) != 0))[0].tolist())
            assert t == sorted(np.nonzero(sel & ((flags & 2) != 0))[0].tolist())


@pytest.mark.parametrize("shrink,depth", [(0, 1), (5, 1), (0, 2), (5, 2), (0, 3)])
def test_dirty_gather_fixed_capacity_gloo_world2(shrink, depth):
    """The bench's per-step collective (shard.DirtyGather, one all-gather per
    step): node-wide dirty sets equal the single-rank view; a capacity below a
    rank's count is regrown inside the step (depth 1) or reported (pipelined),
    never truncated silently."""
    rnd = np.random.default_rng(4)
    n = 4000
    clusters = rnd.integers(0, 61, n)
    flags = rnd.integers(0, 4, n).astype(np.uint8)
    owners = np.zeros(n, dtype=np.int32)
    for r, idx in enumerate(shard.shard_pairs(clusters, 2)):
        owners[idx] = r
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_fixed, args=(r, 2, port, flags, owners, shrink, q, depth)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want_s = sorted(np.nonzero(flags & 1)[0].tolist())
    want_t = sorted(np.nonzero(flags & 2)[0].tolist())
    for rank, ok, s, t, regrows in res:
        if shrink and depth > 1:
            assert not ok  # pipelined: an overflow in any step is reported, never accepted
        else:
            # depth 1: a capacity below a rank's count is regrown inside the step, the sets stay exact
            assert ok and s == want_s and t == want_t
            assert regrows == (1 if shrink else 0)


# ---------------------------------------------------------------- byte-weighted sharding
def _pair_compare_bytes_py(r):
    """Restatement of gpudiff_format.h gpudiff_pair_compare_bytes for one ROW_DTYPE record."""
    from kcp_amd import gpudiff as G
    b = 65
    if (int(r["flags_a"]) | int(r["flags_b"])) & G.OBJ_DECODE_ERR:
        return b
    seg = lambda l, ar: 16 * int(l) + int(ar)  # noqa: E731
    spec_sz = r["spec_l_a"] == r["spec_l_b"] and r["spec_ar_a"] == r["spec_ar_b"]
    stat_sz = bool(int(r["flags_b"]) & G.OBJ_HAS_STATUS) and r["stat_l_a"] == r["stat_l_b"] and \
        r["stat_ar_a"] == r["stat_ar_b"]
    ss, st = seg(r["spec_l_a"], r["spec_ar_a"]), seg(r["stat_l_a"], r["stat_ar_a"])
    up = lambda x: (x + 127) & ~127  # noqa: E731
    if spec_sz and stat_sz:
        per = up(ss + st)
    elif spec_sz:
        per = ss if (int(r["stat_l_a"]) | int(r["stat_l_b"]) | int(r["stat_ar_a"]) | int(r["stat_ar_b"])) else up(ss)
    elif stat_sz:
        per = st
    else:
        per = 0
    return b + 2 * per


def test_shard_lpt_c_equals_restatement():
    from kcp_amd import gpudiff as G
    rnd = np.random.default_rng(5)
    for world in (1, 2, 3, 8, 16):
        for w in (rnd.integers(0, 1 << 40, 3000), rnd.integers(0, 5, 500), np.zeros(7, np.int64)):
            assert np.array_equal(G.shard_lpt(w.astype(np.uint64), world), shard.lpt_assign(w, world))
    with pytest.raises(G.GpuDiffError):
        G.shard_lpt(np.ones(3, np.uint64), 0)


def test_cluster_bytes_equal_row_formula():
    """gpudiff_cluster_bytes sums gpudiff_pair_compare_bytes by cluster; held to a Python restatement over
    encoded synthetic rows of every kind (and the engine's own compare_bytes total)."""
    from kcp_amd import gpudiff as G
    e = G.Engine(device=G.DEVICE_NONE)
    for name in ("config3", "config4"):
        cfg = S.make_cfg(name, n_pairs=3000, n_clusters=40)
        p = S.Population(cfg)
        ch = p.chunk(e, 0, p.n, 4)
        rows = ch.hb.rows()
        got = G.cluster_bytes(rows, cfg.n_clusters)
        want = np.zeros(cfg.n_clusters, np.uint64)
        for r in rows:
            want[int(r["cluster_id"])] += _pair_compare_bytes_py(r)
        assert np.array_equal(got, want)
        # the synth's per-cluster weights are the same sums
        assert np.array_equal(S.cluster_bytes(cfg, threads=4), want)
        with pytest.raises(G.GpuDiffError):
            G.cluster_bytes(rows, 1)  # cluster ids past n_clusters
        ch.hb.free()
        p.close()
    e.close()


@pytest.mark.parametrize("world", [2, 8])
def test_byte_weighted_shards_partition_and_balance(world):
    """Ranks packed by Σ B_pair: every pair exactly once, whole clusters, the same owner as gpudiff_shard_lpt,
    and byte loads at least as balanced as the pair-count rule's."""
    from kcp_amd import gpudiff as G
    cfg = S.make_cfg("config3", n_pairs=60000, n_clusters=600)
    w = S.cluster_bytes(cfg, threads=4)
    sizes = S.cluster_sizes(cfg)
    owner = G.shard_lpt(w, world)
    seen = []
    for r in range(world):
        p = S.Population(cfg, world, r, cluster_weight=w)
        assert p.n == int(sizes[owner == r].sum())
        seen.append(p.local_ids().astype(np.int64))
        p.close()
    allg = np.concatenate(seen)
    assert allg.size == cfg.n_pairs and np.unique(allg).size == cfg.n_pairs
    lb = np.bincount(owner, weights=w.astype(float), minlength=world)
    lc = np.bincount(shard.lpt_assign(sizes, world), weights=w.astype(float), minlength=world)
    assert lb.max() <= lc.max() and lb.max() / lb.mean() < 1.01


def _weights_worker(rank, world, port, q):
    """bench.py's shard_population at world 2 over gloo: the stride-split weight computation summed by an
    all-reduce equals one rank computing every cluster."""
    import argparse
    import bench
    from kcp_amd import gpudiff as G
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = S.make_cfg("config3", n_pairs=20000, n_clusters=300)
    args = argparse.Namespace(emulate_world=0, emulate_rank=-1, shard_weight="bytes")
    info, pop = bench.shard_population(args, cfg, world, rank, 2, torch.device("cpu"), dist, G, S)
    q.put((rank, info, pop.local_ids().tolist()))
    dist.destroy_process_group()


def test_bench_shard_population_gloo_world2():
    from kcp_amd import gpudiff as G
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_weights_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = sorted(q.get(timeout=300) for _ in range(world))
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    cfg = S.make_cfg("config3", n_pairs=20000, n_clusters=300)
    w = S.cluster_bytes(cfg, threads=4)
    owner = G.shard_lpt(w, world)
    sizes = S.cluster_sizes(cfg)
    for r, info, ids in out:
        assert info["rule"] == "LPT by sum of B_pair" and info["rank_pairs"] == int(sizes[owner == r].sum())
        assert info["total_bytes"] == int(w.sum())
    assert sorted(sum((o[2] for o in out), [])) == list(range(cfg.n_pairs))
