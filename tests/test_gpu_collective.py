"""The multi-GPU step's collective over RCCL ("nccl" backend = RCCL on ROCm) on
real hardware at world_size 1: shard.DirtyGather (the bench's per-step
all-gather, IDs exported straight from HBM with gpudiff_dbatch_export, a
capacity overflow regrown inside the step) and shard.gather_dirty return the node-wide dirty sets
of a diffed device batch.  World size 2 of the same code runs on CPU (gloo) in
tests/test_multirank.py."""
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist

from kcp_amd import gpudiff as G
from kcp_amd import shard
from tests.workload import make_pairs

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_dirty_gather_over_rccl_world1():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % _port(), rank=0, world_size=1,
                            device_id=dev)
    try:
        stream = torch.cuda.Stream(device=dev)  # shared with the engine and current: exports, copies and the
        torch.cuda.set_stream(stream)            # collectives order on one stream (the null stream cannot be shared)
        eng = G.Engine(device=0, stream=stream.cuda_stream)
        pairs, _, _ = make_pairs(3000, seed=21, mutate_frac=0.3, pretty_frac=0)
        hb = eng.encode(pairs)
        db = eng.device_batch(hb.info().pool_bytes + 4096, len(pairs))
        db.append(hb)
        want = eng.wait(eng.diff(db))
        counts = torch.zeros(8, dtype=torch.int32, device=dev)
        db.export(G.EXPORT_COUNTS, counts.data_ptr(), 8)
        torch.cuda.synchronize()
        cap_s, cap_t = shard.DirtyGather.agree_capacity(counts, 1, dist)
        assert (cap_s, cap_t) == (want.spec_dirty_ids.size + 1, want.status_dirty_ids.size + 1)

        def fill_counts(t):
            db.export(G.EXPORT_COUNTS, t.data_ptr(), 8)

        def fill_ids(col, buf):
            db.export(G.EXPORT_SPEC_IDS if col == 0 else G.EXPORT_STATUS_IDS, buf.data_ptr(), buf.numel(),
                      buf.numel())
        for depth in (1, 2, 3):  # serial, and pipelined (step s's collective overlaps step s+1's diff)
            g = shard.DirtyGather(1, cap_s, cap_t, dev, dist, depth=depth)
            for _ in range(5):  # diff + collective, no host sync in between
                eng.diff(db)
                g.step(fill_counts, fill_ids)
            g.finish()
            torch.cuda.synchronize()
            for b in range(depth):  # every buffer of the ring holds a full step's gather
                rows = g.alls[b].view(1, g.width)
                assert int(rows[0, 0]) == want.spec_dirty_ids.size and int(rows[0, 1]) == want.status_dirty_ids.size
            sa, ta = g.result()
            assert np.array_equal(sa.cpu().numpy().astype(np.uint32), want.spec_dirty_ids)
            assert np.array_equal(ta.cpu().numpy().astype(np.uint32), want.status_dirty_ids)
        # the engine writes counts + IDs into the send buffer itself (gpudiff_dbatch_bind_gather): no export
        # copies per step; the fills run only after a regrow (capacity below the count: the first step)
        bind = lambda send, cs, ct: db.bind_gather(send.data_ptr(), cs, ct)  # noqa: E731
        for depth, caps in ((1, (cap_s, cap_t)), (2, (cap_s, cap_t)), (1, (max(1, cap_s // 2), max(1, cap_t // 3)))):
            g = shard.DirtyGather(1, caps[0], caps[1], dev, dist, depth=depth, bind=bind)
            for _ in range(4):
                g.begin_step()
                eng.diff(db)
                g.step(fill_counts, fill_ids)
            g.finish()
            torch.cuda.synchronize()
            sa, ta = g.result()
            assert np.array_equal(sa.cpu().numpy().astype(np.uint32), want.spec_dirty_ids)
            assert np.array_equal(ta.cpu().numpy().astype(np.uint32), want.status_dirty_ids)
            assert g.n_regrows == (1 if caps[0] < cap_s else 0)
            cnt = g._rows()[0, :8].cpu().tolist()
            assert cnt[:3] == [want.spec_dirty_ids.size, want.status_dirty_ids.size, want.dirty_ids.size]
            if not g.n_regrows:  # words 4..7: zero from the binding (a regrow's export copies the summary's)
                assert cnt[4:] == [0, 0, 0, 0]
        # lookahead: step s checked after step s + 1 is queued; a capacity below the count is found one step
        # late and re-gathered from the engine's alternate result slot (and so is the in-flight step)
        for caps in ((cap_s, cap_t), (max(1, cap_s // 2), max(1, cap_t // 3))):
            g = shard.DirtyGather(1, caps[0], caps[1], dev, dist, bind=bind, slot=lambda k: db.result_slot(k))
            for _ in range(5):
                g.begin_step()
                eng.diff(db)
                g.step(fill_counts, fill_ids)
            g.finish()
            torch.cuda.synchronize()
            ok, cc = g.check()
            assert ok and g.n_regrows == (1 if caps[0] < cap_s else 0)
            sa, ta = g.result()
            assert np.array_equal(sa.cpu().numpy().astype(np.uint32), want.spec_dirty_ids)
            assert np.array_equal(ta.cpu().numpy().astype(np.uint32), want.status_dirty_ids)
        db.result_slot(0)
        # each slot keeps the lists of the last diff made under it
        r0 = eng.wait(eng.diff(db))
        db.result_slot(1)
        r1 = eng.wait(eng.diff(db))
        assert np.array_equal(r0.spec_dirty_ids, r1.spec_dirty_ids) and np.array_equal(r1.spec_dirty_ids, want.spec_dirty_ids)
        db.result_slot(0)
        db.bind_gather(0, 0, 0)
        # a capacity below the dirty count: regrown inside the first step, exact from then on
        g = shard.DirtyGather(1, max(1, cap_s // 2), max(1, cap_t // 3), dev, dist)
        for _ in range(3):
            eng.diff(db)
            g.step(fill_counts, fill_ids)
        g.finish()
        assert g.n_regrows == 1 and g.cap[0] >= want.spec_dirty_ids.size
        sa, ta = g.result()
        assert np.array_equal(sa.cpu().numpy().astype(np.uint32), want.spec_dirty_ids)
        assert np.array_equal(ta.cpu().numpy().astype(np.uint32), want.status_dirty_ids)
        # the general (trimmed) form
        s2, t2 = shard.gather_dirty(counts, lambda col, buf, k: db.export(
            G.EXPORT_SPEC_IDS if col == 0 else G.EXPORT_STATUS_IDS, buf.data_ptr(), buf.numel(), k), 0, 1, dist, dev)
        assert np.array_equal(s2.cpu().numpy().astype(np.uint32), want.spec_dirty_ids)
        assert np.array_equal(t2.cpu().numpy().astype(np.uint32), want.status_dirty_ids)
        # two passes in flight (shard.PipelinedGather, the bench's default): a second context on its own stream
        # diffs a view of the batch on alternate steps, each pass's compaction writes its own bound send buffer,
        # its collective runs on its stream; a capacity below the count is found one step late and both
        # passes' steps are re-gathered from their still-intact lists
        stream2 = torch.cuda.Stream(device=dev)
        eng2 = G.Engine(device=0, stream=stream2.cuda_stream)
        db2 = db.view(eng2)
        engs, dbs = [eng, eng2], [db, db2]
        binds = [lambda send, cs, ct, d=d: d.bind_gather(send.data_ptr(), cs, ct) for d in dbs]

        def fill_counts2(p, t):
            dbs[p].export(G.EXPORT_COUNTS, t.data_ptr(), 8, 8)

        def fill_ids2(p, col, buf):
            dbs[p].export(G.EXPORT_SPEC_IDS if col == 0 else G.EXPORT_STATUS_IDS, buf.data_ptr(), buf.numel(),
                          buf.numel())
        for caps in ((cap_s, cap_t), (max(1, cap_s // 2), max(1, cap_t // 3))):
            g = shard.PipelinedGather(1, caps[0], caps[1], dev, dist, [stream, stream2], binds)
            for s in range(6):
                engs[s % 2].diff(dbs[s % 2])
                g.step(fill_counts2, fill_ids2)
            g.finish()
            torch.cuda.synchronize()
            ok, cc = g.check()
            assert ok and g.n_regrows == (1 if caps[0] < cap_s else 0)
            assert [int(x) for x in cc[0, :2]] == [want.spec_dirty_ids.size, want.status_dirty_ids.size]
            sa, ta = g.result()
            assert np.array_equal(sa.cpu().numpy().astype(np.uint32), want.spec_dirty_ids)
            assert np.array_equal(ta.cpu().numpy().astype(np.uint32), want.status_dirty_ids)
        for d in dbs:
            d.bind_gather(0, 0, 0)
        db2.free()  # the view before its base
        eng2.close()
        db.free()
        hb.free()
        eng.close()
    finally:
        torch.cuda.set_stream(torch.cuda.default_stream(dev))
        dist.destroy_process_group()


def test_lookahead_regrow_with_changing_counts():
    """with lookahead, a capacity overflow found one step late re-gathers step s from its result
    slot after step s + 1 has run.  The counts must be step s's too (the summary is per result slot): here step
    0 diffs 3000 pairs, then 1000 more are appended, so step 1's counts differ from step 0's; every gather --
    the regrow's re-gathers included -- must carry its own step's counts and exactly its own step's IDs."""
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % _port(), rank=0, world_size=1,
                            device_id=dev)
    try:
        stream = torch.cuda.Stream(device=dev)
        torch.cuda.set_stream(stream)
        eng = G.Engine(device=0, stream=stream.cuda_stream)
        pa, _, _ = make_pairs(3000, seed=31, mutate_frac=0.3, pretty_frac=0)
        pb, _, _ = make_pairs(1000, seed=32, mutate_frac=0.6, pretty_frac=0)
        ha, hb = eng.encode(pa), eng.encode(pb)
        cap = ha.info().pool_bytes + hb.info().pool_bytes + 8192
        want = []
        for parts in ((ha,), (ha, hb)):
            d = eng.device_batch(cap, len(pa) + len(pb))
            for h in parts:
                d.append(h)
            r = eng.wait(eng.diff(d))
            want.append((r.spec_dirty_ids.copy(), r.status_dirty_ids.copy()))
            d.free()
        # pair IDs of the appended batch continue after the first one's
        assert want[1][0].size > want[0][0].size and want[1][1].size > want[0][1].size
        db = eng.device_batch(cap, len(pa) + len(pb))
        db.append(ha)
        bind = lambda send, cs, ct: db.bind_gather(send.data_ptr(), cs, ct)  # noqa: E731

        def fill_counts(t):
            db.export(G.EXPORT_COUNTS, t.data_ptr(), 8)

        def fill_ids(col, buf):
            db.export(G.EXPORT_SPEC_IDS if col == 0 else G.EXPORT_STATUS_IDS, buf.data_ptr(), buf.numel(),
                      buf.numel())
        caps = (max(1, want[0][0].size // 2), max(1, want[0][1].size // 2))
        g = shard.DirtyGather(1, caps[0], caps[1], dev, dist, bind=bind, slot=lambda k: db.result_slot(k))
        g.trace = True
        for s in range(4):
            if s == 1:
                db.append(hb)
            g.begin_step()
            eng.diff(db)
            g.step(fill_counts, fill_ids)
        g.finish()
        torch.cuda.synchronize()
        assert g.n_regrows >= 1
        seen = set()
        for step, (cs, ct), rows in g.gathered:
            w = want[0] if step == 0 else want[1]
            n_s, n_t = int(rows[0, 0]), int(rows[0, 1])
            assert (n_s, n_t) == (w[0].size, w[1].size), (step, n_s, n_t)
            if n_s <= cs and n_t <= ct:  # a complete gather: exactly that step's lists
                seen.add(step)
                assert np.array_equal(rows[0, 8:8 + n_s].numpy().astype(np.uint32), w[0]), step
                assert np.array_equal(rows[0, 8 + cs:8 + cs + n_t].numpy().astype(np.uint32), w[1]), step
        assert {0, 1, 2, 3} <= seen  # step 0 was re-gathered complete after step 1 ran
        sa, ta = g.result()
        assert np.array_equal(sa.cpu().numpy().astype(np.uint32), want[1][0])
        db.bind_gather(0, 0, 0)
        db.free()
        ha.free()
        hb.free()
        eng.close()
    finally:
        torch.cuda.set_stream(torch.cuda.default_stream(dev))
        dist.destroy_process_group()
