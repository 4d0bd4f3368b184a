"""Gate -> write on the device: for batches diffed
through the device-encode submit path, gpudiff_write_plan_get[_ex] lists the
writes the syncer issues -- spec-dirty pairs: an upsertIntoDownstream body;
status-dirty pairs: an updateStatusInUpstream body -- rendered by K10 from the
JSON still staged in HBM, with the write-path no-op rule (no body, call
skipped).  For informer (old, new) pairs (the default) both render the NEW
object, the one UpdateFunc enqueues (specsyncer.go:47-50); for (upstream,
downstream) pairs the spec write renders A.  Everything is compared with
oracle/upsert_oracle.write_plan, i.e. the oracle's decisions, no-op rule and
Go-exact bodies."""
import json
import random

import pytest

from kcp_amd import gpudiff as G
from oracle import upsert_oracle as U
from tests.golden.kat_cases import BASE, J, cases
from tests.parity import assert_matches
from tests.workload import make_pairs

pytestmark = pytest.mark.gpu


def _check(eng, pairs, mode=G.PLAN_INFORMER):
    t = eng.submit(pairs)
    res = eng.wait(t)
    assert_matches(res, pairs)
    plan = eng.write_plan(t, mode)
    want = U.write_plan(pairs, mode)
    got = list(zip(plan.pair_index.tolist(), plan.kind.tolist(), [bool(x) for x in plan.noop], plan.bodies))
    assert len(got) == len(want)
    for g, w in zip(got, want):
        assert g == w, (g[:3], w[:3], (g[3] or b"")[:200], (w[3] or b"")[:200])
    return plan


def _noop_pairs(n, seed):
    """int <-> integral-float retypes (no-op writes) mixed with real edits."""
    rnd = random.Random(seed)
    out = []
    for i in range(n):
        a = json.loads(J(BASE))
        a["spec"]["replicas"] = rnd.randint(0, 50)
        a["status"]["readyReplicas"] = rnd.randint(0, 50)
        ja = J(a)
        k = i % 5
        if k == 0:    # spec no-op
            jb = ja.replace(b'"replicas":%d,"selector"' % a["spec"]["replicas"],
                            b'"replicas":%d.0,"selector"' % a["spec"]["replicas"])
        elif k == 1:  # status no-op
            jb = ja.replace(b'"readyReplicas":%d' % a["status"]["readyReplicas"],
                            b'"readyReplicas":%de0' % a["status"]["readyReplicas"])
        elif k == 2:  # a real spec edit beside a retype
            jb = ja.replace(b'"replicas":%d,"selector"' % a["spec"]["replicas"],
                            b'"replicas":%d.0,"selector"' % a["spec"]["replicas"]).replace(
                b'"revisionHistoryLimit":10', b'"revisionHistoryLimit":12')
        elif k == 3:  # no status on either side: the status write is a no-op
            b = json.loads(ja)
            del b["status"]
            ja = jb = J(b)
        else:         # identical
            jb = ja
        out.append((ja, jb))
    return out


def test_write_plan_kat_and_noops():
    eng = G.Engine(device=0, device_encode=True)
    pairs = [(a, b) for _, a, b, _, _ in cases()]
    plan = _check(eng, pairs)
    assert plan.noop.any()
    np_ = _noop_pairs(200, 1)
    plan = _check(eng, np_)
    assert plan.noop.sum() >= 100 and (plan.noop == 0).any()
    eng.close()


@pytest.mark.parametrize("seed", [2, 3])
def test_write_plan_populations(seed):
    eng = G.Engine(device=0, device_encode=True, encode_threads=8)
    pairs, _, _ = make_pairs(1500, seed=seed, mutate_frac=0.3)
    _check(eng, pairs)
    deep, _, _ = make_pairs(100, seed=seed + 10, mix=(("crd", 1.0),), mutate_frac=0.6, crd_leaves=1200)
    _check(eng, deep)
    eng.close()


def test_write_plan_two_batches_in_flight_and_state_errors():
    eng = G.Engine(device=0, device_encode=True)
    p1, _, _ = make_pairs(300, seed=7, mutate_frac=0.3)
    p2, _, _ = make_pairs(400, seed=8, mutate_frac=0.3)
    t1 = eng.submit(p1)
    t2 = eng.submit(p2)
    with pytest.raises(G.GpuDiffError):  # not waited yet
        eng.write_plan(t2)
    eng.wait(t1)
    eng.wait(t2)
    want2 = U.write_plan(p2)
    want1 = U.write_plan(p1)
    plan2 = eng.write_plan(t2)
    plan1 = eng.write_plan(t1)
    assert [(int(i), int(k), bool(z), b) for i, k, z, b in zip(plan1.pair_index, plan1.kind, plan1.noop,
                                                               plan1.bodies)] == want1
    assert [(int(i), int(k), bool(z), b) for i, k, z, b in zip(plan2.pair_index, plan2.kind, plan2.noop,
                                                               plan2.bodies)] == want2
    t3 = eng.submit(p1)
    eng.wait(t3)
    with pytest.raises(G.GpuDiffError):  # t1's staging was reused by t3
        eng.write_plan(t1)
    host = G.Engine(device=0)  # host-encoded batches keep no JSON in HBM
    th = host.submit(p1)
    host.wait(th)
    with pytest.raises(G.GpuDiffError):
        host.write_plan(th)
    host.close()
    eng.close()


def test_write_plan_informer_renders_new_object():
    """an informer Update (old, new) that changes the spec must write NEW downstream
    (UpdateFunc -> AddToQueue(gvr, newObj), specsyncer.go:47-50 -> upsertIntoDownstream); rendering old
    would push the stale version and undo the change."""
    eng = G.Engine(device=0, device_encode=True)
    pairs = []
    for i in range(40):
        a = json.loads(J(BASE))
        a["spec"]["replicas"] = i
        b = json.loads(J(a))
        b["spec"]["replicas"] = i + 100
        b["status"]["readyReplicas"] = i + 7
        b["metadata"]["resourceVersion"] = "rv-%d" % i
        pairs.append((J(a), J(b)))
    t = eng.submit(pairs)
    eng.wait(t)
    for mode in (G.PLAN_INFORMER, G.PLAN_SPEC, G.PLAN_STATUS, G.PLAN_UPSTREAM_DOWNSTREAM,
                 G.PLAN_UPSTREAM_DOWNSTREAM | G.PLAN_SPEC):
        plan = eng.write_plan(t, mode)
        want = U.write_plan(pairs, mode)
        got = list(zip(plan.pair_index.tolist(), plan.kind.tolist(), [bool(x) for x in plan.noop], plan.bodies))
        assert got == want, mode
        kinds = set(plan.kind.tolist())
        assert kinds == ({G.UPSERT_SPEC} if mode & 3 == G.PLAN_SPEC else {G.UPSERT_STATUS} if mode & 3 == G.PLAN_STATUS
                         else {G.UPSERT_SPEC, G.UPSERT_STATUS})
        for i, k, body in zip(plan.pair_index.tolist(), plan.kind.tolist(), plan.bodies):
            side = 0 if (k == G.UPSERT_SPEC and mode & G.PLAN_UPSTREAM_DOWNSTREAM) else 1
            assert body == U.upsert_body(pairs[i][side], k)
            if side == 1:
                assert b'"replicas":%d' % (i + 100) in body
    eng.close()


def _escaped_key_pairs(n, seed):
    """Pairs whose new object has a key that needs unescaping (K10 hands such documents to the host path)
    beside plain edits."""
    rnd = random.Random(seed)
    out = []
    for i in range(n):
        a = json.loads(J(BASE))
        a["spec"]["replicas"] = rnd.randint(0, 50)
        ja = J(a)
        a["spec"]["replicas"] += 1
        jb = J(a)
        if i % 3 == 0:  # a key written with an escape: "maxSurge"-style, same decoded key
            jb = jb.replace(b'"replicas"', b'"r\\u0065plicas"')
            jb = jb.replace(b'"revisionHistoryLimit":10', b'"revisionHistoryLimit":%d' % (11 + i))
        out.append((ja, jb))
    return out


def test_write_plan_zero_copy_batches_host_deferrals():
    """a zero-copy batch (gpudiff_host_alloc buffer) has no copy in the ring slot's pinned
    staging, so the write plan's host path for the documents K10 defers must not read the staging (null on a
    slot that never staged; another batch's JSON otherwise).  Fresh engine: the first batch is zero-copy (its
    slot never staged); then staged batches fill both slots with other JSON before another zero-copy batch."""
    import numpy as np
    eng = G.Engine(device=0, device_encode=True)

    def pinned(pairs):
        lens = [len(x) for p in pairs for x in p]
        offs = np.zeros(len(lens) + 1, dtype=np.int64)
        offs[1:] = np.cumsum(lens)
        buf = np.frombuffer(b"".join(x for p in pairs for x in p), dtype=np.uint8)
        return G.PinnedJson(eng, buf, offs)

    def check_plan(t, pairs):
        plan = eng.write_plan(t)
        want = U.write_plan(pairs)
        got = list(zip(plan.pair_index.tolist(), plan.kind.tolist(), [bool(x) for x in plan.noop], plan.bodies))
        assert got == want
        return plan

    zc1 = _escaped_key_pairs(60, 1)
    pj = pinned(zc1)
    t = eng.submit_array(pj.pairs)
    res = eng.wait(t)
    assert_matches(res, zc1)
    plan = check_plan(t, zc1)
    assert (plan.source == G.BODY_HOST).sum() >= 20  # the escaped-key documents went to the host path
    assert eng.submit_stats().zero_copy_batches >= 1
    # the caller may reuse its buffer once wait returned: scribble over it, the plan must not see it
    np.ctypeslib.as_array(G.C.cast(pj.ptr, G.C.POINTER(G.C.c_uint8)), (pj.nbytes,))[:] = ord("x")
    plan2 = eng.write_plan(t)
    assert plan2.bodies == plan.bodies
    pj.free()
    for seed in (2, 3):  # staged batches into both ring slots
        st = _escaped_key_pairs(40, 10 + seed)
        t2 = eng.submit(st)
        eng.wait(t2)
        check_plan(t2, st)
    zc2 = _escaped_key_pairs(50, 4)
    pj2 = pinned(zc2)
    t3 = eng.submit_array(pj2.pairs)
    eng.wait(t3)
    check_plan(t3, zc2)
    pj2.free()
    eng.close()
