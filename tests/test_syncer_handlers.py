"""Handler wiring of the syncer mirror (specsyncer.go:43-55,
statussyncer.go:29-39): which events reach AddToQueue, in what order.

CPU tests drive the batcher through its decision seam with the oracle as the
decider (test infrastructure); the GPU test drives the real engine and checks
the queue equals the one the oracle-decided reference handlers produce."""
import json

import pytest

from kcp_amd import gpudiff as G
from kcp_amd import syncer as Y
from oracle import gpudiff_oracle as O
from tests.golden.kat_cases import BASE, J, cases
from tests.parity import expected_flags, oracle_batch


def _events():
    return [(a, b) for _, a, b, _, _ in cases()]


def _reference_queue(events):
    """What the Go handlers enqueue, decided by the oracle."""
    spec_q, stat_q = [], []
    for old, new in events:
        r = O.diff_pair(old, new)
        if r["spec_dirty"]:
            spec_q.append(("deployments.apps", new))
        if r["status_dirty"]:
            stat_q.append(("deployments.apps", new))
    return spec_q, stat_q


def _oracle_decide(pairs):
    return [expected_flags(r) for r in oracle_batch(pairs)]


def test_add_delete_always_enqueue_and_status_has_no_add():
    c = Y.Controller()
    h = Y.spec_handlers(c, "deployments.apps", Y.UpdateBatcher(decide=_oracle_decide))
    h.on_add(b"{}")
    h.on_delete(b"{}")
    assert len(c.queue) == 2
    c2 = Y.Controller()
    hs = Y.status_handlers(c2, "deployments.apps", Y.UpdateBatcher(decide=_oracle_decide))
    hs.on_add(b"{}")
    hs.on_delete(b"{}")
    assert c2.queue == []


def test_batched_update_gate_matches_reference_order():
    events = _events()
    spec_c, stat_c = Y.Controller(), Y.Controller()
    b = Y.UpdateBatcher(max_batch=7, decide=_oracle_decide)
    hs = Y.spec_handlers(spec_c, "deployments.apps", b)
    ht = Y.status_handlers(stat_c, "deployments.apps", b)
    for old, new in events:
        hs.on_update(old, new)
        ht.on_update(old, new)
    b.flush()
    want_spec, want_stat = _reference_queue(events)
    assert spec_c.queue == want_spec
    assert stat_c.queue == want_stat


@pytest.mark.gpu
@pytest.mark.parametrize("dev", [False, True], ids=["host_encode", "device_encode"])
def test_gpu_handlers_match_reference(dev):
    events = _events()
    eng = G.Engine(device=0, device_encode=dev)
    spec_c, stat_c = Y.Controller(), Y.Controller()
    b = Y.UpdateBatcher(engine=eng, max_batch=16)
    hs = Y.spec_handlers(spec_c, "deployments.apps", b)
    ht = Y.status_handlers(stat_c, "deployments.apps", b)
    for old, new in events:
        hs.on_update(old, new)
        ht.on_update(old, new)
    b.flush()
    want_spec, want_stat = _reference_queue(events)
    assert spec_c.queue == want_spec and stat_c.queue == want_stat
    # synchronous one-pair drop-ins give the same gate
    Y._default_engine = eng
    sc2 = Y.Controller()
    h2 = Y.spec_handlers(sc2, "deployments.apps")
    for old, new in events:
        h2.on_update(old, new)
    assert sc2.queue == want_spec
    eng.close()
    Y._default_engine = None
