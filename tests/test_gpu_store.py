"""Device-resident object store (gpudiff_store_*, watch replay): each event's
new object is diffed against its slot's resident version, bit-exact with the
oracle's diff_pair(previous version, new version) -- previous = the empty
object {} on a first sighting without an old object -- including chained
events on one slot inside a batch, forced path-hash collisions (8-bit
hashes: re-seeds through old_json), compactions of the two spaces, Delete
events (forget) and undecodable new objects."""
import copy
import json
import random

import numpy as np
import pytest

from kcp_amd import gpudiff as G
from tests.parity import assert_matches
from tests.workload import _noise, configmap, crd, deployment, mutate

pytestmark = pytest.mark.gpu


def _obj(rnd, i):
    k = rnd.random()
    if k < 0.3:
        return configmap(rnd, i, i % 7)
    if k < 0.45:
        return configmap(rnd, i, i % 7, True)
    if k < 0.8:
        return deployment(rnd, i, i % 7)
    return crd(rnd, i, i % 7, 60)


def _next_version(rnd, o):
    o = _noise(rnd, copy.deepcopy(o))
    if "status" not in o and o.get("kind") not in ("ConfigMap", "Secret"):
        # a status that an earlier version dropped comes back
        o["status"] = {"readyReplicas": 1, "conditions": [{"type": "Ready", "status": "True"}]}
        return o
    c = rnd.random()
    if c < 0.45:
        return o  # metadata churn only: clean
    if c < 0.9:
        return mutate(rnd, o)
    if c < 0.95 and "status" in o:
        del o["status"]
        return o
    o.setdefault("spec", {})["extra"] = [1, 2, {"x": None}]
    return o


def _stream(seed, n_slots, n_batches, per_batch):
    """[(batch events [(slot, new_json, old_json)], expected pairs [(old, new)])]."""
    rnd = random.Random(seed)
    cur = {}
    out = []
    for b in range(n_batches):
        evs, pairs = [], []
        for _ in range(per_batch):
            s = rnd.randrange(n_slots)
            old = cur.get(s)
            new = _obj(rnd, s) if old is None else _next_version(rnd, old)
            nj = json.dumps(new, separators=(",", ":")).encode()
            oj = json.dumps(old, separators=(",", ":")).encode() if old is not None else None
            evs.append((s, nj, oj))
            pairs.append((oj if oj is not None else b"{}", nj))
            cur[s] = new
        out.append((evs, pairs))
    return out


def _run(eng, st, stream, drop_old=False):
    for evs, pairs in stream:
        items = [(s, nj, None if drop_old else oj, i, s % 7) for i, (s, nj, oj) in enumerate(evs)]
        res = eng.wait(st.submit(items))
        assert_matches(res, pairs, hash_bits=eng.path_hash_bits)


@pytest.mark.parametrize("drop_old", [False, True])
def test_replay_matches_oracle(drop_old):
    """Events on 60 slots, 6 batches of 150 (many slots get several events
    per batch: they chain)."""
    e = G.Engine(device=0, encode_threads=4)
    st = e.object_store(max_slots=60, space_bytes=64 << 20, max_events=256)
    _run(e, st, _stream(1, 60, 6, 150), drop_old)
    s = st.stats()
    assert s.events == 900 and s.live_slots == 60 and s.collisions_unresolved == 0
    st.free()
    e.close()


def test_compaction_keeps_results_exact():
    """A space of 512 KiB forces compactions while batches still read blobs of
    the previous versions."""
    e = G.Engine(device=0, encode_threads=4)
    st = e.object_store(max_slots=40, space_bytes=512 << 10, max_events=128)
    _run(e, st, _stream(2, 40, 12, 60))
    s = st.stats()
    assert s.compactions >= 3, s.compactions
    assert s.used_bytes <= 512 << 10
    st.free()
    e.close()


def test_forced_collisions_reseed_through_old_json():
    e = G.Engine(device=0, encode_threads=2, path_hash_bits=8)
    st = e.object_store(max_slots=30, space_bytes=64 << 20, max_events=128)
    _run(e, st, _stream(3, 30, 5, 80))
    s = st.stats()
    assert s.reseeded > 0 and s.collisions_unresolved == 0
    st.free()
    e.close()


def test_forget_and_decode_error():
    e = G.Engine(device=0, encode_threads=1)
    st = e.object_store(max_slots=4, space_bytes=1 << 20, max_events=16)
    rnd = random.Random(4)
    a = deployment(rnd, 0, 0)
    aj = json.dumps(a).encode()
    b = mutate(rnd, _noise(rnd, copy.deepcopy(a)))
    bj = json.dumps(b).encode()
    # first sighting without old: diffed against {}
    r = e.wait(st.submit([(0, aj, None)]))
    assert_matches(r, [(b"{}", aj)])
    r = e.wait(st.submit([(0, bj, None)]))
    assert_matches(r, [(aj, bj)])
    # Delete: the slot is empty again
    st.forget(0)
    r = e.wait(st.submit([(0, aj, None)]))
    assert_matches(r, [(b"{}", aj)])
    # undecodable new object: conservative dirty + error, the slot empties
    r = e.wait(st.submit([(0, b'{"spec": ', None), (1, aj, None)]))
    assert r.pair_flags.tolist() == [G.SPEC_DIRTY | G.STATUS_DIRTY | G.DECODE_ERROR,
                                     r.pair_flags[1]]
    assert_matches(r, [(aj, b'{"spec": '), (b"{}", aj)])
    r = e.wait(st.submit([(0, bj, None)]))
    assert_matches(r, [(b"{}", bj)])
    st.free()
    e.close()


def test_two_submits_in_flight():
    e = G.Engine(device=0, encode_threads=4)
    st = e.object_store(max_slots=50, space_bytes=32 << 20, max_events=200)
    stream = _stream(5, 50, 4, 120)
    tickets = []
    for k, (evs, pairs) in enumerate(stream):
        items = [(s, nj, oj, i) for i, (s, nj, oj) in enumerate(evs)]
        tickets.append(st.submit(items))
        if k >= 1:
            assert_matches(e.wait(tickets[k - 1]), stream[k - 1][1])
    assert_matches(e.wait(tickets[-1]), stream[-1][1])
    st.free()
    e.close()
