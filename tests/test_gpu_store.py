"""Device-resident object store (gpudiff_store_*, watch replay): each event's
new object is diffed against its slot's resident version, bit-exact with the
oracle's diff_pair(previous version, new version) -- previous = the empty
object {} on a first sighting without an old object -- including chained
events on one slot inside a batch, forced path-hash collisions (8-bit
hashes: re-seeds through old_json), compactions of the two spaces, Delete
events (forget) and undecodable new objects.  Every test runs in both modes:
host encoding, and device encoding (raw JSON up, kernel K0 encodes, the host
re-does only the events K0 defers) -- and device encoding with the events' JSON
written into one engine-pinned buffer in the zero-copy layout (no staging
copy)."""
import copy
import json
import random

import numpy as np
import pytest

from kcp_amd import gpudiff as G
from tests.parity import assert_matches
from tests.workload import _noise, configmap, crd, deployment, mutate

pytestmark = pytest.mark.gpu

MODES = pytest.mark.parametrize("dev", [False, True, "zc"], ids=["host_encode", "device_encode", "device_zero_copy"])


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


def _run(eng, st, stream, drop_old=False, zc=False):
    z0 = st.stats().zero_copy_batches
    for evs, pairs in stream:
        items = [(s, nj, None if drop_old else oj, i, s % 7) for i, (s, nj, oj) in enumerate(evs)]
        res = eng.wait(st.submit(items, zero_copy=zc))
        assert_matches(res, pairs, hash_bits=eng.path_hash_bits)
    # zero copy: every batch uploaded straight from its pinned buffer
    assert st.stats().zero_copy_batches - z0 == (len(stream) if zc else 0)


@MODES
@pytest.mark.parametrize("drop_old", [False, True])
def test_replay_matches_oracle(drop_old, dev):
    """Events on 60 slots, 6 batches of 150 (many slots get several events
    per batch: they chain)."""
    e = G.Engine(device=0, encode_threads=4)
    st = e.object_store(max_slots=60, space_bytes=64 << 20, max_events=256, device_encode=bool(dev))
    _run(e, st, _stream(1, 60, 6, 150), drop_old, zc=dev == "zc")
    s = st.stats()
    assert s.events == 900 and s.live_slots == 60 and s.collisions_unresolved == 0
    assert s.deferred == 0 or drop_old  # regular objects: K0 encodes and K0c confirms every event
    st.free()
    e.close()


@MODES
def test_compaction_keeps_results_exact(dev):
    """A space of 512 KiB forces compactions while batches still read blobs of
    the previous versions."""
    e = G.Engine(device=0, encode_threads=4)
    st = e.object_store(max_slots=40, space_bytes=512 << 10, max_events=128, device_encode=bool(dev))
    _run(e, st, _stream(2, 40, 12, 60), zc=dev == "zc")
    s = st.stats()
    assert s.compactions >= 3, s.compactions
    assert s.used_bytes <= 512 << 10
    st.free()
    e.close()


@MODES
def test_compaction_keeps_path_tables(dev):
    """Blobs moved by compactions keep their path tables whole: with room for
    every batch, K0c confirms every event after the moves (no false collision
    defers one to the host)."""
    e = G.Engine(device=0, encode_threads=4)
    st = e.object_store(max_slots=40, space_bytes=2 << 20, max_events=128, device_encode=bool(dev))
    _run(e, st, _stream(6, 40, 40, 60), zc=dev == "zc")
    s = st.stats()
    assert s.compactions >= 2, s.compactions
    assert s.deferred == 0 and s.reseeded == 0
    st.free()
    e.close()


@MODES
def test_forced_collisions_reseed_through_old_json(dev):
    e = G.Engine(device=0, encode_threads=2, path_hash_bits=8)
    st = e.object_store(max_slots=30, space_bytes=64 << 20, max_events=128, device_encode=bool(dev))
    _run(e, st, _stream(3, 30, 5, 80), zc=dev == "zc")
    s = st.stats()
    assert s.reseeded > 0 and s.collisions_unresolved == 0
    st.free()
    e.close()


@MODES
def test_path_tables_exact_at_16_bits(dev):
    """16-bit path hashes: paths of an object's old and new versions share hashes
    by chance in a good fraction of the events; the path tables (K0c on the
    device, tab_agree on the host) catch every such collision exactly and the
    pair is re-encoded from old_json, so every result equals the oracle's."""
    e = G.Engine(device=0, encode_threads=4, path_hash_bits=16)
    st = e.object_store(max_slots=40, space_bytes=64 << 20, max_events=256, device_encode=bool(dev))
    _run(e, st, _stream(9, 40, 6, 120), zc=dev == "zc")
    s = st.stats()
    assert s.reseeded > 0 and s.collisions_unresolved == 0
    st.free()
    e.close()


@MODES
def test_adversarial_collisions_never_equal(dev):
    """Objects built so that the old and new versions' segments are identical
    key for key and value for value under 16-bit path hashes although the paths
    differ (same parent, other key; other parent): with old_json the result is
    the oracle's, without it the event is reported dirty (conservative), never
    equal."""
    from tests.test_path_table import adversarial_pairs
    pairs = adversarial_pairs(16)
    e = G.Engine(device=0, encode_threads=2, path_hash_bits=16)
    st = e.object_store(max_slots=8, space_bytes=8 << 20, max_events=16, device_encode=bool(dev))
    olds = [json.dumps(a, separators=(",", ":")).encode() for a, _b in pairs]
    news = [json.dumps(b, separators=(",", ":")).encode() for _a, b in pairs]
    k = len(pairs)
    # first sightings (slots 0..k-1 and k..2k-1 hold the old versions), diffed against {}
    zc = dev == "zc"
    r = e.wait(st.submit([(i, olds[i % k], None, i) for i in range(2 * k)], zero_copy=zc))
    assert_matches(r, [(b"{}", olds[i % k]) for i in range(2 * k)], hash_bits=16)
    # the new versions with old_json (slots 0..k-1): the oracle's results
    r = e.wait(st.submit([(i, news[i], olds[i], i) for i in range(k)], zero_copy=zc))
    exp = assert_matches(r, [(olds[i], news[i]) for i in range(k)], hash_bits=16)
    assert all(x["spec_dirty"] and x["seed"] != 0 for x in exp)
    # without old_json (slots k..2k-1): conservative, never equal
    r = e.wait(st.submit([(k + i, news[i], None, i) for i in range(k)], zero_copy=zc))
    assert r.pair_flags.tolist() == [G.SPEC_DIRTY | G.STATUS_DIRTY | G.DECODE_ERROR] * k
    s = st.stats()
    assert s.collisions_unresolved == k
    st.free()
    e.close()


@MODES
def test_forget_and_decode_error(dev):
    e = G.Engine(device=0, encode_threads=1)
    st = e.object_store(max_slots=4, space_bytes=1 << 20, max_events=16, device_encode=bool(dev))
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


@MODES
def test_two_submits_in_flight(dev):
    e = G.Engine(device=0, encode_threads=4)
    st = e.object_store(max_slots=50, space_bytes=32 << 20, max_events=200, device_encode=bool(dev))
    stream = _stream(5, 50, 4, 120)
    tickets = []
    for k, (evs, pairs) in enumerate(stream):
        items = [(s, nj, oj, i) for i, (s, nj, oj) in enumerate(evs)]
        tickets.append(st.submit(items, zero_copy=dev == "zc"))
        if k >= 1:
            assert_matches(e.wait(tickets[k - 1]), stream[k - 1][1])
    assert_matches(e.wait(tickets[-1]), stream[-1][1])
    assert st.stats().zero_copy_batches == (len(stream) if dev == "zc" else 0)
    st.free()
    e.close()


_IRREGULAR = [
    b',"zz":1,"zz":2}',                      # duplicate key (last wins): K0 defers (HASH)
    b',"k\\u0065y":"v"}',                   # escaped key: K0 defers (KEY)
    b',"bad":"\xff\xfe x"}',                 # invalid UTF-8 (U+FFFD repair): K0 defers (STRING)
    b',"big":123456789012345678901234567}',  # > 19 significant digits: K0 defers (NUMBER)
    b',"f":0.30886104750414978,"g":-1.5e-7}',  # floats K0 converts itself (Eisel-Lemire)
    b',"spec":',                             # Go decode error (truncated)
]


def _raw_stream(seed, n_slots, n_batches, per_batch):
    """Like _stream, but ~1 in 6 new versions gets an irregular tail spliced
    into its JSON bytes; the next event's old object is those exact bytes."""
    rnd = random.Random(seed)
    cur, cur_b = {}, {}
    out = []
    for _b in range(n_batches):
        evs, pairs = [], []
        for _ in range(per_batch):
            s = rnd.randrange(n_slots)
            old = cur.get(s)
            new = _obj(rnd, s) if old is None else _next_version(rnd, old)
            nj = json.dumps(new, separators=(",", ":")).encode()
            if rnd.random() < 0.17:
                nj = nj[:-1] + rnd.choice(_IRREGULAR)
            oj = cur_b.get(s)
            # without old objects, a slot emptied by an undecodable version diffs against {}
            prev_bad = oj is not None and oj.endswith(b',"spec":')
            evs.append((s, nj, oj))
            pairs.append((oj if oj is not None else b"{}", nj, b"{}" if (oj is None or prev_bad) else oj))
            cur[s] = new
            cur_b[s] = nj
        out.append((evs, pairs))
    return out


@pytest.mark.parametrize("drop_old", [False, True])
def test_device_encode_deferrals_exact(drop_old):
    """Host encoding and device encoding on the same stream with irregular
    objects spliced in: both bit-exact with the oracle, and the device mode
    really deferred events to the host."""
    stream = _raw_stream(11, 40, 6, 120)
    for dev in (False, True):
        e = G.Engine(device=0, encode_threads=4)
        st = e.object_store(max_slots=40, space_bytes=32 << 20, max_events=256, device_encode=bool(dev))
        for evs, pairs in stream:
            items = [(s, nj, None if drop_old else oj, i, s % 5) for i, (s, nj, oj) in enumerate(evs)]
            res = e.wait(st.submit(items))
            pairs = [(p[2] if drop_old else p[0], p[1]) for p in pairs]
            assert_matches(res, pairs)
        s = st.stats()
        if dev:
            assert s.deferred > 0
        st.free()
        e.close()


def test_device_store_space_pressure_stays_usable():
    """under space pressure K0 defers documents that do not fit (SPACE) and the
    host's re-encoded blobs may not fit either; those events must come back dirty (DECODE_ERROR, never
    "equal", slot emptied) and the store must stay usable -- every other event exact, later batches
    exact."""
    e = G.Engine(device=0, encode_threads=4)
    st = e.object_store(max_slots=64, space_bytes=192 << 10, max_events=64, device_encode=True)
    rnd = random.Random(17)
    objs = [crd(rnd, i, i % 3, 60) for i in range(60)]
    docs = [json.dumps(o, separators=(",", ":")).encode() for o in objs]
    assert 100 << 10 < sum(len(d) for d in docs) < 192 << 10  # the JSON fits, its blobs + tables do not
    res = e.wait(st.submit([(i, d, None) for i, d in enumerate(docs)]))
    pairs = [(b"{}", d) for d in docs]
    from tests.parity import oracle_batch, expected_flags, expected_paths
    exp = oracle_batch(pairs)
    cons = 0
    dirty = 0
    for i, r in enumerate(exp):
        f = int(res.pair_flags[i])
        if f == G.SPEC_DIRTY | G.STATUS_DIRTY | G.DECODE_ERROR:
            cons += 1
            assert res.paths_of(dirty) == []
        else:
            assert f == expected_flags(r), i
            assert res.paths_of(dirty) == expected_paths(r), i
        if f & (G.SPEC_DIRTY | G.STATUS_DIRTY):
            dirty += 1
    s = st.stats()
    assert cons > 0 and s.space_conservative == cons
    # the store goes on: forget most slots, then small batches are exact again
    for i in range(8, 64):
        st.forget(i)
    rnd2 = random.Random(18)
    for b in range(3):
        items, pairs = [], []
        for i in range(8):
            o = _next_version(rnd2, objs[i])
            nj = json.dumps(o, separators=(",", ":")).encode()
            items.append((i, nj, docs[i]))
            pairs.append((docs[i] if b == 0 else prev[i], nj))
        prev = {i: it[1] for i, it in enumerate(items)}
        r = e.wait(st.submit(items))
        # a slot emptied by the conservative path stages the event's old object again: same as the oracle's
        assert_matches(r, pairs)
        for i in range(8):
            objs[i] = json.loads(prev[i])
        docs = [prev[i] for i in range(8)]
    st.free()
    e.close()


def test_zero_copy_store_layout_rules():
    """Store-mode zero copy takes a batch only in the documented layout: the documents the store encodes in
    submit order inside one engine-pinned buffer, 16-B aligned, each followed by its staged span.  Old objects the
    store does not encode may lie anywhere (here: outside the buffer); any other layout (documents out of order)
    takes the staging copy.  Results equal the oracle's either way."""
    e = G.Engine(device=0, encode_threads=2)
    st = e.object_store(max_slots=64, space_bytes=32 << 20, max_events=64, device_encode=True)
    stream = _stream(21, 32, 3, 40)
    # batch 0: every event staged zero-copy (old objects in the buffer too, first sightings among them)
    evs, pairs = stream[0]
    assert_matches(e.wait(st.submit([(s, nj, oj, i) for i, (s, nj, oj) in enumerate(evs)], zero_copy=True)), pairs)
    assert st.stats().zero_copy_batches == 1
    # batch 1: only the new objects in the buffer, the old objects as ordinary host memory -- still zero copy (a
    # slot seen before reads its old object only on a collision; a first sighting here has none)
    evs, pairs = stream[1]
    news = G.PinnedDocs.of_bytes(e, [nj for _, nj, _ in evs])
    items = [(s, int(news.ptrs[i]), int(news.lens[i]), C_buf(oj)) for i, (s, nj, oj) in enumerate(evs)]
    arr, n = _events_raw(items)
    assert_matches(e.wait(st.submit_raw(arr, n, (news, items))), pairs)
    assert st.stats().zero_copy_batches == 2
    # batch 2: the same documents written in reverse order -- not the layout: staged, same results
    evs, pairs = stream[2]
    rev = G.PinnedDocs.of_bytes(e, [nj for _, nj, _ in reversed(evs)])
    items = [(s, int(rev.ptrs[len(evs) - 1 - i]), int(rev.lens[len(evs) - 1 - i]), C_buf(oj) if oj else None)
             for i, (s, nj, oj) in enumerate(evs)]
    arr, n = _events_raw(items)
    assert_matches(e.wait(st.submit_raw(arr, n, (rev, items))), pairs)
    assert st.stats().zero_copy_batches == 2
    st.free()
    news.free()
    rev.free()
    e.close()


def C_buf(b):
    import ctypes
    return ctypes.create_string_buffer(b, len(b)) if b is not None else None


def _events_raw(items):
    """[(slot, new_ptr, new_len, old ctypes buffer or None)] -> (Event array, n)."""
    import ctypes
    arr = (G.Event * len(items))()
    for i, (s, p, ln, old) in enumerate(items):
        arr[i].slot, arr[i].pair_id, arr[i].new_json, arr[i].new_len = s, i, p, ln
        if old is not None:
            arr[i].old_json, arr[i].old_len = ctypes.cast(old, ctypes.c_void_p), len(old)
    return arr, len(items)
