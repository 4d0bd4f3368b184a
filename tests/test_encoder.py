"""CPU tests of the host canonical encoder (product code) against the oracle's
independent restatement of the leaf extraction (oracle/gpudiff_oracle.py).

These run without a GPU: the encoder is host code behind the C-ABI
(gpudiff_encode_pairs on a GPUDIFF_DEVICE_NONE context)."""
import json
import random

import numpy as np
import pytest
from hypothesis import given, settings, strategies as st

from kcp_amd import gpudiff as G
from oracle import gpudiff_oracle as O
from tests.golden.kat_cases import BASE, J, cases

CASES = cases()


@pytest.fixture(scope="module")
def host_engine():
    e = G.Engine(device=G.DEVICE_NONE, encode_threads=4)
    yield e
    e.close()


def expected_segments(a_json: bytes, b_json: bytes, bits: int = O.PATH_HASH_BITS):
    """Oracle view: (seed, [(key, tag, bytes)] for spec/status of A and B, flags)."""
    if O._nesting_bound(a_json) + O._nesting_bound(b_json) > 1000:  # 10000-deep KATs: a thread with a big stack
        return O._on_big_stack(_expected_segments, a_json, b_json, bits)
    return _expected_segments(a_json, b_json, bits)


def _expected_segments(a_json: bytes, b_json: bytes, bits: int):
    try:
        a = O.informer_decode(a_json)
        b = O.informer_decode(b_json)
    except O.DecodeError:
        return None
    sa, sb, ta, tb = O.spec_leaves(a), O.spec_leaves(b), O.status_leaves(a), O.status_leaves(b)
    seed = O.pair_seed(sa, sb, ta, tb, bits)
    if seed < 0:
        return None
    mask = (1 << bits) - 1

    def seg(leaves):
        out = [(O.path_hash(p, seed) & mask, tag, vb) for p, (tag, vb) in leaves.items()]
        return sorted(out)

    fa = (O.OBJ_HAS_STATUS if False else 0)
    return dict(seed=seed, spec_a=seg(sa), spec_b=seg(sb), stat_a=seg(ta), stat_b=seg(tb),
                has_a="status" in a, has_b="status" in b)


def actual_segments(hb: G.HostBatch):
    pool = hb.pool()
    out = []
    for r in hb.rows():
        if r["flags_a"] & G.OBJ_DECODE_ERR:
            out.append(None)
            continue

        def segs(off, sl, sar, tl, tar):
            s = G.decode_segment(pool, off, sl, sar)
            t = G.decode_segment(pool, off + G.segment_bytes(sl, sar), tl, tar)
            f = lambda lst: [(k, m & 7, vb) for (k, v, m, vb) in lst]
            return f(s), f(t)

        sa, ta = segs(int(r["off_a"]), int(r["spec_l_a"]), int(r["spec_ar_a"]), int(r["stat_l_a"]), int(r["stat_ar_a"]))
        sb, tb = segs(int(r["off_b"]), int(r["spec_l_b"]), int(r["spec_ar_b"]), int(r["stat_l_b"]), int(r["stat_ar_b"]))
        out.append(dict(seed=int(r["flags_a"]) >> G.OBJ_SEED_SHIFT, spec_a=sa, spec_b=sb, stat_a=ta, stat_b=tb,
                        has_a=bool(r["flags_a"] & G.OBJ_HAS_STATUS), has_b=bool(r["flags_b"] & G.OBJ_HAS_STATUS)))
    return out


def check_pairs(engine, pairs, bits=O.PATH_HASH_BITS):
    hb = engine.encode(pairs)
    got = actual_segments(hb)
    for (a, b), g in zip(pairs, got):
        exp = expected_segments(G.to_json_bytes(a), G.to_json_bytes(b), bits)
        assert g == exp, (a, b)
    return hb


def test_kat_encoding(host_engine):
    hb = check_pairs(host_engine, [(a, b) for _, a, b, _, _ in CASES])
    inf = hb.info()
    # x11 truncated JSON, x20 trailing garbage, x21-x25 the list probe, x29 nesting depth 10001
    assert inf.n_decode_errors == 8


def test_rows_layout(host_engine):
    hb = host_engine.encode([(J(BASE), J(BASE))], ids=[77], clusters=[5])
    r = hb.rows()[0]
    assert r["pair_id"] == 77 and r["cluster_id"] == 5
    assert r["off_a"] % 128 == 0 and r["off_b"] % 128 == 0  # GPUDIFF_BLOB_ALIGN: blobs start on HBM lines
    assert r["spec_ar_a"] % 16 == 0
    # identical objects -> byte-identical segments
    pool = hb.pool()
    la = G.segment_bytes(int(r["spec_l_a"]), int(r["spec_ar_a"])) + G.segment_bytes(int(r["stat_l_a"]),
                                                                                        int(r["stat_ar_a"]))
    assert pool[r["off_a"]:r["off_a"] + la] == pool[r["off_b"]:r["off_b"] + la]
    # the body: segments zero padded to 128 B (the decision kernel streams the pad)
    body = G.blob_body(int(r["spec_l_a"]), int(r["spec_ar_a"]), int(r["stat_l_a"]), int(r["stat_ar_a"]))
    assert body % 128 == 0 and body - la < 128 and pool[r["off_a"] + la:r["off_a"] + body] == bytes(body - la)


def test_bodies_line_aligned_and_zero_padded(host_engine):
    """Every blob of a mixed batch starts on a 128-B line and its body's pad is zero (K2 compares the pad
    of both sides whenever their sizes match, so a nonzero pad would be a false 'dirty')."""
    pairs = [(a, b) for _, a, b, _, _ in CASES]
    hb = host_engine.encode(pairs)
    pool = hb.pool()
    for r in hb.rows():
        if r["flags_a"] & G.OBJ_DECODE_ERR:
            continue
        for s in ("a", "b"):
            off = int(r["off_" + s])
            la = G.segment_bytes(int(r["spec_l_" + s]), int(r["spec_ar_" + s])) + \
                G.segment_bytes(int(r["stat_l_" + s]), int(r["stat_ar_" + s]))
            body = G.blob_body(int(r["spec_l_" + s]), int(r["spec_ar_" + s]), int(r["stat_l_" + s]),
                               int(r["stat_ar_" + s]))
            assert off % 128 == 0 and off + body <= len(pool)
            assert pool[off + la:off + body] == bytes(body - la)


def test_long_values_head_in_record_tail_in_arena():
    """A long string (> 8 bytes) keeps its first 8 bytes in the leaf's value slot and the rest in the
    arena at a 4-byte aligned offset, zero padded (include/gpudiff_format.h): decode_segment reads every
    value of the KAT base object back whole, and the arena holds exactly the tails."""
    e = G.Engine(device=G.DEVICE_NONE)
    hb = e.encode([(J(BASE), J(BASE))])
    pool = hb.pool()
    r = hb.rows()[0]
    off, sl, sar = int(r["off_a"]), int(r["spec_l_a"]), int(r["spec_ar_a"])
    seg = G.decode_segment(pool, off, sl, sar)
    longs = [(v, m, vb) for (k, v, m, vb) in seg if (m & 7) == 5 and (m >> 3) > 8]
    assert len(longs) > 5
    arena = pool[off + 16 * sl:off + 16 * sl + sar]
    pos = 0
    for v, m, vb in longs:
        assert len(vb) == m >> 3 and int(v).to_bytes(8, "little") == vb[:8]
        tail = vb[8:]
        assert arena[pos:pos + len(tail)] == tail
        pad = (len(tail) + 3) & ~3
        assert arena[pos + len(tail):pos + pad] == bytes(pad - len(tail))
        pos += pad
    assert sar == (pos + 15) & ~15 and arena[pos:] == bytes(sar - pos)
    strings = set()

    def walk(x):
        if isinstance(x, str):
            strings.add(x.encode())
        elif isinstance(x, dict):
            for y in x.values():
                walk(y)
        elif isinstance(x, list):
            for y in x:
                walk(y)
    walk(json.loads(J(BASE)))
    assert all(vb in strings for (v, m, vb) in longs)
    e.close()


def test_multithreaded_matches_single(host_engine):
    rnd = random.Random(7)
    pairs = []
    for i in range(600):
        o = json.loads(J(BASE))
        o["spec"]["replicas"] = rnd.randint(0, 5)
        o["metadata"]["labels"]["k%d" % (i % 7)] = "v" * rnd.randint(0, 20)
        pairs.append((J(BASE), J(o)))
    e1 = G.Engine(device=G.DEVICE_NONE, encode_threads=1)
    h1 = e1.encode(pairs)
    h4 = host_engine.encode(pairs)
    assert h1.pool() == h4.pool()
    assert (h1.rows() == h4.rows()).all()
    e1.close()


def test_collision_reseed_small_hash():
    e = G.Engine(device=G.DEVICE_NONE, path_hash_bits=8)
    pairs = [(a, b) for _, a, b, _, _ in CASES[:12]]
    hb = check_pairs(e, pairs, bits=8)
    assert hb.info().n_reseeded > 0
    e.close()


_scalar = st.one_of(st.none(), st.booleans(), st.integers(-(1 << 63), (1 << 63) - 1),
                    st.floats(allow_nan=False, allow_infinity=False),
                    st.text(max_size=20))
_tree = st.recursive(_scalar, lambda ch: st.one_of(st.lists(ch, max_size=4),
                                                   st.dictionaries(st.text(max_size=6), ch, max_size=4)),
                     max_leaves=20)
_obj = st.fixed_dictionaries({}, optional={
    "spec": _tree, "status": _tree, "data": _tree, "kind": _scalar,
    "metadata": st.fixed_dictionaries({}, optional={
        "labels": st.one_of(st.none(), st.dictionaries(st.text(max_size=5), st.one_of(st.text(max_size=12),
                                                                                       st.integers(0, 1)),
                                                       max_size=3)),
        "annotations": st.dictionaries(st.text(max_size=5), st.text(max_size=30), max_size=3)})})


@settings(max_examples=150, deadline=None)
@given(st.lists(st.tuples(_obj, _obj), min_size=1, max_size=6))
def test_random_encoding(pairs):
    e = G.Engine(device=G.DEVICE_NONE, encode_threads=1)
    check_pairs(e, [(json.dumps(a).encode(), json.dumps(b).encode()) for a, b in pairs])
    e.close()


def test_resolve_path():
    a = J(BASE)
    o = json.loads(a)
    o["spec"]["template"]["spec"]["containers"][0]["image"] = "busybox:1.26"
    r = O.diff_pair(a, J(o))
    (h, region, kind, p), = r["paths"]
    assert G.resolve_path(a, J(o), h, kind | (0x80 if region else 0)) == "spec.template.spec.containers[0].image"
