"""The object store's path table (include/gpudiff_format.h), host encoder side
(CPU): the table a blob carries names exactly the region leaves' paths and
their ancestors -- checked against the oracle's leaf sets by walking every
entry's parent chain back to the root -- is sorted and unique with no entry
equal to the root's hash, and the agreement rule the store applies (a hash two
tables share must have the same parent hash and the same last component)
separates adversarially colliding paths at reduced hash widths, where the path
hash alone cannot.  The device side (K0 writes the same bytes, K0c applies the
rule) is in test_gpu_tokenize.py and test_gpu_store.py."""
import json
import random

import pytest
import xxhash

from kcp_amd import gpudiff as G
from oracle import gpudiff_oracle as O
from tests.golden.kat_cases import cases as kat_cases
from tests.workload import configmap, crd, deployment

SEEDS_BITS = [(0, 32), (5, 32), (0, 16), (3, 16)]


def _objects():
    rnd = random.Random(11)
    objs = [configmap(rnd, 0, 1), configmap(rnd, 1, 1, True), deployment(rnd, 2, 1), crd(rnd, 3, 1, 120)]
    objs += [{"apiVersion": "v1", "metadata": {"labels": {"a": "b"}, "annotations": {"x": 1}}, "spec": {}},
             {"metadata": {"labels": {}}, "status": 5, "spec": [1, [2, {}], {"k": None}]},
             {"kind": "K", "status": None, "top": None, "l": [[[]]]}]
    for _n, a, b, _se, _st in kat_cases():
        for x in (a, b):
            data = G.to_json_bytes(x)
            if O._nesting_bound(data) > 200:  # the depth-10000 rows: K0 and the host defer them anyway
                continue
            try:
                objs.append(O.informer_decode(data))
            except O.DecodeError:
                pass
    return objs


def _table_paths(tab, seed, mask):
    """Every entry's path, rebuilt by following parent hashes to the root."""
    by_h = {h: (ph, c) for h, ph, c in tab}
    root = seed & mask
    paths = set()
    for h in by_h:
        p, x = [], h
        for _ in range(len(by_h) + 1):
            if x == root:
                break
            ph, (kind, c) = by_h[x]
            p.append(("K", c.decode("utf-8")) if kind == "K" else ("I", c))
            x = ph
        else:
            raise AssertionError("parent chain does not reach the root")
        paths.add(tuple(reversed(p)))
    return paths


def _expected_paths(obj):
    leaves = set(O.spec_leaves(obj)) | set(O.status_leaves(obj))
    return {p[:k] for p in leaves for k in range(1, len(p) + 1)}


@pytest.mark.parametrize("seed,bits", SEEDS_BITS)
def test_table_names_region_paths_and_ancestors(seed, bits):
    mask = (1 << bits) - 1
    n_checked = 0
    for obj in _objects():
        doc = json.dumps(obj).encode()
        info, blob = G.encode_object_host(doc, seed, bits)
        if info["status"] != G.TOK_OK:
            assert info["status"] == G.TOK_HASH and bits < 64, info
            continue
        assert info["bytes"] % 16 == 0 and len(blob) == info["bytes"]
        tab = G.decode_path_table(blob, info)
        hs = [h for h, _ph, _c in tab]
        assert hs == sorted(set(hs)), "not ascending / not unique"
        assert (seed & mask) not in hs
        assert all(ph == (seed & mask) or ph in set(hs) for _h, ph, _c in tab)
        for h, _ph, _c in tab:
            assert h <= mask
        got = _table_paths(tab, seed, mask)
        assert got == _expected_paths(obj), obj
        # each entry's hash is the chained path hash of the path it names
        for p in got:
            assert O.path_hash(p, seed) & mask in set(hs)
        n_checked += 1
    assert n_checked >= 20


def _agree(ta, tb):
    """The store's rule (encoder.cpp tab_agree, dstore.hip k_collide)."""
    a = {h: (ph, c) for h, ph, c in ta}
    return all(a[h] == (ph, c) for h, ph, c in tb if h in a)


def _collide(parent_a, parent_b, bits, prefix="f"):
    """Two keys ka != kb with hash(parent_a + ka) == hash(parent_b + kb) under `bits` (seed 0)."""
    mask = (1 << bits) - 1
    pa, pb = O.path_hash(parent_a, 0), O.path_hash(parent_b, 0)
    seen_a, seen_b = {}, {}
    for i in range(1 << 20):
        k = "%s%d" % (prefix, i)
        ha = xxhash.xxh64_intdigest(O.encode_path((("K", k),)), seed=pa) & mask
        hb = xxhash.xxh64_intdigest(O.encode_path((("K", k),)), seed=pb) & mask
        if ha in seen_b and seen_b[ha] != k:
            return k, seen_b[ha]
        if hb in seen_a and seen_a[hb] != k:
            return seen_a[hb], k
        seen_a[ha], seen_b[hb] = k, k
    raise AssertionError("no collision found")


def adversarial_pairs(bits=16):
    """(old, new) objects whose region segments are equal key for key and value
    for value under `bits`-bit path hashes at seed 0, though the objects differ:
    the same parent with another key, and another parent.  Each object on its
    own encodes at seed 0."""
    base = {"apiVersion": "v1", "kind": "Widget", "metadata": {"name": "w"}}
    out = []
    ka, kb = _collide((("K", "spec"),), (("K", "spec"),), bits)
    out.append((dict(base, spec={ka: 1}), dict(base, spec={kb: 1})))
    xa, yb = _collide((("K", "a"),), (("K", "b"),), bits, prefix="g")
    out.append((dict(base, a={xa: "v"}), dict(base, b={yb: "v"})))
    return out


def test_agreement_rule_separates_colliding_paths():
    bits = 16
    for old, new in adversarial_pairs(bits):
        ia, ba = G.encode_object_host(json.dumps(old).encode(), 0, bits)
        ib, bb = G.encode_object_host(json.dumps(new).encode(), 0, bits)
        assert ia["status"] == ib["status"] == G.TOK_OK
        # the spec segments are identical: the path hash alone would call the pair equal
        sa = G.decode_segment(ba, 0, ia["spec_l"], ia["spec_ar"])
        sb = G.decode_segment(bb, 0, ib["spec_l"], ib["spec_ar"])
        assert [tuple(map(int, e[:3])) + (e[3],) for e in sa] == [tuple(map(int, e[:3])) + (e[3],) for e in sb]
        assert not O.deep_equal_apart_from_status(old, new)
        # the tables disagree (the store re-encodes the pair from old_json, or reports it dirty)
        assert not _agree(G.decode_path_table(ba, ia), G.decode_path_table(bb, ib))
        # and the oracle's pair seed moves off 0 for this pair
        assert O.diff_pair(json.dumps(old).encode(), json.dumps(new).encode(), bits)["seed"] != 0


def test_agreement_holds_for_versions_of_one_object():
    rnd = random.Random(5)
    for seed, bits in SEEDS_BITS:
        for make in (lambda i: deployment(rnd, i, 0), lambda i: crd(rnd, i, 0, 80)):
            a = make(1)
            b = json.loads(json.dumps(a))
            b["metadata"]["resourceVersion"] = "999"
            b.setdefault("spec", {})["extra"] = [1, {"z": 2}]
            ia, ba = G.encode_object_host(json.dumps(a).encode(), seed, bits)
            ib, bb = G.encode_object_host(json.dumps(b).encode(), seed, bits)
            if ia["status"] != G.TOK_OK or ib["status"] != G.TOK_OK:
                assert bits < 64
                continue
            assert _agree(G.decode_path_table(ba, ia), G.decode_path_table(bb, ib))
