"""Kernel K10 (the write path's request bodies) on the
GPU: every body K10 emits is byte-identical to the host path's (itself pinned
to the oracle and the known-answer bodies by tests/test_upsert.py), and the
documents K10 leaves to the host carry one of the documented reasons."""
import json
import random

import pytest

from kcp_amd import gpudiff as G
from tests import upsert_cases as UC
from tests.test_gpu_tokenize import EDGE_DEFER, EDGE_OK

pytestmark = pytest.mark.gpu

REASONS = {G.TOK_NUMBER, G.TOK_KEY, G.TOK_STRING, G.TOK_HASH, G.TOK_DEPTH, G.TOK_FLOAT, G.TOK_WIDE, G.TOK_SPACE}


def _check(eng, docs, mode, must_device=True, allowed=()):
    res = eng.upsert_bodies(docs, mode)
    assert len(res.bodies) == len(docs)
    codes = []
    for i, d in enumerate(docs):
        want = G.upsert_body_host(d, mode)
        assert res.bodies[i] == want, (i, d[:300], res.bodies[i][:300] if res.bodies[i] else None, want[:300]
                                       if want else None)
        k = int(res.k10_status[i])
        codes.append(k)
        if res.source[i] == G.BODY_DEVICE:
            assert k == G.TOK_OK
        else:
            assert k != G.TOK_OK
            if want is not None:
                assert k in REASONS, (i, k, d[:200])
                if must_device and k not in allowed:
                    raise AssertionError("K10 deferred doc %d (status %d): %r" % (i, k, d[:300]))
    return codes


@pytest.mark.parametrize("mode", [UC.SPEC, UC.STATUS])
def test_kat_bodies(mode):
    eng = G.Engine(device=0)
    kat = [k for k in UC.KAT if k[2] == mode or mode == UC.SPEC]
    res = eng.upsert_bodies([k[1] for k in kat], mode)
    for (name, doc, m, want), got in zip(kat, res.bodies):
        if m == mode:
            assert got == want, name
    eng.close()


def test_kat_device_subset():
    """Every KAT document outside the documented exceptions is emitted by K10."""
    eng = G.Engine(device=0)
    docs = [k[1] for k in UC.KAT if k[2] == UC.SPEC]
    codes = _check(eng, docs, UC.SPEC, must_device=False)
    by_name = {k[0]: c for k, c in zip([k for k in UC.KAT if k[2] == UC.SPEC], codes)}
    assert by_name["floats"] == G.TOK_FLOAT
    assert by_name["duplicate keys last wins"] == G.TOK_HASH
    assert by_name["surrogates and invalid UTF-8"] == G.TOK_STRING
    assert by_name["ints"] == G.TOK_FLOAT  # 9223372036854775808 decodes to a float64
    assert by_name["key byte order"] == G.TOK_KEY  # a non-ASCII key
    for name in ("uid+rv removed", "kept ref normalized", "owned ref dropped, field removed", "refs not a list",
                 "refs with a non-map element", "non-string label collapses owned-by", "html-safe escaping",
                 "raw U+2028 in input", "escaped key", "whitespace", "empty object", "refs empty list",
                 "empty ref object kept", "non-bool controller omitted", "nested metadata untouched"):
        assert by_name[name] == G.TOK_OK, name
    eng.close()


@pytest.mark.parametrize("mode", [UC.SPEC, UC.STATUS])
def test_fixtures_and_synthetic(mode):
    eng = G.Engine(device=0)
    # the KAT pairs hold floats, duplicate keys, escaped keys and invalid UTF-8 on purpose, the
    # reference's manifests a few floats; the config populations none of these
    codes = _check(eng, UC.fixture_docs(), mode, allowed=(G.TOK_FLOAT, G.TOK_NUMBER, G.TOK_KEY, G.TOK_HASH,
                                                           G.TOK_STRING))
    assert sum(c == G.TOK_OK for c in codes) >= 0.85 * len(codes)  # config3/4 CRDs carry random floats
    _check(eng, UC.synthetic_docs(floats=False), mode)
    codes = _check(eng, UC.synthetic_docs(seed=12), mode, allowed=(G.TOK_FLOAT,))
    assert G.TOK_OK in codes and G.TOK_FLOAT in codes
    eng.close()


def test_edges_and_scan_boundaries():
    eng = G.Engine(device=0)
    _check(eng, UC.boundary_docs(), UC.SPEC)
    _check(eng, list(EDGE_OK), UC.SPEC, allowed=(G.TOK_FLOAT,))
    _check(eng, [d for d, _ in EDGE_DEFER], UC.SPEC, must_device=False)
    eng.close()


def test_wide_object_and_big_batch():
    eng = G.Engine(device=0)
    wide = b'{"d":{' + b",".join(b'"k%05d":%d' % (4999 - i, i) for i in range(3000)) + b'}}'
    codes = _check(eng, [wide, b'{"d":{' + b",".join(b'"k%05d":"v"' % (999 - i) for i in range(1000)) + b'}}'],
                   UC.SPEC, must_device=False)
    assert codes == [G.TOK_WIDE, G.TOK_OK]
    rnd = random.Random(9)
    docs = UC.synthetic_docs(n=400, seed=21, floats=False)
    rnd.shuffle(docs)
    _check(eng, docs, UC.SPEC)
    eng.close()


def test_staged_batch_reruns_identical():
    """gpudiff_wbatch: the resident batch re-run gives identical bodies and a timed K10."""
    eng = G.Engine(device=0, timing=True)
    docs = UC.synthetic_docs(n=80, seed=4, floats=False)
    wb = eng.wbatch(docs, UC.SPEC)
    wb.run()
    a = wb.fetch()
    for _ in range(3):
        wb.run()
    b = wb.fetch()
    st = wb.stats()
    wb.close()
    assert a.bodies == b.bodies and a.n_host == 0
    assert st.runs == 4 and st.k10_ms > 0 and st.body_bytes == sum(len(x) for x in a.bodies)
    eng.close()
