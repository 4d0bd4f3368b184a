"""Kernel K10 (the write path's request bodies) on the
GPU: every body is byte-identical to the oracle's (oracle/upsert_oracle.py,
test_k10_bodies_equal_oracle) and to the product's host path (itself pinned to
the oracle and the known-answer bodies by tests/test_upsert.py), and the
documents K10 leaves to the host carry one of the documented reasons."""
import json
import random

import pytest

from kcp_amd import gpudiff as G
from oracle import upsert_oracle as U
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
    assert by_name["floats"] == G.TOK_NUMBER  # 5e-324: a subnormal, outside the device's exact float parse
    assert by_name["duplicate keys last wins"] == G.TOK_HASH
    assert by_name["surrogates and invalid UTF-8"] == G.TOK_STRING
    assert by_name["key byte order"] == G.TOK_KEY  # a non-ASCII key
    for name in ("uid+rv removed", "kept ref normalized", "owned ref dropped, field removed", "refs not a list",
                 "refs with a non-map element", "non-string label collapses owned-by", "html-safe escaping",
                 "raw U+2028 in input", "escaped key", "whitespace", "empty object", "refs empty list",
                 "empty ref object kept", "non-bool controller omitted", "nested metadata untouched", "ints"):
        assert by_name[name] == G.TOK_OK, name
    eng.close()


@pytest.mark.parametrize("mode", [UC.SPEC, UC.STATUS])
def test_fixtures_and_synthetic(mode):
    eng = G.Engine(device=0)
    # the KAT pairs hold floats, duplicate keys, escaped keys and invalid UTF-8 on purpose, the
    # reference's manifests a few floats; the config populations none of these
    # (and the KAT table its 10000-deep documents: TOK_DEPTH)
    codes = _check(eng, UC.fixture_docs(), mode,
                   allowed=(G.TOK_NUMBER, G.TOK_KEY, G.TOK_HASH, G.TOK_STRING, G.TOK_DEPTH))
    assert sum(c == G.TOK_OK for c in codes) >= 0.95 * len(codes)
    _check(eng, UC.synthetic_docs(floats=False), mode)
    _check(eng, UC.synthetic_docs(seed=12), mode, allowed=(G.TOK_NUMBER,))
    eng.close()


def test_edges_and_scan_boundaries():
    eng = G.Engine(device=0)
    _check(eng, UC.boundary_docs(), UC.SPEC)
    _check(eng, list(EDGE_OK), UC.SPEC, allowed=(G.TOK_NUMBER,))
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


def test_float_text_matches_host():
    """Go's shortest float64 text (Ryu on the device, std::to_chars on the
    host): random doubles of every magnitude, %.17g and repr literals, the
    'e' switch boundaries and negative zeros."""
    import struct
    eng = G.Engine(device=0)
    rnd = random.Random(17)
    vals = [rnd.uniform(-1, 1) * 10 ** rnd.randint(-300, 300) for _ in range(6000)]
    vals += [struct.unpack("<d", struct.pack("<Q", rnd.getrandbits(64)))[0] for _ in range(6000)]
    vals += [1e-6, 9.999999999999999e-7, 1e21, 9.999999999999999e20, 1.7976931348623157e308, 0.1, 0.5,
             2.0 ** 63, 2.0 ** 53 + 2, 123456789012345680000.0, 1e22, 1e23, 4.35e-5]
    vals += [float(k) for k in range(-70, 70)] + [2.0 ** k for k in range(-80, 80)]  # exact integers / powers of 2
    vals = [v for v in vals if v == v and abs(v) != float("inf")]
    lits = [repr(v).encode() for v in vals] + [b"%.17g" % v for v in vals[:3000]] + \
        [b"-0.0", b"-0e5", b"0.000", b"-1e-400", b"1E+2", b"-12.50"]
    docs = [b'{"f":[' + b",".join(lits[i:i + 40]) + b']}' for i in range(0, len(lits), 40)]
    codes = _check(eng, docs, UC.SPEC, must_device=False)
    # only literals the device cannot parse exactly (subnormals, undecidable halfway cases) go to the host
    assert sum(c == G.TOK_OK for c in codes) >= 0.5 * len(codes)
    assert set(codes) <= {G.TOK_OK, G.TOK_NUMBER}
    single = [b'{"f":%s}' % x for x in lits[:4000]]
    codes = _check(eng, single, UC.SPEC, must_device=False)
    assert sum(c == G.TOK_OK for c in codes) >= 0.95 * len(codes), sum(c == G.TOK_OK for c in codes)
    eng.close()


@pytest.mark.parametrize("mode", [UC.SPEC, UC.STATUS])
def test_k10_bodies_equal_oracle(mode):
    """K10 (with its host completion) against the Python oracle directly, not the
    product's host path: the known-answer documents, the reference's fixtures,
    synthetic kcp-shaped objects with and without floats, K0's edge corpus and
    the 64-byte scan boundaries; the synthetic populations must come from the
    device."""
    eng = G.Engine(device=0)
    groups = [([k[1] for k in UC.KAT], False), (UC.fixture_docs(), False), (UC.synthetic_docs(floats=False), True),
              (UC.synthetic_docs(seed=12), False), (UC.boundary_docs(), True),
              (list(EDGE_OK) + [d for d, _ in EDGE_DEFER], False)]
    for docs, all_device in groups:
        res = eng.upsert_bodies(docs, mode)
        for i, d in enumerate(docs):
            assert res.bodies[i] == U.upsert_body(d, mode), (i, d[:300])
        if all_device:
            assert res.n_host == 0 and all(int(s) == G.BODY_DEVICE for s in res.source)
    eng.close()
