"""Write path on the CPU: the oracle and the product's
host path (gpudiff_upsert_body_host, which completes K10's deferrals) against
the known-answer bodies, and against each other on a corpus of reference
fixtures, synthetic kcp-shaped objects and edge cases, in both modes."""
import random
import struct

import pytest

from kcp_amd import gpudiff as G
from oracle import upsert_oracle as U
from tests import upsert_cases as UC
from tests.test_gpu_tokenize import EDGE_DEFER, EDGE_OK


@pytest.mark.parametrize("name,doc,mode,want", UC.KAT, ids=[k[0] for k in UC.KAT])
def test_kat_oracle_and_host(name, doc, mode, want):
    assert U.upsert_body(doc, mode) == want
    assert G.upsert_body_host(doc, mode) == want


def _corpus():
    return (UC.fixture_docs() + UC.synthetic_docs() + list(EDGE_OK) + [d for d, _ in EDGE_DEFER] +
            UC.boundary_docs())


@pytest.mark.parametrize("mode", [UC.SPEC, UC.STATUS])
def test_host_matches_oracle_on_corpus(mode):
    docs = _corpus()
    assert len(docs) > 700
    for d in docs:
        assert G.upsert_body_host(d, mode) == U.upsert_body(d, mode), d[:200]


def test_float_formatting_matches_oracle():
    """strconv.AppendFloat(-1) restated twice (numpy Dragon4 in the oracle,
    std::to_chars on the host) agree on random doubles of every magnitude."""
    rnd = random.Random(5)
    vals = [rnd.uniform(-1, 1) * 10 ** rnd.randint(-30, 30) for _ in range(3000)]
    vals += [struct.unpack("<d", struct.pack("<Q", rnd.getrandbits(64)))[0] for _ in range(3000)]
    vals += [1e-6, 9.999999999999999e-7, 1e21, 9.999999999999999e20, 5e-324, 1.7976931348623157e308, 0.5, 2.0 ** 60]
    vals = [v for v in vals if v == v and abs(v) != float("inf")]
    for v in vals:
        doc = b'{"f":%s}' % repr(v).encode()
        assert G.upsert_body_host(doc) == U.upsert_body(doc), repr(v)


def test_transform_does_not_touch_other_fields():
    """Property: the body decodes to the input object minus exactly the
    transformed metadata fields (oracle.transform on the decoded object)."""
    from oracle.gpudiff_oracle import go_json_decode
    for d in UC.synthetic_docs(n=40, seed=3):
        body = G.upsert_body_host(d)
        got = go_json_decode(body)
        want = U.transform(go_json_decode(d))
        assert got == want
        md = got.get("metadata", {})
        assert "uid" not in md and "resourceVersion" not in md


@pytest.mark.parametrize("mode", [UC.SPEC, UC.STATUS])
def test_cpp_restatement_matches_oracle(mode):
    """The C++ restatement (CPU baseline of the write-path bench) agrees with
    the Python oracle body for body."""
    from oracle import cpu_ref
    docs = [k[1] for k in UC.KAT] + _corpus()
    dd = cpu_ref.DecodedDocs(docs)
    for i, d in enumerate(docs):
        assert dd.body(i, mode) == U.upsert_body(d, mode), d[:200]
    dd.close()
