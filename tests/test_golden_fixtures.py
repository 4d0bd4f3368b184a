"""Golden fixtures (tests/golden/*.json.gz): pairs built from the reference's
own manifests and CRD schema plus samples of the bench populations, with the
expected decisions and changed paths.  CPU side: the Python oracle, the C++
restatement (CPU baseline) and the host encoder's path hashes are pinned to
them; tests/test_gpu_golden.py holds the HIP path to the same vectors."""
import numpy as np
import pytest

from kcp_amd import gpudiff as G
from oracle import cpu_ref
from oracle import gpudiff_oracle as O
from tests.golden import fixtures as F


@pytest.fixture(scope="module", params=F.NAMES)
def fixture(request):
    return request.param, F.load(request.param)


def test_oracle_reproduces_fixtures(fixture):
    name, pairs = fixture
    for pname, a, b, e in pairs:
        r = O.diff_pair(a, b)
        got = [(h, k | (0x80 if region else 0), O.render_path(p)) for (h, region, k, p) in r["paths"]]
        assert (r["spec_dirty"], r["status_dirty"], r["decode_error"], r["seed"]) == (
            e["spec_dirty"], e["status_dirty"], e["decode_error"], e["seed"]), pname
        assert got == e["paths"], pname


def test_cpp_restatement_decisions(fixture):
    name, pairs = fixture
    d = cpu_ref.DecodedPairs([(a, b) for _, a, b, _ in pairs])
    flags, _, _ = d.decide(2)
    d.close()
    exp = np.array([F.expected_flags(e) for *_, e in pairs], dtype=np.uint8)
    bad = np.nonzero(flags != exp)[0]
    assert bad.size == 0, [pairs[i][0] for i in bad[:5]]


def test_host_encoder_paths_resolve(fixture):
    """Every expected (hash, kind) resolves, through the C-ABI's host-side
    gpudiff_resolve_path, to the oracle's rendered path: the encoder's path
    bytes, seeds and hashes agree with the fixture."""
    name, pairs = fixture
    for pname, a, b, e in pairs[:60]:
        for h, k, rendered in e["paths"][:40]:
            assert G.resolve_path(a, b, h, k) == rendered, (pname, rendered)


def test_fixture_coverage():
    """The fixtures exercise the cases SURVEY.md §8(c) asks for."""
    m = {n: e for n, _, _, e in F.load("manifests")}
    assert not m["contrib/examples/deployment.yaml:metadata-churn"]["spec_dirty"]
    assert m["contrib/examples/deployment.yaml:command-trailing-space"]["spec_dirty"]
    assert m["contrib/examples/deployment.yaml:replicas-float"]["spec_dirty"]
    assert m["contrib/examples/deployment.yaml:status-removed"]["status_dirty"]
    assert any(len(e["paths"]) > 100 for e in m.values())  # CRD list shifts
    c2 = F.load("config2")
    assert all(e["status_dirty"] for *_, e in c2)  # no status key: statussyncer.go:22-26
