"""Kernels K11 (roll-up fields, roll-up mode of k_encode_docs) and K12 (device
grouping by owned-by label) on the GPU -- SURVEY.md §8(f) row 4,
pkg/reconciler/deployment/deployment.go:41-91.  Every batch's groups, int32
sums, others[0] and per-document group ids must equal the oracle's
(oracle/rollup_oracle.py, pinned by tests/rollup_cases.py); API-server-shaped
populations must be decided entirely on the device; every document K11 leaves
to the host must carry a documented reason."""
import pytest

from kcp_amd import gpudiff as G
from kcp_amd import synth as S
from oracle import rollup_oracle as R
from tests import rollup_cases as C
from tests.test_gpu_tokenize import EDGE_DEFER, EDGE_OK
from tests.test_rollup import fuzz_docs

pytestmark = pytest.mark.gpu

REASONS = {G.TOK_SYNTAX, G.TOK_NUMBER, G.TOK_KEY, G.TOK_STRING, G.TOK_DEPTH, G.TOK_SIZE, G.TOK_FIELD}


def _check(eng, docs):
    res = eng.rollup_status(docs)
    want = R.rollup(docs)
    got = res.as_dict()
    assert got["doc_group"] == want["doc_group"], [
        (i, g, w, docs[i][:200]) for i, (g, w) in enumerate(zip(got["doc_group"], want["doc_group"])) if g != w][:5]
    wg = [{"first_doc": g["first_doc"], "n_members": g["n_members"], "sums": g["sums"]} for g in want["groups"]]
    assert got["groups"] == wg
    for i, k in enumerate(res.k11_status.tolist()):
        assert k == G.TOK_OK or k in REASONS, (i, k)
        if k == G.TOK_OK:  # decided on the device: Go must accept the document
            assert want["doc_group"][i] != R.GROUP_DECODE, (i, docs[i][:200])
    assert res.n_host == int((res.k11_status != 0).sum())
    assert res.host_grouped == (res.n_host > 0)
    return res


def test_kat_batch():
    eng = G.Engine(device=0)
    _check(eng, [c[1] for c in C.CASES])
    eng.close()


def test_kat_device_subset():
    """The canonical KAT documents (no folds, duplicates, escapes or type errors) are decided by K11."""
    eng = G.Engine(device=0)
    names = {"plain leaf", "root (no owned-by)", "no labels, no status", "empty status", "status null (struct: no-op)",
             "counter null (int32: no-op)", "int32 max / min", "negative zero", "metadata null", "labels null",
             "labels empty", "owned-by empty string", "label key case matters (map)", "other status fields ignored",
             "nested status not read", "whitespace"}
    docs = [c[1] for c in C.CASES if c[0] in names]
    assert len(docs) == len(names)
    res = _check(eng, docs)
    assert res.n_host == 0 and not res.host_grouped
    eng.close()


def test_edge_documents():
    eng = G.Engine(device=0)
    _check(eng, EDGE_OK + [d for d, _ in EDGE_DEFER])
    eng.close()


def test_population_all_on_device():
    eng = G.Engine(device=0)
    docs, roots = S.rollup_population(2000, 4)
    res = _check(eng, docs)
    assert res.n_host == 0 and not res.host_grouped
    assert len(res.first_doc) == 2000 and set(res.n_members.tolist()) == {4}
    assert all(res.doc_group[i] == G.ROLLUP_NONE for i in roots)
    eng.close()


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_fuzzed_population(seed):
    eng = G.Engine(device=0)
    _check(eng, fuzz_docs(2000, 20211004 + seed))
    eng.close()


def test_staged_runs_repeat():
    """gpudiff_rbatch: several K11+K12 runs over the resident documents give the same answer."""
    eng = G.Engine(device=0, timing=True)
    docs, _ = S.rollup_population(500, 3, seed=7)
    docs = docs + [c[1] for c in C.CASES]
    rb = eng.rbatch(docs)
    want = R.rollup(docs)
    for _ in range(3):
        rb.run()
        got = rb.fetch().as_dict()
        assert got["doc_group"] == want["doc_group"]
        assert [g["sums"] for g in got["groups"]] == [g["sums"] for g in want["groups"]]
    st = rb.stats()
    assert st.runs == 3 and st.k11_ms > 0 and st.k12_ms > 0
    rb.close()
    eng.close()


def test_empty_and_single():
    eng = G.Engine(device=0)
    r = eng.rollup_status([])
    assert len(r.doc_group) == 0 and len(r.first_doc) == 0
    _check(eng, [C.dep({C.O: "r"}, {"replicas": 3})])
    _check(eng, [b"{}"])
    eng.close()


def test_root_member_order_and_decoys():
    """Root members reordered (status first, metadata last at times) and decoy metadata / status
    objects nested in spec: R2/R3 look only inside the root's metadata and status subtrees."""
    import random

    from tests.test_gpu_negotiate import _reorder_root
    rng = random.Random(79)
    docs, _ = S.rollup_population(200, 4, seed=80)
    eng = G.Engine(device=0)
    res = _check(eng, [_reorder_root(d, rng) for d in docs])
    assert res.n_host < len(docs) // 10  # clean API-server JSON: decided on the device
    eng.close()


@pytest.mark.parametrize("phase", ["created", "available"])
def test_kubecon_transcript(phase):
    """K11 + K12 against the reference's own transcript (contrib/demo/kubecon.result:196-208): the two
    leaves createLeafs makes from contrib/demo/deployment.yaml roll up into the root's 0/10 10 0 while
    the pods start and 10/10 10 10 once Available -- decided on the device, equal to the oracle."""
    from tests import kubecon_demo as K
    docs, root, _leaves = K.cache(phase)
    eng = G.Engine(device=0)
    res = _check(eng, docs)
    assert res.n_host == 0
    assert res.doc_group.tolist() == [G.ROLLUP_NONE, 0, 0]
    st = K.root_status_from_sums(res.sums[0])
    assert K.kubectl_row(root["spec"]["replicas"], st) == K.TRANSCRIPT[phase][K.ROOT_NAME]
    assert int(res.first_doc[0]) == 1  # others[0]: the us-east1 leaf's conditions go to the root
    eng.close()
