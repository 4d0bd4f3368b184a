"""CPU tests of the Deployment splitter roll-up (SURVEY.md §8(f) row 4,
pkg/reconciler/deployment/deployment.go:41-91): the oracle against the
hand-written known answers, the C++ host path (the product's path for the
documents K11 defers) against the oracle on the known answers and on seeded
fuzzed populations, and the batch grouping rules."""
import random

import numpy as np
import pytest

from kcp_amd import gpudiff as G
from kcp_amd import synth as S
from oracle import rollup_oracle as R
from tests import rollup_cases as C


def _oracle(d):
    try:
        e = R.extract(d)
    except R.DecodeError:
        return C.DECODE
    return (e["status"], e["owned_by"])


def _host(d):
    h = G.rollup_doc_host(d)
    if h is None:
        return C.DECODE
    return (h[0], None if h[1] is None else h[1].decode("utf-8"))


@pytest.mark.parametrize("name,doc,exp", C.CASES, ids=[c[0] for c in C.CASES])
def test_oracle_kat(name, doc, exp):
    assert _oracle(doc) == exp


@pytest.mark.parametrize("name,doc,exp", C.CASES, ids=[c[0] for c in C.CASES])
def test_host_path_kat(name, doc, exp):
    assert _host(doc) == exp


def fuzz_docs(n, seed):
    """Deployments with seeded edits aimed at the typed-decode rules."""
    docs, _ = S.rollup_population(max(1, n // 5), 4, seed=seed)
    rng = random.Random(seed)
    edits = [
        (b'"replicas":', b'"Replicas":'), (b'"status":{', b'"Status":{'), (b'"labels":{', b'"LABELS":{'),
        (b'"readyReplicas":', b'"readyReplicas":null,"readyReplicas":'), (b'"status":{', b'"status":null,"status":{'),
        (b'"replicas":', b'"replicas":1.0,"x":'), (b'"updatedReplicas":', b'"updatedReplicas":"7","y":'),
        (b'"kcp.dev/owned-by":"', b'"kcp.dev/owned-by":"\\u00e9'), (b'"labels":{', b'"labels":{"n":5,'),
        (b'"metadata":{', b'"metadata":{"labels":{"kcp.dev/owned-by":"zz"},'), (b'"unavailableReplicas":',
                                                                            b'"unavailableReplicas":2147483648,"u":'),
        (b'"availableReplicas":', b'"availableReplicas":-2147483648,"a":'), (b'}}', b'}} '), (b'"kind"', b'"kind":1,"k"'),
        (b'"spec":{', b'"spec":{"q":tru,'), (b'"labels":{', b'"labels":null,"labels":{'),
        (b'"status":{', b'"statu\xc5\xbf":{"replicas":3},"status":{'),
    ]
    out = []
    for d in docs:
        if rng.random() < 0.5:
            a, b = rng.choice(edits)
            d = d.replace(a, b, 1)
        out.append(d)
    return out


def test_host_path_matches_oracle_fuzz():
    docs = fuzz_docs(3000, 20211004 + 61)
    bad = [i for i, d in enumerate(docs) if _host(d) != _oracle(d)]
    assert not bad, (len(bad), docs[bad[0]][:300], _host(docs[bad[0]]), _oracle(docs[bad[0]]))


def test_rollup_grouping_rules():
    docs = [C.dep({C.O: "a"}, {"replicas": 2147483647}), C.dep({C.O: "b"}, {"replicas": 1}),
            C.dep({"app": "x"}, {"replicas": 9}), b'{"status":[]}', C.dep({C.O: "a"}, {"replicas": 1,
                                                                                    "readyReplicas": 3}),
            C.dep({C.O: ""}, {}), C.dep({C.O: "b"}, {"unavailableReplicas": -5})]
    r = R.rollup(docs)
    assert r["doc_group"] == [0, 1, R.GROUP_NONE, R.GROUP_DECODE, 0, 2, 1]
    g = r["groups"]
    assert [x["first_doc"] for x in g] == [0, 1, 5]
    assert g[0]["sums"] == [-2147483648, 0, 3, 0, 0] and g[0]["n_members"] == 2  # Go int32 wrap-around
    assert g[1]["sums"] == [1, 0, 0, 0, -5]
    assert g[2]["owned_by"] == "" and g[2]["n_members"] == 1


def test_population_shape():
    docs, roots = S.rollup_population(50, 4)
    r = R.rollup(docs)
    assert len(r["groups"]) == 50 and all(x["n_members"] == 4 for x in r["groups"])
    assert all(r["doc_group"][i] == R.GROUP_NONE for i in roots)
    assert sorted(x["first_doc"] for x in r["groups"]) == [x["first_doc"] for x in r["groups"]]
    assert np.all(np.array([len(d) for d in docs]) > 1000)


def _strip(r):
    return {"doc_group": r["doc_group"], "groups": [{"first_doc": g["first_doc"], "n_members": g["n_members"],
                                                     "sums": g["sums"]} for g in r["groups"]]}


def test_cpp_restatement_matches_oracle():
    """oracle/rollup_ref.cpp (the CPU baseline) == oracle/rollup_oracle.py on the KATs and fuzzed populations."""
    from oracle import cpu_ref
    for docs in ([c[1] for c in C.CASES], fuzz_docs(3000, 20211004 + 62)):
        rd = cpu_ref.RollupDocs(docs)
        _, _, got = rd.run(threads=4)
        rd.close()
        assert got == _strip(R.rollup(docs))


# ---------------------------------------------------------------- the reference's own transcript
@pytest.mark.parametrize("phase", ["created", "available"])
def test_kubecon_transcript_oracle_and_host_path(phase):
    """contrib/demo/kubecon.result:196-208 (the one reference-held outcome of the roll-up): the root's
    READY / UP-TO-DATE / AVAILABLE from the sums of createLeafs' two leaves equal the transcript's row,
    by the oracle and by the product's host path (summed per owned-by label)."""
    from tests import kubecon_demo as K
    docs, root, leaves = K.cache(phase)
    want = K.TRANSCRIPT[phase]
    for lf in leaves:  # the leaves' own rows
        assert K.kubectl_row(lf["spec"]["replicas"], lf["status"]) == want[lf["metadata"]["name"]]
    res = R.rollup(docs)
    assert res["doc_group"] == [R.GROUP_NONE, 0, 0]  # the root is no leaf; both leaves roll up into one group
    (g,) = res["groups"]
    assert g["first_doc"] == 1 and g["n_members"] == 2
    st = K.root_status_from_sums(g["sums"])
    assert K.kubectl_row(root["spec"]["replicas"], st) == want[K.ROOT_NAME]
    sums = [0] * 5
    for d in docs:
        h = G.rollup_doc_host(d)
        assert h is not None
        if h[1] == K.ROOT_NAME.encode():
            sums = [a + b for a, b in zip(sums, h[0])]
    assert sums == g["sums"]
