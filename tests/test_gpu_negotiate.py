"""Kernels K13 (negotiation fields, negotiation mode of k_encode_docs) and K14
(per-pair classification) on the GPU -- SURVEY.md §8(f) row 4,
pkg/reconciler/apiresource/controller.go:238-295.  Every batch's actions must
equal the oracle's (oracle/negotiate_oracle.py, pinned by
tests/negotiate_cases.py); API-server-shaped populations must be classified
entirely on the device."""
import pytest

from kcp_amd import gpudiff as G
from kcp_amd import synth as S
from oracle import negotiate_oracle as N
from tests import negotiate_cases as C
from tests.test_negotiate import fuzz_pairs

pytestmark = pytest.mark.gpu


def _check(eng, pairs):
    nb = eng.nbatch(pairs)
    try:
        nb.run()
        got = nb.fetch().tolist()
        st = nb.stats()
    finally:
        nb.close()
    want = [N.classify(a, b) for a, b in pairs]
    bad = [i for i, (g, w) in enumerate(zip(got, want)) if g != w]
    assert not bad, (len(bad), bad[:5], [(got[i], want[i], pairs[i]) for i in bad[:2]])
    return st


def test_kat_batch():
    eng = G.Engine(device=0)
    pairs = [(a, b) for _, a, b, _ in C.cases()]
    _check(eng, pairs)
    eng.close()


def test_clean_population_all_on_device():
    eng = G.Engine(device=0)
    pairs, want = S.negotiate_population(20000, seed=5, variants=False)
    st = _check(eng, pairs)
    assert st.n_host == 0
    got = eng.classify_updates(pairs)
    assert got.tolist() == want.tolist()
    eng.close()


def test_population_with_variants():
    eng = G.Engine(device=0)
    pairs, want = S.negotiate_population(20000, seed=6)
    st = _check(eng, pairs)
    # the fold-case metadata keys (0.5% of the ignorable events) are the only deferrals
    assert 0 < st.n_host < 200
    eng.close()


def test_fuzz():
    eng = G.Engine(device=0)
    _check(eng, fuzz_pairs(4000, 20211004 + 72))
    eng.close()


def test_empty_and_repeated_runs():
    eng = G.Engine(device=0)
    assert eng.classify_updates([]).tolist() == []
    pairs, want = S.negotiate_population(3000, seed=8, variants=False)
    nb = eng.nbatch(pairs)
    for _ in range(3):
        nb.run()
        assert nb.fetch().tolist() == want.tolist()
    nb.close()
    eng.close()


def test_many_members_and_conditions_defer():
    eng = G.Engine(device=0)
    base = C.obj(rv="1", labels={"k%d" % i: "v" for i in range(20)}, conds=[C.cond(t="T%d" % i) for i in range(10)])
    new = C.obj(rv="2", labels={"k%d" % i: "v" for i in range(20)}, conds=[C.cond(t="T%d" % i) for i in range(10)])
    new2 = C.obj(rv="2", labels={"k%d" % i: "v" for i in range(20)}, conds=[C.cond(t="T%d" % i) for i in range(9)])
    st = _check(eng, [(base, new), (base, new2), (new, base)])
    assert st.n_host == 3
    eng.close()


def test_condition_times_vs_oracle():
    """K13's strict-shape RFC3339 parser (or its deferral) against the oracle over random time strings."""
    from tests.test_negotiate import random_times
    eng = G.Engine(device=0)
    times = random_times(3000, 4)
    pairs = []
    for i, t in enumerate(times):
        a = C.obj(rv="1", conds=[C.cond(ltt=times[i - 1])])
        b = C.obj(rv="2", conds=[C.cond(ltt=t)])
        pairs.append((a, b))
        pairs.append((b, C.obj(rv="3", conds=[C.cond(ltt=t.replace("Z", "+00:00"))])))
    st = _check(eng, pairs)
    assert st.n_host < len(pairs) // 3  # most shapes are parsed on the device, not deferred
    eng.close()


# ---------------------------------------------------------------- CustomResourceDefinition events (controller.go:186-199)
def _check_kinds(eng, pairs, kinds):
    nb = eng.nbatch(pairs, kinds)
    try:
        nb.run()
        got = nb.fetch().tolist()
        st = nb.stats()
    finally:
        nb.close()
    ks = [kinds] * len(pairs) if isinstance(kinds, int) else list(kinds)
    want = [N.classify(a, b, k) for (a, b), k in zip(pairs, ks)]
    bad = [i for i, (g, w) in enumerate(zip(got, want)) if g != w]
    assert not bad, (len(bad), bad[:5], [(got[i], want[i], pairs[i]) for i in bad[:2]])
    return st


def test_crd_kat_batch():
    eng = G.Engine(device=0)
    _check_kinds(eng, [(a, b) for _, a, b, _ in C.crd_cases()], G.NEG_KIND_CRD)
    _check_kinds(eng, [(a, b) for _, a, b, _ in C.kcp_kind_ignores_crd_status()], G.NEG_KIND_API)
    eng.close()


def test_crd_population_all_on_device():
    eng = G.Engine(device=0)
    pairs, want = S.crd_population(8000, seed=9)
    st = _check_kinds(eng, pairs, G.NEG_KIND_CRD)
    assert st.n_host == 0
    assert eng.classify_updates(pairs, G.NEG_KIND_CRD).tolist() == want.tolist()
    eng.close()


def test_crd_fuzz():
    from tests.test_negotiate import crd_fuzz_pairs
    eng = G.Engine(device=0)
    _check_kinds(eng, crd_fuzz_pairs(4000, 20211004 + 74), G.NEG_KIND_CRD)
    eng.close()


def test_mixed_kinds_batch():
    eng = G.Engine(device=0)
    api, _ = S.negotiate_population(3000, seed=10, variants=False)
    crd, _ = S.crd_population(3000, seed=10, n_props=4)
    pairs = [p for ab in zip(api, crd) for p in ab]
    kinds = [k for _ in range(3000) for k in (G.NEG_KIND_API, G.NEG_KIND_CRD)]
    st = _check_kinds(eng, pairs, kinds)
    assert st.n_host == 0
    eng.close()


def test_crd_long_lists_defer():
    """More than kNegMaxList (8) stored versions / short names: the host path decides."""
    eng = G.Engine(device=0)
    many = ["v%d" % i for i in range(10)]
    pairs = [(C.crd(rv="1", stored=many), C.crd(rv="2", stored=many + ["v10"])),
             (C.crd(rv="1", names=dict(C.NAMES, shortNames=many)), C.crd(rv="2", names=dict(C.NAMES, shortNames=many))),
             (C.crd(rv="1", stored=many[:8]), C.crd(rv="2", stored=many[:8]))]
    st = _check_kinds(eng, pairs, G.NEG_KIND_CRD)
    assert st.n_host == 2
    eng.close()


def _reorder_root(doc: bytes, rng) -> bytes:
    """The same object with its root members in another order, plus decoy "metadata" / "status"
    members nested in spec (only the root's count): the passes after N1 / R1 look inside the
    metadata and status subtrees by their pre-order ranges, which this moves around."""
    import json
    o = json.loads(doc)
    if isinstance(o.get("spec"), dict):
        o["spec"]["metadata"] = {"labels": {"kcp.dev/owned-by": "decoy"}, "resourceVersion": "9"}
        o["spec"]["status"] = {"conditions": [{"type": "Decoy", "status": "True"}], "replicas": 99}
    keys = list(o)
    rng.shuffle(keys)
    if rng.random() < 0.5 and "status" in keys:  # status first / metadata last at times
        keys.remove("status")
        keys.insert(0, "status")
    return json.dumps({k: o[k] for k in keys}, separators=(",", ":")).encode()


def test_root_member_order_and_decoys():
    import random
    rng = random.Random(77)
    eng = G.Engine(device=0)
    pairs, _ = S.negotiate_population(600, seed=78)
    moved = [(_reorder_root(a, rng), _reorder_root(b, rng)) for a, b in pairs]
    _check(eng, moved)
    eng.close()
