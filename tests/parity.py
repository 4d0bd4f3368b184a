"""Helpers: compare a gpudiff DiffResult with the oracle on the same pairs."""
import numpy as np

from kcp_amd import gpudiff as G
from oracle import gpudiff_oracle as O


def oracle_batch(pairs, hash_bits=O.PATH_HASH_BITS):
    return [O.diff_pair(G.to_json_bytes(a), G.to_json_bytes(b), hash_bits) for a, b in pairs]


def expected_flags(r):
    f = 0
    if r["spec_dirty"]:
        f |= G.SPEC_DIRTY
    if r["status_dirty"]:
        f |= G.STATUS_DIRTY
    if r["decode_error"]:
        f |= G.DECODE_ERROR
    if r.get("spec_noop"):
        f |= G.SPEC_NOOP
    if r.get("status_noop"):
        f |= G.STATUS_NOOP
    return f


def expected_paths(r):
    return [(h, k | (G.PATH_REGION_STATUS if region else 0)) for (h, region, k, _p) in r["paths"]]


def assert_matches(res: G.DiffResult, pairs, ids=None, hash_bits=O.PATH_HASH_BITS, exp=None):
    n = len(pairs)
    ids = list(range(n)) if ids is None else list(ids)
    exp = oracle_batch(pairs, hash_bits) if exp is None else exp
    flags = np.array([expected_flags(r) for r in exp], dtype=np.uint8)
    assert res.pair_flags.shape == (n,)
    bad = np.nonzero(res.pair_flags != flags)[0]
    assert bad.size == 0, "flag mismatch at pairs %s: got %s want %s" % (
        bad[:10].tolist(), res.pair_flags[bad[:10]].tolist(), flags[bad[:10]].tolist())
    ids_a = np.array(ids, dtype=np.uint32)
    assert res.spec_dirty_ids.tolist() == ids_a[(flags & G.SPEC_DIRTY) != 0].tolist()
    assert res.status_dirty_ids.tolist() == ids_a[(flags & G.STATUS_DIRTY) != 0].tolist()
    dirty = np.nonzero(flags & (G.SPEC_DIRTY | G.STATUS_DIRTY))[0]
    assert res.dirty_ids.tolist() == ids_a[dirty].tolist()
    assert res.path_offsets.shape == (len(dirty) + 1,)
    for k, p in enumerate(dirty.tolist()):
        got = res.paths_of(k)
        want = expected_paths(exp[p])
        assert got == want, "paths differ for pair %d:\n got %s\nwant %s" % (p, got, want)
    return exp
