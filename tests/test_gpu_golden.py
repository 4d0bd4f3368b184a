"""HIP path (through the C-ABI) against the committed golden fixtures:
decisions, dirty-ID lists and the changed-path CSR (hashes, kinds, order),
bit-exact, for every fixture file, also with every pair deferred to K4."""
import numpy as np
import pytest

from kcp_amd import gpudiff as G
from oracle import gpudiff_oracle as O
from tests.golden import fixtures as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", F.NAMES)
@pytest.mark.parametrize("shrink", [0, 14])
def test_fixture_parity(name, shrink):
    pairs = F.load(name)
    e = G.Engine(device=0, encode_threads=8, flags=shrink << 21)
    res = e.diff_pairs([(a, b) for _, a, b, _ in pairs])
    exp_flags = np.array([F.expected_flags(x) for *_, x in pairs], dtype=np.uint8)
    bad = np.nonzero((res.pair_flags & 7) != exp_flags)[0]
    assert bad.size == 0, [pairs[i][0] for i in bad[:5]]
    # the write-path no-op hints (not stored in the fixtures): against the oracle
    for (pname, a, b, _), f in zip(pairs, res.pair_flags.tolist()):
        r = O.diff_pair(a, b)
        assert ((f & G.SPEC_NOOP) != 0, (f & G.STATUS_NOOP) != 0) == (r["spec_noop"], r["status_noop"]), pname
    ids = np.arange(len(pairs), dtype=np.uint32)
    assert res.spec_dirty_ids.tolist() == ids[(exp_flags & G.SPEC_DIRTY) != 0].tolist()
    assert res.status_dirty_ids.tolist() == ids[(exp_flags & G.STATUS_DIRTY) != 0].tolist()
    dirty = ids[(exp_flags & (G.SPEC_DIRTY | G.STATUS_DIRTY)) != 0]
    assert res.dirty_ids.tolist() == dirty.tolist()
    for j, i in enumerate(dirty):
        lo, hi = int(res.path_offsets[j]), int(res.path_offsets[j + 1])
        got = list(zip(res.path_hashes[lo:hi].tolist(), res.path_kinds[lo:hi].tolist()))
        want = [(h, k) for h, k, _ in pairs[i][3]["paths"]]
        assert got == want, pairs[i][0]
    e.close()
