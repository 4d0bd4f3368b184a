"""the Go drop-in's transfer, emulated end to end on the GPU.

Every known-answer and golden pair is decoded as the informer would
(oracle.informer_decode), re-emitted with the Go binding's marker rules
(tests/goshim.py restating integration/go/gpudiff/gpudiff.go:jsonOf), and
submitted through the C-ABI (gpudiff_submit / gpudiff_wait), with host and with
device (K0) encoding.  The flags, ID lists and changed-path lists must equal
the oracle's on the ORIGINAL JSON pair; pairs the shim cannot transfer are the
ones the batcher reports dirty itself, and they must be dirty in the oracle too."""
import numpy as np
import pytest

from kcp_amd import gpudiff as G
from oracle import gpudiff_oracle as O
from tests import goshim as S
from tests.parity import assert_matches
from tests.test_goshim import PAIRS

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("device_encode", [False, True])
def test_shim_transfer_matches_oracle_on_original_pairs(device_encode):
    orig, shim, bad = [], [], []
    for name, a, b in PAIRS:
        sp = S.shim_pair(a, b)
        if sp is None:
            bad.append((name, a, b))
        else:
            orig.append((a, b))
            shim.append(sp)
    eng = G.Engine(device=0, encode_threads=8, device_encode=device_encode)
    exp = [O.diff_pair(a, b) for a, b in orig]
    res = eng.diff_pairs(shim)
    assert_matches(res, shim, exp=exp)
    # the KAT rows whose answer the old MarshalJSON transfer flipped are dirty here
    kat7 = [i for i, (name, *_r) in enumerate([p for p in PAIRS if S.shim_pair(p[1], p[2]) is not None])
            if name.startswith("07")]
    assert all(res.pair_flags[i] & G.SPEC_DIRTY for i in kat7)
    for name, a, b in bad:
        r = O.diff_pair(a, b)
        assert r["spec_dirty"] and r["status_dirty"], name
    eng.close()


def test_shim_one_pair_drop_ins():
    """gpudiff_spec_equal / gpudiff_status_equal through the shim (DeepEqualApartFromStatus /
    DeepEqualStatus of the Go binding)."""
    eng = G.Engine(device=0)
    for name, a, b in PAIRS[:120]:
        sp = S.shim_pair(a, b)
        r = O.diff_pair(a, b)
        if sp is None:
            continue
        assert eng.spec_equal(*sp) == (not r["spec_dirty"]), name
        assert eng.status_equal(*sp) == (not r["status_dirty"]), name
    eng.close()
