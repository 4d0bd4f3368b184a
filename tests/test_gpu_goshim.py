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


def test_stored_flushes_upload_zero_copy():
    """The Go batcher's store flushes (tests/goshim.py stage_stored, gpudiff.go submitStored) written into
    engine-pinned memory are uploaded without the staging copy (every batch counts as zero-copy) and decide every
    event as the oracle does on (previous version, new version)."""
    import ctypes as C
    import json
    import random
    rnd = random.Random(14)

    def doc(i, v):
        return json.dumps({"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "c%d" % i, "namespace": "ns"},
                           "data": {"k": "v%d" % v, "pad": "x" * rnd.randrange(1, 200)}}, separators=(",", ":")).encode()

    e = G.Engine(device=0, encode_threads=2)
    st = e.object_store(max_slots=32, space_bytes=16 << 20, max_events=64, device_encode=True)
    cur, seen = {}, set()
    for batch in range(4):
        evs, pairs = [], []
        for s in rnd.sample(range(24), 16):
            new = doc(s, rnd.randrange(3))
            old = cur.get(s)
            evs.append((s, old, new))
            pairs.append((old if old is not None else b"{}", new))
            cur[s] = new
        pin, plain, entries = S.stage_stored(evs, seen)
        p = C.c_void_p()
        assert G.lib().gpudiff_host_alloc(e.ctx, len(pin), C.byref(p)) == G.OK
        C.memmove(p.value, pin, len(pin))
        pb = C.create_string_buffer(plain, max(1, len(plain)))
        arr = (G.Event * len(entries))()
        for i, (slot, n, o, in_jb) in enumerate(entries):
            arr[i].slot, arr[i].pair_id = slot, i
            arr[i].new_json, arr[i].new_len = p.value + n[0], n[1]
            if o is not None:
                base = p.value if in_jb else C.addressof(pb)
                arr[i].old_json, arr[i].old_len = base + o[0], o[1]
        z0 = st.stats().zero_copy_batches
        r = e.wait(st.submit_raw(arr, len(entries), (pb,)))
        assert st.stats().zero_copy_batches == z0 + 1
        assert_matches(r, pairs)
        G.lib().gpudiff_host_free(e.ctx, p)
    st.free()
    e.close()
