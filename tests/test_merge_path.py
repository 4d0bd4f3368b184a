"""CPU restatement of K4's merge-path slicing (kcp_amd/csrc/kernels.hip: merge_split, join_slice,
k_join_slices / k_join_gather), checked against the unsliced merge-join.

A deferred pair's region join is cut into slices of D merged keys of the two sorted key lists (A before B
on equal keys); a slice's split points come from a 64-ary search, and an equal key straddling a split stays
with the slice holding its A side.  Joining every slice on its own and concatenating the outputs in slice
order must give exactly the unsliced join -- for any D, any overlap of the key sets, keys shared at slice
boundaries, empty sides.  (The GPU path is held to the oracle by
tests/test_gpu_parity.py::test_deep_joins_merge_path; this pins the slicing rule itself.)"""
import random

import pytest


def merge_split(ka, kb, dg):
    """Number of A keys among the first dg merged keys -- the 64-ary search of kernels.hip:merge_split,
    with the 64 lanes' probes restated as a loop."""
    La, Lb = len(ka), len(kb)
    lo, hi = max(0, dg - Lb), min(dg, La)
    while lo < hi:
        span = hi - lo
        step = (span + 63) // 64
        probes = [lo + l * step for l in range(64) if lo + l * step < hi]
        inc = [ka[ia] <= kb[dg - ia - 1] for ia in probes]
        if all(inc):
            last = len(probes) - 1
            lo = lo + last * step + 1
            if step == 1:
                break
            hi = min(hi, lo + step - 1)
        else:
            f = inc.index(False)
            nhi = lo + f * step
            lo = lo + (f - 1) * step + 1 if f else lo
            hi = nhi
    return lo


def join(ka, kb, va, vb):
    """The merge-join of one region: (key, kind) in ascending key order; kind 'C' changed, 'R' only in A,
    'A' only in B (join_region's emission order)."""
    out = []
    i = j = 0
    while i < len(ka) or j < len(kb):
        if j >= len(kb) or (i < len(ka) and ka[i] < kb[j]):
            out.append((ka[i], "R"))
            i += 1
        elif i >= len(ka) or kb[j] < ka[i]:
            out.append((kb[j], "A"))
            j += 1
        else:
            if va[i] != vb[j]:
                out.append((ka[i], "C"))
            i += 1
            j += 1
    return out


def join_sliced(ka, kb, va, vb, D):
    L = len(ka) + len(kb)
    out = []
    for dg0 in range(0, L, D):
        dg1 = min(dg0 + D, L)
        ia0 = merge_split(ka, kb, dg0)
        ib0 = dg0 - ia0
        ia1 = merge_split(ka, kb, dg1)
        ib1 = dg1 - ia1
        if ia0 > 0 and ib0 < len(kb) and ka[ia0 - 1] == kb[ib0]:
            ib0 += 1
        if ia1 > 0 and ib1 < len(kb) and ka[ia1 - 1] == kb[ib1]:
            ib1 += 1
        ib1 = max(ib1, ib0)
        part = join(ka[ia0:ia1], kb[ib0:ib1], va[ia0:ia1], vb[ib0:ib1])
        assert len(part) <= D  # a slice's paths fit its scratch slot (defer_cap)
        out += part
    return out


def brute_split(ka, kb, dg):
    merged = sorted([(k, 0) for k in ka] + [(k, 1) for k in kb])
    return sum(1 for k, side in merged[:dg] if side == 0)


def lists(rnd, na, nb, shared, space):
    keys = rnd.sample(range(space), na + nb)
    common = keys[:shared]
    a = sorted(common + keys[shared:na])
    b = sorted(common + keys[na:na + nb - shared])
    return a, b


@pytest.mark.parametrize("seed", range(40))
def test_merge_split_matches_merged_order(seed):
    rnd = random.Random(seed)
    na, nb = rnd.randint(0, 3000), rnd.randint(0, 3000)
    shared = rnd.randint(0, min(na, nb))
    ka, kb = lists(rnd, na, nb, shared, 10 * (na + nb) + 10)
    for dg in sorted(set([0, na + nb] + [rnd.randint(0, na + nb) for _ in range(30)])):
        assert merge_split(ka, kb, dg) == brute_split(ka, kb, dg)


@pytest.mark.parametrize("seed", range(60))
def test_sliced_join_equals_join(seed):
    rnd = random.Random(1000 + seed)
    na, nb = rnd.randint(0, 5000), rnd.randint(0, 5000)
    shared = rnd.randint(0, min(na, nb))
    if seed % 3 == 0:  # mostly equal lists (an unchanged deep object with a few edits)
        shared = min(na, nb)
    ka, kb = lists(rnd, na, nb, shared, 4 * (na + nb) + 10)
    va = [rnd.randint(0, 3) for _ in ka]
    pos = {k: i for i, k in enumerate(ka)}
    vb = [va[pos[k]] if k in pos and rnd.random() < 0.9 else rnd.randint(0, 3) for k in kb]
    want = join(ka, kb, va, vb)
    for D in (1, 2, 3, 64, 1024, rnd.randint(5, 700)):
        assert join_sliced(ka, kb, va, vb, D) == want, D


def test_equal_keys_on_every_boundary():
    # identical lists: every merged pair (A[i], B[i]) straddles an odd D's boundaries somewhere
    ka = list(range(0, 4000, 2))
    kb = list(ka)
    va = [i % 5 for i in range(len(ka))]
    vb = [(v + (i % 7 == 0)) % 5 for i, v in enumerate(va)]
    want = join(ka, kb, va, vb)
    for D in (1, 3, 7, 1023, 1024, 1025):
        assert join_sliced(ka, kb, va, vb, D) == want


def _defer_cap(ls, lt, sent, slice_=1024):
    """Restatement of kernels.hip defer_cap: exact entries for a whole deferral (need <= one slice), else
    whole slices per region and at least need."""
    need = ls + lt + sent
    if need <= slice_:
        return need
    sl = -(-ls // slice_) + -(-lt // slice_)
    return max(sl, -(-need // slice_)) * slice_


def _place(caps, slice_=1024):
    """Restatement of kernels.hip place_deferred over a batch's deferred pairs (in dirty order): slot q
    (starting at entry q * slice) belongs to the pair whose entries contain its start; a whole deferral
    marks it 'none'."""
    owner = {}
    so = 0
    offs = []
    for d, cap in enumerate(caps):
        offs.append(so)
        b0, b1 = -(-so // slice_), -(-(so + cap) // slice_)
        for q in range(b0, b1):
            assert q not in owner
            owner[q] = d if cap > slice_ else None
            if cap <= slice_:
                assert b1 - b0 == 1  # a whole deferral holds at most one slot start
        so += cap
    return owner, offs, so


@pytest.mark.parametrize("seed", range(20))
def test_deferred_scratch_placement(seed):
    """whole deferrals take exact entries, sliced ones whole slices at unaligned offsets.  Every
    slot starting inside the batch's entries is written exactly once; a sliced pair owns exactly cap / 1024
    consecutive slots starting at slot_ceil(so), and its slice i's window [so + 1024 i, +1024) lies inside
    its entries -- what K4a (slice i = s - slot_ceil(so)) and K4b (first slot = slot_ceil(so)) rely on."""
    rnd = random.Random(seed)
    caps, kinds = [], []
    for _ in range(rnd.randint(1, 400)):
        if rnd.random() < 0.8:
            ls, lt = rnd.randint(0, 600), rnd.randint(0, 400)
        else:
            ls, lt = rnd.randint(0, 9000), rnd.randint(0, 5000)
        sent = rnd.randint(0, 1)
        if ls + lt + sent == 0:
            sent = 1
        cap = _defer_cap(ls, lt, sent)
        assert cap >= ls + lt + sent
        if cap > 1024:
            assert cap % 1024 == 0 and cap >= 2048 and cap // 1024 >= -(-ls // 1024) + -(-lt // 1024)
        caps.append(cap)
    owner, offs, total = _place(caps)
    assert sorted(owner) == list(range(-(-total // 1024)))
    for d, (cap, so) in enumerate(zip(caps, offs)):
        mine = sorted(q for q, o in owner.items() if o == d)
        if cap <= 1024:
            assert not mine
            continue
        first = -(-so // 1024)
        assert mine == list(range(first, first + cap // 1024))
        for q in mine:
            i = q - first
            assert so <= so + 1024 * i and so + 1024 * (i + 1) <= so + cap
