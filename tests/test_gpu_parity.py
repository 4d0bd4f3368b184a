"""GPU parity: the HIP path (through the C-ABI) against the oracle, bit-exact.

Covers the Appendix A.4 KAT table, mixed synthetic populations (configs 1-4
shapes, 5% mutated), deep objects (>64 leaves per region -> multi-window
merge-join, long values split into an 8-B head and an arena tail), forced
path-hash collisions, multi-chunk batches (scan tiles), appends and
single-pair drop-ins."""
import json
import random

import numpy as np
import pytest
import torch

from kcp_amd import gpudiff as G
from oracle import gpudiff_oracle as O
from tests.golden.kat_cases import BASE, J, cases
from tests.parity import assert_matches, oracle_batch
from tests.workload import deep_pairs, make_pairs

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", params=[False, True], ids=["host_encode", "device_encode"])
def eng(request):
    """Both submit paths: host encoding, and device encoding (raw JSON up,
    kernel K0 encodes, the host re-does only what K0 defers)."""
    assert G.device_count() > 0, "no GPU visible"
    e = G.Engine(device=0, encode_threads=8, timing=True, device_encode=request.param)
    yield e
    e.close()


def test_kat(eng):
    cs = cases()
    pairs = [(a, b) for _, a, b, _, _ in cs]
    res = eng.diff_pairs(pairs)
    exp = assert_matches(res, pairs)
    for (name, a, b, se, st), r in zip(cs, exp):
        if se is not None:
            assert r["spec_dirty"] == (not se), name


def test_empty_batch(eng):
    res = eng.diff_pairs([])
    assert res.pair_flags.size == 0 and res.dirty_ids.size == 0 and res.path_offsets.tolist() == [0]


def test_mixed_population(eng):
    pairs, cl, muts = make_pairs(3000, seed=1)
    ids = [1000 + 3 * i for i in range(len(pairs))]
    res = eng.diff_pairs(pairs, ids=ids, clusters=cl)
    assert_matches(res, pairs, ids=ids)


def test_all_mutated_many_chunks(eng):
    # > SCAN_TILE dirty pairs and > 64-pair chunks, every pair dirty
    pairs, _, _ = make_pairs(5000, seed=2, mix=(("cm", 0.5), ("deploy", 0.5)), mutate_frac=1.0, pretty_frac=0)
    res = eng.diff_pairs(pairs)
    assert_matches(res, pairs)


def test_deep_objects(eng):
    pairs, _, _ = make_pairs(300, seed=3, mix=(("crd", 1.0),), mutate_frac=0.5, crd_leaves=1500)
    res = eng.diff_pairs(pairs)
    assert_matches(res, pairs)


def test_long_values_and_list_shift(eng):
    rnd = random.Random(4)
    pairs = []
    for i in range(200):
        a = json.loads(J(BASE))
        a["spec"]["blob"] = "".join(rnd.choice("ab") for _ in range(rnd.randint(9, 300)))
        a["spec"]["items"] = ["item-%03d-%s" % (k, "x" * rnd.randint(0, 40)) for k in range(rnd.randint(60, 200))]
        b = json.loads(json.dumps(a))
        c = i % 4
        if c == 0:
            b["spec"]["blob"] = b["spec"]["blob"][:-1] + ("a" if b["spec"]["blob"][-1] == "b" else "b")
        elif c == 1:
            del b["spec"]["items"][len(b["spec"]["items"]) // 2]
        elif c == 2:
            b["spec"]["items"].insert(3, "new")
        pairs.append((J(a), J(b)))
    res = eng.diff_pairs(pairs)
    assert_matches(res, pairs)


@pytest.mark.parametrize("shrink", [9, 10, 12, 14])
def test_deferred_join_path(shrink):
    """Wave arenas shrunk until most dirty pairs do not fit: those pairs take the
    deferred K4 path (and with shrink 14 every pair with a path does);
    results must not change."""
    pairs, _, _ = make_pairs(1500, seed=14, mutate_frac=0.4, crd_leaves=300, pretty_frac=0)
    e = G.Engine(device=0, flags=shrink << G.OPT_ARENA_SHIFT)
    res = e.diff_pairs(pairs)
    assert_matches(res, pairs)
    e.close()


def test_scratch_overflow_keeps_arena_paths():
    """Deferred pairs whose paths overflow the initial K4 scratch (64Ki entries)
    force the grow-and-rejoin path in gpudiff_wait, while the small pairs' paths
    already sit in the K2 wave arenas: both sets must survive the re-run."""
    rnd = random.Random(15)
    pairs = []
    for i in range(800):
        a = json.loads(J(BASE))
        a["spec"]["m"] = {"k%04d" % k: rnd.randint(0, 1 << 40) for k in range(260)}
        b = json.loads(json.dumps(a))
        if i % 2:  # ~260 changed paths: deferred to K4
            b["spec"]["m"] = {k: v + 1 for k, v in b["spec"]["m"].items()}
        else:  # one changed path: joined inside K2
            b["spec"]["m"]["k0007"] += 1
        pairs.append((J(a), J(b)))
    e = G.Engine(device=0, flags=10 << 21)
    res = e.diff_pairs(pairs)
    assert res.path_hashes.size > 65536 + 65536 // 8
    assert_matches(res, pairs)
    e.close()


def test_small_deferrals_take_exact_scratch():
    """a small pair deferred only because its K2 wave arena is full (here: no arena at all, so
    every dirty pair is deferred) gets exactly its merged keys + sentinel as K4 scratch and is joined whole
    by K3 -- not two 1024-entry slices -- and deep pairs in the same batch still go through the slices.
    The scratch need (summary word 3) must be the exact sum, the first pass overflows the default 64Ki
    scratch (the grow-and-rejoin path re-places and re-joins whole deferrals), and every flag, ID and path
    equals the oracle's."""
    small, _, _ = make_pairs(9000, seed=91, mix=(("cm", 0.6), ("deploy", 0.4)), mutate_frac=0.9, pretty_frac=0)
    deep = deep_pairs()[:6]
    pairs = small + deep
    e = G.Engine(device=0, flags=15 << 21)  # arena_per_wave = 16384 >> 15 = 0
    hb = e.encode(pairs)
    rows = hb.rows()
    db = e.device_batch(hb.info().pool_bytes + 4096, len(pairs))
    db.append(hb)
    res = e.wait(e.diff(db))
    exp = assert_matches(res, pairs)
    import torch
    cnt = torch.zeros(8, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()  # the engine's stream does not order against torch's null stream
    db.export(G.EXPORT_COUNTS, cnt.data_ptr(), 8)
    e.sync()
    scratch = int(cnt[3].item()) & 0xFFFFFFFF
    # expected: per dirty pair (not a decode error) need = joined regions' leaves + sentinel, whole when
    # <= 1024, else whole 1024-entry slices (spec slices + status slices, at least need)
    want, n_whole = 0, 0
    for r, x in zip(rows, exp):
        if not (x["spec_dirty"] or x["status_dirty"]) or x.get("decode_error"):
            continue
        ls = int(r["spec_l_a"]) + int(r["spec_l_b"]) if x["spec_dirty"] else 0
        has_st_b = bool(int(r["flags_b"]) & G.OBJ_HAS_STATUS)
        lt = int(r["stat_l_a"]) + int(r["stat_l_b"]) if x["status_dirty"] else 0
        need = ls + lt + (1 if (x["status_dirty"] and not has_st_b) else 0)
        if need <= 1024:
            want += need
            n_whole += 1
        else:
            sl = -(-ls // 1024) + -(-lt // 1024)
            want += max(sl, -(-need // 1024)) * 1024
    assert n_whole > 5000 and want > 65536
    assert scratch == want, (scratch, want)
    db.free()
    hb.free()
    e.close()


@pytest.mark.parametrize("dev", [False, True], ids=["host_encode", "device_encode"])
def test_forced_collisions(dev):
    e = G.Engine(device=0, path_hash_bits=8, device_encode=dev)
    pairs, _, _ = make_pairs(200, seed=5, mix=(("cm", 0.5), ("deploy", 0.5)), mutate_frac=0.5)
    res = e.diff_pairs(pairs)
    assert_matches(res, pairs, hash_bits=8)
    e.close()


@pytest.mark.parametrize("shrink", [0, 14])
def test_tail_confirmation(shrink):
    """Long values of equal length whose first 8 bytes (the head, in the leaf record) agree are decided by
    the byte confirmation of their tails in the arenas: one flipped byte anywhere in a 9-400 byte value,
    at least half of them past the head, both for joins inside K2 (shrink 0) and in K4 (shrink 14: every
    pair deferred)."""
    rnd = random.Random(12)
    pairs = []
    for i in range(300):
        a = json.loads(J(BASE))
        a["spec"]["vals"] = ["".join(rnd.choice("xy") for _ in range(rnd.randint(9, 400))) for _ in range(12)]
        b = json.loads(json.dumps(a))
        if i % 2:
            k = rnd.randrange(12)
            s = b["spec"]["vals"][k]
            j = rnd.randrange(8, len(s)) if i % 4 == 1 else rnd.randrange(len(s))
            b["spec"]["vals"][k] = s[:j] + ("x" if s[j] == "y" else "y") + s[j + 1:]  # same length, one byte
        pairs.append((J(a), J(b)))
    e = G.Engine(device=0, flags=shrink << 21)
    res = e.diff_pairs(pairs)
    assert_matches(res, pairs)
    e.close()


def _long_value_corpus():
    """Long values of every length class the format splits differently: 9-70 B (tails of 1-62 B), values
    around 128-B lines, a 5 KB value, non-ASCII bytes, and one object with 700 long values; in spec and
    status segments of both objects."""
    rnd = random.Random(11)
    out = []
    for n in list(range(9, 70)) + [95, 96, 97, 127, 128, 129, 130, 159, 160, 161, 255, 256, 257, 511, 512, 513, 5000]:
        a = {"kind": "ConfigMap", "metadata": {"name": "lv-%d" % n},
             "data": {"v%d" % j: "".join(rnd.choice("abcdefgh\u00e9") for _ in range(n + j)) for j in range(3)},
             "status": {"s": "x" * (n + 5), "short": "y" * 7}}
        b = json.loads(json.dumps(a))
        b["data"]["v1"] = b["data"]["v1"][::-1]
        out.append((json.dumps(a).encode(), json.dumps(b).encode()))
    many = {"kind": "Big", "metadata": {"name": "many"}, "spec": {"k%04d" % j: "v" * (9 + j % 200) for j in range(700)}}
    out.append((json.dumps(many).encode(), json.dumps(many).encode()))
    return out


def _json_strings(x, out):
    if isinstance(x, str):
        out.append(x.encode())
    elif isinstance(x, dict):
        for v in x.values():
            _json_strings(v, out)
    elif isinstance(x, list):
        for v in x:
            _json_strings(v, out)
    return out


def test_value_heads_and_tails_resident(eng):
    """After the upload the resident pool is the host encoder's byte for byte, and every long string reads
    back whole from its head (the leaf's 8-B value slot) and its tail (the arena): the multiset of long
    values per object equals the JSON's strings longer than 8 bytes in the compared regions."""
    pairs = _long_value_corpus()
    hb = eng.encode(pairs)
    info = hb.info()
    db = eng.device_batch(info.pool_bytes + 1024, len(pairs))
    db.append(hb)
    eng.sync()
    pool = db.read_pool(0, info.pool_bytes)
    assert pool == hb.pool()
    checked = 0
    for r, (ja, jb) in zip(hb.rows(), pairs):
        for side, js in (("a", ja), ("b", jb)):
            off, sl, sar = int(r["off_" + side]), int(r["spec_l_" + side]), int(r["spec_ar_" + side])
            tl, tar = int(r["stat_l_" + side]), int(r["stat_ar_" + side])
            got = [vb for (k, v, m, vb) in G.decode_segment(pool, off, sl, sar) +
                   G.decode_segment(pool, off + G.segment_bytes(sl, sar), tl, tar) if (m & 7) == 5 and (m >> 3) > 8]
            obj = json.loads(js)
            want = [x for x in _json_strings({k: v for k, v in obj.items() if k != "metadata"}, []) if len(x) > 8]
            assert sorted(got) == sorted(want)
            checked += len(got)
    assert checked > 1000
    res = eng.wait(eng.diff(db))
    assert_matches(res, pairs)
    db.free()
    hb.free()


@pytest.mark.parametrize("dev", [False, True], ids=["host_encode", "device_encode"])
@pytest.mark.parametrize("n_pairs", [1, 37, 3000])
def test_long_value_corpus_vs_oracle(n_pairs, dev):
    """The long-value corpus plus mixed populations through both encoders (host CSR / K0): flags, ID lists
    and changed paths equal the oracle's."""
    e = G.Engine(device=0, encode_threads=8, device_encode=dev)
    pairs, _, _ = make_pairs(n_pairs, seed=70 + n_pairs, mutate_frac=0.2)
    if n_pairs > 1:
        pairs = _long_value_corpus() + pairs
    res = e.diff_pairs(pairs)
    assert_matches(res, pairs)
    e.close()


def test_append_chunks_and_rediff(eng):
    pairs, cl, _ = make_pairs(1500, seed=8, mutate_frac=0.1)
    chunks = [pairs[0:100], pairs[100:900], pairs[900:]]
    hbs = [eng.encode(c, ids=list(range(s, s + len(c)))) for c, s in zip(chunks, (0, 100, 900))]
    total = sum(h.info().pool_bytes for h in hbs)
    db = eng.device_batch(total + 4096, len(pairs))
    for h in hbs:
        db.append(h)
    st = db.stats()
    assert st.n_pairs == len(pairs) and st.pool_bytes == total
    r1 = eng.wait(eng.diff(db))
    exp = assert_matches(r1, pairs)
    r2 = eng.wait(eng.diff(db))  # re-diff of the resident batch is identical
    assert_matches(r2, pairs, exp=exp)
    t = eng.timings()
    assert t.compare_ms > 0 and t.total_ms >= t.compare_ms
    db.free()


def test_single_pair_dropins(eng):
    for name, a, b, se, st in cases():
        r = O.diff_pair(a, b)
        assert eng.spec_equal(a, b) == (not r["spec_dirty"]), name
        assert eng.status_equal(a, b) == (not r["status_dirty"]), name


def test_submit_pipelining(eng):
    # two tickets in flight on the submit ring
    p1, _, _ = make_pairs(300, seed=9, mutate_frac=0.2)
    p2, _, _ = make_pairs(500, seed=10, mutate_frac=0.2)
    t1 = eng.submit(p1)
    t2 = eng.submit(p2)
    assert_matches(eng.wait(t2), p2)
    assert_matches(eng.wait(t1), p1)


@pytest.mark.parametrize("timeline", [False, True], ids=["default", "timeline_build"])
def test_k2_kernels_bit_exact(timeline):
    """The four decision kernels -- 8 chunks a side in flight (mixed pairs) and 16 (deep pairs, >= 16 KiB a pair),
    each also as the per-wave timeline build (selected while gpudiff_k2_profile has a buffer installed) -- against
    the oracle, with joins in K2 and with every join deferred to K4."""
    pairs, _, _ = make_pairs(1200, seed=31, mutate_frac=0.3, pretty_frac=0)
    deep, _, _ = make_pairs(120, seed=32, mix=(("crd", 1.0),), mutate_frac=0.5, crd_leaves=2500, pretty_frac=0)
    for shrink in (0, 12):
        e = G.Engine(device=0, flags=shrink << G.OPT_ARENA_SHIFT)
        if timeline:
            prof = torch.zeros(12 << 16, dtype=torch.int64, device="cuda")
            e.k2_profile(prof.data_ptr(), 1 << 16)
        assert_matches(e.diff_pairs(pairs), pairs)
        hb = e.encode(deep)
        assert hb.info().pool_bytes / len(deep) > 2 * 16384  # the deep-pair kernel
        hb.free()
        assert_matches(e.diff_pairs(deep), deep)
        if timeline:
            e.sync()
            assert int((prof.view(-1, 12)[:, 4] != 0).sum()) > 0  # the timeline build ran and recorded waves
            e.k2_profile(0, 0)
        e.close()


@pytest.mark.parametrize("n", [1, 63, 64, 65, 4095, 6000, 20000])
def test_k2_hand_out_shapes_bit_exact(n):
    """Batch sizes around the chunk and item boundaries: 64-pair chunks split into items, the tail of half-size
    items, dynamic tickets -- against the oracle."""
    pairs, _, _ = make_pairs(n, seed=33 + n, mutate_frac=0.2, pretty_frac=0)
    e = G.Engine(device=0)
    res = e.diff_pairs(pairs)
    assert_matches(res, pairs)
    e.close()


def test_k2_largest_first_round():
    """Large pairs (>= 16 KiB compared on average): K2's final round of items is handed out largest first
    (k_tail_order's permutation, cached per batch under the exact launch shape and the rows' generation);
    repeated passes over the same batch (the cached order), over a view (its own order) and after the batch
    was reset and refilled with other pairs of the same count (a new order): identical to the oracle."""
    pairs, _, _ = make_pairs(900, seed=61, mix=(("crd", 1.0),), mutate_frac=0.4, crd_leaves=2500, pretty_frac=0)
    other, _, _ = make_pairs(900, seed=62, mix=(("crd", 1.0),), mutate_frac=0.6, crd_leaves=3000, pretty_frac=0)
    e = G.Engine(device=0)
    hb = e.encode(pairs)
    ho = e.encode(other)
    assert hb.info().pool_bytes / len(pairs) > 2 * 16384  # the large-pair path
    db = e.device_batch(max(hb.info().pool_bytes, ho.info().pool_bytes) + 4096, len(pairs))
    db.append(hb)
    exp = assert_matches(e.wait(e.diff(db)), pairs)
    assert_matches(e.wait(e.diff(db)), pairs, exp=exp)
    e2 = G.Engine(device=0)
    v = db.view(e2)
    assert_matches(e2.wait(e2.diff(v)), pairs, exp=exp)
    v.free()
    db.reset()
    db.append(ho)
    assert_matches(e.wait(e.diff(db)), other)
    db.free()
    hb.free()
    ho.free()
    e2.close()
    e.close()


@pytest.mark.parametrize("mode", ["slices", "slices_all"])
def test_deep_joins_merge_path(mode):
    """Joins over 2048 keys go to K4's merge-path slices (1024 merged keys each: several slices per
    region, equal keys straddling slice boundaries, list shifts with thousands of changed paths);
    "slices_all": a shrunken K2 arena sends every dirty pair, small ones included, through the slices.
    Flags, IDs and paths equal the oracle's."""
    pairs = deep_pairs() + make_pairs(300, seed=43, mutate_frac=0.4)[0]
    flags = {"slices": 0, "slices_all": 14 << G.OPT_ARENA_SHIFT}[mode]
    e = G.Engine(device=0, flags=flags)
    assert_matches(e.diff_pairs(pairs), pairs)
    e.close()


def test_k2_hand_out_orders_agree_on_deep_batches():
    """A deep batch large enough for every K2 hand-out stage (config4 shape, 40k pairs: 4-pair main items, a
    round of whole items and a round of single pairs both handed out largest first, their joins over 1024 keys
    deferred to K4): the default and every join deferred to K4's slices (a shrunken arena) give identical flags,
    ID lists and changed paths, and the flags equal the generator's ground truth."""
    from kcp_amd import synth as S
    pop = S.Population(S.make_cfg("config4", n_pairs=40000))
    res = {}
    for name, flags in (("default", 0), ("all_joins_in_k4", 14 << G.OPT_ARENA_SHIFT)):
        e = G.Engine(device=0, encode_threads=16, flags=flags)
        ch = pop.chunk(e, 0, pop.n, 16)
        db = e.device_batch(ch.hb.info().pool_bytes + 4096, pop.n)
        db.append(ch.hb)
        r = e.wait(e.diff(db))
        r2 = e.wait(e.diff(db))  # the cached order
        assert np.array_equal(r.pair_flags, r2.pair_flags) and np.array_equal(r.path_hashes, r2.path_hashes)
        res[name] = r
        truth = ch.truth
        db.free()
        ch.hb.free()
        e.close()
    want = res["default"]
    assert np.array_equal(want.pair_flags & (G.SPEC_DIRTY | G.STATUS_DIRTY), pop.expected_flags(truth))
    for name, r in res.items():
        for f in ("pair_flags", "spec_dirty_ids", "status_dirty_ids", "path_offsets", "path_hashes", "path_kinds"):
            assert np.array_equal(getattr(r, f), getattr(want, f)), (name, f)
