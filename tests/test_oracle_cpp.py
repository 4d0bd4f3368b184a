"""Pins the C++ restatements (CPU baselines) to the Python oracle and the
Appendix A.4 table: the tree-walk restatement of the predicates (decisions and
its field-path diff), the CPU merge over the canonical CSR encoding
("cpu-csr", oracle/csr_ref.cpp) and the oracle's own XXH64."""
import random

import numpy as np
import xxhash

from kcp_amd import gpudiff as G
from oracle import cpu_ref
from tests.golden.kat_cases import cases
from tests.parity import expected_flags, expected_paths, oracle_batch
from tests.workload import make_pairs


def _paths_of(offs, hs, ks, k):
    b, e = int(offs[k]), int(offs[k + 1])
    return list(zip(hs[b:e].tolist(), ks[b:e].tolist()))


def _check(pairs, threads=1, paths=True):
    exp = oracle_batch(pairs)
    want = np.array([expected_flags(r) for r in exp], dtype=np.uint8) & 7  # the C++ baselines: decisions only
    d = cpu_ref.DecodedPairs(pairs)
    flags, sweeps, sec = d.decide(threads)
    assert (flags == want).all(), np.nonzero(flags != want)[0][:10]
    if not paths:
        d.close()
        return
    dirty = np.nonzero(want & 3)[0].tolist()
    offs, hs, ks = d.paths([r["seed"] for r in exp])
    assert offs.size == len(dirty) + 1
    for k, i in enumerate(dirty):
        assert _paths_of(offs, hs, ks, k) == expected_paths(exp[i]), i
    d.close()
    # the CPU merge over the encoder's CSR blobs
    eng = G.Engine(device=G.DEVICE_NONE, encode_threads=2)
    hb = eng.encode(pairs)
    csr = cpu_ref.CsrPairs(hb.pool(), hb.rows())
    f2, offs2, hs2, ks2 = csr.paths()
    assert (f2 == want).all(), np.nonzero(f2 != want)[0][:10]
    for k, i in enumerate(dirty):
        assert _paths_of(offs2, hs2, ks2, k) == expected_paths(exp[i]), i
    f3, sweeps, sec, npaths = csr.run(threads=threads)
    assert (f3 == want).all() and sweeps >= 1 and npaths == hs2.size
    eng.close()


def test_kat():
    _check([(a, b) for _, a, b, _, _ in cases()])


def test_population_threads():
    pairs, _, _ = make_pairs(1500, seed=11, mutate_frac=0.2)
    _check(pairs, threads=4)


def test_deep_objects_and_short_hashes():
    pairs, _, _ = make_pairs(120, seed=16, mix=(("crd", 1.0),), mutate_frac=0.6, crd_leaves=800)
    _check(pairs, threads=2)


def test_xxh64_ref_matches_xxhash():
    """The oracle's independent XXH64 (via the chained path hash of the tree
    restatement) against the xxhash package: a one-component path's hash is
    XXH64(0x01 u32le(len) key, seed)."""
    rnd = random.Random(5)
    for n in list(range(0, 70)) + [127, 128, 1000]:
        key = "".join(rnd.choice("abcxyz") for _ in range(n))
        seed = rnd.randrange(256)
        a = b'{"k":1,"status":{}}'
        b = ('{"k":1,"%s":2,"status":{}}' % key).encode() if key not in ("k", "metadata", "status") else a
        if a == b:
            continue
        d = cpu_ref.DecodedPairs([(a, b)])
        offs, hs, ks = d.paths([seed])
        comp = b"\x01" + len(key.encode()).to_bytes(4, "little") + key.encode()
        assert hs.tolist() == [xxhash.xxh64_intdigest(comp, seed=seed) & 0xFFFFFFFF], key  # reported at 32 bits
        d.close()


def test_csr_paths_ptr_threads_equal_single_pass():
    """bench.py's full-size path check (cpu_ref.csr_paths_ptr: the CPU merge over a host batch in place,
    split over threads) equals the single-threaded CSR checker and the oracle's paths."""
    from kcp_amd import gpudiff as G
    from oracle import cpu_ref
    from tests.parity import expected_paths, oracle_batch
    from tests.workload import make_pairs
    pairs, _, _ = make_pairs(9000, seed=31, mutate_frac=0.2)
    e = G.Engine(device=G.DEVICE_NONE, encode_threads=4)
    hb = e.encode(pairs)
    rows = hb.rows()
    f1, o1, h1, k1 = cpu_ref.CsrPairs(hb.pool(), rows).paths()
    f2, o2, h2, k2 = cpu_ref.csr_paths_ptr(hb.info().pool, rows, threads=5)
    assert np.array_equal(f1, f2) and np.array_equal(o1.astype(np.int64), o2.astype(np.int64))
    assert np.array_equal(h1, h2) and np.array_equal(k1, k2)
    exp = oracle_batch(pairs[:800])
    dirty = [i for i in range(800) if f2[i] & 3]
    for j, i in enumerate(dirty):
        got = list(zip(h2[o2[j]:o2[j + 1]].tolist(), k2[o2[j]:o2[j + 1]].tolist()))
        assert got == expected_paths(exp[i])
    hb.free()
    e.close()


def test_tree_check_equals_decoded_pairs_and_python_oracle():
    """oracle_tree_check (the full-size checker's JSON-in tree walk, threaded, own decoder) gives the same
    flags and changed paths as the per-pair oracle functions and the Python oracle, on a synthetic config3
    population (its seeds from the host encoder's rows) plus the KAT pairs (decode errors included)."""
    from kcp_amd import synth as S
    cfg = S.make_cfg("config3", n_pairs=3000, n_clusters=30, mutate_frac=0.3)
    pop = S.Population(cfg)
    buf, offs, _ = pop.json_range(0, pop.n, 4)
    e = G.Engine(device=G.DEVICE_NONE)
    pairs = [(bytes(buf[offs[2 * i]:offs[2 * i + 1]]), bytes(buf[offs[2 * i + 1]:offs[2 * i + 2]]))
             for i in range(pop.n)]
    pairs += [(a, b) for _, a, b, _, _ in cases()]
    hb = e.encode(pairs)
    seeds = ((hb.rows()["flags_a"] >> G.OBJ_SEED_SHIFT) & 0xFF).astype(np.uint8)
    jb = np.frombuffer(b"".join(a + b for a, b in pairs), np.uint8)
    jo = np.zeros(2 * len(pairs) + 1, np.uint64)
    pos = 0
    for i, (a, b) in enumerate(pairs):
        jo[2 * i], jo[2 * i + 1] = pos, pos + len(a)
        pos += len(a) + len(b)
    jo[-1] = pos
    for threads in (1, 7):
        f, o, h, k = cpu_ref.tree_check(jb, jo, seeds, threads)
        dp = cpu_ref.DecodedPairs(pairs)
        f2, _, _ = dp.decide()
        o2, h2, k2 = dp.paths(seeds)
        dp.close()
        assert np.array_equal(f, f2) and np.array_equal(o, o2) and np.array_equal(h, h2) and np.array_equal(k, k2)
    exp = oracle_batch(pairs)
    assert [int(x) & 7 for x in f] == [expected_flags(r) & 7 for r in exp]
    dirty = [i for i, r in enumerate(exp) if expected_flags(r) & 3]
    for j, i in enumerate(dirty):
        got = list(zip(h[o[j]:o[j + 1]].tolist(), k[o[j]:o[j + 1]].tolist()))
        assert got == expected_paths(exp[i]), i
    hb.free()
    e.close()
