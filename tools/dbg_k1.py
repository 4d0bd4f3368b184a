"""Locate K1 digest mismatches: encode pairs, let K1 (variant from argv) hash them on the device, and
report every 8-B value slot that differs from the host encoder's XXH64 digest."""
import sys
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from kcp_amd import gpudiff as G
from tests.golden.kat_cases import cases
from tests.workload import make_pairs

variant = int(sys.argv[1]) if len(sys.argv) > 1 else 0
sets = {"kat": [(a, b) for _, a, b, _, _ in cases()], "mix": make_pairs(500, seed=5, mutate_frac=0.2)[0]}
host = G.Engine(device=G.DEVICE_NONE, host_value_hash=True)
eng = G.Engine(device=0, flags=variant << 30, device_value_hash=True)
for name, pairs in sets.items():
    ref = host.encode(pairs)
    hb = eng.encode(pairs)
    info = hb.info()
    db = eng.device_batch(info.pool_bytes + 1024, len(pairs))
    db.append(hb)
    eng.sync()
    got = np.frombuffer(db.read_pool(0, info.pool_bytes), np.uint8)
    want = np.frombuffer(ref.pool(), np.uint8)
    rows = hb.rows()
    bad = 0
    for pi, r in enumerate(rows):
        for side in ("a", "b"):
            off, sl, sar, tl, tar = (int(r["off_" + side]), int(r["spec_l_" + side]), int(r["spec_ar_" + side]),
                                     int(r["stat_l_" + side]), int(r["stat_ar_" + side]))
            for reg, (so, L, AR) in enumerate(((off, sl, sar), (off + 16 * sl + sar, tl, tar))):
                if not L:
                    continue
                m = np.frombuffer(want[so + 12 * L: so + 16 * L].tobytes(), np.uint32)
                run = 0
                for i in range(L):
                    w = want[so + 8 * i: so + 8 * i + 8].tobytes()
                    g = got[so + 8 * i: so + 8 * i + 8].tobytes()
                    ln = int(m[i] >> 3)
                    lg = (m[i] & 7) == 5 and ln > 8
                    if w != g:
                        bad += 1
                        if bad <= 12:
                            print(name, "pair", pi, side, "region", reg, "leaf", i, "of", L, "len", ln, "long", lg,
                                  "arena_off", run, "AR", AR, "got", g.hex(), "want", w.hex())
                    if lg:
                        run += (ln + 3) & ~3
    rest = int((got != want).sum())
    print(name, "variant", variant, "bad slots", bad, "differing bytes", rest, flush=True)
    db.free(); hb.free(); ref.free()
