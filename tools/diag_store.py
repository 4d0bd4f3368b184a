"""Diagnostic (GPU box): where a device-encode store's deferrals come from on the
config5 population -- K0 statuses of both versions, K0-vs-host blob identity,
path-table agreement of each object's two versions, and per-batch deferrals of
a short replay.  usage: python tools/diag_store.py [objects] [batch]"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from kcp_amd import gpudiff as G  # noqa: E402
from kcp_amd import synth as S  # noqa: E402
from bench_replay import EVENT_DTYPE  # noqa: E402


def agree(ta, tb):
    a = {h: (ph, c) for h, ph, c in ta}
    bad = [(h, a[h], (ph, c)) for h, ph, c in tb if h in a and a[h] != (ph, c)]
    return bad


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
    cfg = S.make_cfg("config3", n_pairs=M, n_clusters=max(1, M // 100))
    pop = S.Population(cfg)
    buf, offs, truth = pop.json_range(0, M, 16)
    raw = buf.tobytes()
    docs = [raw[offs[i]:offs[i + 1]] for i in range(2 * M)]
    eng = G.Engine(device=0, encode_threads=16)
    n_s = min(4000, M)
    samp = []
    for i in range(n_s):
        samp += [docs[2 * i], docs[2 * i + 1]]
    dev = eng.encode_objects(samp)
    hist = {}
    for di, _db in dev:
        hist[di["status"]] = hist.get(di["status"], 0) + 1
    print("K0 statuses over %d docs: %s" % (len(samp), hist), flush=True)
    ident = mism = dis = 0
    for k, (doc, (di, db)) in enumerate(zip(samp, dev)):
        if di["status"] != G.TOK_OK:
            continue
        hi, hb = G.encode_object_host(doc, 0, G.PATH_HASH_BITS)
        if hb == db:
            ident += 1
        else:
            mism += 1
            if mism <= 3:
                print("blob mismatch doc %d: dev %s host %s" % (k, di, hi), flush=True)
    for i in range(n_s):
        (ia, ba), (ib, bb) = dev[2 * i], dev[2 * i + 1]
        if ia["status"] or ib["status"]:
            continue
        bad = agree(G.decode_path_table(ba, ia), G.decode_path_table(bb, ib))
        if bad:
            dis += 1
            if dis <= 3:
                print("tables disagree for object %d: %s" % (i, bad[:3]), flush=True)
    print("K0 vs host: %d identical, %d differ; version tables disagree for %d of %d objects" % (
        ident, mism, dis, n_s), flush=True)
    # short replay
    base = buf.ctypes.data
    starts = offs[:-1].astype(np.uint64) + np.uint64(base)
    lens = np.diff(offs).astype(np.uint64)
    a_ptr, b_ptr, a_len, b_len = starts[0::2], starts[1::2], lens[0::2], lens[1::2]
    st = eng.object_store(M, int(float(lens.mean()) * 2.2 * M * 2.5) + (256 << 20), B, device_encode=True)

    def submit(slots, new_is_b, with_old):
        ev = np.zeros(slots.size, dtype=EVENT_DTYPE)
        ev["slot"] = slots
        ev["pair_id"] = np.arange(slots.size, dtype=np.uint32)
        ev["new_json"] = np.where(new_is_b, b_ptr[slots], a_ptr[slots])
        ev["new_len"] = np.where(new_is_b, b_len[slots], a_len[slots])
        if with_old:
            ev["old_json"] = np.where(new_is_b, a_ptr[slots], b_ptr[slots])
            ev["old_len"] = np.where(new_is_b, a_len[slots], b_len[slots])
        arr = (G.Event * ev.size).from_buffer(ev)
        return eng.wait(st.submit_raw(arr, ev.size, ev))

    prev = 0
    for s0 in range(0, M, B):
        sl = np.arange(s0, min(M, s0 + B), dtype=np.uint32)
        submit(sl, np.zeros(sl.size, bool), False)
    s = st.stats()
    print("initial list: deferred %d, live %d, used %.2f GB, compactions %d" % (
        s.deferred, s.live_slots, s.used_bytes / 1e9, s.compactions), flush=True)
    prev = s.deferred
    rng = np.random.default_rng(5)
    on_b = np.zeros(M, bool)
    for k in range(8):
        sl = rng.choice(M, size=B, replace=False).astype(np.uint32)
        nb = ~on_b[sl]
        on_b[sl] = nb
        submit(sl, nb, True)
        s = st.stats()
        print("batch %d: deferred %d (reseeded %d total, unresolved %d, compactions %d, used %.2f GB)" % (
            k, s.deferred - prev, s.reseeded, s.collisions_unresolved, s.compactions, s.used_bytes / 1e9),
            flush=True)
        prev = s.deferred
    st.free()
    eng.close()


if __name__ == "__main__":
    main()
