#!/usr/bin/env python3
"""Where a K0 blob differs from the host encoder's, section by section (include/gpudiff_format.h): the spec and
status segments (vals u64 | keys u32 | metas u32 | arena) and the path table (hashes, parent hashes, components,
key bytes). A debugging aid for K0 changes, run on the GPU box:

    python tools/k0_diff.py [--lib kcp_amd/_exp/libgpudiff_x.so] [--kat N]

Prints one line per library: the documents compared, how many differ, and for the first differing ones the
sections and entry indices that differ."""
import argparse
import os
import struct
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def sections(info, blob):
    sl, sar, tl, tar = info["spec_l"], info["spec_ar"], info["stat_l"], info["stat_ar"]
    out = {}
    off = 0
    for name, L, ar in (("spec", sl, sar), ("status", tl, tar)):
        out[name + ".vals"] = (off, 8, L)
        out[name + ".keys"] = (off + 8 * L, 4, L)
        out[name + ".metas"] = (off + 12 * L, 4, L)
        out[name + ".arena"] = (off + 16 * L, 1, ar)
        off += 16 * L + ar
    body = (off + 127) & ~127
    n = info["n_tab"]
    out["tab.hash"] = (body, 8, n)
    out["tab.parent"] = (body + 8 * n, 8, n)
    out["tab.comp"] = (body + 16 * n, 8, n)
    out["tab.keys"] = (body + 24 * n, 1, len(blob) - body - 24 * n)
    return out


def diff(info, db, hb):
    res = []
    for name, (o, w, n) in sections(info, hb).items():
        bad = [k for k in range(n) if db[o + w * k:o + w * (k + 1)] != hb[o + w * k:o + w * (k + 1)]]
        if bad:
            ex = [(k, db[o + w * k:o + w * (k + 1)].hex(), hb[o + w * k:o + w * (k + 1)].hex()) for k in bad[:3]]
            res.append((name, len(bad), bad[:6], ex if w > 1 else None))
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", action="append", default=[])
    ap.add_argument("--kat", type=int, default=0, help="also the synthetic config3 sample of this many documents")
    a = ap.parse_args()
    from kcp_amd import gpudiff as G
    from tests.golden.kat_cases import cases as kat_cases
    from tests.golden import fixtures as FX
    docs = []
    for _n, x, y, _se, _st in kat_cases():
        docs += [G.to_json_bytes(x), G.to_json_bytes(y)]
    for name in FX.NAMES:
        for _n, x, y, _e in FX.load(name):
            docs += [x, y]
    host = [G.encode_object_host(d, 0, G.PATH_HASH_BITS) for d in docs]
    for lib in a.lib or [""]:
        if lib:
            G.LIB_PATH = os.path.abspath(lib)
            G._lib = G._load()
        eng = G.Engine(device=0)
        dev = eng.encode_objects(docs, [0] * len(docs))
        eng.close()
        nd, shown = 0, []
        for k, ((di, db), (hi, hb)) in enumerate(zip(dev, host)):
            if di["status"] != 0 or hi["status"] != 0:
                continue
            if db != hb or any(di[f] != hi[f] for f in ("spec_l", "spec_ar", "stat_l", "stat_ar", "n_tab", "bytes")):
                nd += 1
                if len(shown) < 4:
                    shown.append(dict(doc=k, n_nodes=di.get("n_nodes"), fields={f: (di[f], hi[f]) for f in
                                      ("spec_l", "spec_ar", "stat_l", "stat_ar", "n_tab", "bytes") if di[f] != hi[f]},
                                      sections=diff(hi, db, hb) if len(db) == len(hb) else "length",
                                      json=docs[k][:400].decode("utf-8", "replace")))
        print(lib or "kcp_amd/libgpudiff.so", "docs", len(docs), "differing", nd, shown, flush=True)


if __name__ == "__main__":
    main()
