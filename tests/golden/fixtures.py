"""Loader of the committed golden fixtures (tests/golden/*.json.gz, written by
tests/golden/make_fixtures.py)."""
import base64
import gzip
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
NAMES = ("manifests", "config1", "config2", "config3", "config4")


def load(name):
    """[(name, a_json, b_json, expect)] with expect = dict(spec_dirty,
    status_dirty, decode_error, seed, paths=[(hash, kind_with_region_bit,
    rendered_path)])."""
    with gzip.open(os.path.join(HERE, name + ".json.gz")) as f:
        doc = json.load(f)
    assert doc["format"] == 1
    out = []
    for p in doc["pairs"]:
        e = dict(p["expect"])
        e["paths"] = [(int(h, 16), k, s) for h, k, s in e["paths"]]
        out.append((p["name"], base64.b64decode(p["a"]), base64.b64decode(p["b"]), e))
    return out


def expected_flags(e):
    return (1 if e["spec_dirty"] else 0) | (2 if e["status_dirty"] else 0) | (4 if e["decode_error"] else 0)
