"""What libgpudiff.so is built from, and the build ID that ties a loaded library to those sources.

`kcp_amd/build.py` compiles `source_id()` into both libraries (`gpudiff_build_id()`,
`gpudiff_synth_build_id()`); `kcp_amd/gpudiff.py` recomputes it from the sources that ship beside the
library and refuses a library whose ID differs, as it refuses another ABI.  The ID hashes file CONTENTS
(never mtimes, which a fresh checkout or a push can reorder), the compiler flags included (they live
in build.py, which is hashed too).  Pure stdlib, no side effects at import: build.py loads it by path.
"""
import hashlib
import os

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")

SOURCES = ["kernels.hip", "tokenize.hip", "rollup.hip", "negotiate.hip", "dstore.hip", "api.cpp", "store.cpp",
           "dstore.cpp", "devenc.cpp", "upsert.cpp", "rollup.cpp", "negotiate.cpp", "encoder.cpp", "json.cpp",
           "buildid.cpp"]
SYNTH_SOURCES = ["synth.cpp", "encoder.cpp", "json.cpp", "buildid.cpp"]
HEADERS = ["kernels.h", "pool.h", "tokenize.h", "tokdev.h", "marshal_phases.inc", "rollup_phases.inc",
           "negotiate_phases.inc", "goscan.h", "rollup.h", "ryu_tables.h", "dstore.h", "decfloat.h", "pow10_128.h",
           "encoder.h", "engine.h", "json.h", "xxh64.h"]
MAPS = ["gpudiff.map", "synth.map"]
INCLUDE_NAMES = ["gpudiff.h", "gpudiff_format.h", "gpudiff_synth.h"]
INCLUDES = [os.path.join(ROOT, "include", h) for h in INCLUDE_NAMES]
BUILD_SCRIPTS = [os.path.join(HERE, "build.py"), os.path.join(HERE, "buildinfo.py")]


def input_files():
    """Every file whose content can change either library, as (name relative to the repo, path)."""
    names = sorted(set(SOURCES) | set(SYNTH_SOURCES) | set(HEADERS) | set(MAPS))
    paths = [os.path.join(CSRC, n) for n in names] + INCLUDES + BUILD_SCRIPTS
    return [(os.path.relpath(p, ROOT).replace(os.sep, "/"), p) for p in paths]


def source_id(root_override=None):
    """16 hex digits of SHA-256 over (relative name, NUL, length, content) of every input file, in name order.

    root_override: hash the same relative names under another tree (a test's edited copy)."""
    h = hashlib.sha256()
    for rel, path in sorted(input_files()):
        if root_override is not None:
            path = os.path.join(root_override, rel)
        with open(path, "rb") as f:
            data = f.read()
        h.update(rel.encode() + b"\0" + str(len(data)).encode() + b"\0")
        h.update(data)
    return h.hexdigest()[:16]


def sources_present(root_override=None):
    base = root_override if root_override is not None else ROOT
    return all(os.path.exists(os.path.join(base, rel)) for rel, _ in input_files())
