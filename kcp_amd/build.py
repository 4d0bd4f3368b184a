"""In-tree build of libgpudiff.so (hipcc, gfx950) -- no JIT cache, the .so
travels to the GPU box with the repo snapshot.

Rebuilds are decided by content, not mtimes (a fresh checkout or a push can
reorder those): every object carries a stamp of its command line and the
contents of its source and of every header, and a library the stamps of its
objects.  The sources' content hash (kcp_amd/buildinfo.py) is compiled in as
gpudiff_build_id(), which the Python binding checks at load."""
import hashlib
import importlib.util
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
OUT = os.path.join(HERE, "_build")
LIB = os.path.join(HERE, "libgpudiff.so")
SYNTH_LIB = os.path.join(HERE, "libgpudiff_synth.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"


def _buildinfo():
    # by path: importing kcp_amd.buildinfo would run the package __init__, which loads the library
    spec = importlib.util.spec_from_file_location("_kcp_amd_buildinfo", os.path.join(HERE, "buildinfo.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


BI = _buildinfo()
CSRC = BI.CSRC
SOURCES, SYNTH_SOURCES, HEADERS, INCLUDES = BI.SOURCES, BI.SYNTH_SOURCES, BI.HEADERS, BI.INCLUDES
CFLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function", f"--offload-arch={ARCH}",
          "-I" + os.path.join(ROOT, "include")]
# kernels.hip: no wave-level atomic aggregation.  K2 takes its next item's ticket with one lane's
# atomicAdd as an item starts and reads it only at the item's end; the optimizer's broadcast of the
# returned value (readfirstlane + per-lane prefix) waited for the atomic's round trip right where it
# was issued -- a full, queue-loaded HBM latency at the start of every item.
# tokenize.hip: no promotion of private arrays to LDS.  LLVM moved the marshal mode's (K10) per-lane arrays into
# 5 KiB of LDS per one-wave workgroup, which halved K10's resident waves: 9.28 -> 6.45 ms per 131k bodies without it
# (profiles/r06h, interleaved A/B; K0 / K11 / K13 have no promoted arrays and are unchanged)
FILE_FLAGS = {"kernels.hip": ["-mllvm", "-amdgpu-atomic-optimizer-strategy=None"],
              "tokenize.hip": ["-mllvm", "-disable-promote-alloca-to-lds"]}


def _digest(parts, files):
    h = hashlib.sha256()
    for p in parts:
        h.update(p.encode() + b"\0")
    for f in files:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def _up_to_date(target, stamp):
    try:
        with open(target + ".stamp") as f:
            return os.path.exists(target) and f.read() == stamp
    except OSError:
        return False


def _write_stamp(target, stamp):
    with open(target + ".stamp", "w") as f:
        f.write(stamp)


def _compile(src, build_id, verbose):
    s = os.path.join(CSRC, src)
    o = os.path.join(OUT, src + ".o")
    cmd = [HIPCC] + CFLAGS + FILE_FLAGS.get(src, [])
    if src.endswith(".hip"):
        # zstd-compressed code objects: the fat binary shrinks ~8x (rocPRIM's radix sort alone carried 3.7 MB of
        # per-architecture dispatch stubs), so every push to a GPU box is smaller; unpacked once at load
        cmd += ["--offload-compress"]
    if src == "buildid.cpp":
        cmd += ['-DGPUDIFF_BUILD_ID="%s"' % build_id]
    cmd += ["-c", s, "-o", o]
    stamp = _digest(cmd, [s] + [os.path.join(CSRC, h) for h in HEADERS] + INCLUDES)
    if _up_to_date(o, stamp):
        return o, stamp
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("hipcc failed for %s:\n%s%s" % (src, r.stdout, r.stderr))
    _write_stamp(o, stamp)
    return o, stamp


def _link(lib, objs, mapfile, verbose):
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib] + [o for o, _ in objs] + [
        "-lpthread", "-Wl,--version-script=" + mapfile]
    stamp = _digest(cmd + [st for _, st in objs], [mapfile])
    if _up_to_date(lib, stamp):
        return
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("link failed:\n%s%s" % (r.stdout, r.stderr))
    _write_stamp(lib, stamp)


def build(verbose: bool = False) -> str:
    """Builds libgpudiff.so (the product) and libgpudiff_synth.so (bench /
    test workload generator); returns the library's path."""
    os.makedirs(OUT, exist_ok=True)
    build_id = BI.source_id()
    srcs = sorted(set(SOURCES) | set(SYNTH_SOURCES))
    with ThreadPoolExecutor(max_workers=5) as ex:
        objs = dict(zip(srcs, ex.map(lambda s: _compile(s, build_id, verbose), srcs)))
    _link(LIB, [objs[s] for s in SOURCES], os.path.join(CSRC, "gpudiff.map"), verbose)
    _link(SYNTH_LIB, [objs[s] for s in SYNTH_SOURCES], os.path.join(CSRC, "synth.map"), verbose)
    return LIB


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv))
