"""In-tree build of libgpudiff.so (hipcc, gfx950) -- no JIT cache, the .so
travels to the GPU box with the repo snapshot."""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "_build")
LIB = os.path.join(HERE, "libgpudiff.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

SOURCES = ["kernels.hip", "tokenize.hip", "rollup.hip", "negotiate.hip", "dstore.hip", "api.cpp", "store.cpp", "dstore.cpp", "devenc.cpp", "upsert.cpp", "rollup.cpp", "negotiate.cpp",
           "encoder.cpp", "json.cpp"]
SYNTH_SOURCES = ["synth.cpp", "encoder.cpp", "json.cpp"]
SYNTH_LIB = os.path.join(HERE, "libgpudiff_synth.so")
HEADERS = ["kernels.h", "pool.h", "tokenize.h", "tokdev.h", "marshal_phases.inc", "rollup_phases.inc", "negotiate_phases.inc", "goscan.h", "rollup.h", "ryu_tables.h", "dstore.h", "decfloat.h", "pow10_128.h", "encoder.h", "engine.h", "json.h", "xxh64.h"]
INCLUDES = [os.path.join(ROOT, "include", h) for h in ("gpudiff.h", "gpudiff_format.h", "gpudiff_synth.h")]
CFLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function", f"--offload-arch={ARCH}",
          "-I" + os.path.join(ROOT, "include")]
# kernels.hip: no wave-level atomic aggregation.  K2 takes its next item's ticket with one lane's
# atomicAdd as an item starts and reads it only at the item's end; the optimizer's broadcast of the
# returned value (readfirstlane + per-lane prefix) waited for the atomic's round trip right where it
# was issued -- a full, queue-loaded HBM latency at the start of every item.
FILE_FLAGS = {"kernels.hip": ["-mllvm", "-amdgpu-atomic-optimizer-strategy=None"]}


def _newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _compile(src, verbose):
    s = os.path.join(CSRC, src)
    o = os.path.join(OUT, src + ".o")
    deps = [s, os.path.abspath(__file__)] + [os.path.join(CSRC, h) for h in HEADERS] + INCLUDES
    if not _newer(o, deps):
        return o
    cmd = [HIPCC] + CFLAGS + FILE_FLAGS.get(src, []) + ["-c", s, "-o", o]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("hipcc failed for %s:\n%s%s" % (src, r.stdout, r.stderr))
    return o


def _link(lib, objs, mapfile, verbose):
    if not _newer(lib, objs + [mapfile]):
        return
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib] + objs + [
        "-lpthread", "-Wl,--version-script=" + mapfile]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("link failed:\n%s%s" % (r.stdout, r.stderr))


def build(verbose: bool = False) -> str:
    """Builds libgpudiff.so (the product) and libgpudiff_synth.so (bench /
    test workload generator)."""
    os.makedirs(OUT, exist_ok=True)
    srcs = sorted(set(SOURCES) | set(SYNTH_SOURCES))
    with ThreadPoolExecutor(max_workers=5) as ex:
        objs = dict(zip(srcs, ex.map(lambda s: _compile(s, verbose), srcs)))
    _link(LIB, [objs[s] for s in SOURCES], os.path.join(CSRC, "gpudiff.map"), verbose)
    _link(SYNTH_LIB, [objs[s] for s in SYNTH_SOURCES], os.path.join(CSRC, "synth.map"), verbose)
    return LIB


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv))
