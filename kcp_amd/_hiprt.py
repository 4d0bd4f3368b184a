"""One HIP runtime per process.

PyTorch-ROCm ships its own libamdhip64 / libhsa-runtime64 (torch/lib) and
loads them by file name; libgpudiff.so needs the soname libamdhip64.so.7.  If
libgpudiff.so is loaded first, the dynamic loader resolves it to /opt/rocm's
runtime and torch later maps a second copy of its own: two HSA runtimes then
compete for the GPU (one of them sees no device).  Loading torch's runtime
file first, globally, makes both resolve to that single copy (glibc reuses an
already-mapped file and matches the soname).  Without torch installed the
library keeps /opt/rocm's runtime."""
import ctypes
import importlib.util
import os

_done = False


def preload() -> None:
    global _done
    if _done:
        return
    _done = True
    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.submodule_search_locations:
        return
    lib = os.path.join(list(spec.submodule_search_locations)[0], "lib")
    for name in ("libhsa-runtime64.so", "libamdhip64.so"):
        path = os.path.join(lib, name)
        if os.path.exists(path):
            ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
