"""kcp_amd: MI355X-native batched reconciliation-diff engine for kcp's syncer.

The hot path (the syncer's change-detection predicates, sttts/kcp
pkg/syncer/specsyncer.go:17-41 and pkg/syncer/statussyncer.go:15-27) runs in
hand-written HIP kernels behind the C-ABI in include/gpudiff.h; this package
is the Python host side above that ABI.
"""
from . import gpudiff  # noqa: F401  (fails loudly if libgpudiff.so is missing)
from .gpudiff import Engine, DiffResult, GpuDiffError, resolve_path  # noqa: F401

__all__ = ["gpudiff", "Engine", "DiffResult", "GpuDiffError", "resolve_path"]
