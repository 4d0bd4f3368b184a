"""The C-ABI libraries load and export every function the headers declare
(no compute calls: these run without a GPU)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared(header):
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(gpudiff_[a-z0-9_]+)\s*\(", src)) -
                  {"gpudiff_seg_bytes", "gpudiff_meta", "gpudiff_meta_tag", "gpudiff_meta_len",
                   "gpudiff_meta_is_long", "gpudiff_meta_arena"})


@pytest.mark.parametrize("header,lib", [("gpudiff.h", "kcp_amd/libgpudiff.so"),
                                        ("gpudiff_synth.h", "kcp_amd/libgpudiff_synth.so")])
def test_exports(header, lib):
    names = declared(header)
    assert len(names) > 5
    so = ctypes.CDLL(os.path.join(ROOT, lib))
    missing = [n for n in names if not hasattr(so, n)]
    assert not missing, missing


def test_python_binding_covers_header():
    from kcp_amd import gpudiff as G
    bound = {n for n, _, _ in G.SIGNATURES}
    assert set(declared("gpudiff.h")) == bound


def test_host_only_context_refuses_device_work():
    from kcp_amd import gpudiff as G
    e = G.Engine(device=G.DEVICE_NONE)
    with pytest.raises(G.GpuDiffError) as ei:
        e.submit([(b"{}", b"{}")])
    assert ei.value.code == G.E_NODEVICE
    assert G.lib().gpudiff_abi_version() == G.ABI_VERSION == 6
    # pinned zero-copy buffers need a device; freeing a pointer the context never handed out is refused
    import ctypes as C
    p = C.c_void_p()
    assert G.lib().gpudiff_host_alloc(e.ctx, 4096, C.byref(p)) == G.E_NODEVICE and not p.value
    assert G.lib().gpudiff_host_alloc(e.ctx, 0, C.byref(p)) == G.E_INVAL
    buf = C.create_string_buffer(64)
    assert G.lib().gpudiff_host_free(e.ctx, C.cast(buf, C.c_void_p)) == G.E_INVAL
    e.close()


def test_binding_abi_matches_header():
    """The Python binding's ABI_VERSION is the header's, and its loader checks the library against it
    (gpudiff_write_plan_get kept its name while its default mode changed in ABI 4)."""
    from kcp_amd import gpudiff as G
    src = open(os.path.join(ROOT, "include", "gpudiff.h")).read()
    assert int(re.search(r"#define GPUDIFF_ABI_VERSION (\d+)", src).group(1)) == G.ABI_VERSION
    assert G.lib().gpudiff_abi_version() == G.ABI_VERSION
    import inspect
    assert "gpudiff_abi_version" in inspect.getsource(G._load)


def test_engine_refuses_the_null_stream():
    """stream=0 would silently give the engine its own non-blocking stream, which never orders against
    the caller's null-stream copies and collectives (the r04 gloo rehearsal read exports before they
    landed): refused."""
    from kcp_amd import gpudiff as G
    with pytest.raises(ValueError):
        G.Engine(device=G.DEVICE_NONE, stream=0)


def test_header_compiles_as_c():
    import subprocess
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        open(c, "w").write('#include "gpudiff.h"\n#include "gpudiff_synth.h"\nint main(void){return 0;}\n')
        r = subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), c, "-o",
                            os.path.join(d, "t")], capture_output=True, text=True)
        assert r.returncode == 0, r.stderr


def test_open_rejects_removed_tuning_bits():
    """ABI 5: the tuning bits of earlier rounds are gone; gpudiff_open refuses any bit outside
    GPUDIFF_OPT_KNOWN (timing, the K2 timeline hook, the arena test hook, device encode) instead of ignoring it."""
    from kcp_amd import gpudiff as G
    for bad in (0x2, 0x4, 0x8, 0x80, 0x100, 14 << 8, 3 << 16, 0x100000, 1 << 26, 1 << 28, 1 << 30):
        with pytest.raises(G.GpuDiffError) as ei:
            G.Engine(device=G.DEVICE_NONE, flags=bad)
        assert ei.value.code == G.E_INVAL, hex(bad)
    for ok in (0, G.OPT_TIMING, 12 << G.OPT_ARENA_SHIFT, G.OPT_DEVICE_ENCODE):
        G.Engine(device=G.DEVICE_NONE, flags=ok).close()


def test_build_id_equals_shipped_sources():
    """The loaded library's gpudiff_build_id() is the content hash of the sources beside it."""
    from kcp_amd import buildinfo, gpudiff as G
    from kcp_amd import synth as S
    assert G.BUILD_VERIFIED
    assert G.BUILD_ID == buildinfo.source_id() == G.lib().gpudiff_build_id().decode()
    assert S._lib.gpudiff_synth_build_id().decode() == G.BUILD_ID
    assert len(G.BUILD_ID) == 16 and int(G.BUILD_ID, 16) >= 0


def _copy_tree(dst):
    import shutil
    for d in ("kcp_amd", "include"):
        shutil.copytree(os.path.join(ROOT, d), os.path.join(dst, d),
                        ignore=shutil.ignore_patterns("_build", "__pycache__"))


def _import_in(tree):
    import subprocess
    import sys
    return subprocess.run([sys.executable, "-c", "import kcp_amd.gpudiff as G; print(G.BUILD_ID, G.BUILD_VERIFIED)"],
                          cwd=tree, capture_output=True, text=True, timeout=120)


def test_stale_library_is_refused(tmp_path):
    """A library pushed beside sources it was not built from is refused at import, whatever the mtimes say:
    a copy of the tree with one header's content changed (and its mtime set back before the library's)
    no longer loads; the untouched copy does."""
    _copy_tree(str(tmp_path))
    ok = _import_in(str(tmp_path))
    assert ok.returncode == 0, ok.stderr
    assert ok.stdout.split() == [__import__("kcp_amd").gpudiff.BUILD_ID, "True"]
    hdr = tmp_path / "kcp_amd" / "csrc" / "engine.h"
    hdr.write_text(hdr.read_text() + "\n// an edit the library was not built from\n")
    lib_m = os.path.getmtime(tmp_path / "kcp_amd" / "libgpudiff.so")
    os.utime(hdr, (lib_m - 3600, lib_m - 3600))
    bad = _import_in(str(tmp_path))
    assert bad.returncode != 0
    assert "built from other sources" in bad.stderr


def test_build_id_hashes_contents_not_mtimes(tmp_path):
    from kcp_amd import buildinfo
    _copy_tree(str(tmp_path))
    a = buildinfo.source_id(str(tmp_path))
    for rel, _ in buildinfo.input_files():
        os.utime(tmp_path / rel, (1, 1))
    assert buildinfo.source_id(str(tmp_path)) == a == buildinfo.source_id()
    f = tmp_path / "include" / "gpudiff_format.h"
    f.write_bytes(f.read_bytes() + b" ")
    assert buildinfo.source_id(str(tmp_path)) != a
