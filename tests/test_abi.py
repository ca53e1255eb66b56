"""libsbam.so loads (no GPU needed) and exports every symbol include/sbam.h declares; host-only entry
points (no device work) behave like the reference's split rule."""
import ctypes
import os
import re

from conftest import ROOT


def header_functions():
    src = open(os.path.join(ROOT, "include", "sbam.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(sbam_[a-z_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    import sbam
    L = sbam.load_library()
    declared = header_functions()
    assert declared, "no declarations parsed"
    missing = [f for f in declared if not hasattr(L, f)]
    assert not missing, missing
    assert sorted(sbam.EXPORTS) == declared


def test_version_and_file_splits_host_only():
    import sbam
    L = sbam.load_library()
    assert b"gfx950" in L.sbam_version()
    assert sbam.hadoop_splits(597482, 230 * 1024) == [(0, 235520), (235520, 471040), (471040, 597482)]


def test_no_cpu_fallback(tmp_path):
    """The product path raises when the HIP library is missing (no silent fallback)."""
    import importlib
    import pytest
    import sbam
    with pytest.raises(ImportError):
        sbam._lib, saved = None, sbam._lib
        try:
            sbam.load_library(str(tmp_path / "missing.so"))
        finally:
            sbam._lib = saved


def test_library_is_gfx950_code_object():
    so = os.path.join(ROOT, "spark-bam_amd", "build", "libsbam.so")
    data = open(so, "rb").read()
    assert b"gfx950" in data


def test_load_replaces_window_on_gpu_marker():
    """(CPU) sbam_load is declared and bound like sbam_open (GPU behaviour: test_load_window_gpu)."""
    import sbam
    assert "sbam_load" in sbam.EXPORTS


import pytest  # noqa: E402


@pytest.mark.gpu
def test_load_window_gpu():
    """sbam_load: a context re-filled with another file (and back) gives the same blocks, stream and checker
    calls as a fresh sbam_open of that file, with its allocations reused."""
    import numpy as np
    import sbam
    from conftest import fixture_bytes
    a, b = fixture_bytes("1.bam"), fixture_bytes("2.bam")
    with sbam.BamFile(b) as fresh:
        want_blocks = [x.copy() for x in fresh.blocks()]
        want_calls = fresh.check_eager(0, fresh.uncompressed_size)
    with sbam.BamFile(a) as f:
        for _ in range(2):
            f.load(b)
            f.run()
            assert all(np.array_equal(x, y) for x, y in zip(f.blocks(), want_blocks))
            assert np.array_equal(f.check_eager(0, f.uncompressed_size), want_calls)
            f.load(a)
            f.run()
            assert f.blocks()[0].size == 25 and int(f.check_eager(0, f.uncompressed_size).sum()) == 4917
