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


def header_prototypes():
    """name -> (return type, [parameter types]) for every function include/sbam.h declares."""
    src = open(os.path.join(ROOT, "include", "sbam.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    out = {}
    for m in re.finditer(r"([A-Za-z_][\w \*]*?)\b(sbam_[a-z_]+)\s*\(([^)]*)\)\s*;", src):
        params = [p.strip() for p in m.group(3).split(",") if p.strip() and p.strip() != "void"]
        out[m.group(2)] = (m.group(1).strip(), [re.sub(r"\s*\b\w+$", "", p) if not p.endswith("*") else p
                                                for p in params])
    return out


def _kind(c_type: str) -> str:
    t = c_type.replace("const", "").strip()
    if "*" in t:
        return "ptr"
    return {"int64_t": "i64", "int32_t": "i32", "int": "i32", "uint32_t": "i32", "double": "f64",
            "sbam_pos": "pos"}.get(t, t)


def _ctypes_kind(ct) -> str:
    import ctypes as C
    import sbam
    if ct in (C.c_void_p, C.c_char_p) or isinstance(ct, type(C.POINTER(C.c_int))):
        return "ptr"
    return {C.c_int64: "i64", C.c_int32: "i32", C.c_int: "i32", C.c_uint32: "i32", C.c_double: "f64",
            sbam._Pos: "pos"}.get(ct, repr(ct))


def test_ctypes_bindings_match_header_prototypes():
    """Every declared function's ctypes binding has the header's arity and argument widths (i64 / i32 / pointer /
    sbam_pos by value): a mismatch would pass wrong-width arguments silently through the C ABI."""
    import sbam
    L = sbam.load_library()
    protos = header_prototypes()
    assert sorted(protos) == header_functions()
    for name, (ret, params) in protos.items():
        fn = getattr(L, name)
        want = [_kind(p) for p in params]
        got = [_ctypes_kind(a) for a in (fn.argtypes or [])]
        assert got == want, (name, got, want)


def test_reserve_rejects_bad_arguments_host_only():
    """sbam_reserve checks its arguments before any device call: a null context or a negative size is
    SBAM_ERR_ARG (no GPU needed)."""
    import sbam
    L = sbam.load_library()
    assert L.sbam_reserve(None, 1 << 20, 16, 1 << 22, 0) == sbam.ERR_ARG
    assert L.sbam_reserve(None, -1, 0, 0, 0) == sbam.ERR_ARG


import pytest  # noqa: E402


@pytest.mark.gpu
def test_reserve_then_larger_window_gpu():
    """sbam_reserve sizes a context opened on a small file for a larger one; loading the larger file then gives
    the same blocks, checker calls and full-check counts as a fresh context, and a negative size raises."""
    import numpy as np
    import sbam
    from conftest import fixture_bytes
    a, b = fixture_bytes("1.bam"), fixture_bytes("2.bam")
    with sbam.BamFile(b) as fresh:
        want_blocks = [x.copy() for x in fresh.blocks()]
        want_calls = fresh.check_eager(0, fresh.uncompressed_size)
        nb, ub = int(fresh.n_blocks), int(fresh.uncompressed_size)
    with sbam.BamFile(a) as f:
        f.reserve(2 * len(b), 2 * nb, 2 * ub, 0)
        f.load(b)
        f.run()
        assert all(np.array_equal(x, y) for x, y in zip(f.blocks(), want_blocks))
        assert np.array_equal(f.check_eager(0, f.uncompressed_size), want_calls)
        with pytest.raises(sbam.SbamError):
            f.reserve(-1, 0, 0, 0)


@pytest.mark.gpu
def test_reserve_after_run_drops_stages_gpu():
    """sbam_reserve on a context that has already scanned, inflated and checked, growing its buffers,
    must not leave stale stage state over fresh (uninitialised) allocations: the C context drops its stages (a
    stream query is then SBAM_ERR_STATE) and the Python wrapper re-runs them, so the calls equal a fresh context's."""
    import numpy as np
    import sbam
    from conftest import fixture_bytes
    a = fixture_bytes("2.bam")
    with sbam.BamFile(a) as fresh:
        want_calls = fresh.check_eager(0, fresh.uncompressed_size)
        want_counts = fresh.check_full_counts(0, fresh.uncompressed_size)
        L_, nb = int(fresh.uncompressed_size), int(fresh.n_blocks)
    L = sbam.load_library()
    with sbam.BamFile(a) as f:
        f.check_full_counts(0, L_)
        # raw ABI: the grown context reports that inflate has to run again
        assert L.sbam_reserve(f.ctx, 8 * len(a), 8 * nb, 8 * L_, 0) == sbam.SBAM_OK
        assert L.sbam_read_uncompressed(f.ctx, 0, 0, None) == sbam.ERR_STATE
        f.n_blocks = f._scan()
        f.inflate()
        assert np.array_equal(f.check_eager(0, L_), want_calls)
        # the wrapper: reserve larger again, then query without re-running by hand
        f.reserve(16 * len(a), 16 * nb, 16 * L_, 1 << 16)
        assert f.uncompressed_size == L_
        c = f.check_full_counts(0, L_)
        assert np.array_equal(c.totals, want_counts.totals) and c.n_success == want_counts.n_success
        assert np.array_equal(f.check_eager(0, L_), want_calls)
        # nothing grows: the stages stay
        f.reserve(len(a), nb, L_, 0)
        assert L.sbam_read_uncompressed(f.ctx, 0, 0, None) == sbam.SBAM_OK


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


def test_struct_layout_matches_compiled_c(tmp_path):
    """sizeof/offsetof of the ABI structs as a C compiler lays out include/sbam.h, against the ctypes mirror and
    the offsets INTEGRATION.md's Panama binding reads (message @32, sizeof(sbam_error) = 544)."""
    import subprocess
    import sbam
    probe = tmp_path / "probe.c"
    fields = {
        "sbam_error": ["code", "idx", "actual", "expected", "position", "message"],
        "sbam_pos": ["block_pos", "offset", "reserved"],
        "sbam_split": ["start", "end"],
        "sbam_counts": ["totals", "counts", "positions", "reads_before_error", "pair_hist", "n_positions",
                        "n_success", "n_too_few_fixed", "n_halo"],
        "sbam_split_args": ["split_size", "bgzf_blocks_to_check", "reads_to_check", "max_read_size",
                            "use_success_bitmap"],
        "sbam_record_columns": list(sbam.RECORD_COLUMNS),
    }
    lines = ["#include <stdio.h>", "#include <stddef.h>", f'#include "{ROOT}/include/sbam.h"', "int main(void) {"]
    for t, fs in fields.items():
        lines.append(f'  printf("{t} sizeof %zu\\n", sizeof({t}));')
        for f in fs:
            lines.append(f'  printf("{t} {f} %zu\\n", offsetof({t}, {f}));')
    lines += ["  return 0;", "}"]
    probe.write_text("\n".join(lines))
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-o", str(exe), str(probe)], check=True)
    c = {}
    for ln in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.splitlines():
        t, f, v = ln.split()
        c[(t, f)] = int(v)
    mirror = {"sbam_error": sbam._Error, "sbam_pos": sbam._Pos, "sbam_split": sbam._Split,
              "sbam_counts": sbam._Counts, "sbam_split_args": sbam._SplitArgs,
              "sbam_record_columns": sbam._RecordColumns}
    for t, cls in mirror.items():
        assert c[(t, "sizeof")] == ctypes.sizeof(cls), t
        for f in fields[t]:
            assert c[(t, f)] == getattr(cls, f).offset, (t, f)
    assert c[("sbam_error", "message")] == 32 and c[("sbam_error", "sizeof")] == 544
    assert c[("sbam_error", "position")] == 24 and c[("sbam_error", "actual")] == 8
    assert c[("sbam_error", "expected")] == 16
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    assert "err.getString(32)" in text and "byteSize() == 544" in text


@pytest.mark.gpu
def test_error_messages_name_the_path():
    """HeaderSearchFailedException / NoReadFoundException messages as the reference formats them
    (HeaderSearchFailedException.scala:7-12, FindRecordStart.scala:66-71) with the path set by sbam_set_path, and
    the structured fields a JVM shim rebuilds them from."""
    import numpy as np
    import sbam
    from conftest import fixture_bytes
    # a shard whose first 65536 bytes hold no BGZF header: FindBlockStart(1000) fails
    with pytest.raises(sbam.HeaderSearchFailedException) as ei:
        sbam.BamFile(np.zeros(140000, np.uint8), base_offset=1000, file_size=141000, path="holes.bam")
    assert str(ei.value) == "holes.bam: failed to find BGZF header in 65536 bytes from 1000"
    # a Hadoop split starting past the last data block: FindBlockStart returns the EOF marker, the stream from
    # there is empty, FindRecordStart throws
    data = fixture_bytes("2.bam")
    L = len(data)
    with sbam.BamFile(data, path="test_bams/2.bam") as f:
        st = f.blocks()[0]
        last, eof = int(st[-1]), L - 28
        S = next(S for S in range(max(1, (eof - last) // 3), eof - last + 1)
                 if any(last < a <= eof for a, _ in sbam.hadoop_splits(L, S)))
        with pytest.raises(sbam.NoReadFoundException) as ei:
            f.compute_splits(S)
        e = f.L.sbam_last_error(f.ctx).contents
        assert e.code == sbam.ERR_NO_READ_FOUND and e.position == eof and e.expected == sbam.MAX_READ_SIZE
        assert str(ei.value) == f"Failed to find a valid read-start in {sbam.MAX_READ_SIZE} attempts in test_bams/2.bam from {eof}"


@pytest.mark.gpu
def test_concurrent_handles_match_serial():
    """§8(b) reentrancy: 4 threads × 4 handles (one per thread at a time, all on one GPU) give the serial results
    — no global mutable state, each handle its own stream and allocations."""
    import threading
    import numpy as np
    import sbam
    from conftest import fixture_bytes
    names = ["1.bam", "2.bam", "5k.bam", "1.2203053-2211029.bam"]
    want = {}
    for nm in names:
        with sbam.BamFile(fixture_bytes(nm), path=nm) as f:
            c = f.check_full_counts()
            want[nm] = (f.uncompressed_size, c.totals.copy(), c.n_success,
                        [str(s) for s in f.compute_splits(100000)], f.check_eager().copy())
    errors = []

    def worker(k):
        try:
            for j in range(4):
                nm = names[(k + j) % 4]
                with sbam.BamFile(fixture_bytes(nm), path=nm) as f:
                    c = f.check_full_counts()
                    got = (f.uncompressed_size, c.totals, c.n_success, [str(s) for s in f.compute_splits(100000)],
                           f.check_eager())
                    w = want[nm]
                    ok = got[0] == w[0] and np.array_equal(got[1], w[1]) and got[2] == w[2] and got[3] == w[3] \
                        and np.array_equal(got[4], w[4])
                    if not ok:
                        errors.append((k, nm))
        except Exception as e:  # noqa: BLE001
            errors.append((k, repr(e)))

    ts = [threading.Thread(target=worker, args=(k,)) for k in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["1.bam", "2.bam", "5k.bam"])
def test_block_table_before_inflate_gpu(name):
    """The fast scan leaves the block table's host copy in flight (pinned staging filled on a side stream; the host
    picks it up on its first read, or while inflate's kernels run).  Read straight after the scan, after a second
    scan whose predecessor's copy was never read, and for a shard whose first block is found by FindBlockStart, the
    table equals the oracle's, and the stream inflated afterwards has the oracle's length."""
    import numpy as np
    import oracle
    import sbam
    from conftest import fixture_bytes
    data = fixture_bytes(name)
    o = oracle.BamFile(data)
    want = (o.start, o.csize, o.usize, o.uoff[:-1])
    with sbam.BamFile(data, inflate=False) as f:
        assert all(np.array_equal(x, y) for x, y in zip(f.blocks(), want))
        f.reset()
        f.n_blocks = f._scan()
        f.n_blocks = f._scan()
        assert f.inflate() == o.L
        assert all(np.array_equal(x, y) for x, y in zip(f.blocks(), want))
    k0 = o.nblocks // 3
    lo = int(o.start[k0]) - 7  # inside the previous block: the shard starts at block k0
    with sbam.BamFile(data[lo:], base_offset=lo, file_size=len(data), inflate=False) as f:
        st, cs, us, uo = f.blocks()
        assert np.array_equal(st, o.start[k0:]) and np.array_equal(cs, o.csize[k0:])
        assert np.array_equal(us, o.usize[k0:]) and np.array_equal(uo, o.uoff[k0:-1] - o.uoff[k0])
        assert f.inflate() == o.L - int(o.uoff[k0])
