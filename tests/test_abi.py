"""CPU tests of the C-ABI library: it loads, and exports every symbol include/dbslmm_hip.h
declares.  No compute call is made without a GPU."""
import ctypes
import os
import re
import subprocess

import pytest

from _common import ROOT

HEADER = os.path.join(ROOT, "include", "dbslmm_hip.h")
LIB = os.path.join(ROOT, "dbslmm_amd", "libdbslmm_hip.so")


def declared_symbols():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|void|const char\*)\s+(dbslmm_\w+)\s*\(", src, re.M)))


def test_header_declares_entry_points():
    syms = declared_symbols()
    assert "dbslmm_est" in syms and "dbslmm_plan_run" in syms and len(syms) >= 14


def test_library_exports_every_declared_symbol():
    assert os.path.exists(LIB), "build first: __graft_entry__.build()"
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True,
                         check=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if l.strip()}
    missing = [s for s in declared_symbols() if s not in exported]
    assert not missing, missing


def test_python_binding_lists_all_exports():
    from dbslmm_amd import _lib
    assert sorted(_lib.EXPORTS) == declared_symbols()


def test_library_loads_and_reports_abi():
    from dbslmm_amd import _lib
    import re
    L = _lib.load()
    hdr = open(os.path.join(ROOT, "include", "dbslmm_hip.h")).read()
    ver = int(re.search(r"#define DBSLMM_ABI_VERSION (\d+)", hdr).group(1))
    assert L.dbslmm_abi_version() == ver == _lib.ABI_VERSION
    n = int(re.search(r"#define DBSLMM_WORKLOAD_LEN (\d+)", hdr).group(1))
    assert n == _lib.WORKLOAD_LEN
    assert len(_lib.KERNEL_NAMES) == int(re.search(r"DBSLMM_K_COUNT = (\d+)", hdr).group(1))


def test_kernels_are_gfx950_code_objects():
    """The fat binary carries a gfx950 code object (and no other target)."""
    data = open(LIB, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data
    for other in (b"--gfx942", b"--gfx90a", b"--gfx1100"):
        assert other not in data


def test_ctx_create_without_gpu_fails_cleanly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from dbslmm_amd import Context, DbslmmError
    with pytest.raises(DbslmmError):
        Context(0)


def test_multi_ctx_create_without_gpu_fails_cleanly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from dbslmm_amd import Context, DbslmmError
    with pytest.raises(DbslmmError):
        Context([0, 0])


def test_options_struct_matches_header():
    """The ctypes mirror of dbslmm_options / dbslmm_problem has the header's field order."""
    from dbslmm_amd import _lib
    src = open(HEADER).read()
    body = re.search(r"typedef struct dbslmm_options \{(.*?)\} dbslmm_options;", src, re.S).group(1)
    names = re.findall(r"(\w+);", body)
    assert names == [f[0] for f in _lib.Options._fields_]
    body = re.search(r"typedef struct dbslmm_problem \{(.*?)\} dbslmm_problem;", src, re.S).group(1)
    names = re.findall(r"(\w+);", body)
    assert names == [f[0] for f in _lib.Problem._fields_]


def test_no_null_stream_transfers_in_library():
    """Round-3 parity failure (config 3, first run of a fresh plan): plan_create zeroed the matrix
    buffer with a null-stream hipMemset, which returns before it completes and is not ordered
    against the context's non-blocking streams, so it zeroed Sigma entries the lead group's Gram
    had just written.  Every memset and host -> device copy of the library must be stream-ordered
    (hipMemsetAsync / hipMemcpyAsync on the stream its consumers run on or are forked from)."""
    import pathlib
    import re
    root = pathlib.Path(__file__).resolve().parents[1] / "dbslmm_amd" / "csrc"
    bad = []
    for f in sorted(root.glob("*.hip")):
        # comments out first (keeping the line count), then whole calls matched across line breaks:
        # the library wraps long calls, so a HostToDevice argument may sit on a continuation line
        text = re.sub(r"//[^\n]*", "", f.read_text())
        text = re.sub(r"/\*.*?\*/", lambda m: "\n" * m.group(0).count("\n"), text, flags=re.S)
        for m in re.finditer(r"\bhipMemset\s*\(|\bhipMemcpy\s*\([^;]*?HostToDevice[^;]*?\)\s*;", text, re.S):
            i = text.count("\n", 0, m.start()) + 1
            bad.append(f"{f.name}:{i}: {' '.join(m.group(0).split())}")
    assert not bad, "null-stream transfers:\n" + "\n".join(bad)


def test_null_stream_lint_sees_wrapped_calls(tmp_path):
    """The lint above matches a synchronous H2D copy whose direction sits on a continuation line."""
    import re
    text = "x = 1;\n    HIP_TRY(ctx, hipMemcpy(dst, src, n,\n                         hipMemcpyHostToDevice));\n"
    assert re.search(r"\bhipMemcpy\s*\([^;]*?HostToDevice[^;]*?\)\s*;", text, re.S)
