"""The C-ABI library loads, exports every entry point include/dgl_hip.h
declares, and reports errors through DGLGetLastError (no GPU calls)."""
import ctypes
import os
import re

import pytest
import torch

import dgl
from dgl import _ffi
from dgl.base import DGLError

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                      "include", "dgl_hip.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    # type declarations are not entry points: struct typedefs, then the rest
    text = re.sub(r"typedef\s+(?:struct|union)[^{]*\{.*?\}\s*\w+\s*;", "", text, flags=re.S)
    text = re.sub(r"typedef[^;]*;", "", text, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[\w\*\s]+?\b(\w+)\s*\(", text, flags=re.M)
    return sorted(set(n for n in names if n not in ("if", "for", "while", "sizeof")))


def test_header_symbols_exported():
    lib = ctypes.CDLL(_ffi.lib_path())
    names = declared_functions()
    assert len(names) >= 50
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_version_and_build_info():
    assert _ffi.LIB.dglhip_abi_version() == 1
    assert b"gfx950" in _ffi.LIB.dglhip_build_info()


def test_error_convention():
    # out-of-range edge endpoint -> -1 and a message, raised as DGLError
    row = torch.tensor([0, 5], dtype=torch.int64)
    col = torch.tensor([1, 1], dtype=torch.int64)
    indptr = torch.empty(3, dtype=torch.int64)
    indices = torch.empty(2, dtype=torch.int32)
    eid = torch.empty(2, dtype=torch.int64)
    rc = _ffi.LIB.dglhip_coo_to_csr_host(2, 2, 2, _ffi.ptr(row), _ffi.ptr(col), 0,
                                          _ffi.ptr(indptr), _ffi.ptr(indices), _ffi.ptr(eid))
    assert rc == -1
    assert b"out of range" in _ffi.LIB.DGLGetLastError()
    with pytest.raises(DGLError):
        _ffi.check_call(rc)


def test_registry_names_and_unknown():
    names = dgl.list_global_func_names()
    for n in ("dglhip._CAPI_GSpMM", "dglhip._CAPI_GSDDMM", "dglhip._CAPI_COOToCSR",
              "dglhip._CAPI_RowsByDegree"):
        assert n in names
    with pytest.raises(DGLError):
        _ffi.call_packed("dglhip._CAPI_NoSuchThing")


def test_registry_call_host_csr_and_spmm():
    row = torch.tensor([2, 0, 2, 1], dtype=torch.int64)
    col = torch.tensor([0, 1, 1, 2], dtype=torch.int64)
    indptr = torch.empty(4, dtype=torch.int64)
    indices = torch.empty(4, dtype=torch.int32)
    eid = torch.empty(4, dtype=torch.int64)
    _ffi.call_packed("dglhip._CAPI_COOToCSR", 3, 3, row, col, 0, indptr, indices, eid)
    assert indptr.tolist() == [0, 1, 2, 4]
    assert indices.tolist() == [1, 2, 0, 1]
    assert eid.tolist() == [1, 3, 0, 2]
    h = torch.arange(6, dtype=torch.float32).reshape(3, 2)
    out = torch.empty(3, 2)
    _ffi.call_packed("dglhip._CAPI_GSpMM", 0, 0, indptr, indices, eid, h, None, out, None,
                     None, None)
    assert out.tolist() == [[2, 3], [4, 5], [2, 4]]
    with pytest.raises(DGLError):  # wrong dtype is rejected, not reinterpreted
        _ffi.call_packed("dglhip._CAPI_GSpMM", 0, 0, indptr, indices.long(), eid, h, None,
                         out, None, None, None)


def test_plain_c_client(tmp_path):
    """A plain-C program (tests/c_client/capi_demo.c) links libdgl_hip.so and
    drives the graph index through the registry, the host g-SpMM and the
    error convention."""
    import shutil
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no C compiler")
    libdir = os.path.dirname(_ffi.lib_path())
    exe = str(tmp_path / "capi_demo")
    subprocess.check_call([cc, "-std=c99", "-O1", "-Wall", "-Werror",
                           "-I", os.path.join(root, "include"),
                           os.path.join(root, "tests", "c_client", "capi_demo.c"),
                           "-o", exe, "-L", libdir, "-ldgl_hip", "-Wl,-rpath," + libdir])
    res = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert res.returncode == 0, (res.returncode, res.stdout, res.stderr)
    assert "capi_demo ok" in res.stdout
