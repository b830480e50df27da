"""The C-ABI libraries load (no GPU needed) and export every function the
headers in include/ declare."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "dealii-ns-gls_amd", "lib")


def declared(header):
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(gls_[a-z0-9_]+)\s*\(", src)))


@pytest.mark.parametrize("header,lib", [("gls_op.h", "libglsamd.so"), ("gls_mesh.h", "libglsmesh.so")])
def test_exports(header, lib):
    path = os.path.join(LIB, lib)
    assert os.path.exists(path), f"{path} not built (make)"
    L = ctypes.CDLL(path)
    names = declared(header)
    assert len(names) > 5
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, f"{lib} does not export {missing}"


def test_python_export_list_matches_header():
    import glsamd
    assert sorted(glsamd.EXPORTS) == declared("gls_op.h")


def test_error_reporting_without_gpu():
    """Invalid descriptors are rejected with a message (status != 0) before
    any device call."""
    import glsamd
    L = glsamd.lib()
    d = glsamd.OpDesc(4, 2, 0, 1, 1, 1, None, None, None, None, None)  # dim 4 invalid
    h = ctypes.c_void_p()
    rc = L.gls_op_create(ctypes.byref(d), ctypes.byref(h))
    assert rc != 0
    assert b"invalid" in L.gls_last_error()
