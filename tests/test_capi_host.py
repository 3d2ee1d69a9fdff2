"""CPU tests of the boundary: the C-ABI library loads and exports every symbol
declared in include/nbkd.h; the pybind module imports; without a GPU every
entry point fails loudly (no silent CPU fallback); host-side validation
produces the reference's error messages."""
import ctypes
import os

import numpy as np
import pytest

from nbodyhpc_amd import capi


def test_library_exports_header_symbols():
    syms = capi.header_symbols()
    assert len(syms) >= 14
    L = ctypes.CDLL(capi.LIB_PATH)
    for s in syms:
        assert hasattr(L, s), f"{s} declared in include/nbkd.h but not exported"


def test_library_is_gfx950_code_object():
    data = open(capi.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_pybind_module_imports():
    from nbodyhpc import kdtree
    from nbodyhpc.kdtree import _impl
    assert kdtree.KDTree.__mro__[1] is _impl.KDTree
    assert _impl.__file__.startswith(os.path.dirname(capi.PKG))  # in-tree build


def test_shape_error_message():
    from nbodyhpc import kdtree
    with pytest.raises(RuntimeError, match=r"positions must be a 2D array of shape \(N, 3\)"):
        kdtree.KDTree(np.zeros((10, 2), np.float32))


@pytest.mark.skipif(capi.device_count() > 0, reason="only meaningful without a GPU")
def test_no_gpu_fails_loudly():
    from nbodyhpc import kdtree
    with pytest.raises(RuntimeError, match="requires a GPU"):
        kdtree.KDTree(np.zeros((10, 3), np.float32))
    with pytest.raises(capi.NbkdError):
        capi.Tree(np.zeros((10, 3), np.float32))


def test_null_arguments_rejected():
    L = capi.lib()
    h = ctypes.c_void_p()
    assert L.nbkd_build(None, 10, 16, 0, 0.0, 0, 0, None, ctypes.byref(h)) == capi.NBKD_EINVAL
    assert L.nbkd_query_knn(None, None, 0, 1, None, None, 0, None) == capi.NBKD_EINVAL
    assert b"NULL" in L.nbkd_last_error()
    n8 = ctypes.c_uint64()
    assert L.nbkd_tree_info(None, ctypes.byref(n8), None, None, None, None) == capi.NBKD_EINVAL


def test_timing_api_roundtrip():
    capi.timing_enable(True)
    capi.timing_reset()
    assert capi.timing_read("knn") == (0.0, 0)
    capi.timing_enable(False)
