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


def test_deposit_arguments_rejected_before_any_device_call():
    """nbkd_deposit validates its arguments first (EINVAL with a message), so
    these fail the same way with or without a GPU."""
    xyz = np.zeros((4, 3), np.float32)
    w = np.ones(4, np.float32)
    cases = [
        (dict(grid=(0, 8, 8), ppu=1.0), "grid extents"),
        (dict(grid=(8, 8, 8), ppu=0.0), "pixels_per_unit"),
        (dict(grid=(8, 8, 8), ppu=float("nan")), "pixels_per_unit"),
        (dict(grid=(8, 8, 8), ppu=1.0, subsample=0), "subsample"),
        (dict(grid=(8, 8, 8), ppu=1.0, subsample=17), "subsample"),
        (dict(grid=(8, 8, 2), ppu=1.0, mode=1), "mode"),
        (dict(grid=(8, 8, 8), ppu=1.0, window=(6, 3)), "column window"),
        (dict(grid=(8, 8, 8), ppu=1.0, window=(0, 0)), "column window"),
    ]
    for kw, msg in cases:
        with pytest.raises(capi.NbkdError, match=msg) as e:
            capi.deposit(xyz, w, w, **kw)
        assert e.value.status == capi.NBKD_EINVAL
    L = capi.lib()
    assert L.nbkd_deposit(None, None, None, 4, 8, 8, 8, 1.0, None, 4, 0, 0, 8, None, -1, 0,
                          None) == capi.NBKD_EINVAL
    assert b"NULL" in L.nbkd_last_error()


def test_production_library_reads_no_environment():
    """Algorithm choices cannot change with the caller's environment: the
    production libnbkd.so imports no getenv (the A/B overrides exist only in
    the -DNBKD_EXPERIMENTS build, lib/exp/, loaded through NBKD_LIB)."""
    import subprocess

    out = subprocess.run(["nm", "-D", "--undefined-only", capi.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    assert "getenv" not in out


def test_tuning_knobs_validated():
    old = capi.get_tuning("knn_seed_margin")
    assert old > 0
    try:
        capi.set_tuning("knn_seed_margin", 2.0)
        assert capi.get_tuning("knn_seed_margin") == 2.0
        for bad in (0.0, -1.0, float("nan"), float("inf")):
            with pytest.raises(capi.NbkdError, match="out of range"):
                capi.set_tuning("knn_seed_margin", bad)
        with pytest.raises(capi.NbkdError, match="unknown knob"):
            capi.set_tuning("no_such_knob", 1.0)
        with pytest.raises(capi.NbkdError, match="out of range"):
            capi.set_tuning("candidate_bytes", -5.0)
    finally:
        capi.set_tuning("knn_seed_margin", old)


def test_row_and_forward_arguments_rejected():
    L = capi.lib()
    c = ctypes.c_uint64()
    assert L.nbkd_slab_forward(None, None, 5, 4, 0.0, 1.0, None, None, 0, ctypes.byref(c), 0,
                               None) == capi.NBKD_EINVAL
    assert L.nbkd_slab_forward(None, None, 0, 0, 0.0, 1.0, None, None, 0, ctypes.byref(c), 0,
                               None) == capi.NBKD_EINVAL
    assert L.nbkd_rows_gather(None, 6, None, 0, None, 0, None) == capi.NBKD_EINVAL  # 6 % 4 != 0
    assert L.nbkd_rows_scatter(None, 8, None, 3, None, 0, None) == capi.NBKD_EINVAL
    # zero rows: nothing to do, no device touched
    assert L.nbkd_rows_gather(None, 8, None, 0, None, 0, None) == capi.NBKD_OK


def test_type_stub_names_the_reference_surface():
    """_impl.pyi ships beside the extension (and beside the nbodyhpc.kdtree
    re-export) and declares every member of the reference's stub
    (kdtree/src/python/nbodyhpc/kdtree/_impl.pyi:1-18)."""
    import ast
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for rel in ("nbodyhpc_amd/kdtree/_impl.pyi", "nbodyhpc/kdtree/_impl.pyi"):
        tree = ast.parse(open(os.path.join(root, rel)).read())
        cls = [n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == "KDTree"][0]
        names = {f.name for f in cls.body if isinstance(f, ast.FunctionDef)}
        assert {"__init__", "query", "n", "size", "periodic", "boxsize"} <= names
        init = [f for f in cls.body if isinstance(f, ast.FunctionDef) and f.name == "__init__"][0]
        assert [a.arg for a in init.args.args][:5] == ["self", "points", "leafsize", "max_threads",
                                                       "boxsize"]


def test_build_ext_and_kth_out_arguments_rejected():
    """nbkd_build_ext checks its extents and nbkd_set_kth_out its tree before
    any device call; self_order is a 0 / 1 knob like the others."""
    L = capi.lib()
    h = ctypes.c_void_p()
    pts = np.zeros((16, 3), np.float32)
    for bad in ((0.0, 1.0, 1.0), (1.0, -1.0, 1.0), (1.0, 1.0, float("inf")),
                (float("nan"), 1.0, 1.0)):
        ext = (ctypes.c_float * 3)(*bad)
        assert L.nbkd_build_ext(pts.ctypes.data, 16, 16, 0, 0.0, ctypes.cast(ext, ctypes.c_void_p),
                                0, 0, None, ctypes.byref(h)) == capi.NBKD_EINVAL
        assert "extents must be positive" in L.nbkd_last_error().decode()
    assert L.nbkd_set_kth_out(None, None, 0) == capi.NBKD_EINVAL
    old = capi.get_tuning("self_order")
    assert old == 1.0
    try:
        capi.set_tuning("self_order", 0.0)
        assert capi.get_tuning("self_order") == 0.0
    finally:
        capi.set_tuning("self_order", old)


def test_reference_build_never_travels():
    """no reference source, object or bytecode travels to the GPU
    box.  oracle/_ref (the reference compiled here, the checker's checker) must
    stay listed in .gpurunignore (round 5 had dropped the entry)."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(root, ".gpurunignore")) as f:
        pats = {ln.strip() for ln in f if ln.strip() and not ln.startswith("#")}
    assert "./oracle/_ref" in pats
    # and the bench (which runs on the box) names nothing there; build() in
    # __graft_entry__.py compiles it in this container only
    with open(os.path.join(root, "bench.py")) as f:
        assert "oracle/_ref" not in f.read()
