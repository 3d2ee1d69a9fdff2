"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes access to the CPU checkers:
  * ``Oracle``    -> oracle/liborc.so, the plain-C restatement of the reference
                     kd-tree hot path (oracle/kdtree_oracle.c, see its header for
                     the reference file:line each function follows);
  * ``Reference`` -> oracle/_ref/libnbkd_ref.so, the reference's own C++ built from
                     /root/reference by oracle/Makefile (present only where it was
                     built; the built .so travels with the repo snapshot).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module.  The product (nbodyhpc_amd) never does.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORC_PATH = os.path.join(HERE, "liborc.so")
REF_PATH = os.path.join(HERE, "_ref", "libnbkd_ref.so")
VERTEX_REF_PATH = os.path.join(HERE, "_ref", "libvertex_ref.so")

NODE_DTYPE = np.dtype([("dim", "<i4"), ("split", "<f4"), ("left", "<u4"), ("right", "<u4")])

_fp = ctypes.POINTER(ctypes.c_float)
_up = ctypes.POINTER(ctypes.c_uint32)
_u64p = ctypes.POINTER(ctypes.c_uint64)


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def _ptr(a, t):
    return a.ctypes.data_as(t) if a is not None else None


def build_oracle(force: bool = False) -> str:
    """Compile liborc.so (and _ref when /root/reference exists)."""
    if force or not os.path.exists(ORC_PATH):
        subprocess.check_call(["make", "-s", "-C", HERE, "liborc.so"])
    return ORC_PATH


def build_reference(force: bool = False) -> str | None:
    if os.path.isdir("/root/reference/kdtree") and (force or not os.path.exists(REF_PATH)):
        subprocess.check_call(["make", "-s", "-C", HERE, "ref"])
    return REF_PATH if os.path.exists(REF_PATH) else None


class _Lib:
    prefix = ""

    def __init__(self, path):
        self.lib = ctypes.CDLL(path)
        p = self.prefix
        L = self.lib
        getattr(L, p + "build").argtypes = [_fp, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                                            ctypes.c_float, ctypes.POINTER(ctypes.c_void_p)]
        getattr(L, p + "build").restype = ctypes.c_int
        getattr(L, p + "free").argtypes = [ctypes.c_void_p]
        getattr(L, p + "n8").argtypes = [ctypes.c_void_p]
        getattr(L, p + "n8").restype = ctypes.c_int64
        getattr(L, p + "num_nodes").argtypes = [ctypes.c_void_p]
        getattr(L, p + "num_nodes").restype = ctypes.c_int64
        getattr(L, p + "export").argtypes = [ctypes.c_void_p, ctypes.c_void_p, _fp, _fp, _fp, _up]
        getattr(L, p + "knn").argtypes = [ctypes.c_void_p, _fp, ctypes.c_int64, ctypes.c_int32,
                                          ctypes.c_int32, ctypes.c_int32, _fp, _up, _u64p]
        getattr(L, p + "knn").restype = ctypes.c_int


class Tree:
    """Handle over one CPU tree (oracle or reference)."""

    def __init__(self, lib: _Lib, points, leafsize=128, boxsize=None):
        self._lib = lib
        self._p = lib.prefix
        pts = _f32(points)
        if pts.ndim != 2 or pts.shape[1] != 3:
            raise RuntimeError("positions must be a 2D array of shape (N, 3)")
        h = ctypes.c_void_p()
        periodic = boxsize is not None
        st = getattr(lib.lib, self._p + "build")(
            _ptr(pts, _fp), pts.shape[0], int(leafsize), 1 if periodic else 0,
            float(boxsize) if periodic else 0.0, ctypes.byref(h))
        if st == 2:
            raise RuntimeError("When using periodic boundary conditions, all points must be "
                               "within the box (0 <= x <= box_size).")
        if st != 0:
            raise RuntimeError(f"build failed with status {st}")
        self._h = h
        self.periodic = periodic
        self.boxsize = float(np.float32(boxsize)) if periodic else 0.0

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            getattr(self._lib.lib, self._p + "free")(h)
            self._h = None

    @property
    def n(self):
        return int(getattr(self._lib.lib, self._p + "n8")(self._h))

    @property
    def size(self):
        return int(getattr(self._lib.lib, self._p + "num_nodes")(self._h))

    def export(self):
        nodes = np.empty(self.size, dtype=NODE_DTYPE)
        n8 = self.n
        x, y, z = (np.empty(n8, np.float32) for _ in range(3))
        idx = np.empty(n8, np.uint32)
        getattr(self._lib.lib, self._p + "export")(
            self._h, nodes.ctypes.data_as(ctypes.c_void_p), _ptr(x, _fp), _ptr(y, _fp),
            _ptr(z, _fp), _ptr(idx, _up))
        return nodes, x, y, z, idx

    def query(self, q, k=1, workers=1, sqrt=True, stats=False):
        q = _f32(q)
        if k <= 0:
            raise RuntimeError("k must be positive integer")
        if q.ndim != 2 or q.shape[1] != 3:
            raise RuntimeError("positions must be a 2D array of shape (N, 3)")
        m = q.shape[0]
        d = np.empty((m, k), np.float32)
        i = np.empty((m, k), np.uint32)
        st = np.zeros(3, np.uint64)
        if workers <= 0:
            workers = os.cpu_count() or 1
        rc = getattr(self._lib.lib, self._p + "knn")(
            self._h, _ptr(q, _fp), m, int(k), int(workers), 1 if sqrt else 0, _ptr(d, _fp),
            _ptr(i, _up), _ptr(st, _u64p))
        if rc != 0:
            raise RuntimeError(f"knn failed with status {rc}")
        if stats:
            return d, i, {"nodes_visited": int(st[0]), "nodes_pruned": int(st[1]),
                          "points_visited": int(st[2])}
        return d, i


class Oracle(_Lib):
    prefix = "orc_"

    def __init__(self, path=None):
        super().__init__(path or build_oracle())
        L = self.lib
        L.orc_knn_brute.argtypes = [_fp, ctypes.c_int64, ctypes.c_int32, ctypes.c_float, _fp,
                                    ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, _fp, _up]
        L.orc_ball_count_brute.argtypes = [_fp, ctypes.c_int64, ctypes.c_int32, ctypes.c_float,
                                           _fp, ctypes.c_int64, ctypes.c_float, _up]
        L.orc_ball_count.argtypes = [ctypes.c_void_p, _fp, ctypes.c_int64, ctypes.c_float, _up]
        L.orc_ball_count_stats.argtypes = [ctypes.c_void_p, _fp, ctypes.c_int64, ctypes.c_float,
                                           _up, ctypes.POINTER(ctypes.c_uint64),
                                           ctypes.POINTER(ctypes.c_uint64)]
        L.orc_point_d2.argtypes = [_fp, _fp, ctypes.c_int32, ctypes.c_float]
        L.orc_point_d2.restype = ctypes.c_float
        L.orc_box_d2.argtypes = [_fp, _fp, ctypes.c_int32, ctypes.c_float]
        L.orc_box_d2.restype = ctypes.c_float
        L.orc_deposit.argtypes = [_fp, _fp, _fp, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                                  ctypes.c_int32, ctypes.c_float, _fp, ctypes.c_int32,
                                  ctypes.c_int32, ctypes.POINTER(ctypes.c_double)]
        L.orc_deposit.restype = ctypes.c_int
        L.orc_deposit_images.argtypes = [_fp, _fp, ctypes.c_int64, _fp, _fp,
                                         ctypes.POINTER(ctypes.c_int32)]

    def deposit_images(self, xyz, radius, period):
        """Periodic images of each ball as the restated rasteriser makes them:
        a list of (k_i, 3) float32 arrays."""
        p, r = _f32(xyz), _f32(radius)
        per = np.asarray(period, np.float32)
        n = p.shape[0]
        out = np.empty((n, 27, 3), np.float32)
        cnt = np.empty(n, np.int32)
        self.lib.orc_deposit_images(_ptr(p, _fp), _ptr(r, _fp), n, _ptr(per, _fp),
                                    _ptr(out, _fp), cnt.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
        return [out[i, :cnt[i]] for i in range(n)]

    def deposit(self, xyz, weight, radius, grid, ppu, period=(-1.0, -1.0, -1.0), subsample=4,
                mode=0):
        """Restated rasteriser (deposit_oracle.c): float64 grid of shape (gx, gy, nz),
        Fortran order, as the reference's render_points_volume returns it."""
        p, w, r = _f32(xyz), _f32(weight), _f32(radius)
        gx, gy, nz = (int(v) for v in grid)
        per = np.asarray(period, np.float32)
        out = np.zeros(gx * gy * nz, np.float64)
        st = self.lib.orc_deposit(_ptr(p, _fp), _ptr(w, _fp), _ptr(r, _fp), p.shape[0], gx, gy, nz,
                                  float(ppu), _ptr(per, _fp), int(subsample), int(mode),
                                  out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
        if st:
            raise ValueError("orc_deposit: bad arguments")
        return out.reshape((gx, gy, nz), order="F")

    def tree(self, points, leafsize=128, boxsize=None):
        return Tree(self, points, leafsize, boxsize)

    def knn_brute(self, points, q, k, boxsize=None, sqrt=True):
        p = _f32(points)
        q = _f32(q)
        m = q.shape[0]
        d = np.empty((m, k), np.float32)
        i = np.empty((m, k), np.uint32)
        self.lib.orc_knn_brute(_ptr(p, _fp), p.shape[0], 1 if boxsize is not None else 0,
                               float(boxsize or 0.0), _ptr(q, _fp), m, int(k), 1 if sqrt else 0,
                               _ptr(d, _fp), _ptr(i, _up))
        return d, i

    def ball_count_brute(self, points, q, r, boxsize=None):
        p = _f32(points)
        q = _f32(q)
        out = np.empty(q.shape[0], np.uint32)
        self.lib.orc_ball_count_brute(_ptr(p, _fp), p.shape[0], 1 if boxsize is not None else 0,
                                      float(boxsize or 0.0), _ptr(q, _fp), q.shape[0], float(r),
                                      _ptr(out, _up))
        return out

    def ball_count(self, tree: Tree, q, r):
        q = _f32(q)
        out = np.empty(q.shape[0], np.uint32)
        self.lib.orc_ball_count(tree._h, _ptr(q, _fp), q.shape[0], float(r), _ptr(out, _up))
        return out

    def ball_count_stats(self, tree: Tree, q, r):
        """(counts, nodes visited, points scanned) of the one-query DFS."""
        q = _f32(q)
        out = np.empty(q.shape[0], np.uint32)
        nn, npt = ctypes.c_uint64(), ctypes.c_uint64()
        self.lib.orc_ball_count_stats(tree._h, _ptr(q, _fp), q.shape[0], float(r),
                                      _ptr(out, _up), ctypes.byref(nn), ctypes.byref(npt))
        return out, int(nn.value), int(npt.value)

    def point_d2(self, q, p, boxsize=None):
        q = _f32(q)
        p = _f32(p)
        return self.lib.orc_point_d2(_ptr(q, _fp), _ptr(p, _fp), 1 if boxsize is not None else 0,
                                     float(boxsize or 0.0))

    def box_d2(self, q, box, boxsize=None):
        q = _f32(q)
        b = _f32(box)
        return self.lib.orc_box_d2(_ptr(q, _fp), _ptr(b, _fp), 1 if boxsize is not None else 0,
                                   float(boxsize or 0.0))


class Reference(_Lib):
    prefix = "ref_"

    def __init__(self, path=None):
        path = path or build_reference()
        if path is None:
            raise FileNotFoundError("oracle/_ref/libnbkd_ref.so not built (needs /root/reference)")
        super().__init__(path)

    def tree(self, points, leafsize=128, boxsize=None):
        return Tree(self, points, leafsize, boxsize)


class VertexReference:
    """The reference rasteriser's own augment_vertices_periodic
    (rasterization/src/cpp/vertex_utilities.cpp:13-42), compiled from its
    sources into oracle/_ref/libvertex_ref.so (oracle/Makefile `ref`)."""

    def __init__(self, path=None):
        path = path or VERTEX_REF_PATH
        if not os.path.exists(path):
            if os.path.isdir("/root/reference/rasterization"):
                subprocess.check_call(["make", "-s", "-C", HERE, "ref"])
            else:
                raise FileNotFoundError("oracle/_ref/libvertex_ref.so not built")
        self.lib = ctypes.CDLL(path)
        f = self.lib.ref_augment_vertices_periodic
        f.argtypes = [_fp, _fp, _fp, ctypes.c_int64, _fp, _fp, ctypes.c_int64]
        f.restype = ctypes.c_int64

    def augment(self, xyz, weight, radius, box):
        """(m, 5) float32 vertices (x, y, z, weight, radius) after augmentation,
        in the reference's order."""
        p, w, r = _f32(xyz), _f32(weight), _f32(radius)
        b = np.asarray(box, np.float32)
        n = p.shape[0]
        cap = 27 * n
        out = np.empty((cap, 5), np.float32)
        m = self.lib.ref_augment_vertices_periodic(_ptr(p, _fp), _ptr(w, _fp), _ptr(r, _fp), n,
                                                   _ptr(b, _fp), _ptr(out, _fp), cap)
        return out[:m]


def reference_available() -> bool:
    return os.path.exists(REF_PATH) or os.path.isdir("/root/reference/kdtree")
