"""ctypes binding of the C ABI (include/nbkd.h) — the binding a ctypes caller
of the reference's hot path would add.  Loads the in-tree
nbodyhpc_amd/lib/libnbkd.so and raises if it is missing: there is no fallback.
"""
from __future__ import annotations

import ctypes
import os
import re

import numpy as np

PKG = os.path.dirname(os.path.abspath(__file__))
# NBKD_LIB: an alternative build of the library (A/B experiments)
LIB_PATH = os.environ.get("NBKD_LIB") or os.path.join(PKG, "lib", "libnbkd.so")
HEADER = os.path.join(os.path.dirname(PKG), "include", "nbkd.h")

NBKD_OK, NBKD_EINVAL, NBKD_EBOX, NBKD_ETOOMANY, NBKD_ENOMEM, NBKD_EDEVICE, NBKD_EINTR = range(7)
NBKD_INPUT_DEVICE = 0x1
NBKD_OUTPUT_DEVICE = 0x2
NBKD_ACCUMULATE = 0x4
NBKD_SQUARED = 0x8
NBKD_SORTED = 0x10

NODE_DTYPE = np.dtype([("dim", "<i4"), ("split", "<f4"), ("left", "<u4"), ("right", "<u4")])


class NbkdError(RuntimeError):
    def __init__(self, status, msg):
        super().__init__(msg)
        self.status = status


_c_p = ctypes.c_void_p
_u64 = ctypes.c_uint64
_i32 = ctypes.c_int32
_u32 = ctypes.c_uint32

_PROTOS = {
    "nbkd_build": (_i32, [_c_p, _u64, _i32, _i32, ctypes.c_float, _i32, _u32, _c_p,
                          ctypes.POINTER(_c_p)]),
    "nbkd_set_kth_out": (_i32, [_c_p, _c_p, _u64]),
    "nbkd_build_ext": (_i32, [_c_p, _u64, _i32, _i32, ctypes.c_float, _c_p, _i32, _u32, _c_p,
                              ctypes.POINTER(_c_p)]),
    "nbkd_query_knn": (_i32, [_c_p, _c_p, _u64, _i32, _c_p, _c_p, _u32, _c_p]),
    "nbkd_query_kth": (_i32, [_c_p, _c_p, _u64, _i32, _c_p, _u32, _c_p]),
    "nbkd_query_ball_count": (_i32, [_c_p, _c_p, _u64, ctypes.c_float, _c_p, _u32, _c_p]),
    "nbkd_query_ball_csr": (_i32, [_c_p, _c_p, _u64, ctypes.c_float, _c_p, _c_p, _u64, _u32,
                                   _c_p]),
    "nbkd_tree_info": (_i32, [_c_p, ctypes.POINTER(_u64), ctypes.POINTER(_u64),
                              ctypes.POINTER(_i32), ctypes.POINTER(ctypes.c_float),
                              ctypes.POINTER(_i32)]),
    "nbkd_export": (_i32, [_c_p, _c_p, _c_p, _c_p, _c_p, _c_p]),
    "nbkd_free": (None, [_c_p]),
    "nbkd_last_error": (ctypes.c_char_p, []),
    "nbkd_device_count": (_i32, [ctypes.POINTER(_i32)]),
    "nbkd_timing_enable": (_i32, [_i32]),
    "nbkd_timing_reset": (_i32, []),
    "nbkd_timing_read": (_i32, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_double),
                                ctypes.POINTER(_u64)]),
    "nbkd_stats_enable": (_i32, [_i32]),
    "nbkd_stats_read": (_i32, [ctypes.POINTER(_u64), ctypes.POINTER(_u64)]),
    "nbkd_stats_read_all": (_i32, [ctypes.POINTER(_u64), _i32]),
    "nbkd_set_ids": (_i32, [_c_p, _c_p, _u32, _c_p]),
    "nbkd_slab_select": (_i32, [_c_p, _c_p, _u64, ctypes.c_float, ctypes.c_float, _c_p, _c_p,
                                _u64, ctypes.POINTER(_u64), _i32, _c_p]),
    "nbkd_slab_violations": (_i32, [_c_p, _c_p, _u64, _i32, ctypes.c_float, ctypes.c_float,
                                    ctypes.c_float, ctypes.POINTER(_u64), _i32, _c_p]),
    "nbkd_slab_forward": (_i32, [_c_p, _c_p, _u64, _i32, ctypes.c_float, ctypes.c_float, _c_p,
                                 _c_p, _u64, ctypes.POINTER(_u64), _i32, _c_p]),
    "nbkd_slab_forward_async": (_i32, [_c_p, _c_p, _u64, _i32, ctypes.c_float, ctypes.c_float,
                                       _c_p, _c_p, _u64, _c_p, _i32, _c_p]),
    "nbkd_rows_gather": (_i32, [_c_p, _u64, _c_p, _u64, _c_p, _i32, _c_p]),
    "nbkd_rows_scatter": (_i32, [_c_p, _u64, _c_p, _u64, _c_p, _i32, _c_p]),
    "nbkd_set_tuning": (_i32, [ctypes.c_char_p, ctypes.c_double]),
    "nbkd_set_interrupt": (_i32, [_c_p, _c_p]),
    "nbkd_get_tuning": (_i32, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_double)]),
    "nbkd_comm_probe": (_i32, []),
    "nbkd_comm_unique_id": (_i32, [_c_p]),
    "nbkd_comm_init": (_i32, [_c_p, _i32, _i32, _i32, ctypes.POINTER(_c_p)]),
    "nbkd_comm_exchange": (_i32, [_c_p, _i32, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p]),
    "nbkd_comm_free": (None, [_c_p]),
    "nbkd_deposit": (_i32, [_c_p, _c_p, _c_p, _u64, _i32, _i32, _i32, ctypes.c_float, _c_p, _i32,
                            _i32, _i32, _i32, _c_p, _i32, _u32, _c_p]),
}
COMM_ID_BYTES = 128


def header_symbols() -> list[str]:
    """Function names declared in include/nbkd.h."""
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(nbkd_[a-z_]+)\s*\(", txt)))


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not built: run `python -m nbodyhpc_amd.build`")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _PROTOS.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _check(st):
    if st != NBKD_OK:
        raise NbkdError(st, lib().nbkd_last_error().decode())


def device_count() -> int:
    c = _i32(0)
    _check(lib().nbkd_device_count(ctypes.byref(c)))
    return c.value


def _host_f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


class Tree:
    """Owning handle over an nbkd_tree*.  Inputs are numpy arrays (host) or raw
    device pointers (int) with `device_ptrs=True`."""

    def __init__(self, points=None, leafsize=128, boxsize=None, device=-1, *, n=None,
                 dev_ptr=None, stream=None, extent=None):
        L = lib()
        h = _c_p()
        flags = 0
        if dev_ptr is not None:
            ptr, count, flags = dev_ptr, n, NBKD_INPUT_DEVICE
        else:
            pts = _host_f32(points)
            if pts.ndim != 2 or pts.shape[1] != 3:
                raise RuntimeError("positions must be a 2D array of shape (N, 3)")
            ptr, count = pts.ctypes.data, pts.shape[0]
            self._keep = pts
        periodic = boxsize is not None
        # extent (ex, ey, ez): nbkd_build_ext, split axes by the points' extent
        # (slab trees); None: the reference's depth % 3
        ext = None if extent is None else (ctypes.c_float * 3)(*[float(e) for e in extent])
        ext = None if ext is None else ctypes.cast(ext, ctypes.c_void_p)
        st = L.nbkd_build_ext(ptr, count, int(leafsize), 1 if periodic else 0,
                              float(boxsize) if periodic else 0.0, ext, int(device), flags,
                              stream, ctypes.byref(h))
        _check(st)
        self.h = h
        self._keep = None
        n8, nn, per, box, dev = _u64(), _u64(), _i32(), ctypes.c_float(), _i32()
        _check(L.nbkd_tree_info(h, ctypes.byref(n8), ctypes.byref(nn), ctypes.byref(per),
                                ctypes.byref(box), ctypes.byref(dev)))
        self.n, self.size = n8.value, nn.value
        self.periodic, self.boxsize, self.device = bool(per.value), box.value, dev.value

    def close(self):
        if getattr(self, "h", None):
            lib().nbkd_free(self.h)
            self.h = None

    __del__ = close

    def export(self):
        nodes = np.empty(self.size, NODE_DTYPE)
        x, y, z = (np.empty(self.n, np.float32) for _ in range(3))
        idx = np.empty(self.n, np.uint32)
        _check(lib().nbkd_export(self.h, nodes.ctypes.data, x.ctypes.data, y.ctypes.data,
                                 z.ctypes.data, idx.ctypes.data))
        return nodes, x, y, z, idx

    def query(self, q, k, squared=False):
        """(m, k) distances and ids; squared=True: d2 instead of sqrtf(d2)."""
        q = _host_f32(q).reshape(-1, 3)
        m = q.shape[0]
        d = np.empty((m, k), np.float32)
        i = np.empty((m, k), np.uint32)
        _check(lib().nbkd_query_knn(self.h, q.ctypes.data, m, int(k), d.ctypes.data,
                                    i.ctypes.data, NBKD_SQUARED if squared else 0, None))
        return d, i

    def query_device(self, q_ptr, m, k, d_ptr, i_ptr, stream=None, input_device=True,
                     squared=False):
        flags = (NBKD_OUTPUT_DEVICE | (NBKD_INPUT_DEVICE if input_device else 0)
                 | (NBKD_SQUARED if squared else 0))
        _check(lib().nbkd_query_knn(self.h, q_ptr, int(m), int(k), d_ptr, i_ptr, flags, stream))

    def query_kth(self, q, k):
        """Distance to the k-th neighbour (column k-1 of query()), float32 (m,)."""
        q = _host_f32(q)
        out = np.empty(q.shape[0], np.float32)
        _check(lib().nbkd_query_kth(self.h, q.ctypes.data, q.shape[0], int(k), out.ctypes.data, 0,
                                    None))
        return out

    def query_kth_device(self, q_ptr, m, k, d_ptr, stream=None, input_device=True):
        flags = NBKD_OUTPUT_DEVICE | (NBKD_INPUT_DEVICE if input_device else 0)
        _check(lib().nbkd_query_kth(self.h, q_ptr, int(m), int(k), d_ptr, flags, stream))

    def set_kth_out(self, dev_ptr=None, capacity=0):
        """nbkd_set_kth_out: self queries with device rows also write each row's
        k-th distance to dev_ptr[row] (None detaches)."""
        _check(lib().nbkd_set_kth_out(self.h, dev_ptr, int(capacity) if dev_ptr else 0))

    def set_ids(self, ids=None, *, dev_ptr=None, stream=None):
        """Map the tree's point ids through `ids` (host array or device pointer)."""
        if dev_ptr is not None:
            _check(lib().nbkd_set_ids(self.h, dev_ptr, NBKD_INPUT_DEVICE, stream))
        else:
            a = np.ascontiguousarray(ids, dtype=np.uint32)
            _check(lib().nbkd_set_ids(self.h, a.ctypes.data, 0, stream))

    def ball_count(self, q, r):
        q = _host_f32(q)
        out = np.empty(q.shape[0], np.uint32)
        _check(lib().nbkd_query_ball_count(self.h, q.ctypes.data, q.shape[0], float(r),
                                           out.ctypes.data, 0, None))
        return out

    def ball_count_device(self, q_ptr, m, r, out_ptr, stream=None):
        _check(lib().nbkd_query_ball_count(self.h, q_ptr, int(m), float(r), out_ptr,
                                           NBKD_INPUT_DEVICE | NBKD_OUTPUT_DEVICE, stream))

    def ball_csr(self, q, r, sorted=False):
        """CSR radius query of host queries: (offsets (m + 1,) uint64, ids);
        sorted=True: each row ascending (NBKD_SORTED, sorted on the device)."""
        q = _host_f32(q)
        m = q.shape[0]
        fl = NBKD_SORTED if sorted else 0
        off = np.empty(m + 1, np.uint64)
        _check(lib().nbkd_query_ball_csr(self.h, q.ctypes.data, m, float(r), off.ctypes.data,
                                         None, 0, fl, None))
        idx = np.empty(int(off[-1]), np.uint32)
        _check(lib().nbkd_query_ball_csr(self.h, q.ctypes.data, m, float(r), off.ctypes.data,
                                         idx.ctypes.data if idx.size else None, idx.size, fl,
                                         None))
        return off, idx

    def ball_csr_device(self, q_ptr, m, r, off, idx_ptr, capacity, sorted=False, stream=None):
        """Device queries and device ids (offsets in host memory `off`,
        (m + 1,) uint64); idx_ptr None: the counts pass only."""
        fl = NBKD_INPUT_DEVICE | NBKD_OUTPUT_DEVICE | (NBKD_SORTED if sorted else 0)
        _check(lib().nbkd_query_ball_csr(self.h, q_ptr, int(m), float(r), off.ctypes.data,
                                         idx_ptr, int(capacity), fl, stream))
        return off


def deposit(xyz, weight, radius, grid, ppu, period=(-1.0, -1.0, -1.0), subsample=4, mode=0,
            device=-1, out=None, window=None):
    """Host arrays in, float32 grid (gx, gy, nz) in Fortran order out (nbkd_deposit).
    `window` = (x0, wx): only columns [x0, x0 + wx) of the gx-wide grid, shape
    (wx, gy, nz).  `out` (that shape, Fortran-contiguous float32): accumulate into it."""
    p, w, r = _host_f32(xyz), _host_f32(weight), _host_f32(radius)
    gx, gy, nz = (int(v) for v in grid)
    x0, wx = (0, gx) if window is None else (int(window[0]), int(window[1]))
    per = np.ascontiguousarray(period, np.float32)
    flags = 0
    if out is None:
        out = np.empty((wx, gy, nz), np.float32, order="F")
    else:
        if out.dtype != np.float32 or out.shape != (wx, gy, nz) or not out.flags.f_contiguous:
            raise ValueError("out must be a Fortran-ordered float32 array of the grid's shape")
        flags |= NBKD_ACCUMULATE
    _check(lib().nbkd_deposit(p.ctypes.data, w.ctypes.data, r.ctypes.data, p.shape[0], gx, gy, nz,
                              float(ppu), per.ctypes.data, int(subsample), int(mode), x0, wx,
                              out.ctypes.data, int(device), flags, None))
    return out


def deposit_device(xyz_ptr, weight_ptr, radius_ptr, n, grid, ppu, out_ptr,
                   period=(-1.0, -1.0, -1.0), subsample=4, mode=0, device=-1, accumulate=False,
                   stream=None, window=None):
    """Device pointers in and out; returns once the deposit is enqueued."""
    gx, gy, nz = (int(v) for v in grid)
    x0, wx = (0, gx) if window is None else (int(window[0]), int(window[1]))
    per = np.ascontiguousarray(period, np.float32)
    flags = NBKD_INPUT_DEVICE | NBKD_OUTPUT_DEVICE | (NBKD_ACCUMULATE if accumulate else 0)
    _check(lib().nbkd_deposit(xyz_ptr, weight_ptr, radius_ptr, int(n), gx, gy, nz, float(ppu),
                              per.ctypes.data, int(subsample), int(mode), x0, wx, out_ptr,
                              int(device), flags, stream))


def set_tuning(name, value):
    """nbkd_set_tuning: "knn_seed_margin" (default 3.5), "candidate_bytes" (0 = auto)."""
    _check(lib().nbkd_set_tuning(name.encode(), float(value)))


def get_tuning(name):
    v = ctypes.c_double()
    _check(lib().nbkd_get_tuning(name.encode(), ctypes.byref(v)))
    return v.value


def timing_enable(on=True):
    _check(lib().nbkd_timing_enable(1 if on else 0))


def timing_reset():
    _check(lib().nbkd_timing_reset())


def timing_read(name):
    ms, cnt = ctypes.c_double(), _u64()
    _check(lib().nbkd_timing_read(name.encode(), ctypes.byref(ms), ctypes.byref(cnt)))
    return ms.value, cnt.value


def stats_enable(on=True):
    _check(lib().nbkd_stats_enable(1 if on else 0))


def stats_read():
    a, b = _u64(), _u64()
    _check(lib().nbkd_stats_read(ctypes.byref(a), ctypes.byref(b)))
    return a.value, b.value


# work counters of the last kNN call (collect kernel, knn_collect.hip): nodes
# entered x packet lanes, (query, point) distance evaluations, dense point steps,
# sparse (lane-compacted) iterations, leaf points staged, packets (waves),
# candidates appended, leaves scanned, queries sent to the exact kernel,
# queries retried with a larger seed ball; then the collect kernel's phase
# clocks (shader cycles summed over waves): tree walk, leaf staging wait, leaf
# need test, dense scan, sparse scan, bound update; lanes needing a staged
# chunk, summed over chunks
STATS_NAMES = ("node_visits", "pair_evals", "leaves_reached", "sparse_iters", "points_staged",
               "packets", "candidates", "leaves_scanned", "fallback_queries", "retry_queries",
               "clk_walk", "clk_wait", "clk_leaf_test", "clk_dense", "clk_sparse", "clk_tighten",
               "chunk_lanes")


# the same slots after a radius count with stats enabled (ball.hip STATS instance)
BALL_STATS_NAMES = ("node_visits", "points_evaluated", "leaves_needed", "transposed_steps",
                    "points_staged", "packets", "full_lane_leaves", "partial_lane_leaves",
                    "lane_loop_chunks", "unused9", "clk_walk", "clk_leaf_test", "clk_wait",
                    "clk_transposed", "clk_lane_loop", "unused15", "unused16")


def ball_stats_read_all():
    arr = (_u64 * len(BALL_STATS_NAMES))()
    _check(lib().nbkd_stats_read_all(arr, len(BALL_STATS_NAMES)))
    return dict(zip(BALL_STATS_NAMES, [int(v) for v in arr]))


def stats_read_all():
    arr = (_u64 * len(STATS_NAMES))()
    _check(lib().nbkd_stats_read_all(arr, len(STATS_NAMES)))
    return dict(zip(STATS_NAMES, [int(v) for v in arr]))


# ------------------------------------------------------------------ slabs / RCCL
def slab_select(xyz_ptr, ids_ptr, n, lo, hi, out_xyz_ptr=None, out_ids_ptr=None, capacity=0,
                device=0, stream=None):
    """Device-side stable selection of points with lo <= x < hi; returns the count."""
    c = _u64()
    _check(lib().nbkd_slab_select(xyz_ptr, ids_ptr, int(n), float(lo), float(hi), out_xyz_ptr,
                                  out_ids_ptr, int(capacity), ctypes.byref(c), int(device), stream))
    return c.value


def slab_violations(q_ptr, dist_ptr, m, k, lo, hi, h, device=0, stream=None):
    c = _u64()
    _check(lib().nbkd_slab_violations(q_ptr, dist_ptr, int(m), int(k), float(lo), float(hi),
                                      float(h), ctypes.byref(c), int(device), stream))
    return c.value


def slab_forward_async(q_ptr, dist_ptr, m, k, cl, ch, count_ptr, list_ptr=None, sides_ptr=None,
                       capacity=0, device=0, stream=None):
    """nbkd_slab_forward_async: the same test, its total in the device word
    count_ptr when the stream gets there (nothing is waited for)."""
    _check(lib().nbkd_slab_forward_async(q_ptr, dist_ptr, int(m), int(k), float(cl), float(ch),
                                         list_ptr, sides_ptr, int(capacity), count_ptr,
                                         int(device), stream))


def slab_forward(q_ptr, dist_ptr, m, k, cl, ch, list_ptr=None, sides_ptr=None, capacity=0,
                 device=0, stream=None):
    """nbkd_slab_forward: total count of own queries whose k-th distance reaches
    past cl (left) or ch (right); up to `capacity` (index, side bits) entries."""
    c = _u64()
    _check(lib().nbkd_slab_forward(q_ptr, dist_ptr, int(m), int(k), float(cl), float(ch), list_ptr,
                                   sides_ptr, int(capacity), ctypes.byref(c), int(device), stream))
    return c.value


def rows_gather(src_ptr, row_bytes, idx_ptr, n, dst_ptr, device=0, stream=None):
    _check(lib().nbkd_rows_gather(src_ptr, int(row_bytes), idx_ptr, int(n), dst_ptr, int(device),
                                  stream))


def rows_scatter(src_ptr, row_bytes, idx_ptr, n, dst_ptr, device=0, stream=None):
    _check(lib().nbkd_rows_scatter(src_ptr, int(row_bytes), idx_ptr, int(n), dst_ptr, int(device),
                                   stream))


def comm_probe() -> None:
    """Raises unless RCCL loads (no bootstrap listener is started)."""
    _check(lib().nbkd_comm_probe())


def comm_unique_id() -> bytes:
    buf = (ctypes.c_uint8 * COMM_ID_BYTES)()
    _check(lib().nbkd_comm_unique_id(buf))
    return bytes(buf)


class Comm:
    """RCCL communicator over librccl (dlopen'ed by libnbkd)."""

    def __init__(self, uid: bytes, rank: int, world: int, device: int):
        buf = (ctypes.c_uint8 * COMM_ID_BYTES).from_buffer_copy(uid)
        h = _c_p()
        _check(lib().nbkd_comm_init(buf, int(rank), int(world), int(device), ctypes.byref(h)))
        self.h = h

    def exchange(self, pairs, stream=None):
        """pairs: list of (send_ptr, send_bytes, send_peer, recv_ptr, recv_bytes, recv_peer)."""
        n = len(pairs)
        sp = (_c_p * n)(*[p[0] for p in pairs])
        sb = (_u64 * n)(*[int(p[1]) for p in pairs])
        speer = (_i32 * n)(*[int(p[2]) for p in pairs])
        rp = (_c_p * n)(*[p[3] for p in pairs])
        rb = (_u64 * n)(*[int(p[4]) for p in pairs])
        rpeer = (_i32 * n)(*[int(p[5]) for p in pairs])
        _check(lib().nbkd_comm_exchange(self.h, n, sp, sb, speer, rp, rb, rpeer, stream))

    def close(self):
        if getattr(self, "h", None):
            lib().nbkd_comm_free(self.h)
            self.h = None

    __del__ = close
