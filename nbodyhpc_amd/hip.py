"""Minimal HIP runtime plumbing over ctypes (device buffers, copies, streams,
events, synchronisation) for bench.py and the device-pointer tests.

It binds the SAME libamdhip64.so.7 that libnbkd.so links (ROCm 7.2), so there
is exactly one HIP runtime in the process.  torch wheels bundle their own HIP
runtime (ROCm 7.0); two initialised runtimes in one process do not coexist
(the second reports "No HIP GPUs are available"), so processes that drive
libnbkd never touch torch.cuda — torch is used only for torch.distributed
(gloo) coordination.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_LIB = None
H2D, D2H, D2D = 1, 2, 3


def _hip():
    global _LIB
    if _LIB is None:
        path = os.environ.get("NBKD_HIP_RUNTIME", "/opt/rocm/lib/libamdhip64.so.7")
        L = ctypes.CDLL(path)
        vp, sz = ctypes.c_void_p, ctypes.c_size_t
        L.hipMalloc.argtypes = [ctypes.POINTER(vp), sz]
        L.hipFree.argtypes = [vp]
        L.hipMemcpy.argtypes = [vp, vp, sz, ctypes.c_int]
        L.hipMemcpyAsync.argtypes = [vp, vp, sz, ctypes.c_int, vp]
        L.hipHostMalloc.argtypes = [ctypes.POINTER(vp), sz, ctypes.c_uint]
        L.hipHostFree.argtypes = [vp]
        L.hipMemset.argtypes = [vp, ctypes.c_int, sz]
        L.hipMemGetInfo.argtypes = [ctypes.POINTER(sz), ctypes.POINTER(sz)]
        L.hipDeviceSynchronize.argtypes = []
        L.hipSetDevice.argtypes = [ctypes.c_int]
        L.hipGetDeviceCount.argtypes = [ctypes.POINTER(ctypes.c_int)]
        L.hipStreamCreate.argtypes = [ctypes.POINTER(vp)]
        L.hipStreamDestroy.argtypes = [vp]
        L.hipStreamSynchronize.argtypes = [vp]
        L.hipStreamQuery.argtypes = [vp]
        L.hipEventCreate.argtypes = [ctypes.POINTER(vp)]
        L.hipEventDestroy.argtypes = [vp]
        L.hipEventRecord.argtypes = [vp, vp]
        L.hipEventSynchronize.argtypes = [vp]
        L.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), vp, vp]
        L.hipGetErrorString.restype = ctypes.c_char_p
        L.hipGetErrorString.argtypes = [ctypes.c_int]
        _LIB = L
    return _LIB


def preload():
    """Load the ROCm 7.2 HIP runtime and libnbkd.so NOW.  Call before anything
    imports torch: torch's bundled libamdhip64.so.7 / libhsa-runtime64.so.1
    (ROCm 7.0) carry the same sonames, so whichever loads first serves the
    process; loading ours second fails (missing ROCR_1 symbols)."""
    _hip()
    from . import capi

    capi.lib()
    # RCCL too (nbkd_comm_probe: a dlopen, nothing starts): the image's librccl,
    # bound to this runtime.  Loaded after torch, the soname would resolve to
    # torch's bundled librccl, whose own HIP runtime sees no device here.
    try:
        capi.comm_probe()
    except Exception:
        pass  # no RCCL: the multi-GPU paths stage over gloo


def _ok(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what}: {_hip().hipGetErrorString(rc).decode()}")


def device_count() -> int:
    c = ctypes.c_int(0)
    rc = _hip().hipGetDeviceCount(ctypes.byref(c))
    return c.value if rc == 0 else 0


def set_device(d: int):
    _ok(_hip().hipSetDevice(int(d)), "hipSetDevice")


def synchronize():
    _ok(_hip().hipDeviceSynchronize(), "hipDeviceSynchronize")


def stream_synchronize(handle):
    """hipStreamSynchronize on a raw stream handle (None: the null stream)."""
    _ok(_hip().hipStreamSynchronize(handle), "hipStreamSynchronize")


def mem_info():
    """(free, total) bytes of the current device (hipMemGetInfo)."""
    f, t = ctypes.c_size_t(), ctypes.c_size_t()
    _ok(_hip().hipMemGetInfo(ctypes.byref(f), ctypes.byref(t)), "hipMemGetInfo")
    return int(f.value), int(t.value)


class DeviceArray:
    """A raw device allocation with numpy-style shape/dtype bookkeeping."""

    def __init__(self, shape, dtype):
        self.shape = tuple(int(s) for s in np.atleast_1d(shape)) if not isinstance(shape, tuple) \
            else tuple(int(s) for s in shape)
        self.dtype = np.dtype(dtype)
        self.nbytes = int(np.prod(self.shape)) * self.dtype.itemsize
        p = ctypes.c_void_p()
        _ok(_hip().hipMalloc(ctypes.byref(p), max(self.nbytes, 16)), "hipMalloc")
        self.ptr = p.value

    @classmethod
    def from_numpy(cls, a):
        a = np.ascontiguousarray(a)
        d = cls(a.shape, a.dtype)
        _ok(_hip().hipMemcpy(d.ptr, a.ctypes.data, a.nbytes, H2D), "hipMemcpy H2D")
        return d

    def numpy(self):
        out = np.empty(self.shape, self.dtype)
        _ok(_hip().hipMemcpy(out.ctypes.data, self.ptr, self.nbytes, D2H), "hipMemcpy D2H")
        return out

    def numpy_head(self, rows):
        """copy only the first `rows` rows (leading dimension) to the host"""
        rows = min(int(rows), self.shape[0])
        out = np.empty((rows,) + self.shape[1:], self.dtype)
        _ok(_hip().hipMemcpy(out.ctypes.data, self.ptr, out.nbytes, D2H), "hipMemcpy D2H")
        return out

    def zero(self):
        _ok(_hip().hipMemset(self.ptr, 0, self.nbytes), "hipMemset")

    def free(self):
        if getattr(self, "ptr", None):
            _hip().hipFree(self.ptr)
            self.ptr = None

    __del__ = free


def memcpy(dst_ptr, src_ptr, nbytes, kind=D2D):
    """Synchronous copy between raw pointers (kind: H2D / D2H / D2D)."""
    if nbytes:
        _ok(_hip().hipMemcpy(dst_ptr, src_ptr, int(nbytes), int(kind)), "hipMemcpy")


def memcpy_async(dst_ptr, src_ptr, nbytes, kind, stream_handle):
    """hipMemcpyAsync on a stream (with pinned host memory a true async copy)."""
    if nbytes:
        _ok(_hip().hipMemcpyAsync(dst_ptr, src_ptr, int(nbytes), int(kind), stream_handle),
            "hipMemcpyAsync")


class HostBuffer:
    """Pinned host memory (hipHostMalloc) viewed as a numpy array."""

    def __init__(self, shape, dtype):
        self.dtype = np.dtype(dtype)
        self.shape = tuple(int(s) for s in np.atleast_1d(shape))
        self.nbytes = int(np.prod(self.shape)) * self.dtype.itemsize
        p = ctypes.c_void_p()
        _ok(_hip().hipHostMalloc(ctypes.byref(p), max(self.nbytes, 16), 0), "hipHostMalloc")
        self.ptr = p.value
        buf = (ctypes.c_char * max(self.nbytes, 16)).from_address(self.ptr)
        self.array = np.frombuffer(buf, self.dtype, count=int(np.prod(self.shape))).reshape(
            self.shape)

    def free(self):
        if getattr(self, "ptr", None):
            self.array = None
            _hip().hipHostFree(self.ptr)
            self.ptr = None

    __del__ = free


class Stream:
    def __init__(self):
        s = ctypes.c_void_p()
        _ok(_hip().hipStreamCreate(ctypes.byref(s)), "hipStreamCreate")
        self.handle = s.value

    def synchronize(self):
        _ok(_hip().hipStreamSynchronize(self.handle), "hipStreamSynchronize")

    def busy(self) -> bool:
        """hipStreamQuery: True while work enqueued on the stream is pending."""
        rc = _hip().hipStreamQuery(self.handle)
        if rc == 600:  # hipErrorNotReady
            return True
        _ok(rc, "hipStreamQuery")
        return False


class Event:
    def __init__(self):
        e = ctypes.c_void_p()
        _ok(_hip().hipEventCreate(ctypes.byref(e)), "hipEventCreate")
        self.handle = e.value

    def record(self, stream=None):
        h = stream.handle if isinstance(stream, Stream) else stream
        _ok(_hip().hipEventRecord(self.handle, h), "hipEventRecord")

    def synchronize(self):
        _ok(_hip().hipEventSynchronize(self.handle), "hipEventSynchronize")

    def elapsed_ms(self, end: "Event") -> float:
        _ok(_hip().hipEventSynchronize(end.handle), "hipEventSynchronize")
        t = ctypes.c_float()
        _ok(_hip().hipEventElapsedTime(ctypes.byref(t), self.handle, end.handle),
            "hipEventElapsedTime")
        return float(t.value)
