"""MI355X-native kd-tree (build + batched kNN / radius queries) for N-body particle data.

Product layout:
  include/nbkd.h            C ABI (drop-in boundary)
  nbodyhpc_amd/csrc/        HIP kernels (gfx950) + C ABI + pybind11 module sources
  nbodyhpc_amd/lib/         built libnbkd.so
  nbodyhpc_amd/kdtree/      Python surface (mirror of nbodyhpc.kdtree) + built _impl
  nbodyhpc_amd/capi.py      ctypes binding of the C ABI
"""
__version__ = "0.1.0"
