"""Build recipe for the in-tree native artefacts (no cmake / setuptools needed).

  nbodyhpc_amd/lib/libnbkd.so              hipcc --offload-arch=gfx950: C ABI + HIP kernels
  nbodyhpc_amd/kdtree/_impl<ext-suffix>    g++: pybind11 module over the C ABI

Both are built in-tree so they travel with the repo snapshot to the GPU box.
`python -m nbodyhpc_amd.build [--force]`.
"""
from __future__ import annotations

import os
import subprocess
import sys
import sysconfig

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB_DIR = os.path.join(PKG, "lib")
OBJ_DIR = os.path.join(LIB_DIR, "obj")
LIB = os.path.join(LIB_DIR, "libnbkd.so")
EXT = os.path.join(PKG, "kdtree", "_impl" + sysconfig.get_config_var("EXT_SUFFIX"))

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("NBKD_ARCH", "gfx950")
# -ffp-contract=off: the reference is built -mavx2 without -mfma
# (kdtree/CMakeLists.txt:74); no multiply may be fused into an add or the
# squared distances stop being bit-identical.
HIP_FLAGS = ["--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
             "-Wall", "-Wno-unused-function", "-Wno-unused-const-variable"]
SOURCES = ["api.cpp", "build.hip", "query.hip", "knn_packet.hip", "knn_collect.hip", "ball.hip",
           "slab.hip", "deposit.hip"]
HEADERS = [os.path.join(CSRC, "internal.hpp"), os.path.join(CSRC, "metric.hpp"),
           os.path.join(CSRC, "packet.hpp"),
           os.path.join(ROOT, "include", "nbkd.h")]


def _newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    return subprocess.Popen(cmd)


def build_lib(force=False, verbose=True):
    os.makedirs(OBJ_DIR, exist_ok=True)
    procs, objs = [], []
    for src in SOURCES:
        path = os.path.join(CSRC, src)
        obj = os.path.join(OBJ_DIR, src + ".o")
        objs.append(obj)
        if force or _newer(obj, [path] + HEADERS):
            lang = [] if src.endswith(".hip") else ["-x", "hip"]
            procs.append(_run([HIPCC] + HIP_FLAGS + lang + ["-c", path, "-o", obj], verbose))
    for p in procs:
        if p.wait() != 0:
            raise RuntimeError("hipcc failed")
    if force or procs or _newer(LIB, objs):
        cmd = [HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", LIB] + objs + ["-ldl"]
        if _run(cmd, verbose).wait() != 0:
            raise RuntimeError("link of libnbkd.so failed")
    return LIB


def build_ext(force=False, verbose=True):
    src = os.path.join(CSRC, "pybind_impl.cpp")
    if not (force or _newer(EXT, [src, LIB] + HEADERS)):
        return EXT
    import pybind11

    inc = [pybind11.get_include(), sysconfig.get_paths()["include"]]
    cmd = (["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-fvisibility=hidden"]
           + ["-I" + i for i in inc]
           + [src, "-o", EXT, "-L" + LIB_DIR, "-lnbkd", "-Wl,-rpath,$ORIGIN/../lib"])
    if _run(cmd, verbose).wait() != 0:
        raise RuntimeError("build of the pybind11 module failed")
    return EXT


def build(force=False, verbose=True):
    build_lib(force, verbose)
    build_ext(force, verbose)
    return LIB, EXT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
