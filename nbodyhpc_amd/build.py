"""Build recipe for the in-tree native artefacts (no cmake / setuptools needed).

  nbodyhpc_amd/lib/libnbkd.so              hipcc --offload-arch=gfx950: C ABI + HIP kernels
  nbodyhpc_amd/kdtree/_impl<ext-suffix>    g++: pybind11 module over the C ABI
  nbodyhpc_amd/lib/exp/libnbkd.so          (--experiments only) the same sources with
                                           -DNBKD_EXPERIMENTS: the NBKD_* environment
                                           overrides of the tuning knobs (A/B runs);
                                           loaded only through NBKD_LIB, never by default

Both are built in-tree so they travel with the repo snapshot to the GPU box.
`python -m nbodyhpc_amd.build [--force] [--experiments]`.
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
SOURCES = ["api.cpp", "build.hip", "query.hip", "knn_collect.hip", "ball.hip", "slab.hip",
           "deposit.hip"]
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


EXP_DIR = os.path.join(LIB_DIR, "exp")
EXP_LIB = os.path.join(EXP_DIR, "libnbkd.so")


def build_lib(force=False, verbose=True, experiments=False):
    obj_dir = os.path.join(EXP_DIR, "obj") if experiments else OBJ_DIR
    lib = EXP_LIB if experiments else LIB
    flags = HIP_FLAGS + (["-DNBKD_EXPERIMENTS"] if experiments else [])
    os.makedirs(obj_dir, exist_ok=True)
    procs, objs = [], []
    for src in SOURCES:
        path = os.path.join(CSRC, src)
        obj = os.path.join(obj_dir, src + ".o")
        objs.append(obj)
        if force or _newer(obj, [path] + HEADERS):
            lang = [] if src.endswith(".hip") else ["-x", "hip"]
            procs.append(_run([HIPCC] + flags + lang + ["-c", path, "-o", obj], verbose))
    for p in procs:
        if p.wait() != 0:
            raise RuntimeError("hipcc failed")
    if force or procs or _newer(lib, objs):
        cmd = [HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", lib] + objs + ["-ldl"]
        if _run(cmd, verbose).wait() != 0:
            raise RuntimeError("link of libnbkd.so failed")
    return lib


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
    if "--experiments" in sys.argv:
        build_lib(force="--force" in sys.argv, experiments=True)
    else:
        build(force="--force" in sys.argv)
