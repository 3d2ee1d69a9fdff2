"""One library build, one workload: per-phase kNN times (HIP events on the
launch stream) and a SHA of the full distance and id arrays, as one JSON line.
The library is the one NBKD_LIB names (A/B runs: scripts/lib_ab.py).
python scripts/knn_time.py --n 1e8 --k 32 --leaf 64 [--lognormal] [--indep]"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nbodyhpc_amd import capi, hip, synth  # noqa: E402

PHASES = ("leaf_key", "sort", "knn_collect", "knn_select", "knn_retry", "knn_retry_order",
          "knn_fallback", "knn")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=float, default=1e8)
    ap.add_argument("--k", type=int, default=32)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--leaf", type=int, default=64)
    ap.add_argument("--lognormal", action="store_true")
    ap.add_argument("--kth", action="store_true", help="k-th distance only (nbkd_query_kth)")
    ap.add_argument("--ball", type=float, default=0.0, help="radius count at this r instead")
    a = ap.parse_args()
    hip.preload()
    hip.set_device(0)
    n, k = int(a.n), a.k
    pts = synth.lognormal(n) if a.lognormal else synth.uniform(n)
    s = hip.Stream()
    d = hip.DeviceArray.from_numpy(pts)
    del pts
    t = capi.Tree(n=n, dev_ptr=d.ptr, leafsize=a.leaf, boxsize=1.0, stream=s.handle)
    if a.ball > 0:
        od = hip.DeviceArray((n,), np.uint32)
        oi = None
        run = lambda: t.ball_count_device(d.ptr, n, a.ball, od.ptr, s.handle)  # noqa: E731
    elif a.kth:
        od = hip.DeviceArray((n,), np.float32)
        oi = None
        run = lambda: t.query_kth_device(d.ptr, n, k, od.ptr, s.handle)  # noqa: E731
    else:
        od = hip.DeviceArray((n, k), np.float32)
        oi = hip.DeviceArray((n, k), np.uint32)
        run = lambda: t.query_device(d.ptr, n, k, od.ptr, oi.ptr, s.handle)  # noqa: E731
    run()
    s.synchronize()
    capi.timing_enable(True)
    capi.timing_reset()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        run()
    s.synchronize()
    wall = (time.perf_counter() - t0) / a.steps * 1e3
    ph = {}
    for p in PHASES:
        ms, cnt = capi.timing_read(p)
        ph[p] = round(ms / a.steps, 3)
    capi.timing_enable(False)
    h = hashlib.sha256(od.numpy().tobytes())
    if oi is not None:
        h.update(oi.numpy().tobytes())
    lib = os.environ.get("NBKD_LIB", "production")
    print(json.dumps({"lib": lib, "n": n, "k": k, "leaf": a.leaf, "lognormal": a.lognormal,
                      "kth": a.kth, "ball": a.ball, "wall_ms": round(wall, 3), "qps": n / wall * 1e3,
                      "phases_ms": ph, "sha": h.hexdigest()[:16]}), flush=True)


if __name__ == "__main__":
    main()
