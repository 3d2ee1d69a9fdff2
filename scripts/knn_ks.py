"""kNN timing over several k on one 1e8 tree (device in / device out), with
the per-kernel breakdown (HIP events) and a checksum of the first rows:
    python scripts/knn_ks.py --ks 32,64,100,200 [--n 1e8] [--leaf 64]"""
import argparse
import hashlib
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nbodyhpc_amd import capi, hip, synth  # noqa: E402

PARTS = ("self_order", "leaf_key", "sort", "knn_collect", "knn_select", "knn_retry", "knn_fallback",
         "knn_exact")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=float, default=1e8)
    ap.add_argument("--ks", default="32,64,100")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--leaf", type=int, default=64)
    a = ap.parse_args()
    hip.preload()
    hip.set_device(0)
    n = int(a.n)
    ks = [int(x) for x in a.ks.split(",")]
    pts = synth.uniform(n)
    s = hip.Stream()
    d = hip.DeviceArray.from_numpy(pts)
    del pts
    t = capi.Tree(n=n, dev_ptr=d.ptr, leafsize=a.leaf, boxsize=1.0, stream=s.handle)
    od = hip.DeviceArray((n, max(ks)), np.float32)
    oi = hip.DeviceArray((n, max(ks)), np.uint32)
    for k in ks:
        t.query_device(d.ptr, n, k, od.ptr, oi.ptr, s.handle)
        hip.synchronize()
        capi.timing_reset()
        capi.timing_enable(True)
        t0 = time.perf_counter()
        for _ in range(a.steps):
            t.query_device(d.ptr, n, k, od.ptr, oi.ptr, s.handle)
        hip.synchronize()
        ms = (time.perf_counter() - t0) / a.steps * 1e3
        br = {p: round(capi.timing_read(p)[0] / a.steps, 3) for p in PARTS}
        capi.timing_enable(False)
        h = od.numpy_head(min(n, 1_000_000) * k // max(ks) + 1)
        print(f"k={k} leaf={a.leaf} n={n:.0e} ms={ms:.2f} q/s={n / ms * 1e3:.3e} {br} "
              f"sha={hashlib.sha256(h.tobytes()).hexdigest()[:16]}", flush=True)


if __name__ == "__main__":
    main()
