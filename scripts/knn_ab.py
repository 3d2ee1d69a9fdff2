"""kNN timing at one setting of the env knobs, for A/B runs in separate
processes:  NBKD_KNN_ANCHOR=128 python scripts/knn_ab.py --lognormal --n 1e8
Prints ms per query pass, the retry count and a checksum of the distances
(must not change between knobs)."""
import argparse
import hashlib
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nbodyhpc_amd import capi, hip, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=float, default=1e8)
    ap.add_argument("--k", type=int, default=32)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--leaf", type=int, default=64)
    ap.add_argument("--lognormal", action="store_true")
    ap.add_argument("--grid", type=int, default=512)
    a = ap.parse_args()
    hip.preload()
    hip.set_device(0)
    n, k = int(a.n), a.k
    pts = synth.lognormal(n, grid=a.grid) if a.lognormal else synth.uniform(n)
    s = hip.Stream()
    d = hip.DeviceArray.from_numpy(pts)
    del pts
    t = capi.Tree(n=n, dev_ptr=d.ptr, leafsize=a.leaf, boxsize=1.0, stream=s.handle)
    od = hip.DeviceArray((n, k), np.float32)
    oi = hip.DeviceArray((n, k), np.uint32)
    t.query_device(d.ptr, n, k, od.ptr, oi.ptr, s.handle)
    hip.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        t.query_device(d.ptr, n, k, od.ptr, oi.ptr, s.handle)
    hip.synchronize()
    ms = (time.perf_counter() - t0) / a.steps * 1e3
    capi.stats_enable(True)
    t.query_device(d.ptr, n, k, od.ptr, oi.ptr, s.handle)
    hip.synchronize()
    st = capi.stats_read_all()
    capi.stats_enable(False)
    h = od.numpy()
    knobs = " ".join(f"{kk}={v}" for kk, v in sorted(os.environ.items()) if kk.startswith("NBKD_"))
    print(f"[{knobs or 'defaults'}] leaf={a.leaf} n={n:.0e} k={k} lognormal={a.lognormal} "
          f"ms={ms:.2f} q/s={n / ms * 1e3:.3e} retry={st['retry_queries']} "
          f"fallback={st['fallback_queries']} cand/q={st['candidates'] / n:.1f} "
          f"sha={hashlib.sha256(h.tobytes()).hexdigest()[:16]}", flush=True)


if __name__ == "__main__":
    main()
