"""Radius-count timing at one setting of the ball-kernel knobs (env), for A/B
runs in separate processes:  NBKD_BALL_T=0 python scripts/ball_ab.py --n 1e8
Prints ms per pass and a checksum of the counts (must not change between knobs)."""
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
    ap.add_argument("--r", type=float, default=0.01)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--lognormal", action="store_true")
    ap.add_argument("--leaf", type=int, default=32)
    a = ap.parse_args()
    hip.preload()
    hip.set_device(0)
    n = int(a.n)
    pts = synth.lognormal(n) if a.lognormal else synth.uniform(n)
    s = hip.Stream()
    d = hip.DeviceArray.from_numpy(pts)
    del pts
    t = capi.Tree(n=n, dev_ptr=d.ptr, leafsize=a.leaf, boxsize=1.0, stream=s.handle)
    c = hip.DeviceArray((n,), np.uint32)
    t.ball_count_device(d.ptr, n, a.r, c.ptr, s.handle)
    hip.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        t.ball_count_device(d.ptr, n, a.r, c.ptr, s.handle)
    hip.synchronize()
    ms = (time.perf_counter() - t0) / a.steps * 1e3
    h = c.numpy()
    knobs = " ".join(f"{k}={v}" for k, v in sorted(os.environ.items()) if k.startswith("NBKD_"))
    print(f"[{knobs or 'defaults'}] leaf={a.leaf} n={n:.0e} "
          f"lognormal={a.lognormal} ms={ms:.2f} q/s={n / ms * 1e3:.3e} mean={h.mean():.3f} "
          f"sha={hashlib.sha256(h.tobytes()).hexdigest()[:16]}", flush=True)


if __name__ == "__main__":
    main()
