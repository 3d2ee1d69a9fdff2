"""The C3 radius count alone (for rocprofv3 PMC passes of ball_count2_kernel):
1e8 uniform periodic points (the bench's), leafsize 64, r = 0.01 L, every
particle counted, `--steps` timed passes after one untimed."""
import argparse
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
    ap.add_argument("--leaf", type=int, default=64)
    ap.add_argument("--steps", type=int, default=2)
    a = ap.parse_args()
    hip.preload()
    hip.set_device(0)
    n = int(a.n)
    pts = synth.uniform(n)
    d = hip.DeviceArray.from_numpy(pts)
    del pts
    s = hip.Stream()
    t = capi.Tree(n=n, dev_ptr=d.ptr, leafsize=a.leaf, boxsize=1.0, stream=s.handle)
    cnt = hip.DeviceArray((n,), np.uint32)
    t.ball_count_device(d.ptr, n, a.r, cnt.ptr, s.handle)
    hip.synchronize()
    capi.timing_reset()
    capi.timing_enable(True)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        t.ball_count_device(d.ptr, n, a.r, cnt.ptr, s.handle)
    hip.synchronize()
    ms = (time.perf_counter() - t0) / a.steps * 1e3
    kms = capi.timing_read("ball_count")[0] / a.steps
    print(f"radius count n={n:.0e} r={a.r} leaf={a.leaf}: {ms:.2f} ms/pass ({kms:.2f} ms kernel), "
          f"{n / ms * 1e3:.3e} q/s, mean count {cnt.numpy().mean():.2f}", flush=True)


if __name__ == "__main__":
    main()
