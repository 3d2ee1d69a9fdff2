"""Deposit benchmark: kNN smoothing lengths -> render_points_volume on the GPU.

The reference quotes its Vulkan rasteriser at ~2.5 s for a 256^3-particle
snapshot on a 1024^3 grid (rasterization/README.md "Performance", RTX 6000,
after host-side vertex preparation).  This runs the same shape: N particles
(uniform or the C5 log-normal field) in the unit periodic box, radii = distance
to the k-th neighbour (GPU kd-tree), weights 1/N, grid G^3, S^3 sub-samples;
inputs resident on the device; the deposit kernel timed with HIP events.

    python scripts/bench_deposit.py [--n 16777216] [--grid 1024] [--k 32] [--dist lognormal]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from nbodyhpc_amd import hip  # noqa: E402

hip.preload()
from nbodyhpc_amd import capi, synth  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=256 ** 3)
    p.add_argument("--grid", type=int, default=1024)
    p.add_argument("--k", type=int, default=32)
    p.add_argument("--S", type=int, default=4)
    p.add_argument("--dist", choices=("uniform", "lognormal"), default="uniform")
    p.add_argument("--reps", type=int, default=3)
    p.add_argument("--cpu-sample", type=int, default=2000)
    p.add_argument("--no-cpu", action="store_true")
    a = p.parse_args()

    t0 = time.time()
    if a.dist == "uniform":
        pts = synth.uniform(a.n, box=1.0)
    else:
        pts = synth.lognormal(a.n, box=1.0, grid=256)
    gen_s = time.time() - t0
    tree = capi.Tree(pts, leafsize=64, boxsize=1.0)
    radii = tree.query_kth(pts, a.k)
    tree.close()
    w = np.full(a.n, 1.0 / a.n, np.float32)
    G = a.grid
    ppu = float(G)
    dx = hip.DeviceArray.from_numpy(pts)
    dw = hip.DeviceArray.from_numpy(w)
    dr = hip.DeviceArray.from_numpy(radii)
    dg = hip.DeviceArray((G, G, G), np.float32)
    per = (1.0, 1.0, 1.0)

    def run():
        capi.deposit_device(dx.ptr, dw.ptr, dr.ptr, a.n, (G, G, G), ppu, dg.ptr, period=per,
                            subsample=a.S)

    run()
    hip.synchronize()
    capi.timing_enable(True)
    times = []
    for _ in range(a.reps):
        capi.timing_reset()
        e0, e1 = hip.Event(), hip.Event()
        e0.record()
        run()
        e1.record()
        times.append(e0.elapsed_ms(e1))
        kms, _ = capi.timing_read("deposit")
    capi.timing_enable(False)
    ms = float(np.median(times))
    # the grid holds the total weight (sampling error of the S^3 rule)
    total = 0.0
    plane = G * G
    for s0 in range(0, G, 64):
        blk = np.empty(plane * min(64, G - s0), np.float32)
        hip.memcpy(blk.ctypes.data, dg.ptr + s0 * plane * 4, blk.nbytes, hip.D2H)
        total += float(blk.sum(dtype=np.float64))
    rvox = radii.astype(np.float64) * G
    out = {"workload": "deposit", "dist": a.dist, "n": a.n, "grid": G, "k": a.k, "S": a.S,
           "ms": round(ms, 3), "kernel_ms": round(kms, 3),
           "particles_per_s": a.n / (ms * 1e-3), "mass": total,
           "radius_vox_mean": float(rvox.mean()), "radius_vox_p99": float(np.percentile(rvox, 99)),
           "sphere_voxels_mean": float((4.0 / 3.0 * np.pi * rvox ** 3).mean()),
           "gen_s": round(gen_s, 1)}
    if not a.no_cpu:
        from oracle.oracle import Oracle
        o = Oracle()
        m = min(a.cpu_sample, a.n)
        sel = np.random.default_rng(0).choice(a.n, m, replace=False)
        # the oracle accumulates into a full double grid: the sample's positions
        # are squeezed into a sub-box of Gc^3 voxels with the radii (in voxels) kept
        Gc = G if G <= 512 else 512
        scale = Gc / G
        t = time.time()
        o.deposit(pts[sel] * np.float32(scale), w[sel], radii[sel], (Gc, Gc, Gc), ppu,
                  (scale, scale, scale), a.S)
        dt = time.time() - t
        out["cpu_baseline"] = {"particles_per_s": m / dt, "cores": 1, "kind": "port",
                               "sample": f"{m} particles, grid {Gc}^3 at the same voxel radii"}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
