"""One library build, one workload: per-phase kNN times (HIP events on the
launch stream) and a SHA of the full distance and id arrays, as one JSON line.
The library is the one NBKD_LIB names (A/B runs: scripts/lib_ab.py).
python scripts/knn_time.py --n 1e8 --k 32 --leaf 64 [--lognormal]

--slab-world W --slab-rank r [--scaling strong|weak]: rank r's part of the
bench's W-GPU run, alone on this GPU (scripts/slab_traffic.sh profiles it):
the same own particles (slab.gen_uniform_slab / gen_slab_points), the same
halo strips of its two ring neighbours (width slab.halo_width, the strip tests
of DeviceSlab.exchange, own then left then right), global ids, and only the
own particles queried, so the counters see one rank's kNN step."""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nbodyhpc_amd import capi, hip, synth  # noqa: E402

PHASES = ("self_order", "leaf_key", "sort", "knn_collect", "knn_select", "knn_retry", "knn_retry_order",
          "knn_fallback", "knn", "ball_count")


def slab_points(a, k):
    """(points, global ids, own count) of rank a.slab_rank's local tree in the
    bench's a.slab_world-GPU run: own particles first, then the strip from the
    left neighbour (its x >= hi - h), then the one from the right (x < lo + h)."""
    from nbodyhpc_amd import slab
    W, r, L = a.slab_world, a.slab_rank, 1.0
    n = int(a.n)

    def own_of(rank):
        if a.scaling == "strong":
            return slab.gen_uniform_slab(n, a.seed, L, rank, W)
        return slab.gen_slab_points(n, a.seed, L, rank, W)

    total = n if a.scaling == "strong" else n * W
    h = slab.halo_width(total, k, L)
    bounds = slab.bounds_list(W, L)
    slab.check_halo(h, bounds)
    left, right = slab.neighbours(r, W)
    ox, oi = own_of(r)
    lx, li = own_of(left)
    m = lx[:, 0] >= np.float32(bounds[left + 1] - h)
    fl = (lx[m], li[m])
    rx, ri = (lx, li) if right == left else own_of(right)
    m = rx[:, 0] < np.float32(bounds[right] + h)
    fr = (rx[m], ri[m])
    xyz = np.concatenate([ox, fl[0], fr[0]])
    ids = np.concatenate([oi, fl[1], fr[1]]).astype(np.uint32)
    print(f"[knn_time] slab {r}/{W} {a.scaling}: {len(ox)} own + {len(fl[0])} + {len(fr[0])} "
          f"halo, h = {h:.4g}", file=sys.stderr, flush=True)
    ext = (min(L, bounds[r + 1] - bounds[r] + 2.0 * h), L, L)  # DeviceSlab.extent
    return xyz, ids, len(ox), ext


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=float, default=1e8)
    ap.add_argument("--k", type=int, default=32)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--leaf", type=int, default=64)
    ap.add_argument("--lognormal", action="store_true")
    ap.add_argument("--kth", action="store_true", help="k-th distance only (nbkd_query_kth)")
    ap.add_argument("--ball", type=float, default=0.0, help="radius count at this r instead")
    ap.add_argument("--slab-world", type=int, default=1)
    ap.add_argument("--slab-rank", type=int, default=0)
    ap.add_argument("--scaling", choices=("strong", "weak"), default="strong")
    ap.add_argument("--no-extent", action="store_true",
                    help="slab tree with the reference's depth %% 3 axes (A/B of nbkd_build_ext)")
    ap.add_argument("--seed", type=int, default=20261015)
    ap.add_argument("--no-timing", action="store_true",
                    help="time the steps with the library's phase timers off (no phases)")
    ap.add_argument("--tune", action="append", default=[], metavar="NAME=VALUE",
                    help="nbkd_set_tuning before the runs (e.g. self_order=0)")
    ap.add_argument("--stats", action="store_true",
                    help="one more (untimed) pass with the work counters and phase clocks on")
    a = ap.parse_args()
    hip.preload()
    hip.set_device(0)
    for kv in a.tune:
        name, val = kv.split("=")
        capi.set_tuning(name, float(val))
    n, k = int(a.n), a.k
    ids = None
    ext = None
    if a.slab_world > 1:
        pts, ids, n_own, ext = slab_points(a, k)
        if a.no_extent:
            ext = None
    else:
        pts = synth.lognormal(n) if a.lognormal else synth.uniform(n, a.seed)
        n_own = n
    s = hip.Stream()
    d = hip.DeviceArray.from_numpy(pts)
    n_tree = pts.shape[0]
    del pts
    t = capi.Tree(n=n_tree, dev_ptr=d.ptr, leafsize=a.leaf, boxsize=1.0, stream=s.handle,
                  extent=ext)
    if ids is not None:
        di = hip.DeviceArray.from_numpy(ids)
        t.set_ids(dev_ptr=di.ptr, stream=s.handle)
    n = n_own
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
    capi.timing_enable(not a.no_timing)
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
    st = None
    if a.stats:
        capi.stats_enable(True)
        run()
        s.synchronize()
        st = capi.ball_stats_read_all() if a.ball > 0 else capi.stats_read_all()
        capi.stats_enable(False)
    h = hashlib.sha256(od.numpy().tobytes())
    if oi is not None:
        h.update(oi.numpy().tobytes())
    lib = os.environ.get("NBKD_LIB", "production")
    print(json.dumps({"lib": lib, "n": n, "n_tree": n_tree, "slab_world": a.slab_world,
                      "slab_rank": a.slab_rank, "scaling": a.scaling, "n_arg": int(a.n),
                      "seed": a.seed, "k": k, "leaf": a.leaf, "lognormal": a.lognormal,
                      "kth": a.kth, "ball": a.ball, "wall_ms": round(wall, 3), "qps": n / wall * 1e3,
                      "phases_ms": ph, "sha": h.hexdigest()[:16], "tune": a.tune,
                      "extent": ext, "stats": st}),
          flush=True)


if __name__ == "__main__":
    main()
