"""Tuning sweep: time packet-kNN variants (NBKD_KNN_VARIANT) on one tree.
python scripts/variants.py --n 1e8 --variants 0,5,6,7 [--stats]"""
import argparse, json, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from nbodyhpc_amd import capi, hip
from bench import gen_uniform

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=float, default=1e8)
ap.add_argument("--k", type=int, default=32)
ap.add_argument("--leafsize", type=int, default=32)
ap.add_argument("--variants", default="0")
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--stats", action="store_true")
a = ap.parse_args()
n, k = int(a.n), a.k
pts = gen_uniform(n, 20261015, 1.0)
dp = hip.DeviceArray.from_numpy(pts)
s = hip.Stream()
tree = capi.Tree(n=n, dev_ptr=dp.ptr, leafsize=a.leafsize, boxsize=1.0, stream=s.handle)
od = hip.DeviceArray((n, k), np.float32)
oi = hip.DeviceArray((n, k), np.uint32)
ref = None
res = {}
for v in a.variants.split(","):
    os.environ["NBKD_KNN_VARIANT"] = v
    tree.query_device(dp.ptr, n, k, od.ptr, oi.ptr, s.handle)
    s.synchronize()
    capi.timing_enable(True); capi.timing_reset()
    for _ in range(a.reps):
        tree.query_device(dp.ptr, n, k, od.ptr, oi.ptr, s.handle)
    s.synchronize()
    ms, cnt = capi.timing_read("knn")
    capi.timing_enable(False)
    r = {"knn_ms": ms / cnt, "qps_kernel": n / (ms / cnt * 1e-3)}
    head = od.numpy_head(200000)
    if ref is None:
        ref = head
    r["dist_equal_to_first"] = bool(np.array_equal(head, ref))
    if a.stats:
        capi.stats_enable(True)
        tree.query_device(dp.ptr, n, k, od.ptr, oi.ptr, s.handle)
        s.synchronize()
        st = capi.stats_read_all()
        capi.stats_enable(False)
        p = max(st["packets"], 1)
        r.update({kk: round(st[kk] / p, 2) for kk in ("dense_rounds", "sparse_iters", "merges",
                                                       "candidates", "fill_merges")})
    res[v] = r
    print(v, json.dumps(r), flush=True)
json.dump(res, open(os.path.join(ROOT, "gpurun_out", "variants.json"), "w"), indent=1)
