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
ap.add_argument("--dist", default="uniform", choices=["uniform", "lognormal"])
a = ap.parse_args()
n, k = int(a.n), a.k
if a.dist == "uniform":
    pts = gen_uniform(n, 20261015, 1.0)
else:
    from nbodyhpc_amd import synth
    pts = synth.lognormal(n)
dp = hip.DeviceArray.from_numpy(pts)
s = hip.Stream()
tree = capi.Tree(n=n, dev_ptr=dp.ptr, leafsize=a.leafsize, boxsize=1.0, stream=s.handle)
od = hip.DeviceArray((n, k), np.float32)
oi = hip.DeviceArray((n, k), np.uint32)
ref = None
res = {}
for spec in a.variants.split(","):
    # "V" or "V/S": kernel variant V, seed parameter S (NBKD_KNN_SEED; 0 = off)
    # "V[/S[/C[/D]]]": kernel variant V, seed parameter S (NBKD_KNN_SEED; 0 = off),
    # collect path C (NBKD_KNN_COLLECT; 0 = off), dense threshold D (NBKD_DENSE_MIN)
    parts = spec.split("/")
    v = parts[0]
    os.environ["NBKD_KNN_VARIANT"] = v
    for i, var in ((1, "NBKD_KNN_SEED"), (2, "NBKD_KNN_COLLECT"), (3, "NBKD_DENSE_MIN"),
                   (4, "NBKD_COLLECT_OCC"), (5, "NBKD_KNN_ANCHOR")):
        if len(parts) > i and parts[i] != "":
            os.environ[var] = parts[i]
        else:
            os.environ.pop(var, None)
    tree.query_device(dp.ptr, n, k, od.ptr, oi.ptr, s.handle)
    s.synchronize()
    capi.timing_enable(True); capi.timing_reset()
    for _ in range(a.reps):
        tree.query_device(dp.ptr, n, k, od.ptr, oi.ptr, s.handle)
    s.synchronize()
    ms, cnt = capi.timing_read("knn")
    fb_ms, _ = capi.timing_read("knn_fallback")
    col_ms, _ = capi.timing_read("knn_collect")
    sel_ms, _ = capi.timing_read("knn_select")
    lk_ms, _ = capi.timing_read("leaf_key")
    rt_ms, _ = capi.timing_read("knn_retry")
    so_ms, _ = capi.timing_read("sort")
    ro_ms, _ = capi.timing_read("knn_retry_order")
    capi.timing_enable(False)
    r = {"knn_ms": ms / cnt, "collect_ms": col_ms / cnt, "select_ms": sel_ms / cnt,
         "fallback_ms": fb_ms / cnt, "retry_ms": rt_ms / cnt, "leaf_key_ms": lk_ms / cnt,
         "sort_ms": so_ms / cnt, "retry_order_ms": ro_ms / cnt,
         "total_ms": (ms + fb_ms + rt_ms + ro_ms + lk_ms + so_ms) / cnt,
         "qps_kernel": n / (ms / cnt * 1e-3)}
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
        r.update({kk: round(st[kk] / p, 2) for kk in capi.STATS_NAMES if kk not in ("packets", "fallback_queries", "retry_queries")})
        r["fallback_queries"] = st["fallback_queries"]
        r["retry_queries"] = st["retry_queries"]
    res[spec] = r
    print(spec, json.dumps(r), flush=True)
json.dump(res, open(os.path.join(ROOT, "gpurun_out", "variants.json"), "w"), indent=1)
