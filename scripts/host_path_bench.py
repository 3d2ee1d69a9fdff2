"""Where the host-buffer kNN path (KDTree.query: host queries in, host rows
out) spends its time at 1e8 self-queries, k = 32:

  * pinned DMA rates (hipMemcpyAsync D2H / H2D, 1 GiB, pinned host memory);
  * first-touch write rate of fresh pageable numpy memory (one thread);
  * the whole host-to-host call at host_threads = 1, 4, 8, 16 (0 = auto).

    python scripts/host_path_bench.py [--n 1e8] [--k 32]
"""
import argparse
import json
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
    ap.add_argument("--threads", type=int, nargs="+", default=[0, 1, 4, 16])
    a = ap.parse_args()
    hip.preload()
    hip.set_device(0)
    out = {}
    nb = 1 << 30
    hb = hip.HostBuffer((nb,), np.uint8)
    db = hip.DeviceArray((nb,), np.uint8)
    s = hip.Stream()
    for name, kind, dst, src in (("d2h", hip.D2H, hb.ptr, db.ptr), ("h2d", hip.H2D, db.ptr, hb.ptr)):
        hip.memcpy_async(dst, src, nb, kind, s.handle)
        s.synchronize()
        t0 = time.perf_counter()
        for _ in range(4):
            hip.memcpy_async(dst, src, nb, kind, s.handle)
        s.synchronize()
        out[f"pinned_{name}_GBps"] = 4 * nb / (time.perf_counter() - t0) / 1e9
    t0 = time.perf_counter()
    x = np.empty(nb // 4, np.float32)
    x[:] = 1.0
    out["first_touch_write_1thread_GBps"] = nb / (time.perf_counter() - t0) / 1e9
    t0 = time.perf_counter()
    x[:] = 2.0
    out["rewrite_1thread_GBps"] = nb / (time.perf_counter() - t0) / 1e9
    del x
    hb.free()
    db.free()
    print(json.dumps(out), flush=True)

    n, k = int(a.n), a.k
    pts = synth.uniform(n)
    d = hip.DeviceArray.from_numpy(pts)
    t = capi.Tree(n=n, dev_ptr=d.ptr, leafsize=64, boxsize=1.0, stream=s.handle)
    t.query(pts[:100_000], k)
    rates = {}
    for th in a.threads:
        capi.set_tuning("host_threads", th)
        t.query(pts[:1_000_000], k)
        t0 = time.perf_counter()
        dd, ii = t.query(pts, k)
        sec = time.perf_counter() - t0
        ok = bool(np.all(dd[:, 0] == 0.0))
        rates[str(th)] = {"queries_per_s": n / sec, "s": sec,
                          "GBps_out": (dd.nbytes + ii.nbytes) / sec / 1e9, "self_zero": ok}
        del dd, ii
        print(json.dumps({"host_threads": th, **rates[str(th)]}), flush=True)
    capi.set_tuning("host_threads", 0)
    out["host_to_host"] = rates
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
