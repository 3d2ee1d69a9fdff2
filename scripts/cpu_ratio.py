"""Port / reference CPU speed ratio (the bench's cpu_baseline is the port,
oracle/liborc.so; the compiled reference oracle/_ref exists only in the build
container).  Same points, same tree parameters, same thread counts, runs
interleaved (port, reference, port, ...) so host noise hits both:

    python scripts/cpu_ratio.py --n 1e7 --threads 1 8 --reps 3 > profiles/r05_cpu_ratio.json

Reports the single-threaded build times and the query rates (k = 32,
periodic, leafsize 64, self-queries of the first --queries points) with the
per-rep values, min and median, and the port/reference ratios of the medians."""
import argparse
import json
import os
import statistics
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle.oracle import Oracle, Reference  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=float, default=1e7)
    ap.add_argument("--queries", type=int, default=1_000_000)
    ap.add_argument("--threads", type=int, nargs="+", default=[1, 8])
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--leafsize", type=int, default=64)
    ap.add_argument("--k", type=int, default=32)
    a = ap.parse_args()
    n = int(a.n)
    rng = np.random.Generator(np.random.PCG64(20261015))
    pts = rng.uniform(0.0, 1.0, size=(n, 3)).astype(np.float32)
    libs = {"port": Oracle(), "reference": Reference()}
    build = {nm: [] for nm in libs}
    trees = {}
    for _ in range(a.reps):
        for nm, lib in libs.items():
            trees.pop(nm, None)
            t0 = time.perf_counter()
            trees[nm] = lib.tree(pts, a.leafsize, 1.0)
            build[nm].append(time.perf_counter() - t0)
    q = pts[: a.queries]
    rates = {nm: {t: [] for t in a.threads} for nm in libs}
    for t in a.threads:
        for _ in range(a.reps):
            for nm in libs:
                t0 = time.perf_counter()
                trees[nm].query(q, a.k, workers=t)
                rates[nm][t].append(len(q) / (time.perf_counter() - t0))
    med = statistics.median
    out = {
        "n": n, "queries": len(q), "k": a.k, "leafsize": a.leafsize, "periodic": True,
        "host_cpus": os.cpu_count(),
        "build_s": {nm: {"runs": v, "min": min(v), "median": med(v)} for nm, v in build.items()},
        "build_port_over_reference_time": med(build["port"]) / med(build["reference"]),
        "query_qps": {nm: {str(t): {"runs": v, "max": max(v), "median": med(v)}
                           for t, v in r.items()} for nm, r in rates.items()},
        "query_port_over_reference_rate": {
            str(t): med(rates["port"][t]) / med(rates["reference"][t]) for t in a.threads},
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
