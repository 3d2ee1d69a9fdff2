#!/usr/bin/env python3
"""Benchmark of the MI355X kd-tree hot path: batched k=32 kNN self-queries over
1e8 uniform periodic particles (BASELINE.json metric), plus build time.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

One step = one pass of the hot path over one batch: every particle queried
for its k=32 nearest neighbours (query bucketing + radix sort + packet collect /
select kernels), inputs and outputs resident in HBM.  N > 1 (strong scaling by
default: --particles is the total, the same 1e8 points at every N): the
particles are sharded by x-slab, each rank holds its slab plus a periodic halo
exchanged over RCCL at setup, queries its own particles, and the rows whose
k-th neighbour lies past the halo go through the second-round exchange
(slab.second_round) inside the step, so every row is
exact.  --scaling weak: --particles per GPU.

Rank 0 prints ONE JSON line.  Device plumbing goes through the same HIP
runtime as libnbkd (nbodyhpc_amd/hip.py); torch is used only for
torch.distributed (gloo) coordination.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PROFILES = os.path.join(ROOT, "profiles")  # the committed PMC summaries bench.py matches
METRIC = "kNN queries/sec (k=32, 1e8 periodic particles)"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
# Algorithmic bytes per kNN query: B_q = 16*N + 12*P + 12 + 8k,
# N = nodes visited, P = points scanned by the REFERENCE traversal at leafsize 32
# (its KDTreeQueryStatistics), uniform periodic k=32 at 1e8 points: N=61.8, P=307.9.
REF_NODES_1E8, REF_POINTS_1E8 = 61.8, 307.9
# Radius count (C3: 1e8 uniform periodic, r = 0.01 L, leafsize 32): B_r = 16*N + 12*P + 16
# with N, P of the one-query DFS (tests/tools/ref_ball_counters.py --n 1e8: N=175.19, P=1302.53)
REF_BALL_NODES_1E8, REF_BALL_POINTS_1E8 = 175.19, 1302.53


def _phase_frac(st):
    keys = ("clk_walk", "clk_wait", "clk_leaf_test", "clk_dense", "clk_sparse", "clk_tighten")
    tot = sum(st.get(kk, 0) for kk in keys)
    return {kk[4:]: st[kk] / tot for kk in keys} if tot else None


def lib_sha256():
    import hashlib

    from nbodyhpc_amd import capi
    h = hashlib.sha256()
    with open(capi.LIB_PATH, "rb") as f:
        for blk in iter(lambda: f.read(1 << 20), b""):
            h.update(blk)
    return h.hexdigest()


def pmc_traffic(n_particles, k, q_per_launch, kind="knn"):
    """(HBM bytes per launch, source file) from the PMC summary measured with
    this very library build, or (None, None).  kind: "knn" (the collect
    kernel) or "ball" (the C3 radius count, k ignored)."""
    import glob
    sha = lib_sha256()
    if kind == "ball":
        for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_ball.json"))):
            try:
                pm = json.load(open(path))
            except Exception:
                continue
            if pm.get("lib_sha256") == sha and pm.get("n_particles") == n_particles:
                return pm.get("hbm_bytes_per_launch"), os.path.relpath(path, ROOT)
        return None, None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_knn.json"))):
        try:
            pm = json.load(open(path))
        except Exception:
            continue
        if (pm.get("lib_sha256") != sha or pm.get("n_particles") != n_particles
                or pm.get("k") != k or not str(pm.get("kernel", "")).startswith("knn_collect")):
            continue
        # per-query HBM bytes over every first-pass launch of the PMC runs x this
        # run's queries per launch (the batch split follows the free memory)
        if pm.get("hbm_bytes_per_query"):
            return pm["hbm_bytes_per_query"] * q_per_launch, os.path.relpath(path, ROOT)
        if abs(float(pm.get("queries_per_launch") or 0) - q_per_launch) <= 1e-9 * q_per_launch:
            return pm.get("hbm_bytes_per_launch"), os.path.relpath(path, ROOT)
    return None, None


def pmc_step_traffic(n_particles, k):
    """(HBM bytes of one whole kNN step, source file) from a committed
    profiles/r*_pmc_step.json (scripts/gpu_run.sh STEPS=step + summarize_step.py:
    every kernel of the query, the build and warmup differenced out) measured
    with this very library build, or (None, None)."""
    import glob
    sha = lib_sha256()
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_step.json"))):
        try:
            pm = json.load(open(path))
        except Exception:
            continue
        if pm.get("lib_sha256") == sha and pm.get("n_particles") == n_particles and pm.get("k") == k:
            return pm.get("hbm_bytes_per_step"), os.path.relpath(path, ROOT)
    return None, None


def pmc_slab(args, world, k):
    """N > 1: (entry, source) of a committed profiles/r*_pmc_slab.json measured
    with this very library build for this decomposition, or (None, None).
    Each entry is one rank's slab (own particles + halo) profiled alone on one
    GPU by scripts/gpu_run.sh STEPS=slab (scripts/knn_time.py --slab-world N
    --slab-rank r: the same points, halo and ids the bench's rank builds), with
    the HBM bytes per own query of the collect kernel and of the whole step."""
    import glob
    sha = lib_sha256()
    want = {"world": world, "scaling": args.scaling, "n_arg": int(args.n), "k": k,
            "leafsize": args.leafsize, "seed": args.seed}
    for path in sorted(glob.glob(os.path.join(PROFILES, "r*_pmc_slab.json"))):
        try:
            pm = json.load(open(path))
        except Exception:
            continue
        if pm.get("lib_sha256") != sha:
            continue
        for e in pm.get("entries", []):
            if all(e.get(kk) == v for kk, v in want.items()):
                return e, os.path.relpath(path, ROOT)
    return None, None


def slab_roofline(ent, src, world, bq, q_per_launch, own, col_avg_ms, step_sec, allsum, allmax):
    """The whole job's roofline terms at N > 1 (a collective: every rank calls
    it).  Each rank's HBM bytes = its own queries x the bytes per own query of
    its slab's profile (ent, same build and decomposition); the sums over the
    ranks go over the slowest rank's collect launch / step time, against N x the
    per-GPU peak.  Without a profile on every rank the traffic terms are None."""
    have = allsum(1.0 if ent else 0.0) == world
    col_max = allmax(col_avg_ms)
    out = {"kernel_ms": col_max, "peak": HBM_PEAK_GBS * world,
           "work_achieved": allsum(bq * q_per_launch) / (col_max * 1e-3) / 1e9,
           "traffic": None, "step_traffic": None, "step_achieved": None, "source": None,
           "basis": None}
    if not have:
        return out
    out["traffic"] = allsum(ent["collect_bytes_per_query"] * q_per_launch)
    out["step_traffic"] = allsum(ent["step_bytes_per_query"] * own)
    out["step_achieved"] = out["step_traffic"] / step_sec / 1e9
    out["source"] = src
    out["basis"] = (f"sum over the {world} ranks of own queries x HBM bytes per own query of "
                    f"rank {ent['rank']}'s slab (own + halo, {ent['n_local']} points) profiled "
                    f"alone on one GPU (scripts/gpu_run.sh STEPS=slab), over the slowest rank's time, "
                    f"against {world} x {HBM_PEAK_GBS:.0f} GB/s")
    return out


def roofline_entry(traffic, traffic_source, kernel_ms, work_achieved, peak=HBM_PEAK_GBS, **extra):
    """The roofline object of one kernel.  `achieved` / `frac` are HBM
    bandwidth as the counters see it: HBM bytes per launch (rocprofv3 PMC of
    THIS library build: FETCH_SIZE x2 + WRITE_SIZE, each scaled by the
    calibration of this code's access shapes, profiles/*_pmc_calibration.json)
    / the launch's HIP-event duration / 8 TB/s, so frac <= 1.  Without a PMC
    summary of this build both are null.  `work_achieved` / `work_frac` are
    the reference's algorithmic bytes per launch / the same
    duration: a work rate, which exceeds the HBM peak because one staged leaf
    serves 64 queries of a packet."""
    sec = kernel_ms * 1e-3
    ach = None if traffic is None or sec <= 0 else traffic / sec / 1e9
    out = {"bound": "hbm", "achieved": ach, "peak": peak, "unit": "GB/s",
           "frac": None if ach is None else ach / peak,
           "traffic": traffic, "traffic_source": traffic_source,
           "basis": "PMC HBM bytes per launch (calibrated) / HIP-event launch time",
           "work_achieved": work_achieved, "work_frac": work_achieved / peak,
           "kernel_ms_per_launch": kernel_ms}
    out.update(extra)
    return out


def bytes_per_query(k, nodes=REF_NODES_1E8, points=REF_POINTS_1E8):
    return 16.0 * nodes + 12.0 * points + 12.0 + 8.0 * k


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--particles", dest="n", type=float, default=1e8,
                   help="particles: the total over all GPUs (strong scaling, default) or per "
                        "GPU (--scaling weak)")
    p.add_argument("--scaling", choices=("strong", "weak"), default="strong",
                   help="strong: the same --particles points at every N, split by x-slab (the "
                        "metric's 1/2/4/8-GPU curve); weak: --particles per GPU (C4 = --scaling "
                        "weak --particles 1.25e8 at 8 GPUs)")
    p.add_argument("--k", type=int, default=32)
    p.add_argument("--leafsize", type=int, default=64,
                   help="tree leaf size (default 64: the reference _impl.KDTree default, "
                        "kdtree/src/cpp/pybind.cpp:200-205)")
    p.add_argument("--box", type=float, default=1.0)
    p.add_argument("--seed", type=int, default=20261015)
    p.add_argument("--cpu-sample", type=int, default=10_000_000,
                   help="queries timed on the CPU baseline (rank 0, N=1)")
    p.add_argument("--cpu-threads", type=int, default=0,
                   help="CPU baseline workers (default: every core this process may use)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-parity", action="store_true")
    p.add_argument("--suite", action="store_true",
                   help="also measure SURVEY §8(d)'s secondary runs (independent uniform "
                        "queries, C3 radius count + CSR batch, log-normal kNN) into 'suite'")
    p.add_argument("--radius", type=float, default=0.01, help="C3 radius, units of L")
    p.add_argument("--deposit-grid", type=int, default=1024,
                   help="--suite: grid side of the smoothing-radius deposit (0: skip)")
    p.add_argument("--csr-batch", type=int, default=10_000_000)
    p.add_argument("--lognormal-grid", type=int, default=512)
    p.add_argument("--redistribute", action="store_true",
                   help="with --input at N > 1: each rank reads a contiguous row chunk and the "
                        "particles go to their slab owners by all-to-all-v (RCCL), instead of "
                        "every rank scanning the file for its slab")
    p.add_argument("--workload", choices=("knn", "c5"), default="knn",
                   help="knn: the headline line (default).  c5: config C5 - log-normal "
                        "particles sharded at count-quantile x-slabs, radius count at "
                        "--radius plus the k-th-neighbour density, exact over the halo "
                        "(a secondary line, never the headline)")
    p.add_argument("--input", default=None,
                   help="raw float32 (N, 3) particle file (reference main.cpp -f format) "
                        "instead of the synthetic set; N > 1 streams each rank's slab")
    p.add_argument("--launch-probe", action="store_true", help=argparse.SUPPRESS)
    p.add_argument("--probe-rccl-fail", default="", help=argparse.SUPPRESS)
    p.add_argument("--input-format", choices=("raw", "gadget"), default="raw",
                   help="gadget: a Gadget-2 snapshot (format 1/2, multi-file; N > 1 streams each "
                        "rank's slab unless --redistribute); the box is its BoxSize")
    return p.parse_args()


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def gen_uniform(n, seed, box):
    rng = np.random.Generator(np.random.PCG64(seed))
    out = np.empty((n, 3), np.float32)
    chunk = 1 << 24
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        out[s:e] = rng.uniform(0.0, box, size=(e - s, 3))
    return out


# port / reference CPU speed ratios measured in the build container, where the
# compiled reference exists (scripts/cpu_ratio.py -> profiles/r05_cpu_ratio.json,
# 1e7 points, k = 32, periodic, leafsize 64, interleaved runs, medians): the
# single-threaded build and the query rate at 1 and 8 threads
CPU_RATIO_SOURCE = "profiles/r05_cpu_ratio.json"


def cpu_ratio():
    try:
        r = json.load(open(os.path.join(ROOT, CPU_RATIO_SOURCE)))
        return {"source": CPU_RATIO_SOURCE,
                "build_time_port_over_reference": r["build_port_over_reference_time"],
                "query_rate_port_over_reference": r["query_port_over_reference_rate"]}
    except (OSError, KeyError, ValueError):
        return None


def host_cpus():
    """The host cores this process may use: the affinity mask, capped by the
    cgroup CPU quota (a GPU box shares its machine: nproc and os.cpu_count()
    show every CPU of it), plus nproc and the CPU model for the report."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(period)
    except (OSError, ValueError):
        pass
    usable = max(1, min(aff, int(math.ceil(quota)) if quota else aff))
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"usable": usable, "nproc": os.cpu_count(), "affinity": aff, "cgroup_quota": quota,
            "model": model}


def cpu_baseline(points, k, leafsize, box, sample, gpu_d, gpu_i, threads=0):
    """The C restatement of the reference (oracle/liborc.so, pinned bit for bit to
    the reference's own compiled C++ by tests/test_oracle.py; same median-split
    tree, 8-wide leaf scan + loser tree, contiguous-block thread pool), timed on
    this host's cores on a bounded sample: `threads` workers, by default every
    core this process may use (host_cpus; BASELINE.md "workers = nproc").  The
    reference itself does not travel to the GPU box; the
    port/reference speed ratios measured in the build container are reported
    beside it (cpu_ratio)."""
    from oracle.oracle import Oracle
    kind = "port"
    lib = Oracle()
    host = host_cpus()
    cores = threads if threads > 0 else host["usable"]
    t0 = time.perf_counter()
    tree = lib.tree(points, leafsize, box)
    build_s = time.perf_counter() - t0
    q = points[:sample]
    t0 = time.perf_counter()
    d, i = tree.query(q, k, workers=cores)
    query_s = time.perf_counter() - t0
    parity = None
    if gpu_d is not None:
        from tests.parity import assert_knn_equal
        try:
            tie_rows = assert_knn_equal(gpu_d, gpu_i, d, i, points, q, box)
            parity = {"rows": int(sample), "bit_exact_distances": True,
                      "rows_with_tie_order_differences": int(tie_rows)}
        except AssertionError as e:  # reported, never hidden
            parity = {"rows": int(sample), "FAILED": str(e)[:500]}
    return {"value": sample / query_s, "unit": "queries/s", "cores": cores, "kind": kind,
            "sample": f"{sample} self-queries (first {sample} particles) of the same "
                      f"{len(points):.0e}-point periodic tree, k={k}, leafsize={leafsize}, "
                      f"{cores} threads on {host['model']} ({host['usable']} usable of nproc "
                      f"{host['nproc']}); the port's single-threaded CPU build {build_s:.2f} s",
            "host": host, "build_s": build_s}, parity


def cpu_build_entry(build_s):
    r = cpu_ratio()
    out = {"port_ms": build_s * 1e3, "kind": "port", "threads": 1, "ratio": r}
    if r:
        out["reference_estimate_ms"] = build_s * 1e3 / r["build_time_port_over_reference"]
    return out


def gloo_halo() -> bool:
    """NBKD_HALO_TRANSPORT=gloo: stage the (setup-time) halo exchange over gloo
    instead of RCCL, e.g. where RCCL cannot run; the timed step has no collective
    either way."""
    return os.environ.get("NBKD_HALO_TRANSPORT", "rccl").lower() == "gloo"


def rank_report(dist, rank, world, local, same_dev):
    """N > 1: what every rank saw, gathered over gloo so a
    first multi-GPU run can be read from its line alone.  `local` holds this
    rank's numbers (step / collect ms, transports); the RCCL failures come from
    slab.RCCL_ERRORS.  Returns
      rccl_error  every rank's fallback reasons ("rank r: what: message"), or None;
      degraded    True when the ranks sit on distinct devices, gloo was not
                  asked for (NBKD_HALO_TRANSPORT=gloo) and some rank's halo or second
                  round did not run over RCCL;
      per_rank    each key of `local` as a list over the ranks."""
    from nbodyhpc_amd import slab
    mine = dict(local, rccl_errors=list(slab.RCCL_ERRORS))
    got = [None] * world
    dist.all_gather_object(got, mine)
    errs = [e for g in got for e in g["rccl_errors"]]
    tr = [g.get(kk) for g in got for kk in ("halo_transport", "second_round_transport")]
    tr = [t for t in tr if t not in (None, "none")]
    degraded = (not same_dev) and (not gloo_halo()) and any(t != "rccl" for t in tr)
    keys = [kk for kk in local]
    return {"rccl_error": errs or None, "degraded": bool(degraded),
            "per_rank": {kk: [g.get(kk) for g in got] for kk in keys}}


def timed(fn, steps, hip):
    """fn() `steps` times between device synchronisations; seconds per call."""
    hip.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    hip.synchronize()
    return (time.perf_counter() - t0) / steps


def suite(args, capi, hip, tree, dev_pts, n, k, L, stream, od, oi):
    """SURVEY.md §8(d) secondary runs on one GPU (not the headline `value`)."""
    from nbodyhpc_amd import synth
    out = {}
    steps = max(1, min(args.steps, 3))
    # (ii) independent uniform query set of the same size, same tree
    qh = synth.uniform(n, synth.SEED_QUERIES, L)
    dq = hip.DeviceArray.from_numpy(qh)
    del qh
    tree.query_device(dq.ptr, n, k, od.ptr, oi.ptr, stream.handle)
    sec = timed(lambda: tree.query_device(dq.ptr, n, k, od.ptr, oi.ptr, stream.handle), steps, hip)
    out["knn_independent_queries"] = {"queries_per_s": n / sec, "ms": sec * 1e3, "k": k,
                                      "queries": n, "query_seed": synth.SEED_QUERIES}
    log(f"suite: independent queries {n / sec:.3e} q/s")
    # the drop-in surface with host buffers (PCIe-inclusive, never `value`): the
    # same self-queries from a host (n, 3) array into host (n, k) arrays, as
    # KDTree.query returns them; batches of host_batch queries stream through
    # two device slots (query.hip host_pipeline)
    ph = dev_pts.numpy_head(n)
    # the first call of this size pins the two host staging slots (kept by
    # the tree's workspace for later calls): timed apart, as first_call_ms
    t0 = time.perf_counter()
    hd, hi_ = tree.query(ph, k)
    first = time.perf_counter() - t0
    del hd, hi_
    t0 = time.perf_counter()
    hd, hi_ = tree.query(ph, k)
    sec = time.perf_counter() - t0
    ok = bool(np.array_equal(hd[:, 0], np.zeros(n, np.float32)))
    out["knn_host_to_host"] = {"queries_per_s": n / sec, "ms": sec * 1e3, "k": k, "queries": n,
                               "first_call_ms": first * 1e3,
                               "output_bytes": int(hd.nbytes + hi_.nbytes),
                               "output_GBps": (hd.nbytes + hi_.nbytes) / sec / 1e9,
                               "self_distance_zero": ok}
    del hd, hi_, ph
    log(f"suite: host-to-host kNN {n / sec:.3e} q/s")
    # the same self-queries over a leafsize-128 tree (the reference wrapper's
    # default, kdtree/src/python/nbodyhpc/kdtree/__init__.py:17): 65..128-point
    # leaves are staged as two halves with their own tight boxes
    if args.leafsize != 128:
        t128 = capi.Tree(n=n, dev_ptr=dev_pts.ptr, leafsize=128, boxsize=L, stream=stream.handle)
        t128.query_device(dev_pts.ptr, n, k, od.ptr, oi.ptr, stream.handle)
        capi.timing_reset()
        capi.timing_enable(True)
        sec = timed(lambda: t128.query_device(dev_pts.ptr, n, k, od.ptr, oi.ptr, stream.handle),
                    steps, hip)
        br = {nm: capi.timing_read(nm)[0] / steps for nm in
              ("self_order", "leaf_key", "sort", "knn_collect", "knn_select", "knn_retry")}
        capi.timing_enable(False)
        out["knn_leafsize128"] = {"queries_per_s": n / sec, "ms": sec * 1e3, "k": k,
                                  "queries": n, "breakdown_ms": br}
        if not args.no_parity:
            rows = min(1_000_000, n)
            _, parity = cpu_baseline(dev_pts.numpy_head(n), k, 128, L, rows,
                                     od.numpy_head(rows), oi.numpy_head(rows))
            out["knn_leafsize128"]["parity_vs_cpu"] = parity
        t128.close()
        log(f"suite: leafsize 128 {n / sec:.3e} q/s")
    # kNN with k = 100 (scipy-style callers): the wave-per-query select path
    k2 = 100
    od2 = hip.DeviceArray((n, k2), np.float32)
    oi2 = hip.DeviceArray((n, k2), np.uint32)
    tree.query_device(dev_pts.ptr, n, k2, od2.ptr, oi2.ptr, stream.handle)
    capi.timing_reset()
    capi.timing_enable(True)
    sec = timed(lambda: tree.query_device(dev_pts.ptr, n, k2, od2.ptr, oi2.ptr, stream.handle),
                steps, hip)
    br = {nm: capi.timing_read(nm)[0] / steps for nm in
          ("self_order", "leaf_key", "sort", "knn_collect", "knn_select", "knn_retry",
           "knn_fallback")}
    capi.timing_enable(False)
    out["knn_k100"] = {"queries_per_s": n / sec, "ms": sec * 1e3, "k": k2, "queries": n,
                       "breakdown_ms": br}
    if not args.no_parity:
        rows = min(200_000, n)
        _, parity = cpu_baseline(dev_pts.numpy_head(n), k2, args.leafsize, L, rows,
                                 od2.numpy_head(rows), oi2.numpy_head(rows))
        out["knn_k100"]["parity_vs_cpu"] = parity
    od2.free()
    oi2.free()
    log(f"suite: k=100 {n / sec:.3e} q/s")
    # k-th neighbour distance only (densities / smoothing radii): same search,
    # m floats out instead of the (m, k) rows
    rk = hip.DeviceArray((n,), np.float32)
    tree.query_kth_device(dev_pts.ptr, n, k, rk.ptr, stream.handle)
    sec = timed(lambda: tree.query_kth_device(dev_pts.ptr, n, k, rk.ptr, stream.handle), steps, hip)
    out["knn_kth_distance_only"] = {"queries_per_s": n / sec, "ms": sec * 1e3, "k": k,
                                    "queries": n}
    log(f"suite: k-th distance only {n / sec:.3e} q/s")
    # those k-th distances as smoothing radii, deposited
    # onto a G^3 periodic grid (render_points_volume semantics, S = 4)
    if args.deposit_grid > 0:
        G = args.deposit_grid
        wd = hip.DeviceArray.from_numpy(np.full(n, 1.0 / n, np.float32))
        gd = hip.DeviceArray((G, G, G), np.float32)

        def dep():
            capi.deposit_device(dev_pts.ptr, wd.ptr, rk.ptr, n, (G, G, G), G / L, gd.ptr,
                                period=(L, L, L), stream=stream.handle)
        dep()
        capi.timing_reset()
        capi.timing_enable(True)
        sec = timed(dep, 1, hip)
        parts = {nm: capi.timing_read(nm)[0] for nm in
                 ("deposit_pairs", "deposit_fill", "deposit", "deposit_tiny")}
        capi.timing_enable(False)
        mass, plane = 0.0, G * G
        for s0 in range(0, G, 64):
            blk = np.empty(plane * min(64, G - s0), np.float32)
            hip.memcpy(blk.ctypes.data, gd.ptr + s0 * plane * 4, blk.nbytes, hip.D2H)
            mass += float(blk.sum(dtype=np.float64))
        out["deposit"] = {"balls_per_s": n / sec, "ms": sec * 1e3, "breakdown_ms": parts,
                          "grid": G, "subsample": 4, "radius": f"k={k} neighbour distance",
                          "mass_on_grid": mass, "mass_expected": 1.0}
        log(f"suite: deposit {n / sec:.3e} balls/s on {G}^3, mass {mass:.6f}")
        gd.free()
        wd.free()
    rk.free()
    # C3: radius count of every particle (self-queries), r = 0.01 L
    r = args.radius * L
    cnt = hip.DeviceArray((n,), np.uint32)
    tree.ball_count_device(dev_pts.ptr, n, r, cnt.ptr, stream.handle)
    capi.timing_reset()
    capi.timing_enable(True)
    sec = timed(lambda: tree.ball_count_device(dev_pts.ptr, n, r, cnt.ptr, stream.handle),
                steps, hip)
    kern_ms, _ = capi.timing_read("ball_count")
    capi.timing_enable(False)
    c = cnt.numpy()
    expect = n * 4.0 / 3.0 * math.pi * args.radius ** 3
    out["radius_count"] = {"queries_per_s": n / sec, "ms": sec * 1e3,
                           "kernel_ms": kern_ms / steps, "r": r, "mean_count": float(c.mean()),
                           "expected_mean_count": expect, "queries": n}
    if n == 100_000_000 and abs(args.radius - 0.01) < 1e-12:
        # algorithmic bytes per query / kernel time; work_frac > 1 means the leaves are
        # re-read from cache (the kernel is VALU-bound: profiles/r01k_ball_pmc.txt)
        br = 16.0 * REF_BALL_NODES_1E8 + 12.0 * REF_BALL_POINTS_1E8 + 16.0
        ach = br * n / (kern_ms / steps * 1e-3) / 1e9
        traffic, tsrc = pmc_traffic(n, k, n, kind="ball")
        out["radius_count"]["roofline"] = roofline_entry(
            traffic, tsrc, kern_ms / steps, ach,
            kernel="ball_count2_kernel<periodic> (nbodyhpc_amd/csrc/ball.hip)",
            bytes_per_query=br, queries_per_launch=n)
    log(f"suite: radius count {n / sec:.3e} q/s, mean {c.mean():.1f} (expect {expect:.1f})")
    # C3: CSR of the first 1e7 particles (host in / host out: PCIe-inclusive),
    # rows sorted on the device (NBKD_SORTED), streamed in batches
    # (VERDICT r05 #4): ~4.2e9 ids at r = 0.01, ~17 GB of host output
    b = min(args.csr_batch, n)
    qb = dev_pts.numpy_head(b)
    t0 = time.perf_counter()
    off, idx = tree.ball_csr(qb, r, sorted=True)
    sec = time.perf_counter() - t0
    ok = bool(np.array_equal(np.diff(off.astype(np.int64)), c[:b].astype(np.int64)))
    # a sample of rows: strictly ascending ids
    srt = all(bool(np.all(np.diff(idx[int(off[j]):int(off[j + 1])].astype(np.int64)) > 0))
              for j in range(0, b, max(1, b // 997)))
    out["radius_csr_batch"] = {"queries": b, "ms_host_to_host": sec * 1e3,
                               "queries_per_s": b / sec, "neighbours": int(off[-1]),
                               "ids_GBps": int(off[-1]) * 4 / sec / 1e9, "sorted_rows": True,
                               "counts_match_count_pass": ok, "sampled_rows_ascending": srt}
    log(f"suite: CSR of {b} queries host to host {sec:.2f} s ({int(off[-1])} ids)")
    del off, idx, qb, c
    cnt.free()
    dq.free()
    # C5-style log-normal set at the same N (GRF 512^3, P(k) ~ k^-2), self-queries
    t0 = time.perf_counter()
    lp = synth.lognormal(n, box=L, grid=args.lognormal_grid)
    gen_s = time.perf_counter() - t0
    dl = hip.DeviceArray.from_numpy(lp)
    bt = []
    for _ in range(2):
        hip.synchronize()
        t0 = time.perf_counter()
        lt = capi.Tree(n=n, dev_ptr=dl.ptr, leafsize=args.leafsize, boxsize=L,
                       stream=stream.handle)
        hip.synchronize()
        bt.append((time.perf_counter() - t0) * 1e3)
        if _ == 0:
            lt.close()
    lt.query_device(dl.ptr, n, k, od.ptr, oi.ptr, stream.handle)
    capi.timing_reset()
    capi.timing_enable(True)
    sec = timed(lambda: lt.query_device(dl.ptr, n, k, od.ptr, oi.ptr, stream.handle), steps, hip)
    br = {nm: capi.timing_read(nm)[0] / steps for nm in
          ("self_order", "leaf_key", "sort", "knn_collect", "knn_select", "knn_retry_order",
           "knn_retry", "knn_fallback")}
    capi.timing_enable(False)
    capi.stats_enable(True)
    lt.query_device(dl.ptr, n, k, od.ptr, oi.ptr, stream.handle)
    stream.synchronize()
    st = capi.stats_read_all()
    capi.stats_enable(False)
    out["knn_lognormal"] = {"queries_per_s": n / sec, "ms": sec * 1e3, "build_ms": min(bt),
                            "breakdown_ms": br, "retry_queries": st["retry_queries"],
                            "fallback_queries": st["fallback_queries"],
                            "grid": args.lognormal_grid, "generate_s": gen_s,
                            "seed": synth.SEED_LOGNORMAL}
    if not args.no_parity:
        # the first 1e6 rows (retried queries included) against the compiled
        # reference over the same log-normal points (the checker, not timed)
        rows = min(1_000_000, n)
        _, parity = cpu_baseline(lp, k, args.leafsize, L, rows, od.numpy_head(rows),
                                 oi.numpy_head(rows))
        out["knn_lognormal"]["parity_vs_cpu"] = parity
    del lp
    log(f"suite: log-normal kNN {n / sec:.3e} q/s, build {min(bt):.1f} ms")
    lt.close()
    dl.free()
    return out


def run_c5(args, rank, world, local_rank, dist, same_dev, barrier, allmax, allsum):
    """Config C5: log-normal particles (synth.lognormal_slab,
    the C5 recipe) cut into x-slabs at particle-count quantiles, one halo of
    width max(r, kNN halo) over RCCL, then two timed passes over every own
    particle: the radius count at r (-> count density) and the k-th neighbour
    distance (-> k-NN density).  The halo is widened until no k-th distance
    reaches past it (nbkd_slab_violations); the radius count is exact by
    construction (halo >= r).  Weak scaling: --particles per GPU on average."""
    from nbodyhpc_amd import capi, hip, slab, synth

    n_total = int(args.n) * (world if args.scaling == "weak" else 1)
    k, L = args.k, args.box
    r = args.radius * L
    h_r = slab.ball_halo(r, L)
    h = max(h_r, slab.halo_width(n_total, k, L))
    stream = hip.Stream()
    t0 = time.perf_counter()
    own_xyz, own_ids, bounds = synth.lognormal_slab(n_total, rank, world, box=L,
                                                    grid=args.lognormal_grid, min_width=4 * h)
    gen_s = time.perf_counter() - t0
    own = own_xyz.shape[0]
    ds = None
    if world == 1:
        dev_pts, n_local = hip.DeviceArray.from_numpy(own_xyz), own
    else:
        comm = None if (same_dev or gloo_halo()) else slab.init_comm(dist, rank, world, local_rank, log)
        ds = slab.DeviceSlab(own_xyz, own_ids, rank, world, L, local_rank, dist, comm, log,
                             bounds=bounds)
        ds.exchange(h, stream.handle)
        dev_pts, n_local = ds.xyz, ds.n_local
    del own_xyz, own_ids
    log(f"rank {rank}: {own} own log-normal particles ({n_local} with halo h={h:.4g}), "
        f"generated in {gen_s:.1f} s")

    def build_tree():
        # slab trees split by their points' extent (nbkd_build_ext)
        t = capi.Tree(n=n_local, dev_ptr=dev_pts.ptr, leafsize=args.leafsize, boxsize=L,
                      device=local_rank, stream=stream.handle,
                      extent=None if ds is None else ds.extent())
        if ds is not None:
            t.set_ids(dev_ptr=ds.ids.ptr, stream=stream.handle)
        return t

    build_tree().close()
    hip.synchronize()
    t0 = time.perf_counter()
    tree = build_tree()
    hip.synchronize()
    build_ms = allmax((time.perf_counter() - t0) * 1e3)
    cnt = hip.DeviceArray((max(own, 1),), np.uint32)
    rk = hip.DeviceArray((max(own, 1),), np.float32)

    def radius_step():
        tree.ball_count_device(dev_pts.ptr, own, r, cnt.ptr, stream.handle)

    def kth_step():
        tree.query_kth_device(dev_pts.ptr, own, k, rk.ptr, stream.handle)

    # the k-th distances reaching past the halo go through the second-round
    # exchange inside the timed step: every one is exact
    rows = None if ds is None else slab.DeviceRows(ds, tree, k, kth_ptr=rk.ptr,
                                                   stream=stream.handle)
    sr_acc = {"rows_forwarded": 0, "forwards": 0, "hops": 0, "calls": 0}

    def kth_pass():
        tree.query_kth_device(dev_pts.ptr, own, k, rk.ptr, stream.handle)
        if rows is not None:
            # the forward test enqueued behind the pass, its count read behind
            # an event (no device synchronisation)
            rows.start(*slab.covered_range(bounds, rank, ds.h))
            st = slab.second_round(rows, rank, world, bounds, L, ds.h, k, dist)
            for kk in ("rows_forwarded", "forwards"):
                sr_acc[kk] += st[kk]
            sr_acc["hops"] = max(sr_acc["hops"], st["hops"])
            sr_acc["calls"] += 1

    kth_step = kth_pass
    kth_step()
    stream.synchronize()
    violations = 0 if ds is None else int(allsum(float(sr_acc["rows_forwarded"])))

    def timed_max(fn):
        for _ in range(args.warmup):
            fn()
        barrier()
        hip.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            fn()
        hip.synchronize()
        barrier()
        return allmax(time.perf_counter() - t0)

    t_r = timed_max(radius_step)
    t_k = timed_max(kth_step)
    # density estimates (host, from the last passes), in units of the mean density
    rho_bar = n_total / L ** 3
    c = cnt.numpy_head(own).astype(np.float64)
    d = rk.numpy_head(own).astype(np.float64)
    dens_r = c / (4.0 / 3.0 * math.pi * r ** 3) / rho_bar
    dens_k = k / (4.0 / 3.0 * math.pi * np.maximum(d, 1e-30) ** 3) / rho_bar
    sums = [float(own), float(c.sum()), float(dens_r.sum()), float(dens_k.sum()),
            float(np.log(dens_k).sum())]
    if dist is not None:
        import torch
        t = torch.tensor(sums, dtype=torch.float64)
        dist.all_reduce(t)
        sums = t.tolist()
        counts = [torch.zeros(1, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(counts, torch.tensor([float(own)], dtype=torch.float64))
        per_rank = [int(x.item()) for x in counts]
    else:
        per_rank = [own]
    # collectives on every rank, before rank 0 alone writes the line
    sr_fwd = 0.0 if ds is None else allsum(float(sr_acc["rows_forwarded"])) / max(sr_acc["calls"], 1)
    sr_hops = 0 if ds is None else int(allmax(float(sr_acc["hops"])))
    rep = None if ds is None else rank_report(dist, rank, world, {
        "own_particles": own, "local_points": n_local,
        "halo_transport": ds.transport, "second_round_transport": rows.transport}, same_dev)
    if rank != 0:
        return
    q_total = sums[0] * args.steps
    out = {
        "metric": "C5 radius-count + k-th-neighbour density queries/sec (log-normal)",
        "value": q_total / t_r,
        "unit": "queries/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": t_r / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "f32",
        "data": (f"synthetic: C5 log-normal recipe (GRF {args.lognormal_grid}^3, P(k)~k^-2, "
                 f"sigma_g=1, seed {synth.SEED_LOGNORMAL}), periodic L={L}; self-queries"),
        "config": {
            "workload": (f"C5: radius count r={r:g} and k={k} k-th neighbour distance of every "
                         f"particle, {n_total:.3g} log-normal particles over {world} GPU(s)"),
            "n_particles": int(sums[0]), "particles_per_rank": per_rank, "k": k, "r": r,
            "leafsize": args.leafsize,
            "parallelism": ("single" if world == 1 else
                            f"count-quantile x-slab x{world} + halo over "
                            f"{getattr(ds, 'transport', 'rccl')}"),
        },
        "radius_count": {"queries_per_s": q_total / t_r, "ms_per_step": t_r / args.steps * 1e3,
                         "mean_count": sums[1] / sums[0],
                         "mean_density_over_mean": sums[2] / sums[0]},
        "kth_density": {"queries_per_s": q_total / t_k, "ms_per_step": t_k / args.steps * 1e3,
                        "mean_density_over_mean": sums[3] / sums[0],
                        "geomean_density_over_mean": math.exp(sums[4] / sums[0])},
        "halo": None if ds is None else {
            "h": ds.h, "h_radius": h_r, "transport": ds.transport,
            # k-th distances of the first pass that reached past the halo: each
            # was resolved by the second-round exchange (no rebuild, no widening)
            "kth_rows_past_halo": violations,
            "second_round": {"transport": rows.transport,
                             "rows_forwarded_per_pass": sr_fwd,
                             "max_hops": sr_hops},
            **rep},
        "bounds": bounds,
        "build_ms": build_ms,
        "generate_s": gen_s,
    }
    print(json.dumps(out), flush=True)


def visible_gpus() -> int:
    """GPUs this process may use, counted without initialising the HIP runtime
    (torch.cuda.device_count() does not initialise it on this image)."""
    import torch
    return int(torch.cuda.device_count())


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args) -> int:
    """`python bench.py --gpus N` (N > 1) without a launcher: start the N ranks
    as children (torch.distributed.run, one process per GPU, rendezvous on
    127.0.0.1) before this process touches the GPU, and exit with their exit
    code; rank 0's JSON line reaches stdout through the inherited descriptor.
    Never execs: the parent only waits.  With fewer visible GPUs than N it
    fails, unless NBKD_BENCH_SAME_DEVICE=1 (every rank on GPU 0: a rehearsal of
    the N > 1 path on a one-GPU box)."""
    import subprocess
    same_dev = os.environ.get("NBKD_BENCH_SAME_DEVICE") == "1"
    if not same_dev and not args.launch_probe:
        have = visible_gpus()
        if have < args.gpus:
            log(f"error: --gpus {args.gpus} but only {have} GPU(s) visible; refusing to "
                f"report an N={args.gpus} line from fewer GPUs (NBKD_BENCH_SAME_DEVICE=1 "
                f"rehearses N ranks on GPU 0)")
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1",
           f"--master-port={free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    log("starting ranks: " + " ".join(cmd))
    sys.stdout.flush()
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "16")
    return subprocess.call(cmd, env=env)


def init_gloo(rank, world):
    import torch.distributed as dist  # gloo: CPU-side coordination only
    # gloo prints "[Gloo] Rank r is connected to ..." on stdout (C++, every
    # rank): stdout carries only rank 0's JSON line, so send it to stderr
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    finally:
        os.dup2(saved, 1)
        os.close(saved)
    return dist


def launch_probe(rank, world, dist, fail_rccl=()):
    """--launch-probe (tests): the ranks meet over gloo and rank 0 prints one
    JSON line naming them; no GPU is touched.  --probe-rccl-fail R,..: those
    ranks' RCCL probe fails (a forced failure: slab.init_comm with a probe
    that raises), and the line carries the N > 1 report fields the bench line
    would (rank_report: rccl_error, degraded, per-rank numbers)."""
    import torch
    from nbodyhpc_amd import slab
    out = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(out, torch.tensor([rank], dtype=torch.int64))

    def probe():
        if rank in fail_rccl:
            raise RuntimeError("forced RCCL failure (launch probe)")

    slab.init_comm(dist, rank, world, None, probe=probe)  # None: a probe starts no communicator
    # every rank holds the same list: with a failure every rank stages over gloo
    transport = "gloo-staged" if fail_rccl else "rccl"
    rep = rank_report(dist, rank, world, {"step_ms": 1.0 + rank, "collect_ms": 0.5 + rank,
                                          "halo_transport": transport,
                                          "second_round_transport": transport}, False)
    if rank == 0:
        print(json.dumps({"n_gpus": world, "ranks": [int(x.item()) for x in out],
                          "launch_probe": True, "halo": rep}), flush=True)


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE")
    if args.launch_probe:
        dist = init_gloo(rank, world)
        fail = [int(x) for x in args.probe_rccl_fail.split(",") if x != ""]
        launch_probe(rank, world, dist, fail)
        dist.destroy_process_group()
        return
    from nbodyhpc_amd import capi, hip

    hip.preload()  # before torch: see hip.preload
    dist = None
    if world > 1:
        dist = init_gloo(rank, world)
    # rehearsal of the N > 1 path on a one-GPU box: every rank on device 0 and
    # the halo staged over gloo (RCCL needs one GPU per rank)
    same_dev = os.environ.get("NBKD_BENCH_SAME_DEVICE") == "1"
    if same_dev:
        local_rank = 0
    hip.set_device(local_rank)

    def barrier():
        if dist is not None:
            dist.barrier()

    def allsum(v):
        if dist is None:
            return v
        import torch
        t = torch.tensor([v], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return float(t.item())

    def allgather_int(v):
        if dist is None:
            return [int(v)]
        import torch
        out = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(out, torch.tensor([int(v)], dtype=torch.int64))
        return [int(x.item()) for x in out]

    def allmax(v):
        if dist is None:
            return v
        import torch
        t = torch.tensor([v], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    if args.workload == "c5":
        return run_c5(args, rank, world, local_rank, dist, same_dev, barrier, allmax, allsum)

    n = int(args.n)
    k, L = args.k, args.box
    gadget = None
    if args.input and args.input_format == "gadget":
        from nbodyhpc_amd import io as nio
        if world == 1 or args.redistribute:
            gadget, _, gh = nio.read_gadget(args.input, ids=False)
        else:  # each rank streams its own slab (read_gadget_slab below)
            gh = nio._gadget_pos_blocks(args.input)[1]
        L = float(gh["BoxSize"])
    stream = hip.Stream()
    t_gen = time.perf_counter()
    ds = None
    halo = None
    if world == 1:
        if gadget is not None:
            points, gadget = gadget, None
            n = points.shape[0]
        elif args.input:
            from nbodyhpc_amd import io as nio
            points = nio.read_positions(args.input, mmap=False)
            n = points.shape[0]
        else:
            points = gen_uniform(n, args.seed, L)
        own = n
        dev_pts = hip.DeviceArray.from_numpy(points)
        n_local = n
    else:
        from nbodyhpc_amd import slab
        points = None
        comm = None if (same_dev or gloo_halo()) else slab.init_comm(dist, rank, world, local_rank, log)
        if args.input and args.redistribute:
            # each rank reads its contiguous row chunk; all-to-all-v to the owners
            from nbodyhpc_amd import io as nio
            rows = gadget if gadget is not None else nio.read_positions(args.input)
            lo_r, hi_r = rank * rows.shape[0] // world, (rank + 1) * rows.shape[0] // world
            own_xyz, own_ids = slab.redistribute(
                np.array(rows[lo_r:hi_r]), np.arange(lo_r, hi_r, dtype=np.uint32), rank, world,
                L, dist, comm=comm, device=local_rank, log=log)
            del rows
        elif args.input and args.input_format == "gadget":
            from nbodyhpc_amd import io as nio
            own_xyz, own_ids, _ = nio.read_gadget_slab(args.input, rank, world, L)
        elif args.input:
            from nbodyhpc_amd import io as nio
            own_xyz, own_ids = nio.read_slab(args.input, rank, world, L)
        elif args.scaling == "strong":  # the one-GPU point set, cut into slabs
            own_xyz, own_ids = slab.gen_uniform_slab(n, args.seed, L, rank, world)
        else:
            own_xyz, own_ids = slab.gen_slab_points(n, args.seed, L, rank, world)
        own = own_xyz.shape[0]
        ds = slab.DeviceSlab(own_xyz, own_ids, rank, world, L, local_rank, dist, comm, log)
        del own_xyz, own_ids
        h = slab.halo_width(int(allsum(float(own))), k, L)  # file inputs: the real total
        barrier()
        t_x = time.perf_counter()
        ds.exchange(h, stream.handle)
        barrier()
        halo = {"h": h, "exchange_ms": (time.perf_counter() - t_x) * 1e3}
        dev_pts, n_local = ds.xyz, ds.n_local
    log(f"rank {rank}: {own} own particles ({n_local} with halo) ready in "
        f"{time.perf_counter() - t_gen:.1f} s")

    def build_tree():
        # slab trees split by their points' extent (nbkd_build_ext)
        t = capi.Tree(n=n_local, dev_ptr=dev_pts.ptr, leafsize=args.leafsize, boxsize=L,
                      device=local_rank, stream=stream.handle,
                      extent=None if ds is None else ds.extent())
        if ds is not None:
            t.set_ids(dev_ptr=ds.ids.ptr, stream=stream.handle)
        return t

    # build: one untimed (code-object load; also the process's first build,
    # which pays the shape enumeration and the allocations the later builds
    # reuse), then timed rebuilds of the same size
    hip.synchronize()
    t0 = time.perf_counter()
    build_tree().close()
    hip.synchronize()
    build_ms_first = allmax((time.perf_counter() - t0) * 1e3)
    build_ms = []
    for _ in range(2):
        hip.synchronize()
        t0 = time.perf_counter()
        tree = build_tree()
        hip.synchronize()
        build_ms.append((time.perf_counter() - t0) * 1e3)
        if _ == 0:
            tree.close()
    build_ms = allmax(min(build_ms))

    # N > 1: two row buffers, so a step's second round overlaps the next step
    bufs = [(hip.DeviceArray((own, k), np.float32), hip.DeviceArray((own, k), np.uint32))
            for _ in range(1 if ds is None else 2)]
    od, oi = bufs[0]

    # N > 1: rows whose k-th neighbour lies past the halo are forwarded to the
    # neighbours and merged (second-round exchange) inside
    # every step, so every row of every step is exact; no rebuild, no widening
    # the rows' k-th distances beside them (nbkd_set_kth_out): the forward test
    # reads 4 B per own row instead of each row's last line
    side = None if ds is None else hip.DeviceArray((own,), np.float32)
    if side is not None:
        tree.set_kth_out(side.ptr, own)
    rows_b = None if ds is None else [slab.DeviceRows(ds, tree, k, b[0].ptr, b[1].ptr,
                                                      stream=stream.handle,
                                                      side_ptr=side.ptr) for b in bufs]
    rows = None if rows_b is None else rows_b[0]
    cover = None if ds is None else slab.covered_range(ds.bounds, rank, ds.h)
    sr_acc = {"rows_forwarded": 0, "forwards": 0, "hops": 0, "calls": 0, "host_s": 0.0}

    counters = {"timing": False, "stats": False}
    pipe = {"cur": 0, "pending": None, "last": 0}

    def resolve(j):
        # the second round's small host-in kNN calls stay out of the kernel
        # timers and work counters (they describe the slab-local pass); its
        # time is in the step's wall clock
        capi.timing_enable(False)
        capi.stats_enable(False)
        rows_b[j].wait()  # the count is behind that step's kNN: not the round's own time
        t_r = time.perf_counter()
        st = slab.second_round(rows_b[j], rank, world, ds.bounds, L, ds.h, k, dist)
        sr_acc["host_s"] += time.perf_counter() - t_r
        capi.timing_enable(counters["timing"])
        capi.stats_enable(counters["stats"])
        for kk in ("rows_forwarded", "forwards"):
            sr_acc[kk] += st[kk]
        sr_acc["hops"] = max(sr_acc["hops"], st["hops"])
        sr_acc["calls"] += 1

    def step():
        j = pipe["cur"]
        tree.query_device(dev_pts.ptr, own, k, bufs[j][0].ptr, bufs[j][1].ptr, stream.handle)
        pipe["last"] = j
        if ds is None:
            return
        # the forward test and its count are enqueued behind this step's kNN;
        # the previous step's second round (its count agreed over gloo, and
        # any forwarded rows) runs while this step computes on the device
        rows_b[j].start(*cover)
        if pipe["pending"] is not None:
            resolve(pipe["pending"])
        pipe["pending"], pipe["cur"] = j, 1 - j

    def drain():
        if pipe["pending"] is not None:
            resolve(pipe["pending"])
            pipe["pending"] = None

    for _ in range(args.warmup):
        step()
    drain()
    stream.synchronize()
    if ds is not None:
        # the slab-local rows before the second round: how many reach past the halo
        tree.query_device(dev_pts.ptr, own, k, od.ptr, oi.ptr, stream.handle)
        stream.synchronize()
        halo["rows_past_halo_before_second_round"] = int(
            allsum(float(ds.violations(od.ptr, k, stream.handle))))
        step()  # and resolved again, so the checked rows below are the exact ones
        drain()
        stream.synchronize()
        halo.update({"h": ds.h, "local_points": n_local, "transport": ds.transport})
        for kk in sr_acc:
            sr_acc[kk] = 0
    capi.timing_enable(True)
    counters["timing"] = True
    capi.timing_reset()
    barrier()
    hip.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    drain()
    hip.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    sr_timed = dict(sr_acc)
    od, oi = bufs[pipe["last"]]  # the last step's (exact) rows
    knn_ms, knn_launches = capi.timing_read("knn")
    sort_ms, _ = capi.timing_read("sort")
    key_ms, _ = capi.timing_read("leaf_key")
    self_ms, _ = capi.timing_read("self_order")
    oob_ms, _ = capi.timing_read("knn_outside_box")
    fb_ms, _ = capi.timing_read("knn_fallback")
    rt_ms, _ = capi.timing_read("knn_retry")
    rto_ms, _ = capi.timing_read("knn_retry_order")
    col_ms, col_launches = capi.timing_read("knn_collect")
    sel_ms, _ = capi.timing_read("knn_select")
    capi.timing_enable(False)
    counters["timing"] = False
    elapsed_max = allmax(elapsed)
    own_total = int(allsum(float(own)))  # file inputs: slabs differ in size

    # work counters of our own traversal (one extra, untimed pass)
    capi.stats_enable(True)
    counters["stats"] = True
    step()
    stream.synchronize()
    st = capi.stats_read_all()
    pts_scanned = st["pair_evals"]
    capi.stats_enable(False)
    counters["stats"] = False
    drain()  # that step's second round: its rows are the exact ones read below
    stream.synchronize()
    od, oi = bufs[pipe["last"]]

    gpu_d = gpu_i = None
    parity_rows = min(args.cpu_sample, own)
    if rank == 0 and not args.no_parity:
        gpu_d = od.numpy_head(parity_rows)
        gpu_i = oi.numpy_head(parity_rows)

    if ds is not None:
        # the same steps without the second round (rows then inexact, never
        # reported): what the round adds to a step, on the same (possibly
        # shared) device
        barrier()
        hip.synchronize()
        t_k = time.perf_counter()
        for _ in range(args.steps):
            tree.query_device(dev_pts.ptr, own, k, bufs[0][0].ptr, bufs[0][1].ptr, stream.handle)
        hip.synchronize()
        barrier()
        knn_only_local = (time.perf_counter() - t_k) / args.steps
        knn_only = allmax(knn_only_local * args.steps) / args.steps
        halo["second_round"] = {
            "transport": rows.transport,
            "rows_forwarded_per_step": allsum(float(sr_timed["rows_forwarded"])) / max(args.steps, 1),
            "forwards_per_step": allsum(float(sr_timed["forwards"])) / max(args.steps, 1),
            "max_hops": int(allmax(float(sr_timed["hops"]))),
            # overlapped with the next step's kNN (pipelined steps); the host's
            # time in it once the count is known (agreement over gloo, any
            # forwarded rows), and the step time over the same steps without it
            "host_ms_per_step": allmax(sr_timed["host_s"]) / args.steps * 1e3,
            "ms_per_step": (elapsed_max / args.steps - knn_only) * 1e3,
            "knn_only_ms_per_step": knn_only * 1e3,
        }
        counts = allgather_int(own)
        # every rank's own numbers beside the max-over-ranks step (VERDICT r05
        # #6: set them against profiles/r05ao_slab_ranks.txt's per-rank steps)
        halo.update(rank_report(dist, rank, world, {
            "step_ms": elapsed / args.steps * 1e3,
            "collect_ms_per_launch": col_ms / max(col_launches, 1),
            "select_ms_per_step": sel_ms / args.steps,
            "knn_only_ms_per_step": knn_only_local * 1e3,
            "second_round_host_ms_per_step": sr_timed["host_s"] / args.steps * 1e3,
            "own_particles": own, "local_points": n_local,
            "halo_transport": ds.transport, "second_round_transport": rows.transport},
            same_dev))
    else:
        counts = [own]
    total_q = own_total * args.steps
    value = total_q / elapsed_max
    ms_per_step = elapsed_max / args.steps * 1e3
    bq = bytes_per_query(k)
    # dominant kernel: the collect kernel (knn_collect_grp_kernel), launched once
    # per query batch (the candidate-column budget); achieved = algorithmic bytes
    # of the queries one launch processes / that launch's average duration (HIP
    # events on the launch stream)
    col_launches = max(col_launches, 1)
    col_avg_ms = col_ms / col_launches
    q_per_launch = own * args.steps / col_launches
    achieved = bq * q_per_launch / (col_avg_ms * 1e-3) / 1e9
    # HBM bytes per collect launch from rocprofv3 PMC passes of THIS build: a
    # committed profiles/rNN_pmc_knn.json (scripts/summarize_prof.py: FETCH_SIZE
    # x2 (gfx950) + WRITE_SIZE, separate runs) whose recorded libnbkd.so SHA-256
    # equals the loaded library's, for the same workload; else null
    traffic, traffic_source = pmc_traffic(own, k, q_per_launch)
    # the whole step's HBM bytes (every kernel of the query), same build, one GPU
    step_traffic, step_source = pmc_step_traffic(own, k) if world == 1 else (None, None)
    step_sec = elapsed_max / args.steps
    useful = float(own_total) * k * 8 + 16.0 * (own_total if world == 1 else allsum(float(n_local))) \
        + 16.0 * (tree.size if world == 1 else allsum(float(tree.size)))
    step_ach = None if step_traffic is None else step_traffic / step_sec / 1e9
    peak = HBM_PEAK_GBS
    basis = None
    if world > 1:
        ent, src = pmc_slab(args, world, k)
        sr = slab_roofline(ent, src, world, bq, q_per_launch, own, col_avg_ms, step_sec,
                           allsum, allmax)
        traffic, step_traffic = sr["traffic"], sr["step_traffic"]
        traffic_source = step_source = sr["source"]
        achieved, col_avg_ms, step_ach = sr["work_achieved"], sr["kernel_ms"], sr["step_achieved"]
        peak, basis = sr["peak"], sr["basis"]
    if rank != 0:
        return
    extra = None
    if world == 1 and args.suite:
        extra = suite(args, capi, hip, tree, dev_pts, n, k, L, stream, od, oi)
    cpu = None
    parity = None
    if world == 1 and not args.no_cpu_baseline:
        cpu, parity = cpu_baseline(points, k, args.leafsize, L, parity_rows, gpu_d, gpu_i,
                                   threads=args.cpu_threads)
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "queries/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "f32",
        "data": (f"file: {os.path.basename(args.input)} ({args.input_format}); self-queries"
                 if args.input else
                 "synthetic: numpy PCG64 uniform [0,L)^3, L=1, float32; self-queries"),
        "config": {
            "workload": (f"kNN k={k} self-query of every particle of {os.path.basename(args.input)}"
                         f" ({own_total} particles, periodic L={L}), leafsize {args.leafsize}"
                         if args.input else
                         f"kNN k={k} self-query of every particle, {own_total:.3g} uniform "
                         f"periodic particles{' per GPU' if args.scaling == 'weak' else ''} "
                         f"(L={L}), leafsize {args.leafsize}"),
            "n_particles": own_total, "n_particles_per_gpu": own, "particles_per_rank": counts,
            "k": k, "leafsize": args.leafsize,
            "queries_per_step": own_total,
            "parallelism": ("single" if world == 1 else
                            f"x-slab x{world} + halo over {(halo or {}).get('transport', 'rccl')}"),
        },
        "halo": halo,
        "build_ms": build_ms,
        "build_ms_first": build_ms_first,
        "roofline": roofline_entry(
            traffic, traffic_source, col_avg_ms, achieved, peak=peak,
            kernel="knn_collect_grp_kernel<periodic> (nbodyhpc_amd/csrc/knn_collect.hip)",
            step_work_frac=value * bq / (HBM_PEAK_GBS * 1e9 * world),
            launches_per_step=col_launches / args.steps, queries_per_launch=q_per_launch,
            bytes_per_query=bq, peak_per_gpu=HBM_PEAK_GBS, traffic_basis=basis,
            # the whole pipeline (bucketing, sort, collect, select, retries):
            # PMC HBM bytes of one step / the step's wall time
            step_traffic=step_traffic, step_traffic_source=step_source,
            step_achieved=step_ach,
            step_frac=None if step_ach is None else step_ach / peak,
            # the bytes a step cannot avoid: the k-column rows
            # written (f32 + u32), the packed points read once (16 B) and the
            # node table (16 B per node); the step's PMC traffic over this is
            # the step's waste factor
            useful_bytes=useful,
            useful_frac_of_step_traffic=None if step_traffic is None else useful / step_traffic,
            useful_achieved=useful / step_sec / 1e9),
        "breakdown_ms_per_step": {
            "self_order": self_ms / args.steps, "leaf_key": key_ms / args.steps,
            "sort": sort_ms / args.steps, "knn": knn_ms / args.steps, "knn_collect": col_ms / args.steps,
            "knn_select": sel_ms / args.steps, "outside_box_check": oob_ms / args.steps,
            "retry": (rt_ms + rto_ms) / args.steps, "fallback": fb_ms / args.steps,
        },
        # one packet = 64 queries walking the tree together: node visits are
        # per packet walk; distance evaluations are per (query, point) pair
        "traversal_per_query": {"distance_evals": pts_scanned / own,
                                "candidates": st["candidates"] / own},
        "traversal_per_packet": {kk: st[kk] / max(st["packets"], 1)
                                 for kk in ("node_visits", "leaves_reached", "sparse_iters",
                                            "points_staged", "candidates", "leaves_scanned")},
        "lanes_per_scanned_chunk": st["chunk_lanes"] / max(st["leaves_scanned"], 1),
        "fallback_queries": st["fallback_queries"], "retry_queries": st["retry_queries"],
        # where a collect wave's cycles go (work-counter pass, s_memtime clocks)
        "collect_phase_frac": _phase_frac(st),
        "cpu_baseline": None if cpu is None else dict(
            {kk: cpu[kk] for kk in ("value", "unit", "cores", "kind", "sample")},
            port_over_reference=cpu_ratio()),
        "cpu_build_ms": None if cpu is None else cpu["build_s"] * 1e3,
        # the port's build selects with a scalar partition where the reference
        # runs its AVX2 one: the measured build-time ratio scales it to the
        # reference's (an estimate; the reference cannot run on the GPU box)
        "cpu_build": None if cpu is None else cpu_build_entry(cpu["build_s"]),
        "cpu_host": None if cpu is None else cpu["host"],
        "parity_vs_cpu": parity,
    }
    if extra is not None:
        out["suite"] = extra
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
