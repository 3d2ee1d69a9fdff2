"""Turn one gpu_run.sh output directory (steps trace, pmc) into the committed profile summaries.

    python scripts/summarize_prof.py gpurun_out/<tag> <round-tag>

writes
  profiles/<round>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (copied)
  profiles/<round>_launches.json      per-launch durations of the kNN / radius kernels by
                                      grid size (full-size collect launches vs retries)
  profiles/<round>_pmc_knn.json       HBM bytes per knn launch from the FETCH_SIZE and
                                      WRITE_SIZE passes (separate runs), gfx950-corrected
  profiles/<round>_bench.json         the bench line of the same call
FETCH_SIZE / WRITE_SIZE are rocprofv3 derived counters in KiB, calibrated on this
code's access shapes by scripts/calib/pmc_calib.hip (profiles/r04a_pmc_calibration.json):
FETCH_SIZE reports exactly half the bytes of every read shape measured (16-B and
4-B per lane loads, 4-B global_load_lds), so fetched bytes = 2 * 1024 * FETCH_SIZE;
WRITE_SIZE reports full-line stores exactly at any width (16, 8 or 4 B per lane:
the select kernel's row stores) and a partly written 128-B line as 32-B sectors
(one 8-B or 4-B store alone in a line counts 32 B), i.e. the bytes the L2
actually writes back, so it is taken as reported: the collect kernel's candidate
columns show their sector write-amplification in it, not an undercount.
"""
import csv
import glob
import json
import os
import shutil
import sys


def find(d, pat):
    hits = sorted(glob.glob(os.path.join(d, "**", pat), recursive=True))
    return hits[-1] if hits else None


def _stats_instance(name):
    """knn_collect_grp_kernel<PER, OCC, STATS, LOOP, AHEAD>: STATS is the third
    template argument (the work-counter instance; its timing and traffic are not
    the production kernel's)."""
    if "knn_collect_grp_kernel<" not in name:
        return False
    args = name.split("knn_collect_grp_kernel<", 1)[1].split(">", 1)[0].split(",")
    return len(args) >= 3 and args[2].strip() == "true"


def per_dispatch(path, regex):
    """Counter sum per dispatch of the full-size launches of the kernel (the
    work-counter instance and the small retry launches are left out)."""
    vals, grid = {}, {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if regex not in row["Kernel_Name"]:
                continue
            if _stats_instance(row["Kernel_Name"]):  # the work-counter (STATS) instance
                continue
            key = row["Dispatch_Id"]
            vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
            grid[key] = int(row["Grid_Size"])
    gmax = max(grid.values())
    return [v for kk, v in vals.items() if grid[kk] == gmax]


def per_query(path, regex):
    """(counter sum, grid sum) over the first-pass launches of the kernel: the
    production instance (not STATS, not the LOOP retry instance), grids of at
    least 1 M threads (one query per thread).  The launch split depends on the
    free memory at the call, so bytes are kept per query."""
    vals, grid = {}, {}
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row["Kernel_Name"]
            if regex not in name or _stats_instance(name):
                continue
            if "knn_collect_grp_kernel<" in name:
                args = name.split("knn_collect_grp_kernel<", 1)[1].split(">", 1)[0].split(",")
                if len(args) >= 4 and args[3].strip() == "true":  # LOOP: retry rounds
                    continue
            if int(row["Grid_Size"]) < (1 << 20):
                continue
            key = row["Dispatch_Id"]
            vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
            grid[key] = int(row["Grid_Size"])
    return sum(vals.values()), sum(grid.values())


def main():
    src, tag = sys.argv[1], sys.argv[2]
    regex = sys.argv[3] if len(sys.argv) > 3 else "knn_collect"
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prof = os.path.join(root, "profiles")
    stats = find(os.path.join(src, "trace"), "*kernel_stats.csv")
    if stats:
        shutil.copy(stats, os.path.join(prof, f"{tag}_kernel_stats.csv"))
    trace = find(os.path.join(src, "trace"), "*kernel_trace.csv")
    if trace:
        # the stats summary averages every launch of a kernel; the collect
        # kernel also runs small retry launches, so list the per-launch
        # durations by (kernel, grid size): the full-size rows are what the
        # bench's roofline.kernel_ms_per_launch measures with HIP events
        launches = {}
        with open(trace) as f:
            for row in csv.DictReader(f):
                name = row["Kernel_Name"]
                if not any(r in name for r in (regex, "knn_select", "ball_count2")):
                    continue
                key = (name[:120], int(row["Grid_Size_X"]))
                ms = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-6
                launches.setdefault(key, []).append(ms)
        rows = [{"kernel": k[0], "grid_size": k[1], "launches": len(v),
                 "avg_ms": sum(v) / len(v), "min_ms": min(v), "max_ms": max(v)}
                for k, v in sorted(launches.items(), key=lambda kv: -kv[0][1])]
        json.dump(rows, open(os.path.join(prof, f"{tag}_launches.json"), "w"), indent=1)
    bench = os.path.join(src, "bench.json")
    b = None
    if os.path.exists(bench) and os.path.getsize(bench) > 0:
        b = json.loads(open(bench).read().strip().splitlines()[-1])
        json.dump(b, open(os.path.join(prof, f"{tag}_bench.json"), "w"), indent=1)
    fetch = find(os.path.join(src, "fetch"), "*counter_collection.csv")
    write = find(os.path.join(src, "write"), "*counter_collection.csv")
    if fetch and write:
        fv = per_dispatch(fetch, regex)
        wv = per_dispatch(write, regex)
        f_kib = sum(fv) / len(fv)
        w_kib = sum(wv) / len(wv)
        hbm = 2.0 * 1024.0 * f_kib + 1024.0 * w_kib
        fs, fg = per_query(fetch, regex)
        ws_, wg = per_query(write, regex)
        bpq = (2.0 * 1024.0 * fs / fg + 1024.0 * ws_ / wg) if fg and wg else None
        cfg = (b or {}).get("config", {})
        shaf = os.path.join(src, "lib.sha256")
        lib_sha = open(shaf).read().split()[0] if os.path.exists(shaf) else None
        out = {
            # the libnbkd.so these counters were measured with (bench.py uses the
            # file only when the loaded library has the same SHA-256)
            "lib_sha256": lib_sha,
            "kernel": (b or {}).get("roofline", {}).get("kernel", regex),
            "command": f"rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE --kernel-include-regex {regex} -- "
                       "python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity",
            "n_particles": cfg.get("n_particles_per_gpu", 100_000_000), "k": cfg.get("k", 32),
            "queries_per_launch": (b or {}).get("roofline", {}).get("queries_per_launch"),
            "dispatches": [len(fv), len(wv)],
            "FETCH_SIZE_KiB_per_launch": f_kib, "WRITE_SIZE_KiB_per_launch": w_kib,
            "fetch_bytes_per_launch_corrected": 2.0 * 1024.0 * f_kib,
            "write_bytes_per_launch": 1024.0 * w_kib,
            "hbm_bytes_per_launch": hbm,
            # over every first-pass launch of the runs (any batch split): bench.py
            # multiplies it by the queries of its own launches
            "hbm_bytes_per_query": bpq,
            "queries_in_passes": [fg, wg],
            "note": "FETCH_SIZE doubled, WRITE_SIZE as reported (calibration: "
                    "profiles/r04a_pmc_calibration.json); Infinity-Cache hits are counted "
                    "by these counters, not excluded",
        }
        json.dump(out, open(os.path.join(prof, f"{tag}_pmc_knn.json"), "w"), indent=1)
        print(json.dumps(out, indent=1))
    # the C3 radius count's passes (scripts/ball_run.py under rocprofv3)
    bf = find(os.path.join(src, "ball_fetch"), "*counter_collection.csv")
    bw = find(os.path.join(src, "ball_write"), "*counter_collection.csv")
    if bf and bw:
        fv = per_dispatch(bf, "ball_count2")
        wv = per_dispatch(bw, "ball_count2")
        f_kib, w_kib = sum(fv) / len(fv), sum(wv) / len(wv)
        shaf = os.path.join(src, "lib.sha256")
        out = {
            "lib_sha256": open(shaf).read().split()[0] if os.path.exists(shaf) else None,
            "kernel": "ball_count2_kernel<periodic> (nbodyhpc_amd/csrc/ball.hip)",
            "command": "rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE --kernel-include-regex "
                       "ball_count2 -- python3 scripts/ball_run.py",
            "n_particles": 100_000_000, "r": 0.01, "queries_per_launch": 100_000_000,
            "dispatches": [len(fv), len(wv)],
            "FETCH_SIZE_KiB_per_launch": f_kib, "WRITE_SIZE_KiB_per_launch": w_kib,
            "hbm_bytes_per_launch": 2.0 * 1024.0 * f_kib + 1024.0 * w_kib,
            "note": "FETCH_SIZE doubled (gfx950 wide-read correction)",
        }
        json.dump(out, open(os.path.join(prof, f"{tag}_pmc_ball.json"), "w"), indent=1)
        print(json.dumps(out, indent=1))
    if b:
        print(json.dumps(b)[:2000])


if __name__ == "__main__":
    main()
