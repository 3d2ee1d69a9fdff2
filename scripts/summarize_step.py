"""Per-step HBM bytes of the whole kNN query (scripts/gpu_run.sh STEPS=step output):

    python scripts/summarize_step.py gpurun_out/<tag> <round-tag>

writes profiles/<round-tag>_pmc_step.json: for FETCH_SIZE and WRITE_SIZE, the
counter total of the 3-step run minus the 1-step run, / 2 (the tree build and
the warmup call cancel), per kernel and in all; bytes as in summarize_prof.py
(FETCH_SIZE x 2, WRITE_SIZE as reported, KiB -> B: profiles/r04a_pmc_calibration.json).
bench.py reports it as roofline.step_traffic when the loaded library's SHA-256
matches lib_sha256."""
import csv
import glob
import json
import os
import re
import sys


def totals(d):
    path = sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True))[-1]
    per = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            m = re.search(r"([A-Za-z_0-9]+)(<[^(]*>)?\(", row["Kernel_Name"])
            name = m.group(1) + (m.group(2) or "") if m else row["Kernel_Name"][:60]
            per[name] = per.get(name, 0.0) + float(row["Counter_Value"])
    return per


def main():
    src, tag = sys.argv[1], sys.argv[2]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    f1, f3 = totals(os.path.join(src, "f1")), totals(os.path.join(src, "f3"))
    w1, w3 = totals(os.path.join(src, "w1")), totals(os.path.join(src, "w3"))
    kern = {}
    for name in sorted(set(f3) | set(w3)):
        fb = 2.0 * 1024.0 * (f3.get(name, 0.0) - f1.get(name, 0.0)) / 2.0
        wb = 1024.0 * (w3.get(name, 0.0) - w1.get(name, 0.0)) / 2.0
        if abs(fb) + abs(wb) > 1e6:
            kern[name] = {"fetch_bytes": fb, "write_bytes": wb, "hbm_bytes": fb + wb}
    tot_f = sum(v["fetch_bytes"] for v in kern.values())
    tot_w = sum(v["write_bytes"] for v in kern.values())
    shaf = os.path.join(src, "lib.sha256")
    if not os.path.exists(shaf):  # gpu_run.sh keeps it one level up (<tag>/step/)
        shaf = os.path.join(os.path.dirname(os.path.normpath(src)), "lib.sha256")
    out = {
        "lib_sha256": open(shaf).read().split()[0] if os.path.exists(shaf) else None,
        "workload": "nbkd_query_knn of every particle, 1e8 uniform periodic, k = 32, leafsize 64",
        "n_particles": 100_000_000, "k": 32,
        "command": "rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE -- python3 scripts/knn_time.py "
                   "--n 1e8 --k 32 --steps 1 | 3 (separate runs)",
        "method": "(3-step total - 1-step total) / 2 per counter",
        "fetch_bytes_per_step": tot_f, "write_bytes_per_step": tot_w,
        "hbm_bytes_per_step": tot_f + tot_w,
        "per_kernel_per_step": dict(sorted(kern.items(), key=lambda kv: -kv[1]["hbm_bytes"])),
        "note": "FETCH_SIZE doubled, WRITE_SIZE as reported; Infinity-Cache hits are counted",
    }
    json.dump(out, open(os.path.join(root, "profiles", f"{tag}_pmc_step.json"), "w"), indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "per_kernel_per_step"}, indent=1))
    for k, v in list(out["per_kernel_per_step"].items())[:10]:
        print(f"{v['hbm_bytes'] / 1e9:8.2f} GB  {k}")


if __name__ == "__main__":
    main()
