"""Per-rank HBM bytes of the N-GPU bench (scripts/gpu_run.sh STEPS=slab):

    python scripts/summarize_slab.py gpurun_out/<tag> <round-tag>

Each gpurun_out/<tag>/slab_<W>_<scaling>/ holds FETCH_SIZE / WRITE_SIZE passes
over 1- and 3-step knn_time.py runs of rank 0's slab (own particles + halo,
global ids, own particles queried) alone on one GPU.  As summarize_step.py:
(3-step - 1-step) / 2 per kernel, FETCH_SIZE x 2, WRITE_SIZE as reported
(profiles/r04a_pmc_calibration.json); divided by the rank's own queries.
Writes profiles/<round-tag>_pmc_slab.json; bench.py at N > 1 multiplies the
per-query bytes by every rank's own queries (roofline.traffic / step_traffic)
when the loaded library's SHA-256 equals lib_sha256."""
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from summarize_step import totals  # noqa: E402


def run_info(log):
    for line in reversed(open(log).read().splitlines()):
        if line.startswith("{"):
            return json.loads(line)
    raise RuntimeError(f"no JSON line in {log}")


def main():
    src, tag = sys.argv[1], sys.argv[2]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    shaf = os.path.join(src, "lib.sha256")
    entries = []
    for d in sorted(glob.glob(os.path.join(src, "slab_*"))):
        if not os.path.isdir(d):
            continue
        f1, f3 = totals(os.path.join(d, "f1")), totals(os.path.join(d, "f3"))
        w1, w3 = totals(os.path.join(d, "w1")), totals(os.path.join(d, "w3"))
        info = run_info(os.path.join(d, "f3.log"))
        own = info["n"]
        kern = {}
        for name in set(f3) | set(w3):
            fb = 2.0 * 1024.0 * (f3.get(name, 0.0) - f1.get(name, 0.0)) / 2.0
            wb = 1024.0 * (w3.get(name, 0.0) - w1.get(name, 0.0)) / 2.0
            if abs(fb) + abs(wb) > 1e6:
                kern[name] = fb + wb
        step = sum(kern.values())
        # the first pass: knn_collect_grp_kernel<PER, OCC, STATS, LOOP, AHEAD>
        # with LOOP = false (the LOOP retry launches hold few queries; they
        # are counted in the step only)
        first = [kk for kk in kern if kk.startswith("knn_collect_grp_kernel<")
                 and kk.split("<", 1)[1].rstrip(">").split(",")[3].strip() == "false"]
        collect = sum(kern[kk] for kk in first)
        entries.append({
            "world": info["slab_world"], "rank": info["slab_rank"], "scaling": info["scaling"],
            "n_arg": int(info["n_arg"]), "k": info["k"], "leafsize": info["leaf"],
            "seed": info["seed"], "own": own, "n_local": info["n_tree"],
            "collect_bytes_per_query": collect / own,
            "step_bytes_per_query": step / own,
            "step_bytes": step, "collect_kernels": first,
            "per_kernel_bytes_per_step": dict(sorted(kern.items(), key=lambda kv: -kv[1])),
            "wall_ms_per_step": info["wall_ms"],
        })
    out = {
        "lib_sha256": open(shaf).read().split()[0] if os.path.exists(shaf) else None,
        "command": "rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE -- python3 scripts/knn_time.py --n N "
                   "--k 32 --slab-world W --slab-rank 0 --scaling S --steps 1 | 3 (separate runs)",
        "method": "(3-step total - 1-step total) / 2 per counter, / the rank's own queries",
        "note": "FETCH_SIZE doubled, WRITE_SIZE as reported; Infinity-Cache hits are counted",
        "entries": entries,
    }
    json.dump(out, open(os.path.join(root, "profiles", f"{tag}_pmc_slab.json"), "w"), indent=1)
    for e in entries:
        print(f"W={e['world']} {e['scaling']} n_arg={e['n_arg']}: own {e['own']}, local "
              f"{e['n_local']}, collect {e['collect_bytes_per_query']:.1f} B/q, step "
              f"{e['step_bytes_per_query']:.1f} B/q")


if __name__ == "__main__":
    main()
