"""Print the bench lines of one gpu_ab.sh output directory as a table."""
import glob
import json
import os
import sys

for f in sorted(glob.glob(os.path.join(sys.argv[1], "b_*.json"))):
    try:
        d = json.load(open(f))
    except Exception as e:  # noqa: BLE001
        print(os.path.basename(f), "unreadable", e)
        continue
    b = d["breakdown_ms_per_step"]
    ph = d.get("collect_phase_frac") or {}
    print(f"{os.path.basename(f)[2:-5]:28s} {d['value']:.4g} q/s  collect {b['knn_collect']:6.2f} "
          f"wrap {b.get('knn_collect_wrap', 0):5.2f} select {b['knn_select']:5.2f} key {b['leaf_key']:4.2f} retry {b['retry']:5.2f}  "
          f"evals/q {d['traversal_per_query']['distance_evals']:6.1f} "
          f"cand/q {d['traversal_per_query']['candidates']:5.1f} "
          f"nodes/pk {d['traversal_per_packet']['node_visits']:5.1f}  build {d['build_ms']:5.1f}  "
          + " ".join(f"{k}={v:.2f}" for k, v in ph.items()))
