"""Per-kernel (name, grid) means of every PMC counter in a rocprofv3 csv tree,
over its dispatches:
    python scripts/pmc_summary.py gpurun_out/<tag> [kernel-substring] [dir-glob]
(dir-glob default "pmc*", e.g. "ball_sq*" for the radius-count sets)."""
import collections
import csv
import glob
import sys

root = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else ""
pat = sys.argv[3] if len(sys.argv) > 3 else "pmc*"
for f in sorted(glob.glob(f"{root}/{pat}/run_counter_collection.csv")):
    agg = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(f)):
        if sub not in r["Kernel_Name"]:
            continue
        key = (r["Kernel_Name"].replace("void nbkd::(anonymous namespace)::", "").split("(")[0],
               r.get("Grid_Size", "?"))
        agg[key + (r["Counter_Name"],)] += float(r["Counter_Value"])
        disp[key].add(r["Dispatch_Id"])
    rows = collections.defaultdict(dict)
    for (k, g, c), v in agg.items():
        rows[(k, g)][c] = "%.4g" % (v / len(disp[(k, g)]))
    for (k, g), cs in sorted(rows.items()):
        print(f.split("/")[-2], k, "grid", g, "dispatches", len(disp[(k, g)]), dict(sorted(cs.items())))
