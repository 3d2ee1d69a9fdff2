"""Per-kernel mean of every PMC counter in a rocprofv3 csv tree:
    python scripts/pmc_summary.py gpurun_out/<tag> [kernel-substring]"""
import collections
import csv
import glob
import sys

root = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else ""
for f in sorted(glob.glob(f"{root}/pmc*/run_counter_collection.csv")):
    agg = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if sub not in r["Kernel_Name"]:
            continue
        agg[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    byc = collections.defaultdict(list)
    for (_, c), v in agg.items():
        byc[c].append(v)
    print(f.split("/")[-2], {c: "%.4g" % (sum(v) / len(v)) for c, v in sorted(byc.items())})
