"""Sum rocprofv3 --pmc counter_collection CSVs per kernel (all dispatches).
python scripts/pmc_table.py gpurun_out/<tag>"""
import csv, glob, os, re, sys
from collections import defaultdict
root = sys.argv[1]
tot = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
for f in sorted(glob.glob(os.path.join(root, "pmc*", "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        mm = re.search(r"(\w+_kernel)(<[^(]*>)?", r["Kernel_Name"])
        name = (mm.group(1) + (mm.group(2) or "")) if mm else r["Kernel_Name"][:40]
        tot[name][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[name].add((f, r["Dispatch_Id"]))
for name, c in tot.items():
    waves = c.get("SQ_WAVES", 0) or 1
    print(f"== {name}  dispatches(all passes)={len(disp[name])}")
    for key in sorted(c):
        v = c[key]
        print(f"   {key:24s} {v:16.4g}   per wave {v / waves:12.1f}")
