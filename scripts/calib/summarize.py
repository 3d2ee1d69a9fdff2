"""Join the calibration kernels' known byte counts with their rocprofv3 PMC
passes (WRITE_SIZE and FETCH_SIZE, separate runs) into the per-shape scale
factors bench.py / summarize_prof.py apply.

    python scripts/calib/summarize.py gpurun_out/<tag>/calib profiles/<round>_pmc_calibration.json

<dir>/known.json is pmc_calib's stdout; <dir>/write, <dir>/fetch the
rocprofv3 -d directories.  Each kernel runs twice (warm-up, measured): the
second dispatch of each name is used.  Counters are KiB.
"""
import csv
import glob
import json
import os
import sys


def per_kernel(d):
    hits = sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True))
    if not hits:
        return {}
    vals = {}
    with open(hits[-1]) as f:
        for row in csv.DictReader(f):
            key = (row["Kernel_Name"], int(row["Dispatch_Id"]))
            vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    out = {}
    for (name, did), v in sorted(vals.items(), key=lambda kv: kv[0][1]):
        base = name.split("(")[0].split("<")[0].replace("void ", "").strip()
        if "col8_append" in name:
            base = "col8_append_4k" if "4096" in name else "col8_append_noload"
        out.setdefault(base, []).append(v * 1024.0)
    return out


def main():
    src, dst = sys.argv[1], sys.argv[2]
    known = json.load(open(os.path.join(src, "known.json")))
    w = per_kernel(os.path.join(src, "write"))
    f = per_kernel(os.path.join(src, "fetch"))
    rows = {}
    for name, kv in known.items():
        r = {"known_write_bytes": kv["write_bytes"], "known_read_bytes": kv["read_bytes"],
             "ms": kv["ms"]}
        if name in w:
            r["WRITE_SIZE_bytes"] = w[name][-1]
            if kv["write_bytes"]:
                r["write_counter_over_known"] = w[name][-1] / kv["write_bytes"]
        if name in f:
            r["FETCH_SIZE_bytes"] = f[name][-1]
            if kv["read_bytes"]:
                r["fetch_counter_over_known"] = f[name][-1] / kv["read_bytes"]
        rows[name] = r
    out = {"command": "rocprofv3 --pmc WRITE_SIZE | FETCH_SIZE -- scripts/calib/pmc_calib "
                      "(scripts/calib/pmc_calib.hip: each kernel moves a known byte count in one "
                      "access shape)",
           "kernels": rows}
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
