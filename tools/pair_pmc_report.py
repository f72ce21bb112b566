"""Per-dispatch means of the counters of the last K k_env_step dispatches of one lanes instance (Q = lanes in the
mangled name: Li1E / Li2E) from rocprofv3 counter CSVs.  Usage: python tools/pair_pmc_report.py DIR LANES K"""
import collections
import csv
import glob
import json
import os
import sys

root, lanes, K = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
tag = "Li%dE" % lanes
per = collections.defaultdict(dict)  # counter -> dispatch -> value
for f in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        if "k_env_step" in r["Kernel_Name"] and tag in r["Kernel_Name"]:
            d = int(r["Dispatch_Id"])
            per[r["Counter_Name"]][d] = per[r["Counter_Name"]].get(d, 0.0) + float(r["Counter_Value"])
out = {}
for c, dv in per.items():
    ds = sorted(dv)[-K:]
    out[c] = sum(dv[d] for d in ds) / len(ds)
print(json.dumps({"lanes": lanes, "dispatches": K, "counters": out}))
