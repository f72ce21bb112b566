"""Summarise rocprofv3 counter CSVs: per-dispatch mean of each counter for k_env_step."""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
kern = sys.argv[2] if len(sys.argv) > 2 else "k_env_step"
vals = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        if kern in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
waves = None
if vals.get("SQ_WAVES"):
    waves = sum(vals["SQ_WAVES"]) / len(vals["SQ_WAVES"])
for k in sorted(vals):
    m = sum(vals[k]) / len(vals[k])
    extra = "  per-wave %.1f" % (m / waves) if waves and k.startswith("SQ_") else ""
    print("%-28s %16.1f%s" % (k, m, extra))
