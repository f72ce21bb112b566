#!/usr/bin/env python3
"""Average k_env_step duration over the LAST ``n`` dispatches of a rocprofv3 kernel trace (the bench's
timed window + its kernel-timing replays), next to the all-dispatch average of --stats.
Usage: trace_window.py <trace dir> [n] [kernel substring] [out.json] [skip_last]
(skip_last: dispatches after the window, e.g. the bench's 1000-step long window)"""
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1128
kern = sys.argv[3] if len(sys.argv) > 3 else "k_env_step"
rows = []
for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
    rows += [r for r in csv.DictReader(open(f)) if kern in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
skip = int(sys.argv[5]) if len(sys.argv) > 5 else 0
w = dur[len(dur) - skip - n:len(dur) - skip]
out = {"kernel": kern, "dispatches": len(dur), "all_avg_us": sum(dur) / len(dur), "window": len(w), "skipped_last": skip,
       "window_avg_us": sum(w) / len(w), "window_min_us": min(w), "window_max_us": max(w)}
print(json.dumps(out))
if len(sys.argv) > 4:
    with open(sys.argv[4], "w") as f:
        json.dump(out, f, indent=1)
