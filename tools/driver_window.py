#!/usr/bin/env python3
"""Per-launch durations of the bench's timed window from a rocprofv3 kernel trace of
`bench.py --gpus 1 --steps K --warmup W` (the driver's command).

The timed engine's k_env_step dispatches come first in the trace, in this order: 1 eager step, the
96-step early regime, the prep steps up to --prep (1000), W warm-up steps, the K timed steps, then the
long window (and after it the stats replay, the open-loop and fp64 legs).  So the timed window is
dispatches [prep + W, prep + W + K) of the float k_env_step instances.
Usage: driver_window.py <trace dir> [K=20] [W=5] [prep=1000] [out.json]"""
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
K = int(sys.argv[2]) if len(sys.argv) > 2 else 20
W = int(sys.argv[3]) if len(sys.argv) > 3 else 5
prep = int(sys.argv[4]) if len(sys.argv) > 4 else 1000
rows = []
for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
    rows += [r for r in csv.DictReader(open(f)) if ("k_env_step<float" in r["Kernel_Name"] or "k_env_stepIf" in r["Kernel_Name"])]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
a = prep + W
w = dur[a:a + K]
gaps = [(int(rows[i + 1]["Start_Timestamp"]) - int(rows[i]["End_Timestamp"])) / 1e3 for i in range(a, a + K - 1)]
span = (int(rows[a + K - 1]["End_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e3
out = {"kernel": rows[a]["Kernel_Name"][:120], "float_k_env_step_dispatches": len(dur), "window_first_dispatch": a,
       "window": K, "per_launch_us": [round(x, 2) for x in w], "window_avg_us": sum(w) / K,
       "window_span_us_per_step": span / K, "gap_avg_us": sum(gaps) / max(len(gaps), 1),
       "window_max_us": max(w), "window_min_us": min(w),
       "long_window_avg_us": (sum(dur[a + K:a + K + 1000]) / 1000) if len(dur) >= a + K + 1000 else None}
print(json.dumps(out))
if len(sys.argv) > 5:
    with open(sys.argv[5], "w") as f:
        json.dump(out, f, indent=1)
