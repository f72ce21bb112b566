#!/usr/bin/env python3
"""Idle gaps between the kernels of the fused collect step from a rocprofv3 kernel trace: for every
k_env_step -> k_policy_mfma and k_policy_mfma -> k_env_step pair of consecutive dispatches on the collect's
queue, start(next) - end(prev).  Usage: tools/graph_gaps.py <trace dir> [--last N]"""
import argparse, csv, glob, json
import numpy as np

ap = argparse.ArgumentParser()
ap.add_argument("trace_dir"); ap.add_argument("--last", type=int, default=2048)
a = ap.parse_args()
rows = list(csv.DictReader(open(glob.glob(a.trace_dir + "/**/*kernel_trace.csv", recursive=True)[0])))
rows = [r for r in rows if "k_env_step" in r["Kernel_Name"] or "k_policy_mfma" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-2 * a.last:]
gaps = {"env->policy": [], "policy->env": []}
busy = {"k_env_step": [], "k_policy_mfma": []}
for p, n in zip(rows, rows[1:]):
    g = (int(n["Start_Timestamp"]) - int(p["End_Timestamp"])) / 1e3
    if "k_env_step" in p["Kernel_Name"] and "k_policy_mfma" in n["Kernel_Name"]:
        gaps["env->policy"].append(g)
    elif "k_policy_mfma" in p["Kernel_Name"] and "k_env_step" in n["Kernel_Name"]:
        gaps["policy->env"].append(g)
for r in rows:
    k = "k_env_step" if "k_env_step" in r["Kernel_Name"] else "k_policy_mfma"
    busy[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3
out = {"pairs": {k: len(v) for k, v in gaps.items()},
       "gap_us_median": {k: float(np.median(v)) for k, v in gaps.items()},
       "gap_us_mean": {k: float(np.mean(v)) for k, v in gaps.items()},
       "kernel_us_mean": {k: float(np.mean(v)) for k, v in busy.items()},
       "span_us_per_step": span / (len(rows) / 2)}
print(json.dumps(out, indent=1))
