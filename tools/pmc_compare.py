#!/usr/bin/env python3
"""fp32 vs fp64 SQ counters of the one-lane k_env_step from two rocprofv3 --pmc counter_collection.csv files
(tools/r05_final.sh, tools/tail.py): the last ``--last`` k_env_step dispatches averaged per counter."""
import argparse, collections, csv, glob


def per_dispatch(path, last):
    rows = collections.defaultdict(dict)
    for r in csv.DictReader(open(path)):
        if "k_env_step" in r["Kernel_Name"]:
            d = rows[int(r["Dispatch_Id"])]
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    ids = sorted(rows)[-last:]
    out = collections.defaultdict(float)
    for i in ids:
        for k, v in rows[i].items():
            out[k] += v / len(ids)
    return out


ap = argparse.ArgumentParser()
ap.add_argument("f32_dir"); ap.add_argument("f64_dir"); ap.add_argument("--last", type=int, default=30)
a = ap.parse_args()
p32 = per_dispatch(glob.glob(a.f32_dir + "/**/*counter_collection.csv", recursive=True)[0], a.last)
p64 = per_dispatch(glob.glob(a.f64_dir + "/**/*counter_collection.csv", recursive=True)[0], a.last)
print(f"{'counter':28s}{'fp32':>12s}{'fp64':>15s}    ratio")
for k in sorted(set(p32) | set(p64)):
    x, y = p32.get(k, 0.0), p64.get(k, 0.0)
    print(f"{k:28s}{x:12.0f}{y:15.0f}{(y / x if x else float('nan')):9.2f}")
