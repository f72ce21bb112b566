"""Summary of tools/r06_pair_pmc.sh: per (aircraft, lanes) the means over the last K k_env_step dispatches of that
lanes instance (demangled names: `..., false, 1>` / `..., false, 2>`), profiled launch durations from the kernel trace.
Usage: python tools/pair_pmc_summary.py DIR [K]"""
import collections
import csv
import glob
import json
import os
import sys

root = sys.argv[1]
K = int(sys.argv[2]) if len(sys.argv) > 2 else 40
for N in (65536, 32768):
    for L in (1, 2):
        tag = "false, %d>" % L
        cnt = collections.defaultdict(dict)
        dur = []
        for f in sorted(glob.glob(os.path.join(root, "n%d_l%d_p*" % (N, L), "**", "*counter_collection.csv"), recursive=True)):
            for r in csv.DictReader(open(f)):
                if "k_env_step" in r["Kernel_Name"] and tag in r["Kernel_Name"]:
                    d = (f, int(r["Dispatch_Id"]))
                    cnt[r["Counter_Name"]][d] = cnt[r["Counter_Name"]].get(d, 0.0) + float(r["Counter_Value"])
        for f in sorted(glob.glob(os.path.join(root, "n%d_l%d_p1" % (N, L), "**", "*kernel_trace.csv"), recursive=True)):
            rows = [r for r in csv.DictReader(open(f)) if "k_env_step" in r["Kernel_Name"] and tag in r["Kernel_Name"]]
            dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows][-K:]
        res = {}
        for c, dv in cnt.items():
            ks = sorted(dv)[-K:]
            res[c] = round(sum(dv[k] for k in ks) / len(ks), 1)
        w = res.get("SQ_WAVES", 0) or 1
        derived = {"valu_per_wave": round(res.get("SQ_INSTS_VALU", 0) / w, 1),
                   "wait_any_frac": round(res.get("SQ_WAIT_ANY", 0) / max(res.get("SQ_WAVE_CYCLES", 1), 1), 3),
                   "wait_inst_frac": round(res.get("SQ_WAIT_INST_ANY", 0) / max(res.get("SQ_WAVE_CYCLES", 1), 1), 3),
                   "active_valu_frac": round(res.get("SQ_ACTIVE_INST_VALU", 0) / max(res.get("SQ_WAVE_CYCLES", 1), 1), 3)}
        print(json.dumps({"envs": N, "lanes": L, "dispatches": K,
                          "launch_us_profiled_mean": round(sum(dur) / max(len(dur), 1), 1),
                          "launch_us_profiled_p50": round(sorted(dur)[len(dur) // 2], 1) if dur else None,
                          "derived": derived, "counters": res}))
