#!/usr/bin/env python3
"""HBM bytes per k_env_step launch in the NORESET and STEADY windows of tools/traffic_split.py, corrected
with the fetch_calib factors (tools/traffic_report.py), against the algorithmic accounting
(bench.algorithmic_bytes_per_env_step).  Writes profiles/r04_traffic_split.json."""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def series(d, kernel, counter):
    vals = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals.append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    return [v for _, v in sorted(vals)]


def main(base):
    sys.path.insert(0, ROOT)
    import bench  # noqa: E402
    from tum_adlr_deep_reinforcement_learning_amd import config as C  # noqa: E402
    lines = open(os.path.join(base, "calib_fetch.log")).read().splitlines()
    calib = json.loads([ln for ln in lines if ln.startswith('{"n"')][-1])
    cf = series(os.path.join(base, "calib_fetch"), "k_calib_read", "FETCH_SIZE")
    cw = series(os.path.join(base, "calib_write"), "k_calib_write", "WRITE_SIZE")
    f_read = calib["read_bytes_k_calib_read"] / (sum(cf) / len(cf) * 1024.0)
    f_write = calib["write_bytes_k_calib_write"] / (sum(cw) / len(cw) * 1024.0)
    w = json.loads([ln for ln in open(os.path.join(base, "split_fetch.log")).read().splitlines()
                    if ln.startswith('{"n"')][-1])
    fe = series(os.path.join(base, "split_fetch"), "k_env_step", "FETCH_SIZE")
    wr = series(os.path.join(base, "split_write"), "k_env_step", "WRITE_SIZE")
    spec = C.EnvSpec(sim_config_kw={"turbulence": False})
    rd_alg, wr_alg = bench.algorithmic_bytes_per_env_step(spec, 4)
    n = w["n"]
    out = {"workload": "65536 aircraft fp32, default task with metrics, turbulence off (tools/traffic_split.py)",
           "calibration": {"factor_read": f_read, "factor_write": f_write},
           "algorithmic_bytes_per_env_step": {"read": rd_alg, "write": wr_alg, "total": rd_alg + wr_alg},
           "windows": {}}
    for name in ("noreset", "steady"):
        a, b = w["dispatches"][name]
        r = sum(fe[a:b]) / (b - a) * 1024.0 * f_read
        x = sum(wr[a:b]) / (b - a) * 1024.0 * f_write
        dones = w[name + "_dones"]
        out["windows"][name] = {
            "dispatches": [a, b], "dones_per_launch": sum(dones) / len(dones),
            "hbm_read_bytes_per_launch": r, "hbm_write_bytes_per_launch": x,
            "read_over_algorithmic": r / (rd_alg * n), "write_over_algorithmic": x / (wr_alg * n),
            "total_over_algorithmic": (r + x) / ((rd_alg + wr_alg) * n)}
    q, s = out["windows"]["noreset"], out["windows"]["steady"]
    dd = s["dones_per_launch"] - q["dones_per_launch"]
    if dd > 0:
        extra = (s["hbm_read_bytes_per_launch"] + s["hbm_write_bytes_per_launch"]
                 - q["hbm_read_bytes_per_launch"] - q["hbm_write_bytes_per_launch"])
        out["reset_path_bytes_per_done_aircraft"] = extra / dd
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    for path in (os.path.join(ROOT, "profiles", "r04_traffic_split.json"), os.path.join(base, "r04_traffic_split.json")):
        with open(path, "w") as f:
            json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "split"))
