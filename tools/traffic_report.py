#!/usr/bin/env python3
"""Turn the FETCH_SIZE / WRITE_SIZE passes of tools/traffic.sh into HBM bytes per k_env_step launch.

Correction: FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950 their bytes-per-request
accounting depends on the access width (MI355X guide, HBM section), so the
factor is measured on tools/fetch_calib.hip, whose kernels use k_env_step's
4-B-per-lane SoA pattern with a known byte count:
    factor_read  = known read bytes of k_calib_read   / (FETCH_SIZE * 1024)
    factor_write = known write bytes of k_calib_write / (WRITE_SIZE * 1024)
    traffic      = factor_read * FETCH_SIZE*1024 + factor_write * WRITE_SIZE*1024   (k_env_step, per launch)
Writes profiles/pmc_env_step.json (read by bench.py for roofline.traffic).
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_launch(d, kernel, counter, last=None):
    """Mean per-dispatch value of ``counter`` for ``kernel``; ``last``: only the last N dispatches (the
    bench's timed window, in dispatch order)."""
    vals = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals.append((int(r.get("Dispatch_Id") or len(vals)), float(r["Counter_Value"])))
    if not vals:
        raise SystemExit("no %s samples for %s under %s" % (counter, kernel, d))
    vals = [v for _, v in sorted(vals)]
    if last:
        vals = vals[-last:]
    return sum(vals) / len(vals), len(vals)


def main(base):
    lines = open(os.path.join(base, "calib_fetch.log")).read().splitlines()
    calib = json.loads([ln for ln in lines if ln.startswith('{"n"')][-1])
    cf, _ = per_launch(os.path.join(base, "calib_fetch"), "k_calib_read", "FETCH_SIZE")
    cw, _ = per_launch(os.path.join(base, "calib_write"), "k_calib_write", "WRITE_SIZE")
    f_read = calib["read_bytes_k_calib_read"] / (cf * 1024.0)
    f_write = calib["write_bytes_k_calib_write"] / (cw * 1024.0)
    last = int(os.environ.get("PMC_LAST", "200"))  # the bench's timed (steady-state) dispatches
    ef, nf = per_launch(os.path.join(base, "env_fetch"), "k_env_step", "FETCH_SIZE", last)
    ew, nw = per_launch(os.path.join(base, "env_write"), "k_env_step", "WRITE_SIZE", last)
    valu = {}
    if os.path.isdir(os.path.join(base, "env_valu")):
        for ctr in ("SQ_INSTS_VALU", "SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY",
                    "SQ_ACTIVE_INST_VALU"):
            valu[ctr] = per_launch(os.path.join(base, "env_valu"), "k_env_step", ctr, last)[0]
    read_b = ef * 1024.0 * f_read
    write_b = ew * 1024.0 * f_write
    sys.path.insert(0, ROOT)
    import bench  # noqa: E402
    from tum_adlr_deep_reinforcement_learning_amd import config as C  # noqa: E402
    spec = C.EnvSpec(sim_config_kw={"turbulence": False})
    alg = sum(bench.algorithmic_bytes_per_env_step(spec, 4)) * 65536
    out = {
        "kernel": "k_env_step", "workload": "65536 aircraft fp32, turbulence off, U(-1,1) actions",
        "envs": 65536, "precision": "float32", "turbulence": False, "metrics": bool(spec.metrics_enabled),
        "regime": "steady", "dispatches": os.environ.get("PMC_WINDOW", "last %d k_env_step dispatches of the bench "
                                                                      "(its timed window)" % last),
        "valu_insts_per_launch": valu.get("SQ_INSTS_VALU"), "sq_counters_per_launch": valu or None,
        "fetch_size_kib_per_launch": ef, "write_size_kib_per_launch": ew, "launches": [nf, nw],
        "calibration": {"fetch_kib_k_calib_read": cf, "write_kib_k_calib_write": cw, "factor_read": f_read,
                        "factor_write": f_write, "pattern": "4 B/lane SoA rows, coalesced"},
        "hbm_read_bytes_per_launch": read_b, "hbm_write_bytes_per_launch": write_b,
        "hbm_bytes_per_launch": read_b + write_b, "algorithmic_bytes_per_launch": alg,
        "traffic_over_algorithmic": (read_b + write_b) / alg,
    }
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    for path in (os.path.join(ROOT, "profiles", "pmc_env_step.json"), os.path.join(base, "pmc_env_step.json")):
        with open(path, "w") as f:  # the gpurun_out copy is the one that travels back from the GPU box
            json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "traffic"))
