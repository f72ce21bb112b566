#!/usr/bin/env python3
"""The fp64 bench population's extreme stragglers: step the fp64 kernel (65536 aircraft, bench seeds)
with stats, and for every step whose largest RHS-evaluation count exceeds `thresh`, re-run that
aircraft's pre-step state through the fp64 C oracle (test infrastructure, checker only): is the count
the reference's own (scipy RK45 restated) or a device artefact?  Usage (GPU):
    python tools/fp64_stuck.py [steps=500] [thresh=20000]"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from tum_adlr_deep_reinforcement_learning_amd import config as C  # noqa: E402
from tum_adlr_deep_reinforcement_learning_amd.engine import Engine  # noqa: E402
from oracle import oracle as O  # noqa: E402  (checker only)

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 500
thresh = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
n = 65536
spec = C.EnvSpec(sim_config_kw={"turbulence": False, "turbulence_intensity": "light"})
ec = spec.struct()
lo = np.array([ec.act_low[k] for k in range(3)])
hi = np.array([ec.act_high[k] for k in range(3)])
eng = Engine(spec.sim, spec, n, device="cuda:0", precision="float64")
eng.seed(1234)
eng.reset()
gen = torch.Generator(device="cuda:0")
gen.manual_seed(1)
pool = torch.rand(16, n, 3, generator=gen, device="cuda:0", dtype=torch.float64) * 2 - 1
BL = (C.FW_BLK_ODE, C.FW_BLK_DERIVED, C.FW_BLK_WIND)
found, t0 = 0, time.time()
for s in range(steps):
    pre = {b: eng.get_block(b) for b in BL}
    a = pool[s % 16]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    eng.env_step(a, stats=True)
    e1.record()
    torch.cuda.synchronize()
    nf = eng.stats & 0xFFFF
    mx, am = int(nf.max()), int(nf.argmax())
    if s % 25 == 0:
        print(json.dumps({"step": s, "max_nfev": mx, "launch_ms": round(e0.elapsed_time(e1), 3),
                          "elapsed_s": round(time.time() - t0, 1)}), flush=True)
    if mx > thresh and found < 6:
        found += 1
        i = am
        act = np.clip(a[i].cpu().numpy(), -1, 1)
        cmd = lo + (act + 1) / 2 * (hi - lo)  # linear_action_scaling (fixed_wing.py:630-652)
        y = pre[C.FW_BLK_ODE][:, i].cpu().numpy()[None]
        der = pre[C.FW_BLK_DERIVED][:, i].cpu().numpy()[None]
        wind = pre[C.FW_BLK_WIND][:, i].cpu().numpy()[None]
        t1 = time.time()
        o = O.sim_step(spec.sim.struct(), y, der, wind, np.zeros((1, 6)), cmd[None])
        print(json.dumps({"step": s, "env": i, "device_nfev": int(nf[i]), "launch_ms": round(e0.elapsed_time(e1), 3),
                          "oracle_nfev": int(o["nfev"][0]), "oracle_naccept": int(o["naccept"][0]),
                          "oracle_term": int(o["term"][0]), "oracle_s": round(time.time() - t1, 2),
                          "state": {"omega": y[0, 4:7].round(3).tolist(), "vel": y[0, 10:13].round(3).tolist(),
                                    "act": y[0, 13:19].round(3).tolist(), "Va": round(float(der[0, 3]), 4),
                                    "alpha": round(float(der[0, 4]), 3), "beta": round(float(der[0, 5]), 3)}}),
              flush=True)
