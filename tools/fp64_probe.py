#!/usr/bin/env python3
"""fp64 closed-loop step times of the bench population (65536 aircraft): per-launch ms and the largest
RHS-evaluation count, for steps [a, b) after the global reset.  Usage (GPU):
    [FWSIM_TAIL_QUAD=0] python tools/fp64_probe.py [a=200] [b=260] [n=65536]"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tum_adlr_deep_reinforcement_learning_amd import config as C  # noqa: E402
from tum_adlr_deep_reinforcement_learning_amd.engine import Engine  # noqa: E402

a = int(sys.argv[1]) if len(sys.argv) > 1 else 200
b = int(sys.argv[2]) if len(sys.argv) > 2 else 260
n = int(sys.argv[3]) if len(sys.argv) > 3 else 65536
spec = C.EnvSpec(sim_config_kw={"turbulence": False, "turbulence_intensity": "light"})
eng = Engine(spec.sim, spec, n, device="cuda:0", precision=os.environ.get("PROBE_PREC", "float64"))
eng.seed(1234)
eng.reset()
gen = torch.Generator(device="cuda:0")
gen.manual_seed(1)
pool = torch.rand(16, n, 3, generator=gen, device="cuda:0", dtype=eng.dtype) * 2 - 1
t0 = time.time()
for s in range(a):
    eng.env_step(pool[s % 16])
    if s % 50 == 0:
        torch.cuda.synchronize()
        print(json.dumps({"prep_step": s, "elapsed_s": round(time.time() - t0, 2)}), flush=True)
ms, mx = [], []
st = torch.cuda.current_stream()
for s in range(a, b):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    eng.env_step(pool[s % 16], stats=True)
    e1.record(st)
    torch.cuda.synchronize()
    ms.append(e0.elapsed_time(e1))
    mx.append(int((eng.stats & 0xFFFF).max()))
ms, mx = np.array(ms), np.array(mx)
coef = np.polyfit(mx, ms, 1)
print(json.dumps({"precision": eng.precision, "tail_quad": os.environ.get("FWSIM_TAIL_QUAD", "default"),
                  "steps": [a, b], "ms_mean": float(ms.mean()), "ms_p50": float(np.median(ms)),
                  "ms_max": float(ms.max()), "max_nfev_mean": float(mx.mean()), "max_nfev_max": int(mx.max()),
                  "fit_us_per_rhs": float(coef[0] * 1e3), "fit_intercept_ms": float(coef[1])}))
