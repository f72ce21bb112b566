#!/usr/bin/env python3
"""The bench workload's per-step RK45 work in its timed window: max nfev, solver failures, slowest aircraft.
Usage: FWSIM_LIB=... python tools/window_probe.py [prep] [steps]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tum_adlr_deep_reinforcement_learning_amd import config as C  # noqa: E402
from tum_adlr_deep_reinforcement_learning_amd.engine import Engine  # noqa: E402

prep = int(sys.argv[1]) if len(sys.argv) > 1 else 1016
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 500
n = 65536
spec = C.EnvSpec(sim_config_kw={"turbulence": False, "turbulence_intensity": "light"})
eng = Engine(spec.sim, spec, n, device="cuda:0")
eng.seed(1234)
eng.reset()
gen = torch.Generator(device="cuda:0")
gen.manual_seed(1)
pool = torch.rand(16, n, 3, generator=gen, device="cuda:0") * 2 - 1
for s in range(prep):
    eng.env_step(pool[s % 16])
tot, fails, big = 0, 0, []
for s in range(steps):
    eng.env_step(pool[(prep + s) % 16], stats=True)
    nf, _, failed = eng.decode_stats(eng.stats)
    mx = int(nf.max())
    tot += mx
    fails += int(failed.sum())
    if mx > 500:
        i = int(nf.argmax())
        big.append((s, mx, i))
print(json.dumps({"prep": prep, "steps": steps, "mean_max_nfev": tot / steps, "solver_failures": fails,
                  "steps_over_500": len(big), "first": big[:30]}))
