#!/usr/bin/env python3
"""Open-loop throughput of fw_env_rollout (k_env_rollout) for one precision, for A/B builds (FWSIM_LIB).

  ROLL_PREC=float64 ROLL_N=65536 ROLL_K=64 ROLL_LAUNCHES=4 python tools/rollout_probe.py

Prep: ROLL_PREP closed-loop steps after the reset (steady state), then ROLL_LAUNCHES timed launches of
ROLL_K steps each on U(-1,1) actions.  Prints one JSON line (env-steps/s, ms per step)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tum_adlr_deep_reinforcement_learning_amd import config as C  # noqa: E402
from tum_adlr_deep_reinforcement_learning_amd.engine import Engine  # noqa: E402

prec = os.environ.get("ROLL_PREC", "float64")
n = int(os.environ.get("ROLL_N", "65536"))
K = int(os.environ.get("ROLL_K", "64"))
L = int(os.environ.get("ROLL_LAUNCHES", "4"))
prep = int(os.environ.get("ROLL_PREP", "200"))
prep_mode = os.environ.get("ROLL_PREP_MODE", "closed")  # closed: eager env steps; open: rollouts (as bench.py)
spec = C.EnvSpec(sim_config_kw={"turbulence": False})
eng = Engine(spec.sim, spec, n, device="cuda:0", precision=prec)
eng.seed(1234)
eng.reset()
gen = torch.Generator(device="cuda:0")
gen.manual_seed(1)
acts = torch.rand(K, n, 3, generator=gen, device="cuda:0", dtype=eng.dtype) * 2 - 1
if prep_mode == "open":
    for _ in range(max(prep // K, 1)):
        eng.env_rollout(acts)
else:
    for s in range(prep):
        eng.env_step(acts[s % K])
    eng.env_rollout(acts)  # warm-up launch (allocates the stacked outputs)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(L):
    eng.env_rollout(acts)
torch.cuda.synchronize()
el = time.perf_counter() - t0
print(json.dumps({"precision": prec, "n": n, "k": K, "launches": L, "prep": prep, "prep_mode": prep_mode, "lib": os.environ.get("FWSIM_LIB", "in-tree"),
                  "env_steps_per_s": n * K * L / el, "ms_per_step": el / (K * L) * 1e3}))
