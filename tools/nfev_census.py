#!/usr/bin/env python3
"""RHS-evaluation census of the bench population: how often a step needs many evaluations, and whether
any step ever reaches the max_nfev budget (a step scipy's solve_ivp would have continued).

Runs the bench population (bench._Schedule: seed 1234, the bench's 16-batch action pool, cycled) for
`steps` env steps after the global reset with stats enabled, one launch per step, and counts per
aircraft-step: nfev above each threshold, budget hits (stats bit 30), solver
failures, plus the largest nfev seen (and where).  Usage (GPU):
    python tools/nfev_census.py [steps=4000] [out.json]"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from tum_adlr_deep_reinforcement_learning_amd import config as C  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 4000
out = sys.argv[2] if len(sys.argv) > 2 else None
n = int(os.environ.get("CENSUS_N", "65536"))


class A:  # the bench's defaults
    precision, lanes = os.environ.get("CENSUS_PREC", "float32"), 0


spec = C.EnvSpec(sim_config_kw={"turbulence": False, "turbulence_intensity": "light"})
sch = bench._Schedule(n, A, spec, torch.device("cuda", 0), 0, 0)
eng = sch.eng
edges = [64, 128, 256, 512, 1024, 2048, 4096, 6000, 8192, 16384, 65535]
cnt = torch.zeros(len(edges), dtype=torch.int64, device="cuda:0")
per_step = torch.zeros(steps, 4, dtype=torch.int64, device="cuda:0")  # max nfev, argmax, failures, budget hits
edges_t = torch.tensor(edges, device="cuda:0")
t0 = time.time()
for s in range(steps):
    eng.env_step(sch.pool[s % 16], stats=True)
    st = eng.stats
    nf = (st & 0xFFFF).to(torch.int64)
    m, am = nf.max(0)
    per_step[s, 0], per_step[s, 1] = m, am
    per_step[s, 2] = (st < 0).sum()
    per_step[s, 3] = ((st & (1 << 30)) != 0).sum()
    cnt += (nf[None, :] > edges_t[:, None]).sum(1)
    mx = int(m)  # (one sync per step: the census is not timed)
    if mx > 8000:
        print(json.dumps({"step": s, "max_nfev": mx, "env": int(am), "elapsed_s": round(time.time() - t0, 1)}),
              flush=True)
    if s % 100 == 0:
        print(json.dumps({"step": s, "elapsed_s": round(time.time() - t0, 1)}), flush=True)
torch.cuda.synchronize()
r = per_step.cpu().numpy()
top = np.argsort(-r[:, 0])[:12]
res = {"what": "RHS-evaluation census of the bench population (65536 aircraft, fp32, bench seeds and actions)",
       "aircraft": n, "steps": steps, "aircraft_steps": n * steps, "precision": A.precision,
       "max_nfev_budget": 1000000,
       "aircraft_steps_over": {str(e): int(c) for e, c in zip(edges, cnt.cpu().numpy())},
       "budget_hits": int(r[:, 3].sum()), "solver_failures": int(r[:, 2].sum()),
       "max_nfev": int(r[:, 0].max()), "per_step_max_nfev_p50": float(np.median(r[:, 0])),
       "per_step_max_nfev_mean": float(r[:, 0].mean()),
       "largest": [{"step_after_reset": int(j) + 1, "env": int(r[j, 1]), "nfev": int(r[j, 0])} for j in top]}
print(json.dumps(res))
if out:
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
