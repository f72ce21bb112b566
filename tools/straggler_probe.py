#!/usr/bin/env python3
"""Per-step k_env_step duration vs the RK45 work of its slowest aircraft (nfev max, stragglers)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tum_adlr_deep_reinforcement_learning_amd import config as C  # noqa: E402
from tum_adlr_deep_reinforcement_learning_amd.engine import Engine  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
total = int(sys.argv[2]) if len(sys.argv) > 2 else 1500
spec = C.EnvSpec(sim_config_kw={"turbulence": False})
eng = Engine(spec.sim, spec, n, device="cuda:0")
eng.seed(1234)
eng.reset()
pool = torch.rand(16, n, 3, device="cuda:0") * 2 - 1
evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(total)]
nf = torch.zeros(total, n, dtype=torch.int32, device="cuda:0")
for s in range(total):
    evs[s][0].record()
    eng.env_step(pool[s % 16], stats=True)
    evs[s][1].record()
    nf[s].copy_(eng.stats & 0xFFFF)
torch.cuda.synchronize()
ms = [a.elapsed_time(b) for a, b in evs]
mx = nf.max(1).values.cpu().tolist()
big = (nf > 64).sum(1).cpu().tolist()
for s in range(total):
    if s % 10 == 0 or ms[s] > 0.15:
        print(json.dumps({"step": s, "ms": round(ms[s], 4), "nfev_max": mx[s], "n_gt64": big[s]}))
hist = torch.bincount(nf.flatten().clamp(max=2200).long()).cpu()
print("nfev>64 lanes total", int((nf > 64).sum()), "of", nf.numel())
print("hist(>=44)", {i: int(hist[i]) for i in range(44, len(hist)) if hist[i] > 0})
