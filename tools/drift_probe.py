#!/usr/bin/env python3
"""k_env_step cost vs episode progress: ms/launch, nfev mean / wave-max and done rate per block of launches."""
import json
import time
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tum_adlr_deep_reinforcement_learning_amd import config as C  # noqa: E402
from tum_adlr_deep_reinforcement_learning_amd.engine import Engine  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
total = int(sys.argv[2]) if len(sys.argv) > 2 else 3000
blk = 100
idle = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0  # host sleep between blocks (s)
spec = C.EnvSpec(sim_config_kw={"turbulence": False})
eng = Engine(spec.sim, spec, n, device="cuda:0")
eng.seed(1234)
eng.reset()
pool = torch.rand(16, n, 3, device="cuda:0") * 2 - 1
s = 0
for b in range(total // blk):
    a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(blk - 1):
        eng.env_step(pool[s % 16], stats=False)
        s += 1
    e.record()
    eng.env_step(pool[s % 16], stats=True)
    s += 1
    nf = (eng.stats & 0xFFFF).float()
    torch.cuda.synchronize()
    w = nf[: n // 64 * 64].view(-1, 64).max(1).values
    print(json.dumps({"step": s, "ms": a.elapsed_time(e) / (blk - 1), "nfev_mean": nf.mean().item(),
                      "nfev_wave_max": w.mean().item(), "done_frac": eng.done.float().mean().item()}), flush=True)
    if idle > 0:
        time.sleep(idle)
