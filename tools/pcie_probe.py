#!/usr/bin/env python3
"""PCIe-inclusive rate of the SB3 VecEnv surface: FixedWingVecEnv.step with host
numpy actions in and numpy obs/reward/done/infos out (return_tensors=False), next to the same
surface with device tensors (return_tensors=True). Not bench.py's ``value``."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tum_adlr_deep_reinforcement_learning_amd.vec_env import FixedWingVecEnv  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
out = {"n": n, "steps": steps}
for mode in ("numpy", "device"):
    env = FixedWingVecEnv(n, device="cuda:0", seed=0, sim_config_kw={"turbulence": False},
                          return_tensors=(mode == "device"))
    env.reset()
    rng = np.random.default_rng(1)
    acts = [rng.uniform(-1, 1, (n, 3)).astype(np.float32) for _ in range(8)]
    if mode == "device":
        acts = [torch.as_tensor(a, device="cuda:0") for a in acts]
    for k in range(50):
        env.step(acts[k % 8])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        obs, rew, done, infos = env.step(acts[k % 8])
        if mode == "numpy":
            _ = [infos[int(j)] for j in np.flatnonzero(done)]  # materialise done infos like Monitor would
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    out[mode] = {"env_steps_per_s": n * steps / dt, "ms_per_step": 1e3 * dt / steps}
    env.close()
print(json.dumps(out))
