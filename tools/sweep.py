#!/usr/bin/env python3
"""Scaling sweep of k_env_step: ms/step vs aircraft count, plus RK45 work statistics."""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tum_adlr_deep_reinforcement_learning_amd import config as C  # noqa: E402
from tum_adlr_deep_reinforcement_learning_amd.engine import Engine  # noqa: E402


def run(n, precision, steps, turbulence):
    spec = C.EnvSpec(sim_config_kw={"turbulence": turbulence})
    eng = Engine(spec.sim, spec, n, device="cuda:0", precision=precision)
    eng.seed(7)
    eng.reset()
    pool = torch.rand(8, n, 3, device="cuda:0", dtype=eng.dtype) * 2 - 1
    for s in range(10):
        eng.env_step(pool[s % 8], stats=True)
    torch.cuda.synchronize()
    nfev = []
    for s in range(5):
        eng.env_step(pool[s % 8], stats=True)
        nfev.append((eng.stats & 0xFFFF).cpu().numpy())
    nfev = np.stack(nfev)
    lanes = nfev.reshape(nfev.shape[0], -1)
    waves = lanes[:, : (lanes.shape[1] // 64) * 64].reshape(lanes.shape[0], -1, 64)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for s in range(steps):
        eng.env_step(pool[s % 8])
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    eng.close()
    return {"n": n, "precision": precision, "turb": turbulence, "ms_per_step": ms, "env_steps_per_s": n / ms * 1e3,
            "nfev_mean": float(lanes.mean()), "nfev_wave_max_mean": float(waves.max(-1).mean()) if waves.size else None}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1024,4096,16384,65536,131072,262144")
    ap.add_argument("--precision", default="float32")
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--turbulence", action="store_true")
    a = ap.parse_args()
    for n in [int(x) for x in a.sizes.split(",")]:
        print(json.dumps(run(n, a.precision, a.steps, a.turbulence)), flush=True)
