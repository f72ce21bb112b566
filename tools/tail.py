#!/usr/bin/env python3
"""Tail analysis of k_env_step: per-launch time vs the largest per-aircraft RHS count.

With one wave per SIMD (65536 aircraft), a launch lasts as long as its slowest
wave, and a wave iterates as long as its slowest lane: launch time ~ a + b * max_nfev.
This fits a and b (b = latency of one RHS iteration of a lone wave) and prints
the nfev distribution."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tum_adlr_deep_reinforcement_learning_amd import config as C  # noqa: E402
from tum_adlr_deep_reinforcement_learning_amd.engine import Engine  # noqa: E402

n = int(os.environ.get("TAIL_N", "65536"))
steps = int(os.environ.get("TAIL_STEPS", "300"))
spec = C.EnvSpec(sim_config_kw={"turbulence": False})
spec.metrics_enabled = os.environ.get("TAIL_METRICS", "1") == "1"
eng = Engine(spec.sim, spec, n, device="cuda:0", precision=os.environ.get("TAIL_PREC", "float32"))
eng.seed(1234)
eng.reset()
gen = torch.Generator(device="cuda:0")
gen.manual_seed(1)
pool = torch.rand(16, n, 3, generator=gen, device="cuda:0", dtype=eng.dtype) * 2 - 1
MODE = os.environ.get("TAIL_MODE", "env")  # env | env_noreset | sim


def step(a):
    if MODE == "sim":
        eng.sim_step(a, stats=True)
    else:
        eng.env_step(a, stats=True, auto_reset=(MODE == "env"))


for s in range(int(os.environ.get("TAIL_PREP", "20"))):  # (20: the round-2..4 protocol; 1000: steady state)
    step(pool[s % 16])
torch.cuda.synchronize()
ms, mx, p999, mean, wmax = [], [], [], [], []
stream = torch.cuda.current_stream()
for s in range(steps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    step(pool[s % 16])
    e1.record(stream)
    torch.cuda.synchronize()
    nf = (eng.stats & 0xFFFF).cpu().numpy().astype(np.int64)
    ms.append(e0.elapsed_time(e1))
    mx.append(nf.max())
    p999.append(np.percentile(nf, 99.9))
    mean.append(nf.mean())
    w = nf[: n // 64 * 64].reshape(-1, 64).max(1)
    wmax.append(np.median(w))
ms, mx = np.array(ms), np.array(mx)
A = np.stack([np.ones_like(mx, dtype=float), mx.astype(float)], 1)
coef, *_ = np.linalg.lstsq(A, ms, rcond=None)
out = {"mode": MODE, "n": n, "steps": steps, "ms_mean": float(ms.mean()), "ms_p50": float(np.median(ms)),
       "max_nfev_mean": float(mx.mean()), "max_nfev_p50": float(np.median(mx)), "max_nfev_max": int(mx.max()),
       "nfev_p999_mean": float(np.mean(p999)), "nfev_mean": float(np.mean(mean)),
       "wave_max_nfev_median": float(np.mean(wmax)),
       "fit_ms_intercept": float(coef[0]), "fit_us_per_iteration": float(coef[1] * 1e3),
       "corr": float(np.corrcoef(mx, ms)[0, 1])}
print(json.dumps(out))
hist = np.histogram(mx, bins=[0, 50, 75, 100, 150, 200, 300, 500, 1000, 7000])
print("max-nfev histogram:", list(zip(hist[1][:-1].tolist(), hist[0].tolist())))
