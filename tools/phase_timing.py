#!/usr/bin/env python3
"""Per-wave phase timing of k_env_step (debug build with -DFW_TIMING).

    python tools/ab.py build timing -DFW_TIMING          (CPU)
    FWSIM_LIB=tools/_build/variants/timing.so python tools/phase_timing.py   (GPU)

Lane 0 of each wave stamps the 100 MHz real-time counter at: 0 kernel entry, 1 after the
prologue loads / turbulence, 2 after PyFly.step (RK loop + post-step save), 3 after reward /
obs / metrics, 4 end (5 = end of the auto-reset path).  Stamps are taken after s_waitcnt(0).
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tum_adlr_deep_reinforcement_learning_amd import config as C  # noqa: E402
from tum_adlr_deep_reinforcement_learning_amd.engine import Engine  # noqa: E402

n = int(os.environ.get("TIM_N", "65536"))
spec = C.EnvSpec(sim_config_kw={"turbulence": False})
eng = Engine(spec.sim, spec, n, device="cuda:0", precision="float32")
eng.seed(1234)
eng.reset()
gen = torch.Generator(device="cuda:0")
gen.manual_seed(1)
pool = torch.rand(16, n, 3, generator=gen, device="cuda:0") * 2 - 1
for s in range(20):
    eng.env_step(pool[s % 16], stats=True)
torch.cuda.synchronize()
lanes = eng.lanes  # FWSIM_LANES=1|4 selects the integrator
per = 64 // lanes  # aircraft per wave
waves = (n * lanes + 63) // 64
rows = []
for s in range(60):
    eng.episode.zero_()
    eng.env_step(pool[s % 16], stats=True)
    torch.cuda.synchronize()
    st = eng.episode.view(-1).view(torch.int64)[: waves * 8].view(waves, 8).cpu().numpy().astype(np.float64) * 10.0
    nf = (eng.stats & 0xFFFF).cpu().numpy()
    wmax = nf[: waves * per].reshape(waves, per).max(1) if n % per == 0 else None
    t0 = st[:, 0]
    end = np.where(st[:, 4] > 0, st[:, 4], st[:, 5])
    k0 = t0.min()
    slow = int(np.argmax(end))
    rows.append({"span_us": (end.max() - k0) / 1e3, "entry_spread_us": (t0.max() - k0) / 1e3,
                 "prologue_us": float(np.median(st[:, 1] - st[:, 0]) / 1e3),
                 "sim_us_median": float(np.median(st[:, 2] - st[:, 1]) / 1e3),
                 "epilogue_us": float(np.median(st[:, 3] - st[:, 2]) / 1e3),
                 "tail_us": float(np.median(end - st[:, 3]) / 1e3),
                 "slow_wave": {"entry_us": (t0[slow] - k0) / 1e3, "prologue_us": (st[slow, 1] - st[slow, 0]) / 1e3,
                               "sim_us": (st[slow, 2] - st[slow, 1]) / 1e3, "epi_us": (st[slow, 3] - st[slow, 2]) / 1e3,
                               "end_us": (end[slow] - st[slow, 3]) / 1e3,
                               "wave_max_nfev": int(wmax[slow]) if wmax is not None else None}})
keys = ["span_us", "entry_spread_us", "prologue_us", "sim_us_median", "epilogue_us", "tail_us"]
print(json.dumps(dict({k: round(float(np.median([r[k] for r in rows])), 2) for k in keys}, n=n, lanes=lanes)))
for r in rows[:6]:
    print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in r["slow_wave"].items()}),
          "span", round(r["span_us"], 1))
