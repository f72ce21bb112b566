#!/usr/bin/env python3
"""Capture the rare extreme stragglers of the bench workload and re-run them in fp32, fp64 and the oracle.

Runs the bench workload (N aircraft, fp32, U(-1,1) actions, auto-reset) for `steps` env steps, keeping a
copy of the pre-step state.  Whenever an aircraft needs more than `thresh` RHS evaluations in one step,
its pre-step state and command are re-run through k_sim_step in fp32 and fp64 and through the fp64 C
oracle (checker only): is the straggler physics (all three need the work) or fp32 arithmetic?
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from tum_adlr_deep_reinforcement_learning_amd import config as C  # noqa: E402
from tum_adlr_deep_reinforcement_learning_amd.engine import Engine  # noqa: E402
from oracle import oracle as O  # noqa: E402  (checker only)

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3000
thresh = int(sys.argv[3]) if len(sys.argv) > 3 else 400
dev = "cuda:0"
spec = C.EnvSpec(sim_config_kw={"turbulence": False})
ec = spec.struct()
lo = np.array([ec.act_low[k] for k in range(3)])
hi = np.array([ec.act_high[k] for k in range(3)])
env = Engine(spec.sim, spec, n, device=dev, precision="float32")
env.seed(1234)
env.reset()
gen = torch.Generator(device=dev)
gen.manual_seed(1)
pool = torch.rand(16, n, 3, generator=gen, device=dev) * 2 - 1
s32 = Engine(spec.sim, None, 1, device=dev, precision="float32")
s64 = Engine(spec.sim, None, 1, device=dev, precision="float64")
BL = (C.FW_BLK_ODE, C.FW_BLK_DERIVED, C.FW_BLK_WIND, C.FW_BLK_STEPS)
hist = np.zeros(7, np.int64)  # nfev > 64, 128, 256, 512, 1024, 2048, 4096
edges = [64, 128, 256, 512, 1024, 2048, 4096]
found = []
for s in range(steps):
    pre = {b: env.get_block(b) for b in BL}
    a = pool[s % 16]
    env.env_step(a, stats=True)
    nf = (env.stats & 0xFFFF)
    mx = int(nf.max())
    for k, e in enumerate(edges):
        hist[k] += int((nf > e).sum())
    if mx > thresh and len(found) < 40:
        for i in torch.nonzero(nf > thresh).flatten().tolist()[:4]:
            act = np.clip(a[i].double().cpu().numpy(), -1, 1)
            cmd = lo + (act + 1) / 2 * (hi - lo)  # linear_action_scaling (fixed_wing.py:630-652)
            rec = {"step": s, "env": i, "nfev_env_step": int(nf[i])}
            for name, e in (("f32", s32), ("f64", s64)):
                for b in BL:
                    v = pre[b][:, i:i + 1]
                    e.set_block(b, v if b == C.FW_BLK_STEPS else v.to(e.dtype))
                e.sim_step(torch.tensor(cmd[None], dtype=e.dtype, device=dev), stats=True)
                nfev, nacc, failed = e.decode_stats(e.stats)
                rec[name] = [int(nfev[0]), int(nacc[0]), bool(failed[0]), int(e.term[0])]
            y = pre[C.FW_BLK_ODE][:, i].double().cpu().numpy()[None]
            der = pre[C.FW_BLK_DERIVED][:, i].double().cpu().numpy()[None]
            wind = pre[C.FW_BLK_WIND][:, i].double().cpu().numpy()[None]
            o = O.sim_step(spec.sim.struct(), y, der, wind, np.zeros((1, 6)), cmd[None])
            rec["oracle"] = [int(o["nfev"][0]), int(o["naccept"][0]), int(o["term"][0])]
            rec["state"] = {"omega": y[0, 4:7].round(3).tolist(), "vel": y[0, 10:13].round(2).tolist(),
                            "act": y[0, 13:19].round(3).tolist(), "Va": round(float(der[0, 3]), 2),
                            "alpha": round(float(der[0, 4]), 3)}
            found.append(rec)
            print(json.dumps(rec), flush=True)
    if s % 500 == 0:
        print(json.dumps({"step": s, "max_nfev": mx}), flush=True)
print(json.dumps({"steps": steps, "n": n, "aircraft_steps_over": dict(zip(edges, hist.tolist()))}))
