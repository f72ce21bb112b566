#!/usr/bin/env python3
"""Straggler tail: fp32 kernel vs fp64 kernel vs the CPU oracle on IDENTICAL steady-state states.

Drives N aircraft with U(-1,1) actions through `warm` env steps (fp32, the bench workload), then
takes `snaps` snapshots (every `gap` steps) of the ODE state, derived states, wind and step counter.
From each snapshot ONE PyFly.step with the same random commands is run by
  - the fp32 kernel  (k_sim_step, float32 state),
  - the fp64 kernel  (k_sim_step, the same state widened to float64),
  - the fp64 C oracle (oracle/fw_oracle.c, the same state) -- test infrastructure, used as checker,
and the three RHS-evaluation counts (nfev) per aircraft are compared: histograms, tails, and for the
fp32 stragglers what the fp64 paths needed from the very same state.  Prints JSON lines.
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

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
warm = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
snaps = int(sys.argv[3]) if len(sys.argv) > 3 else 4
gap = int(sys.argv[4]) if len(sys.argv) > 4 else 100
dev = "cuda:0"

from oracle import oracle as O  # noqa: E402  (checker only)

spec = C.EnvSpec(sim_config_kw={"turbulence": False})
env = Engine(spec.sim, spec, n, device=dev, precision="float32")
env.seed(1234)
env.reset()
gen = torch.Generator(device=dev)
gen.manual_seed(1)
pool = torch.rand(16, n, 3, generator=gen, device=dev) * 2 - 1
s32 = Engine(spec.sim, None, n, device=dev, precision="float32")
s64 = Engine(spec.sim, None, n, device=dev, precision="float64")
lo = np.array([-0.5236, -0.5672, 0.0])
hi = np.array([0.6109, 0.5672, 1.0])
rng = np.random.RandomState(5)
BLKS = (C.FW_BLK_ODE, C.FW_BLK_DERIVED, C.FW_BLK_WIND, C.FW_BLK_STEPS)
EDGES = [0, 27, 33, 39, 45, 51, 64, 100, 200, 400, 1000, 2000, 6001]


def hist(x):
    return [int(((x >= a) & (x < b)).sum()) for a, b in zip(EDGES[:-1], EDGES[1:])]


step = 0
all32, all64, allo = [], [], []
for s in range(snaps):
    target = warm + s * gap
    while step < target:
        env.env_step(pool[step % 16])
        step += 1
    torch.cuda.synchronize()
    st = {b: env.get_block(b) for b in BLKS}
    cmd = rng.uniform(lo, hi, (n, 3))
    res = {}
    for name, e in (("f32", s32), ("f64", s64)):
        for b in BLKS:
            e.set_block(b, st[b] if b == C.FW_BLK_STEPS else st[b].to(e.dtype))
        e.sim_step(torch.tensor(cmd, device=dev, dtype=e.dtype), stats=True)
        torch.cuda.synchronize()
        res[name] = ((e.stats & 0xFFFF).cpu().numpy(), e.term.cpu().numpy().copy())
    y = st[C.FW_BLK_ODE].double().cpu().numpy().T
    der = st[C.FW_BLK_DERIVED].double().cpu().numpy().T
    wind = st[C.FW_BLK_WIND].double().cpu().numpy().T
    o = O.sim_step(spec.sim.struct(), y, der, wind, np.zeros((n, 6)), cmd)
    n32, t32 = res["f32"]
    n64, t64 = res["f64"]
    no = o["nfev"]
    all32.append(n32)
    all64.append(n64)
    allo.append(no)
    top = np.argsort(-n32)[:12]
    print(json.dumps({
        "snapshot_step": target, "n": n,
        "max": {"f32": int(n32.max()), "f64": int(n64.max()), "oracle": int(no.max())},
        "mean": {"f32": float(n32.mean()), "f64": float(n64.mean()), "oracle": float(no.mean())},
        "gt64": {"f32": int((n32 > 64).sum()), "f64": int((n64 > 64).sum()), "oracle": int((no > 64).sum())},
        "nfev_equal_f64_oracle": float((n64 == no).mean()), "nfev_equal_f32_oracle": float((n32 == no).mean()),
        "term_fail": {"f32": int((t32 != 0).sum()), "f64": int((t64 != 0).sum()), "oracle": int((o["term"] != 0).sum())},
        "top_f32_stragglers": [[int(i), int(n32[i]), int(n64[i]), int(no[i])] for i in top],
    }), flush=True)
a32, a64, ao = (np.concatenate(x) for x in (all32, all64, allo))
print(json.dumps({"histogram_edges": EDGES, "f32": hist(a32), "f64": hist(a64), "oracle": hist(ao),
                  "samples": int(a32.size),
                  "wave_max_mean": {k: float(v.reshape(-1, 64).max(1).mean()) for k, v in
                                    (("f32", a32), ("f64", a64), ("oracle", ao))}}))
for k in (64, 200, 1000):
    m = a32 > k
    print(json.dumps({"f32_gt": k, "count": int(m.sum()), "f64_same_states_gt": int((a64[m] > k).sum()),
                      "oracle_same_states_gt": int((ao[m] > k).sum()),
                      "f64_gt_total": int((a64 > k).sum()), "oracle_gt_total": int((ao > k).sum())}))
