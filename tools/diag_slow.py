#!/usr/bin/env python3
"""Find aircraft whose env step needs pathologically many RHS evaluations."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tum_adlr_deep_reinforcement_learning_amd import config as C  # noqa: E402
from tum_adlr_deep_reinforcement_learning_amd.engine import Engine  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
seed = int(sys.argv[2]) if len(sys.argv) > 2 else 1234
spec = C.EnvSpec(sim_config_kw={"turbulence": False, "turbulence_intensity": "light"})
eng = Engine(spec.sim, spec, n, device="cuda:0", precision="float32")
eng.seed(seed)
eng.reset()
gen = torch.Generator(device="cuda:0")
gen.manual_seed(1)
pool = torch.rand(16, n, 3, generator=gen, device="cuda:0") * 2 - 1
dump = {"y0": [], "der0": [], "wind": [], "steps": [], "action": [], "nfev": []}
for s in range(int(os.environ.get("DIAG_STEPS", "40"))):
    y0 = eng.get_block(C.FW_BLK_ODE).clone()
    d0 = eng.get_block(C.FW_BLK_DERIVED).clone()
    w0 = eng.get_block(C.FW_BLK_WIND).clone()
    st0 = eng.get_block(C.FW_BLK_STEPS).clone()
    o, r, d, t = eng.env_step(pool[s % 16], stats=True)
    nf = (eng.stats & 0xFFFF).cpu().numpy()
    bad = np.nonzero(nf > 200)[0]
    nan_state = (~torch.isfinite(eng.get_block(C.FW_BLK_ODE))).any(0).cpu().numpy()
    if nf.max() > 150 or s % 50 == 0: print("step %d max nfev %d  #>200: %d  #nan-state: %d  done %d" % (s, nf.max(), len(bad), nan_state.sum(),
                                                                       int(d.sum())), flush=True)
    for i in bad:
        dump["y0"].append(y0[:, i].double().cpu().numpy())
        dump["der0"].append(d0[:, i].double().cpu().numpy())
        dump["wind"].append(w0[:, i].double().cpu().numpy())
        dump["steps"].append(int(st0[0, i]))
        dump["action"].append(pool[s % 16][i].double().cpu().numpy())
        dump["nfev"].append(int(nf[i]))
    for i in bad[:1]:
        print("  lane %d nfev %d term %d" % (i, nf[i], int(t[i])))
        print("    y0", np.array2string(y0[:, i].cpu().numpy(), precision=4, max_line_width=200))
        print("    der0", np.array2string(d0[:, i].cpu().numpy(), precision=4), "wind", w0[:, i].cpu().numpy(),
              "steps", int(st0[0, i]))
        print("    action", pool[s % 16][i].cpu().numpy())
        print("    y1", np.array2string(eng.get_block(C.FW_BLK_ODE)[:, i].cpu().numpy(), precision=4,
                                        max_line_width=200))

np.savez("gpurun_out/slow_lanes.npz", **{k: np.array(v) for k, v in dump.items()})
