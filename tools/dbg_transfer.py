"""Debug: block transfer between two engines with different lifetime counters (which state differs)."""
import sys
sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import numpy as np
import torch
from tum_adlr_deep_reinforcement_learning_amd import config as C
from tum_adlr_deep_reinforcement_learning_amd.engine import Engine
from test_gpu_r05 import _goal_spec

DEV = "cuda:0"
spec = _goal_spec()
n = 512
a, b = (Engine(spec.sim, spec, n, device=DEV, precision="float64") for _ in range(2))
a.seed(3); b.seed(4); a.reset(); b.reset()
gen = torch.Generator(device=DEV); gen.manual_seed(9)
rnd = lambda: torch.rand(n, 3, generator=gen, device=DEV, dtype=torch.float64) * 2 - 1
for _ in range(int(sys.argv[1])):
    a.env_step(rnd())
for _ in range(int(sys.argv[2])):
    b.env_step(rnd())
blocks = [C.FW_BLK_ODE, C.FW_BLK_DERIVED, C.FW_BLK_WIND, C.FW_BLK_TARGET, C.FW_BLK_STEPS, C.FW_BLK_COMMAND,
          C.FW_BLK_ACT_RING, C.FW_BLK_GOAL]
for blk in blocks:
    b.set_block(blk, a.get_block(blk))
for blk in blocks:
    print("blk", blk, "equal after set:", torch.equal(a.get_block(blk), b.get_block(blk)))
print("n_rew", spec.cfg["reward"]["factors"])
act = rnd()
oa, ra, da, ta = (x.clone() for x in a.env_step(act, auto_reset=False))
ob, rb, db, tb = b.env_step(act, auto_reset=False)
print("reward diff", float((ra - rb).abs().max()), "obs diff per col", (oa - ob).abs().max(0).values.cpu().numpy())
for blk in blocks:
    print("blk", blk, "equal after step:", torch.equal(a.get_block(blk), b.get_block(blk)))
ga, gb = a.get_block(C.FW_BLK_ACT_RING), b.get_block(C.FW_BLK_ACT_RING)
d = (ga != gb)
print("ring rows", ga.shape, "differing rows", d.any(1).nonzero().flatten().tolist(), "lanes", int(d.any(0).sum()))
print("nan a", bool(torch.isnan(ga).any()), "nan b", bool(torch.isnan(gb).any()))
j = int(d.any(0).nonzero()[0]) if d.any() else 0
sa = a.get_block(C.FW_BLK_STEPS)[0, j]
print("lane", j, "steps", int(sa) & 0xFFFF, "\na", ga[:, j].cpu().numpy().reshape(-1, 3), "\nb", gb[:, j].cpu().numpy().reshape(-1, 3))
x = a.get_block(C.FW_BLK_ACT_RING)
a.set_block(C.FW_BLK_ACT_RING, x)
print("a get-set-get identity", torch.equal(a.get_block(C.FW_BLK_ACT_RING), x))
