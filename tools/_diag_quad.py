import sys, numpy as np, torch
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
import test_gpu_quad as T
from tum_adlr_deep_reinforcement_learning_amd import config as C
from oracle import oracle as O
DEV = "cuda:0"
spec = C.EnvSpec(sim_config_kw={"turbulence": False})
n = 256
rng = np.random.default_rng(4)
y = np.zeros((C.FW_NY, n))
ang = rng.uniform(-np.pi, np.pi, (3, n))
cr, sr = np.cos(ang / 2), np.sin(ang / 2)
y[0] = cr[0] * cr[1] * cr[2] + sr[0] * sr[1] * sr[2]
y[1] = sr[0] * cr[1] * cr[2] - cr[0] * sr[1] * sr[2]
y[2] = cr[0] * sr[1] * cr[2] + sr[0] * cr[1] * sr[2]
y[3] = cr[0] * cr[1] * sr[2] - sr[0] * sr[1] * cr[2]
y[4:7] = rng.uniform(-2, 2, (3, n))
y[7:10] = rng.uniform(-50, 50, (3, n))
y[10] = rng.uniform(-0.3, 0.3, n)
y[11] = rng.choice([-1.0, 1.0], n) * rng.uniform(9, 21, n)
y[12] = rng.uniform(-3.5, 0.1, n)
y[13:16] = rng.uniform(-0.3, 0.3, (3, n))
y[15] = rng.uniform(0.4, 0.6, n)
y[16:18] = rng.choice([-1.0, 1.0], (2, n)) * 3.491
cmd = torch.tensor(rng.uniform(-0.5, 0.5, (n, 3)), device=DEV)
cmd[:, 2] = cmd[:, 2].abs() * 2
from tum_adlr_deep_reinforcement_learning_amd.engine import Engine
res = {}
for lanes in (1, 4):
    e = Engine(spec.sim, None, n, device=DEV, precision="float64", lanes=lanes)
    e.set_block(C.FW_BLK_ODE, y); e.set_block(C.FW_BLK_DERIVED, np.zeros((8, n)))
    e.set_block(C.FW_BLK_WIND, np.zeros((3, n))); e.set_block(C.FW_BLK_STEPS, np.zeros(n, np.int32))
    succ, term = e.sim_step(cmd.double(), stats=True)
    nfev, nacc, failed = e.decode_stats(e.stats)
    res[lanes] = (e.get_block(C.FW_BLK_ODE).double().cpu().numpy(), term.cpu().numpy().copy(), nfev.cpu().numpy().copy())
    e.close()
(y1, t1, n1), (y4, t4, n4) = res[1], res[4]
o = O.sim_step(spec.sim.struct(), y.T.copy(), np.zeros((n, 8)), np.zeros((n, 3)), np.zeros((n, 6)), cmd.double().cpu().numpy())
yo, no, to = o["y"].T, o["nfev"], o["term"]
ok = (t1 == 0) & (t4 == 0)
same = ok & (n1 == n4)
tol = 0.1 * (1e-6 + 1e-3 * np.abs(y1))
r = np.abs(y1 - y4) / tol
idx = np.argwhere((r > 1) & same[None, :])
print("viol count", len(idx), "nfev diff frac", (n1 != n4).mean())
for comp, j in idx[:10]:
    print(comp, j, n1[j], n4[j], no[j], y1[comp, j], y4[comp, j], yo[comp, j] if yo.shape == y1.shape else None, r[comp, j])
print("vs oracle nfev equal 1:", (n1 == no).mean(), " 4:", (n4 == no).mean())
