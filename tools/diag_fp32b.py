import sys, numpy as np, torch
sys.path.insert(0,'tests'); sys.path.insert(0,'.')
import _fixtures as F
from tum_adlr_deep_reinforcement_learning_amd import config as C
from tum_adlr_deep_reinforcement_learning_amd.engine import Engine
d = F.load("pyfly_traj.npz")
name="pid_on"
g = lambda k: d[name + "__" + k]
spec = C.build_sim(config_kw={"turbulence": True, "turbulence_sim_length": int(g("L"))})
eng = Engine(spec, None, 1, device="cuda:0", precision="float32")
eng.set_block(C.FW_BLK_ODE, g("y")[0][:, None])
der = np.zeros((8, 1)); der[:6, 0] = g("derived")[0][:6]
eng.set_block(C.FW_BLK_DERIVED, der); eng.set_block(C.FW_BLK_WIND, g("wind")[:, None]); eng.set_block(C.FW_BLK_STEPS, np.zeros(1, np.int32))
eng.set_noise(g("noise")[None])
cmds = torch.tensor(g("cmd"), dtype=eng.dtype, device="cuda:0")
np.set_printoptions(precision=3, linewidth=200)
for s in range(12):
    eng.sim_step(cmds[s:s+1], stats=True)
    y = eng.get_block(C.FW_BLK_ODE)[:, 0].double().cpu().numpy(); r=g("y")[s+1]
    e = np.abs(y-r)/(np.abs(r)+1e-3); k=e.argmax()
    print(s, 'nfev', int(eng.stats[0]&0xFFFF), g("nfev")[s], 'worst comp', k, 'abs', abs(y[k]-r[k]), 'ref', r[k], 'rel', e[k])
