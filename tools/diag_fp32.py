import sys, numpy as np, torch
sys.path.insert(0,'tests'); sys.path.insert(0,'.')
import _fixtures as F
from tum_adlr_deep_reinforcement_learning_amd import config as C
from tum_adlr_deep_reinforcement_learning_amd.engine import Engine
d = F.load("pyfly_traj.npz")
for name in ["rand_off","rand_on","pid_off"]:
  for prec in ["float32","float64"]:
    g = lambda k: d[name + "__" + k]
    turb = bool(g("turb_on"))
    spec = C.build_sim(config_kw={"turbulence": turb, "turbulence_sim_length": int(g("L"))})
    eng = Engine(spec, None, 1, device="cuda:0", precision=prec)
    eng.set_block(C.FW_BLK_ODE, g("y")[0][:, None])
    der = np.zeros((8, 1)); der[:6, 0] = g("derived")[0][:6]
    eng.set_block(C.FW_BLK_DERIVED, der); eng.set_block(C.FW_BLK_WIND, g("wind")[:, None]); eng.set_block(C.FW_BLK_STEPS, np.zeros(1, np.int32))
    if turb: eng.set_noise(g("noise")[None])
    cmds = torch.tensor(g("cmd"), dtype=eng.dtype, device="cuda:0")
    errs=[]
    for s in range(len(cmds)):
        eng.sim_step(cmds[s:s+1])
        y = eng.get_block(C.FW_BLK_ODE)[:, 0].double().cpu().numpy()
        e = np.abs(y - g("y")[s+1]) / (np.abs(g("y")[s+1]) + 1e-3)
        errs.append(e)
    E=np.array(errs)
    print(name, prec, 'per-component max', np.round(E.max(0),5))
    print('   first step any comp >1e-3:', np.argmax(E.max(1)>1e-3) if (E.max(1)>1e-3).any() else None, ' excluding rates(16-18):', (E[:,:16].max()))
