"""Cost of the VecNormalize statistics at the end of the env step, on IDENTICAL states (the RK45 work, and so
the straggler tail, is the same for every variant): per state, the engine's blocks are saved, then each variant
runs one fw_env_step from the saved state, timed with HIP events on the launching stream:
  plain    no collect epilogue
  records  epilogue writing the block records, + the separate fw_vecnorm_merge_update launch (timed apart)
  tree     epilogue with the in-launch merge tree and update_from_moments (fw_collect_epilogue.merged / .rms)
Usage: python tools/epilogue_ab.py [states] [envs]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from tum_adlr_deep_reinforcement_learning_amd import _native, config as C  # noqa
from tum_adlr_deep_reinforcement_learning_amd.vec_env import FixedWingVecEnv  # noqa

S = int(sys.argv[1]) if len(sys.argv) > 1 else 24
n = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
dev = torch.device("cuda:0")
venv = FixedWingVecEnv(n, sim_config_kw={"turbulence": False}, device=dev, seed=1234, return_tensors=True,
                       info_target=False)
eng = venv.engine
lib = _native.load()
venv.reset()
g = torch.Generator(device=dev)
g.manual_seed(0)
acts = [(torch.rand(n, 3, generator=g, device=dev) * 2 - 1) for _ in range(8)]
for k in range(300):  # into the steady state
    eng.env_step(acts[k % 8])
d = eng.n_obs_values
D = d + 1
nrec, nmax = eng.collect_records()
rec = torch.zeros(nmax * (1 + 2 * D), dtype=torch.float64, device=dev)
merged = torch.zeros(1 + 2 * D, dtype=torch.float64, device=dev)
ret = torch.zeros(n, dtype=torch.float64, device=dev)
rms = torch.ones(2 * d + 4, dtype=torch.float64, device=dev)
ctrl = torch.zeros(2, dtype=torch.int32, device=dev)
blocks = [C.FW_BLK_ODE, C.FW_BLK_DERIVED, C.FW_BLK_TARGET, C.FW_BLK_WIND, C.FW_BLK_STEPS, C.FW_BLK_COMMAND,
          C.FW_BLK_ACT_RING, C.FW_BLK_GOAL]
stream = torch.cuda.current_stream(dev)
P = ctypes = __import__("ctypes")


def ptr(t):
    return P.c_void_p(t.data_ptr())


def timed(fn):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3  # us


rows = []
for s in range(S):
    snap = {b: eng.get_block(b).clone() for b in blocks}
    a = acts[s % 8]
    r = {}
    for var in ("plain", "records", "tree", "plain2"):
        for b in blocks:
            eng.set_block(b, snap[b])
        if var == "records":
            eng.set_collect_epilogue(ret=ret, gamma=0.99, records=rec, row_ctrl=ctrl)
        elif var == "tree":
            eng.set_collect_epilogue(ret=ret, gamma=0.99, records=rec, row_ctrl=ctrl, merged=merged, rms=rms)
        else:
            eng.set_collect_epilogue()
        torch.cuda.synchronize()
        r[var] = timed(lambda: eng.env_step(a))
        if var == "records":
            nr = eng.collect_records()[0]
            r["merge_kernel"] = timed(lambda: _native.check(lib.fw_vecnorm_merge_update(
                ptr(rec), nr, d, 1, ptr(rms), ptr(merged), P.c_void_p(stream.cuda_stream)), "merge_update"))
    eng.set_collect_epilogue()
    rows.append(r)
    print(json.dumps({k: round(v, 2) for k, v in r.items()}), flush=True)
    for b in blocks:
        eng.set_block(b, snap[b])
    for k in range(7):  # a new state
        eng.env_step(acts[(s + k) % 8])
mean = {k: sum(r[k] for r in rows) / len(rows) for k in rows[0]}
med = {k: sorted(r[k] for r in rows)[len(rows) // 2] for k in rows[0]}
print(json.dumps({"summary_mean_us": {k: round(v, 2) for k, v in mean.items()},
                  "summary_median_us": {k: round(v, 2) for k, v in med.items()},
                  "tree_minus_plain_us": round(mean["tree"] - mean["plain"], 2),
                  "records_plus_merge_minus_plain_us": round(mean["records"] + mean["merge_kernel"] - mean["plain"], 2),
                  "envs": n, "states": S}))
