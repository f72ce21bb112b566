"""A/B of the VecNormalize statistics in the fused PPO collect (65536 envs): merged + updated inside the env
step's launch (VecNormalize.merge_in_launch, 2 kernels per step) vs a separate fw_vecnorm_merge_update launch
(3 kernels).  Two collectors built from the same seeds (the same envs, policy weights and exploration draws, so
the same flight population up to the statistics' last-bit differences), one per setting, collecting T steps in
turn; each collection timed with a device sync around it.  Usage: python tools/merge_ab.py [T] [reps]"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from tum_adlr_deep_reinforcement_learning_amd.rollout import MlpActorCritic, RolloutBuffer, RolloutCollector  # noqa
from tum_adlr_deep_reinforcement_learning_amd.vec_env import FixedWingVecEnv  # noqa
from tum_adlr_deep_reinforcement_learning_amd.vec_normalize import VecNormalize  # noqa

T = int(sys.argv[1]) if len(sys.argv) > 1 else 512
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
n = int(os.environ.get("AB_ENVS", "65536"))
dev = torch.device("cuda:0")


def make(flag):
    torch.manual_seed(0)
    venv = FixedWingVecEnv(n, sim_config_kw={"turbulence": False}, device=dev, seed=1234, return_tensors=True,
                           info_target=False)
    env = VecNormalize(venv)
    env.merge_in_launch = flag
    pol = MlpActorCritic(env.observation_space.shape[0], env.action_space.shape[0]).to(dev)
    buf = RolloutBuffer(T, env.observation_space, env.action_space, device=dev, gae_lambda=0.95, gamma=0.99, n_envs=n)
    col = RolloutCollector(env, pol, buf)
    torch.manual_seed(1)
    col.collect(16)
    torch.manual_seed(2)
    col.collect(16, graph=True)
    return col


cols = {True: make(True), False: make(False)}
res = {True: [], False: []}
for r in range(reps):
    for flag in (True, False):
        col = cols[flag]
        torch.manual_seed(100 + r)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        col.collect(graph=True)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        res[flag].append(dt)
        print(json.dumps({"merge_in_launch": flag, "rep": r, "collect_s": round(dt, 5),
                          "us_per_step": round(dt / T * 1e6, 2), "env_steps_per_s": n * T / dt,
                          "kernel_nodes": [t.count(0) for t in col.graph_nodes()]}), flush=True)
print(json.dumps({"summary": {str(k): {"us_per_step_each": [round(x / T * 1e6, 2) for x in v],
                                       "mean_us_per_step": round(sum(v) / len(v) / T * 1e6, 2),
                                       "env_steps_per_s_mean": n * T * len(v) / sum(v)} for k, v in res.items()},
                  "T": T, "envs": n}))
