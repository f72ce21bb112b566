#!/usr/bin/env python3
"""Launch overhead probe: k_env_step launched one by one vs replayed from a captured HIP graph
(torch.cuda.CUDAGraph around fw_env_step calls on the capture stream)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tum_adlr_deep_reinforcement_learning_amd import config as C  # noqa: E402
from tum_adlr_deep_reinforcement_learning_amd.engine import Engine  # noqa: E402

n = int(os.environ.get("GP_N", "65536"))
K = 16
spec = C.EnvSpec(sim_config_kw={"turbulence": False})
eng = Engine(spec.sim, spec, n, device="cuda:0", precision="float32")
eng.seed(1234)
eng.reset()
gen = torch.Generator(device="cuda:0")
gen.manual_seed(1)
pool = torch.rand(K, n, 3, generator=gen, device="cuda:0") * 2 - 1
for s in range(40):
    eng.env_step(pool[s % K])
torch.cuda.synchronize()

reps = 20
t0 = time.perf_counter()
for r in range(reps):
    for s in range(K):
        eng.env_step(pool[s])
torch.cuda.synchronize()
eager_ms = (time.perf_counter() - t0) / (reps * K) * 1e3

g = torch.cuda.CUDAGraph()
side = torch.cuda.Stream()
side.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(side):
    eng.env_step(pool[0])  # warm on the capture stream
torch.cuda.current_stream().wait_stream(side)
torch.cuda.synchronize()
with torch.cuda.graph(g):
    for s in range(K):
        eng.env_step(pool[s])
torch.cuda.synchronize()
for _ in range(3):
    g.replay()
torch.cuda.synchronize()
t0 = time.perf_counter()
for r in range(reps):
    g.replay()
torch.cuda.synchronize()
graph_ms = (time.perf_counter() - t0) / (reps * K) * 1e3
print(json.dumps({"n": n, "eager_ms_per_step": eager_ms, "graph_ms_per_step": graph_ms}))
