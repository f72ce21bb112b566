#!/usr/bin/env python3
"""Steady-state env-steps/s of 65536 aircraft as S concurrent shards (one engine + HIP graph + stream each)
vs one lockstep batch; warm-up long enough for straggler (high-nfev) aircraft to appear."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tum_adlr_deep_reinforcement_learning_amd import config as C  # noqa: E402
from tum_adlr_deep_reinforcement_learning_amd.engine import Engine, StepGraph  # noqa: E402

N = int(os.environ.get("SP_N", "65536"))
warm, steps, G = int(os.environ.get("SP_WARM", "1024")), int(os.environ.get("SP_STEPS", "1024")), 16
spec = C.EnvSpec(sim_config_kw={"turbulence": False})
for S in [int(x) for x in os.environ.get("SP_SHARDS", "1,2,4,8").split(",")]:
    n = N // S
    engs, graphs, streams, pools = [], [], [], []
    for k in range(S):
        st = torch.cuda.Stream()
        with torch.cuda.stream(st):
            e = Engine(spec.sim, spec, n, device="cuda:0")
            e.seed(1234, env_offset=k * n)
            e.reset()
            g = torch.Generator(device="cuda:0")
            g.manual_seed(1 + k)
            p = torch.rand(G, n, 3, generator=g, device="cuda:0") * 2 - 1
            e.env_step(p[0])
            gr = StepGraph(e, p)
        engs.append(e), graphs.append(gr), streams.append(st), pools.append(p)
    torch.cuda.synchronize()

    def run(k):
        for _ in range(k // G):
            for s in range(S):
                with torch.cuda.stream(streams[s]):
                    graphs[s].replay()
    run(warm)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(json.dumps({"shards": S, "envs_per_shard": n, "ms_per_step": dt / steps * 1e3,
                      "env_steps_per_s": N * steps / dt}), flush=True)
    for e in engs:
        e.close()
    del graphs
