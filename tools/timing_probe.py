#!/usr/bin/env python3
"""Compare ways of timing k_env_step on the device (bench.py's roofline.kernel_ms) and the host enqueue cost."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tum_adlr_deep_reinforcement_learning_amd import config as C  # noqa: E402
from tum_adlr_deep_reinforcement_learning_amd.engine import Engine  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
spec = C.EnvSpec(sim_config_kw={"turbulence": False})
eng = Engine(spec.sim, spec, n, device="cuda:0")
eng.seed(1234)
eng.reset()
pool = torch.rand(16, n, 3, device="cuda:0") * 2 - 1
it = [0]


def launch():
    eng.env_step(pool[it[0] % 16], stats=False)
    it[0] += 1


for _ in range(50):
    launch()
torch.cuda.synchronize()
ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
K = 100
# (a) warm queue, one event pair around K launches
for _ in range(8):
    launch()
a, b = ev(), ev()
a.record()
t0 = time.perf_counter()
for _ in range(K):
    launch()
t1 = time.perf_counter()
b.record()
torch.cuda.synchronize()
print("warm block   ms/launch %.4f   host enqueue us/launch %.1f" % (a.elapsed_time(b) / K, (t1 - t0) / K * 1e6))
# (b) spin-parked queue, one event pair
torch.cuda._sleep(50_000_000)
a, b = ev(), ev()
a.record()
for _ in range(K):
    launch()
b.record()
torch.cuda.synchronize()
print("parked block ms/launch %.4f" % (a.elapsed_time(b) / K))
# (c) per-launch events
es = [(ev(), ev()) for _ in range(K)]
for x, y in es:
    x.record()
    launch()
    y.record()
torch.cuda.synchronize()
print("per-launch   ms/launch %.4f" % (sum(x.elapsed_time(y) for x, y in es) / K))
# (d) sustained wall
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(500):
    launch()
torch.cuda.synchronize()
print("wall         ms/launch %.4f" % ((time.perf_counter() - t0) / 500 * 1e3))
