#!/usr/bin/env python3
"""Workload for the HBM-traffic split of k_env_step (tools/r04_traffic.sh runs it under rocprofv3 --pmc).

65536 aircraft, fp32, the bench's default task (streaming metrics on), turbulence off, in dispatch order:
  1. fw_reset
  2. NORESET window: 20 steps with zero actions right after the reset -- no aircraft is done, so no
     terminal observation, Monitor record, metric record or auto-reset is written
  3. 1000 untimed steps with U(-1,1) actions (the bench's --prep), then the STEADY window: 20 more
     (auto-resets happen: the done aircraft re-sample their state, metrics and observation)
Prints one JSON line with the dones of every window step, so per-launch PMC bytes can be split into
the steady-state step (window 2) and the reset path ((window 3 - window 2) / dones).
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tum_adlr_deep_reinforcement_learning_amd import config as C  # noqa: E402
from tum_adlr_deep_reinforcement_learning_amd.engine import Engine  # noqa: E402


def main():
    n, K, prep = 65536, 20, int(os.environ.get("SPLIT_PREP", "1000"))
    kw = {"steps_max": int(os.environ["SPLIT_STEPS_MAX"])} if os.environ.get("SPLIT_STEPS_MAX") else None
    spec = C.EnvSpec(config_kw=kw, sim_config_kw={"turbulence": False})
    eng = Engine(spec.sim, spec, n, device="cuda:0", precision="float32")
    eng.seed(1234)
    eng.reset()
    zero = torch.zeros(n, 3, device="cuda:0")
    g = torch.Generator(device="cuda:0")
    g.manual_seed(5)
    pool = torch.rand(16, n, 3, generator=g, device="cuda:0") * 2 - 1
    quiet = []
    for _ in range(K):
        eng.env_step(zero)
        quiet.append(int(eng.done.sum()))
    prep_dones = []
    for s in range(prep):
        eng.env_step(pool[s % 16])
        prep_dones.append(eng.done.sum())
    prep_dones = [int(x) for x in torch.stack(prep_dones).cpu()] if prep else []
    steady = []
    for s in range(K):
        eng.env_step(pool[s % 16])
        steady.append(int(eng.done.sum()))
    torch.cuda.synchronize()
    print(json.dumps({"n": n, "window": K, "prep": prep, "noreset_dones": quiet, "steady_dones": steady,
                      "prep_dones": prep_dones, "steps_max": spec.steps_max,
                      "dispatches": {"noreset": [0, K], "steady": [K + prep, 2 * K + prep]}}))
    eng.close()


if __name__ == "__main__":
    main()
