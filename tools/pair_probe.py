"""Round 6: the pair integrator (lanes = 2, csrc/fw_pair.hpp) against the one-lane integrator (with and without the
tail handoff) and the quad, on IDENTICAL states.

Part 1, PyFly.step alone (k_sim_step): a steady-state population of N aircraft (the bench's env after --prep
closed-loop steps) is copied into a sim-only handle per lanes setting; each handle then runs the same K steps
of U(-1,1)-scaled commands.  Per setting: device ms per launch (HIP events around K launches), the total and
maximum RHS evaluations per step (stats word), and the kernel's VGPR / scratch line.
Part 2, the env step (k_env_step): the same population continued K steps by an env handle per setting.

Usage: python tools/pair_probe.py [N] [K] [PREP]
"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tum_adlr_deep_reinforcement_learning_amd import config as C  # noqa: E402
from tum_adlr_deep_reinforcement_learning_amd.engine import Engine  # noqa: E402

DEV = "cuda:0"
N = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
K = int(sys.argv[2]) if len(sys.argv) > 2 else 200
PREP = int(sys.argv[3]) if len(sys.argv) > 3 else 1000
BLOCKS = [C.FW_BLK_ODE, C.FW_BLK_DERIVED, C.FW_BLK_TARGET, C.FW_BLK_WIND, C.FW_BLK_STEPS, C.FW_BLK_COMMAND,
          C.FW_BLK_ACT_RING, C.FW_BLK_GOAL]


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    spec = C.EnvSpec(sim_config_kw={"turbulence": False})
    spec.metrics_enabled = False
    src = Engine(spec.sim, spec, N, device=DEV, precision="float32", lanes=1)
    src.seed(1234)
    src.reset()
    gen = torch.Generator(device=DEV)
    gen.manual_seed(1)
    pool = torch.rand(16, N, 3, generator=gen, device=DEV) * 2 - 1
    for k in range(PREP):
        src.env_step(pool[k % 16], stats=False)
    torch.cuda.synchronize()
    log("prep done")
    state = {b: src.get_block(b).clone() for b in BLOCKS}
    acts = (torch.rand(K, N, 3, generator=gen, device=DEV) * 2 - 1).contiguous()
    # the commands PyFly.step sees: the env's action scaling (fixed_wing.py:497-504), computed on the host
    lo = torch.tensor(spec.action_scale_to_low, device=DEV, dtype=torch.float32)
    hi = torch.tensor(spec.action_scale_to_high, device=DEV, dtype=torch.float32)
    cmds = ((hi - lo) * (acts.clamp(-1, 1) + 1) / 2 + lo).contiguous()
    out = {"N": N, "K": K, "prep": PREP, "sim": {}, "env": {}}
    settings = [("lanes1", 1, None), ("lanes1_nohandoff", 1, "0"), ("lanes2", 2, None), ("lanes4", 4, None)]
    for name, lanes, th in settings:
        if th is not None:
            os.environ["FWSIM_TAIL_QUAD"] = th
        else:
            os.environ.pop("FWSIM_TAIL_QUAD", None)
        for kind in ("sim", "env"):
            eng = Engine(spec.sim, spec if kind == "env" else None, N, device=DEV, precision="float32", lanes=lanes)
            if kind == "env":
                eng.seed(1234)
                eng.reset()
                for b in BLOCKS:
                    eng.set_block(b, state[b])
            else:
                for b in (C.FW_BLK_ODE, C.FW_BLK_DERIVED, C.FW_BLK_WIND, C.FW_BLK_STEPS, C.FW_BLK_COMMAND):
                    eng.set_block(b, state[b])
            torch.cuda.synchronize()
            st = torch.cuda.current_stream()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
            nf_sum, nf_max = 0, 0
            stats = []
            for k in range(K):
                ev[k][0].record(st)
                if kind == "sim":
                    eng.sim_step(cmds[k], stats=True)
                else:
                    eng.env_step(acts[k], stats=True)
                ev[k][1].record(st)
                stats.append(eng.stats.clone())
            torch.cuda.synchronize()
            ms = np.array([a.elapsed_time(b) for a, b in ev])
            nf = torch.stack(stats).to(torch.int64) & 0xFFFF
            rec = {"lanes": lanes, "tail_quad": th or "default", "ms_mean": float(ms.mean()), "ms_p50": float(np.median(ms)),
                   "ms_min": float(ms.min()), "ms_max": float(ms.max()),
                   "nfev_sum_per_step": float(nf.sum(1).double().mean()), "nfev_max_per_step_mean": float(nf.max(1).values.double().mean()),
                   "nfev_wavemax_mean": float(nf.view(K, -1, 64).max(2).values.double().mean())}
            out[kind][name] = rec
            log(kind, name, json.dumps(rec))
            eng.close()
    src.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
