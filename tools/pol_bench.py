#!/usr/bin/env python3
"""Per-launch time of the fused policy forward (fw_policy_forward, 65536 envs, SB3 default MlpPolicy) and of
the collect-mode launch (fw_collect_policy, rows + VecNormalize normalisation).  FW_POL_VALU=1 selects the
VALU kernel; FW_POL_BLOCKS_PER_CU the persistent grid."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tum_adlr_deep_reinforcement_learning_amd import _native  # noqa: E402
from tum_adlr_deep_reinforcement_learning_amd.rollout import MlpActorCritic  # noqa: E402


def main():
    n, d, A, reps = int(os.environ.get("POL_N", "65536")), 14, 3, 50
    dev = "cuda:0"
    torch.manual_seed(0)
    pol = MlpActorCritic(d, A).to(dev)
    obs = torch.randn(n, d, device=dev)
    noise = torch.randn(n, A, device=dev)
    low, high = -torch.ones(A, device=dev), torch.ones(A, device=dev)
    out = (torch.empty(n, A, device=dev), torch.empty(n, A, device=dev), torch.empty(n, device=dev),
           torch.empty(n, device=dev))
    for _ in range(3):
        pol.collect_step(obs, low, high, out=out, noise=noise)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        pol.collect_step(obs, low, high, out=out, noise=noise)
    b.record()
    torch.cuda.synchronize()
    print(json.dumps({"kernel": "valu" if os.environ.get("FW_POL_VALU") else "mfma", "n": n,
                      "blocks_per_cu": os.environ.get("FW_POL_BLOCKS_PER_CU", "1"),
                      "us_per_launch": a.elapsed_time(b) / reps * 1e3}), flush=True)


if __name__ == "__main__":
    main()
