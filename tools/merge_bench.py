#!/usr/bin/env python3
"""Per-launch time of the VecNormalize statistics kernels on the record count of a 65536-env step
(1024 column-major block records, D = 15): fw_moments_merge, fw_vecnorm_merge_update, fw_rms_update."""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tum_adlr_deep_reinforcement_learning_amd import _native  # noqa: E402


def timed(fn, reps=200):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    lib = _native.load()
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    d, nrec = 14, int(os.environ.get("MB_NREC", "1024"))
    D = d + 1
    rec = torch.rand(1 + 2 * D, nrec, device="cuda:0", dtype=torch.float64)
    rec[0] = 64.0
    rms = torch.ones(2 * d + 4, device="cuda:0", dtype=torch.float64)
    out = torch.empty(1 + 2 * D, device="cuda:0", dtype=torch.float64)
    r = {"n_records": nrec, "D": D,
         "merge_us": timed(lambda: lib.fw_moments_merge(P(rec), nrec, D, P(out), None)),
         "merge_update_us": timed(lambda: lib.fw_vecnorm_merge_update(P(rec), nrec, d, 1, P(rms), P(out), None)),
         "rms_update_us": timed(lambda: lib.fw_rms_update(P(out), 1, d, 1, P(rms), 1, 1, None)),
         "empty_fill_us": timed(lambda: out.fill_(0.0))}
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
