#!/usr/bin/env python3
"""Diagnose the fp32 single-step gate: worst cases (same RK45 step sequence as the reference)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import _fixtures as F  # noqa: E402
from test_gpu_parity import _run_single_steps  # noqa: E402

d = F.load("pyfly_single_step.npz")
o32 = _run_single_steps(d, "float32")
o64 = _run_single_steps(d, "float64")
rows = []
for i, r in o32.items():
    if not (d["success"][i] and r["term"] == 0):
        continue
    rel = np.abs(r["y"] - d["y1"][i]) / (np.abs(d["y1"][i]) + 1e-3)
    rel[16:] = np.abs(r["y"][16:] - d["y1"][i][16:]) / 3.4907 * 0.1  # in units of the 1e-4 gate
    same = r["nfev"] == d["nfev"][i] and r["nacc"] == d["naccept"][i]
    rows.append((rel.max() / 1e-4, i, int(rel.argmax()), same, r["nfev"], int(d["nfev"][i]), r["nacc"]))
rows.sort(reverse=True)
print("worst cases: ratio-to-bound, case, component, same-seq, nfev32, nfev_ref, nacc32")
for r in rows[:15]:
    i, c = r[1], r[2]
    print(r, "y0=%.6g y1ref=%.6g y1_32=%.6g y1_64=%.6g turb=%d" % (d["y0"][i][c], d["y1"][i][c], o32[i]["y"][c],
                                                                   o64[i]["y"][c], d["turb_on"][i]))
print("fraction over bound (same seq):", np.mean([r[0] > 1 for r in rows if r[3]]))
