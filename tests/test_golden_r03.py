"""CPU checks of round-3 fixtures (no GPU).

  gae_fma_column.npz  one env column on which FMA contraction of GAE's fp64 running advantage changes the
                      result: the oracle (numpy's separate multiply and add, buffers.py:321-331) and an
                      FMA-contracted recurrence differ at the recorded step, so the GPU regression test
                      (test_gpu_rollout.test_gae_kernel_no_fma_contraction) can tell them apart.
"""
from fractions import Fraction

import numpy as np

import _fixtures as F
from oracle import rollout_oracle as R


def _gae_fma(rew, val, st, lv, ld, gamma, lam):
    """The GAE recurrence with last = fma(coef, last, delta) in fp64 (exact product + sum, one rounding)."""
    g32, gl = np.float32(gamma), gamma * lam
    T = len(rew)
    v = val[T - 1]
    nnt = 0.0 if ld else 1.0
    last = (float(rew[T - 1]) + float(np.float32(g32 * lv)) * nnt) - float(v)
    out = np.zeros(T, np.float32)
    out[T - 1] = np.float32(last)
    nv, ns = v, st[T - 1]
    for t in range(T - 2, -1, -1):
        nn = np.float32(0.0) if ns else np.float32(1.0)
        b = np.float32(np.float32(g32 * nv) * nn)
        dl = np.float32(np.float32(rew[t] + b) - val[t])
        coef = np.float32(np.float32(gl) * nn)
        last = float(Fraction(float(coef)) * Fraction(last) + Fraction(float(dl)))
        out[t] = np.float32(last)
        nv, ns = val[t], st[t]
    return out


def test_gae_fma_fixture_separates_fused_and_unfused():
    d = F.load("gae_fma_column.npz")
    rew, val, st = d["rewards"], d["values"], d["starts"]
    lv, ld, t = np.float32(d["last_value"]), bool(d["last_done"]), int(d["t"])
    a_ref, _ = R.gae(rew[:, None], val[:, None], st[:, None], np.array([lv]), np.array([ld]), 0.99, 0.95)
    fused = _gae_fma(rew, val, st, lv, ld, 0.99, 0.95)
    assert fused[t] != a_ref[t, 0]
    assert np.array_equal(np.delete(fused, t), np.delete(a_ref[:, 0], t))  # the only step where they differ
