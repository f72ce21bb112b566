"""Host (CPU) build of the device physics, for debugging only -- not a test and not the product.

fw_device.hpp's functions are __host__ __device__; this harness compiles them for the CPU (libm in
place of the hardware rcp/exp/atan2 approximations) so a single aircraft step can be replayed and
instrumented in fp32 or fp64 without a GPU.  Used e.g. to show that the fp32 single-step deviations
of tests/test_gpu_r02.py::test_single_step_fp32_all_components_gate2 come from the fp32 algorithm
(initial-step probe cancellation), not from the device.  Usage (from the repo root):

    import sys; sys.path.insert(0, "tools/host_harness"); import harness as H
    H.sim_step(0 /*fp32*/ or 1, cfg, y, der, wind, turb, cmd)
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
OUT = os.path.join(HERE, "_build", "libfw_host_harness.so")
SRCS = [os.path.join(HERE, "fw_host_harness.hip"),
        os.path.join(ROOT, "tum_adlr_deep_reinforcement_learning_amd", "csrc", "fw_kernels.hip"),
        os.path.join(ROOT, "tum_adlr_deep_reinforcement_learning_amd", "csrc", "fw_device.hpp"),
        os.path.join(ROOT, "include", "fwsim.h")]
_lib = None
_d = ctypes.POINTER(ctypes.c_double)
_i = ctypes.POINTER(ctypes.c_int32)


def build():
    if os.path.exists(OUT) and os.path.getmtime(OUT) >= max(os.path.getmtime(s) for s in SRCS):
        return OUT
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    subprocess.check_call([hipcc, "--offload-arch=gfx950", "-O2", "-std=c++17", "-fPIC", "-shared",
                           "-ffp-contract=off", "-o", OUT, SRCS[0]])
    return OUT


def lib():
    global _lib
    if _lib is None:
        L = ctypes.CDLL(build())
        L.fwt_sim_step.restype = None
        L.fwt_sim_step.argtypes = [ctypes.c_int32, ctypes.c_void_p, ctypes.c_int64] + [_d] * 8 + [_i] * 3
        L.fwt_reset_derived.restype = None
        L.fwt_reset_derived.argtypes = [ctypes.c_void_p, _d, _d, _d, _d]
        L.fwt_philox.restype = None
        L.fwt_philox.argtypes = [ctypes.c_uint32] * 6 + [ctypes.POINTER(ctypes.c_uint32)]
        _lib = L
    return _lib


def _p(a, t=_d):
    return a.ctypes.data_as(t)


def sim_step(precision, cfg, y, der, wind, turb, cmd):
    c = lambda a: np.ascontiguousarray(a, dtype=np.float64)
    y, der, wind, turb, cmd = c(y), c(der), c(wind), c(turb), c(cmd)
    n = y.shape[0]
    yo, do, co = np.zeros_like(y), np.zeros_like(der), np.zeros_like(cmd)
    term, nfev, nacc = (np.zeros(n, np.int32) for _ in range(3))
    lib().fwt_sim_step(precision, ctypes.byref(cfg), n, _p(y), _p(der), _p(wind), _p(turb), _p(cmd), _p(yo), _p(do),
                       _p(co), _p(term, _i), _p(nfev, _i), _p(nacc, _i))
    return dict(y=yo, der=do, cmd=co, term=term, nfev=nfev, naccept=nacc)
