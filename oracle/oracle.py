"""ctypes front-end of the CPU oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module.  It loads oracle/_build/libfworacle.so (built from fw_oracle.c by
oracle/Makefile; ``build()`` below runs make if the library is missing).
Parity anchor: tests/golden/*.npz, generated from the reference itself.
"""
import ctypes
import os
import subprocess

import numpy as np

from tum_adlr_deep_reinforcement_learning_amd import config as C

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "libfworacle.so")
_lib = None

_d = ctypes.POINTER(ctypes.c_double)
_i32 = ctypes.POINTER(ctypes.c_int32)


def build(force=False):
    srcs = [os.path.join(HERE, "fw_oracle.c"), os.path.join(HERE, "..", "include", "fwsim.h")]
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(s) for s in srcs):
        subprocess.check_call(["make", "-s", "-C", HERE])
    return LIB


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(LIB)
        L.orc_sim_step.restype = ctypes.c_int
        L.orc_sim_step.argtypes = [ctypes.c_void_p, _d, _d, _d, _d, _d, _d, _i32, _i32]
        L.orc_sim_step_p.restype = ctypes.c_int
        L.orc_sim_step_p.argtypes = [ctypes.c_void_p, _d, _d, _d, _d, _d, _d, _d, _i32, _i32]
        L.orc_env_set_params.restype = None
        L.orc_env_set_params.argtypes = [ctypes.c_void_p, ctypes.c_void_p, _d]
        L.orc_sim_step_batch.restype = None
        L.orc_sim_step_batch.argtypes = [ctypes.c_void_p, ctypes.c_int64, _d, _d, _d, _d, _d, _d, _i32, _i32, _i32]
        L.orc_turbulence.restype = None
        L.orc_turbulence.argtypes = [ctypes.c_void_p, _d, ctypes.c_int64, ctypes.c_int64, _d]
        L.orc_reset_derived.restype = None
        L.orc_reset_derived.argtypes = [ctypes.c_void_p, _d, _d, _d, _d]
        L.orc_euler_to_quat.restype = None
        L.orc_euler_to_quat.argtypes = [_d, _d]
        L.orc_env_reset.restype = ctypes.c_int
        L.orc_env_reset.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, _d, _d, _d]
        L.orc_env_step.restype = ctypes.c_int
        L.orc_env_step.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, _d, _d, ctypes.c_int64, _d, _d,
                                   _i32, _i32]
        L.orc_env_set_state.restype = None
        L.orc_env_set_state.argtypes = [ctypes.c_void_p, _d, _d, _d, _d, ctypes.c_int32, ctypes.c_int32, _d,
                                        ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32]
        L.orc_env_observe.restype = None
        L.orc_env_observe.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, _d]
        for f in ("orc_env_state_size", "orc_sizeof_sim_config", "orc_sizeof_env_config"):
            getattr(L, f).restype = ctypes.c_int
        _lib = L
    return _lib


def _p(a, t=_d):
    return a.ctypes.data_as(t)


def sim_step(cfg, y, der, wind, turb, cmd):
    """One PyFly.step for a batch (arrays copied).  Returns dict."""
    L = lib()
    y = np.ascontiguousarray(y, dtype=np.float64).copy()
    n = y.shape[0]
    der = np.ascontiguousarray(der, dtype=np.float64).copy()
    hist = np.zeros((n, 9))
    wind = np.ascontiguousarray(wind, dtype=np.float64)
    turb = np.ascontiguousarray(turb, dtype=np.float64)
    cmd = np.ascontiguousarray(cmd, dtype=np.float64).copy()
    term = np.zeros(n, np.int32)
    nfev = np.zeros(n, np.int32)
    nacc = np.zeros(n, np.int32)
    L.orc_sim_step_batch(ctypes.byref(cfg), n, _p(y), _p(der), _p(hist), _p(wind), _p(turb), _p(cmd),
                         _p(term, _i32), _p(nfev, _i32), _p(nacc, _i32))
    return dict(y=y, der=der, hist=hist, cmd=cmd, term=term, nfev=nfev, naccept=nacc)


def sim_step_params(cfg, params, y, der, wind, turb, cmd):
    """PyFly.step of aircraft with their own parameters ``params`` [n][FW_NPARAM] (simulator parameter
    randomisation): _forces reads them, the frozen inertia / gammas / aspect ratio stay ``cfg``'s."""
    L = lib()
    n = len(y)
    out = dict(y=np.array(y, dtype=np.float64), der=np.array(der, dtype=np.float64), hist=np.zeros((n, 9)),
               cmd=np.array(cmd, dtype=np.float64), term=np.zeros(n, np.int32), nfev=np.zeros(n, np.int32),
               naccept=np.zeros(n, np.int32))
    p0 = np.ascontiguousarray(np.array(cfg.param[:]), dtype=np.float64)
    for i in range(n):
        c = C.FwSimConfig.from_buffer_copy(cfg)
        for k in range(C.FW_NPARAM):
            c.param[k] = float(params[i][k])
        yi, di, hi = out["y"][i].copy(), out["der"][i].copy(), out["hist"][i].copy()
        ci = out["cmd"][i].copy()
        nf, na = np.zeros(1, np.int32), np.zeros(1, np.int32)
        out["term"][i] = L.orc_sim_step_p(ctypes.byref(c), _p(p0), _p(yi), _p(di), _p(hi),
                                          _p(np.ascontiguousarray(wind[i], dtype=np.float64)),
                                          _p(np.ascontiguousarray(turb[i], dtype=np.float64)), _p(ci),
                                          _p(nf, _i32), _p(na, _i32))
        out["y"][i], out["der"][i], out["hist"][i], out["cmd"][i] = yi, di, hi, ci
        out["nfev"][i], out["naccept"][i] = nf[0], na[0]
    return out


def turbulence(cfg, noise, k):
    L = lib()
    noise = np.ascontiguousarray(noise, dtype=np.float64)
    out = np.zeros(6)
    L.orc_turbulence(ctypes.byref(cfg), _p(noise), noise.shape[1], int(k), _p(out))
    return out


def euler_to_quat(eul):
    q = np.zeros(4)
    lib().orc_euler_to_quat(_p(np.ascontiguousarray(eul, dtype=np.float64)), _p(q))
    return q


def reset_derived(cfg, y, euler, wind):
    der = np.zeros(8)
    lib().orc_reset_derived(ctypes.byref(cfg), _p(np.ascontiguousarray(y, dtype=np.float64)),
                            _p(np.ascontiguousarray(euler, dtype=np.float64)),
                            _p(np.ascontiguousarray(wind, dtype=np.float64)), _p(der))
    return der


class OracleEnv:
    """One FixedWingAircraft (fixed_wing.py:483-628) on the CPU oracle."""

    def __init__(self, sim_cfg, env_cfg, n_obs):
        if getattr(env_cfg, "resample_every", 0):
            # the device draws resampled targets from its Philox streams, the reference from np_random: no
            # common sequence to restate (tests/test_gpu_r05.py checks the device's draws structurally)
            raise NotImplementedError("oracle: target.resample_every")
        if any(env_cfg.rew[k].randomize for k in range(env_cfg.n_rew)):
            raise NotImplementedError("oracle: reward.randomize_scaling (the device's Philox draws)")
        # round 6 (ABI 11): pinned by the reference's own episodes on the device (tests/test_gpu_r06.py), not
        # restated here
        if any(env_cfg.target_class[k] >= C.FW_TGT["linear"] for k in range(3)) or env_cfg.on_success == 2 or \
                any(env_cfg.rew[k].kind >= C.FW_REW_SUCCESS for k in range(env_cfg.n_rew)):
            raise NotImplementedError("oracle: linear / sinusoidal targets, on_success new, success / step / goal "
                                      "rewards")
        self.L = lib()
        self.sim_cfg, self.env_cfg, self.n_obs = sim_cfg, env_cfg, n_obs
        self.buf = ctypes.create_string_buffer(self.L.orc_env_state_size())
        self.noise = np.zeros((4, 1))

    def reset(self, init, target, noise=None):
        init = np.ascontiguousarray(init, dtype=np.float64)
        target = np.ascontiguousarray(target, dtype=np.float64)
        obs = np.zeros(self.n_obs)
        t = self.L.orc_env_reset(ctypes.byref(self.sim_cfg), ctypes.byref(self.env_cfg), self.buf, _p(init),
                                 _p(target), _p(obs))
        if t:
            raise RuntimeError("reset constraint violation code %d" % t)
        self.noise = np.ascontiguousarray(noise if noise is not None else np.zeros((4, 1)), dtype=np.float64)
        return obs

    def set_state(self, y, der, wind, target, steps, steps_tgt, act_hist, goals):
        """Teacher forcing: the env continues from a device state (orc_env_set_state).  act_hist: the last
        raw actions, oldest first ([k][3]); goals: the last "all" goal bits, oldest first."""
        a = np.ascontiguousarray(np.asarray(act_hist, dtype=np.float64).reshape(-1, 3))
        g = np.ascontiguousarray(np.asarray(goals, dtype=np.uint8))
        self.L.orc_env_set_state(self.buf, _p(np.ascontiguousarray(y, dtype=np.float64)),
                                 _p(np.ascontiguousarray(der, dtype=np.float64)),
                                 _p(np.ascontiguousarray(wind, dtype=np.float64)),
                                 _p(np.ascontiguousarray(target, dtype=np.float64)), int(steps), int(steps_tgt),
                                 _p(a), a.shape[0], g.ctypes.data_as(ctypes.c_void_p), g.shape[0])

    def set_params(self, params):
        """This aircraft's own simulator parameters (after reset, which clears them)."""
        self.L.orc_env_set_params(self.buf, ctypes.byref(self.sim_cfg),
                                  _p(np.ascontiguousarray(params, dtype=np.float64)))

    def step(self, action):
        a = np.ascontiguousarray(action, dtype=np.float64)
        obs = np.zeros(self.n_obs)
        rew = np.zeros(1)
        term = np.zeros(1, np.int32)
        nfev = np.zeros(1, np.int32)
        done = self.L.orc_env_step(ctypes.byref(self.sim_cfg), ctypes.byref(self.env_cfg), self.buf, _p(a),
                                   _p(self.noise), self.noise.shape[1], _p(obs), _p(rew), _p(term, _i32),
                                   _p(nfev, _i32))
        return obs, float(rew[0]), bool(done), int(term[0]), int(nfev[0])


def term_name(code):
    if code == 0:
        return ""
    if code == C.FW_TERM_STEPS:
        return "steps"
    if code == C.FW_TERM_SUCCESS:
        return "success"
    v = code - 1
    if C.FW_V_ACT0 <= v <= C.FW_V_ACT2:
        return ["elevon_right", "elevon_left", "throttle"][v - C.FW_V_ACT0]
    return C.VAR_NAMES[v]
