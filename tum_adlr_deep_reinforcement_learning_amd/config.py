"""Configuration: reference-format JSON/dicts -> the POD structs of include/fwsim.h.

Mirrors how the reference builds its simulator and task from config files:
  * PyFly.__init__              magpie/libs/pyfly/pyfly/pyfly.py:1054-1249
    (config_kw dict recursion :1067-1073, Variable radians conversion :60-64,
     ControlVariable coefficients :296-304, Actuation.finalize limits :584-623,
     inertia "gammas" :1086-1116)
  * FixedWingAircraft.__init__  magpie/libs/fixed-wing-gym/gym_fixed_wing/fixed_wing.py:14-306
    (config_kw recursion into dicts *and lists by index* :34-40, forced
     actuation inputs / turbulence_sim_length :54-62, observation/action
     spaces :91-276)
  * set_curriculum_level        fixed_wing.py:334-412
  * DrydenGustModel             magpie/libs/pyfly/pyfly/dryden.py:51-146, as wired
    (positionally) by Wind in pyfly.py:781-783

Anything the device path does not implement raises NotImplementedError here, so
an unsupported config fails loudly at construction instead of silently
diverging from the reference.
"""
import copy
import ctypes
import json
import math
import os

import numpy as np

from . import defaults

FLOAT32_MAX = float(np.finfo(np.float32).max)
INF = float("inf")

# ---------------------------------------------------------------------------
# ctypes mirrors of include/fwsim.h
# ---------------------------------------------------------------------------
FW_NY = 19
(FW_V_ROLL, FW_V_PITCH, FW_V_YAW, FW_V_OMEGA_P, FW_V_OMEGA_Q, FW_V_OMEGA_R, FW_V_POS_N, FW_V_POS_E, FW_V_POS_D,
 FW_V_VEL_U, FW_V_VEL_V, FW_V_VEL_W, FW_V_VA, FW_V_ALPHA, FW_V_BETA, FW_V_ACT0, FW_V_ACT1, FW_V_ACT2,
 FW_V_ELEVATOR, FW_V_AILERON, FW_V_THROTTLE, FW_NVAR) = range(22)

PARAM_NAMES = [
    "mass", "Jx", "Jy", "Jz", "Jxz", "S_wing", "b", "c", "S_prop", "C_prop",
    "k_motor", "k_T_P", "k_Omega", "e", "M", "a_0",
    "C_L_0", "C_L_alpha", "C_L_q", "C_L_delta_e",
    "C_D_p", "C_D_q", "C_D_beta1", "C_D_beta2", "C_D_delta_e",
    "C_m_0", "C_m_alpha", "C_m_q", "C_m_delta_e", "C_m_fp",
    "C_Y_0", "C_Y_beta", "C_Y_p", "C_Y_r", "C_Y_delta_a", "C_Y_delta_r",
    "C_l_0", "C_l_beta", "C_l_p", "C_l_r", "C_l_delta_a", "C_l_delta_r",
    "C_n_0", "C_n_beta", "C_n_p", "C_n_r", "C_n_delta_a", "C_n_delta_r",
]
FW_NPARAM = len(PARAM_NAMES)

FW_TERM_NONE, FW_TERM_STEPS, FW_TERM_SUCCESS = 0, 100, 101

FW_OBS_STATE, FW_OBS_TARGET_ABS, FW_OBS_TARGET_REL, FW_OBS_ACTION_WINDOW, FW_OBS_TARGET_INT = range(5)
(FW_REW_STATE_ERROR, FW_REW_STATE_VALUE, FW_REW_ACTION_DELTA, FW_REW_ACTION_BOUND, FW_REW_ACTION_VALUE,
 FW_REW_STATE_INT_ERROR, FW_REW_SUCCESS, FW_REW_STEP, FW_REW_GOAL) = range(9)
FW_FUN = {"linear": 0, "quadratic": 1, "exponential": 2}
FW_TGT = {"constant": 0, "compensate": 1, "linear": 2, "sinusoidal": 3}
FW_ON_SUCCESS = {"none": 0, "done": 1, "new": 2}
FW_MAX_OBS, FW_MAX_REW, FW_MAX_WINDOW, FW_MAX_IWIN = 32, 12, 16, 256
FW_MAX_OBS_LEN, FW_MAX_OBS_HIST = 16, 64

(FW_I_ROLL, FW_I_PITCH, FW_I_YAW, FW_I_P, FW_I_Q, FW_I_R, FW_I_PN, FW_I_PE, FW_I_PD, FW_I_U, FW_I_V, FW_I_W,
 FW_I_ACT0, FW_I_ACT0_DOT, FW_I_ACT1, FW_I_ACT1_DOT, FW_I_ACT2, FW_I_ACT2_DOT, FW_I_WIND_N, FW_I_WIND_E,
 FW_I_WIND_D, FW_NINIT) = range(22)

(FW_BLK_ODE, FW_BLK_DERIVED, FW_BLK_TARGET, FW_BLK_WIND, FW_BLK_STEPS, FW_BLK_COMMAND, FW_BLK_PARAMS,
 FW_BLK_ACT_RING, FW_BLK_CMD_RING, FW_BLK_GOAL, FW_BLK_TARGET_PROPS) = range(11)
FW_DIST_GAUSSIAN, FW_DIST_UNIFORM = 0, 1

# episode-metric record (include/fwsim.h FW_M_*): name -> (first column, info keys)
FW_NMETRIC = 28
METRIC_LAYOUT = {
    "rise_time": (0, ["roll", "pitch", "Va"]), "settling_time": (3, ["roll", "pitch", "Va", "all"]),
    "overshoot": (7, ["roll", "pitch", "Va"]), "total_error": (10, ["roll", "pitch", "Va"]),
    "avg_error": (13, ["roll", "pitch", "Va"]), "control_variation": (16, ["all"]),
    "success": (17, ["roll", "pitch", "Va", "all"]), "success_time_frac": (21, ["roll", "pitch", "Va", "all"]),
    "end_error": (25, ["roll", "pitch", "Va"]),
}

# name of every variable slot (termination strings match the reference's
# ConstraintException.variable, pyfly.py:11-16)
VAR_NAMES = ["roll", "pitch", "yaw", "omega_p", "omega_q", "omega_r", "position_n", "position_e", "position_d",
             "velocity_u", "velocity_v", "velocity_w", "Va", "alpha", "beta", None, None, None,
             "elevator", "aileron", "throttle"]

STATE_VAR_IDS = {n: i for i, n in enumerate(VAR_NAMES) if n is not None}


class FwLimits(ctypes.Structure):
    _fields_ = [("value_min", ctypes.c_double), ("value_max", ctypes.c_double),
                ("constraint_min", ctypes.c_double), ("constraint_max", ctypes.c_double),
                ("init_min", ctypes.c_double), ("init_max", ctypes.c_double),
                ("wrap", ctypes.c_int32), ("pad_", ctypes.c_int32)]


class FwActuator(ctypes.Structure):
    _fields_ = [("order", ctypes.c_int32), ("pad_", ctypes.c_int32), ("tau", ctypes.c_double),
                ("omega_0", ctypes.c_double), ("zeta", ctypes.c_double), ("dot_max", ctypes.c_double)]


class FwSimConfig(ctypes.Structure):
    _fields_ = [("dt", ctypes.c_double), ("rho", ctypes.c_double), ("g", ctypes.c_double),
                ("rtol", ctypes.c_double), ("atol", ctypes.c_double),
                ("param", ctypes.c_double * FW_NPARAM),
                ("lim", FwLimits * FW_NVAR),
                ("act", FwActuator * 3),
                ("elevon", ctypes.c_int32), ("disabled_inputs", ctypes.c_int32),
                ("wind_random", ctypes.c_int32), ("max_nfev", ctypes.c_int32),
                ("wind_mag_min", ctypes.c_double), ("wind_mag_max", ctypes.c_double),
                ("wind_init_min", ctypes.c_double * 3), ("wind_init_max", ctypes.c_double * 3),
                ("turbulence", ctypes.c_int32), ("turb_len", ctypes.c_int32),
                ("dryden_g0", ctypes.c_double * 6), ("dryden_g1", ctypes.c_double * 6),
                ("dryden_state", ctypes.c_int32), ("dryden_ncut", ctypes.c_int32),
                ("dryden_ad", ctypes.c_double * 28), ("dryden_e1", ctypes.c_double * 28),
                ("dryden_b0", ctypes.c_double * 12), ("dryden_b1", ctypes.c_double * 12),
                ("dryden_c", ctypes.c_double * 12)]


class FwObsEntry(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("var", ctypes.c_int32), ("window", ctypes.c_int32),
                ("norm", ctypes.c_int32), ("mean", ctypes.c_double), ("var_", ctypes.c_double)]


class FwRewFactor(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("var", ctypes.c_int32), ("window", ctypes.c_int32),
                ("fun", ctypes.c_int32), ("shaping", ctypes.c_int32), ("randomize", ctypes.c_int32),
                ("scaling", ctypes.c_double), ("max", ctypes.c_double), ("sign", ctypes.c_double),
                ("scaling_hi", ctypes.c_double), ("value", ctypes.c_double)]


class FwRandParam(ctypes.Structure):
    _fields_ = [("param", ctypes.c_int32), ("dist", ctypes.c_int32), ("original", ctypes.c_double),
                ("var", ctypes.c_double), ("clip", ctypes.c_double)]


class FwEnvConfig(ctypes.Structure):
    _fields_ = [("steps_max", ctypes.c_int32), ("n_obs", ctypes.c_int32),
                ("obs", FwObsEntry * FW_MAX_OBS),
                ("scale_actions", ctypes.c_int32), ("has_bounds", ctypes.c_int32),
                ("scale_low", ctypes.c_double), ("scale_high", ctypes.c_double),
                ("bounds_multiplier", ctypes.c_double),
                ("act_low", ctypes.c_double * 3), ("act_high", ctypes.c_double * 3),
                ("target_class", ctypes.c_int32 * 3), ("target_wrap", ctypes.c_int32 * 3),
                ("target_low", ctypes.c_double * 3), ("target_high", ctypes.c_double * 3),
                ("target_delta", ctypes.c_double * 3), ("target_bound", ctypes.c_double * 3),
                ("streak_req", ctypes.c_int32), ("on_success", ctypes.c_int32),
                ("streak_frac", ctypes.c_double),
                ("n_rew", ctypes.c_int32), ("step_fail_timesteps", ctypes.c_int32),
                ("step_fail_value", ctypes.c_double),
                ("term_weight", ctypes.c_double * 3), ("term_present", ctypes.c_int32 * 3),
                ("reward_potential", ctypes.c_int32),
                ("rew", FwRewFactor * FW_MAX_REW),
                ("metrics", ctypes.c_int32), ("resample_every", ctypes.c_int32),
                ("rise_low", ctypes.c_double), ("rise_high", ctypes.c_double),
                ("obs_length", ctypes.c_int32), ("obs_step", ctypes.c_int32),
                ("obs_noise", ctypes.c_int32), ("integration_window", ctypes.c_int32),
                ("obs_noise_mean", ctypes.c_double), ("obs_noise_std", ctypes.c_double),
                ("n_rand", ctypes.c_int32), ("pad4_", ctypes.c_int32),
                ("rand", FwRandParam * FW_NPARAM),
                ("target_radians", ctypes.c_int32 * 3), ("pad11_", ctypes.c_int32),
                ("target_slope_low", ctypes.c_double * 3), ("target_slope_high", ctypes.c_double * 3),
                ("target_amp_low", ctypes.c_double * 3), ("target_amp_high", ctypes.c_double * 3),
                ("target_period_low", ctypes.c_double * 3), ("target_period_high", ctypes.c_double * 3),
                ("tape_skip", ctypes.c_int32), ("ang_targets", ctypes.c_int32), ("ang_max_vel", ctypes.c_double * 3)]


# ---------------------------------------------------------------------------
# config_kw recursion semantics
# ---------------------------------------------------------------------------
def _set_attrs_pyfly(parent, kws):
    """PyFly.__init__.set_config_attrs (pyfly.py:1067-1073): recurse into dicts only."""
    for attr, val in kws.items():
        if isinstance(val, dict):
            _set_attrs_pyfly(parent[attr], val)
        else:
            parent[attr] = val


def _set_attrs_env(parent, kws):
    """FixedWingAircraft.__init__.set_config_attrs (fixed_wing.py:34-40): dicts and lists by index."""
    for attr, val in kws.items():
        if isinstance(val, dict) or isinstance(parent[attr], list):
            _set_attrs_env(parent[attr], val)
        else:
            parent[attr] = val


def _load_json(path):
    with open(path) as f:
        return json.load(f)


def load_params(parameter_path=None):
    """Aircraft parameters (x8_param.mat / .json keys)."""
    if parameter_path is None:
        return dict(defaults.X8_PARAMS)
    ext = os.path.splitext(parameter_path)[1]
    if ext == ".json":
        p = _load_json(parameter_path)
    elif ext == ".mat":
        import scipy.io  # noqa: WPS433 (host-side config only)
        p = {k: v for k, v in scipy.io.loadmat(parameter_path, squeeze_me=True).items() if not k.startswith("__")}
    else:
        raise Exception("Unsupported parameter file extension.")
    out = {}
    for k in PARAM_NAMES:
        out[k] = float(np.asarray(p[k]).reshape(-1)[0]) if np.ndim(p[k]) else float(p[k])
    return out


def load_pyfly_config(config_path=None, config_kw=None):
    cfg = defaults.default_pyfly_config() if config_path is None else _load_json(config_path)
    if config_kw is not None:
        _set_attrs_pyfly(cfg, copy.deepcopy(config_kw))
    return cfg


def load_env_config(config_path=None, config_kw=None):
    cfg = defaults.default_env_config() if config_path is None else _load_json(config_path)
    if config_kw is not None:
        _set_attrs_env(cfg, copy.deepcopy(config_kw))
    return cfg


# ---------------------------------------------------------------------------
# Variables (Variable / ControlVariable __init__ semantics)
# ---------------------------------------------------------------------------
class VarSpec:
    """Host-side mirror of a reference ``Variable``/``ControlVariable`` (limits only)."""

    RAD_ATTRS = ("value_min", "value_max", "init_min", "init_max", "constraint_min", "constraint_max")

    def __init__(self, name, value_min=None, value_max=None, init_min=None, init_max=None, constraint_min=None,
                 constraint_max=None, convert_to_radians=False, wrap=False, order=None, tau=None, omega_0=None,
                 zeta=None, dot_max=None, disabled=False, **_unused):
        self.name = name
        self.value_min, self.value_max = value_min, value_max
        self.init_min = init_min if init_min is not None else value_min
        self.init_max = init_max if init_max is not None else value_max
        self.constraint_min, self.constraint_max = constraint_min, constraint_max
        if convert_to_radians:  # pyfly.py:60-64 (only the Variable attributes)
            for a in self.RAD_ATTRS:
                v = getattr(self, a)
                if v is not None:
                    setattr(self, a, float(np.radians(v)))
        self.wrap = bool(wrap)
        self.order, self.tau, self.omega_0, self.zeta, self.dot_max = order, tau, omega_0, zeta, dot_max
        self.disabled = bool(disabled)

    def limits(self):
        L = FwLimits()
        f = (lambda v, d: d if v is None else float(v))
        L.value_min, L.value_max = f(self.value_min, -INF), f(self.value_max, INF)
        L.constraint_min, L.constraint_max = f(self.constraint_min, -INF), f(self.constraint_max, INF)
        L.init_min, L.init_max = f(self.init_min, float("nan")), f(self.init_max, float("nan"))
        L.wrap = int(self.wrap)
        return L


# ---------------------------------------------------------------------------
# Dryden FIR taps (dryden.py:51-146 + scipy lsim FOH, scipy/signal/_ltisys.py)
# ---------------------------------------------------------------------------
def dryden_filters(dt_d, b, h=100.0, V_a=25.0, intensity=None):
    """Transfer functions (num, den) of the six shaping filters (dryden.py:51-146)."""
    m2f = 3.281
    f2m = 1 / m2f
    kn = 0.5144
    W20 = {None: 15, "light": 15, "moderate": 30, "severe": 45}
    if intensity not in W20:
        raise Exception("Unsupported intensity type")
    W_20 = W20[intensity] * kn
    h, b, V_a, W_20 = h * m2f, b * m2f, V_a * m2f, W_20 * m2f
    sigma_w = 0.1 * W_20
    sigma_u = sigma_w / (0.177 + 0.000823 * h) ** 0.4
    sigma_v = sigma_u
    L_u = h / (0.177 + 0.000823 * h) ** 1.2
    L_v, L_w = L_u, h
    K_u = sigma_u * math.sqrt((2 * L_u) / (math.pi * V_a))
    K_v = sigma_v * math.sqrt(L_v / (math.pi * V_a))
    K_w = sigma_w * math.sqrt(L_w / (math.pi * V_a))
    T_u = L_u / V_a
    T_v1, T_v2 = math.sqrt(3.0) * L_v / V_a, L_v / V_a
    T_w1, T_w2 = math.sqrt(3.0) * L_w / V_a, L_w / V_a
    K_p = sigma_w * math.sqrt(0.8 / V_a) * ((math.pi / (4 * b)) ** (1 / 6)) / (L_w ** (1 / 3))
    K_q = 1 / V_a
    K_r = K_q
    T_p = 4 * b / (math.pi * V_a)
    T_q = T_p
    T_r = 3 * b / (math.pi * V_a)
    return {
        "H_u": ([f2m * K_u], [T_u, 1]),
        "H_v": ([f2m * K_v * T_v1, f2m * K_v], [T_v2 ** 2, 2 * T_v2, 1]),
        "H_w": ([f2m * K_w * T_w1, f2m * K_w], [T_w2 ** 2, 2 * T_w2, 1]),
        "H_p": ([K_p], [T_p, 1]),
        "H_q": ([-K_w * K_q * T_w1, -K_w * K_q, 0], [T_q * T_w2 ** 2, T_w2 ** 2 + 2 * T_q * T_w2, T_q + 2 * T_w2, 1]),
        "H_r": ([K_v * K_r * T_v1, K_v * K_r, 0], [T_r * T_v2 ** 2, T_v2 ** 2 + 2 * T_r * T_v2, T_r + 2 * T_v2, 1]),
    }


def _tf2ss(num, den):
    """Controllable canonical realisation of a strictly proper SISO num/den."""
    den = np.atleast_1d(np.asarray(den, dtype=np.float64))
    num = np.atleast_1d(np.asarray(num, dtype=np.float64))
    num = num / den[0]
    den = den / den[0]
    n = len(den) - 1
    num = np.concatenate([np.zeros(n + 1 - len(num)), num])
    if abs(num[0]) > 0:
        raise NotImplementedError("Dryden filter with direct feed-through")
    A = np.zeros((n, n))
    A[0, :] = -den[1:]
    if n > 1:
        A[1:, :-1] = np.eye(n - 1)
    B = np.zeros((n, 1))
    B[0, 0] = 1.0
    C = num[1:].reshape(1, n)
    return A, B, C


DRYDEN_NAMES = ["H_u", "H_v", "H_w", "H_p", "H_q", "H_r"]
DRYDEN_CHAN = [0, 1, 2, 3, 1, 2]  # noise channel of each filter (dryden.py:238-252)
DRYDEN_ORDERS = [1, 2, 2, 1, 3, 3]


def _foh(A, B, dT):
    """scipy lsim's first-order-hold discretisation (scipy/signal/_ltisys.py lsim, interp=True): Ad, Bd0, Bd1
    with x[i] = Ad x[i-1] + Bd0 u[i-1] + Bd1 u[i] (column-vector form)."""
    from scipy.linalg import expm  # host-side config only
    n = A.shape[0]
    M = np.zeros((n + 2, n + 2))
    M[:n, :n] = A * dT
    M[:n, n:n + 1] = B * dT
    M[n, n + 1] = 1.0
    E = expm(M)
    Bd1 = E[:n, n + 1:n + 2]
    return E[:n, :n], E[:n, n:n + 1] - Bd1, Bd1


def dryden_bank(turb_len, dt, wingspan, intensity):
    """The six shaping filters as wired by pyfly.py:781-783 in discretised state-space form, for chunks too short
    for the FIR reduction (dryden_fir): per filter (Ad, Bd0, Bd1, C, E1) with E1 = e^{A L^2}, the zero-input
    propagation lsim applies between chunks (X0 carried from the previous chunk's last state over
    t[0] = c L^2, scipy lsim: ``xout[0] = X0 @ expm(A.T * T[0])``).  Returns the flat fw_sim_config arrays and
    ncut, the first chunk from which the carried state is negligible (max |E1^c| < 1e-30)."""
    from scipy.linalg import expm  # host-side config only
    L = int(turb_len)
    if L < 2:
        raise NotImplementedError("Dryden chunk length %d: lsim of a single sample" % L)
    filt = dryden_filters(turb_len, dt, wingspan, 25.0, intensity)
    dT = (L * float(turb_len)) / (L - 1)
    T0 = L * float(turb_len)
    ad, e1, b0, b1, cc, ncut = [], [], [], [], [], 1
    for name in DRYDEN_NAMES:
        A, B, C = _tf2ss(*filt[name])
        Ad, Bd0, Bd1 = _foh(A, B, dT)
        E1 = expm(A * T0)
        ad += list(Ad.ravel())
        e1 += list(E1.ravel())
        b0 += list(Bd0[:, 0])
        b1 += list(Bd1[:, 0])
        cc += list(C[0])
        P, c = E1.copy(), 1
        while np.max(np.abs(P)) >= 1e-30:
            c += 1
            P = P @ E1
            if c > 64:
                raise NotImplementedError("Dryden chunk length %d: the carried filter state does not decay within "
                                          "64 chunks" % L)
        ncut = max(ncut, c)
    return dict(ad=ad, e1=e1, b0=b0, b1=b1, c=cc, ncut=ncut)


def dryden_bank_sim(bank, noise, L, k_end):
    """Restatement of the filter bank for tests: outputs [6][k_end] for N(0,1) noise [4][len] (wrapped)."""
    noise = np.asarray(noise, dtype=np.float64)
    ln = noise.shape[1]
    s = math.sqrt(math.pi / L)
    out = np.zeros((6, k_end))
    off_a = off_x = 0
    for f, n in enumerate(DRYDEN_ORDERS):
        Ad = np.array(bank["ad"][off_a:off_a + n * n]).reshape(n, n)
        E1 = np.array(bank["e1"][off_a:off_a + n * n]).reshape(n, n)
        B0 = np.array(bank["b0"][off_x:off_x + n])
        B1 = np.array(bank["b1"][off_x:off_x + n])
        Cf = np.array(bank["c"][off_x:off_x + n])
        x = np.zeros(n)
        for k in range(k_end):
            c, j = divmod(k, L)
            if j == 0:
                if c > 0:
                    x = np.linalg.matrix_power(E1, c) @ x if c < bank["ncut"] else np.zeros(n)
            else:
                x = Ad @ x + B0 * (s * noise[DRYDEN_CHAN[f], (k - 1) % ln]) + B1 * (s * noise[DRYDEN_CHAN[f], k % ln])
            out[f, k] = Cf @ x
        off_a += n * n
        off_x += n
    return out


def dryden_fir(turb_len, dt, wingspan, intensity):
    """FIR taps g0 (u[k-1]) and g1 (u[k]) of the six Dryden outputs for the reference's wiring, or None when
    the chunk is too short for the reduction (then dryden_bank, the stateful filter bank, applies).

    Wind passes (sim_length, dt, b) positionally into DrydenGustModel(dt, b, h)
    (pyfly.py:781-783 vs dryden.py:52), so the filter's noise spacing is
    ``turb_len`` s, its "wingspan" ``dt`` and its altitude the real wingspan.
    lsim (first-order hold, _foh) then steps L*L/(L-1) seconds per sample; where the
    state transition e^{A*dT} vanishes (|Ad| <= 1e-30) each output is exactly
    g0*u[k-1] + g1*u[k] (and 0 at the first sample of every chunk).
    """
    filt = dryden_filters(turb_len, dt, wingspan, 25.0, intensity)
    L = int(turb_len)
    dT = (L * float(turb_len)) / (L - 1) if L > 1 else float(turb_len)
    g0, g1 = np.zeros(6), np.zeros(6)
    for i, name in enumerate(["H_u", "H_v", "H_w", "H_p", "H_q", "H_r"]):
        A, B, C = _tf2ss(*filt[name])
        Ad, Bd0, Bd1 = _foh(A, B, dT)
        if np.max(np.abs(Ad)) > 1e-30:
            return None  # not reducible: the filters keep state between samples
        g0[i] = float((C @ Bd0)[0, 0])
        g1[i] = float((C @ Bd1)[0, 0])
    return g0, g1


# ---------------------------------------------------------------------------
# Simulator config
# ---------------------------------------------------------------------------
class SimSpec:
    """Everything the host needs about a PyFly configuration."""

    def __init__(self, cfg, params):
        self.cfg = cfg
        self.params = params
        # RHS-evaluation budget of one RK45 step (fw_sim_config.max_nfev; 0 = the library default 65535, a safety net: scipy has none).
        # scipy has none; exhausting it is handled like solve_ivp's TOO_SMALL_STEP failure.
        self.max_nfev = 0
        self.vars = {}
        for v in cfg["variables"]:
            self.vars[v["name"]] = VarSpec(**v)
        for n in ["elevator", "aileron", "rudder", "throttle"]:  # pyfly.py:1217-1221
            if n not in self.vars:
                self.vars[n] = VarSpec(name=n, disabled=True)
        missing = set(["alpha", "beta", "roll", "pitch", "yaw", "omega_p", "omega_q", "omega_r", "position_n",
                       "position_e", "position_d", "velocity_u", "velocity_v", "velocity_w", "Va", "elevator",
                       "aileron", "rudder", "throttle"]) - set(self.vars)
        if missing:
            raise Exception("Missing required variable(s) in config file: {}".format(",".join(missing)))
        self.dynamics = list(cfg["actuation"]["dynamics"])
        self.inputs = list(cfg["actuation"]["inputs"])
        self.elevon = "elevon_left" in self.dynamics or "elevon_right" in self.dynamics
        if self.elevon:
            if self.dynamics != ["elevon_right", "elevon_left", "throttle"]:
                raise NotImplementedError("elevon dynamics must be ordered [elevon_right, elevon_left, throttle]")
            er, el = self.vars["elevon_right"], self.vars["elevon_left"]
            # Actuation.finalize pyfly.py:599-623
            self.vars["elevator"].value_min = (er.value_min + el.value_min) / 2
            self.vars["elevator"].value_max = (er.value_max + el.value_max) / 2
            self.vars["aileron"].value_min = (-er.value_max + el.value_min) / 2
            self.vars["aileron"].value_max = (-er.value_min + el.value_max) / 2
        elif self.dynamics != ["elevator", "aileron", "throttle"]:
            raise NotImplementedError("actuation.dynamics must be elevons+throttle or [elevator, aileron, throttle]")
        if self.inputs != ["elevator", "aileron", "throttle"]:
            raise NotImplementedError("actuation.inputs must be [elevator, aileron, throttle]")
        for n in self.dynamics:
            o = self.vars[n].order
            if o not in (1, 2):
                raise ValueError("actuator %s must have order 1 or 2" % n)
        if any(k in cfg for k in ("recorder",)):
            raise NotImplementedError("recorder")

    # attitude constraints during integration would re-check the previous saved
    # attitude only (pyfly.py:1865-1869) -- a no-op; value limits on roll/pitch/yaw are honoured at save.

    def struct(self):
        c = FwSimConfig()
        cfg = self.cfg
        c.dt, c.rho, c.g = float(cfg["dt"]), float(cfg["rho"]), float(cfg["g"])
        c.rtol, c.atol = 1e-3, 1e-6
        c.max_nfev = int(self.max_nfev)
        for i, n in enumerate(PARAM_NAMES):
            c.param[i] = float(self.params[n])
        slot = {}
        for n in ["roll", "pitch", "yaw", "omega_p", "omega_q", "omega_r", "position_n", "position_e", "position_d",
                  "velocity_u", "velocity_v", "velocity_w", "Va", "alpha", "beta", "elevator", "aileron", "throttle"]:
            slot[n] = STATE_VAR_IDS[n]
        for n, i in slot.items():
            c.lim[i] = self.vars[n].limits()
        for j, n in enumerate(self.dynamics):
            v = self.vars[n]
            c.lim[FW_V_ACT0 + j] = v.limits()
            a = c.act[j]
            a.order = int(v.order)
            a.tau = float(v.tau) if v.tau is not None else 0.0
            a.omega_0 = float(v.omega_0) if v.omega_0 is not None else 0.0
            a.zeta = float(v.zeta) if v.zeta is not None else 0.0
            a.dot_max = float(v.dot_max) if v.dot_max is not None else INF
        c.elevon = int(self.elevon)
        c.disabled_inputs = (1 if self.vars["elevator"].disabled else 0) | (2 if self.vars["aileron"].disabled else 0)
        mmin, mmax = cfg.get("wind_magnitude_min"), cfg.get("wind_magnitude_max")
        c.wind_random = int(not (mmin is None and mmax is None))
        c.wind_mag_min = float(mmin) if mmin is not None else 0.0
        c.wind_mag_max = float(mmax) if mmax is not None else 0.0
        for i, n in enumerate(["wind_n", "wind_e", "wind_d"]):
            v = self.vars.get(n)
            c.wind_init_min[i] = float(v.init_min) if v is not None and v.init_min is not None else 0.0
            c.wind_init_max[i] = float(v.init_max) if v is not None and v.init_max is not None else 0.0
        c.turbulence = int(bool(cfg["turbulence"]))
        c.turb_len = int(cfg.get("turbulence_sim_length", 300))
        if c.turbulence:
            fir = dryden_fir(c.turb_len, c.dt, float(self.params["b"]), cfg["turbulence_intensity"])
            if fir is not None:
                for i in range(6):
                    c.dryden_g0[i], c.dryden_g1[i] = fir[0][i], fir[1][i]
            else:  # short chunks: the stateful filter bank (fw_sim_config.dryden_state)
                bank = dryden_bank(c.turb_len, c.dt, float(self.params["b"]), cfg["turbulence_intensity"])
                c.dryden_state, c.dryden_ncut = 1, int(bank["ncut"])
                for name, n in (("ad", 28), ("e1", 28), ("b0", 12), ("b1", 12), ("c", 12)):
                    arr = getattr(c, "dryden_" + name)
                    for i in range(n):
                        arr[i] = bank[name][i]
        return c


def build_sim(config_path=None, parameter_path=None, config_kw=None):
    return SimSpec(load_pyfly_config(config_path, config_kw), load_params(parameter_path))


# ---------------------------------------------------------------------------
# Env config
# ---------------------------------------------------------------------------
TARGET_INDEX = {"roll": 0, "pitch": 1, "Va": 2}
# attitude_angular targets (fixed_wing.py:671-675, 1558-1642): include/fwsim.h FW_TGT_OMEGA_P + k
ANG_TARGETS = ["omega_p", "omega_q", "omega_r"]
ANG_INDEX = {n: 3 + k for k, n in enumerate(ANG_TARGETS)}
ACTION_INDEX = {"elevator": 0, "aileron": 1, "throttle": 2}


class EnvSpec:
    """Host-side mirror of FixedWingAircraft's configuration (fixed_wing.py:14-306)."""

    def __init__(self, config_path=None, config_kw=None, sim_config_path=None, sim_parameter_path=None,
                 sim_config_kw=None, curriculum_level=1):
        self.cfg = load_env_config(config_path, config_kw)
        cfg = self.cfg
        skw = copy.deepcopy(sim_config_kw) if sim_config_kw else {}
        skw.update({"actuation": {"inputs": [a["name"] for a in cfg["action"]["states"]]}})
        skw["turbulence_sim_length"] = cfg["steps_max"]  # fixed_wing.py:62
        self.sim = build_sim(sim_config_path, sim_parameter_path, skw)
        self.steps_max = int(cfg["steps_max"])
        obs_cfg = cfg["observation"]
        # observation history (get_observation, fixed_wing.py:1133-1258): `length` rows, `step` apart
        self.obs_length = int(obs_cfg.get("length", 1))
        self.obs_step = int(obs_cfg.get("step", 1))
        self.obs_shape_kind = obs_cfg.get("shape", "vector")
        if self.obs_shape_kind not in ("vector", "matrix"):
            raise ValueError("Unexpected observation shape {}".format(self.obs_shape_kind))
        if not 1 <= self.obs_length <= FW_MAX_OBS_LEN or self.obs_step < 1:
            raise NotImplementedError("observation.length %d / step %d" % (self.obs_length, self.obs_step))
        if (self.obs_length - 1) * self.obs_step + 2 > FW_MAX_OBS_HIST:
            raise NotImplementedError("observation history deeper than %d steps" % FW_MAX_OBS_HIST)
        # observation noise: val += np_random.normal(loc=mean, scale=var) (fixed_wing.py:1241-1242);
        # a zero-mean, zero-scale draw adds exactly 0.0, so it is not drawn at all
        noise = obs_cfg.get("noise")
        self.obs_noise = None
        if noise is not None and (noise.get("var", 0) != 0 or noise.get("mean", 0) != 0):
            self.obs_noise = (float(noise.get("mean", 0)), float(noise.get("var", 0)))
        if cfg["reward"].get("form", "absolute") not in ("absolute", "potential"):
            raise NotImplementedError("reward.form %r" % cfg["reward"].get("form"))
        if cfg["target"].get("on_success", "none") not in FW_ON_SUCCESS:
            raise ValueError("Unexpected goal action {}".format(cfg["target"].get("on_success")))  # fixed_wing.py:553-559
        self.sim_attrs = self._parse_sim_attrs(cfg.get("simulator", {}))
        self.rand_params = self._parse_model(cfg.get("simulator", {}).get("model"))
        self.scale_actions = bool(cfg["action"].get("scale_space", False))
        self.metrics_enabled = True  # track cfg["metrics"] on the device (False: skip that state traffic)
        # the spaces (and derived normalisation constants) read the simulator's bounds BEFORE the env config's
        # "simulator" states are applied: the reference builds them in __init__ (fixed_wing.py:95-247) and
        # applies those states in set_curriculum_level afterwards (:300)
        self._build_spaces()
        self.set_curriculum_level(curriculum_level)
        self.ang_targets = self._check_targets()

    def _check_targets(self):
        """[roll, pitch, Va], optionally followed by omega_p / q / r of class attitude_angular (all three: the
        reference computes all three rates, fixed_wing.py:741-746, reading each one's props).  Returns whether
        the attitude_angular targets are present."""
        cfg = self.cfg
        states = cfg["target"]["states"]
        tnames = [s["name"] for s in states]
        if tnames[:3] != ["roll", "pitch", "Va"] or sorted(tnames[3:]) not in ([], sorted(ANG_TARGETS)):
            raise NotImplementedError("targets must be [roll, pitch, Va] (+ omega_p / q / r of class attitude_angular)")
        if len(tnames) == 3:
            return False
        for st in states[3:]:
            if st.get("class", "constant") != "attitude_angular":
                raise NotImplementedError("target %s of class %r" % (st["name"], st.get("class", "constant")))
            if st.get("bound") is not None:
                # the goal status would count an omega target (fixed_wing.py:1346-1361): the device's goal history
                # holds roll / pitch / Va
                raise NotImplementedError("a bound on attitude_angular target %s" % st["name"])
        if cfg.get("metrics"):
            raise NotImplementedError("episode metrics with attitude_angular targets (get_metric covers every target)")
        if self.obs_length > 1 or self.obs_noise is not None:
            raise NotImplementedError("observation history / noise with attitude_angular targets")
        return True

    # PyFly attributes PyFly.step / reset read (pyfly.py:1251-1482): the numbers among them change the dynamics
    # (dt: the RK45 interval, cur_sim_step: the turbulence sample index), the objects the next step would fail on
    _SIM_STEP_NUMBERS = ("dt", "cur_sim_step")
    _SIM_STEP_OBJECTS = ("actuation", "cfg", "energy_states", "model_inputs", "params", "plots", "rec", "state",
                         "viewer", "wind")

    @classmethod
    def _parse_sim_attrs(cls, sim):
        """The other keys of the "simulator" block (sample_simulator_parameters, fixed_wing.py:802-813): at every
        reset np_random.choice(values, p=probabilities) or np_random.uniform(low, high) (bool if low is a bool)
        is set as an attribute of the PyFly object.  PyFly's step and reset never read an attribute of any other
        name, so for those the draw leaves the episode unchanged: they are accepted (validated as the reference
        reads them) and have no device-side effect -- the device draws nothing for them (its draws are keyed
        per purpose, so no other draw moves).  Randomised dt / cur_sim_step change the integration interval or
        the turbulence index per episode: refused.  An object attribute replaced by a number makes the
        reference's next step fail: refused as invalid."""
        out = {}
        for key, value in sim.items():
            if key in ("states", "model"):
                continue
            if key in cls._SIM_STEP_NUMBERS:
                raise NotImplementedError("randomised simulator attribute %r (a per-episode %s on the device)" % (
                    key, "integration interval" if key == "dt" else "turbulence sample index"))
            if key in cls._SIM_STEP_OBJECTS:
                raise ValueError("simulator attribute %r is a PyFly object; a sampled number in its place breaks "
                                 "PyFly.step" % key)
            if "values" in value:
                probs = value.get("probabilities")
                if probs is not None and len(probs) != len(value["values"]):
                    raise ValueError("simulator attribute %r: probabilities and values differ in length" % key)
                out[key] = ("choice", list(value["values"]), probs)
            else:
                out[key] = ("uniform", value["low"], value["high"])  # (KeyError without low / high, as there)
        return out

    def _parse_model(self, m):
        """The "simulator": {"model": ...} block -> fw_rand_param entries (sample_simulator_parameters,
        fixed_wing.py:748-800): gaussian N(original, var) clipped to original -+ clip, or uniform
        U(original -+ var); "relative" var_type scales var by |original| and clip by original (sign kept,
        like the reference); parameters whose original value is 0 are skipped, as there."""
        if not m:
            return []
        dist = m.get("distribution", "gaussian")
        if dist not in ("gaussian", "uniform"):
            raise ValueError("Unexpected distribution type {}".format(dist))
        out = []
        for pa in m["parameters"]:
            name = pa["name"]
            if name not in PARAM_NAMES:
                raise NotImplementedError("randomised parameter %r (not a simulator parameter read by the "
                                          "dynamics)" % name)
            orig = pa.get("original")
            orig = float(self.sim.params[name] if orig is None else orig)
            if orig == 0:
                continue
            var = float(pa.get("var", m["var"]))
            if m["var_type"] == "relative":
                var *= abs(orig)
            clip = pa.get("clip", m.get("clip"))
            if clip is not None and dist == "gaussian":
                clip = float(clip) * (orig if m["var_type"] == "relative" else 1.0)
            else:
                clip = None
            out.append((PARAM_NAMES.index(name), FW_DIST_GAUSSIAN if dist == "gaussian" else FW_DIST_UNIFORM,
                        orig, var, clip))
        return out

    # fixed_wing.py:334-412
    def set_curriculum_level(self, level):
        assert 0 <= level <= 1
        self.curriculum_level = level
        cfg = self.cfg
        for state in cfg.get("simulator", {}).get("states", []):
            state = copy.copy(state)
            name = state.pop("name")
            rad = state.pop("convert_to_radians", False)
            var = self.sim.vars[name]
            for prop, val in state.items():
                if val is not None:
                    if "constraint" not in prop and any(m in prop for m in ["min", "max"]):
                        midpoint = (state[prop[:-3] + "max"] + state[prop[:-3] + "min"]) / 2
                        val = midpoint - level * (midpoint - val)
                    if rad:
                        val = float(np.radians(val))
                setattr(var, prop, val)
        self.target_props = {}
        for st in cfg["target"]["states"]:
            props = {}
            for k, v in st.items():
                if k == "name":
                    continue
                if k not in ["bound", "class"] and v is not None and not isinstance(v, bool):
                    if k == "low":
                        midpoint = (st["high"] + v) / 2
                    elif k == "high":
                        midpoint = (v + st["low"]) / 2
                    else:
                        midpoint = 0
                    v = midpoint - level * (midpoint - v)
                props[k] = v
            self.target_props[st["name"]] = props

    def _state_bound(self, name, which):
        v = self.sim.vars[name]
        if which == "high":
            if v.value_max is not None:
                return v.value_max
            if v.constraint_max is not None:
                return v.constraint_max
            return FLOAT32_MAX
        if v.value_min is not None:
            return v.value_min
        if v.constraint_min is not None:
            return v.constraint_min
        return -FLOAT32_MAX

    def _build_spaces(self):
        cfg = self.cfg
        lo, hi = [], []
        self._obs_bounds = []  # (high, low) per entry, before the relative-target span (fixed_wing.py:98-125)
        for o in cfg["observation"]["states"]:
            h = o.get("high")
            if h is None:
                h = self._state_bound(o["name"], "high")
            elif o.get("convert_to_radians", False):
                h = float(np.radians(h))
            low = o.get("low")
            if low is None:
                low = self._state_bound(o["name"], "low")
            elif o.get("convert_to_radians", False):
                low = float(np.radians(low))
            self._obs_bounds.append((h, low))
            if o["type"] == "target" and o.get("value") == "relative":
                if h != FLOAT32_MAX and low != -FLOAT32_MAX:
                    hi.append(h - low)
                    lo.append(low - h)
                else:
                    hi.append(FLOAT32_MAX)
                    lo.append(-FLOAT32_MAX)
            else:
                hi.append(h)
                lo.append(low)
        self.obs_low = np.array(lo, dtype=np.float32)
        self.obs_high = np.array(hi, dtype=np.float32)
        if self.obs_length > 1:  # fixed_wing.py:177-191: repeat per row (vector) or stack rows (matrix)
            L = self.obs_length
            if self.obs_shape_kind == "vector":
                self.obs_low, self.obs_high = np.tile(self.obs_low, L), np.tile(self.obs_high, L)
            else:
                self.obs_low, self.obs_high = np.tile(self.obs_low, (L, 1)), np.tile(self.obs_high, (L, 1))
        alo, ahi, slo, shi = [], [], [], []
        for a in cfg["action"]["states"]:
            s_hi = self._state_bound(a["name"], "high")
            s_lo = self._state_bound(a["name"], "low")
            sp_hi, sp_lo = a.get("high"), a.get("low")
            ahi.append(FLOAT32_MAX if sp_hi == "max" else (s_hi if sp_hi is None else sp_hi))
            alo.append(-FLOAT32_MAX if sp_lo == "max" else (s_lo if sp_lo is None else sp_lo))
            shi.append(s_hi)
            slo.append(s_lo)
        self.action_space_low = np.array(alo, dtype=np.float32)
        self.action_space_high = np.array(ahi, dtype=np.float32)
        self.action_scale_to_low = np.array(slo, dtype=np.float64)
        self.action_scale_to_high = np.array(shi, dtype=np.float64)

    @property
    def n_obs_row(self):
        """Entries of one observation row (the observation.states list)."""
        return len(self.cfg["observation"]["states"])

    @property
    def n_obs(self):
        """Values of one env's observation: length rows x n_obs_row entries (flat on the device)."""
        return self.obs_length * self.n_obs_row

    @property
    def obs_shape(self):
        return tuple(self.obs_low.shape)

    def obs_names(self):
        out = []
        for o in self.cfg["observation"]["states"]:
            out.append(o["name"] + ("_target" if o["type"] == "target" else "") +
                       ("_delta" if o["type"] == "action" else ""))
        return out

    def struct(self):
        cfg = self.cfg
        e = FwEnvConfig()
        e.steps_max = self.steps_max
        e.n_rand = len(self.rand_params)
        for r, (pi, dist, orig, var, clip) in enumerate(self.rand_params):
            R = e.rand[r]
            R.param, R.dist, R.original, R.var = pi, dist, orig, var
            R.clip = float("nan") if clip is None else clip
        states = cfg["observation"]["states"]
        if len(states) > FW_MAX_OBS:
            raise NotImplementedError("more than %d observation entries" % FW_MAX_OBS)
        e.n_obs = len(states)
        norm_all = bool(cfg["observation"].get("normalize", False))
        for i, o in enumerate(states):
            E = e.obs[i]
            t = o["type"]
            if t == "state":
                if o["name"] not in STATE_VAR_IDS:
                    raise NotImplementedError("observation of state %r" % o["name"])
                E.kind, E.var = FW_OBS_STATE, STATE_VAR_IDS[o["name"]]
            elif t == "target":
                val = o.get("value")
                if val == "absolute":
                    E.kind = FW_OBS_TARGET_ABS
                elif val == "relative":
                    E.kind = FW_OBS_TARGET_REL
                elif val == "integrator":  # fixed_wing.py:1160-1182
                    E.kind = FW_OBS_TARGET_INT
                else:
                    raise NotImplementedError("target observation value %r" % val)
                if o["name"] in ANG_INDEX and self.ang_targets:
                    if val == "integrator":
                        raise NotImplementedError("integrator observation of an attitude_angular target")
                    E.var = ANG_INDEX[o["name"]]
                else:
                    E.var = TARGET_INDEX[o["name"]]
            elif t == "action":
                E.kind, E.var = FW_OBS_ACTION_WINDOW, ACTION_INDEX[o["name"]]
                E.window = int(o.get("window_size", 1))
                if E.window > FW_MAX_WINDOW:
                    raise NotImplementedError("action window > %d" % FW_MAX_WINDOW)
            else:
                raise Exception("Unexpected observation variable type: {}".format(t))
            E.norm = int(norm_all and o.get("norm", True))
            E.mean = float(o.get("mean", 0.0) or 0.0)
            E.var_ = float(o.get("var", 1.0) or 1.0)
            if norm_all:  # mean / var not given: derived from the bounds (fixed_wing.py:142-161), as written there
                h, low = self._obs_bounds[i]
                finite = h != FLOAT32_MAX and low != -FLOAT32_MAX
                if o.get("mean") is None:
                    E.mean = float(h - low) if finite else 0.0
                if o.get("var") is None:
                    E.var_ = float((h - low) / (4 ** 2)) if finite else 1.0
        a = cfg["action"]
        e.scale_actions = int(self.scale_actions)
        e.scale_low = float(a.get("scale_low", -1) if a.get("scale_low") is not None else -1)
        e.scale_high = float(a.get("scale_high", 1) if a.get("scale_high") is not None else 1)
        bm = a.get("bounds_multiplier")
        e.has_bounds = int(bm is not None)
        e.bounds_multiplier = float(bm) if bm is not None else 0.0
        for i in range(3):
            e.act_low[i] = float(self.action_scale_to_low[i])
            e.act_high[i] = float(self.action_scale_to_high[i])
        tnames = [s["name"] for s in cfg["target"]["states"]]
        for k, name in enumerate(ANG_TARGETS):  # fixed_wing.py:671-675, 741-746, 1558-1642
            if self.ang_targets:
                e.ang_max_vel[k] = float(self.target_props[name].get("max_vel", np.radians(180)))
        e.ang_targets = int(self.ang_targets)
        for i, name in enumerate(tnames[:3]):
            p = self.target_props[name]
            cls = p.get("class", "constant")
            if cls == "attitude_angular":  # _get_next_target (:1455-1459)
                raise ValueError("Invalid state for class attitude_angular {}".format(name))
            if cls not in FW_TGT:
                raise ValueError("Unexpected target class {}".format(cls))
            if cls == "compensate" and name != "Va":
                # Va only (fixed_wing.py:1378-1431: pitch raises NotImplementedError, others ValueError)
                raise NotImplementedError("compensate target for %s" % name)
            if cls == "compensate" and self.target_props["pitch"].get("class", "constant") not in \
                    ("constant", "linear", "sinusoidal"):
                raise ValueError("Invalid combination of state Va target class compensate and pitch target class "
                                 "{}".format(self.target_props["pitch"].get("class")))
            e.target_class[i] = FW_TGT[cls]
            e.target_wrap[i] = int(self.sim.vars[name].wrap)
            rad = p.get("convert_to_radians", False)
            cv = (lambda x: float(np.radians(x)) if rad else float(x))
            e.target_low[i] = cv(p["low"])
            e.target_high[i] = cv(p["high"])
            e.target_delta[i] = cv(p["delta"]) if p.get("delta") is not None else float("nan")
            e.target_bound[i] = cv(p["bound"]) if p.get("bound") is not None else float("nan")
            # the class draws of sample_target (fixed_wing.py:698-722), in config units: np.radians on the device
            e.target_radians[i] = int(bool(rad))
            if cls == "linear":
                e.target_slope_low[i], e.target_slope_high[i] = float(p["slope_low"]), float(p["slope_high"])
            elif cls == "sinusoidal":
                e.target_amp_low[i], e.target_amp_high[i] = float(p["amplitude_low"]), float(p["amplitude_high"])
                e.target_period_low[i] = float(p.get("period_low", 250))
                e.target_period_high[i] = float(p.get("period_high", 500))
        e.tape_skip = len(self.sim_attrs)  # (inert simulator attributes: their reset draws, skipped on a tape)
        t = cfg["target"]
        names = [m["name"] for m in cfg.get("metrics", [])]
        unknown = set(names) - set(METRIC_LAYOUT)
        if unknown:
            raise NotImplementedError("metrics %s" % sorted(unknown))
        e.metrics = int(bool(names) and self.metrics_enabled)
        rise = [m for m in cfg.get("metrics", []) if m["name"] == "rise_time"]
        e.rise_low = float(rise[0].get("low", 0.1)) if rise else 0.1
        e.rise_high = float(rise[0].get("high", 0.9)) if rise else 0.9
        e.obs_length, e.obs_step = self.obs_length, self.obs_step
        if self.obs_noise is not None:
            e.obs_noise, (e.obs_noise_mean, e.obs_noise_std) = 1, self.obs_noise
        e.streak_req = int(t["success_streak_req"])
        if e.streak_req > 4096:  # (the goal-history ring grows with it: 4096 entries = 2 KB per aircraft)
            raise NotImplementedError("success_streak_req > 4096")
        e.streak_frac = float(t["success_streak_fraction"])
        e.on_success = FW_ON_SUCCESS[t.get("on_success", "none")]  # fixed_wing.py:548-559
        r = cfg["reward"]
        fails = r.get("step_fail", 0)
        e.step_fail_timesteps = int(fails == "timesteps")
        e.step_fail_value = 0.0 if fails == "timesteps" else float(fails)
        e.reward_potential = int(r.get("form", "absolute") == "potential")  # fixed_wing.py:566, 1080-1108
        e.resample_every = int(cfg["target"].get("resample_every", 0) or 0)  # fixed_wing.py:570-574
        e.integration_window = int(cfg.get("integration_window", 0) or 0)   # fixed_wing.py:83
        if e.integration_window > FW_MAX_IWIN:
            raise NotImplementedError("integration_window > %d" % FW_MAX_IWIN)
        for term in r["terms"]:
            fc = term["function_class"]
            if fc not in FW_FUN:
                raise ValueError("Unexpected function class {}".format(fc))
            e.term_present[FW_FUN[fc]] = 1
            e.term_weight[FW_FUN[fc]] = float(term["weight"])
        if len(r["factors"]) > FW_MAX_REW:
            raise NotImplementedError("more than %d reward factors" % FW_MAX_REW)
        e.n_rew = len(r["factors"])
        for i, f in enumerate(r["factors"]):
            F = e.rew[i]
            cls, typ = f["class"], f.get("type")
            if cls == "action":
                if typ == "value":
                    F.kind = FW_REW_ACTION_VALUE
                elif typ == "delta":
                    F.kind = FW_REW_ACTION_DELTA
                    F.window = int(f["window_size"])
                    if F.window > FW_MAX_WINDOW:
                        raise NotImplementedError("reward window > %d" % FW_MAX_WINDOW)
                elif typ == "bound":
                    F.kind = FW_REW_ACTION_BOUND
                    if bm is None:
                        raise NotImplementedError("action bound reward without bounds_multiplier")
                else:
                    raise ValueError("Unexpected type {} for reward class action".format(typ))
            elif cls == "state":
                if typ == "error":
                    F.kind = FW_REW_STATE_ERROR
                    F.var = ANG_INDEX[f["name"]] if (self.ang_targets and f["name"] in ANG_INDEX) else \
                        TARGET_INDEX[f["name"]]
                elif typ == "value":
                    F.kind, F.var = FW_REW_STATE_VALUE, STATE_VAR_IDS[f["name"]]
                elif typ == "int_error":  # fixed_wing.py:1001-1012
                    F.kind, F.var = FW_REW_STATE_INT_ERROR, TARGET_INDEX[f["name"]]
                else:
                    raise NotImplementedError("state reward type %r" % typ)
            elif cls == "success":  # fixed_wing.py:1020-1026
                F.kind = FW_REW_SUCCESS
                if f["value"] == "timesteps":
                    F.var = 1
                else:
                    F.value = float(f["value"])
            elif cls == "step":  # :1028-1029
                F.kind, F.value = FW_REW_STEP, float(f["value"])
            elif cls == "goal":  # :1031-1048
                if typ not in ("per_state", "all"):
                    raise ValueError("Unexpected reward type {} for class goal".format(typ))
                F.kind, F.var, F.value = FW_REW_GOAL, int(typ == "all"), float(f["value"])
            else:
                raise ValueError("Unexpected reward component type {}".format(cls))
            fc = f["function_class"]
            if fc not in FW_FUN:
                raise ValueError("Unexpected function class {} for {}".format(fc, f["name"]))
            F.fun = FW_FUN[fc]
            if not e.term_present[F.fun]:
                raise KeyError(fc)
            F.shaping = int(bool(f.get("shaping", False)))
            sc = f["scaling"]
            if isinstance(sc, (list, tuple)):
                # reward.randomize_scaling (fixed_wing.py:473-479): U(low, high) per episode on the device
                if not r.get("randomize_scaling", False):
                    raise TypeError("reward factor %r: list scaling without randomize_scaling" % f["name"])
                F.randomize, F.scaling, F.scaling_hi = 1, float(sc[0]), float(sc[1])
            else:
                F.scaling = F.scaling_hi = float(sc)
            F.max = float(f["max"]) if f.get("max") is not None else INF
            F.sign = float(f.get("sign", -1))
        uses_iw = any(e.obs[o].kind == FW_OBS_TARGET_INT for o in range(e.n_obs)) or \
            any(e.rew[k].kind == FW_REW_STATE_INT_ERROR for k in range(e.n_rew))
        if uses_iw and e.integration_window <= 0:
            # the reference sums the whole history then ([-0:]); no config does that
            raise NotImplementedError("integrator / int_error with integration_window 0")
        return e

    def target_sampling(self):
        """(low, high, delta) per target in radians where configured (sample_target, fixed_wing.py:654-746)."""
        out = []
        for name in ["roll", "pitch", "Va"]:
            p = self.target_props[name]
            rad = p.get("convert_to_radians", False)
            cv = (lambda x: float(np.radians(x)) if rad else float(x))
            out.append((cv(p["low"]), cv(p["high"]), cv(p["delta"]) if p.get("delta") is not None else None))
        return out


def init_array(states, n, spec=None):
    """Pack explicit reset dicts (reference ``reset(state=...)`` keys) into [FW_NINIT][n] with NaN = sample."""
    arr = np.full((FW_NINIT, n), np.nan, dtype=np.float64)
    if states is None:
        return arr
    if isinstance(states, dict):
        states = [states] * n
    keys = {"roll": FW_I_ROLL, "pitch": FW_I_PITCH, "yaw": FW_I_YAW, "omega_p": FW_I_P, "omega_q": FW_I_Q,
            "omega_r": FW_I_R, "position_n": FW_I_PN, "position_e": FW_I_PE, "position_d": FW_I_PD,
            "velocity_u": FW_I_U, "velocity_v": FW_I_V, "velocity_w": FW_I_W,
            "wind_n": FW_I_WIND_N, "wind_e": FW_I_WIND_E, "wind_d": FW_I_WIND_D}
    dyn = spec.dynamics if spec is not None else ["elevon_right", "elevon_left", "throttle"]
    for i, st in enumerate(states):
        if st is None:
            continue
        for k, v in st.items():
            if k in keys:
                arr[keys[k], i] = v
            elif k == "wind":
                if v is None or isinstance(v, (int, float)):
                    if v is not None:
                        raise NotImplementedError("scalar wind magnitude in reset state")
                    continue
                arr[FW_I_WIND_N:FW_I_WIND_D + 1, i] = v
            elif k in dyn:
                j = dyn.index(k)
                if isinstance(v, (tuple, list, np.ndarray)):
                    arr[FW_I_ACT0 + 2 * j, i] = v[0]
                    arr[FW_I_ACT0 + 2 * j + 1, i] = v[1]
                else:
                    arr[FW_I_ACT0 + 2 * j, i] = v
                    arr[FW_I_ACT0 + 2 * j + 1, i] = 0.0
            elif k in ("Va", "alpha", "beta", "attitude", "elevator", "aileron", "rudder") or "energy" in k:
                continue  # ignored by PyFly.reset (pyfly.py:1273-1282)
            else:
                raise KeyError("unknown reset state key %r" % k)
    return arr
