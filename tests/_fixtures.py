"""Shared helpers: load golden fixtures and build the matching configs."""
import os

import numpy as np

from tum_adlr_deep_reinforcement_learning_amd import config as C

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def pyfly_cfg(turb_on, L=300, omega_limit_deg=180.0, va_limit=np.inf):
    spec = C.build_sim(config_kw={"turbulence": bool(turb_on), "turbulence_sim_length": int(L)})
    cfg = spec.struct()
    for i in (C.FW_V_OMEGA_P, C.FW_V_OMEGA_Q, C.FW_V_OMEGA_R):
        cfg.lim[i].constraint_min = -np.radians(omega_limit_deg)
        cfg.lim[i].constraint_max = np.radians(omega_limit_deg)
    cfg.lim[C.FW_V_VA].constraint_max = float(va_limit)
    return spec, cfg


ENV_CASES = {
    # name -> (config_kw, sim turbulence)
    "rand_off": (None, False), "rand_on": (None, False), "rand_turb": (None, True),
    "short_max": ({"steps_max": 120}, False), "fail_omega": (None, False),
    "fail_va": ({"simulator": {"states": {5: {"constraint_max": 17.5}}}}, False),
    "pid_goal": ({"action": {"scale_space": False}}, False),
    "pid_goal_done": ({"steps_max": 1500, "action": {"scale_space": False},
                       "target": {"on_success": "done", "success_streak_fraction": 1, "success_streak_req": 100}},
                      False),
    "pid_turb": ({"action": {"scale_space": False}}, True),
}


def env_spec(name):
    ckw, turb = ENV_CASES[name]
    return C.EnvSpec(config_kw=ckw, sim_config_kw={"turbulence": turb, "turbulence_intensity": "light"})


def env_init(init_row, n_act_dyn=3):
    """fixture init row (12 states + 3 actuator values + wind) -> FW_NINIT vector."""
    v = np.full(C.FW_NINIT, np.nan)
    v[:12] = init_row[:12]
    for j in range(3):
        v[C.FW_I_ACT0 + 2 * j] = init_row[12 + j]
        v[C.FW_I_ACT0 + 2 * j + 1] = 0.0
    v[C.FW_I_WIND_N:C.FW_I_WIND_D + 1] = init_row[15:18]
    return v


OBS_HIST_CASES = {
    # name -> config_kw (the config file itself is stored in the fixture: "" = default config)
    "cnn_rand": None,
    "cnn_fail_p": {"simulator": {"states": {6: {"constraint_min": -150, "constraint_max": 150}}}},
    "cnn_short": {"steps_max": 40},
    "vec3_rand": {"observation": {"length": 3, "step": 2, "shape": "vector"}},
    "vec3_norm": {"observation": {"length": 3, "step": 2, "shape": "vector", "normalize": True}},
}


def obs_hist_spec(name, tmpdir):
    """EnvSpec of an env_obs_hist.npz case (writes the stored reference config file to tmpdir)."""
    import json
    d = load("env_obs_hist.npz")
    text = str(d[name + "__config_json"])
    path = None
    if text:
        path = os.path.join(str(tmpdir), name + ".json")
        with open(path, "w") as f:
            f.write(text)
    ckw = dict(OBS_HIST_CASES[name] or {})
    ckw["steps_max"] = int(d[name + "__steps_max"])
    return C.EnvSpec(config_path=path, config_kw=ckw, sim_config_kw={"turbulence": False}), d
