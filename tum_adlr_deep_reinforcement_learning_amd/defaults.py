"""Built-in default configurations (Skywalker X8 + attitude-tracking task).

The values are those of the reference's shipped defaults -- the aircraft
parameters in ``magpie/libs/pyfly/pyfly/x8_param.mat``, the simulator config
``magpie/libs/pyfly/pyfly/pyfly_config.json`` and the task config
``magpie/libs/fixed-wing-gym/gym_fixed_wing/fixed_wing_config.json`` -- expressed
here as Python data so the package runs without the reference checkout.  The
dictionaries use the reference's JSON schema, so a user's own reference-format
JSON files can be loaded instead (``config.load_*``).
"""
import copy

# x8_param.mat (52 scalars; r_cg = [0, 0, 0] unused by the dynamics)
X8_PARAMS = {
    "C_D_0": 0.01970001181915082, "C_D_alpha1": 0.07909146315766297, "C_D_alpha2": 1.0554699867680841,
    "C_D_beta1": -0.005842980345415388, "C_D_beta2": 0.14781193079241584,
    "C_D_delta_e": 0.06334739678180232, "C_D_p": 0.0102, "C_D_q": 0.0,
    "C_L_0": 0.08673556671610734, "C_L_alpha": 4.020328244000679, "C_L_delta_e": 0.2780736201734713,
    "C_L_q": 3.87,
    "C_Y_0": 0.0, "C_Y_beta": -0.22387215700254048, "C_Y_delta_a": 0.043276402502774876, "C_Y_delta_r": 0.0,
    "C_Y_p": -0.13735505263157893, "C_Y_r": 0.08386876842105263,
    "C_l_0": 0.0, "C_l_beta": -0.08489628639662417, "C_l_delta_a": 0.12018814125782745, "C_l_delta_r": 0.0,
    "C_l_p": -0.40419799999999995, "C_l_r": 0.055520599999999996,
    "C_m_0": 0.018, "C_m_alpha": -0.2524, "C_m_delta_e": -0.2292, "C_m_fp": -0.2168,
    "C_m_q": -1.3012370370370372,
    "C_n_0": 0.0, "C_n_beta": 0.0283, "C_n_delta_a": -0.00339, "C_n_delta_r": 0.0,
    "C_n_p": 0.004365511578947368, "C_n_r": -0.07200000000000001,
    "C_prop": 0.248, "Jx": 1.229, "Jxz": 0.9343, "Jy": 0.1702, "Jz": 0.8808, "M": 50.0,
    "S_prop": 0.10178760197630929, "S_wing": 0.75, "a_0": 0.267, "b": 2.1, "c": 0.35714285714285715,
    "e": 0.9935, "k_Omega": 797.1268, "k_T_P": 1.1871e-06, "k_motor": 37.42, "mass": 3.364,
}


def _var(name, **kw):
    d = {"name": name}
    d.update(kw)
    return d


def default_pyfly_config():
    """The reference's pyfly_config.json content (plots omitted: rendering is out of scope)."""
    act2 = dict(convert_to_radians=True, order=2, dot_max=3.4907, omega_0=100, zeta=1.71)
    variables = [
        _var("roll", convert_to_radians=True, init_min=-30, init_max=30, wrap=True),
        _var("pitch", convert_to_radians=True, init_min=-30, init_max=30),
        _var("yaw", convert_to_radians=True, init_min=-30, init_max=30, wrap=True),
    ]
    for ax in "pqr":
        variables.append(_var("omega_" + ax, init_min=-40, init_max=40, constraint_min=-180, constraint_max=180,
                              convert_to_radians=True))
    variables += [
        _var("position_n", init_min=-100, init_max=100),
        _var("position_e", init_min=-100, init_max=100),
        _var("position_d", init_min=-20, init_max=-100),
        _var("velocity_u", init_min=13, init_max=22),
        _var("velocity_v", init_min=-5, init_max=5),
        _var("velocity_w", init_min=-5, init_max=5),
        _var("alpha"),
        _var("beta", convert_to_radians=True),
        _var("Va", value_min=1e-6),
        _var("wind_n", init_min=8, init_max=8),
        _var("wind_e", init_min=8, init_max=8),
        _var("wind_d", init_min=8, init_max=8),
        _var("elevon_left", value_min=-30, value_max=35, init_min=0, init_max=0, **act2),
        _var("elevon_right", value_min=-30, value_max=35, init_min=0, init_max=0, **act2),
        _var("elevator", value_min=-30, value_max=35, init_min=0, init_max=0, disabled=True, **act2),
        _var("aileron", value_min=-30, value_max=35, init_min=0, init_max=0, disabled=True, **act2),
        _var("rudder", disabled=True, **act2),
        _var("throttle", value_min=0, value_max=1, init_min=0, init_max=0, order=1, tau=0.2),
        _var("energy_total"), _var("energy_potential"), _var("energy_kinetic_rotational"),
        _var("energy_kinetic_translational"),
    ]
    return {
        "dt": 0.01, "rho": 1.2250, "g": 9.81,
        "wind_magnitude_min": -8, "wind_magnitude_max": 8,
        "turbulence": True, "turbulence_intensity": "light", "turbulence_sim_length": 300,
        "variables": variables,
        "actuation": {"dynamics": ["elevon_right", "elevon_left", "throttle"],
                      "inputs": ["elevator", "aileron", "throttle"]},
        "plots": [],
    }


def default_env_config():
    """The reference's fixed_wing_config.json content (attitude-tracking task)."""
    obs_states = [
        dict(name="roll", low=-180, high=180, convert_to_radians=True, type="state", mean=0, var=0.3),
        dict(name="pitch", low=-85, high=85, convert_to_radians=True, type="state", mean=0, var=0.15),
        dict(name="Va", low=0, high=70, type="state", mean=21, var=2),
    ]
    for ax in "pqr":
        obs_states.append(dict(name="omega_" + ax, low=-720, high=720, convert_to_radians=True, type="state",
                               mean=0, var=0.94))
    obs_states += [
        dict(name="roll", type="target", value="absolute", mean=0, var=0.16),
        dict(name="pitch", type="target", value="absolute", mean=0, var=0.05),
        dict(name="Va", type="target", value="absolute", mean=0, var=2),
        dict(name="alpha", type="state", mean=0, var=0.1),
        dict(name="beta", type="state", mean=0, var=0.1),
    ]
    for a in ["elevator", "aileron", "throttle"]:
        obs_states.append(dict(name=a, type="action", window_size=5, norm=False))
    err = dict(**{"class": "state"}, type="error", function_class="linear", shaping=True, max=0.3, sign=-1)
    sim_states = [
        dict(name="roll", init_min=-110, init_max=110, convert_to_radians=True),
        dict(name="pitch", init_min=-45, init_max=45, convert_to_radians=True),
        dict(name="velocity_u", init_min=10, init_max=23),
        dict(name="velocity_v", init_min=-5, init_max=5),
        dict(name="velocity_w", init_min=-5, init_max=5),
        dict(name="Va", constraint_max=70),
    ]
    for ax in "pqr":
        sim_states.append(dict(name="omega_" + ax, init_min=-60, init_max=60, constraint_min=-720,
                               constraint_max=720, convert_to_radians=True))
    return {
        "steps_max": 2000,
        "integration_window": 0,
        "observation": {"length": 1, "step": 1, "shape": "vector", "normalize": False,
                        "noise": {"mean": 0, "var": 0}, "states": obs_states},
        "action": {"scale_space": True, "scale_low": -1, "scale_high": 1, "bounds_multiplier": 1.5,
                   "states": [dict(name=a, low="max", high="max") for a in ["elevator", "aileron", "throttle"]]},
        "target": {
            "resample_every": 0, "success_streak_req": 100, "success_streak_fraction": 0.95, "on_success": "none",
            "states": [
                dict(name="roll", convert_to_radians=True, low=-60, high=60, delta=180, bound=5,
                     **{"class": "constant"}),
                dict(name="pitch", convert_to_radians=True, low=-25, high=25, delta=45, bound=5,
                     **{"class": "constant"}),
                dict(name="Va", low=15, high=28, delta=6, bound=2, **{"class": "compensate"}),
            ],
        },
        "reward": {
            "form": "absolute", "randomize_scaling": False, "step_fail": "timesteps",
            "terms": [{"function_class": "linear", "weight": 1}],
            "factors": [
                dict(name="roll", scaling=3.2, **copy.deepcopy(err)),
                dict(name="pitch", scaling=3.2, **copy.deepcopy(err)),
                dict(name="Va", scaling=25, **copy.deepcopy(err)),
                dict(name="action", type="delta", function_class="linear", window_size=5, scaling=60, shaping=False,
                     sign=-1, **{"class": "action"}),
                dict(name="action_bound", type="bound", function_class="linear", scaling=1, shaping=False, sign=-1,
                     **{"class": "action"}),
            ],
        },
        "simulator": {"states": sim_states},
        "render": {"plot_action": True, "plot_reward": True, "plot_target": True, "plot_goal": True},
        "metrics": [dict(name="rise_time", high=0.9, low=0.1), dict(name="settling_time"), dict(name="overshoot"),
                    dict(name="total_error"), dict(name="avg_error"), dict(name="control_variation"),
                    dict(name="success"), dict(name="success_time_frac"), dict(name="end_error")],
    }
