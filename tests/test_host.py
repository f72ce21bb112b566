"""CPU tests of the host side: the C ABI library loads and exports every symbol
include/fwsim.h declares (no compute calls), argument validation fails loudly
without touching a device, config translation matches the reference's
numbers, and the VecEnv info plumbing behaves like SB3's."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

from oracle import oracle as O
from tum_adlr_deep_reinforcement_learning_amd import _native
from tum_adlr_deep_reinforcement_learning_amd import config as C
from tum_adlr_deep_reinforcement_learning_amd.spaces import Box
from tum_adlr_deep_reinforcement_learning_amd.vec_env import _Infos, termination_name

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(ROOT, "include", h) for h in ("fwsim.h", "fwrollout.h")]


def _declared():
    names = set()
    for h in HEADERS:
        names |= set(re.findall(r"^(?:int|int64_t|size_t)\s+(fw_\w+)\s*\(", open(h).read(), re.M))
    return sorted(names)


def test_library_exports_every_declared_symbol():
    lib = _native.load()
    names = _declared()
    assert len(names) >= 14
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) == set(_native.SIGNATURES), "python signatures out of sync with include/fwsim.h"
    assert lib.fw_abi_version() == _native.ABI_VERSION


def test_create_validates_without_device():
    lib = _native.load()
    h = ctypes.c_void_p()
    spec = C.EnvSpec()
    sim, env = spec.sim.struct(), spec.struct()
    assert lib.fw_create(ctypes.byref(sim), ctypes.byref(env), 0, 0, 0, ctypes.byref(h)) != 0
    assert "n_envs" in _native.last_error()
    assert lib.fw_create(ctypes.byref(sim), ctypes.byref(env), 8, 7, 0, ctypes.byref(h)) != 0
    assert "precision" in _native.last_error()
    bad = spec.sim.struct()
    bad.dt = 0.0
    assert lib.fw_create(ctypes.byref(bad), None, 8, 0, 0, ctypes.byref(h)) != 0
    assert "dt" in _native.last_error()
    assert lib.fw_create(ctypes.byref(sim), None, 8, 0, 0, None) != 0
    assert h.value is None


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-device path")
def test_engine_refuses_to_run_without_gpu():
    from tum_adlr_deep_reinforcement_learning_amd.engine import Engine
    spec = C.EnvSpec()
    with pytest.raises(_native.FwError, match="no CPU fallback"):
        Engine(spec.sim, spec, 4)


def test_struct_layout_matches_c():
    L = O.lib()
    assert ctypes.sizeof(C.FwSimConfig) == L.orc_sizeof_sim_config()
    assert ctypes.sizeof(C.FwEnvConfig) == L.orc_sizeof_env_config()


def test_default_env_spaces_match_reference():
    """fixed_wing_config.json defaults: 14 observations, actions scaled to the actuator limits."""
    spec = C.EnvSpec()
    assert spec.n_obs == 14 and spec.steps_max == 2000
    np.testing.assert_allclose(spec.action_scale_to_low, [-0.5236, -0.5672, 0.0], atol=1e-4)
    np.testing.assert_allclose(spec.action_scale_to_high, [0.6109, 0.5672, 1.0], atol=1e-4)
    assert spec.scale_actions
    e = spec.struct()
    assert e.n_obs == 14 and e.streak_req == 100 and abs(e.streak_frac - 0.95) < 1e-12
    assert spec.obs_names()[:3] == ["roll", "pitch", "Va"]


def test_curriculum_level_scales_ranges():
    spec = C.EnvSpec()
    lo1, hi1, _ = spec.target_sampling()[0]
    spec.set_curriculum_level(0.5)
    lo5, hi5, _ = spec.target_sampling()[0]
    assert lo5 == pytest.approx(lo1 / 2) and hi5 == pytest.approx(hi1 / 2)
    spec.set_curriculum_level(0.0)
    lo0, hi0, _ = spec.target_sampling()[0]
    assert lo0 == pytest.approx(hi0)


def test_termination_names_match_oracle():
    for code in [1 + v for v in range(C.FW_NVAR) if C.VAR_NAMES[v] is not None or C.FW_V_ACT0 <= v <= C.FW_V_ACT2]:
        assert termination_name(code) == O.term_name(code)
    assert termination_name(C.FW_TERM_STEPS) == "steps"
    assert termination_name(C.FW_TERM_SUCCESS) == "success"


def test_init_array_packs_reference_reset_dicts():
    spec = C.build_sim()
    st = {"roll": 0.1, "velocity_u": 20.0, "wind": [1.0, 2.0, 3.0], "elevon_left": (0.05, 0.2), "Va": 99.0}
    a = C.init_array([st, None], 2, spec)
    assert a.shape == (C.FW_NINIT, 2)
    assert a[C.FW_I_ROLL, 0] == 0.1 and a[C.FW_I_U, 0] == 20.0
    assert list(a[C.FW_I_WIND_N:, 0]) == [1.0, 2.0, 3.0]
    assert a[C.FW_I_ACT1, 0] == 0.05 and a[C.FW_I_ACT1_DOT, 0] == 0.2
    assert np.isnan(a[:, 1]).all() and np.isnan(a[C.FW_I_PITCH, 0])
    with pytest.raises(KeyError):
        C.init_array({"bogus": 1.0}, 1, spec)


def test_infos_are_lazy_and_sb3_shaped():
    n = 5
    done = np.array([0, 1, 0, 0, 1], bool)
    term = np.array([0, C.FW_TERM_STEPS, 0, 0, 1 + C.FW_V_OMEGA_R], np.int32)
    tobs = np.arange(n * 14, dtype=np.float32).reshape(n, 14)
    ep = np.zeros((n, 5))
    ep[1] = [-12.5, 2000, 0.1, 0.2, 21.0]
    ep[4] = [-3.0, 17, 0.0, 0.0, 18.0]
    tgt = np.tile(np.array([[0.3], [0.1], [22.0]]), (1, n))
    infos = _Infos(n, done, term, tobs, ep, tgt, 1.5, ("elevon_right", "elevon_left", "throttle"), True)
    assert len(infos) == n and not infos._cache
    i1 = infos[1]
    assert i1["termination"] == "steps" and i1["episode"] == {"r": -12.5, "l": 2000, "t": 1.5}
    assert np.array_equal(i1["terminal_observation"], tobs[1])
    assert i1["target"] == {"roll": 0.1, "pitch": 0.2, "Va": 21.0}
    assert infos[4]["termination"] == "omega_r"
    assert "terminal_observation" not in infos[0] and infos[0]["target"]["Va"] == 22.0
    assert infos[-1] is infos[4]
    assert len(infos[1:3]) == 2


def test_box_space():
    b = Box(np.array([-1, -2], np.float32), np.array([1, 2], np.float32))
    b.seed(0)
    x = b.sample()
    assert b.contains(x) and x.dtype == np.float32 and b.shape == (2,)
