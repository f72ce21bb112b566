"""CPU: the episode-metric oracle (oracle/metrics_oracle.py) against the metrics the reference
itself reported in info on done (tests/golden/env_metrics.npz)."""
import numpy as np
import pytest

import _fixtures as F
from oracle import metrics_oracle as M
from tum_adlr_deep_reinforcement_learning_amd import config as C

CASES = ["pid300", "pid_done", "rand150", "rand_fail", "pid_turb", "rand_short"]


def _spec(case):
    d = F.load("env_metrics.npz")
    g = lambda k: d[case + "__" + k]
    ckw = {"steps_max": int(g("steps_max"))}
    if case in ("pid300", "pid_turb"):
        ckw["action"] = {"scale_space": False}
    if case == "pid_done":
        ckw.update({"action": {"scale_space": False},
                    "target": {"on_success": "done", "success_streak_fraction": 0.9, "success_streak_req": 60}})
    return C.EnvSpec(config_kw=ckw, sim_config_kw={"turbulence": bool(g("turb_on")), "turbulence_intensity": "light"})


@pytest.mark.parametrize("case", CASES)
def test_metric_oracle_matches_reference(case):
    d = F.load("env_metrics.npz")
    g = lambda k: d[case + "__" + k]
    spec = _spec(case)
    t = spec.cfg["target"]
    errors = {k: list(g("hist_error_" + k)) for k in M.TARGETS}
    goals = {k: list(g("hist_goal_" + k).astype(bool)) for k in M.GOALS}
    res = M.metrics(errors, goals, g("hist_command"), 0.01, t["success_streak_req"], t["success_streak_fraction"],
                    len(g("rew")))
    for name, (col, keys) in C.METRIC_LAYOUT.items():
        got = np.array([float(res[name][k]) for k in keys])
        np.testing.assert_allclose(got, g("metric_" + name), rtol=1e-12, atol=1e-12, equal_nan=True,
                                   err_msg="%s %s" % (case, name))


def test_metric_fixture_covers_the_interesting_cases():
    d = F.load("env_metrics.npz")
    assert str(d["rand_fail__term"][-1]) not in ("steps", "success")      # constraint failure ends it
    assert str(d["pid_done__term"][-1]) == "success"
    assert np.isnan(d["rand_short__metric_control_variation"]).sum() == 0  # 3 commands -> defined
    assert np.isfinite(d["pid300__metric_rise_time"]).any()
