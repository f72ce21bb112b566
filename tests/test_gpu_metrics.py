"""GPU: streaming episode metrics of the fused env step (fw_set_metrics_output) against the
metrics the reference itself reported in info on done (tests/golden/env_metrics.npz), fp64.

Tolerance: values rel 1e-5, as for the env sequences (the reference feeds float32 random actions
through float64 arithmetic, which leaves ~1e-7 relative trajectory differences); indices
(settling / rise time) and success exact."""
import numpy as np
import pytest
import torch

import _fixtures as F
from test_metrics_oracle import CASES, _spec
from tum_adlr_deep_reinforcement_learning_amd import config as C

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case", CASES)
def test_device_metrics_match_reference(case):
    from tum_adlr_deep_reinforcement_learning_amd.engine import Engine
    d = F.load("env_metrics.npz")
    g = lambda k: d[case + "__" + k]
    spec = _spec(case)
    eng = Engine(spec.sim, spec, 1, device="cuda:0", precision="float64")
    assert eng.metrics is not None
    if bool(g("turb_on")):
        eng.set_noise(g("noise")[None])
    eng.reset(init=F.env_init(g("init"))[:, None], target=g("target0")[:, None])
    acts = torch.tensor(g("act"), dtype=torch.float64, device="cuda:0")
    for s in range(len(acts)):
        _, _, done, _ = eng.env_step(acts[s:s + 1], auto_reset=False)
        if bool(done[0]):
            break
    assert s == len(acts) - 1, "episode length differs from the reference"
    row = eng.metrics[:, 0].cpu().numpy()
    for name, (col, keys) in C.METRIC_LAYOUT.items():
        got, want = row[col:col + len(keys)], g("metric_" + name)
        if name in ("success", "settling_time", "rise_time"):
            np.testing.assert_array_equal(got, want, err_msg="%s %s" % (case, name))
        else:
            np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-8, equal_nan=True, err_msg="%s %s" % (case, name))
    eng.close()


def test_vecenv_reports_metrics_in_info():
    from tum_adlr_deep_reinforcement_learning_amd.vec_env import FixedWingVecEnv
    env = FixedWingVecEnv(32, config_kw={"steps_max": 30}, sim_config_kw={"turbulence": False}, device="cuda:0",
                          seed=2)
    env.reset()
    rng = np.random.RandomState(0)
    for _ in range(30):
        _, _, done, infos = env.step(rng.uniform(-1, 1, (32, 3)).astype(np.float32))
    assert done.all()
    info = infos[0]
    for m in env.spec.cfg["metrics"]:
        assert m["name"] in info
    assert set(info["success"]) == {"roll", "pitch", "Va", "all"}
    assert isinstance(info["success"]["all"], bool)
    assert np.isfinite(info["control_variation"]["all"]) and info["total_error"]["Va"] >= 0
    env.close()
