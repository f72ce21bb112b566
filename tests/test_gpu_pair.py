"""The pair integrator (two lanes per aircraft, csrc/fw_pair.hpp, round 6) against the one-lane path.

Its reference parity runs with the other integrators' (``test_gpu_parity.py``: reference single steps fp64
<= 1e-9 with equal RHS-evaluation counts, the fp32 single-step gate, free-running reference trajectories, the
65536-aircraft properties; all parametrised over lanes 1 / 2 / 4).  Here, as test_gpu_quad.py does for the quad:

  env steps fp64, pair vs 1 lane .. identical done / termination / RHS-evaluation counts, obs and reward
                                    within 1e-9 (80 steps, 1000 aircraft, auto-resets, light Dryden)
  env steps fp32 .................. >= 99 % of the aircraft within 1e-4 per step over 10 steps
  stragglers ...................... stiff sideways states integrate to the same states
  lanes API ....................... fw_set_lanes(2) / FWSIM_LANES=2; refused with a wrapped ODE variable;
                                    fw_env_rollout runs the pair too (== K pair env steps bit for bit)
"""
import numpy as np
import pytest
import torch

from tum_adlr_deep_reinforcement_learning_amd import _native
from tum_adlr_deep_reinforcement_learning_amd import config as C
from test_gpu_quad import _run, _engine

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def test_pair_equals_one_lane_fp64():
    spec = C.EnvSpec(config_kw={"steps_max": 60}, sim_config_kw={"turbulence": True, "turbulence_intensity": "light"})
    n = 1000
    a, ya = _run(spec, n, "float64", 1, 80)
    b, yb = _run(spec, n, "float64", 2, 80)
    dones, flips = 0, 0
    for k, ((o1, r1, d1, t1, s1), (o2, r2, d2, t2, s2)) in enumerate(zip(a, b)):
        assert torch.equal(d1, d2) and torch.equal(t1, t2), k
        flips += int((s1 != s2).sum())
        assert torch.allclose(o1, o2, rtol=1e-9, atol=1e-9), (k, (o1 - o2).abs().max())
        assert torch.allclose(r1, r2, rtol=1e-9, atol=1e-9), k
        dones += int(d1.sum())
    assert flips <= 2, flips  # same RHS evaluations and accepted steps (a rounding-level flip at most)
    assert dones >= n
    assert torch.allclose(ya, yb, rtol=1e-9, atol=1e-9)


def test_pair_equals_one_lane_fp32():
    spec = C.EnvSpec(config_kw={"steps_max": 60}, sim_config_kw={"turbulence": False})
    n = 1024
    a, _ = _run(spec, n, "float32", 1, 10)
    b, _ = _run(spec, n, "float32", 2, 10)
    for (o1, r1, d1, t1, s1), (o2, r2, d2, t2, s2) in zip(a, b):
        close = ((o1 - o2).abs() <= 1e-4 * (1 + o2.abs())).all(1) & ((r1 - r2).abs() <= 1e-4 * (1 + r2.abs()))
        assert close.float().mean() >= 0.99, close.float().mean()
        assert (d1 == d2).float().mean() >= 0.99


@pytest.mark.parametrize("precision", ["float64", "float32"])
def test_pair_stragglers(precision):
    """The quad's straggler states (test_gpu_quad.test_quad_stragglers) through the pair."""
    from tum_adlr_deep_reinforcement_learning_amd.engine import Engine
    spec = C.EnvSpec(sim_config_kw={"turbulence": False})
    n = 256
    rng = np.random.default_rng(4)
    y = np.zeros((C.FW_NY, n))
    ang = rng.uniform(-np.pi, np.pi, (3, n))
    cr, sr = np.cos(ang / 2), np.sin(ang / 2)
    y[0] = cr[0] * cr[1] * cr[2] + sr[0] * sr[1] * sr[2]
    y[1] = sr[0] * cr[1] * cr[2] - cr[0] * sr[1] * sr[2]
    y[2] = cr[0] * sr[1] * cr[2] + sr[0] * cr[1] * sr[2]
    y[3] = cr[0] * cr[1] * sr[2] - sr[0] * sr[1] * cr[2]
    y[4:7] = rng.uniform(-2, 2, (3, n))
    y[7:10] = rng.uniform(-50, 50, (3, n))
    y[10] = rng.uniform(-0.3, 0.3, n)
    y[11] = rng.choice([-1.0, 1.0], n) * rng.uniform(9, 21, n)
    y[12] = rng.uniform(-3.5, 0.1, n)
    y[13:16] = rng.uniform(-0.3, 0.3, (3, n))
    y[15] = rng.uniform(0.4, 0.6, n)
    y[16:18] = rng.choice([-1.0, 1.0], (2, n)) * 3.491
    cmd = torch.tensor(rng.uniform(-0.5, 0.5, (n, 3)), device=DEV)
    cmd[:, 2] = cmd[:, 2].abs() * 2
    res = {}
    for lanes in (1, 2):
        e = Engine(spec.sim, None, n, device=DEV, precision=precision, lanes=lanes)
        e.set_block(C.FW_BLK_ODE, y)
        e.set_block(C.FW_BLK_DERIVED, np.zeros((8, n)))
        e.set_block(C.FW_BLK_WIND, np.zeros((3, n)))
        e.set_block(C.FW_BLK_STEPS, np.zeros(n, np.int32))
        succ, term = e.sim_step(cmd.to(e.dtype), stats=True)
        nfev, nacc, failed = e.decode_stats(e.stats)
        res[lanes] = (e.get_block(C.FW_BLK_ODE).double().cpu().numpy(), term.cpu().numpy().copy(),
                      nfev.cpu().numpy().copy(), failed.cpu().numpy().copy())
        e.close()
    (y1, t1, n1, f1), (y2, t2, n2, f2) = res[1], res[2]
    assert n1.max() >= 150
    ok = (t1 == 0) & (t2 == 0)
    if precision == "float64":
        assert np.array_equal(t1, t2) and np.array_equal(f1, f2)
        assert (n1 != n2).mean() <= 0.03
        same = ok & (n1 == n2)
        rel = (np.abs(y1 - y2) / (np.abs(y1) + 1e-3))[:, same].max(0)
        assert np.median(rel) <= 1e-12
        within = (np.abs(y1 - y2)[:, same] <= 0.1 * (1e-6 + 1e-3 * np.abs(y1[:, same]))).all(0)
        assert within.mean() >= 0.98, within.mean()
    else:
        assert (t1 == t2).mean() >= 0.97
        rel = (np.abs(y1 - y2) / (np.abs(y1) + 1e-3))[:13, ok].max(0)
        assert np.median(rel) <= 1e-5 and (rel <= 1e-3).mean() >= 0.9


def test_pair_lanes_api():
    spec = C.EnvSpec()
    e = _engine(spec, 300, "float32", 2)
    assert e.lanes == 2
    e.close()
    spec.sim.vars["omega_p"].wrap = True
    w = _engine(spec, 64, "float64")
    with pytest.raises(_native.FwError):
        w.set_lanes(2)
    w.close()


@pytest.mark.parametrize("precision", ["float64", "float32"])
def test_pair_rollout_equals_pair_steps(precision):
    """fw_env_rollout under lanes 2 runs the pair integrator too (round 6: it had no pair instance and ran one
    lane, which rounds differently): equal to K pair fw_env_step launches bit for bit, with auto-resets."""
    spec = C.EnvSpec(config_kw={"steps_max": 30}, sim_config_kw={"turbulence": False})
    n, K = 300, 40
    a, b = _engine(spec, n, precision, 2), _engine(spec, n, precision, 2)
    for e in (a, b):
        e.seed(5)
        e.reset()
    g = torch.Generator(device=DEV)
    g.manual_seed(8)
    acts = (torch.rand(K, n, 3, generator=g, device=DEV, dtype=a.dtype) * 2.4 - 1.2).contiguous()
    obs, rew, done, term = a.env_rollout(acts)
    for k in range(K):
        o, r, d, t = b.env_step(acts[k])
        assert torch.equal(obs[k], o) and torch.equal(rew[k], r) and torch.equal(done[k], d), k
    a.close()
    b.close()
