"""The quad integrator (four lanes per aircraft, csrc/fw_quad.hpp) against the one-lane path.

Its reference parity is tested where the one-lane path's is, with both integrators
(``test_gpu_parity.py``: reference single steps fp64 <= 1e-9 / fp32 gate, free-running reference
trajectories; ``test_gpu_r02.py``: rollout == steps bit for bit).  Here:

  lanes API ....................... auto = 4 up to FW_QUAD_AUTO_MAX (16384) aircraft, 1 above; explicit 1 / 4;
                                    other values raise
  env steps fp64, quad vs 1 lane .. identical done / termination / RHS-evaluation counts, obs and reward
                                    within 1e-9 (80 steps, 1000 aircraft, auto-resets, light Dryden)
  env steps fp32 .................. >= 99 % of the aircraft within 1e-4 per step over 10 steps (an ulp
                                    can flip an RK45 accept/reject, as in the generic-vs-specialised gate)
  stragglers ...................... a wave whose aircraft need thousands of RHS evaluations (stiff
                                    sideways states) integrates them to the same states in both paths
  tail handoff .................... one-lane kernels moving a wave's last <= 16 integrating aircraft to
                                    quads: fp64 within 1e-9 of the handoff-off kernel (FWSIM_TAIL_QUAD=0),
                                    same terminations; rollout == steps bit for bit above 16384 aircraft
"""
import os

import numpy as np
import pytest
import torch

from tum_adlr_deep_reinforcement_learning_amd import _native
from tum_adlr_deep_reinforcement_learning_amd import config as C

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _engine(spec, n, precision, lanes=None):
    from tum_adlr_deep_reinforcement_learning_amd.engine import Engine
    return Engine(spec.sim, spec, n, device=DEV, precision=precision, lanes=lanes)


AUTO = pytest.mark.skipif(bool(os.environ.get("FWSIM_LANES")), reason="FWSIM_LANES overrides the automatic choice")


@AUTO
def test_lanes_api():
    spec = C.EnvSpec()
    e = _engine(spec, 100, "float32")
    assert e.lanes == 4
    e.set_lanes(1)
    assert e.lanes == 1
    e.set_lanes(0)
    assert e.lanes == 4
    with pytest.raises(_native.FwError):
        e.set_lanes(3)
    e.close()
    big = _engine(spec, 20000, "float32")
    assert big.lanes == 1
    big.set_lanes(4)
    assert big.lanes == 4
    big.close()


def _run(spec, n, precision, lanes, steps, seed=9):
    eng = _engine(spec, n, precision, lanes)
    assert eng.lanes == lanes
    eng.seed(seed)
    eng.reset()
    g = torch.Generator(device=DEV)
    g.manual_seed(3)
    out = []
    for _ in range(steps):
        a = torch.rand(n, 3, generator=g, device=DEV, dtype=eng.dtype) * 2.4 - 1.2
        o, r, d, t = eng.env_step(a, stats=True)
        out.append((o.clone(), r.clone(), d.clone(), t.clone(), eng.stats.clone()))
    ode = eng.get_block(C.FW_BLK_ODE)
    eng.close()
    return out, ode


def test_quad_equals_one_lane_fp64():
    spec = C.EnvSpec(config_kw={"steps_max": 60}, sim_config_kw={"turbulence": True, "turbulence_intensity": "light"})
    n = 1000
    a, ya = _run(spec, n, "float64", 1, 80)
    b, yb = _run(spec, n, "float64", 4, 80)
    dones = 0
    for k, ((o1, r1, d1, t1, s1), (o2, r2, d2, t2, s2)) in enumerate(zip(a, b)):
        assert torch.equal(d1, d2) and torch.equal(t1, t2), k
        assert torch.equal(s1, s2), k  # same RHS evaluations and accepted steps
        assert torch.allclose(o1, o2, rtol=1e-9, atol=1e-9), (k, (o1 - o2).abs().max())
        assert torch.allclose(r1, r2, rtol=1e-9, atol=1e-9), k
        dones += int(d1.sum())
    assert dones >= n  # auto-resets happened
    assert torch.allclose(ya, yb, rtol=1e-9, atol=1e-9)


def test_quad_equals_one_lane_fp32():
    spec = C.EnvSpec(config_kw={"steps_max": 60}, sim_config_kw={"turbulence": False})
    n = 1024
    a, _ = _run(spec, n, "float32", 1, 10)
    b, _ = _run(spec, n, "float32", 4, 10)
    for (o1, r1, d1, t1, s1), (o2, r2, d2, t2, s2) in zip(a, b):
        close = ((o1 - o2).abs() <= 1e-4 * (1 + o2.abs())).all(1) & ((r1 - r2).abs() <= 1e-4 * (1 + r2.abs()))
        assert close.float().mean() >= 0.99, close.float().mean()
        assert (d1 == d2).float().mean() >= 0.99


@pytest.mark.parametrize("precision", ["float64", "float32"])
def test_quad_stragglers(precision):
    """Sideways flight at high rates: the RK45 straggler states.  Same accepted states
    (fp64: same terminations, nfev equal for >= 97 %, y within a tenth of the solver tolerance for >= 98 %
    of the aircraft where it is, median 1e-12; fp32: within the fp32 single-step gate) in both paths."""
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
    y[10] = rng.uniform(-0.3, 0.3, n)  # u ~ 0, v ~ +-(9..21) m/s: the sideways states the stragglers are
    y[11] = rng.choice([-1.0, 1.0], n) * rng.uniform(9, 21, n)  # captured in (profiles/r02_straggler_capture.log)
    y[12] = rng.uniform(-3.5, 0.1, n)
    y[13:16] = rng.uniform(-0.3, 0.3, (3, n))
    y[15] = rng.uniform(0.4, 0.6, n)
    y[16:18] = rng.choice([-1.0, 1.0], (2, n)) * 3.491
    cmd = torch.tensor(rng.uniform(-0.5, 0.5, (n, 3)), device=DEV)
    cmd[:, 2] = cmd[:, 2].abs() * 2
    res = {}
    for lanes in (1, 4):
        from tum_adlr_deep_reinforcement_learning_amd.engine import Engine
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
    (y1, t1, n1, f1), (y4, t4, n4, f4) = res[1], res[4]
    assert n1.max() >= 150, np.sort(n1)[-8:]  # the states are stragglers
    ok = (t1 == 0) & (t4 == 0)
    if precision == "float64":
        assert np.array_equal(t1, t4) and np.array_equal(f1, f4)
        assert (n1 != n4).mean() <= 0.03  # stiff states: a rounding-level difference can flip an accept/reject
        same = ok & (n1 == n4)
        rel = (np.abs(y1 - y4) / (np.abs(y1) + 1e-3))[:, same].max(0)
        assert np.median(rel) <= 1e-12
        # stiff states amplify rounding-level step-size differences: a tenth of the solver's own
        # tolerance (atol 1e-6, rtol 1e-3) on >= 98 % of the aircraft.  The exceptions are chaotic
        # stragglers where the two paths take different step grids of the same length, and the fp64 C
        # oracle differs from both by as much (round 3: one of 254, u and w near 0 after 1406
        # evaluations, one lane / quad / oracle = -4.4e-5 / -6.6e-5 / -4.2e-5 m/s, oracle nfev 1496)
        within = (np.abs(y1 - y4)[:, same] <= 0.1 * (1e-6 + 1e-3 * np.abs(y1[:, same]))).all(0)
        assert within.mean() >= 0.98, within.mean()
    else:
        assert (t1 == t4).mean() >= 0.97
        rel = (np.abs(y1 - y4) / (np.abs(y1) + 1e-3))[:13, ok].max(0)
        assert np.median(rel) <= 1e-5 and (rel <= 1e-3).mean() >= 0.9


@AUTO
def test_one_lane_with_handoff_rollout_equals_steps():
    """20037 aircraft, fp32 (above FW_QUAD_AUTO_MAX: one lane per aircraft with the tail handoff, ragged
    last wave): fw_env_rollout equals fw_env_step launches bit for bit."""
    spec = C.EnvSpec(config_kw={"steps_max": 50}, sim_config_kw={"turbulence": True, "turbulence_intensity": "light"})
    n, K = 20000 + 37, 60
    a, b = _engine(spec, n, "float32"), _engine(spec, n, "float32")
    assert a.lanes == 1
    for e in (a, b):
        e.seed(5)
        e.reset()
    g = torch.Generator(device=DEV)
    g.manual_seed(8)
    acts = (torch.rand(K, n, 3, generator=g, device=DEV) * 2.4 - 1.2).contiguous()
    obs, rew, done, term = a.env_rollout(acts, stats=True)
    assert int(done.sum()) >= n
    for k in range(K):
        o, r, d, t = b.env_step(acts[k], stats=True)
        assert torch.equal(obs[k], o) and torch.equal(rew[k], r) and torch.equal(done[k], d), k
        assert torch.equal(term[k], t) and torch.equal(a.rollout_stats[k], b.stats), k
    assert torch.equal(a.get_block(C.FW_BLK_ODE), b.get_block(C.FW_BLK_ODE))
    a.close()
    b.close()


@pytest.mark.parametrize("precision", ["float64", "float32"])
def test_tail_handoff_matches_one_lane(precision, monkeypatch):
    """One-lane kernels hand a wave's last <= 16 integrating aircraft to lane quads (rk45 HO): against
    the same kernels with the handoff off (FWSIM_TAIL_QUAD=0), fp64 agrees within 1e-9 with the same
    terminations and RHS-evaluation counts (up to rounding-level accept/reject flips); fp32 as the
    generic-vs-specialised gate."""
    spec = C.EnvSpec(config_kw={"steps_max": 60}, sim_config_kw={"turbulence": True, "turbulence_intensity": "light"})
    n = 4096 + 37  # ragged last wave
    steps = 60 if precision == "float64" else 10
    outs = []
    for tq in ("0", "16"):
        monkeypatch.setenv("FWSIM_TAIL_QUAD", tq)
        outs.append(_run(spec, n, precision, 1, steps)[0])
    flips = 0
    for (o1, r1, d1, t1, s1), (o2, r2, d2, t2, s2) in zip(*outs):
        if precision == "float64":
            assert torch.equal(d1, d2) and torch.equal(t1, t2)
            flips += int((s1 != s2).sum())
            same = (s1 == s2)
            assert torch.allclose(o1[same], o2[same], rtol=1e-9, atol=1e-9)
        else:
            close = ((o1 - o2).abs() <= 1e-4 * (1 + o2.abs())).all(1) & ((r1 - r2).abs() <= 1e-4 * (1 + r2.abs()))
            assert close.float().mean() >= 0.99
    if precision == "float64":
        assert flips <= 0.002 * n * steps, flips


def test_quad_refused_with_wrapped_ode_variable():
    """The quad integrator's row conditions have no wrap: a configuration wrapping an ODE-state variable
    runs one lane per aircraft (automatic), and asking for quads fails loudly."""
    spec = C.EnvSpec(sim_config_kw={"turbulence": False})
    spec.sim.vars["omega_p"].wrap = True
    e = _engine(spec, 64, "float64")
    assert e.lanes == 1
    with pytest.raises(_native.FwError):
        e.set_lanes(4)
    e.set_lanes(1)
    assert e.lanes == 1
    e.close()
