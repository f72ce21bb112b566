"""GPU parity: the HIP path (through the C ABI) against the oracle and the
reference-generated golden fixtures.  Run on an MI355X with ``pytest -m gpu``.

Tolerances (relative metric |d| / (|ref| + 1e-3)):
  fp64 kernel, teacher-forced single step ........ <= 1e-9, identical nfev / termination
  fp64 kernel, free-running 1000 steps ........... <= 1e-7 (+ step-count parity)
  fp32 kernel, teacher-forced single step ........ median <= 1e-6, >= 97 % of cases <= 1e-4
                                                    (the rest are RK45 accept/reject flips)
  fp32 kernel, free-running 1000 steps ........... within 5x the reference's own deviation under
                                                    per-step float32 state storage (+ rtol kick after
                                                    the first accept/reject flip), same termination +-1
  PID evaluation set (40 scenarios) .............. fp64: lengths exact (all but <= 1), rewards <= 1e-6;
                                                    fp32: >= 69 % exact, >= 92 % within 4 steps
  env sequences fp64 ............................. obs/reward <= 1e-6 abs, identical done/termination
"""
import numpy as np
import pytest
import torch

import _fixtures as F
from oracle import oracle as O
from tum_adlr_deep_reinforcement_learning_amd import config as C

pytestmark = pytest.mark.gpu


def _engine(sim_spec, env_spec=None, n=1, precision="float64", lanes=None):
    from tum_adlr_deep_reinforcement_learning_amd.engine import Engine
    return Engine(sim_spec, env_spec, n, device="cuda:0", precision=precision, lanes=lanes)


# both integrators: one lane per aircraft and the lane quad (fw_quad.hpp)
LANES = pytest.mark.parametrize("lanes", [1, 2, 4])  # one lane, the pair (round 6), the quad


def _rel(a, b):
    return np.abs(a - b) / (np.abs(b) + 1e-3)


def _groups(d):
    keys = {}
    for i in range(len(d["y0"])):
        k = (bool(d["turb_on"][i]), float(d["omega_limit_deg"][i]), float(d["va_limit"][i]))
        keys.setdefault(k, []).append(i)
    return keys


def _run_single_steps(d, precision, lanes=None):
    out = {}
    for (turb, olim, vlim), idx in _groups(d).items():
        spec = C.build_sim(config_kw={"turbulence": turb, "turbulence_sim_length": 300})
        for v in (C.FW_V_OMEGA_P, C.FW_V_OMEGA_Q, C.FW_V_OMEGA_R):
            spec.vars[C.VAR_NAMES[v]].constraint_min = -np.radians(olim)
            spec.vars[C.VAR_NAMES[v]].constraint_max = np.radians(olim)
        spec.vars["Va"].constraint_max = None if not np.isfinite(vlim) else vlim
        n = len(idx)
        eng = _engine(spec, None, n, precision, lanes)
        eng.set_block(C.FW_BLK_ODE, d["y0"][idx].T)
        der = np.zeros((8, n))
        eng.set_block(C.FW_BLK_DERIVED, der)
        eng.set_block(C.FW_BLK_WIND, d["wind"][idx].T)
        eng.set_block(C.FW_BLK_STEPS, d["k"][idx].astype(np.int32))
        if turb:
            L = int(d["k"][idx].max()) + 1
            noise = np.zeros((n, 4, L))
            for j, i in enumerate(idx):
                k = int(d["k"][i])
                noise[j, :, k - 1] = d["noise_km1"][i]
                noise[j, :, k] = d["noise_k"][i]
            eng.set_noise(noise)
        cmd = torch.tensor(d["cmd_in"][idx], dtype=eng.dtype, device=eng.device)
        succ, term = eng.sim_step(cmd, stats=True)
        torch.cuda.synchronize()
        y = eng.get_block(C.FW_BLK_ODE).T.cpu().numpy()
        dr = eng.get_block(C.FW_BLK_DERIVED).T.cpu().numpy()
        st = eng.stats.cpu().numpy()
        for j, i in enumerate(idx):
            out[i] = dict(y=y[j], der=dr[j], term=int(term[j]), nfev=int(st[j] & 0xFFFF), nacc=int((st[j] >> 16) & 0x3FFF),
                          cmd=eng.cmd_out[j].cpu().numpy())
        eng.close()
    return out


@LANES
def test_single_step_fp64_matches_reference(lanes):
    d = F.load("pyfly_single_step.npz")
    out = _run_single_steps(d, "float64", lanes)
    worst = 0.0
    nfev_bad = 0
    for i, r in out.items():
        assert O.term_name(r["term"]) == str(d["term"][i]), (i, r["term"], d["term"][i])
        nfev_bad += r["nfev"] != d["nfev"][i]
        np.testing.assert_allclose(r["cmd"], d["cmd_out"][i], rtol=0, atol=1e-14)
        if d["success"][i]:
            worst = max(worst, _rel(r["y"], d["y1"][i]).max())
            np.testing.assert_allclose(r["der"], d["derived1"][i], rtol=1e-9, atol=1e-11)
    assert worst < 1e-9, worst
    assert nfev_bad <= 1, nfev_bad  # device libm vs glibc may flip one borderline accept/reject


@LANES
def test_single_step_fp32_tolerance(lanes):
    d = F.load("pyfly_single_step.npz")
    out = _run_single_steps(d, "float32", lanes)
    errs = []
    term_bad = 0
    for i, r in out.items():
        term_bad += O.term_name(r["term"]) != str(d["term"][i])
        if d["success"][i] and r["term"] == 0:
            errs.append(_rel(r["y"][:13], d["y1"][i][:13]).max())
    errs = np.array(errs)
    assert term_bad <= 2, term_bad
    assert np.median(errs) <= 1e-6, np.median(errs)
    assert (errs <= 1e-4).mean() >= 0.97, (errs <= 1e-4).mean()
    assert errs.max() <= 5e-3, errs.max()


@LANES
@pytest.mark.parametrize("name", ["pid_off", "pid_on", "rand_off", "rand_on", "rand_fail"])
def test_free_running_trajectory_fp64(name, lanes):
    d = F.load("pyfly_traj.npz")
    g = lambda k: d[name + "__" + k]
    turb = bool(g("turb_on"))
    spec = C.build_sim(config_kw={"turbulence": turb, "turbulence_sim_length": int(g("L"))})
    for v in ("omega_p", "omega_q", "omega_r"):
        spec.vars[v].constraint_min = -np.radians(float(g("omega_lim_deg")))
        spec.vars[v].constraint_max = np.radians(float(g("omega_lim_deg")))
    eng = _engine(spec, None, 1, "float64", lanes)
    eng.set_block(C.FW_BLK_ODE, g("y")[0][:, None])
    der = np.zeros((8, 1))
    der[:6, 0] = g("derived")[0][:6]
    eng.set_block(C.FW_BLK_DERIVED, der)
    eng.set_block(C.FW_BLK_WIND, g("wind")[:, None])
    eng.set_block(C.FW_BLK_STEPS, np.zeros(1, np.int32))
    if turb:
        eng.set_noise(g("noise")[None])
    cmds = torch.tensor(g("cmd"), dtype=torch.float64, device="cuda:0")
    worst, nfev_ok = 0.0, 0
    for s in range(len(cmds)):
        succ, term = eng.sim_step(cmds[s:s + 1], stats=True)
        ok = int(term[0]) == 0
        assert ok == bool(g("success")[s]), s
        nfev_ok += int(eng.stats[0] & 0xFFFF) == int(g("nfev")[s])
        if not ok:
            assert O.term_name(int(term[0])) == str(g("term"))
            break
        y = eng.get_block(C.FW_BLK_ODE)[:, 0].cpu().numpy()
        worst = max(worst, _rel(y, g("y")[s + 1]).max())
    assert worst < 1e-7, worst
    assert nfev_ok >= len(cmds) - 2


@pytest.mark.parametrize("name", list(F.ENV_CASES))
def test_env_sequences_fp64(name):
    d = F.load("env_seq.npz")
    g = lambda k: d[name + "__" + k]
    spec = F.env_spec(name)
    eng = _engine(spec.sim, spec, 1, "float64")
    if bool(g("turb_on")):
        eng.set_noise(g("noise")[None])
    obs0 = eng.reset(init=F.env_init(g("init"))[:, None], target=g("target0")[:, None]).cpu().numpy()[0]
    np.testing.assert_allclose(obs0, g("obs")[0], rtol=1e-12, atol=1e-12)
    acts = torch.tensor(g("act"), dtype=torch.float64, device="cuda:0")
    for s in range(len(acts)):
        obs, rew, done, term = eng.env_step(acts[s:s + 1], auto_reset=False)
        torch.cuda.synchronize()
        dn = bool(done[0])
        assert dn == bool(g("done")[s]), s
        if dn:
            assert O.term_name(int(term[0])) == str(g("term")[s])
            o = eng.terminal_obs[0].cpu().numpy()
        else:
            o = obs[0].cpu().numpy()
        tol = 1e-6 + 1e-6 * s
        assert abs(float(rew[0]) - g("rew")[s]) <= tol, (s, float(rew[0]), g("rew")[s])
        np.testing.assert_allclose(o, g("obs")[s + 1], rtol=1e-5, atol=tol)
        if dn:
            break


def test_env_matches_oracle_fp64_batch():
    """64 envs, random actions incl. out-of-range, 400 steps: fp64 kernel == oracle step by step."""
    _batch_vs_oracle(64, 400, 5)


@pytest.mark.parametrize("n", [1, 63, 257])
def test_env_matches_oracle_fp64_ragged_batches(n):
    """Batch sizes that fill neither a wave (64) nor a block (256): the lanes past N are masked and
    every live lane still equals the oracle (SubprocVecEnv accepts any env count)."""
    _batch_vs_oracle(n, 150, 11 + n)


def _batch_vs_oracle(n, steps, seed):
    spec = C.EnvSpec(config_kw={"steps_max": 250}, sim_config_kw={"turbulence": False})
    rng = np.random.RandomState(seed)
    init = np.full((C.FW_NINIT, n), np.nan)
    d2r = np.radians
    init[C.FW_I_ROLL] = rng.uniform(d2r(-110), d2r(110), n)
    init[C.FW_I_PITCH] = rng.uniform(d2r(-45), d2r(45), n)
    init[C.FW_I_YAW] = rng.uniform(-np.pi, np.pi, n)
    for k in (C.FW_I_P, C.FW_I_Q, C.FW_I_R):
        init[k] = rng.uniform(d2r(-60), d2r(60), n)
    init[C.FW_I_PN:C.FW_I_PD + 1] = rng.uniform(-100, 100, (3, n))
    init[C.FW_I_PD] = rng.uniform(-100, -20, n)
    init[C.FW_I_U] = rng.uniform(10, 23, n)
    init[C.FW_I_V] = rng.uniform(-5, 5, n)
    init[C.FW_I_W] = rng.uniform(-5, 5, n)
    init[C.FW_I_ACT0:C.FW_I_ACT2_DOT + 1] = 0.0
    init[C.FW_I_WIND_N:] = rng.uniform(-3, 3, (3, n))
    tgt = np.stack([rng.uniform(d2r(-60), d2r(60), n), rng.uniform(d2r(-25), d2r(25), n), rng.uniform(15, 28, n)])
    eng = _engine(spec.sim, spec, n, "float64")
    obs = eng.reset(init=init, target=tgt).cpu().numpy()
    envs = [O.OracleEnv(spec.sim.struct(), spec.struct(), spec.n_obs) for _ in range(n)]
    for j in range(n):
        np.testing.assert_allclose(envs[j].reset(init[:, j], tgt[:, j]), obs[j], rtol=1e-12, atol=1e-12)
    alive = np.ones(n, bool)
    for s in range(steps):
        a = rng.uniform(-1.3, 1.3, (n, 3))
        o, r, dn, tm = eng.env_step(torch.tensor(a, device="cuda:0"), auto_reset=False)
        o, r, dn, tm = o.cpu().numpy(), r.cpu().numpy(), dn.cpu().numpy(), tm.cpu().numpy()
        to = eng.terminal_obs.cpu().numpy()
        for j in np.nonzero(alive)[0]:
            oo, rr, dd, tt, _ = envs[j].step(a[j])
            assert dd == bool(dn[j]) and tt == int(tm[j]), (s, j, dd, dn[j], tt, tm[j])
            assert abs(rr - r[j]) <= 1e-7 + 1e-7 * s, (s, j, rr, r[j])
            np.testing.assert_allclose(to[j] if dd else o[j], oo, rtol=1e-6, atol=1e-7 + 1e-7 * s)
            if dd:
                alive[j] = False
        if not alive.any():
            break


@pytest.mark.parametrize("n,lanes", [(65536, 1), (65536, 2), (65536, 4), (262144 + 37, 1)])
def test_full_size_properties_fp32(n, lanes):
    """65536 envs (configs[2]) and a ragged batch above the largest config (262144 + 37), 300 steps of
    U(-1,1) actions with auto-reset: finite, bounded, deterministic, shard-invariant -- bit for bit for a
    fixed integrator (the automatic lanes choice depends on the shard size, fw_set_lanes)."""
    spec = C.EnvSpec(sim_config_kw={"turbulence": False})

    def run(seed, offset=0, count=n, steps=300):
        eng = _engine(spec.sim, spec, count, "float32", lanes)
        eng.seed(seed, env_offset=offset)
        eng.reset()
        g = torch.Generator(device="cuda:0")
        g.manual_seed(1)
        tot = torch.zeros(count, dtype=torch.float64, device="cuda:0")
        dones = 0
        for s in range(steps):
            a = torch.rand(n, 3, generator=g, device="cuda:0") * 2 - 1
            o, r, d, t = eng.env_step(a[offset:offset + count])
            assert torch.isfinite(o).all() and torch.isfinite(r).all()
            tot += r.double()
            dones += int(d.sum())
        ode = eng.get_block(C.FW_BLK_ODE).cpu()
        eng.close()
        return tot.cpu(), dones, ode

    tot, dones, ode = run(3)
    q = ode[:4]
    assert torch.allclose((q * q).sum(0), torch.ones(n), atol=1e-5)  # saved quaternion is normalised
    tot2, dones2, ode2 = run(3)
    assert torch.equal(tot, tot2) and dones == dones2 and torch.equal(ode, ode2)  # bitwise deterministic
    half = n // 2 // 64 * 64  # shard offsets on wave boundaries: bitwise invariance holds per wave (tail handoff)
    tot_b, _, ode_b = run(3, offset=half, count=n - half)  # shard = the second half of the same batch
    assert torch.equal(tot_b, tot[half:]) and torch.equal(ode_b, ode[:, half:])


@pytest.mark.parametrize("precision", ["float64", "float32"])
def test_generic_and_specialised_kernels_agree(precision, monkeypatch):
    """The structure-specialised kernel (GymX8Cfg) and the generic DevCfg kernel compute the same step.
    Not bitwise: the compiler contracts multiply-adds differently in the two instances, so fp64 agrees to
    ~1e-12 and fp32 to ~1e-6 (both far inside the oracle tolerances above)."""
    spec = C.EnvSpec(config_kw={"steps_max": 60}, sim_config_kw={"turbulence": False})
    n = 1024

    def run(generic):
        if generic:
            monkeypatch.setenv("FWSIM_GENERIC", "1")
        else:
            monkeypatch.delenv("FWSIM_GENERIC", raising=False)
        eng = _engine(spec.sim, spec, n, precision)
        eng.seed(9)
        eng.reset()
        g = torch.Generator(device="cuda:0")
        g.manual_seed(3)
        out = []
        for _ in range(80 if precision == "float64" else 10):  # fp32 trajectories decorrelate after flips
            a = torch.rand(n, 3, generator=g, device="cuda:0", dtype=eng.dtype) * 2.4 - 1.2
            o, r, d, t = eng.env_step(a, stats=True)
            out.append((o.clone(), r.clone(), d.clone(), t.clone(), eng.stats.clone()))
        eng.close()
        return out

    a, b = run(False), run(True)
    if precision == "float64":
        for (o1, r1, d1, t1, s1), (o2, r2, d2, t2, s2) in zip(a, b):
            assert torch.equal(d1, d2) and torch.equal(t1, t2)
            assert torch.allclose(o1, o2, rtol=1e-9, atol=1e-9) and torch.allclose(r1, r2, rtol=1e-9, atol=1e-9)
    else:  # a 1-ulp difference can flip an RK45 accept/reject: require agreement on >= 99 % of the envs
        for (o1, r1, d1, t1, s1), (o2, r2, d2, t2, s2) in zip(a, b):
            close = ((o1 - o2).abs() <= 1e-4 * (1 + o2.abs())).all(1) & ((r1 - r2).abs() <= 1e-4 * (1 + r2.abs()))
            assert close.float().mean() >= 0.99
            assert (d1 == d2).float().mean() >= 0.99


def _free_run(name, precision):
    """Free-running PyFly.step replay of a pyfly_traj.npz case: per-step |y - y_ref| per component, the
    step of the first RK45 accept/reject divergence from the reference (nfev differs), fail steps."""
    d = F.load("pyfly_traj.npz")
    g = lambda k: d[name + "__" + k]  # noqa: E731
    turb = bool(g("turb_on"))
    spec = C.build_sim(config_kw={"turbulence": turb, "turbulence_sim_length": int(g("L"))})
    for v in ("omega_p", "omega_q", "omega_r"):
        spec.vars[v].constraint_min = -np.radians(float(g("omega_lim_deg")))
        spec.vars[v].constraint_max = np.radians(float(g("omega_lim_deg")))
    eng = _engine(spec, None, 1, precision)
    eng.set_block(C.FW_BLK_ODE, g("y")[0][:, None])
    der = np.zeros((8, 1))
    der[:6, 0] = g("derived")[0][:6]
    eng.set_block(C.FW_BLK_DERIVED, der)
    eng.set_block(C.FW_BLK_WIND, g("wind")[:, None])
    eng.set_block(C.FW_BLK_STEPS, np.zeros(1, np.int32))
    if turb:
        eng.set_noise(g("noise")[None])
    cmds = torch.tensor(g("cmd"), dtype=eng.dtype, device="cuda:0")
    dev = np.zeros_like(g("y"))
    fail, first_flip = len(cmds), len(cmds)
    for s in range(len(cmds)):
        succ, term = eng.sim_step(cmds[s:s + 1], stats=True)
        if int(eng.stats[0] & 0xFFFF) != int(g("nfev")[s]) and first_flip == len(cmds):
            first_flip = s
        if int(term[0]) != 0:
            fail = s
            break
        dev[s + 1] = np.abs(eng.get_block(C.FW_BLK_ODE)[:, 0].double().cpu().numpy() - g("y")[s + 1])
    eng.close()
    ref_fail = len(cmds) if bool(g("success")[-1]) else len(cmds) - 1
    rms = np.sqrt(np.mean(g("y") ** 2, axis=0)) + 1e-3  # per-component signal scale
    return dev / rms, rms, fail, ref_fail, first_flip


@pytest.mark.parametrize("name", ["pid_off", "pid_on", "rand_off", "rand_on", "rand_fail"])
def test_free_running_trajectory_fp32_within_reference_envelope(name):
    """SURVEY.md 8(d) gate 3, measured against the reference's OWN sensitivity (pyfly_envelope.npz: the
    reference replaying the same 1000 commands from perturbed inputs).  Error metric per step: max over
    ODE components of |y - y_ref| / rms(y_ref component), a component's error relative to its signal
    scale (|y| + 1e-3 explodes at the zero crossings of the actuator rates).

    Gate: termination step identical +-1, and at every step the error stays inside the band the
    reference itself spans (running maxima) under either
      * its ODE state STORED in float32 after every step (fp64 arithmetic in between; x5), or
      * one solver-tolerance kick (initial state x (1 +- rtol = 1e-3)) -- the size of the state change
        an RK45 accept/reject decision, or a stage crossing an actuator clip boundary, makes when fp32
        rounding puts it on the other side.
    Measured (round 1): max error / band 0.01-0.30; the first accept/reject divergence from the fp64
    reference comes after 68-1000 steps.  A one-off relative 1e-7 perturbation of the initial state
    (the survey's first proposal, also in the fixture as dev_eps) is exceeded 5-85x: fp32 re-rounds the
    state every step and the dynamics amplify each rounding, which that yardstick does not model."""
    E = F.load("pyfly_envelope.npz")
    e, rms_ref, fail, ref_fail, flip = _free_run(name, "float32")
    assert abs(fail - ref_fail) <= 1, (fail, ref_fail)
    n = min(fail, ref_fail) + 1
    err = e[:n].max(axis=1)
    env32 = np.maximum.accumulate((E[name + "__dev_state32"][:n] / rms_ref).max(axis=1))
    env_rtol = np.maximum.accumulate((E[name + "__dev_rtol"][:n] / rms_ref).max(axis=1))
    band = np.maximum(np.maximum(5.0 * env32, env_rtol), 1e-5)
    print("%s: first accept/reject flip at step %d; max err %.2e, max err/band %.2f"
          % (name, flip, err.max(), (err / band).max()))
    assert np.all(err <= band), int((err / band).argmax())


def _pid_batch(precision):
    """The 40-scenario PID evaluation set (env_pid_set.npz) as one batch of envs on the device."""
    from _pid import PID
    d = F.load("env_pid_set.npz")
    ckw = {"steps_max": 1500, "action": {"scale_space": False},
           "target": {"on_success": "done", "success_streak_fraction": 1, "success_streak_req": 100,
                      "states": {0: {"bound": 5}, 1: {"bound": 5}, 2: {"bound": 2}}}}
    spec = C.EnvSpec(config_kw=ckw, sim_config_kw={"turbulence": False})
    n = len(d["length"])
    init = np.full((C.FW_NINIT, n), np.nan)
    init[:12] = d["init"].T
    init[C.FW_I_ACT0:C.FW_I_ACT2_DOT + 1] = 0.0
    init[C.FW_I_WIND_N:] = 0.0
    eng = _engine(spec.sim, spec, n, precision)
    obs = eng.reset(init=init, target=d["target"].T).double().cpu().numpy()
    pids = [PID(*d["target"][i]) for i in range(n)]
    length = np.zeros(n, int)
    rew = np.zeros((n, 1500))
    alive = np.ones(n, bool)
    for s in range(1500):
        a = np.stack([pids[i].action(obs[i]) for i in range(n)])
        o, r, dn, _ = eng.env_step(torch.tensor(a, dtype=eng.dtype, device="cuda:0"), auto_reset=False)
        o, r, dn = o.double().cpu().numpy(), r.double().cpu().numpy(), dn.cpu().numpy().astype(bool)
        for i in np.nonzero(alive)[0]:
            pids[i].set_reference(*o[i, 6:9])
            rew[i, s] = r[i]
            length[i] += 1
            if dn[i]:
                alive[i] = False
        obs = o
        if not alive.any():
            break
    eng.close()
    return d, length, rew


def test_pid_evaluation_set_fp64_episode_lengths_and_rewards():
    """SURVEY.md 8(d) gate 4, fp64: the device reproduces the reference's PID replay of the evaluation
    set (episode lengths exact on all but at most one scenario, per-step rewards within 1e-6 + 1e-6/step)."""
    d, length, rew = _pid_batch("float64")
    exact = int((length == d["length"]).sum())
    assert exact >= len(length) - 1, (exact, length, d["length"])
    for i in np.nonzero(length == d["length"])[0]:
        L = length[i]
        tol = 1e-6 + 1e-6 * np.arange(L)
        assert np.all(np.abs(rew[i, :L] - d["reward"][i, :L]) <= tol), i


def test_pid_evaluation_set_fp32_episode_lengths():
    """SURVEY.md 8(d) gate 4, fp32: within the loose bound the reference itself shows against its stored
    eval_res_PID_none.npy (>= 69% exact episode lengths, >= 92% within 4 steps)."""
    d, length, _ = _pid_batch("float32")
    exact = (length == d["length"]).mean()
    near = (np.abs(length - d["length"]) <= 4).mean()
    print("fp32 PID set: exact %.3f, within 4 steps %.3f" % (exact, near))
    assert exact >= 0.69 and near >= 0.92, (exact, near, length, d["length"])
