"""Generate the golden fixtures that pin the oracle (test infrastructure only).

Runs the *reference itself* (pyfly + gym_fixed_wing from /root/reference, pure
Python, importable in the build container) on seeded inputs and stores inputs +
outputs as small ``.npz`` files next to this script.  Only data leaves this
script; no reference source is copied.  The GPU box never runs this file.

The reference imports ``gym`` (0.18), which is not installed here, so this script
installs a tiny offline stand-in module providing exactly what
``fixed_wing.py`` touches: ``gym.Env``, ``gym.spaces.Box`` and
``gym.utils.seeding.np_random`` (restated from gym 0.18's sha512 seeding scheme).
All env fixtures pass explicit ``state``/``target`` dicts to ``reset`` so they
do not depend on that seeding scheme.

Usage:  python tests/golden/gen_golden.py   (takes ~2-4 minutes)

Fixtures (all float64 unless noted):
  pyfly_single_step.npz   teacher-forced single PyFly.step cases (turbulence off/on)
  pyfly_traj.npz          free-running PyFly trajectories (PID + random commands)
  dryden.npz              Dryden FIR coefficients + raw filter outputs
  dryden_wrap.npz         Dryden outputs for a turbulence_noise sequence shorter than the span (wraps)
  env_seq.npz             FixedWingAircraft reset/step sequences (obs, reward, done, term)
  env_pid_set.npz         PID replay of a synthetic 40-scenario evaluation set
  env_metrics.npz         episode metrics + histories for metric scenarios
  env_obs_hist.npz        observation-history episodes (observation.length > 1)
  pyfly_envelope.npz      the reference's own sensitivity to a 1e-7 initial perturbation (fp32 gate)
  pyfly_solver_fail.npz   PyFly.step when the RK45 integration fails (sol.y[:, -1] committed)
  pyfly_energy.npz        energy states along PID / constraint-terminated trajectories
  env_curriculum.npz      set_curriculum_level ranges/constraints/targets and sampled resets
  env_rand_params.npz     simulator parameter randomisation: sampled parameters and episodes flown with them
  env_history.npz         FixedWingAircraft.history of a PID episode and of a constraint-terminated one
"""
import hashlib
import json
import math
import os
import struct
import sys
import types

import numpy as np

REF = "/root/reference/magpie/libs"
OUT = os.path.dirname(os.path.abspath(__file__))

# ---------------------------------------------------------------------------
# offline gym stand-in (only what fixed_wing.py uses)
# ---------------------------------------------------------------------------


def _install_gym_stub():
    gym = types.ModuleType("gym")
    spaces = types.ModuleType("gym.spaces")
    utils = types.ModuleType("gym.utils")
    seeding = types.ModuleType("gym.utils.seeding")

    class Env:
        metadata = {}

    class Box:
        def __init__(self, low, high, shape=None, dtype=np.float32):
            self.dtype = np.dtype(dtype)
            self.low = np.asarray(low, dtype=self.dtype)
            self.high = np.asarray(high, dtype=self.dtype)
            self.shape = self.low.shape

    def _bigint_from_bytes(b):
        pad = 4 - len(b) % 4
        b = b + b"\0" * pad
        vals = struct.unpack("{}I".format(len(b) // 4), b)
        return sum(v << (32 * i) for i, v in enumerate(vals))

    def _int_list_from_bigint(x):
        if x == 0:
            return [0]
        out = []
        while x > 0:
            x, m = divmod(x, 2 ** 32)
            out.append(m)
        return out

    def np_random(seed=None):
        if seed is None:
            seed = _bigint_from_bytes(os.urandom(8))
        seed = seed % 2 ** 64
        h = _bigint_from_bytes(hashlib.sha512(str(seed).encode("utf8")).digest()[:8])
        rng = np.random.RandomState()
        rng.seed(_int_list_from_bigint(h))
        return rng, seed

    class GoalEnv(Env):
        pass

    gym.Env = Env
    gym.GoalEnv = GoalEnv
    spaces.Box = Box
    gym.spaces = spaces
    seeding.np_random = np_random
    utils.seeding = seeding
    gym.utils = utils
    for name, mod in [("gym", gym), ("gym.spaces", spaces), ("gym.utils", utils),
                      ("gym.utils.seeding", seeding)]:
        sys.modules[name] = mod


_install_gym_stub()
sys.path.insert(0, os.path.join(REF, "pyfly"))
sys.path.insert(0, os.path.join(REF, "fixed-wing-gym"))
import scipy.integrate  # noqa: E402
import pyfly.pyfly as pf  # noqa: E402
from pyfly.dryden import DrydenGustModel  # noqa: E402
from gym_fixed_wing.fixed_wing import FixedWingAircraft  # noqa: E402

PYFLY_CFG = os.path.join(REF, "pyfly/pyfly/pyfly_config.json")
PYFLY_PARAM = os.path.join(REF, "pyfly/pyfly/x8_param.mat")
GYM_CFG = os.path.join(REF, "fixed-wing-gym/gym_fixed_wing/fixed_wing_config.json")

# ---------------------------------------------------------------------------
# instrumentation: solver statistics per PyFly.step
# ---------------------------------------------------------------------------
_orig_solve_ivp = scipy.integrate.solve_ivp
_last = {}


def _solve_ivp_probe(*a, **k):
    _last.clear()
    sol = _orig_solve_ivp(*a, **k)
    _last["nfev"] = sol.nfev
    _last["naccept"] = len(sol.t) - 1
    return sol


scipy.integrate.solve_ivp = _solve_ivp_probe


def _count_rhs(sim):
    counter = {"n": 0}
    inner = sim._dynamics

    def wrapped(t, y, control_sp=None):
        counter["n"] += 1
        return inner(t, y, control_sp)

    sim._dynamics = wrapped
    return counter


ODE_NAMES = ["omega_p", "omega_q", "omega_r", "position_n", "position_e", "position_d",
             "velocity_u", "velocity_v", "velocity_w"]


def ode_vector(sim):
    y = list(sim.state["attitude"].value)
    y += [sim.state[n].value for n in ODE_NAMES]
    y += sim.actuation.get_values()
    return np.array(y, dtype=np.float64)


def derived(sim):
    return np.array([sim.state[n].value for n in ["roll", "pitch", "yaw", "Va", "alpha", "beta",
                                                   "elevator", "aileron"]], dtype=np.float64)


def hist_last(sim):
    """history[-1] of the env-observed states (what FixedWingAircraft.get_observation reads)."""
    return np.array([sim.state[n].history[-1] for n in
                     ["roll", "pitch", "yaw", "Va", "alpha", "beta", "omega_p", "omega_q", "omega_r"]],
                    dtype=np.float64)


def turb_at(sim, k):
    if not sim.wind.turbulence:
        return np.zeros(6)
    return np.concatenate([sim.wind.dryden.vel_lin[:, k], sim.wind.dryden.vel_ang[:, k]])


def random_state(rng, omega_deg=60.0, dots=True):
    """A full explicit initial-state dict in the gym init ranges."""
    d2r = np.radians
    st = {
        "roll": rng.uniform(d2r(-110), d2r(110)),
        "pitch": rng.uniform(d2r(-45), d2r(45)),
        "yaw": rng.uniform(d2r(-180), d2r(180)),
        "omega_p": rng.uniform(d2r(-omega_deg), d2r(omega_deg)),
        "omega_q": rng.uniform(d2r(-omega_deg), d2r(omega_deg)),
        "omega_r": rng.uniform(d2r(-omega_deg), d2r(omega_deg)),
        "position_n": rng.uniform(-100, 100),
        "position_e": rng.uniform(-100, 100),
        "position_d": rng.uniform(-100, -20),
        "velocity_u": rng.uniform(10, 23),
        "velocity_v": rng.uniform(-5, 5),
        "velocity_w": rng.uniform(-5, 5),
    }
    if dots:
        st["elevon_right"] = (rng.uniform(d2r(-30), d2r(35)), rng.uniform(-3.4907, 3.4907))
        st["elevon_left"] = (rng.uniform(d2r(-30), d2r(35)), rng.uniform(-3.4907, 3.4907))
        st["throttle"] = (rng.uniform(0, 1), 0.0)
    else:
        st["elevon_right"] = 0.0
        st["elevon_left"] = 0.0
        st["throttle"] = 0.0
    return st


def random_wind(rng, mag=8.0):
    m = rng.uniform(-mag, mag)
    wn = rng.uniform(-abs(m), abs(m))
    we_max = math.sqrt(max(m * m - wn * wn, 0.0))
    we = rng.uniform(-we_max, we_max)
    wd = math.sqrt(max(m * m - wn * wn - we * we, 0.0))
    return [wn, we, wd]


# ---------------------------------------------------------------------------
# A. teacher-forced single steps
# ---------------------------------------------------------------------------


def gen_single_step():
    rows = {k: [] for k in ["turb_on", "y0", "wind", "k", "turb", "noise_km1", "noise_k", "cmd_in",
                            "cmd_out", "y1", "success", "term", "nfev", "naccept", "derived1",
                            "hist1", "omega_limit_deg", "va_limit"]}
    rng = np.random.RandomState(12345)
    L = 300
    n_cases = 800
    for i in range(n_cases):
        turb_on = i % 2 == 1
        omega_lim = 180.0 if i % 4 < 2 else 720.0
        kw = {"turbulence": turb_on, "turbulence_sim_length": L,
              "variables": {}}
        sim = pf.PyFly(PYFLY_CFG, PYFLY_PARAM, config_kw={"turbulence": turb_on,
                                                          "turbulence_sim_length": L})
        for n in ["omega_p", "omega_q", "omega_r"]:
            sim.state[n].constraint_min = np.radians(-omega_lim)
            sim.state[n].constraint_max = np.radians(omega_lim)
        sim.seed(1000 + i)
        # some cases start near the omega constraint to exercise termination
        st = random_state(rng, omega_deg=(175.0 if i % 16 == 3 else 60.0))
        wind = random_wind(rng) if i % 3 else [0.0, 0.0, 0.0]
        st["wind"] = wind
        noise = rng.standard_normal((4, L)) if turb_on else None
        sim.reset(state=st, turbulence_noise=noise)
        if i % 16 == 3:  # tight omega constraint: exercises mid-integration termination
            lim = max(abs(st[n]) for n in ["omega_p", "omega_q", "omega_r"]) + np.radians(0.5)
            for n in ["omega_p", "omega_q", "omega_r"]:
                sim.state[n].constraint_min, sim.state[n].constraint_max = -lim, lim
            omega_lim = np.degrees(lim)
        if i % 16 == 7:  # tight airspeed constraint (gym config has Va <= 70)
            sim.state["Va"].constraint_max = sim.state["Va"].value + 0.002
        k = int(rng.randint(1, L - 1)) if turb_on else 0
        sim.cur_sim_step = k
        cnt = _count_rhs(sim)
        # commands: elevator, aileron, throttle (gym input ordering), slightly beyond limits sometimes
        cmd = [rng.uniform(np.radians(-40), np.radians(45)), rng.uniform(np.radians(-40), np.radians(40)),
               rng.uniform(-0.2, 1.2)]
        y0 = ode_vector(sim)
        turb = turb_at(sim, k)
        cmd_in = list(cmd)
        ok, info = sim.step(cmd)
        rows["turb_on"].append(turb_on)
        rows["y0"].append(y0)
        rows["wind"].append(np.array(wind, dtype=np.float64))
        rows["k"].append(k)
        rows["turb"].append(turb)
        if turb_on:
            rows["noise_km1"].append(noise[:, k - 1])
            rows["noise_k"].append(noise[:, k])
        else:
            rows["noise_km1"].append(np.zeros(4))
            rows["noise_k"].append(np.zeros(4))
        rows["cmd_in"].append(np.array(cmd_in))
        rows["cmd_out"].append(np.array(cmd, dtype=np.float64))
        rows["y1"].append(ode_vector(sim))
        rows["success"].append(ok)
        rows["term"].append(info.get("termination", ""))
        rows["nfev"].append(cnt["n"])
        rows["naccept"].append(_last.get("naccept", -1) if ok else -1)
        rows["derived1"].append(derived(sim))
        rows["hist1"].append(hist_last(sim))
        rows["omega_limit_deg"].append(omega_lim)
        vc = sim.state["Va"].constraint_max
        rows["va_limit"].append(np.inf if vc is None else vc)
    out = {k: np.array(v) for k, v in rows.items()}
    np.savez_compressed(os.path.join(OUT, "pyfly_single_step.npz"), **out)
    print("single steps: %d cases, %d failures, nfev mean %.1f" % (
        n_cases, int((~out["success"]).sum()), out["nfev"].mean()))


# ---------------------------------------------------------------------------
# B. free-running trajectories
# ---------------------------------------------------------------------------


def pid_action(pid, sim):
    phi = sim.state["roll"].value
    theta = sim.state["pitch"].value
    va = sim.state["Va"].value
    om = [sim.state["omega_p"].value, sim.state["omega_q"].value]
    e_v, e_phi, e_th = va - pid["va"], phi - pid["phi"], theta - pid["theta"]
    pid["iv"] += pid["dt"] * e_v
    pid["ir"] += pid["dt"] * e_phi
    pid["ip"] += pid["dt"] * e_th
    dt_ = 0 - 0.5 * e_v - 0.1 * pid["iv"]
    da = -1 * e_phi - 0 * pid["ir"] - 0.5 * om[0]
    de = 0 - (-4) * e_th - (-0.75) * pid["ip"] - (-0.1) * om[1]
    return [float(np.clip(de, np.radians(-30), np.radians(35))),
            float(np.clip(da, np.radians(-30), np.radians(30))),
            float(np.clip(dt_, 0, 1))]


def run_traj(turb_on, controller, seed, n_steps=1000, L=300, omega_lim_deg=None):
    rng = np.random.RandomState(seed)
    sim = pf.PyFly(PYFLY_CFG, PYFLY_PARAM, config_kw={"turbulence": turb_on,
                                                      "turbulence_sim_length": L})
    if omega_lim_deg is not None:
        for n in ["omega_p", "omega_q", "omega_r"]:
            sim.state[n].constraint_min = np.radians(-omega_lim_deg)
            sim.state[n].constraint_max = np.radians(omega_lim_deg)
    sim.seed(seed)
    st = random_state(rng, omega_deg=60.0 if omega_lim_deg is None else 0.5 * omega_lim_deg, dots=False)
    st["roll"], st["pitch"] = -0.5, 0.15
    wind = random_wind(rng) if turb_on else [0.0, 0.0, 0.0]
    st["wind"] = wind
    n_chunks = (n_steps + L - 1) // L + 1
    noise = rng.standard_normal((4, L * n_chunks)) if turb_on else np.zeros((4, L * n_chunks))
    sim.reset(state=st, turbulence_noise=noise if turb_on else None)
    cnt = _count_rhs(sim)
    pid = {"dt": sim.dt, "va": 22.0, "phi": 0.2, "theta": 0.0, "iv": 0.0, "ir": 0.0, "ip": 0.0}
    y = [ode_vector(sim)]
    der = [derived(sim)]
    cmds, nfev, succ, term = [], [], [], ""
    for s in range(n_steps):
        if controller == "pid":
            cmd = pid_action(pid, sim)
        else:
            cmd = [rng.uniform(np.radians(-30), np.radians(35)), rng.uniform(np.radians(-32.5), np.radians(32.5)),
                   rng.uniform(0, 1)]
        cmds.append(list(cmd))
        cnt["n"] = 0
        ok, info = sim.step(cmd)
        nfev.append(cnt["n"])
        succ.append(ok)
        y.append(ode_vector(sim))
        der.append(derived(sim))
        if not ok:
            term = info["termination"]
            break
    return dict(y=np.array(y), derived=np.array(der), cmd=np.array(cmds), nfev=np.array(nfev),
                success=np.array(succ), term=np.array(term), wind=np.array(wind), noise=noise,
                L=np.array(L), turb_on=np.array(turb_on),
                omega_lim_deg=np.array(180.0 if omega_lim_deg is None else omega_lim_deg))


def gen_traj():
    out = {}
    for name, turb_on, ctrl, seed, olim in [("pid_off", False, "pid", 0, None), ("pid_on", True, "pid", 0, None),
                                            ("rand_off", False, "rand", 1, None),
                                            ("rand_on", True, "rand", 2, None),
                                            ("rand_fail", True, "rand", 3, 45.0)]:
        tr = run_traj(turb_on, ctrl, seed, omega_lim_deg=olim)
        for k, v in tr.items():
            out[name + "__" + k] = v
        print("traj %s: %d steps, term=%r, nfev mean %.1f" % (name, len(tr["nfev"]), str(tr["term"]),
                                                             tr["nfev"].mean()))
    np.savez_compressed(os.path.join(OUT, "pyfly_traj.npz"), **out)


TRAJ_CASES = [("pid_off", False, 0, None), ("pid_on", True, 0, None), ("rand_off", False, 1, None),
              ("rand_on", True, 2, None), ("rand_fail", True, 3, 45.0)]


def _replay_open_loop(name, turb_on, seed, olim, cmds, L, perturb, post=None):
    """Replay a pyfly_traj case open-loop from its recorded commands; perturb(st, cmd, k) edits inputs."""
    rng = np.random.RandomState(seed)
    sim = pf.PyFly(PYFLY_CFG, PYFLY_PARAM, config_kw={"turbulence": turb_on, "turbulence_sim_length": L})
    if olim is not None:
        for n in ["omega_p", "omega_q", "omega_r"]:
            sim.state[n].constraint_min = np.radians(-olim)
            sim.state[n].constraint_max = np.radians(olim)
    sim.seed(seed)
    st = random_state(rng, omega_deg=60.0 if olim is None else 0.5 * olim, dots=False)
    st["roll"], st["pitch"] = -0.5, 0.15
    wind = random_wind(rng) if turb_on else [0.0, 0.0, 0.0]
    n_chunks = (len(cmds) + L - 1) // L + 1
    noise = rng.standard_normal((4, L * n_chunks)) if turb_on else np.zeros((4, L * n_chunks))
    perturb(st, None, -1)
    st["wind"] = wind
    sim.reset(state=st, turbulence_noise=noise if turb_on else None)
    ys, fail = [ode_vector(sim)], len(cmds)
    for s in range(len(cmds)):
        cmd = [float(c) for c in cmds[s]]
        perturb(None, cmd, s)
        ok, _ = sim.step(cmd)
        if not ok:
            fail = s
            break
        if post is not None:
            post(sim, s)
        ys.append(ode_vector(sim))
    return np.array(ys), fail


def gen_envelope(eps=1e-7, n_pert=3):
    """The reference's own sensitivity (SURVEY.md 8 d, gate 3), per step and ODE component, as the
    maximum absolute deviation from the pyfly_traj.npz trajectory when the trajectory is replayed
    open-loop (its recorded commands) with perturbed inputs:
      dev_eps   initial state entries scaled by (1 +- eps), n_pert random sign patterns
      dev_fp32  initial state and every step's commands rounded to float32 (what an fp32 engine is
                handed), the arithmetic still fp64
      dev_rtol  initial state scaled by (1 +- rtol = 1e-3): one solver-tolerance-sized kick, the size
                of the state change an RK45 accept/reject decision that goes the other way makes
      dev_state32  fp32 inputs and the ODE state rounded to float32 after every step (nearest; and
                nearest +- 1 ulp at random for the other patterns)
    plus the perturbed runs' termination steps (fail_*)."""
    d = np.load(os.path.join(OUT, "pyfly_traj.npz"))
    out = {}
    for name, turb_on, seed, olim in TRAJ_CASES:
        g = lambda k: d[name + "__" + k]  # noqa: E731
        cmds, y_ref, L = g("cmd"), g("y"), int(g("L"))

        def dev_of(perturb_factory, reps):
            dev = np.zeros_like(y_ref)
            fails = []
            for k in range(reps):
                yp, f = _replay_open_loop(name, turb_on, seed, olim, cmds, L, perturb_factory(k))
                n = min(len(yp), len(y_ref))
                dev[:n] = np.maximum(dev[:n], np.abs(yp[:n] - y_ref[:n]))
                fails.append(f)
            return dev, np.array(fails)

        def scaled(e):
            def factory(k):
                prng = np.random.RandomState(1000 * (1 + int(e == 1e-3)) + k)

                def pert(st, cmd, kk):
                    if st is not None:
                        for key in ENV_STATE_KEYS:
                            st[key] = st[key] * (1.0 + e * prng.choice([-1.0, 1.0]))
                return pert
            return factory

        def to32_factory(k):
            def to32(st, cmd, kk):
                if st is not None:
                    for key in ENV_STATE_KEYS:
                        st[key] = float(np.float32(st[key]))
                if cmd is not None:
                    cmd[:] = [float(np.float32(c)) for c in cmd]
            return to32

        def state32(k):
            # the ODE state stored in float32 after every step (round to nearest, plus for k > 0 a
            # random +-1 ulp): an fp32 engine's per-step rounding, with fp64 arithmetic in between
            prng = np.random.RandomState(3000 + k)

            def post(sim, s):
                y = ode_vector(sim).astype(np.float32)
                if k > 0:
                    y = np.nextafter(y, np.where(prng.rand(len(y)) < 0.5, -np.inf, np.inf).astype(np.float32))
                sim._set_states_from_ode_solution(y.astype(np.float64), save=False)
            return post

        def dev_state32(reps):
            dev = np.zeros_like(y_ref)
            fails = []
            for k in range(reps):
                yp, f = _replay_open_loop(name, turb_on, seed, olim, cmds, L, to32_factory(k), post=state32(k))
                n = min(len(yp), len(y_ref))
                dev[:n] = np.maximum(dev[:n], np.abs(yp[:n] - y_ref[:n]))
                fails.append(f)
            return dev, np.array(fails)

        for tag, fac, reps in (("eps", scaled(eps), n_pert), ("fp32", to32_factory, 1), ("rtol", scaled(1e-3), n_pert),
                               ("state32", None, n_pert)):
            dev, fails = dev_state32(reps) if tag == "state32" else dev_of(fac, reps)
            out[name + "__dev_" + tag] = dev
            out[name + "__fail_" + tag] = fails
            rms = np.sqrt(np.mean(y_ref ** 2, axis=0)) + 1e-3
            e = np.max(dev / rms, axis=1)
            print("%s %s: scaled deviation at 100 %.2e, 500 %.2e, max %.2e, fails %s"
                  % (name, tag, e[min(100, len(e) - 1)], e[min(500, len(e) - 1)], e.max(), fails))
    out["eps"] = np.array(eps)
    np.savez_compressed(os.path.join(OUT, "pyfly_envelope.npz"), **out)


# ---------------------------------------------------------------------------
# C. Dryden
# ---------------------------------------------------------------------------


def gen_dryden():
    out = {}
    rng = np.random.RandomState(7)
    for L, inten in [(300, "light"), (300, "moderate"), (300, "severe"), (2000, "light"),
                     (2000, "severe")]:
        if True:
            # exactly how pyfly.Wind wires it (pyfly.py:781-783): positional (sim_length, dt, b)
            dm = DrydenGustModel(L, 0.01, 2.1, intensity=inten)
            noise = rng.standard_normal((4, 2 * L))
            dm.reset(noise)
            dm.simulate(L)
            dm.simulate(L)
            keep = np.r_[0:200, L - 20:L + 200]  # both chunk starts, FIR interior
            out["L%d_%s__noise" % (L, inten)] = noise[:, keep]
            out["L%d_%s__idx" % (L, inten)] = keep
            out["L%d_%s__vel_lin" % (L, inten)] = dm.vel_lin[:, keep]
            out["L%d_%s__vel_ang" % (L, inten)] = dm.vel_ang[:, keep]
    np.savez_compressed(os.path.join(OUT, "dryden.npz"), **out)
    print("dryden done")


def gen_dryden_wrap():
    """A turbulence_noise sequence SHORTER than the simulated span (DrydenGustModel.simulate wraps it,
    dryden.py:209-236): lengths 170 (wraps inside chunk 1 and again in chunk 2) and 450 (inside chunk 2)."""
    out = {}
    rng = np.random.RandomState(11)
    L = 300
    for n in (170, 450):
        dm = DrydenGustModel(L, 0.01, 2.1, intensity="moderate")
        noise = rng.standard_normal((4, n))
        dm.reset(noise)
        dm.simulate(L)
        dm.simulate(L)
        out["n%d__noise" % n] = noise
        out["n%d__vel_lin" % n] = dm.vel_lin
        out["n%d__vel_ang" % n] = dm.vel_ang
    np.savez_compressed(os.path.join(OUT, "dryden_wrap.npz"), **out)
    print("dryden_wrap done")


# ---------------------------------------------------------------------------
# D. gym env sequences
# ---------------------------------------------------------------------------

ENV_STATE_KEYS = ["roll", "pitch", "yaw", "omega_p", "omega_q", "omega_r", "position_n", "position_e",
                  "position_d", "velocity_u", "velocity_v", "velocity_w"]


def make_env(turb_on, steps_max=2000, config_kw=None):
    ckw = {"steps_max": steps_max}
    if config_kw:
        ckw.update(config_kw)
    env = FixedWingAircraft(GYM_CFG, config_kw=ckw,
                            sim_config_kw={"turbulence": turb_on, "turbulence_intensity": "light"})
    env.seed(0)
    return env


def env_episode(env, rng, turb_on, n_steps, act_scale=1.2, omega_deg=60.0, policy="rand"):
    st = random_state(rng, omega_deg=omega_deg, dots=False)
    st["wind"] = random_wind(rng) if turb_on else [0.0, 0.0, 0.0]
    d2r = np.radians
    target = {"roll": rng.uniform(d2r(-60), d2r(60)), "pitch": rng.uniform(d2r(-25), d2r(25)),
              "Va": rng.uniform(15, 28)}
    L = env.simulator.wind.turbulence_sim_length
    noise = rng.standard_normal((4, L)) if turb_on else None
    obs0 = env.reset(state=dict(st), target=dict(target), turbulence_noise=noise)
    init = np.array([st[k] for k in ENV_STATE_KEYS] + [0.0, 0.0, 0.0] + list(st["wind"]))
    obs, rew, done, term, acts, tgt = [obs0], [], [], [], [], [
        np.array([env.target["roll"], env.target["pitch"], env.target["Va"]])]
    pid = {"dt": 0.01, "va": target["Va"], "phi": target["roll"], "theta": target["pitch"],
           "iv": 0.0, "ir": 0.0, "ip": 0.0}
    for s in range(n_steps):
        if policy == "rand":
            a = rng.uniform(-act_scale, act_scale, size=3).astype(np.float32)
        else:
            a = np.array(pid_action(pid, env.simulator), dtype=np.float64)
        o, r, d, info = env.step(a)
        env._last_info = info
        acts.append(np.asarray(a, dtype=np.float64))
        obs.append(o)
        rew.append(r)
        done.append(d)
        term.append(info.get("termination", ""))
        tgt.append(np.array([env.target["roll"], env.target["pitch"], env.target["Va"]]))
        if policy != "rand":
            pid["phi"], pid["theta"], pid["va"] = info["target"]["roll"], info["target"]["pitch"], info["target"]["Va"]
        if d:
            break
    return dict(init=init, target0=np.array([target["roll"], target["pitch"], target["Va"]]),
                noise=noise if noise is not None else np.zeros((4, 1)), obs=np.array(obs),
                act=np.array(acts), rew=np.array(rew), done=np.array(done), term=np.array(term),
                target=np.array(tgt))


def gen_env_seq():
    out = {}
    rng = np.random.RandomState(99)
    cases = [
        # name, turb, steps_max, n_steps, omega_deg, policy, config_kw
        ("rand_off", False, 2000, 300, 60.0, "rand", None),
        ("rand_on", False, 2000, 300, 60.0, "rand", None),
        ("rand_turb", True, 2000, 300, 60.0, "rand", None),
        ("short_max", False, 120, 200, 60.0, "rand", None),
        ("fail_omega", False, 2000, 300, 700.0, "rand", None),
        ("fail_va", False, 2000, 600, 60.0, "rand", {"simulator": {"states": {5: {"constraint_max": 17.5}}}}),
        ("pid_goal", False, 2000, 400, 20.0, "pid", {"action": {"scale_space": False}}),
        ("pid_goal_done", False, 1500, 1500, 20.0, "pid",
         {"action": {"scale_space": False},
          "target": {"on_success": "done", "success_streak_fraction": 1, "success_streak_req": 100}}),
        ("pid_turb", True, 2000, 500, 20.0, "pid", {"action": {"scale_space": False}}),
    ]
    for name, turb, smax, n, omd, pol, ckw in cases:
        env = make_env(turb, smax, ckw)
        ep = env_episode(env, rng, turb, n, omega_deg=omd, policy=pol)
        for k, v in ep.items():
            out[name + "__" + k] = v
        out[name + "__steps_max"] = np.array(smax)
        out[name + "__turb_on"] = np.array(turb)
        out[name + "__scale_space"] = np.array(ckw is None)
        print("env %s: %d steps, last term=%r, rew sum %.3f" % (name, len(ep["rew"]), ep["term"][-1],
                                                               ep["rew"].sum()))
    np.savez_compressed(os.path.join(OUT, "env_seq.npz"), **out)


def gen_pid_set(n_scen=40):
    """PID replay on a synthetic evaluation set built like evaluate_controller.py:90-108."""
    rng = np.random.RandomState(2021)
    d2r = np.radians
    ckw = {"steps_max": 1500, "action": {"scale_space": False},
           "target": {"on_success": "done", "success_streak_fraction": 1, "success_streak_req": 100,
                      "states": {0: {"bound": 5}, 1: {"bound": 5}, 2: {"bound": 2}}}}
    env = make_env(False, 1500, ckw)
    lengths, rewards, inits, targets, terms = [], [], [], [], []
    for i in range(n_scen):
        st = {"roll": rng.uniform(d2r(-60), d2r(60)), "pitch": rng.uniform(d2r(-25), d2r(25)),
              "yaw": 0.0, "omega_p": 0.0, "omega_q": 0.0, "omega_r": 0.0,
              "position_n": 0.0, "position_e": 0.0, "position_d": -50.0,
              "velocity_u": rng.uniform(15, 23), "velocity_v": 0.0, "velocity_w": 0.0,
              "elevon_right": 0.0, "elevon_left": 0.0, "throttle": 0.0, "wind": [0.0, 0.0, 0.0]}
        tgt = {"roll": rng.uniform(d2r(-60), d2r(60)), "pitch": rng.uniform(d2r(-25), d2r(25)),
               "Va": rng.uniform(15, 28)}
        env.reset(state=dict(st), target=dict(tgt))
        pid = {"dt": 0.01, "va": tgt["Va"], "phi": tgt["roll"], "theta": tgt["pitch"], "iv": 0.0,
               "ir": 0.0, "ip": 0.0}
        rs = []
        while True:
            a = np.array(pid_action(pid, env.simulator))
            o, r, d, info = env.step(a)
            rs.append(r)
            pid["phi"], pid["theta"], pid["va"] = info["target"]["roll"], info["target"]["pitch"], info["target"]["Va"]
            if d:
                break
        lengths.append(len(rs))
        rr = np.zeros(1500)
        rr[:len(rs)] = rs
        rewards.append(rr)
        inits.append([st[k] for k in ENV_STATE_KEYS])
        targets.append([tgt["roll"], tgt["pitch"], tgt["Va"]])
        terms.append(info.get("termination", ""))
    np.savez_compressed(os.path.join(OUT, "env_pid_set.npz"), length=np.array(lengths),
                        reward=np.array(rewards), init=np.array(inits), target=np.array(targets),
                        term=np.array(terms))
    print("pid set: lengths", lengths)


METRIC_KEYS = {"rise_time": ["roll", "pitch", "Va"], "settling_time": ["roll", "pitch", "Va", "all"],
               "overshoot": ["roll", "pitch", "Va"], "total_error": ["roll", "pitch", "Va"],
               "avg_error": ["roll", "pitch", "Va"], "control_variation": ["all"],
               "success": ["roll", "pitch", "Va", "all"], "success_time_frac": ["roll", "pitch", "Va", "all"],
               "end_error": ["roll", "pitch", "Va"]}


def gen_metrics():
    """Episode metrics reported in info on done (fixed_wing.py:1644-1736), with the histories they
    are computed from, for PID / random-action episodes that end by steps_max, success or failure."""
    out = {}
    rng = np.random.RandomState(4242)
    cases = [
        # name, turb, steps_max, policy, omega_deg, act_scale, config_kw
        ("pid300", False, 300, "pid", 20.0, 1.0, {"action": {"scale_space": False}}),
        ("pid_done", False, 1500, "pid", 20.0, 1.0,
         {"action": {"scale_space": False},
          "target": {"on_success": "done", "success_streak_fraction": 0.9, "success_streak_req": 60}}),
        ("rand150", False, 150, "rand", 60.0, 1.2, None),
        ("rand_fail", False, 2000, "rand", 700.0, 1.2, None),
        ("pid_turb", True, 400, "pid", 20.0, 1.0, {"action": {"scale_space": False}}),
        ("rand_short", False, 3, "rand", 60.0, 1.0, None),
    ]
    for name, turb, smax, pol, omd, asc, ckw in cases:
        env = make_env(turb, smax, ckw)
        ep = env_episode(env, rng, turb, smax + 5, act_scale=asc, omega_deg=omd, policy=pol)
        assert ep["done"][-1], name
        info = env._last_info
        p = name + "__"
        for k, v in ep.items():
            out[p + k] = v
        out[p + "steps_max"] = np.array(smax)
        out[p + "turb_on"] = np.array(turb)
        out[p + "scale_space"] = np.array(ckw is None or "action" not in ckw)
        for m, keys in METRIC_KEYS.items():
            out[p + "metric_" + m] = np.array([float(info[m][k]) for k in keys])
        for k in ("roll", "pitch", "Va"):
            out[p + "hist_error_" + k] = np.array(env.history["error"][k], dtype=np.float64)
        for k in ("roll", "pitch", "Va", "all"):
            out[p + "hist_goal_" + k] = np.array(env.history["goal"][k], dtype=np.float64)
        out[p + "hist_command"] = np.array([env.simulator.state[a].history["command"]
                                            for a in ("elevator", "aileron", "throttle")], dtype=np.float64)
        print("metrics %s: %d steps, term=%r, success=%s" % (name, len(ep["rew"]), ep["term"][-1],
                                                             out[p + "metric_success"]))
    np.savez_compressed(os.path.join(OUT, "env_metrics.npz"), **out)


CNN_CFG = os.path.join(REF, "fixed-wing-gym/gym_fixed_wing/examples/models/cnn_controller/fixed_wing_config.json")


def gen_obs_hist():
    """Observation histories (observation.length > 1, fixed_wing.py:1133-1258): the reference's own
    cnn_controller config (5 rows, matrix, relative targets) and the default config with 3 rows,
    step 2, vector shape, with and without normalisation.  Rows older than the episode carry the
    reference's init_noise (np_random.uniform(-1, 1) * dt, one draw per row); the tests check those
    rows up to a row-constant offset."""
    out = {}
    rng = np.random.RandomState(123)
    hist3 = {"observation": {"length": 3, "step": 2, "shape": "vector"}}
    hist3n = {"observation": {"length": 3, "step": 2, "shape": "vector", "normalize": True}}
    cases = [
        # name, config path, config_kw, steps_max, n_steps, omega_deg, policy
        ("cnn_rand", CNN_CFG, None, 2000, 200, 60.0, "rand"),
        ("cnn_fail_p", CNN_CFG, {"simulator": {"states": {6: {"constraint_min": -150, "constraint_max": 150}}}}, 2000,
         600, 60.0, "rand"),
        ("cnn_short", CNN_CFG, None, 40, 60, 60.0, "rand"),
        ("vec3_rand", GYM_CFG, hist3, 2000, 150, 60.0, "rand"),
        ("vec3_norm", GYM_CFG, hist3n, 2000, 150, 60.0, "rand"),
    ]
    for name, path, ckw, smax, n, omd, pol in cases:
        kw = {"steps_max": smax}
        if ckw:
            kw.update(ckw)
        env = FixedWingAircraft(path, config_kw=kw, sim_config_kw={"turbulence": False})
        env.seed(0)
        ep = env_episode(env, rng, False, n, omega_deg=omd, policy=pol)
        for k in ("init", "target0", "obs", "act", "rew", "done", "term"):
            out[name + "__" + k] = ep[k]
        out[name + "__steps_max"] = np.array(smax)
        # the config file itself travels as data (the GPU box has no reference checkout); "" = default
        out[name + "__config_json"] = np.array("" if path == GYM_CFG else json.dumps(json.load(open(path))))
        out[name + "__config_kw"] = np.array(repr(ckw))
        print("obs_hist %s: %d steps, obs %s, last term=%r" % (name, len(ep["rew"]), ep["obs"].shape[1:],
                                                              ep["term"][-1]))
    np.savez_compressed(os.path.join(OUT, "env_obs_hist.npz"), **out)



# ---------------------------------------------------------------------------
# I. solver failure: sol.y[:, -1] committed (pyfly.py:1393-1396)
# ---------------------------------------------------------------------------


class _Budget(Exception):
    pass


def _budget_rk45(budget):
    """scipy's own RK45 that declares a step failure once ``budget`` RHS evaluations are spent.

    Stands in for a TOO_SMALL_STEP failure, which no reference configuration can reach (pyfly
    calls solve_ivp with the default tolerances on a continuous RHS).  Only the step method
    changes: solve_ivp's loop (ivp.py), its sol.y bookkeeping (accepted steps only) and pyfly's
    save of sol.y[:, -1] after the call are the reference's own code.  The budget is checked
    after each evaluation, a constraint raise inside that evaluation taking precedence -- the
    max_nfev rule of fw_sim_config."""
    from scipy.integrate import RK45

    class BudgetRK45(RK45):
        def __init__(self, fun, t0, y0, t_bound, **kw):
            self._spent = 0

            def counted(t, y):
                out = fun(t, y)
                self._spent += 1
                if self._spent >= budget:
                    raise _Budget()
                return out
            try:
                super().__init__(counted, t0, y0, t_bound, **kw)
                self._init_failed = False
            except _Budget:  # f0 or the initial-step probe hit the budget: no step at all
                self._init_failed = True
                self.t, self.y, self.t_old, self.status = t0, np.array(y0, float), None, "running"
                self.h_abs, self.f, self.direction, self.n, self.nfev = 0.0, None, 1.0, len(y0), budget
                self.njev, self.nlu = 0, 0
                self.t_bound = t_bound

        def _step_impl(self):
            if self._init_failed:
                return False, "budget"
            try:
                return super()._step_impl()
            except _Budget:
                return False, "budget"

    return BudgetRK45


def gen_solver_fail():
    rows = {k: [] for k in ["y0", "wind", "cmd_in", "budget", "y1", "success", "term", "nfev", "naccept",
                            "status", "derived1", "der0"]}
    rng = np.random.RandomState(777)
    orig = scipy.integrate.solve_ivp
    budgets = [2, 8, 14, 20, 26, 32, 44]
    for i in range(112):
        budget = budgets[i % len(budgets)]
        sim = pf.PyFly(PYFLY_CFG, PYFLY_PARAM, config_kw={"turbulence": False})
        for n in ["omega_p", "omega_q", "omega_r"]:
            sim.state[n].constraint_min, sim.state[n].constraint_max = np.radians(-720.0), np.radians(720.0)
        sim.seed(4000 + i)
        st = random_state(rng, omega_deg=120.0)
        wind = random_wind(rng) if i % 3 else [0.0, 0.0, 0.0]
        st["wind"] = wind
        sim.reset(state=st)
        cnt = _count_rhs(sim)
        cmd = [rng.uniform(np.radians(-40), np.radians(45)), rng.uniform(np.radians(-40), np.radians(40)),
               rng.uniform(-0.2, 1.2)]
        y0, der0, cmd_in = ode_vector(sim), derived(sim), list(cmd)
        status = {}

        def patched(*a, **k):
            sol = orig(*a, method=_budget_rk45(budget), **k)
            status["s"] = sol.status
            status["na"] = len(sol.t) - 1
            return sol
        scipy.integrate.solve_ivp = patched
        try:
            ok, info = sim.step(cmd)
        finally:
            scipy.integrate.solve_ivp = orig
        rows["y0"].append(y0)
        rows["der0"].append(der0)
        rows["wind"].append(np.array(wind, dtype=np.float64))
        rows["cmd_in"].append(np.array(cmd_in))
        rows["budget"].append(budget)
        rows["y1"].append(ode_vector(sim))
        rows["success"].append(ok)
        rows["term"].append(info.get("termination", ""))
        rows["nfev"].append(cnt["n"])
        rows["naccept"].append(status.get("na", -1))
        rows["status"].append(status.get("s", 99))
        rows["derived1"].append(derived(sim))
    out = {k: np.array(v) for k, v in rows.items()}
    np.savez_compressed(os.path.join(OUT, "pyfly_solver_fail.npz"), **out)
    print("solver failure: %d cases, %d failed integrations (status -1), %d constraint terminations" % (
        len(out["y0"]), int((out["status"] == -1).sum()), int((~out["success"]).sum())))


# ---------------------------------------------------------------------------
# J. energy states (EnergyVariable, pyfly.py:430-450; updated after successful steps :1408-1411)
# ---------------------------------------------------------------------------

ENERGY_NAMES = ["energy_total", "energy_potential", "energy_kinetic_rotational", "energy_kinetic_translational"]


def gen_energy():
    out = {}
    for name, seed, olim, n_steps in [("pid", 0, None, 300), ("rand_fail", 3, 45.0, 1000)]:
        rng = np.random.RandomState(seed)
        sim = pf.PyFly(PYFLY_CFG, PYFLY_PARAM, config_kw={"turbulence": False})
        if olim is not None:
            for n in ["omega_p", "omega_q", "omega_r"]:
                sim.state[n].constraint_min, sim.state[n].constraint_max = np.radians(-olim), np.radians(olim)
        sim.seed(seed)
        st = random_state(rng, omega_deg=60.0 if olim is None else 0.5 * olim, dots=False)
        st["wind"] = random_wind(rng)
        sim.reset(state=st)
        pid = {"dt": sim.dt, "va": 22.0, "phi": 0.2, "theta": 0.0, "iv": 0.0, "ir": 0.0, "ip": 0.0}
        y, der, en, cmds, succ = [ode_vector(sim)], [derived(sim)], [[sim.state[e].value for e in ENERGY_NAMES]], [], []
        for s in range(n_steps):
            if name == "pid":
                cmd = pid_action(pid, sim)
            else:
                cmd = [rng.uniform(np.radians(-30), np.radians(35)), rng.uniform(np.radians(-32.5), np.radians(32.5)),
                       rng.uniform(0, 1)]
            cmds.append(list(cmd))
            ok, info = sim.step(cmd)
            succ.append(ok)
            y.append(ode_vector(sim))
            der.append(derived(sim))
            en.append([sim.state[e].value for e in ENERGY_NAMES])
            if not ok:
                break
        for k, v in dict(y=np.array(y), derived=np.array(der), energy=np.array(en), cmd=np.array(cmds),
                         success=np.array(succ), wind=np.array(st["wind"]), omega_lim_deg=np.array(olim or 180.0)).items():
            out[name + "__" + k] = v
        print("energy %s: %d steps, last success %s" % (name, len(succ), succ[-1]))
    out["names"] = np.array(ENERGY_NAMES)
    np.savez_compressed(os.path.join(OUT, "pyfly_energy.npz"), **out)


# ---------------------------------------------------------------------------
# K. curriculum levels (FixedWingAircraft.set_curriculum_level, fixed_wing.py:334-412)
# ---------------------------------------------------------------------------


def gen_curriculum():
    out = {}
    levels = [0.0, 0.25, 0.5, 0.75, 1.0]
    props = ["init_min", "init_max", "value_min", "value_max", "constraint_min", "constraint_max"]
    env = make_env(False)
    names = [s_["name"] for s_ in env.cfg["simulator"]["states"]]
    out["state_names"] = np.array(names)
    for li, lvl in enumerate(levels):
        env.set_curriculum_level(lvl)
        tab = np.array([[np.nan if getattr(env.simulator.state[n], p, None) is None else
                         float(getattr(env.simulator.state[n], p)) for p in props] for n in names])
        out["L%d__states" % li] = tab
        tp = env._target_props_init["states"]
        out["L%d__targets" % li] = np.array([[np.nan if tp[t].get(k) is None else float(tp[t][k])
                                             for k in ("low", "high", "delta", "bound")]
                                            for t in ("roll", "pitch", "Va")])
        out["L%d__target_rad" % li] = np.array([bool(tp[t].get("convert_to_radians", False))
                                               for t in ("roll", "pitch", "Va")])
        # sampled episodes: initial state and first target of reset() (gym np_random; distribution only)
        env.seed(100 + li)
        init, tgt = [], []
        for _ in range(300):
            env.reset()
            init.append([env.simulator.state[n].value for n in ("roll", "pitch", "Va", "velocity_u")])
            tgt.append([env.target["roll"], env.target["pitch"], env.target["Va"]])
        out["L%d__init" % li] = np.array(init)
        out["L%d__target" % li] = np.array(tgt)
        if lvl in (0.25, 0.5):
            # episodes from the reference's own sampled reset at this level (init state, target and steady
            # wind drawn by reset()), then random actions: replayed on the device at the same level
            rng = np.random.RandomState(300 + li)
            env.seed(200 + li)
            for ep in range(3):
                obs0 = env.reset()
                act_vals = [env.simulator.state[a].value for a in ("elevon_right", "elevon_left", "throttle")]
                wind = np.asarray(env.simulator.wind.steady, dtype=np.float64).reshape(3)
                init_row = np.array([env.simulator.state[k].value for k in ENV_STATE_KEYS] + act_vals + list(wind))
                target0 = np.array([env.target["roll"], env.target["pitch"], env.target["Va"]])
                obs, rew, done, acts = [obs0], [], [], []
                for s in range(300):
                    a = rng.uniform(-1.2, 1.2, size=3).astype(np.float32)
                    o, r, dn, info = env.step(a)
                    acts.append(np.asarray(a, dtype=np.float64))
                    obs.append(o)
                    rew.append(r)
                    done.append(dn)
                    if dn:
                        break
                pre = "L%d__ep%d__" % (li, ep)
                for k, v in dict(init=init_row, target0=target0, obs=np.array(obs), rew=np.array(rew),
                                 done=np.array(done), act=np.array(acts)).items():
                    out[pre + k] = v
                print("curriculum L%g ep%d: %d steps, init roll %.3f pitch %.3f u %.2f, wind %s" % (
                    lvl, ep, len(rew), init_row[0], init_row[1], init_row[9], wind))
    out["levels"] = np.array(levels)
    out["props"] = np.array(props)
    np.savez_compressed(os.path.join(OUT, "env_curriculum.npz"), **out)
    print("curriculum: %d levels, %d simulator states" % (len(levels), len(names)))


# ---------------------------------------------------------------------------
# L. simulator parameter randomisation (FixedWingAircraft.sample_simulator_parameters,
#    fixed_wing.py:748-813)
# ---------------------------------------------------------------------------

RAND_MODELS = {
    # relative gaussian with a clip: negative originals (C_m_alpha, C_l_p, C_m_q) hit the reference's
    # signed-clip quirk (lo > hi -> always original + clip); inertia / wing geometry exercise the
    # frozen gammas / aspect ratio
    "gauss_rel": {"var_type": "relative", "var": 0.1, "distribution": "gaussian", "clip": 0.25,
                  "parameters": [{"name": "C_L_alpha"}, {"name": "mass"}, {"name": "Jy"}, {"name": "Jx"},
                                 {"name": "C_m_alpha", "var": 0.2}, {"name": "b"}, {"name": "S_wing"},
                                 {"name": "e"}, {"name": "C_D_p"}, {"name": "k_motor"}, {"name": "C_l_p"},
                                 {"name": "C_m_q"}, {"name": "C_n_beta"}, {"name": "c"}]},
    "unif_abs": {"var_type": "absolute", "var": 0.05, "distribution": "uniform",
                 "parameters": [{"name": "C_L_0"}, {"name": "C_m_0", "var": 0.01}, {"name": "a_0"},
                                {"name": "M", "var": 5.0}, {"name": "C_Y_beta"}, {"name": "k_T_P", "var": 1e-4}]},
}


def gen_rand_params():
    import copy
    out = {}
    import tempfile
    for name, model in RAND_MODELS.items():
        # the gym config with a "model" block (config_kw cannot add keys, fixed_wing.py:34-48)
        cfg = json.load(open(GYM_CFG))
        cfg["simulator"]["model"] = copy.deepcopy(model)
        path = os.path.join(tempfile.mkdtemp(), "fixed_wing_config.json")
        with open(path, "w") as f:
            json.dump(cfg, f)
        out[name + "__config_json"] = np.array(json.dumps(cfg))
        env = FixedWingAircraft(path, config_kw={"steps_max": 400},
                                sim_config_kw={"turbulence": False, "turbulence_intensity": "light"})
        env.seed(0)
        pnames = sorted(env.simulator.params.keys())
        out[name + "__model_json"] = np.array(json.dumps(model))
        # distribution: 400 resets, the sampled value of every randomised parameter
        env.seed(77)
        draws = []
        for _ in range(400):
            env.reset()
            draws.append([env.simulator.params[p["name"]] for p in model["parameters"]])
        out[name + "__draws"] = np.array(draws)
        # dynamics: episodes from explicit states with the reference's own draw, random actions
        rng = np.random.RandomState(11)
        for ep in range(3):
            res = env_episode(env, rng, False, 400)
            vals = {}
            for p in pnames:
                if p.startswith("__"):
                    continue
                try:
                    vals[p] = float(np.asarray(env.simulator.params[p]).reshape(-1)[0])
                except (TypeError, ValueError):
                    continue
            out["%s__ep%d__param_names" % (name, ep)] = np.array(sorted(vals))
            out["%s__ep%d__param_values" % (name, ep)] = np.array([vals[p] for p in sorted(vals)])
            for k, v in res.items():
                out["%s__ep%d__%s" % (name, ep, k)] = v
        print("rand params %s: %d draws, episode lengths %s" % (
            name, len(draws), [len(out["%s__ep%d__rew" % (name, e)]) for e in range(3)]))
    np.savez_compressed(os.path.join(OUT, "env_rand_params.npz"), **out)


# ---------------------------------------------------------------------------
# M. FixedWingAircraft.history (fixed_wing.py:455-467, 491-585)
# ---------------------------------------------------------------------------


def gen_history():
    out = {}
    for name, policy, omega, ckw in [("pid", "pid", 60.0, {"action": {"scale_space": False}}),
                                     ("rand_fail", "rand", 700.0, None)]:
        env = make_env(False, steps_max=300, config_kw=ckw)
        for seed in range(5, 200):  # rand_fail: the first seed whose episode ends in a constraint violation
            rng = np.random.RandomState(seed)
            res = env_episode(env, rng, False, 300, policy=policy, omega_deg=omega)
            if name != "rand_fail" or (str(res["term"][-1]) not in ("steps", "") and len(res["rew"]) >= 20):
                break
        h = env.history
        for k, v in res.items():
            out[name + "__" + k] = v
        out[name + "__h_action"] = np.array(h["action"], dtype=np.float64)
        out[name + "__h_reward"] = np.array(h["reward"], dtype=np.float64)
        out[name + "__h_observation"] = np.array(h["observation"], dtype=np.float64)
        for t in ("roll", "pitch", "Va"):
            out[name + "__h_target_" + t] = np.array(h["target"][t], dtype=np.float64)
            out[name + "__h_error_" + t] = np.array(h["error"][t], dtype=np.float64)
        for g in h.get("goal", {}):
            out[name + "__h_goal_" + g] = np.array(h["goal"][g], dtype=bool)
        out[name + "__goal_keys"] = np.array(sorted(h.get("goal", {})))
        print("history %s: %d actions, %d rewards, last term %r" % (name, len(h["action"]), len(h["reward"]),
                                                                   str(res["term"][-1])))
    np.savez_compressed(os.path.join(OUT, "env_history.npz"), **out)

if __name__ == "__main__":
    which = sys.argv[1:] or ["single", "traj", "envelope", "dryden", "dryden_wrap", "env", "pidset", "metrics", "obshist",
                             "solverfail", "energy", "curriculum", "randparams", "history"]
    if "envelope" in which and "traj" not in which:
        gen_envelope()
    if "obshist" in which:
        gen_obs_hist()
    if "single" in which:
        gen_single_step()
    if "traj" in which:
        gen_traj()
        if "envelope" in which:
            gen_envelope()
    if "dryden" in which:
        gen_dryden()
    if "dryden_wrap" in which:
        gen_dryden_wrap()
    if "env" in which:
        gen_env_seq()
    if "pidset" in which:
        gen_pid_set()
    if "metrics" in which:
        gen_metrics()
    if "solverfail" in which:
        gen_solver_fail()
    if "energy" in which:
        gen_energy()
    if "curriculum" in which:
        gen_curriculum()
    if "randparams" in which:
        gen_rand_params()
    if "history" in which:
        gen_history()
