"""Round-5 golden fixtures (test infrastructure only): the reference's Dryden turbulence for SHORT chunks.

Runs the reference itself (pyfly / gym_fixed_wing from /root/reference through gen_golden.py's offline
gym stand-in) and stores inputs + outputs as ``.npz`` next to this script.  Only data leaves this script.

Below ~45 steps per turbulence chunk the Dryden shaping filters, as pyfly wires them (the positional
(sim_length, dt, b) quirk, pyfly.py:781-783), keep state from one sample to the next: the 2-tap FIR that
holds for the shipped configurations (L = 300 / 2000; dryden.npz) no longer applies, and at the start of
every chunk lsim propagates the previous chunk's last state over t[0] = chunk * L * L seconds.

Fixtures:
  dryden_short.npz   DrydenGustModel(L, 0.01, 2.1) outputs over 5 chunks for L in (3, 8, 20, 40) x
                     (light, severe), and a turbulence_noise shorter than the span (wrapped, L = 20)
  pyfly_short_turb.npz  PyFly trajectories with turbulence_sim_length 8 / 20 / 40 over several chunks
                     (injected noise; PID and random commands)
  env_short_turb.npz FixedWingAircraft episodes with steps_max 40 (turbulence chunk = steps_max = 40)
  env_potential.npz  FixedWingAircraft episodes with reward.form "potential" (fixed_wing.py:1080-1108: the
                     shaping terms enter as the change since the previous step), random and PID actions,
                     turbulence off and light

Usage:  python tests/golden/gen_golden_r05.py
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gen_golden as G  # noqa: E402  (installs the gym stand-in and imports the reference)

OUT = G.OUT


def gen_dryden_short():
    out = {}
    rng = np.random.RandomState(505)
    for L in (3, 8, 20, 40):
        for inten in ("light", "severe"):
            dm = G.DrydenGustModel(L, 0.01, 2.1, intensity=inten)
            noise = rng.standard_normal((4, 5 * L))
            dm.reset(noise)
            for _ in range(5):
                dm.simulate(L)
            key = "L%d_%s__" % (L, inten)
            out[key + "noise"] = noise
            out[key + "vel_lin"] = dm.vel_lin
            out[key + "vel_ang"] = dm.vel_ang
    # a noise sequence shorter than the span: simulate() wraps it (dryden.py:209-236)
    L = 20
    dm = G.DrydenGustModel(L, 0.01, 2.1, intensity="moderate")
    noise = rng.standard_normal((4, 37))
    dm.reset(noise)
    for _ in range(4):
        dm.simulate(L)
    out["wrap__noise"] = noise
    out["wrap__L"] = np.array(L)
    out["wrap__vel_lin"] = dm.vel_lin
    out["wrap__vel_ang"] = dm.vel_ang
    np.savez_compressed(os.path.join(OUT, "dryden_short.npz"), **out)
    print("dryden_short done")


def gen_pyfly_short():
    out = {}
    for name, ctrl, seed, n_steps, L in [("pid_L20", "pid", 51, 200, 20), ("rand_L8", "rand", 52, 120, 8),
                                         ("pid_L40", "pid", 53, 200, 40)]:
        tr = G.run_traj(True, ctrl, seed, n_steps=n_steps, L=L)
        for k, v in tr.items():
            out[name + "__" + k] = v
        print("pyfly %s: %d steps, term=%r" % (name, len(tr["nfev"]), str(tr["term"])))
    np.savez_compressed(os.path.join(OUT, "pyfly_short_turb.npz"), **out)


def gen_env_short():
    out = {}
    rng = np.random.RandomState(506)
    for name, n, pol, ckw in [("rand_40", 40, "rand", None), ("pid_40", 40, "pid", {"action": {"scale_space": False}})]:
        env = G.make_env(True, 40, ckw)
        ep = G.env_episode(env, rng, True, n, omega_deg=20.0, policy=pol)
        for k, v in ep.items():
            out[name + "__" + k] = v
        out[name + "__steps_max"] = np.array(40)
        out[name + "__scale_space"] = np.array(ckw is None)
        print("env %s: %d steps, last term=%r" % (name, len(ep["rew"]), ep["term"][-1]))
    np.savez_compressed(os.path.join(OUT, "env_short_turb.npz"), **out)


def gen_env_potential():
    out = {}
    rng = np.random.RandomState(507)
    for name, turb, pol, ckw in [("rand_off", False, "rand", None), ("pid_off", False, "pid", {"action": {"scale_space": False}}),
                                 ("rand_light", True, "rand", None)]:
        kw = {"reward": {"form": "potential"}}
        if ckw:
            kw.update(ckw)
        env = G.make_env(turb, 300, kw)
        assert env.cfg["reward"]["form"] == "potential"
        ep = G.env_episode(env, rng, turb, 300, omega_deg=20.0, policy=pol)
        for k, v in ep.items():
            out[name + "__" + k] = v
        out[name + "__turb"] = np.array(turb)
        out[name + "__scale_space"] = np.array(ckw is None)
        print("env potential %s: %d steps, last term=%r" % (name, len(ep["rew"]), ep["term"][-1]))
    np.savez_compressed(os.path.join(OUT, "env_potential.npz"), **out)


if __name__ == "__main__":
    which = sys.argv[1:] or ["dryden", "pyfly", "env", "potential"]
    if "dryden" in which:
        gen_dryden_short()
    if "pyfly" in which:
        gen_pyfly_short()
    if "env" in which:
        gen_env_short()
    if "potential" in which:
        gen_env_potential()
