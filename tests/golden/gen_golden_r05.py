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
  env_intwin.npz     FixedWingAircraft episodes with integration_window 10: "integrator" target observations
                     (roll, pitch) and "int_error" reward factors (roll, Va), fixed_wing.py:1001-1012, 1160-1182,
                     including episodes that end in a constraint violation (the failure-step observation)

Usage:  python tests/golden/gen_golden_r05.py
"""
import json
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


INTWIN_KW = {"integration_window": 10,
             "observation": {"states": {6: {"value": "integrator"}, 7: {"value": "integrator"}}},
             "reward": {"factors": {0: {"type": "int_error"}, 2: {"type": "int_error"}}}}


def gen_env_intwin():
    import copy
    out = {}
    rng = np.random.RandomState(508)
    for name, pol, ckw, omega, scale in [("rand", "rand", None, 20.0, 1.2), ("pid", "pid", {"action": {"scale_space": False}}, 20.0, 1.2),
                                         ("rand_hot", "rand", None, 200.0, 3.0), ("rand_hot2", "rand", None, 250.0, 3.0)]:
        kw = copy.deepcopy(INTWIN_KW)
        if ckw:
            kw.update(ckw)
        env = G.make_env(False, 300, kw)
        assert env.integration_window == 10
        ep = G.env_episode(env, rng, False, 300, act_scale=scale, omega_deg=omega, policy=pol)
        for k, v in ep.items():
            out[name + "__" + k] = v
        out[name + "__scale_space"] = np.array(ckw is None)
        print("env intwin %s: %d steps, last term=%r" % (name, len(ep["rew"]), ep["term"][-1]))
    for name, steps_before in [("fail_early", 0), ("fail_late", 12)]:
        ep = _fail_episode(G.make_env(False, 300, copy.deepcopy(INTWIN_KW)), rng, steps_before)
        for k, v in ep.items():
            out[name + "__" + k] = v
        out[name + "__scale_space"] = np.array(True)
        print("env intwin %s: %d steps, last term=%r" % (name, len(ep["rew"]), ep["term"][-1]))
    # episodes that end in a constraint violation (the fail_va / fail_omega cases of gen_golden.py): the failed
    # step's observation and reward with the window; the extra config (steps_max too) is stored with the episode
    rng = np.random.RandomState(509)
    for name, extra, omega in [("fail_va", {"simulator": {"states": {5: {"constraint_max": 17.5}}}}, 60.0)]:
        kw = copy.deepcopy(INTWIN_KW)
        kw.update(copy.deepcopy(extra))
        env = G.make_env(False, 2000, kw)
        ep = G.env_episode(env, rng, False, 600, omega_deg=omega, policy="rand")
        for k, v in ep.items():
            out[name + "__" + k] = v
        out[name + "__scale_space"] = np.array(True)
        out[name + "__extra_kw"] = np.array(json.dumps(dict(extra, steps_max=2000)))
        print("env intwin %s: %d steps, last term=%r" % (name, len(ep["rew"]), ep["term"][-1]))
    np.savez_compressed(os.path.join(OUT, "env_intwin.npz"), **out)


def _fail_episode(env, rng, calm):
    """An episode that ends in the Va <= 70 constraint (fixed_wing_config.json): start at 66-69 m/s nose down,
    `calm` gentle steps, then full throttle -- the failed step's observation is the one to pin."""
    st = G.random_state(rng, omega_deg=10.0, dots=False)
    st["velocity_u"], st["velocity_v"], st["velocity_w"] = rng.uniform(66, 69), 0.0, 0.0
    st["pitch"] = -0.5
    st["wind"] = [0.0, 0.0, 0.0]
    target = {"roll": 0.1, "pitch": -0.2, "Va": 25.0}
    obs0 = env.reset(state=dict(st), target=dict(target))
    init = np.array([st[k] for k in G.ENV_STATE_KEYS] + [0.0, 0.0, 0.0] + list(st["wind"]))
    obs, rew, done, term, acts, tgt = [obs0], [], [], [], [], [np.array([env.target["roll"], env.target["pitch"],
                                                                          env.target["Va"]])]
    for s in range(300):
        a = rng.uniform(-0.1, 0.1, 3) if s < calm else np.array([-1.0, 0.0, 1.0])
        o, r, d, info = env.step(a)
        acts.append(np.asarray(a, dtype=np.float64))
        obs.append(o)
        rew.append(r)
        done.append(d)
        term.append(info.get("termination", ""))
        tgt.append(np.array([env.target["roll"], env.target["pitch"], env.target["Va"]]))
        if d:
            break
    return dict(init=init, target0=np.array([target["roll"], target["pitch"], target["Va"]]), noise=np.zeros((4, 1)),
                obs=np.array(obs), act=np.array(acts), rew=np.array(rew), done=np.array(done), term=np.array(term),
                target=np.array(tgt))


def gen_env_intwin_hist():
    """integration_window with an observation history (length 3, step 2, vector): the integrator entries of
    the lagged rows (fixed_wing.py:1165-1180, slice [-W-i:-i]), including an episode that ends in a
    constraint violation (the failed step's lagged rows read the history one entry short)."""
    import copy
    out = {}
    rng = np.random.RandomState(511)
    hist = {"observation": {"length": 3, "step": 2, "shape": "vector"}}
    for name, extra, smax, n, omega, scale in [
            ("rand", {}, 300, 300, 20.0, 1.2),
            ("rand_hot", {}, 300, 300, 200.0, 3.0),
            ("fail_va", {"simulator": {"states": {5: {"constraint_max": 17.5}}}}, 2000, 600, 60.0, 1.2)]:
        kw = copy.deepcopy(INTWIN_KW)
        kw["observation"].update(copy.deepcopy(hist["observation"]))
        kw.update(copy.deepcopy(extra))
        env = G.make_env(False, smax, kw)
        ep = G.env_episode(env, rng, False, n, act_scale=scale, omega_deg=omega, policy="rand")
        for k, v in ep.items():
            out[name + "__" + k] = v
        out[name + "__scale_space"] = np.array(True)
        out[name + "__extra_kw"] = np.array(json.dumps(dict(copy.deepcopy(extra), steps_max=smax, **hist)))
        print("env intwin hist %s: %d steps, last term=%r" % (name, len(ep["rew"]), ep["term"][-1]))
    np.savez_compressed(os.path.join(OUT, "env_intwin_hist.npz"), **out)


# observation.normalize with entries that give no mean / var: the reference derives them from the bounds
# (fixed_wing.py:142-161: mean = high - low, var = (high - low) / 16, or 0 / 1 for unbounded entries)
OBSNORM_KW = {"observation": {"normalize": True, "states": {
    0: {"mean": None, "var": None}, 1: {"mean": None}, 2: {"var": None}, 3: {"mean": None, "var": None},
    6: {"mean": None, "var": None}, 8: {"var": None}, 9: {"mean": None, "var": None}}}}


def gen_env_obsnorm():
    import copy
    out = {}
    rng = np.random.RandomState(510)
    for name, pol, ckw in [("rand", "rand", None), ("pid", "pid", {"action": {"scale_space": False}})]:
        kw = copy.deepcopy(OBSNORM_KW)
        if ckw:
            kw.update(ckw)
        env = G.make_env(False, 300, kw)
        ep = G.env_episode(env, rng, False, 300, omega_deg=20.0, policy=pol)
        for k, v in ep.items():
            out[name + "__" + k] = v
        out[name + "__scale_space"] = np.array(ckw is None)
        out[name + "__obs_mean"] = np.array([float(o["mean"]) for o in env.cfg["observation"]["states"]])
        out[name + "__obs_var"] = np.array([float(o["var"]) for o in env.cfg["observation"]["states"]])
        out[name + "__obs_space"] = np.stack([env.observation_space.low, env.observation_space.high])
        out[name + "__act_space"] = np.stack([env.action_space.low, env.action_space.high])
        print("env obsnorm %s: %d steps, last term=%r" % (name, len(ep["rew"]), ep["term"][-1]))
    out["config_kw"] = np.array(json.dumps(OBSNORM_KW))
    np.savez_compressed(os.path.join(OUT, "env_obsnorm.npz"), **out)


if __name__ == "__main__":
    which = sys.argv[1:] or ["dryden", "pyfly", "env", "potential", "intwin", "obsnorm", "intwin_hist"]
    if "dryden" in which:
        gen_dryden_short()
    if "pyfly" in which:
        gen_pyfly_short()
    if "env" in which:
        gen_env_short()
    if "potential" in which:
        gen_env_potential()
    if "intwin" in which:
        gen_env_intwin()
    if "obsnorm" in which:
        gen_env_obsnorm()
    if "intwin_hist" in which:
        gen_env_intwin_hist()
