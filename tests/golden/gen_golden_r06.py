"""Round-6 golden fixtures (test infrastructure only): the reference's env features whose episodes depend on
the env's own np_random draws -- replayed on the device through fw_set_env_draws.

Runs the reference itself (gym_fixed_wing from /root/reference through gen_golden.py's offline gym
stand-in) and stores inputs + outputs as ``.npz`` next to this script.  Only data leaves this script.

After ``env.seed``, the env's ``np_random`` is replaced by a recorder whose ``uniform(low, high)`` draws
``u = random_sample()`` from the same seeded RandomState, appends u to a tape and returns
``low + (high - low) * u`` (numpy's uniform, computed the same way); the default config's zero observation
noise N(0, 0) is drawn from the same stream (it adds exactly 0); any other method raises, so a fixture can
only contain draws the tape covers.  The tape is stored with the episode: the device consumes
it in the reference's draw order (include/fwsim.h fw_set_env_draws).

Fixtures (env_r06.npz), per case the reference config JSON (config_kw cannot add keys, fixed_wing.py:34-48)
and episodes reset with an explicit state and SAMPLED targets:
  linear     roll / pitch targets of class linear (fixed_wing.py:698-706, 1433-1435), Va compensate
             following the linear pitch target (:1381-1384), random actions
  linear_fix the same config with an explicit roll target at reset: a given target flies as "constant"
             (:444-448), the others stay linear
  sinus      roll / pitch targets of class sinusoidal (:708-722, 1438-1448), Va compensate on the pitch
             sinusoid's bias (:1385-1386)
  resample   target.resample_every 60 (:570-574) + reward.randomize_scaling on two factors (:473-479) --
             the two features round 5 pinned structurally only
  success    on_success "new" (:551-552, 566-572) with reward classes success (value and "timesteps"), step
             and goal (per_state, all) (:1020-1048), a PID controller that reaches its goal streak: the
             success reward fires on the first success of the env's lifetime only (goal_achieved, :81, 546-547)

env_streak.npz: success_streak_req 200 and 300 (fixed_wing.py:540-547 has no limit; rounds 1-5 stopped at 128),
on_success "done", PID episodes from explicit states and targets (no np_random draws involved)

Usage:  python tests/golden/gen_golden_r06.py
"""
import copy
import json
import os
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gen_golden as G  # noqa: E402  (installs the gym stand-in and imports the reference)

OUT = G.OUT


class TapeRNG:
    """np_random stand-in: uniform() only, every underlying random_sample() recorded."""

    def __init__(self, rs):
        self.rs = rs
        self.tape = []

    def uniform(self, low=0.0, high=1.0, size=None):
        assert size is None
        u = float(self.rs.random_sample())
        self.tape.append(u)
        return low + (high - low) * u

    def normal(self, loc=0.0, scale=1.0, size=None):
        # the default config's observation noise N(0, 0) (fixed_wing.py:1241-1247): drawn from the same stream
        # (it moves the state the later uniform draws come from) but adds exactly 0, which the device does not
        # draw; a non-zero noise would not be on the tape
        assert size is None and loc == 0 and scale == 0
        return self.rs.normal(loc, scale)

    def choice(self, a, size=None, replace=True, p=None):
        # numpy RandomState.choice with p: cdf = p.cumsum() / its last entry, one random_sample(), searchsorted
        # right (mtrand.pyx); without p it draws an integer (randint), which a tape of doubles cannot hold
        assert size is None and p is not None
        cdf = np.cumsum(np.asarray(p, dtype=np.float64))
        cdf /= cdf[-1]
        u = float(self.rs.random_sample())
        self.tape.append(u)
        return a[int(cdf.searchsorted(u, side="right"))]

    def __getattr__(self, name):
        raise AttributeError("TapeRNG: np_random.%s is not on the tape" % name)


def _cfg(mod):
    cfg = json.load(open(G.GYM_CFG))
    mod(cfg)
    path = os.path.join(tempfile.mkdtemp(), "fixed_wing_config.json")
    with open(path, "w") as f:
        json.dump(cfg, f)
    return cfg, path


def _linear(cfg):
    for i, (lo, hi) in ((0, (2, 8)), (1, (1, 4))):
        cfg["target"]["states"][i].update({"class": "linear", "slope_low": lo, "slope_high": hi})


def _sinus(cfg):
    cfg["target"]["states"][0].update({"class": "sinusoidal", "amplitude_low": 5, "amplitude_high": 20,
                                       "period_low": 150, "period_high": 300})
    cfg["target"]["states"][1].update({"class": "sinusoidal", "amplitude_low": 2, "amplitude_high": 8})


def _resample(cfg):
    cfg["target"]["resample_every"] = 60
    cfg["reward"]["randomize_scaling"] = True
    cfg["reward"]["factors"][0]["scaling"] = [2.0, 4.5]
    cfg["reward"]["factors"][2]["scaling"] = [15.0, 35.0]


def _success(cfg):
    cfg["target"]["on_success"] = "new"
    f = cfg["reward"]["factors"]
    f.append({"name": "succ", "class": "success", "value": 5.0, "function_class": "linear", "scaling": 1.0,
              "shaping": False, "sign": 1})
    f.append({"name": "succ_t", "class": "success", "value": "timesteps", "function_class": "linear",
              "scaling": 100.0, "shaping": False, "sign": 1})
    f.append({"name": "step", "class": "step", "value": 0.01, "function_class": "linear", "scaling": 1.0,
              "shaping": False, "sign": -1})
    f.append({"name": "goal_ps", "class": "goal", "type": "per_state", "value": 0.3, "function_class": "linear",
              "scaling": 1.0, "shaping": False, "sign": 1})
    f.append({"name": "goal_all", "class": "goal", "type": "all", "value": 0.2, "function_class": "linear",
              "scaling": 1.0, "shaping": True, "sign": 1})
    cfg["action"]["scale_space"] = False  # the PID commands the actuators directly


def _simattr(cfg):
    # "simulator" attributes PyFly never reads (sample_simulator_parameters, fixed_wing.py:802-813): drawn at
    # every reset before sample_target, set on the simulator, no effect on the flight; linear targets so the
    # tape's order matters
    _linear(cfg)
    cfg["simulator"]["inert_gain"] = {"low": 0.5, "high": 2.0}
    cfg["simulator"]["inert_mode"] = {"values": [0, 1, 2], "probabilities": [0.2, 0.5, 0.3]}


def _attang(cfg):
    # target class attitude_angular (fixed_wing.py:671-675, 741-746, 1455-1460, 1558-1642): omega_p / q / r targets
    # low-pass filtered from the roll / pitch errors; observed (relative and absolute), rewarded (an error factor),
    # and a per_state goal reward whose value is divided by len(self.target) = 6; no bound on them (the goal
    # status stays roll / pitch / Va) and no metrics (get_metric would cover every target)
    for name in ("omega_p", "omega_q", "omega_r"):
        cfg["target"]["states"].append({"name": name, "class": "attitude_angular"})
    cfg["target"]["states"][-1]["max_vel"] = 2.5
    cfg["metrics"] = []
    obs = cfg["observation"]["states"]
    obs.append({"name": "omega_p", "type": "target", "value": "relative"})
    obs.append({"name": "omega_q", "type": "target", "value": "relative"})
    obs.append({"name": "omega_r", "type": "target", "value": "absolute"})
    cfg["reward"]["factors"].append({"name": "omega_q", "class": "state", "type": "error", "function_class": "linear",
                                     "scaling": 2.0, "max": 0.5, "shaping": False, "sign": -1})
    cfg["reward"]["factors"].append({"name": "goal_ps", "class": "goal", "type": "per_state", "value": 0.3,
                                     "function_class": "linear", "scaling": 1.0, "shaping": False, "sign": 1})


CASES_B = {
    # round 6, second batch (env_r06b.npz)
    "simattr": (_simattr, "rand", 400, 3, 300, None),
    "attang": (_attang, "rand", 400, 3, 300, None),
}

CASES = {
    # name -> (config modifier, policy, steps_max, episodes, steps per episode, explicit targets at reset)
    "linear": (_linear, "rand", 400, 3, 300, None),
    "linear_fix": (_linear, "rand", 400, 2, 200, {"roll": 0.3}),
    "sinus": (_sinus, "rand", 400, 3, 300, None),
    "resample": (_resample, "rand", 400, 3, 300, None),
    "success": (_success, "pid", 1500, 2, 1400, None),
}


def episode(env, rng, pol, n_steps, target=None):
    st = G.random_state(rng, omega_deg=20.0, dots=False)
    st["wind"] = [0.0, 0.0, 0.0]
    tape = env.np_random
    n0 = len(tape.tape)
    obs0 = env.reset(state=dict(st), target=dict(target) if target else None)
    init = np.array([st[k] for k in G.ENV_STATE_KEYS] + [0.0, 0.0, 0.0] + list(st["wind"]))
    tg = lambda: np.array([env.target["roll"], env.target["pitch"], env.target["Va"]])  # noqa: E731
    ang = "omega_p" in env.target
    tga = lambda: np.array([float(env.target[k]) for k in ("omega_p", "omega_q", "omega_r")])  # noqa: E731
    obs, rew, done, term, acts, tgt = [obs0], [], [], [], [], [tg()]
    tang = [tga()] if ang else []
    pid = {"dt": 0.01, "va": env.target["Va"], "phi": env.target["roll"], "theta": env.target["pitch"],
           "iv": 0.0, "ir": 0.0, "ip": 0.0}
    for _ in range(n_steps):
        if pol == "rand":
            a = rng.uniform(-1.2, 1.2, size=3).astype(np.float32)
        else:
            a = np.array(G.pid_action(pid, env.simulator), dtype=np.float64)
        o, r, d, info = env.step(a)
        acts.append(np.asarray(a, dtype=np.float64))
        obs.append(o)
        rew.append(r)
        done.append(d)
        term.append(info.get("termination", ""))
        tgt.append(tg())
        if ang:
            tang.append(tga())
        pid["phi"], pid["theta"], pid["va"] = info["target"]["roll"], info["target"]["pitch"], info["target"]["Va"]
        if d:
            break
    extra = {"target_ang": np.array(tang)} if ang else {}
    return dict(init=init, tape=np.array(tape.tape[n0:]), obs=np.array(obs), act=np.array(acts), rew=np.array(rew),
                done=np.array(done), term=np.array(term), target=np.array(tgt), **extra,
                target0_given=np.array([np.nan if not target or k not in target else target[k]
                                        for k in ("roll", "pitch", "Va")]))


def gen_env_r06(cases=CASES, fname="env_r06.npz", seed=606):
    out = {}
    rng = np.random.RandomState(seed)
    for name, (mod, pol, smax, eps, n, target) in cases.items():
        cfg, path = _cfg(mod)
        out[name + "__config_json"] = np.array(json.dumps(cfg))
        out[name + "__steps_max"] = np.array(smax)
        env = G.FixedWingAircraft(path, config_kw={"steps_max": smax},
                                  sim_config_kw={"turbulence": False, "turbulence_intensity": "light"})
        env.seed(60 + len(out))
        env.np_random = TapeRNG(env.np_random)
        for ep in range(eps):
            res = episode(env, rng, pol, n, target)
            for k, v in res.items():
                out["%s__ep%d__%s" % (name, ep, k)] = v
            print("r06 %s ep%d: %d steps, %d draws, last term=%r, rew sum %.3f" % (
                name, ep, len(res["rew"]), len(res["tape"]), res["term"][-1], res["rew"].sum()))
        out[name + "__episodes"] = np.array(eps)
    np.savez_compressed(os.path.join(OUT, fname), **out)


STREAK_CASES = {
    # name -> success_streak_req: the goal history beyond rounds 1-5's 128 entries (byte counts up to 255, 16-bit
    # counts above), on_success "done", PID episodes with explicit targets (gen_golden.env_episode)
    "streak200": 200,
    "streak300": 300,
}


def gen_env_streak():
    out = {}
    rng = np.random.RandomState(607)
    for name, req in STREAK_CASES.items():
        ckw = {"action": {"scale_space": False},
               "target": {"on_success": "done", "success_streak_fraction": 0.95, "success_streak_req": req}}
        env = G.make_env(False, 1500, ckw)
        for ep in range(3):
            res = G.env_episode(env, rng, False, 1500, omega_deg=20.0, policy="pid")
            for k, v in res.items():
                out["%s__ep%d__%s" % (name, ep, k)] = v
            print("streak %s ep%d: %d steps, last term=%r" % (name, ep, len(res["rew"]), res["term"][-1]))
        out[name + "__req"] = np.array(req)
    np.savez_compressed(os.path.join(OUT, "env_streak.npz"), **out)


if __name__ == "__main__":
    which = sys.argv[1:] or ["r06", "streak", "r06b"]
    if "r06" in which:
        gen_env_r06()
    if "streak" in which:
        gen_env_streak()
    if "r06b" in which:
        gen_env_r06(CASES_B, "env_r06b.npz", 616)
