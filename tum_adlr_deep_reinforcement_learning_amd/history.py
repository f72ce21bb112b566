"""Host-side episode history of FixedWingAircraft (fixed_wing.py:414-628 ``self.history``).

The device path keeps no per-step history (streaming metrics replace it); code written
against the reference that reads ``env.history`` / ``get_attr("history")`` (plotting, evaluation
scripts) gets it from this recorder, which the single-env facade always runs and the VecEnv runs
with ``record_history=True``.  Layout and update rules follow the reference:

  reset:  {"action": [], "reward": [], "observation": [obs], "target": {k: [v]},
           "error": {k: [err]}, "goal": {state: [status], "all": [...]}}   (goal only if enabled)
  step:   "action" always; on a successful simulator step (done by steps / success included):
          goal status against the targets before the update, then the updated targets and their
          errors, then observation and reward (fixed_wing.py:491-585); nothing else on a failed step.
"""
import numpy as np

from . import config as C

_TNAMES = ("roll", "pitch", "Va")


class EpisodeHistory:
    def __init__(self, spec):
        e = spec.struct()
        self.wrap = [bool(spec.sim.vars[n].wrap) for n in _TNAMES]
        self.bound = [None if np.isnan(e.target_bound[k]) else float(e.target_bound[k]) for k in range(3)]
        self.goal_enabled = int(spec.cfg["target"].get("success_streak_req", 0)) > 0
        self.history = None

    def _error(self, k, tgt, val):
        """_get_error / _get_angle_dist (fixed_wing.py:1318-1344)."""
        if self.wrap[k]:
            d = (val - tgt + np.pi) % (2 * np.pi) - np.pi
            return d + 2 * np.pi if d < -np.pi else d
        return tgt - val

    def _goal(self, tgt, vals):
        """_get_goal_status (fixed_wing.py:1346-1361)."""
        st = {}
        for k, name in enumerate(_TNAMES):
            if self.bound[k] is not None:
                st[name] = bool(np.abs(self._error(k, tgt[k], vals[k])) <= self.bound[k])
        st["all"] = all(st.values())
        return st

    def reset(self, obs, tgt, vals):
        """tgt: targets (roll, pitch, Va); vals: current roll, pitch, Va."""
        self.history = {"action": [], "reward": [], "observation": [np.array(obs)],
                        "target": {n: [float(tgt[k])] for k, n in enumerate(_TNAMES)},
                        "error": {n: [float(self._error(k, tgt[k], vals[k]))] for k, n in enumerate(_TNAMES)}}
        if self.goal_enabled:
            self.history["goal"] = {s: [v] for s, v in self._goal(tgt, vals).items()}

    def step(self, action, success, obs, reward, tgt_before, tgt_after, vals):
        h = self.history
        h["action"].append(np.array(action))
        if not success:
            return
        if self.goal_enabled:
            for s, v in self._goal(tgt_before, vals).items():
                h["goal"][s].append(v)
        for k, n in enumerate(_TNAMES):
            h["target"][n].append(float(tgt_after[k]))
            h["error"][n].append(float(self._error(k, tgt_after[k], vals[k])))
        h["observation"].append(np.array(obs))
        h["reward"].append(float(reward))


def step_succeeded(term):
    """The simulator step of a FixedWingAircraft.step succeeded (it may still be done by steps / success)."""
    term = int(term)
    return term == C.FW_TERM_NONE or term in (C.FW_TERM_STEPS, C.FW_TERM_SUCCESS)
