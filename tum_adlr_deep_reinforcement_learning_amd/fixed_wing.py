"""FixedWingAircraft-compatible single-env facade (gym API, fixed_wing.py:13-628).

One aircraft on the GPU, stepped with ``auto_reset=False`` so ``step`` after
``done`` behaves like the reference (the caller resets).  ``info`` carries
``termination`` ("steps", "success" or the violated variable) and ``target``
like fixed_wing.py:519-628, plus the episode metrics of ``cfg["metrics"]``
(fixed_wing.py:1644-1736) on done.
"""
import os

import numpy as np
import torch

from . import config as C
from .engine import Engine
from .history import EpisodeHistory, step_succeeded
from .pyfly import SimulatorView
from .spaces import Box
from .vec_env import metric_info, termination_name


class FixedWingAircraft:
    metadata = {"render.modes": []}

    def __init__(self, config_path=None, sim_config_path=None, sim_parameter_path=None, config_kw=None,
                 sim_config_kw=None, device=None, precision="float64"):
        self.spec = C.EnvSpec(config_path, config_kw, sim_config_path, sim_parameter_path, sim_config_kw)
        self.cfg = self.spec.cfg
        self.observation_space = Box(self.spec.obs_low, self.spec.obs_high, dtype=np.float32)
        self.action_space = Box(self.spec.action_space_low, self.spec.action_space_high, dtype=np.float32)
        self.engine = Engine(self.spec.sim, self.spec, 1, device=device, precision=precision)
        self.simulator = SimulatorView(self.engine, 0)
        self.steps_max = self.spec.steps_max
        self.training = True
        self._act = torch.zeros(1, 3, dtype=self.engine.dtype, device=self.engine.device)
        self._hist = EpisodeHistory(self.spec)
        self.seed(None)

    @property
    def history(self):
        """FixedWingAircraft.history (fixed_wing.py:455-467, 491-585), recorded on the host."""
        return self._hist.history

    def _targets_vals(self):
        t = self.engine.get_block(C.FW_BLK_TARGET)[:, 0].double().cpu().numpy()
        d = self.engine.get_block(C.FW_BLK_DERIVED)[:, 0].double().cpu().numpy()
        return t, d[[0, 1, 3]]

    def seed(self, seed=None):
        """FixedWingAircraft.seed (fixed_wing.py:324-332) -> Philox stream (seed, 0).

        ``None`` draws a fresh seed from the OS entropy pool and returns it, as gym's
        ``seeding.np_random(None)`` does (8 bytes; the reference's stream itself is replaced by Philox)."""
        s = int.from_bytes(os.urandom(8), "little") if seed is None else int(seed)
        self.engine.seed(s)
        return [s]

    def set_curriculum_level(self, level):
        self.spec.set_curriculum_level(level)
        self.engine.update_config(self.spec.sim, self.spec)

    @property
    def target(self):
        t = self.engine.get_block(C.FW_BLK_TARGET)[:, 0].double().cpu().numpy()
        return self._with_ang({"roll": float(t[0]), "pitch": float(t[1]), "Va": float(t[2])})

    def _with_ang(self, d):
        """+ the attitude_angular targets omega_p / q / r (rows 12..14 of FW_BLK_TARGET_PROPS) when configured."""
        if getattr(self.spec, "ang_targets", False):
            o = self.engine.get_block(C.FW_BLK_TARGET_PROPS)[12:15, 0].double().cpu().numpy()
            d.update({n: float(v) for n, v in zip(C.ANG_TARGETS, o)})
        return d

    @property
    def steps_count(self):
        s, _ = self.engine.steps()
        return int(s[0])

    def reset(self, state=None, target=None, turbulence_noise=None):
        """FixedWingAircraft.reset (fixed_wing.py:414-481)."""
        self.engine.set_noise(turbulence_noise)  # Dryden.reset(noise): None draws fresh noise (dryden.py:174-188)
        init = C.init_array(state, 1, self.spec.sim) if state is not None else None
        tgt = None
        if target is not None:
            tgt = np.full((3, 1), np.nan)
            for k, v in target.items():
                tgt[C.TARGET_INDEX[k], 0] = v
        obs = self.engine.reset(init=init, target=tgt)
        o = obs[0].cpu().numpy().astype(np.float32).reshape(self.spec.obs_shape)
        t, v = self._targets_vals()
        self._hist.reset(o, t, v)
        self._tgt = t
        return o

    def step(self, action):
        a = np.asarray(action, dtype=np.float64).reshape(1, 3)
        assert not np.any(np.isnan(a))
        self._act.copy_(torch.as_tensor(a))
        obs, rew, done, term = self.engine.env_step(self._act, auto_reset=False, terminal_obs=False, episode=False)
        d = bool(done[0].item())
        t, v = self._targets_vals()
        o = obs[0].cpu().numpy().astype(np.float32).reshape(self.spec.obs_shape)
        self._hist.step(np.asarray(action).reshape(-1), step_succeeded(term[0].item()), o, float(rew[0].item()),
                        self._tgt, t, v)
        self._tgt = t
        info = {}
        if d:
            info["termination"] = termination_name(term[0].item(), tuple(self.spec.sim.dynamics))
            if self.engine.metrics is not None:
                info.update(metric_info(self.engine.metrics[:, 0].cpu().numpy(),
                                        [m["name"] for m in self.cfg.get("metrics", [])]))
        info["target"] = self._with_ang({"roll": float(t[0]), "pitch": float(t[1]), "Va": float(t[2])})
        return o, float(rew[0].item()), d, info

    def render(self, mode="plot", **kw):
        raise NotImplementedError("rendering is host-side plotting; out of scope for the device engine")

    def close(self):
        self.engine.close()
