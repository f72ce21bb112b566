"""Device-resident VecEnv with the Stable-Baselines3 0.10 surface.

``FixedWingVecEnv`` replaces ``VecNormalize(SubprocVecEnv([FixedWingAircraft(...)] * n))``'s
inner part -- the reference runs one OS process per env
(stable_baselines3/common/vec_env/subproc_vec_env.py:17-208) and pickles every
observation through a pipe; here all N aircraft live in HBM and one fused
kernel steps them.  Method names, signatures and auto-reset semantics follow
``VecEnv`` (base_vec_env.py:48-200) and the SubprocVecEnv worker
(subproc_vec_env.py:25-31): when an env is done, ``info["terminal_observation"]``
holds its last observation and the returned observation is the first one of
the next episode.  Monitor statistics (common/monitor.py:88-115) are reported
as ``info["episode"] = {"r", "l", "t"}`` for done envs.

Step results are numpy arrays (SB3 semantics) unless ``return_tensors=True``,
in which case they stay on the device as torch tensors (no host sync).
"""
import collections.abc
import time

import numpy as np
import torch

from . import config as C
from .engine import Engine
from .spaces import Box

try:  # subclass SB3's VecEnv when available so isinstance checks pass
    from stable_baselines3.common.vec_env.base_vec_env import VecEnv as _SB3VecEnv  # pragma: no cover
except Exception:  # noqa: BLE001
    _SB3VecEnv = None


class VecEnv(_SB3VecEnv if _SB3VecEnv is not None else object):
    """Minimal restatement of SB3's abstract VecEnv (base_vec_env.py:48-200)."""

    metadata = {"render.modes": []}

    def __init__(self, num_envs, observation_space, action_space):
        self.num_envs = num_envs
        self.observation_space = observation_space
        self.action_space = action_space

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def get_images(self):
        raise NotImplementedError

    def render(self, mode="human"):
        raise NotImplementedError("rendering is not part of the device engine")

    @property
    def unwrapped(self):
        return self

    def getattr_depth_check(self, name, already_found):
        return None

    def _get_indices(self, indices):
        if indices is None:
            indices = range(self.num_envs)
        elif isinstance(indices, int):
            indices = [indices]
        return indices


def quad_auto_max():
    """The library's automatic-rule threshold (fw_quad_auto_max: the build's FW_QUAD_AUTO_MAX)."""
    from . import _native
    return int(_native.load().fw_quad_auto_max())


def auto_lanes(global_envs, world_size=None):
    """Lanes per aircraft for every shard of ``global_envs`` envs split over ``world_size`` ranks (default:
    the initialised process group's size, else 1): the library's automatic rule applied to the largest
    shard (sharding.shard_range gives the remainder to the first ranks)."""
    if world_size is None:
        import torch.distributed as dist
        world_size = dist.get_world_size() if (dist.is_available() and dist.is_initialized()) else 1
    largest = -(-int(global_envs) // int(world_size))
    return 4 if largest <= quad_auto_max() else 1


def termination_name(code, dynamics=("elevon_right", "elevon_left", "throttle")):
    """Termination code -> the reference's info["termination"] string."""
    code = int(code)
    if code == C.FW_TERM_STEPS:
        return "steps"
    if code == C.FW_TERM_SUCCESS:
        return "success"
    v = code - 1
    if C.FW_V_ACT0 <= v <= C.FW_V_ACT2:
        return dynamics[v - C.FW_V_ACT0]
    if 0 <= v < len(C.VAR_NAMES):
        return C.VAR_NAMES[v]
    return "solver"


def metric_info(row, names):
    """One FW_NMETRIC record -> the info entries get_metric produces (fixed_wing.py:1644-1736)."""
    out = {}
    for name in names:
        col, keys = C.METRIC_LAYOUT[name]
        vals = {}
        for j, k in enumerate(keys):
            v = float(row[col + j])
            if name == "success":
                v = bool(v)
            elif name in ("settling_time", "rise_time") and np.isfinite(v):
                v = int(round(v))
            vals[k] = v
        out[name] = vals
    return out


class _Infos(collections.abc.Sequence):
    """Per-env info dicts, materialised on first access (65536 dicts per step are
    the dominant host cost of the SB3 surface, and most callers touch few)."""

    def __init__(self, n, done, term, tobs, episode, targets, t_elapsed, dynamics, with_target, metrics=None,
                 metric_names=(), stats=None):
        self._n = n
        self._done, self._term, self._tobs, self._ep = done, term, tobs, episode
        self._tgt = targets
        self._t = t_elapsed
        self._dyn = dynamics
        self._with_target = with_target
        self._met, self._met_names = metrics, metric_names
        self._stats = stats
        self._cache = {}

    def __len__(self):
        return self._n

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[j] for j in range(*i.indices(self._n))]
        if i < 0:
            i += self._n
        d = self._cache.get(i)
        if d is None:
            d = {}
            if self._done[i]:
                d["terminal_observation"] = self._tobs[i]
                d["termination"] = termination_name(self._term[i], self._dyn)
                ep = self._ep[i]
                d["episode"] = {"r": round(float(ep[0]), 6), "l": int(round(float(ep[1]))), "t": round(self._t, 6)}
                if self._met is not None:
                    d.update(metric_info(self._met[:, i], self._met_names))
                if self._with_target:
                    d["target"] = {"roll": float(ep[2]), "pitch": float(ep[3]), "Va": float(ep[4])}
            elif self._with_target:
                t = self._tgt[:, i]
                d["target"] = {"roll": float(t[0]), "pitch": float(t[1]), "Va": float(t[2])}
            if self._stats is not None and (int(self._stats[i]) >> 30) & 1:
                # the step ended on the RHS-evaluation budget (fw_sim_config.max_nfev; scipy has none): the
                # last accepted sub-step was committed, where solve_ivp would have kept integrating
                d["solver_budget_exhausted"] = True
            self._cache[i] = d
        return d


class FixedWingVecEnv(VecEnv):
    """N FixedWingAircraft environments stepped by one fused MI355X kernel.

    Construction mirrors ``FixedWingAircraft(config_path, sim_config_path=...,
    sim_parameter_path=..., config_kw=..., sim_config_kw=...)``
    (fixed_wing.py:14-24) plus the batch size and device.
    """

    def __init__(self, num_envs=1, config_path=None, config_kw=None, sim_config_path=None, sim_parameter_path=None,
                 sim_config_kw=None, device=None, precision="float32", seed=None, return_tensors=False,
                 info_target=True, curriculum_level=1, env_offset=0, record_history=False, lanes=None,
                 global_envs=None):
        self.spec = C.EnvSpec(config_path, config_kw, sim_config_path, sim_parameter_path, sim_config_kw,
                              curriculum_level=curriculum_level)
        obs_space = Box(self.spec.obs_low, self.spec.obs_high, dtype=np.float32)
        act_space = Box(self.spec.action_space_low, self.spec.action_space_high, dtype=np.float32)
        VecEnv.__init__(self, int(num_envs), obs_space, act_space)
        # lanes: integrator (fw_set_lanes; None = automatic by num_envs).  A shard of a sharded batch
        # (global_envs = the envs of all ranks) picks it from the LARGEST shard of the split, so every rank
        # runs the same integrator (the automatic rule alone could give 16385 one lane and 16384 quads)
        if lanes is None and global_envs is not None:
            lanes = auto_lanes(global_envs)
        self.engine = Engine(self.spec.sim, self.spec, self.num_envs, device=device, precision=precision, lanes=lanes)
        self.device = self.engine.device
        self.return_tensors = return_tensors
        self.info_target = info_target
        self.env_offset = int(env_offset)
        self.training = True
        self._actions = None
        self._t_start = time.time()
        self._dyn = tuple(self.spec.sim.dynamics)
        self.seed(seed if seed is not None else 0)
        self._reset_pending = True
        # per-env FixedWingAircraft.history on the host (get_attr("history")): pulls every step's data
        # to the host, meant for evaluation with few envs
        self._hists = None
        if record_history:
            if getattr(self.spec, "ang_targets", False):
                # history["target"] / ["error"] would carry omega_p / q / r as well (fixed_wing.py:575-580)
                raise NotImplementedError("record_history with attitude_angular targets")
            from .history import EpisodeHistory
            self._hists = [EpisodeHistory(self.spec) for _ in range(self.num_envs)]

    @property
    def cfg(self):
        return self.spec.cfg

    # ---------------------------------------------------------------- VecEnv API
    def seed(self, seed=None):
        """SubprocVecEnv.seed gives env i the seed ``seed + i`` (subproc_vec_env.py:120-123); here env i
        draws from Philox stream (seed, env_offset + i)."""
        s = 0 if seed is None else int(seed)
        self.engine.seed(s, env_offset=self.env_offset)
        return [s + i for i in range(self.num_envs)]

    def reset(self):
        # every SubprocVecEnv worker resets without turbulence_noise (Dryden.reset(None) draws fresh noise,
        # dryden.py:174-188): a per-env injection ends here
        self.engine.set_env_noise(range(self.num_envs), None)
        obs = self.engine.reset()
        self._reset_pending = False
        if self._hists is not None:
            o = obs.cpu().numpy().astype(np.float32)
            t, v = self._targets_vals()
            for i, h in enumerate(self._hists):
                h.reset(self._shaped(o[i:i + 1])[0], t[:, i], v[:, i])
            self._tgt = t
        return self._out(obs)

    def _targets_vals(self):
        t = self.engine.get_block(C.FW_BLK_TARGET).double().cpu().numpy()
        d = self.engine.get_block(C.FW_BLK_DERIVED).double().cpu().numpy()
        return t, d[[0, 1, 3]]

    def _step_recording(self, actions):
        """env step with the history recorder: step without auto-reset, record every env's step from its
        post-step state, then reset the done envs (what the SubprocVecEnv worker does, subproc_vec_env.py:
        25-31) and restart their histories with the reset observation."""
        from .history import step_succeeded
        eng = self.engine
        obs, rew, done, term = eng.env_step(actions, auto_reset=False, stats=True)
        dn = done.cpu().numpy().astype(bool)
        tm, r = term.cpu().numpy(), rew.double().cpu().numpy()
        o = self._shaped(obs.cpu().numpy().astype(np.float32))
        to = self._shaped(eng.terminal_obs.cpu().numpy().astype(np.float32))
        t, v = self._targets_vals()
        a = actions.double().cpu().numpy()
        for i, h in enumerate(self._hists):
            h.step(a[i], step_succeeded(tm[i]), to[i] if dn[i] else o[i], r[i], self._tgt[:, i], t[:, i], v[:, i])
        if dn.any():
            eng.set_env_noise(np.nonzero(dn)[0], None)  # as the auto-reset of fw_env_step: the injection ends
            obs = eng.reset(mask=dn)
            o = self._shaped(obs.cpu().numpy().astype(np.float32))
            t, v = self._targets_vals()
            for i in np.nonzero(dn)[0]:
                self._hists[i].reset(o[i], t[:, i], v[:, i])
        self._tgt = t
        return obs, rew, done, term

    def step_async(self, actions):
        if isinstance(actions, torch.Tensor):
            a = actions.to(device=self.device, dtype=self.engine.dtype)
        else:
            a = torch.as_tensor(np.asarray(actions), dtype=self.engine.dtype).to(self.device, non_blocking=True)
        self._actions = a.reshape(self.num_envs, -1).contiguous()

    def step_wait(self):
        if self._actions is None:
            raise RuntimeError("step_wait() without step_async()")
        eng = self.engine
        if self._hists is not None:
            obs, rew, done, term = self._step_recording(self._actions)
        else:
            obs, rew, done, term = eng.env_step(self._actions, auto_reset=True, stats=True)
        self._actions = None
        if self.return_tensors:
            # a bool view of the engine's uint8 done buffer (no conversion kernel); like obs and rew it is
            # the engine's buffer, overwritten by the next step
            return self._shaped(obs), rew, done.view(torch.bool), self._infos_lazy_device()
        done_np = done.cpu().numpy().astype(bool)
        infos = self._infos(done_np)
        return self._shaped(obs.cpu().numpy().astype(np.float32)), rew.cpu().numpy().astype(np.float32), done_np, infos

    def rollout(self, actions):
        """``K`` consecutive ``step`` calls for actions known in advance ([K][N][3] device tensor), in one
        fused launch (Engine.env_rollout): the SAC / TD3 warm-up with uniform actions, scripted command
        sequences.  Auto-reset as in ``step``.  Returns device tensors (obs [K, N, *obs_shape], reward
        [K][N], done [K][N] bool, termination code [K][N]); terminal observations and Monitor records of
        the done steps are in ``engine.rollout_terminal_obs`` / ``engine.rollout_episode``; the episode
        metrics (``engine.metrics``) hold the last episode each env finished inside the launch."""
        if self._hists is not None:
            raise NotImplementedError("rollout() resets envs inside the launch, so per-env histories cannot be "
                                      "recorded: use step() with record_history=True")
        a = torch.as_tensor(actions).to(device=self.device, dtype=self.engine.dtype)
        obs, rew, done, term = self.engine.env_rollout(a.reshape(a.shape[0], self.num_envs, -1).contiguous())
        shape = self.observation_space.shape
        o = obs if len(shape) == 1 else obs.reshape(obs.shape[:2] + tuple(shape))
        return o, rew, done.bool(), term

    def _shaped(self, o):
        """[N][length * n_row] device layout -> [N, *observation_space.shape] ("matrix" observations)."""
        shape = self.observation_space.shape
        return o if len(shape) == 1 else o.reshape((o.shape[0],) + tuple(shape))

    def _infos(self, done_np):
        eng = self.engine
        term = eng.term.cpu().numpy()
        anyd = bool(done_np.any())
        tobs = self._shaped(eng.terminal_obs.cpu().numpy().astype(np.float32)) if anyd else None
        ep = eng.episode.cpu().numpy() if anyd else None
        tgt = eng.get_block(C.FW_BLK_TARGET).cpu().numpy() if self.info_target else None
        met = eng.metrics.cpu().numpy() if (anyd and eng.metrics is not None) else None
        return _Infos(self.num_envs, done_np, term, tobs, ep, tgt, time.time() - self._t_start, self._dyn,
                      self.info_target, met, [m["name"] for m in self.spec.cfg.get("metrics", [])],
                      eng.stats.cpu().numpy())

    def _infos_lazy_device(self):
        """Device mode: infos are built only if the caller asks for them (triggers a sync)."""
        env = self

        class _Lazy(collections.abc.Sequence):
            _inner = None

            def _get(self):
                if self._inner is None:
                    self._inner = env._infos(env.engine.done.cpu().numpy().astype(bool))
                return self._inner

            def __len__(self):
                return env.num_envs

            def __getitem__(self, i):
                return self._get()[i]

        return _Lazy()

    def close(self):
        self.engine.close()

    def graph_key(self):
        """What a captured step bakes in (rollout.RolloutCollector recaptures when it changes)."""
        return (self.engine.lanes, self.engine.config_version, self._hists is not None)

    def get_attr(self, attr_name, indices=None):
        idx = list(self._get_indices(indices))
        if attr_name == "target":
            t = self.engine.get_block(C.FW_BLK_TARGET).cpu().numpy()
            out = [{"roll": float(t[0, i]), "pitch": float(t[1, i]), "Va": float(t[2, i])} for i in idx]
            if getattr(self.spec, "ang_targets", False):  # + omega_p / q / r (FW_BLK_TARGET_PROPS rows 12..14)
                o = self.engine.get_block(C.FW_BLK_TARGET_PROPS)[12:15].double().cpu().numpy()
                for d, i in zip(out, idx):
                    d.update({n: float(o[k, i]) for k, n in enumerate(C.ANG_TARGETS)})
            return out
        if attr_name == "simulator":
            from .pyfly import SimulatorView
            return [SimulatorView(self.engine, i) for i in idx]
        if attr_name in ("cfg", "observation_space", "action_space", "training", "steps_max"):
            val = {"cfg": self.spec.cfg, "observation_space": self.observation_space,
                   "action_space": self.action_space, "training": self.training,
                   "steps_max": self.spec.steps_max}[attr_name]
            return [val for _ in idx]
        if attr_name == "history":
            if self._hists is None:
                raise AttributeError("history is recorded on the host only with FixedWingVecEnv(record_history=True)")
            return [self._hists[i].history for i in idx]
        if attr_name == "steps_count":
            s, _ = self.engine.steps()
            s = s.cpu().numpy()
            return [int(s[i]) for i in idx]
        host = self._host_attrs()
        if attr_name == "use_curriculum" and all(attr_name in host[i] for i in idx):
            # a plain attribute in the reference (fixed_wing.py:299, 412: set True by __init__ and
            # set_curriculum_level, never read): a set_attr value stands until the next set_curriculum_level
            return [host[i][attr_name] for i in idx]
        if attr_name in ("scale_actions", "goal_enabled", "integration_window", "curriculum_level", "use_curriculum",
                         "obs_norm"):
            val = {"scale_actions": self.spec.scale_actions,
                   "goal_enabled": self.spec.cfg["target"]["success_streak_req"] > 0,
                   "integration_window": self.spec.cfg.get("integration_window", 0),
                   "curriculum_level": getattr(self.spec, "curriculum_level", 1),
                   "use_curriculum": True, "obs_norm": self.spec.cfg["observation"].get("normalize", False)}[attr_name]
            return [val for _ in idx]
        if all(attr_name in host[i] for i in idx):  # set earlier by set_attr
            return [host[i][attr_name] for i in idx]
        raise AttributeError("FixedWingVecEnv has no per-env attribute %r" % attr_name)

    def _host_attrs(self):
        """Per-env attributes set through set_attr that the device step does not read (a plain ``setattr`` on
        the worker's FixedWingAircraft, subproc_vec_env.py:156-161): kept on the host, returned by get_attr."""
        if getattr(self, "_hattrs", None) is None:
            self._hattrs = [dict() for _ in range(self.num_envs)]
        return self._hattrs

    def set_attr(self, attr_name, value, indices=None):
        """SubprocVecEnv.set_attr (subproc_vec_env.py:156-161: ``setattr(env, name, value)`` on each chosen
        worker's FixedWingAircraft).  Attributes the device step reads: ``training`` (the reference's
        callbacks, train_rl_controller.py:320), ``target`` (a {"roll", "pitch", "Va"} dict, partial allowed:
        the chosen envs track it from their next step), ``steps_count`` (their step counter), ``steps_max``
        and ``curriculum_level`` (one device configuration, so ``indices`` must cover all envs; like the
        reference, the turbulence sequence length fixed at construction does not change).  Configuration
        attributes (cfg, spaces, simulator, ...) are refused: they are compiled into the device config.
        Any other name is stored per env on the host and returned by get_attr, as a plain attribute of the
        worker's env object would be (the device step never reads it); render_on_reset / save_on_reset may
        be set False only (plotting is out of scope)."""
        idx = list(self._get_indices(indices))
        if attr_name == "training":
            self.training = value
            return
        if attr_name == "target":
            t = self.engine.get_block(C.FW_BLK_TARGET)
            for k, v in dict(value).items():
                t[C.TARGET_INDEX[k], idx] = float(v)
            self.engine.set_block(C.FW_BLK_TARGET, t)
            return
        if attr_name == "steps_count":
            sw = self.engine.get_block(C.FW_BLK_STEPS)
            keep = sw[0, idx] & ~0xFFFF
            sw[0, idx] = keep | (int(value) & 0xFFFF)
            self.engine.set_block(C.FW_BLK_STEPS, sw)
            return
        if attr_name == "steps_max":
            if sorted(set(i % self.num_envs for i in idx)) != list(range(self.num_envs)):
                raise NotImplementedError("steps_max is one device configuration: set it for all envs (indices=None)")
            self.spec.steps_max = int(value)
            self.engine.update_config(self.spec.sim, self.spec)
            return
        if attr_name in ("curriculum_level",):  # FixedWingAircraft.set_curriculum_level's state (fixed_wing.py:334)
            if sorted(set(i % self.num_envs for i in idx)) != list(range(self.num_envs)):
                raise NotImplementedError("curriculum_level is one device configuration: set it for all envs")
            self.set_curriculum_level(value)
            return
        if attr_name in ("render_on_reset", "save_on_reset") and value:
            raise NotImplementedError("%s is host-side plotting; out of scope for the device engine" % attr_name)
        if attr_name in ("cfg", "observation_space", "action_space", "simulator", "history", "scale_actions",
                         "integration_window", "goal_enabled", "obs_norm"):
            # attributes the reference reads while stepping: on the device they are the compiled configuration
            raise AttributeError("setting %r would change the compiled device configuration: rebuild the env "
                                 "(config_kw) or use update_config" % attr_name)
        host = self._host_attrs()  # any other attribute: the device step does not read it (e.g. a callback's flag)
        for i in idx:
            host[i][attr_name] = value

    def env_method(self, method_name, *method_args, indices=None, **method_kwargs):
        idx = list(self._get_indices(indices))
        if method_name == "reset":
            return self._reset_some(idx, *method_args, **method_kwargs)
        if method_name == "set_curriculum_level":
            self.set_curriculum_level(*method_args, **method_kwargs)
            return [None for _ in idx]
        if method_name == "seed":
            return [self.seed(*method_args, **method_kwargs)[i] for i in idx]
        if method_name in ("render", "save_history"):
            raise NotImplementedError("%s is host-side plotting; out of scope for the device engine" % method_name)
        raise AttributeError("unsupported env_method %r" % method_name)

    # --------------------------------------------------------------- extras
    def set_curriculum_level(self, level):
        """FixedWingAircraft.set_curriculum_level (fixed_wing.py:334-412) for all envs."""
        self.spec.set_curriculum_level(level)
        self.engine.update_config(self.spec.sim, self.spec)
        for h in self._host_attrs():  # fixed_wing.py:412: use_curriculum = True again
            h.pop("use_curriculum", None)

    def _reset_some(self, idx, state=None, target=None, turbulence_noise=None):
        """FixedWingAircraft.reset(state=..., target=...) for the envs in ``idx``."""
        n = self.num_envs
        mask = np.zeros(n, np.uint8)
        mask[idx] = 1
        init = None
        if state is not None:
            states = [None] * n
            for i in idx:
                states[i] = state
            init = C.init_array(states, n, self.spec.sim)
        tgt = None
        if target is not None:
            tgt = np.full((3, n), np.nan)
            for i in idx:
                for k, v in target.items():
                    tgt[C.TARGET_INDEX[k], i] = v
        # FixedWingAircraft.reset(**sim_reset_kw) -> PyFly.reset(turbulence_noise=...) -> Dryden.reset(noise)
        # (fixed_wing.py:441, pyfly.py:1294, dryden.py:174-188): these envs' episodes read the given noise,
        # and a reset without it draws fresh noise again
        self.engine.set_env_noise(idx, turbulence_noise)
        obs = self.engine.reset(mask=mask, init=init, target=tgt)
        o = self._shaped(obs.cpu().numpy().astype(np.float32))
        return [o[i] for i in idx]

    def _out(self, t):
        return self._shaped(t if self.return_tensors else t.cpu().numpy().astype(np.float32))
