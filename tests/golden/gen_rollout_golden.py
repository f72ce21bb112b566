"""Golden fixtures for the rollout-side kernels (test infrastructure only).

Runs the reference's vendored Stable-Baselines3 0.10.0 (``RolloutBuffer``,
``RunningMeanStd``, ``VecNormalize``, ``ReplayBuffer``) from /root/reference on
seeded synthetic data and stores inputs + outputs as ``.npz``.  Only data
leaves this script.  The GPU box never runs it.

gym 0.18 is not installed, so a minimal offline stand-in module is installed
first (class names only; SB3's buffer / normalisation code uses nothing but
``spaces.Box`` shapes and dtypes).  The ``stable_baselines3`` package
``__init__`` (which imports every algorithm) is bypassed by registering the
package path directly.

Usage:  python tests/golden/gen_rollout_golden.py

Fixtures:
  rollout_gae.npz    RolloutBuffer.add x T + compute_returns_and_advantage, several (T, N, gamma, lambda)
  vecnormalize.npz   VecNormalize(reset + K step_wait) over a scripted VecEnv: normalised obs/rewards, rms states
  replay.npz         ReplayBuffer add sequence (wrap-around) + _get_samples, optimize_memory_usage on/off
"""
import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference/magpie/libs/stable-baselines3"
OUT = os.path.dirname(os.path.abspath(__file__))


def _install_gym_stub():
    gym = types.ModuleType("gym")
    spaces = types.ModuleType("gym.spaces")

    class Space:
        def __init__(self, shape=None, dtype=None):
            self.shape = shape
            self.dtype = None if dtype is None else np.dtype(dtype)

    class Box(Space):
        def __init__(self, low, high, shape=None, dtype=np.float32):
            if shape is not None and np.isscalar(low):
                low, high = np.full(shape, low), np.full(shape, high)
            self.low = np.asarray(low, dtype=dtype)
            self.high = np.asarray(high, dtype=dtype)
            Space.__init__(self, self.low.shape, dtype)

    class Discrete(Space):
        def __init__(self, n):
            self.n = n
            Space.__init__(self, (), np.int64)

    class MultiDiscrete(Space):
        def __init__(self, nvec):
            self.nvec = np.asarray(nvec)
            Space.__init__(self, self.nvec.shape, np.int64)

    class MultiBinary(Space):
        def __init__(self, n):
            self.n = n
            Space.__init__(self, (n,), np.int8)

    class Dict(Space):
        def __init__(self, spaces_=None):
            self.spaces = spaces_ or {}
            Space.__init__(self, None, None)

    class Tuple(Space):
        def __init__(self, spaces_):
            self.spaces = spaces_
            Space.__init__(self, None, None)

    for c in (Space, Box, Discrete, MultiDiscrete, MultiBinary, Dict, Tuple):
        setattr(spaces, c.__name__, c)

    class Env:
        metadata = {}

    class Wrapper(Env):
        def __init__(self, env):
            self.env = env

    gym.Env, gym.GoalEnv, gym.Space, gym.Wrapper = Env, Env, Space, Wrapper
    gym.ObservationWrapper = gym.RewardWrapper = gym.ActionWrapper = Wrapper
    gym.spaces = spaces
    error = types.ModuleType("gym.error")
    error.Error = type("Error", (Exception,), {})
    gym.error = error
    wrappers = types.ModuleType("gym.wrappers")
    monitoring = types.ModuleType("gym.wrappers.monitoring")
    video = types.ModuleType("gym.wrappers.monitoring.video_recorder")
    video.VideoRecorder = type("VideoRecorder", (), {})
    monitoring.video_recorder = video
    wrappers.monitoring = monitoring
    gym.wrappers = wrappers
    envs = types.ModuleType("gym.envs")
    reg = types.ModuleType("gym.envs.registration")
    reg.EnvSpec = type("EnvSpec", (), {})
    envs.registration = reg
    gym.envs = envs
    utils = types.ModuleType("gym.utils")
    seeding = types.ModuleType("gym.utils.seeding")
    utils.seeding = seeding
    gym.utils = utils
    for name, mod in {"gym": gym, "gym.spaces": spaces, "gym.error": error, "gym.wrappers": wrappers,
                      "gym.wrappers.monitoring": monitoring, "gym.wrappers.monitoring.video_recorder": video,
                      "gym.envs": envs, "gym.envs.registration": reg, "gym.utils": utils,
                      "gym.utils.seeding": seeding}.items():
        sys.modules[name] = mod
    return gym


def _import_sb3():
    pkg = types.ModuleType("stable_baselines3")
    pkg.__path__ = [os.path.join(REF, "stable_baselines3")]
    sys.modules["stable_baselines3"] = pkg
    import stable_baselines3.common.base_class  # noqa: F401  -- the package's own import order (breaks a cycle)
    from stable_baselines3.common.buffers import RolloutBuffer
    from stable_baselines3.common.running_mean_std import RunningMeanStd
    from stable_baselines3.common.vec_env.base_vec_env import VecEnv
    from stable_baselines3.common.vec_env.vec_normalize import VecNormalize
    return RolloutBuffer, RunningMeanStd, VecEnv, VecNormalize


def gen_gae(RolloutBuffer, gym):
    cases = [("a", 64, 37, 0.99, 0.95, 0.05), ("b", 33, 16, 0.98, 1.0, 0.2), ("c", 1, 8, 0.99, 0.95, 0.5),
             ("d", 200, 5, 0.999, 0.9, 0.01)]
    out = {}
    rng = np.random.RandomState(123)
    obs_space = gym.spaces.Box(-np.inf, np.inf, shape=(14,), dtype=np.float32)
    act_space = gym.spaces.Box(-1.0, 1.0, shape=(3,), dtype=np.float32)
    for name, T, N, gamma, lam, p_done in cases:
        buf = RolloutBuffer(T, obs_space, act_space, device="cpu", gae_lambda=lam, gamma=gamma, n_envs=N)
        last_dones = rng.rand(N) < p_done
        starts = np.zeros((T, N), bool)
        for t in range(T):
            obs = rng.randn(N, 14).astype(np.float32)
            act = rng.uniform(-1, 1, (N, 3)).astype(np.float32)
            rew = rng.randn(N) * 3.0  # float64, as the VecEnv returns it
            val = torch.tensor(rng.randn(N, 1) * 5.0, dtype=torch.float32)
            logp = torch.tensor(rng.randn(N), dtype=torch.float32)
            starts[t] = last_dones
            buf.add(obs, act, rew, last_dones, val, logp)
            last_dones = rng.rand(N) < p_done
        last_values = torch.tensor(rng.randn(N, 1) * 5.0, dtype=torch.float32)
        buf.compute_returns_and_advantage(last_values=last_values, dones=last_dones)
        p = name + "__"
        out.update({p + "gamma": gamma, p + "lam": lam, p + "rewards": buf.rewards, p + "values": buf.values,
                    p + "starts": starts.astype(np.uint8), p + "dones_stored": buf.dones,
                    p + "last_values": last_values.numpy().ravel(), p + "last_dones": last_dones.astype(np.uint8),
                    p + "advantages": buf.advantages, p + "returns": buf.returns})
        # flattening order used by RolloutBuffer.get (swap_and_flatten, buffers.py:70-80)
        out[p + "flat_advantages"] = buf.swap_and_flatten(buf.advantages.copy()).ravel()
    np.savez_compressed(os.path.join(OUT, "rollout_gae.npz"), **out)


def gen_vecnormalize(VecEnv, VecNormalize, gym):
    N, D, K = 16, 14, 60
    rng = np.random.RandomState(7)
    scale = rng.uniform(0.1, 30.0, D)
    seq_obs = (rng.randn(K + 1, N, D) * scale + rng.randn(D) * 10).astype(np.float32)
    seq_rew = (rng.randn(K, N) * 2 - 1).astype(np.float32).astype(np.float64)
    seq_done = rng.rand(K, N) < 0.08

    class Scripted(VecEnv):
        def __init__(self):
            VecEnv.__init__(self, N, gym.spaces.Box(-np.inf, np.inf, shape=(D,), dtype=np.float32),
                            gym.spaces.Box(-1, 1, shape=(3,), dtype=np.float32))
            self.k = 0

        def reset(self):
            self.k = 0
            return seq_obs[0].copy()

        def step_async(self, actions):
            pass

        def step_wait(self):
            k = self.k
            self.k += 1
            return seq_obs[k + 1].copy(), seq_rew[k].copy(), seq_done[k].copy(), [{} for _ in range(N)]

        def close(self):
            pass

        def get_attr(self, *a, **k):
            return []

        def set_attr(self, *a, **k):
            pass

        def env_method(self, *a, **k):
            return []

        def seed(self, seed=None):
            return []

        def get_images(self):
            return []

        def env_is_wrapped(self, *a, **k):
            return [False] * N

    vn = VecNormalize(Scripted(), gamma=0.99, clip_obs=10.0, clip_reward=10.0)
    o0 = vn.reset()
    nobs, nrew, rms = [], [], []
    for k in range(K):
        vn.step_async(np.zeros((N, 3), np.float32))
        o, r, d, _ = vn.step_wait()
        nobs.append(o)
        nrew.append(r)
        rms.append(np.concatenate([vn.obs_rms.mean, vn.obs_rms.var, [vn.obs_rms.count], [vn.ret_rms.mean],
                                   [vn.ret_rms.var], [vn.ret_rms.count]]))
    np.savez_compressed(os.path.join(OUT, "vecnormalize.npz"), obs=seq_obs, rew=seq_rew, done=seq_done.astype(np.uint8),
                        norm_obs0=o0, norm_obs=np.stack(nobs), norm_rew=np.stack(nrew), rms=np.stack(rms),
                        gamma=0.99, clip_obs=10.0, clip_reward=10.0, epsilon=1e-8)


def gen_replay(gym):
    """ReplayBuffer (n_envs = 1) add sequence that wraps around, then _get_samples on every slot,
    with and without optimize_memory_usage (buffers.py:151-257)."""
    from stable_baselines3.common.buffers import ReplayBuffer
    rng = np.random.RandomState(77)
    B, K = 7, 11
    obs_space = gym.spaces.Box(-np.inf, np.inf, shape=(14,), dtype=np.float32)
    act_space = gym.spaces.Box(-1.0, 1.0, shape=(3,), dtype=np.float32)
    out = {}
    adds = {"obs": rng.randn(K, 14).astype(np.float32), "next_obs": rng.randn(K, 14).astype(np.float32),
            "action": rng.uniform(-1, 1, (K, 3)).astype(np.float32), "reward": rng.randn(K),
            "done": (rng.rand(K) < 0.3)}
    for k, v in adds.items():
        out["add_" + k] = v
    for opt in (False, True):
        buf = ReplayBuffer(B, obs_space, act_space, device="cpu", n_envs=1, optimize_memory_usage=opt)
        for t in range(K):
            buf.add(adds["obs"][t][None], adds["next_obs"][t][None], adds["action"][t][None],
                    np.array([adds["reward"][t]]), np.array([adds["done"][t]]))
        inds = np.arange(B)
        s = buf._get_samples(inds)
        p = "opt%d__" % int(opt)
        out[p + "pos"] = np.array(buf.pos)
        out[p + "full"] = np.array(buf.full)
        for name, t in zip(["observations", "actions", "next_observations", "dones", "rewards"], s):
            out[p + name] = t.numpy()
    np.savez_compressed(os.path.join(OUT, "replay.npz"), **out)


if __name__ == "__main__":
    gym = _install_gym_stub()
    RolloutBuffer, RunningMeanStd, VecEnv, VecNormalize = _import_sb3()
    which = sys.argv[1:] or ["gae", "vecnormalize", "replay"]
    if "gae" in which:
        gen_gae(RolloutBuffer, gym)
    if "vecnormalize" in which:
        gen_vecnormalize(VecEnv, VecNormalize, gym)
    if "replay" in which:
        gen_replay(gym)
    print("wrote", which)
