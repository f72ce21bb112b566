"""Device multi-env ReplayBuffer and the off-policy (SAC/TD3) collection loop.

SURVEY.md 8(f) row 4 / BASELINE configs[4] (SAC replay-buffer fill at 262144 envs).
SB3 0.10's ``ReplayBuffer`` (stable_baselines3/common/buffers.py:151-257) keeps
``n_envs == 1`` numpy arrays and ``OffPolicyAlgorithm.collect_rollouts``
(common/off_policy_algorithm.py:356-470) asserts a single env; here both are
lifted to N envs on the device -- a deliberate API extension -- while keeping
the reference's storage semantics: float32 rewards / dones, the scaled action
in [-1, 1] stored (``scale_action``, policies.py:309-318), ``next_obs`` = the
observation returned by the step (after auto-reset for done envs, as in
SB3 0.10), the unnormalised observation / reward when a VecNormalize is used,
and ``optimize_memory_usage`` (next observation read from slot + 1).

Layout: ``buffer_size`` counts transitions like SB3 1.x multi-env buffers; the
device arrays are ``[steps][n_envs][...]`` with ``steps = buffer_size // n_envs``
and transition ``k = step * n_envs + env``.  ``add`` moves one step for all envs
with ONE ``fw_replay_add`` launch (obs, next_obs, action, reward, done).
"""
import collections
import ctypes

import numpy as np
import torch

from . import _native

ReplayBufferSamples = collections.namedtuple(
    "ReplayBufferSamples", ["observations", "actions", "next_observations", "dones", "rewards"])


def _stream(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


class ReplayBuffer:
    def __init__(self, buffer_size, observation_space, action_space, device=None, n_envs=1,
                 optimize_memory_usage=False):
        self.n_envs = int(n_envs)
        self.buffer_size = max(int(buffer_size) // self.n_envs, 1)  # steps
        self.obs_dim = int(np.prod(observation_space.shape))
        self.action_dim = int(np.prod(action_space.shape))
        self.device = torch.device(device if device is not None else "cuda")
        self.optimize_memory_usage = optimize_memory_usage
        B, N, dev = self.buffer_size, self.n_envs, self.device
        self.observations = torch.zeros(B, N, self.obs_dim, dtype=torch.float32, device=dev)
        self.next_observations = None if optimize_memory_usage else torch.zeros_like(self.observations)
        self.actions = torch.zeros(B, N, self.action_dim, dtype=torch.float32, device=dev)
        self.rewards = torch.zeros(B, N, dtype=torch.float32, device=dev)
        self.dones = torch.zeros(B, N, dtype=torch.float32, device=dev)
        self.pos, self.full = 0, False
        self._segs = (_native.FwCopySeg * 5)()

    def size(self):
        """Stored transitions (all envs)."""
        return (self.buffer_size if self.full else self.pos) * self.n_envs

    def reset(self):
        self.pos, self.full = 0, False

    def add(self, obs, next_obs, action, reward, done):
        """buffers.py:222-235 for all envs of one step (device tensors [N][...], any float dtype)."""
        dev, N = self.device, self.n_envs
        f32 = lambda t, shape: torch.as_tensor(t, device=dev).to(torch.float32).reshape(shape).contiguous()
        src = [f32(obs, (N, self.obs_dim)), f32(next_obs, (N, self.obs_dim)), f32(action, (N, self.action_dim)),
               f32(reward, (N,)), f32(done, (N,))]
        p = self.pos
        nxt = self.observations[(p + 1) % self.buffer_size] if self.optimize_memory_usage else self.next_observations[p]
        dst = [self.observations[p], nxt, self.actions[p], self.rewards[p], self.dones[p]]
        for k, (a, b) in enumerate(zip(src, dst)):
            self._segs[k].src, self._segs[k].dst, self._segs[k].bytes = a.data_ptr(), b.data_ptr(), a.numel() * 4
        self._keep = src  # the copies are asynchronous: keep the sources alive until the next add
        _native.check(_native.load().fw_replay_add(self._segs, 5, _stream(dev)), "fw_replay_add")
        self.pos += 1
        if self.pos == self.buffer_size:
            self.full = True
            self.pos = 0

    # ---------------------------------------------------------------- sampling
    def sample(self, batch_size, env=None, generator=None):
        """buffers.py:95-106 / 237-254: uniform over stored transitions (excluding the slot being
        overwritten when optimize_memory_usage and full)."""
        N, dev = self.n_envs, self.device
        if self.optimize_memory_usage:
            if self.full:
                steps = (torch.randint(1, self.buffer_size, (batch_size,), device=dev, generator=generator) + self.pos) \
                    % self.buffer_size
            else:
                steps = torch.randint(0, self.pos, (batch_size,), device=dev, generator=generator)
        else:
            upper = self.buffer_size if self.full else self.pos
            steps = torch.randint(0, upper, (batch_size,), device=dev, generator=generator)
        envs = torch.randint(0, N, (batch_size,), device=dev, generator=generator)
        return self.get_samples(steps * N + envs, env)

    def get_samples(self, transitions, env=None):
        """buffers.py:239-254 for explicit transition indices k = step * n_envs + env."""
        N = self.n_envs
        k = torch.as_tensor(transitions, device=self.device).long()
        st, en = k // N, k % N
        obs = self.observations[st, en]
        if self.optimize_memory_usage:
            nxt = self.observations[(st + 1) % self.buffer_size, en]
        else:
            nxt = self.next_observations[st, en]
        rew = self.rewards[st, en]
        if env is not None:  # VecNormalize: normalise with the current statistics (buffers.py:125-138)
            obs, nxt = env.normalize_obs(obs), env.normalize_obs(nxt)
            rew = env.normalize_reward(rew) if hasattr(env, "normalize_reward") else rew
        return ReplayBufferSamples(obs, self.actions[st, en], nxt, self.dones[st, en].reshape(-1, 1),
                                   rew.reshape(-1, 1))


class OffPolicyCollector:
    """OffPolicyAlgorithm.collect_rollouts (off_policy_algorithm.py:356-470) over N device envs.

    Warm-up (``num_timesteps < learning_starts``): actions uniform over the action space
    (``action_space.sample()``, _sample_action :299-302), drawn on the device; afterwards
    ``actor(obs)`` (a callable returning actions in [-1, 1]).  The scaled action is stored
    (policies.py:309-328).  ``env`` is a FixedWingVecEnv or device VecNormalize with
    ``return_tensors=True``; with a VecNormalize the original obs / rewards are stored."""

    def __init__(self, env, buffer, learning_starts=100, actor=None, seed=0):
        self.env, self.buffer, self.learning_starts, self.actor = env, buffer, learning_starts, actor
        dev = buffer.device
        space = env.action_space
        self.low = torch.as_tensor(space.low, dtype=torch.float32, device=dev)
        self.high = torch.as_tensor(space.high, dtype=torch.float32, device=dev)
        self.num_timesteps = 0
        self.gen = torch.Generator(device=dev)
        self.gen.manual_seed(seed)
        self.last_obs = None
        self.last_original_obs = None
        self._vecnorm = hasattr(env, "get_original_obs")

    def scale_action(self, a):
        return 2.0 * ((a - self.low) / (self.high - self.low)) - 1.0

    def unscale_action(self, a):
        return self.low + (0.5 * (a + 1.0) * (self.high - self.low))

    def _warmup(self, k):
        """True if the next ``k`` steps all draw uniform warm-up actions (no policy in the loop)."""
        return self.actor is None or self.num_timesteps + k * self.env.num_envs <= self.learning_starts

    @torch.no_grad()
    def collect(self, n_steps, chunk=0):
        """``n_steps`` steps of all envs.  ``chunk`` > 1: warm-up steps (uniform actions, which do not depend
        on the observations) run ``chunk`` at a time through the fused open-loop rollout
        (FixedWingVecEnv.rollout) -- same actions, transitions and buffer contents as stepping one by one."""
        env, buf = self.env, self.buffer
        n = env.num_envs
        if self.last_obs is None:
            self.last_obs = env.reset().clone()
            self.last_original_obs = (env.get_original_obs() if self._vecnorm else self.last_obs).clone()
        done_steps = 0
        if chunk > 1 and not self._vecnorm and hasattr(env, "rollout"):
            while n_steps - done_steps >= chunk and self._warmup(chunk):
                scaled = []
                for _ in range(chunk):  # the per-step draws of the loop below, in the same order
                    u = torch.rand(n, self.low.numel(), device=buf.device, generator=self.gen)
                    scaled.append(self.scale_action(self.low + u * (self.high - self.low)))
                scaled = torch.stack(scaled)
                obs, reward, done, _ = env.rollout(self.unscale_action(scaled))
                for k in range(chunk):
                    buf.add(self.last_original_obs, obs[k], scaled[k], reward[k], done[k])
                    self.last_original_obs = obs[k]
                self.num_timesteps += n * chunk
                self.last_obs = obs[chunk - 1].clone()
                self.last_original_obs = self.last_obs
                done_steps += chunk
        for _ in range(n_steps - done_steps):
            if self.num_timesteps < self.learning_starts or self.actor is None:
                u = torch.rand(n, self.low.numel(), device=buf.device, generator=self.gen)
                unscaled = self.low + u * (self.high - self.low)
                scaled = self.scale_action(unscaled)
            else:
                scaled = self.actor(self.last_obs).clamp(-1, 1)
            action = self.unscale_action(scaled)
            new_obs, reward, done, _ = env.step(action)
            self.num_timesteps += n
            if self._vecnorm:
                new_obs_, reward_ = env.get_original_obs(), env.get_original_reward()
            else:
                new_obs_, reward_ = new_obs, reward
            buf.add(self.last_original_obs, new_obs_, scaled, reward_, done)
            self.last_obs = new_obs.clone()
            self.last_original_obs = new_obs_.clone()
        return buf
