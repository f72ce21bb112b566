"""CPU ORACLE for the rollout-side kernels (test infrastructure only; never shipped).

NumPy restatements, with the reference's exact dtypes and operation order, of
  RolloutBuffer.compute_returns_and_advantage   stable_baselines3/common/buffers.py:304-333
  RolloutBuffer.swap_and_flatten                buffers.py:70-80
  RunningMeanStd.update / update_from_moments   stable_baselines3/common/running_mean_std.py:20-40
  VecNormalize.reset / step_wait / normalize_*  stable_baselines3/common/vec_env/vec_normalize.py:106-169, 209-220
(paths relative to magpie/libs/stable-baselines3/).  Pinned by tests/golden/rollout_gae.npz and
tests/golden/vecnormalize.npz, produced by running the reference's SB3 itself
(tests/golden/gen_rollout_golden.py).  Only tests/ may import this module.
"""
import numpy as np


def gae(rewards, values, starts, last_values, last_dones, gamma, gae_lambda):
    """buffers.py:304-333.  rewards/values float32 [T][N]; starts = the stored `dones` column
    ([T][N], 0/1); last_values float32 [N]; last_dones bool [N].  Returns (advantages, returns)."""
    rewards = np.asarray(rewards, np.float32)
    values = np.asarray(values, np.float32)
    dones = np.asarray(starts).astype(np.float32)  # RolloutBuffer stores dones as float32
    last_values = np.asarray(last_values, np.float32).ravel()
    last_dones = np.asarray(last_dones).astype(bool)
    T = rewards.shape[0]
    advantages = np.zeros_like(rewards)
    last_gae_lam = 0
    for step in reversed(range(T)):
        if step == T - 1:
            next_non_terminal = 1.0 - last_dones
            next_values = last_values
        else:
            next_non_terminal = 1.0 - dones[step + 1]
            next_values = values[step + 1]
        delta = rewards[step] + gamma * next_values * next_non_terminal - values[step]
        last_gae_lam = delta + gamma * gae_lambda * next_non_terminal * last_gae_lam
        advantages[step] = last_gae_lam
    return advantages, advantages + values


def swap_and_flatten(arr):
    """[T][N][...] -> [N*T][...] (env-major), buffers.py:70-80."""
    shape = arr.shape
    if len(shape) < 3:
        shape = shape + (1,)
    return arr.swapaxes(0, 1).reshape(shape[0] * shape[1], *shape[2:])


class RunningMeanStd:
    """running_mean_std.py:6-40."""

    def __init__(self, epsilon=1e-4, shape=()):
        self.mean = np.zeros(shape, np.float64)
        self.var = np.ones(shape, np.float64)
        self.count = epsilon

    def update(self, arr):
        self.update_from_moments(np.mean(arr, axis=0), np.var(arr, axis=0), arr.shape[0])

    def update_from_moments(self, batch_mean, batch_var, batch_count):
        delta = batch_mean - self.mean
        tot_count = self.count + batch_count
        new_mean = self.mean + delta * batch_count / tot_count
        m_a = self.var * self.count
        m_b = batch_var * batch_count
        m_2 = m_a + m_b + np.square(delta) * self.count * batch_count / (self.count + batch_count)
        self.mean, self.var, self.count = new_mean, m_2 / (self.count + batch_count), batch_count + self.count


def chan_merge(records):
    """Merge (n, mean, M2) moment records in order (parallel-variance formula); the
    sharded-batch equivalent of np.mean / np.var over the concatenated batch."""
    n, mean, m2 = records[0]
    for nb, mb, qb in records[1:]:
        tot = n + nb
        delta = mb - mean
        mean = mean + delta * (nb / tot)
        m2 = m2 + qb + delta * delta * (n * nb / tot)
        n = tot
    return n, mean, m2


class VecNormalizeOracle:
    """The normalisation arithmetic of VecNormalize (vec_normalize.py:106-169, 209-220) on
    explicit arrays (no wrapped env)."""

    def __init__(self, num_envs, obs_dim, training=True, norm_obs=True, norm_reward=True, clip_obs=10.0,
                 clip_reward=10.0, gamma=0.99, epsilon=1e-8):
        self.obs_rms = RunningMeanStd(shape=(obs_dim,))
        self.ret_rms = RunningMeanStd(shape=())
        self.ret = np.zeros(num_envs)
        self.training, self.norm_obs, self.norm_reward = training, norm_obs, norm_reward
        self.clip_obs, self.clip_reward, self.gamma, self.epsilon = clip_obs, clip_reward, gamma, epsilon

    def normalize_obs(self, obs):
        if not self.norm_obs:
            return obs
        return np.clip((obs - self.obs_rms.mean) / np.sqrt(self.obs_rms.var + self.epsilon), -self.clip_obs,
                       self.clip_obs).astype(np.float32)

    def normalize_reward(self, reward):
        if self.norm_reward:
            reward = np.clip(reward / np.sqrt(self.ret_rms.var + self.epsilon), -self.clip_reward, self.clip_reward)
        return reward

    def reset(self, obs):
        self.ret = np.zeros(len(self.ret))
        if self.training:
            self.ret = self.ret * self.gamma + self.ret  # _update_reward(self.ret) with ret == 0
            self.ret_rms.update(self.ret)
        return self.normalize_obs(obs)

    def step(self, obs, rews, news):
        if self.training:
            self.obs_rms.update(obs)
        obs = self.normalize_obs(obs)
        if self.training:
            self.ret = self.ret * self.gamma + rews
            self.ret_rms.update(self.ret)
        rews = self.normalize_reward(rews)
        self.ret[np.asarray(news, bool)] = 0
        return obs, rews

    def state(self):
        return np.concatenate([self.obs_rms.mean, self.obs_rms.var, [self.obs_rms.count], [self.ret_rms.mean],
                               [self.ret_rms.var], [self.ret_rms.count]])
