"""CPU ORACLE for the device ReplayBuffer (test infrastructure only; never shipped).

NumPy restatement of ReplayBuffer.add / _get_samples
(magpie/libs/stable-baselines3/stable_baselines3/common/buffers.py:151-257) for one env,
pinned by tests/golden/replay.npz (the reference's own buffer, gen_rollout_golden.py).
"""
import numpy as np


class ReplayOracle:
    def __init__(self, buffer_size, obs_dim, act_dim, optimize_memory_usage=False):
        self.B, self.opt = buffer_size, optimize_memory_usage
        self.obs = np.zeros((buffer_size, obs_dim), np.float32)
        self.next_obs = None if optimize_memory_usage else np.zeros((buffer_size, obs_dim), np.float32)
        self.act = np.zeros((buffer_size, act_dim), np.float32)
        self.rew = np.zeros(buffer_size, np.float32)
        self.done = np.zeros(buffer_size, np.float32)
        self.pos, self.full = 0, False

    def add(self, obs, next_obs, action, reward, done):  # buffers.py:222-235
        self.obs[self.pos] = obs
        if self.opt:
            self.obs[(self.pos + 1) % self.B] = next_obs
        else:
            self.next_obs[self.pos] = next_obs
        self.act[self.pos] = action
        self.rew[self.pos] = reward
        self.done[self.pos] = done
        self.pos += 1
        if self.pos == self.B:
            self.full, self.pos = True, 0

    def get_samples(self, inds):  # buffers.py:239-254
        nxt = self.obs[(inds + 1) % self.B] if self.opt else self.next_obs[inds]
        return (self.obs[inds], self.act[inds], nxt, self.done[inds].reshape(-1, 1), self.rew[inds].reshape(-1, 1))
