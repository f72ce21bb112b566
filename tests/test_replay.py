"""ReplayBuffer: the CPU restatement against the reference's own buffer (tests/golden/replay.npz),
and the device buffer (one fw_replay_add launch per step) against both, bit for bit (GPU)."""
import numpy as np
import pytest
import torch

import _fixtures as F
from oracle.replay_oracle import ReplayOracle

FIELDS = ["observations", "actions", "next_observations", "dones", "rewards"]


def _adds(d):
    return [(d["add_obs"][t], d["add_next_obs"][t], d["add_action"][t], d["add_reward"][t], d["add_done"][t])
            for t in range(len(d["add_reward"]))]


@pytest.mark.parametrize("opt", [False, True])
def test_replay_oracle_matches_reference(opt):
    d = F.load("replay.npz")
    o = ReplayOracle(7, 14, 3, optimize_memory_usage=opt)
    for a in _adds(d):
        o.add(*a)
    p = "opt%d__" % int(opt)
    assert o.pos == int(d[p + "pos"]) and o.full == bool(d[p + "full"])
    for name, got in zip(FIELDS, o.get_samples(np.arange(7))):
        assert np.array_equal(got, d[p + name]), name


@pytest.mark.gpu
@pytest.mark.parametrize("opt", [False, True])
def test_device_replay_matches_reference(opt):
    from tum_adlr_deep_reinforcement_learning_amd.replay import ReplayBuffer
    from tum_adlr_deep_reinforcement_learning_amd.spaces import Box
    d = F.load("replay.npz")
    buf = ReplayBuffer(7, Box(-np.inf, np.inf, (14,)), Box(-1, 1, (3,)), device="cuda:0", n_envs=1,
                       optimize_memory_usage=opt)
    for obs, nxt, act, rew, done in _adds(d):
        t = lambda x: torch.as_tensor(np.asarray(x)).reshape(1, -1).cuda()
        buf.add(t(obs), t(nxt), t(act), t(rew), t(float(done)))
    p = "opt%d__" % int(opt)
    assert buf.pos == int(d[p + "pos"]) and buf.full == bool(d[p + "full"])
    s = buf.get_samples(torch.arange(7))
    for name, got in zip(FIELDS, s):
        assert np.array_equal(got.cpu().numpy(), d[p + name]), name


@pytest.mark.gpu
def test_sac_warmup_fill_on_device():
    """OffPolicyCollector with uniform warm-up actions over 512 real envs: the buffer holds the
    scaled actions, next_obs of step t is obs of step t+1 unless the env was reset, sampling works."""
    from tum_adlr_deep_reinforcement_learning_amd.replay import OffPolicyCollector, ReplayBuffer
    from tum_adlr_deep_reinforcement_learning_amd.vec_env import FixedWingVecEnv
    n, steps = 512, 12
    # the default action space is +-FLT_MAX, where SB3's scale_action overflows to NaN too: a SAC setup
    # uses a bounded space, here [-1, 1] scaled onto the actuator ranges (scale_space)
    unit = {i: {"low": -1.0, "high": 1.0} for i in range(3)}  # lists by index (fixed_wing.py:34-40)
    env = FixedWingVecEnv(n, config_kw={"steps_max": 8, "action": {"scale_space": True, "states": unit}},
                          sim_config_kw={"turbulence": False}, device="cuda:0", seed=3, return_tensors=True)
    buf = ReplayBuffer(n * 16, env.observation_space, env.action_space, device="cuda:0", n_envs=n)
    col = OffPolicyCollector(env, buf, learning_starts=10 ** 9, seed=1)
    col.collect(steps)
    assert buf.pos == steps and buf.size() == n * steps
    obs, nxt = buf.observations[:steps].cpu(), buf.next_observations[:steps].cpu()
    dones = buf.dones[:steps].cpu()
    cont = dones[:-1] == 0
    assert torch.isfinite(obs).all() and torch.isfinite(nxt).all()
    assert torch.equal(nxt[:-1][cont], obs[1:][cont])
    assert dones.sum() >= n  # steps_max = 8 < 12
    a = buf.actions[:steps]
    assert torch.isfinite(a).all() and float(a.abs().max()) <= 1.0 + 1e-6
    s = buf.sample(4096, generator=torch.Generator(device="cuda:0").manual_seed(0))
    assert s.observations.shape == (4096, 14) and s.rewards.shape == (4096, 1)
    env.close()
