"""GPU: the rollout-side kernels through the C ABI.

  fw_gae            bit-exact vs the reference's own RolloutBuffer (fixtures) and vs the oracle
                    at PPO size (T = 2048)
  fw_moments / fw_rms_update / fw_vecnorm_apply (device VecNormalize)
                    vs the oracle fed the same float32 observations in float64: statistics
                    rel <= 1e-12, normalised obs within 1 float32 ulp (+1e-6 abs);
                    vs the reference fixture (whose batch moments are float32 np.mean/np.var):
                    statistics rel <= 1e-5, normalised obs abs <= 1e-3
  RolloutCollector  end to end on the real env: stored advantages == oracle GAE of the stored
                    rollout, bit for bit
"""
import ctypes

import numpy as np
import pytest
import torch

import _fixtures as F
from oracle import rollout_oracle as R

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _gae_dev(rew, val, starts, lv, ld, gamma, lam):
    from tum_adlr_deep_reinforcement_learning_amd.rollout import gae
    t = lambda a, dt: torch.tensor(np.ascontiguousarray(a), dtype=dt, device=DEV)
    adv, ret = gae(t(rew, torch.float32), t(val, torch.float32), t(starts, torch.uint8), t(lv, torch.float32),
                   t(ld, torch.uint8), gamma, lam)
    return adv.cpu().numpy(), ret.cpu().numpy()


@pytest.mark.parametrize("case", ["a", "b", "c", "d"])
def test_gae_kernel_bit_exact_vs_reference(case):
    d = F.load("rollout_gae.npz")
    g = lambda k: d[case + "__" + k]
    adv, ret = _gae_dev(g("rewards"), g("values"), g("starts"), g("last_values"), g("last_dones"), float(g("gamma")),
                        float(g("lam")))
    assert np.array_equal(adv, g("advantages"))
    assert np.array_equal(ret, g("returns"))


def test_gae_kernel_no_fma_contraction():
    """One env column of a 65536 x 256 collect on which an FMA-contracted running advantage
    (fma(coef, last, delta) in fp64) rounds 1 ulp away from numpy's separate multiply and add at step
    190 (tests/golden/gae_fma_column.npz, captured from test_c3_rollout_collector_full_size's population):
    the kernel must equal the oracle there bit for bit."""
    d = F.load("gae_fma_column.npz")
    rew, val, st = d["rewards"][:, None], d["values"][:, None], d["starts"][:, None]
    lv, ld = np.array([d["last_value"]], np.float32), np.array([d["last_done"]], np.uint8)
    adv, ret = _gae_dev(rew, val, st, lv, ld, 0.99, 0.95)
    a_ref, r_ref = R.gae(rew, val, st, lv, ld, 0.99, 0.95)
    t = int(d["t"])
    assert adv[t, 0] == a_ref[t, 0]
    assert np.array_equal(adv, a_ref) and np.array_equal(ret, r_ref)


def test_gae_kernel_ppo_size_vs_oracle():
    rng = np.random.RandomState(9)
    T, N = 2048, 4099  # ragged N (not a multiple of the block)
    rew = (rng.randn(T, N) * 2).astype(np.float32)
    val = (rng.randn(T, N) * 10).astype(np.float32)
    starts = (rng.rand(T, N) < 0.002).astype(np.uint8)
    lv = (rng.randn(N) * 10).astype(np.float32)
    ld = (rng.rand(N) < 0.01).astype(np.uint8)
    adv, ret = _gae_dev(rew, val, starts, lv, ld, 0.99, 0.95)
    a_ref, r_ref = R.gae(rew, val, starts, lv, ld, 0.99, 0.95)
    assert np.array_equal(adv, a_ref) and np.array_equal(ret, r_ref)


class _ScriptedDeviceEnv:
    """Replays recorded (obs, rew, done) as device tensors behind the VecEnv step API."""

    def __init__(self, obs, rew, done):
        from tum_adlr_deep_reinforcement_learning_amd.spaces import Box
        self.obs = torch.tensor(obs, device=DEV)
        self.rew = torch.tensor(rew.astype(np.float32), device=DEV)
        self.done = torch.tensor(done.astype(bool), device=DEV)
        self.num_envs, d = obs.shape[1], obs.shape[2]
        self.observation_space = Box(-np.inf, np.inf, (d,))
        self.action_space = Box(-1, 1, (3,))
        self.device = torch.device(DEV)
        self.return_tensors = True
        self.k = 0

    def reset(self):
        self.k = 0
        return self.obs[0]

    def step_async(self, a):
        pass

    def step_wait(self):
        k = self.k
        self.k += 1
        return self.obs[k + 1], self.rew[k], self.done[k], [{}] * self.num_envs

    def close(self):
        pass


def test_device_vecnormalize_vs_oracle_and_reference():
    from tum_adlr_deep_reinforcement_learning_amd.vec_normalize import VecNormalize
    d = F.load("vecnormalize.npz")
    n, dim = d["obs"].shape[1:]
    env = VecNormalize(_ScriptedDeviceEnv(d["obs"], d["rew"], d["done"]), gamma=float(d["gamma"]),
                       clip_obs=float(d["clip_obs"]), clip_reward=float(d["clip_reward"]), epsilon=float(d["epsilon"]),
                       return_tensors=False)
    orc = R.VecNormalizeOracle(n, dim, gamma=float(d["gamma"]), clip_obs=float(d["clip_obs"]),
                               clip_reward=float(d["clip_reward"]), epsilon=float(d["epsilon"]))
    o = env.reset()
    o_ref = orc.reset(d["obs"][0].astype(np.float64))
    np.testing.assert_allclose(o, o_ref, rtol=1.2e-7, atol=1e-6)
    np.testing.assert_allclose(o, d["norm_obs0"], atol=1e-3)
    for k in range(len(d["rew"])):
        o, r, dn, _ = env.step(np.zeros((n, 3), np.float32))
        oo, rr = orc.step(d["obs"][k + 1].astype(np.float64), d["rew"][k], d["done"][k].astype(bool))
        st = env.rms.cpu().numpy()
        np.testing.assert_allclose(st, orc.state(), rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(o, oo, rtol=1.2e-7, atol=1e-6)
        np.testing.assert_allclose(r, rr, rtol=1.2e-7, atol=1e-7)
        # the reference computes batch moments in float32 (np.mean/np.var of float32 obs)
        np.testing.assert_allclose(st, d["rms"][k], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(o, d["norm_obs"][k], atol=1e-3)
        np.testing.assert_allclose(r, d["norm_rew"][k], rtol=1e-4, atol=1e-5)


def test_rollout_collector_end_to_end():
    from tum_adlr_deep_reinforcement_learning_amd.rollout import MlpActorCritic, RolloutBuffer, RolloutCollector
    from tum_adlr_deep_reinforcement_learning_amd.vec_env import FixedWingVecEnv
    from tum_adlr_deep_reinforcement_learning_amd.vec_normalize import VecNormalize
    torch.manual_seed(0)
    n, T = 512, 96
    venv = FixedWingVecEnv(n, config_kw={"steps_max": 40}, sim_config_kw={"turbulence": False}, device=DEV, seed=4,
                           return_tensors=True)
    env = VecNormalize(venv)
    policy = MlpActorCritic(env.observation_space.shape[0], env.action_space.shape[0]).to(DEV)
    buf = RolloutBuffer(T, env.observation_space, env.action_space, device=DEV, gae_lambda=0.95, gamma=0.99, n_envs=n)
    col = RolloutCollector(env, policy, buf)
    col.collect()
    assert buf.full and buf.pos == T
    starts = buf.dones.cpu().numpy()
    assert starts.sum() >= n  # steps_max = 40 < T: every env restarted at least once
    with torch.no_grad():
        lv = policy.predict_values(col.last_obs).reshape(-1).cpu().numpy()
    a_ref, r_ref = R.gae(buf.rewards.cpu().numpy(), buf.values.cpu().numpy(), starts, lv,
                         col.last_dones.cpu().numpy(), 0.99, 0.95)
    assert np.array_equal(buf.advantages.cpu().numpy(), a_ref)
    assert np.array_equal(buf.returns.cpu().numpy(), r_ref)
    obs = buf.observations.cpu().numpy()
    assert np.isfinite(obs).all() and np.abs(obs).max() <= 10.0  # VecNormalize clip
    g = buf.all_gather()  # single process: identity gather
    batches = list(g.get(batch_size=4096))
    assert sum(len(b.observations) for b in batches) == n * T
    flat = g.flatten()
    assert np.array_equal(flat[4].cpu().numpy().ravel(), R.swap_and_flatten(buf.advantages.cpu().numpy()).ravel())
    venv.close()


@pytest.mark.parametrize("d", [7, 16, 32])
def test_fused_policy_forward_vs_torch_module(d):
    """fw_policy_forward (MlpActorCritic.collect_step: both MLPs, Gaussian sample, log-prob and clip in one
    launch) == the torch module's forward + torch.max(torch.min(...)) on the same noise draws: fp32,
    rel/abs 2e-5 (a different FMA order than the BLAS GEMMs; the fast tanh adds ~1e-7 absolute).  Ragged n
    (not a multiple of the 128-env block), random (trained-like) weights, wide inputs."""
    from tum_adlr_deep_reinforcement_learning_amd.rollout import MlpActorCritic
    torch.manual_seed(3)
    n, A = 5000 + d, 3
    pol = MlpActorCritic(d, A).to(DEV)
    with torch.no_grad():
        for prm in pol.parameters():
            prm.add_(0.3 * torch.randn_like(prm))
    obs = 3 * torch.randn(n, d, device=DEV)
    low = torch.tensor([-0.5, -1.0, 0.0], device=DEV)
    high = torch.tensor([0.5, 1.0, 1.0], device=DEV)
    assert pol.fused_ok(obs)
    torch.manual_seed(11)
    with torch.no_grad():
        a_ref, v_ref, lp_ref = pol(obs)
    torch.manual_seed(11)
    a, c, v, lp = pol.collect_step(obs, low, high)
    tol = dict(rtol=2e-5, atol=2e-5)
    torch.testing.assert_close(a, a_ref, **tol)
    torch.testing.assert_close(v, v_ref.reshape(-1), **tol)
    torch.testing.assert_close(lp, lp_ref, **tol)
    torch.testing.assert_close(c, torch.max(torch.min(a, high), low), rtol=0, atol=0)
    pol.deterministic_rollout = True
    a2, _, v2, lp2 = pol.collect_step(obs, low, high)
    with torch.no_grad():
        m_ref, _, _ = pol(obs, deterministic=True)
    torch.testing.assert_close(a2, m_ref, **tol)
    assert torch.equal(v2, v)  # the critic does not depend on the noise


@pytest.mark.parametrize("n", [1, 255, 256, 70001])
def test_moments_kernel_vs_numpy(n):
    """fw_moments (block two-pass records + two-pass record merge) vs numpy's np.mean / np.var in fp64:
    rel 1e-12, including a constant column (var exactly 0) and a column with a large offset."""
    from tum_adlr_deep_reinforcement_learning_amd import _native
    lib = _native.load()
    d = 5
    g = torch.Generator(device=DEV)
    g.manual_seed(n)
    x = torch.randn(n, d, generator=g, device=DEV)
    x[:, 2] = 0.25
    x[:, 3] = 1000.0 + x[:, 3]
    rew = torch.randn(n, generator=g, device=DEV)
    ret = torch.randn(n, generator=g, device=DEV, dtype=torch.float64)
    ret0 = ret.clone()
    ws = torch.empty(int(lib.fw_moments_workspace_bytes(n, d)), dtype=torch.uint8, device=DEV)
    out = torch.empty(1 + 2 * (d + 1), dtype=torch.float64, device=DEV)
    P = lambda t: ctypes.c_void_p(t.data_ptr())
    _native.check(lib.fw_moments(P(x), n, d, d, P(rew), P(ret), 0.99, P(ws), P(out), None), "fw_moments")
    torch.cuda.synchronize()
    xs = np.concatenate([x.cpu().double().numpy(), (ret0.cpu().numpy() * 0.99 + rew.cpu().double().numpy())[:, None]], 1)
    np.testing.assert_array_equal(ret.cpu().numpy(), xs[:, -1])
    o = out.cpu().numpy()
    assert o[0] == n
    np.testing.assert_allclose(o[1:d + 2], xs.mean(0), rtol=1e-12, atol=1e-13)
    np.testing.assert_allclose(o[d + 2:] / n, xs.var(0), rtol=1e-12, atol=1e-13)
    assert o[d + 2 + 2] == 0.0
