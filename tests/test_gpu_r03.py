"""GPU tests of round 3, all through the C ABI.

  max_nfev budget     the stats word's budget bit (bit 30) and info["solver_budget_exhausted"] are
                      set exactly on the steps that end on fw_sim_config.max_nfev; the default budget
                      is never reached by the bench population
  RCCL, world 1       an in-process ``nccl`` process group on cuda:0: the VecNormalize moment
                      all-gather and the rollout-slab all_gather_into_tensor run through RCCL, and a
                      collection under the group (eager, and graphed as two graphs around the
                      collective) equals the same collection without a process group, bit for bit
  configs[3]          emulated on one GPU: eight 8192-aircraft shards at env_offset = r * 8192 collect
                      the same rollout as one 65536-aircraft batch (slabs concatenated in rank order ==
                      the 65536 slab, GAE included, bit for bit); eight shard VecNormalize records
                      merged in rank order == the whole batch's statistics
  configs[2]          65536 aircraft x the 2048-step PPO horizon, graphed collect: GAE == oracle bit for
                      bit on a sampled subset of envs (reference: buffers.py:304-333)
  curriculum          device reset draws at levels 0 / 0.25 / 0.5 / 0.75 inside the level's ranges and
                      KS-matched to the reference's draws; the reference's episodes at levels 0.25 / 0.5
                      (from its own sampled resets) replayed on the device in fp64 and fp32
  facade seed         FixedWingAircraft.seed(None) draws a fresh seed (gym seeding semantics)
"""
import socket

import numpy as np
import pytest
import torch
from torch import nn

from oracle import rollout_oracle as R
from tum_adlr_deep_reinforcement_learning_amd import config as C

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


# ---------------------------------------------------------------------------- max_nfev budget
def test_budget_bit_surfaced_in_stats_and_info():
    from tum_adlr_deep_reinforcement_learning_amd.engine import Engine
    from tum_adlr_deep_reinforcement_learning_amd.vec_env import FixedWingVecEnv
    n = 256
    env = FixedWingVecEnv(n, sim_config_kw={"turbulence": False}, device=DEV, seed=5, info_target=False)
    env.reset()
    rng = np.random.RandomState(0)
    # default budget: 40 steps, no step ends on it
    for _ in range(40):
        _, _, _, infos = env.step(rng.uniform(-1, 1, (n, 3)))
        assert not bool(Engine.budget_hits(env.engine.stats).any())
        assert not any("solver_budget_exhausted" in infos[i] for i in range(n))
    # a budget of 20 RHS evaluations (a step needs 14-44): the bit marks exactly the budget failures
    env.spec.sim.max_nfev = 20
    env.engine.update_config(env.spec.sim, env.spec)
    hits = 0
    for _ in range(10):
        _, _, _, infos = env.step(rng.uniform(-1, 1, (n, 3)))
        st = env.engine.stats
        nfev, _, failed = Engine.decode_stats(st)
        bud = Engine.budget_hits(st)
        assert torch.equal(bud, failed & (nfev >= 20))
        assert bool((nfev <= 20).all())
        b = bud.cpu().numpy()
        for i in range(n):
            assert ("solver_budget_exhausted" in infos[i]) == bool(b[i])
        hits += int(b.sum())
    assert hits > 0
    env.close()


# ---------------------------------------------------------------------------- RCCL world 1
class _Det(nn.Module):
    def __init__(self, d, a):
        super().__init__()
        from tum_adlr_deep_reinforcement_learning_amd.rollout import MlpActorCritic
        self.m = MlpActorCritic(d, a)

    def forward(self, obs):
        return self.m(obs, deterministic=True)

    def predict_values(self, obs):
        return self.m.predict_values(obs)


def _setup(n, T, seed=21, steps_max=30):
    from tum_adlr_deep_reinforcement_learning_amd.rollout import RolloutBuffer, RolloutCollector
    from tum_adlr_deep_reinforcement_learning_amd.vec_env import FixedWingVecEnv
    from tum_adlr_deep_reinforcement_learning_amd.vec_normalize import VecNormalize
    torch.manual_seed(5)
    venv = FixedWingVecEnv(n, config_kw={"steps_max": steps_max}, sim_config_kw={"turbulence": False}, device=DEV,
                           seed=seed, return_tensors=True, info_target=False)
    env = VecNormalize(venv)
    policy = _Det(env.observation_space.shape[0], env.action_space.shape[0]).to(DEV)
    buf = RolloutBuffer(T, env.observation_space, env.action_space, device=DEV, gae_lambda=0.95, gamma=0.99, n_envs=n)
    return venv, env, buf, RolloutCollector(env, policy, buf)


def _snapshot(env, buf, col):
    return [t.clone() for t in (buf.slab, buf.rewards, buf.dones, col.last_obs, col.last_dones, env.rms, env.ret)]


def test_rccl_world1_collect_equals_no_group():
    """The same collections first without a process group, then under an nccl group of size 1 on
    cuda:0, where the VecNormalize moment exchange and the slab gather go through RCCL.  In each, an
    eager collector and a graphed one (after the same warm-up) store the same rollouts bit for bit over
    two consecutive collections, and the grouped run equals the group-less one bit for bit.  Under the
    group the graphed collect is two graphs around the collective (3 host launches per step)."""
    import torch.distributed as dist
    n, T = 4096, 48
    runs = []
    for grouped in (False, True):
        if grouped:
            dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % _free_port(), rank=0, world_size=1,
                                    device_id=torch.device(DEV))
        try:
            va, ea, ba, ca = _setup(n, T)
            vb, eb, bb, cb = _setup(n, T)
            ca.collect(8)
            cb.collect(8)
            snaps = []
            for _ in range(2):
                ca.collect()
                cb.collect(graph=True)
                sa, sb = _snapshot(ea, ba, ca), _snapshot(eb, bb, cb)
                for x, y in zip(sa, sb):
                    assert torch.equal(x, y)
                snaps += sb
            assert int(bb.dones.sum()) > 0 and float(bb.log_probs.abs().max()) > 0
            snaps.append(len(cb._graphs))
            if grouped:
                assert dist.get_backend() == "nccl" and eb._parts.shape[0] == 1
                g = bb.all_gather()  # one all_gather_into_tensor on RCCL
                assert len(g.slabs) == 1 and torch.equal(g.slabs[0], bb.slab)
            va.close()
            vb.close()
        finally:
            if grouped:
                dist.destroy_process_group()
        runs.append(snaps)
    a, b = runs
    assert a[-1] == 1 and b[-1] == 2  # one graph without a group; two around the collective under one
    for x, y in zip(a[:-1], b[:-1]):
        assert torch.equal(x, y)


# ---------------------------------------------------------------------------- configs[3] on one GPU
class _Scripted(nn.Module):
    """A policy with no cross-row arithmetic (so a shard and the whole batch compute the same bits): the
    actions of step k are rows [off, off + n) of a pre-drawn global table; value and log-prob are
    elementwise functions of the observation."""

    def __init__(self, table, off, n):
        super().__init__()
        self.table, self.off, self.n, self.k = table, off, n, 0

    def forward(self, obs):
        a = self.table[self.k % self.table.shape[0], self.off:self.off + self.n]
        self.k += 1
        return a.clone(), (obs[:, 0] * 0.5)[:, None], obs[:, 1] * 0.25 - obs[:, 2]

    def predict_values(self, obs):
        return (obs[:, 0] * 0.5)[:, None]


def test_configs3_eight_shards_equal_one_batch():
    from tum_adlr_deep_reinforcement_learning_amd.rollout import GatheredRollout, RolloutBuffer, RolloutCollector
    from tum_adlr_deep_reinforcement_learning_amd.vec_env import FixedWingVecEnv
    W, n, T = 8, 8192, 64
    N = W * n
    g = torch.Generator(device=DEV)
    g.manual_seed(3)
    table = torch.rand(T, N, 3, generator=g, device=DEV) * 2.4 - 1.2  # some clipped by the action space

    def collect(off, cnt):
        env = FixedWingVecEnv(cnt, config_kw={"steps_max": 40}, sim_config_kw={"turbulence": False}, device=DEV,
                              seed=99, env_offset=off, return_tensors=True, info_target=False, lanes=1)
        buf = RolloutBuffer(T, env.observation_space, env.action_space, device=DEV, gae_lambda=0.95, gamma=0.99,
                            n_envs=cnt)
        col = RolloutCollector(env, _Scripted(table, off, cnt), buf)
        col.collect()
        out = (buf, col.last_obs.clone(), col.last_dones.clone())
        env.close()
        return out

    whole, wobs, wdone = collect(0, N)
    shards = [collect(r * n, n) for r in range(W)]
    gathered = GatheredRollout([s[0].slab for s in shards], shards[0][0])  # what the all-gather returns
    wflat = GatheredRollout([whole.slab], whole).flatten()
    for got, want in zip(gathered.flatten(), wflat):
        assert torch.equal(got, want)
    assert torch.equal(torch.cat([s[0].rewards for s in shards], 1), whole.rewards)
    assert torch.equal(torch.cat([s[0].dones for s in shards], 1), whole.dones)
    assert torch.equal(torch.cat([s[1] for s in shards], 0), wobs)
    assert torch.equal(torch.cat([s[2] for s in shards], 0), wdone)
    assert int(whole.dones.sum()) > 0  # episodes end and restart inside the horizon


def test_configs3_sharded_vecnormalize_statistics():
    """Eight shard VecNormalize wrappers whose moment records are exchanged (stacked in rank order, as
    the RCCL all-gather delivers them) hold the statistics of one VecNormalize over the whole batch,
    to rounding (the records merge in a different tree), on every rank identically."""
    from tum_adlr_deep_reinforcement_learning_amd.vec_env import FixedWingVecEnv
    from tum_adlr_deep_reinforcement_learning_amd.vec_normalize import VecNormalize
    W, n, steps = 8, 8192, 24
    N = W * n

    def make(off, cnt):
        venv = FixedWingVecEnv(cnt, config_kw={"steps_max": 15}, sim_config_kw={"turbulence": False}, device=DEV,
                               seed=7, env_offset=off, return_tensors=True, info_target=False, lanes=1)
        return venv, VecNormalize(venv)

    wv, we = make(0, N)
    sh = [make(r * n, n) for r in range(W)]
    for _, e in sh:
        e._parts = torch.empty(W, e._rec.numel(), dtype=torch.float64, device=DEV)
    we.reset()
    for _, e in sh:  # reset updates the return statistics only: exchange those records too
        e.venv.reset()
        e.old_obs = e.venv.engine.obs
    rng = torch.Generator(device=DEV)
    rng.manual_seed(1)
    for _ in range(steps):
        a = torch.rand(N, 3, generator=rng, device=DEV) * 2 - 1
        we.step(a)
        for r, (_, e) in enumerate(sh):
            e.step_async(a[r * n:(r + 1) * n])
            e.step_wait_local()
        recs = torch.stack([e._rec for _, e in sh])
        for _, e in sh:
            e._parts.copy_(recs)
            e.step_wait_finish()
    d = we.obs_dim
    for _, e in sh:
        assert torch.equal(e.rms, sh[0][1].rms)
    got, want = sh[0][1].rms.cpu().numpy(), we.rms.cpu().numpy()
    # obs mean / var and counts (the return statistics started from different reset records: skip)
    np.testing.assert_allclose(got[:2 * d + 1], want[:2 * d + 1], rtol=1e-10, atol=1e-12)
    for v, _ in sh:
        v.close()
    wv.close()


# ---------------------------------------------------------------------------- configs[2] full horizon
def test_configs2_full_2048_horizon_graphed():
    from tum_adlr_deep_reinforcement_learning_amd.rollout import MlpActorCritic, RolloutBuffer, RolloutCollector
    from tum_adlr_deep_reinforcement_learning_amd.vec_env import FixedWingVecEnv
    from tum_adlr_deep_reinforcement_learning_amd.vec_normalize import VecNormalize
    torch.manual_seed(0)
    n, T = 65536, 2048
    venv = FixedWingVecEnv(n, sim_config_kw={"turbulence": False}, device=DEV, seed=17, return_tensors=True,
                           info_target=False)
    env = VecNormalize(venv)
    policy = MlpActorCritic(env.observation_space.shape[0], env.action_space.shape[0]).to(DEV)
    buf = RolloutBuffer(T, env.observation_space, env.action_space, device=DEV, gae_lambda=0.95, gamma=0.99, n_envs=n)
    col = RolloutCollector(env, policy, buf)
    col.collect(16)
    col.collect(graph=True)
    assert buf.full and buf.pos == T
    with torch.no_grad():
        lv = policy.predict_values(col.last_obs).reshape(-1)
    idx = torch.randperm(n, generator=torch.Generator().manual_seed(4))[:512].sort().values.to(DEV)
    sub = lambda t: t[:, idx].cpu().numpy()  # noqa: E731
    a_ref, r_ref = R.gae(sub(buf.rewards), sub(buf.values), sub(buf.dones), lv[idx].cpu().numpy(),
                         col.last_dones[idx].cpu().numpy(), 0.99, 0.95)
    assert np.array_equal(sub(buf.advantages), a_ref)
    assert np.array_equal(sub(buf.returns), r_ref)
    assert bool(torch.isfinite(buf.slab).all()) and float(buf.observations.abs().max()) <= 10.0
    assert int(buf.dones.sum()) > 0 and float(buf.log_probs.abs().max()) > 0
    venv.close()


# ---------------------------------------------------------------------------- teacher-forced env step
def _device_state(eng):
    """The pre-step state of every env as the oracle's orc_env_set_state takes it (numpy, fp64 of the
    engine's values): ODE state, derived values, wind, targets, step counters, action ring, goal bits."""
    g = {name: eng.get_block(b).cpu().numpy() for name, b in
         (("ode", C.FW_BLK_ODE), ("der", C.FW_BLK_DERIVED), ("wind", C.FW_BLK_WIND), ("tgt", C.FW_BLK_TARGET),
          ("steps", C.FW_BLK_STEPS), ("ring", C.FW_BLK_ACT_RING), ("goal", C.FW_BLK_GOAL))}
    for k in ("ode", "der", "wind", "tgt", "ring"):
        g[k] = g[k].astype(np.float64)
    return g


def _force(env, g, j):
    """Teacher forcing: oracle env j continues from the device's state of env j (the device keeps the
    last `window` raw actions in slots (k - 1) % window and the last 128 goal bits newest-first)."""
    sw = int(g["steps"][0, j]) & 0xFFFFFFFF
    steps, steps_tgt = sw & 0xFFFF, sw >> 16
    window = g["ring"].shape[0] // 3
    ring = g["ring"][:, j].reshape(window, 3)
    act = [ring[(k - 1) % window] for k in range(max(1, steps - window + 1), steps + 1)]
    words = [int(w) & 0xFFFFFFFF for w in g["goal"][:, j]]
    n_goal = min(steps + 1, 128)
    bits = [(words[b // 32] >> (b % 32)) & 1 for b in range(n_goal)]  # bit 0 = newest
    env.set_state(g["ode"][:, j], g["der"][:, j], g["wind"][:, j], g["tgt"][:, j], steps, steps_tgt,
                  np.array(act).reshape(-1, 3), bits[::-1])


@pytest.mark.parametrize("precision", ["float64", "float32"])
def test_env_step_teacher_forced(precision):
    """FixedWingAircraft.step (fixed_wing.py:483-628) teacher-forced on every env-step: before each of 24
    steps the fp64 C oracle of every env is put into the device's exact pre-step state (ODE state, derived
    values, targets, counters, action ring, goal register; oracle/fw_oracle.c orc_env_set_state) and takes
    the same (fp32-rounded) action; auto-reset on, so finished episodes continue from their device reset.

    An env-step whose RK45 evaluation count differs from the oracle's is an accept/reject flip (counted,
    bounded).  On every other env-step: done and termination identical; fp64: obs and reward within 1e-9
    (1 + |ref|); fp32: obs and reward within 1e-4 (1 + |ref|) (SURVEY 8(d) gate 2 at the env level) on
    >= 99.9 % of them -- an equal count is not an equal step grid, see the gate-2 test -- and every one
    within 2e-3 (1 + |ref|); flips <= 0.5 %.  The angle of attack is weighed by its conditioning 1 / |cos beta| (round 3:
    one fp32 env-step in 49152 flew sideways and its alpha moved 0.12 rad with the reward equal to
    1.5e-6)."""
    from tum_adlr_deep_reinforcement_learning_amd.engine import Engine
    from oracle import oracle as O
    spec = C.EnvSpec(sim_config_kw={"turbulence": False})
    n = 2048 if precision == "float32" else 512
    eng = Engine(spec.sim, spec, n, device=DEV, precision=precision)
    eng.seed(11)
    eng.reset()
    gen = torch.Generator(device=DEV)
    gen.manual_seed(4)
    for _ in range(150):  # a steady-state mix: mid-episode, tumbling, freshly reset aircraft
        eng.env_step(torch.rand(n, 3, generator=gen, device=DEV, dtype=eng.dtype) * 2 - 1)
    envs = [O.OracleEnv(spec.sim.struct(), spec.struct(), spec.n_obs) for _ in range(n)]
    names = [(o["name"], o["type"]) for o in spec.cfg["observation"]["states"]]
    i_alpha, i_beta = names.index(("alpha", "state")), names.index(("beta", "state"))
    rng = np.random.RandomState(8)
    tight = 1e-9 if precision == "float64" else 1e-4
    total = flips = tight_ok = 0
    worst, worst_at = 0.0, None
    for _ in range(24):
        g = _device_state(eng)
        a = rng.uniform(-1, 1, (n, 3)).astype(np.float32).astype(np.float64)
        o, r, dn, tm = eng.env_step(torch.tensor(a, dtype=eng.dtype, device=DEV), auto_reset=True, stats=True)
        o, r = o.double().cpu().numpy(), r.double().cpu().numpy()
        dn, tm = dn.cpu().numpy().astype(bool), tm.cpu().numpy()
        to = eng.terminal_obs.double().cpu().numpy()
        nf = (eng.stats & 0xFFFF).cpu().numpy()
        for j in range(n):
            _force(envs[j], g, j)
            oo, rr, dd, tt, nfo = envs[j].step(a[j])
            total += 1
            if nfo != nf[j]:
                flips += 1
                continue
            assert dd == dn[j] and tt == tm[j], (j, dd, dn[j], tt, tm[j])
            got = to[j] if dn[j] else o[j]
            eo = np.abs(got - oo) / (1 + np.abs(oo))
            # alpha = atan2(w_r, u_r) is ill-conditioned when the aircraft flies sideways (beta near
            # +-90 deg: the x-z airspeed Va cos(beta) is small): its error is weighed by that conditioning
            eo[i_alpha] /= max(1.0, 1.0 / max(abs(np.cos(oo[i_beta])), 1e-12))
            err = max(float(eo.max()), abs(rr - r[j]) / (1 + abs(rr)))
            if err > worst:
                worst = err
                worst_at = dict(env=j, obs_entry=int(eo.argmax()), got=float(got[eo.argmax()]),
                                want=float(oo[eo.argmax()]), reward=(float(r[j]), rr), nfev=int(nfo), done=bool(dd))
            tight_ok += err <= tight
    same = total - flips
    print("teacher-forced %s: %d env-steps, %d flips; %.6f of the rest within %g, worst %.2e at %s"
          % (precision, total, flips, tight_ok / same, tight, worst, worst_at))
    if precision == "float64":
        assert flips <= 0.002 * total and tight_ok == same
    else:
        # measured (round 3): 17 flips in 49152, 99.996 % within 1e-4, worst 7.5e-4 (a sideways flyer)
        assert flips <= 0.005 * total and tight_ok >= 0.999 * same and worst <= 2e-3
    eng.close()


# ---------------------------------------------------------------------------- curriculum levels on the device
def _curriculum_spec(lvl):
    spec = C.EnvSpec(config_kw={"steps_max": 2000}, sim_config_kw={"turbulence": False})
    spec.set_curriculum_level(lvl)
    return spec


@pytest.mark.parametrize("li", [0, 1, 2, 3])
def test_curriculum_device_reset_draws(li):
    """Resets the device samples at curriculum level 0 / 0.25 / 0.5 / 0.75 (set_curriculum_level,
    fixed_wing.py:334-412; reset / sample_target, :414-481, 654-746): every draw inside the level's init
    and target ranges, and (levels > 0) the roll / pitch / Va / velocity_u and target marginals match the
    reference's 300 draws at the same level (env_curriculum.npz; two-sample KS, p > 1e-3).  The draws
    themselves differ: Philox replaces gym's np_random."""
    import _fixtures as F
    from scipy import stats
    from tum_adlr_deep_reinforcement_learning_amd.engine import Engine
    d = F.load("env_curriculum.npz")
    lvl = float(d["levels"][li])
    spec = _curriculum_spec(lvl)
    n = 8192
    eng = Engine(spec.sim, spec, n, device=DEV, precision="float64")
    eng.seed(31 + li)
    eng.reset()
    der = eng.get_block(C.FW_BLK_DERIVED).cpu().numpy()
    y = eng.get_block(C.FW_BLK_ODE).cpu().numpy()
    tgt = eng.get_block(C.FW_BLK_TARGET).cpu().numpy()
    eng.close()
    dev = np.stack([der[0], der[1], der[3], y[10]], axis=1)  # roll pitch Va u: the fixture's columns
    for k, name in ((0, "roll"), (1, "pitch"), (3, "velocity_u")):
        v = spec.sim.vars[name]
        assert np.all(dev[:, k] >= v.init_min - 1e-9) and np.all(dev[:, k] <= v.init_max + 1e-9), (name, lvl)
    for k, (lo, hi, delta) in enumerate(spec.target_sampling()):
        cur = dev[:, k if k < 2 else 2]
        low = np.maximum(lo, cur - delta) if delta is not None else np.full_like(cur, lo)
        high = np.maximum(np.minimum(hi, cur + delta), low) if delta is not None else np.full_like(cur, hi)
        assert np.all(tgt[k] >= low - 1e-9) and np.all(tgt[k] <= high + 1e-9), (k, lvl)
    ref_init, ref_tgt = d["L%d__init" % li], d["L%d__target" % li]
    if lvl == 0.0:  # collapsed ranges: every draw is the midpoint, as the reference's
        for k in (0, 1, 3):
            np.testing.assert_allclose(dev[:, k], ref_init[0, k], rtol=0, atol=1e-9)
        return
    for k in range(4):
        assert stats.ks_2samp(dev[:, k], ref_init[:, k]).pvalue > 1e-3, ("init", k, lvl)
    for k in range(3):
        assert stats.ks_2samp(tgt[k], ref_tgt[:, k]).pvalue > 1e-3, ("target", k, lvl)


@pytest.mark.parametrize("precision", ["float64", "float32"])
@pytest.mark.parametrize("li", [1, 2])
def test_curriculum_reference_episodes_replayed(li, precision):
    """The reference's episodes at curriculum level 0.25 / 0.5, each from the reference's own sampled reset
    (state, target and steady wind drawn by reset() at that level) under random actions, flown on the
    device configured at the same level: fp64 obs / rewards within 1e-6 + 1e-6 per step, fp32 within
    2e-3 (1 + |ref|) over the first 100 steps (the tolerances of the parameter-randomisation replay)."""
    import _fixtures as F
    from tum_adlr_deep_reinforcement_learning_amd.engine import Engine
    d = F.load("env_curriculum.npz")
    spec = _curriculum_spec(float(d["levels"][li]))
    g = lambda ep, k: d["L%d__ep%d__%s" % (li, ep, k)]  # noqa: E731
    eps = 3
    eng = Engine(spec.sim, spec, eps, device=DEV, precision=precision)
    init = np.stack([F.env_init(g(ep, "init")) for ep in range(eps)], axis=1)
    obs0 = eng.reset(init=init, target=np.stack([g(ep, "target0") for ep in range(eps)], axis=1))
    for ep in range(eps):
        np.testing.assert_allclose(obs0[ep].double().cpu().numpy(), g(ep, "obs")[0], rtol=1e-5, atol=1e-5)
    steps = max(len(g(ep, "rew")) for ep in range(eps)) if precision == "float64" else 100
    for s in range(steps):
        a = np.stack([g(ep, "act")[min(s, len(g(ep, "act")) - 1)] for ep in range(eps)])
        o, r, dn, _ = eng.env_step(torch.tensor(a, dtype=eng.dtype, device=DEV), auto_reset=False)
        o, r, dn = o.double().cpu().numpy(), r.double().cpu().numpy(), dn.cpu().numpy()
        for ep in range(eps):
            if s >= len(g(ep, "rew")):
                continue
            ref_o = eng.terminal_obs[ep].double().cpu().numpy() if dn[ep] else o[ep]
            want_o, want_r = g(ep, "obs")[s + 1], g(ep, "rew")[s]
            if precision == "float64":
                tol = 1e-6 + 1e-6 * s
                assert abs(r[ep] - want_r) <= tol, (ep, s)
                np.testing.assert_allclose(ref_o, want_o, rtol=1e-5, atol=tol)
            else:
                assert abs(r[ep] - want_r) <= 2e-3 * (1 + abs(want_r)), (ep, s)
                assert np.all(np.abs(ref_o - want_o) <= 2e-3 * (1 + np.abs(want_o))), (ep, s)
            assert bool(dn[ep]) == bool(g(ep, "done")[s]), (ep, s)
    eng.close()


def test_facade_seed_none_draws_a_seed():
    """FixedWingAircraft.seed(None) draws a fresh seed and returns it (gym seeding.np_random(None),
    fixed_wing.py:324-332); an explicit seed is returned as given and reproduces the sampled reset."""
    from tum_adlr_deep_reinforcement_learning_amd.fixed_wing import FixedWingAircraft
    env = FixedWingAircraft(config_kw={"steps_max": 60}, sim_config_kw={"turbulence": False}, device=DEV)
    a, b = env.seed(None)[0], env.seed()[0]
    assert a != b and 0 <= a < 2 ** 64
    assert env.seed(5) == [5]
    o1 = env.reset()
    env.seed(5)
    np.testing.assert_array_equal(env.reset(), o1)
    env.close()
