"""GPU tests of round 5, all through the C ABI.

  in-launch merge tree  fw_env_step's collect epilogue with ``merged`` / ``rms`` (ABI 9): the merged record
                        equals a numpy restatement of the same tree over the launch's own block records BIT
                        FOR BIT on every step (one, two and three tree levels; one lane and quads), numpy's
                        mean / var of the step's observations and returns to 1e-12, and the in-launch
                        update_from_moments equals fw_rms_update of that record bit for bit; two engines with
                        the same seed produce the same bits (the tree does not depend on block timing)
  fused collect         one graph of TWO kernels per step (policy, env step) with VecNormalize; graphed ==
                        eager bit for bit; GAE == oracle
  noise injection       set_noise after set_env_noise replaces the per-env lengths (no stale pointer: every
                        env reads the shared sequence); a full VecEnv reset and a recording-mode auto-reset end
                        a per-env injection (the env draws Philox again, as Dryden.reset(None) draws fresh noise)
"""
import ctypes

import numpy as np
import pytest
import torch

from tum_adlr_deep_reinforcement_learning_amd import config as C

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
FANIN = 64  # fw_stats::MERGE_FANIN


def _P(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _merge_node(n, m, q):
    """k_env_step's merge_node: sums in record order, each product and sum rounded (no FMA)."""
    D = m.shape[1]
    S, N = np.zeros(D), 0.0
    for k in range(len(n)):
        S = S + n[k] * m[k]
        N = N + n[k]
    mean = S / N
    M2 = np.zeros(D)
    for k in range(len(n)):
        dm = m[k] - mean
        M2 = M2 + (q[k] + n[k] * (dm * dm))
    return N, mean, M2


def _merge_tree(n, m, q):
    """fw_stats' tree: levels of 64-record groups until at most 64 records remain, then the final node."""
    levels = 0
    while len(n) > FANIN:
        out = [_merge_node(n[g:g + FANIN], m[g:g + FANIN], q[g:g + FANIN]) for g in range(0, len(n), FANIN)]
        n = np.array([o[0] for o in out])
        m = np.stack([o[1] for o in out])
        q = np.stack([o[2] for o in out])
        levels += 1
    return _merge_node(n, m, q), levels + 1


@pytest.mark.parametrize("n,lanes,levels", [(1000, 4, 1), (20037, 1, 2), (70001, 4, 3)])
def test_in_launch_merge_tree_bitwise(n, lanes, levels):
    from tum_adlr_deep_reinforcement_learning_amd import _native
    from tum_adlr_deep_reinforcement_learning_amd.vec_env import FixedWingVecEnv
    lib = _native.load()
    envs = [FixedWingVecEnv(n, config_kw={"steps_max": 12}, sim_config_kw={"turbulence": False}, device=DEV, seed=9,
                            return_tensors=True, info_target=False, lanes=lanes) for _ in range(2)]
    for v in envs:
        v.reset()
    eng = envs[0].engine
    d = eng.n_obs_values
    D = d + 1
    nrec, nmax = eng.collect_records()
    g = torch.Generator(device=DEV)
    g.manual_seed(n)
    ret0 = torch.randn(n, generator=g, device=DEV, dtype=torch.float64)
    rms0 = torch.rand(2 * d + 4, generator=g, device=DEV, dtype=torch.float64) + 0.5
    bufs = []
    for v in envs:
        bufs.append(dict(ret=ret0.clone(), rms=rms0.clone(),
                         rec=torch.full((nmax * (1 + 2 * D),), float("nan"), dtype=torch.float64, device=DEV),
                         merged=torch.full((1 + 2 * D,), float("nan"), dtype=torch.float64, device=DEV),
                         ctrl=torch.zeros(2, dtype=torch.int32, device=DEV)))
    gamma = 0.99
    for k in range(14):  # episodes end at step 12: done envs reset inside the window
        a = torch.rand(n, 3, generator=g, device=DEV) * 2 - 1
        ret_before = bufs[0]["ret"].clone()
        rms_before = bufs[0]["rms"].clone()
        outs = []
        for v, b in zip(envs, bufs):
            v.engine.set_collect_epilogue(ret=b["ret"], gamma=gamma, records=b["rec"], row_ctrl=b["ctrl"],
                                          merged=b["merged"], rms=b["rms"])
            outs.append(v.engine.env_step(a))
            v.engine.set_collect_epilogue()
        torch.cuda.synchronize()
        b = bufs[0]
        # the tree over the launch's own block records, restated in numpy: bit for bit
        R = b["rec"][:nrec * (1 + 2 * D)].reshape(1 + 2 * D, nrec).cpu().numpy()
        (N, mean, M2), lv = _merge_tree(R[0], R[1:D + 1].T, R[D + 1:].T)
        assert lv == levels
        got = b["merged"].cpu().numpy()
        assert got[0] == N == n
        assert np.array_equal(got[1:D + 1], mean) and np.array_equal(got[D + 1:], M2), k
        # ... and numpy's statistics of the step
        obs, rew, done, _ = outs[0]
        r_new = ret_before.cpu().numpy() * gamma + rew.cpu().numpy().astype(np.float32).astype(np.float64)
        xs = np.concatenate([obs.cpu().numpy().astype(np.float32).astype(np.float64), r_new[:, None]], 1)
        np.testing.assert_allclose(got[1:D + 1], xs.mean(0), rtol=1e-12, atol=1e-13)
        np.testing.assert_allclose(got[D + 1:] / n, xs.var(0), rtol=1e-12, atol=1e-13)
        # the in-launch update_from_moments == fw_rms_update of the merged record
        want = rms_before.clone()
        _native.check(lib.fw_rms_update(_P(b["merged"]), 1, d, 1, _P(want), 1, 1, None), "fw_rms_update")
        torch.cuda.synchronize()
        assert torch.equal(b["rms"], want) and not torch.equal(b["rms"], rms_before)
        # the second engine (same seed, same actions): the same bits
        for f in ("merged", "rms", "ret"):
            assert torch.equal(bufs[1][f], b[f]), f
        assert int(b["ctrl"][0]) == k + 1
    for v in envs:
        v.close()


def test_fused_collect_is_two_launches_and_equals_eager():
    """With VecNormalize the fused collect step is one graph of two kernels (fw_collect_policy, fw_env_step
    merging + updating the statistics in its own launch); graphed == eager bit for bit; GAE == oracle; the
    statistics equal the three-launch form (merge as its own launch) to rounding."""
    from oracle import rollout_oracle as R
    from test_gpu_r04 import _collect_setup
    va, ea, ba, ca = _collect_setup(2048, 40)
    vb, eb, bb, cb = _collect_setup(2048, 40)
    vc, ec, bc, cc = _collect_setup(2048, 40)
    ec.merge_in_launch = False
    for c in (ca, cb, cc):
        torch.manual_seed(40)
        c.collect(8)
    for i in range(2):
        for c, gr in ((ca, False), (cb, True), (cc, True)):
            torch.manual_seed(41 + i)
            c.collect(graph=gr)
        for f in ("slab", "rewards", "dones"):
            assert torch.equal(getattr(ba, f), getattr(bb, f)), f
        assert torch.equal(ca.last_obs, cb.last_obs) and torch.equal(ea.rms, eb.rms) and torch.equal(ea.ret, eb.ret)
        np.testing.assert_allclose(eb.rms.cpu().numpy(), ec.rms.cpu().numpy(), rtol=1e-9, atol=1e-12)
    nodes = cb.graph_nodes()
    assert len(nodes) == 1 and nodes[0].count(0) == 2, nodes
    assert cc.graph_nodes()[0].count(0) == 3
    with torch.no_grad():
        lv = cb.policy.predict_values(cb.last_obs).reshape(-1).cpu().numpy()
    a_ref, _ = R.gae(bb.rewards.cpu().numpy(), bb.values.cpu().numpy(), bb.dones.cpu().numpy(), lv,
                     cb.last_dones.cpu().numpy(), 0.99, 0.95)
    assert np.array_equal(bb.advantages.cpu().numpy(), a_ref)
    for v in (va, vb, vc):
        v.close()


# ---------------------------------------------------------------------------- noise injection lifetime
_STATE = {"roll": 0.2, "pitch": 0.05, "yaw": 0.0, "omega_p": 0.0, "omega_q": 0.0, "omega_r": 0.0,
          "position_n": 0.0, "position_e": 0.0, "position_d": -50.0, "velocity_u": 19.0, "velocity_v": 0.0,
          "velocity_w": 0.5, "wind": [0.0, 0.0, 0.0],
          "elevon_right": (0.0, 0.0), "elevon_left": (0.0, 0.0), "throttle": (0.5, 0.0)}


def test_set_noise_after_set_env_noise_reads_the_shared_sequence():
    """set_env_noise on a subset, then set_noise(shared): every env flies on the shared sequence (the
    handle drops the per-env lengths with the old buffer), equal to an engine that only saw set_noise."""
    from tum_adlr_deep_reinforcement_learning_amd.engine import Engine
    spec = C.build_sim(config_kw={"turbulence": True, "turbulence_sim_length": 300, "turbulence_intensity": "severe"})
    n = 64
    z = np.random.RandomState(5).standard_normal((4, 300))
    zj = np.random.RandomState(6).standard_normal((4, 40))
    a, b = (Engine(spec, None, n, device=DEV, precision="float64") for _ in range(2))
    a.set_env_noise([3, 17], zj)
    a.set_noise(z)
    b.set_noise(z)
    for e in (a, b):
        e.seed(1)
        e.reset(want_obs=False)
    rng = np.random.RandomState(0)
    for _ in range(60):
        cmd = torch.tensor(rng.uniform(-0.2, 0.2, (n, 3)) + [0.0, 0.0, 0.6], device=DEV)
        a.sim_step(cmd)
        b.sim_step(cmd)
    assert torch.equal(a.get_block(C.FW_BLK_ODE), b.get_block(C.FW_BLK_ODE))
    a.close()
    b.close()


def test_set_env_noise_keeps_a_set_noise_injection():
    """A per-env injection on top of a set_noise buffer: the other envs keep reading the set_noise sequence."""
    from tum_adlr_deep_reinforcement_learning_amd.engine import Engine
    spec = C.build_sim(config_kw={"turbulence": True, "turbulence_sim_length": 300, "turbulence_intensity": "severe"})
    n = 64
    z = np.random.RandomState(5).standard_normal((4, 300))
    zj = np.random.RandomState(6).standard_normal((4, 40))
    a, b = (Engine(spec, None, n, device=DEV, precision="float64") for _ in range(2))
    for e in (a, b):
        e.set_noise(z)
    a.set_env_noise([3], zj)
    for e in (a, b):
        e.seed(1)
        e.reset(want_obs=False)
    rng = np.random.RandomState(0)
    for _ in range(60):
        cmd = torch.tensor(rng.uniform(-0.2, 0.2, (n, 3)) + [0.0, 0.0, 0.6], device=DEV)
        a.sim_step(cmd)
        b.sim_step(cmd)
    ya, yb = a.get_block(C.FW_BLK_ODE), b.get_block(C.FW_BLK_ODE)
    others = torch.arange(n, device=DEV) != 3
    assert torch.equal(ya[:, others], yb[:, others]) and not torch.equal(ya[:, 3], yb[:, 3])
    a.close()
    b.close()


@pytest.mark.parametrize("record", [False, True])
def test_reset_ends_per_env_injection(record):
    """After env_method("reset", indices=[j], turbulence_noise=Z): a full VecEnv reset (record=False) or the
    recording step's auto-reset (record=True) ends the injection -- env j's next episode equals the one of a
    run that never injected, as the reference's worker resets with Dryden.reset(None)."""
    from tum_adlr_deep_reinforcement_learning_amd.vec_env import FixedWingVecEnv
    n, j, steps_max = 8, 5, 120  # (turbulence chunk = steps_max; shorter chunks need the stateful filter)
    z = np.random.RandomState(2).standard_normal((4, 50))
    runs = []
    for inject in (True, False):
        env = FixedWingVecEnv(n, config_kw={"steps_max": steps_max},
                              sim_config_kw={"turbulence": True, "turbulence_intensity": "moderate"},
                              device=DEV, precision="float64", seed=3, return_tensors=True, info_target=False,
                              record_history=record)
        env.reset()
        env.env_method("reset", state=_STATE, indices=[j], **({"turbulence_noise": z} if inject else {}))
        rng = np.random.RandomState(9)
        obs = []
        if record:  # run env j's episode out: the recording step resets it (eng.reset(mask=done))
            for _ in range(steps_max):
                env.step(torch.tensor(rng.uniform(-1, 1, (n, 3)), device=DEV))
        else:
            env.reset()
        for _ in range(30):
            o, _, _, _ = env.step(torch.tensor(rng.uniform(-1, 1, (n, 3)), device=DEV))
            obs.append(o.cpu().numpy().copy())
        runs.append(np.array(obs))
        env.close()
    assert np.array_equal(runs[0][:, j], runs[1][:, j])


# ---------------------------------------------------------------------------- Dryden filter bank (short chunks)
def _rel(a, b):
    return np.abs(a - b) / (np.abs(b) + 1e-3)


@pytest.mark.parametrize("lanes", [1, 4])
@pytest.mark.parametrize("name", ["pid_L20", "rand_L8", "pid_L40"])
def test_short_chunk_dryden_trajectory_fp64(name, lanes):
    """PyFly trajectories whose turbulence chunk (8 / 20 / 40 steps) is too short for the 2-tap FIR: the device's
    filter bank (state carried step to step and across chunks) stays on the REFERENCE's trajectory
    (pyfly_short_turb.npz) within 1e-7, nfev identical, on both integrators."""
    import _fixtures as F
    from tum_adlr_deep_reinforcement_learning_amd.engine import Engine
    d = F.load("pyfly_short_turb.npz")
    g = lambda k: d[name + "__" + k]
    spec = C.build_sim(config_kw={"turbulence": True, "turbulence_sim_length": int(g("L"))})
    assert spec.struct().dryden_state == 1
    eng = Engine(spec, None, 1, device=DEV, precision="float64", lanes=lanes)
    eng.set_block(C.FW_BLK_ODE, g("y")[0][:, None])
    der = np.zeros((8, 1))
    der[:6, 0] = g("derived")[0][:6]
    eng.set_block(C.FW_BLK_DERIVED, der)
    eng.set_block(C.FW_BLK_WIND, g("wind")[:, None])
    eng.set_block(C.FW_BLK_STEPS, np.zeros(1, np.int32))
    eng.set_noise(g("noise")[None])
    cmds = torch.tensor(g("cmd"), dtype=torch.float64, device=DEV)
    worst, nfev_ok = 0.0, 0
    for s in range(len(cmds)):
        _, term = eng.sim_step(cmds[s:s + 1], stats=True)
        assert (int(term[0]) == 0) == bool(g("success")[s]), s
        nfev_ok += int(eng.stats[0] & 0xFFFF) == int(g("nfev")[s])
        y = eng.get_block(C.FW_BLK_ODE)[:, 0].cpu().numpy()
        worst = max(worst, _rel(y, g("y")[s + 1]).max())
    assert worst < 1e-7, worst
    assert nfev_ok >= len(cmds) - 2
    eng.close()


@pytest.mark.parametrize("precision", ["float64", "float32"])
@pytest.mark.parametrize("name", ["rand_40", "pid_40"])
def test_short_chunk_dryden_env_episode(name, precision):
    """FixedWingAircraft episodes with steps_max 40 (turbulence chunk 40: the filter bank) vs the reference's
    own episode (env_short_turb.npz): fp64 obs / reward within the env-sequence tolerance, fp32 within 2e-3."""
    import _fixtures as F
    from tum_adlr_deep_reinforcement_learning_amd.engine import Engine
    d = F.load("env_short_turb.npz")
    g = lambda k: d[name + "__" + k]
    ckw = {"steps_max": 40} if bool(g("scale_space")) else {"steps_max": 40, "action": {"scale_space": False}}
    spec = C.EnvSpec(config_kw=ckw, sim_config_kw={"turbulence": True, "turbulence_intensity": "light"})
    eng = Engine(spec.sim, spec, 1, device=DEV, precision=precision)
    eng.set_noise(g("noise")[None])
    obs0 = eng.reset(init=F.env_init(g("init"))[:, None], target=g("target0")[:, None]).double().cpu().numpy()[0]
    np.testing.assert_allclose(obs0, g("obs")[0], rtol=1e-5 if precision == "float32" else 1e-12, atol=1e-6)
    acts = torch.tensor(g("act"), dtype=eng.dtype, device=DEV)
    for s in range(len(acts)):
        obs, rew, done, _ = eng.env_step(acts[s:s + 1], auto_reset=False)
        assert bool(done[0]) == bool(g("done")[s]), s
        o, r = obs.double().cpu().numpy()[0], float(rew[0])
        if precision == "float64":
            tol = 1e-6 + 1e-6 * s
            assert abs(r - g("rew")[s]) <= tol, (s, r)
            np.testing.assert_allclose(o, g("obs")[s + 1], rtol=1e-5, atol=tol)
        else:
            assert abs(r - g("rew")[s]) <= 2e-3 * (1 + abs(g("rew")[s])), (s, r)
            np.testing.assert_allclose(o, g("obs")[s + 1], rtol=2e-3, atol=2e-3)
        if bool(done[0]):
            break
    eng.close()


def test_short_chunk_dryden_philox_equals_injected_over_resets():
    """L = 3 (state carried into later chunks), 64 aircraft, Philox noise, two episodes (the reset restarts
    the filters): the device drawing its own noise equals a second engine fed the host restatement of the
    same Philox draws (oracle/rng_oracle.py) through fw_set_noise (fp64, 1e-9 per step)."""
    from oracle import rng_oracle as RNG
    from tum_adlr_deep_reinforcement_learning_amd.engine import Engine
    spec = C.build_sim(config_kw={"turbulence": True, "turbulence_sim_length": 3, "turbulence_intensity": "severe"})
    assert spec.struct().dryden_state == 1 and spec.struct().dryden_ncut > 1
    n, seed = 64, 91
    a, b = (Engine(spec, None, n, device=DEV, precision="float64") for _ in range(2))
    for e in (a, b):
        e.seed(seed)
    rng = np.random.RandomState(0)
    lo, hi = np.array([-0.5236, -0.5672, 0.0]), np.array([0.6109, 0.5672, 1.0])
    for episode, steps in ((1, 40), (2, 25)):
        b.set_noise(RNG.turbulence_noise(seed, np.arange(n), episode, steps + 2))
        a.reset(want_obs=False)
        b.reset(want_obs=False)
        alive = np.ones(n, bool)
        for s in range(steps):
            cmd = torch.tensor(rng.uniform(0.3 * lo, 0.3 * hi, (n, 3)), device=DEV)
            _, ta = a.sim_step(cmd)
            _, tb = b.sim_step(cmd)
            ta, tb = ta.cpu().numpy(), tb.cpu().numpy()
            assert np.array_equal(ta[alive], tb[alive]), s
            alive &= ta == 0
            ya, yb = a.get_block(C.FW_BLK_ODE).cpu().numpy(), b.get_block(C.FW_BLK_ODE).cpu().numpy()
            assert _rel(ya[:, alive], yb[:, alive]).max() < 1e-9 * (1 + s), (episode, s)
        assert alive.mean() > 0.5
    a.close()
    b.close()


def test_set_attr_any_attribute():
    """SubprocVecEnv.set_attr sets ANY attribute on the chosen workers (subproc_vec_env.py:156-161): names the
    device step does not read are kept per env on the host and read back by get_attr; curriculum_level goes to
    the device configuration; compiled configuration attributes are refused loudly."""
    from tum_adlr_deep_reinforcement_learning_amd.vec_env import FixedWingVecEnv
    env = FixedWingVecEnv(8, sim_config_kw={"turbulence": False}, device=DEV, return_tensors=True, info_target=False)
    env.reset()
    env.set_attr("eval_tag", "a", indices=[1, 2])
    assert env.get_attr("eval_tag", indices=[1, 2]) == ["a", "a"]
    with pytest.raises(AttributeError):
        env.get_attr("eval_tag", indices=[0])
    env.set_attr("render_on_reset", False)
    assert env.get_attr("render_on_reset") == [False] * 8
    with pytest.raises(NotImplementedError):
        env.set_attr("render_on_reset", True)
    with pytest.raises(AttributeError):
        env.set_attr("cfg", {})
    env.set_attr("curriculum_level", 0.5)
    assert env.get_attr("curriculum_level") == [0.5] * 8
    env.step(torch.zeros(8, 3, device=DEV))  # the env still steps
    env.close()


def _goal_spec():
    """success_streak_req 5 at 60 % with wide bounds: random actions reach the goal often."""
    ckw = {"steps_max": 400, "target": {"on_success": "done", "success_streak_fraction": 0.6, "success_streak_req": 5,
                                        "states": {0: {"bound": 60}, 1: {"bound": 60}, 2: {"bound": 20}}}}
    return C.EnvSpec(config_kw=ckw, sim_config_kw={"turbulence": False})


def test_goal_history_block_transfer():
    """FW_BLK_GOAL (the 128-bit "all" register of the ABI) over the round-5 goal history (nibble ring by lifetime
    position + window counts + entry count): bits before an episode's first entry read 0; copying the blocks
    into a handle whose lifetime counter differs (FW_BLK_STEPS first, then the rings) reproduces the register
    and every following step bit for bit, successes (the streak window) included."""
    from tum_adlr_deep_reinforcement_learning_amd.engine import Engine
    spec = _goal_spec()
    n = 512
    a, b = (Engine(spec.sim, spec, n, device=DEV, precision="float64") for _ in range(2))
    a.seed(3)
    b.seed(4)
    a.reset()
    b.reset()
    gen = torch.Generator(device=DEV)
    gen.manual_seed(9)
    rnd = lambda: torch.rand(n, 3, generator=gen, device=DEV, dtype=torch.float64) * 2 - 1  # noqa: E731
    succ = 0
    for _ in range(60):
        _, _, _, t = a.env_step(rnd())
        succ += int((t == C.FW_TERM_SUCCESS).sum())
    for _ in range(23):
        b.env_step(rnd())
    assert succ > 0
    reg = a.get_block(C.FW_BLK_GOAL).cpu().numpy().astype(np.uint32)
    steps = (a.get_block(C.FW_BLK_STEPS)[0].cpu().numpy().astype(np.uint32) & 0xFFFF).astype(np.int64)
    for i in range(n):  # auto-reset: every episode's history has steps + 1 entries
        bits = np.array([(int(reg[j // 32, i]) >> (j % 32)) & 1 for j in range(128)])
        assert not bits[steps[i] + 1:].any(), i
    blocks = [C.FW_BLK_ODE, C.FW_BLK_DERIVED, C.FW_BLK_WIND, C.FW_BLK_TARGET, C.FW_BLK_STEPS, C.FW_BLK_COMMAND,
              C.FW_BLK_ACT_RING, C.FW_BLK_GOAL]
    for blk in blocks:
        b.set_block(blk, a.get_block(blk))
    assert torch.equal(b.get_block(C.FW_BLK_GOAL), a.get_block(C.FW_BLK_GOAL))
    succ = 0
    for s in range(40):
        act = rnd()
        oa, ra, da, ta = (x.clone() for x in a.env_step(act, auto_reset=False))
        ob, rb, db, tb = b.env_step(act, auto_reset=False)
        assert torch.equal(ta, tb) and torch.equal(da, db), s
        assert torch.equal(ra, rb) and torch.equal(oa, ob), s
        assert torch.equal(a.get_block(C.FW_BLK_GOAL), b.get_block(C.FW_BLK_GOAL)), s
        succ += int((ta == C.FW_TERM_SUCCESS).sum())
    assert succ > 0


@pytest.mark.parametrize("precision", ["float64", "float32"])
@pytest.mark.parametrize("name", ["rand_off", "pid_off", "rand_light"])
def test_env_potential_reward_episode(name, precision):
    """reward.form "potential" on the device (State::shp, reward_of) against the reference's own episodes
    (env_potential.npz): done flags identical; fp64 rewards within 1e-6 + 1e-6 / step (the env-level gate of
    the other episode fixtures), fp32 within 1e-3 (1 + |r|) -- the shaping difference of two fp32 errors."""
    import _fixtures as F
    from tum_adlr_deep_reinforcement_learning_amd.engine import Engine
    d = F.load("env_potential.npz")
    g = lambda k: d[name + "__" + k]  # noqa: E731
    ckw = {"steps_max": 300, "reward": {"form": "potential"}}
    if not bool(g("scale_space")):
        ckw["action"] = {"scale_space": False}
    turb = bool(g("turb"))
    spec = C.EnvSpec(config_kw=ckw, sim_config_kw={"turbulence": turb, "turbulence_intensity": "light"})
    eng = Engine(spec.sim, spec, 1, device=DEV, precision=precision)
    if turb:
        eng.set_noise(g("noise")[None])
    eng.reset(init=F.env_init(g("init"))[:, None], target=g("target0")[:, None])
    acts = torch.tensor(g("act"), dtype=eng.dtype, device=DEV)
    for s in range(len(acts)):
        _, rew, done, _ = eng.env_step(acts[s:s + 1], auto_reset=False)
        assert bool(done[0]) == bool(g("done")[s]), s
        r, ref = float(rew[0]), float(g("rew")[s])
        tol = (1e-6 + 1e-6 * s) if precision == "float64" else 1e-3 * (1 + abs(ref))
        assert abs(r - ref) <= tol, (s, r, ref)
        if bool(done[0]):
            break
    eng.close()


def test_target_resample_every():
    """target.resample_every (fixed_wing.py:570-574, sample_target :654-746): after every `resample_every` steps
    with the same targets the env draws new ones -- U(low, high) narrowed to the post-step value -+ delta --
    and the target step count restarts (FW_BLK_STEPS >> 16).  The constant-class roll / pitch targets change
    exactly at those steps and stay inside their intervals; a second engine with the same seed draws the same
    targets (the reference draws from np_random: distribution-level parity only, parity unpinned)."""
    from tum_adlr_deep_reinforcement_learning_amd.engine import Engine
    R = 25
    spec = C.EnvSpec(config_kw={"steps_max": 400, "target": {"resample_every": R}},
                     sim_config_kw={"turbulence": False})
    assert spec.struct().resample_every == R
    n = 256
    a, b = (Engine(spec.sim, spec, n, device=DEV, precision="float64") for _ in range(2))
    for e in (a, b):
        e.seed(21)
        e.reset()
    gen = torch.Generator(device=DEV)
    gen.manual_seed(5)
    e = spec.struct()
    lo, hi, dl = (np.array(list(v))[:2] for v in (e.target_low, e.target_high, e.target_delta))
    alive = np.ones(n, bool)
    tprev = a.get_block(C.FW_BLK_TARGET).cpu().numpy()
    changes = 0
    for s in range(1, 3 * R + 1):
        act = torch.rand(n, 3, generator=gen, device=DEV, dtype=torch.float64) * 0.2 - 0.1  # gentle: few failures
        _, _, da, _ = a.env_step(act, auto_reset=False)
        b.env_step(act, auto_reset=False)
        alive &= ~da.cpu().numpy().astype(bool)
        t = a.get_block(C.FW_BLK_TARGET).cpu().numpy()
        der = a.get_block(C.FW_BLK_DERIVED).cpu().numpy()
        st = (a.get_block(C.FW_BLK_STEPS)[0].cpu().numpy().astype(np.int64) >> 16) & 0xFFFF
        assert torch.equal(a.get_block(C.FW_BLK_TARGET), b.get_block(C.FW_BLK_TARGET)), s
        idx = np.nonzero(alive)[0]
        moved = np.any(t[:2, idx] != tprev[:2, idx], axis=0)
        if s % R == 0:
            assert moved.all(), s
            assert (st[idx] == 0).all(), s
            vals = der[:2, idx]  # roll, pitch after the step
            l2 = np.maximum(lo[:, None], vals - dl[:, None])
            h2 = np.maximum(np.minimum(hi[:, None], vals + dl[:, None]), l2)
            assert np.all(t[:2, idx] >= l2 - 1e-12) and np.all(t[:2, idx] <= h2 + 1e-12), s
            changes += 1
        else:
            assert not moved.any(), s
            assert (st[idx] == s % R).all(), s
        tprev = t
    assert changes == 3 and alive.sum() > n // 2
    a.close()
    b.close()


def test_reward_randomize_scaling(tmp_path):
    """reward.randomize_scaling (fixed_wing.py:473-479): a factor with "scaling": [low, high] gets a new
    U(low, high) scaling at every reset (Philox stream 7 on the device; the reference draws from np_random, so
    parity is distribution-level: unpinned).  With the roll error as the only reward term the scaling each env
    used is |error| / -reward: constant within an episode, inside [low, high], spread over the envs, redrawn by
    a reset, and the same bits on a second engine with the same seed."""
    from tum_adlr_deep_reinforcement_learning_amd.engine import Engine
    import json
    from tum_adlr_deep_reinforcement_learning_amd import defaults
    lo, hi = 0.5, 2.0
    cfg = defaults.default_env_config()
    cfg["steps_max"] = 400
    cfg["reward"].update({"form": "absolute", "randomize_scaling": True,
                          "terms": [{"function_class": "linear", "weight": 1.0}],
                          "factors": [{"name": "roll", "class": "state", "type": "error", "function_class": "linear",
                                       "scaling": [lo, hi], "shaping": False, "sign": -1}]})
    path = tmp_path / "fixed_wing_config.json"
    path.write_text(json.dumps(cfg))
    spec = C.EnvSpec(config_path=str(path), sim_config_kw={"turbulence": False})
    assert spec.struct().rew[0].randomize == 1
    n = 128
    a, b = (Engine(spec.sim, spec, n, device=DEV, precision="float64") for _ in range(2))
    for e in (a, b):
        e.seed(8)
        e.reset()
    gen = torch.Generator(device=DEV)
    gen.manual_seed(2)

    def scalings(steps):
        seen = np.full((steps, n), np.nan)
        alive = np.ones(n, bool)
        for s in range(steps):
            act = torch.rand(n, 3, generator=gen, device=DEV, dtype=torch.float64) * 0.2 - 0.1
            _, ra, da, _ = a.env_step(act, auto_reset=False)
            ra = ra.clone()
            _, rb, _, _ = b.env_step(act, auto_reset=False)
            assert torch.equal(ra, rb), s
            alive &= ~da.cpu().numpy().astype(bool)
            t = a.get_block(C.FW_BLK_TARGET)[0].cpu().numpy()
            roll = a.get_block(C.FW_BLK_DERIVED)[0].cpu().numpy()
            err = np.abs((roll - t + np.pi) % (2 * np.pi) - np.pi)
            r = ra.cpu().numpy()
            ok = alive & (err > 1e-3)
            seen[s, ok] = err[ok] / -r[ok]
        return seen

    s1 = scalings(20)
    per_env = np.nanmedian(s1, axis=0)
    dev = np.nanmax(np.abs(s1 - per_env) / per_env, axis=0)
    assert np.nanmax(dev) < 1e-9
    got = per_env[~np.isnan(per_env)]
    assert len(got) > n // 2 and got.min() >= lo and got.max() <= hi and got.std() > 0.2
    for e in (a, b):
        e.reset()
    s2 = np.nanmedian(scalings(5), axis=0)
    both = ~np.isnan(per_env) & ~np.isnan(s2)
    assert both.sum() > n // 2 and np.mean(np.abs(s2[both] - per_env[both]) > 1e-6) > 0.9  # redrawn
    a.close()
    b.close()


def _intwin_spec(steps_max=300, scale_space=True):
    import copy
    from test_golden_r05 import INTWIN_KW
    ckw = copy.deepcopy(INTWIN_KW)
    ckw["steps_max"] = steps_max
    if not scale_space:
        ckw["action"] = {"scale_space": False}
    return C.EnvSpec(config_kw=ckw, sim_config_kw={"turbulence": False})


@pytest.mark.parametrize("precision", ["float64", "float32"])
@pytest.mark.parametrize("name", ["rand", "pid", "rand_hot", "fail_late", "fail_va"])
def test_env_integration_window_episode(name, precision):
    """integration_window 10: "integrator" observations and "int_error" rewards on the device (State::iws /
    iwr) against the reference's own episodes (env_intwin.npz, fail_va ending in a Va constraint violation):
    fp64 observations and rewards within 1e-6 + 1e-6 / step, fp32 within 2e-3 (1 + |ref|)."""
    import _fixtures as F
    from test_golden_r05 import intwin_config_kw
    from tum_adlr_deep_reinforcement_learning_amd.engine import Engine
    d = F.load("env_intwin.npz")
    g = lambda k: d[name + "__" + k]  # noqa: E731
    spec = C.EnvSpec(config_kw=intwin_config_kw(d, name), sim_config_kw={"turbulence": False})
    eng = Engine(spec.sim, spec, 1, device=DEV, precision=precision)
    obs0 = eng.reset(init=F.env_init(g("init"))[:, None], target=g("target0")[:, None])
    f64 = precision == "float64"
    np.testing.assert_allclose(obs0[0].double().cpu().numpy(), g("obs")[0], rtol=1e-12 if f64 else 1e-5, atol=1e-6)
    acts = torch.tensor(g("act"), dtype=eng.dtype, device=DEV)
    for s in range(len(acts)):
        obs, rew, done, _ = eng.env_step(acts[s:s + 1], auto_reset=False)
        assert bool(done[0]) == bool(g("done")[s]), s
        r, ref = float(rew[0]), float(g("rew")[s])
        o = obs[0].double().cpu().numpy()
        if f64:
            tol = 1e-6 + 1e-6 * s
            assert abs(r - ref) <= tol, (s, r, ref)
            np.testing.assert_allclose(o, g("obs")[s + 1], rtol=1e-5, atol=tol)
        else:
            assert abs(r - ref) <= 2e-3 * (1 + abs(ref)), (s, r, ref)
            np.testing.assert_allclose(o, g("obs")[s + 1], rtol=2e-3, atol=2e-3)
        if bool(done[0]):
            break
    eng.close()


def test_integration_window_reset_reads_previous_history():
    """FixedWingAircraft.reset observes before it replaces self.history (fixed_wing.py:452-459): an
    "integrator" entry of a reset observation is the PREVIOUS episode's window sum padded as at steps_count 0
    (the current error x W at the first reset).  Device (fp64) against the oracle: an explicit second reset
    after 16 steps, and the auto-reset at steps_max (only the integrator entries: the new episode's other
    entries come from the device's own draws)."""
    import _fixtures as F
    from oracle import oracle as O
    from tum_adlr_deep_reinforcement_learning_amd.engine import Engine
    d = F.load("env_intwin.npz")
    spec = _intwin_spec(17)
    ints = [o for o in range(spec.n_obs) if spec.struct().obs[o].kind == C.FW_OBS_TARGET_INT]
    eng = Engine(spec.sim, spec, 1, device=DEV, precision="float64")
    ora = O.OracleEnv(spec.sim.struct(), spec.struct(), spec.n_obs)
    iA, tA = F.env_init(d["rand__init"]), d["rand__target0"]
    iB, tB = F.env_init(d["pid__init"]), d["pid__target0"]
    np.testing.assert_allclose(eng.reset(init=iA[:, None], target=tA[:, None])[0].cpu().numpy(), ora.reset(iA, tA),
                               rtol=1e-12, atol=1e-12)
    acts = d["rand__act"][:17]
    for s in range(16):
        eng.env_step(torch.tensor(acts[s:s + 1], device=DEV), auto_reset=False)
        ora.step(acts[s])
    o_dev = eng.reset(init=iB[:, None], target=tB[:, None])[0].cpu().numpy()
    o_ora = ora.reset(iB, tB)
    np.testing.assert_allclose(o_dev, o_ora, rtol=1e-9, atol=1e-9)
    for s in range(17):  # the 17th step ends the episode (steps_max) and auto-resets
        obs, _, done, _ = eng.env_step(torch.tensor(acts[s:s + 1], device=DEV), auto_reset=True)
        ora.step(acts[s])
    assert bool(done[0])
    o_ora = ora.reset(iA, tA)
    np.testing.assert_allclose(obs[0].cpu().numpy()[ints], o_ora[ints], rtol=1e-9, atol=1e-9)
    eng.close()


@pytest.mark.parametrize("precision", ["float64", "float32"])
@pytest.mark.parametrize("name", ["rand", "pid"])
def test_env_obs_normalize_derived(name, precision):
    """observation.normalize with mean / var derived from the bounds (fixed_wing.py:142-161) on the device
    against the reference's episodes (env_obsnorm.npz): fp64 within 1e-6 + 1e-6 / step, fp32 2e-3 (1 + |ref|)."""
    import _fixtures as F
    from test_golden_r05 import obsnorm_config_kw
    from tum_adlr_deep_reinforcement_learning_amd.engine import Engine
    d = F.load("env_obsnorm.npz")
    g = lambda k: d[name + "__" + k]  # noqa: E731
    spec = C.EnvSpec(config_kw=obsnorm_config_kw(d, name), sim_config_kw={"turbulence": False})
    eng = Engine(spec.sim, spec, 1, device=DEV, precision=precision)
    f64 = precision == "float64"
    obs0 = eng.reset(init=F.env_init(g("init"))[:, None], target=g("target0")[:, None])
    np.testing.assert_allclose(obs0[0].double().cpu().numpy(), g("obs")[0], rtol=1e-12 if f64 else 1e-5, atol=1e-6)
    acts = torch.tensor(g("act"), dtype=eng.dtype, device=DEV)
    for s in range(len(acts)):
        obs, rew, done, _ = eng.env_step(acts[s:s + 1], auto_reset=False)
        assert bool(done[0]) == bool(g("done")[s]), s
        r, ref = float(rew[0]), float(g("rew")[s])
        o = obs[0].double().cpu().numpy()
        if f64:
            tol = 1e-6 + 1e-6 * s
            assert abs(r - ref) <= tol, (s, r, ref)
            np.testing.assert_allclose(o, g("obs")[s + 1], rtol=1e-5, atol=tol)
        else:
            assert abs(r - ref) <= 2e-3 * (1 + abs(ref)), (s, r, ref)
            np.testing.assert_allclose(o, g("obs")[s + 1], rtol=2e-3, atol=2e-3)
        if bool(done[0]):
            break
    eng.close()


def test_integration_window_with_observation_noise():
    """Observation noise applies to "integrator" entries as to every other (fixed_wing.py:1240-1247:
    normalise, then add N(mean, std)).  With std 0 the draw is exactly the mean, so every entry of the noisy
    run -- the integrator ones included -- is the plain run's plus the mean (fp64, 40 steps with an
    auto-reset at steps_max 17, 64 aircraft)."""
    import copy
    from test_golden_r05 import INTWIN_KW
    from tum_adlr_deep_reinforcement_learning_amd.engine import Engine
    outs = []
    for noise in (None, {"mean": 0.25, "var": 0.0}):
        ckw = copy.deepcopy(INTWIN_KW)
        ckw["steps_max"] = 17
        if noise:
            ckw["observation"]["noise"] = noise
        spec = C.EnvSpec(config_kw=ckw, sim_config_kw={"turbulence": False})
        eng = Engine(spec.sim, spec, 64, device=DEV, precision="float64")
        eng.seed(11)
        rows = [eng.reset().cpu().numpy()]
        g = torch.Generator().manual_seed(5)
        for _ in range(40):
            a = (torch.rand(64, 3, generator=g, dtype=torch.float64) * 2 - 1).to(DEV)
            obs, _, _, _ = eng.env_step(a, auto_reset=True)
            rows.append(obs.cpu().numpy())
        eng.close()
        outs.append(np.stack(rows))
    np.testing.assert_allclose(outs[1], outs[0] + 0.25, rtol=0, atol=1e-9)


@pytest.mark.parametrize("name", ["rand", "rand_hot", "fail_va"])
def test_integration_window_observation_history(name):
    """integration_window 10 with an observation history (length 3, step 2): the integrator entries of the
    lagged rows read slice [-W-i:-i] (fixed_wing.py:1165-1180), the reset rows the first reset's err x W,
    and a failed step's lagged rows the history one entry short -- fp64 against the reference's own
    episodes (env_intwin_hist.npz), rows beyond the episode up to their init-noise offset as in
    test_gpu_obs.py."""
    import _fixtures as F
    from test_golden_r05 import intwin_config_kw
    from test_gpu_obs import _check_obs
    from tum_adlr_deep_reinforcement_learning_amd.engine import Engine
    d = F.load("env_intwin_hist.npz")
    g = lambda k: d[name + "__" + k]  # noqa: E731
    spec = C.EnvSpec(config_kw=intwin_config_kw(d, name), sim_config_kw={"turbulence": False})
    assert spec.obs_length == 3 and spec.n_obs == g("obs").shape[1]
    eng = Engine(spec.sim, spec, 1, device=DEV, precision="float64")
    eng.seed(3)
    obs0 = eng.reset(init=F.env_init(g("init"))[:, None], target=g("target0")[:, None]).cpu().numpy()[0]
    _check_obs(spec, obs0, g("obs")[0], 0, 1e-12, "reset")
    acts = torch.tensor(g("act"), dtype=torch.float64, device=DEV)
    for s in range(len(acts)):
        obs, rew, done, _ = eng.env_step(acts[s:s + 1], auto_reset=False)
        dn = bool(done[0])
        assert dn == bool(g("done")[s]), s
        o = eng.terminal_obs[0].cpu().numpy() if dn else obs[0].cpu().numpy()
        tol = 1e-6 + 1e-6 * s
        assert abs(float(rew[0]) - g("rew")[s]) <= tol, (s, float(rew[0]), g("rew")[s])
        _check_obs(spec, o, g("obs")[s + 1], s + 1, tol, "step %d" % s)
        if dn:
            break
    assert s == len(acts) - 1
    eng.close()
