"""GPU tests of the reference-shaped Python surface: FixedWingVecEnv (SB3 VecEnv
semantics: auto-reset, terminal_observation, Monitor episode stats, seeding and
sharding), the FixedWingAircraft facade and the PyFly facade -- each checked
against the CPU oracle on the same states (fp64 build, tolerances as in
test_gpu_parity.py)."""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from tum_adlr_deep_reinforcement_learning_amd import config as C

pytestmark = pytest.mark.gpu


def _init_from_device(eng, j):
    """Rebuild an oracle reset vector from aircraft j's device state (euler from the derived block)."""
    y = eng.get_block(C.FW_BLK_ODE)[:, j].double().cpu().numpy()
    der = eng.get_block(C.FW_BLK_DERIVED)[:, j].double().cpu().numpy()
    wind = eng.get_block(C.FW_BLK_WIND)[:, j].double().cpu().numpy()
    v = np.zeros(C.FW_NINIT)
    v[0:3] = der[0:3]
    v[3:12] = y[4:13]
    for k in range(3):
        v[C.FW_I_ACT0 + 2 * k] = y[13 + k]
        v[C.FW_I_ACT0 + 2 * k + 1] = y[16 + k]
    v[C.FW_I_WIND_N:] = wind
    tgt = eng.get_block(C.FW_BLK_TARGET)[:, j].double().cpu().numpy()
    return v, tgt


def test_vecenv_auto_reset_terminal_obs_and_monitor():
    from tum_adlr_deep_reinforcement_learning_amd.vec_env import FixedWingVecEnv
    n, steps_max = 16, 40
    env = FixedWingVecEnv(n, config_kw={"steps_max": steps_max}, sim_config_kw={"turbulence": False},
                          device="cuda:0", precision="float64", seed=11)
    obs = env.reset()
    assert obs.shape == (n, env.spec.n_obs) and obs.dtype == np.float32
    eng = env.engine
    orc = []
    for j in range(n):
        init, tgt = _init_from_device(eng, j)
        e = O.OracleEnv(env.spec.sim.struct(), env.spec.struct(), env.spec.n_obs)
        np.testing.assert_allclose(e.reset(init, tgt), obs[j], rtol=1e-6, atol=1e-6)
        orc.append(e)
    ret = np.zeros(n)
    length = np.zeros(n, int)
    rng = np.random.RandomState(2)
    n_done = 0
    for s in range(steps_max + 20):
        a = rng.uniform(-1, 1, (n, 3)).astype(np.float32)
        obs, rew, done, infos = env.step(a)
        assert obs.shape == (n, env.spec.n_obs) and rew.shape == (n,) and done.dtype == bool
        assert len(infos) == n
        for j in range(n):
            oo, rr, dd, tt, _ = orc[j].step(a[j].astype(np.float64))
            assert dd == bool(done[j]), (s, j)
            assert abs(rr - rew[j]) <= 1e-5 * (1 + abs(rr)), (s, j, rr, rew[j])
            ret[j] += rr
            length[j] += 1
            if dd:
                n_done += 1
                info = infos[j]
                np.testing.assert_allclose(info["terminal_observation"], oo, rtol=1e-5, atol=1e-5)
                assert info["termination"] == O.term_name(tt)
                assert info["episode"]["l"] == length[j]
                assert abs(info["episode"]["r"] - ret[j]) <= 1e-5 * (1 + abs(ret[j]))
                assert set(info["target"]) == {"roll", "pitch", "Va"}
                # auto-reset: the returned obs is the first of the next episode
                init, tgt = _init_from_device(eng, j)
                np.testing.assert_allclose(orc[j].reset(init, tgt), obs[j], rtol=1e-6, atol=1e-6)
                ret[j], length[j] = 0.0, 0
            else:
                np.testing.assert_allclose(obs[j], oo, rtol=1e-5, atol=1e-5)
                assert "terminal_observation" not in infos[j]
    assert n_done >= n  # every env finished at least one episode (steps_max = 40)
    env.close()


def test_vecenv_seeding_is_shard_invariant():
    from tum_adlr_deep_reinforcement_learning_amd.vec_env import FixedWingVecEnv
    # a fixed integrator (the quad one: per-aircraft results independent of the wave's other aircraft,
    # so shards at any offset agree bit for bit)
    kw = dict(sim_config_kw={"turbulence": False}, device="cuda:0", precision="float32", seed=5, lanes=4)
    full = FixedWingVecEnv(8, **kw)
    a = FixedWingVecEnv(4, env_offset=0, **kw)
    b = FixedWingVecEnv(4, env_offset=4, **kw)
    o = full.reset()
    assert np.array_equal(o, np.concatenate([a.reset(), b.reset()]))
    assert full.seed(5) == list(range(5, 13))
    acts = np.random.RandomState(0).uniform(-1, 1, (30, 8, 3)).astype(np.float32)
    for s in range(30):
        of, rf, df, _ = full.step(acts[s])
        oa, ra, da, _ = a.step(acts[s, :4])
        ob, rb, db, _ = b.step(acts[s, 4:])
        assert np.array_equal(of, np.concatenate([oa, ob])) and np.array_equal(rf, np.concatenate([ra, rb]))
    for e in (full, a, b):
        e.close()


def test_vecenv_env_method_reset_and_attrs():
    from tum_adlr_deep_reinforcement_learning_amd.vec_env import FixedWingVecEnv
    env = FixedWingVecEnv(4, sim_config_kw={"turbulence": False}, device="cuda:0", precision="float64", seed=1)
    env.reset()
    state = {"roll": 0.3, "pitch": -0.1, "yaw": 0.0, "omega_p": 0.0, "omega_q": 0.0, "omega_r": 0.0,
             "position_n": 0.0, "position_e": 0.0, "position_d": -50.0, "velocity_u": 20.0, "velocity_v": 0.0,
             "velocity_w": 0.0, "wind": [0.0, 0.0, 0.0]}
    target = {"roll": 0.1, "pitch": 0.05, "Va": 21.0}
    out = env.env_method("reset", state=state, target=target, indices=[1, 3])
    assert len(out) == 2
    tg = env.get_attr("target")
    assert tg[1] == pytest.approx(target) and tg[3] == pytest.approx(target)
    assert tg[0] != pytest.approx(target)
    sims = env.get_attr("simulator", indices=[1])
    assert sims[0].state["roll"].value == pytest.approx(0.3)
    assert sims[0].state["velocity_u"].value == pytest.approx(20.0)
    assert env.get_attr("steps_count") == [0, 0, 0, 0]
    env.env_method("set_curriculum_level", 0.5)
    assert env.spec.curriculum_level == 0.5
    env.close()


def test_fixed_wing_facade_matches_oracle():
    from tum_adlr_deep_reinforcement_learning_amd.fixed_wing import FixedWingAircraft
    env = FixedWingAircraft(config_kw={"steps_max": 60}, sim_config_kw={"turbulence": False}, device="cuda:0")
    state = {"roll": -0.4, "pitch": 0.1, "yaw": 0.2, "omega_p": 0.1, "omega_q": -0.05, "omega_r": 0.0,
             "position_n": 0.0, "position_e": 0.0, "position_d": -40.0, "velocity_u": 19.0, "velocity_v": 1.0,
             "velocity_w": -0.5, "wind": [1.0, -0.5, 0.0], "elevon_right": 0.02, "elevon_left": -0.01,
             "throttle": 0.4}
    target = {"roll": 0.2, "pitch": 0.0, "Va": 22.0}
    obs = env.reset(state=state, target=target)
    o = O.OracleEnv(env.spec.sim.struct(), env.spec.struct(), env.spec.n_obs)
    init = C.init_array(state, 1, env.spec.sim)[:, 0]
    assert not np.isnan(init).any()
    np.testing.assert_allclose(o.reset(init, [target["roll"], target["pitch"], target["Va"]]), obs, rtol=1e-6,
                               atol=1e-6)
    rng = np.random.RandomState(4)
    for s in range(80):
        a = rng.uniform(-1, 1, 3)
        obs, rew, done, info = env.step(a)
        oo, rr, dd, tt, _ = o.step(a)
        assert done == dd and abs(rew - rr) < 1e-7
        np.testing.assert_allclose(obs, oo, rtol=1e-6, atol=1e-6)
        assert info["target"] == pytest.approx(target)
        if done:
            assert info["termination"] == O.term_name(tt)
            break
    assert done and env.steps_count == s + 1
    env.close()


def test_pyfly_facade_matches_oracle():
    from tum_adlr_deep_reinforcement_learning_amd.pyfly import PyFly
    sim = PyFly(config_kw={"turbulence": False}, device="cuda:0")
    state = {"roll": -0.5, "pitch": 0.15, "yaw": 0.0, "omega_p": 0.0, "omega_q": 0.0, "omega_r": 0.0,
             "position_n": 0.0, "position_e": 0.0, "position_d": -50.0, "velocity_u": 22.0, "velocity_v": 0.0,
             "velocity_w": 0.0, "wind": [0.0, 0.0, 0.0]}
    sim.seed(0)
    sim.reset(state=state)
    assert sim.state["roll"].value == pytest.approx(-0.5)
    assert sim.state["Va"].value == pytest.approx(22.0)
    cfg = sim.engine.sim_spec.struct()
    y = sim.engine.get_block(C.FW_BLK_ODE).T.cpu().numpy()
    der = sim.engine.get_block(C.FW_BLK_DERIVED).T.cpu().numpy()
    wind = np.zeros((1, 3))
    rng = np.random.RandomState(0)
    for s in range(100):
        cmd = [rng.uniform(-0.5, 0.6), rng.uniform(-0.5, 0.5), rng.uniform(0, 1)]
        ok, info = sim.step(cmd)
        r = O.sim_step(cfg, y, der, wind, np.zeros((1, 6)), np.array([cmd]))
        assert ok == (r["term"][0] == 0)
        if not ok:
            assert info["termination"] == O.term_name(int(r["term"][0]))
            break
        y, der = r["y"], r["der"]
        for name, row in (("roll", 0), ("pitch", 1), ("yaw", 2), ("Va", 3), ("alpha", 4), ("beta", 5)):
            assert sim.state[name].value == pytest.approx(der[0, row], rel=1e-7, abs=1e-9), (s, name)
        assert sim.state["omega_p"].value == pytest.approx(y[0, 4], rel=1e-7, abs=1e-9)
    assert sim.cur_sim_step == s + 1
    e = sim.state["energy_total"].value
    assert np.isfinite(e) and e > 0
    sim.engine.close()


def test_step_graph_replay_matches_eager_steps():
    """engine.StepGraph: K captured env steps replayed from a HIP graph leave exactly the state (and
    last-step outputs) that K eager launches leave, including auto-resets inside the graph."""
    from tum_adlr_deep_reinforcement_learning_amd.engine import Engine, StepGraph
    spec = C.EnvSpec(config_kw={"steps_max": 12}, sim_config_kw={"turbulence": False})
    n, K = 4096, 8
    engs = [Engine(spec.sim, spec, n, device="cuda:0", precision="float32") for _ in range(2)]
    for e in engs:
        e.seed(5)
        e.reset()
    g = torch.Generator(device="cuda:0")
    g.manual_seed(3)
    pool = torch.rand(K, n, 3, generator=g, device="cuda:0") * 2 - 1
    for e in engs:
        e.env_step(pool[0])
    graph = StepGraph(engs[1], pool)
    for r in range(3):  # 24 steps: crosses steps_max, so done/auto-reset happen inside the graph
        for k in range(K):
            engs[0].env_step(pool[k])
        graph.replay()
        pool.mul_(-1.0)  # refilled in place between replays: the graph reads the new values
    torch.cuda.synchronize()
    for blk in (C.FW_BLK_ODE, C.FW_BLK_DERIVED, C.FW_BLK_TARGET, C.FW_BLK_STEPS):
        assert torch.equal(engs[0].get_block(blk), engs[1].get_block(blk)), blk
    for name in ("obs", "reward", "done", "term", "terminal_obs", "episode"):
        assert torch.equal(getattr(engs[0], name), getattr(engs[1], name)), name
    assert int(engs[1].steps()[0].max()) <= 12
    for e in engs:
        e.close()
