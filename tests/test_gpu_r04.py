"""GPU tests of round 4, all through the C ABI.

  per-env turbulence   env_method("reset", indices=[j], turbulence_noise=Z) (FixedWingAircraft.reset
                       (**sim_reset_kw) -> PyFly.reset -> Dryden.reset, fixed_wing.py:441, pyfly.py:1294):
                       env j's episode flies on Z (shorter than the episode: wrapped as dryden.py:209-236
                       does) and matches the fp64 oracle given Z; every other env is bit-identical to a run
                       without the injection; env j's next episode (after the VecEnv auto-reset) draws
                       from Philox again
  noise wrap           an injected sequence shorter than the episode == the same sequence tiled to the
                       episode length, bit for bit
  set_attr             target / steps_count / steps_max / training through SubprocVecEnv.set_attr's
                       surface (subproc_vec_env.py:156-161)
  graph key            a captured collect step is recaptured when the policy's exploration flag or the
                       policy module changes (actions then equal the mean / the new module's)
"""
import numpy as np
import pytest
import torch

from tum_adlr_deep_reinforcement_learning_amd import config as C

pytestmark = pytest.mark.gpu
DEV = "cuda:0"

_STATE = {"roll": 0.2, "pitch": 0.05, "yaw": 0.0, "omega_p": 0.0, "omega_q": 0.0, "omega_r": 0.0,
          "position_n": 0.0, "position_e": 0.0, "position_d": -50.0, "velocity_u": 19.0, "velocity_v": 0.0,
          "velocity_w": 0.5, "wind": [0.0, 0.0, 0.0],
          "elevon_right": (0.0, 0.0), "elevon_left": (0.0, 0.0), "throttle": (0.5, 0.0)}  # (the oracle draws nothing)
_TARGET = {"roll": -0.3, "pitch": 0.1, "Va": 21.0}


def _env(n, steps_max, seed=3):
    from tum_adlr_deep_reinforcement_learning_amd.vec_env import FixedWingVecEnv
    return FixedWingVecEnv(n, config_kw={"steps_max": steps_max},
                           sim_config_kw={"turbulence": True, "turbulence_intensity": "moderate"}, device=DEV,
                           precision="float64", seed=seed, return_tensors=True, info_target=False)


def test_per_env_turbulence_noise_vs_oracle_and_philox():
    from oracle import oracle as O
    n, j, steps_max = 64, 17, 120  # (turbulence_sim_length = steps_max; 40 is too short for the 2-tap FIR)
    z = np.random.RandomState(2).standard_normal((4, 50))  # shorter than the 120-step episode: wraps
    runs = []
    for inject in (True, False):
        env = _env(n, steps_max)
        env.reset()
        kw = {"turbulence_noise": z} if inject else {}
        env.env_method("reset", state=_STATE, target=_TARGET, indices=[j], **kw)
        rng = np.random.RandomState(9)
        obs, rew, dones = [], [], []
        for _ in range(steps_max + 20):  # the whole episode, its auto-reset, 20 steps of the next
            o, r, d, _ = env.step(torch.tensor(rng.uniform(-1, 1, (n, 3)), device=DEV))
            obs.append(o.cpu().numpy().copy())
            rew.append(r.cpu().numpy().copy())
            dones.append(d.cpu().numpy().copy())
        lens = env.engine._env_len.cpu().numpy().copy() if inject else None
        tobs = env.engine.terminal_obs.cpu().numpy().copy()
        runs.append((np.array(obs), np.array(rew), np.array(dones), lens, tobs))
        env.close()
    (oa, ra, da, lens, _), (ob, rb, db, _, _) = runs
    assert lens[j] == 0  # the auto-reset ended the injection
    others = np.arange(n) != j
    assert np.array_equal(oa[:, others], ob[:, others]) and np.array_equal(ra[:, others], rb[:, others])
    assert np.array_equal(da, db)
    assert da[steps_max - 1, j] and not da[:steps_max - 1, j].any()  # the steps_max termination of env j
    # env j's injected episode vs the oracle given the same noise (fp64 env-sequence tolerance)
    spec = C.EnvSpec(config_kw={"steps_max": steps_max},
                     sim_config_kw={"turbulence": True, "turbulence_intensity": "moderate"})
    orc = O.OracleEnv(spec.sim.struct(), spec.struct(), spec.n_obs)
    init = C.init_array([_STATE], 1, spec.sim)[:, 0]
    tgt = np.array([_TARGET["roll"], _TARGET["pitch"], _TARGET["Va"]])
    orc.reset(init, tgt, z)
    rng = np.random.RandomState(9)
    differs = False
    for s in range(steps_max - 1):  # the done step's obs is the reset observation: compare before it
        a = rng.uniform(-1, 1, (n, 3))[j]
        oo, rr, dd, _, _ = orc.step(a)
        tol = 1e-6 + 1e-7 * s
        np.testing.assert_allclose(oa[s, j], oo, rtol=tol, atol=tol, err_msg="step %d" % s)
        assert abs(ra[s, j] - rr) <= tol * (1 + abs(rr)) and not dd
        differs |= not np.allclose(oa[s, j], ob[s, j], rtol=1e-6, atol=1e-6)
    assert differs  # the injected noise moved env j's flight
    # the next episode of env j draws Philox again: equal to the run that never injected
    assert np.array_equal(oa[steps_max:, j], ob[steps_max:, j])


def test_injected_noise_wraps_like_tiled_sequence():
    from tum_adlr_deep_reinforcement_learning_amd.engine import Engine
    spec = C.build_sim(config_kw={"turbulence": True, "turbulence_sim_length": 300, "turbulence_intensity": "severe"})
    n = 64
    z = np.random.RandomState(4).standard_normal((n, 4, 70))
    tiled = np.concatenate([z] * 5, axis=2)[:, :, :301]
    engs = [Engine(spec, None, n, device=DEV, precision="float64") for _ in range(2)]
    engs[0].set_noise(z)
    engs[1].set_noise(tiled)
    for e in engs:
        e.seed(1)
        e.reset(want_obs=False)
    rng = np.random.RandomState(0)
    for s in range(300):
        cmd = torch.tensor(rng.uniform(-0.2, 0.2, (n, 3)) + [0.0, 0.0, 0.6], device=DEV)
        ta = engs[0].sim_step(cmd)[1].cpu().numpy()
        tb = engs[1].sim_step(cmd)[1].cpu().numpy()
        assert np.array_equal(ta, tb), s
    assert torch.equal(engs[0].get_block(C.FW_BLK_ODE), engs[1].get_block(C.FW_BLK_ODE))
    for e in engs:
        e.close()


def test_set_attr_surface():
    from tum_adlr_deep_reinforcement_learning_amd.vec_env import FixedWingVecEnv
    n = 8
    env = FixedWingVecEnv(n, sim_config_kw={"turbulence": False}, device=DEV, seed=2, return_tensors=True)
    env.reset()
    before = env.get_attr("target")
    env.set_attr("target", {"roll": 0.25, "Va": 23.0}, indices=[2, 5])
    after = env.get_attr("target")
    for i in range(n):
        if i in (2, 5):
            assert after[i]["roll"] == pytest.approx(0.25) and after[i]["Va"] == pytest.approx(23.0)
            assert after[i]["pitch"] == pytest.approx(before[i]["pitch"])
        else:
            assert after[i] == before[i]
    env.set_attr("steps_count", 7, indices=[1])
    assert env.get_attr("steps_count") == [0, 7, 0, 0, 0, 0, 0, 0]
    with pytest.raises(NotImplementedError):
        env.set_attr("steps_max", 5, indices=[0])
    env.set_attr("steps_max", 12)
    assert env.get_attr("steps_max", indices=[3]) == [12]
    env.set_attr("training", False)
    assert env.get_attr("training") == [False] * n
    # the new limit is what the kernel applies: env 1 (steps_count 7) ends after 5 steps, the others after 12
    # (an aircraft a constraint ends first is not counted)
    first, term = np.full(n, -1), np.zeros(n, np.int64)
    for s in range(12):
        _, _, d, _ = env.step(torch.zeros(n, 3, device=DEV))
        d, tm = d.cpu().numpy(), env.engine.term.cpu().numpy()
        for i in np.nonzero(d & (first < 0))[0]:
            first[i], term[i] = s, tm[i]
    by_steps = term == C.FW_TERM_STEPS
    assert by_steps[1] and first[1] == 4
    assert by_steps.sum() >= n // 2 and (first[by_steps & (np.arange(n) != 1)] == 11).all()
    env.close()


def test_graph_recaptured_when_policy_changes():
    """the captured collect step baked in the policy's exploration flag and module.  Toggling
    ``deterministic_rollout`` or swapping the policy recaptures: a deterministic graphed collection's
    actions equal the policy mean, and two stochastic collections draw different noise."""
    from tum_adlr_deep_reinforcement_learning_amd.rollout import MlpActorCritic, RolloutBuffer, RolloutCollector
    from tum_adlr_deep_reinforcement_learning_amd.vec_env import FixedWingVecEnv
    from tum_adlr_deep_reinforcement_learning_amd.vec_normalize import VecNormalize
    n, T = 1024, 16
    torch.manual_seed(0)
    venv = FixedWingVecEnv(n, sim_config_kw={"turbulence": False}, device=DEV, seed=4, return_tensors=True,
                           info_target=False)
    env = VecNormalize(venv)
    pol = MlpActorCritic(env.observation_space.shape[0], env.action_space.shape[0]).to(DEV)
    buf = RolloutBuffer(T, env.observation_space, env.action_space, device=DEV, n_envs=n)
    col = RolloutCollector(env, pol, buf)
    col.collect(4)
    col.collect(graph=True)
    g0 = col._graphs
    a1 = buf.actions.clone()
    col.collect(graph=True)
    assert col._graphs is g0 and not torch.equal(buf.actions, a1)  # fresh draws, same graph
    pol.deterministic_rollout = True
    col.collect(graph=True)
    assert col._graphs is not g0
    with torch.no_grad():
        mean = pol.action_net(pol.pi(buf.observations.reshape(-1, buf.obs_dim))).reshape(buf.actions.shape)
    assert torch.allclose(buf.actions, mean, rtol=1e-5, atol=1e-6)
    g1 = col._graphs
    col.policy = MlpActorCritic(env.observation_space.shape[0], env.action_space.shape[0]).to(DEV)
    col.policy.deterministic_rollout = True
    col.collect(graph=True)
    assert col._graphs is not g1
    with torch.no_grad():
        mean2 = col.policy.action_net(col.policy.pi(buf.observations.reshape(-1, buf.obs_dim))).reshape(
            buf.actions.shape)
    assert torch.allclose(buf.actions, mean2, rtol=1e-5, atol=1e-6)
    venv.close()


# ---------------------------------------------------------------------------- fused collect step (round 4)
def _P(t):
    import ctypes
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


@pytest.mark.parametrize("n,lanes", [(1000, 4), (20037, 1)])
def test_collect_epilogue_records_and_return_vs_numpy(n, lanes):
    """fw_env_step's collect epilogue (fw_set_collect_epilogue): the block records merged by fw_moments_merge
    equal numpy's mean / var of the step's float32 observation and of ret*gamma + reward (fp64, rel 1e-12);
    ret after the step = that value, 0 where done (bit for bit, multiply and add unfused as numpy); the row
    counter advances by one per launch; one record per launch block of the lanes setting."""
    from tum_adlr_deep_reinforcement_learning_amd import _native
    from tum_adlr_deep_reinforcement_learning_amd.vec_env import FixedWingVecEnv
    lib = _native.load()
    venv = FixedWingVecEnv(n, config_kw={"steps_max": 12}, sim_config_kw={"turbulence": False}, device=DEV, seed=9,
                           return_tensors=True, info_target=False, lanes=lanes)
    eng = venv.engine
    venv.reset()
    D = eng.n_obs_values + 1
    nrec, nmax = eng.collect_records()
    assert nrec == -(-n * lanes // 64) and nmax == -(-n * 4 // 64)
    g = torch.Generator(device=DEV)
    g.manual_seed(n)
    ret = torch.randn(n, generator=g, device=DEV, dtype=torch.float64)
    rec = torch.full((nmax * (1 + 2 * D),), float("nan"), dtype=torch.float64, device=DEV)
    ctrl = torch.zeros(2, dtype=torch.int32, device=DEV)
    out = torch.empty(1 + 2 * D, dtype=torch.float64, device=DEV)
    gamma = 0.99
    seen_done = 0
    for k in range(15):  # episodes end at step 12: done envs reset inside the window
        a = torch.rand(n, 3, generator=g, device=DEV) * 2 - 1
        ret0 = ret.clone()
        eng.set_collect_epilogue(ret=ret, gamma=gamma, records=rec, row_ctrl=ctrl)
        obs, rew, done, _ = eng.env_step(a)
        eng.set_collect_epilogue()
        _native.check(lib.fw_moments_merge(_P(rec), nrec, D, _P(out), None), "fw_moments_merge")
        torch.cuda.synchronize()
        r_new = ret0.cpu().numpy() * gamma + rew.cpu().numpy().astype(np.float32).astype(np.float64)
        dn = done.cpu().numpy().astype(bool)
        seen_done += int(dn.sum())
        np.testing.assert_array_equal(ret.cpu().numpy(), np.where(dn, 0.0, r_new))
        xs = np.concatenate([obs.cpu().numpy().astype(np.float32).astype(np.float64), r_new[:, None]], 1)
        o = out.cpu().numpy()
        assert o[0] == n
        np.testing.assert_allclose(o[1:D + 1], xs.mean(0), rtol=1e-12, atol=1e-13)
        np.testing.assert_allclose(o[D + 1:] / n, xs.var(0), rtol=1e-12, atol=1e-13)
        assert int(ctrl[0]) == k + 1
    assert seen_done >= n  # every env's episode ended (steps_max) inside the window
    venv.close()


def test_merge_update_equals_merge_then_update():
    """fw_vecnorm_merge_update (one launch) == fw_moments_merge + fw_rms_update of the merged record, bit for
    bit (the same device functions), over records of uneven block sizes."""
    from tum_adlr_deep_reinforcement_learning_amd import _native
    lib = _native.load()
    d, nrec = 14, 1029
    D = d + 1
    g = torch.Generator(device=DEV)
    g.manual_seed(7)
    rec = torch.randn(1 + 2 * D, nrec, generator=g, device=DEV, dtype=torch.float64)  # column-major records
    rec[0] = torch.randint(1, 65, (nrec,), generator=g, device=DEV).double()
    rec[1 + D:] = rec[1 + D:].abs() * 10
    rms0 = torch.rand(2 * d + 4, generator=g, device=DEV, dtype=torch.float64) + 0.5
    a, b = rms0.clone(), rms0.clone()
    out_a = torch.empty(1 + 2 * D, dtype=torch.float64, device=DEV)
    out_b = torch.empty_like(out_a)
    _native.check(lib.fw_vecnorm_merge_update(_P(rec), nrec, d, 1, _P(a), _P(out_a), None), "merge_update")
    _native.check(lib.fw_moments_merge(_P(rec), nrec, D, _P(out_b), None), "merge")
    _native.check(lib.fw_rms_update(_P(out_b), 1, d, 1, _P(b), 1, 1, None), "rms_update")
    torch.cuda.synchronize()
    assert torch.equal(out_a, out_b) and torch.equal(a, b) and not torch.equal(a, rms0)


@pytest.mark.parametrize("d,A", [(14, 1), (20, 5), (9, 8)])
def test_mfma_policy_forward_vs_torch_module(d, A):
    """The matrix-core policy launch (v_mfma_f32_16x16x4_f32, fw_policy_forward) for action heads beyond
    four rows (rows 4..7 come from the next lane group), one action, and observations wider than 16 (eight
    k-steps) == the torch module within fp32 rounding (rel/abs 2e-5), ragged n."""
    from tum_adlr_deep_reinforcement_learning_amd.rollout import MlpActorCritic
    torch.manual_seed(d * 10 + A)
    n = 3001
    pol = MlpActorCritic(d, A).to(DEV)
    with torch.no_grad():
        for prm in pol.parameters():
            prm.add_(0.3 * torch.randn_like(prm))
    obs = 3 * torch.randn(n, d, device=DEV)
    low = -0.7 * torch.ones(A, device=DEV)
    high = 0.8 * torch.ones(A, device=DEV)
    torch.manual_seed(11)
    with torch.no_grad():
        a_ref, v_ref, lp_ref = pol(obs)
    torch.manual_seed(11)
    a, c, v, lp = pol.collect_step(obs, low, high)
    tol = dict(rtol=2e-5, atol=2e-5)
    torch.testing.assert_close(a, a_ref, **tol)
    torch.testing.assert_close(v, v_ref.reshape(-1), **tol)
    torch.testing.assert_close(lp, lp_ref, **tol)
    assert torch.equal(c, torch.max(torch.min(a, high), low))


def _collect_setup(n, T, vecnorm=True, seed=21):
    from tum_adlr_deep_reinforcement_learning_amd.rollout import MlpActorCritic, RolloutBuffer, RolloutCollector
    from tum_adlr_deep_reinforcement_learning_amd.vec_env import FixedWingVecEnv
    from tum_adlr_deep_reinforcement_learning_amd.vec_normalize import VecNormalize
    torch.manual_seed(5)
    venv = FixedWingVecEnv(n, config_kw={"steps_max": 30}, sim_config_kw={"turbulence": False}, device=DEV,
                           seed=seed, return_tensors=True, info_target=False)
    env = VecNormalize(venv) if vecnorm else venv
    policy = MlpActorCritic(env.observation_space.shape[0], env.action_space.shape[0]).to(DEV)
    buf = RolloutBuffer(T, env.observation_space, env.action_space, device=DEV, gae_lambda=0.95, gamma=0.99, n_envs=n)
    return venv, env, buf, RolloutCollector(env, policy, buf)


@pytest.mark.parametrize("vecnorm", [True, False])
def test_fused_collect_step_launches_and_equals_eager(vecnorm):
    """The fused graphed collect step is ONE graph of 3 kernels with VecNormalize (fw_collect_policy,
    fw_env_step with its collect epilogue, fw_vecnorm_merge_update), 2 without; it stores the same rollout
    as the eager collect bit for bit (slab, rewards, episode starts, last obs / dones, statistics, return)."""
    from oracle import rollout_oracle as R
    va, ea, ba, ca = _collect_setup(2048, 40, vecnorm)
    vb, eb, bb, cb = _collect_setup(2048, 40, vecnorm)
    for c in (ca, cb):
        torch.manual_seed(40)
        c.collect(8)
    for i in range(2):
        torch.manual_seed(41 + i)
        ca.collect()
        torch.manual_seed(41 + i)
        cb.collect(graph=True)
        assert cb._fused_graph
        for f in ("slab", "rewards", "dones"):
            assert torch.equal(getattr(ba, f), getattr(bb, f)), f
        assert torch.equal(ca.last_obs, cb.last_obs) and torch.equal(ca.last_dones, cb.last_dones)
        if vecnorm:
            assert torch.equal(ea.rms, eb.rms) and torch.equal(ea.ret, eb.ret)
    nodes = cb.graph_nodes()
    assert len(nodes) == 1 and nodes[0].count(0) == 2, nodes  # VecNormalize merges inside the env step (r05)
    assert cb.host_launches_per_step() <= 1
    assert int(bb.dones.sum()) > 0 and float(bb.log_probs.abs().max()) > 0
    with torch.no_grad():
        lv = cb.policy.predict_values(cb.last_obs).reshape(-1).cpu().numpy()
    a_ref, _ = R.gae(bb.rewards.cpu().numpy(), bb.values.cpu().numpy(), bb.dones.cpu().numpy(), lv,
                     cb.last_dones.cpu().numpy(), 0.99, 0.95)
    assert np.array_equal(bb.advantages.cpu().numpy(), a_ref)
    va.close()
    vb.close()


def test_fused_collect_rccl_world1_single_graph():
    """Under an nccl process group of size 1 the fused collect step captures the RCCL all-gather of the
    moment records inside its one graph (1 host launch per step), and the collection equals the group-less
    one and the eager one bit for bit."""
    import socket
    import torch.distributed as dist

    def port():
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            return s.getsockname()[1]

    runs = []
    for grouped in (False, True):
        if grouped:
            dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % port(), rank=0, world_size=1,
                                    device_id=torch.device(DEV))
        try:
            va, ea, ba, ca = _collect_setup(4096, 32)
            vb, eb, bb, cb = _collect_setup(4096, 32)
            for c in (ca, cb):
                torch.manual_seed(40)
                c.collect(8)
            snaps = []
            for i in range(2):
                torch.manual_seed(41 + i)
                ca.collect()
                torch.manual_seed(41 + i)
                cb.collect(graph=True)
                sa = [t.clone() for t in (ba.slab, ba.rewards, ba.dones, ca.last_obs, ca.last_dones, ea.rms, ea.ret)]
                sb = [t.clone() for t in (bb.slab, bb.rewards, bb.dones, cb.last_obs, cb.last_dones, eb.rms, eb.ret)]
                for x, y in zip(sa, sb):
                    assert torch.equal(x, y)
                snaps += sb
            assert cb._fused_graph and cb.host_launches_per_step() <= 1 and len(cb._graphs) == 1
            if grouped:
                assert dist.get_backend() == "nccl" and eb.exchanged()
            va.close()
            vb.close()
        finally:
            if grouped:
                dist.destroy_process_group()
        runs.append(snaps)
    for x, y in zip(*runs):
        assert torch.equal(x, y)


def test_fused_collect_falls_back_when_the_collective_cannot_be_captured():
    """If the RCCL exchange refuses stream capture (forced here: the all-gather raises while the stream is
    capturing), the fused sharded step is recaptured as two graphs around an eager all-gather, says why in
    `capture_error`, and still equals the eager collection bit for bit (world-1 nccl group)."""
    import socket
    import torch.distributed as dist

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % port, rank=0, world_size=1,
                            device_id=torch.device(DEV))
    try:
        va, ea, ba, ca = _collect_setup(4096, 32)
        vb, eb, bb, cb = _collect_setup(4096, 32)
        gather = eb._gather

        def refusing_gather(rec):
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("collective not capturable (forced by the test)")
            return gather(rec)

        eb._gather = refusing_gather
        for c in (ca, cb):
            torch.manual_seed(40)
            c.collect(8)
        for i in range(2):
            torch.manual_seed(41 + i)
            ca.collect()
            torch.manual_seed(41 + i)
            if i == 0:  # the first graphed collection captures (and falls back), the second replays
                with pytest.warns(UserWarning, match="could not be captured"):
                    cb.collect(graph=True)
            else:
                cb.collect(graph=True)
            for x, y in zip((ba.slab, ba.rewards, ba.dones, ca.last_obs, ca.last_dones, ea.rms, ea.ret),
                            (bb.slab, bb.rewards, bb.dones, cb.last_obs, cb.last_dones, eb.rms, eb.ret)):
                assert torch.equal(x, y)
        assert cb._fused_graph and len(cb._graphs) == 2 and "forced by the test" in cb.capture_error
        assert cb.host_launches_per_step() == 3
        va.close()
        vb.close()
    finally:
        dist.destroy_process_group()


def test_fused_collect_ragged_batch_equals_eager():
    """A ragged batch (1037 envs: a partial last policy tile, a partial last env block, an env count the unfused
    graphed step -- dword row copies -- cannot take) through the fused collect step, 40 steps = two 16-step
    graph replays + 8 single-step replays: graphed == eager bit for bit, GAE == oracle, and the statistics'
    count advances by 1037 per step."""
    from oracle import rollout_oracle as R
    va, ea, ba, ca = _collect_setup(1037, 40, True, seed=33)
    vb, eb, bb, cb = _collect_setup(1037, 40, True, seed=33)
    for c in (ca, cb):
        torch.manual_seed(50)
        c.collect(8)
    d = ea.obs_dim
    count0 = float(eb.rms[2 * d])
    torch.manual_seed(51)
    ca.collect()
    torch.manual_seed(51)
    cb.collect(graph=True)
    assert cb._fused_graph and cb.host_launches_per_step() <= 1
    for f in ("slab", "rewards", "dones"):
        assert torch.equal(getattr(ba, f), getattr(bb, f)), f
    assert torch.equal(ca.last_obs, cb.last_obs) and torch.equal(ea.rms, eb.rms) and torch.equal(ea.ret, eb.ret)
    assert abs(float(eb.rms[2 * d]) - (count0 + 40 * 1037)) < 1e-6  # (the count starts at SB3's epsilon)
    with torch.no_grad():
        lv = cb.policy.predict_values(cb.last_obs).reshape(-1).cpu().numpy()
    a_ref, _ = R.gae(bb.rewards.cpu().numpy(), bb.values.cpu().numpy(), bb.dones.cpu().numpy(), lv,
                     cb.last_dones.cpu().numpy(), 0.99, 0.95)
    assert np.array_equal(bb.advantages.cpu().numpy(), a_ref)
    va.close()
    vb.close()
