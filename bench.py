#!/usr/bin/env python3
"""Throughput benchmark: env-steps/s of the fused fixed-wing env step on MI355X.

One "step" = one FixedWingAircraft.step (PyFly.step with scipy-RK45 step
control + env epilogue + masked auto-reset) for every aircraft of the batch,
i.e. one launch of k_env_step per GPU.  Actions are uniform random in [-1, 1]^3,
pre-generated on the device (a pool of 16 batches cycled), so the timed region
contains only the hot path.

Workload (BASELINE.json metric / configs[2]-[3]): 65536 aircraft in TOTAL
(``--envs``), attitude-tracking task (fixed_wing_config.json defaults), fp32,
turbulence off.  With ``--gpus N`` the 65536 aircraft are split over N GPUs
(8192 per GPU at N = 8: strong scaling, configs[3]); one process per GPU, each
rank owns a contiguous env range with disjoint Philox streams, no collective on
the data path.  ``python bench.py --gpus N`` launches the N ranks itself (before
any GPU call) unless it already runs under torchrun, where WORLD_SIZE must equal N.

Steady state: after the global reset the population first runs ``--prep`` (1000)
untimed steps, so the timed window always sees the steady-state mix of
mid-episode, tumbling (straggler) and freshly reset aircraft whatever
``--warmup`` is; the first 96 steps after the reset are timed separately and
reported as ``early_regime``.

Prints ONE JSON line (rank 0).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from tum_adlr_deep_reinforcement_learning_amd import config as C  # noqa: E402
from tum_adlr_deep_reinforcement_learning_amd.engine import Engine, StepGraph  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md: 8.0 TB/s spec)
_T0 = time.time()


def _log(msg):
    """Progress on stderr (rank 0): the JSON line stays the only stdout output."""
    if os.environ.get("RANK", "0") == "0":
        print("[bench %7.1fs] %s" % (time.time() - _T0, msg), file=sys.stderr, flush=True)


def algorithmic_bytes_per_env_step(spec, esz=4):
    """HBM bytes one aircraft moves per env step in k_env_step (steady state, no reset).

    reads : ODE state 19, elevator/aileron 2, steady wind 3, targets 3, action 3,
            the previous actions the step reads (act_need*3: window - 1), ep_return 1   -> T
            steps word, life word (+ episode word with turbulence or observation noise:
            the Philox key); goal history (success_streak_req > 0, round 5): the ring
            words of the new and of the leaving entry, the window counts, the entry count -> u32
    writes: ODE state 19, derived 8, the targets that can change (compensate class; a
            constant-class row is stored only when some lane changed it), ring slot 3,
            last command 3, ep_return 1, observation n_obs, reward 1                    -> T
            steps word, term code, life word; goal history: the new entry's ring word,
            the counts, the entry count                                                 -> u32
            done flag                                                                   -> u8
    (life: the lifetime step counter the ring slots are indexed by, round 4.)  Not counted: the kernel's
    deliberate re-reads after the RK loop (pre-step state 19, targets 3, actions 3 -- held across the
    integration they would cost VGPRs), which PMC shows partly served from HBM (profiles/r04_traffic_split.json, r06_traffic_split.json).
    """
    act_need = 0
    for o in spec.cfg["observation"]["states"]:
        if o["type"] == "action" and spec.scale_actions:
            act_need = max(act_need, int(o.get("window_size", 1)) - 1)
    for f in spec.cfg["reward"]["factors"]:
        if f["class"] == "action" and f["type"] == "delta":
            act_need = max(act_need, int(f["window_size"]) - 1)
    tgt_var = sum(1 for t in spec.cfg["target"]["states"] if t.get("class", "constant") != "constant")
    philox = bool(spec.sim.cfg.get("turbulence")) or bool(spec.obs_noise)
    metrics = bool(spec.cfg.get("metrics") and spec.metrics_enabled)
    goal = int(spec.cfg["target"].get("success_streak_req", 0)) > 0
    rd = (19 + 2 + 3 + 3 + 3 + act_need * 3 + 1) * esz + (1 + 1 + (1 if philox else 0)) * 4
    wr = (19 + 8 + tgt_var + 3 + 3 + 1 + spec.n_obs + 1) * esz + (1 + 1 + 1) * 4 + 1
    rd += (4 if goal else 1 if metrics else 0) * 4
    wr += (3 if goal else 1 if metrics else 0) * 4
    if metrics:
        # streaming episode metrics, packed (round 5; csrc/fw_kernels.hip Met): previous command 3 (recomputed
        # from the previous action when the action ring delivers it), control variation 1, e0 / sum / |sum| /
        # overshoot extremum / end-window sum x3, the ring's previous error and the entry the new error overwrites
        # x3 each (T); goal counts, settling x4, rise crossings x6 (u16).  Written: control variation, sum / |sum| /
        # window sum x3, ring entry x3 (T).  The goal statuses and the entry count are the goal history's (above).
        # Rows that change now and then (extrema, goal counts, settling and rise indices) are stored only when a
        # lane changed them and are not counted.
        rd += ((0 if act_need >= 1 else 3) + 1 + 15 + 3 + 3) * esz + 14 * 2
        wr += (1 + 9 + 3) * esz
    return rd, wr


def device_ms_per_launch(launch, reps, dev):
    """Average device duration of ``launch()``: one HIP event pair on the launching stream around
    ``reps`` back-to-back launches, divided by ``reps``.

    The stream is first parked behind a spin kernel (torch.cuda._sleep) long enough for the host to
    enqueue every launch, so host-side Python overhead between launches never shows up as device time;
    no event sits between two launches (an event per launch serialises the queue and inflates each
    launch by the marker's own cost).  Inter-launch dispatch gaps are included (conservative)."""
    stream = torch.cuda.current_stream(dev)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(stream)
    torch.cuda._sleep(1 << 20)
    b.record(stream)
    torch.cuda.synchronize(dev)
    ms_per_cycle = max(a.elapsed_time(b), 1e-3) / float(1 << 20)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    host_ms = 2.0 + 0.2 * reps  # generous upper bound for enqueuing reps launches from Python
    torch.cuda._sleep(int(host_ms / ms_per_cycle))
    e0.record(stream)
    for _ in range(reps):
        launch()
    e1.record(stream)
    torch.cuda.synchronize(dev)
    return e0.elapsed_time(e1) / reps


def _cpu_worker(args):
    """One host process of the CPU baseline: 64 oracle envs stepped with U(-1,1) actions for ``seconds``."""
    seed, seconds = args
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle import oracle as O
    spec = C.EnvSpec(sim_config_kw={"turbulence": False})
    sc, ec = spec.sim.struct(), spec.struct()
    rng = np.random.RandomState(seed)
    envs = []
    for _ in range(64):
        e = O.OracleEnv(sc, ec, spec.n_obs)
        init = np.zeros(C.FW_NINIT)
        init[C.FW_I_ROLL], init[C.FW_I_PITCH] = rng.uniform(-1.9, 1.9), rng.uniform(-0.78, 0.78)
        init[C.FW_I_U] = rng.uniform(10, 23)
        init[C.FW_I_PD] = -50.0
        tgt = np.array([rng.uniform(-1, 1), rng.uniform(-0.4, 0.4), rng.uniform(15, 28)])
        e.reset(init, tgt)
        envs.append((e, init, tgt))
    steps = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        for e, init, tgt in envs:
            _, _, done, _, _ = e.step(rng.uniform(-1, 1, 3))
            steps += 1
            if done:
                e.reset(init, tgt)
    return steps, time.perf_counter() - t0


def cpu_baseline(seconds=12.0, procs=None):
    """The CPU oracle (oracle/fw_oracle.c, fp64 C port of the reference step) in one process per host
    core, the way the reference runs its envs (SubprocVecEnv: one env process per core).  Must run
    before this process touches the GPU (the workers are forked)."""
    import multiprocessing as mp
    if procs is None:
        procs = max(1, min(16, os.cpu_count() or 1))  # the GPU box's CPU share is 16 cores
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle import oracle as O
    O.build()  # compile once in the parent (workers only load it)
    # close() + join() let the workers exit on their own: leaving a `with Pool` block calls terminate(), whose
    # SIGTERM put two "*** Aborted at" stacks into every profiler log of this command (round-5 review)
    pool = mp.get_context("fork").Pool(procs)
    try:
        res = pool.map(_cpu_worker, [(1000 + k, seconds) for k in range(procs)])
    finally:
        pool.close()
        pool.join()
    steps = sum(r[0] for r in res)
    dt = max(r[1] for r in res)
    return {"value": steps / dt, "unit": "env-steps/s", "cores": procs, "kind": "port",
            "sample": "%d env steps (%d processes x 64 envs, U(-1,1) actions, default task, turbulence off, "
                      "auto-reset) of the fp64 C oracle in %.1f s on %d host cores"
                      % (steps, procs, dt, procs)}


def rollout_leg(spec, n, T, dev, rank, world, precision):
    """BASELINE configs[2]/[3]: one PPO collect_rollouts of T steps on the device (policy forward,
    VecNormalize with global statistics, env step, buffer writes, GAE kernel) plus, when sharded, the
    RCCL all-gather of the rollout slab.  Returns timings of rank-local phases (max over ranks)."""
    from tum_adlr_deep_reinforcement_learning_amd.rollout import MlpActorCritic, RolloutBuffer, RolloutCollector
    from tum_adlr_deep_reinforcement_learning_amd.vec_env import FixedWingVecEnv
    from tum_adlr_deep_reinforcement_learning_amd.vec_normalize import VecNormalize
    torch.manual_seed(rank)
    venv = FixedWingVecEnv(n, sim_config_kw={"turbulence": False}, device=dev, precision=precision, seed=1234,
                           env_offset=rank * n, return_tensors=True, info_target=False, global_envs=n * world)
    env = VecNormalize(venv)
    policy = MlpActorCritic(env.observation_space.shape[0], env.action_space.shape[0]).to(dev)
    buf = RolloutBuffer(T, env.observation_space, env.action_space, device=dev, gae_lambda=0.95, gamma=0.99, n_envs=n)
    col = RolloutCollector(env, policy, buf)
    # the collect step is replayed from ONE HIP graph per step (RolloutCollector.collect(graph=True), the fused
    # step: fw_collect_policy, fw_env_step + its VecNormalize epilogue, the statistics update; on N > 1 the
    # per-step RCCL all-gather of the moment records is captured inside the same graph)
    graph = True
    col.collect(min(T, 16))  # warm-up (kernels, allocator, RCCL communicator)
    col.collect(min(T, 16), graph=True)  # captures the step graph(s)
    buf.all_gather()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    col.collect(graph=graph)
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    gathered = buf.all_gather()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t2 = time.perf_counter()
    # GAE kernel alone (same inputs again)
    lv = torch.zeros(n, device=dev)
    gae_ms = device_ms_per_launch(lambda: buf.compute_returns_and_advantage(lv, col.last_dones), 5, dev)
    t = torch.tensor([t1 - t0, t2 - t1, t2 - t0, gae_ms], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    collect_s, gather_s, total_s, gae_ms = [float(x) for x in t]
    gae_bytes = (4 + 4 + 1 + 4 + 4) * T * n + (4 + 1) * n
    out = {"horizon": T, "envs_per_gpu": n, "global_envs": n * world, "collect_graphed": graph,
           "host_launches_per_step": col.host_launches_per_step(), "fused_step": bool(getattr(col, "_fused_graph", False)),
           "capture_error": getattr(col, "capture_error", None),
           "graph_kernel_nodes": [t.count(0) for t in col.graph_nodes()] if getattr(col, "_fused_graph", False) else None,
           "collect_s": collect_s,
           "allgather_s": gather_s if world > 1 else 0.0, "env_steps_per_s": n * world * T / total_s,
           "gathered_bytes_per_gpu": sum(s.numel() * 4 for s in gathered.slabs),
           "gae_kernel": {"ms": gae_ms, "bytes": gae_bytes, "achieved_GBs": gae_bytes / (gae_ms * 1e-3) / 1e9,
                          "frac_of_hbm_peak": gae_bytes / (gae_ms * 1e-3) / 1e9 / HBM_PEAK_GBS}}
    del gathered
    venv.close()
    return out


def sac_fill_leg(n, K, dev, rank, world, precision):
    """BASELINE configs[4]: SAC replay-buffer fill (OffPolicyCollector warm-up: uniform actions, env step
    with light Dryden turbulence + the default actuator constraints, one fused fw_replay_add per step)
    over n envs per GPU for K steps.  The action space is the bounded [-1, 1] scaled onto the actuator
    ranges: with the default +-FLT_MAX space SB3's scale_action overflows to NaN (see tests/test_replay.py)."""
    from tum_adlr_deep_reinforcement_learning_amd.replay import OffPolicyCollector, ReplayBuffer
    from tum_adlr_deep_reinforcement_learning_amd.vec_env import FixedWingVecEnv
    unit = {i: {"low": -1.0, "high": 1.0} for i in range(3)}
    env = FixedWingVecEnv(n, config_kw={"action": {"scale_space": True, "states": unit}},
                          sim_config_kw={"turbulence": True, "turbulence_intensity": "light"}, device=dev,
                          precision=precision, seed=4321, env_offset=rank * n, return_tensors=True, info_target=False,
                          global_envs=n * world)
    buf = ReplayBuffer(n * (K + 8), env.observation_space, env.action_space, device=dev, n_envs=n)
    col = OffPolicyCollector(env, buf, learning_starts=1 << 62, seed=7 + rank)
    col.collect(8)  # warm-up
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    col.collect(K, chunk=100)  # warm-up actions do not depend on obs: fused open-loop rollouts
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    fill_s = time.perf_counter() - t0
    # the add kernel alone (re-adding the last step's tensors into the first slots)
    src = (col.last_original_obs, col.last_original_obs, buf.actions[0].clone(), buf.rewards[0].clone(),
           buf.dones[0].clone())
    buf.pos = 0
    add_ms = device_ms_per_launch(lambda: buf.add(*src), 8, dev)
    t = torch.tensor([fill_s, add_ms], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    fill_s, add_ms = float(t[0]), float(t[1])
    d, a = buf.obs_dim, buf.action_dim
    add_bytes = 2 * (2 * d + a + 2) * 4 * n  # read + write of obs, next_obs, action, reward, done
    out = {"envs_per_gpu": n, "global_envs": n * world, "steps": K, "fill_s": fill_s,
           "env_steps_per_s": n * world * K / fill_s, "transitions_stored": buf.size() * world,
           "replay_add_kernel": {"ms": add_ms, "bytes": add_bytes, "achieved_GBs": add_bytes / (add_ms * 1e-3) / 1e9,
                                 "frac_of_hbm_peak": add_bytes / (add_ms * 1e-3) / 1e9 / HBM_PEAK_GBS}}
    env.close()
    return out


VALU_ISSUE_PEAK = 256 * 4 * 2.4e9 / 2.0  # wave64 VALU instructions/s: 1024 SIMDs, one per 2 cycles at 2.4 GHz
REFERENCE_CPU = {"value": 814.0, "unit": "env-steps/s", "cores": 8, "kind": "reference",
                 "sample": "reference VecNormalize(SubprocVecEnv([FixedWingAircraft] x 8)), default task, turbulence "
                           "off, U(-1,1) actions, 300 steps per env; measured in the survey container (8 vCPU Xeon, "
                           "SURVEY.md 6 / BASELINE.md 2) -- the reference is not shipped to the GPU box"}


def _self_launch(args):
    """--gpus N outside torchrun: start N ranks as child processes (nothing here has touched the GPU)."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % args.gpus,
           "--master-addr=127.0.0.1", "--master-port=%d" % port, os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd, env=env)


def _pmc_record(n, args, spec):
    """profiles/pmc_env_step.json when it was measured on this very workload (else None)."""
    pmc = os.path.join(ROOT, "profiles", "pmc_env_step.json")
    try:
        with open(pmc) as f:
            pm = json.load(f)
    except (OSError, ValueError):
        return None
    if pm.get("envs") == n and pm.get("precision") == args.precision and \
            bool(pm.get("turbulence")) == bool(args.turbulence) and \
            bool(pm.get("metrics", True)) == bool(spec.metrics_enabled) and pm.get("regime") == "steady":
        return pm
    return None


class _Schedule:
    """The bench's step schedule on one engine: a first eager step, then replays of a HIP graph of ``G``
    captured ``fw_env_step`` launches (engine.StepGraph: one host call per G steps, so the box's host
    jitter never leaves the device idle between steps) cycling over a pool of 16 action batches.
    ``run(k)`` = k // G replays + k % G eager steps on pool[0 .. k % G - 1]; ``actions_of(k)`` lists
    the pool index of each of those steps (the stats replay walks exactly the same sequence)."""
    G = 16

    def __init__(self, n, args, spec, dev, rank, env_offset, precision=None):
        self.eng = Engine(spec.sim, spec, n, device=dev, precision=precision or args.precision, lanes=args.lanes)
        self.eng.seed(1234, env_offset=env_offset)
        self.eng.reset()
        gen = torch.Generator(device=dev)
        gen.manual_seed(1 + rank)
        self.pool = torch.rand(16, n, 3, generator=gen, device=dev, dtype=self.eng.dtype) * 2 - 1
        self.eng.env_step(self.pool[0], stats=False)  # first step eager (kernel load outside the capture)
        self.graph = StepGraph(self.eng, self.pool)
        self.done = 1

    def run(self, k):
        for _ in range(k // self.G):
            self.graph.replay()
        for s in range(k % self.G):
            self.eng.env_step(self.pool[s], stats=False)
        self.done += k

    def actions_of(self, k):
        return list(range(self.G)) * (k // self.G) + list(range(k % self.G))

    def close(self):
        self.eng.close()
        del self.graph


def timed_env_steps(n, args, spec, dev, rank, world, env_offset, early=True, precision=None, replay=False):
    """Steady-state timing of ``args.steps`` env steps of ``n`` aircraft on this rank.

    Returns (elapsed_s, kernel_ms, early_ms, long_ms, window) with elapsed/kernel_ms max-reduced over
    ranks; ``window`` (replay=True) = the per-launch statistics of a stats-enabled replay of the same
    steps (window_replay)."""
    sch = _Schedule(n, args, spec, dev, rank, env_offset, precision)
    eng = sch.eng
    _log("timed_env_steps: %d aircraft, %s" % (n, precision or args.precision))
    timed_env_steps.lanes = eng.lanes  # the integrator this shard size runs (fw_set_lanes)
    stream = torch.cuda.current_stream(dev)
    early_ms = None
    plan = []  # (phase, steps) in order, for the replay
    if early:  # early-episode regime: the first 96 steps after the global reset (no stragglers yet)
        torch.cuda.synchronize(dev)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        sch.run(96)
        b.record(stream)
        torch.cuda.synchronize(dev)
        early_ms = a.elapsed_time(b) / 96
        plan.append(("early", 96))
    plan.append(("prep", max(args.prep - sch.done, 0)))
    # steady-state population.  Progress lines every 192 steps: chunks that are multiples
    # of the graph length keep exactly the action sequence of one run(prep) call
    k_prep = plan[-1][1]
    for k in range(0, k_prep - k_prep % sch.G, 192):
        sch.run(min(192, k_prep - k_prep % sch.G - k))
        torch.cuda.synchronize(dev)
        _log("  prep %d / %d" % (min(k + 192, k_prep), k_prep))
    sch.run(k_prep % sch.G)
    plan.append(("warmup", args.warmup))
    sch.run(args.warmup)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    sch.run(args.steps)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    _log("  timed window: %.4f ms/step" % (elapsed / args.steps * 1e3))
    plan.append(("timed", args.steps))
    obs_after = eng.obs.clone() if replay else None
    # k_env_step device duration per launch: HIP events on the launch stream around the timed steps
    # themselves (graph replays keep the queue full, so this is kernel time plus dispatch gaps)
    kern_ms = ev0.elapsed_time(ev1) / args.steps
    # the same population over a long window: rare extreme stragglers (an aircraft needing thousands of
    # RHS evaluations in one step) make a short window's mean depend on luck
    long_ms = 0.0
    if args.long_window > 0:
        l0, l1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        l0.record(stream)
        sch.run(args.long_window)
        l1.record(stream)
        torch.cuda.synchronize(dev)
        long_ms = l0.elapsed_time(l1) / args.long_window
        plan.append(("long", args.long_window))
        _log("  long window: %.4f ms/step" % long_ms)
    el = torch.tensor([elapsed, kern_ms, early_ms or 0.0, long_ms], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    sch.close()
    window = window_replay(n, args, spec, dev, rank, env_offset, precision, plan, obs_after) if replay else None
    return float(el[0]), float(el[1]), (float(el[2]) if early else None), float(el[3]), window


def window_replay(n, args, spec, dev, rank, env_offset, precision, plan, obs_after):
    """Per-launch statistics of the timed window (and of the long window), OUTSIDE the timed region: a
    second engine with the same seeds walks the same step schedule; the untimed phases run as before,
    the ``timed`` and ``long`` phases run eagerly with stats enabled and a HIP event pair around every
    launch.  Per step it records the launch duration, the largest RHS-evaluation count (and its aircraft),
    the solver failures and the max_nfev budget hits.  ``bitwise_equal_to_timed_run`` compares the
    replay's observations after the timed window with the timed engine's."""
    sch = _Schedule(n, args, spec, dev, rank, env_offset, precision)
    eng = sch.eng
    stream = torch.cuda.current_stream(dev)
    out = {}
    _log("window replay")
    for phase, k in plan:
        if phase not in ("timed", "long"):
            sch.run(k)
            continue
        _log("  replay %s (%d steps)" % (phase, k))
        rec = torch.zeros(k, 4, dtype=torch.int64, device=dev)  # max nfev, argmax, failures, budget hits
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(k)]
        for j, ai in enumerate(sch.actions_of(k)):
            evs[j][0].record(stream)
            eng.env_step(sch.pool[ai], stats=True)
            evs[j][1].record(stream)
            st = eng.stats
            nf = (st & 0xFFFF).to(torch.int64)
            m, am = nf.max(0)
            rec[j, 0], rec[j, 1] = m, am
            rec[j, 2] = (st < 0).sum()
            rec[j, 3] = ((st & (1 << 30)) != 0).sum()
        torch.cuda.synchronize(dev)
        ms = np.array([a.elapsed_time(b) for a, b in evs])
        r = rec.cpu().numpy()
        top = np.argsort(-ms)[:5]
        blk = {"steps": k, "launch_ms": {"mean": float(ms.mean()), "p50": float(np.median(ms)),
                                         "p99": float(np.percentile(ms, 99)), "max": float(ms.max()),
                                         "sum": float(ms.sum())},
               "max_nfev": int(r[:, 0].max()), "max_nfev_p50": float(np.median(r[:, 0])),
               "solver_failures": int(r[:, 2].sum()), "max_nfev_budget_hits": int(r[:, 3].sum()),
               "slowest_launches": [{"step_in_window": int(j), "launch_ms": round(float(ms[j]), 4),
                                     "max_nfev": int(r[j, 0]), "env": int(r[j, 1]) + env_offset} for j in top]}
        if phase == "timed" and obs_after is not None:
            blk["bitwise_equal_to_timed_run"] = bool(torch.equal(eng.obs, obs_after))
        out[phase] = blk
    sch.close()
    out["source"] = ("stats-enabled replay of the same steps (same seeds, same action sequence) outside the "
                     "timed region, one HIP event pair per launch (eager launches: the means include each "
                     "launch's dispatch overhead)")
    return out


def open_loop_leg(n, args, spec, dev, rank, world, env_offset, K=256, launches=16):
    """The same workload through the open-loop rollout kernel (fw_env_rollout: K steps per launch,
    actions pre-generated): the rate of a SAC / TD3 warm-up fill or a scripted-command evaluation, where
    the actions do not depend on the observations.  Steady state as above (prep steps first).  A launch
    lasts as long as its slowest wave's K steps, so one aircraft needing thousands of RHS evaluations adds
    milliseconds to its launch: 16 launches (4096 steps) instead of round 2's 4, whose rate moved by
    0.98e9 .. 1.26e9 with the population (profiles/r03_open_loop_probe.log)."""
    eng = Engine(spec.sim, spec, n, device=dev, precision=args.precision)
    eng.seed(1234, env_offset=env_offset)
    eng.reset()
    gen = torch.Generator(device=dev)
    gen.manual_seed(1 + rank)
    acts = (torch.rand(K, n, 3, generator=gen, device=dev, dtype=eng.dtype) * 2 - 1).contiguous()
    for _ in range(max(args.prep // K, 1)):  # steady-state population
        eng.env_rollout(acts)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    stream = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(launches):
        eng.env_rollout(acts)
    e1.record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    el = torch.tensor([time.perf_counter() - t0, e0.elapsed_time(e1)], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    eng.close()
    steps = K * launches
    return {"kernel": "k_env_rollout", "steps_per_launch": K, "steps": steps, "envs_per_gpu": n,
            "global_envs": n * world, "value": n * world * steps / float(el[0]), "unit": "env-steps/s",
            "ms_per_step": float(el[0]) / steps * 1e3, "kernel_ms_per_step": float(el[1]) / steps}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=16)
    ap.add_argument("--prep", type=int, default=1000,
                    help="untimed steps after the global reset that build the steady-state population")
    ap.add_argument("--envs", type=int, default=65536, help="aircraft in total, split over the GPUs")
    ap.add_argument("--precision", default="float32", choices=["float32", "float64"])
    ap.add_argument("--turbulence", action="store_true", help="light Dryden turbulence + random steady wind")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-procs", type=int, default=None, help="CPU baseline processes (default: min(16, cores))")
    ap.add_argument("--no-metrics", action="store_true",
                    help="do not track the config's streaming episode metrics (fixed_wing.py:1644-1736)")
    ap.add_argument("--no-weak", action="store_true", help="skip the weak-scaling line (65536 aircraft per GPU)")
    ap.add_argument("--no-open-loop", action="store_true", help="skip the open-loop rollout line (fw_env_rollout)")
    ap.add_argument("--long-window", type=int, default=1000,
                    help="after the timed steps, time this many more for the long-window steady-state line")
    ap.add_argument("--rollout-steps", type=int, default=2048,
                    help="also run one PPO collect_rollouts of this horizon (default 2048 = BASELINE configs[2]; on "
                         "N > 1 GPUs configs[3]: sharded collection + the RCCL all-gather of the slab); 0 = skip")
    ap.add_argument("--sac-fill-steps", type=int, default=1000,
                    help="also run a SAC replay-buffer fill of this many steps (BASELINE configs[4], default 1000 "
                         "steps of --sac-envs envs); 0 = skip")
    ap.add_argument("--sac-envs", type=int, default=262144, help="global envs of the SAC fill leg")
    ap.add_argument("--no-replay", action="store_true",
                    help="skip the stats-enabled replay of the timed window (per-launch times, nfev, budget hits)")
    ap.add_argument("--no-fp64", action="store_true",
                    help="skip the secondary line at the reference's own precision (fp64 kernels)")
    ap.add_argument("--fp64-prep", type=int, default=-1,
                    help="untimed steps before the fp64 line's window (default: --prep)")
    ap.add_argument("--lanes", type=int, default=0,
                    help="lanes per aircraft of k_env_step: 0 = automatic by shard size, 1, or 4 (quad integrator)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(_self_launch(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world), file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.envs % world:
        print("bench.py: --envs %d does not split evenly over %d GPUs" % (args.envs, world), file=sys.stderr)
        sys.exit(2)
    # CPU baseline first: its worker processes are forked, which must happen before any HIP call
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.cpu_seconds, args.cpu_procs)
        _log("cpu baseline done")
    # FW_BENCH_ONE_DEVICE=1 / FW_BENCH_BACKEND=gloo: rehearsal of the N > 1 code path with every rank on
    # cuda:0 (RCCL refuses two ranks on one GPU); never used for a reported line
    if os.environ.get("FW_BENCH_ONE_DEVICE") == "1":
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        backend = os.environ.get("FW_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    # pyfly_config.json defaults: random steady wind |w| <= 8 m/s; Dryden only with --turbulence
    spec = C.EnvSpec(sim_config_kw={"turbulence": bool(args.turbulence), "turbulence_intensity": "light"})
    spec.metrics_enabled = not args.no_metrics
    n = args.envs // world  # strong scaling: the global batch is split over the GPUs
    elapsed, kern_ms, early_ms, long_ms, window = timed_env_steps(n, args, spec, dev, rank, world, rank * n,
                                                                  replay=not args.no_replay)
    lanes = timed_env_steps.lanes
    value = args.envs * args.steps / elapsed

    weak = None
    if world > 1 and not args.no_weak:  # secondary: 65536 aircraft per GPU
        nw = 65536
        w_el, w_k, _, _, _ = timed_env_steps(nw, args, spec, dev, rank, world, rank * nw, early=False)
        weak = {"envs_per_gpu": nw, "global_envs": nw * world, "value": nw * world * args.steps / w_el,
                "ms_per_step": w_el / args.steps * 1e3, "kernel_ms": w_k}

    _log("open-loop leg")
    open_loop = None if args.no_open_loop else open_loop_leg(n, args, spec, dev, rank, world, rank * n)

    fp64 = None
    if not args.no_fp64 and args.precision == "float32":  # secondary: the reference's own precision
        _log("fp64 line")
        # the same schedule as the fp32 line (seeds, prep, window, long window) on the fp64 kernels
        a64 = argparse.Namespace(**vars(args))
        a64.prep = args.fp64_prep if args.fp64_prep >= 0 else args.prep
        f_el, f_k, f_early, f_long, _ = timed_env_steps(n, a64, spec, dev, rank, world, rank * n,
                                                        precision="float64")
        fp64 = {"dtype": "f64", "value": args.envs * args.steps / f_el, "ms_per_step": f_el / args.steps * 1e3,
                "kernel_ms": f_k, "prep_steps": a64.prep, "steps": args.steps,
                "early_regime": {"steps": 96, "kernel_ms": f_early,
                                 "env_steps_per_s_per_gpu": n / (f_early * 1e-3)},
                "long_window": ({"steps": args.long_window, "kernel_ms": f_long,
                                 "env_steps_per_s": args.envs / (f_long * 1e-3)} if f_long > 0 else None),
                "isa": "profiles/r06_isa_resources.txt (VGPR / spill counts per kernel instance)"}

    esz = 4 if args.precision == "float32" else 8
    rd, wr = algorithmic_bytes_per_env_step(spec, esz)
    achieved = (rd + wr) * n / (kern_ms * 1e-3) / 1e9  # GB/s per GPU, dominant kernel
    pm = _pmc_record(n, args, spec)
    traffic = pm.get("hbm_bytes_per_launch") if pm else None
    roof_valu = None
    if pm and pm.get("valu_insts_per_launch"):
        valu_rate = pm["valu_insts_per_launch"] / (kern_ms * 1e-3)
        roof_valu = {"bound": "valu", "achieved": valu_rate / 1e9, "peak": VALU_ISSUE_PEAK / 1e9,
                     "unit": "Ginst/s (wave64 VALU issue)", "frac": valu_rate / VALU_ISSUE_PEAK,
                     "valu_insts_per_launch": pm["valu_insts_per_launch"],
                     "valu_insts_per_wave": pm["valu_insts_per_launch"] * 64.0 / n,
                     "source": "SQ_INSTS_VALU per k_env_step dispatch from profiles/pmc_env_step.json (%s) over "
                               "this window's kernel_ms" % pm.get("dispatches")}

    # the configs[2]/[3] and configs[4] legs come last: a failure there is reported in the line instead of
    # costing the headline (an error that strikes every rank alike; a one-rank failure inside a collective
    # still hangs the job)
    rollout = None
    if args.rollout_steps > 0:
        _log("rollout leg (%d steps)" % args.rollout_steps)
        try:
            rollout = rollout_leg(spec, n, args.rollout_steps, dev, rank, world, args.precision)
        except Exception as e:  # noqa: BLE001
            rollout = {"horizon": args.rollout_steps, "error": "%s: %s" % (type(e).__name__, e)}
        torch.cuda.empty_cache()
    sac = None
    if args.sac_fill_steps > 0:
        _log("SAC fill leg (%d envs x %d steps)" % (args.sac_envs, args.sac_fill_steps))
        try:
            sac = sac_fill_leg(args.sac_envs // world, args.sac_fill_steps, dev, rank, world, args.precision)
        except Exception as e:  # noqa: BLE001
            sac = {"steps": args.sac_fill_steps, "error": "%s: %s" % (type(e).__name__, e)}
        torch.cuda.empty_cache()

    if rank == 0:
        out = {
            "metric": "env-steps/sec at 64k parallel aircraft, 1/2/4/8 MI355X; % HBM roofline",
            "value": value,
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32" if args.precision == "float32" else "f64",
            "data": "synthetic: seeded Philox initial states, U(-1,1) actions pre-generated on device (a pool of 16 "
                    "batches replayed cyclically); timed in the "
                    "steady state (%d untimed steps after the global reset, then %d warm-up steps)"
                    % (args.prep, args.warmup),
            "config": {"workload": "FixedWingAircraft.step x %d aircraft in total, %d per GPU (attitude task, "
                                   "fixed_wing_config defaults, %s, RK45 rtol=1e-3 atol=1e-6, auto-reset)"
                                   % (args.envs, n, "light Dryden + steady wind" if args.turbulence else
                                      "steady wind, turbulence off")
                                   + (", streaming episode metrics" if spec.metrics_enabled else ""),
                       "global_envs": args.envs, "envs_per_gpu": n, "kernel": "k_env_step",
                       "lanes_per_aircraft": lanes,
                       "parallelism": "env-dp%d" % world},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "algorithmic_bytes_per_env_step": rd + wr, "kernel_ms": kern_ms,
                         "traffic_source": ("profiles/pmc_env_step.json: calibrated FETCH_SIZE + WRITE_SIZE per "
                                            "k_env_step dispatch, %s" % pm.get("dispatches")) if traffic is not None
                         else None,
                         "binding_limit": "valu issue + RK45 straggler latency (see roofline_valu, DESIGN.md 3)"},
            "roofline_valu": roof_valu,
            "early_regime": {"steps": 96, "kernel_ms": early_ms, "env_steps_per_s_per_gpu": n / (early_ms * 1e-3)},
            "long_window": ({"steps": args.long_window, "kernel_ms": long_ms,
                             "env_steps_per_s": args.envs / (long_ms * 1e-3)} if long_ms > 0 else None),
            "window": window,
            "cpu_baseline": cpu,
            "cpu_baseline_reference": REFERENCE_CPU,
        }
        if fp64 is not None:
            out["fp64"] = fp64
        if open_loop is not None:
            out["open_loop_rollout"] = open_loop
        if weak is not None:
            out["weak_scaling"] = weak
        if rollout is not None:
            out["rollout"] = rollout
        if sac is not None:
            out["sac_fill"] = sac
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
