"""Device-resident PPO rollout collection: RolloutBuffer + GAE kernel + RCCL all-gather.

SURVEY.md 8(f) row 1 and 8(e): the consumer directly downstream of the env step.
The reference keeps the rollout in host numpy arrays and copies every step
through ``.cpu()`` (``OnPolicyAlgorithm.collect_rollouts``,
stable_baselines3/common/on_policy_algorithm.py:126-190; ``RolloutBuffer``,
stable_baselines3/common/buffers.py:259-389).  Here the buffer is one HBM slab
per GPU, the advantage scan is the ``fw_gae`` kernel (bit-exact with the
reference's numpy loop), and a sharded run gathers the slab with ONE
``all_gather_into_tensor`` (RCCL over xGMI) at the end of the collection -- the
only collective on the path.

Slab layout (float32, one allocation, so the all-gather is a single call):
    observations [T][N][D] | actions [T][N][A] | values [T][N] | log_probs [T][N]
    | advantages [T][N] | returns [T][N]
84 B per (step, env) for the default task (D = 14, A = 3).  Rewards and
episode starts live outside the slab (inputs of the scan, not of the update).
"""
import collections
import ctypes
import os
import warnings

import numpy as np
import torch
from torch import nn

from . import _native
from .sharding import all_gather_flat

RolloutBufferSamples = collections.namedtuple(
    "RolloutBufferSamples", ["observations", "actions", "old_values", "old_log_prob", "advantages", "returns"])


def _p(t):
    return ctypes.c_void_p(t.data_ptr())


def _stream(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _dim(space):
    return int(np.prod(space.shape))


def gae(rewards, values, episode_starts, last_values, last_dones, gamma, gae_lambda, advantages=None, returns=None):
    """fw_gae on device tensors ([T][N] float32, starts / last_dones uint8); returns (advantages, returns)."""
    T, N = rewards.shape
    for t, dt in ((rewards, torch.float32), (values, torch.float32), (episode_starts, torch.uint8)):
        if t.shape != (T, N) or t.dtype != dt or not t.is_contiguous() or t.device.type != "cuda":
            raise ValueError("gae: expected contiguous [T][N] device tensors (float32 rewards/values, uint8 starts)")
    last_values = last_values.reshape(N).to(torch.float32).contiguous()
    last_dones = last_dones.reshape(N).to(torch.uint8).contiguous()
    advantages = torch.empty_like(rewards) if advantages is None else advantages
    returns = torch.empty_like(rewards) if returns is None else returns
    lib = _native.load()
    _native.check(lib.fw_gae(_p(rewards), _p(values), _p(episode_starts), _p(last_values), _p(last_dones), T, N,
                             float(gamma), float(gae_lambda), _p(advantages), _p(returns), _stream(rewards.device)),
                  "fw_gae")
    return advantages, returns


class RolloutBuffer:
    """Device RolloutBuffer with SB3 0.10's API (buffers.py:259-389)."""

    def __init__(self, buffer_size, observation_space, action_space, device=None, gae_lambda=1, gamma=0.99, n_envs=1):
        self.buffer_size, self.n_envs = int(buffer_size), int(n_envs)
        self.obs_shape = tuple(observation_space.shape)
        self.obs_dim, self.action_dim = _dim(observation_space), _dim(action_space)
        self.gae_lambda, self.gamma = gae_lambda, gamma
        self.device = torch.device(device if device is not None else "cuda")
        T, N, D, A = self.buffer_size, self.n_envs, self.obs_dim, self.action_dim
        self.slab = torch.zeros(T * N * (D + A + 4), dtype=torch.float32, device=self.device)
        self._bind(self.slab, T, N)
        self.rewards = torch.zeros(T, N, dtype=torch.float32, device=self.device)
        self.dones = torch.zeros(T, N, dtype=torch.uint8, device=self.device)  # episode starts (SB3's `dones`)
        self.reset()

    def _bind(self, slab, T, N):
        D, A = self.obs_dim, self.action_dim
        o = 0
        self.observations = slab[o:o + T * N * D].view(T, N, D)
        o += T * N * D
        self.actions = slab[o:o + T * N * A].view(T, N, A)
        o += T * N * A
        self.values, self.log_probs, self.advantages, self.returns = (
            slab[o + k * T * N:o + (k + 1) * T * N].view(T, N) for k in range(4))

    def reset(self, zero=True):
        """buffers.py RolloutBuffer.reset.  zero=False skips clearing the arrays (11.3 GB at configs[2]'s shape):
        for a collection that rewrites every row it later reads (the fused graphed collect)."""
        self.pos, self.full, self.generator_ready = 0, False, False
        if zero:
            self.slab.zero_()
            self.rewards.zero_()
            self.dones.zero_()
        self._flat = None

    def size(self):
        return self.buffer_size if self.full else self.pos

    def add(self, obs, action, reward, done, value, log_prob):
        """buffers.py:335-361: store one step for all envs (device tensors or arrays)."""
        p = self.pos
        dev = self.device
        self.observations[p].copy_(torch.as_tensor(obs).reshape(self.n_envs, -1).to(dev), non_blocking=True)
        self.actions[p].copy_(torch.as_tensor(action).reshape(self.n_envs, -1).to(dev), non_blocking=True)
        self.rewards[p].copy_(torch.as_tensor(reward).reshape(-1).to(dev), non_blocking=True)
        self.dones[p].copy_(torch.as_tensor(done).reshape(-1).to(dev), non_blocking=True)
        self.values[p].copy_(value.reshape(-1), non_blocking=True)
        self.log_probs[p].copy_(log_prob.reshape(-1), non_blocking=True)
        self.pos += 1
        if self.pos == self.buffer_size:
            self.full = True

    def compute_returns_and_advantage(self, last_values, dones):
        """buffers.py:304-333 on the device (fw_gae) over the rows stored so far (``size()``): the
        bootstrap value enters at the last stored row, as the reference's loop over buffer_size does
        when the buffer is full."""
        lv = torch.as_tensor(last_values).to(self.device).reshape(-1)
        ld = torch.as_tensor(np.asarray(dones) if not isinstance(dones, torch.Tensor) else dones).to(self.device)
        n = self.size() or self.buffer_size
        gae(self.rewards[:n], self.values[:n], self.dones[:n], lv, ld, self.gamma, self.gae_lambda,
            self.advantages[:n], self.returns[:n])

    # ------------------------------------------------------------- sharding
    def all_gather(self, group=None):
        """Gather every rank's slab (one all_gather_into_tensor) -> GatheredRollout over W*N envs.
        Env g = rank * N + e, i.e. the global env order of the sharded VecEnv.  Every rank must hold
        the same number of envs (all_gather_into_tensor needs equal slabs): an uneven split raises."""
        counts = all_gather_flat(torch.tensor([self.n_envs], dtype=torch.int64, device=self.device), group)
        if counts.numel() > 1 and bool((counts != self.n_envs).any()):
            raise ValueError("RolloutBuffer.all_gather: uneven env shards %s; split the envs evenly over the ranks"
                             % counts.flatten().tolist())
        return GatheredRollout(list(all_gather_flat(self.slab, group)), self)

    def get(self, batch_size=None, generator=None):
        """buffers.py:363-380: minibatches over the (local) rollout, env-major flattening."""
        return self.all_gather_local().get(batch_size, generator)

    def all_gather_local(self):
        return GatheredRollout([self.slab], self)


class GatheredRollout:
    """Rollout slabs of W ranks; ``get`` yields SB3 RolloutBufferSamples over all W*N envs."""

    def __init__(self, slabs, like):
        self.slabs, self.T, self.N = slabs, like.buffer_size, like.n_envs
        self.D, self.A = like.obs_dim, like.action_dim
        self.n_envs = len(slabs) * self.N
        self._flat = None

    def _field_views(self, slab):
        T, N, D, A = self.T, self.N, self.D, self.A
        o = 0
        obs = slab[o:o + T * N * D].view(T, N, D)
        o += T * N * D
        act = slab[o:o + T * N * A].view(T, N, A)
        o += T * N * A
        rest = [slab[o + k * T * N:o + (k + 1) * T * N].view(T, N, 1) for k in range(4)]
        return [obs, act] + rest

    def flatten(self):
        """swap_and_flatten (buffers.py:70-80) of every field over the global env axis: index g*T + t."""
        if self._flat is None:
            per = [self._field_views(s) for s in self.slabs]
            self._flat = [torch.cat([p[k] for p in per], dim=1).transpose(0, 1).reshape(self.n_envs * self.T, -1)
                          for k in range(6)]
        return self._flat

    def get(self, batch_size=None, generator=None, indices=None):
        obs, act, val, logp, adv, ret = self.flatten()
        total = self.n_envs * self.T
        if indices is None:
            indices = torch.randperm(total, device=obs.device, generator=generator)
        batch_size = total if batch_size is None else batch_size
        for s in range(0, total, batch_size):
            idx = indices[s:s + batch_size]
            yield RolloutBufferSamples(obs[idx], act[idx], val[idx].flatten(), logp[idx].flatten(),
                                       adv[idx].flatten(), ret[idx].flatten())


# ---------------------------------------------------------------------------
# policy (the caller of the path; SB3 PPO MlpPolicy defaults, policies.py ActorCriticPolicy)
# ---------------------------------------------------------------------------
class MlpActorCritic(nn.Module):
    """SB3 0.10 PPO ``MlpPolicy`` defaults: separate pi/vf MLPs [64, 64] with tanh, orthogonal
    init (gains sqrt(2), 0.01 for the action head, 1 for the value head), state-independent
    log-std initialised to 0, diagonal Gaussian actions."""

    def __init__(self, obs_dim, act_dim, hidden=(64, 64), log_std_init=0.0):
        super().__init__()

        def mlp():
            layers, d = [], obs_dim
            for h in hidden:
                layers += [nn.Linear(d, h), nn.Tanh()]
                d = h
            return nn.Sequential(*layers)

        self.pi, self.vf = mlp(), mlp()
        self.action_net = nn.Linear(hidden[-1], act_dim)
        self.value_net = nn.Linear(hidden[-1], 1)
        self.log_std = nn.Parameter(torch.full((act_dim,), float(log_std_init)))
        for m, g in ((self.pi, np.sqrt(2)), (self.vf, np.sqrt(2)), (self.action_net, 0.01), (self.value_net, 1.0)):
            for layer in m.modules() if isinstance(m, nn.Sequential) else [m]:
                if isinstance(layer, nn.Linear):
                    nn.init.orthogonal_(layer.weight, gain=g)
                    nn.init.zeros_(layer.bias)

    deterministic_rollout = False  # collect_step without exploration noise (actions = mean)

    def fused_ok(self, obs):
        """collect_step can run as the fused fw_policy_forward kernel: SB3's default shapes on the device."""
        hid = [m.out_features for m in self.pi if isinstance(m, nn.Linear)]
        return (obs.is_cuda and obs.dtype == torch.float32 and obs.dim() == 2 and obs.shape[1] <= 32
                and hid == [64, 64] and [m.out_features for m in self.vf if isinstance(m, nn.Linear)] == [64, 64]
                and self.action_net.out_features <= 8 and self.log_std.dtype == torch.float32)

    @torch.no_grad()
    def collect_step(self, obs, low, high, out=None, noise=None, noise_row=None):
        """One collect step's policy work (ActorCriticPolicy.forward, policies.py:539-553, + the action
        clip, on_policy_algorithm.py:158-161) as ONE fw_policy_forward launch: returns (actions, clipped,
        values [N], log_probs).  The exploration noise is torch.randn (the module's own sampler): drawn
        here, or given -- ``noise`` [N][A], or the whole collection's draws [T][N][A] with ``noise_row`` a
        device int32 holding this step's row (a captured step then draws no RNG).  ``out`` = four
        preallocated tensors to write into.  Equal to forward() within ~1e-6 (FMA order), not bit for bit."""
        n, d = obs.shape
        A = self.action_net.out_features
        if out is None:
            out = (torch.empty(n, A, device=obs.device), torch.empty(n, A, device=obs.device),
                   torch.empty(n, device=obs.device), torch.empty(n, device=obs.device))
        act, clip, val, logp = out
        if self.deterministic_rollout:
            noise, noise_row = None, None
        elif noise is None:
            noise, noise_row = torch.randn(n, A, device=obs.device), None
        if not hasattr(self, "_fw_p"):
            self._fw_p = _native.FwMlpPolicy()
        lin = [m for m in self.pi if isinstance(m, nn.Linear)] + [self.action_net] + \
              [m for m in self.vf if isinstance(m, nn.Linear)] + [self.value_net]
        p = self._fw_p
        for k, m in zip((("pi_w0", "pi_b0"), ("pi_w1", "pi_b1"), ("act_w", "act_b"), ("vf_w0", "vf_b0"),
                         ("vf_w1", "vf_b1"), ("val_w", "val_b")), lin):
            assert m.weight.is_contiguous() and m.bias.is_contiguous()
            setattr(p, k[0], m.weight.data_ptr())
            setattr(p, k[1], m.bias.data_ptr())
        p.log_std, p.d, p.hidden, p.act_dim = self.log_std.data_ptr(), d, 64, A
        p.noise_row = noise_row.data_ptr() if noise_row is not None else None
        obs = obs.contiguous()
        lib = _native.load()
        _native.check(lib.fw_policy_forward(ctypes.byref(p), _p(obs), n, _p(noise) if noise is not None else None,
                                            _p(low), _p(high), _p(act), _p(clip), _p(val), _p(logp),
                                            _stream(obs.device)), "fw_policy_forward")
        return act, clip, val, logp

    def forward(self, obs, deterministic=False):
        mean = self.action_net(self.pi(obs))
        values = self.value_net(self.vf(obs))
        std = self.log_std.exp()
        actions = mean if deterministic else mean + std * torch.randn_like(mean)
        log_prob = (-((actions - mean) ** 2) / (2 * std * std) - self.log_std - 0.5 * np.log(2 * np.pi)).sum(-1)
        return actions, values, log_prob

    def predict_values(self, obs):
        return self.value_net(self.vf(obs))


class RolloutCollector:
    capture_collective = True  # a sharded fused step captures its RCCL exchange inside the one graph
    steps_per_graph = 16       # the fused step is also captured K times in one graph (one replay per K steps)
    # round 6: the env step leaves its VecNormalize merge's final level to the next step's policy launch (every
    # policy block merges it under its weight fill; fwsim.h fw_collect_epilogue.defer), off the env step's tail;
    # the collection's last level is applied by fw_vecnorm_pending_update.  Same bits either way.
    defer_final_merge = os.environ.get("FW_DEFER_FINAL_MERGE", "1") != "0"  # (A/B: tools/r06_collect_ab.sh)

    """OnPolicyAlgorithm.collect_rollouts (on_policy_algorithm.py:126-190) with everything on the device.

    ``env`` is a FixedWingVecEnv (or a VecNormalize-style wrapper around one) built with
    ``return_tensors=True``.  Per step: copy the last observation into the buffer slot, run the
    policy on it, clip the actions to the action space, step the env, store reward / episode start /
    value / log-prob.  No host synchronisation inside the loop."""

    def __init__(self, env, policy, buffer):
        self.env, self.policy, self.buffer = env, policy, buffer
        dev = buffer.device
        space = env.action_space
        self.low = torch.as_tensor(space.low, device=dev)
        self.high = torch.as_tensor(space.high, device=dev)
        self.last_obs = None
        self.last_dones = torch.zeros(env.num_envs, dtype=torch.uint8, device=dev)

    @torch.no_grad()
    def collect(self, n_rollout_steps=None, graph=False):
        """``graph=True``: the step body (policy forward, action clip, env step incl. VecNormalize, the
        buffer row stores) is captured into a HIP graph and replayed per step; same kernels, same results
        (bit for bit, tests/test_gpu_r02.py, tests/test_gpu_r03.py).  Under a process group (a sharded
        VecNormalize exchanges its moment records every step) the step is captured as two graphs around
        the RCCL all-gather: 3 launches per step (graph, collective, graph) instead of ~30.  The captured
        step reads the policy's parameters in place, so optimiser steps between collections are seen; it
        is recaptured when a host-side choice it baked in changes (``graph_key``: VecNormalize training /
        norm flags, the engine's lanes and configuration, the buffer)."""
        buf, env = self.buffer, self.env
        n = n_rollout_steps or buf.buffer_size
        if self.last_obs is None:
            self.last_obs = env.reset()
        if graph and self._graph_ok():
            return self._collect_graphed(n)
        buf.reset()
        fused = self._fused(buf.observations[0])
        noise = self._draw_noise(n) if fused else None
        for t in range(n):
            obs_slot = buf.observations[t]
            obs_slot.copy_(self.last_obs)
            if fused:
                actions, clipped, values, log_probs = self.policy.collect_step(
                    obs_slot, self.low, self.high, noise=noise[t] if noise is not None else None)
            else:
                actions, values, log_probs = self.policy(obs_slot)
                clipped = torch.max(torch.min(actions, self.high), self.low)
            new_obs, rewards, dones, _ = env.step(clipped)
            buf.actions[t].copy_(actions)
            buf.rewards[t].copy_(rewards)
            buf.dones[t].copy_(self.last_dones)
            buf.values[t].copy_(values.reshape(-1))
            buf.log_probs[t].copy_(log_probs)
            self.last_obs = new_obs
            self.last_dones = dones.to(torch.uint8).clone()
        buf.pos, buf.full = n, n == buf.buffer_size
        last_values = self.policy.predict_values(self.last_obs)
        buf.compute_returns_and_advantage(last_values, self.last_dones)
        self._eager_done = True
        return buf

    def _draw_noise(self, n):
        """The exploration noise of a whole fused collection in one torch.randn ([buffer_size][N][A], rows
        0..n-1 drawn): the eager and the captured collection read the same draws, and a replayed step
        draws nothing (torch's per-replay RNG bookkeeping costs two fill kernels + a randn per step)."""
        if getattr(self.policy, "deterministic_rollout", False):
            return None
        buf = self.buffer
        shape = (buf.buffer_size, buf.n_envs, buf.action_dim)
        if getattr(self, "_noise", None) is None or tuple(self._noise.shape) != shape:
            self._noise = torch.empty(shape, dtype=torch.float32, device=buf.device)
        if n > 0:
            self._noise[:n].normal_()
        return self._noise

    def _fused(self, obs):
        """The policy's step runs as one fw_policy_forward launch (MlpActorCritic with SB3's default shapes;
        any other policy module runs its own forward)."""
        pol = self.policy
        return (hasattr(pol, "collect_step") and type(pol).forward is MlpActorCritic.forward and
                self.low.dtype == torch.float32 and pol.fused_ok(obs))

    # ------------------------------------------------------------ graphed collection
    def _graph_ok(self):
        buf = self.buffer
        if buf.device.type != "cuda":
            return False
        venv = getattr(self.env, "venv", self.env)
        if getattr(venv, "_hists", None) is not None:  # a history recorder syncs to the host every step
            return False
        # the unfused captured step's fw_rollout_store moves whole dwords (uint8 rows); the fused step's
        # fw_collect_policy stores each env's episode start on its own
        return buf.n_envs % 4 == 0 or self._fused_collect_ok()

    def _split(self):
        """The env exchanges statistics between shards every step: capture around the collective."""
        import torch.distributed as dist
        return hasattr(self.env, "step_exchange") and dist.is_available() and dist.is_initialized()

    def graph_key(self):
        """Everything a captured step bakes in: the env's host-side choices, the split around the collective,
        the buffer, and the policy -- which module, where its parameters live (the launch reads them in
        place, so optimiser steps are seen but a replaced tensor is not), whether it explores."""
        env_key = self.env.graph_key() if hasattr(self.env, "graph_key") else None
        pol = self.policy
        pol_key = (id(pol), bool(getattr(pol, "deterministic_rollout", False)),
                   tuple(p.data_ptr() for p in pol.parameters()) if isinstance(pol, nn.Module) else None)
        return (env_key, self._split(), self.buffer.slab.data_ptr(), self.buffer.buffer_size, pol_key,
                self.capture_collective, self.steps_per_graph, self.defer_final_merge)

    def _capture(self):
        """Capture one collect step on static tensors: s_obs (the observation the policy acts on, then
        the next one), s_start (episode starts: the last dones), and the step's outputs, which the
        step's own fw_rollout_store launch writes into buffer row ctrl[0] (then ctrl[0] += 1)."""
        # kernels, the policy's BLAS handles and the allocator were warmed by an eager collect(); the
        # capture itself records only, so no env state moves here
        if not getattr(self, "_eager_done", False):
            raise RuntimeError("collect(graph=True): run one eager collect() first (warms kernels outside the capture)")
        if self._fused_collect_ok():
            return self._capture_fused()
        self._fused_graph = False
        buf, env, dev = self.buffer, self.env, self.buffer.device
        N, D, A = buf.n_envs, buf.obs_dim, buf.action_dim
        self.s_obs = torch.empty(N, D, dtype=torch.float32, device=dev)
        self.s_start = torch.empty(N, dtype=torch.uint8, device=dev)
        self.s_act = torch.empty(N, A, dtype=torch.float32, device=dev)
        self.s_clip = torch.empty(N, A, dtype=torch.float32, device=dev)
        self.s_val = torch.empty(N, dtype=torch.float32, device=dev)
        self.s_logp = torch.empty(N, dtype=torch.float32, device=dev)
        self._ctrl = torch.zeros(2, dtype=torch.int32, device=dev)  # {row, n_rows} of fw_rollout_store
        lib = _native.load()
        split = self._split()
        fused = self._fused(self.s_obs)

        def head():
            if fused:  # one fw_policy_forward launch writes the step's outputs in place
                noise = self._draw_noise(0)  # the buffer only; each collection draws its rows
                self.policy.collect_step(self.s_obs, self.low, self.high,
                                         out=(self.s_act, self.s_clip, self.s_val, self.s_logp),
                                         noise=noise, noise_row=self._ctrl if noise is not None else None)
                clipped = self.s_clip
            else:
                actions, values, log_probs = self.policy(self.s_obs)
                clipped = torch.max(torch.min(actions, self.high), self.low)
                self.s_act.copy_(actions)
                self.s_val.copy_(values.reshape(-1))
                self.s_logp.copy_(log_probs)
            if split:
                env.step_async(clipped)
                env.step_wait_local()
                return None
            return env.step(clipped)

        def tail(res):
            new_obs, rewards, dones, _ = env.step_wait_finish() if res is None else res
            self.s_obs.copy_(new_obs.reshape(N, D))  # the next step's policy input
            d8 = dones.reshape(N)
            if d8.dtype == torch.bool and d8.is_contiguous():
                d8 = d8.view(torch.uint8)  # the env's done buffer itself, no conversion kernel
            else:
                self.s_start.copy_(d8)
                d8 = self.s_start
            self._dsrc = d8  # the episode starts of the next row (and, after the last step, last_dones)
            # the step's rows straight from where they were produced (the captured env outputs keep their
            # addresses on every replay); the episode starts of row t + 1 from the static s_start
            rew = rewards.reshape(N)
            if rew.dtype != buf.rewards.dtype or not rew.is_contiguous():  # e.g. an fp64 env: convert once
                self.s_rew = torch.empty(N, dtype=buf.rewards.dtype, device=dev)
                self.s_rew.copy_(rew)
                rew = self.s_rew
            rows = ((self.s_obs, buf.observations, 1), (d8, buf.dones, 1), (self.s_act, buf.actions, 0),
                    (rew, buf.rewards, 0), (self.s_val, buf.values, 0), (self.s_logp, buf.log_probs, 0))
            self._rsegs = (_native.FwRowSeg * len(rows))()
            for k, (src, dst, off) in enumerate(rows):
                assert src.dtype == dst.dtype and src.is_contiguous()
                rb = dst[0].numel() * dst.element_size()
                g = self._rsegs[k]
                g.src, g.dst, g.bytes, g.stride, g.row_off = src.data_ptr(), dst.data_ptr(), rb, rb, off
            # the stream is read here, inside the capture: torch.cuda.graph captures on its own side stream
            _native.check(lib.fw_rollout_store(self._rsegs, len(rows), _p(self._ctrl), 1, _stream(dev)),
                          "fw_rollout_store")

        self._graphs = [torch.cuda.CUDAGraph()]
        if split:
            self._graphs.append(torch.cuda.CUDAGraph())
            with torch.cuda.graph(self._graphs[0]):
                head()
            with torch.cuda.graph(self._graphs[1]):
                tail(None)
        else:
            with torch.cuda.graph(self._graphs[0]):
                tail(head())
        self._key = self.graph_key()

    def _collect_graphed(self, n):
        buf = self.buffer
        if getattr(self, "_graphs", None) is None or self._key != self.graph_key():
            self._capture()
        if self._fused_graph:
            return self._collect_fused(n)
        N, D = buf.n_envs, buf.obs_dim
        buf.reset()
        if self._fused(self.s_obs):
            self._draw_noise(n)  # into the buffer the captured policy launch reads (row = ctrl[0])
        self.s_obs.copy_(self.last_obs.reshape(N, D))
        buf.observations[0].copy_(self.s_obs)  # the inputs of step 0; step t stores those of t + 1
        buf.dones[0].copy_(self.last_dones)
        self._ctrl[0] = 0
        self._ctrl[1] = n
        if len(self._graphs) == 1:
            g = self._graphs[0]
            for _ in range(n):
                g.replay()
        else:
            g0, g1 = self._graphs
            for _ in range(n):
                g0.replay()
                self.env.step_exchange()  # the RCCL all-gather of the moment records
                g1.replay()
        self.last_obs = self.s_obs.clone().reshape(self.last_obs.shape)
        self.last_dones = self._dsrc.clone()
        buf.pos, buf.full = n, n == buf.buffer_size
        last_values = self.policy.predict_values(self.last_obs)
        buf.compute_returns_and_advantage(last_values, self.last_dones)
        return buf

    # ------------------------------------------------------------ the fused collect step
    # One captured step = fw_collect_policy (VecNormalize's normalisation of the env's raw output, the
    # policy, the rollout rows at row ctrl[0]) -> fw_env_step (+ its collect epilogue: the moment records,
    # the return update, ctrl[0] += 1) -> the statistics update (fw_vecnorm_merge_update; sharded:
    # fw_moments_merge -> RCCL all-gather -> fw_rms_update).  3 launches per step unsharded, and one host
    # launch (graph replay) per step sharded too when the collective is captured.
    def _vecnorm(self):
        from .vec_normalize import VecNormalize
        return self.env if isinstance(self.env, VecNormalize) else None

    def _fused_collect_ok(self):
        buf, pol = self.buffer, self.policy
        vn = self._vecnorm()
        venv = vn.venv if vn is not None else self.env
        eng = getattr(venv, "engine", None)
        if eng is None or eng.dtype != torch.float32 or getattr(venv, "_hists", None) is not None:
            return False
        if vn is not None and not vn.fused_stats:
            return False
        if not (isinstance(pol, MlpActorCritic) and self._fused(eng.obs)):
            return False
        lin = [m for m in pol.modules() if isinstance(m, nn.Linear)]
        return all(t.data_ptr() % 16 == 0 for m in lin for t in (m.weight, m.bias)) and \
            eng.n_obs_values == buf.obs_dim and buf.action_dim == pol.action_net.out_features

    def _capture_fused(self):
        buf, pol, dev = self.buffer, self.policy, self.buffer.device
        vn = self._vecnorm()
        venv = vn.venv if vn is not None else self.env
        eng = venv.engine
        lib = _native.load()
        N, A = buf.n_envs, buf.action_dim
        self.s_clip = torch.empty(N, A, dtype=torch.float32, device=dev)
        self._ctrl = torch.zeros(2, dtype=torch.int32, device=dev)
        noise = self._draw_noise(0)
        if not hasattr(pol, "_fw_p"):
            pol._fw_p = _native.FwMlpPolicy()
        p = pol._fw_p
        lin = [m for m in pol.pi if isinstance(m, nn.Linear)] + [pol.action_net] + \
              [m for m in pol.vf if isinstance(m, nn.Linear)] + [pol.value_net]
        for k, m in zip((("pi_w0", "pi_b0"), ("pi_w1", "pi_b1"), ("act_w", "act_b"), ("vf_w0", "vf_b0"),
                         ("vf_w1", "vf_b1"), ("val_w", "val_b")), lin):
            setattr(p, k[0], m.weight.data_ptr())
            setattr(p, k[1], m.bias.data_ptr())
        p.log_std, p.d, p.hidden, p.act_dim, p.noise_row = pol.log_std.data_ptr(), buf.obs_dim, 64, A, None
        io = _native.FwCollectIO()
        io.obs, io.reward, io.done = eng.obs.data_ptr(), eng.reward.data_ptr(), eng.done.data_ptr()
        if vn is not None:
            io.rms, io.epsilon, io.clip_obs, io.clip_reward = vn.rms.data_ptr(), vn.epsilon, vn.clip_obs, vn.clip_reward
            io.norm_obs, io.norm_reward = int(vn.norm_obs), int(vn.norm_reward)
        io.noise = noise.data_ptr() if noise is not None else None
        io.low, io.high, io.clipped, io.ctrl = self.low.data_ptr(), self.high.data_ptr(), self.s_clip.data_ptr(), \
            self._ctrl.data_ptr()
        io.obs_rows, io.act_rows = buf.observations.data_ptr(), buf.actions.data_ptr()
        io.val_rows, io.logp_rows = buf.values.data_ptr(), buf.log_probs.data_ptr()
        io.rew_rows, io.start_rows, io.n = buf.rewards.data_ptr(), buf.dones.data_ptr(), N
        self._io = io
        grouped = vn is not None and vn.exchanged()
        if vn is not None:
            vn._ensure_parts()
        # the exchange is captured only on RCCL (nccl backend); gloo runs collectives on host threads, which a
        # stream capture cannot record (the one-device rehearsals of the N > 1 bench path use it)
        split = grouped and not (self.capture_collective and self._capturable_group())

        def policy():
            _native.check(lib.fw_collect_policy(ctypes.byref(p), ctypes.byref(io), _stream(dev)), "fw_collect_policy")

        def env_step():
            eng.env_step(self.s_clip, auto_reset=True, stats=True)

        def stats_local():
            if vn is None or vn.merge_in_launch:  # the env step's launch merged (and, unsharded, updated)
                return
            if grouped:
                vn.merge_records(vn._rec)
            else:
                vn.merge_update()

        def stats_exchange():
            if grouped:
                vn._gather(vn._rec)

        def stats_finish():
            if grouped:
                vn._merge()

        def capture(split):
            self._graphs = [torch.cuda.CUDAGraph(keep_graph=True)]  # keep_graph: graph_nodes() lists the launches
            self._graphK = None
            if split:
                self._graphs.append(torch.cuda.CUDAGraph(keep_graph=True))
                with torch.cuda.graph(self._graphs[0]):
                    policy()
                    env_step()
                    stats_local()
                with torch.cuda.graph(self._graphs[1]):
                    stats_finish()
            else:
                def step():
                    policy()
                    env_step()
                    stats_local()
                    stats_exchange()  # an RCCL all-gather captured into the graph (nccl backend)
                    stats_finish()
                with torch.cuda.graph(self._graphs[0]):
                    step()
                # and K steps in one graph: one host replay (and one inter-graph gap) per K steps; the rows,
                # noise row and counter advance on the device, so the K copies are the same launches
                K = max(1, int(self.steps_per_graph))
                if K > 1:
                    self._graphK = torch.cuda.CUDAGraph(keep_graph=True)
                    with torch.cuda.graph(self._graphK):
                        for _ in range(K):
                            step()
            for g in self._graphs:
                g.instantiate()
            if self._graphK is not None:
                self._graphK.instantiate()

        self._deferred = None  # the deferred level's fields (fw_collect_pending) when the step defers
        if vn is not None:
            vn.set_epilogue(row_ctrl=self._ctrl, defer=self.defer_final_merge and not grouped)
            pf = vn.pending_fields()
            if pf is not None and (1 + 2 * (buf.obs_dim + 1)) * pf[2] > vn.PEND_MAX:  # too big to stage: no deferral
                vn.set_epilogue(row_ctrl=self._ctrl)
                pf = None
            if pf is not None:
                io.pend, io.pend_stride, io.pend_cnt, io.has_ret, io.merged, io.rms_prev = pf
                self._deferred = vn._pend
            else:
                io.pend = None
        else:
            eng.set_collect_epilogue(row_ctrl=self._ctrl)
        self.capture_error = None
        try:
            try:
                capture(split)
            except Exception as e:  # noqa: BLE001 -- the collective would not capture: split around it instead
                if split or not grouped:
                    raise
                self.capture_error = "%s: %s" % (type(e).__name__, e)
                warnings.warn("the RCCL exchange could not be captured into the collect graph (%s); "
                              "replaying two graphs around an eager all-gather" % self.capture_error)
                torch.cuda.synchronize(dev)
                split = True
                capture(split)
        finally:
            eng.set_collect_epilogue()
        self._fused_graph = True
        self._fused_parts = (vn, eng, grouped, stats_exchange)
        self._key = self.graph_key()

    def _capturable_group(self):
        import torch.distributed as dist
        if not (dist.is_available() and dist.is_initialized()):
            return True
        vn = self._vecnorm()
        return dist.get_backend(getattr(vn, "group", None)) == "nccl"

    def graph_nodes(self):
        """Node types of each captured step graph of the fused path (hipGraphGetNodes / hipGraphNodeGetType:
        0 = kernel, 1 = memcpy, 2 = memset, 5 = empty, 6 / 7 = event wait / record)."""
        hip = _native.load()  # dlsym through libfwsim.so reaches its HIP runtime
        out = []
        for g in self._graphs:
            raw = ctypes.c_void_p(g.raw_cuda_graph())
            cnt = ctypes.c_size_t(0)
            if hip.hipGraphGetNodes(raw, None, ctypes.byref(cnt)) != 0:
                raise _native.FwError("hipGraphGetNodes failed")
            nodes = (ctypes.c_void_p * cnt.value)()
            hip.hipGraphGetNodes(raw, nodes, ctypes.byref(cnt))
            types = []
            for k in range(cnt.value):
                t = ctypes.c_int(-1)
                hip.hipGraphNodeGetType(ctypes.c_void_p(nodes[k]), ctypes.byref(t))
                types.append(t.value)
            out.append(types)
        return out

    def host_launches_per_step(self):
        """Host-side launches per replayed collect step: graph replays + an eager collective between them (split
        path), or 1 / steps_per_graph when the fused step is replayed K steps per graph."""
        g = getattr(self, "_graphs", None) or []
        if len(g) == 1 and getattr(self, "_graphK", None) is not None:
            return 1.0 / int(self.steps_per_graph)
        return len(g) + (1 if len(g) > 1 else 0)

    def _collect_fused(self, n):
        buf = self.buffer
        vn, eng, grouped, exchange = self._fused_parts
        buf.reset(zero=n < buf.buffer_size)  # a full collection writes every row of every field
        self._draw_noise(n)
        buf.dones[0].copy_(self.last_dones)  # the episode starts of row 0; row t >= 1 comes from the step
        self._ctrl[0] = 0
        self._ctrl[1] = n
        if len(self._graphs) == 1:
            g, gK = self._graphs[0], getattr(self, "_graphK", None)
            done = 0
            if gK is not None:
                K = int(self.steps_per_graph)
                for _ in range(n // K):
                    gK.replay()
                done = (n // K) * K
            for _ in range(n - done):
                g.replay()
        else:
            g0, g1 = self._graphs
            for _ in range(n):
                g0.replay()
                exchange()
                g1.replay()
        # the last step's reward row and the VecNormalize outputs of the last step (its obs_out is the
        # policy input of the next collection)
        if vn is not None:
            if self._deferred is not None:  # the last env step's final merge level (no policy launch follows it)
                vn.pending_update(self._deferred)
            vn._apply(eng.obs, eng.reward, None)
            vn.old_obs, vn.old_reward = eng.obs, eng.reward
            buf.rewards[n - 1].copy_(vn.rew_out)
            self.last_obs = vn.obs_out.clone().reshape(self.last_obs.shape)
        else:
            buf.rewards[n - 1].copy_(eng.reward)
            self.last_obs = eng.obs.clone().reshape(self.last_obs.shape)
        self.last_dones = eng.done.clone()
        buf.pos, buf.full = n, n == buf.buffer_size
        last_values = self.policy.predict_values(self.last_obs)
        buf.compute_returns_and_advantage(last_values, self.last_dones)
        return buf
