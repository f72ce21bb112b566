"""Engine: one libfwsim handle = N aircraft resident on one GPU.

Thin, allocation-free-per-step wrapper over the C ABI (include/fwsim.h): device
buffers are torch tensors on the handle's device, passed by data_ptr() together
with torch's current HIP stream, so every call is asynchronous and ordered with
the caller's torch work (policy forward, rollout buffer writes, RCCL).
"""
import ctypes

import numpy as np
import torch

from . import _native
from . import config as C

F32, F64 = 0, 1


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


class Engine:
    def __init__(self, sim_spec, env_spec=None, num_envs=1, device=None, precision="float32", lanes=None):
        if not torch.cuda.is_available():
            raise _native.FwError("no HIP device visible: the fixed-wing engine runs on MI355X only (no CPU fallback)")
        self.lib = _native.load()
        self.device = torch.device(device if device is not None else "cuda")
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        if precision not in ("float32", "float64"):
            raise ValueError("precision must be 'float32' or 'float64'")
        self.precision = precision
        self.dtype = torch.float32 if precision == "float32" else torch.float64
        self.n = int(num_envs)
        self.sim_spec, self.env_spec = sim_spec, env_spec
        self._sim_cfg = sim_spec.struct()
        self._env_cfg = env_spec.struct() if env_spec is not None else None
        h = ctypes.c_void_p()
        _native.check(self.lib.fw_create(ctypes.byref(self._sim_cfg),
                                         ctypes.byref(self._env_cfg) if self._env_cfg is not None else None,
                                         self.n, F32 if precision == "float32" else F64, self.device.index,
                                         ctypes.byref(h)), "fw_create")
        self.h = h
        self.n_obs = env_spec.n_obs if env_spec is not None else 0
        dev, dt = self.device, self.dtype
        n = self.n
        # persistent per-step I/O buffers (no allocation in the step path)
        self.obs = torch.zeros(n, max(self.n_obs, 1), dtype=dt, device=dev)
        self.terminal_obs = torch.zeros_like(self.obs)
        self.reward = torch.zeros(n, dtype=dt, device=dev)
        self.done = torch.zeros(n, dtype=torch.uint8, device=dev)
        self.term = torch.zeros(n, dtype=torch.int32, device=dev)
        self.episode = torch.zeros(n, 5, dtype=dt, device=dev)  # return, length, final target x3
        self.stats = torch.zeros(n, dtype=torch.int32, device=dev)
        self.success = torch.zeros(n, dtype=torch.uint8, device=dev)
        self.cmd_out = torch.zeros(n, 3, dtype=dt, device=dev)
        # episode-metric records of done envs (fixed_wing.py:1644-1736), when the config lists metrics
        self.metrics = None
        if self._env_cfg is not None and self._env_cfg.metrics:
            self.metrics = torch.full((C.FW_NMETRIC, n), float("nan"), dtype=dt, device=dev)  # SoA
            _native.check(self.lib.fw_set_metrics_output(self.h, _ptr(self.metrics)), "fw_set_metrics_output")
        self._noise = None
        self.config_version = 0  # bumped by every call that changes what a launch does (captured graphs check it)
        self.seed(0)
        if lanes is not None:
            self.set_lanes(lanes)

    def set_lanes(self, lanes):
        """Lanes per aircraft of the step kernels: 1, 4 (quad integrator) or 0 = automatic (fw_set_lanes)."""
        _native.check(self.lib.fw_set_lanes(self.h, int(lanes)), "fw_set_lanes")
        self.config_version += 1

    @property
    def lanes(self):
        """Lanes per aircraft the next fw_env_step / fw_sim_step launch uses."""
        v = ctypes.c_int32()
        _native.check(self.lib.fw_get_lanes(self.h, ctypes.byref(v)), "fw_get_lanes")
        return v.value

    # ------------------------------------------------------------------
    def stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def close(self):
        if getattr(self, "h", None):
            self.lib.fw_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 -- interpreter shutdown
            pass

    def seed(self, seed, env_offset=0):
        """Philox key; env i of this engine draws from stream (seed, env_offset + i)."""
        seed = 0 if seed is None else int(seed)
        _native.check(self.lib.fw_seed(self.h, seed % (1 << 64), int(env_offset)), "fw_seed")
        self._seed = seed

    def update_config(self, sim_spec=None, env_spec=None):
        if sim_spec is not None:
            self.sim_spec = sim_spec
        if env_spec is not None:
            self.env_spec = env_spec
        self._sim_cfg = self.sim_spec.struct()
        self._env_cfg = self.env_spec.struct() if self.env_spec is not None else None
        _native.check(self.lib.fw_update_config(self.h, ctypes.byref(self._sim_cfg),
                                                ctypes.byref(self._env_cfg) if self._env_cfg is not None else None),
                      "fw_update_config")
        self.config_version += 1

    def _push_noise(self):
        """Hand the current noise buffer (and per-env lengths) to the handle.  A captured step bakes in the
        buffer's address and length (not the per-env lengths, which the kernel reads from device memory), so
        config_version moves only when those change."""
        buf, lens = self._noise, getattr(self, "_env_len", None)
        key = (buf.data_ptr() if buf is not None else None, int(buf.shape[1]) if buf is not None else 0,
               lens.data_ptr() if lens is not None else None)
        _native.check(self.lib.fw_set_noise(self.h, _ptr(buf), key[1]), "fw_set_noise")  # (clears the lengths)
        if lens is not None:
            _native.check(self.lib.fw_set_noise_lengths(self.h, _ptr(lens)), "fw_set_noise_lengths")
        if key != getattr(self, "_noise_key", (None, 0, None)):
            self._noise_key = key
            self.config_version += 1

    def set_noise(self, noise):
        """Inject N(0,1) turbulence noise for every env, array-like [n][4][len] or [4][len] (shared), or None.
        Step k of an episode reads sample k mod len (dryden.py:209-236).  Replaces any per-env injection
        (set_env_noise)."""
        self._env_len = None
        if noise is None:
            self._noise = None
            self._push_noise()
            return
        a = torch.as_tensor(np.asarray(noise), dtype=self.dtype)
        if a.dim() == 2:
            a = a.unsqueeze(0).expand(self.n, *a.shape)
        if a.shape[0] != self.n or a.shape[1] != 4:
            raise ValueError("noise must be [n][4][len] or [4][len]")
        L = a.shape[2]
        ld = (self.n + 63) // 64 * 64
        buf = torch.zeros(4, L, ld, dtype=self.dtype, device=self.device)
        buf[:, :, :self.n] = a.permute(1, 2, 0).to(self.device)
        self._noise = buf
        self._push_noise()

    def set_env_draws(self, tape):
        """fw_set_env_draws: the env's own np_random draws (sample_target at every reset / resample, the
        randomised reward scalings, fixed_wing.py:436-479, 566-575, 654-746) taken in order from ``tape``
        [len][n] (numpy's ``random_sample()`` values: each draw is used as ``low + (high - low) * u``) instead
        of the Philox streams, so a device episode replays the reference's.  None: Philox again.  Restarts
        every env's cursor at draw 0; draws past the end are NaN."""
        if tape is None:
            self._tape = None
            _native.check(self.lib.fw_set_env_draws(self.h, None, 0), "fw_set_env_draws")
            return
        a = torch.as_tensor(np.asarray(tape), dtype=self.dtype)
        if a.dim() != 2 or a.shape[1] != self.n or a.shape[0] < 1:
            raise ValueError("tape must be [len][n] with len >= 1")
        self._tape = a.to(self.device).contiguous()
        torch.cuda.current_stream(self.device).synchronize()
        _native.check(self.lib.fw_set_env_draws(self.h, _ptr(self._tape), int(a.shape[0])), "fw_set_env_draws")
        self.config_version += 1  # a captured step bakes in the tape's address

    def set_env_noise(self, indices, noise):
        """Per-env injection (PyFly.reset(turbulence_noise=...) of the envs in ``indices``, pyfly.py:1262):
        ``noise`` [4][len] N(0,1) samples for all of them, or None = those envs draw from Philox again.
        The other envs keep what they had (a set_noise injection included); an env's injection ends at its
        next VecEnv auto-reset (fw_set_noise_lengths) or at a reset of it without noise (FixedWingVecEnv).
        Applies to the envs' next reset (call before ``reset(mask=...)``).  A set_noise sequence is an engine-wide
        override: the envs that never got their own injection keep reading it across resets, whatever the call
        history (round-5 advice); an env whose own injection ends draws from Philox."""
        idx = torch.as_tensor(np.asarray(list(indices), dtype=np.int64))
        if getattr(self, "_env_len", None) is None:
            if noise is None:
                return
            ld = (self.n + 63) // 64 * 64
            if self._noise is not None:  # a set_noise buffer: every env keeps reading it until its own injection
                # (a negative length marks the shared sequence: it survives resets, as it does without per-env lengths)
                self._env_len = torch.full((self.n,), -int(self._noise.shape[1]), dtype=torch.int32, device=self.device)
                self._noise = self._noise.clone()
            else:
                self._env_len = torch.zeros(self.n, dtype=torch.int32, device=self.device)
                self._noise = torch.zeros(4, 1, ld, dtype=self.dtype, device=self.device)
        if noise is None:  # ends the per-env injections of these envs (a shared set_noise sequence stays)
            cols = idx.to(self.device)
            self._env_len[cols] = torch.where(self._env_len[cols] > 0, 0, self._env_len[cols])
        else:
            a = torch.as_tensor(np.asarray(noise), dtype=self.dtype)
            if a.dim() != 2 or a.shape[0] != 4 or a.shape[1] < 1:
                raise ValueError("turbulence_noise must be [4][len] with len >= 1")
            L = a.shape[1]
            if L > self._noise.shape[1]:  # grow the buffer, keeping the other envs' samples
                grown = torch.zeros(4, L, self._noise.shape[2], dtype=self.dtype, device=self.device)
                grown[:, :self._noise.shape[1]] = self._noise
                self._noise = grown
            cols = idx.to(self.device)
            self._noise[:, :L, cols] = a.to(self.device)[:, :, None]
            self._env_len[cols] = L
        torch.cuda.current_stream(self.device).synchronize()  # host -> device copies of the pageable input
        self._push_noise()

    # ------------------------------------------------------------------
    def reset(self, mask=None, init=None, target=None, want_obs=True):
        """Masked reset.  init: [FW_NINIT][n] (NaN = sample), target: [3][n] (NaN = sample)."""
        m = None
        if mask is not None:
            m = torch.as_tensor(mask, device=self.device).to(torch.uint8).contiguous()
        it = None
        if init is not None:
            it = torch.as_tensor(np.asarray(init), dtype=self.dtype).to(self.device).contiguous()
            assert it.shape == (C.FW_NINIT, self.n)
        tg = None
        if target is not None:
            tg = torch.as_tensor(np.asarray(target), dtype=self.dtype).to(self.device).contiguous()
            assert tg.shape == (3, self.n)
        obs = self.obs if (want_obs and self.n_obs) else None
        _native.check(self.lib.fw_reset(self.h, _ptr(m), _ptr(it), _ptr(tg), _ptr(obs), self.stream()), "fw_reset")
        return self.obs if obs is not None else None

    def sim_step(self, commands, stats=False):
        """PyFly.step for all aircraft.  commands: tensor [n][3] on device (elevator, aileron, throttle)."""
        cmd = commands.to(device=self.device, dtype=self.dtype).contiguous()
        _native.check(self.lib.fw_sim_step(self.h, _ptr(cmd), _ptr(self.cmd_out), _ptr(self.success), _ptr(self.term),
                                           _ptr(self.stats) if stats else None, self.stream()), "fw_sim_step")
        return self.success, self.term

    def env_step(self, actions, auto_reset=True, stats=False, terminal_obs=True, episode=True):
        act = actions if (actions.dtype == self.dtype and actions.device == self.device and actions.is_contiguous()) \
            else actions.to(device=self.device, dtype=self.dtype).contiguous()
        _native.check(self.lib.fw_env_step(self.h, _ptr(act), _ptr(self.obs), _ptr(self.reward), _ptr(self.done),
                                           _ptr(self.term), _ptr(self.terminal_obs) if terminal_obs else None,
                                           _ptr(self.episode) if episode else None,
                                           _ptr(self.stats) if stats else None, int(bool(auto_reset)),
                                           self.stream()), "fw_env_step")
        self._stepped = True
        return self.obs, self.reward, self.done, self.term

    def env_rollout(self, actions, auto_reset=True, stats=False, terminal_obs=True, episode=True):
        """K consecutive ``env_step`` calls in ONE launch (fw_env_rollout) for actions known in advance.

        ``actions``: device tensor [K][n][3].  Returns (obs [K][n][n_obs], reward [K][n], done [K][n],
        term [K][n]); ``self.rollout_terminal_obs`` [K][n][n_obs], ``self.rollout_episode`` [K][n][5] and
        ``self.rollout_stats`` [K][n] hold the other per-step outputs.  The buffers are reused by the next
        call with the same K.  Bitwise the same as K ``env_step`` calls."""
        if actions.dim() != 3 or actions.shape[1:] != (self.n, 3):
            raise ValueError("actions must be [K][%d][3]" % self.n)
        act = actions if (actions.dtype == self.dtype and actions.device == self.device and actions.is_contiguous()) \
            else actions.to(device=self.device, dtype=self.dtype).contiguous()
        K = int(act.shape[0])
        if getattr(self, "_roll_k", None) != K:
            dev, dt, n = self.device, self.dtype, self.n
            w = max(self.n_obs, 1)
            self._roll_k = K
            self.rollout_obs = torch.zeros(K, n, w, dtype=dt, device=dev)
            self.rollout_terminal_obs = torch.zeros(K, n, w, dtype=dt, device=dev)
            self.rollout_reward = torch.zeros(K, n, dtype=dt, device=dev)
            self.rollout_done = torch.zeros(K, n, dtype=torch.uint8, device=dev)
            self.rollout_term = torch.zeros(K, n, dtype=torch.int32, device=dev)
            self.rollout_episode = torch.zeros(K, n, 5, dtype=dt, device=dev)
            self.rollout_stats = torch.zeros(K, n, dtype=torch.int32, device=dev)
        _native.check(self.lib.fw_env_rollout(self.h, K, _ptr(act), _ptr(self.rollout_obs), _ptr(self.rollout_reward),
                                              _ptr(self.rollout_done), _ptr(self.rollout_term),
                                              _ptr(self.rollout_terminal_obs) if terminal_obs else None,
                                              _ptr(self.rollout_episode) if episode else None,
                                              _ptr(self.rollout_stats) if stats else None, int(bool(auto_reset)),
                                              self.stream()), "fw_env_rollout")
        self._stepped = True
        return self.rollout_obs, self.rollout_reward, self.rollout_done, self.rollout_term

    def observe(self):
        _native.check(self.lib.fw_observe(self.h, _ptr(self.obs), self.stream()), "fw_observe")
        return self.obs

    def set_collect_epilogue(self, ret=None, gamma=0.0, records=None, row_ctrl=None, merged=None, rms=None,
                             defer=False):
        """fw_set_collect_epilogue: every following ``env_step`` also updates VecNormalize's discounted return
        ``ret`` (fp64 [n]: ret*gamma + reward, then 0 where done) and writes one moment record per launch block
        of (observation, ret) into ``records`` (fp64, ``collect_records()[1]`` x (1 + 2 D) rows); ``row_ctrl``
        (int32 device tensor) gets ``[0] += 1`` per launch.  ``merged`` (fp64 [1 + 2 D]): the launch merges its
        block records itself (in-launch tree) into that record; ``rms`` (the fw_rms_update buffer, with
        ``merged``): it also applies update_from_moments.  ``defer`` (ABI 12, with ``merged``): the launch stops
        the tree one level short and leaves that level (``collect_pending()``) to the next fw_collect_policy or
        to fw_vecnorm_pending_update.  All None turns it off.  A captured step keeps the setting it was
        captured with."""
        if ret is None and records is None and row_ctrl is None:
            _native.check(self.lib.fw_set_collect_epilogue(self.h, None), "fw_set_collect_epilogue")
            self._collect = None
            return
        for t, dt in ((ret, torch.float64), (records, torch.float64), (row_ctrl, torch.int32),
                      (merged, torch.float64), (rms, torch.float64)):
            if t is not None and (t.dtype != dt or t.device != self.device or not t.is_contiguous()):
                raise ValueError("set_collect_epilogue: ret / records / merged / rms fp64, row_ctrl int32, "
                                 "contiguous on the device")
        if ret is not None and ret.numel() != self.n:
            raise ValueError("set_collect_epilogue: ret must hold one value per env")
        D = self.n_obs_values + (1 if ret is not None else 0)
        if records is not None and records.numel() < self.collect_records()[1] * (1 + 2 * D):
            raise ValueError("set_collect_epilogue: records buffer too small")
        if merged is not None and merged.numel() < 1 + 2 * D:
            raise ValueError("set_collect_epilogue: merged must hold 1 + 2 D values")
        if rms is not None and rms.numel() < 2 * self.n_obs_values + 4:
            raise ValueError("set_collect_epilogue: rms must hold 2 d + 4 values")
        ptr = (lambda t: t.data_ptr() if t is not None else None)
        e = _native.FwCollectEpilogue(ptr(ret), float(gamma), ptr(records), ptr(row_ctrl), ptr(merged), ptr(rms),
                                      int(bool(defer)), 0)
        _native.check(self.lib.fw_set_collect_epilogue(self.h, ctypes.byref(e)), "fw_set_collect_epilogue")
        self._collect = (ret, records, row_ctrl, merged, rms)  # keep the buffers alive while the handle writes them

    def collect_pending(self):
        """fw_collect_pending: where the next env_step leaves its deferred final merge level --
        (records pointer, stride, count, D, the statistics' copy the next policy launch reads)."""
        p = _native.FwCollectPend()
        _native.check(self.lib.fw_collect_pending(self.h, ctypes.byref(p)), "fw_collect_pending")
        return p.records, p.stride, p.count, p.D, p.rms_prev

    def collect_records(self):
        """(records the next env_step writes, the most any lanes setting writes)."""
        a, b = ctypes.c_int64(), ctypes.c_int64()
        _native.check(self.lib.fw_collect_records(self.h, ctypes.byref(a), ctypes.byref(b)), "fw_collect_records")
        return a.value, b.value

    @property
    def n_obs_values(self):
        """Values per observation (rows x entries: observation.length x n_obs)."""
        return int(self.obs.shape[1])

    # ------------------------------------------------------------------
    _U32 = (C.FW_BLK_STEPS, C.FW_BLK_GOAL)

    def block_rows(self, blk):
        """Rows of a state block on this handle (fw_block_rows): [rows][n]."""
        v = ctypes.c_int32()
        _native.check(self.lib.fw_block_rows(self.h, int(blk), ctypes.byref(v)), "fw_block_rows")
        return v.value

    def get_block(self, blk):
        rows = self.block_rows(blk)
        dt = torch.int32 if blk in self._U32 else self.dtype
        out = torch.empty(rows, self.n, dtype=dt, device=self.device)
        _native.check(self.lib.fw_get_state(self.h, blk, _ptr(out), self.stream()), "fw_get_state")
        return out

    def set_block(self, blk, value):
        rows = self.block_rows(blk)
        dt = torch.int32 if blk in self._U32 else self.dtype
        v = torch.as_tensor(value, dtype=dt).to(self.device).reshape(rows, self.n).contiguous()
        _native.check(self.lib.fw_set_state(self.h, blk, _ptr(v), self.stream()), "fw_set_state")
        torch.cuda.current_stream(self.device).synchronize()

    def steps(self):
        s = self.get_block(C.FW_BLK_STEPS)[0]
        return s & 0xFFFF, (s >> 16) & 0xFFFF

    @staticmethod
    def decode_stats(stats):
        """fw_sim_step / fw_env_step stats -> (nfev, n_accepted, solver_failed) tensors.

        nfev saturates at 65535 and n_accepted at 16383 (include/fwsim.h); ``budget_hits`` tells the
        failures that were the max_nfev budget apart."""
        return stats & 0xFFFF, (stats >> 16) & 0x3FFF, (stats < 0)

    @staticmethod
    def budget_hits(stats):
        """stats -> bool tensor: the step ended on the max_nfev budget (FW_STATS_BUDGET, bit 30), a step
        scipy's solve_ivp would have continued (it has no budget)."""
        return (stats & (1 << 30)) != 0


class StepGraph:
    """``K`` consecutive ``Engine.env_step`` launches captured into one HIP graph.

    ``actions`` is a device tensor ``[K][n][3]`` of the engine's dtype; step ``k`` of every replay reads
    ``actions[k]`` at replay time, so a caller (e.g. an off-policy warm-up that draws uniform actions
    on the device, or a benchmark) refills it in place between replays.  One host call then issues K
    kernels, so the device never idles behind Python between steps.  The outputs (``eng.obs``,
    ``eng.reward``, ``eng.done``, ...) hold step K-1's values after a replay; the per-step values of the
    earlier steps are not kept (use eager ``env_step`` when every step's outputs are consumed).
    """

    def __init__(self, eng, actions, auto_reset=True, terminal_obs=True, episode=True):
        if actions.dim() != 3 or actions.shape[1:] != (eng.n, 3) or actions.dtype != eng.dtype \
                or actions.device != eng.device or not actions.is_contiguous():
            raise ValueError("actions must be a contiguous [K][n][3] %s tensor on %s" % (eng.dtype, eng.device))
        self.eng, self.actions, self.k = eng, actions, actions.shape[0]
        kw = dict(auto_reset=auto_reset, terminal_obs=terminal_obs, episode=episode)
        if not getattr(eng, "_stepped", False):
            raise RuntimeError("StepGraph: run one eager env_step first (loads the kernels outside the capture)")
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            for k in range(self.k):
                eng.env_step(actions[k], **kw)

    def replay(self):
        self.graph.replay()
        return self.eng.obs, self.eng.reward, self.eng.done, self.eng.term
