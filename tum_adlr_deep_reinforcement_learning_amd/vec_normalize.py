"""Device VecNormalize: SB3 0.10's normalising wrapper with its statistics in HBM.

Mirrors ``VecNormalize`` (stable_baselines3/common/vec_env/vec_normalize.py:13-260)
and ``RunningMeanStd`` (common/running_mean_std.py:6-40): same constructor
arguments, same ``reset`` / ``step_wait`` order of updates (obs statistics, obs
normalisation, discounted-return update, return statistics, reward
normalisation, ``ret[news] = 0``), same ``obs_rms`` / ``ret_rms`` attributes.
Per step it runs ``fw_moments`` (batch mean / M2, fp64) -> ``fw_rms_update``
(update_from_moments) -> ``fw_vecnorm_apply`` on the device: no host sync.

Sharded runs (one process per GPU, each owning a slice of the envs): the
statistics must be those of the GLOBAL batch, as with one VecNormalize over all
envs.  Each rank's moment record (n, mean, M2: 1 + 2D doubles) is all-gathered
over RCCL and every rank merges the records in rank order (parallel-variance
formula), so all ranks hold bit-identical statistics.  That is ~250 B per rank
per step: latency-bound (~10-20 us on xGMI); ``sync_every`` > 1 trades exactness
for fewer collectives (default 1 = the reference's semantics).

Persistence: ``save`` / ``load`` write the statistics as ``.npz`` (the reference
pickles the whole wrapper; pickles are not produced or read here).
"""
import ctypes

import numpy as np
import torch
import torch.distributed as dist

from . import _native
from .sharding import all_gather_flat


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


class _RMSView:
    """Read-only RunningMeanStd-like view (mean / var / count as numpy, copied on access)."""

    def __init__(self, owner, which):
        self._o, self._w = owner, which

    def _s(self):
        return self._o.rms.cpu().numpy()

    @property
    def mean(self):
        s, d = self._s(), self._o.obs_dim
        return s[:d].copy() if self._w == "obs" else float(s[2 * d + 1])

    @property
    def var(self):
        s, d = self._s(), self._o.obs_dim
        return s[d:2 * d].copy() if self._w == "obs" else float(s[2 * d + 2])

    @property
    def count(self):
        s, d = self._s(), self._o.obs_dim
        return float(s[2 * d]) if self._w == "obs" else float(s[2 * d + 3])


class VecNormalize:
    def __init__(self, venv, training=True, norm_obs=True, norm_reward=True, clip_obs=10.0, clip_reward=10.0,
                 gamma=0.99, epsilon=1e-8, group=None, return_tensors=None):
        self.venv = venv
        self.num_envs = venv.num_envs
        self.observation_space, self.action_space = venv.observation_space, venv.action_space
        self.training, self.norm_obs, self.norm_reward = training, norm_obs, norm_reward
        self.clip_obs, self.clip_reward, self.gamma, self.epsilon = clip_obs, clip_reward, gamma, epsilon
        self.group = group
        self.return_tensors = getattr(venv, "return_tensors", False) if return_tensors is None else return_tensors
        venv.return_tensors = True  # the wrapped device env hands over device tensors
        self.device = venv.device
        self.obs_dim = int(np.prod(self.observation_space.shape))
        d, n, dev = self.obs_dim, self.num_envs, self.device
        rms = np.zeros(2 * d + 4)
        rms[d:2 * d] = 1.0            # var = 1, count = epsilon 1e-4 (running_mean_std.py:14-16)
        rms[2 * d] = 1e-4
        rms[2 * d + 2] = 1.0
        rms[2 * d + 3] = 1e-4
        self.rms = torch.tensor(rms, dtype=torch.float64, device=dev)
        self.ret = torch.zeros(n, dtype=torch.float64, device=dev)
        self.lib = _native.load()
        self._ws = torch.empty(int(self.lib.fw_moments_workspace_bytes(n, d)), dtype=torch.uint8, device=dev)
        self._rec = torch.empty(1 + 2 * (d + 1), dtype=torch.float64, device=dev)
        self._rec_ret = torch.empty(3, dtype=torch.float64, device=dev)
        self._parts = None
        self._ensure_parts()
        self._zero_rew = torch.zeros(n, dtype=torch.float32, device=dev)
        self.obs_out = torch.empty(n, d, dtype=torch.float32, device=dev)
        self.rew_out = torch.empty(n, dtype=torch.float32, device=dev)
        self.old_obs = None
        self.old_reward = None
        self.obs_rms = _RMSView(self, "obs")
        self.ret_rms = _RMSView(self, "ret")
        # the env step's own epilogue computes the moment records and the return update (fwsim.h
        # fw_set_collect_epilogue) when the wrapped env is the device engine without a host recorder
        eng = getattr(venv, "engine", None)
        self._epi_ok = (eng is not None and getattr(venv, "_hists", None) is None and hasattr(eng, "collect_records")
                        and d + 1 <= 33)
        self._records, self._n_rec, self._epi_last = None, None, False
        if self._epi_ok:
            self._records = torch.empty(eng.collect_records()[1] * (1 + 2 * (d + 1)), dtype=torch.float64, device=dev)

    # --------------------------------------------------------------- internals
    def _world(self):
        return dist.get_world_size(self.group) if (dist.is_available() and dist.is_initialized()) else 1

    def _ensure_parts(self):
        """Rank-ordered records of the global batch, at fixed addresses (a captured collect step reads them),
        sized for the current process group: a wrapper built before init_process_group is re-sized on first
        use under the group (graph_key carries the world size, so a captured step is recaptured)."""
        W = self._world()
        grouped = dist.is_available() and dist.is_initialized()
        if self._parts is not None and (self._parts.shape[0] == W or not grouped):
            return  # (without a group a caller may stack records itself, as the configs[3] emulation does)
        dev = self.device
        n_rec = 1 + 2 * (self.obs_dim + 1)
        self._parts = torch.empty(W, n_rec, dtype=torch.float64, device=dev)
        self._parts_ret = torch.empty(W, 3, dtype=torch.float64, device=dev)
        # W == 1: the record is written where update_from_moments reads it (no copy per step)
        self._rec = self._parts[0] if W == 1 else torch.empty(n_rec, dtype=torch.float64, device=dev)

    def _s(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def _gather(self, rec):
        """Rank-ordered moment records of the global batch ([W][len]), into the static parts buffer."""
        import torch.distributed as dist
        if rec is self._rec and self._parts.shape[0] == 1 and not (dist.is_available() and dist.is_initialized()):
            return self._parts, 1  # no process group: the record was written in place (_rec aliases _parts[0])
        out = all_gather_flat(rec, self.group, out=self._parts if rec is self._rec else self._parts_ret)
        return out, out.shape[0]

    def _moments(self, obs, rew):
        """This shard's moment record (fw_moments) of obs and of the updated discounted return."""
        d, n = self.obs_dim, self.num_envs
        _native.check(self.lib.fw_moments(_p(obs), n, d, d, _p(rew), _p(self.ret), float(self.gamma), _p(self._ws),
                                          _p(self._rec), self._s()), "fw_moments")

    def _merge(self):
        """RunningMeanStd.update_from_moments over the gathered records (rank order)."""
        d = self.obs_dim
        _native.check(self.lib.fw_rms_update(_p(self._parts), self._parts.shape[0], d, 1, _p(self.rms), 1, 1,
                                             self._s()), "fw_rms_update")

    def _update(self, obs, rew):
        """obs_rms.update(obs) and ret = ret*gamma + rew; ret_rms.update(ret)  (training only)."""
        d, n = self.obs_dim, self.num_envs
        L = self.lib
        s = self._s()
        self._ensure_parts()
        if obs is not None:
            self._moments(obs, rew)
            self._gather(self._rec)
            self._merge()
        else:  # return statistics only (reset)
            _native.check(L.fw_moments(None, n, 0, 0, _p(rew), _p(self.ret), float(self.gamma), _p(self._ws),
                                       _p(self._rec_ret), s), "fw_moments")
            parts, W = self._gather(self._rec_ret)
            # a [1+2*1] record has the layout of a d=0 record with a return column
            self._ret_only_update(parts, W)

    def _ret_only_update(self, parts, W):
        d = self.obs_dim
        tmp = torch.cat([self.rms[2 * d:2 * d + 1], self.rms[2 * d + 1:]])  # [obs_count, ret_mean, ret_var, ret_count]
        _native.check(self.lib.fw_rms_update(_p(parts), W, 0, 1, _p(tmp), 0, 1, self._s()), "fw_rms_update")
        self.rms[2 * d + 1:].copy_(tmp[1:])

    def _apply(self, obs, rew, done, obs_out=None):
        d, n = self.obs_dim, self.num_envs
        obs_out = self.obs_out if obs_out is None else obs_out
        _native.check(self.lib.fw_vecnorm_apply(_p(obs), n, d, d, _p(self.rms), float(self.epsilon),
                                                int(self.norm_obs), float(self.clip_obs),
                                                _p(obs_out) if obs is not None else None, d, _p(rew),
                                                int(self.norm_reward), float(self.clip_reward),
                                                _p(self.rew_out) if rew is not None else None, _p(done),
                                                _p(self.ret), self._s()), "fw_vecnorm_apply")

    def _out(self, t):
        return t if self.return_tensors else t.cpu().numpy()

    # --------------------------------------------------------------- VecEnv API
    def reset(self):
        """vec_normalize.py:209-220."""
        obs = self.venv.reset()
        obs = obs if isinstance(obs, torch.Tensor) else torch.as_tensor(obs, device=self.device)
        obs = obs.to(torch.float32).contiguous()
        self.old_obs = obs
        self.ret.zero_()
        if self.training:
            self._update(None, self._zero_rew)
        self._apply(obs, None, None)
        return self._out(self.obs_out)

    def step_async(self, actions):
        self.venv.step_async(actions)

    def step_wait(self):
        """vec_normalize.py:106-131."""
        self.step_wait_local()
        self.step_exchange()
        return self.step_wait_finish()

    # step_wait in three phases, for a collect step captured as HIP graphs around the collective:
    # local (env step + this shard's moments) | exchange (RCCL all-gather of the records) | finish
    # (update_from_moments in rank order, normalisation).  Phase 1 and 3 launch only kernels.
    def step_wait_local(self):
        epi = self._epi_ok and self.training
        if epi:  # only around this wrapper's own env step: a direct step of the inner env leaves ret alone
            self.set_epilogue()
        try:
            obs, rews, news, infos = self.venv.step_wait()
        finally:
            if epi:
                self.venv.engine.set_collect_epilogue()
        self._epi_last = epi
        obs = obs.to(torch.float32).contiguous()
        rews = rews.to(torch.float32).contiguous()
        self.old_obs, self.old_reward = obs, rews
        self._ensure_parts()
        u8 = news.view(torch.uint8) if (news.dtype == torch.bool and news.is_contiguous()) else news.to(torch.uint8)
        self._news, self._infos, self._done_u8 = news, infos, u8.contiguous()
        if self.training:
            if not epi:
                self._moments(obs, rews)
            elif self.exchanged() and not self.merge_in_launch:  # this shard's record, for the exchange
                self.merge_records(self._rec)

    def step_exchange(self):
        if self.training:
            self._gather(self._rec)

    def step_wait_finish(self):
        if self.training:
            if self._epi_last and not self.exchanged():
                if not self.merge_in_launch:
                    self.merge_update()
            else:
                self._merge()
        self._apply(self.old_obs, self.old_reward, self._done_u8)
        news, infos = self._news, self._infos
        if self.return_tensors:
            return self.obs_out, self.rew_out, news, infos
        return self.obs_out.cpu().numpy(), self.rew_out.cpu().numpy().astype(np.float64), \
            news.cpu().numpy().astype(bool), infos

    # ---- the fused path: records from the env step's epilogue (fwsim.h fw_set_collect_epilogue)
    def exchanged(self):
        """The statistics combine several records (a process group, or a caller stacking shard records)."""
        return self._parts.shape[0] > 1 or (dist.is_available() and dist.is_initialized())

    @property
    def fused_stats(self):
        """The env step writes this wrapper's moment records and return update (training on the engine)."""
        return self._epi_ok and self.training

    # the env step's own launch merges its block records (and, unsharded, updates the statistics): a
    # collect step is then two launches (fwsim.h fw_collect_epilogue.merged / .rms); False = the merge (+
    # update) as a separate launch after the env step (fw_vecnorm_merge_update / fw_moments_merge)
    merge_in_launch = True

    def set_epilogue(self, row_ctrl=None, defer=False):
        """Point the engine's collect epilogue at this wrapper's return and record buffers (and, for a
        captured collect step, the rollout row counter).  With ``merge_in_launch`` the launch also writes the
        merged record into ``_rec`` and, without an exchange, applies it to ``rms``.  ``defer`` (unsharded,
        with ``merge_in_launch``): the launch stops the merge one level short; the fused collect's next policy
        launch finishes it (``pending_fields``), or ``pending_update`` does."""
        eng = self.venv.engine
        self._ensure_parts()
        merged = self._rec if self.merge_in_launch else None
        rms = self.rms if (self.merge_in_launch and not self.exchanged()) else None
        defer = bool(defer and rms is not None)
        eng.set_collect_epilogue(ret=self.ret, gamma=self.gamma, records=self._records, row_ctrl=row_ctrl,
                                 merged=merged, rms=rms, defer=defer)
        self._n_rec = eng.collect_records()[0]
        self._pend = eng.collect_pending() if defer else None

    # the deferred final level fits one policy block's LDS staging (fw_rollout.hip PEND_MAX fields x records)
    PEND_MAX = 2048

    def pending_fields(self):
        """(pend, stride, count, has_ret, merged, rms_prev) for fw_collect_io, or None when the epilogue set by
        ``set_epilogue`` does not defer."""
        if getattr(self, "_pend", None) is None:
            return None
        rec, stride, cnt, D, rms_prev = self._pend
        return rec, stride, cnt, 1, self._rec.data_ptr(), rms_prev

    def pending_update(self, pend=None):
        """fw_vecnorm_pending_update: apply a deferred final merge (after a collection's last env step)."""
        rec, stride, cnt, D, _ = pend if pend is not None else self._pend
        _native.check(self.lib.fw_vecnorm_pending_update(rec, stride, cnt, self.obs_dim, 1, _p(self.rms),
                                                         _p(self._rec), self._s()), "fw_vecnorm_pending_update")

    def merge_records(self, out):
        """fw_moments_merge of the env step's block records into one (obs + return) record."""
        d = self.obs_dim
        _native.check(self.lib.fw_moments_merge(_p(self._records), self._n_rec, d + 1, _p(out), self._s()),
                      "fw_moments_merge")

    def merge_update(self):
        """fw_vecnorm_merge_update: the records merged and applied to the running statistics, one launch
        (the merged record also lands in _rec)."""
        d = self.obs_dim
        _native.check(self.lib.fw_vecnorm_merge_update(_p(self._records), self._n_rec, d, 1, _p(self.rms),
                                                       _p(self._rec), self._s()), "fw_vecnorm_merge_update")

    def graph_key(self):
        """Host-side choices a captured step bakes in (RolloutCollector recaptures when this changes)."""
        inner = self.venv.graph_key() if hasattr(self.venv, "graph_key") else None
        return (self.training, self.norm_obs, self.norm_reward, self.clip_obs, self.clip_reward, self.gamma,
                self.epsilon, self._world(), self._epi_ok, self.merge_in_launch, inner)

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def normalize_obs(self, obs):
        """vec_normalize.py:148-159 with the current statistics, any number of rows."""
        o = torch.as_tensor(obs, dtype=torch.float32, device=self.device).reshape(-1, self.obs_dim).contiguous()
        out = torch.empty_like(o)
        d = self.obs_dim
        _native.check(self.lib.fw_vecnorm_apply(_p(o), o.shape[0], d, d, _p(self.rms), float(self.epsilon),
                                                int(self.norm_obs), float(self.clip_obs), _p(out), d, None, 0, 0.0,
                                                None, None, None, self._s()), "fw_vecnorm_apply")
        return self._out(out)

    def normalize_reward(self, reward):
        """vec_normalize.py:161-169 with the current statistics (device tensors in, same shape out)."""
        r = torch.as_tensor(reward, device=self.device)
        if not self.norm_reward:
            return r
        d = self.obs_dim
        scale = torch.sqrt(self.rms[2 * d + 2] + self.epsilon)
        return torch.clamp(r.double() / scale, -self.clip_reward, self.clip_reward).to(r.dtype)

    def get_original_obs(self):
        return self._out(self.old_obs)

    def get_original_reward(self):
        return self._out(self.old_reward)

    def close(self):
        self.venv.close()

    def __getattr__(self, name):  # env_method / get_attr / set_attr / seed ... pass through
        if name in ("venv",):
            raise AttributeError(name)
        return getattr(self.venv, name)

    def save(self, path):
        np.savez(path, rms=self.rms.cpu().numpy(), obs_dim=self.obs_dim, gamma=self.gamma, epsilon=self.epsilon,
                 clip_obs=self.clip_obs, clip_reward=self.clip_reward, norm_obs=self.norm_obs,
                 norm_reward=self.norm_reward)

    def load_stats(self, path):
        with np.load(path, allow_pickle=False) as z:
            if int(z["obs_dim"]) != self.obs_dim:
                raise ValueError("observation size mismatch")
            self.rms.copy_(torch.as_tensor(z["rms"]))
