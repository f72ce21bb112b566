/*
 * fwrollout.h -- C ABI of the rollout-side kernels in libfwsim.so: the device
 * RolloutBuffer's GAE scan and the device VecNormalize statistics.
 *
 * These are the consumers directly downstream of fw_env_step in SB3's
 * collect_rollouts.  Same conventions as fwsim.h:
 * device pointers, `void* stream` = hipStream_t, int return codes,
 * fw_last_error() for the message.  All buffers are row-major
 * [n_steps][n_envs] like SB3's numpy buffers (buffer_size, n_envs).
 *
 * Reference interfaces replaced (paths relative to magpie/libs/stable-baselines3/):
 *   fw_gae            RolloutBuffer.compute_returns_and_advantage
 *                     stable_baselines3/common/buffers.py:304-333
 *   fw_moments_*      RunningMeanStd.update (np.mean / np.var over the batch)
 *                     stable_baselines3/common/running_mean_std.py:20-24
 *   fw_rms_update     RunningMeanStd.update_from_moments  running_mean_std.py:26-40,
 *                     merged over ranks (the global batch of a sharded VecEnv)
 *   fw_vecnorm_apply  VecNormalize.step_wait's normalisation + return reset
 *                     stable_baselines3/common/vec_env/vec_normalize.py:106-131, 133-169
 *   fw_replay_add     ReplayBuffer.add   stable_baselines3/common/buffers.py:222-235
 *   fw_rollout_store  RolloutBuffer.add  stable_baselines3/common/buffers.py:335-361, with the row
 *                     index on the device so a captured collect step stores its own row
 *   fw_policy_forward ActorCriticPolicy.forward of the default PPO MlpPolicy
 *                     stable_baselines3/common/policies.py:539-553 (+ the action clip of
 *                     on_policy_algorithm.py:158-161), one launch per collect step
 */
#ifndef FWROLLOUT_H
#define FWROLLOUT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* GAE(lambda) + returns over a [n_steps][n_envs] rollout, float32 storage like SB3.
 *   rewards, values      [n_steps][n_envs] float
 *   episode_starts       [n_steps][n_envs] uint8   (SB3's `dones` column: done flag of the
 *                                                   PREVIOUS step, i.e. _last_dones at add())
 *   last_values          [n_envs] float            (value of the obs after the last step)
 *   last_dones           [n_envs] uint8            (dones returned by the last step)
 *   advantages, returns  [n_steps][n_envs] float   (outputs; may not alias inputs)
 * Arithmetic reproduces numpy's promotions in the reference loop bit for bit: fp32
 * deltas, an fp64 running advantage (the last step's 1.0 - bool promotes to float64),
 * fp32 stores.  One lane per env, sequential in time. */
int fw_gae(const float* rewards, const float* values, const uint8_t* episode_starts, const float* last_values,
           const uint8_t* last_dones, int64_t n_steps, int64_t n_envs, double gamma, double gae_lambda,
           float* advantages, float* returns, void* stream);

/* Batch moments of the columns of x [n][d] (float, row stride ldx >= d) and, optionally,
 * of the discounted return after the update ret <- ret * gamma + rew (rew may be NULL =
 * no return column; ret is fp64 [n] and updated in place).
 * Output (fp64, D = d + (rew != NULL)):  out[0] = n, out[1 .. D] = mean, out[1+D .. 2D] = M2
 * (sum of squared deviations; np.var = M2 / n).  `workspace` must hold
 * fw_moments_workspace_bytes(n, d) bytes of device memory. */
size_t fw_moments_workspace_bytes(int64_t n, int32_t d);
int fw_moments(const float* x, int64_t n, int32_t d, int64_t ldx, const float* rew, double* ret, double gamma,
               void* workspace, double* out, void* stream);

/* Merge `n_parts` moment records (each 1 + 2D doubles, rank order, e.g. the all-gather of
 * fw_moments outputs) into the running statistics with RunningMeanStd.update_from_moments.
 *   rms layout (fp64): [obs_mean d][obs_var d][obs_count][ret_mean][ret_var][ret_count]
 * update_obs / update_ret select which RunningMeanStd objects are updated. */
int fw_rms_update(const double* parts, int32_t n_parts, int32_t d, int32_t has_ret, double* rms, int32_t update_obs,
                  int32_t update_ret, void* stream);

/* Normalise one step: obs_out = float(clip((obs - mean) / sqrt(var + eps), +-clip_obs)),
 * rew_out = float(clip(rew / sqrt(ret_var + eps), +-clip_rew)), then ret[done] = 0.
 * obs_out / rew_out may be NULL (not requested); norm_obs / norm_rew = 0 copies through. */
int fw_vecnorm_apply(const float* obs, int64_t n, int32_t d, int64_t ldx, const double* rms, double epsilon,
                     int32_t norm_obs, double clip_obs, float* obs_out, int64_t ld_out, const float* rew,
                     int32_t norm_rew, double clip_rew, float* rew_out, const uint8_t* done, double* ret,
                     void* stream);

/* ReplayBuffer.add (stable_baselines3/common/buffers.py:222-235) for n_envs transitions at once:
 * one launch copies up to FW_MAX_COPY_SEGS device ranges (obs, next_obs, action, reward, done of
 * the current step into their replay slots).  Ranges must not overlap; bytes % 4 == 0; 16-byte
 * aligned ranges move as 16-byte vectors. */
#define FW_MAX_COPY_SEGS 8
typedef struct fw_copy_seg {
  const void* src;
  void* dst;
  int64_t bytes;
} fw_copy_seg;
int fw_replay_add(const fw_copy_seg* segs, int32_t n_segs, void* stream);

/* RolloutBuffer.add (stable_baselines3/common/buffers.py:335-361) as a graph-capturable launch: the
 * buffer row comes from device memory, ctrl_dev = {row, n_rows} (int32).  Segment k copies `bytes`
 * from src to dst + (row + row_off) * stride, skipped when row + row_off is outside [0, n_rows);
 * then, if advance != 0, ctrl_dev[0] += 1 (a second, single-thread launch on the same stream).
 * A captured collect step replays the same launch every step and still fills row t at step t.
 * Ranges must not overlap; bytes % 4 == 0. */
typedef struct fw_row_seg {
  const void* src;
  void* dst;
  int64_t bytes;
  int64_t stride;
  int32_t row_off;
  int32_t pad;
} fw_row_seg;
int fw_rollout_store(const fw_row_seg* segs, int32_t n_segs, int32_t* ctrl_dev, int32_t advance, void* stream);

/* The default PPO MlpPolicy's forward for one collect step (SB3 ActorCriticPolicy.forward,
 * stable_baselines3/common/policies.py:539-553, DiagGaussianDistribution distributions.py:143-171):
 * two tanh MLPs [d -> hidden -> hidden] (actor, critic; nn.Linear weights [out][in], row-major),
 * mean = act_w h + act_b, value = val_w h + val_b, action = mean + exp(log_std) * noise (noise [n][A],
 * NULL = deterministic), log_prob = sum_a (-(action-mean)^2 / (2 std^2) - log_std - log(2 pi)/2),
 * clipped = min(max(action, low), high) (on_policy_algorithm.py:158-161; clipped may be NULL).
 * Parameters are read in place (device pointers), so an optimiser step is seen by the next launch.
 * Limits: d <= 32, hidden == 64 (SB3's default net_arch [64, 64]), act_dim <= 8.  fp32 FMA arithmetic: equal to the torch module's
 * forward within ~1e-6, not bit for bit (a different summation order than the BLAS GEMMs). */
typedef struct fw_mlp_policy {
  const float *pi_w0, *pi_b0, *pi_w1, *pi_b1, *act_w, *act_b;
  const float *vf_w0, *vf_b0, *vf_w1, *vf_b1, *val_w, *val_b;
  const float* log_std;
  /* optional device int32: the noise rows of the whole collection are in `noise` ([T][n][A]) and this
   * launch reads row *noise_row (e.g. fw_rollout_store's ctrl[0]), so a captured step draws no RNG */
  const int32_t* noise_row;
  int32_t d, hidden, act_dim, pad;
} fw_mlp_policy;
int fw_policy_forward(const fw_mlp_policy* p, const float* obs, int64_t n, const float* noise, const float* low,
                      const float* high, float* actions, float* clipped, float* values, float* log_probs, void* stream);

/* Two-pass merge of n_records moment records (1 + 2D doubles each: n_b, mean_b[D], M2_b[D], e.g. the
 * per-block records of fw_env_step's collect epilogue, fwsim.h fw_set_collect_epilogue; stored
 * column-major, field f of record b at records[f * n_records + b]) into one record `out` (1 + 2D doubles):
 * mean = sum n_b mean_b / N, M2 = sum (M2_b + n_b (mean_b - mean)^2), every sum in
 * a fixed order.  The batch moments of RunningMeanStd.update (running_mean_std.py:20-24). */
int fw_moments_merge(const double* records, int32_t n_records, int32_t D, double* out, void* stream);

/* fw_moments_merge of the records (obs columns d, plus the return column when has_ret) followed by
 * fw_rms_update of that single record, in ONE launch (the unsharded VecNormalize statistics update,
 * vec_normalize.py:106-131 -> running_mean_std.py:20-40): bit-identical to the two calls.  rec_out (may be
 * NULL) receives the merged record. */
int fw_vecnorm_merge_update(const double* records, int32_t n_records, int32_t d, int32_t has_ret, double* rms,
                            double* rec_out, void* stream);

/* One PPO collect step's policy side, fused (OnPolicyAlgorithm.collect_rollouts,
 * on_policy_algorithm.py:140-176 for the default MlpPolicy): reads the env's RAW step output, normalises the
 * observation with VecNormalize's current statistics (vec_normalize.py:148-159), runs the policy (as
 * fw_policy_forward), and stores the rollout rows (RolloutBuffer.add, buffers.py:335-361) at row t = ctrl[0]:
 *   obs_rows[t] = normalised obs, act_rows[t], val_rows[t], logp_rows[t];  the clipped actions -> `clipped`
 *   (the env's next action input); when t >= 1 also rew_rows[t-1] = the normalised reward of the previous
 *   step (vec_normalize.py:161-169) and start_rows[t] = that step's done flags (the next episode start).
 * rms NULL: observation and reward taken raw (no VecNormalize).  The row index advances elsewhere (the env
 * step's collect epilogue), so a captured graph of {this, fw_env_step, ...} fills row t at its t-th replay.
 * Noise (NULL = deterministic): [T][n][A], row t read.  Limits as fw_policy_forward; float32. */
typedef struct fw_collect_io {
  const float* obs;         /* [n][d] raw observation of the previous env step */
  const float* reward;      /* [n] raw reward of the previous env step */
  const uint8_t* done;      /* [n] done flags of the previous env step */
  const double* rms;        /* fwrollout.h rms layout, or NULL */
  double epsilon, clip_obs, clip_reward;
  int32_t norm_obs, norm_reward;
  const float* noise;       /* [T][n][A] or NULL */
  const float *low, *high;  /* action space bounds [A] */
  float* clipped;           /* [n][A] */
  const int32_t* ctrl;      /* device {t, n_rows} */
  float *obs_rows, *act_rows, *val_rows, *logp_rows, *rew_rows;
  uint8_t* start_rows;
  int64_t n;
  /* ABI 12: the statistics update the env step deferred (fwsim.h fw_collect_epilogue.defer; the fields of
   * fw_collect_pending).  When pend is set and t >= 1, every block merges the pend_cnt records and applies
   * update_from_moments to the statistics the env step found (rms_prev) before normalising; block 0 writes
   * the updated statistics to rms (in place) and the merged record (merged [1 + 2D], may be NULL).  At
   * t = 0 nothing is pending (the previous collection ended with fw_vecnorm_pending_update).  NULL: off. */
  const double* pend;
  int64_t pend_stride;
  int32_t pend_cnt, has_ret;
  double* merged;
  const double* rms_prev;
} fw_collect_io;
int fw_collect_policy(const fw_mlp_policy* p, const fw_collect_io* io, void* stream);

/* ABI 12: the deferred final merge on its own (after a collection's last env step): merges the cnt records
 * (fw_collect_pending's layout), applies update_from_moments to rms [2d + 4] and writes the merged record
 * (merged may be NULL) -- the same bits as the merging fw_collect_policy launch and as the env step's own
 * final node. */
int fw_vecnorm_pending_update(const double* pend, int64_t stride, int32_t cnt, int32_t d, int32_t has_ret,
                              double* rms, double* merged, void* stream);

#ifdef __cplusplus
}
#endif
#endif
