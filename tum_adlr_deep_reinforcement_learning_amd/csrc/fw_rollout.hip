// fw_rollout.hip -- rollout-side kernels of libfwsim.so (include/fwrollout.h):
// the device RolloutBuffer's GAE scan and the device VecNormalize statistics.
//
//   k_gae              RolloutBuffer.compute_returns_and_advantage
//                      (stable_baselines3/common/buffers.py:304-333).  One lane per env,
//                      reverse scan over time; rows [t][N] are read coalesced and
//                      prefetched GAE_PF steps ahead (the recurrence is serial, the loads
//                      are not).  HBM-bound: 4+4+1 B read, 4+4 B written per (step, env).
//   k_moments_partial  RunningMeanStd.update's batch mean/var (running_mean_std.py:20-24):
//   k_moments_merge    per-block two-pass records, then a two-pass merge of the records, every
//                      sum in a fixed order -> deterministic.
//   k_rms_update       update_from_moments (running_mean_std.py:26-40) over rank-ordered
//                      moment records (the RCCL all-gather of a sharded batch).
//   k_vecnorm_apply    VecNormalize.normalize_obs / normalize_reward + ret[news] = 0
//                      (vec_normalize.py:106-131, 133-169).
//   k_copy_segs        ReplayBuffer.add (buffers.py:222-235): all fields of one step, one launch.
//
// Floating point follows the reference's numpy promotions exactly where the reference
// is deterministic (GAE: bit-exact), so contraction into FMA is disabled in this file.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <string>

#include "../../include/fwrollout.h"
#include "../../include/fwsim.h"
#include "fw_stats.hpp"

#pragma clang fp contract(off)

namespace fw {
int set_error(int code, const std::string& msg);
}

namespace {

constexpr int BLOCK = 256;
constexpr int GAE_PF = 16;   // time steps loaded ahead per lane
constexpr int MAXD = 33;     // observation dims (FW_MAX_OBS) + the return column

#define FW_HIP(expr)                                                                                     \
  do {                                                                                                   \
    hipError_t e_ = (expr);                                                                              \
    if (e_ != hipSuccess) return fw::set_error(FW_E_HIP, std::string(#expr ": ") + hipGetErrorString(e_)); \
  } while (0)

// ---------------------------------------------------------------------------
// GAE.  numpy's evaluation of buffers.py:321-331, per element:
//   step T-1: nnt = 1.0 - dones (bool -> float64); a = f32(gamma)*last_value (f32);
//             delta = ((f64)r + (f64)a*nnt) - (f64)v      (float64)
//             last  = delta + (gamma*lam*nnt)*0            (float64)
//   step t  : nnt = 1.0 - starts[t+1] (float32); a = f32(gamma)*values[t+1]; b = a*nnt;
//             delta = (r + b) - v                          (float32, each op rounded)
//             last  = (f64)delta + (f64)(f32(gamma*lam)*nnt) * last   (float64)
//   adv[t] = f32(last); ret[t] = adv[t] + v                 (float32)
// ---------------------------------------------------------------------------
// A product that feeds an addition goes through this barrier: the __dmul_rn / __dadd_rn (and f32) header
// functions carry the default fp-contract flags, so after inlining the backend fused them into an FMA
// despite the file's contract(off) -- one element in 16.7M of a 65536 x 256 rollout was 1 ulp off
// numpy's (test_c3_rollout_collector_full_size); an opaque register keeps multiply and add separate.
template <typename F>
__device__ __forceinline__ F nofuse(F x) {
  asm volatile("" : "+v"(x));
  return x;
}

__global__ __launch_bounds__(BLOCK) void k_gae(const float* __restrict__ rew, const float* __restrict__ val,
                                               const uint8_t* __restrict__ starts, const float* __restrict__ last_v,
                                               const uint8_t* __restrict__ last_d, int64_t T, int64_t N, float gamma_f,
                                               double gl, float gl_f, float* __restrict__ adv, float* __restrict__ ret) {
  const int64_t e = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
  if (e >= N) return;
  int64_t t = T - 1;
  float v = val[t * N + e];
  {
    const double nnt = last_d[e] ? 0.0 : 1.0;
    const float a = __fmul_rn(gamma_f, last_v[e]);
    const double delta = __dsub_rn(__dadd_rn((double)rew[t * N + e], nofuse(__dmul_rn((double)a, nnt))), (double)v);
    const double last0 = __dadd_rn(delta, nofuse(__dmul_rn(__dmul_rn(gl, nnt), 0.0)));
    const float af = (float)last0;
    adv[t * N + e] = af;
    ret[t * N + e] = __fadd_rn(af, v);
    double last = last0;
    float nv = v;
    uint8_t nstart = starts[t * N + e];
    for (int64_t t0 = T - 2; t0 >= 0; t0 -= GAE_PF) {
      float rr[GAE_PF], vv[GAE_PF];
      uint8_t ss[GAE_PF];
#pragma unroll
      for (int k = 0; k < GAE_PF; k++) {
        const int64_t tt = t0 - k;
        if (tt >= 0) {
          rr[k] = rew[tt * N + e];
          vv[k] = val[tt * N + e];
          ss[k] = starts[tt * N + e];
        }
      }
#pragma unroll
      for (int k = 0; k < GAE_PF; k++) {
        const int64_t tt = t0 - k;
        if (tt >= 0) {
          const float nnt = nstart ? 0.f : 1.f;
          const float b = nofuse(__fmul_rn(__fmul_rn(gamma_f, nv), nnt));
          const float dl = __fsub_rn(__fadd_rn(rr[k], b), vv[k]);
          const float coef = __fmul_rn(gl_f, nnt);
          last = __dadd_rn((double)dl, nofuse(__dmul_rn((double)coef, last)));
          const float a2 = (float)last;
          adv[tt * N + e] = a2;
          ret[tt * N + e] = __fadd_rn(a2, vv[k]);
          nv = vv[k];
          nstart = ss[k];
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// batch moments
// ---------------------------------------------------------------------------
using fw_stats::Mom;  // (fw_stats.hpp: shared with k_env_step's in-launch merge)
using fw_stats::chan;
using fw_stats::rms_update;

// Batch moments in two kernels, both exact two-pass (numpy's np.mean then np.var of the deviations):
//   k_moments_partial  one block per MROWS rows: the rows staged column-major in LDS, the block's mean
//                      (column sum / rows) then its M2 = sum (x - mean)^2 from LDS -> record (n_b, mean_b, M2_b)
//   k_moments_merge    the records of the whole batch: mean = sum n_b mean_b / N, then
//                      M2 = sum (M2_b + n_b (mean_b - mean)^2) -- sums only, no per-record division
// Every sum runs in a fixed order (strided lane partials, then a butterfly), so results are deterministic.
// Round 2's per-thread Welford + Chan LDS tree (a division per element, 8 barriers per column) took
// 44 + 35 us per call at 65536 x 16 (profiles/r03_collect_kernels.csv); this is memory-bound.
constexpr int MROWS = BLOCK;  // rows per moment record
constexpr int MGRP = 8;       // threads per column in k_moments_partial

__device__ __forceinline__ double grp_sum8(double s) {  // sum over an aligned group of 8 lanes, same bits on all
  s += __shfl_xor(s, 1);
  s += __shfl_xor(s, 2);
  s += __shfl_xor(s, 4);
  return s;
}
__device__ __forceinline__ double wave_sum(double s) {  // butterfly over the 64 lanes, same bits on all
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) s += __shfl_xor(s, m);
  return s;
}

__global__ __launch_bounds__(BLOCK) void k_moments_partial(const float* __restrict__ x, int64_t n, int d, int64_t ldx,
                                                           const float* __restrict__ rew, double* __restrict__ retv,
                                                           double gamma, double* __restrict__ part) {
  __shared__ float sx[MAXD - 1][MROWS + 8];  // the block's rows, column-major (fp32: exact); +8: the columns a
                                             // wave reads at once start 8 banks apart
  __shared__ double sr[MROWS];           // the updated discounted return column
  __shared__ double smean[MAXD];
  const int D = d + (rew ? 1 : 0);
  const int64_t r0 = (int64_t)blockIdx.x * MROWS;
  const int nb = (int)std::min<int64_t>(MROWS, n - r0);
  if (d > 0) {
    if (ldx == d) {  // contiguous chunk: flat coalesced reads
      const float* src = x + r0 * d;
      for (int f = threadIdx.x; f < nb * d; f += BLOCK) {
        const int r = f / d;
        sx[f - r * d][r] = src[f];
      }
    } else {
      for (int f = threadIdx.x; f < nb * d; f += BLOCK) {
        const int r = f / d, j = f - r * d;
        sx[j][r] = x[(r0 + r) * ldx + j];
      }
    }
  }
  if (rew && (int)threadIdx.x < nb) {  // VecNormalize._update_reward: ret = ret * gamma + reward (vec_normalize.py:126-129)
    const int64_t r = r0 + threadIdx.x;
    const double v = retv[r] * gamma + (double)rew[r];
    retv[r] = v;
    sr[threadIdx.x] = v;
  }
  __syncthreads();
  const int sub = threadIdx.x % MGRP, cg = threadIdx.x / MGRP;
  constexpr int NCG = BLOCK / MGRP;
  const double dn = (double)nb;
  for (int j = cg; j < D; j += NCG) {  // pass 1: column sums -> block mean
    double s = 0.0;
    for (int k = sub; k < nb; k += MGRP) s += j < d ? (double)sx[j][k] : sr[k];
    s = grp_sum8(s);
    if (sub == 0) smean[j] = s / dn;
  }
  __syncthreads();
  // column-major records (field q of block b at part[q * blocks + b]): merge_records reads them coalesced
  double* out = part + blockIdx.x;
  const int64_t qs = gridDim.x;
  for (int j = cg; j < D; j += NCG) {  // pass 2: sum of squared deviations
    const double m = smean[j];
    double q = 0.0;
    for (int k = sub; k < nb; k += MGRP) {
      const double dv = (j < d ? (double)sx[j][k] : sr[k]) - m;
      q += dv * dv;
    }
    q = grp_sum8(q);
    if (sub == 0) {
      out[(1 + j) * qs] = m;
      out[(1 + D + j) * qs] = q;
    }
  }
  if (threadIdx.x == 0) out[0] = dn;  // field 0
}

// merges `parts` records (column-major: field q of record k at part[q * parts + k]; q = 0 count, 1..D means,
// D+1..2D M2) into one record `out` (contiguous 1 + 2D), two-pass: mean = sum n_b mean_b / N, then
// M2 = sum (M2_b + n_b (mean_b - mean)^2).  Thread t folds records t, t + MERGE_THREADS, ... (coalesced per
// field, every field of a record in one batch of loads), the per-thread partials go through LDS, and thread
// j sums column j over the threads in 8 interleaved chains combined in a fixed order: deterministic, and no
// fp64 cross-lane shuffles (a butterfly per column and pass serialised ~180 LDS round trips: 30 us).
constexpr int MERGE_THREADS = 256;
__device__ __forceinline__ double col_sum(const double* c) {  // c[0..MERGE_THREADS), fixed order
  double p[8];
#pragma unroll
  for (int k = 0; k < 8; k++) p[k] = c[k];
  for (int t = 8; t < MERGE_THREADS; t += 8)
#pragma unroll
    for (int k = 0; k < 8; k++) p[k] += c[t + k];
  return ((p[0] + p[1]) + (p[2] + p[3])) + ((p[4] + p[5]) + (p[6] + p[7]));
}
__device__ __forceinline__ void merge_records(const double* __restrict__ part, int parts, int D, double* __restrict__ out) {
  __shared__ double tp[MAXD + 1][MERGE_THREADS];  // per-thread partials, column-major; row MAXD: the counts
  __shared__ double smean[MAXD + 1];              // column means; [MAXD]: N
  const int tid = threadIdx.x;
  double acc[MAXD], cn = 0.0;
#pragma unroll
  for (int j = 0; j < MAXD; j++) acc[j] = 0.0;
  // loads from clamped indices, unconditionally (a load in a D-guarded block is waited for right there)
  for (int k = tid; k < parts; k += MERGE_THREADS) {  // pass 1
    const double* r = part + k;
    const double nk = r[0];
    double m[MAXD];
#pragma unroll
    for (int j = 0; j < MAXD; j++) m[j] = r[(int64_t)(1 + (j < D ? j : D - 1)) * parts];
    cn += nk;
#pragma unroll
    for (int j = 0; j < MAXD; j++) acc[j] += j < D ? nk * m[j] : 0.0;
  }
#pragma unroll
  for (int j = 0; j < MAXD; j++)
    if (j < D) tp[j][tid] = acc[j];
  tp[MAXD][tid] = cn;
  __syncthreads();
  if (tid <= D) {
    const int j = tid == D ? MAXD : tid;
    smean[j] = col_sum(tp[j]);
  }
  __syncthreads();
  const double N = smean[MAXD];
  if (tid < D) smean[tid] = smean[tid] / N;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < MAXD; j++) acc[j] = 0.0;
  for (int k = tid; k < parts; k += MERGE_THREADS) {  // pass 2
    const double* r = part + k;
    const double nk = r[0];
    double m[MAXD], q[MAXD];
#pragma unroll
    for (int j = 0; j < MAXD; j++) {
      const int jc = j < D ? j : D - 1;
      m[j] = r[(int64_t)(1 + jc) * parts];
      q[j] = r[(int64_t)(1 + D + jc) * parts];
    }
#pragma unroll
    for (int j = 0; j < MAXD; j++) {
      const double dm = m[j] - smean[j < D ? j : D - 1];
      acc[j] += j < D ? q[j] + nk * (dm * dm) : 0.0;
    }
  }
  __syncthreads();  // (every thread has read smean; tp is rewritten below)
#pragma unroll
  for (int j = 0; j < MAXD; j++)
    if (j < D) tp[j][tid] = acc[j];
  __syncthreads();
  if (tid < D) {
    out[1 + tid] = smean[tid];
    out[1 + D + tid] = col_sum(tp[tid]);
    if (tid == 0) out[0] = N;
  }
}

// The common case, D <= 15 columns (the default task: 14 observation values + the return; the count takes
// column D of the 16-column staging), 256 threads: a
// thread's records (four at 65536 envs) are loaded in ONE batch per pass (the general kernel waits a memory
// round trip per record), only the D live columns are read, and the column sums are two-level through LDS
// (16 threads per column, 16 values each, in order; then the 16 partials in order) -- fp64 cross-lane
// butterflies serialised ~100 dependent LDS round trips per pass (tools/merge_bench.py: 19 us at 64 records).
constexpr int MERGE16_THREADS = 256, MERGE16_BATCH = 4;
__device__ __forceinline__ double sum16_cols(double (*tp)[MERGE16_THREADS + 1], double (*pp)[17], int ncols) {
  // column j (< ncols) of tp summed over the 256 threads: thread 16 j + h sums threads h, h + 16, ..., h + 240
  // (the 16 lanes of a column read 16 consecutive doubles per step: no LDS bank conflicts; contiguous runs of
  // 16 per lane, 128 B apart, conflicted 16 ways)
  const int tid = threadIdx.x, j = tid >> 4, h = tid & 15;
  if (j < ncols) {
    double a = 0.0;
#pragma unroll
    for (int k = 0; k < 16; k++) a += tp[j][h + 16 * k];
    pp[j][h] = a;
  }
  __syncthreads();
  double r = 0.0;
  if (tid < ncols)
#pragma unroll
    for (int k = 0; k < 16; k++) r += pp[tid][k];
  return r;  // on thread j
}
__device__ __forceinline__ void merge_records16(const double* __restrict__ part, int parts, int D,
                                                double* __restrict__ out) {
  // parts <= MERGE16_THREADS * MERGE16_BATCH: a thread's records are loaded ONCE (one memory round trip) and
  // both passes run from registers
  constexpr int MD = 16, BT = MERGE16_BATCH;
  __shared__ double tp[MD + 1][MERGE16_THREADS + 1];  // per-thread partials
  __shared__ double pp[MD + 1][17];
  __shared__ double smean[MD + 1];
  const int tid = threadIdx.x;
  double nk[BT], m[BT][MD], q[BT][MD];
#pragma unroll
  for (int b = 0; b < BT; b++) {
    const int k = tid + b * MERGE16_THREADS, kc = k < parts ? k : parts - 1;
    nk[b] = part[kc];
#pragma unroll
    for (int j = 0; j < MD; j++) {
      const int jc = j < D ? j : D - 1;
      m[b][j] = part[(int64_t)(1 + jc) * parts + kc];
      q[b][j] = part[(int64_t)(1 + D + jc) * parts + kc];
    }
    if (k >= parts) nk[b] = -1.0;  // padding slot
  }
  double acc[MD], cn = 0.0;
#pragma unroll
  for (int j = 0; j < MD; j++) acc[j] = 0.0;
#pragma unroll
  for (int b = 0; b < BT; b++) {  // pass 1
    const double w = nk[b] >= 0.0 ? nk[b] : 0.0;
    cn += w;
#pragma unroll
    for (int j = 0; j < MD; j++) acc[j] += j < D ? w * m[b][j] : 0.0;
  }
#pragma unroll
  for (int j = 0; j < MD; j++) tp[j][tid] = acc[j];
  __syncthreads();
  tp[D][tid] = cn;  // the count in column D (D <= 15: a zero column of acc)
  __syncthreads();
  {
    const double v = sum16_cols(tp, pp, D + 1);
    if (tid <= D) smean[tid == D ? MD : tid] = v;
  }
  __syncthreads();
  const double N = smean[MD];
  if (tid < D) smean[tid] = smean[tid] / N;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < MD; j++) acc[j] = 0.0;
#pragma unroll
  for (int b = 0; b < BT; b++)  // pass 2
#pragma unroll
    for (int j = 0; j < MD; j++) {
      const double dm = m[b][j] - smean[j < D ? j : D - 1];
      acc[j] += (j < D && nk[b] >= 0.0) ? q[b][j] + nk[b] * (dm * dm) : 0.0;
    }
#pragma unroll
  for (int j = 0; j < MD; j++) tp[j][tid] = acc[j];
  __syncthreads();
  const double m2 = sum16_cols(tp, pp, D);
  if (tid < D) {
    out[1 + tid] = smean[tid];
    out[1 + D + tid] = m2;
    if (tid == 0) out[0] = N;
  }
}

__global__ __launch_bounds__(MERGE16_THREADS) void k_moments_merge16(const double* __restrict__ part, int parts, int D,
                                                                     double* __restrict__ out) {
  merge_records16(part, parts, D, out);
}

__global__ __launch_bounds__(MERGE_THREADS) void k_moments_merge(const double* __restrict__ part, int parts, int D,
                                                                    double* __restrict__ out) {
  merge_records(part, parts, D, out);
}

__global__ void k_rms_update(const double* __restrict__ parts, int n_parts, int d, int has_ret, double* __restrict__ rms,
                             int update_obs, int update_ret) {
  __shared__ double old_count[2];
  rms_update(parts, n_parts, d, has_ret, rms, update_obs, update_ret, old_count);
}

__global__ __launch_bounds__(MERGE16_THREADS) void k_merge_update16(const double* __restrict__ part, int parts, int d,
                                                                    int has_ret, double* __restrict__ rms,
                                                                    double* __restrict__ rec_out) {
  __shared__ double rec[1 + 2 * MAXD];
  __shared__ double old_count[2];
  const int D = d + (has_ret ? 1 : 0);
  merge_records16(part, parts, D, rec);
  __syncthreads();
  if (rec_out)
    for (int k = threadIdx.x; k < 1 + 2 * D; k += blockDim.x) rec_out[k] = rec[k];
  rms_update(rec, 1, d, has_ret, rms, 1, 1, old_count);
}

// The env step's deferred final merge (fw_collect_epilogue.defer) on its own: one wave, lane j < D owns column
// j; the same functions (fw_stats::merge_col / update_col) as k_policy_mfma's prologue and the same bits as the
// in-launch final node + rms_update.
__global__ __launch_bounds__(64) void k_pending_update(const double* __restrict__ pend, int64_t stride, int cnt, int d,
                                                       int has_ret, double* __restrict__ rms, double* __restrict__ merged) {
  const int j = threadIdx.x, D = d + has_ret;
  const double c_obs = rms[2 * d], c_ret = rms[2 * d + 3];
  const bool is_ret = has_ret && j == d;
  double N = 0.0, mu = 0.0, m2 = 0.0, mean = 0.0, var = 0.0;
  if (j < D) {
    fw_stats::merge_col(pend, pend + (1 + j) * stride, pend + (1 + D + j) * stride, cnt, N, mu, m2);
    mean = rms[is_ret ? 2 * d + 1 : j];
    var = rms[is_ret ? 2 * d + 2 : d + j];
    fw_stats::update_col(mu, m2 / N, N, is_ret ? c_ret : c_obs, mean, var);
  }
  __syncthreads();  // (every lane read the counts before lane 0 / the return lane rewrites them)
  if (j < D) {
    rms[is_ret ? 2 * d + 1 : j] = mean;
    rms[is_ret ? 2 * d + 2 : d + j] = var;
    if (j == 0) rms[2 * d] = N + c_obs;
    if (is_ret) rms[2 * d + 3] = N + c_ret;
    if (merged) {
      if (j == 0) merged[0] = N;
      merged[1 + j] = mu;
      merged[1 + D + j] = m2;
    }
  }
}

// k_moments_merge + k_rms_update of the single merged record in one launch (the unsharded statistics
// update of a collect step): the same device functions, so the same bits as the two launches.
__global__ __launch_bounds__(MERGE_THREADS) void k_merge_update(const double* __restrict__ part, int parts, int d,
                                                                   int has_ret, double* __restrict__ rms,
                                                                   double* __restrict__ rec_out) {
  __shared__ double rec[1 + 2 * MAXD];
  __shared__ double old_count[2];
  const int D = d + (has_ret ? 1 : 0);
  merge_records(part, parts, D, rec);
  __syncthreads();
  if (rec_out)
    for (int k = threadIdx.x; k < 1 + 2 * D; k += blockDim.x) rec_out[k] = rec[k];
  rms_update(rec, 1, d, has_ret, rms, 1, 1, old_count);  // every thread: it holds a barrier
}

__global__ __launch_bounds__(BLOCK) void k_vecnorm_apply(const float* __restrict__ obs, int64_t n, int d, int64_t ldx,
                                                         const double* __restrict__ rms, double eps, int norm_obs,
                                                         double clip_obs, float* __restrict__ obs_out, int64_t ld_out,
                                                         const float* __restrict__ rew, int norm_rew, double clip_rew,
                                                         float* __restrict__ rew_out, const uint8_t* __restrict__ done,
                                                         double* __restrict__ retv) {
  __shared__ double sden[MAXD];  // np.sqrt(var + eps) per column, once per block
  if (norm_obs && (int)threadIdx.x < d) sden[threadIdx.x] = sqrt(rms[d + threadIdx.x] + eps);
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
  if (i >= n) return;
  if (obs_out) {
    for (int j = 0; j < d; j++) {
      const float o = obs[i * ldx + j];
      if (norm_obs) {  // np.clip((obs - mean) / np.sqrt(var + eps), -clip, clip).astype(float32)
        double y = ((double)o - rms[j]) / sden[j];
        y = fmin(fmax(y, -clip_obs), clip_obs);
        obs_out[i * ld_out + j] = (float)y;
      } else {
        obs_out[i * ld_out + j] = o;
      }
    }
  }
  if (rew_out) {
    double r = (double)rew[i];
    if (norm_rew) r = fmin(fmax(r / sqrt(rms[2 * d + 2] + eps), -clip_rew), clip_rew);
    rew_out[i] = (float)r;
  }
  if (done && retv && done[i]) retv[i] = 0.0;  // self.ret[news] = 0
}

// ---------------------------------------------------------------------------
// ReplayBuffer.add: several independent device copies in one launch.  Each segment is
// split into 16-byte vectors (when aligned) or dwords; the grid strides over the sum.
// ---------------------------------------------------------------------------
struct CopySegs {
  const uint8_t* src[FW_MAX_COPY_SEGS];
  uint8_t* dst[FW_MAX_COPY_SEGS];
  int64_t units[FW_MAX_COPY_SEGS];   // number of 16-B (vec) or 4-B units
  int64_t start[FW_MAX_COPY_SEGS + 1];
  int vec[FW_MAX_COPY_SEGS];
  int n;
};

__global__ __launch_bounds__(BLOCK) void k_copy_segs(CopySegs cs) {
  const int64_t total = cs.start[cs.n];
  for (int64_t u = (int64_t)blockIdx.x * BLOCK + threadIdx.x; u < total; u += (int64_t)gridDim.x * BLOCK) {
    int k = 0;
#pragma unroll
    for (int j = 1; j < FW_MAX_COPY_SEGS; j++) k += (j < cs.n && u >= cs.start[j]) ? 1 : 0;
    const int64_t off = u - cs.start[k];
    if (cs.vec[k]) {
      reinterpret_cast<uint4*>(cs.dst[k])[off] = reinterpret_cast<const uint4*>(cs.src[k])[off];
    } else {
      reinterpret_cast<uint32_t*>(cs.dst[k])[off] = reinterpret_cast<const uint32_t*>(cs.src[k])[off];
    }
  }
}

// RolloutBuffer.add with the row read on the device (fw_rollout_store): the same copy as k_copy_segs,
// destinations offset by (ctrl[0] + row_off) * stride, segments outside [0, ctrl[1]) skipped.
struct RowSegs {
  const uint8_t* src[FW_MAX_COPY_SEGS];
  uint8_t* dst[FW_MAX_COPY_SEGS];
  int64_t stride[FW_MAX_COPY_SEGS];
  int64_t start[FW_MAX_COPY_SEGS + 1];  // 4-byte units
  int row_off[FW_MAX_COPY_SEGS];
  int n;
};

__global__ __launch_bounds__(BLOCK) void k_store_rows(RowSegs rs, const int32_t* __restrict__ ctrl) {
  const int row = ctrl[0], n_rows = ctrl[1];
  const int64_t total = rs.start[rs.n];
  for (int64_t u = (int64_t)blockIdx.x * BLOCK + threadIdx.x; u < total; u += (int64_t)gridDim.x * BLOCK) {
    int k = 0;
#pragma unroll
    for (int j = 1; j < FW_MAX_COPY_SEGS; j++) k += (j < rs.n && u >= rs.start[j]) ? 1 : 0;
    const int r = row + rs.row_off[k];
    if (r < 0 || r >= n_rows) continue;
    const int64_t off = u - rs.start[k];
    reinterpret_cast<uint32_t*>(rs.dst[k] + (int64_t)r * rs.stride[k])[off] = reinterpret_cast<const uint32_t*>(rs.src[k])[off];
  }
}

__global__ void k_row_advance(int32_t* ctrl) { ctrl[0] += 1; }


// ---------------------------------------------------------------------------
// The default PPO MlpPolicy forward of one collect step (SB3 ActorCriticPolicy.forward,
// stable_baselines3/common/policies.py:539-553; DiagGaussianDistribution, distributions.py:143-171):
//   latent_pi = tanh(W1 tanh(W0 x + b0) + b1), mean = Wa latent_pi + ba        (actor MLP)
//   latent_vf = tanh(V1 tanh(V0 x + c0) + c1), value = Wv latent_vf + bv       (critic MLP)
//   action = mean + exp(log_std) * noise, log_prob = sum_a N(action | mean, std), clipped = clip(action)
// (on_policy_algorithm.py:152-161).  Two lanes per env: the even lane runs the actor MLP, the odd lane
// the critic, both from one LDS image of the nets per block (the critic's 32 banks after the actor's,
// so a pair's reads do not collide); hidden units stay in VGPRs.  The grid is persistent (at most
// POL_BLOCKS_PER_CU blocks per CU): a block stages the weights once and walks env tiles of 128.
// MACs are FMAs in input order; tanh = 1 - 2 / (exp(2x) + 1) on the hardware exp / rcp: results equal the
// torch module to ~1e-6, not bit for bit.  Measured alternatives (65536 envs, us per launch,
// profiles/r03_collect_kernels.csv): this layout 39 (non-persistent); weights through SGPRs 51; one net per
// wave with packed input pairs 94; two envs per lane 100 (register-bound).
// ---------------------------------------------------------------------------
constexpr int POL_MAXD = 32, POL_MAXH = 64, POL_MAXA = 8;
// fields x records of a deferred final merge a k_policy_mfma block stages in LDS (fw_collect_io.pend)
constexpr int PEND_MAX = 2048;
constexpr int POL_BLOCK = 256;  // 128 envs per tile
constexpr int POL_BLOCKS_PER_CU = 2;
#ifndef FW_POL_ROWPF
#define FW_POL_ROWPF 0  // 1: hidden-layer rows and heads read whole, four partial sums per unit (A/B: 38.0 vs
                        // 38.7 us, within noise, profiles/r03_collect_kernels.csv)
#endif

__host__ __device__ inline int pol_net_floats(int d, int H, int out) { return H * d + H + H * H + H + out * H + out; }
__host__ __device__ inline int pol_vf_offset(int d, int H, int A) { return ((pol_net_floats(d, H, A) + 63) / 64) * 64 + 32; }

__device__ __forceinline__ float ftanh(float x) {
  const float e = __builtin_amdgcn_exp2f(x * 2.8853900817779268f);  // exp(2x)
  return 1.0f - 2.0f * __builtin_amdgcn_rcpf(e + 1.0f);
}
// the same of x2 = 2 log2(e) x (the scale folded into the producing layer)
__device__ __forceinline__ float ftanh2(float x2) {
  return fmaf(-2.0f, __builtin_amdgcn_rcpf(__builtin_amdgcn_exp2f(x2) + 1.0f), 1.0f);
}

template <int H>
__global__ __launch_bounds__(POL_BLOCK) void k_policy_forward(fw_mlp_policy P, const float* __restrict__ obs, int64_t n,
                                                               const float* __restrict__ noise,
                                                               const float* __restrict__ low, const float* __restrict__ high,
                                                               float* __restrict__ act_out, float* __restrict__ clip_out,
                                                               float* __restrict__ val_out, float* __restrict__ logp_out) {
  extern __shared__ float W[];  // actor image, critic image: W0^T [d][H] | b0 | W1 [H][H] | b1 | head [out][H] | head b
  const int d = P.d, A = P.act_dim;
  const int off_vf = pol_vf_offset(d, H, A);
  {
    const float* src[2][6] = {{P.pi_w0, P.pi_b0, P.pi_w1, P.pi_b1, P.act_w, P.act_b},
                              {P.vf_w0, P.vf_b0, P.vf_w1, P.vf_b1, P.val_w, P.val_b}};
    for (int net = 0; net < 2; net++) {
      float* img = W + (net ? off_vf : 0);
      const int out = net ? 1 : A;
      for (int i = threadIdx.x; i < H * d; i += POL_BLOCK) {  // nn.Linear [H][d] -> [d][H]
        const int r = i / d, c = i - r * d;
        img[c * H + r] = src[net][0][i];
      }
      img += d * H;
      const int len[5] = {H, H * H, H, out * H, out};
      for (int k = 0; k < 5; k++) {
        for (int i = threadIdx.x; i < len[k]; i += POL_BLOCK) img[i] = src[net][k + 1][i];
        img += len[k];
      }
    }
  }
  __syncthreads();
  const bool critic = threadIdx.x & 1;
  const float* w0 = W + (critic ? off_vf : 0);
  const float* b0 = w0 + H * d;
  const float* w1 = b0 + H;
  const float* b1 = w1 + H * H;
  const float* wh = b1 + H;
  const float* bh = wh + (critic ? 1 : A) * H;
  const float half_log_2pi = 0.91893853320467274f;  // 0.5 * log(2 pi)
  if (noise && P.noise_row) noise += (int64_t)P.noise_row[0] * n * A;  // this step's row of the collection's draws
  for (int64_t tile = blockIdx.x; tile * (POL_BLOCK / 2) < n; tile += gridDim.x) {
    const int64_t env = tile * (POL_BLOCK / 2) + (threadIdx.x >> 1);
    if (env >= n) break;
    float h0[H], h1[H];
#pragma unroll
    for (int i = 0; i < H; i++) h0[i] = 0.0f;
    for (int k = 0; k < d; k++) {  // every unit sums its inputs in order k = 0 .. d-1
      const float xk = obs[env * d + k];
      const float4* col = reinterpret_cast<const float4*>(w0 + k * H);
#pragma unroll
      for (int j = 0; j < H / 4; j++) {
        const float4 q = col[j];
        h0[4 * j] = fmaf(q.x, xk, h0[4 * j]);
        h0[4 * j + 1] = fmaf(q.y, xk, h0[4 * j + 1]);
        h0[4 * j + 2] = fmaf(q.z, xk, h0[4 * j + 2]);
        h0[4 * j + 3] = fmaf(q.w, xk, h0[4 * j + 3]);
      }
    }
#pragma unroll
    for (int i = 0; i < H; i++) h0[i] = ftanh(h0[i] + b0[i]);
#if FW_POL_ROWPF
#pragma unroll
    for (int i = 0; i < H; i++) {
      // the whole row in flight, then four independent partial sums (inputs k mod 4, combined as
      // (s0 + s1) + (s2 + s3)): one dependent chain per unit left each LDS read's latency exposed
      __builtin_amdgcn_sched_barrier(0);
      const float4* r = reinterpret_cast<const float4*>(w1 + i * H);
      float4 rw[H / 4];
#pragma unroll
      for (int k = 0; k < H / 4; k++) rw[k] = r[k];
      float c0 = 0.0f, c1 = 0.0f, c2 = 0.0f, c3 = 0.0f;
#pragma unroll
      for (int k = 0; k < H / 4; k++) {
        c0 = fmaf(rw[k].x, h0[4 * k], c0);
        c1 = fmaf(rw[k].y, h0[4 * k + 1], c1);
        c2 = fmaf(rw[k].z, h0[4 * k + 2], c2);
        c3 = fmaf(rw[k].w, h0[4 * k + 3], c3);
      }
      h1[i] = ftanh(((c0 + c1) + (c2 + c3)) + b1[i]);
    }
    auto head = [&](const float* row) {  // four partial sums, as the hidden layer
      const float4* r4 = reinterpret_cast<const float4*>(row);
      float c0 = 0.0f, c1 = 0.0f, c2 = 0.0f, c3 = 0.0f;
#pragma unroll
      for (int k = 0; k < H / 4; k++) {
        const float4 q = r4[k];
        c0 = fmaf(q.x, h1[4 * k], c0);
        c1 = fmaf(q.y, h1[4 * k + 1], c1);
        c2 = fmaf(q.z, h1[4 * k + 2], c2);
        c3 = fmaf(q.w, h1[4 * k + 3], c3);
      }
      return (c0 + c1) + (c2 + c3);
    };
    if (critic) {
      val_out[env] = head(wh) + bh[0];
      continue;
    }
    float lp = 0.0f;
    for (int a = 0; a < A; a++) {
      const float m = head(wh + a * H) + bh[a];
      const float ls = P.log_std[a];
      const float sd = expf(ls);
      // the module's arithmetic (rollout.py MlpActorCritic.forward): separate mul / add, as torch's kernels
      const float act = noise ? m + sd * noise[env * A + a] : m;
      const float dv = act - m;
      lp = lp + (((-(dv * dv)) / ((2.0f * sd) * sd) - ls) - half_log_2pi);
      act_out[env * A + a] = act;
      if (clip_out) clip_out[env * A + a] = fmaxf(fminf(act, high[a]), low[a]);
    }
#else
#pragma unroll
    for (int i = 0; i < H; i++) {
      const float4* r = reinterpret_cast<const float4*>(w1 + i * H);
      float acc = 0.0f;
#pragma unroll
      for (int k = 0; k < H / 4; k++) {
        const float4 q = r[k];
        acc = fmaf(q.x, h0[4 * k], acc);
        acc = fmaf(q.y, h0[4 * k + 1], acc);
        acc = fmaf(q.z, h0[4 * k + 2], acc);
        acc = fmaf(q.w, h0[4 * k + 3], acc);
      }
      h1[i] = ftanh(acc + b1[i]);
    }
    if (critic) {
      float v = 0.0f;
#pragma unroll
      for (int k = 0; k < H; k++) v = fmaf(wh[k], h1[k], v);
      val_out[env] = v + bh[0];
      continue;
    }
    float lp = 0.0f;
    for (int a = 0; a < A; a++) {
      float m = 0.0f;
#pragma unroll
      for (int k = 0; k < H; k++) m = fmaf(wh[a * H + k], h1[k], m);
      m = m + bh[a];
      const float ls = P.log_std[a];
      const float sd = expf(ls);
      // the module's arithmetic (rollout.py MlpActorCritic.forward): separate mul / add, as torch's kernels
      const float act = noise ? m + sd * noise[env * A + a] : m;
      const float dv = act - m;
      lp = lp + (((-(dv * dv)) / ((2.0f * sd) * sd) - ls) - half_log_2pi);
      act_out[env * A + a] = act;
      if (clip_out) clip_out[env * A + a] = fmaxf(fminf(act, high[a]), low[a]);
    }
#endif
    logp_out[env] = lp;
  }
}

// ---------------------------------------------------------------------------
// The same policy forward on the matrix cores (v_mfma_f32_16x16x4_f32: f32 in, f32 accumulate, exact f32
// products), one wave per tile of 16 envs, every weight resident in registers for the wave's lifetime.
//
// The layers are computed transposed, H^T = W . X^T, so the env index is the MFMA's N (column) dimension
// and a layer's output tile is directly the next layer's B operand: the 16x16 D tile of out-tile O holds, in
// lane l's register v, unit 16 O + 4 (l >> 4) + v of env l & 15 -- and a B operand of the 16x16x4 form takes
// in lane l the k-row l >> 4 of column l & 15.  Reading the K dimension of the next layer in the order
// k-step (T, v) = units {16 T + 4 g + v : g = 0..3} makes D register v of tile T exactly the B operand of
// k-step (T, v), with no lane exchange; the A operands (weights) are loaded in that order once per wave:
//   layer 0   A(O, s)    lane l: W0[16 O + (l & 15)][4 s + (l >> 4)]          (B = obs features 4s..4s+3)
//   layer 1   A(O, T, v) lane l: W1[16 O + (l & 15)][16 T + 4 (l >> 4) + v]    (a float4 per (O, T))
//   heads     rows 0..A-1 = action means (actor latent), row 15 = value (critic latent), one D tile
// Per 16 envs: 2 x (4 S + 64 + 16) MFMAs (S = k-steps of the observation, 4 for d <= 16).  Sums run in
// the k-step order above (not the torch GEMM's): equal to the module within fp32 rounding.
// ---------------------------------------------------------------------------
typedef float f32x4 __attribute__((ext_vector_type(4)));

struct PolArgs {
  fw_mlp_policy P;
  const float* obs;
  const float* reward;
  const uint8_t* done;
  const double* rms;
  double eps, clip_obs, clip_rew;
  int norm_obs, norm_rew;
  const float* noise;
  const int32_t* noise_row;  // device row of `noise` ([T][n][A]) or null
  const float *low, *high;
  float* clipped;
  const int32_t* ctrl;       // collect mode: rows at ctrl[0]; null: row 0 and no reward / start rows
  float *obs_rows, *act, *val, *logp, *rew_rows;
  uint8_t* start_rows;
  int64_t n;
  // the env step's deferred final merge (fw_collect_io.pend, ABI 12), or pend null
  const double* pend;
  int64_t pend_stride;
  int pend_cnt, has_ret;
  double* rms_w;     // = rms, written by block 0
  double* merged;    // [1 + 2D] or null
  const double* rms_prev;  // the statistics before the update (the env step's copy)
};

#ifndef FW_POL_VHEADS
// 1: the 4-action / 8-wave instance computes the heads (<= 4 actor rows + the critic row) on the VALU -- 80
// multiply-adds per lane and a butterfly over the four lane groups -- instead of 32 MFMAs of which 12 of 16
// output rows are padding (A/B: tools/r05_pol.sh)
#define FW_POL_VHEADS 0
#endif
#ifndef FW_POL_WAVES
// waves per block of the k_policy_mfma instance of SB3's default shapes (d <= 16, act_dim <= 4); two blocks per
// CU share the CU's LDS (one weight image each).  8: four resident waves per SIMD at <= 128 VGPRs (one 16-env
// tile per wave at 65536 envs); 4: two per SIMD (the wider instances, whose registers do not fit 128)
#define FW_POL_WAVES 8
#endif
#ifndef FW_POL_STAGGER
#define FW_POL_STAGGER 0  // s_sleep units (64 cycles) the second half of the grid waits (A/B, below)
#endif
#ifndef FW_POL_TILES
#define FW_POL_TILES 1  // 16-env tiles per wave iteration of k_policy_mfma (A/B: tools/r05_pol.sh)
#endif
#ifndef FW_POL_DIAG
// timing diagnostics only (tools/r04_poldiag.sh builds library variants; their results are wrong): 1 = no tanh,
// 2 = no hidden-layer MFMA, 3 = no LDS weight fill, 4 = no row / output stores, 5 = no observation normalisation
#define FW_POL_DIAG 0
#endif

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float norm_obs_val(float o, double mean, double den, double clip) {
  double y = ((double)o - mean) / den;  // np.clip((obs - mean) / np.sqrt(var + eps), -clip, clip) (k_vecnorm_apply)
  y = fmin(fmax(y, -clip), clip);
  return (float)y;
}

// LDS image of the A operands (per block, read by every wave of it): lane l's fragment of a k-step group is
// 16 contiguous bytes, consecutive lanes consecutive (ds_read_b128, conflict-free).  Floats:
//   L1 [net][O][T][lane][v]   K2 W1[16 O + (l & 15)][16 T + 4 (l >> 4) + v]
//   L0 [net][O][lane][s]      K2 W0[16 O + (l & 15)][4 s + (l >> 4)]
//   HD [net][T][lane][v]      actor rows l & 15 < A / critic row 15 of the heads (unscaled)
//   B  [layer][net][O][16]    K2 bias of unit 16 O + 4 g + v (read as lane group g's float4)
//   BH [16]                   head bias of rows 0..15
template <int S>
struct PolLds {
  static constexpr int L1 = 0, L0 = L1 + 2 * 4 * 4 * 64 * 4, HD = L0 + 2 * 4 * 64 * S, B = HD + 2 * 4 * 64 * 4,
                       BH = B + 2 * 2 * 4 * 16, NRM = BH + 16, HV = NRM + 2 * 2 * 4 * S, RV = HV + 4 * 5 * 16,
                       PO = RV + 2, FLOATS = PO + 2 * (2 * POL_MAXD + 4 + 1 + 2 * (POL_MAXD + 1));
  // RV: the return variance (double) and PO: the updated statistics [2d + 4] then the merged record [1 + 2D]
  // (doubles) of the deferred final merge (PolArgs.pend); its records are staged past FLOATS (dynamic LDS)
  static_assert(RV % 2 == 0 && FLOATS % 2 == 0, "RV / PO hold doubles");
  // HV: the heads for the VALU form (FW_POL_VHEADS): [g][row][16] with rows 0..3 = actor rows (0 past act_dim),
  // row 4 = the critic; entry 4 T + v of lane group g = hidden unit 16 T + 4 g + v (the layer-1 B-operand slot)
  // NRM: the VecNormalize mean and sqrt(var + eps) of features 0 .. 4 S - 1 as doubles (8-wave blocks read
  // them from here instead of holding them in VGPRs)
  static_assert(NRM % 2 == 0, "NRM holds doubles");
};

// The image is filled region by region with unrolled, independent loads (a load-then-store loop with a region
// switch in its body issued one global load per iteration and waited for each: ~15 us of a 34-us launch).
template <int S, int PM_WAVES>
__device__ __forceinline__ void pol_fill_lds(const fw_mlp_policy& P, float* W) {
  using L = PolLds<S>;
  constexpr int NT = 64 * PM_WAVES;  // threads of the block; every region below is a multiple of 256 entries
  const int d = P.d, A = P.act_dim, H = POL_MAXH, t0 = threadIdx.x;
  const float K2 = 2.8853900817779268f;  // 2 log2(e): tanh(x) = 1 - 2 / (exp2(K2 x) + 1)
#pragma unroll
  for (int base = 0; base < 256; base += NT) {  // (NT = 256: one pass; NT = 512: the upper half idles)
    const int t = t0 + base;
    if (NT > 256 && t >= 256) break;
    {  // L1: 2048 float4 fragments, 8 per 256-thread stripe; fragment q = ((net * 4 + O) * 4 + T) * 64 + l
      f32x4 v[8];
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const int q = t + 256 * k, l = q & 63, T = (q >> 6) & 3, O = (q >> 8) & 3, net = q >> 10;
        const float* w = net ? P.vf_w1 : P.pi_w1;
        v[k] = *reinterpret_cast<const f32x4*>(w + (16 * O + (l & 15)) * H + 16 * T + 4 * (l >> 4));
      }
#pragma unroll
      for (int k = 0; k < 8; k++) *reinterpret_cast<f32x4*>(W + L::L1 + 4 * (t + 256 * k)) = K2 * v[k];
    }
    {  // L0: 512 S floats, 2 S per stripe; element q = ((net * 4 + O) * 64 + l) * S + s
      float v[2 * S];
#pragma unroll
      for (int k = 0; k < 2 * S; k++) {
        const int q = t + 256 * k, sidx = q % S, l = (q / S) & 63, O = (q / (S * 64)) & 3, net = q / (S * 256);
        const int f = 4 * sidx + (l >> 4);
        const float* w = net ? P.vf_w0 : P.pi_w0;
        v[k] = w[(16 * O + (l & 15)) * d + (f < d ? f : d - 1)];
        v[k] = f < d ? K2 * v[k] : 0.0f;
      }
#pragma unroll
      for (int k = 0; k < 2 * S; k++) W[L::L0 + t + 256 * k] = v[k];
    }
    {  // HD: 512 float4 fragments, 2 per stripe; fragment q = (net * 4 + T) * 64 + l (row r = l & 15)
      f32x4 v[2];
#pragma unroll
      for (int k = 0; k < 2; k++) {
        const int q = t + 256 * k, l = q & 63, T = (q >> 6) & 3, net = q >> 8, r = l & 15;
        const int kk = 16 * T + 4 * (l >> 4);
        const float* src = net ? P.val_w + kk : P.act_w + (r < A ? r : 0) * H + kk;
        v[k] = *reinterpret_cast<const f32x4*>(src);
        if (net ? r != 15 : r >= A) v[k] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
      }
#pragma unroll
      for (int k = 0; k < 2; k++) *reinterpret_cast<f32x4*>(W + L::HD + 4 * (t + 256 * k)) = v[k];
    }
    {  // B: 256 floats, one per stripe entry; q = ((layer * 2 + net) * 4 + O) * 16 + u
      const int u = t & 15, O = (t >> 4) & 3, net = (t >> 6) & 1, layer = t >> 7;
      const float* b = layer ? (net ? P.vf_b1 : P.pi_b1) : (net ? P.vf_b0 : P.pi_b0);
      W[L::B + t] = K2 * b[16 * O + u];
    }
  }
  const int t = t0;
  if (t < 16) W[L::BH + t] = t < A ? P.act_b[t] : (t == 15 ? P.val_b[0] : 0.0f);
  for (int q = t; q < 4 * 5 * 16; q += NT) {  // HV
    const int gq = q / 80, r = (q / 16) % 5, kk = q % 16, u = 16 * (kk >> 2) + 4 * gq + (kk & 3);
    W[L::HV + q] = r < 4 ? (r < A ? P.act_w[r * H + u] : 0.0f) : P.val_w[u];
  }
  __syncthreads();
}

__device__ __forceinline__ f32x4 lds4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }

// S: k-steps of 4 observation features (d <= 4 S); AM: actions held per lane (act_dim <= AM, 4 or POL_MAXA);
// PM_WAVES: waves per block (4 or 8; two blocks per CU)
template <int S, int AM, int PM_WAVES>
__global__ __launch_bounds__(64 * PM_WAVES, PM_WAVES / 2) void k_policy_mfma(PolArgs G) {  // (min waves per SIMD)
  constexpr bool FW_POL_DBUF_ = PM_WAVES <= 4;  // layer-1 fragments double-buffered in VGPRs (32 extra)
  using L = PolLds<S>;
  extern __shared__ float Wl[];
  const int lane = threadIdx.x & 63;
  const int c16 = lane & 15, g = lane >> 4;
  const int d = G.P.d, A = G.P.act_dim;
  const int64_t n = G.n;
  // ---- the block's A-operand image in LDS (filled below; two blocks per CU, two waves per SIMD: one wave's MFMAs overlap
  // the other's tanh / loads; with the weights in registers a wave took 430 VGPRs and ran alone on its SIMD)
  const float* W0 = Wl + L::L0 + lane * S;
  const float* W1 = Wl + L::L1 + lane * 4;
  const float* WH = Wl + L::HD + lane * 4;
  const float* WB = Wl + L::B + 4 * g;
  // ---- this launch's rows and the VecNormalize statistics of this lane's features
  const int64_t row = G.ctrl ? (int64_t)G.ctrl[0] : 0;
  const float* noise = G.noise;
  if (noise) noise += (G.ctrl ? row : (G.noise_row ? (int64_t)G.noise_row[0] : 0)) * n * A;
  const bool nobs = G.rms && G.norm_obs;
  // The prologue's loads are issued together from clamped, valid addresses under wave-uniform conditions, then
  // selected: a load per feature / action under its own lane condition compiled to a branch with a wait each,
  // eight dependent round trips before the first tile (fp64 statistics) plus the action constants.
  constexpr bool NRM_LDS = PM_WAVES > 4;  // (register budget of four waves per SIMD)
  double mean[NRM_LDS ? 1 : S], den[NRM_LDS ? 1 : S];
  const bool nrew = G.rms && G.norm_rew;
  double rvar = 0.0;
  if (nobs || nrew) {
    double mr[S], vr[S];
#pragma unroll
    for (int s = 0; s < S; s++) {
      const int f = 4 * s + g, fc = f < d ? f : d - 1;
      mr[s] = G.rms[fc];
      vr[s] = G.rms[d + fc];
    }
    rvar = G.rms[2 * d + 2];
    if constexpr (!NRM_LDS) {
#pragma unroll
      for (int s = 0; s < S; s++) {
        const bool on = nobs && 4 * s + g < d;
        mean[s] = on ? mr[s] : 0.0;
        den[s] = on ? sqrt(vr[s] + G.eps) : 1.0;
      }
    } else if (threadIdx.x < 64 && c16 == 0) {  // lanes 0, 16, 32, 48 of wave 0: features 4 s + g
      double* nl = reinterpret_cast<double*>(Wl + L::NRM);
#pragma unroll
      for (int s = 0; s < S; s++) {
        const bool on = nobs && 4 * s + g < d;
        nl[4 * s + g] = on ? mr[s] : 0.0;
        nl[4 * S + 4 * s + g] = on ? sqrt(vr[s] + G.eps) : 1.0;
      }
    }
  } else {
    if constexpr (!NRM_LDS) {
#pragma unroll
      for (int s = 0; s < S; s++) {
        mean[s] = 0.0;
        den[s] = 1.0;
      }
    }
  }
  // the env step's deferred final merge (fw_collect_epilogue.defer): from row 1 on, the statistics this launch
  // normalises with are the ones the previous env step's records update (stream order: they are complete)
  const bool pend = G.pend != nullptr && G.ctrl != nullptr && row >= 1;
  double* const PD = reinterpret_cast<double*>(Wl + L::FLOATS);
  // staged: the records (field f of record k at PD[f * cnt + k]), then the statistics before the update
  const int pcnt = pend ? (1 + 2 * (d + G.has_ret)) * G.pend_cnt : 0, ptot = pend ? pcnt + 2 * d + 4 : 0;
  auto pend_at = [&](int e) {
    return e < pcnt ? G.pend[(int64_t)(e / G.pend_cnt) * G.pend_stride + e % G.pend_cnt] : G.rms_prev[e - pcnt];
  };
  // 8-wave blocks: the upper half of the block (idle in the weight fill) stages them, two loads in flight per
  // lane, before its (empty) part of the fill; 4-wave blocks: one element per thread in flight under the fill
  constexpr int NT = 64 * PM_WAVES;
  double sv = 0.0;
  if constexpr (NT > 256) {
    if (pend && threadIdx.x >= 256) {
      for (int e = (int)threadIdx.x - 256; e < ptot; e += 512) {
        const double a = pend_at(e), b = e + 256 < ptot ? pend_at(e + 256) : 0.0;
        PD[e] = a;
        if (e + 256 < ptot) PD[e + 256] = b;
      }
    }
  } else {
    if (pend) sv = pend_at((int)threadIdx.x < ptot ? (int)threadIdx.x : 0);  // (in flight under the weight fill)
  }
  float* obs_rows = G.obs_rows ? G.obs_rows + row * n * d : nullptr;
  float* act = G.act + row * n * A;
  float* val = G.val + row * n;
  float* logp = G.logp + row * n;
  const float half_log_2pi = 0.91893853320467274f;
  // per-action constants, loaded once (uniform: scalar registers), not per tile inside the lane-divergent
  // action stage (where each load waited for every outstanding load, the next tile's prefetch included)
  float lsA[AM], sdA[AM], hiA[AM], loA[AM];
  {
    float l_[AM], h_[AM], o_[AM];
#pragma unroll
    for (int a = 0; a < AM; a++) l_[a] = G.P.log_std[a < A ? a : A - 1];
    if (G.clipped) {
#pragma unroll
      for (int a = 0; a < AM; a++) {
        h_[a] = G.high[a < A ? a : A - 1];
        o_[a] = G.low[a < A ? a : A - 1];
      }
    } else {
#pragma unroll
      for (int a = 0; a < AM; a++) h_[a] = o_[a] = 0.0f;
    }
#pragma unroll
    for (int a = 0; a < AM; a++) {
      lsA[a] = a < A ? l_[a] : 0.0f;
      sdA[a] = expf(lsA[a]);
      hiA[a] = a < A ? h_[a] : 0.0f;
      loA[a] = a < A ? o_[a] : 0.0f;
    }
  }

  const int64_t tiles = (n + 15) / 16;
  const int64_t wid = (int64_t)blockIdx.x * PM_WAVES + (threadIdx.x >> 6), nw = (int64_t)gridDim.x * PM_WAVES;
  // A tile's inputs are loaded one iteration ahead (their HBM latency hides under the previous iteration's
  // MFMAs): the raw observation features of this lane, and -- for the row stores -- the previous step's reward
  // and done flag (lanes g == 1) and this step's noise draws (lanes g == 0).  Restrict-qualified locals: the
  // output stores cannot alias the inputs, so the loads are not serialised behind them.
  const float* __restrict__ obs_in = G.obs;
  const float* __restrict__ rew_in = G.reward;
  const uint8_t* __restrict__ done_in = G.done;
  const float* __restrict__ noise_in = noise;
  const bool rows_prev = G.ctrl && row >= 1;
  struct In {
    float o[S];
    float r;
    uint32_t dn;
    float z[AM];
  };
  // branch-free, and not selected on load: every lane loads from a clamped, valid address straight into the
  // register it is consumed from one iteration later; the validity masks apply at the use (a select right after
  // the load, or a load inside an exec-masked block, makes the compiler wait for it there)
  auto fetch = [&](int64_t t, In& in) {
    const int64_t e = t * 16 + c16;
    const int64_t ec = (t < tiles && e < n) ? e : 0;
#pragma unroll
    for (int s = 0; s < S; s++) {
      const int f = 4 * s + g;
      in.o[s] = obs_in[ec * d + (f < d ? f : d - 1)];
    }
    if (rows_prev) {
      in.r = rew_in[ec];
      in.dn = done_in[ec];
    }
#pragma unroll
    for (int a = 0; a < AM; a++)
      if (noise_in && a < A) in.z[a] = noise_in[ec * A + a];
  };
  // PT tiles per iteration, interleaved stage by stage: each A operand read from LDS serves PT tiles, and one
  // tile's tanh overlaps the other's MFMAs within the wave (the per-tile arithmetic, and so every bit of the
  // outputs, is the same for any PT)
  constexpr int PT = FW_POL_TILES;
  In nxt[PT];
#pragma unroll
  for (int p = 0; p < PT; p++) nxt[p] = In{};
#pragma unroll
  for (int p = 0; p < PT; p++) fetch(wid * PT + p, nxt[p]);
  // the block's weight image after the first tiles' loads are issued (their latency hides under the fill)
  if (FW_POL_DIAG != 3) pol_fill_lds<S, PM_WAVES>(G.P, Wl);
  if (pend) {
    if constexpr (NT <= 256) {
      if ((int)threadIdx.x < ptot) PD[threadIdx.x] = sv;
      for (int e = (int)threadIdx.x + NT; e < ptot; e += NT) PD[e] = pend_at(e);
      __syncthreads();
    }  // (8-wave blocks: staged before the fill's closing barrier)
    double* const po = reinterpret_cast<double*>(Wl + L::PO);
    double* const nl = reinterpret_cast<double*>(Wl + L::NRM);
    double* const rv = reinterpret_cast<double*>(Wl + L::RV);
    if (threadIdx.x < 64) {
      // every block computes the same bits; block 0 writes them back (the other blocks read the env step's copy
      // of the old statistics, so the write cannot race their reads; a ticket on one counter from 512 blocks
      // serialised on its address: +5 us per launch, profiles/r06_collect_ab.log)
      const int j = lane, D = d + G.has_ret, nr = 2 * d + 4, cnt = G.pend_cnt;
      const double* ro = PD + pcnt;  // the statistics before the update
      for (int e = j; e < nr; e += 64) po[e] = ro[e];  // (what the update leaves alone: no return column)
      const double c_obs = ro[2 * d], r_m = ro[2 * d + 1], r_v = ro[2 * d + 2], c_ret = ro[2 * d + 3];
      const double o_m = ro[j < d ? j : 0], o_v = ro[d + (j < d ? j : 0)];
      double rvar_new = r_v;
      if (j < D) {
        double N, mu, m2;
        fw_stats::merge_col(PD, PD + (1 + j) * cnt, PD + (1 + D + j) * cnt, cnt, N, mu, m2);
        const bool is_ret = G.has_ret && j == d;
        double mean = is_ret ? r_m : o_m, var = is_ret ? r_v : o_v;
        fw_stats::update_col(mu, m2 / N, N, is_ret ? c_ret : c_obs, mean, var);
        po[is_ret ? 2 * d + 1 : j] = mean;
        po[is_ret ? 2 * d + 2 : d + j] = var;
        if (j == 0) po[2 * d] = N + c_obs;
        if (is_ret) po[2 * d + 3] = N + c_ret;
        double* mg = po + nr;
        if (j == 0) mg[0] = N;
        mg[1 + j] = mu;
        mg[1 + D + j] = m2;
        if (j < 4 * S) {
          const bool on = nobs && j < d;
          nl[j] = on ? mean : 0.0;
          nl[4 * S + j] = on ? sqrt(var + G.eps) : 1.0;
        }
        if (is_ret) rvar_new = var;
      } else if (j < 4 * S) {
        nl[j] = 0.0;
        nl[4 * S + j] = 1.0;
      }
      if (j == (G.has_ret ? d : 0)) rv[0] = rvar_new;
      if (blockIdx.x == 0) {
        asm volatile("" ::: "memory");  // (po's stores above are this wave's own: LDS completes them in order)
        const int nm = 1 + 2 * D;
        for (int e = lane; e < nr; e += 64) G.rms_w[e] = po[e];
        if (G.merged)
          for (int e = lane; e < nm; e += 64) G.merged[e] = po[nr + e];
      }
    }
    __syncthreads();
    if constexpr (!NRM_LDS) {
#pragma unroll
      for (int s = 0; s < S; s++) {
        mean[s] = nl[4 * s + g];
        den[s] = nl[4 * S + 4 * s + g];
      }
    }
    rvar = rv[0];
  }
  const double rden = nrew ? sqrt(rvar + G.eps) : 1.0;
#if FW_POL_STAGGER
  // A/B (tools/r05_pol.sh): the CU's second block starts FW_POL_STAGGER x 64 cycles late, so its waves' tanh
  // phases meet their SIMD partners' MFMA phases instead of running in lockstep with them
  if (blockIdx.x >= gridDim.x / 2)
#pragma unroll
    for (int k = 0; k < FW_POL_STAGGER / 32; k++) __builtin_amdgcn_s_sleep(32);
#endif
  for (int64_t base = wid * PT; base < tiles; base += nw * PT) {
    In cur[PT];
#pragma unroll
    for (int p = 0; p < PT; p++) {
      cur[p] = nxt[p];
      fetch(base + nw * PT + p, nxt[p]);
    }
    int64_t env[PT];
    bool valid[PT];
    // ---- observation (normalised) = B operands of layer 0; the rollout's observation row
    float x[PT][S];
#pragma unroll
    for (int p = 0; p < PT; p++) {
      env[p] = (base + p) * 16 + c16;
      valid[p] = base + p < tiles && env[p] < n;
#pragma unroll
      for (int s = 0; s < S; s++) {
        const int f = 4 * s + g;
        float o = (valid[p] && f < d) ? cur[p].o[s] : 0.0f;
        if (FW_POL_DIAG != 5 && nobs && valid[p] && f < d) {
          if constexpr (NRM_LDS) {
            const double* nl = reinterpret_cast<const double*>(Wl + L::NRM);
            o = norm_obs_val(o, nl[f], nl[4 * S + f], G.clip_obs);
          } else {
            o = norm_obs_val(o, mean[s], den[s], G.clip_obs);
          }
        }
        x[p][s] = o;
        if (FW_POL_DIAG != 4 && obs_rows && valid[p] && f < d) obs_rows[env[p] * d + f] = o;
      }
      // ---- the previous step's reward row (normalised) and the episode starts of this row
      if (rows_prev && g == 1 && valid[p]) {
        double r = (double)cur[p].r;
        if (G.rms && G.norm_rew) r = fmin(fmax(r / rden, -G.clip_rew), G.clip_rew);
        if (FW_POL_DIAG != 4) G.rew_rows[(row - 1) * n + env[p]] = (float)r;
        G.start_rows[row * n + env[p]] = (uint8_t)cur[p].dn;
      }
    }
    asm volatile("" ::: "memory");  // the A operands are re-read from LDS every iteration (not hoisted into VGPRs)
    // ---- layer 0 (8 independent accumulators per tile, starting at the scaled bias)
    f32x4 cp[PT][4], cv[PT][4];
#pragma unroll
    for (int O = 0; O < 4; O++) {
      const f32x4 bp = lds4(WB + (0 * 4 + O) * 16), bv = lds4(WB + (1 * 4 + O) * 16);
#pragma unroll
      for (int p = 0; p < PT; p++) {
        cp[p][O] = bp;
        cv[p][O] = bv;
      }
    }
    // every fragment of a k-group first, then the MFMAs round-robin over the eight accumulators (a dependent
    // MFMA every 8 issues, past its 40-cycle latency; the per-accumulator order -- s4, then k -- is unchanged)
#pragma unroll
    for (int s4 = 0; s4 < S; s4 += 4) {
      f32x4 ap[4], av[4];
#pragma unroll
      for (int O = 0; O < 4; O++) {
        ap[O] = lds4(W0 + (0 * 4 + O) * 64 * S + s4);
        av[O] = lds4(W0 + (1 * 4 + O) * 64 * S + s4);
      }
#pragma unroll
      for (int k = 0; k < 4; k++)
#pragma unroll
        for (int O = 0; O < 4; O++)
#pragma unroll
          for (int p = 0; p < PT; p++) {
            cp[p][O] = mfma4(ap[O][k], x[p][s4 + k], cp[p][O]);
            cv[p][O] = mfma4(av[O][k], x[p][s4 + k], cv[p][O]);
          }
    }
    f32x4 hpv[PT][4], hvv[PT][4];  // tanh(layer 0): the B operands of layer 1, k-step (T, v) = register v of tile T
#pragma unroll
    for (int p = 0; p < PT; p++)
#pragma unroll
      for (int T = 0; T < 4; T++)
#pragma unroll
        for (int v = 0; v < 4; v++) {
          hpv[p][T][v] = FW_POL_DIAG == 1 ? cp[p][T][v] : ftanh2(cp[p][T][v]);
          hvv[p][T][v] = FW_POL_DIAG == 1 ? cv[p][T][v] : ftanh2(cv[p][T][v]);
        }
    // ---- layer 1
#pragma unroll
    for (int O = 0; O < 4; O++) {
      const f32x4 bp = lds4(WB + (2 * 4 + O) * 16), bv = lds4(WB + (3 * 4 + O) * 16);
#pragma unroll
      for (int p = 0; p < PT; p++) {
        cp[p][O] = bp;
        cv[p][O] = bv;
      }
    }
    // the k-step group T + 1's eight fragments are read while group T's MFMAs issue (FW_POL_DBUF: registers,
    // double buffered); MFMAs round-robin over the eight accumulators; per accumulator the order (T, then v)
    // is unchanged
    if constexpr (PM_WAVES <= 4) {
    {
      constexpr int NB = FW_POL_DBUF_ ? 2 : 1;
      f32x4 ap[NB][4], av[NB][4];
      if constexpr (NB == 2) {
#pragma unroll
        for (int O = 0; O < 4; O++) {
          ap[0][O] = lds4(W1 + ((0 * 4 + O) * 4 + 0) * 256);
          av[0][O] = lds4(W1 + ((1 * 4 + O) * 4 + 0) * 256);
        }
      }
#pragma unroll
      for (int T = 0; T < 4; T++) {
        const int cb = NB == 2 ? (T & 1) : 0, nb = NB == 2 ? (cb ^ 1) : 0;
        if (NB == 1) {
#pragma unroll
          for (int O = 0; O < 4; O++) {
            ap[0][O] = lds4(W1 + ((0 * 4 + O) * 4 + T) * 256);
            av[0][O] = lds4(W1 + ((1 * 4 + O) * 4 + T) * 256);
          }
        } else if (T < 3) {
#pragma unroll
          for (int O = 0; O < 4; O++) {
            ap[nb][O] = lds4(W1 + ((0 * 4 + O) * 4 + T + 1) * 256);
            av[nb][O] = lds4(W1 + ((1 * 4 + O) * 4 + T + 1) * 256);
          }
        }
        if (FW_POL_DIAG == 2) {
#pragma unroll
          for (int O = 0; O < 4; O++)
#pragma unroll
            for (int p = 0; p < PT; p++) {
              cp[p][O] += hpv[p][T];
              cv[p][O] += hvv[p][T];
            }
          continue;
        }
#pragma unroll
        for (int v = 0; v < 4; v++)
#pragma unroll
          for (int O = 0; O < 4; O++)
#pragma unroll
            for (int p = 0; p < PT; p++) {
              cp[p][O] = mfma4(ap[cb][O][v], hpv[p][T][v], cp[p][O]);
              cv[p][O] = mfma4(av[cb][O][v], hvv[p][T][v], cv[p][O]);
            }
      }
    }
    } else {  // (8-wave blocks: two fragments at a time, the round-4 order; the same per-accumulator order)
#pragma unroll
      for (int T = 0; T < 4; T++)
#pragma unroll
        for (int O = 0; O < 4; O++) {
          const f32x4 ap = lds4(W1 + ((0 * 4 + O) * 4 + T) * 256), av = lds4(W1 + ((1 * 4 + O) * 4 + T) * 256);
#pragma unroll
          for (int v = 0; v < 4; v++)
#pragma unroll
            for (int p = 0; p < PT; p++) {
              cp[p][O] = mfma4(ap[v], hpv[p][T][v], cp[p][O]);
              cv[p][O] = mfma4(av[v], hvv[p][T][v], cv[p][O]);
            }
        }
    }
#pragma unroll
    for (int p = 0; p < PT; p++)
#pragma unroll
      for (int T = 0; T < 4; T++)
#pragma unroll
        for (int v = 0; v < 4; v++) {
          hpv[p][T][v] = FW_POL_DIAG == 1 ? cp[p][T][v] : ftanh2(cp[p][T][v]);
          hvv[p][T][v] = FW_POL_DIAG == 1 ? cv[p][T][v] : ftanh2(cv[p][T][v]);
        }
    constexpr bool VH = FW_POL_VHEADS && AM <= 4 && PM_WAVES > 4;
    // ---- heads: actor rows 0..A-1 and the value row 15 of one tile (two accumulators, disjoint rows)
    f32x4 ha[PT], hc[PT];
#pragma unroll
    for (int p = 0; p < PT; p++) {
      ha[p] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
      hc[p] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    }
    if constexpr (VH) {
      // VALU form: lane group g's partial dot products over its 16 hidden units (order T, v), then the sum over
      // the four groups as a butterfly (the same bits on every lane)
      const float* hvw = Wl + L::HV + g * 80;
#pragma unroll
      for (int r = 0; r < 5; r++) {
        const f32x4 w0 = lds4(hvw + 16 * r), w1 = lds4(hvw + 16 * r + 4), w2 = lds4(hvw + 16 * r + 8),
                    w3 = lds4(hvw + 16 * r + 12);
        const f32x4 wr[4] = {w0, w1, w2, w3};
#pragma unroll
        for (int p = 0; p < PT; p++) {
          float acc = 0.0f;
#pragma unroll
          for (int T = 0; T < 4; T++)
#pragma unroll
            for (int v = 0; v < 4; v++) acc = fmaf(wr[T][v], r < 4 ? hpv[p][T][v] : hvv[p][T][v], acc);
          acc += __shfl_xor(acc, 16);
          acc += __shfl_xor(acc, 32);
          // the MFMA form's C layout: lane group 0 holds actor rows 0..3, group 3 row 15 (the critic)
          if (r < 4) ha[p][r] = g == 0 ? acc : 0.0f;
          else hc[p][3] = g == 3 ? acc : 0.0f;
        }
      }
    } else {
#pragma unroll
      for (int T = 0; T < 4; T++) {
        const f32x4 ap = lds4(WH + (0 * 4 + T) * 256), av = lds4(WH + (1 * 4 + T) * 256);
#pragma unroll
        for (int v = 0; v < 4; v++)
#pragma unroll
          for (int p = 0; p < PT; p++) {
            ha[p] = mfma4(ap[v], hpv[p][T][v], ha[p]);
            hc[p] = mfma4(av[v], hvv[p][T][v], hc[p]);
          }
      }
    }
    const f32x4 bh = lds4(Wl + L::BH + 4 * g);
#pragma unroll
    for (int p = 0; p < PT; p++) {
      f32x4 out;
#pragma unroll
      for (int v = 0; v < 4; v++) out[v] = (ha[p][v] + hc[p][v]) + bh[v];  // one of ha / hc is 0 in each row
      // rows 4..7 (A > 4) from the lanes 16 up
      f32x4 hi = out;
      if constexpr (AM > 4)
#pragma unroll
        for (int v = 0; v < 4; v++) hi[v] = __shfl(out[v], (lane + 16) & 63);
      if (FW_POL_DIAG != 4 && g == 3 && valid[p]) val[env[p]] = out[3];
      if (g == 0 && valid[p]) {
        float lp = 0.0f;
#pragma unroll
        for (int a = 0; a < AM; a++) {
          if (a < A) {
            const float m = a < 4 ? out[a & 3] : hi[a & 3];
            const float ls = lsA[a];
            const float sd = sdA[a];
            // the module's arithmetic (rollout.py MlpActorCritic.forward): separate mul / add, as torch's kernels
            const float ac = noise ? m + sd * cur[p].z[a] : m;
            const float dv = ac - m;
            lp = lp + (((-(dv * dv)) / ((2.0f * sd) * sd) - ls) - half_log_2pi);
            if (FW_POL_DIAG != 4) act[env[p] * A + a] = ac;
            if (FW_POL_DIAG != 4 && G.clipped) G.clipped[env[p] * A + a] = fmaxf(fminf(ac, hiA[a]), loA[a]);
          }
        }
        if (FW_POL_DIAG != 4) logp[env[p]] = lp;
      }
    }
  }
}

unsigned grid_for(int64_t n) { return (unsigned)((n + BLOCK - 1) / BLOCK); }

int64_t moments_parts(int64_t n) { return std::max<int64_t>(1, (n + MROWS - 1) / MROWS); }

int cu_count(int* out) {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    FW_HIP(hipGetDevice(&dev));
    FW_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  }
  *out = cus;
  return FW_OK;
}

// the matrix-core kernel reads the hidden / head weights and the biases as 16-byte vectors; the VALU
// kernel (k_policy_forward) stays for unaligned parameters and as the A/B reference (FW_POL_VALU=1)
bool use_mfma(const fw_mlp_policy* p) {
  static const bool valu = std::getenv("FW_POL_VALU") != nullptr;
  if (valu) return false;
  const void* v16[] = {p->pi_w1, p->vf_w1, p->act_w, p->val_w, p->pi_b0, p->vf_b0, p->pi_b1, p->vf_b1};
  for (const void* q : v16)
    if ((uintptr_t)q % 16) return false;
  return true;
}

int launch_mfma(const PolArgs& G, hipStream_t s) {
  int cus = 0;
  if (int rc = cu_count(&cus)) return rc;
  const int64_t tiles = (G.n + 15) / 16;
  static const int per_cu = std::getenv("FW_POL_BLOCKS_PER_CU") ? std::atoi(std::getenv("FW_POL_BLOCKS_PER_CU")) : 2;
  const bool small = G.P.d <= 16 && G.P.act_dim <= 4;  // SB3's default shapes for this env
  const int waves = small ? FW_POL_WAVES : 4;
  const int64_t groups = (tiles + FW_POL_TILES - 1) / FW_POL_TILES;
  const unsigned grid = (unsigned)std::max<int64_t>(
      1, std::min<int64_t>((groups + waves - 1) / waves, (int64_t)cus * std::max(per_cu, 1)));
  // (+ the deferred merge's records and the statistics before the update, staged per block)
  const size_t pst =
      G.pend ? ((size_t)(1 + 2 * (G.P.d + G.has_ret)) * G.pend_cnt + 2 * G.P.d + 4) * sizeof(double) : 0;
  if (small)
    hipLaunchKernelGGL((k_policy_mfma<4, 4, FW_POL_WAVES>), dim3(grid), dim3(64 * FW_POL_WAVES),
                       PolLds<4>::FLOATS * sizeof(float) + pst, s, G);
  else if (G.P.d <= 16)
    hipLaunchKernelGGL((k_policy_mfma<4, POL_MAXA, 4>), dim3(grid), dim3(256), PolLds<4>::FLOATS * sizeof(float) + pst, s, G);
  else
    hipLaunchKernelGGL((k_policy_mfma<8, POL_MAXA, 4>), dim3(grid), dim3(256), PolLds<8>::FLOATS * sizeof(float) + pst, s, G);
  FW_HIP(hipGetLastError());
  return FW_OK;
}

// A/B switch (tools/merge_bench.py): FW_MERGE256=1 runs the 256-thread general merge for every D
bool merge256() {
  static const bool v = std::getenv("FW_MERGE256") != nullptr;
  return v;
}

int check_policy(const fw_mlp_policy* p, const char* who) {
  if (p->d < 1 || p->d > POL_MAXD || p->hidden != POL_MAXH || p->act_dim < 1 || p->act_dim > POL_MAXA)
    return fw::set_error(FW_E_INVALID, std::string(who) + ": d 1..32, hidden 64 (SB3's default net_arch), act_dim 1..8");
  const void* ptrs[13] = {p->pi_w0, p->pi_b0, p->pi_w1, p->pi_b1, p->act_w, p->act_b, p->vf_w0,
                          p->vf_b0, p->vf_w1, p->vf_b1, p->val_w, p->val_b, p->log_std};
  for (const void* q : ptrs)
    if (!q) return fw::set_error(FW_E_INVALID, std::string(who) + ": NULL parameter");
  return FW_OK;
}

}  // namespace

extern "C" {

int fw_gae(const float* rewards, const float* values, const uint8_t* episode_starts, const float* last_values,
           const uint8_t* last_dones, int64_t n_steps, int64_t n_envs, double gamma, double gae_lambda,
           float* advantages, float* returns, void* stream) {
  if (!rewards || !values || !episode_starts || !last_values || !last_dones || !advantages || !returns)
    return fw::set_error(FW_E_INVALID, "fw_gae: NULL buffer");
  if (n_steps < 1 || n_envs < 1) return fw::set_error(FW_E_INVALID, "fw_gae: n_steps and n_envs must be >= 1");
  const double gl = gamma * gae_lambda;  // Python float product (float64)
  hipLaunchKernelGGL(k_gae, dim3(grid_for(n_envs)), dim3(BLOCK), 0, (hipStream_t)stream, rewards, values,
                     episode_starts, last_values, last_dones, n_steps, n_envs, (float)gamma, gl, (float)gl, advantages,
                     returns);
  FW_HIP(hipGetLastError());
  return FW_OK;
}

size_t fw_moments_workspace_bytes(int64_t n, int32_t d) {
  return (size_t)moments_parts(n) * (size_t)(1 + 2 * (d + 1)) * sizeof(double);
}

int fw_moments(const float* x, int64_t n, int32_t d, int64_t ldx, const float* rew, double* ret, double gamma,
               void* workspace, double* out, void* stream) {
  if (n < 1) return fw::set_error(FW_E_INVALID, "fw_moments: n must be >= 1");
  if (d < 0 || d + 1 > MAXD) return fw::set_error(FW_E_INVALID, "fw_moments: d out of range");
  if ((d > 0 && (!x || ldx < d)) || !workspace || !out || (rew && !ret))
    return fw::set_error(FW_E_INVALID, "fw_moments: bad buffer / stride");
  const int64_t parts = moments_parts(n);
  if (parts > INT32_MAX / 2) return fw::set_error(FW_E_INVALID, "fw_moments: n too large");
  const int D = d + (rew ? 1 : 0);
  if (D == 0) return fw::set_error(FW_E_INVALID, "fw_moments: nothing to reduce");
  hipStream_t s = (hipStream_t)stream;
  double* part = (double*)workspace;
  hipLaunchKernelGGL(k_moments_partial, dim3((unsigned)parts), dim3(BLOCK), 0, s, x, n, d, ldx, rew, ret, gamma, part);
  FW_HIP(hipGetLastError());
  hipLaunchKernelGGL(k_moments_merge, dim3(1), dim3(MERGE_THREADS), 0, s, part, (int)parts, D, out);
  FW_HIP(hipGetLastError());
  return FW_OK;
}

int fw_rms_update(const double* parts, int32_t n_parts, int32_t d, int32_t has_ret, double* rms, int32_t update_obs,
                  int32_t update_ret, void* stream) {
  if (!parts || !rms || n_parts < 1) return fw::set_error(FW_E_INVALID, "fw_rms_update: bad arguments");
  if (d < 0 || d + 1 > MAXD) return fw::set_error(FW_E_INVALID, "fw_rms_update: d out of range");
  hipLaunchKernelGGL(k_rms_update, dim3(1), dim3(64), 0, (hipStream_t)stream, parts, n_parts, d, has_ret, rms,
                     update_obs, update_ret);
  FW_HIP(hipGetLastError());
  return FW_OK;
}

int fw_vecnorm_apply(const float* obs, int64_t n, int32_t d, int64_t ldx, const double* rms, double epsilon,
                     int32_t norm_obs, double clip_obs, float* obs_out, int64_t ld_out, const float* rew,
                     int32_t norm_rew, double clip_rew, float* rew_out, const uint8_t* done, double* ret,
                     void* stream) {
  if (n < 1 || d < 0 || d + 1 > MAXD || !rms) return fw::set_error(FW_E_INVALID, "fw_vecnorm_apply: bad arguments");
  if (obs_out && (!obs || ldx < d || ld_out < d)) return fw::set_error(FW_E_INVALID, "fw_vecnorm_apply: bad obs");
  if (rew_out && !rew) return fw::set_error(FW_E_INVALID, "fw_vecnorm_apply: rew_out without rew");
  hipLaunchKernelGGL(k_vecnorm_apply, dim3(grid_for(n)), dim3(BLOCK), 0, (hipStream_t)stream, obs, n, d, ldx, rms,
                     epsilon, norm_obs, clip_obs, obs_out, ld_out, rew, norm_rew, clip_rew, rew_out, done, ret);
  FW_HIP(hipGetLastError());
  return FW_OK;
}

int fw_replay_add(const fw_copy_seg* segs, int32_t n_segs, void* stream) {
  if (!segs || n_segs < 1 || n_segs > FW_MAX_COPY_SEGS)
    return fw::set_error(FW_E_INVALID, "fw_replay_add: 1..FW_MAX_COPY_SEGS segments");
  CopySegs cs{};
  cs.n = n_segs;
  cs.start[0] = 0;
  for (int k = 0; k < n_segs; k++) {
    const fw_copy_seg& g = segs[k];
    if (!g.src || !g.dst || g.bytes < 0 || g.bytes % 4) return fw::set_error(FW_E_INVALID, "fw_replay_add: bad segment");
    const bool v = g.bytes % 16 == 0 && ((uintptr_t)g.src % 16) == 0 && ((uintptr_t)g.dst % 16) == 0;
    cs.src[k] = (const uint8_t*)g.src;
    cs.dst[k] = (uint8_t*)g.dst;
    cs.vec[k] = v;
    cs.units[k] = g.bytes / (v ? 16 : 4);
    cs.start[k + 1] = cs.start[k] + cs.units[k];
  }
  const int64_t total = cs.start[n_segs];
  if (total == 0) return FW_OK;
  const unsigned grid = (unsigned)std::min<int64_t>((total + BLOCK - 1) / BLOCK, 8192);
  hipLaunchKernelGGL(k_copy_segs, dim3(grid), dim3(BLOCK), 0, (hipStream_t)stream, cs);
  FW_HIP(hipGetLastError());
  return FW_OK;
}

int fw_rollout_store(const fw_row_seg* segs, int32_t n_segs, int32_t* ctrl_dev, int32_t advance, void* stream) {
  if (!segs || !ctrl_dev || n_segs < 1 || n_segs > FW_MAX_COPY_SEGS)
    return fw::set_error(FW_E_INVALID, "fw_rollout_store: 1..FW_MAX_COPY_SEGS segments and a ctrl buffer");
  RowSegs rs{};
  rs.n = n_segs;
  rs.start[0] = 0;
  for (int k = 0; k < n_segs; k++) {
    const fw_row_seg& g = segs[k];
    if (!g.src || !g.dst || g.bytes < 0 || g.bytes % 4 || g.stride % 4 || (uintptr_t)g.src % 4 || (uintptr_t)g.dst % 4)
      return fw::set_error(FW_E_INVALID, "fw_rollout_store: bad segment (NULL, or not dword-aligned)");
    rs.src[k] = (const uint8_t*)g.src;
    rs.dst[k] = (uint8_t*)g.dst;
    rs.stride[k] = g.stride;
    rs.row_off[k] = g.row_off;
    rs.start[k + 1] = rs.start[k] + g.bytes / 4;
  }
  hipStream_t s = (hipStream_t)stream;
  const int64_t total = rs.start[n_segs];
  if (total > 0) {
    const unsigned grid = (unsigned)std::min<int64_t>((total + BLOCK - 1) / BLOCK, 8192);
    hipLaunchKernelGGL(k_store_rows, dim3(grid), dim3(BLOCK), 0, s, rs, (const int32_t*)ctrl_dev);
    FW_HIP(hipGetLastError());
  }
  if (advance) {  // a second launch: a last-block increment inside k_store_rows serialises ~5k atomics
                  // on one address (198 vs 7 us per step, profiles/r03_collect_kernels.csv)
    hipLaunchKernelGGL(k_row_advance, dim3(1), dim3(1), 0, s, ctrl_dev);
    FW_HIP(hipGetLastError());
  }
  return FW_OK;
}


int fw_policy_forward(const fw_mlp_policy* p, const float* obs, int64_t n, const float* noise, const float* low,
                      const float* high, float* actions, float* clipped, float* values, float* log_probs, void* stream) {
  if (!p || !obs || !actions || !values || !log_probs || n < 1)
    return fw::set_error(FW_E_INVALID, "fw_policy_forward: NULL buffer or n < 1");
  if (int rc = check_policy(p, "fw_policy_forward")) return rc;
  if (clipped && (!low || !high)) return fw::set_error(FW_E_INVALID, "fw_policy_forward: clipped needs low and high");
  if (use_mfma(p)) {
    PolArgs G{};
    G.P = *p;
    G.obs = obs;
    G.noise = noise;
    G.noise_row = p->noise_row;
    G.low = low;
    G.high = high;
    G.clipped = clipped;
    G.act = actions;
    G.val = values;
    G.logp = log_probs;
    G.n = n;
    return launch_mfma(G, (hipStream_t)stream);
  }
  const int d = p->d, H = p->hidden, A = p->act_dim;
  const size_t lds = (size_t)(pol_vf_offset(d, H, A) + pol_net_floats(d, H, 1)) * sizeof(float);
  int cus = 0;
  if (int rc = cu_count(&cus)) return rc;
  const int64_t tiles = (n + POL_BLOCK / 2 - 1) / (POL_BLOCK / 2);
  const unsigned grid = (unsigned)std::min<int64_t>(tiles, (int64_t)cus * POL_BLOCKS_PER_CU);
  hipLaunchKernelGGL(k_policy_forward<POL_MAXH>, dim3(grid), dim3(POL_BLOCK), lds, (hipStream_t)stream, *p, obs, n, noise,
                     low, high, actions, clipped, values, log_probs);
  FW_HIP(hipGetLastError());
  return FW_OK;
}

int fw_moments_merge(const double* records, int32_t n_records, int32_t D, double* out, void* stream) {
  if (!records || !out || n_records < 1 || D < 1 || D > MAXD)
    return fw::set_error(FW_E_INVALID, "fw_moments_merge: bad arguments");
  if (D <= 15 && n_records <= MERGE16_THREADS * MERGE16_BATCH && !merge256())
    hipLaunchKernelGGL(k_moments_merge16, dim3(1), dim3(MERGE16_THREADS), 0, (hipStream_t)stream, records,
                       (int)n_records, (int)D, out);
  else
    hipLaunchKernelGGL(k_moments_merge, dim3(1), dim3(MERGE_THREADS), 0, (hipStream_t)stream, records,
                       (int)n_records, (int)D, out);
  FW_HIP(hipGetLastError());
  return FW_OK;
}

int fw_vecnorm_merge_update(const double* records, int32_t n_records, int32_t d, int32_t has_ret, double* rms,
                            double* rec_out, void* stream) {
  const int D = d + (has_ret ? 1 : 0);
  if (!records || !rms || n_records < 1 || d < 0 || D < 1 || D > MAXD)
    return fw::set_error(FW_E_INVALID, "fw_vecnorm_merge_update: bad arguments");
  if (D <= 15 && n_records <= MERGE16_THREADS * MERGE16_BATCH && !merge256())
    hipLaunchKernelGGL(k_merge_update16, dim3(1), dim3(MERGE16_THREADS), 0, (hipStream_t)stream, records,
                       (int)n_records, (int)d, (int)(has_ret != 0), rms, rec_out);
  else
    hipLaunchKernelGGL(k_merge_update, dim3(1), dim3(MERGE_THREADS), 0, (hipStream_t)stream, records, (int)n_records,
                       (int)d, (int)(has_ret != 0), rms, rec_out);
  FW_HIP(hipGetLastError());
  return FW_OK;
}

int fw_collect_policy(const fw_mlp_policy* p, const fw_collect_io* io, void* stream) {
  if (!p || !io) return fw::set_error(FW_E_INVALID, "fw_collect_policy: NULL argument");
  if (int rc = check_policy(p, "fw_collect_policy")) return rc;
  if (io->n < 1 || !io->obs || !io->reward || !io->done || !io->low || !io->high || !io->clipped || !io->ctrl ||
      !io->obs_rows || !io->act_rows || !io->val_rows || !io->logp_rows || !io->rew_rows || !io->start_rows)
    return fw::set_error(FW_E_INVALID, "fw_collect_policy: NULL buffer or n < 1");
  if (!use_mfma(p)) return fw::set_error(FW_E_UNSUPPORTED, "fw_collect_policy: parameters must be 16-byte aligned");
  PolArgs G{};
  G.P = *p;
  G.obs = io->obs;
  G.reward = io->reward;
  G.done = io->done;
  G.rms = io->rms;
  G.eps = io->epsilon;
  G.clip_obs = io->clip_obs;
  G.clip_rew = io->clip_reward;
  G.norm_obs = io->norm_obs;
  G.norm_rew = io->norm_reward;
  G.noise = io->noise;
  G.low = io->low;
  G.high = io->high;
  G.clipped = io->clipped;
  G.ctrl = io->ctrl;
  G.obs_rows = io->obs_rows;
  G.act = io->act_rows;
  G.val = io->val_rows;
  G.logp = io->logp_rows;
  G.rew_rows = io->rew_rows;
  G.start_rows = io->start_rows;
  G.n = io->n;
  if (io->pend) {
    const int D = p->d + (io->has_ret ? 1 : 0);
    if (!io->rms || !io->rms_prev || io->pend_cnt < 1 || io->pend_cnt > 64 || io->pend_stride < io->pend_cnt ||
        (1 + 2 * D) * io->pend_cnt > PEND_MAX)
      return fw::set_error(FW_E_INVALID, "fw_collect_policy: pend needs rms, rms_prev and 1..64 records of at most "
                                         "PEND_MAX fields in all");
    G.pend = io->pend;
    G.pend_stride = io->pend_stride;
    G.pend_cnt = io->pend_cnt;
    G.has_ret = io->has_ret ? 1 : 0;
    G.rms_w = const_cast<double*>(io->rms);
    G.merged = io->merged;
    G.rms_prev = io->rms_prev;
  }
  return launch_mfma(G, (hipStream_t)stream);
}

int fw_vecnorm_pending_update(const double* pend, int64_t stride, int32_t cnt, int32_t d, int32_t has_ret,
                              double* rms, double* merged, void* stream) {
  if (!pend || !rms || cnt < 1 || cnt > 64 || stride < cnt || d < 0 || d + (has_ret ? 1 : 0) < 1 ||
      d + (has_ret ? 1 : 0) > 64)
    return fw::set_error(FW_E_INVALID, "fw_vecnorm_pending_update: bad arguments");
  hipLaunchKernelGGL(k_pending_update, dim3(1), dim3(64), 0, (hipStream_t)stream, pend, stride, (int)cnt, (int)d,
                     (int)(has_ret != 0), rms, merged);
  FW_HIP(hipGetLastError());
  return FW_OK;
}

}  // extern "C"
