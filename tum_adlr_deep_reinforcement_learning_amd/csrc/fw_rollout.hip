// fw_rollout.hip -- rollout-side kernels of libfwsim.so (include/fwrollout.h):
// the device RolloutBuffer's GAE scan and the device VecNormalize statistics.
//
//   k_gae              RolloutBuffer.compute_returns_and_advantage
//                      (stable_baselines3/common/buffers.py:304-333).  One lane per env,
//                      reverse scan over time; rows [t][N] are read coalesced and
//                      prefetched GAE_PF steps ahead (the recurrence is serial, the loads
//                      are not).  HBM-bound: 4+4+1 B read, 4+4 B written per (step, env).
//   k_moments_partial  RunningMeanStd.update's batch mean/var (running_mean_std.py:20-24):
//   k_moments_merge    per-lane Welford, Chan merges in a fixed tree -> deterministic.
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
#include <string>

#include "../../include/fwrollout.h"
#include "../../include/fwsim.h"

#pragma clang fp contract(off)

namespace fw {
int set_error(int code, const std::string& msg);
}

namespace {

constexpr int BLOCK = 256;
constexpr int GAE_PF = 16;   // time steps loaded ahead per lane
constexpr int MAXD = 33;     // observation dims (FW_MAX_OBS) + the return column
constexpr int MAX_PARTS = 1024;

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
    const double delta = __dsub_rn(__dadd_rn((double)rew[t * N + e], __dmul_rn((double)a, nnt)), (double)v);
    const double last0 = __dadd_rn(delta, __dmul_rn(__dmul_rn(gl, nnt), 0.0));
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
          const float b = __fmul_rn(__fmul_rn(gamma_f, nv), nnt);
          const float dl = __fsub_rn(__fadd_rn(rr[k], b), vv[k]);
          const float coef = __fmul_rn(gl_f, nnt);
          last = __dadd_rn((double)dl, __dmul_rn((double)coef, last));
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
struct Mom {
  double n, mean, m2;
};

__device__ __forceinline__ Mom chan(Mom a, Mom b) {  // parallel-variance merge, a then b
  if (b.n == 0.0) return a;
  if (a.n == 0.0) return b;
  const double n = a.n + b.n;
  const double delta = b.mean - a.mean;
  Mom r;
  r.n = n;
  r.mean = a.mean + delta * (b.n / n);
  r.m2 = a.m2 + b.m2 + delta * delta * (a.n * b.n / n);
  return r;
}

// LDS tree over BLOCK records; returns the merged record on thread 0.
__device__ Mom block_merge(Mom m, double* sn, double* sm, double* sq) {
  const int tid = threadIdx.x;
  sn[tid] = m.n;
  sm[tid] = m.mean;
  sq[tid] = m.m2;
  __syncthreads();
  for (int s = BLOCK / 2; s > 0; s >>= 1) {
    if (tid < s) {
      const Mom r = chan(Mom{sn[tid], sm[tid], sq[tid]}, Mom{sn[tid + s], sm[tid + s], sq[tid + s]});
      sn[tid] = r.n;
      sm[tid] = r.mean;
      sq[tid] = r.m2;
    }
    __syncthreads();
  }
  const Mom out{sn[0], sm[0], sq[0]};
  __syncthreads();
  return out;
}

__global__ __launch_bounds__(BLOCK) void k_moments_partial(const float* __restrict__ x, int64_t n, int d, int64_t ldx,
                                                           const float* __restrict__ rew, double* __restrict__ retv,
                                                           double gamma, int64_t rows_per, double* __restrict__ part) {
  __shared__ double sn[BLOCK], sm[BLOCK], sq[BLOCK];
  const int D = d + (rew ? 1 : 0);
  const int64_t r0 = (int64_t)blockIdx.x * rows_per;
  const int64_t r1 = std::min(n, r0 + rows_per);
  double cnt = 0.0, mean[MAXD], m2[MAXD];
#pragma unroll
  for (int j = 0; j < MAXD; j++) mean[j] = m2[j] = 0.0;
  for (int64_t r = r0 + threadIdx.x; r < r1; r += BLOCK) {
    cnt += 1.0;
#pragma unroll
    for (int j = 0; j < MAXD; j++) {
      if (j < D) {
        double xv;
        if (j < d) {
          xv = (double)x[r * ldx + j];
        } else {  // VecNormalize._update_reward: ret = ret * gamma + reward  (vec_normalize.py:126-129)
          xv = retv[r] * gamma + (double)rew[r];
          retv[r] = xv;
        }
        const double delta = xv - mean[j];
        mean[j] += delta / cnt;
        m2[j] += delta * (xv - mean[j]);
      }
    }
  }
  double* out = part + (int64_t)blockIdx.x * (1 + 2 * D);
  for (int j = 0; j < D; j++) {
    double mj = 0.0, qj = 0.0;
#pragma unroll
    for (int k = 0; k < MAXD; k++)
      if (k == j) mj = mean[k], qj = m2[k];
    const Mom m = block_merge(Mom{cnt, mj, qj}, sn, sm, sq);
    if (threadIdx.x == 0) {
      out[0] = m.n;
      out[1 + j] = m.mean;
      out[1 + D + j] = m.m2;
    }
  }
}

// merges `parts` records (stride 1+2D) in a fixed order into one record
__global__ __launch_bounds__(BLOCK) void k_moments_merge(const double* __restrict__ part, int parts, int D,
                                                         double* __restrict__ out) {
  __shared__ double sn[BLOCK], sm[BLOCK], sq[BLOCK];
  const int S = 1 + 2 * D;
  for (int j = 0; j < D; j++) {
    Mom m{0.0, 0.0, 0.0};
    for (int k = threadIdx.x; k < parts; k += BLOCK) m = chan(m, Mom{part[k * S], part[k * S + 1 + j], part[k * S + 1 + D + j]});
    const Mom r = block_merge(m, sn, sm, sq);
    if (threadIdx.x == 0) {
      out[0] = r.n;
      out[1 + j] = r.mean;
      out[1 + D + j] = r.m2;
    }
  }
}

// RunningMeanStd.update_from_moments, one thread per column; parts merged in rank order.
__global__ void k_rms_update(const double* __restrict__ parts, int n_parts, int d, int has_ret, double* __restrict__ rms,
                             int update_obs, int update_ret) {
  const int D = d + (has_ret ? 1 : 0);
  const int S = 1 + 2 * D;
  const int j = threadIdx.x;
  __shared__ double old_count[2];
  if (j == 0) {
    old_count[0] = rms[2 * d];
    old_count[1] = rms[2 * d + 3];
  }
  __syncthreads();
  if (j < D) {
    const bool is_ret = j == d;
    if ((is_ret && update_ret) || (!is_ret && update_obs)) {
      Mom m{0.0, 0.0, 0.0};
      for (int k = 0; k < n_parts; k++) m = chan(m, Mom{parts[k * S], parts[k * S + 1 + j], parts[k * S + 1 + D + j]});
      const double bmean = m.mean, bvar = m.m2 / m.n, bc = m.n;
      double* mean_p = is_ret ? rms + 2 * d + 1 : rms + j;
      double* var_p = is_ret ? rms + 2 * d + 2 : rms + d + j;
      const double count = old_count[is_ret ? 1 : 0];
      const double mean = *mean_p, var = *var_p;
      // running_mean_std.py:26-40, same operation order
      const double delta = bmean - mean;
      const double tot = count + bc;
      const double new_mean = mean + delta * bc / tot;
      const double m_a = var * count;
      const double m_b = bvar * bc;
      const double m_2 = m_a + m_b + delta * delta * count * bc / (count + bc);
      *mean_p = new_mean;
      *var_p = m_2 / (count + bc);
      if (j == (is_ret ? d : 0)) {
        if (is_ret)
          rms[2 * d + 3] = bc + count;
        else
          rms[2 * d] = bc + count;
      }
    }
  }
}

__global__ __launch_bounds__(BLOCK) void k_vecnorm_apply(const float* __restrict__ obs, int64_t n, int d, int64_t ldx,
                                                         const double* __restrict__ rms, double eps, int norm_obs,
                                                         double clip_obs, float* __restrict__ obs_out, int64_t ld_out,
                                                         const float* __restrict__ rew, int norm_rew, double clip_rew,
                                                         float* __restrict__ rew_out, const uint8_t* __restrict__ done,
                                                         double* __restrict__ retv) {
  const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
  if (i >= n) return;
  if (obs_out) {
    for (int j = 0; j < d; j++) {
      const float o = obs[i * ldx + j];
      if (norm_obs) {  // np.clip((obs - mean) / np.sqrt(var + eps), -clip, clip).astype(float32)
        double y = ((double)o - rms[j]) / sqrt(rms[d + j] + eps);
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

unsigned grid_for(int64_t n) { return (unsigned)((n + BLOCK - 1) / BLOCK); }

int moments_parts(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>(MAX_PARTS, (n + BLOCK - 1) / BLOCK)); }

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
  const int parts = moments_parts(n);
  const int64_t rows_per = (n + parts - 1) / parts;
  const int D = d + (rew ? 1 : 0);
  if (D == 0) return fw::set_error(FW_E_INVALID, "fw_moments: nothing to reduce");
  hipStream_t s = (hipStream_t)stream;
  double* part = (double*)workspace;
  hipLaunchKernelGGL(k_moments_partial, dim3(parts), dim3(BLOCK), 0, s, x, n, d, ldx, rew, ret, gamma, rows_per, part);
  FW_HIP(hipGetLastError());
  hipLaunchKernelGGL(k_moments_merge, dim3(1), dim3(BLOCK), 0, s, part, parts, D, out);
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
  if (advance) {
    hipLaunchKernelGGL(k_row_advance, dim3(1), dim3(1), 0, s, ctrl_dev);
    FW_HIP(hipGetLastError());
  }
  return FW_OK;
}

}  // extern "C"
