// fw_stats.hpp -- RunningMeanStd arithmetic shared by two translation units of libfwsim.so:
//   fw_rollout.hip  fw_rms_update / fw_vecnorm_merge_update (rank-ordered records, the sharded path)
//   fw_kernels.hip  k_env_step's collect epilogue, which merges the step's block records and applies
//                   update_from_moments inside the launch (fw_collect_epilogue.merged / .rms)
// Both must produce the same bits for the same record, so every function body disables FP contraction
// itself (fw_kernels.hip is compiled with the default contraction; fw_rollout.hip turns it off file-wide):
// numpy evaluates each product and sum with its own rounding.
#pragma once

#include <hip/hip_runtime.h>

namespace fw_stats {

struct Mom {
  double n, mean, m2;
};

// parallel-variance merge (Chan et al.), a then b
__device__ __forceinline__ Mom chan(Mom a, Mom b) {
#pragma clang fp contract(off)
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

// update_from_moments of one column (running_mean_std.py:26-40, same operation order): the batch's mean, var
// and count folded into (mean, var) that held `count` samples.  Shared by rms_update and the deferred final
// merge (fw_rollout.hip k_policy_mfma / k_pending_update), so every path produces the same bits.
__device__ __forceinline__ void update_col(double bmean, double bvar, double bc, double count, double& mean,
                                           double& var) {
#pragma clang fp contract(off)
  const double delta = bmean - mean;
  const double tot = count + bc;
  const double new_mean = mean + delta * bc / tot;
  const double m_a = var * count;
  const double m_b = bvar * bc;
  const double m_2 = m_a + m_b + delta * delta * count * bc / (count + bc);
  mean = new_mean;
  var = m_2 / (count + bc);
}

// The final node of the in-launch merge tree for one column, computed by one lane from the node's cnt records
// (record k's n / mean_j / M2_j at nrow[k] / mrow[k] / qrow[k]): N = sum n_k, mean = (sum n_k mean_k) / N,
// M2 = sum (M2_k + n_k (mean_k - mean)^2), every sum in record order -- the arithmetic of fw_kernels.hip
// merge_node, whose 64-slot row sums add +0.0 for absent records (which leaves these sums unchanged), so the
// bits are the same.
__device__ __forceinline__ void merge_col(const double* nrow, const double* mrow, const double* qrow, int cnt,
                                          double& N, double& mean, double& m2) {
#pragma clang fp contract(off)
  // (reads in batches of 8, issued together; the sums stay in record order)
  constexpr int B = 8;
  double a = 0.0, s = 0.0;
  int k = 0;
  for (; k + B <= cnt; k += B) {
    double nv[B], mv[B];
#pragma unroll
    for (int u = 0; u < B; u++) {
      nv[u] = nrow[k + u];
      mv[u] = mrow[k + u];
    }
#pragma unroll
    for (int u = 0; u < B; u++) {
      a += nv[u];
      s += nv[u] * mv[u];
    }
  }
  for (; k < cnt; k++) {
    a += nrow[k];
    s += nrow[k] * mrow[k];
  }
  N = a;
  mean = s / a;
  double q = 0.0;
  k = 0;
  for (; k + B <= cnt; k += B) {
    double nv[B], mv[B], qv[B];
#pragma unroll
    for (int u = 0; u < B; u++) {
      nv[u] = nrow[k + u];
      mv[u] = mrow[k + u];
      qv[u] = qrow[k + u];
    }
#pragma unroll
    for (int u = 0; u < B; u++) {
      const double dm = mv[u] - mean;
      q += qv[u] + nv[u] * (dm * dm);
    }
  }
  for (; k < cnt; k++) {
    const double dm = mrow[k] - mean;
    q += qrow[k] + nrow[k] * (dm * dm);
  }
  m2 = q;
}

// RunningMeanStd.update_from_moments (running_mean_std.py:26-40, same operation order) over n_parts records
// (contiguous, 1 + 2D each: n, mean[D], M2[D]; D = d + has_ret) merged in order; rms = [mean d | var d |
// count | ret mean | ret var | ret count].  Thread j < D owns column j.  Every thread of the block calls
// it (old_count, two doubles in LDS, is shared behind a barrier).
__device__ __forceinline__ void rms_update(const double* __restrict__ parts, int n_parts, int d, int has_ret,
                                           double* __restrict__ rms, int update_obs, int update_ret,
                                           double* old_count) {
#pragma clang fp contract(off)
  const int D = d + (has_ret ? 1 : 0);
  const int S = 1 + 2 * D;
  const int j = threadIdx.x;
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
      double mean = *mean_p, var = *var_p;
      update_col(bmean, bvar, bc, count, mean, var);
      *mean_p = mean;
      *var_p = var;
      if (j == (is_ret ? d : 0)) {
        if (is_ret)
          rms[2 * d + 3] = bc + count;
        else
          rms[2 * d] = bc + count;
      }
    }
  }
}

// The in-launch merge tree of k_env_step's block records (fw_collect_epilogue.merged): level 0 holds one
// record per launch block; a level with more than MERGE_FANIN records is merged in groups of MERGE_FANIN
// consecutive records into the next level; a level with at most MERGE_FANIN records is merged into the
// final one.  Every node is merged by the last block to arrive at it, in record order, so the bits do not
// depend on which block finishes when.  merge_tree_size gives the workspace the levels above 0 need.
constexpr int MERGE_FANIN = 64;

__host__ __device__ inline int64_t merge_ceil(int64_t a, int64_t b) { return (a + b - 1) / b; }

// (record slots, counters) needed above level 0 for a launch of `blocks` blocks
__host__ __device__ inline void merge_tree_size(int64_t blocks, int64_t* records, int64_t* counters) {
  int64_t r = 0, c = 0, nodes = blocks;
  while (nodes > MERGE_FANIN) {
    const int64_t up = merge_ceil(nodes, MERGE_FANIN);
    r += up;
    c += up;
    nodes = up;
  }
  *records = r;
  *counters = c + 1;  // + the final node's
}

}  // namespace fw_stats
