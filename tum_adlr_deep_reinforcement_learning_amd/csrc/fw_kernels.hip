// fw_kernels.hip -- gfx950 kernels and the C ABI of libfwsim.so (include/fwsim.h).
//
// Data layout in HBM (one handle = one GPU): every per-aircraft quantity is a
// row of a structure-of-arrays block, [rows][ld] with ld = N rounded up to a
// multiple of 64, so lane i of a wave touches element i of each row: every
// global access below is a coalesced dword (or dwordx2 for fp64) per lane.
//
// Kernels (one lane = one aircraft, one-wave blocks, the RK45 state and
// stage vectors staged in LDS, no MFMA -- the work is elementwise ODE
// integration):
//   k_env_step   FixedWingAircraft.step + PyFly.step + masked auto-reset (hot path)
//   k_env_rollout K such steps per launch with actions given in advance (open loop)
//   k_sim_step   PyFly.step only
//   k_reset      masked reset (sampled with Philox or injected values)
//   k_observe    get_observation of the current state
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>

#include "fw_device.hpp"
#include "fw_stats.hpp"

// Parallel build (_native.py): this file is compiled as several translation units.  FW_PART = 0 holds
// the host code, the C ABI and the small kernels; FW_PART = 1..6 each instantiate one launch helper
// (fwl:: below) and with it one step kernel's template instances for one precision.  FW_PART
// undefined: everything in one unit.
#ifndef FW_PART
#define FW_PART -1
#endif
#define FW_HOST_PART (FW_PART <= 0)

using namespace fw;

#if FW_HOST_PART
namespace {
thread_local std::string g_err;
}  // namespace

// shared by every translation unit of libfwsim.so (fw_rollout.hip), read by fw_last_error
int fw::set_error(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
#endif

namespace {

int set_err(int code, const std::string& msg) { return fw::set_error(code, msg); }

#define FW_HIP(expr)                                                                              \
  do {                                                                                            \
    hipError_t e_ = (expr);                                                                       \
    if (e_ != hipSuccess) return set_err(FW_E_HIP, std::string(#expr ": ") + hipGetErrorString(e_)); \
  } while (0)

#ifndef FW_BLOCK
#define FW_BLOCK 64  // threads per block: one wave (measured 1-2% faster than 256, profiles/r01_ab_block.log)
#endif
constexpr int BLOCK = FW_BLOCK;
#ifndef FW_MIN_WAVES
#define FW_MIN_WAVES 1  // __launch_bounds__ minimum waves per SIMD of the env-step kernels (VGPR budget 512 / this)
#endif
#ifndef FW_QUAD_MIN_WAVES
#define FW_QUAD_MIN_WAVES 1  // ... of their quad (Q = 4) instances
#endif
#ifndef FW_PAIR_MIN_WAVES
#define FW_PAIR_MIN_WAVES 2  // ... of their pair (Q = 2) instances: two waves per SIMD (256 registers), the point of the pair
#endif
#define FW_WAVES(Q) ((Q) == 4 ? FW_QUAD_MIN_WAVES : (Q) == 2 ? FW_PAIR_MIN_WAVES : FW_MIN_WAVES)
#ifndef FW_HALF_WAVE
// A/B only (tools/r05_halfwave.sh; with FW_MIN_WAVES=2): one-lane k_env_step waves step 32 aircraft (lanes 0..31),
// twice the waves, so a second wave can share each SIMD.  No collect epilogue, no tail handoff to the idle lanes.
#define FW_HALF_WAVE 0
#endif
#ifndef FW_PREF_Q4_F64
// 1: the fp64 quad instances prefetch the epilogue's loads like the fp32 ones.  In fp64 the prefetched
// rows spill (339 VGPRs): 8192 aircraft 0.137 -> 0.099 ms per step without it (profiles/r03_ab_pref64.log)
#define FW_PREF_Q4_F64 0
#endif
#ifndef FW_PREF_Q4_F32
#define FW_PREF_Q4_F32 1  // 0: the fp32 quad instances load the epilogue's inputs after the integration (A/B)
#endif
#ifndef FW_PREF_Q1
#define FW_PREF_Q1 0  // 1: the one-lane k_env_step instances prefetch the epilogue's loads too (A/B)
#endif
#ifndef FW_LDS_STATE
#define FW_LDS_STATE 1  // 0 = y/f in VGPRs (measured: 512 VGPRs + spills, slower)
#endif
constexpr int RING = FW_MAX_WINDOW - 1;  // max previous actions kept

// ---------------------------------------------------------------------------
// SoA state block pointers
// ---------------------------------------------------------------------------
template <typename T>
struct State {
  int64_t n, ld;
  T* y;            // [19][ld]
  T* der;          // [8][ld]
  T* wind;         // [3][ld]
  T* target;       // [3][ld]
  T* cmd;          // [3][ld] last constrained commands
  T* ep_ret;       // [ld]
  T* act_ring;     // [act_window][3][ld], action k of an episode in slot (L_ep + k - 1) % act_window
  T* cmd_ring;     // [cmd_window][3][ld] or null, the same slots
  uint32_t* steps;    // [ld]: steps_count | steps_for_current_target << 16
  uint32_t* goal;     // [GB_ROWS][ld] goal-status history: nibble ring, window counts, entry count (below)
  uint32_t* episode;  // [ld]
  uint32_t* life;     // [ld] LIFE0 + env steps since the handle was created (never reset): every launch steps
                      // every aircraft, so the value is the same on all lanes -- ring slots are indexed by it
                      // (below).  Starting at LIFE0 >= 2^16 + any window keeps life - steps_count - window > 0
                      // whatever FW_BLK_STEPS a caller sets, so no slot expression wraps below 0.
  T* dry;             // [12][ld] Dryden filter-bank state of the current step (short chunks; null: FIR or off)
  T* shp;             // [3][ld] reward.form "potential": the previous step's shaping per function class (NaN =
                      // the reference's None, after a reset), or null
  T* rsc;             // [FW_MAX_REW][ld] reward.randomize_scaling: this episode's scaling per factor, or null
  // integration_window W (fixed_wing.py:1001-1012, 1160-1182): the error history's sums.  iwr: ring of the last W
  // errors per target, entry e in slot (L_ep + e) % W; iws rows IW_Q + k: sum of the last W of the n entries
  // so far, IW_QP + k: the same before the newest entry (what an "integrator" observation reads), IW_E0 + k:
  // entry 0 (the padding).  Null without an integration window.
  T* iwr;             // [W][3][ld]
  T* iws;             // [9][ld]
  const T* noise;     // injected N(0,1) turbulence noise [4][noise_len][ld] or null
  int64_t noise_len;
  int32_t* noise_env_len;  // [ld] per-env injected length (> 0 own, zeroed by the auto-reset; < 0 shared; 0 Philox) or null
  uint32_t key0, key1;  // Philox key = seed
  uint32_t env_offset;
  T* met;             // [MT_ROWS][ld] streaming episode-metric sums (null: metrics off)
  uint16_t* metu16;   // [M16_ROWS][ld] counters / indices
  T* met_out;         // [FW_NMETRIC][N] (SoA) record of done envs (null: not requested)
  T* obs_init;        // [n_obs][ld] raw observation row at the episode's reset (null: length-1 observations)
  T* obs_ring;        // [obs_hist][n_obs][ld] raw rows of past steps, slot = (L_ep + step) % obs_hist
  T* prm;             // [FW_NPARAM][ld] per-aircraft parameters (null: no randomisation)
  T* tpr;             // [12][ld] linear / sinusoidal target properties, per target: slope or amplitude, period,
                      // phase, bias (null: constant / compensate targets only)
  uint32_t* gflag;    // [ld] bit 0: goal_achieved, never cleared (fixed_wing.py:81, 546-547; null: no success reward)
  uint32_t* dcur;     // [ld] next draw of the env-draw tape (fw_set_env_draws)
  const T* tape;      // [tape_len][n] the env's np_random draws, or null: Philox
  int32_t tape_len;
  // collect epilogue of k_env_step (fw_set_collect_epilogue; all null: off)
  double* col_ret;    // [n] VecNormalize discounted return, or null
  double col_gamma;
  double* col_rec;    // [blocks][1 + 2 D] per-block moment records, or null
  int32_t* col_ctrl;  // rollout row counter advanced by the launch, or null
  double* col_merged; // [1 + 2 D] the launch's merged record (in-launch merge tree), or null: merged later
  double* col_rms;    // RunningMeanStd buffer update_from_moments is applied to (with col_merged), or null
  double* col_lvl;    // merge-tree records above level 0 (handle workspace, fw_stats::merge_tree_size)
  // merge-tree arrival counters (handle workspace, zero between launches); bit 0 of the address set: the tree
  // stops one level short (fw_collect_epilogue.defer; a flag bit, not a field: a larger State costs the quad
  // instances 64 B of scratch)
  uint32_t* col_cnt;
};

// streaming episode-metric state (fixed_wing.py:1644-1736 restated over running sums), packed (round 5):
// T rows: e0, sum, |sum|, the extremum overshoot reads (the minimum where e0 > 0, else the maximum), the sum of
// the last FW_M_END_WINDOW errors (x3 targets), control variation, ring of the last FW_M_END_WINDOW errors.  Not
// kept: the previous error (the ring's previous entry).  The window sum stays streaming (+ the new error - the
// one it overwrites in the ring): summed from the ring when the episode ends, the 150 scattered loads of every
// done aircraft put ~16 us on the steady-state launch (long-window median 0.080 -> 0.096 ms, tools/r05_longwin_ab.sh).
constexpr int MR_E0 = 0, MR_ESUM = 3, MR_EABS = 6, MR_EXT = 9, MR_WSUM = 12, MR_CV = 15, MR_RING = 16;
constexpr int MT_ROWS = MR_RING + 3 * FW_M_END_WINDOW;
// uint16 rows: goal counts (4), settling index (4, 0xFFFF = none), first crossings below the high / low rise
// limits (3 x 2)
constexpr int M16_GC = 0, M16_SET = 4, M16_RISE = 8;
constexpr int M16_ROWS = M16_RISE + 6;
constexpr uint32_t M_NONE = 0xFFFFu;
// goal-status history of the env (round 5; s.goal, uint32 rows).  The history entry e of the episode (0 = the
// reset state, one entry per successful step, fixed_wing.py:462-466, 536-538) keeps its four statuses
// (goal_status_bits: roll / pitch / Va within bound, all) in nibble (lep + e) % 8 of ring word ((lep + e) % 128) / 8
// -- indexed by the LIFETIME position, so every lane of a wave touches the same word row.  GB_CNT holds the ones
// among the last success_streak_req entries per status (one byte each, "all" in byte 3; 16 bits each in two words
// when success_streak_req > 255, round 6: GCnt), GB_N the entry count.  Round 6: the ring holds a power of two
// >= success_streak_req entries (at least 128); words beyond 16 follow the count rows (gring_row).
// A step reads the word the new entry goes to, the word holding the entry that leaves the window, the counts and
// the entry count (16 B) and writes three of them back: the 128-bit shift register of rounds 1-4 plus the
// metrics' per-target bit buffers moved 76 B per step.
constexpr int GB_RING = 0, GB_CNT = 16, GB_N = 17, GB_ROWS = 18;
constexpr uint32_t LIFE0 = 1u << 20;  // State::life at handle creation
// ring word w of the history (mask = entries - 1): words 0..15 in rows 0..15, words 16.. (success_streak_req > 128,
// round 6) after the count rows
__host__ __device__ __forceinline__ int gring_row(uint32_t pos, uint32_t mask) {
  const int w = (int)((pos & mask) >> 3);
  return GB_RING + (w < 16 ? w : w + 2);
}
// the window counts per status (roll, pitch, Va, all): four bytes in GB_CNT, or -- streak_req > 255 -- 16-bit
// fields in GB_CNT (roll, pitch) and the row gcnt2_row (Va, all)
struct GCnt {
  uint32_t w0, w1;
  bool wide;
  __device__ __forceinline__ uint32_t get(int k) const {
    return wide ? ((k < 2 ? w0 : w1) >> (16 * (k & 1))) & 0xFFFFu : (w0 >> (8 * k)) & 0xFFu;
  }
  __device__ __forceinline__ void set(int k, uint32_t v) {
    if (wide) {
      const int sh = 16 * (k & 1);
      if (k < 2) w0 = (w0 & ~(0xFFFFu << sh)) | (v << sh);
      else w1 = (w1 & ~(0xFFFFu << sh)) | (v << sh);
    } else {
      w0 = (w0 & ~(0xFFu << (8 * k))) | (v << (8 * k));
    }
  }
};
__device__ __forceinline__ uint32_t gring_get(uint32_t w, uint32_t pos) { return (w >> (4u * (pos & 7u))) & 0xFu; }
__device__ __forceinline__ uint32_t gring_set(uint32_t w, uint32_t pos, uint32_t nib) {
  const uint32_t sh = 4u * (pos & 7u);
  return (w & ~(0xFu << sh)) | (nib << sh);
}
constexpr int MD_EXT = 0, MD_U = 3;  // Met::dirty bits: 3 extremum rows, then the M16_ROWS - M16_GC rare u16 rows
static_assert(MD_U + (M16_ROWS - M16_GC) <= 32, "Met::dirty holds one bit per rarely-changing row");

// Debug build only (-DFW_TIMING, tools/phase_timing.py): lane 0 of every wave stamps the
// 100 MHz real-time clock at phase boundaries into the episode_out buffer (8 x u64 per wave),
// after draining all outstanding memory operations.
#ifdef FW_TIMING
#define FW_TSTAMP(k)                                                                                 \
  do {                                                                                               \
    __builtin_amdgcn_s_waitcnt(0);                                                                   \
    if ((threadIdx.x & 63) == 0 && episode_out)                                                      \
      ((unsigned long long*)episode_out)[(((int64_t)blockIdx.x * BLOCK + threadIdx.x) >> 6) * 8 + (k)] = \
          __builtin_amdgcn_s_memrealtime();                                                          \
  } while (0)
#else
#define FW_TSTAMP(k) \
  do {               \
  } while (0)
#endif

template <typename T>
__device__ __forceinline__ T ld_(const T* p, int64_t row, int64_t ld, int64_t i) {
  return p[row * ld + i];
}
template <typename T>
__device__ __forceinline__ void st_(T* p, int64_t row, int64_t ld, int64_t i, T v) {
  p[row * ld + i] = v;
}

// N(0,1) turbulence noise sample (4 channels) of step index k of the current episode.  Injected noise
// shorter than the episode wraps: DrydenGustModel.simulate reads noise[:, (t_span[0] + j) % len] in every
// branch of dryden.py:209-236 (slice, modulo start, concatenation, np.pad(mode="wrap")).
template <typename T>
__device__ __forceinline__ void noise4(const State<T>& s, int64_t i, uint32_t episode, int k, T u[4]) {
  if (s.noise) {
    // per-env lengths: > 0 an env's own injection, < 0 the shared set_noise sequence (kept across resets), 0 Philox
    const int64_t len = s.noise_env_len ? (int64_t)abs(s.noise_env_len[i]) : s.noise_len;
    if (len > 0) {
      const int64_t kk = (int64_t)((uint32_t)k % (uint32_t)len);  // len < 2^31 (fw_set_noise)
#pragma unroll
      for (int ch = 0; ch < 4; ch++) u[ch] = s.noise[((int64_t)ch * s.noise_len + kk) * s.ld + i];
      return;
    }
  }
  uint32_t r[4];
  philox(s.key0, s.key1, s.env_offset + (uint32_t)i, episode, 1u, (uint32_t)k, r);
  normal4<T>(r, u);
}

// The Dryden filter bank for chunks too short for the FIR (fw_sim_config.dryden_state, fwsim.h): State::dry
// holds x_k, the filters' state at step k (0 at reset); the turbulence of step k is C x_k, and the step
// (lead lane only: a quad's four lanes compute the same) stores x_{k+1} = Ad x_k + Bd0 u_k + Bd1 u_{k+1} --
// scipy lsim's first-order hold inside a chunk (dryden.py:238-252 as wired by pyfly.py:781-783) -- or, at
// a chunk boundary, E1^c x_k (lsim's zero-input step to t[0] = c L^2 for chunk c; 0 from dryden_ncut on).
template <typename T>
__device__ __forceinline__ void dryden_bank_at(const DevCfg<T>& c, const State<T>& s, int64_t i, uint32_t episode,
                                               int k, T tl[3], T ta[3], bool lead) {
  constexpr int ord[6] = {1, 2, 2, 1, 3, 3}, chan[6] = {0, 1, 2, 3, 1, 2};
  T x[12], out[6];
#pragma unroll
  for (int r = 0; r < 12; r++) x[r] = ld_(s.dry, r, s.ld, i);
  {
    int ox = 0;
#pragma unroll
    for (int f = 0; f < 6; f++) {
      T y = T(0);
#pragma unroll
      for (int r = 0; r < ord[f]; r++) y += c.dry_c[ox + r] * x[ox + r];
      out[f] = y;
      ox += ord[f];
    }
  }
  tl[0] = out[0];
  tl[1] = out[1];
  tl[2] = out[2];
  ta[0] = out[3];
  ta[1] = out[4];
  ta[2] = out[5];
  if (!lead) return;
  const int kn = k + 1;
  T xn[12];
  if (kn % c.turb_len == 0) {  // the next step opens chunk ch: zero-input propagation of the last state
    const int ch = kn / c.turb_len;
#pragma unroll
    for (int r = 0; r < 12; r++) xn[r] = T(0);
    if (ch < c.dry_ncut) {
#pragma unroll
      for (int r = 0; r < 12; r++) xn[r] = x[r];
      for (int p = 0; p < ch; p++) {
        int oa = 0, ox = 0;
#pragma unroll
        for (int f = 0; f < 6; f++) {
          T t[3];
#pragma unroll
          for (int r = 0; r < ord[f]; r++) {
            t[r] = T(0);
#pragma unroll
            for (int q = 0; q < ord[f]; q++) t[r] += c.dry_e1[oa + r * ord[f] + q] * xn[ox + q];
          }
#pragma unroll
          for (int r = 0; r < ord[f]; r++) xn[ox + r] = t[r];
          oa += ord[f] * ord[f];
          ox += ord[f];
        }
      }
    }
  } else {
    T u0[4], u1[4];
    noise4(s, i, episode, k, u0);
    noise4(s, i, episode, kn, u1);
    int oa = 0, ox = 0;
#pragma unroll
    for (int f = 0; f < 6; f++) {
      const T a = c.noise_scale * u0[chan[f]], b = c.noise_scale * u1[chan[f]];
#pragma unroll
      for (int r = 0; r < ord[f]; r++) {
        T t = c.dry_b0[ox + r] * a + c.dry_b1[ox + r] * b;
#pragma unroll
        for (int q = 0; q < ord[f]; q++) t += c.dry_ad[oa + r * ord[f] + q] * x[ox + q];
        xn[ox + r] = t;
      }
      oa += ord[f] * ord[f];
      ox += ord[f];
    }
  }
#pragma unroll
  for (int r = 0; r < 12; r++) st_(s.dry, r, s.ld, i, xn[r]);
}

template <typename T>
__device__ __forceinline__ void turbulence_at(const DevCfg<T>& c, const State<T>& s, int64_t i, uint32_t episode, int k,
                                              T tl[3], T ta[3], bool lead = true) {
  tl[0] = tl[1] = tl[2] = ta[0] = ta[1] = ta[2] = T(0);
  if (!c.turbulence) return;
  if (c.dry_state && s.dry) {  // (fw_update_config refuses the filter bank on a handle without its rows)
    dryden_bank_at(c, s, i, episode, k, tl, ta, lead);
    return;
  }
  if (k % c.turb_len == 0) return;
  T un1[4], u0[4];
  noise4(s, i, episode, k - 1, un1);
  noise4(s, i, episode, k, u0);
  dryden(c, k, un1, u0, tl, ta);
}

// a[k] for a runtime k by selects: a register array indexed at run time would be placed in scratch
template <typename T>
__device__ __forceinline__ T pick3(const T* a, int k) {
  return k == 0 ? a[0] : (k == 1 ? a[1] : a[2]);
}

// the same from three values that pass an opaque register copy first: a select of three ELEMENTS of a register
// array (y) is folded into a select of their addresses, which puts the array in scratch
template <typename T>
__device__ __forceinline__ T pick3v(T a0, T a1, T a2, int k) {
  asm volatile("" : "+v"(a0), "+v"(a1), "+v"(a2));
  return k == 0 ? a0 : (k == 1 ? a1 : a2);
}

// value of an observed / rewarded state variable from the stored state
template <typename T>
__device__ __forceinline__ T state_value(int var, const T* y, const T* der) {
  switch (var) {
    case FW_V_ROLL: return der[0];
    case FW_V_PITCH: return der[1];
    case FW_V_YAW: return der[2];
    case FW_V_VA: return der[3];
    case FW_V_ALPHA: return der[4];
    case FW_V_BETA: return der[5];
    case FW_V_ELEVATOR: return der[6];
    case FW_V_AILERON: return der[7];
    case FW_V_THROTTLE: return y[15];
    case FW_V_ACT0: return y[13];
    case FW_V_ACT1: return y[14];
    case FW_V_ACT2: return y[15];
    default: {  // omega p q r, position n e d, velocity u v w = y[4 .. 12]
      const int k = var - FW_V_OMEGA_P;
      if constexpr (sizeof(T) == 4) {
        return y[4 + k];  // (fp32: the 19-float state stays a register vector at a runtime index)
      } else {
        // fp64: y at a runtime index (the factor / entry loops are not unrolled) put the 19-double state in
        // scratch, and plain selects were folded back into a select of addresses: each candidate passes an
        // opaque register copy, so the pick is a select of values
        T v = y[12];
#pragma unroll
        for (int j = 0; j < 8; j++) {
          T yj = y[4 + j];
          asm volatile("" : "+v"(yj));
          v = k == j ? yj : v;
        }
        return v;
      }
    }
  }
}

// get_observation (fixed_wing.py:1113-1262): length-1 vector observation.
// seqA / seqC: newest-first sequences of raw actions / constrained commands
// (index 0 = latest), nseq = number of valid entries (= steps_count).
template <typename T>
__device__ __forceinline__ T obs_raw(const DevCfg<T>& c, const fw_obs_entry& E, const T* y, const T* der,
                                     const T* tgt, int steps, const T (*seqA)[3], const T (*seqC)[3]) {
  {
    T val;
    if (E.kind == FW_OBS_STATE) {
      val = state_value(E.var, y, der);
    } else if ((E.kind == FW_OBS_TARGET_ABS || E.kind == FW_OBS_TARGET_REL) && E.var >= FW_TGT_OMEGA_P) {
      val = T(0);  // (an attitude_angular target: written afterwards, ang_obs)
    } else if (E.kind == FW_OBS_TARGET_ABS) {
      val = pick3(tgt, E.var);
    } else if (E.kind == FW_OBS_TARGET_REL) {
      const int tv = E.var == 0 ? FW_V_ROLL : (E.var == 1 ? FW_V_PITCH : FW_V_VA);
      val = target_error(c, E.var, pick3(tgt, E.var), state_value(tv, y, der));
    } else if (E.kind == FW_OBS_TARGET_INT) {
      val = T(0);  // (written afterwards from the window sums: iw_obs)
    } else {  // action window
      const int ai = E.var;
      if (steps - 1 < 0) {
        const int av[3] = {FW_V_ELEVATOR, FW_V_AILERON, FW_V_THROTTLE};
        val = state_value(av[ai], y, der);
        if (c.scale_actions) val = scale_bwd(c, ai, val);
      } else {
        // all indices static (runtime-indexed private arrays would go to scratch)
        const bool sa = c.scale_actions;
        const int w = E.window < steps ? E.window : steps;  // entries in the window
        float acc = 0.0f;                                    // np.sum(..., dtype=np.float32)
#pragma unroll
        for (int j = RING - 1; j >= 0; j--) {                // oldest diff first
          if (j + 1 < w) {
            const T d0 = sa ? seqA[j][0] - seqA[j + 1][0] : seqC[j][0] - seqC[j + 1][0];
            const T d1 = sa ? seqA[j][1] - seqA[j + 1][1] : seqC[j][1] - seqC[j + 1][1];
            const T d2 = sa ? seqA[j][2] - seqA[j + 1][2] : seqC[j][2] - seqC[j + 1][2];
            acc += (float)fabs(ai == 0 ? d0 : (ai == 1 ? d1 : d2));
          }
        }
        val = (T)acc;
      }
    }
    return val;
  }
}

template <typename T>
__device__ __forceinline__ T obs_norm(const fw_obs_entry& E, T val) {
  return E.norm ? (val - (T)E.mean) / (T)E.var_ : val;
}

// integration_window (State::iws): rows of the window sums
constexpr int IW_Q = 0, IW_QP = 3, IW_E0 = 6;
// the sum plus the padding of an integrator value: s + (W - x) e0 when x < W (fixed_wing.py:1009-1012, 1177-1181)
template <typename T>
__device__ __forceinline__ T iw_value(const DevCfg<T>& c, T sum, int x, T e0) {
  return x < c.iwin ? sum + T(c.iwin - x) * e0 : sum;
}
// the "integrator" entries of observation row r (v3: the raw values per target).  The row was written with
// 0 in their place; on the general path (observation noise, or a history row's init noise) that entry
// already carries its draws (fixed_wing.py:1236-1247: + init noise, normalise, + noise), so the value goes
// in as the difference.
template <typename T>
__device__ __forceinline__ void iw_obs(const DevCfg<T>& c, const T* v3, T* out, int r = 0) {
  if (!out) return;
  for (int o = 0; o < c.n_obs; o++) {
    const fw_obs_entry E = c.obs[o];
    if (E.kind == FW_OBS_TARGET_INT) {
      const T v = obs_norm(E, pick3(v3, E.var));
      T& dst = out[r * c.n_obs + o];
      dst = c.obs_general ? dst + (v - obs_norm(E, T(0))) : v;
    }
  }
}
// a reset observation: every history row is the lag-1 row (i > steps_count -> i = steps_count + 1 = 1)
template <typename T>
__device__ __forceinline__ void iw_obs_all_rows(const DevCfg<T>& c, const T* v3, T* out) {
  for (int r = 0; r < c.obs_len; r++) iw_obs(c, v3, out, r);
}
// the attitude_angular target entries of an observation (obs_raw wrote 0 in their place; plain length-1,
// noise-free observations only, config.py): the omega target (absolute) or its error target - omega (relative,
// _get_error: omega does not wrap), normalised (fixed_wing.py:1133-1247)
template <typename T>
__device__ __forceinline__ void ang_obs(const DevCfg<T>& c, const T* ot, const T* y, T* out) {
  if (!out) return;
  for (int o = 0; o < c.n_obs; o++) {
    const fw_obs_entry E = c.obs[o];
    if ((E.kind == FW_OBS_TARGET_ABS || E.kind == FW_OBS_TARGET_REL) && E.var >= FW_TGT_OMEGA_P) {
      const int k = E.var - FW_TGT_OMEGA_P;
      const T t = pick3(ot, k);
      out[o] = obs_norm(E, E.kind == FW_OBS_TARGET_ABS ? t : t - pick3v(y[4], y[5], y[6], k));
    }
  }
}
// the attitude_angular targets as stored (State::tpr rows 12..14)
template <typename T>
__device__ __forceinline__ void ang_load(const State<T>& s, int64_t i, T* ot) {
#pragma unroll
  for (int k = 0; k < 3; k++) ot[k] = s.tpr[(int64_t)(12 + k) * s.ld + i];
}
// observation history (observation.length > 1): the raw row kept for later lags holds the integrator
// entries' lag-1 values, so a lagged row reads slice [-W-i:-i] as the reference does (its padding condition
// steps - i < W is the lag-1 one at step steps - i + 1).  dst: the history row just written by observe_full.
template <typename T>
__device__ __forceinline__ void iw_hist_row(const DevCfg<T>& c, const State<T>& s, int64_t i, const T* v3, T* dst) {
  for (int o = 0; o < c.n_obs; o++)
    if (c.obs[o].kind == FW_OBS_TARGET_INT) dst[(int64_t)o * s.ld + i] = pick3(v3, c.obs[o].var);
}
// the reset row kept for lags beyond the episode: slice [-W-steps-1:-steps-1] is empty and the padding
// (W + 1) e0 (the current episode's entry 0), whatever the reset observation itself read
template <typename T>
__device__ __forceinline__ void iw_hist_init(const DevCfg<T>& c, const State<T>& s, int64_t i, const T* tgt,
                                             const T* der) {
  if (c.obs_hist == 0) return;
  const T vals[3] = {der[0], der[1], der[3]};
  T v3[3];
#pragma unroll
  for (int k = 0; k < 3; k++) v3[k] = target_error(c, k, tgt[k], vals[k]) * T(c.iwin + 1);
  iw_hist_row(c, s, i, v3, s.obs_init);
}
// a failed step (ConstraintException): the error history was not appended, so a lagged row's slice ends one
// entry earlier relative to steps_count, and its padding (W - (steps - i)) e0 holds one e0 less than the
// stored lag-1 value of that step whenever the stored value was padded (row step at <= W)
template <typename T>
__device__ __forceinline__ void iw_obs_fail(const DevCfg<T>& c, const State<T>& s, int64_t i, int steps, uint32_t lep,
                                            T* out) {
  if (!out || c.obs_len <= 1) return;
  const int64_t ld = s.ld;
  for (int r = 1; r < c.obs_len; r++) {
    const int lag = 1 + r * c.obs_step;
    if (lag > steps) break;  // clamped rows: the reset row, (W + 1) e0 either way
    const int at = steps - lag;
    if (at > c.iwin) continue;
    for (int o = 0; o < c.n_obs; o++) {
      const fw_obs_entry E = c.obs[o];
      if (E.kind != FW_OBS_TARGET_INT) continue;
      const T v = at <= 0 ? s.obs_init[(int64_t)o * ld + i]
                          : s.obs_ring[((int64_t)((lep + (uint32_t)at) % (uint32_t)c.obs_hist) * c.n_obs + o) * ld + i];
      const T e0 = ld_(s.iws, IW_E0 + E.var, ld, i);
      T& dst = out[r * c.n_obs + o];
      dst = dst + (obs_norm(E, v - e0) - obs_norm(E, v));
    }
  }
}
// a fresh episode's error history: entry 0 in its ring slot, the sums of one entry
template <typename T>
__device__ __forceinline__ void iw_init(const DevCfg<T>& c, const State<T>& s, int64_t i, const T* tgt, const T* der,
                                        uint32_t lep) {
  const int64_t ld = s.ld;
  const int slot = (int)(lep % (uint32_t)c.iwin);
  const T vals[3] = {der[0], der[1], der[3]};
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const T e0 = target_error(c, k, tgt[k], vals[k]);
    st_(s.iwr, slot * 3 + k, ld, i, e0);
    st_(s.iws, IW_Q + k, ld, i, e0);
    st_(s.iws, IW_QP + k, ld, i, T(0));
    st_(s.iws, IW_E0 + k, ld, i, e0);
  }
}

// length-1 observation without noise (the default task): one row straight from the state
template <typename T>
__device__ __forceinline__ void observe(const DevCfg<T>& c, const T* y, const T* der, const T* tgt, int steps,
                                        const T (*seqA)[3], const T (*seqC)[3], T* out, int64_t stride) {
  for (int o = 0; o < c.n_obs; o++) {
    const fw_obs_entry E = c.obs[o];
    out[(int64_t)o * stride] = obs_norm(E, obs_raw(c, E, y, der, tgt, steps, seqA, seqC));
  }
}

// get_observation with history rows and/or noise (fixed_wing.py:1113-1262).  Row r is the
// observation at lag i = 1 + r * step, built from the raw (un-normalised, noise-free) rows this
// env stored at earlier steps: the reference reads state.history[-i], history["target"/"error"][-i]
// and the action window ending i-1 steps ago, which are exactly the values its lag-1 row had at
// step t-i+1.  On a failed step (ConstraintException) the state/target/error histories were not
// appended, so those entries come from step t-i while the action window (appended before the
// integration) still ends at step t-i+1.  Lags beyond the episode (i > steps_count) repeat the
// episode's first row (actions: the actuator's current value) plus one U(-1,1)*dt offset per row
// (init_noise).  Then normalisation, then N(mean, std) noise per value.
constexpr int OBS_STEP = 0, OBS_FAIL = 1, OBS_RESET = 2, OBS_PEEK = 3;

template <typename T>
__device__ __forceinline__ void observe_full(const DevCfg<T>& c, const State<T>& s, int64_t i, uint32_t episode,
                                          int mode, const T* y, const T* der, const T* tgt, int steps,
                                          const T (*seqA)[3], const T (*seqC)[3], T* out, uint32_t lep) {
  const int64_t ld = s.ld;
  const int nr = c.n_obs;
  const bool hist = c.obs_hist > 0;
  const uint32_t ctr = s.env_offset + (uint32_t)i;
  uint32_t rnd[4] = {0u, 0u, 0u, 0u};
  T z[4] = {T(0), T(0), T(0), T(0)};
  int e = 0;  // value index across rows (noise block = e / 4)
  for (int r = 0; r < c.obs_len; r++) {
    const int lag = 1 + r * c.obs_step;
    const bool clamp = lag > steps;
    T inoise = T(0);
    if (clamp && c.obs_len > 1) {  // self.np_random.uniform(-1, 1) * dt
      philox(s.key0, s.key1, ctr, episode, 3u, (uint32_t)steps * 16u + (uint32_t)r, rnd);
      inoise = (T(2) * u01<T>(rnd[0]) - T(1)) * c.dt;
    }
    for (int o = 0; o < nr; o++, e++) {
      const fw_obs_entry E = c.obs[o];
      const bool act = E.kind == FW_OBS_ACTION_WINDOW;
      T v;
      if (!clamp && lag == 1) {
        v = obs_raw(c, E, y, der, tgt, steps, seqA, seqC);
      } else if (!clamp) {
        const int at = (mode == OBS_FAIL && !act) ? steps - lag : steps - lag + 1;  // step whose row holds it
        v = at <= 0 ? s.obs_init[(int64_t)o * ld + i]
                    : s.obs_ring[((int64_t)((lep + (uint32_t)at) % (uint32_t)c.obs_hist) * nr + o) * ld + i];
      } else if (act || steps == 0) {
        v = obs_raw(c, E, y, der, tgt, 0, seqA, seqC);  // current values (steps_count - i < 0 branch)
      } else {
        v = s.obs_init[(int64_t)o * ld + i];
      }
      v = obs_norm(E, v + inoise);
      if (c.obs_noise) {
        if ((e & 3) == 0) {
          philox(s.key0, s.key1, ctr, episode, 2u, (uint32_t)steps * 256u + (uint32_t)(e >> 2), rnd);
          normal4<T>(rnd, z);
        }
        v += c.obs_noise_mean + c.obs_noise_std * z[e & 3];
      }
      if (out) out[e] = v;
    }
  }
  if (hist && (mode == OBS_RESET || mode == OBS_STEP)) {  // this step's raw row for later lags
    T* dst = mode == OBS_RESET ? s.obs_init
                               : s.obs_ring + (int64_t)((lep + (uint32_t)steps) % (uint32_t)c.obs_hist) * nr * ld;
    for (int o = 0; o < nr; o++) dst[(int64_t)o * ld + i] = obs_raw(c, c.obs[o], y, der, tgt, steps, seqA, seqC);
  }
}

// dispatch: the plain row for the default task, the general path otherwise (compiled out of the
// structural specialisations, whose obs_general is a constant 0)
template <typename T, typename C>
__device__ __forceinline__ void observe_env(const C& c, const State<T>& s, int64_t i, uint32_t episode, int mode,
                                            const T* y, const T* der, const T* tgt, int steps, const T (*seqA)[3],
                                            const T (*seqC)[3], T* out, uint32_t lep) {
  if (c.obs_general) observe_full<T>(c, s, i, episode, mode, y, der, tgt, steps, seqA, seqC, out, lep);
  else observe<T>(c, y, der, tgt, steps, seqA, seqC, out, 1);
}

// get_reward (fixed_wing.py:941-1111), form "absolute"
template <typename T>
// shp (when pot): with reward.form "potential", the previous step's shaping per function class (NaN = None)
// on input, this step's on output (fixed_wing.py:1080-1108)
// rsc: with reward.randomize_scaling, this aircraft's column of State::rsc (row stride ld), else null
// iwq (when iw): with an integration window, the sums of the last W errors (3) then entry 0 (3)
// (shp / iwq are register arrays taken by reference with a flag: a pointer that may be null would take their
// address and place them in scratch)
// succ: goal_achieved_on_step (fixed_wing.py:546, 565): the first success of the env's lifetime, this step
// ot: the attitude_angular targets omega_p / q / r (c.ang; factors with var FW_TGT_OMEGA_P + k)
__device__ __forceinline__ T reward_of(const DevCfg<T>& c, const T* y, const T* der, const T* tgt, int steps,
                                       const T (*seqA)[3], T (&shp)[3], bool pot, const T* rsc, int64_t ld,
                                       const T (&iwq)[6], bool iw, bool succ, const T (&ot)[3]) {
  T tv[3] = {T(0), T(0), T(0)}, ts[3] = {T(0), T(0), T(0)};
  for (int f = 0; f < c.n_rew; f++) {
    const fw_rew_factor F = c.rew[f];
    const T scl = (rsc && F.randomize) ? rsc[f * ld] : (T)F.scaling;
    T val = T(0);
    if (F.kind == FW_REW_ACTION_VALUE) {
      val = fabs(seqA[0][0]) + fabs(seqA[0][1]) + fabs(seqA[0][2]);
    } else if (F.kind == FW_REW_ACTION_DELTA) {
      if (steps > 1) {
        const int w = F.window < steps ? F.window : steps;
#pragma unroll
        for (int j = RING - 1; j >= 0; j--) {
          if (j + 1 < w) {
#pragma unroll
            for (int a = 0; a < 3; a++) val += fabs(seqA[j][a] - seqA[j + 1][a]);
          }
        }
      }
    } else if (F.kind == FW_REW_ACTION_BOUND) {
#pragma unroll
      for (int a = 0; a < 3; a++) {
        const T x = seqA[0][a];
        const T hi = x > c.bmax ? x - c.bmax : T(0);
        const T lo = x < c.bmin ? x - c.bmin : T(0);
        val += fabs(hi) + fabs(lo);
      }
    } else if (F.kind == FW_REW_STATE_VALUE) {
      val = state_value(F.var, y, der);
    } else if (F.kind == FW_REW_STATE_INT_ERROR) {  // fixed_wing.py:1001-1012
      val = iw ? iw_value(c, pick3(iwq, F.var), steps, pick3(iwq + 3, F.var)) : T(0);
    } else if (F.kind == FW_REW_SUCCESS) {  // fixed_wing.py:1020-1026
      val = succ ? (F.var ? (T)(c.steps_max - steps) : (T)F.value) : T(0);
    } else if (F.kind == FW_REW_STEP) {  // :1028-1029
      val = (T)F.value;
    } else if (F.kind == FW_REW_GOAL) {  // :1031-1048, _get_goal_status of the step's targets (:1346-1361)
      const T vals[3] = {der[0], der[1], der[3]};
      const uint32_t gb = goal_status_bits(c, tgt, vals);
      if (F.var) {
        val = (gb >> 3) & 1u ? (T)F.value : T(0);
      } else {
#pragma unroll
        for (int k = 0; k < 3; k++)  // value / len(self.target) per bounded target within its bound
          val += ((gb >> k) & 1u) ? (T)F.value / c.n_targets : T(0);  // (len(self.target): 6 with omega)
      }
    } else if (F.var >= FW_TGT_OMEGA_P) {  // an attitude_angular target's error (no wrap): target - omega
      const int k = F.var - FW_TGT_OMEGA_P;
      val = pick3(ot, k) - pick3v(y[4], y[5], y[6], k);
    } else {  // (by selects: the factor loop is not unrolled at FW_MAX_REW 12, and tgt[F.var] went to scratch)
      const int tv_ = F.var == 0 ? FW_V_ROLL : (F.var == 1 ? FW_V_PITCH : FW_V_VA);
      val = target_error(c, F.var, pick3(tgt, F.var), state_value(tv_, y, der));
    }
    if (F.fun == FW_FUN_LINEAR) {
      val = fabs(val) / scl;
      val = val < T(0) ? T(0) : val;
      val = val > (T)F.max ? (T)F.max : val;
    } else {
      val = val * val / scl;
    }
    const T add = val * sgn((T)F.sign);
#pragma unroll
    for (int k = 0; k < 3; k++) {  // by selects: tv[F.fun] at a runtime index would live in scratch
      if (F.fun == k) {
        if (F.shaping) ts[k] += add;
        else tv[k] += add;
      }
    }
  }
  T r = T(0);
#pragma unroll
  for (int k = 0; k < 3; k++) {
    if (!c.term_present[k]) continue;
    T v;
    if (pot) {  // potential: the shaping's change since the previous step, or nothing after a reset
      const T prev = shp[k];
      const T a = isnan(prev) ? tv[k] : tv[k] + (ts[k] - prev);
      v = (k == FW_FUN_EXPONENTIAL) ? T(-1) + exp(a) : a;
      shp[k] = ts[k];
    } else {
      v = (k == FW_FUN_EXPONENTIAL) ? T(-1) + exp(tv[k] + ts[k]) : tv[k] + ts[k];
    }
    r += c.term_weight[k] * v;
  }
  return r;
}

// ---------------------------------------------------------------------------
// Streaming episode metrics.  The reference keeps the whole episode history and
// evaluates get_metric on done (fixed_wing.py:1644-1736); every metric it reports
// is a function of running sums, extrema, first-crossing indices, the goal-status
// shift registers and the last FW_M_END_WINDOW errors, which is what is kept per
// aircraft here (history["error"] / ["goal"] entry 0 = the reset state, one entry
// per successful step; one command per step).
// ---------------------------------------------------------------------------
// the deque condition of success / settling_time from a window count: `n` entries so far, `cnt` ones among
// the last success_streak_req of them
template <typename T>
__device__ __forceinline__ bool settled_n(const DevCfg<T>& c, uint32_t cnt, uint32_t n) {
  const int req = c.streak_req;
  return req > 0 && (int64_t)n >= req && (double)cnt / (double)req >= (double)c.streak_frac;
}

template <typename T>
__device__ __forceinline__ void metrics_init(const DevCfg<T>& c, const State<T>& s, int64_t i, const T* tgt,
                                             const T* vals, uint32_t lep) {
  const int slot0 = (int)(lep % (uint32_t)FW_M_END_WINDOW);  // entry 0 of the episode
  const int64_t ld = s.ld;
  const uint32_t gb = goal_status_bits(c, tgt, vals);  // (the goal history itself: goal_init)
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const T err = target_error(c, k, tgt[k], vals[k]);
    st_(s.met, MR_E0 + k, ld, i, err);
    st_(s.met, MR_ESUM + k, ld, i, err);
    st_(s.met, MR_EABS + k, ld, i, T(fabs(err)));
    st_(s.met, MR_EXT + k, ld, i, err);
    st_(s.met, MR_WSUM + k, ld, i, err);
    st_(s.met, MR_RING + 3 * slot0 + k, ld, i, err);
  }
  st_(s.met, MR_CV, ld, i, T(0));
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint32_t bit = (gb >> k) & 1u;
    st_(s.metu16, M16_GC + k, ld, i, (uint16_t)bit);
    st_(s.metu16, M16_SET + k, ld, i, (uint16_t)(settled_n(c, bit, 1u) ? 0u : M_NONE));
  }
#pragma unroll
  for (int r = 0; r < 6; r++) st_(s.metu16, M16_RISE + r, ld, i, (uint16_t)M_NONE);
}

__device__ __forceinline__ bool bits_differ(float a, float b) { return __float_as_uint(a) != __float_as_uint(b); }
__device__ __forceinline__ bool bits_differ(double a, double b) {
  return __double_as_longlong(a) != __double_as_longlong(b);
}

// The per-step metric state of one aircraft, loaded with ONE batch of independent loads
// (no load depends on another, none follows a store) and written back in one batch.
template <typename T>
struct Met {
  T row[MR_RING];          // e0 / sum / |sum| / extremum (x3), cv
  uint32_t u[M16_ROWS];    // goal counts, settling, rise (uint16 rows)
  T prev[3];               // the previous entry's errors (ring)
  T old[3];                // the ring entries the new error overwrites (leaving the end-error window)
  uint32_t b;              // the entry index the loads assumed
  // rows that change only now and then (the extrema, goal counts, settling and rise indices): a set
  // bit k marks row MD_* k as changed in this lane; store() writes such a row when some lane of the wave
  // changed it (whole-row coalesced stores), so a steady step writes the rows the traffic accounting counts
  uint32_t dirty;
  // entry e lives in ring slot (lep + e) % FW_M_END_WINDOW (lep = the episode's first `life`, the same on every
  // lane for the same e: coalesced rows)
  __device__ __forceinline__ void fetch_entry(const State<T>& s, int64_t i, uint32_t lep) {
    const int ps = (int)((lep + b - 1u) % (uint32_t)FW_M_END_WINDOW);
    const int ns = (int)((lep + b) % (uint32_t)FW_M_END_WINDOW);
#pragma unroll
    for (int k = 0; k < 3; k++) {
      prev[k] = ld_(s.met, MR_RING + 3 * ps + k, s.ld, i);
      old[k] = ld_(s.met, MR_RING + 3 * ns + k, s.ld, i);
    }
  }
  // b_guess: the new entry's index as the goal history assumes it (GoalHist)
  __device__ __forceinline__ void load(const State<T>& s, int64_t i, uint32_t lep, uint32_t b_guess) {
#pragma unroll
    for (int r = 0; r < MR_RING; r++) row[r] = ld_(s.met, r, s.ld, i);
#pragma unroll
    for (int r = 0; r < M16_ROWS; r++) u[r] = ld_(s.metu16, r, s.ld, i);
    b = b_guess;
    dirty = 0u;
    fetch_entry(s, i, lep);
  }
  __device__ __forceinline__ void store(const State<T>& s, int64_t i) const {
    // MR_E0 (the episode's initial errors) never changes after metrics_init: not written back
#pragma unroll
    for (int r = MR_ESUM; r < MR_RING; r++) {
      const bool rare = r >= MR_EXT && r < MR_EXT + 3;  // the extrema
      if (!rare || __ballot((dirty >> (MD_EXT + r - MR_EXT)) & 1u)) st_(s.met, r, s.ld, i, row[r]);
    }
#pragma unroll
    for (int r = 0; r < M16_ROWS; r++) {
      // goal counts, settling, rise indices: all rows change only now and then
      if (__ballot((dirty >> (MD_U + r - M16_GC)) & 1u)) st_(s.metu16, r, s.ld, i, (uint16_t)u[r]);
    }
  }
};

// one successful step appending history entry b: errors w.r.t. the NEW targets (fixed_wing.py:575-579), goal
// statuses `gb` w.r.t. the old ones (:534-537); gcnt = the goal history's window counts with entry b included.
// Writes the new error into the end-error ring.
template <typename T>
__device__ __forceinline__ void metrics_step(const DevCfg<T>& c, const State<T>& s, int64_t i, Met<T>& M,
                                             const T* tgt, const T* vals, uint32_t gb, const GCnt& gcnt, uint32_t b,
                                             uint32_t lep) {
  const uint32_t n0 = b;  // entries before this one
  if (b != M.b) {  // stepping on after a failed (done) step without reset: the entry's slots moved
    M.b = b;
    M.fetch_entry(s, i, lep);
  }
  const int slot = (int)((lep + b) % (uint32_t)FW_M_END_WINDOW);
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const T err = target_error(c, k, tgt[k], vals[k]);
    const T prev = M.prev[k], e0 = M.row[MR_E0 + k];
    M.row[MR_ESUM + k] += err;
    M.row[MR_EABS + k] += T(fabs(err));
    {  // overshoot's extremum (fixed_wing.py:1722-1730): the minimum where e0 > 0, else the maximum
      const T x = e0 > T(0) ? fmin(M.row[MR_EXT + k], err) : fmax(M.row[MR_EXT + k], err);
      if (bits_differ(x, M.row[MR_EXT + k])) M.dirty |= 1u << (MD_EXT + k);
      M.row[MR_EXT + k] = x;
    }
    M.row[MR_WSUM + k] += n0 >= (uint32_t)FW_M_END_WINDOW ? err - M.old[k] : err;
    st_(s.met, MR_RING + 3 * slot + k, s.ld, i, err);
    // rise_time: earliest downward crossing of |error| through each limit
    const T lims[2] = {T(fabs(c.rise_high * e0)), T(fabs(c.rise_low * e0))};
#pragma unroll
    for (int w = 0; w < 2; w++) {
      uint32_t& r = M.u[M16_RISE + 2 * k + w];
      if (r == M_NONE && fabs(prev) >= lims[w] && fabs(err) < lims[w]) {
        r = b;
        M.dirty |= 1u << (MD_U + M16_RISE - M16_GC + 2 * k + w);
      }
    }
  }
  if (c.streak_req > 0) {
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t bit = (gb >> k) & 1u;
      const bool set = settled_n(c, gcnt.get(k), n0 + 1u);
      M.u[M16_GC + k] += bit;
      M.dirty |= bit << (MD_U + k);
      if (M.u[M16_SET + k] == M_NONE && set) {
        M.u[M16_SET + k] = b;
        M.dirty |= 1u << (MD_U + M16_SET - M16_GC + k);
      }
    }
  }
}

// the record of a done episode (get_metric for every cfg metric), layout FW_M_* of fwsim.h
// n: the history entries; out: column of the SoA record [FW_NMETRIC][N] (element m at out[m * stride]).
template <typename T>
__device__ __forceinline__ void metrics_final(const DevCfg<T>& c, const Met<T>& M, uint32_t n, int n_commands, T* out,
                                              int64_t stride) {
  const T nan = T(NAN);
  const int cnt = n < (uint32_t)FW_M_END_WINDOW ? (int)n : FW_M_END_WINDOW;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const T e0 = M.row[MR_E0 + k];
    const uint32_t rs = M.u[M16_RISE + 2 * k], re = M.u[M16_RISE + 2 * k + 1];
    out[(FW_M_RISE_TIME + k) * stride] = (rs != M_NONE && re != M_NONE) ? T((double)re - (double)rs) : nan;
    const T m = M.row[MR_EXT + k];
    out[(FW_M_OVERSHOOT + k) * stride] = sgn(m) == sgn(e0) ? nan : T(fabs(m / e0));
    out[(FW_M_TOTAL_ERROR + k) * stride] = M.row[MR_EABS + k];
    out[(FW_M_AVG_ERROR + k) * stride] = fabs(e0) >= T(0.01) ? T(fabs(M.row[MR_ESUM + k] / (T)n / e0)) : nan;
    out[(FW_M_END_ERROR + k) * stride] = T(fabs(M.row[MR_WSUM + k] / (T)cnt));
  }
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint32_t st = M.u[M16_SET + k];
    out[(FW_M_SETTLING_TIME + k) * stride] = st != M_NONE ? (T)st : nan;
    out[(FW_M_SUCCESS + k) * stride] = st != M_NONE ? T(1) : T(0);
    out[(FW_M_SUCCESS_TIME_FRAC + k) * stride] = (T)((double)M.u[M16_GC + k] / (double)n);
  }
  out[FW_M_CONTROL_VARIATION * stride] = n_commands >= 2 ? M.row[MR_CV] / (T(3) * c.dt * (T)(n_commands - 1)) : nan;
}

// ---------------------------------------------------------------------------
// reset of one lane: PyFly.reset (pyfly.py:1262-1311) + FixedWingAircraft.reset
// (fixed_wing.py:414-481) incl. sample_target (:654-746).  init: FW_NINIT values
// (NaN = sample) or null; tin: 3 targets (NaN = sample) or null.
// ---------------------------------------------------------------------------
template <typename T>
struct Draws {
  uint32_t k0, k1, cid, ep, blk;
  uint32_t r[4];
  int used;
  uint32_t stream = 0u;
  __device__ __forceinline__ T next() {
    if (used == 4) {
      philox(k0, k1, cid, ep, stream, blk++, r);
      used = 0;
    }
    // r[used] by selects: where the draw count depends on the configuration (sample_target's class draws) the
    // index is not a compile-time constant, and an indexed register array is placed in scratch (round 6: 60 B
    // and ~15 scratch instructions per wave on every step of the fp32 instances)
    const uint32_t v = used == 0 ? r[0] : (used == 1 ? r[1] : (used == 2 ? r[2] : r[3]));
    used++;
    return u01<T>(v);
  }
  __device__ __forceinline__ T uniform(T lo, T hi) { return lo + (hi - lo) * next(); }  // numpy uniform
};

// The env's own np_random (FixedWingAircraft.np_random, fixed_wing.py:324-332): the caller's tape
// (fw_set_env_draws: aircraft i's column, from its cursor `cur`, State::dcur) or the Philox source D.  Free
// functions on the caller's locals: an object holding references to them placed the Draws (48 B) in scratch.
template <typename T>
__device__ __forceinline__ T env_draw(const State<T>& s, int64_t i, Draws<T>& D, uint32_t& cur) {
  if (!s.tape) return D.next();
  const T u = cur < (uint32_t)s.tape_len ? s.tape[(int64_t)cur * s.n + i] : T(NAN);
  cur++;
  return u;
}
template <typename T>
__device__ __forceinline__ T env_uniform(const State<T>& s, int64_t i, Draws<T>& D, uint32_t& cur, T lo, T hi) {
  return lo + (hi - lo) * env_draw(s, i, D, cur);  // numpy uniform
}

// sample_target (fixed_wing.py:654-746) of one aircraft: per target (roll, pitch, Va) the initial value
// U(low, high) narrowed to the current value -+ delta, then the class's draws -- linear: the slope
// U(slope_low, slope_high), negated when U() < 0.5, in radians where configured (:698-706); sinusoidal: the
// amplitude (radians where configured), the period, the phase U(0, 2 pi) / (2 pi / period) and the bias that
// puts the sinusoid through the initial value at steps_count `steps` (:708-722) -- into State::tpr.  tin:
// explicit targets (NaN = sample); such a target is drawn all the same and then flies as "constant" for the
// episode (reset, :436-448): slope 0, or amplitude 0 and bias = the given value.
template <typename T>
__device__ __forceinline__ void sample_target(const DevCfg<T>& c, const State<T>& s, int64_t i, Draws<T>& D, uint32_t& cur,
                                              const T* vals, int steps, const T* tin, int64_t tin_ld, T* tgt) {
  const T two_pi = T(2.0 * PI_D);
  T drawn[3];
#pragma unroll
  for (int k = 0; k < 3; k++) {
    T lo = c.target_low[k], hi = c.target_high[k];
    if (c.has_delta[k]) {
      lo = fmax(lo, vals[k] - c.target_delta[k]);
      hi = fmax(fmin(hi, vals[k] + c.target_delta[k]), lo);
    }
    const T init = env_uniform(s, i, D, cur, lo, hi);
    const T given = tin ? tin[k * tin_ld + i] : T(NAN);
    const bool fixed = !isnan(given);
    if (c.tprops && s.tpr) {
      T* tp = s.tpr + (int64_t)(4 * k) * s.ld + i;
      if (c.target_class[k] == FW_TGT_LINEAR) {
        T slope = env_uniform(s, i, D, cur, c.tgt_slo[k], c.tgt_shi[k]);
        if (env_draw(s, i, D, cur) < T(0.5)) slope = -slope;
        tp[0] = fixed ? T(0) : slope * c.tgt_rad[k];
      } else if (c.target_class[k] == FW_TGT_SINUSOIDAL) {
        const T amp = env_uniform(s, i, D, cur, c.tgt_alo[k], c.tgt_ahi[k]) * c.tgt_rad[k];
        const T per = env_uniform(s, i, D, cur, c.tgt_plo[k], c.tgt_phi[k]);
        const T ph = env_uniform(s, i, D, cur, T(0), two_pi) / (two_pi / per);
        tp[0] = fixed ? T(0) : amp;
        tp[s.ld] = per;
        tp[2 * s.ld] = ph;
        tp[3 * s.ld] = fixed ? given : init - amp * sin(two_pi / per * ((T)steps + ph));
      }
    }
    tgt[k] = fixed ? given : init;
    drawn[k] = init;
  }
  if (c.ang && s.tpr) {
    // the omega targets (:662-675, 741-746): 0, then all three rates from those zeros and the DRAWN roll / pitch
    // targets (an explicit target replaces its draw only afterwards, in reset, :444-448)
    const T z[3] = {T(0), T(0), T(0)};
#pragma unroll
    for (int k = 0; k < 3; k++) s.tpr[(int64_t)(12 + k) * s.ld + i] = att_ang_rate(c, k, drawn, z, vals[0], vals[1]);
  }
}

template <typename T>
__device__ __forceinline__ void reset_lane(const DevCfg<T>& c, const State<T>& s, int64_t i, const T* init, const T* tin,
                                           T* y, T* der, T* wind, T* tgt) {
  const int64_t ld = s.n;  // injected init / target arrays are dense [rows][N]
  const uint32_t episode = s.episode[i] + 1u;
  s.episode[i] = episode;
  Draws<T> D{s.key0, s.key1, s.env_offset + (uint32_t)i, episode, 0u, {0, 0, 0, 0}, 4};
  int term = 0;
  T st[12];
#pragma unroll
  for (int k = 0; k < 12; k++) {  // roll pitch yaw p q r n e d u v w
    const T given = init ? init[k * ld + i] : T(NAN);
    const int var = k;  // fw_var order matches for these 12
    const T smp = D.uniform(c.init_min[var], c.init_max[var]);
    st[k] = isnan(given) ? smp : cond(c, var, given, term);  // Variable.reset (pyfly.py:83-104)
  }
#pragma unroll
  for (int j = 0; j < 3; j++) {  // ControlVariable.reset (pyfly.py:340-366)
    const T gv = init ? init[(FW_I_ACT0 + 2 * j) * ld + i] : T(NAN);
    const T gd = init ? init[(FW_I_ACT0 + 2 * j + 1) * ld + i] : T(NAN);
    const T smp = D.uniform(c.init_min[FW_V_ACT0 + j], c.init_max[FW_V_ACT0 + j]);
    if (isnan(gv)) {
      y[13 + j] = smp;
      y[16 + j] = T(0);
    } else {
      y[13 + j] = cond(c, FW_V_ACT0 + j, gv, term);
      const T d = isnan(gd) ? T(0) : gd;
      y[16 + j] = (c.dotmask & (1u << j)) ? clipv(d, -c.dot_max[j], c.dot_max[j]) : d;
    }
  }
  // Wind.reset (pyfly.py:799-830)
  {
    T wn, we, wdn;
    if (c.wind_random) {
      const T m = D.uniform(c.wind_mag_min, c.wind_mag_max);
      wn = D.uniform(-m, m);
      const T we_max = sqrt(m * m - wn * wn);
      we = D.uniform(-we_max, we_max);
      wdn = sqrt(fmax(m * m - wn * wn - we * we, T(0)));
    } else {
      wn = D.uniform(c.wind_init_min[0], c.wind_init_max[0]);
      we = D.uniform(c.wind_init_min[1], c.wind_init_max[1]);
      wdn = D.uniform(c.wind_init_min[2], c.wind_init_max[2]);
    }
    const T gn = init ? init[FW_I_WIND_N * ld + i] : T(NAN);
    const T ge = init ? init[FW_I_WIND_E * ld + i] : T(NAN);
    const T gd = init ? init[FW_I_WIND_D * ld + i] : T(NAN);
    const bool given = !isnan(gn) && !isnan(ge) && !isnan(gd);
    wind[0] = given ? gn : wn;
    wind[1] = given ? ge : we;
    wind[2] = given ? gd : wdn;
  }
#pragma unroll
  for (int k = 0; k < 9; k++) y[4 + k] = st[3 + k];
  euler_to_quat(st[0], st[1], st[2], y);
  der[0] = st[0];
  der[1] = st[1];
  der[2] = st[2];
  reset_derived(c, y, wind, der);
  if (c.rand_params && s.prm) {
    // sample_simulator_parameters (fixed_wing.py:748-813; FixedWingAircraft.reset calls it after
    // PyFly.reset and before sample_target): Philox stream 5, one block per entry
#pragma unroll 1
    for (int k = 0; k < FW_NPARAM; k++) s.prm[k * s.ld + i] = c.pdef[k];
#pragma unroll 1
    for (int r = 0; r < c.n_rand; r++) {
      uint32_t rnd[4];
      philox(s.key0, s.key1, s.env_offset + (uint32_t)i, episode, 5u, (uint32_t)r, rnd);
      const T orig = c.rp[r].orig, var = c.rp[r].var;
      T v;
      if (c.rp[r].dist == FW_DIST_UNIFORM) {
        v = (orig - var) + (T(2) * var) * u01<T>(rnd[0]);  // np_random.uniform(orig - var, orig + var)
      } else {
        T z[4];
        normal4<T>(rnd, z);
        v = orig + var * z[0];  // np_random.normal(loc=orig, scale=var)
        if (c.rp[r].has_clip)  // np.clip(v, orig - clip, orig + clip) = min(max(v, lo), hi)
          v = fmin(fmax(v, orig - c.rp[r].clip), orig + c.rp[r].clip);
      }
      s.prm[c.rp[r].param * s.ld + i] = v;
    }
  }
  if (c.has_env) {
    // sample_target (fixed_wing.py:654-746): Philox stream 0 after the state draws, or the env-draw tape
    const T vals[3] = {der[0], der[1], der[3]};
    uint32_t cur = s.tape ? s.dcur[i] : 0u;
    // sample_simulator_parameters' draws for simulator attributes PyFly never reads come first (:802-813);
    // they change nothing, so a tape replay only steps over them
    if (s.tape) cur += (uint32_t)c.tape_skip;
    sample_target(c, s, i, D, cur, vals, 0, tin, ld, tgt);
    if (s.tape && s.rsc)  // reward.randomize_scaling from the tape, after the targets (fixed_wing.py:473-479)
      for (int r = 0; r < c.n_rew; r++)
        if (c.rew[r].randomize)
          st_(s.rsc, r, s.ld, i, env_uniform(s, i, D, cur, (T)c.rew[r].scaling, (T)c.rew[r].scaling_hi));
    if (s.tape) s.dcur[i] = cur;
  }
}

// sample_target (fixed_wing.py:654-746) during an episode (target.resample_every, on_success "new"): as at the
// reset, from the env-draw tape or Philox stream 6 keyed by (env, episode, 16 x env step)
template <typename T>
__device__ __forceinline__ void resample_targets(const DevCfg<T>& c, const State<T>& s, int64_t i, int steps,
                                                 const T* vals, T* tgt) {
  Draws<T> D{s.key0, s.key1, s.env_offset + (uint32_t)i, s.episode[i], (uint32_t)steps << 4, {0, 0, 0, 0}, 4, 6u};
  uint32_t cur = s.tape ? s.dcur[i] : 0u;
  sample_target(c, s, i, D, cur, vals, steps, (const T*)nullptr, 0, tgt);
  if (s.tape) s.dcur[i] = cur;
}

template <typename T>
__device__ __forceinline__ void load_row(const T* p, int rows, int64_t ld, int64_t i, T* dst) {
  for (int r = 0; r < rows; r++) dst[r] = p[r * ld + i];
}

// the goal history of a fresh episode: entry 0 (the reset state) at lifetime position lep.  The other nibbles of
// its word are entries of an earlier episode or ones this episode writes before reading: a plain store, no
// read-modify-write.
template <typename T>
__device__ __forceinline__ void goal_init(const DevCfg<T>& c, const State<T>& s, int64_t i, const T* tgt,
                                          const T* der, uint32_t lep) {
  const int64_t ld = s.ld;
  if (c.streak_req > 0) {
    const T vals[3] = {der[0], der[1], der[3]};
    const uint32_t gb = goal_status_bits(c, tgt, vals);
    st_(s.goal, gring_row(lep, c.gring_mask), ld, i, gring_set(0u, lep, gb));
    if (c.gcnt_wide) {
      st_(s.goal, GB_CNT, ld, i, (gb & 1u) | ((gb >> 1) & 1u) << 16);
      st_(s.goal, c.gcnt2_row, ld, i, ((gb >> 2) & 1u) | ((gb >> 3) & 1u) << 16);
    } else {
      st_(s.goal, GB_CNT, ld, i, (gb & 1u) | ((gb >> 1) & 1u) << 8 | ((gb >> 2) & 1u) << 16 | ((gb >> 3) & 1u) << 24);
    }
  }
  st_(s.goal, GB_N, ld, i, 1u);
}

// lep: the fresh episode's first `life`
template <typename T>
__device__ __forceinline__ void store_env_fresh(const DevCfg<T>& c, const State<T>& s, int64_t i, const T* y, const T* der,
                                                const T* wind, const T* tgt, uint32_t lep) {
  const int64_t ld = s.ld;
#pragma unroll
  for (int k = 0; k < NY; k++) st_(s.y, k, ld, i, y[k]);
#pragma unroll
  for (int k = 0; k < 8; k++) st_(s.der, k, ld, i, der[k]);
#pragma unroll
  for (int k = 0; k < 3; k++) st_(s.wind, k, ld, i, wind[k]);
  if (s.dry)  // Dryden.reset: lsim restarts from X0 = None (dryden.py:41-48, 190-191)
#pragma unroll
    for (int r = 0; r < 12; r++) st_(s.dry, r, ld, i, T(0));
  if (c.has_env) {
#pragma unroll
    for (int k = 0; k < 3; k++) st_(s.target, k, ld, i, tgt[k]);
    goal_init(c, s, i, tgt, der, lep);
    st_(s.ep_ret, 0, ld, i, T(0));
    // (State::gflag, goal_achieved, is not touched: the reference never clears it, fixed_wing.py:81)
    if (s.shp)  // self.prev_shaping[*] = None (fixed_wing.py:469-470)
#pragma unroll
      for (int k = 0; k < 3; k++) st_(s.shp, k, ld, i, T(NAN));
    if (s.rsc && !s.tape)  // reward.randomize_scaling (fixed_wing.py:473-479): Philox stream 7, one block per factor
      for (int r = 0; r < c.n_rew; r++)
        if (c.rew[r].randomize) {
          uint32_t rnd[4];
          philox(s.key0, s.key1, s.env_offset + (uint32_t)i, s.episode[i], 7u, (uint32_t)r, rnd);
          const T lo = (T)c.rew[r].scaling, hi = (T)c.rew[r].scaling_hi;
          st_(s.rsc, r, ld, i, lo + (hi - lo) * u01<T>(rnd[0]));  // np_random.uniform(low, high)
        }
  }
  s.steps[i] = 0u;
}

// ===========================================================================
// kernels
// ===========================================================================
template <typename T>
__global__ __launch_bounds__(BLOCK) void k_reset(const DevCfg<T>* __restrict__ cfgp, State<T> s,
                                                 const uint8_t* __restrict__ mask, const T* __restrict__ init,
                                                 const T* __restrict__ tin, T* __restrict__ obs) {
  const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
  if (i >= s.n) return;
  if (mask && !mask[i]) return;
  const DevCfg<T>& c = *cfgp;
  T y[NY], der[8], wind[3], tgt[3] = {T(0), T(0), T(0)};
  // integrator observations at the reset read the previous episode's history (None before the first reset:
  // the current error x W), fixed_wing.py:452-459, 1163-1167
  T rv[3] = {T(0), T(0), T(0)};
  const bool iw_first = s.iws ? ld_(s.goal, GB_N, s.ld, i) == 0u : true;
  if (s.iws && !iw_first)
#pragma unroll
    for (int k = 0; k < 3; k++)
      rv[k] = iw_value(c, ld_(s.iws, IW_QP + k, s.ld, i), -1, ld_(s.iws, IW_E0 + k, s.ld, i));
  reset_lane(c, s, i, init, tin, y, der, wind, tgt);
  store_env_fresh(c, s, i, y, der, wind, tgt, s.life[i]);
  if (s.iws) {
    iw_init(c, s, i, tgt, der, s.life[i]);
    if (iw_first) {
      const T vals[3] = {der[0], der[1], der[3]};
#pragma unroll
      for (int k = 0; k < 3; k++) rv[k] = target_error(c, k, tgt[k], vals[k]) * T(c.iwin);
    }
  }
  if (c.has_env && c.metrics) {
    const T vr[3] = {der[0], der[1], der[3]};
    metrics_init(c, s, i, tgt, vr, s.life[i]);
  }
  if (c.has_env && (obs || c.obs_hist)) {  // the history needs the reset row even without an output
    T seq[RING + 1][3];
#pragma unroll
    for (int j = 0; j <= RING; j++)
#pragma unroll
      for (int a = 0; a < 3; a++) seq[j][a] = T(0);
    observe_env(c, s, i, s.episode[i], OBS_RESET, y, der, tgt, 0, seq, seq,
                obs ? obs + i * (int64_t)c.n_obs * c.obs_len : nullptr, s.life[i]);
    if (c.ang && obs) {
      T ot[3];
      ang_load(s, i, ot);
      ang_obs(c, ot, y, obs + i * (int64_t)c.n_obs * c.obs_len);
    }
    if (s.iws) {
      iw_obs_all_rows(c, rv, obs ? obs + i * (int64_t)c.n_obs * c.obs_len : nullptr);
      iw_hist_init(c, s, i, tgt, der);
    }
  }
}

template <typename T>
__global__ __launch_bounds__(BLOCK) void k_observe(const DevCfg<T>* __restrict__ cfgp, State<T> s, T* __restrict__ obs) {
  const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
  if (i >= s.n) return;
  const DevCfg<T>& c = *cfgp;
  const int64_t ld = s.ld;
  T y[NY], der[8], tgt[3];
  load_row(s.y, NY, ld, i, y);
  load_row(s.der, 8, ld, i, der);
  load_row(s.target, 3, ld, i, tgt);
  const int steps = (int)(s.steps[i] & 0xFFFFu);
  const uint32_t life = s.life[i];
  T seqA[RING + 1][3], seqC[RING + 1][3];
#pragma unroll
  for (int j = 0; j <= RING; j++)
#pragma unroll
    for (int a = 0; a < 3; a++) seqA[j][a] = seqC[j][a] = T(0);
  // newest-first from the rings
#pragma unroll
  for (int j = 0; j <= RING; j++) {
    if (j < c.act_window && steps - 1 - j >= 0) {
      const int slot = (int)((life - 1u - (uint32_t)j) % (uint32_t)c.act_window);
#pragma unroll
      for (int a = 0; a < 3; a++) seqA[j][a] = s.act_ring[((int64_t)slot * 3 + a) * ld + i];
    }
    if (j < c.cmd_window && steps - 1 - j >= 0) {
      const int slot = (int)((life - 1u - (uint32_t)j) % (uint32_t)c.cmd_window);
#pragma unroll
      for (int a = 0; a < 3; a++) seqC[j][a] = s.cmd_ring[((int64_t)slot * 3 + a) * ld + i];
    }
  }
  observe_env(c, s, i, s.episode[i], OBS_PEEK, y, der, tgt, steps, seqA, seqC, obs + i * (int64_t)c.n_obs * c.obs_len,
              life - (uint32_t)steps);
  if (c.ang) {
    T ot[3];
    ang_load(s, i, ot);
    ang_obs(c, ot, y, obs + i * (int64_t)c.n_obs * c.obs_len);
  }
  if (s.iws) {  // get_observation with the current history: the sum before the newest entry + padding
    T v[3];
#pragma unroll
    for (int k = 0; k < 3; k++) v[k] = iw_value(c, ld_(s.iws, IW_QP + k, ld, i), steps - 1, ld_(s.iws, IW_E0 + k, ld, i));
    if (steps == 0) iw_obs_all_rows(c, v, obs + i * (int64_t)c.n_obs * c.obs_len);
    else iw_obs(c, v, obs + i * (int64_t)c.n_obs * c.obs_len);
  }
}

// Re-reads the pre-step ODE state after the RK loop (sim_step_masked's reload hook): the
// barrier keeps the compiler from reusing the prologue's loads, which would pin 19
// values in registers for the whole integration.
template <typename T>
struct ReloadRow {
  const T* y;
  int64_t ld, i;
  __device__ __forceinline__ void operator()(T* out) const {
    asm volatile("" ::: "memory");
#pragma unroll
    for (int r = 0; r < NY; r++) out[r] = y[r * ld + i];
  }
};

template <typename T, typename C, bool RP = false, int Q = 1>
__global__ __launch_bounds__(BLOCK, FW_WAVES(Q)) void k_sim_step(const DevCfg<T>* __restrict__ cfgp, State<T> s,
                                                    const T* __restrict__ cmd_in, T* __restrict__ cmd_out,
                                                    uint8_t* __restrict__ success, int32_t* __restrict__ term_out,
                                                    int32_t* __restrict__ stats) {
  const int64_t tid = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
  const int64_t i = tid / Q;  // Q = 4: lanes 4i..4i+3 integrate aircraft i (fw_quad.hpp); Q = 2: lanes 2i, 2i+1
  const int qr = (int)(tid % Q);
  if (i >= s.n) return;
  const C& c = *reinterpret_cast<const C*>(cfgp);  // structural specialisation view (fw_device.hpp SpecCfg)
  const int64_t ld = s.ld;
  T y[NY], der[8], wind[3], cmd[3];
  load_row(s.y, NY, ld, i, y);
  der[6] = ld_(s.der, 6, ld, i);
  der[7] = ld_(s.der, 7, ld, i);
  load_row(s.wind, 3, ld, i, wind);
#pragma unroll
  for (int a = 0; a < 3; a++) cmd[a] = cmd_in[i * 3 + a];
  const uint32_t sw = s.steps[i];
  const int k = (int)(sw & 0xFFFFu);
  T tl[3], ta[3];
  turbulence_at(c, s, i, s.episode[i], k, tl, ta, qr == 0);
  int nfev = 0, nacc = 0;
  uint32_t dmask = 0;
  __shared__ V2<T> lds[(Q == 1 ? lds_slots<T>() * NP : Q == 2 ? pr::LDS_PAIRS : 1) * BLOCK];  // y, f (+ error sum)
  constexpr bool HO = Q == 1 && !RP && FW_TAIL_QUAD > 0;
  static_assert(!HO || BLOCK == 64, "the tail handoff works per one-wave block");
  __shared__ qd::HoSlot<T> ho[HO ? BLOCK : 1];
  int term;
  if constexpr (RP) {
    const AeroP<T> ap = aero_from<T>(c, [&](int k) { return s.prm[k * ld + i]; });
    term = sim_step_masked<Q>(c, ap, y, der, cmd, wind, tl, ta, nfev, nacc, dmask, lds + threadIdx.x,
                              lds + NP * BLOCK + threadIdx.x, BLOCK, ReloadRow<T>{s.y, ld, i}, qr);
  } else {
    term = sim_step_masked<Q, HO>(c, c, y, der, cmd, wind, tl, ta, nfev, nacc, dmask, lds + threadIdx.x,
                                  lds + NP * BLOCK + threadIdx.x, BLOCK, ReloadRow<T>{s.y, ld, i}, qr, ho);
  }
  if (qr != 0) return;  // the quad's other lanes hold the same result
  if (term) {  // uncommitted derived values keep their previous (history[-1]) value
#pragma unroll
    for (int r = 0; r < 6; r++)
      if (!(dmask & (1u << r))) der[r] = ld_(s.der, r, ld, i);
  }
#pragma unroll
  for (int r = 0; r < NY; r++) st_(s.y, r, ld, i, y[r]);
#pragma unroll
  for (int r = 0; r < 8; r++) st_(s.der, r, ld, i, der[r]);
#pragma unroll
  for (int a = 0; a < 3; a++) st_(s.cmd, a, ld, i, cmd[a]);
  s.steps[i] = (sw & 0xFFFF0000u) | (uint32_t)((k + 1) & 0xFFFF);  // cur_sim_step += 1 (pyfly.py:1418)
  s.life[i] += 1u;
  if (cmd_out)
#pragma unroll
    for (int a = 0; a < 3; a++) cmd_out[i * 3 + a] = cmd[a];
  if (success) success[i] = term == 0;
  if (term_out) term_out[i] = term;
  if (stats) stats[i] = pack_stats(nfev, nacc, dmask);
}

// FixedWingAircraft.step of aircraft i (the body of k_env_step and of one k_env_rollout step).
// lds: this block's RK45 slots (lds_slots<T>() * NP * BLOCK pairs).
// Q = 4: called on the four lanes of aircraft i's quad (qr = 0..3); they integrate together, then
// lane 0 alone runs the epilogue.  PREF: the epilogue's loads (rings, goal register, metric state) are
// issued before the integration, so their latency hides under it instead of following it; that keeps
// ~90 more values live across the RK loop, which the one-wave quad instances have room for.
// YF: the one-lane integrator keeps the accepted y / f in registers (FW_YF_REGS) -- false: in LDS (A/B only; the
// bits differ, profiles/r06_openloop_yf_ab.log)
template <typename T, typename C, bool RP = false, int Q = 1, bool PREF = false, bool YF = true>
__device__ __forceinline__ void env_step_lane(const C& c, const State<T>& s, const int64_t i, V2<T>* lds,
                                              const T* __restrict__ actions, T* __restrict__ obs_out,
                                              T* __restrict__ rew_out, uint8_t* __restrict__ done_out,
                                              int32_t* __restrict__ term_out, T* __restrict__ tobs_out,
                                              T* __restrict__ episode_out, int32_t* __restrict__ stats,
                                              int auto_reset, int qr = 0, void* ho = nullptr) {
  const int64_t ld = s.ld;
  constexpr bool HO = Q == 1 && !RP && FW_TAIL_QUAD > 0;  // ho: the block's qd::HoSlot<T>[64] (tail handoff)
  FW_TSTAMP(0);

  T y[NY], der[8], wind[3], tgt[3], a[3];
  load_row(s.y, NY, ld, i, y);
  der[6] = ld_(s.der, 6, ld, i);
  der[7] = ld_(s.der, 7, ld, i);
  load_row(s.wind, 3, ld, i, wind);
  load_row(s.target, 3, ld, i, tgt);
#pragma unroll
  for (int q = 0; q < 3; q++) a[q] = actions[i * 3 + q];
  const uint32_t sw = s.steps[i];
  const int steps0 = (int)(sw & 0xFFFFu);
  const int steps_tgt0 = (int)(sw >> 16);
  // the episode counter keys the Philox streams of turbulence and observation noise (the reset path reads it
  // itself): without either it is not loaded
  const uint32_t episode = (c.turbulence || c.obs_noise) ? s.episode[i] : 0u;
  // ring slots by `life` (the same on every lane: coalesced rows however the episodes are staggered; slots by
  // the episode step scattered a wave's ring accesses over up to 64 rows once resets desynchronised the
  // episodes, +30 % HBM traffic per launch at the bench's steady state, profiles/r04_traffic_split.json)
  uint32_t life0 = 0u, lep = 0u;  // loaded with the epilogue's inputs: lep = the episode's first `life` (fixed_wing.py:491-506) ----
  T cmd[3];
#pragma unroll
  for (int q = 0; q < 3; q++) cmd[q] = c.scale_actions ? scale_fwd(c, q, clipv(a[q], c.scale_low, c.scale_high)) : a[q];

  const int steps = steps0 + 1;
  int steps_tgt = steps_tgt0 + 1;
  // ---- epilogue inputs: action / command histories (newest first), goal register, metric state ----
  T seqA[RING + 1][3], seqC[RING + 1][3];
  // goal history (GB_*): entry count, counts, the ring words of the new entry and of the entry leaving the window
  uint32_t gn = 1u, gw_new = 0u, gw_old = 0u;
  GCnt gcnt{0u, 0u, c.gcnt_wide != 0};
  const bool goal_on = c.streak_req > 0;
  const uint32_t req = goal_on ? (uint32_t)c.streak_req : 0u;
  // every step but a terminal failure appends a history entry, so the new entry's index is steps0 + 1 unless the
  // caller stepped on after a failure without reset: the loads below assume it (no load waits on GB_N)
  const uint32_t b_guess = (uint32_t)steps0 + 1u;
  Met<T> M;
  T prev_cmd[3];
  T ep_ret0;
  T shp[3] = {T(0), T(0), T(0)};  // reward.form "potential": the previous step's shaping (State::shp)
  // integration window (State::iws): the window sums before this step, entry 0, the entry leaving the window
  T iwq[6] = {T(0), T(0), T(0), T(0), T(0), T(0)}, iqp[3] = {T(0), T(0), T(0)}, iold[3] = {T(0), T(0), T(0)};
  auto load_epilogue = [&]() {
    life0 = s.life[i];
    lep = life0 - (uint32_t)steps0;
#pragma unroll
    for (int j = 1; j <= RING; j++) {
#pragma unroll
      for (int q = 0; q < 3; q++) seqA[j][q] = seqC[j][q] = T(0);
      // previous action j = action number steps-j (1-based) -> slot (life0 - j) % window
      if (j <= c.act_need && steps - j >= 1) {
        const int slot = (int)((life0 - (uint32_t)j) % (uint32_t)c.act_window);
#pragma unroll
        for (int q = 0; q < 3; q++) seqA[j][q] = s.act_ring[((int64_t)slot * 3 + q) * ld + i];
      }
      if (j <= c.cmd_need && steps - j >= 1) {
        const int slot = (int)((life0 - (uint32_t)j) % (uint32_t)c.cmd_window);
#pragma unroll
        for (int q = 0; q < 3; q++) seqC[j][q] = s.cmd_ring[((int64_t)slot * 3 + q) * ld + i];
      }
    }
    if (goal_on || c.metrics || s.iws) gn = ld_(s.goal, GB_N, ld, i);
    if (s.iws) {
      const int os = (int)((lep + b_guess) % (uint32_t)c.iwin);  // entry b - W shares the new entry's slot
#pragma unroll
      for (int k = 0; k < 3; k++) {
        iwq[k] = ld_(s.iws, IW_Q + k, ld, i);
        iwq[3 + k] = ld_(s.iws, IW_E0 + k, ld, i);
        iqp[k] = ld_(s.iws, IW_QP + k, ld, i);
        iold[k] = ld_(s.iwr, os * 3 + k, ld, i);
      }
    }
    if (goal_on) {
      gw_new = ld_(s.goal, gring_row(lep + b_guess, c.gring_mask), ld, i);
      gw_old = ld_(s.goal, gring_row(lep + b_guess - req, c.gring_mask), ld, i);
      gcnt.w0 = ld_(s.goal, GB_CNT, ld, i);
      if (c.gcnt_wide) gcnt.w1 = ld_(s.goal, c.gcnt2_row, ld, i);
    }
    if (c.metrics) {
      M.load(s, i, lep, b_guess);
      // the previous constrained command: recomputed from the previous raw action where the action ring
      // already delivered it (scale_fwd(clip(.)) and constrain_commands are pure functions of the action),
      // else the command row
      if (c.act_need >= 1) {
#pragma unroll
        for (int q = 0; q < 3; q++)
          prev_cmd[q] =
              c.scale_actions ? scale_fwd(c, q, clipv(seqA[1][q], c.scale_low, c.scale_high)) : seqA[1][q];
        T sp_unused[3];
        (void)constrain_commands(c, prev_cmd, sp_unused);
      } else {
        load_row(s.cmd, 3, ld, i, prev_cmd);
      }
    }
    ep_ret0 = ld_(s.ep_ret, 0, ld, i);
    if (s.shp)
#pragma unroll
      for (int k = 0; k < 3; k++) shp[k] = ld_(s.shp, k, ld, i);
  };
  if constexpr (PREF) load_epilogue();

  // ---- PyFly.step ----
  T tl[3], ta[3];
  turbulence_at(c, s, i, episode, steps0, tl, ta, qr == 0);
  FW_TSTAMP(1);
  int nfev = 0, nacc = 0;
  uint32_t dmask = 0;
  int sterm;
  if constexpr (RP) {  // this aircraft's own parameters (simulator parameter randomisation)
    const AeroP<T> ap = aero_from<T>(c, [&](int k) { return s.prm[k * ld + i]; });
    sterm = sim_step_masked<Q, false, YF>(c, ap, y, der, cmd, wind, tl, ta, nfev, nacc, dmask, lds + threadIdx.x,
                                          lds + NP * BLOCK + threadIdx.x, BLOCK, ReloadRow<T>{s.y, ld, i}, qr);
  } else {
    sterm = sim_step_masked<Q, HO, YF>(c, c, y, der, cmd, wind, tl, ta, nfev, nacc, dmask, lds + threadIdx.x,
                                       lds + NP * BLOCK + threadIdx.x, BLOCK, ReloadRow<T>{s.y, ld, i}, qr, ho);
  }
  if (Q > 1 && qr != 0) return;
  if constexpr (!PREF) {
    // keep the epilogue's loads (action ring, goal bits, ...) below the integrator:
    // hoisted above it they would sit in VGPRs for the whole RK loop.  Actions and
    // targets are re-read for the same reason.
    asm volatile("" ::: "memory");
    load_row(s.target, 3, ld, i, tgt);
#pragma unroll
    for (int q = 0; q < 3; q++) a[q] = actions[i * 3 + q];
  }
  FW_TSTAMP(2);
  if (sterm) {
#pragma unroll
    for (int r = 0; r < 6; r++)
      if (!(dmask & (1u << r))) der[r] = ld_(s.der, r, ld, i);
  }
  if constexpr (!PREF) load_epilogue();
#pragma unroll
  for (int q = 0; q < 3; q++) {
    seqA[0][q] = a[q];
    seqC[0][q] = cmd[q];
  }
  {
    const int slot = (int)(life0 % (uint32_t)c.act_window);
#pragma unroll
    for (int q = 0; q < 3; q++) s.act_ring[((int64_t)slot * 3 + q) * ld + i] = a[q];
    if (c.cmd_window) {
      const int cs = (int)(life0 % (uint32_t)c.cmd_window);
#pragma unroll
      for (int q = 0; q < 3; q++) s.cmd_ring[((int64_t)cs * 3 + q) * ld + i] = cmd[q];
    }
  }

  // ---- epilogue (fixed_wing.py:511-628) ----
  bool done = false;
  int term = FW_TERM_NONE;
  if (steps >= c.steps_max && c.steps_max > 0) {
    done = true;
    term = FW_TERM_STEPS;
  }
  T reward;
  // command history (control_variation): one constrained command per step, success or not
  if (c.metrics) {
    if (steps0 >= 1)
#pragma unroll
      for (int q = 0; q < 3; q++) M.row[MR_CV] += fabs(cmd[q] - prev_cmd[q]);
  }
#pragma unroll
  for (int q = 0; q < 3; q++) st_(s.cmd, q, ld, i, cmd[q]);
  const T tgt_in[3] = {tgt[0], tgt[1], tgt[2]};  // a target row is stored only where some lane changed it
  T ot[3] = {T(0), T(0), T(0)};  // attitude_angular targets omega_p / q / r (c.ang; a constant 0 in the specialisations)
  if (c.ang)
#pragma unroll
    for (int k = 0; k < 3; k++) ot[k] = s.tpr[(int64_t)(12 + k) * ld + i];
  if (sterm == 0) {
    const T vals[3] = {der[0], der[1], der[3]};
    uint32_t gb = 0;
    bool success = false, succ_first = false, resample = false;
    const uint32_t b = gn;  // the new history entry
    if (goal_on) {
      // history["goal"][*].append (fixed_wing.py:536-538): the entry's nibble, and per status the window count
      // + the new status - the one leaving the req-deep window (the deque of get_metric, :1682-1700)
      gb = goal_status_bits(c, tgt, vals);
      const uint32_t pn = lep + b, po = pn - req;
      if (b != b_guess) {
        gw_new = ld_(s.goal, gring_row(pn, c.gring_mask), ld, i);
        gw_old = ld_(s.goal, gring_row(po, c.gring_mask), ld, i);
      }
      const uint32_t leave = b >= req ? gring_get(gw_old, po) : 0u;
#pragma unroll
      for (int k = 0; k < 4; k++) gcnt.set(k, gcnt.get(k) - ((leave >> k) & 1u) + ((gb >> k) & 1u));
      st_(s.goal, gring_row(pn, c.gring_mask), ld, i, gring_set(gw_new, pn, gb));
      st_(s.goal, GB_CNT, ld, i, gcnt.w0);
      if (c.gcnt_wide) st_(s.goal, c.gcnt2_row, ld, i, gcnt.w1);
      // np.mean(history["goal"]["all"][-streak_req:]) >= success_streak_fraction (:540-547)
      if (steps_tgt >= c.streak_req && (double)gcnt.get(3) / (double)c.streak_req >= (double)c.streak_frac) {
        success = true;
        if (c.on_success == 1) {
          done = true;
          term = FW_TERM_SUCCESS;
        } else if (c.on_success == 2) {
          resample = true;  // on_success "new" (:551-552)
        }
      }
    }
    if (success && s.gflag) {  // goal_achieved_on_step = not self.goal_achieved; self.goal_achieved = True (:546-547)
      const uint32_t f = s.gflag[i];
      succ_first = !(f & 1u);
      if (succ_first) s.gflag[i] = f | 1u;
    }
    if (goal_on || c.metrics || s.iws) st_(s.goal, GB_N, ld, i, b + 1u);
    if (s.shp || s.rsc || s.iws) {
      reward = reward_of(c, y, der, tgt, steps, seqA, shp, s.shp != nullptr, s.rsc ? s.rsc + i : nullptr, ld,
                         iwq, s.iws != nullptr, succ_first, ot);
      if (s.shp)
#pragma unroll
        for (int k = 0; k < 3; k++) st_(s.shp, k, ld, i, shp[k]);
    } else {
      reward = reward_of(c, y, der, tgt, steps, seqA, shp, false, (const T*)nullptr, 0, iwq, false, succ_first, ot);
    }
    if (resample || (c.resample_every > 0 && steps_tgt >= c.resample_every)) {
      // on_success "new" or target.resample_every (fixed_wing.py:566-574): sample_target (:654-746) from the
      // state after the step, then _get_next_target with the target step count restarted
      resample_targets(c, s, i, steps, vals, tgt);
      steps_tgt = 0;
      if (c.ang) ang_load(s, i, ot);  // (sample_target's omega targets, from zero)
    }
    if (c.ang) {  // _get_next_target's attitude_angular part (:1455-1460), from the targets before the update
      const T o0[3] = {ot[0], ot[1], ot[2]};
#pragma unroll
      for (int k = 0; k < 3; k++) ot[k] = att_ang_rate(c, k, tgt, o0, vals[0], vals[1]);
#pragma unroll
      for (int k = 0; k < 3; k++) s.tpr[(int64_t)(12 + k) * ld + i] = ot[k];
    }
    next_target(c, steps_tgt, steps, [&](int r) { return s.tpr[(int64_t)r * ld + i]; }, tgt);
    if (s.iws) {  // history["error"][k].append(self._get_error(k)) (fixed_wing.py:575-579): the window sums move on
      const int ns = (int)((lep + b) % (uint32_t)c.iwin);
      if (b != b_guess)
#pragma unroll
        for (int k = 0; k < 3; k++) iold[k] = ld_(s.iwr, ns * 3 + k, ld, i);
      // every W entries, once the ring holds exactly the window (slot W - 1 just written, b + 1 >= W), the sum is
      // formed afresh from the ring, oldest entry first as np.sum over the slice (fixed_wing.py:1004-1012): the
      // running total's rounding cannot build up over a long episode (round-5 advice).  ns = (life + 1) % W is
      // the same on every lane, so the branch is wave-uniform
      const bool resum = ns == c.iwin - 1 && b + 1u >= (uint32_t)c.iwin;
#pragma unroll
      for (int k = 0; k < 3; k++) {
        const T err = target_error(c, k, tgt[k], vals[k]);
        iqp[k] = iwq[k];
        iwq[k] = b >= (uint32_t)c.iwin ? (iwq[k] + err) - iold[k] : iwq[k] + err;
        if (resum) {
          T q = T(0);
          for (int j = 0; j + 1 < c.iwin; j++) q += ld_(s.iwr, j * 3 + k, ld, i);
          iwq[k] = q + err;
        }
        st_(s.iwr, ns * 3 + k, ld, i, err);
        st_(s.iws, IW_Q + k, ld, i, iwq[k]);
        st_(s.iws, IW_QP + k, ld, i, iqp[k]);
      }
    }
#ifndef FW_MET_SKIP_STEP
    if (c.metrics) metrics_step(c, s, i, M, tgt, vals, gb, gcnt, b, lep);
#endif
    gn = b + 1u;
  } else {
    done = true;
    reward = c.step_fail_timesteps ? (T)(steps - c.steps_max) : c.step_fail_value;
    term = sterm;
  }
  const T ep_ret = ep_ret0 + reward;

  // ---- observation (also the terminal observation) ----
  const int64_t ow = (int64_t)c.n_obs * c.obs_len;  // values per observation (rows x entries)
  const int omode = sterm ? OBS_FAIL : OBS_STEP;
  T* orow = obs_out + i * ow;
  // the "integrator" observation entries: the sum before the newest entry + padding (i = 1, fixed_wing.py:1168-1181)
  T iwv[3] = {T(0), T(0), T(0)};
  if (s.iws)
#pragma unroll
    for (int k = 0; k < 3; k++) iwv[k] = iw_value(c, iqp[k], steps - 1, iwq[3 + k]);
  if (done && tobs_out) {
    observe_env(c, s, i, episode, omode, y, der, tgt, steps, seqA, seqC, tobs_out + i * ow, lep);
    if (c.ang) ang_obs(c, ot, y, tobs_out + i * ow);
    if (s.iws) {
      iw_obs(c, iwv, tobs_out + i * ow);
      if (omode == OBS_FAIL) iw_obs_fail(c, s, i, steps, lep, tobs_out + i * ow);
    }
  }

  rew_out[i] = reward;
  done_out[i] = done ? 1 : 0;
  if (term_out) term_out[i] = term;
  if (stats) stats[i] = pack_stats(nfev, nacc, dmask);

  // Monitor episode record + the episode's final target (info["target"] of the done step)
  if (done && episode_out) {
    T* e = episode_out + i * 5;
    e[0] = ep_ret;
    e[1] = (T)steps;
    e[2] = tgt[0];
    e[3] = tgt[1];
    e[4] = tgt[2];
  }
  if (c.metrics) {
#ifndef FW_MET_SKIP_STORE
    M.store(s, i);
#endif
#ifndef FW_MET_SKIP_FINAL
    if (done && s.met_out) metrics_final(c, M, gn, steps, s.met_out + i, s.n);
#endif
  }
  FW_TSTAMP(3);
  // wavefront-uniform skip of the reset path when no lane of the wave is done
  const bool do_reset = done && auto_reset;
  if (__ballot(do_reset)) {
    if (do_reset) {
      T yr[NY], dr[8], wr[3], tr[3];
      // the worker's env.reset() passes no turbulence_noise: Dryden.reset(None) (dryden.py:184-188)
      if (s.noise_env_len && s.noise_env_len[i] > 0) s.noise_env_len[i] = 0;  // (the shared sequence stays)
      reset_lane(c, s, i, (const T*)nullptr, (const T*)nullptr, yr, dr, wr, tr);
      store_env_fresh(c, s, i, yr, dr, wr, tr, life0 + 1u);
#ifndef FW_MET_SKIP_INIT
      if (c.metrics) {
        const T vr[3] = {dr[0], dr[1], dr[3]};
        metrics_init(c, s, i, tr, vr, life0 + 1u);
      }
#endif
      T seq0[RING + 1][3];
      observe_env(c, s, i, s.episode[i], OBS_RESET, yr, dr, tr, 0, seq0, seq0, orow, life0 + 1u);  // (reset_lane's +1)
      if (c.ang) {
        T otr[3];
        ang_load(s, i, otr);
        ang_obs(c, otr, yr, orow);
      }
      if (s.iws) {
        // FixedWingAircraft.reset observes BEFORE it replaces the history (fixed_wing.py:452-459): the finished
        // episode's sums, padded as at steps_count 0; then the new episode's entry 0
        T rv[3];
#pragma unroll
        for (int k = 0; k < 3; k++) rv[k] = iw_value(c, iqp[k], -1, iwq[3 + k]);
        iw_obs_all_rows(c, rv, orow);
        iw_init(c, s, i, tr, dr, life0 + 1u);
        iw_hist_init(c, s, i, tr, dr);
      }
      s.life[i] = life0 + 1u;
      FW_TSTAMP(5);
      return;
    }
  }
#ifndef FW_SKIP_OBS
  observe_env(c, s, i, episode, omode, y, der, tgt, steps, seqA, seqC, orow, lep);
  if (c.ang) ang_obs(c, ot, y, orow);
  if (s.iws) {
    iw_obs(c, iwv, orow);
    if (omode == OBS_FAIL) iw_obs_fail(c, s, i, steps, lep, orow);
    else if (c.obs_hist) iw_hist_row(c, s, i, iwv, s.obs_ring + (int64_t)((lep + (uint32_t)steps) % (uint32_t)c.obs_hist) * c.n_obs * ld);
  }
#endif
#pragma unroll
  for (int r = 0; r < NY; r++) st_(s.y, r, ld, i, y[r]);
#pragma unroll
  for (int r = 0; r < 8; r++) st_(s.der, r, ld, i, der[r]);
#pragma unroll
  for (int k = 0; k < 3; k++)  // (constant-class targets never change within an episode)
    if (__ballot(bits_differ(tgt[k], tgt_in[k]))) st_(s.target, k, ld, i, tgt[k]);
  st_(s.ep_ret, 0, ld, i, ep_ret);
  s.steps[i] = (uint32_t)(steps & 0xFFFF) | ((uint32_t)(steps_tgt & 0xFFFF) << 16);
  s.life[i] = life0 + 1u;
  FW_TSTAMP(4);
}

// ---- in-launch merge of the block records (fw_collect_epilogue.merged) ---------------------------------
// Hand-off between blocks of one launch (MI355X_MICROARCH.md, hand-off table row 1): every word handed over
// is stored with an agent-scope store (write-through, `sc1`), every storing wave waits for its stores
// (s_waitcnt vmcnt(0)) and then ONE lane adds to the node's agent-scope counter; the block whose add returns
// the last count loads the words with agent-scope loads (`sc1`, L1 bypassed) only after that add returned.
// No cache write-back / invalidate fence (several us each at four blocks per CU).  The first version moved
// the words with agent-scope read-modify-write atomics instead: each lane's atomic is its own memory-side
// transaction, and the tree cost 16 us per launch (tools/epilogue_ab.py).
// (global address space: `global_` instructions -- the hand-off is not valid through `flat_` ones)
typedef __attribute__((address_space(1))) unsigned long long g_u64;
__device__ __forceinline__ void pub64(double* p, double v) {
  __hip_atomic_store((g_u64*)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double get64(const double* p) {
  return __longlong_as_double((long long)__hip_atomic_load((const g_u64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

constexpr int COL_MAXD = FW_MAX_OBS + 1;
constexpr int MN_COLS = 16;  // columns staged per LDS pass of merge_node
constexpr int MN_LD = 66;    // staging row stride (doubles): lane j reads row j with 16-B loads, 4 banks apart
// LDS staging of merge_node: MN_COLS + 1 rows x 64 records, the column means, update_from_moments' counts
constexpr size_t MN_BYTES = ((MN_COLS + 1) * MN_LD + COL_MAXD + 2) * sizeof(double);
// the handle's copy of the statistics a deferring env step found (fw_collect_pending.rms_prev): right below the
// merge tree's level records (State::col_lvl)
constexpr size_t COL_SHADOW_BYTES = ((2 * COL_MAXD + 4) * sizeof(double) + 255) / 256 * 256;

// sum of row[0 .. 64) in index order (row 16-B aligned): all loads issued first.  The slots of absent
// records hold +0.0, and adding +0.0 leaves any partial sum that can occur here unchanged (it starts at
// +0.0, so it is never -0.0): the same bits as summing only the present records, without 64 masks.
__device__ __forceinline__ double row_sum(const double* row) {
#pragma clang fp contract(off)
  double v[64];
#pragma unroll
  for (int k = 0; k < 32; k++) {
    const double2 t = reinterpret_cast<const double2*>(row)[k];
    v[2 * k] = t.x;
    v[2 * k + 1] = t.y;
  }
  double a = 0.0;
#pragma unroll
  for (int k = 0; k < 64; k++) a += v[k];
  return a;
}

// One wave merges cnt <= 64 records (field f of record k at src[f * stride + k], published with pub64)
// exactly as fw_moments_merge does, two-pass, every sum in record order: N = sum n_k,
// mean_j = (sum n_k mean_kj) / N, M2_j = sum (M2_kj + n_k (mean_kj - mean_j)^2).  Lane k loads record k
// (coalesced per field), MN_COLS columns at a time; the column sums go through LDS (lane j sums column
// j).  Returns N on every lane, mean_j / M2_j on lane j < D.
__device__ __forceinline__ void merge_node(const double* src, int64_t stride, int cnt, int D, double* st,
                                           double& N, double& mean, double& m2) {
#pragma clang fp contract(off)
  const int l = (int)(threadIdx.x & 63);
  const bool act = l < cnt;
  // the record addresses are formed in VGPRs from a per-lane base and an opaque stride: as wave-uniform
  // values the field addresses went to SGPRs (and spilled)
  const double* pl = src + l;
  int64_t sd = stride;
  asm volatile("" : "+v"(pl), "+v"(sd));
  const double nl = act ? get64(pl) : 0.0;
  N = 0.0;
  mean = 0.0;
  m2 = 0.0;
  for (int cb = 0; cb < D; cb += MN_COLS) {
    double m[MN_COLS], q[MN_COLS];
#pragma unroll
    for (int jj = 0; jj < MN_COLS; jj++) {  // (in flight together with nl's load)
      const bool v = act && cb + jj < D;
      m[jj] = v ? get64(pl + (int64_t)(1 + cb + jj) * sd) : 0.0;
      q[jj] = v ? get64(pl + (int64_t)(1 + D + cb + jj) * sd) : 0.0;
    }
    if (cb == 0) {
      st[MN_COLS * MN_LD + l] = nl;
      __syncthreads();
      N = row_sum(st + MN_COLS * MN_LD);  // (a broadcast read)
    }
    const bool mine = l >= cb && l < cb + MN_COLS && l < D;  // lane l owns column l
#pragma unroll
    for (int jj = 0; jj < MN_COLS; jj++) st[jj * MN_LD + l] = nl * m[jj];  // pass 1
    __syncthreads();
    double mu = 0.0;
    if (mine) mu = row_sum(st + (l - cb) * MN_LD) / N;
    __syncthreads();
    if (l >= cb && l < cb + MN_COLS) st[(MN_COLS + 1) * MN_LD + (l - cb)] = mu;  // this block's means
    if (mine) mean = mu;
    __syncthreads();
#pragma unroll
    for (int jj = 0; jj < MN_COLS; jj++) {  // pass 2
      const double dm = m[jj] - st[(MN_COLS + 1) * MN_LD + jj];
      st[jj * MN_LD + l] = q[jj] + nl * (dm * dm);
    }
    __syncthreads();
    if (mine) m2 = row_sum(st + (l - cb) * MN_LD);
    __syncthreads();
  }
}

// After this block published its record (level 0, column-major at col_rec with stride gridDim.x): draw a
// ticket on the block's node; the last block to arrive at a node merges the node's records in order and
// publishes the node's record one level up (fw_stats::merge_tree_size), until the final node, whose last
// arriver writes col_merged and -- with col_rms -- applies RunningMeanStd.update_from_moments
// (running_mean_std.py:26-40) through the same function fw_rms_update runs.  The node a block merges and
// the order inside it are fixed by block index, so the bits do not depend on the order blocks finish in;
// each node's counter is reset by its last arriver, for the next launch.  The merged record equals the one
// merge over all block records (fw_moments_merge) to rounding, not bit for bit (another summation tree).
__device__ __forceinline__ void collect_merge(const double* rec0, double* lvl, uint32_t* cnt, double* merged, double* rms,
                                           int D, int d, bool has_ret, double* st, bool defer) {
  const int l = (int)(threadIdx.x & 63);
  int64_t nodes = gridDim.x, idx = blockIdx.x, stride = gridDim.x;
  const double* src = rec0;
  while (true) {
    const bool fin = nodes <= fw_stats::MERGE_FANIN;
    // deferred (fw_collect_epilogue.defer, round 6): the final node's records stay where they are published;
    // the next fw_collect_policy launch merges them in its prologue (fw_collect_pending), off this launch's tail
    if (fin && defer) return;
    const int64_t g = fin ? 0 : idx / fw_stats::MERGE_FANIN;
    const int gs = fin ? (int)nodes : (int)std::min<int64_t>(fw_stats::MERGE_FANIN, nodes - g * fw_stats::MERGE_FANIN);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this block's published words have left the CU
    uint32_t t = 0;
    if (l == 0) t = __hip_atomic_fetch_add(cnt + g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    t = __shfl(t, 0);
    if (t != (uint32_t)(gs - 1)) return;  // not the last arrival: the node's last block merges it
    // acquire side of the ticket: no load of merge_node's (get64, which bypasses the CU's L1) may be issued
    // before the ticket's result is known (round-5 advice: only the loop-head clobber ordered them)
    asm volatile("" ::: "memory");
    if (l == 0) __hip_atomic_store(cnt + g, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // for the next launch
    double N, mean, m2;
    double warm = 0.0;  // the statistics' lines, fetched under the merge (update_from_moments re-reads them)
    if (fin && rms && l < 2 * d + 4) warm = rms[l];
    merge_node(src + g * fw_stats::MERGE_FANIN, stride, gs, D, st, N, mean, m2);
    asm volatile("" ::"v"(warm));
    if (fin) {
      double* out = merged;
      if (l < D) {
        out[1 + l] = mean;
        out[1 + D + l] = m2;
      }
      if (l == 0) out[0] = N;
      if (rms) {
        __syncthreads();  // (merge_node's last reads of st are done)
        if (l < D) {
          st[1 + l] = mean;
          st[1 + D + l] = m2;
        }
        if (l == 0) st[0] = N;
        __syncthreads();
        fw_stats::rms_update(st, 1, d, has_ret ? 1 : 0, rms, 1, 1, st + (MN_COLS + 1) * MN_LD + COL_MAXD);
      }
      return;
    }
    const int64_t up = fw_stats::merge_ceil(nodes, fw_stats::MERGE_FANIN);
    if (l < D) {
      pub64(lvl + (1 + l) * up + g, mean);
      pub64(lvl + (1 + D + l) * up + g, m2);
    }
    if (l == 0) pub64(lvl + g, N);
    src = lvl;
    stride = up;
    lvl += up * (1 + 2 * COL_MAXD);
    cnt += up;
    nodes = up;
    idx = g;
  }
}

// The env-side half of VecNormalize.step_wait (vec_normalize.py:106-131) after the env step, while the
// block's observations are still in cache (fw_set_collect_epilogue): per env ret = ret * gamma + reward
// (vec_normalize.py:126-129, multiply and add kept separate as numpy does) then ret[done] = 0 (:130), and
// per block one exact two-pass moment record (n_b, mean_b, M2_b) of the float32 observation columns and of
// ret before its reset -- the batch moments of RunningMeanStd.update (running_mean_std.py:20-24), merged
// over the blocks by the in-launch tree above (col_merged) or later by fw_moments_merge /
// fw_vecnorm_merge_update.  Row lanes: one per aircraft (lane 0 of each quad when Q = 4).  Four lanes per
// column, each summing 16 rows in order, then a quad butterfly: every sum in a fixed order, so the records
// are deterministic.  Every lane of the block calls this.
template <typename T>
__device__ __forceinline__ void collect_epilogue(const State<T>& s, int64_t i, bool row, int ow, const T* obs_out,
                                                 const T* rew_out, const uint8_t* done_out, float* sx, double* sr,
                                                 double* mst) {
  const int lane = (int)(threadIdx.x & 63);
  const bool has_ret = s.col_ret != nullptr;
  double ret = 0.0;
  if (row && has_ret) {
    double g = s.col_ret[i] * s.col_gamma;
    asm volatile("" : "+v"(g));  // no FMA contraction of ret * gamma + reward
    ret = g + (double)(float)rew_out[i];
    s.col_ret[i] = done_out[i] ? 0.0 : ret;
  }
  const bool defer = ((uintptr_t)s.col_cnt & 1u) != 0;  // (fw_collect_epilogue.defer)
  if (defer && blockIdx.x == 0) {  // the statistics the next policy launch updates (its blocks read this copy
    double* shadow = (double*)((char*)s.col_lvl - COL_SHADOW_BYTES);  // while its block 0 rewrites col_rms)
    for (int e = lane; e < 2 * ow + 4; e += 64) shadow[e] = s.col_rms[e];
  }
  if (s.col_rec) {
    const int D = ow + (has_ret ? 1 : 0);
    const bool tree = s.col_merged != nullptr;
    if (row) {
      for (int j = 0; j < ow; j++) sx[lane * COL_MAXD + j] = (float)obs_out[i * ow + j];
      sr[lane] = ret;
    }
    const unsigned long long rm = __ballot(row);
    const double nb = (double)__popcll(rm);
    __syncthreads();
    double* rec = s.col_rec + blockIdx.x;  // column-major: field q at rec[q * blocks] (coalesced merge reads)
    const int64_t qs = gridDim.x;
    const int p = lane & 3;
    for (int c0 = 0; c0 < D; c0 += 16) {
      const int col = c0 + (lane >> 2);
      const bool cv = col < D;
      auto at = [&](int r) { return col < ow ? (double)sx[r * COL_MAXD + col] : sr[r]; };
      double sum = 0.0;
      if (cv)
        for (int k = 0; k < 16; k++) {
          const int r = p * 16 + k;
          if ((rm >> r) & 1ull) sum += at(r);
        }
      sum += __shfl_xor(sum, 1);
      sum += __shfl_xor(sum, 2);
      const double mean = sum / nb;
      double q = 0.0;
      if (cv)
        for (int k = 0; k < 16; k++) {
          const int r = p * 16 + k;
          if ((rm >> r) & 1ull) {
            const double dv = at(r) - mean;
            q += dv * dv;
          }
        }
      q += __shfl_xor(q, 1);
      q += __shfl_xor(q, 2);
      if (cv && p == 0) {
        if (tree) {
          pub64(rec + (1 + col) * qs, mean);
          pub64(rec + (1 + D + col) * qs, q);
        } else {
          rec[(1 + col) * qs] = mean;
          rec[(1 + D + col) * qs] = q;
        }
      }
    }
    if (lane == 0) {
      if (tree)
        pub64(rec, nb);
      else
        rec[0] = nb;
    }
    if (tree) {
      __syncthreads();  // (the staging area is reused by the merge)
      collect_merge(s.col_rec, s.col_lvl, (uint32_t*)((uintptr_t)s.col_cnt & ~(uintptr_t)1), s.col_merged, s.col_rms, D,
                    ow, has_ret, mst, defer);
    }
  }
  if (s.col_ctrl && blockIdx.x == 0 && lane == 0) s.col_ctrl[0] += 1;  // the stream's next launch sees it
}

template <typename T, typename C, bool RP = false, int Q = 1>
__global__ __launch_bounds__(BLOCK, FW_WAVES(Q)) void k_env_step(const DevCfg<T>* __restrict__ cfgp, State<T> s,
                                                    const T* __restrict__ actions, T* __restrict__ obs_out,
                                                    T* __restrict__ rew_out, uint8_t* __restrict__ done_out,
                                                    int32_t* __restrict__ term_out, T* __restrict__ tobs_out,
                                                    T* __restrict__ episode_out, int32_t* __restrict__ stats,
                                                    int auto_reset) {
#if FW_HALF_WAVE
  const int64_t tid = Q == 1 ? (threadIdx.x < 32 ? (int64_t)blockIdx.x * 32 + threadIdx.x : (int64_t)s.n)
                             : (int64_t)blockIdx.x * BLOCK + threadIdx.x;
#else
  const int64_t tid = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
#endif
  const int64_t i = tid / Q;  // Q = 4: lanes 4i..4i+3 integrate aircraft i (fw_quad.hpp)
  const bool collect = s.col_rec || s.col_ret || s.col_ctrl;
  if (i >= s.n && !collect) return;
  const C& c = *reinterpret_cast<const C*>(cfgp);  // structural specialisation view (fw_device.hpp SpecCfg)
  __shared__ __attribute__((aligned(16))) V2<T> lds[(Q == 1 ? lds_slots<T>() * NP : Q == 2 ? pr::LDS_PAIRS : 1) * BLOCK];  // y, f (+ error sum) of the block's aircraft (pairs; Q = 2: the pair integrator's Y / F / ER)
  static_assert(Q != 1 || RP || FW_TAIL_QUAD == 0 || BLOCK == 64, "the tail handoff works per one-wave block");
  __shared__ qd::HoSlot<T> ho[Q == 1 && !RP ? BLOCK : 1];
  static_assert(BLOCK == 64, "collect_epilogue: one-wave blocks");
  // the epilogue's staging (64 rows x COL_MAXD floats + 64 doubles) reuses the integrator's LDS slots once
  // the step is done (one-lane instances; LDS bounds how many fp64 blocks fit a CU); quads get their own
  constexpr size_t COL_STAGE = 64 * COL_MAXD * sizeof(float) + 64 * sizeof(double);
  constexpr size_t COL_BYTES = COL_STAGE > MN_BYTES ? COL_STAGE : MN_BYTES;  // the merge tree reuses it
  constexpr bool COL_ALIAS = sizeof(lds) >= COL_BYTES;
  __shared__ __attribute__((aligned(16))) double col_sep[COL_ALIAS ? 1 : COL_BYTES / sizeof(double)];
  char* const col_base = COL_ALIAS ? (char*)lds : (char*)col_sep;
  float* const col_x = (float*)col_base;
  double* const col_r = (double*)(col_base + 64 * COL_MAXD * sizeof(float));
  if (i < s.n)
    env_step_lane<T, C, RP, Q, ((Q == 4 && (sizeof(T) == 4 ? FW_PREF_Q4_F32 : FW_PREF_Q4_F64)) || FW_PREF_Q1)>(c, s, i, lds, actions, obs_out, rew_out, done_out, term_out, tobs_out,
                                                    episode_out, stats, auto_reset, (int)(tid % Q), ho);
  if (collect) {
    if (COL_ALIAS) __syncthreads();  // (one wave: orders the slot reuse after the integrator's last accesses)
    collect_epilogue<T>(s, i, i < s.n && tid % Q == 0, c.n_obs * c.obs_len, obs_out, rew_out, done_out, col_x, col_r,
                        (double*)col_base);
  }
}

// One env step of k_env_rollout.  fp32: inlined, and scratch-free since the step loop re-materialises
// the aircraft index (below); behind a call boundary it ran 5 % slower (profiles/r02_ab_rollout.log).
// fp64: inlined, the step loop spills 660-810 VGPRs (the fp64 live state does not fit 512); behind a call
// boundary the step runs 1.39x faster (65536 aircraft, 1.86e8 -> 2.58e8 env-steps/s,
// profiles/r03_ab_rollout64.log), so FW_ROLLOUT_CALL64 = 1 ships.
#ifndef FW_ROLLOUT_CALL
#define FW_ROLLOUT_CALL 0  // 1: every instance's step behind a call
#endif
#ifndef FW_ROLLOUT_CALL64
#define FW_ROLLOUT_CALL64 1
#endif
template <typename T, typename C, bool RP, int Q>
__device__ __forceinline__ void env_step_inl(const C& c, const State<T>& s, const int64_t i, V2<T>* lds,
                                             const T* actions, T* obs_out, T* rew_out, uint8_t* done_out,
                                             int32_t* term_out, T* tobs_out, T* episode_out, int32_t* stats,
                                             int auto_reset, int qr, void* ho) {
  // no prefetch (the open loop needs no overlap); y / f in registers as in k_env_step, although the open loop alone
  // runs 7 % faster with them in LDS: the two forms round differently (contraction), and the open loop must equal
  // K k_env_step launches bit for bit (profiles/r06_openloop_yf_ab.log)
  env_step_lane<T, C, RP, Q, false, true>(c, s, i, lds, actions, obs_out, rew_out, done_out, term_out, tobs_out,
                                          episode_out, stats, auto_reset, qr, ho);
}
template <typename T, typename C, bool RP, int Q>
__device__ __noinline__ void env_step_noinl(const C& c, const State<T>& s, const int64_t i, V2<T>* lds,
                                            const T* actions, T* obs_out, T* rew_out, uint8_t* done_out,
                                            int32_t* term_out, T* tobs_out, T* episode_out, int32_t* stats,
                                            int auto_reset, int qr, void* ho) {
  env_step_inl<T, C, RP, Q>(c, s, i, lds, actions, obs_out, rew_out, done_out, term_out, tobs_out, episode_out, stats,
                            auto_reset, qr, ho);
}
template <typename T, typename C, bool RP, int Q>
__device__ __forceinline__ void env_step_call(const C& c, const State<T>& s, const int64_t i, V2<T>* lds,
                                              const T* actions, T* obs_out, T* rew_out, uint8_t* done_out,
                                              int32_t* term_out, T* tobs_out, T* episode_out, int32_t* stats,
                                              int auto_reset, int qr, void* ho) {
  if constexpr (FW_ROLLOUT_CALL || (FW_ROLLOUT_CALL64 && sizeof(T) == 8))
    env_step_noinl<T, C, RP, Q>(c, s, i, lds, actions, obs_out, rew_out, done_out, term_out, tobs_out, episode_out,
                                stats, auto_reset, qr, ho);
  else
    env_step_inl<T, C, RP, Q>(c, s, i, lds, actions, obs_out, rew_out, done_out, term_out, tobs_out, episode_out, stats,
                              auto_reset, qr, ho);
}

// Open-loop rollout: n_steps consecutive FixedWingAircraft.step calls per aircraft in ONE launch, actions
// given in advance ([K][N][3]; outputs per step [K][N][...]).  Identical per-step code to k_env_step, so
// the results equal K k_env_step launches bit for bit; what changes is synchronisation: a wave moves on
// to its next step as soon as its own aircraft are done, instead of every step waiting for the slowest
// aircraft of the whole batch (the RK45 straggler tail).
// Q = 4: the quad integrator as in k_env_step (lanes 1..3 of a quad skip each step's epilogue; lane 0's
// stores of step k precede the quad's loads of step k + 1 in the wave's program order).
template <typename T, typename C, bool RP = false, int Q = 1>
__global__ __launch_bounds__(BLOCK, FW_WAVES(Q)) void k_env_rollout(const DevCfg<T>* __restrict__ cfgp, State<T> s, int n_steps,
                                                       const T* __restrict__ actions, T* __restrict__ obs_out,
                                                       T* __restrict__ rew_out, uint8_t* __restrict__ done_out,
                                                       int32_t* __restrict__ term_out, T* __restrict__ tobs_out,
                                                       T* __restrict__ episode_out, int32_t* __restrict__ stats,
                                                       int auto_reset) {
  const int64_t tid = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
  const int64_t i = tid / Q;
  const int qr = (int)(tid % Q);
  if (i >= s.n) return;
  // (Q = 2: the pair integrator's Y / F / ER, as k_env_step -- fw_set_lanes(2) runs the open loop on pairs too, so
  // it equals K k_env_step launches bit for bit under every lanes setting)
  __shared__ V2<T> lds[(Q == 1 ? lds_slots<T>() * NP : Q == 2 ? pr::LDS_PAIRS : 1) * BLOCK];
  __shared__ qd::HoSlot<T> ho[Q == 1 && !RP ? BLOCK : 1];
  const int64_t n = s.n, ow = (int64_t)cfgp->n_obs * cfgp->obs_len;
  for (int k = 0; k < n_steps; k++) {
    // the aircraft index re-materialised per step: otherwise the backend hoists the ~70 per-lane 64-bit
    // row addresses of the step (every SoA row at i) out of the step loop, where they stay live across
    // the RK loop and spill (292 VGPRs, profiles/r03_isa_resources.txt); recomputed they cost an add each
    int64_t ik = i;
    asm volatile("" : "+v"(ik));
    const C& c = *reinterpret_cast<const C*>(cfgp);
    env_step_call<T, C, RP, Q>(c, s, ik, lds, actions + k * n * 3, obs_out + k * n * ow, rew_out + k * n, done_out + k * n,
                  term_out ? term_out + k * n : nullptr, tobs_out ? tobs_out + k * n * ow : nullptr,
                  episode_out ? episode_out + k * n * 5 : nullptr, stats ? stats + k * n : nullptr, auto_reset, qr, ho);
  }
}

}  // namespace

// ===========================================================================
// host side: handle, config conversion, launches, C ABI
// ===========================================================================
struct fw_handle {
  int device = 0;
  int precision = FW_F32;
  int64_t n = 0, ld = 0;
  fw_sim_config sim{};
  fw_env_config env{};
  bool has_env = false;
  int act_window = 1, cmd_window = 0;
  void* dcfg = nullptr;
  void* base = nullptr;
  size_t base_bytes = 0;
  uint64_t seed = 0;
  int64_t env_offset = 0;
  const void* noise = nullptr;
  int64_t noise_len = 0;
  int32_t* noise_env_len = nullptr;
  int spec = 0;  // 0 = generic DevCfg kernels, 1 = GymX8Cfg, 2 = PyflyX8Cfg (structure matched at upload)
  int metrics = 0;          // streaming episode-metric state allocated (env->metrics at create)
  void* met_out = nullptr;  // [FW_NMETRIC][N] done-episode records (fw_set_metrics_output)
  // offsets (bytes) of the SoA blocks inside base
  size_t o_y, o_der, o_wind, o_target, o_cmd, o_epret, o_act, o_cmdring, o_steps, o_goal, o_episode, o_life;
  size_t o_met = 0, o_metu16 = 0;
  int obs_hist = 0;         // past raw observation rows kept per env ((length - 1) * step + 2, 0 = none)
  size_t o_obs_init = 0, o_obs_ring = 0;
  size_t o_prm = 0;         // per-aircraft parameter rows (env->n_rand > 0 at create; 0 = none)
  size_t o_dry = 0;         // Dryden filter-bank state rows (turbulence on at create; 0 = none)
  size_t o_shp = 0;         // potential-form shaping rows (env->reward_potential at create; 0 = none)
  size_t o_rsc = 0;         // per-episode reward scalings (a randomised factor at create; 0 = none)
  size_t o_iwr = 0, o_iws = 0;  // integration-window ring and sums (env->integration_window > 0 at create)
  size_t o_tpr = 0;         // linear / sinusoidal target properties (such a target class at create; 0 = none)
  size_t o_gflag = 0;       // goal_achieved flags (a success reward factor at create; 0 = none)
  size_t o_dcur = 0;        // env-draw tape cursors (env handles)
  const void* tape = nullptr;  // fw_set_env_draws
  int32_t tape_len = 0;
  int iwin = 0;
  int rand_active = 0;      // the current config randomises parameters (kernels read the rows)
  int lanes_opt = FW_LANES_AUTO;  // fw_set_lanes: 0 = automatic, 1, 4
  int quad_ok = 1;          // the config allows the quad integrator (no wrapped ODE-state variable)
  fw_collect_epilogue col{};  // fw_set_collect_epilogue (all null: off)
  size_t o_colws = 0, o_colcnt = 0;  // in-launch merge tree workspace (records above level 0, counters)
  size_t colcnt_bytes = 0;           // bytes of the tree's arrival counters (zeroed again by clear_tree)
  size_t o_colshadow = 0;            // the statistics as a deferring env step found them (fw_collect_pending)
  bool tree_dirty = false;           // an env step with the tree failed: counters may hold stale arrivals
  uint32_t gring_mask = 127u;        // goal-history ring entries - 1 (a power of two >= 128, >= success_streak_req)
  int goal_rows = 18;                // GB_* rows (18 + ring words beyond 16 + a second count word when wide)
};

namespace {

template <typename T>
void fill_devcfg(const fw_handle* h, DevCfg<T>& d) {
  std::memset(&d, 0, sizeof(d));
  const fw_sim_config& s = h->sim;
  const double* P = s.param;
  d.tail_quad = std::getenv("FWSIM_TAIL_QUAD") ? std::atoi(std::getenv("FWSIM_TAIL_QUAD")) : FW_TAIL_QUAD;  // A/B switch
  d.tail_quad = std::min(std::max(d.tail_quad, 0), 16);  // at most 16 quads in a wave
  d.t_bound = s.dt;
  d.dt = (T)s.dt;
  d.rtol = (T)s.rtol;
  d.atol = (T)s.atol;
  d.half_rho = (T)(0.5 * s.rho);
  d.rho = (T)s.rho;
  d.grav = (T)s.g;
  d.ar0 = (T)(P[FW_P_B] * P[FW_P_B] / P[FW_P_S_WING]);
  for (int k = 0; k < FW_NPARAM; k++) d.pdef[k] = (T)P[k];
  d.S = (T)P[FW_P_S_WING];
  d.b = (T)P[FW_P_B];
  d.c = (T)P[FW_P_C];
  d.mass = (T)P[FW_P_MASS];
  d.inv_mass = (T)(1.0 / P[FW_P_MASS]);
  d.mg = (T)(P[FW_P_MASS] * s.g);
  d.inv_Jy = (T)(1.0 / P[FW_P_JY]);
  {  // gammas pyfly.py:1098-1116
    const double Jx = P[FW_P_JX], Jy = P[FW_P_JY], Jz = P[FW_P_JZ], I02 = -P[FW_P_JXZ];
    double G[9];
    G[0] = Jx * Jz - I02 * I02;
    G[1] = (std::fabs(I02) * (Jx - Jy + Jz)) / G[0];
    G[2] = (Jz * (Jz - Jy) + I02 * I02) / G[0];
    G[3] = Jz / G[0];
    G[4] = std::fabs(I02) / G[0];
    G[5] = (Jz - Jx) / Jy;
    G[6] = std::fabs(I02) / Jy;
    G[7] = ((Jx - Jy) * Jx + I02 * I02) / G[0];
    G[8] = Jx / G[0];
    for (int k = 0; k < 9; k++) d.gam[k] = (T)G[k];
  }
  d.M = (T)P[FW_P_M];
  d.a0 = (T)P[FW_P_A0];
  d.pi_e_ar = (T)(3.141592653589793 * P[FW_P_E] * (P[FW_P_B] * P[FW_P_B] / P[FW_P_S_WING]));
  d.sig_c = (T)std::exp(2.0 * P[FW_P_M] * P[FW_P_A0]);
  {
    const double qS = 0.5 * s.rho * P[FW_P_S_WING];
    d.qS = (T)qS;
    d.qSc = (T)(qS * P[FW_P_C]);
    d.qSb = (T)(qS * P[FW_P_B]);
    d.kCLq = (T)(P[FW_P_C_L_Q] * P[FW_P_C] * 0.5);
    d.kCDq = (T)(P[FW_P_C_D_Q] * P[FW_P_C] * 0.5);
    d.kCmq = (T)(P[FW_P_C_M_Q] * P[FW_P_B] * 0.5);
    d.hb = (T)(P[FW_P_B] * 0.5);
    d.inv_pi_e_ar = (T)(1.0 / (3.141592653589793 * P[FW_P_E] * (P[FW_P_B] * P[FW_P_B] / P[FW_P_S_WING])));
    d.kTP2 = (T)(P[FW_P_K_T_P] * P[FW_P_K_OMEGA] * P[FW_P_K_OMEGA]);
  }
  d.CL0 = (T)P[FW_P_C_L_0]; d.CLa = (T)P[FW_P_C_L_ALPHA]; d.CLq = (T)P[FW_P_C_L_Q]; d.CLde = (T)P[FW_P_C_L_DELTA_E];
  d.CDp = (T)P[FW_P_C_D_P]; d.CDq = (T)P[FW_P_C_D_Q]; d.CDb1 = (T)P[FW_P_C_D_BETA1]; d.CDb2 = (T)P[FW_P_C_D_BETA2];
  d.CDde = (T)P[FW_P_C_D_DELTA_E];
  d.Cm0 = (T)P[FW_P_C_M_0]; d.Cma = (T)P[FW_P_C_M_ALPHA]; d.Cmq = (T)P[FW_P_C_M_Q]; d.Cmde = (T)P[FW_P_C_M_DELTA_E];
  d.Cmfp = (T)P[FW_P_C_M_FP];
  d.CY0 = (T)P[FW_P_C_Y_0]; d.CYb = (T)P[FW_P_C_Y_BETA]; d.CYp = (T)P[FW_P_C_Y_P]; d.CYr = (T)P[FW_P_C_Y_R];
  d.CYda = (T)P[FW_P_C_Y_DELTA_A]; d.CYdr = (T)P[FW_P_C_Y_DELTA_R];
  d.Cl0 = (T)P[FW_P_C_L0_ROLL]; d.Clb = (T)P[FW_P_C_L_BETA]; d.Clp = (T)P[FW_P_C_L_P]; d.Clr = (T)P[FW_P_C_L_R];
  d.Clda = (T)P[FW_P_C_L_DELTA_A]; d.Cldr = (T)P[FW_P_C_L_DELTA_R];
  d.Cn0 = (T)P[FW_P_C_N_0]; d.Cnb = (T)P[FW_P_C_N_BETA]; d.Cnp = (T)P[FW_P_C_N_P]; d.Cnr = (T)P[FW_P_C_N_R];
  d.Cnda = (T)P[FW_P_C_N_DELTA_A]; d.Cndr = (T)P[FW_P_C_N_DELTA_R];
  d.kmotor = (T)P[FW_P_K_MOTOR];
  d.prop_k = (T)(0.5 * s.rho * P[FW_P_S_PROP] * P[FW_P_C_PROP]);
  d.kTP = (T)P[FW_P_K_T_P];
  d.kOmega = (T)P[FW_P_K_OMEGA];
  d.Sprop = (T)P[FW_P_S_PROP];
  d.Cprop = (T)P[FW_P_C_PROP];
  for (int j = 0; j < 3; j++) {
    const fw_actuator& A = s.act[j];
    if (A.order == 1) {
      d.ac[j][0] = (T)(-1.0 / A.tau); d.ac[j][1] = 0; d.ac[j][2] = (T)(1.0 / A.tau);
      d.ac[j][3] = 0; d.ac[j][4] = 0; d.ac[j][5] = 0;
    } else {
      d.ac[j][0] = 0; d.ac[j][1] = 1; d.ac[j][2] = 0;
      d.ac[j][3] = (T)(-(A.omega_0 * A.omega_0)); d.ac[j][4] = (T)(-2 * A.zeta * A.omega_0);
      d.ac[j][5] = (T)(A.omega_0 * A.omega_0);
    }
    d.dot_max[j] = (T)A.dot_max;
    if (std::isfinite(A.dot_max)) d.dotmask |= 1u << j;
  }
  for (int v = 0; v < FW_NVAR; v++) {
    const fw_limits& L = s.lim[v];
    d.lim[v] = Lim<T>{(T)L.value_min, (T)L.value_max, (T)L.constraint_min, (T)L.constraint_max};
    d.init_min[v] = (T)L.init_min;
    d.init_max[v] = (T)L.init_max;
    if (std::isfinite(L.constraint_min) || std::isfinite(L.constraint_max)) d.cmask |= 1u << v;
    if (std::isfinite(L.value_min) || std::isfinite(L.value_max)) d.clipmask |= 1u << v;
    if (L.wrap) d.wrapmask |= 1u << v;
  }
  auto limited = [&](int v) { return ((d.clipmask | d.wrapmask) >> v) & 1u; };
  d.trig_alpha = limited(FW_V_ALPHA);
  d.trig_beta = limited(FW_V_BETA);
  // Euler-angle clipping (not the +-pi wrap, a no-op on atan2 output) changes the post-step rotation
  d.euler_exact = ((d.clipmask >> FW_V_ROLL) | (d.clipmask >> FW_V_PITCH) | (d.clipmask >> FW_V_YAW)) & 1u;
  d.elevon = s.elevon;
  d.disabled_inputs = s.disabled_inputs;
  d.turbulence = s.turbulence;
  d.turb_len = s.turb_len > 0 ? s.turb_len : 1;
  d.wind_random = s.wind_random;
  d.max_nfev = s.max_nfev > 0 ? s.max_nfev : MAX_NFEV;
  d.wind_mag_min = (T)s.wind_mag_min;
  d.wind_mag_max = (T)s.wind_mag_max;
  for (int k = 0; k < 3; k++) {
    d.wind_init_min[k] = (T)s.wind_init_min[k];
    d.wind_init_max[k] = (T)s.wind_init_max[k];
  }
  for (int k = 0; k < 6; k++) {
    d.g0[k] = (T)s.dryden_g0[k];
    d.g1[k] = (T)s.dryden_g1[k];
  }
  d.noise_scale = (T)std::sqrt(3.141592653589793 / (double)d.turb_len);
  d.dry_state = s.turbulence ? s.dryden_state : 0;
  d.dry_ncut = s.dryden_ncut;
  for (int k = 0; k < 28; k++) {
    d.dry_ad[k] = (T)s.dryden_ad[k];
    d.dry_e1[k] = (T)s.dryden_e1[k];
  }
  for (int k = 0; k < 12; k++) {
    d.dry_b0[k] = (T)s.dryden_b0[k];
    d.dry_b1[k] = (T)s.dryden_b1[k];
    d.dry_c[k] = (T)s.dryden_c[k];
  }

  d.has_env = h->has_env;
  d.act_window = h->act_window;
  d.cmd_window = h->cmd_window;
  d.act_need = d.cmd_need = 0;
  if (h->has_env) {
    const fw_env_config& e = h->env;
    // an env step reads previous action j for j < window (obs_raw / reward_of: entries 0 .. window - 1, entry 0
    // the current action)
    for (int o = 0; o < e.n_obs; o++)
      if (e.obs[o].kind == FW_OBS_ACTION_WINDOW) {
        if (e.scale_actions) d.act_need = std::max(d.act_need, e.obs[o].window - 1);
        else d.cmd_need = std::max(d.cmd_need, e.obs[o].window - 1);
      }
    for (int r = 0; r < e.n_rew; r++)
      if (e.rew[r].kind == FW_REW_ACTION_DELTA) d.act_need = std::max(d.act_need, e.rew[r].window - 1);
    d.steps_max = e.steps_max;
    d.n_obs = e.n_obs;
    d.scale_actions = e.scale_actions;
    d.has_bounds = e.has_bounds;
    d.streak_req = e.streak_req;
    d.gring_mask = h->gring_mask;
    d.gcnt_wide = e.streak_req > 255;
    d.gcnt2_row = GB_ROWS + (int)((h->gring_mask + 1u) / 8u - 16u);
    d.on_success = e.on_success;
    d.n_rew = e.n_rew;
    d.step_fail_timesteps = e.step_fail_timesteps;
    d.scale_low = (T)e.scale_low;
    d.scale_high = (T)e.scale_high;
    d.bmax = (T)(e.scale_high * e.bounds_multiplier);
    d.bmin = (T)(e.scale_low * e.bounds_multiplier);
    for (int k = 0; k < 3; k++) {
      d.act_low[k] = (T)e.act_low[k];
      d.act_high[k] = (T)e.act_high[k];
      d.target_class[k] = e.target_class[k];
      d.target_wrap[k] = e.target_wrap[k];
      d.target_low[k] = (T)e.target_low[k];
      d.target_high[k] = (T)e.target_high[k];
      d.has_delta[k] = !std::isnan(e.target_delta[k]);
      d.target_delta[k] = d.has_delta[k] ? (T)e.target_delta[k] : T(0);
      d.has_bound[k] = !std::isnan(e.target_bound[k]);
      d.target_bound[k] = d.has_bound[k] ? (T)e.target_bound[k] : T(0);
      d.term_weight[k] = (T)e.term_weight[k];
      d.term_present[k] = e.term_present[k];
    }
    d.tprops = 0;
    for (int k = 0; k < 3; k++) {
      d.tprops |= (e.target_class[k] == FW_TGT_LINEAR || e.target_class[k] == FW_TGT_SINUSOIDAL) ? 1 : 0;
      d.tgt_rad[k] = e.target_radians[k] ? (T)(3.141592653589793 / 180.0) : T(1);  // np.radians: x * (pi / 180)
      d.tgt_slo[k] = (T)e.target_slope_low[k];
      d.tgt_shi[k] = (T)e.target_slope_high[k];
      d.tgt_alo[k] = (T)e.target_amp_low[k];
      d.tgt_ahi[k] = (T)e.target_amp_high[k];
      d.tgt_plo[k] = (T)e.target_period_low[k];
      d.tgt_phi[k] = (T)e.target_period_high[k];
    }
    d.tprops = d.tprops && h->o_tpr;
    d.tape_skip = e.tape_skip > 0 ? e.tape_skip : 0;
    d.ang = e.ang_targets ? 1 : 0;
    for (int k = 0; k < 3; k++) d.ang_max_vel[k] = (T)e.ang_max_vel[k];
    d.n_targets = d.ang ? T(6) : T(3);
    d.goal_flag = h->o_gflag != 0;
    d.streak_frac = (T)e.streak_frac;
    d.step_fail_value = (T)e.step_fail_value;
    d.metrics = h->metrics && e.metrics;
    d.reward_potential = e.reward_potential ? 1 : 0;
    d.resample_every = e.resample_every > 0 ? e.resample_every : 0;
    d.iwin = e.integration_window > 0 ? e.integration_window : 0;
    d.rise_low = (T)e.rise_low;
    d.rise_high = (T)e.rise_high;
    d.obs_len = e.obs_length > 1 ? e.obs_length : 1;
    d.obs_step = e.obs_step > 1 ? e.obs_step : 1;
    d.obs_hist = h->obs_hist;
    d.obs_noise = e.obs_noise != 0;
    d.obs_noise_mean = (T)e.obs_noise_mean;
    d.obs_noise_std = (T)e.obs_noise_std;
    d.obs_general = d.obs_len > 1 || d.obs_noise;
    std::memcpy(d.obs, e.obs, sizeof(d.obs));
    std::memcpy(d.rew, e.rew, sizeof(d.rew));
    d.rand_params = e.n_rand > 0 && h->o_prm != 0;
    d.n_rand = d.rand_params ? e.n_rand : 0;
    for (int r = 0; r < d.n_rand; r++) {
      const fw_rand_param& R = e.rand[r];
      d.rp[r].param = R.param;
      d.rp[r].dist = R.dist;
      d.rp[r].has_clip = !std::isnan(R.clip);
      d.rp[r].orig = (T)R.original;
      d.rp[r].var = (T)R.var;
      d.rp[r].clip = d.rp[r].has_clip ? (T)R.clip : T(0);
    }
  }
}

int validate(const fw_sim_config* s, const fw_env_config* e) {
  if (!s) return set_err(FW_E_INVALID, "sim config is NULL");
  if (!(s->dt > 0)) return set_err(FW_E_INVALID, "dt must be > 0");
  for (int j = 0; j < 3; j++)
    if (s->act[j].order != 1 && s->act[j].order != 2) return set_err(FW_E_INVALID, "actuator order must be 1 or 2");
  if (s->turbulence && s->turb_len < 2) return set_err(FW_E_INVALID, "turb_len must be >= 2");
  if (s->max_nfev < 0) return set_err(FW_E_INVALID, "max_nfev must be >= 0 (0 = default budget)");
  if (e) {
    if (e->n_obs < 1 || e->n_obs > FW_MAX_OBS) return set_err(FW_E_INVALID, "n_obs out of range");
    if (e->n_rew < 0 || e->n_rew > FW_MAX_REW) return set_err(FW_E_INVALID, "n_rew out of range");
    if (e->steps_max > 65535) return set_err(FW_E_UNSUPPORTED, "steps_max > 65535");
    if (e->metrics && (e->steps_max < 1 || e->steps_max > 65534))  // 16-bit entry indices, 0xFFFF = none
      return set_err(FW_E_UNSUPPORTED, "episode metrics need 1 <= steps_max <= 65534");
    if (e->streak_req > 4096) return set_err(FW_E_UNSUPPORTED, "success_streak_req > 4096");
    if (e->obs_length < 0 || e->obs_length > FW_MAX_OBS_LEN || e->obs_step < 0 ||
        (e->obs_length > 1 && (e->obs_length - 1) * std::max(e->obs_step, 1) + 2 > FW_MAX_OBS_HIST))
      return set_err(FW_E_UNSUPPORTED, "observation length / step out of range");
    if (e->obs_noise && !(e->obs_noise_std >= 0)) return set_err(FW_E_INVALID, "observation noise scale < 0");
    if (e->n_rand < 0 || e->n_rand > FW_NPARAM) return set_err(FW_E_INVALID, "n_rand out of range");
    for (int r = 0; r < e->n_rand; r++)
      if (e->rand[r].param < 0 || e->rand[r].param >= FW_NPARAM ||
          (e->rand[r].dist != FW_DIST_GAUSSIAN && e->rand[r].dist != FW_DIST_UNIFORM))
        return set_err(FW_E_INVALID, "bad parameter randomisation entry");
    for (int o = 0; o < e->n_obs; o++)
      if (e->obs[o].kind == FW_OBS_ACTION_WINDOW && (e->obs[o].window < 1 || e->obs[o].window > FW_MAX_WINDOW))
        return set_err(FW_E_UNSUPPORTED, "action window out of range");
    for (int r = 0; r < e->n_rew; r++) {
      if (e->rew[r].kind == FW_REW_ACTION_DELTA && (e->rew[r].window < 1 || e->rew[r].window > FW_MAX_WINDOW))
        return set_err(FW_E_UNSUPPORTED, "reward window out of range");
      if (e->rew[r].kind < FW_REW_STATE_ERROR || e->rew[r].kind > FW_REW_GOAL)
        return set_err(FW_E_INVALID, "unknown reward factor kind");
    }
    for (int k = 0; k < 3; k++)
      if (e->target_class[k] < FW_TGT_CONSTANT || e->target_class[k] > FW_TGT_SINUSOIDAL)
        return set_err(FW_E_INVALID, "unknown target class");
    if (e->target_class[2] == FW_TGT_COMPENSATE && e->target_class[1] == FW_TGT_COMPENSATE)
      return set_err(FW_E_UNSUPPORTED, "compensate Va with a compensate pitch target (fixed_wing.py:1386-1392)");
    if (e->on_success < 0 || e->on_success > 2) return set_err(FW_E_INVALID, "on_success must be 0 (none), 1 (done) or 2 (new)");
    // attitude_angular targets (ABI 12): entries / factors address them as FW_TGT_OMEGA_P + k only when present;
    // plain observations only (ang_obs writes row 0); metrics cover roll / pitch / Va
    for (int o = 0; o < e->n_obs; o++) {
      const fw_obs_entry& E = e->obs[o];
      const bool tgt = E.kind == FW_OBS_TARGET_ABS || E.kind == FW_OBS_TARGET_REL || E.kind == FW_OBS_TARGET_INT;
      if (tgt && (E.var < 0 || E.var > (e->ang_targets && E.kind != FW_OBS_TARGET_INT ? FW_TGT_OMEGA_P + 2 : 2)))
        return set_err(FW_E_INVALID, "target observation entry: bad target index");
    }
    for (int r = 0; r < e->n_rew; r++)
      if (e->rew[r].kind == FW_REW_STATE_ERROR &&
          (e->rew[r].var < 0 || e->rew[r].var > (e->ang_targets ? FW_TGT_OMEGA_P + 2 : 2)))
        return set_err(FW_E_INVALID, "state error reward factor: bad target index");
    if (e->ang_targets) {
      if (e->obs_length > 1 || e->obs_noise || e->metrics)
        return set_err(FW_E_UNSUPPORTED, "attitude_angular targets with observation history / noise or metrics");
      for (int k = 0; k < 3; k++)
        if (!(e->ang_max_vel[k] >= 0)) return set_err(FW_E_INVALID, "attitude_angular max_vel < 0");
    }
  }
  return FW_OK;
}

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Which compiled structural specialisation (fw_device.hpp SpecCfg) matches this config.
template <typename S, typename T>
bool same_limits(const DevCfg<T>& d) {
  if constexpr (S::const_limits) {
    for (int v = 0; v < FW_NVAR; v++)
      if (std::memcmp(&d.lim[v], &S::lim[v], sizeof(Lim<T>)) != 0) return false;
    if (std::memcmp(d.dot_max, S::dot_max, sizeof(d.dot_max)) != 0) return false;
  }
  return true;
}

template <typename S, typename T>
bool same_params(const DevCfg<T>& d) {
  if constexpr (S::const_params) {
#define FW_X8_CMP(name, val) \
  if (std::memcmp(&d.name, &S::name, sizeof(T)) != 0) return false;
    FW_X8_SCALARS(FW_X8_CMP)
#undef FW_X8_CMP
    if (std::memcmp(d.gam, S::gam, sizeof(d.gam)) != 0) return false;
    if (std::memcmp(d.ac, S::ac, sizeof(d.ac)) != 0) return false;
  }
  return true;
}

template <typename S, typename T>
bool same_structure(const DevCfg<T>& d) {
  if (!same_limits<S>(d) || !same_params<S>(d)) return false;
  return d.rand_params == S::rand_params && d.cmask == S::cmask && d.clipmask == S::clipmask &&
         d.wrapmask == S::wrapmask && d.dotmask == S::dotmask &&
         d.elevon == S::elevon && d.trig_alpha == S::trig_alpha && d.trig_beta == S::trig_beta &&
         d.euler_exact == S::euler_exact && d.obs_general == S::obs_general && d.ang == S::ang;
}

template <typename T>
int spec_of(const DevCfg<T>& d) {
  if (std::getenv("FWSIM_GENERIC")) return 0;  // A/B switch for tests and profiling
  if (same_structure<GymX8Cfg<T>>(d)) return 1;
  if (same_structure<PyflyX8Cfg<T>>(d)) return 2;
  return 0;
}

// the quad integrator's conditions have no wrap (fw_quad.hpp qcond): ODE-state variables must not wrap
constexpr uint32_t ODE_VAR_MASK = (7u << FW_V_OMEGA_P) | (7u << FW_V_POS_N) | (7u << FW_V_VEL_U) | (7u << FW_V_ACT0);

int upload_cfg(fw_handle* h) {
  if (h->precision == FW_F64) {
    DevCfg<double> d;
    fill_devcfg(h, d);
    h->rand_active = d.rand_params;
    h->spec = spec_of(d);
    h->quad_ok = (d.wrapmask & ODE_VAR_MASK) == 0;
    FW_HIP(hipMemcpy(h->dcfg, &d, sizeof(d), hipMemcpyHostToDevice));
  } else {
    DevCfg<float> d;
    fill_devcfg(h, d);
    h->rand_active = d.rand_params;
    h->spec = spec_of(d);
    h->quad_ok = (d.wrapmask & ODE_VAR_MASK) == 0;
    FW_HIP(hipMemcpy(h->dcfg, &d, sizeof(d), hipMemcpyHostToDevice));
  }
  return FW_OK;
}

// Lanes per aircraft of the step kernels.  Automatic: the quad integrator while one quad wave per SIMD
// holds the shard (FW_QUAD_AUTO_MAX aircraft: lower per-aircraft latency), beyond that one lane per
// aircraft with the tail handoff to quads (rk45 HO); profiles/r02_lanes.log.
#ifndef FW_QUAD_AUTO_MAX
#define FW_QUAD_AUTO_MAX 16384
#endif
int lanes_of(const fw_handle* h) {
  if (!h->quad_ok) return 1;
  if (h->lanes_opt != FW_LANES_AUTO) return h->lanes_opt;
  static const int env_lanes = [] {  // A/B switch for tests and profiling: FWSIM_LANES=1|4 replaces auto
    const char* e = std::getenv("FWSIM_LANES");
    return e ? std::atoi(e) : 0;
  }();
  if (env_lanes == 1 || env_lanes == 2 || env_lanes == 4) return env_lanes;
  return h->n <= FW_QUAD_AUTO_MAX ? 4 : 1;
}

// launch KERNEL<T, C> with C chosen by the handle's structural specialisation (G / P: the gym / pyfly
// X8 view types of this kernel)
#define FW_LAUNCH_SPEC_GRID(KERNEL, G, P, T, h, st, grid, ...)                                                  \
  do {                                                                                                           \
    const dim3 gg_(grid), b_(BLOCK);                                                                             \
    if ((h)->rand_active)                                                                                        \
      hipLaunchKernelGGL((KERNEL<T, DevCfg<T>, true>), gg_, b_, 0, st, (const DevCfg<T>*)(h)->dcfg, __VA_ARGS__);  \
    else if ((h)->spec == 1)                                                                                     \
      hipLaunchKernelGGL((KERNEL<T, G<T>>), gg_, b_, 0, st, (const DevCfg<T>*)(h)->dcfg, __VA_ARGS__);             \
    else if ((h)->spec == 2)                                                                                     \
      hipLaunchKernelGGL((KERNEL<T, P<T>>), gg_, b_, 0, st, (const DevCfg<T>*)(h)->dcfg, __VA_ARGS__);             \
    else                                                                                                         \
      hipLaunchKernelGGL((KERNEL<T, DevCfg<T>>), gg_, b_, 0, st, (const DevCfg<T>*)(h)->dcfg, __VA_ARGS__);        \
  } while (0)
#define FW_LAUNCH_SPEC_AS(KERNEL, G, P, T, h, st, ...) \
  FW_LAUNCH_SPEC_GRID(KERNEL, G, P, T, h, st, grid_of(h), __VA_ARGS__)
#define FW_LAUNCH_SPEC(KERNEL, T, h, st, ...) FW_LAUNCH_SPEC_AS(KERNEL, GymX8Cfg, PyflyX8Cfg, T, h, st, __VA_ARGS__)

// ... and Q = lanes per aircraft (1, or 4 for the quad integrator)
#define FW_LAUNCH_SPEC_Q(KERNEL, PAIR, T, h, st, ...)                                                             \
  do {                                                                                                             \
    const dim3 b_(BLOCK);                                                                                          \
    const int q0_ = lanes_of(h);                                                                                   \
    const int q_ = (!(PAIR) && q0_ == 2) ? 1 : q0_; /* no pair instances of this kernel: one lane */               \
    const dim3 g_((unsigned)(((h)->n * q_ + (FW_HALF_WAVE && q_ == 1 ? 32 : BLOCK) - 1) /                          \
                             (FW_HALF_WAVE && q_ == 1 ? 32 : BLOCK)));                                            \
    const DevCfg<T>* d_ = (const DevCfg<T>*)(h)->dcfg;                                                             \
    bool done_ = false;                                                                                            \
    if constexpr (PAIR) {                                                                                          \
      if (q_ == 2) {                                                                                               \
        done_ = true;                                                                                              \
        if ((h)->rand_active) hipLaunchKernelGGL((KERNEL<T, DevCfg<T>, true, 2>), g_, b_, 0, st, d_, __VA_ARGS__); \
        else if ((h)->spec == 1) hipLaunchKernelGGL((KERNEL<T, GymX8Cfg<T>, false, 2>), g_, b_, 0, st, d_, __VA_ARGS__); \
        else if ((h)->spec == 2) hipLaunchKernelGGL((KERNEL<T, PyflyX8Cfg<T>, false, 2>), g_, b_, 0, st, d_, __VA_ARGS__); \
        else hipLaunchKernelGGL((KERNEL<T, DevCfg<T>, false, 2>), g_, b_, 0, st, d_, __VA_ARGS__);                \
      }                                                                                                            \
    }                                                                                                              \
    if (done_) {                                                                                                   \
    } else if (q_ == 4) {                                                                                          \
      if ((h)->rand_active) hipLaunchKernelGGL((KERNEL<T, DevCfg<T>, true, 4>), g_, b_, 0, st, d_, __VA_ARGS__);   \
      else if ((h)->spec == 1) hipLaunchKernelGGL((KERNEL<T, GymX8Cfg<T>, false, 4>), g_, b_, 0, st, d_, __VA_ARGS__); \
      else if ((h)->spec == 2) hipLaunchKernelGGL((KERNEL<T, PyflyX8Cfg<T>, false, 4>), g_, b_, 0, st, d_, __VA_ARGS__); \
      else hipLaunchKernelGGL((KERNEL<T, DevCfg<T>, false, 4>), g_, b_, 0, st, d_, __VA_ARGS__);                  \
    } else {                                                                                                       \
      FW_LAUNCH_SPEC_GRID(KERNEL, GymX8Cfg, PyflyX8Cfg, T, h, st, g_, __VA_ARGS__);                                \
    }                                                                                                              \
  } while (0)

template <typename T>
State<T> state_of(const fw_handle* h) {
  State<T> s;
  char* b = (char*)h->base;
  s.n = h->n;
  s.ld = h->ld;
  s.y = (T*)(b + h->o_y);
  s.der = (T*)(b + h->o_der);
  s.wind = (T*)(b + h->o_wind);
  s.target = (T*)(b + h->o_target);
  s.cmd = (T*)(b + h->o_cmd);
  s.ep_ret = (T*)(b + h->o_epret);
  s.act_ring = (T*)(b + h->o_act);
  s.cmd_ring = h->cmd_window ? (T*)(b + h->o_cmdring) : nullptr;
  s.steps = (uint32_t*)(b + h->o_steps);
  s.goal = (uint32_t*)(b + h->o_goal);
  s.episode = (uint32_t*)(b + h->o_episode);
  s.life = (uint32_t*)(b + h->o_life);
  s.noise = (const T*)h->noise;
  s.noise_len = h->noise_len;
  s.noise_env_len = h->noise_env_len;
  s.key0 = (uint32_t)(h->seed & 0xFFFFFFFFu);
  s.key1 = (uint32_t)(h->seed >> 32);
  s.env_offset = (uint32_t)h->env_offset;
  s.met = h->metrics ? (T*)(b + h->o_met) : nullptr;
  s.metu16 = h->metrics ? (uint16_t*)(b + h->o_metu16) : nullptr;
  s.met_out = (T*)h->met_out;
  s.obs_init = h->obs_hist ? (T*)(b + h->o_obs_init) : nullptr;
  s.obs_ring = h->obs_hist ? (T*)(b + h->o_obs_ring) : nullptr;
  s.prm = h->o_prm ? (T*)(b + h->o_prm) : nullptr;
  s.dry = (h->o_dry && h->sim.turbulence && h->sim.dryden_state) ? (T*)(b + h->o_dry) : nullptr;
  s.shp = (h->o_shp && h->has_env && h->env.reward_potential) ? (T*)(b + h->o_shp) : nullptr;
  s.rsc = h->o_rsc ? (T*)(b + h->o_rsc) : nullptr;
  s.iwr = h->o_iwr ? (T*)(b + h->o_iwr) : nullptr;
  s.iws = h->o_iws ? (T*)(b + h->o_iws) : nullptr;
  s.tpr = h->o_tpr ? (T*)(b + h->o_tpr) : nullptr;
  s.gflag = h->o_gflag ? (uint32_t*)(b + h->o_gflag) : nullptr;
  s.dcur = h->o_dcur ? (uint32_t*)(b + h->o_dcur) : nullptr;
  s.tape = (h->tape && h->o_dcur) ? (const T*)h->tape : nullptr;
  s.tape_len = h->tape_len;
  s.col_ret = h->col.ret;
  s.col_gamma = h->col.gamma;
  s.col_rec = h->col.records;
  s.col_ctrl = h->col.row_ctrl;
  s.col_merged = h->col.merged;
  s.col_rms = h->col.rms;
  s.col_lvl = h->o_colws ? (double*)(b + h->o_colws) : nullptr;
  s.col_cnt = h->o_colws ? (uint32_t*)(b + h->o_colcnt + (h->col.defer ? 1 : 0)) : nullptr;
  return s;
}

unsigned grid_of(const fw_handle* h) { return (unsigned)((h->n + BLOCK - 1) / BLOCK); }

int check_launch() {
  FW_HIP(hipGetLastError());
  return FW_OK;
}

// The merge tree's arrival counters are reset by each node's last arriver; a launch that did not run to
// its end leaves counts behind that would make every later tree merge at the wrong arrival.  A failed env
// step with the tree on zeroes them on its stream and marks the handle, and the next
// fw_set_collect_epilogue that turns the tree on zeroes them again after a device synchronisation.
void clear_tree(fw_handle* h, hipStream_t st) {
  if (h->o_colws && h->colcnt_bytes) (void)hipMemsetAsync((char*)h->base + h->o_colcnt, 0, h->colcnt_bytes, st);
}

}  // namespace

// Launch helpers of the step kernels: one explicit instance per build part (FW_PART 1..6), called
// from the C ABI in part 0.  Only plain types cross the parts.
namespace fwl {
template <typename T>
int sim_step(fw_handle* h, hipStream_t st, const void* cmd, void* cmd_out, uint8_t* success, int32_t* term,
             int32_t* stats) {
  FW_LAUNCH_SPEC_Q(k_sim_step, true, T, h, st, state_of<T>(h), (const T*)cmd, (T*)cmd_out, success, term, stats);
  return check_launch();
}
template <typename T>
int env_step(fw_handle* h, hipStream_t st, const void* actions, void* obs, void* reward, uint8_t* done, int32_t* term,
             void* tobs, void* episode, int32_t* stats, int32_t auto_reset) {
  FW_LAUNCH_SPEC_Q(k_env_step, true, T, h, st, state_of<T>(h), (const T*)actions, (T*)obs, (T*)reward, done, term, (T*)tobs,
                   (T*)episode, stats, auto_reset);
  return check_launch();
}
template <typename T>
int env_rollout(fw_handle* h, hipStream_t st, int32_t n_steps, const void* actions, void* obs, void* reward,
                uint8_t* done, int32_t* term, void* tobs, void* episode, int32_t* stats, int32_t auto_reset) {
  FW_LAUNCH_SPEC_Q(k_env_rollout, true, T, h, st, state_of<T>(h), n_steps, (const T*)actions, (T*)obs, (T*)reward, done,
                   term, (T*)tobs, (T*)episode, stats, auto_reset);
  return check_launch();
}
}  // namespace fwl

#define FW_SIG_SIM(T) int fwl::sim_step<T>(fw_handle*, hipStream_t, const void*, void*, uint8_t*, int32_t*, int32_t*)
#define FW_SIG_ENV(T)                                                                                           \
  int fwl::env_step<T>(fw_handle*, hipStream_t, const void*, void*, void*, uint8_t*, int32_t*, void*, void*, \
                       int32_t*, int32_t)
#define FW_SIG_ROLL(T)                                                                                              \
  int fwl::env_rollout<T>(fw_handle*, hipStream_t, int32_t, const void*, void*, void*, uint8_t*, int32_t*, void*, \
                          void*, int32_t*, int32_t)
#if FW_PART == 0
extern template FW_SIG_SIM(float);
extern template FW_SIG_SIM(double);
extern template FW_SIG_ENV(float);
extern template FW_SIG_ENV(double);
extern template FW_SIG_ROLL(float);
extern template FW_SIG_ROLL(double);
#elif FW_PART == 1
template FW_SIG_ENV(float);
#elif FW_PART == 2
template FW_SIG_ENV(double);
#elif FW_PART == 3
template FW_SIG_ROLL(float);
#elif FW_PART == 4
template FW_SIG_ROLL(double);
#elif FW_PART == 5
template FW_SIG_SIM(float);
#elif FW_PART == 6
template FW_SIG_SIM(double);
#endif

#if FW_HOST_PART
extern "C" {

int fw_abi_version(void) { return FWSIM_ABI_VERSION; }

int fw_last_error(char* buf, size_t len) {
  if (!buf || !len) return FW_E_INVALID;
  std::snprintf(buf, len, "%s", g_err.c_str());
  return FW_OK;
}

int fw_create(const fw_sim_config* sim, const fw_env_config* env, int64_t n_envs, int32_t precision, int32_t device,
              fw_handle** out) {
  if (!out) return set_err(FW_E_INVALID, "out is NULL");
  *out = nullptr;
  int v = validate(sim, env);
  if (v) return v;
  if (n_envs < 1 || n_envs > (int64_t)1 << 31) return set_err(FW_E_INVALID, "n_envs out of range");
  if (precision != FW_F32 && precision != FW_F64) return set_err(FW_E_INVALID, "precision must be FW_F32 or FW_F64");
  fw_handle* h = new (std::nothrow) fw_handle();
  if (!h) return set_err(FW_E_NOMEM, "host allocation failed");
  h->device = device;
  h->precision = precision;
  h->n = n_envs;
  h->ld = (n_envs + 63) / 64 * 64;
  h->sim = *sim;
  h->has_env = env != nullptr;
  h->metrics = env != nullptr && env->metrics != 0;
  if (env) {
    h->env = *env;
    int wa = 1, wc = 0;
    for (int o = 0; o < env->n_obs; o++)
      if (env->obs[o].kind == FW_OBS_ACTION_WINDOW) {
        if (env->scale_actions) wa = std::max(wa, env->obs[o].window);  // window entries: fw_observe re-reads the newest too
        else wc = std::max(wc, env->obs[o].window);
      }
    for (int r = 0; r < env->n_rew; r++)
      if (env->rew[r].kind == FW_REW_ACTION_DELTA) wa = std::max(wa, env->rew[r].window - 1);
    h->act_window = std::max(wa, 1);
    h->cmd_window = wc;
  }
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) {
    delete h;
    return set_err(FW_E_HIP, std::string("hipSetDevice: ") + hipGetErrorString(e));
  }
  const size_t T_ = precision == FW_F64 ? 8 : 4;
  const size_t row = align_up((size_t)h->ld * T_, 256), row32 = align_up((size_t)h->ld * 4, 256);
  size_t off = 0;
  h->o_y = off; off += FW_NY * row;
  h->o_der = off; off += 8 * row;
  h->o_wind = off; off += 3 * row;
  h->o_target = off; off += 3 * row;
  h->o_cmd = off; off += 3 * row;
  h->o_epret = off; off += row;
  h->o_act = off; off += (size_t)h->act_window * 3 * row;
  h->o_cmdring = off; off += (size_t)h->cmd_window * 3 * row;
  h->o_steps = off; off += row32;
  if (env) {  // goal ring: the power of two >= success_streak_req entries (at least the 128 of rounds 1-5)
    uint32_t entries = 128u;
    while ((int64_t)entries < (int64_t)env->streak_req) entries <<= 1;
    h->gring_mask = entries - 1u;
    h->goal_rows = GB_ROWS + (int)(entries / 8u - 16u) + (env->streak_req > 255 ? 1 : 0);
  }
  h->o_goal = off; off += (size_t)h->goal_rows * row32;
  h->o_episode = off; off += row32;
  h->o_life = off; off += row32;
  if (h->metrics) {
    h->o_met = off; off += (size_t)MT_ROWS * row;
    h->o_metu16 = off; off += (size_t)M16_ROWS * align_up((size_t)h->ld * 2, 256);
  }
  if (sim->turbulence) {  // Dryden filter-bank state (used when the chunk is too short for the FIR)
    h->o_dry = off; off += (size_t)12 * row;
  }
  if (env && env->reward_potential) {  // the previous step's reward shaping (reward.form "potential")
    h->o_shp = off; off += (size_t)3 * row;
  }
  if (env && env->integration_window > 0) {  // the error history's window sums (integration_window)
    h->iwin = env->integration_window;
    h->o_iwr = off; off += (size_t)3 * h->iwin * row;
    h->o_iws = off; off += (size_t)9 * row;
  }
  if (env) {  // per-episode reward scalings (reward.randomize_scaling)
    bool any = false;
    for (int r = 0; r < env->n_rew; r++) any = any || env->rew[r].randomize;
    if (any) { h->o_rsc = off; off += (size_t)FW_MAX_REW * row; }
  }
  if (env && env->n_rand > 0) {  // per-aircraft parameters (simulator parameter randomisation)
    h->o_prm = off; off += (size_t)FW_NPARAM * row;
  }
  if (env) {  // linear / sinusoidal targets: their drawn properties; success rewards: goal_achieved; tape cursors
    bool tp = false, sf = false;
    for (int k = 0; k < 3; k++) tp = tp || env->target_class[k] == FW_TGT_LINEAR || env->target_class[k] == FW_TGT_SINUSOIDAL;
    for (int r = 0; r < env->n_rew; r++) sf = sf || env->rew[r].kind == FW_REW_SUCCESS;
    if (tp || env->ang_targets) { h->o_tpr = off; off += (size_t)(env->ang_targets ? 15 : 12) * row; }
    if (sf) { h->o_gflag = off; off += align_up((size_t)h->ld * 4, 256); }
    h->o_dcur = off; off += align_up((size_t)h->ld * 4, 256);
  }
  if (env && env->obs_length > 1) {  // observation history: first row of the episode + ring of past rows
    const int step = env->obs_step > 1 ? env->obs_step : 1;
    h->obs_hist = (env->obs_length - 1) * step + 2;
    h->o_obs_init = off; off += (size_t)env->n_obs * row;
    h->o_obs_ring = off; off += (size_t)h->obs_hist * env->n_obs * row;
  }
  if (env) {  // the collect epilogue's in-launch merge tree (fw_collect_epilogue.merged), sized for 4 lanes
    int64_t mr = 0, mc = 0;
    fw_stats::merge_tree_size((h->n * 4 + BLOCK - 1) / BLOCK, &mr, &mc);
    // the statistics a deferring launch found (fw_collect_pending.rms_prev), right below the tree's records
    h->o_colshadow = off; off += COL_SHADOW_BYTES;
    h->o_colws = off; off += align_up((size_t)mr * (1 + 2 * COL_MAXD) * sizeof(double), 256);
    h->o_colcnt = off; off += align_up((size_t)mc * sizeof(uint32_t), 256);  // zeroed below, reset by the tree
    h->colcnt_bytes = (size_t)mc * sizeof(uint32_t);
  }
  // rows are ld elements apart: the padding above is folded into ld for simplicity
  h->base_bytes = off;
  e = hipMalloc(&h->base, off);
  if (e == hipSuccess) e = hipMemset(h->base, 0, off);
  if (e == hipSuccess) e = hipMemsetD32((hipDeviceptr_t)((char*)h->base + h->o_life), (int)LIFE0, (size_t)h->ld);
  if (e == hipSuccess) e = hipMalloc(&h->dcfg, precision == FW_F64 ? sizeof(DevCfg<double>) : sizeof(DevCfg<float>));
  if (e != hipSuccess) {
    if (h->base) (void)hipFree(h->base);
    delete h;
    return set_err(FW_E_HIP, std::string("device allocation: ") + hipGetErrorString(e));
  }
  v = upload_cfg(h);
  if (v) {
    (void)hipFree(h->base);
    (void)hipFree(h->dcfg);
    delete h;
    return v;
  }
  *out = h;
  return FW_OK;
}

int fw_destroy(fw_handle* h) {
  if (!h) return FW_OK;
  (void)hipSetDevice(h->device);
  if (h->base) (void)hipFree(h->base);
  if (h->dcfg) (void)hipFree(h->dcfg);
  delete h;
  return FW_OK;
}

int fw_num_envs(const fw_handle* h, int64_t* n) {
  if (!h || !n) return set_err(FW_E_INVALID, "NULL argument");
  *n = h->n;
  return FW_OK;
}

int fw_num_obs(const fw_handle* h, int32_t* n) {
  if (!h || !n) return set_err(FW_E_INVALID, "NULL argument");
  *n = h->has_env ? h->env.n_obs * std::max(h->env.obs_length, 1) : 0;
  return FW_OK;
}

int fw_seed(fw_handle* h, uint64_t seed, int64_t env_offset) {
  if (!h) return set_err(FW_E_INVALID, "NULL handle");
  h->seed = seed;
  h->env_offset = env_offset;
  // a re-seed restarts every env's stream: the episode counters (the Philox counter's episode word)
  // go back to 0, so the next reset draws what the first reset after fw_create drew
  FW_HIP(hipSetDevice(h->device));
  FW_HIP(hipDeviceSynchronize());
  FW_HIP(hipMemset((char*)h->base + h->o_episode, 0, align_up((size_t)h->ld * 4, 256)));
  FW_HIP(hipDeviceSynchronize());
  return FW_OK;
}

int fw_set_noise(fw_handle* h, const void* noise_dev, int64_t len) {
  if (!h) return set_err(FW_E_INVALID, "NULL handle");
  if (noise_dev && len < 1) return set_err(FW_E_INVALID, "noise length must be >= 1");
  if (len > INT32_MAX) return set_err(FW_E_INVALID, "noise length must be < 2^31");
  h->noise = noise_dev;
  h->noise_len = noise_dev ? len : 0;
  h->noise_env_len = nullptr;  // lengths belong to a buffer: set them again with fw_set_noise_lengths
  return FW_OK;
}

int fw_set_env_draws(fw_handle* h, const void* tape_dev, int32_t len) {
  if (!h) return set_err(FW_E_INVALID, "NULL handle");
  if (!h->has_env || !h->o_dcur) return set_err(FW_E_INVALID, "fw_set_env_draws: handle has no env");
  if (tape_dev && len < 1) return set_err(FW_E_INVALID, "fw_set_env_draws: len must be >= 1");
  FW_HIP(hipSetDevice(h->device));
  FW_HIP(hipDeviceSynchronize());  // (launches in flight keep the tape they were given)
  FW_HIP(hipMemset((char*)h->base + h->o_dcur, 0, (size_t)h->ld * 4));
  h->tape = tape_dev;
  h->tape_len = tape_dev ? len : 0;
  return FW_OK;
}

int fw_set_noise_lengths(fw_handle* h, int32_t* env_len_dev) {
  if (!h) return set_err(FW_E_INVALID, "NULL handle");
  if (env_len_dev && !h->noise) return set_err(FW_E_INVALID, "fw_set_noise_lengths: set the noise buffer first");
  h->noise_env_len = env_len_dev;
  return FW_OK;
}

int fw_update_config(fw_handle* h, const fw_sim_config* sim, const fw_env_config* env) {
  if (!h) return set_err(FW_E_INVALID, "NULL handle");
  int v = validate(sim, env);
  if (v) return v;
  if ((env != nullptr) != h->has_env) return set_err(FW_E_INVALID, "env config presence cannot change");
  if (env) {
    // windows decide the ring sizes allocated at create time
    fw_handle tmp = *h;
    tmp.env = *env;
    int wa = 1, wc = 0;
    for (int o = 0; o < env->n_obs; o++)
      if (env->obs[o].kind == FW_OBS_ACTION_WINDOW) {
        if (env->scale_actions) wa = std::max(wa, env->obs[o].window);  // window entries: fw_observe re-reads the newest too
        else wc = std::max(wc, env->obs[o].window);
      }
    for (int r = 0; r < env->n_rew; r++)
      if (env->rew[r].kind == FW_REW_ACTION_DELTA) wa = std::max(wa, env->rew[r].window - 1);
    if (wa != h->act_window || wc != h->cmd_window || env->n_obs != h->env.n_obs ||
        std::max(env->obs_length, 1) != std::max(h->env.obs_length, 1) ||
        std::max(env->obs_step, 1) != std::max(h->env.obs_step, 1))
      return set_err(FW_E_UNSUPPORTED, "config update may not change observation layout or window sizes");
    if (env->metrics && !h->metrics)
      return set_err(FW_E_UNSUPPORTED, "episode metrics must be enabled when the handle is created");
    if (env->n_rand > 0 && !h->o_prm)
      return set_err(FW_E_UNSUPPORTED, "parameter randomisation must be enabled when the handle is created");
    for (int r = 0; r < env->n_rew; r++)
      if (env->rew[r].randomize && !h->o_rsc)
        return set_err(FW_E_UNSUPPORTED, "reward.randomize_scaling must be set when the handle is created");
    // the per-episode scaling rows are drawn at reset for the factors randomised then: a factor randomised
    // only from now on would divide by its still-zero row until the aircraft's next reset
    if (h->o_rsc) {
      bool same = env->n_rew == h->env.n_rew;
      for (int r = 0; same && r < env->n_rew; r++) same = (env->rew[r].randomize != 0) == (h->env.rew[r].randomize != 0);
      if (!same)
        return set_err(FW_E_UNSUPPORTED, "reward.randomize_scaling: the randomised factors cannot change after create");
    }
    {  // the goal ring and the count width were sized for the streak window at create
      uint32_t entries = 128u;
      while ((int64_t)entries < (int64_t)env->streak_req) entries <<= 1;
      if (entries > h->gring_mask + 1u || (env->streak_req > 255) != (h->env.streak_req > 255))
        return set_err(FW_E_UNSUPPORTED, "success_streak_req beyond the goal history sized at create");
    }
    if (env->integration_window != h->iwin)
      return set_err(FW_E_UNSUPPORTED, "integration_window must be the one the handle was created with");
    if (env->reward_potential && !h->o_shp)
      return set_err(FW_E_UNSUPPORTED, "reward.form \"potential\" must be set when the handle is created");
    for (int k = 0; k < 3; k++)
      if ((env->target_class[k] == FW_TGT_LINEAR || env->target_class[k] == FW_TGT_SINUSOIDAL || env->ang_targets) && !h->o_tpr)
        return set_err(FW_E_UNSUPPORTED, "linear / sinusoidal target classes must be configured when the handle is created");
    if ((env->ang_targets != 0) != (h->env.ang_targets != 0))
      return set_err(FW_E_UNSUPPORTED, "attitude_angular targets must be the ones the handle was created with");
    for (int r = 0; r < env->n_rew; r++)
      if (env->rew[r].kind == FW_REW_SUCCESS && !h->o_gflag)
        return set_err(FW_E_UNSUPPORTED, "a success reward factor must be configured when the handle is created");
    h->env = *env;
  }
  if (sim->turbulence && sim->dryden_state && !h->o_dry)
    return set_err(FW_E_UNSUPPORTED, "turbulence must be enabled when the handle is created (Dryden filter state)");
  h->sim = *sim;
  FW_HIP(hipSetDevice(h->device));
  FW_HIP(hipDeviceSynchronize());
  return upload_cfg(h);
}

int fw_reset(fw_handle* h, const uint8_t* mask_dev, const void* init_dev, const void* target_dev, void* obs_dev,
             void* stream) {
  if (!h) return set_err(FW_E_INVALID, "NULL handle");
  FW_HIP(hipSetDevice(h->device));
  hipStream_t st = (hipStream_t)stream;
  if (h->precision == FW_F64)
    hipLaunchKernelGGL(k_reset<double>, dim3(grid_of(h)), dim3(BLOCK), 0, st, (const DevCfg<double>*)h->dcfg,
                       state_of<double>(h), mask_dev, (const double*)init_dev, (const double*)target_dev,
                       (double*)obs_dev);
  else
    hipLaunchKernelGGL(k_reset<float>, dim3(grid_of(h)), dim3(BLOCK), 0, st, (const DevCfg<float>*)h->dcfg,
                       state_of<float>(h), mask_dev, (const float*)init_dev, (const float*)target_dev, (float*)obs_dev);
  return check_launch();
}

int fw_observe(fw_handle* h, void* obs_dev, void* stream) {
  if (!h || !obs_dev) return set_err(FW_E_INVALID, "NULL argument");
  if (!h->has_env) return set_err(FW_E_INVALID, "handle has no env config");
  FW_HIP(hipSetDevice(h->device));
  hipStream_t st = (hipStream_t)stream;
  if (h->precision == FW_F64)
    hipLaunchKernelGGL(k_observe<double>, dim3(grid_of(h)), dim3(BLOCK), 0, st, (const DevCfg<double>*)h->dcfg,
                       state_of<double>(h), (double*)obs_dev);
  else
    hipLaunchKernelGGL(k_observe<float>, dim3(grid_of(h)), dim3(BLOCK), 0, st, (const DevCfg<float>*)h->dcfg,
                       state_of<float>(h), (float*)obs_dev);
  return check_launch();
}

int fw_sim_step(fw_handle* h, const void* commands_dev, void* commands_out_dev, uint8_t* success_dev, int32_t* term_dev,
                int32_t* stats_dev, void* stream) {
  if (!h || !commands_dev) return set_err(FW_E_INVALID, "NULL argument");
  FW_HIP(hipSetDevice(h->device));
  hipStream_t st = (hipStream_t)stream;
  if (h->precision == FW_F64)
    return fwl::sim_step<double>(h, st, commands_dev, commands_out_dev, success_dev, term_dev, stats_dev);
  return fwl::sim_step<float>(h, st, commands_dev, commands_out_dev, success_dev, term_dev, stats_dev);
}

int fw_env_step(fw_handle* h, const void* actions_dev, void* obs_dev, void* reward_dev, uint8_t* done_dev,
                int32_t* term_dev, void* terminal_obs_dev, void* episode_dev, int32_t* stats_dev, int32_t auto_reset,
                void* stream) {
  if (!h || !actions_dev || !obs_dev || !reward_dev || !done_dev) return set_err(FW_E_INVALID, "NULL argument");
  if (!h->has_env) return set_err(FW_E_INVALID, "handle has no env config");
  FW_HIP(hipSetDevice(h->device));
  hipStream_t st = (hipStream_t)stream;
  const int r = h->precision == FW_F64
                    ? fwl::env_step<double>(h, st, actions_dev, obs_dev, reward_dev, done_dev, term_dev, terminal_obs_dev,
                                            episode_dev, stats_dev, auto_reset)
                    : fwl::env_step<float>(h, st, actions_dev, obs_dev, reward_dev, done_dev, term_dev, terminal_obs_dev,
                                           episode_dev, stats_dev, auto_reset);
  if (r != FW_OK && h->col.merged) {
    clear_tree(h, st);
    h->tree_dirty = true;
  }
  return r;
}

int fw_env_rollout(fw_handle* h, int32_t n_steps, const void* actions_dev, void* obs_dev, void* reward_dev,
                   uint8_t* done_dev, int32_t* term_dev, void* terminal_obs_dev, void* episode_dev, int32_t* stats_dev,
                   int32_t auto_reset, void* stream) {
  if (!h || !actions_dev || !obs_dev || !reward_dev || !done_dev) return set_err(FW_E_INVALID, "NULL argument");
  if (!h->has_env) return set_err(FW_E_INVALID, "handle has no env config");
  if (n_steps < 1) return set_err(FW_E_INVALID, "n_steps must be >= 1");
  FW_HIP(hipSetDevice(h->device));
  hipStream_t st = (hipStream_t)stream;
  if (h->precision == FW_F64)
    return fwl::env_rollout<double>(h, st, n_steps, actions_dev, obs_dev, reward_dev, done_dev, term_dev,
                                    terminal_obs_dev, episode_dev, stats_dev, auto_reset);
  return fwl::env_rollout<float>(h, st, n_steps, actions_dev, obs_dev, reward_dev, done_dev, term_dev, terminal_obs_dev,
                                 episode_dev, stats_dev, auto_reset);
}

int fw_set_lanes(fw_handle* h, int32_t lanes) {
  if (!h) return set_err(FW_E_INVALID, "NULL handle");
  if (lanes != FW_LANES_AUTO && lanes != 1 && lanes != 2 && lanes != 4)
    return set_err(FW_E_INVALID, "lanes must be 0 (auto), 1, 2 or 4");
  if ((lanes == 4 || lanes == 2) && !h->quad_ok)
    return set_err(FW_E_INVALID, "lanes = 2 / 4 need a config without wrapped ODE-state variables");
  h->lanes_opt = lanes;
  return FW_OK;
}

int fw_get_lanes(const fw_handle* h, int32_t* lanes) {
  if (!h || !lanes) return set_err(FW_E_INVALID, "NULL argument");
  *lanes = lanes_of(h);
  return FW_OK;
}

int64_t fw_quad_auto_max(void) { return FW_QUAD_AUTO_MAX; }

int fw_set_metrics_output(fw_handle* h, void* metrics_dev) {
  if (!h) return set_err(FW_E_INVALID, "NULL handle");
  if (metrics_dev && !h->metrics) return set_err(FW_E_INVALID, "handle was created without episode metrics");
  h->met_out = metrics_dev;
  return FW_OK;
}

int fw_set_collect_epilogue(fw_handle* h, const fw_collect_epilogue* epi) {
  if (!h) return set_err(FW_E_INVALID, "NULL handle");
  if (!epi) {
    h->col = fw_collect_epilogue{};
    return FW_OK;
  }
  if ((epi->ret || epi->records || epi->row_ctrl) && !h->has_env)
    return set_err(FW_E_INVALID, "fw_set_collect_epilogue: handle has no env");
  if (h->has_env && h->env.n_obs * std::max(h->env.obs_length, 1) + 1 > FW_MAX_OBS + 1 && epi->records)
    return set_err(FW_E_UNSUPPORTED, "fw_set_collect_epilogue: more than FW_MAX_OBS observation values per env");
  if (epi->merged && !epi->records)
    return set_err(FW_E_INVALID, "fw_set_collect_epilogue: merged needs the records buffer (the tree's level 0)");
  if (epi->rms && !epi->merged) return set_err(FW_E_INVALID, "fw_set_collect_epilogue: rms needs merged");
  if (epi->defer && !epi->rms)
    return set_err(FW_E_INVALID, "fw_set_collect_epilogue: defer needs rms (the statistics the deferred merge updates)");
  h->col = *epi;
  if (epi->merged && h->tree_dirty) {  // no arrival left over from a failed launch
    FW_HIP(hipSetDevice(h->device));
    FW_HIP(hipDeviceSynchronize());
    FW_HIP(hipMemset((char*)h->base + h->o_colcnt, 0, h->colcnt_bytes));
    h->tree_dirty = false;
  }
  return FW_OK;
}

int fw_collect_pending(const fw_handle* h, fw_collect_pend* p) {
  if (!h || !p) return set_err(FW_E_INVALID, "fw_collect_pending: NULL argument");
  if (!h->has_env || !h->o_colws) return set_err(FW_E_INVALID, "fw_collect_pending: handle has no env");
  if (!h->col.records || !h->col.merged || !h->col.defer)
    return set_err(FW_E_INVALID, "fw_collect_pending: no deferred merge tree (fw_set_collect_epilogue with defer)");
  // the level the tree stops at (collect_merge): level 0 = the caller's records when the launch has at most
  // MERGE_FANIN blocks, else the first level of the handle's workspace with at most MERGE_FANIN nodes
  const int64_t blocks = (h->n * lanes_of(h) + BLOCK - 1) / BLOCK;
  char* const b = (char*)h->base;
  if (blocks <= fw_stats::MERGE_FANIN) {
    p->records = h->col.records;
    p->stride = blocks;
    p->count = (int32_t)blocks;
  } else {
    double* lvl = (double*)(b + h->o_colws);
    int64_t nodes = blocks;
    while (true) {
      const int64_t up = fw_stats::merge_ceil(nodes, fw_stats::MERGE_FANIN);
      if (up <= fw_stats::MERGE_FANIN) {
        p->records = lvl;
        p->stride = up;
        p->count = (int32_t)up;
        break;
      }
      lvl += up * (1 + 2 * COL_MAXD);
      nodes = up;
    }
  }
  p->D = h->env.n_obs * std::max(h->env.obs_length, 1) + (h->col.ret ? 1 : 0);
  p->rms_prev = (const double*)(b + h->o_colshadow);
  return FW_OK;
}

int fw_collect_records(const fw_handle* h, int64_t* n_records, int64_t* max_records) {
  if (!h) return set_err(FW_E_INVALID, "NULL handle");
  if (n_records) *n_records = (h->n * lanes_of(h) + BLOCK - 1) / BLOCK;
  if (max_records) *max_records = (h->n * 4 + BLOCK - 1) / BLOCK;
  return FW_OK;
}

// FW_BLK_ACT_RING / FW_BLK_CMD_RING as the ABI presents them (action k of the current episode in slot
// (k - 1) % W, fwsim.h) <-> the device layout (the action j steps back, k = steps_count + 1 - j, in slot
// (life - j) % W: the expression k_env_step reads it with): a per-aircraft rotation of the W slots.
__global__ void k_ring_xlate(const char* __restrict__ src, char* __restrict__ dst, int W, int64_t n, int esz,
                             int64_t row_dev, int64_t row_abi, const uint32_t* __restrict__ life,
                             const uint32_t* __restrict__ steps, int to_abi) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int st = (int)(steps[i] & 0xFFFFu);
  for (int j = 1; j <= W; j++) {
    const int p = (int)((life[i] - (uint32_t)j) % (uint32_t)W);
    const int q = ((st - j) % W + W) % W;  // (k - 1) % W for k = st + 1 - j (k <= 0: an earlier episode's slot)
    for (int a = 0; a < 3; a++) {
      const int64_t rl = (int64_t)q * 3 + a, rp = (int64_t)p * 3 + a;
      const char* from = to_abi ? src + rp * row_dev + i * esz : src + rl * row_abi + i * esz;
      char* to = to_abi ? dst + rl * row_abi + i * esz : dst + rp * row_dev + i * esz;
      if (esz == 8) *(uint64_t*)to = *(const uint64_t*)from;
      else *(uint32_t*)to = *(const uint32_t*)from;
    }
  }
}

static int ring_copy(fw_handle* h, int32_t block, size_t off, size_t esz, const void* src, void* dst, int to_abi,
                     hipStream_t st) {
  const int W = block == FW_BLK_ACT_RING ? h->act_window : h->cmd_window;
  const int64_t row_dev = (int64_t)align_up((size_t)h->ld * esz, 256), row_abi = h->n * (int64_t)esz;
  char* b = (char*)h->base;
  hipLaunchKernelGGL(k_ring_xlate, dim3((unsigned)((h->n + 255) / 256)), dim3(256), 0, st,
                     to_abi ? (const char*)(b + off) : (const char*)src, to_abi ? (char*)dst : (char*)(b + off), W,
                     h->n, (int)esz, row_dev, row_abi, (const uint32_t*)(b + h->o_life),
                     (const uint32_t*)(b + h->o_steps), to_abi);
  return check_launch();
}

// FW_BLK_GOAL as the ABI presents it (the 128-bit register of the "all" statuses, bit j of row j / 32 = entry
// N - 1 - j of the episode's history, 0 past its start, fwsim.h) <-> the device's goal history (GB_*: nibble ring
// by lifetime position, window counts, entry count N).  Setting takes N = steps_count + 1 from FW_BLK_STEPS (the
// history of an episode without a failed step: a checkpoint sets FW_BLK_STEPS first), rewrites the "all" bit of
// the 128 ring positions and recounts the "all" window; the per-target statuses and counts (metrics) stay.
__global__ void k_goal_xlate(uint32_t* __restrict__ goal, int64_t ld, uint32_t* __restrict__ reg, int64_t n,
                             const uint32_t* __restrict__ life, const uint32_t* __restrict__ steps, int req,
                             int to_abi, uint32_t gm) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint32_t N = to_abi ? goal[GB_N * ld + i] : (steps[i] & 0xFFFFu) + 1u;
  const uint32_t newest = life[i] - (steps[i] & 0xFFFFu) + N - 1u;  // lifetime position of entry N - 1
  if (!to_abi) goal[GB_N * ld + i] = N;
  if (to_abi) {
    uint32_t w[4] = {0u, 0u, 0u, 0u};
    for (uint32_t j = 0; j < 128u && j < N; j++) {
      const uint32_t pos = newest - j;
      w[j >> 5] |= ((gring_get(goal[gring_row(pos, gm) * ld + i], pos) >> 3) & 1u) << (j & 31u);
    }
    for (int r = 0; r < 4; r++) reg[r * n + i] = w[r];
    return;
  }
  uint32_t cnt = 0u;
  for (uint32_t j = 0; j < 128u; j++) {
    const uint32_t pos = newest - j, bit = (reg[(j >> 5) * n + i] >> (j & 31u)) & 1u;
    uint32_t* wp = goal + gring_row(pos, gm) * ld + i;
    *wp = gring_set(*wp, pos, (gring_get(*wp, pos) & 7u) | (bit << 3));
    if ((int)j < req && j < N) cnt += bit;
  }
  uint32_t* cp = goal + GB_CNT * ld + i;
  *cp = (*cp & 0x00FFFFFFu) | (cnt << 24);
}

static int goal_copy(fw_handle* h, const void* src, void* dst, int to_abi, hipStream_t st) {
  char* b = (char*)h->base;
  if (!to_abi && h->has_env && h->env.streak_req > 128)  // the 128-bit register cannot hold the window
    return set_err(FW_E_UNSUPPORTED, "FW_BLK_GOAL: setting the goal history needs success_streak_req <= 128");
  hipLaunchKernelGGL(k_goal_xlate, dim3((unsigned)((h->n + 255) / 256)), dim3(256), 0, st, (uint32_t*)(b + h->o_goal),
                     (int64_t)h->ld, to_abi ? (uint32_t*)dst : (uint32_t*)const_cast<void*>(src), h->n,
                     (const uint32_t*)(b + h->o_life), (const uint32_t*)(b + h->o_steps),
                     h->has_env ? std::max(h->env.streak_req, 0) : 0, to_abi, h->gring_mask);
  return check_launch();
}

static int block_info(const fw_handle* h, int32_t block, size_t* off, int* rows, size_t* esz) {
  const size_t T_ = h->precision == FW_F64 ? 8 : 4;
  switch (block) {
    case FW_BLK_ODE: *off = h->o_y; *rows = FW_NY; *esz = T_; return FW_OK;
    case FW_BLK_DERIVED: *off = h->o_der; *rows = 8; *esz = T_; return FW_OK;
    case FW_BLK_TARGET: *off = h->o_target; *rows = 3; *esz = T_; return FW_OK;
    case FW_BLK_WIND: *off = h->o_wind; *rows = 3; *esz = T_; return FW_OK;
    case FW_BLK_STEPS: *off = h->o_steps; *rows = 1; *esz = 4; return FW_OK;
    case FW_BLK_COMMAND: *off = h->o_cmd; *rows = 3; *esz = T_; return FW_OK;
    case FW_BLK_PARAMS:
      if (!h->o_prm) return set_err(FW_E_INVALID, "handle has no per-aircraft parameters (env n_rand = 0)");
      *off = h->o_prm; *rows = FW_NPARAM; *esz = T_; return FW_OK;
    case FW_BLK_ACT_RING:
      if (!h->has_env) return set_err(FW_E_INVALID, "handle has no env (no action ring)");
      *off = h->o_act; *rows = 3 * h->act_window; *esz = T_; return FW_OK;
    case FW_BLK_CMD_RING:
      if (!h->has_env || !h->cmd_window) return set_err(FW_E_INVALID, "handle keeps no command ring");
      *off = h->o_cmdring; *rows = 3 * h->cmd_window; *esz = T_; return FW_OK;
    case FW_BLK_GOAL:
      if (!h->has_env) return set_err(FW_E_INVALID, "handle has no env (no goal history)");
      *off = h->o_goal; *rows = 4; *esz = 4; return FW_OK;
    case FW_BLK_TARGET_PROPS:
      if (!h->o_tpr) return set_err(FW_E_INVALID, "handle has no linear / sinusoidal / attitude_angular targets");
      *off = h->o_tpr; *rows = h->env.ang_targets ? 15 : 12; *esz = T_; return FW_OK;
    default: return set_err(FW_E_INVALID, "unknown state block");
  }
}

int fw_block_rows(const fw_handle* h, int32_t block, int32_t* rows) {
  if (!h || !rows) return set_err(FW_E_INVALID, "NULL argument");
  size_t off, esz;
  int r;
  const int v = block_info(h, block, &off, &r, &esz);
  if (v) return v;
  *rows = r;
  return FW_OK;
}

// Blocks are exchanged densely as [rows][N].
int fw_get_state(fw_handle* h, int32_t block, void* dst_dev, void* stream) {
  if (!h || !dst_dev) return set_err(FW_E_INVALID, "NULL argument");
  size_t off, esz;
  int rows;
  int v = block_info(h, block, &off, &rows, &esz);
  if (v) return v;
  FW_HIP(hipSetDevice(h->device));
  hipStream_t st = (hipStream_t)stream;
  if (block == FW_BLK_ACT_RING || block == FW_BLK_CMD_RING) return ring_copy(h, block, off, esz, nullptr, dst_dev, 1, st);
  if (block == FW_BLK_GOAL) return goal_copy(h, nullptr, dst_dev, 1, st);
  const size_t row = align_up((size_t)h->ld * esz, 256);
  FW_HIP(hipMemcpy2DAsync(dst_dev, h->n * esz, (char*)h->base + off, row, h->n * esz, rows, hipMemcpyDeviceToDevice,
                          st));
  return FW_OK;
}

int fw_set_state(fw_handle* h, int32_t block, const void* src_dev, void* stream) {
  if (!h || !src_dev) return set_err(FW_E_INVALID, "NULL argument");
  size_t off, esz;
  int rows;
  int v = block_info(h, block, &off, &rows, &esz);
  if (v) return v;
  FW_HIP(hipSetDevice(h->device));
  hipStream_t st = (hipStream_t)stream;
  if (block == FW_BLK_ACT_RING || block == FW_BLK_CMD_RING) return ring_copy(h, block, off, esz, src_dev, nullptr, 0, st);
  if (block == FW_BLK_GOAL) return goal_copy(h, src_dev, nullptr, 0, st);
  const size_t row = align_up((size_t)h->ld * esz, 256);
  FW_HIP(hipMemcpy2DAsync((char*)h->base + off, row, src_dev, h->n * esz, h->n * esz, rows, hipMemcpyDeviceToDevice,
                          st));
  return FW_OK;
}

}  // extern "C"
#endif  // FW_HOST_PART
