// fw_device.hpp -- per-aircraft physics + env epilogue for the fused CDNA4 kernels.
//
// One lane owns one aircraft for a whole env step: the 19-element ODE state and
// the current stage input/derivative sit in per-lane LDS slots, the
// Dormand-Prince accumulators and the error estimate in VGPRs; nothing but the
// SoA state row is read or written in HBM per step.  Every
// function is __host__ __device__ so tests/native can also exercise this exact
// code on the CPU against the independent oracle (oracle/fw_oracle.c).
//
// Reference behaviour replicated (paths relative to the reference checkout):
//   PyFly._dynamics / _forces / _f_*   magpie/libs/pyfly/pyfly/pyfly.py:1450-1747
//   Variable/ControlVariable conditions pyfly.py:114-133, 312-328
//   PyFly.step save + post-step        pyfly.py:1358-1420, 1852-1881
//   scipy 1.15.3 RK45 step control     integrate/_ivp/rk.py:111-173, common.py:68-134
//   FixedWingAircraft.step epilogue    magpie/libs/fixed-wing-gym/gym_fixed_wing/fixed_wing.py:483-628
//
// Code-size rule (measured, profiles/): with one wave per SIMD the kernel is
// instruction-fetch bound as soon as its hot loop outgrows the instruction
// cache, so the integrator below contains exactly ONE inlined RHS, driven by a
// wave-uniform stage loop (initial-step probe, six stages, accept/reject).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "../../include/fwsim.h"

#define FW_HD __host__ __device__ __forceinline__

namespace fw {

// records the message returned by fw_last_error (defined in fw_kernels.hip)
int set_error(int code, const std::string& msg);

constexpr int NY = FW_NY;
constexpr double PI_D = 3.141592653589793;
// default RHS-evaluation budget per step (fw_sim_config.max_nfev): a safety net only -- scipy has no
// budget, and the steady-state bench population never comes near it (profiles/r03_nfev_census.json:
// maximum 6686 in 2.6e8 aircraft-steps).  65535 = the largest count the stats word reports, so a
// saturated nfev field and a budget hit coincide; it bounds one launch at ~30 ms of lone-aircraft work.
constexpr int MAX_NFEV = 65535;
constexpr uint32_t DM_SOLVER_FAIL = 1u << 31;  // sim_step_masked dmask bit: RK45 failed, last accepted sub-step kept
constexpr uint32_t DM_BUDGET = 1u << 30;       // ... and the failure was the max_nfev budget (not TOO_SMALL_STEP)

// per-aircraft stats word of fw_sim_step / fw_env_step (include/fwsim.h): saturated counts + failure bits
FW_HD int32_t pack_stats(int nfev, int nacc, uint32_t dmask) {
  const uint32_t nf = nfev > 0xFFFF ? 0xFFFFu : (uint32_t)nfev;
  const uint32_t na = nacc > 0x3FFF ? 0x3FFFu : (uint32_t)nacc;
  return (int32_t)(nf | (na << 16) | (dmask & (DM_SOLVER_FAIL | DM_BUDGET)));
}
#ifndef FW_Y_PREFETCH
#define FW_Y_PREFETCH 0
#endif
#ifndef FW_ER_LDS
#define FW_ER_LDS 1  // DOPRI error sum in LDS: frees 20 VGPRs of the RK loop (measured -3%)
#endif
#ifndef FW_P_LDS
#define FW_P_LDS 0  // bitmask: RK stage accumulators P3/P4/P5/YB held in LDS instead of VGPRs (fp32)
#endif
#ifndef FW_FOLD_INPLACE
#define FW_FOLD_INPLACE 1  // stage accumulators seeded at the attempt start, every stage folds in place (-1.5..3% per RK iteration, profiles/r02_ab_fold.log)
#endif
#ifndef FW_RK_UNROLL
#define FW_RK_UNROLL 1  // one-lane rk45: a trial step written out with its six RHS sites (0 = stage machine, A/B)
#endif
#if FW_RK_UNROLL && !FW_FOLD_INPLACE
#error "FW_RK_UNROLL needs FW_FOLD_INPLACE"
#endif
#ifndef FW_YF_REGS
#define FW_YF_REGS 1  // one-lane rk45: the accepted y / f in registers (AGPR room at one wave per SIMD) instead of LDS: long window -9 % (profiles/r06_lanes_sweep.log)
#endif
#if FW_YF_REGS && !FW_RK_UNROLL
#error "FW_YF_REGS needs FW_RK_UNROLL"
#endif
#ifndef FW_Q1_SIGMA_1RCP
#define FW_Q1_SIGMA_1RCP 0  // one-lane rhs(): fp32 stall blend with one reciprocal, as rhs_quad (A/B)
#endif
#ifndef FW_Q1_IVA_SEL
#define FW_Q1_IVA_SEL 0  // one-lane rhs(): 1 / Va from 1 / Va_raw where Va clips only from below (A/B)
#endif
#ifndef FW_RELAUNDER
#define FW_RELAUNDER 0  // 1: re-issue config scalar loads per RHS (helped the generic kernel; -4.5% slower on the specialised one)
#endif  // RHS evaluations per step before the step is declared a solver failure

template <typename T>
struct Lim {
  T vmin, vmax, cmin, cmax;
};

// Device-resident configuration (one copy per handle, read with scalar loads:
// every address is wave-uniform).  Precomputed products keep the RHS short.
template <typename T>
struct DevCfg {
  // ---- simulator ----
  double t_bound;            // dt
  T dt, rtol, atol;
  T half_rho, S, b, c, mass, inv_mass, mg, inv_Jy;
  T gam[9];
  T M, a0, pi_e_ar;
  T sig_c;                   // exp(2 M a0) = e^{-M(a-a0)} e^{M(a+a0)} (stall-blend constant)
  // host-folded constant products of the force model (one multiply each in the RHS)
  T qS, qSc, qSb;            // rho/2 S, rho/2 S c, rho/2 S b
  T kCLq, kCDq, kCmq, hb;    // C_L_q c/2, C_D_q c/2, C_m_q b/2 (pyfly.py:1579 uses b), b/2
  T inv_pi_e_ar, kTP2;       // 1/(pi e AR), k_T_P k_Omega^2
  T CL0, CLa, CLq, CLde, CDp, CDq, CDb1, CDb2, CDde, Cm0, Cma, Cmq, Cmde, Cmfp;
  T CY0, CYb, CYp, CYr, CYda, CYdr, Cl0, Clb, Clp, Clr, Clda, Cldr, Cn0, Cnb, Cnp, Cnr, Cnda, Cndr;
  T kmotor, prop_k, kTP, kOmega;
  T Sprop, Cprop;
  T ac[3][6];                // actuator coefs c00 c01 c02 c10 c11 c12 (ControlVariable.coefs)
  T dot_max[3];
  Lim<T> lim[FW_NVAR];
  T init_min[FW_NVAR], init_max[FW_NVAR];
  uint32_t cmask, clipmask, wrapmask;  // per fw_var: has constraint / has clip / wraps
  uint32_t dotmask;                    // per actuator: dot_max finite
  int elevon, disabled_inputs, turbulence, turb_len, wind_random;
  int max_nfev;                        // RHS-evaluation budget of one step
  int tail_quad;                       // one-lane kernels: tail handoff to lane quads at <= this many (0 = off)
  // simulator parameter randomisation (FixedWingAircraft.sample_simulator_parameters,
  // fixed_wing.py:748-813): per-aircraft parameter rows redrawn at every reset
  int rand_params;                     // 1: aircraft read their own parameter rows (State::prm)
  int n_rand;
  struct RandP {
    int param, dist, has_clip, pad;
    T orig, var, clip;
  } rp[FW_NPARAM];
  T pdef[FW_NPARAM];                   // parameter values of the un-randomised aircraft (x8_param.mat)
  T rho, grav, ar0;                    // air density, g, aspect ratio b^2/S of the config (pyfly.py:1119)
  int trig_alpha, trig_beta;           // alpha/beta limited -> use trig of the clipped angle
  int euler_exact;                     // roll/pitch/yaw limited -> Euler-angle rotation post step
  T wind_mag_min, wind_mag_max, wind_init_min[3], wind_init_max[3];
  T g0[6], g1[6], noise_scale;
  // chunks too short for the FIR (fw_sim_config.dryden_state): the shaping filters' discretised state-space
  // blocks (orders 1 2 2 1 3 3), per-aircraft state in State::dry (fw_kernels.hip turbulence_at)
  int dry_state, dry_ncut;
  T dry_ad[28], dry_e1[28], dry_b0[12], dry_b1[12], dry_c[12];
  // ---- env ----
  int has_env;
  int steps_max, n_obs, scale_actions, has_bounds, streak_req, on_success, n_rew;
  int step_fail_timesteps;
  int act_window;                      // ring length of raw actions kept (max window - 1, >= 1)
  int cmd_window;                      // ring length of commands kept (0 if unused)
  int act_need, cmd_need;              // previous actions / commands an env step reads (the rings keep one more
                                       // for fw_observe, which re-reads the newest)
  T scale_low, scale_high, bmax, bmin;
  T act_low[3], act_high[3];
  int target_class[3], target_wrap[3];
  T target_low[3], target_high[3], target_delta[3], target_bound[3];
  int has_delta[3], has_bound[3];
  // linear / sinusoidal target classes (fw_env_config ABI 11): draw bounds, np.radians factor (1 or pi/180)
  int tprops;                          // some target is linear or sinusoidal: State::tpr rows are kept
  int tape_skip;                       // env-draw tape entries before sample_target's at a reset (inert attributes)
  int ang;                             // omega_p / q / r targets of class attitude_angular (State::tpr rows 12..14)
  T ang_max_vel[3];
  T n_targets;                         // len(self.target): 3, or 6 with the attitude_angular targets
  T tgt_rad[3], tgt_slo[3], tgt_shi[3], tgt_alo[3], tgt_ahi[3], tgt_plo[3], tgt_phi[3];
  int goal_flag;                       // a success reward factor: State::gflag keeps goal_achieved
  // goal-status history ring (fw_kernels.hip GB_*): 8 x gring_words entries (a power of two >= 128 and >=
  // success_streak_req), words 16.. after the count rows; window counts as bytes, or (gcnt_wide: streak_req > 255)
  // as 16-bit fields in two words (the second at row gcnt2_row)
  uint32_t gring_mask;
  int gcnt_wide, gcnt2_row;
  T streak_frac;
  T step_fail_value;
  T term_weight[3];
  int term_present[3];
  int metrics;                         // streaming episode metrics tracked (fw_env_config.metrics)
  int reward_potential;                // reward.form "potential" (fw_env_config.reward_potential)
  int resample_every;                  // target.resample_every (fw_env_config.resample_every; 0 = never)
  int iwin;                            // integration_window (fw_env_config.integration_window; 0 = none)
  T rise_low, rise_high;
  int obs_len, obs_step, obs_hist;     // observation rows, their spacing, past rows kept (0: no history)
  int obs_noise;                       // observation.noise drawn
  int obs_general;                     // obs_len > 1 or obs_noise: observe_full instead of the plain row
  T obs_noise_mean, obs_noise_std;
  fw_obs_entry obs[FW_MAX_OBS];
  fw_rew_factor rew[FW_MAX_REW];
  static constexpr int const_limits = 0;  // (SpecCfg views: limit values compile-time constants)
};

// Compile-time specialisations of a configuration's STRUCTURE (which variables
// carry constraints / clips / wraps, which actuators have a rate limit, elevon
// mixing, trig flags).  The values stay in DevCfg (runtime); a SpecCfg view
// hides the structural fields with constants of the same name, so cond() and
// the RHS compile to straight-line code containing only the checks this
// configuration has.  The host picks the instance whose structure equals the
// runtime one (fw_kernels.hip: spec_of), else the generic DevCfg instance.
template <typename T, uint32_t CM, uint32_t CLM, uint32_t WM, uint32_t DM, int ELEVON, int TA, int TB, int EE>
struct SpecCfg : DevCfg<T> {
  static constexpr uint32_t cmask = CM, clipmask = CLM, wrapmask = WM, dotmask = DM;
  static constexpr int elevon = ELEVON, trig_alpha = TA, trig_beta = TB, euler_exact = EE;
  static constexpr int obs_general = 0;  // specialisations serve plain length-1, noise-free observations
  static constexpr int ang = 0;          // ... and the three targets roll / pitch / Va
  static constexpr int const_limits = 0;  // limit values compile-time constants too (see GymX8Cfg)
  static constexpr int const_params = 0;  // airframe constants compile-time too
  static constexpr int rand_params = 0;  // ... with one parameter set for all aircraft
};
// The limit VALUES of the two shipped configurations as compile-time constants as well (the host
// selects a specialisation only if every runtime value equals these bit for bit): the conditions then
// compare against immediates instead of ~20 config scalars that do not fit the SGPR budget next to
// the rest of the loop (they were spilled to VGPR lanes and re-read every RHS, v_readlane).
#ifndef FW_CONST_CFG
#define FW_CONST_CFG 2  // 0: runtime values only; 1: + limit values; 2: + airframe constants (fw_x8_consts.inc)
#endif
#include "fw_x8_consts.inc"
#define FW_X8_MEMBER(name, val) static constexpr T name = (T)(val);
#define FW_INF_ __builtin_inf()
#define FW_X8_LIMS(OM, VACMAX)                                                                          \
  {{(T)-FW_INF_, (T)FW_INF_, (T)-FW_INF_, (T)FW_INF_}, {(T)-FW_INF_, (T)FW_INF_, (T)-FW_INF_, (T)FW_INF_}, \
   {(T)-FW_INF_, (T)FW_INF_, (T)-FW_INF_, (T)FW_INF_}, {(T)-FW_INF_, (T)FW_INF_, (T)-(OM), (T)(OM)},          \
   {(T)-FW_INF_, (T)FW_INF_, (T)-(OM), (T)(OM)},       {(T)-FW_INF_, (T)FW_INF_, (T)-(OM), (T)(OM)},          \
   {(T)-FW_INF_, (T)FW_INF_, (T)-FW_INF_, (T)FW_INF_}, {(T)-FW_INF_, (T)FW_INF_, (T)-FW_INF_, (T)FW_INF_}, \
   {(T)-FW_INF_, (T)FW_INF_, (T)-FW_INF_, (T)FW_INF_}, {(T)-FW_INF_, (T)FW_INF_, (T)-FW_INF_, (T)FW_INF_}, \
   {(T)-FW_INF_, (T)FW_INF_, (T)-FW_INF_, (T)FW_INF_}, {(T)-FW_INF_, (T)FW_INF_, (T)-FW_INF_, (T)FW_INF_}, \
   {(T)0x1.0c6f7a0b5ed8dp-20, (T)FW_INF_, (T)-FW_INF_, (T)(VACMAX)},                                       \
   {(T)-FW_INF_, (T)FW_INF_, (T)-FW_INF_, (T)FW_INF_}, {(T)-FW_INF_, (T)FW_INF_, (T)-FW_INF_, (T)FW_INF_}, \
   {(T)-0x1.0c152382d7365p-1, (T)0x1.38c35418a5bf6p-1, (T)-FW_INF_, (T)FW_INF_},                           \
   {(T)-0x1.0c152382d7365p-1, (T)0x1.38c35418a5bf6p-1, (T)-FW_INF_, (T)FW_INF_},                           \
   {(T)0.0, (T)1.0, (T)-FW_INF_, (T)FW_INF_},                                                               \
   {(T)-0x1.0c152382d7365p-1, (T)0x1.38c35418a5bf6p-1, (T)-FW_INF_, (T)FW_INF_},                           \
   {(T)-0x1.226c3bcdbe7aep-1, (T)0x1.226c3bcdbe7aep-1, (T)-FW_INF_, (T)FW_INF_},                           \
   {(T)0.0, (T)1.0, (T)-FW_INF_, (T)FW_INF_}}
// fixed_wing_config.json (gym): omega +-720 deg/s and Va <= 70 constrained; Va, actuators,
// elevator / aileron / throttle clipped; roll / yaw wrapped; elevon rate limits 200 deg/s
template <typename T>
struct GymX8Cfg : SpecCfg<T, 0x1038u, 0x1F9000u, 0x5u, 0x3u, 1, 0, 0, 0> {
#if FW_CONST_CFG >= 1
  static constexpr int const_limits = 1;
  static constexpr Lim<T> lim[FW_NVAR] = FW_X8_LIMS(0x1.921fb54442d18p+3, 0x1.1800000000000p+6);
  static constexpr T dot_max[3] = {(T)0x1.becf41f212d77p+1, (T)0x1.becf41f212d77p+1, (T)FW_INF_};
#endif
#if FW_CONST_CFG >= 2
  static constexpr int const_params = 1;
  FW_X8_SCALARS(FW_X8_MEMBER)
  static constexpr T gam[9] = FW_X8_GAM;
  static constexpr T ac[3][6] = FW_X8_AC;
#endif
};
// pyfly_config.json: omega +-180 deg/s, no Va constraint, otherwise as above
template <typename T>
struct PyflyX8Cfg : SpecCfg<T, 0x38u, 0x1F9000u, 0x5u, 0x3u, 1, 0, 0, 0> {
#if FW_CONST_CFG >= 1
  static constexpr int const_limits = 1;
  static constexpr Lim<T> lim[FW_NVAR] = FW_X8_LIMS(0x1.921fb54442d18p+1, FW_INF_);
  static constexpr T dot_max[3] = {(T)0x1.becf41f212d77p+1, (T)0x1.becf41f212d77p+1, (T)FW_INF_};
#endif
#if FW_CONST_CFG >= 2
  static constexpr int const_params = 1;
  FW_X8_SCALARS(FW_X8_MEMBER)
  static constexpr T gam[9] = FW_X8_GAM;
  static constexpr T ac[3][6] = FW_X8_AC;
#endif
};
#undef FW_X8_LIMS

// Re-materialise the (wave-uniform) config pointer so the scalar loads of the
// ~90 aircraft constants are issued where they are used instead of being
// hoisted out of the RK loop and pinned in SGPRs (which spills them into VGPR
// lanes).  s_load from the scalar cache costs nothing next to the VALU work.
template <typename C>
FW_HD const C& relaunder(const C& c) {
#if defined(__HIP_DEVICE_COMPILE__) && FW_RELAUNDER
  using CPtr = const __attribute__((address_space(4))) C*;
  CPtr q = (CPtr)(&c);
  asm volatile("" : "+s"(q));
  return *(const C*)q;
#else
  return c;
#endif
}

// ---------------------------------------------------------------------------
// arithmetic helpers.  fp64 = IEEE-exact (the parity build); fp32 = the
// hardware single-instruction forms (v_rcp_f32 / v_sqrt_f32 / v_exp_f32 /
// v_log_f32, ~1 ulp) instead of the multi-instruction correctly-rounded
// sequences: an fp32 trajectory differs from fp64 at the 1e-7 level anyway.
// ---------------------------------------------------------------------------
FW_HD double fdiv(double a, double b) { return a / b; }
FW_HD double frcp(double a) { return 1.0 / a; }
FW_HD double fsqrt(double a) { return sqrt(a); }
FW_HD double fexp(double a) { return exp(a); }
FW_HD double fpow(double a, double p) { return pow(a, p); }
FW_HD float frcp(float a) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_rcpf(a);
#else
  return 1.0f / a;
#endif
}
FW_HD float fdiv(float a, float b) { return a * frcp(b); }
FW_HD float fsqrt(float a) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_sqrtf(a);
#else
  return sqrtf(a);
#endif
}
FW_HD float fexp(float a) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_exp2f(a * 1.4426950408889634f);
#else
  return expf(a);
#endif
}
FW_HD float fpow(float a, float p) {  // a > 0
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_exp2f(p * __builtin_amdgcn_logf(a));
#else
  return powf(a, p);
#endif
}

// max / min of |a|, |b| as ONE v_max_f32 / v_min_f32 with abs source modifiers.  fmaxf / fminf (and
// v_med3 against +-inf, which the backend folds back into them) canonicalise each input first in IEEE
// mode: three instructions for what the hardware does in one (NaN behaviour is the same: the other input).
FW_HD float fmax_abs(float a, float b) {
#if defined(__HIP_DEVICE_COMPILE__)
  float r;
  asm("v_max_f32_e64 %0, |%1|, |%2|" : "=v"(r) : "v"(a), "v"(b));
  return r;
#else
  return fmaxf(fabsf(a), fabsf(b));
#endif
}
FW_HD float fmin_abs(float a, float b) {
#if defined(__HIP_DEVICE_COMPILE__)
  float r;
  asm("v_min_f32_e64 %0, |%1|, |%2|" : "=v"(r) : "v"(a), "v"(b));
  return r;
#else
  return fminf(fabsf(a), fabsf(b));
#endif
}
FW_HD double fmax_abs(double a, double b) { return fmax(fabs(a), fabs(b)); }

// atan2 for the RHS.  fp64: libm.  fp32: octant reduction + a degree-8 polynomial
// in t^2 for atan(t), t in [0, 1] (fitted by tools/atan_fit in DESIGN.md; max abs
// error 1.0e-7 rad, i.e. ~1 ulp at pi/4) -- ~20 instructions instead of the ~45 of
// the correctly-rounded library routine, which matters because every RHS needs two.
FW_HD double fatan2(double y, double x) { return atan2(y, x); }
FW_HD float fatan2(float y, float x) {
#if defined(__HIP_DEVICE_COMPILE__)
  const float mx = fmax_abs(x, y), mn = fmin_abs(x, y);
  const float t = mn * __builtin_amdgcn_rcpf(mx);
  const float q = t * t;
  float p = 0.0029030926525592804f;
  p = fmaf(p, q, -0.016281209886074066f);
  p = fmaf(p, q, 0.043036505579948425f);
  p = fmaf(p, q, -0.07533437758684158f);
  p = fmaf(p, q, 0.10654566437005997f);
  p = fmaf(p, q, -0.14207105338573456f);
  p = fmaf(p, q, 0.19993050396442413f);
  p = fmaf(p, q, -0.3333309292793274f);
  p = fmaf(p, q, 1.0f);
  float r = t * p;
  r = fabsf(y) > fabsf(x) ? 1.5707963267948966f - r : r;
  r = x < 0.0f ? 3.141592653589793f - r : r;
  r = mx == 0.0f ? 0.0f : r;
  return copysignf(r, y);
#else
  return atan2f(y, x);
#endif
}

// Two atan2 at once (the one-lane RHS needs alpha and beta): the same function as fatan2, the
// polynomial of both run as packed pairs (v_pk_fma_f32: one instruction per degree for the two).
FW_HD void fatan2_2(double y0, double x0, double y1, double x1, double& r0, double& r1) {
  r0 = atan2(y0, x0);
  r1 = atan2(y1, x1);
}
FW_HD void fatan2_2(float y0, float x0, float y1, float x1, float& r0, float& r1) {
#if defined(__HIP_DEVICE_COMPILE__)
  typedef float F2 __attribute__((ext_vector_type(2)));
  const float mx0 = fmax_abs(x0, y0), mn0 = fmin_abs(x0, y0);
  const float mx1 = fmax_abs(x1, y1), mn1 = fmin_abs(x1, y1);
  F2 t;
  t.x = mn0 * __builtin_amdgcn_rcpf(mx0);
  t.y = mn1 * __builtin_amdgcn_rcpf(mx1);
  const F2 q = t * t;
  F2 p = q * 0.0029030926525592804f + -0.016281209886074066f;
  p = p * q + 0.043036505579948425f;
  p = p * q + -0.07533437758684158f;
  p = p * q + 0.10654566437005997f;
  p = p * q + -0.14207105338573456f;
  p = p * q + 0.19993050396442413f;
  p = p * q + -0.3333309292793274f;
  p = p * q + 1.0f;
  const F2 rr = t * p;
  float a0 = rr.x, a1 = rr.y;
  a0 = fabsf(y0) > fabsf(x0) ? 1.5707963267948966f - a0 : a0;
  a1 = fabsf(y1) > fabsf(x1) ? 1.5707963267948966f - a1 : a1;
  a0 = x0 < 0.0f ? 3.141592653589793f - a0 : a0;
  a1 = x1 < 0.0f ? 3.141592653589793f - a1 : a1;
  a0 = mx0 == 0.0f ? 0.0f : a0;
  a1 = mx1 == 0.0f ? 0.0f : a1;
  r0 = copysignf(a0, y0);
  r1 = copysignf(a1, y1);
#else
  r0 = fatan2(y0, x0);
  r1 = fatan2(y1, x1);
#endif
}

// ---------------------------------------------------------------------------
// small helpers
// ---------------------------------------------------------------------------
FW_HD bool any_lane(bool p) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_ballot_w64(p) != 0;  // an SGPR mask test (the __any form round-trips through a VGPR)
#else
  return p;
#endif
}

template <typename T>
FW_HD T sgn(T x) {
  return (T)((x > T(0)) - (x < T(0)));
}

template <typename T>
FW_HD T clipv(T x, T lo, T hi) {
  // np.clip for every non-NaN x in one v_med3_f32 (fp32) / v_max+v_min (fp64).  A NaN x
  // clamps to lo instead of propagating: NaN states fail the step via the step-size
  // control anyway (rk45: !(h_abs >= min_step)).
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (sizeof(T) == 4) {
    if (__builtin_constant_p(hi) && hi == __builtin_inff()) {
      // a lower bound only (a constant +inf upper bound of a specialised configuration): the backend turns
      // the med3 into fmaxf, which canonicalises x first in IEEE mode -- one v_max instead of two
      float r;
      asm("v_max_f32_e64 %0, %1, %2" : "=v"(r) : "v"(x), "v"(lo));
      return r;
    }
    return __builtin_amdgcn_fmed3f(x, lo, hi);
  }
#endif
  return fmin(fmax(x, lo), hi);
}

// Variable.apply_conditions (pyfly.py:114-133).  Records the first violation.
template <typename T, typename C>
FW_HD T cond(const C& c, int v, T x, int& term) {
  const uint32_t bit = 1u << v;
  if (c.cmask & bit) {  // branch-free: first violation wins
    const bool viol = (x < c.lim[v].cmin) | (x > c.lim[v].cmax);
    term = (term == 0 && viol) ? FW_TERM_VAR(v) : term;
  }
  if (c.clipmask & bit) x = clipv(x, c.lim[v].vmin, c.lim[v].vmax);
  if (c.wrapmask & bit) {
    const T pi = T(PI_D);
    if (fabs(x) > pi) x = sgn(x) * (fmod(fabs(x), pi) - pi);
  }
  return x;
}

// Philox4x32-10 counter-based RNG (Salmon et al., SC'11).
FW_HD void philox(uint32_t k0, uint32_t k1, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t out[4]) {
#pragma unroll
  for (int r = 0; r < 10; r++) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    c0 = hi1 ^ c1 ^ k0;
    c1 = lo1;
    c2 = hi0 ^ c3 ^ k1;
    c3 = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  out[0] = c0;
  out[1] = c1;
  out[2] = c2;
  out[3] = c3;
}

// uniform in (0, 1]: 32 random bits
template <typename T>
FW_HD T u01(uint32_t x) {
  return (T)((double)x * 2.3283064365386963e-10 + 1.1641532182693481e-10);
}

// 4 standard normals from one Philox block (Box-Muller)
template <typename T>
FW_HD void normal4(const uint32_t r[4], T z[4]) {
  const double two_pi = 6.283185307179586;
  for (int k = 0; k < 2; k++) {
    double u1 = (double)r[2 * k] * 2.3283064365386963e-10 + 1.1641532182693481e-10;
    double u2 = (double)r[2 * k + 1] * 2.3283064365386963e-10;
    T rad = (T)sqrt(-2.0 * log(u1));
    T ang = (T)(two_pi * u2);
    z[2 * k] = rad * cos(ang);
    z[2 * k + 1] = rad * sin(ang);
  }
}

// ---------------------------------------------------------------------------
// per-step context held constant across RK stages
// ---------------------------------------------------------------------------
template <typename T>
struct StepCtx {
  T sp[3];      // constrained dynamics set-points
  T wind[3];    // steady wind (vehicle frame)
  T tl[3];      // turbulence, linear (body)  -- ZOH over the step (pyfly.py:1502, 1839)
  T ta[3];      // turbulence, angular
  T elev0, ail0;  // stored elevator/aileron .value used by the t == 0 evaluation
};

// wind_b = R(q)·w + turb (quaternion branch of _rot_b_v, pyfly.py:1780-1800; 1843)
template <typename T>
FW_HD void airspeed_vec(const T* q, const T* w, const T* tl, const T* v, T va[3]) {
  const T e0 = q[0], e1 = q[1], e2 = q[2], e3 = q[3];
  const T R00 = T(-1) + T(2) * (e0 * e0 + e1 * e1), R01 = T(2) * (e1 * e2 + e3 * e0), R02 = T(2) * (e1 * e3 - e2 * e0);
  const T R10 = T(2) * (e1 * e2 - e3 * e0), R11 = T(-1) + T(2) * (e0 * e0 + e2 * e2), R12 = T(2) * (e2 * e3 + e1 * e0);
  const T R20 = T(2) * (e1 * e3 + e2 * e0), R21 = T(2) * (e2 * e3 - e1 * e0), R22 = T(-1) + T(2) * (e0 * e0 + e3 * e3);
  va[0] = v[0] - (R00 * w[0] + R01 * w[1] + R02 * w[2] + tl[0]);
  va[1] = v[1] - (R10 * w[0] + R11 * w[1] + R12 * w[2] + tl[1]);
  va[2] = v[2] - (R20 * w[0] + R21 * w[1] + R22 * w[2] + tl[2]);
}

// Euler branch of _rot_b_v (pyfly.py:1757-1777) -- used post step when the Euler
// angles may have been clipped (otherwise R(q_normalised) is the same matrix).
template <typename T>
FW_HD void airspeed_vec_euler(T phi, T th, T psi, const T* w, const T* tl, const T* v, T va[3]) {
  const T cph = cos(phi), sph = sin(phi), cth = cos(th), sth = sin(th), cps = cos(psi), sps = sin(psi);
  const T R00 = cth * cps, R01 = cth * sps, R02 = -sth;
  const T R10 = sph * sth * cps - cph * sps, R11 = sph * sth * sps + cph * cps, R12 = sph * cth;
  const T R20 = cph * sth * cps + sph * sps, R21 = cph * sth * sps - sph * cps, R22 = cph * cth;
  va[0] = v[0] - (R00 * w[0] + R01 * w[1] + R02 * w[2] + tl[0]);
  va[1] = v[1] - (R10 * w[0] + R11 * w[1] + R12 * w[2] + tl[1]);
  va[2] = v[2] - (R20 * w[0] + R21 * w[1] + R22 * w[2] + tl[2]);
}

// ---------------------------------------------------------------------------
// RHS: PyFly._dynamics (pyfly.py:1450-1482).  first == (t == 0): the stored,
// already-conditioned state is used as is; otherwise the stage vector is
// conditioned first (_set_states_from_ode_solution(save=False)), which can
// terminate the step.  Returns the first violated condition (0 = none).
// ---------------------------------------------------------------------------
// `a` supplies the parameter-derived constants (qS, C_L_0, mass, ...): the config itself (same
// field names, uniform) or a per-aircraft AeroP when simulator parameters are randomised.
template <typename T, typename C, typename A>
FW_HD int rhs(const C& c0, const A& a, const StepCtx<T>& X, bool first, const T* y, T* dy) {
#ifdef FW_RHS_TRIVIAL  // ISA accounting experiment only (tools/isa_loop.sh -DFW_RHS_TRIVIAL)
  for (int i = 0; i < NY; i++) dy[i] = y[i] * X.sp[0];
  return 0;
#endif
  const C& c = relaunder(c0);
  int term = 0;
  T om[3] = {y[4], y[5], y[6]};
  T vel[3] = {y[10], y[11], y[12]};
  T av[3] = {y[13], y[14], y[15]};
  T ad[3] = {y[16], y[17], y[18]};
  T elev = X.elev0, ail = X.ail0;
  if (!first) {
#pragma unroll
    for (int i = 0; i < 3; i++) om[i] = cond(c, FW_V_OMEGA_P + i, om[i], term);
#pragma unroll
    for (int i = 0; i < 3; i++) (void)cond(c, FW_V_POS_N + i, y[7 + i], term);
#pragma unroll
    for (int i = 0; i < 3; i++) vel[i] = cond(c, FW_V_VEL_U + i, vel[i], term);
#pragma unroll
    for (int j = 0; j < 3; j++) {  // Actuation.set_states (pyfly.py:479-492)
      av[j] = cond(c, FW_V_ACT0 + j, av[j], term);
      if (c.dotmask & (1u << j)) ad[j] = clipv(ad[j], -c.dot_max[j], c.dot_max[j]);
    }
    if (c.elevon) {
      ail = (-av[0] + av[1]) * T(0.5);
      elev = (av[0] + av[1]) * T(0.5);
      ail = cond(c, FW_V_AILERON, ail, term);
      elev = cond(c, FW_V_ELEVATOR, elev, term);
    } else {
      elev = av[0];
      ail = av[1];
    }
  }
  const T thr = av[2];
  const T e0 = y[0], e1 = y[1], e2 = y[2], e3 = y[3];  // raw attitude (pyfly.py:1464)

  // ---- _forces (pyfly.py:1484-1643) ----
  // angular turbulence (0 when the config has none: turbulence_at zeroes it, and x - 0 is x exactly)
  const T p = om[0] - X.ta[0], q = om[1] - X.ta[1], r = om[2] - X.ta[2];
  T va[3];
  airspeed_vec(y, X.wind, X.tl, vel, va);
  // Va = |va|, alpha = atan2(w, u), beta = asin(v / Va) = atan2(v, sqrt(u^2 + w^2))
  // (pyfly.py:1506-1511, _calculate_airspeed_factors :1830-1850)
  const T rxz2 = va[0] * va[0] + va[2] * va[2];
  const T rxz = fsqrt(rxz2);
  const T Va_raw = fsqrt(rxz2 + va[1] * va[1]);
  T alpha, beta;
  fatan2_2(va[2], va[0], va[1], rxz, alpha, beta);
  const T Va = cond(c, FW_V_VA, Va_raw, term);
  alpha = cond(c, FW_V_ALPHA, alpha, term);
  beta = cond(c, FW_V_BETA, beta, term);

  T sa, ca, sb, cb;
  if (c.trig_alpha) {
    sa = sin(alpha);
    ca = cos(alpha);
  } else {  // sin/cos of atan2(z, x) without the transcendental
    const T irxz = frcp(rxz);
    sa = rxz2 > T(0) ? va[2] * irxz : T(0);
    ca = rxz2 > T(0) ? va[0] * irxz : T(1);
  }
  T iVr = T(0);
  if (c.trig_beta) {
    sb = sin(beta);
    cb = cos(beta);
  } else {  // sin / cos of beta = asin(v / Va): v / Va and sqrt(u^2 + w^2) / Va
    iVr = frcp(Va_raw);
    sb = va[1] * iVr;
    cb = rxz * iVr;
  }

  const T V2a = Va * Va;
  const T fg0 = a.mg * (T(2) * (e1 * e3 - e2 * e0));
  const T fg1 = a.mg * (T(2) * (e2 * e3 + e1 * e0));
  const T fg2 = a.mg * (e3 * e3 + e0 * e0 - e1 * e1 - e2 * e2);
  T ex1, ex2;
  if constexpr (sizeof(T) == 4) {  // exp(-M (alpha - a0)), exp(M (alpha + a0)) as exp2 of one fma each
    const T l2e = T(1.4426950408889634), k = a.M * l2e, k0 = a.M * a.a0 * l2e;
    if constexpr (FW_Q1_SIGMA_1RCP) {  // exponents clamped at 2^120: S + C below stays finite (rhs_quad)
      ex1 = __builtin_amdgcn_exp2f(fminf(fmaf(-k, alpha, k0), T(120)));
      ex2 = __builtin_amdgcn_exp2f(fminf(fmaf(k, alpha, k0), T(120)));
    } else {
      ex1 = __builtin_amdgcn_exp2f(fmaf(-k, alpha, k0));
      ex2 = __builtin_amdgcn_exp2f(fmaf(k, alpha, k0));
    }
  } else {
    ex1 = fexp(-a.M * (alpha - a.a0));
    ex2 = fexp(a.M * (alpha + a.a0));
  }
  // stall blend sigma = (1+e1+e2) / ((1+e1)(1+e2)) (pyfly.py:1541-1543).  Since
  // e1 e2 = exp(2 M a0) = C, the denominator is S + C with S = 1+e1+e2, so
  // sigma = 1 / (1 + C/S): the same value, but it never forms the ~1e38 product
  // (whose fp32 reciprocal flushes to 0 and flips sigma from 1 to 0 deep in
  // stall) and it is exactly 1 when an exponential overflows.  FW_Q1_SIGMA_1RCP (fp32): S / (S + C) with
  // the exponents clamped, one reciprocal (where the clamp acts C / S < 1e-15 and sigma rounds to 1 either way)
  T sigma;
  if constexpr (sizeof(T) == 4 && FW_Q1_SIGMA_1RCP) {
    const T S = T(1) + ex1 + ex2;
    sigma = S * frcp(S + a.sig_c);
  } else {
    sigma = frcp(T(1) + a.sig_c * frcp(T(1) + ex1 + ex2));
  }
  const T osig = T(1) - sigma;
  // sgn(alpha) sin(alpha)^2 = sin(alpha) |sin(alpha)|: sin has alpha's sign on [-pi, pi] and the
  // product is 0 where it does not (pyfly.py:1547-1579 multiply by np.sign(alpha))
  const T ssa = sa * fabs(sa);
  const T CLlin = a.CL0 + a.CLa * alpha;
  const T CL = osig * CLlin + sigma * (T(2) * ssa * ca);
  T iVa;
  if constexpr (FW_Q1_IVA_SEL && C::const_limits) {
    // X8 limits: Va clips only from below (at 1e-6), so Va == Va_raw unless Va_raw < vmin, and 1 / Va is the
    // reciprocal already formed for beta (the trig_beta-free branch above needs iVr)
    if (!c.trig_beta && !(c.lim[FW_V_VA].vmax < T(__builtin_inf())))  // (compile-time for the X8 views)
      iVa = Va_raw >= c.lim[FW_V_VA].vmin ? iVr : T(1) / c.lim[FW_V_VA].vmin;  // Va = max(Va_raw, vmin)
    else
      iVa = frcp(Va);
  } else {
    iVa = frcp(Va);
  }
  const T qn = q * iVa;  // q / Va
  // lift / drag / pitch moment per unit dynamic pressure (pyfly.py:1529-1579)
  const T flift = a.qS * V2a * (CL + a.kCLq * qn + a.CLde * elev);
  const T CD = a.CDp + osig * (CLlin * CLlin) * a.inv_pi_e_ar + sigma * (T(2) * (ssa * sa));
  const T CDb = a.CDb1 * beta + a.CDb2 * beta * beta;
  const T fdrag = a.qS * V2a * (CD + CDb + a.kCDq * qn + a.CDde * elev * elev);
  const T Cm = osig * (a.Cm0 + a.Cma * alpha) + sigma * (a.Cmfp * ssa);
  const T mm = a.qSc * V2a * (Cm + a.kCmq * qn + a.Cmde * elev);
  const T bp = a.hb * p * iVa, br = a.hb * r * iVa;
  const T fy = a.qS * V2a * (a.CY0 + a.CYb * beta + a.CYp * bp + a.CYr * br + a.CYda * ail);
  const T ll = a.qSb * V2a * (a.Cl0 + a.Clb * beta + a.Clp * bp + a.Clr * br + a.Clda * ail);
  const T nn = a.qSb * V2a * (a.Cn0 + a.Cnb * beta + a.Cnp * bp + a.Cnr * br + a.Cnda * ail);
  // f_aero = R_euler(0, alpha, beta) . [-D, Y, -L] = R_alpha . (R_beta . [-D, Y, -L])
  const T U = cb * (-fdrag) + sb * fy;
  const T fa0 = ca * U + sa * flift;
  const T fa1 = sb * fdrag + cb * fy;
  const T fa2 = sa * U - ca * flift;
  const T Vd = Va + thr * (a.kmotor - Va);
  const T fprop = a.prop_k * Vd * (Vd - Va);
  const T tprop = -a.kTP2 * (thr * thr);
  const T f0 = fprop + fg0 + fa0, f1 = fg1 + fa1, f2 = fg2 + fa2;
  const T t0 = ll + tprop, t1 = mm, t2 = nn;

  const T P0 = om[0], Q0 = om[1], R0 = om[2];
  // _f_attitude_dot (pyfly.py:1645-1657)
  dy[0] = T(0.5) * (-P0 * e1 - Q0 * e2 - R0 * e3);
  dy[1] = T(0.5) * (P0 * e0 + R0 * e2 - Q0 * e3);
  dy[2] = T(0.5) * (Q0 * e0 - R0 * e1 + P0 * e3);
  dy[3] = T(0.5) * (R0 * e0 + Q0 * e1 - P0 * e2);
  // _f_omega_dot (pyfly.py:1659-1683)
  dy[4] = c.gam[1] * P0 * Q0 - c.gam[2] * Q0 * R0 + c.gam[3] * t0 + c.gam[4] * t2;
  dy[5] = c.gam[5] * P0 * R0 - c.gam[6] * (P0 * P0 - R0 * R0) + t1 * c.inv_Jy;
  dy[6] = c.gam[7] * P0 * Q0 - c.gam[1] * Q0 * R0 + c.gam[4] * t0 + c.gam[8] * t2;
  // _f_p_dot (pyfly.py:1706-1737)
  dy[7] = (e1 * e1 + e0 * e0 - e2 * e2 - e3 * e3) * vel[0] + T(2) * (e1 * e2 - e3 * e0) * vel[1] +
          T(2) * (e1 * e3 + e2 * e0) * vel[2];
  dy[8] = T(2) * (e1 * e2 + e3 * e0) * vel[0] + (e2 * e2 + e0 * e0 - e1 * e1 - e3 * e3) * vel[1] +
          T(2) * (e2 * e3 - e1 * e0) * vel[2];
  dy[9] = T(2) * (e1 * e3 - e2 * e0) * vel[0] + T(2) * (e2 * e3 + e1 * e0) * vel[1] +
          (e3 * e3 + e0 * e0 - e1 * e1 - e2 * e2) * vel[2];
  // _f_v_dot (pyfly.py:1685-1704)
  dy[10] = R0 * vel[1] - Q0 * vel[2] + f0 * a.inv_mass;
  dy[11] = P0 * vel[2] - R0 * vel[0] + f1 * a.inv_mass;
  dy[12] = Q0 * vel[0] - P0 * vel[1] + f2 * a.inv_mass;
  // Actuation.rhs (pyfly.py:519-543)
#pragma unroll
  for (int j = 0; j < 3; j++) {
    dy[13 + j] = av[j] * c.ac[j][0] + X.sp[j] * c.ac[j][2] + ad[j] * c.ac[j][1];
    dy[16 + j] = av[j] * c.ac[j][3] + X.sp[j] * c.ac[j][5] + ad[j] * c.ac[j][4];
  }
  return term;
}

// ---------------------------------------------------------------------------
// scipy RK45 (Dormand-Prince 5(4), FSAL) integrating y from 0 to dt with the
// solve_ivp default controller; t/h bookkeeping in fp64 for both precisions so
// the step-size sequence follows scipy's.
//
// Each lane runs its own phase machine around ONE rhs() evaluation per loop
// iteration:  phase 0  f0 = f(0, y0)                       (RungeKutta.__init__)
//             phase 1  probe f(h0, y0 + h0 f0)             (select_initial_step)
//             phase 2..7  stage s = phase - 1 of an attempt, s = 6 is f(t_new, y_new)
// Stage vectors are folded into running sums as soon as they are produced
// (P_s = sum_j A[s][j] K_j for the stages to come, YB = sum_j B_j K_j,
// ER = sum_j E_j K_j); per element the sums run j = 0, 1, ... as scipy's
// np.dot(K[:s].T, a[:s]) (rk.py:58-64).
// ---------------------------------------------------------------------------

// Each wave walks ONE uniform sequence of RHS evaluations -- f0, the initial
// step probe, then stages 1..6 of trial steps -- around a single inlined rhs()
// call; lanes whose integration has finished (or terminated) sit masked.  The
// stage index is wave-uniform, so every Butcher coefficient is a scalar
// literal and each stage's fold is straight-line code.  Stage vectors are
// folded into running sums as soon as they are produced (P_s = sum_j A[s][j]
// K_j for the stages to come, YB = sum_j B_j K_j, ER = sum_j E_j K_j); per
// element the sums run j = 0, 1, ... as scipy's np.dot(K[:s].T, a[:s])
// (rk.py:58-64).
// Pair layout: the 19-element state is processed as NP = 10 two-element
// vectors (element 19 is a zero pad), so fp32 folds issue as packed
// v_pk_fma_f32 / v_pk_mul_f32 (two elements per instruction) and the LDS slots
// move 8 bytes per access.  fp64 uses the same code (scalarised by the backend).
template <typename T>
using V2 = T __attribute__((ext_vector_type(2)));
constexpr int NP = (NY + 1) / 2;

// LDS slots (pairs per lane) the integrator needs: y, f, error sum, stage accumulators
template <typename T>
constexpr int lds_slots() {
  return 2 + FW_ER_LDS + ((sizeof(T) == 4 && FW_P_LDS) ? 4 : 0);
}

// Dormand-Prince 5(4) tableau (scipy rk.py RK45.A / B / E)
namespace dp5 {
constexpr double A10 = 1.0 / 5;
constexpr double A20 = 3.0 / 40, A21 = 9.0 / 40;
constexpr double A30 = 44.0 / 45, A31 = -56.0 / 15, A32 = 32.0 / 9;
constexpr double A40 = 19372.0 / 6561, A41 = -25360.0 / 2187, A42 = 64448.0 / 6561, A43 = -212.0 / 729;
constexpr double A50 = 9017.0 / 3168, A51 = -355.0 / 33, A52 = 46732.0 / 5247, A53 = 49.0 / 176, A54 = -5103.0 / 18656;
constexpr double B0 = 35.0 / 384, B2 = 500.0 / 1113, B3 = 125.0 / 192, B4 = -2187.0 / 6784, B5 = 11.0 / 84;
constexpr double E0 = -71.0 / 57600, E2 = 71.0 / 16695, E3 = -71.0 / 1920, E4 = 17253.0 / 339200, E5 = -22.0 / 525,
                 E6 = 1.0 / 40;
}  // namespace dp5

// scipy's min_step = 10 * np.abs(np.nextafter(t, np.inf) - t) (rk.py:116) for t in [0, t_bound]:
// on the device from the exponent (v_frexp_exp / v_ldexp, 3 instructions) instead of libm's nextafter
// (~25): for normal t = m 2^e, m in [0.5, 1), the spacing above t is 2^(e - 53); at t = 0 it is the
// smallest subnormal.  t never lies in (0, 2^-1022): steps start at h0 >= ~1e-300.
FW_HD double min_step_at(double t) {
#if defined(__HIP_DEVICE_COMPILE__)
  return t > 0.0 ? 10.0 * __builtin_amdgcn_ldexp(1.0, __builtin_amdgcn_frexp_exp(t) - 53) : 10.0 * 0x1p-1074;
#else
  return 10.0 * fabs(nextafter(t, 1e300) - t);
#endif
}

#include "fw_quad.hpp"
#include "fw_pair.hpp"

#ifndef FW_TAIL_QUAD
#define FW_TAIL_QUAD 16  // one-lane waves hand their last <= this many integrating aircraft to lane quads (0 = off)
#endif

// HO: tail handoff (one-wave blocks, stride = 64): once at most FW_TAIL_QUAD aircraft of the wave are
// still integrating, at the start of a trial step, they continue on lane quads of the same wave
// (qd::handoff, fw_quad.hpp; ho = the block's handoff slots in LDS) -- the straggler tail at the
// quad integrator's per-evaluation latency instead of the one-lane one.
template <typename T, typename C, typename A, bool HO = false, bool YF = true>
FW_HD int rk45(const C& c, const A& a, const StepCtx<T>& X, T* y_io, V2<T>* __restrict__ sy, V2<T>* __restrict__ sf, int stride,
               int& nfev, int& nacc, V2<T>* __restrict__ se = nullptr, void* ho = nullptr) {
  using V = V2<T>;
  using namespace dp5;
  const T rtol = c.rtol, atol = c.atol;
  const double t_bound = c.t_bound;
  const T inv_sqrt_n = T(0.22941573387056177);  // 1 / sqrt(19)

  // y and f (the accepted state and its derivative) live in LDS slots of this
  // lane (pair p at s[p * stride]); the stage accumulators stay in VGPRs.
  // FW_YF_REGS (fp32): in registers instead (written to the LDS slots before a tail handoff, which reads them there)
  constexpr bool YFR = FW_YF_REGS && sizeof(T) == 4 && YF;  // (fp64: the instances already spill; not measured)
  V Yr[YFR ? NP : 1], Fr[YFR ? NP : 1];
  auto Yp = [&](int p) -> V& {
    if constexpr (YFR) return Yr[p];
    else return sy[p * stride];
  };
  auto Fp = [&](int p) -> V& {
    if constexpr (YFR) return Fr[p];
    else return sf[p * stride];
  };
#define Y(p) Yp(p)
#define F(p) Fp(p)
#if FW_ER_LDS
  // error accumulator in this lane's third LDS slot (registers go to the live stage vectors)
#define ERV(p) se[(p) * stride]
  V ys[NP], K[NP];
#else
  V ER[NP], ys[NP], K[NP];
#define ERV(p) ER[p]
#endif
  // stage accumulators P3, P4, P5, YB (k = 0..3): VGPRs, or (fp32, bit k of FW_P_LDS) four more
  // LDS slots of this lane after the error sum (the kernels size their LDS with lds_slots<T>())
  constexpr unsigned PL = sizeof(T) == 4 ? (unsigned)FW_P_LDS : 0u;
  V* const sp = (se ? se : sf) + NP * stride;
  V Preg[4][NP];
#if FW_FOLD_INPLACE
  V P2v[NP];  // stage-3 input accumulator A20 K1 (+ A21 K2), seeded at the attempt start
#endif
  auto PA = [&](int k, int p) -> V& {
    if ((PL >> k) & 1u) return sp[(k * NP + p) * stride];
    return Preg[k][p];
  };
#define P3 (0)
#define P4 (1)
#define P5 (2)
#define YB (3)
#pragma unroll
  for (int p = 0; p < NP; p++) {
    V v;
    v.x = y_io[2 * p];
    v.y = 2 * p + 1 < NY ? y_io[2 * p + 1] : T(0);
    ys[p] = v;
    Y(p) = v;
  }
  double t = 0.0, h_abs = 0.0, h0 = 0.0, t_new = 0.0, min_step = 0.0;
  T ht = T(0), d1 = T(0);
  bool rejected = false, active = true;
  int result = 0;
  nfev = 0;
  nacc = 0;
  // 1 / (atol + |y| rtol) for both lanes of a pair
  auto iscale = [&](V y) {
    V r;
    r.x = frcp(atol + fabs(y.x) * rtol);
    r.y = frcp(atol + fabs(y.y) * rtol);
    return r;
  };
  auto sq2 = [](V v) { return v.x * v.x + v.y * v.y; };

  // stage: 0 = f0, 1 = probe, 2..7 = RK stage s = stage - 1 (s = 6: f(t_new, y_new)).
  // The RHS and the stage folds run on EVERY lane (finished lanes compute on
  // dead data): only the writes that define a lane's result (Y/F on accept,
  // result, counters) are predicated.  Unpredicated folds keep the stage
  // arrays in place across the wave-uniform stage switch (no phi copies).
  bool handoff = false;
#if FW_RK_UNROLL
  // The stage sequence is wave-uniform (f0, probe, then trial steps of exactly six RHS evaluations,
  // accepted or rejected; see rk45_quad_core): one trial step is written out with its six RHS sites,
  // so the accumulators have static lifetimes instead of merging at a stage switch.
  bool begin_step = false;
  // K = f(ys) at evaluation site k of a sequence that started with `nfev` evaluations done (f0 / probe:
  // k = 1 / 2 from 0; a trial step: k = 1..6 from its start, nfev += 6 at its step control).  `room` =
  // evaluations left before the max_nfev budget, set at the sequence start, so the common path is one
  // compare against the site's constant plus the violated-condition test (counting per evaluation cost ~9
  // VALU per RHS on the lone-wave tail).  A lane stops on a violated condition (result = its code) or when
  // this evaluation reaches the budget (hard bound on the work of one step so that no input can keep a wave
  // spinning; scipy has none; ends the step like its TOO_SMALL_STEP failure, reported in the stats).
  // Returns false once no lane of the wave integrates any more.  `tight` (wave-uniform): some lane may
  // reach its budget within the sequence; otherwise the common path is one ballot of the condition codes.
  int room = c.max_nfev;
  bool tight = true;
  auto eval = [&](bool first, int k) {
    const int term = rhs(c, a, X, first, (const T*)ys, (T*)K);
    K[NP - 1].y = T(0);  // pad element
    if (!tight && !any_lane(term != 0)) return true;
    const bool stop = active && (term != 0 || k >= room);
    if (any_lane(stop)) {
      if (stop) {
        result = term ? term : -2;
        nfev += k;
        active = false;
      }
      return any_lane(active);
    }
    return true;  // every lane that was integrating still is (the caller only evaluates while one is)
  };
  if (!eval(true, 1)) goto rk_done;
  {  // ---- f0; select_initial_step (common.py:68-110)
    T d0s = T(0), d1s = T(0);
#pragma unroll
    for (int p = 0; p < NP; p++) {
      F(p) = K[p];
      const V isc = iscale(Y(p));
      d0s += sq2(Y(p) * isc);
      d1s += sq2(K[p] * isc);
    }
    const T d0 = fsqrt(d0s) * inv_sqrt_n;
    d1 = fsqrt(d1s) * inv_sqrt_n;
    h0 = (d0 < T(1e-5) || d1 < T(1e-5)) ? 1e-6 : 0.01 * (double)d0 / (double)d1;
    if (h0 > t_bound) h0 = t_bound;
    const T h0t = (T)h0;
#pragma unroll
    for (int p = 0; p < NP; p++) ys[p] = Y(p) + h0t * F(p);
  }
  if (!eval(false, 2)) goto rk_done;
  if (active) nfev = 2;
  {  // ---- probe; select_initial_step (common.py:111-134)
    T d2s = T(0);
#pragma unroll
    for (int p = 0; p < NP; p++) d2s += sq2((K[p] - F(p)) * iscale(Y(p)));
    const double d2 = (double)(fsqrt(d2s) * inv_sqrt_n) / h0;
    double h1;
    if ((double)d1 <= 1e-15 && d2 <= 1e-15) h1 = fmax(1e-6, h0 * 1e-3);
    else h1 = pow(0.01 / fmax((double)d1, d2), 1.0 / 5.0);
    h_abs = fmin(fmin(100 * h0, h1), t_bound);
    begin_step = active;
  }
  for (;;) {
    if (begin_step) {  // RungeKutta._step_impl entry (rk.py:111-124)
      min_step = min_step_at(t);
      if (h_abs < min_step) h_abs = min_step;
      rejected = false;
    }
    room = c.max_nfev - nfev;
    tight = any_lane(active && room <= 6);
    {  // one trial step (rk.py:126-137); stage 1 input, accumulators seeded
      double h = h_abs;
      t_new = t + h;
      if (t_new - t_bound > 0) t_new = t_bound;
      h = t_new - t;
      h_abs = fabs(h);
      ht = (T)h;
#pragma unroll
      for (int p = 0; p < NP; p++) {
        const V f = F(p);
        ys[p] = Y(p) + (f * T(A10)) * ht;
        P2v[p] = f * T(A20);
        PA(P3, p) = f * T(A30);
        PA(P4, p) = f * T(A40);
        PA(P5, p) = f * T(A50);
        PA(YB, p) = f * T(B0);
        ERV(p) = f * T(E0);
      }
    }
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (HO && FW_TAIL_QUAD > 0) {  // every integrating lane is at the start of a trial step
      const unsigned long long am = __ballot(active);
      const int na = __popcll(am);  // (lanes of the wave's aircraft past N have returned: quads need 4 na live lanes)
      if (na > 0 && na <= c.tail_quad && 4 * na <= __popcll(__ballot(true))) {
        handoff = true;
        if constexpr (YFR) {
#pragma unroll
          for (int p = 0; p < NP; p++) {
            sy[p * stride] = Yr[p];
            sf[p * stride] = Fr[p];
          }
        }
        break;
      }
    }
#endif
    if (!eval(false, 1)) break;  // K1
#pragma unroll
    for (int p = 0; p < NP; p++) {
      ys[p] = Y(p) + (P2v[p] + K[p] * T(A21)) * ht;
      PA(P3, p) += K[p] * T(A31);
      PA(P4, p) += K[p] * T(A41);
      PA(P5, p) += K[p] * T(A51);
    }
    if (!eval(false, 2)) break;  // K2
#pragma unroll
    for (int p = 0; p < NP; p++) {
      PA(P3, p) += K[p] * T(A32);
      PA(P4, p) += K[p] * T(A42);
      PA(P5, p) += K[p] * T(A52);
      PA(YB, p) += K[p] * T(B2);
      ERV(p) += K[p] * T(E2);
      ys[p] = Y(p) + PA(P3, p) * ht;
    }
    if (!eval(false, 3)) break;  // K3
#pragma unroll
    for (int p = 0; p < NP; p++) {
      PA(P4, p) += K[p] * T(A43);
      PA(P5, p) += K[p] * T(A53);
      PA(YB, p) += K[p] * T(B3);
      ERV(p) += K[p] * T(E3);
      ys[p] = Y(p) + PA(P4, p) * ht;
    }
    if (!eval(false, 4)) break;  // K4
#pragma unroll
    for (int p = 0; p < NP; p++) {
      PA(P5, p) += K[p] * T(A54);
      PA(YB, p) += K[p] * T(B4);
      ERV(p) += K[p] * T(E4);
      ys[p] = Y(p) + PA(P5, p) * ht;
    }
    if (!eval(false, 5)) break;  // K5; ys <- y_new
#pragma unroll
    for (int p = 0; p < NP; p++) {
      PA(YB, p) += K[p] * T(B5);
      ERV(p) += K[p] * T(E5);
      ys[p] = Y(p) + ht * PA(YB, p);
    }
    if (!eval(false, 6)) break;  // K = f(t_new, y_new): error norm + step control (rk.py:138-173)
    if (active) nfev += 6;
    {
      T es = T(0);
#pragma unroll
      for (int p = 0; p < NP; p++) {
        const V e = (ERV(p) + K[p] * T(E6)) * ht;
        const V y0 = Y(p), y1 = ys[p];
        V sc;
        sc.x = frcp(atol + fmax_abs(y0.x, y1.x) * rtol);
        sc.y = frcp(atol + fmax_abs(y0.y, y1.y) * rtol);
        es += sq2(e * sc);
      }
      const T en = fsqrt(es) * inv_sqrt_n;
      begin_step = false;
      if (active) {
        if (en < T(1)) {
          double factor = (en == T(0)) ? 10.0 : fmin(10.0, 0.9 * (double)fpow(en, T(-0.2)));
          if (rejected) factor = fmin(1.0, factor);
          h_abs *= factor;
          t = t_new;
#pragma unroll
          for (int p = 0; p < NP; p++) {
            Y(p) = ys[p];
            F(p) = K[p];
          }
          nacc++;
          if (t - t_bound >= 0.0) active = false;  // OdeSolver.step: finished (base.py:203-204)
          else begin_step = true;
        } else {
          h_abs *= fmax(0.2, 0.9 * (double)fpow(en, T(-0.2)));
          rejected = true;
          if (!(h_abs >= min_step)) {  // TOO_SMALL_STEP (or a NaN step size): solver failure
            result = -1;
            active = false;
          }
        }
      }
    }
    if (!any_lane(active)) break;
  }
rk_done:
#else
  for (int stage = 0;;) {
    if (!any_lane(active)) break;
#if FW_Y_PREFETCH
    // the accepted state is read by every stage's fold: issue the LDS reads before the
    // RHS so their latency hides under it (Y changes only on accept, after the folds)
    V yv[NP];
#pragma unroll
    for (int p = 0; p < NP; p++) yv[p] = Y(p);
#define YR(p) yv[p]
#else
#define YR(p) Y(p)
#endif
    {
      const int term = rhs(c, a, X, stage == 0, (const T*)ys, (T*)K);
      K[NP - 1].y = T(0);  // pad element
      if (active) {
        nfev++;
        if (term) {
          result = term;
          active = false;
        }
        // hard bound on work per step so that no input can keep a wave spinning (scipy has
        // none; ends the step like its TOO_SMALL_STEP failure, reported in the stats)
        else if (nfev >= c.max_nfev) {
          result = -2;
          active = false;
        }
      }
    }
    bool begin_step = false, begin_attempt = false;
    if (stage == 0) {  // ---- f0; select_initial_step (common.py:68-110)
      T d0s = T(0), d1s = T(0);
#pragma unroll
      for (int p = 0; p < NP; p++) {
        F(p) = K[p];
        const V isc = iscale(Y(p));
        d0s += sq2(Y(p) * isc);
        d1s += sq2(K[p] * isc);
      }
      const T d0 = fsqrt(d0s) * inv_sqrt_n;
      d1 = fsqrt(d1s) * inv_sqrt_n;
      h0 = (d0 < T(1e-5) || d1 < T(1e-5)) ? 1e-6 : 0.01 * (double)d0 / (double)d1;
      if (h0 > t_bound) h0 = t_bound;
      const T h0t = (T)h0;
#pragma unroll
      for (int p = 0; p < NP; p++) ys[p] = Y(p) + h0t * F(p);
      stage = 1;
    } else if (stage == 1) {  // ---- probe; select_initial_step (common.py:111-134)
      T d2s = T(0);
#pragma unroll
      for (int p = 0; p < NP; p++) d2s += sq2((K[p] - F(p)) * iscale(Y(p)));
      const double d2 = (double)(fsqrt(d2s) * inv_sqrt_n) / h0;
      double h1;
      if ((double)d1 <= 1e-15 && d2 <= 1e-15) h1 = fmax(1e-6, h0 * 1e-3);
      else h1 = pow(0.01 / fmax((double)d1, d2), 1.0 / 5.0);
      h_abs = fmin(fmin(100 * h0, h1), t_bound);
      begin_step = active;
      stage = 2;
    } else if (stage == 2) {  // K = K1
#pragma unroll
      for (int p = 0; p < NP; p++) {
#if FW_FOLD_INPLACE
        ys[p] = YR(p) + (P2v[p] + K[p] * T(A21)) * ht;
        PA(P3, p) += K[p] * T(A31);
        PA(P4, p) += K[p] * T(A41);
        PA(P5, p) += K[p] * T(A51);
#else
        const V f = F(p);
        ys[p] = YR(p) + (f * T(A20) + K[p] * T(A21)) * ht;
        PA(P3, p) = f * T(A30) + K[p] * T(A31);
        PA(P4, p) = f * T(A40) + K[p] * T(A41);
        PA(P5, p) = f * T(A50) + K[p] * T(A51);
        PA(YB, p) = f * T(B0);
        ERV(p) = f * T(E0);
#endif
      }
      stage = 3;
    } else if (stage == 3) {  // K = K2
#pragma unroll
      for (int p = 0; p < NP; p++) {
        PA(P3, p) += K[p] * T(A32);
        PA(P4, p) += K[p] * T(A42);
        PA(P5, p) += K[p] * T(A52);
        PA(YB, p) += K[p] * T(B2);
        ERV(p) += K[p] * T(E2);
        ys[p] = YR(p) + PA(P3, p) * ht;
      }
      stage = 4;
    } else if (stage == 4) {  // K = K3
#pragma unroll
      for (int p = 0; p < NP; p++) {
        PA(P4, p) += K[p] * T(A43);
        PA(P5, p) += K[p] * T(A53);
        PA(YB, p) += K[p] * T(B3);
        ERV(p) += K[p] * T(E3);
        ys[p] = YR(p) + PA(P4, p) * ht;
      }
      stage = 5;
    } else if (stage == 5) {  // K = K4
#pragma unroll
      for (int p = 0; p < NP; p++) {
        PA(P5, p) += K[p] * T(A54);
        PA(YB, p) += K[p] * T(B4);
        ERV(p) += K[p] * T(E4);
        ys[p] = YR(p) + PA(P5, p) * ht;
      }
      stage = 6;
    } else if (stage == 6) {  // K = K5; ys <- y_new
#pragma unroll
      for (int p = 0; p < NP; p++) {
        PA(YB, p) += K[p] * T(B5);
        ERV(p) += K[p] * T(E5);
        ys[p] = YR(p) + ht * PA(YB, p);
      }
      stage = 7;
    } else {  // K = f(t_new, y_new): error norm + step control (rk.py:138-173)
      T es = T(0);
#pragma unroll
      for (int p = 0; p < NP; p++) {
        const V e = (ERV(p) + K[p] * T(E6)) * ht;
        const V y0 = YR(p), y1 = ys[p];
        V sc;
        sc.x = frcp(atol + fmax_abs(y0.x, y1.x) * rtol);
        sc.y = frcp(atol + fmax_abs(y0.y, y1.y) * rtol);
        es += sq2(e * sc);
      }
      const T en = fsqrt(es) * inv_sqrt_n;
      if (active) {
        if (en < T(1)) {
          double factor = (en == T(0)) ? 10.0 : fmin(10.0, 0.9 * (double)fpow(en, T(-0.2)));
          if (rejected) factor = fmin(1.0, factor);
          h_abs *= factor;
          t = t_new;
#pragma unroll
          for (int p = 0; p < NP; p++) {
            Y(p) = ys[p];
            F(p) = K[p];
          }
          nacc++;
          if (t - t_bound >= 0.0) active = false;  // OdeSolver.step: finished (base.py:203-204)
          else begin_step = true;
        } else {
          h_abs *= fmax(0.2, 0.9 * (double)fpow(en, T(-0.2)));
          rejected = true;
          if (!(h_abs >= min_step)) {  // TOO_SMALL_STEP (or a NaN step size): solver failure
            result = -1;
            active = false;
          } else {
            begin_attempt = true;
          }
        }
      }
      stage = 2;
    }
    if (begin_step) {  // RungeKutta._step_impl entry (rk.py:111-124)
      min_step = min_step_at(t);
      if (h_abs < min_step) h_abs = min_step;
      rejected = false;
      begin_attempt = true;
    }
    if (begin_attempt) {  // one trial step (rk.py:126-137); stage 1 input
      double h = h_abs;
      t_new = t + h;
      if (t_new - t_bound > 0) t_new = t_bound;
      h = t_new - t;
      h_abs = fabs(h);
      ht = (T)h;
#pragma unroll
      for (int p = 0; p < NP; p++) {
        const V f = F(p);
        ys[p] = Y(p) + (f * T(A10)) * ht;
#if FW_FOLD_INPLACE
        P2v[p] = f * T(A20);
        PA(P3, p) = f * T(A30);
        PA(P4, p) = f * T(A40);
        PA(P5, p) = f * T(A50);
        PA(YB, p) = f * T(B0);
        ERV(p) = f * T(E0);
#endif
      }
    }
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (HO && FW_TAIL_QUAD > 0) {
      if (stage == 2) {  // every integrating lane is at the start of a trial step
        const unsigned long long am = __ballot(active);
        const int na = __popcll(am);  // (lanes of the wave's aircraft past N have returned: quads need 4 na live lanes)
        if (na > 0 && na <= c.tail_quad && 4 * na <= __popcll(__ballot(true))) {
          handoff = true;
          break;
        }
      }
    }
#endif
  }
#endif  // FW_RK_UNROLL
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (HO && FW_TAIL_QUAD > 0) {
    if (handoff) {
      qd::QRun R{t, t_new, h_abs, min_step, rejected ? 1 : 0, nfev, nacc};
      if (qd::handoff<T>(c, a, X, sy, sf, stride, active, R, result, ho)) {
        nfev = R.nfev;
        nacc = R.nacc;
      }
    }
  }
#endif
#pragma unroll
  for (int p = 0; p < NP; p++) {
    V v = Y(p);
    if constexpr (YFR) {
      if (handoff) v = sy[p * stride];  // (the quads wrote the handed-off aircraft's y to the slots)
    }
    y_io[2 * p] = v.x;
    if (2 * p + 1 < NY) y_io[2 * p + 1] = v.y;
  }
#undef Y
#undef F
#undef ERV
#undef YR
#undef P3
#undef P4
#undef P5
#undef YB
  return result;
}

// ---------------------------------------------------------------------------
// Actuation.set_and_constrain_commands (pyfly.py:545-582).  cmd in/out in input
// order (elevator, aileron, throttle); sp = dynamics set-points.
// ---------------------------------------------------------------------------
template <typename T, typename C>
FW_HD int constrain_commands(const C& c, T* cmd, T* sp) {
  int term = 0;
  if (c.elevon) {
    T er = T(-1) * cmd[1] + cmd[0], el = cmd[1] + cmd[0];
    er = cond(c, FW_V_ACT0, er, term);
    el = cond(c, FW_V_ACT1, el, term);
    const T thr = cond(c, FW_V_ACT2, cmd[2], term);
    sp[0] = er;
    sp[1] = el;
    sp[2] = thr;
    T ail = (-er + el) / T(2), elev = (er + el) / T(2);
    elev = cond(c, FW_V_ELEVATOR, elev, term);
    ail = cond(c, FW_V_AILERON, ail, term);
    cmd[0] = elev;
    cmd[1] = ail;
    cmd[2] = thr;
  } else {
#pragma unroll
    for (int j = 0; j < 3; j++) {
      cmd[j] = cond(c, FW_V_ACT0 + j, cmd[j], term);
      sp[j] = cmd[j];
    }
  }
  return term;
}

// Dryden FIR at step k: j = k % L; 0 at chunk starts (dryden.py:193-261 as wired
// by pyfly.py:781-783).  un1 / u0: N(0,1) samples of channels (u0,u1,u2,u3) at k-1, k.
template <typename T>
FW_HD void dryden(const DevCfg<T>& c, int k, const T* un1, const T* u0, T* tl, T* ta) {
  const bool zero = (k % c.turb_len) == 0;
  const int chan[6] = {0, 1, 2, 3, 1, 2};
  T out[6];
#pragma unroll
  for (int f = 0; f < 6; f++)
    out[f] = zero ? T(0) : c.g0[f] * (c.noise_scale * un1[chan[f]]) + c.g1[f] * (c.noise_scale * u0[chan[f]]);
  tl[0] = out[0];
  tl[1] = out[1];
  tl[2] = out[2];
  ta[0] = out[3];
  ta[1] = out[4];
  ta[2] = out[5];
}

// ---------------------------------------------------------------------------
// Per-aircraft parameter-derived constants of the RHS (simulator parameter randomisation).  The
// reference samples simulator.params at every reset and _forces reads them at every RHS call
// (pyfly.py:1514-1643); the inertia gammas / I (pyfly.py:1086-1116) and the aspect ratio ar
// (pyfly.py:1119) are computed once in PyFly.__init__ and are NOT refreshed (quirk kept: they stay
// the config's values, DevCfg.gam / inv_Jy / ar0), nor are the EnergyVariable mass and inertia.
// ---------------------------------------------------------------------------
template <typename T>
struct AeroP {
  T qS, qSc, qSb, kCLq, kCDq, kCmq, hb, inv_pi_e_ar, kTP2, prop_k, mg, inv_mass, sig_c, M, a0, kmotor;
  T CL0, CLa, CLde, CDp, CDb1, CDb2, CDde, Cm0, Cma, Cmde, Cmfp;
  T CY0, CYb, CYp, CYr, CYda, Cl0, Clb, Clp, Clr, Clda, Cn0, Cnb, Cnp, Cnr, Cnda;
};

// P: the aircraft's parameter values in fw_param order (P(k) -> value)
template <typename T, typename C, typename PF>
FW_HD AeroP<T> aero_from(const C& c, PF P) {
  AeroP<T> a;
  const T S = P(FW_P_S_WING), b = P(FW_P_B), ch = P(FW_P_C);
  a.qS = T(0.5) * c.rho * S;
  a.qSc = a.qS * ch;
  a.qSb = a.qS * b;
  a.kCLq = P(FW_P_C_L_Q) * ch * T(0.5);
  a.kCDq = P(FW_P_C_D_Q) * ch * T(0.5);
  a.kCmq = P(FW_P_C_M_Q) * b * T(0.5);  // pyfly.py:1579 uses b, not c
  a.hb = b * T(0.5);
  a.inv_pi_e_ar = T(1) / (T(PI_D) * P(FW_P_E) * c.ar0);
  a.kTP2 = P(FW_P_K_T_P) * P(FW_P_K_OMEGA) * P(FW_P_K_OMEGA);
  a.prop_k = T(0.5) * c.rho * P(FW_P_S_PROP) * P(FW_P_C_PROP);
  a.mg = P(FW_P_MASS) * c.grav;
  a.inv_mass = T(1) / P(FW_P_MASS);
  a.M = P(FW_P_M);
  a.a0 = P(FW_P_A0);
  a.sig_c = exp(T(2) * a.M * a.a0);
  a.kmotor = P(FW_P_K_MOTOR);
  a.CL0 = P(FW_P_C_L_0); a.CLa = P(FW_P_C_L_ALPHA); a.CLde = P(FW_P_C_L_DELTA_E);
  a.CDp = P(FW_P_C_D_P); a.CDb1 = P(FW_P_C_D_BETA1); a.CDb2 = P(FW_P_C_D_BETA2); a.CDde = P(FW_P_C_D_DELTA_E);
  a.Cm0 = P(FW_P_C_M_0); a.Cma = P(FW_P_C_M_ALPHA); a.Cmde = P(FW_P_C_M_DELTA_E); a.Cmfp = P(FW_P_C_M_FP);
  a.CY0 = P(FW_P_C_Y_0); a.CYb = P(FW_P_C_Y_BETA); a.CYp = P(FW_P_C_Y_P); a.CYr = P(FW_P_C_Y_R);
  a.CYda = P(FW_P_C_Y_DELTA_A);
  a.Cl0 = P(FW_P_C_L0_ROLL); a.Clb = P(FW_P_C_L_BETA); a.Clp = P(FW_P_C_L_P); a.Clr = P(FW_P_C_L_R);
  a.Clda = P(FW_P_C_L_DELTA_A);
  a.Cn0 = P(FW_P_C_N_0); a.Cnb = P(FW_P_C_N_BETA); a.Cnp = P(FW_P_C_N_P); a.Cnr = P(FW_P_C_N_R);
  a.Cnda = P(FW_P_C_N_DELTA_A);
  return a;
}

// ---------------------------------------------------------------------------
// One PyFly.step for one aircraft (pyfly.py:1358-1420).
//   y[19]     ODE state (in/out)            der[8] roll pitch yaw Va alpha beta elev ail (in/out;
//             only der[6..7] are read: the t == 0 elevator/aileron values)
//   cmd[3]    raw commands in, constrained out
//   dmask     bit r set <=> der[r] was (re)computed.  On failure the stored state
//             holds the committed part of the save (history[-1] semantics); the
//             caller keeps its previous der[r] for the clear bits.  Bit 31
//             (DM_SOLVER_FAIL): the integration failed (TOO_SMALL_STEP, NaN step
//             or the max_nfev budget) and, like solve_ivp's sol.y[:, -1], the last
//             accepted sub-step went through the normal save (pyfly.py:1393-1396).
// Returns termination code (0 = success).
// ---------------------------------------------------------------------------
struct KeepY {  // default: y stays live in registers across the integration
  template <typename T>
  FW_HD void operator()(T*) const {}
};

// `reload(y)` runs right after the integration and may re-read the pre-step
// state from memory (the kernels do: keeping 19 values live across the RK loop
// costs registers the loop needs).
// Q = 4: the integration runs on the lane quad of the aircraft (fw_quad.hpp; qr = lane in the quad,
// every lane of the quad returns the same result); Q = 2: on its lane pair (fw_pair.hpp, round 6).
// HO: the one-lane integration's tail handoff (rk45; ho = the block's qd::HoSlot array in LDS).
template <int Q = 1, bool HO = false, bool YF = true, typename T, typename C, typename A, typename R = KeepY>
FW_HD int sim_step_masked(const C& c, const A& a, T* y, T* der, T* cmd, const T* wind, const T* tl, const T* ta, int& nfev,
                          int& nacc, uint32_t& dmask, V2<T>* sy, V2<T>* sf, int stride, R reload = R(), int qr = 0,
                          void* ho = nullptr) {
  dmask = 0;
  StepCtx<T> X;
#pragma unroll
  for (int i = 0; i < 3; i++) {
    X.wind[i] = wind[i];
    X.tl[i] = tl[i];
    X.ta[i] = ta[i];
  }
  X.elev0 = der[6];
  X.ail0 = der[7];
  nfev = 0;
  nacc = 0;
  int term = constrain_commands(c, cmd, X.sp);
  if (term) return term;
  T y1[NY];
#pragma unroll
  for (int i = 0; i < NY; i++) y1[i] = y[i];
  if constexpr (Q == 4) term = qd::rk45_quad(c, a, X, y1, nfev, nacc, qr);
  else if constexpr (Q == 2) term = pr::rk45_pair(c, a, X, y1, nfev, nacc, qr, sy, stride);
  else term = rk45<T, C, A, HO, YF>(c, a, X, y1, sy, sf, stride, nfev, nacc, FW_ER_LDS ? sf + NP * stride : nullptr, ho);
  reload(y);
  if (term < 0) {  // solver failure: y1 = the last accepted sub-step (rk45 wrote Y back), saved as usual
    dmask = DM_SOLVER_FAIL | (term == -2 ? DM_BUDGET : 0u);
    term = 0;
  }
  if (term) return term;

  // ---- _set_states_from_ode_solution(save=True) (pyfly.py:1852-1881) ----
  const T n = sqrt(y1[0] * y1[0] + y1[1] * y1[1] + y1[2] * y1[2] + y1[3] * y1[3]);
  const T e0 = y1[0] / n, e1 = y1[1] / n, e2 = y1[2] / n, e3 = y1[3] / n;
  y[0] = e0;
  y[1] = e1;
  y[2] = e2;
  y[3] = e3;
  T eul[3];
  eul[0] = atan2(T(2) * (e0 * e1 + e2 * e3), e0 * e0 + e3 * e3 - e1 * e1 - e2 * e2);
  // fp32: the rounded argument can exceed 1 in magnitude at pitch +-90 deg (NaN in asin); the fp64 parity
  // build keeps the reference's unclamped np.arcsin (pyfly.py:702)
  const T sp2 = T(2) * (e0 * e2 - e1 * e3);
  eul[1] = asin(sizeof(T) == 4 ? clipv(sp2, T(-1), T(1)) : sp2);
  eul[2] = atan2(T(2) * (e0 * e3 + e1 * e2), e0 * e0 + e1 * e1 - e2 * e2 - e3 * e3);
#pragma unroll
  for (int i = 0; i < 3; i++) {
    eul[i] = cond(c, FW_V_ROLL + i, eul[i], term);
    if (term) return term;
    der[i] = eul[i];
    dmask |= 1u << i;
  }
  // ODE states: the last RHS evaluation saw the very same y1, so these conditions
  // cannot fail here; they still clip/commit in order.
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const T v = cond(c, FW_V_OMEGA_P + i, y1[4 + i], term);
    if (term) return term;
    y[4 + i] = v;
  }
#pragma unroll
  for (int j = 0; j < 3; j++) {
    const T v = cond(c, FW_V_ACT0 + j, y1[13 + j], term);
    if (term) return term;
    y[13 + j] = v;
    y[16 + j] = (c.dotmask & (1u << j)) ? clipv(y1[16 + j], -c.dot_max[j], c.dot_max[j]) : y1[16 + j];
  }
  if (c.elevon) {
    const T ail = cond(c, FW_V_AILERON, (-y[13] + y[14]) / T(2), term);
    if (term) return term;
    der[7] = ail;
    dmask |= 1u << 7;
    const T elev = cond(c, FW_V_ELEVATOR, (y[13] + y[14]) / T(2), term);
    if (term) return term;
    der[6] = elev;
    dmask |= 1u << 6;
  } else {
    der[6] = y[13];
    der[7] = y[14];
    dmask |= 3u << 6;
  }
  // ---- post-step airspeed factors, Euler branch (pyfly.py:1398-1406) ----
  T va[3];
  if (c.euler_exact) airspeed_vec_euler(der[0], der[1], der[2], wind, tl, y + 10, va);
  else airspeed_vec(y, wind, tl, y + 10, va);
  const T Va_raw = sqrt(va[0] * va[0] + va[1] * va[1] + va[2] * va[2]);
  const T al = atan2(va[2], va[0]);
  const T sb1 = va[1] / Va_raw;  // (fp32: clamped like the pitch above; pyfly.py:1848)
  const T be = asin(sizeof(T) == 4 ? clipv(sb1, T(-1), T(1)) : sb1);
  const T Va = cond(c, FW_V_VA, Va_raw, term);
  if (term) return term;
  der[3] = Va;
  dmask |= 1u << 3;
  const T alc = cond(c, FW_V_ALPHA, al, term);
  if (term) return term;
  der[4] = alc;
  dmask |= 1u << 4;
  const T bec = cond(c, FW_V_BETA, be, term);
  if (term) return term;
  der[5] = bec;
  dmask |= 1u << 5;
  return 0;
}

// AttitudeQuaternion._from_euler_angles (pyfly.py:714-737)
template <typename T>
FW_HD void euler_to_quat(T phi, T th, T psi, T* q) {
  const T cps = cos(psi / T(2)), sps = sin(psi / T(2)), cth = cos(th / T(2)), sth = sin(th / T(2)),
          cph = cos(phi / T(2)), sph = sin(phi / T(2));
  q[0] = cps * cth * cph + sps * sth * sph;
  q[1] = cps * cth * sph - sps * sth * cph;
  q[2] = cps * sth * cph + sps * cth * sph;
  q[3] = sps * cth * cph - cps * sth * sph;
}

// Post-reset derived states (pyfly.py:1296-1311): Va/alpha/beta from Euler
// angles (turbulence is 0 at k = 0), elevator/aileron .value.
template <typename T, typename C>
FW_HD void reset_derived(const C& c, const T* y, const T* wind, T* der) {
  const T zero[3] = {T(0), T(0), T(0)};
  T va[3];
  airspeed_vec_euler(der[0], der[1], der[2], wind, zero, y + 10, va);
  const T Va_raw = sqrt(va[0] * va[0] + va[1] * va[1] + va[2] * va[2]);
  int term = 0;
  der[4] = cond<T>(c, FW_V_ALPHA, (T)atan2(va[2], va[0]), term);
  der[5] = cond<T>(c, FW_V_BETA, (T)asin(va[1] / Va_raw), term);
  der[3] = cond(c, FW_V_VA, Va_raw, term);
  if (c.elevon) {
    der[6] = cond(c, FW_V_ELEVATOR, (y[13] + y[14]) / T(2), term);
    der[7] = cond(c, FW_V_AILERON, (-y[13] + y[14]) / T(2), term);
  } else {
    der[6] = y[13];
    der[7] = y[14];
  }
  if (c.disabled_inputs & 1) der[6] = T(0);  // disabled ControlVariable.reset (pyfly.py:359-363)
  if (c.disabled_inputs & 2) der[7] = T(0);
}

// ===========================================================================
// gym env epilogue (fixed_wing.py)
// ===========================================================================
template <typename T>
FW_HD T pymod(T a, T b) {
  T r = fmod(a, b);
  if (r != T(0) && ((r < T(0)) != (b < T(0)))) r += b;
  return r;
}

// _get_error (fixed_wing.py:1318-1344); val = current .value of the target state
template <typename T>
FW_HD T target_error(const DevCfg<T>& c, int k, T tgt, T val) {
  if (c.target_wrap[k]) {
    const T pi = T(PI_D);
    T dist = pymod(val - tgt + pi, T(2) * pi) - pi;
    if (dist < -pi) dist += T(2) * pi;
    return dist;
  }
  return tgt - val;
}

// _get_goal_status()["all"] (fixed_wing.py:1346-1361)
template <typename T>
FW_HD bool goal_all(const DevCfg<T>& c, const T* tgt, const T* vals) {
  bool all = true;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    if (!c.has_bound[k]) continue;
    const T err = target_error(c, k, tgt[k], vals[k]);
    if (!(fabs(err) <= c.target_bound[k])) all = false;
  }
  return all;
}

// _get_goal_status (fixed_wing.py:1346-1361) as bits: bit k = roll / pitch / Va within its bound
// (targets without a bound report 0), bit 3 = "all" (all bounded targets; True if none)
template <typename T>
FW_HD uint32_t goal_status_bits(const DevCfg<T>& c, const T* tgt, const T* vals) {
  uint32_t bits = 0, all = 1;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    if (!c.has_bound[k]) continue;
    const T err = target_error(c, k, tgt[k], vals[k]);
    const uint32_t ok = fabs(err) <= c.target_bound[k] ? 1u : 0u;
    bits |= ok << k;
    all &= ok;
  }
  return bits | (all << 3);
}

// _get_next_target (fixed_wing.py:1363-1471): constant / compensate(Va) / linear / sinusoidal.  tp: the
// aircraft's target properties (per target: slope or amplitude, period, phase, bias; State::tpr), read only
// for the linear / sinusoidal classes; steps = steps_count after the step (the sinusoid's argument)
template <typename T, typename TP>
FW_HD void next_target(const DevCfg<T>& c, int steps_tgt, int steps, TP tp, T* tgt) {
  T res[3];
#pragma unroll
  for (int k = 0; k < 3; k++) {
    T r = tgt[k];
    if (c.target_class[k] == FW_TGT_LINEAR) {  // :1433-1435
      r = tgt[k] + tp(4 * k) * c.dt;
    } else if (c.target_class[k] == FW_TGT_SINUSOIDAL) {  // :1438-1448
      r = tp(4 * k) * sin(T(2.0 * PI_D) / tp(4 * k + 1) * ((T)steps + tp(4 * k + 2))) + tp(4 * k + 3);
    } else if (c.target_class[k] == FW_TGT_COMPENSATE) {
      // pitch_tar: the pitch target (constant, linear) or the sinusoid's bias (:1381-1392)
      const T pitch_tar = c.target_class[1] == FW_TGT_SINUSOIDAL ? tp(4 * 1 + 3) : tgt[1];
      const T deg = T(PI_D / 180.0);
      if (pitch_tar <= T(-2.5) * deg) {
        const T va_target = tgt[2];
        const T va_end = T(28.434) - T(40.0841) * pitch_tar;
        T slope = T(0);
        if (va_target <= va_end) {
          const T a = va_target < va_end * T(0.95) ? T(1) : T(1) - va_target / (va_end * T(1.5));
          slope = T(7) * (a > T(0) ? a : T(0));
        }
        r = va_target + (slope * (-tgt[1]) - T(0.25)) * c.dt;
      } else if (pitch_tar >= T(5) * deg) {
        const T va_end = T(26.27) - T(41.2529) * pitch_tar;
        const T va_target = tgt[2];
        if (va_target > va_end) r = steps_tgt < 750 ? va_target + (va_end - va_target) * T(1) / T(150) : va_end;
        else r = va_target;
      }
    }
    if (c.target_wrap[k] && fabs(r) > T(PI_D)) r = sgn(r) * (fmod(fabs(r), T(PI_D)) - T(PI_D));
    res[k] = r;
  }
  tgt[0] = res[0];
  tgt[1] = res[1];
  tgt[2] = res[2];
}

// _attitude_to_angular_rates (fixed_wing.py:1558-1642) of target omega_p / q / r (k = 0 / 1 / 2): from the errors
// of the roll / pitch targets `tgt` against the attitude (roll, pitch) and the current omega targets `ot`.  As
// numpy evaluates it: np.clip keeps a NaN, np.sign(0) = 0, a zero sin(roll) divides to +-inf; the damping's
// `<= radians(0.1)` branch is overwritten on the next line there, so it is absent here.
template <typename T>
FW_HD T np_clip(T x, T lo, T hi) {
  return x < lo ? lo : (x > hi ? hi : x);
}
template <typename T>
FW_HD T np_sign(T x) {
  return x > T(0) ? T(1) : (x < T(0) ? T(-1) : x);
}
template <typename T>
FW_HD T att_ang_rate(const DevCfg<T>& c, int k, const T* tgt, const T* ot, T roll, T pitch) {
  const T mv = c.ang_max_vel[k], dt = c.dt, half_pi = T(0.5 * PI_D);
  const T roll_err = target_error(c, 0, tgt[0], roll);
  const T pitch_err = target_error(c, 1, tgt[1], pitch);
  const T qw = cos(roll), rw = sin(roll);
  const T mpc = mv * dt * (qw + rw);
  T res, damp;
  if (k == 0) {
    damp = fabs(roll_err / half_pi);
    const T q_roll = sin(roll) * tan(pitch) * ot[1] * dt;
    const T r_roll = cos(roll) * tan(pitch) * ot[2] * dt;
    res = np_clip(-(roll_err - q_roll - r_roll) / dt, -mv, mv);
  } else if (k == 1) {
    damp = fabs(pitch_err / half_pi);
    res = mpc > fabs(pitch_err) ? -pitch_err / (T(2) * qw) : np_sign(qw) * mv * np_sign(pitch_err);
  } else {
    damp = fabs(pitch_err / half_pi);
    res = mpc > fabs(pitch_err) ? pitch_err / rw : -np_sign(rw) * mv * np_sign(pitch_err);
  }
  damp = isnan(damp) ? T(0.05) : (damp < T(1) ? damp : T(1));  // min(1, damping)
  const T t = ot[k];
  return np_clip(t + (res * damp - t) * T(1) / T(20), -mv, mv);
}

// linear_action_scaling (fixed_wing.py:630-652)
template <typename T>
FW_HD T scale_fwd(const DevCfg<T>& c, int i, T a) {
  return (c.act_high[i] - c.act_low[i]) * (a - c.scale_low) / (c.scale_high - c.scale_low) + c.act_low[i];
}
template <typename T>
FW_HD T scale_bwd(const DevCfg<T>& c, int i, T a) {
  return (c.scale_high - c.scale_low) * (a - c.act_low[i]) / (c.act_high[i] - c.act_low[i]) + c.scale_low;
}

}  // namespace fw
