// fw_quad.hpp -- one aircraft's RK45 integration on a quad of four lanes (included by fw_device.hpp).
//
// The one-lane integrator (rk45 / rhs above) is a serial chain of ~600 instructions per RHS
// evaluation, and a wave is as slow as its slowest aircraft: when aircraft are few (the per-GPU
// shard of the strong-scaling configurations) or one aircraft needs thousands of evaluations (the
// RK45 straggler tail), the step time is the latency of that chain.  Here lanes
// 4a..4a+3 own aircraft a and split every 3-vector operation of the RHS by ROW (SIMT-uniform
// code: lane r computes row r of the same formula):
//
//   lane r < 3 holds   eps_r (quaternion e_{r+1}), omega_r, pos_r, vel_r, actuator r, its rate r
//   lane 3 holds       e0 (and zeros)
//
// so the Dormand-Prince folds, the error norm and the state conditioning run on 6 elements per
// lane instead of 19, and the airspeed rotation, kinematics, force/moment rows and actuator
// dynamics are computed once per row.  The scalar front (Va, alpha, beta, stall blend, the
// aerodynamic coefficients) is computed redundantly on the four lanes.  Row values cross lanes
// with DPP quad permutations (no LDS); norms are quad butterfly sums, bit-identical on the four
// lanes, so the step-size control (and every branch) stays uniform within the quad.
//
// Reference behaviour: the same as rhs() / rk45() (PyFly._dynamics / _forces / _f_*,
// pyfly.py:1450-1747; scipy 1.15.3 RK45, rk.py:111-173, common.py:68-134).  Sums are formed in a
// different order (rows before lanes), so results differ from the one-lane path by rounding.
#pragma once

#ifndef FW_QUAD_SIGMA_1RCP
#define FW_QUAD_SIGMA_1RCP 1  // fp32 stall blend with one reciprocal (0: round 4's two; A/B)
#endif
#ifndef FW_QUAD_RC_NOSEL
#define FW_QUAD_RC_NOSEL 1  // the front's reciprocals without lane selects when Va is not clipped (0: round 4; A/B)
#endif

namespace qd {

// bound_ctrl set and no `old` operand: the form the backend's DPP combiner folds into a single-use
// VOP2 consumer (v_add_f32_dpp / v_mul_f32_dpp ... instead of v_mov_b32_dpp + the op).  A quad_perm never
// reads outside the quad and the four lanes of a quad are always enabled together, so no lane takes
// the bound_ctrl zero.
template <int A, int B, int C, int D>
__device__ __forceinline__ int perm_i(int x) {
  return __builtin_amdgcn_update_dpp(0, x, A | (B << 2) | (C << 4) | (D << 6), 0xF, 0xF, true);
}
template <int A, int B, int C, int D>
__device__ __forceinline__ float perm(float x) {
  return __int_as_float(perm_i<A, B, C, D>(__float_as_int(x)));
}
template <int A, int B, int C, int D>
__device__ __forceinline__ double perm(double x) {
  const unsigned long long v = (unsigned long long)__double_as_longlong(x);
  const unsigned lo = (unsigned)perm_i<A, B, C, D>((int)(unsigned)v);
  const unsigned hi = (unsigned)perm_i<A, B, C, D>((int)(unsigned)(v >> 32));
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
// row K of every quad (lane & 3 == K) takes x_row, the others x_other: one v_cndmask against a
// constant lane mask.  The compiler turns `r == K ? a + b : c` with work in an arm into an exec-masked
// branch (saveexec / xor / andn2 / or, both arms issued) -- the lone-wave tail pays every instruction.
template <int K>
__device__ __forceinline__ float rowsel(float x_row, float x_other) {
  float out;
  asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(out) : "v"(x_other), "v"(x_row), "s"(0x1111111111111111ull << K));
  return out;
}
template <int K>
__device__ __forceinline__ double rowsel(double x_row, double x_other) {
  const unsigned long long a = (unsigned long long)__double_as_longlong(x_row);
  const unsigned long long b = (unsigned long long)__double_as_longlong(x_other);
  const float lo = rowsel<K>(__int_as_float((int)(unsigned)a), __int_as_float((int)(unsigned)b));
  const float hi = rowsel<K>(__int_as_float((int)(unsigned)(a >> 32)), __int_as_float((int)(unsigned)(b >> 32)));
  return __longlong_as_double((long long)(((unsigned long long)(unsigned)__float_as_int(hi) << 32) |
                                          (unsigned)__float_as_int(lo)));
}
// lane K's value on all four lanes
template <int K, typename T>
__device__ __forceinline__ T bc(T x) {
  return perm<K, K, K, K>(x);
}
// row (r + 1) % 3 / (r + 2) % 3 of a row-distributed 3-vector (lane 3 keeps its own)
template <typename T>
__device__ __forceinline__ T nx1(T x) {
  return perm<1, 2, 0, 3>(x);
}
template <typename T>
__device__ __forceinline__ T nx2(T x) {
  return perm<2, 0, 1, 3>(x);
}
// butterfly sum / min over the quad: the same bits on all four lanes
template <typename T>
__device__ __forceinline__ T sum4(T x) {
  x = x + perm<1, 0, 3, 2>(x);
  return x + perm<2, 3, 0, 1>(x);
}
__device__ __forceinline__ int min4(int k) {
  k = min(k, perm_i<1, 0, 3, 2>(k));
  return min(k, perm_i<2, 3, 0, 1>(k));
}

// Violation keys in rhs()'s order of checks (first violation wins = smallest key):
// omega p q r, pos n e d, vel u v w, actuators 0 1 2, aileron, elevator, Va, alpha, beta.
constexpr int KEY_NONE = 64;
__device__ __forceinline__ int key_var(int k) {
  if (k < 12) return (k < 9 ? FW_V_OMEGA_P : FW_V_ACT0 - 9) + k;
  return k == 12 ? FW_V_AILERON : k == 13 ? FW_V_ELEVATOR : k == 14 ? FW_V_VA : k == 15 ? FW_V_ALPHA : FW_V_BETA;
}

// Per-lane constants of one step (lane r's rows; lane 3: no conditions).  Lane 3 carries e0 in slot 0
// and zeros in slots 1..5; its row coefficients are zero, so its slot-1..5 derivatives come out as 0
// without a select (rhs_quad).
template <typename T>
struct QCtx {
  int r;
  bool row;
  T rowf;                 // 1 on lanes 0..2, 0 on lane 3
  T sgn1;                 // +1 on lane 1 (the beta chain's exponential), -1 on the others
  T w0, w1, w2;           // steady wind components r, r+1, r+2 (cyclic)
  T tl, ta, sp;           // linear / angular turbulence and actuator set-point of row r
  T elev0, ail0;          // t == 0 elevator / aileron (StepCtx)
  // conditions: constraint interval (+-inf: none) and clip interval + flag of this lane's variables
  T om_cl, om_ch, om_vl, om_vh, pos_cl, pos_ch, vel_cl, vel_ch, vel_vl, vel_vh, act_cl, act_ch, act_vl, act_vh;
  T dmax;
  bool om_clip, vel_clip, act_clip, dclip;
  T ac0, ac1, ac2, ac3, ac4, ac5;  // actuator coefficients of row r (0 on lane 3)
  // gyroscopic part of _f_omega_dot row r in the lane's cyclic frame (om, om1, om2 = omega_r, _r+1, _r+2):
  // kx om om1 + ky om1 om2 + kz om om2 + kw (om2^2 - om1^2)  (0 on lane 3)
  T kx, ky, kz, kw;
  // rhs_quad's per-lane coefficients of the lift / pitch-moment / drag factor (fK) and of the side-force /
  // torque-row formula (tK, t0 .. tda, the propeller torque tpr); computed once here: with the products in
  // the arms of a per-lane select, the compiler branched on the lane in every RHS evaluation
  T fK, tK, t0, tb, tp, tr, tda, tpr;
  T kprop;  // the propeller force's factor on row 0 (it acts along body x), 0 on the other rows
};

template <typename T, typename C, typename A>
__device__ __forceinline__ QCtx<T> qctx(const C& c, const A& a, const StepCtx<T>& X, int r) {
  QCtx<T> Q;
  auto s3 = [r](T a0, T a1, T a2) { return r == 0 ? a0 : (r == 1 ? a1 : a2); };
  const T inf = T(__builtin_inf());
  const T z = T(0);
  Q.r = r;
  Q.row = r < 3;
  Q.rowf = Q.row ? T(1) : z;
  Q.sgn1 = r == 1 ? T(1) : T(-1);
  Q.w0 = s3(X.wind[0], X.wind[1], X.wind[2]);
  Q.w1 = s3(X.wind[1], X.wind[2], X.wind[0]);
  Q.w2 = s3(X.wind[2], X.wind[0], X.wind[1]);
  Q.tl = s3(X.tl[0], X.tl[1], X.tl[2]);
  Q.ta = s3(X.ta[0], X.ta[1], X.ta[2]);
  Q.sp = s3(X.sp[0], X.sp[1], X.sp[2]);
  Q.elev0 = X.elev0;
  Q.ail0 = X.ail0;
  auto lim = [&](int v0, T& cl, T& ch, T& vl, T& vh, bool& clip) {
    T l[3], h[3], a[3], b[3];
    bool k[3];
#pragma unroll
    for (int j = 0; j < 3; j++) {
      const uint32_t bit = 1u << (v0 + j);
      const bool hc = (c.cmask & bit) != 0;
      l[j] = hc ? c.lim[v0 + j].cmin : -inf;
      h[j] = hc ? c.lim[v0 + j].cmax : inf;
      a[j] = c.lim[v0 + j].vmin;
      b[j] = c.lim[v0 + j].vmax;
      k[j] = (c.clipmask & bit) != 0;
    }
    cl = Q.row ? s3(l[0], l[1], l[2]) : -inf;
    ch = Q.row ? s3(h[0], h[1], h[2]) : inf;
    vl = Q.row ? s3(a[0], a[1], a[2]) : -inf;  // lane 3's zero slots clip to themselves
    vh = Q.row ? s3(b[0], b[1], b[2]) : inf;
    clip = Q.row && (r == 0 ? k[0] : (r == 1 ? k[1] : k[2]));
  };
  bool pclip;
  T pvl, pvh;
  lim(FW_V_OMEGA_P, Q.om_cl, Q.om_ch, Q.om_vl, Q.om_vh, Q.om_clip);
  lim(FW_V_POS_N, Q.pos_cl, Q.pos_ch, pvl, pvh, pclip);  // positions are checked, never clipped (rhs())
  lim(FW_V_VEL_U, Q.vel_cl, Q.vel_ch, Q.vel_vl, Q.vel_vh, Q.vel_clip);
  lim(FW_V_ACT0, Q.act_cl, Q.act_ch, Q.act_vl, Q.act_vh, Q.act_clip);
  Q.dmax = s3(c.dot_max[0], c.dot_max[1], c.dot_max[2]);
  Q.dclip = Q.row && ((c.dotmask >> (r & 3)) & 1u);
  auto s3r = [&](T a0, T a1, T a2) { return Q.row ? s3(a0, a1, a2) : z; };
  Q.ac0 = s3r(c.ac[0][0], c.ac[1][0], c.ac[2][0]);
  Q.ac1 = s3r(c.ac[0][1], c.ac[1][1], c.ac[2][1]);
  Q.ac2 = s3r(c.ac[0][2], c.ac[1][2], c.ac[2][2]);
  Q.ac3 = s3r(c.ac[0][3], c.ac[1][3], c.ac[2][3]);
  Q.ac4 = s3r(c.ac[0][4], c.ac[1][4], c.ac[2][4]);
  Q.ac5 = s3r(c.ac[0][5], c.ac[1][5], c.ac[2][5]);
  // pyfly.py:1659-1683: p' = g1 PQ - g2 QR + g3 l + g4 n;  q' = g5 PR - g6 (P^2 - R^2) + m / Jy;
  //                     r' = g7 PQ - g1 QR + g4 l + g8 n
  //   row 0 (om, om1, om2 = P, Q, R): g1 PQ - g2 QR;  row 1 (Q, R, P): g5 PR - g6 (P^2 - R^2);
  //   row 2 (R, P, Q): g7 PQ - g1 QR
  Q.kx = s3r(c.gam[1], z, z);
  Q.ky = s3r(-c.gam[2], c.gam[5], c.gam[7]);
  Q.kz = s3r(z, z, -c.gam[1]);
  Q.kw = s3r(z, -c.gam[6], z);
  const T jm = a.qSc * c.inv_Jy;
  Q.fK = r == 1 ? jm : a.qS;
  // side force Y on lane 1, roll / yaw torque rows on lanes 0 / 2: row 0 = g3 l + g4 n, row 2 = g4 l + g8 n
  const T g3 = c.gam[3], g4 = c.gam[4], g8 = c.gam[8];
  auto tq = [&](T cl, T cn, T cy) {
    const T r0v = g3 * cl + g4 * cn, r2v = g4 * cl + g8 * cn;
    return s3r(r0v, cy, r2v);
  };
  Q.tK = s3r(a.qSb, a.qS, a.qSb);
  Q.t0 = tq(a.Cl0, a.Cn0, a.CY0);
  Q.tb = tq(a.Clb, a.Cnb, a.CYb);
  Q.tp = tq(a.Clp, a.Cnp, a.CYp);
  Q.tr = tq(a.Clr, a.Cnr, a.CYr);
  Q.tda = tq(a.Clda, a.Cnda, a.CYda);
  const T k3 = -a.kTP2 * g3, k4 = -a.kTP2 * g4;
  Q.tpr = s3r(k3, z, k4);
  Q.kprop = r == 0 ? a.prop_k : z;
  return Q;
}

// Variable.apply_conditions of a row variable (interval form of cond(); the ODE-state variables
// of a quad configuration never wrap, fw_kernels.hip checks that before choosing this path)
template <typename T>
__device__ __forceinline__ T qcond(T x, T cl, T ch, T vl, T vh, bool clip, int& key, int k) {
  const bool viol = (x < cl) | (x > ch);
  key = (key == KEY_NONE && viol) ? k : key;
  return clip ? clipv(x, vl, vh) : x;
}
// ... of a scalar (quad-uniform) variable: cond() itself
template <typename T, typename C>
__device__ __forceinline__ T ucond(const C& c, int v, T x, int& key, int k) {
  int t = 0;
  x = cond(c, v, x, t);
  key = (key == KEY_NONE && t) ? k : key;
  return x;
}

// PyFly._dynamics (pyfly.py:1450-1482) of lane Q.r's rows: s = this lane's 6 stage values,
// ds = their derivatives.  term = the first violated condition of the aircraft (0 = none); returns
// whether any aircraft of the wave violated one (wave-uniform; term is only written then).
// Written for the lone-wave tail, where every VALU instruction costs its issue slot: the checks a
// configuration does not have are compiled out (mask tests fold for the SpecCfg views), lane 3's zero
// rows need no selects (QCtx), and the per-row force rotation shares its beta rotation.
template <typename T, typename C, typename A>
__device__ __forceinline__ bool rhs_quad(const C& c, const A& a, const QCtx<T>& Q, bool first, const T* s, T* ds,
                                         int& term) {
  int key = KEY_NONE;
  T om = s[1], vel = s[3], av = s[4], ad = s[5];
  T elev = Q.elev0, ail = Q.ail0;
  if (!first) {  // _set_states_from_ode_solution(save=False) + Actuation.set_states (pyfly.py:479-492)
    // a row variable: constraint (first violation wins) then clip.  All three rows clipping: lane 3
    // (zeros, clip interval of row 2) clips too, without the per-lane select.
    auto rowcond = [&](T x, int v0, T cl, T ch, T vl, T vh, bool clip, int k) {
      if (c.cmask & (7u << v0)) {
        const bool viol = (x < cl) | (x > ch);
        key = (key == KEY_NONE && viol) ? k : key;
      }
      if (((c.clipmask >> v0) & 7u) == 7u) return clipv(x, vl, vh);
      if (c.clipmask & (7u << v0)) return clip ? clipv(x, vl, vh) : x;
      return x;
    };
    om = rowcond(om, FW_V_OMEGA_P, Q.om_cl, Q.om_ch, Q.om_vl, Q.om_vh, Q.om_clip, Q.r);
    (void)rowcond(s[2], FW_V_POS_N, Q.pos_cl, Q.pos_ch, T(0), T(0), false, 3 + Q.r);  // checked, never clipped
    vel = rowcond(vel, FW_V_VEL_U, Q.vel_cl, Q.vel_ch, Q.vel_vl, Q.vel_vh, Q.vel_clip, 6 + Q.r);
    av = rowcond(av, FW_V_ACT0, Q.act_cl, Q.act_ch, Q.act_vl, Q.act_vh, Q.act_clip, 9 + Q.r);
    if (c.dotmask) ad = Q.dclip ? clipv(ad, -Q.dmax, Q.dmax) : ad;
    const T a0 = bc<0>(av), a1 = bc<1>(av);
    if (c.elevon) {
      ail = (-a0 + a1) * T(0.5);
      elev = (a0 + a1) * T(0.5);
      ail = ucond(c, FW_V_AILERON, ail, key, 12);
      elev = ucond(c, FW_V_ELEVATOR, elev, key, 13);
    } else {
      elev = a0;
      ail = a1;
    }
  }
  const T thr = bc<2>(av);
  const T er = s[0];  // raw attitude (pyfly.py:1464): eps_r, lane 3: e0
  const T e0 = bc<3>(er);
  const T er1 = nx1(er), er2 = nx2(er);

  // ---- _forces (pyfly.py:1484-1643) ----
  const T omt = om - Q.ta;  // angular turbulence (0 without turbulence: turbulence_at zeroes it)
  const T p = bc<0>(omt), q = bc<1>(omt), r = bc<2>(omt);
  // row r of wind_b = R(q) w + turb (_rot_b_v quaternion branch, pyfly.py:1780-1800; 1843)
  const T Rrr = T(-1) + T(2) * (e0 * e0 + er * er);
  const T Rr1 = T(2) * (er * er1 + er2 * e0);
  const T Rr2 = T(2) * (er * er2 - er1 * e0);
  const T var_ = vel - (Rrr * Q.w0 + Rr1 * Q.w1 + Rr2 * Q.w2 + Q.tl);
  const T va0 = bc<0>(var_), va1 = bc<1>(var_), va2 = bc<2>(var_);
  // the scalar front's transcendental work split over the lanes (lane 1: the beta chain, the others:
  // the alpha chain), the results broadcast: the same values as rhs() computes serially
  const bool l1 = Q.r == 1;
  const T rxz2 = va0 * va0 + va2 * va2;
  const T sq = fsqrt(l1 ? rxz2 + va1 * va1 : rxz2);
  const T rxz = bc<0>(sq), Va_raw = bc<1>(sq);
  const T at = fatan2(l1 ? va1 : va2, l1 ? rxz : va0);
  T alpha = bc<0>(at), beta = bc<1>(at);
  const T Va = ucond(c, FW_V_VA, Va_raw, key, 14);
  alpha = ucond(c, FW_V_ALPHA, alpha, key, 15);
  beta = ucond(c, FW_V_BETA, beta, key, 16);
  // 1 / rxz, 1 / Va_raw (, 1 / Va) on lanes 0, 1 (, 2).  A configuration that does not clip Va has Va ==
  // Va_raw bit for bit, and the reciprocal is of this lane's own square root: no selects, one broadcast fewer
  T irxz, iVr, iVa;
  if (FW_QUAD_RC_NOSEL && !((c.clipmask >> FW_V_VA) & 1u)) {  // (compile-time for the SpecCfg views)
    const T rc = frcp(sq);
    irxz = bc<0>(rc);
    iVr = bc<1>(rc);
    iVa = iVr;
  } else {
    const T rc = frcp(Q.r == 0 ? rxz : (l1 ? Va_raw : Va));
    irxz = bc<0>(rc);
    iVr = bc<1>(rc);
    iVa = bc<2>(rc);
  }
  T sa, ca, sb, cb;
  if (c.trig_alpha) {
    sa = sin(alpha);
    ca = cos(alpha);
  } else {
    sa = rxz2 > T(0) ? va2 * irxz : T(0);
    ca = rxz2 > T(0) ? va0 * irxz : T(1);
  }
  if (c.trig_beta) {
    sb = sin(beta);
    cb = cos(beta);
  } else {
    sb = va1 * iVr;
    cb = rxz * iVr;
  }
  const T V2a = Va * Va;
  // lane 1: exp(M (alpha + a0)); the others: exp(-M (alpha - a0)) = exp(-M alpha + M a0)
  T ex, sigma;
  if constexpr (sizeof(T) == 4 && FW_QUAD_SIGMA_1RCP) {
    // sigma = S / (S + C), S = 1 + e1 + e2, with ONE reciprocal: the exponent clamped at 2^120 keeps S + C
    // finite and its reciprocal normal; where the clamp acts, C / S < 1e-15 and sigma rounds to 1 either way
    const T l2e = T(1.4426950408889634);
    ex = __builtin_amdgcn_exp2f(fminf(fmaf(Q.sgn1 * (a.M * l2e), alpha, a.M * a.a0 * l2e), T(120)));
    const T S = T(1) + bc<0>(ex) + bc<1>(ex);
    sigma = S * frcp(S + a.sig_c);
  } else if constexpr (sizeof(T) == 4) {  // (round 4: two reciprocals; A/B switch FW_QUAD_SIGMA_1RCP=0)
    const T l2e = T(1.4426950408889634);
    ex = __builtin_amdgcn_exp2f(fmaf(Q.sgn1 * (a.M * l2e), alpha, a.M * a.a0 * l2e));
    sigma = frcp(T(1) + a.sig_c * frcp(T(1) + bc<0>(ex) + bc<1>(ex)));
  } else {
    ex = fexp(l1 ? a.M * (alpha + a.a0) : -a.M * (alpha - a.a0));
    const T ex1 = bc<0>(ex), ex2 = bc<1>(ex);
    sigma = frcp(T(1) + a.sig_c * frcp(T(1) + ex1 + ex2));  // overflow-safe form, see rhs()
  }
  const T osig = T(1) - sigma;
  // sgn(alpha) sin(alpha)^2 = sin(alpha) |sin(alpha)|: sin has alpha's sign on [-pi, pi] and the
  // product is 0 where it does not (pyfly.py:1547-1579 multiply by np.sign(alpha))
  const T ssa = sa * fabs(sa);
  const T qn = q * iVa;
  // lift / drag / pitch moment (pyfly.py:1529-1579) as ONE formula with row constants, lane r = row r
  // (lane 3 repeats lane 0), then broadcast:
  //   K V2a (c0 + osig (pa + pb alpha)(pg + ph alpha) + sigma ssa (mu ca + mv sa + mw)
  //          + kq q/Va + kde elev + kde2 elev^2 + kb1 beta + kb2 beta^2)
  //   lift:   CL0 + CLa a, stall 2 ca,  C_L_q c/2,  C_L_de elev                       (K = rho/2 S)
  //   moment: Cm0 + Cma a, stall C_m_fp, C_m_q b/2, C_m_de elev                (K = rho/2 S c / Jy)
  //   drag:   CDp + (CL0 + CLa a)^2 / (pi e AR), stall 2 sa, C_D_q c/2, C_D_de elev^2,
  //           C_D_beta1 b + C_D_beta2 b^2                                            (K = rho/2 S)
  // on lanes 0 / 1 / 2: lane 1's pitch moment over Jy is row 1 of _f_omega_dot's torque term as it stands
  const int rr = Q.r == 3 ? 0 : Q.r;
  auto s3r = [rr](T x0, T x1, T x2) { return rr == 0 ? x0 : (rr == 1 ? x1 : x2); };
  const T z = T(0), one = T(1), two = T(2);
  const T pa = s3r(a.CL0, a.Cm0, a.CL0), pb = s3r(a.CLa, a.Cma, a.CLa);
  const T pg = s3r(one, one, a.CL0 * a.inv_pi_e_ar), ph = s3r(z, z, a.CLa * a.inv_pi_e_ar);
  const T c0 = s3r(z, z, a.CDp), mu = s3r(two, z, z), mv = s3r(z, z, two), mw = s3r(z, a.Cmfp, z);
  const T kq = s3r(a.kCLq, a.kCmq, a.kCDq), kde = s3r(a.CLde, a.Cmde, z), kde2 = s3r(z, z, a.CDde);
  const T kb1 = s3r(z, z, a.CDb1), kb2 = s3r(z, z, a.CDb2), K = Q.fK;
  const T P = (pa + pb * alpha) * (pg + ph * alpha);
  const T Cr = c0 + osig * P + (sigma * ssa) * (mu * ca + mv * sa + mw);
  const T Fr = K * V2a * (Cr + kq * qn + kde * elev + kde2 * (elev * elev) + kb1 * beta + kb2 * (beta * beta));
  const T flift = bc<0>(Fr), fdrag = bc<2>(Fr);
  const T bp = a.hb * p * iVa, br = a.hb * r * iVa;
  // side force Y (lane 1) and the roll / yaw torque rows of _f_omega_dot (pyfly.py:1659-1683) on lanes 0 / 2:
  // row 0 = g3 (l + tprop) + g4 n, row 2 = g4 (l + tprop) + g8 n, with l, n, Y linear in the same items
  // (pyfly.py:1581-1643) -- one formula with the torque-combined coefficients per lane; lane 3: zero
  // (coefficients: QCtx; the propeller torque -kTP2 thr^2 adds to l, pyfly.py:1615-1643)
  const T g2 = Q.tK * V2a * (Q.t0 + Q.tb * beta + Q.tp * bp + Q.tr * br + Q.tda * ail) + Q.tpr * (thr * thr);
  const T fy = bc<1>(g2);
  // Row selections below pick among values computed on every lane: selects, not divergent branches
  // (a conditional expression with work in its arms compiles to exec-masked branches here).
  const bool r0 = Q.r == 0, r1 = Q.r == 1;
  // row r of f_aero = R_euler(0, alpha, beta) . [-D, Y, -L] = R_alpha . (R_beta . [-D, Y, -L]):
  // U = cb (-D) + sb Y, then rows (ca U + sa L, sb D + cb Y, sa U - ca L)
  const T U = cb * (-fdrag) + sb * fy;
  const T fa02 = (r0 ? ca : sa) * U + (r0 ? sa : -ca) * flift;
  const T fa = rowsel<1>(sb * fdrag + cb * fy, fa02);
  // gravity: column 2 of R(q) (the diagonal term in the raw-quaternion form of pyfly.py:1493-1499)
  const T Dr = er * er + e0 * e0 - er1 * er1 - er2 * er2;
  const T fg = a.mg * (r0 ? Rr2 : (r1 ? Rr1 : Dr));
  const T Vd = Va + thr * (a.kmotor - Va);
  const T fr = Q.kprop * Vd * (Vd - Va) + fg + fa;  // propeller force on row 0 only (QCtx)

  const T om1 = nx1(om), om2 = nx2(om), vel1 = nx1(vel), vel2 = nx2(vel);
  // _f_attitude_dot (pyfly.py:1645-1657): row r = d eps_r, lane 3 = d e0 = -(P e1 + Q e2 + R e3) / 2, the
  // quad sum of omega_r eps_r (lane 3's omega slot is 0)
  const T deps = T(0.5) * (om * e0 + om2 * er1 - om1 * er2);
  const T de0 = T(-0.5) * sum4(om * er);
  // _f_omega_dot (pyfly.py:1659-1683), row r: gyroscopic terms + the torque row (lane 1: Fr, else g2)
  const T dw = Q.kx * (om * om1) + Q.ky * (om1 * om2) + Q.kz * (om * om2) + Q.kw * (om2 * om2 - om1 * om1) +
               rowsel<1>(Fr, g2);
  // _f_p_dot (pyfly.py:1706-1737), row r
  const T dp = Dr * vel + T(2) * (er * er1 - er2 * e0) * vel1 +
               T(2) * (er * er2 + er1 * e0) * vel2;
  // _f_v_dot (pyfly.py:1685-1704), row r
  const T dv = om2 * vel1 - om1 * vel2 + fr * (a.inv_mass * Q.rowf);
  // Actuation.rhs (pyfly.py:519-543), actuator r
  const T da = av * Q.ac0 + Q.sp * Q.ac2 + ad * Q.ac1;
  const T dd = av * Q.ac3 + Q.sp * Q.ac5 + ad * Q.ac4;
  // lane 3: de0, then zeros -- its slots 1..5 are 0 and its coefficients (QCtx) are 0
  ds[0] = Q.row ? deps : de0;
  ds[1] = dw;
  ds[2] = dp;
  ds[3] = dv;
  ds[4] = da;
  ds[5] = dd;
  if (!any_lane(key != KEY_NONE)) return false;  // (wave-uniform) no condition violated: the common case
  key = min4(key);
  term = key == KEY_NONE ? 0 : FW_TERM_VAR(key_var(key));
  return true;
}

// Where one aircraft's integration stands at the start of a trial step (the resumable part of the
// state besides Y and F): what the one-lane integrator hands over (rk45 handoff, fw_device.hpp).
struct QRun {
  double t, t_new, h_abs, min_step;
  int rejected, nfev, nacc;
};

#ifndef FW_QUAD_DIAG_FOLD
#define FW_QUAD_DIAG_FOLD 3  // timing diagnostics only (below): 3 = all pairs, the shipped integrator
#endif
#ifndef FW_QUAD_UNROLL
#define FW_QUAD_UNROLL 1  // 0 = the stage machine below (one RHS site per loop iteration), A/B switch
#endif

// rk45() on a quad: same step-size control and failure semantics; each lane folds its 3 pairs (6
// elements), norms are quad sums.  Y: this lane's slots of the accepted state (in and out).
// resume = false: a fresh integration from Y (R is output only); resume = true: continue at the
// trial step R describes (begin_attempt done: t, t_new, h_abs, min_step, rejected set; F = f(t, Y)).
//
// Every lane of a wave runs the same sequence of RHS evaluations -- f0, the initial-step probe, then
// trial steps of exactly six (K1..K5 and the FSAL f(t_new, y_new)), accepted or rejected -- so the
// stage is wave-uniform and one trial step is written out with its six RHS sites: the accumulators
// then have static lifetimes (the stage machine's switch merged them at the loop head with register
// copies).  Lanes that finish or fail run on masked, as in rk45().
#if FW_QUAD_UNROLL
template <typename T, typename C, typename A>
__device__ __forceinline__ int rk45_quad_core(const C& c, const A& a, const QCtx<T>& Q, V2<T> (&Y)[3], V2<T> (&F)[3],
                                              QRun& R, bool resume) {
  using V = V2<T>;
  using namespace dp5;
  constexpr int NQ = 3;
  // pairs of the trial-step folds (Dormand-Prince stages, error norm, acceptance): NQ.  Diagnostic builds only
  // (FW_QUAD_DIAG_FOLD=2, tools/r05_fold8.sh; wrong results): the fold load of an 8-lane group (3 elements a lane)
  constexpr int NF = FW_QUAD_DIAG_FOLD;
  static_assert(NF >= 1 && NF <= NQ, "FW_QUAD_DIAG_FOLD: 1..3 pairs");
  const T rtol = c.rtol, atol = c.atol;
  const double t_bound = c.t_bound;
  const T inv_sqrt_n = T(0.22941573387056177);  // 1 / sqrt(19)
  V ER[NQ], ys[NQ], K[NQ], P2v[NQ], P3[NQ], P4[NQ], P5[NQ], YB[NQ];
  double t = 0.0, h_abs = 0.0, t_new = 0.0, min_step = 0.0;
  T ht = T(0);
  bool rejected = false, active = true, begin_step = false, seeded = false;
  int result = 0, nfev = 0, nacc = 0;
  auto iscale = [&](V y) {
    V s;
    s.x = frcp(atol + fabs(y.x) * rtol);
    s.y = frcp(atol + fabs(y.y) * rtol);
    return s;
  };
  auto sq2 = [](V v) { return v.x * v.x + v.y * v.y; };
  // K = f(ys) at evaluation site k of a sequence begun with `nfev` evaluations done; `room` = evaluations
  // left before the budget (the bookkeeping of rk45()'s eval: one compare per evaluation, the count
  // updated per sequence).  False once no lane of the wave integrates any more.  `tight`: some lane of the
  // wave may reach its budget within the sequence (wave-uniform) -- otherwise an evaluation without a
  // violated condition anywhere in the wave goes on with two scalar branches.
  int room = c.max_nfev;
  bool tight = true;
  auto eval = [&](bool first, int k) {
    int term = 0;
    const bool viol = rhs_quad(c, a, Q, first, (const T*)ys, (T*)K, term);
    if (!viol && !tight) return true;
    const bool stop = active && (term != 0 || k >= room);
    if (any_lane(stop)) {
      if (stop) {
        result = term ? term : -2;
        nfev += k;
        active = false;
      }
      return any_lane(active);
    }
    return true;
  };
  auto seed = [&]() {  // stage-1 input and accumulators of a trial step
#pragma unroll
    for (int p = NF; p < NQ; p++) ys[p] = Y[p];  // (diagnostic builds: the pairs the folds skip stay at Y)
#pragma unroll
    for (int p = 0; p < NF; p++) {
      const V f = F[p];
      ys[p] = Y[p] + (f * T(A10)) * ht;
      P2v[p] = f * T(A20);
      P3[p] = f * T(A30);
      P4[p] = f * T(A40);
      P5[p] = f * T(A50);
      YB[p] = f * T(B0);
      ER[p] = f * T(E0);
    }
  };
  if (resume) {
    t = R.t;
    t_new = R.t_new;
    h_abs = R.h_abs;
    min_step = R.min_step;
    rejected = R.rejected != 0;
    nfev = R.nfev;
    nacc = R.nacc;
    ht = (T)(t_new - t);
    seed();
    seeded = true;
  } else {
#pragma unroll
    for (int p = 0; p < NQ; p++) ys[p] = Y[p];
    if (!eval(true, 1)) goto done;
    T d1;
    double h0;
    {  // f0; select_initial_step (common.py:68-110)
      T d0s = T(0), d1s = T(0);
#pragma unroll
      for (int p = 0; p < NQ; p++) {
        F[p] = K[p];
        const V isc = iscale(Y[p]);
        d0s += sq2(Y[p] * isc);
        d1s += sq2(K[p] * isc);
      }
      const T d0 = fsqrt(qd::sum4(d0s)) * inv_sqrt_n;
      d1 = fsqrt(qd::sum4(d1s)) * inv_sqrt_n;
      h0 = (d0 < T(1e-5) || d1 < T(1e-5)) ? 1e-6 : 0.01 * (double)d0 / (double)d1;
      if (h0 > t_bound) h0 = t_bound;
      const T h0t = (T)h0;
#pragma unroll
      for (int p = 0; p < NQ; p++) ys[p] = Y[p] + h0t * F[p];
    }
    if (!eval(false, 2)) goto done;
    if (active) nfev = 2;
    {  // probe; select_initial_step (common.py:111-134)
      T d2s = T(0);
#pragma unroll
      for (int p = 0; p < NQ; p++) d2s += sq2((K[p] - F[p]) * iscale(Y[p]));
      const double d2 = (double)(fsqrt(qd::sum4(d2s)) * inv_sqrt_n) / h0;
      double h1;
      if ((double)d1 <= 1e-15 && d2 <= 1e-15) h1 = fmax(1e-6, h0 * 1e-3);
      else h1 = pow(0.01 / fmax((double)d1, d2), 1.0 / 5.0);
      h_abs = fmin(fmin(100 * h0, h1), t_bound);
      begin_step = active;
    }
  }
  for (;;) {
    if (!seeded) {
      if (begin_step) {  // RungeKutta._step_impl entry (rk.py:111-124)
        min_step = min_step_at(t);
        if (h_abs < min_step) h_abs = min_step;
        rejected = false;
      }
      // one trial step (rk.py:126-137)
      double h = h_abs;
      t_new = t + h;
      if (t_new - t_bound > 0) t_new = t_bound;
      h = t_new - t;
      h_abs = fabs(h);
      ht = (T)h;
      seed();
    }
    seeded = false;
    room = c.max_nfev - nfev;
    tight = any_lane(active && room <= 6);
    if (!eval(false, 1)) break;  // K1
#pragma unroll
    for (int p = 0; p < NF; p++) {
      ys[p] = Y[p] + (P2v[p] + K[p] * T(A21)) * ht;
      P3[p] += K[p] * T(A31);
      P4[p] += K[p] * T(A41);
      P5[p] += K[p] * T(A51);
    }
    if (!eval(false, 2)) break;  // K2
#pragma unroll
    for (int p = 0; p < NF; p++) {
      P3[p] += K[p] * T(A32);
      P4[p] += K[p] * T(A42);
      P5[p] += K[p] * T(A52);
      YB[p] += K[p] * T(B2);
      ER[p] += K[p] * T(E2);
      ys[p] = Y[p] + P3[p] * ht;
    }
    if (!eval(false, 3)) break;  // K3
#pragma unroll
    for (int p = 0; p < NF; p++) {
      P4[p] += K[p] * T(A43);
      P5[p] += K[p] * T(A53);
      YB[p] += K[p] * T(B3);
      ER[p] += K[p] * T(E3);
      ys[p] = Y[p] + P4[p] * ht;
    }
    if (!eval(false, 4)) break;  // K4
#pragma unroll
    for (int p = 0; p < NF; p++) {
      P5[p] += K[p] * T(A54);
      YB[p] += K[p] * T(B4);
      ER[p] += K[p] * T(E4);
      ys[p] = Y[p] + P5[p] * ht;
    }
    if (!eval(false, 5)) break;  // K5; ys <- y_new
#pragma unroll
    for (int p = 0; p < NF; p++) {
      YB[p] += K[p] * T(B5);
      ER[p] += K[p] * T(E5);
      ys[p] = Y[p] + ht * YB[p];
    }
    if (!eval(false, 6)) break;  // K = f(t_new, y_new): error norm + step control (rk.py:138-173)
    if (active) nfev += 6;
    T es = T(0);
#pragma unroll
    for (int p = 0; p < NF; p++) {
      const V e = (ER[p] + K[p] * T(E6)) * ht;
      const V y0 = Y[p], y1 = ys[p];
      V sc;
      sc.x = frcp(atol + fmax_abs(y0.x, y1.x) * rtol);
      sc.y = frcp(atol + fmax_abs(y0.y, y1.y) * rtol);
      es += sq2(e * sc);
    }
    const T en = fsqrt(qd::sum4(es)) * inv_sqrt_n;
    begin_step = false;
    if (active) {
      if (en < T(1)) {
        double factor = (en == T(0)) ? 10.0 : fmin(10.0, 0.9 * (double)fpow(en, T(-0.2)));
        if (rejected) factor = fmin(1.0, factor);
        h_abs *= factor;
        t = t_new;
#pragma unroll
        for (int p = 0; p < NF; p++) {
          Y[p] = ys[p];
          F[p] = K[p];
        }
        nacc++;
        if (t - t_bound >= 0.0) active = false;
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
    if (!any_lane(active)) break;
  }
done:
  R.nfev = nfev;
  R.nacc = nacc;
  return result;
}
#else
template <typename T, typename C, typename A>
__device__ __forceinline__ int rk45_quad_core(const C& c, const A& a, const QCtx<T>& Q, V2<T> (&Y)[3], V2<T> (&F)[3],
                                              QRun& R, bool resume) {
  using V = V2<T>;
  using namespace dp5;
  constexpr int NQ = 3;
  const T rtol = c.rtol, atol = c.atol;
  const double t_bound = c.t_bound;
  const T inv_sqrt_n = T(0.22941573387056177);  // 1 / sqrt(19)
  V ER[NQ], ys[NQ], K[NQ], P2v[NQ], P3[NQ], P4[NQ], P5[NQ], YB[NQ];
  double t = 0.0, h_abs = 0.0, h0 = 0.0, t_new = 0.0, min_step = 0.0;
  T ht = T(0), d1 = T(0);
  bool rejected = false, active = true;
  int result = 0, nfev = 0, nacc = 0;
  int stage = 0;
#pragma unroll
  for (int p = 0; p < NQ; p++) ys[p] = Y[p];
  if (resume) {  // the trial step's stage-1 input and seeded accumulators (rk45 begin_attempt)
    t = R.t;
    t_new = R.t_new;
    h_abs = R.h_abs;
    min_step = R.min_step;
    rejected = R.rejected != 0;
    nfev = R.nfev;
    nacc = R.nacc;
    ht = (T)(t_new - t);
#pragma unroll
    for (int p = 0; p < NQ; p++) {
      const V f = F[p];
      ys[p] = Y[p] + (f * T(A10)) * ht;
      P2v[p] = f * T(A20);
      P3[p] = f * T(A30);
      P4[p] = f * T(A40);
      P5[p] = f * T(A50);
      YB[p] = f * T(B0);
      ER[p] = f * T(E0);
    }
    stage = 2;
  }
  auto iscale = [&](V y) {
    V s;
    s.x = frcp(atol + fabs(y.x) * rtol);
    s.y = frcp(atol + fabs(y.y) * rtol);
    return s;
  };
  auto sq2 = [](V v) { return v.x * v.x + v.y * v.y; };

  for (;;) {
    if (!any_lane(active)) break;
    {
      int term = 0;
      (void)rhs_quad(c, a, Q, stage == 0, (const T*)ys, (T*)K, term);
      if (active) {
        nfev++;
        if (term) {
          result = term;
          active = false;
        } else if (nfev >= c.max_nfev) {
          result = -2;
          active = false;
        }
      }
    }
    bool begin_step = false, begin_attempt = false;
    if (stage == 0) {  // f0; select_initial_step (common.py:68-110)
      T d0s = T(0), d1s = T(0);
#pragma unroll
      for (int p = 0; p < NQ; p++) {
        F[p] = K[p];
        const V isc = iscale(Y[p]);
        d0s += sq2(Y[p] * isc);
        d1s += sq2(K[p] * isc);
      }
      const T d0 = fsqrt(qd::sum4(d0s)) * inv_sqrt_n;
      d1 = fsqrt(qd::sum4(d1s)) * inv_sqrt_n;
      h0 = (d0 < T(1e-5) || d1 < T(1e-5)) ? 1e-6 : 0.01 * (double)d0 / (double)d1;
      if (h0 > t_bound) h0 = t_bound;
      const T h0t = (T)h0;
#pragma unroll
      for (int p = 0; p < NQ; p++) ys[p] = Y[p] + h0t * F[p];
      stage = 1;
    } else if (stage == 1) {  // probe; select_initial_step (common.py:111-134)
      T d2s = T(0);
#pragma unroll
      for (int p = 0; p < NQ; p++) d2s += sq2((K[p] - F[p]) * iscale(Y[p]));
      const double d2 = (double)(fsqrt(qd::sum4(d2s)) * inv_sqrt_n) / h0;
      double h1;
      if ((double)d1 <= 1e-15 && d2 <= 1e-15) h1 = fmax(1e-6, h0 * 1e-3);
      else h1 = pow(0.01 / fmax((double)d1, d2), 1.0 / 5.0);
      h_abs = fmin(fmin(100 * h0, h1), t_bound);
      begin_step = active;
      stage = 2;
    } else if (stage == 2) {  // K = K1
#pragma unroll
      for (int p = 0; p < NQ; p++) {
        ys[p] = Y[p] + (P2v[p] + K[p] * T(A21)) * ht;
        P3[p] += K[p] * T(A31);
        P4[p] += K[p] * T(A41);
        P5[p] += K[p] * T(A51);
      }
      stage = 3;
    } else if (stage == 3) {  // K = K2
#pragma unroll
      for (int p = 0; p < NQ; p++) {
        P3[p] += K[p] * T(A32);
        P4[p] += K[p] * T(A42);
        P5[p] += K[p] * T(A52);
        YB[p] += K[p] * T(B2);
        ER[p] += K[p] * T(E2);
        ys[p] = Y[p] + P3[p] * ht;
      }
      stage = 4;
    } else if (stage == 4) {  // K = K3
#pragma unroll
      for (int p = 0; p < NQ; p++) {
        P4[p] += K[p] * T(A43);
        P5[p] += K[p] * T(A53);
        YB[p] += K[p] * T(B3);
        ER[p] += K[p] * T(E3);
        ys[p] = Y[p] + P4[p] * ht;
      }
      stage = 5;
    } else if (stage == 5) {  // K = K4
#pragma unroll
      for (int p = 0; p < NQ; p++) {
        P5[p] += K[p] * T(A54);
        YB[p] += K[p] * T(B4);
        ER[p] += K[p] * T(E4);
        ys[p] = Y[p] + P5[p] * ht;
      }
      stage = 6;
    } else if (stage == 6) {  // K = K5; ys <- y_new
#pragma unroll
      for (int p = 0; p < NQ; p++) {
        YB[p] += K[p] * T(B5);
        ER[p] += K[p] * T(E5);
        ys[p] = Y[p] + ht * YB[p];
      }
      stage = 7;
    } else {  // K = f(t_new, y_new): error norm + step control (rk.py:138-173)
      T es = T(0);
#pragma unroll
      for (int p = 0; p < NQ; p++) {
        const V e = (ER[p] + K[p] * T(E6)) * ht;
        const V y0 = Y[p], y1 = ys[p];
        V sc;
        sc.x = frcp(atol + fmax_abs(y0.x, y1.x) * rtol);
        sc.y = frcp(atol + fmax_abs(y0.y, y1.y) * rtol);
        es += sq2(e * sc);
      }
      const T en = fsqrt(qd::sum4(es)) * inv_sqrt_n;
      if (active) {
        if (en < T(1)) {
          double factor = (en == T(0)) ? 10.0 : fmin(10.0, 0.9 * (double)fpow(en, T(-0.2)));
          if (rejected) factor = fmin(1.0, factor);
          h_abs *= factor;
          t = t_new;
#pragma unroll
          for (int p = 0; p < NQ; p++) {
            Y[p] = ys[p];
            F[p] = K[p];
          }
          nacc++;
          if (t - t_bound >= 0.0) active = false;
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
    if (begin_attempt) {  // one trial step (rk.py:126-137); stage 1 input, accumulators seeded
      double h = h_abs;
      t_new = t + h;
      if (t_new - t_bound > 0) t_new = t_bound;
      h = t_new - t;
      h_abs = fabs(h);
      ht = (T)h;
#pragma unroll
      for (int p = 0; p < NQ; p++) {
        const V f = F[p];
        ys[p] = Y[p] + (f * T(A10)) * ht;
        P2v[p] = f * T(A20);
        P3[p] = f * T(A30);
        P4[p] = f * T(A40);
        P5[p] = f * T(A50);
        YB[p] = f * T(B0);
        ER[p] = f * T(E0);
      }
    }
  }
  R.nfev = nfev;
  R.nacc = nacc;
  return result;
}
#endif  // FW_QUAD_UNROLL

// a fresh integration of the state y_io (the full 19-element state on every lane of the quad, in and out)
template <typename T, typename C, typename A>
__device__ __forceinline__ int rk45_quad(const C& c, const A& a, const StepCtx<T>& X, T* y_io, int& nfev, int& nacc,
                                         int r) {
  using V = V2<T>;
  constexpr int NQ = 3;
  const QCtx<T> Q = qctx<T>(c, a, X, r);
  V Y[NQ], F[NQ];
  {
    auto s3 = [r](T a0, T a1, T a2) { return r == 0 ? a0 : (r == 1 ? a1 : a2); };
    T v[6];  // slot k of row r = y[1 + 3k + r]; lane 3: e0, 0, ...
    v[0] = Q.row ? s3(y_io[1], y_io[2], y_io[3]) : y_io[0];
#pragma unroll
    for (int k = 1; k < 6; k++) v[k] = Q.row ? s3(y_io[3 * k + 1], y_io[3 * k + 2], y_io[3 * k + 3]) : T(0);
#pragma unroll
    for (int p = 0; p < NQ; p++) {
      Y[p].x = v[2 * p];
      Y[p].y = v[2 * p + 1];
    }
  }
  QRun R;
  const int result = rk45_quad_core(c, a, Q, Y, F, R, false);
  nfev = R.nfev;
  nacc = R.nacc;
  // the accepted state back on every lane of the quad
  T v[6];
#pragma unroll
  for (int p = 0; p < NQ; p++) {
    v[2 * p] = Y[p].x;
    v[2 * p + 1] = Y[p].y;
  }
  y_io[0] = bc<3>(v[0]);
#pragma unroll
  for (int k = 0; k < 6; k++) {
    y_io[1 + 3 * k] = bc<0>(v[k]);
    y_io[2 + 3 * k] = bc<1>(v[k]);
    y_io[3 + 3 * k] = bc<2>(v[k]);
  }
  return result;
}

// ---------------------------------------------------------------------------
// Tail handoff (rk45 HO, fw_device.hpp): the at most 16 aircraft of a one-lane wave still integrating
// continue on lane quads of the same wave.  Their Y / F rows stay in the one-lane integrator's LDS
// slots (the quads read and write them in place); the step-control state and the step context go
// through a per-wave LDS slot array.  Quad k (lanes 4k..4k+3) takes the k-th integrating lane.
// ---------------------------------------------------------------------------
// 160 B in fp64 (QRun's fields unpadded, `rejected` in src's bit 8): 64 slots + the one-lane LDS state
// = 40 KB, four one-wave blocks per CU (at 168 B the fp64 one-lane instances fit three)
template <typename T>
struct HoSlot {
  double t, t_new, h_abs, min_step;
  StepCtx<T> X;
  int nfev, nacc;
  int src;  // source lane | rejected << 8
  int result;
};

// true on the handed-off lanes, whose R (nfev, nacc) and result are then the integration's
template <typename T, typename C, typename A>
__device__ __forceinline__ bool handoff(const C& c, const A& a, const StepCtx<T>& X, V2<T>* sy, V2<T>* sf, int stride,
                                        bool active, QRun& R, int& result, void* ho) {
  HoSlot<T>* st = (HoSlot<T>*)ho;
  const int lane = (int)(threadIdx.x & 63);
  const unsigned long long am = __ballot(active);
  const int na = __popcll(am);
  const int kk = (int)__builtin_amdgcn_mbcnt_hi((unsigned)(am >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)am, 0u));
  if (active) {
    st[kk].t = R.t;
    st[kk].t_new = R.t_new;
    st[kk].h_abs = R.h_abs;
    st[kk].min_step = R.min_step;
    st[kk].nfev = R.nfev;
    st[kk].nacc = R.nacc;
    st[kk].X = X;
    st[kk].src = lane | (R.rejected ? 256 : 0);
  }
  __syncthreads();
  const int k = lane >> 2, r = lane & 3;
  if (k < na) {
    const int src = st[k].src & 255;
    QRun Rq{st[k].t, st[k].t_new, st[k].h_abs, st[k].min_step, st[k].src >> 8, st[k].nfev, st[k].nacc};
    const StepCtx<T> Xs = st[k].X;
    const QCtx<T> Q = qctx<T>(c, a, Xs, r);
    V2<T>* const ysrc = sy - lane + src;
    V2<T>* const fsrc = sf - lane + src;
    auto el = [stride](V2<T>* base, int e) -> T& { return ((T*)(base + (e >> 1) * stride))[e & 1]; };
    int e[6];  // element of this lane's slot m (row r of the m-th 3-vector; lane 3: e0 only)
#pragma unroll
    for (int m = 0; m < 6; m++) e[m] = r < 3 ? 1 + 3 * m + r : (m == 0 ? 0 : -1);
    V2<T> Yq[3], Fq[3];
#pragma unroll
    for (int p = 0; p < 3; p++) {
      Yq[p].x = e[2 * p] >= 0 ? el(ysrc, e[2 * p]) : T(0);
      Yq[p].y = e[2 * p + 1] >= 0 ? el(ysrc, e[2 * p + 1]) : T(0);
      Fq[p].x = e[2 * p] >= 0 ? el(fsrc, e[2 * p]) : T(0);
      Fq[p].y = e[2 * p + 1] >= 0 ? el(fsrc, e[2 * p + 1]) : T(0);
    }
    const int res = rk45_quad_core(c, a, Q, Yq, Fq, Rq, true);
#pragma unroll
    for (int p = 0; p < 3; p++) {
      if (e[2 * p] >= 0) el(ysrc, e[2 * p]) = Yq[p].x;
      if (e[2 * p + 1] >= 0) el(ysrc, e[2 * p + 1]) = Yq[p].y;
    }
    if (r == 0) {
      st[k].result = res;
      st[k].nfev = Rq.nfev;
      st[k].nacc = Rq.nacc;
    }
  }
  __syncthreads();
  if (active) {
    result = st[kk].result;
    R.nfev = st[kk].nfev;
    R.nacc = st[kk].nacc;
  }
  return active;
}

}  // namespace qd
