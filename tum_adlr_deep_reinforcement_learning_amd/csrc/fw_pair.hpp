// fw_pair.hpp -- one aircraft's RK45 integration on a PAIR of lanes (included by fw_device.hpp after fw_quad.hpp).
//
// Round 6 (the round-5 review's first item): at 65536 aircraft the one-lane integrator runs 1024 waves, one per
// SIMD, and a lone wave issues a VALU instruction every ~4 cycles where the SIMD could take one every 2 from two
// waves.  Two lanes per aircraft give 2048 waves; if the instance fits 256 registers (two waves per SIMD) every
// SIMD holds two of them.  The split is fw_quad.hpp's ROW split with two virtual quad rows per lane:
//
//   lane 0 of the pair holds rows 0 and 1, lane 1 rows 2 and 3 (row 3 = e0 and zeros, as quad lane 3)
//
// Every row-valued quantity is a V2 (x = row 2h, y = row 2h + 1, h = lane & 1); the row formulas of rhs_quad
// run on both components (packed where the backend pairs them), row values cross the pair with one DPP swap,
// and the scalar front's transcendental chains are split over the two lanes as the quad splits them (lane 1:
// beta, lane 0: alpha).  The Dormand-Prince folds, error norm and conditions run on 12 elements per lane (19 in
// one lane, 6 on a quad lane); norms are pair sums, the same bits on both lanes.
//
// Reference behaviour: as rhs() / rk45() and fw_quad.hpp (PyFly._dynamics / _forces / _f_*,
// pyfly.py:1450-1747; scipy 1.15.3 RK45, rk.py:111-173, common.py:68-134).  Sums are formed rows before lanes,
// so results differ from the one-lane path by rounding (fp64 parity: tests/test_gpu_pair.py).
#pragma once

namespace pr {

template <typename T>
using R = V2<T>;

// lane h's value on both lanes of the pair (quad_perm inside a quad: pairs are lanes 0-1 and 2-3)
template <int H>
__device__ __forceinline__ int bl_i(int x) {
  return qd::perm_i<H, H, 2 + H, 2 + H>(x);
}
template <int H>
__device__ __forceinline__ float bl(float x) {
  return qd::perm<H, H, 2 + H, 2 + H>(x);
}
template <int H>
__device__ __forceinline__ double bl(double x) {
  return qd::perm<H, H, 2 + H, 2 + H>(x);
}
// the partner lane's value
template <typename T>
__device__ __forceinline__ T swp(T x) {
  return qd::perm<1, 0, 3, 2>(x);
}
// row K's value on both lanes
template <int K, typename T>
__device__ __forceinline__ T bc(R<T> x) {
  return bl<(K >> 1)>((K & 1) ? x.y : x.x);
}
// per-lane select of computed values: a on lane 0 of every pair, b on lane 1 -- one v_cndmask against a constant
// lane mask (a conditional expression with work in its arms compiles to exec-masked branches, fw_quad.hpp rowsel)
__device__ __forceinline__ float psel(float a, float b) {
  float out;
  asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(out) : "v"(b), "v"(a), "s"(0x5555555555555555ull));
  return out;
}
__device__ __forceinline__ double psel(double a, double b) {
  const unsigned long long x = (unsigned long long)__double_as_longlong(a);
  const unsigned long long y = (unsigned long long)__double_as_longlong(b);
  const float lo = psel(__int_as_float((int)(unsigned)x), __int_as_float((int)(unsigned)y));
  const float hi = psel(__int_as_float((int)(unsigned)(x >> 32)), __int_as_float((int)(unsigned)(y >> 32)));
  return __longlong_as_double((long long)(((unsigned long long)(unsigned)__float_as_int(hi) << 32) |
                                          (unsigned)__float_as_int(lo)));
}
// rows (r + 1) % 3 / (r + 2) % 3 of a row-distributed 3-vector (row 3 keeps its own)
template <typename T>
__device__ __forceinline__ R<T> nx1(R<T> x) {
  const T px = swp(x.x);  // lane 0 receives row 2, lane 1 row 0
  R<T> o;
  o.x = psel(x.y, px);    // row 0 <- row 1; row 2 <- row 0
  o.y = psel(px, x.y);    // row 1 <- row 2; row 3 stays
  return o;
}
template <typename T>
__device__ __forceinline__ R<T> nx2(R<T> x) {
  R<T> o;
  o.x = swp(psel(x.y, x.x));  // lane 0 sends row 1, lane 1 row 2: row 0 <- row 2; row 2 <- row 1
  o.y = psel(x.x, x.y);       // row 1 <- row 0; row 3 stays
  return o;
}
// sum over the four rows (the same bits on both lanes)
template <typename T>
__device__ __forceinline__ T sum4(R<T> x) {
  const T s = x.x + x.y;
  return s + swp(s);
}
__device__ __forceinline__ int min2(int k) { return min(k, qd::perm_i<1, 0, 3, 2>(k)); }

// Per-lane constants of one step (rows 2h, 2h + 1; row 3: no conditions, zero coefficients)
template <typename T>
struct PCtx {
  bool h0;
  R<T> rowf;                 // 1 on rows 0..2, 0 on row 3
  T sgn1;                    // +1 on lane 1 (the beta chain's exponential), -1 on lane 0
  R<T> w0, w1, w2;           // steady wind components r, r+1, r+2 (cyclic)
  R<T> tl, ta, sp;           // linear / angular turbulence and actuator set-point of the rows
  T elev0, ail0;
  R<T> om_cl, om_ch, om_vl, om_vh, pos_cl, pos_ch, vel_cl, vel_ch, vel_vl, vel_vh, act_cl, act_ch, act_vl, act_vh;
  R<T> dlo, dhi;             // actuator rate clip interval (+-inf: none)
  R<T> ac0, ac1, ac2, ac3, ac4, ac5;
  R<T> kx, ky, kz, kw;       // gyroscopic terms in the row's cyclic frame (fw_quad.hpp QCtx)
  // lift / moment / drag row formula (rhs_quad) and side-force / torque-row formula coefficients per row
  R<T> pa, pb, pg, ph, c0, mu, mv, mw, kq, kde, kde2, kb1, kb2, fK;
  R<T> tK, t0, tb, tp, tr, tda, tpr;
  R<T> kprop;
};

template <typename T, typename C, typename A>
__device__ __forceinline__ PCtx<T> pctx(const C& c, const A& a, const StepCtx<T>& X, int h) {
  PCtx<T> Q;
  const T inf = T(__builtin_inf());
  const T z = T(0), one = T(1), two = T(2);
  Q.h0 = h == 0;
  // a row-valued constant from the four rows' values
  auto rv = [&](T r0, T r1, T r2, T r3) {
    R<T> v;
    v.x = h == 0 ? r0 : r2;
    v.y = h == 0 ? r1 : r3;
    return v;
  };
  Q.rowf = rv(one, one, one, z);
  Q.sgn1 = h == 1 ? T(1) : T(-1);
  Q.w0 = rv(X.wind[0], X.wind[1], X.wind[2], z);
  Q.w1 = rv(X.wind[1], X.wind[2], X.wind[0], z);
  Q.w2 = rv(X.wind[2], X.wind[0], X.wind[1], z);
  Q.tl = rv(X.tl[0], X.tl[1], X.tl[2], z);
  Q.ta = rv(X.ta[0], X.ta[1], X.ta[2], z);
  Q.sp = rv(X.sp[0], X.sp[1], X.sp[2], z);
  Q.elev0 = X.elev0;
  Q.ail0 = X.ail0;
  auto lim = [&](int v0, R<T>& cl, R<T>& ch, R<T>& vl, R<T>& vh) {
    T l[3], hh[3], lo[3], hi[3];
#pragma unroll
    for (int j = 0; j < 3; j++) {
      const uint32_t bit = 1u << (v0 + j);
      const bool hc = (c.cmask & bit) != 0, hk = (c.clipmask & bit) != 0;
      l[j] = hc ? c.lim[v0 + j].cmin : -inf;
      hh[j] = hc ? c.lim[v0 + j].cmax : inf;
      lo[j] = hk ? c.lim[v0 + j].vmin : -inf;  // no clip: +-inf (clipv is then the identity)
      hi[j] = hk ? c.lim[v0 + j].vmax : inf;
    }
    cl = rv(l[0], l[1], l[2], -inf);
    ch = rv(hh[0], hh[1], hh[2], inf);
    vl = rv(lo[0], lo[1], lo[2], -inf);
    vh = rv(hi[0], hi[1], hi[2], inf);
  };
  R<T> pvl, pvh;
  lim(FW_V_OMEGA_P, Q.om_cl, Q.om_ch, Q.om_vl, Q.om_vh);
  lim(FW_V_POS_N, Q.pos_cl, Q.pos_ch, pvl, pvh);  // positions are checked, never clipped
  lim(FW_V_VEL_U, Q.vel_cl, Q.vel_ch, Q.vel_vl, Q.vel_vh);
  lim(FW_V_ACT0, Q.act_cl, Q.act_ch, Q.act_vl, Q.act_vh);
  T dm[3];
#pragma unroll
  for (int j = 0; j < 3; j++) dm[j] = ((c.dotmask >> j) & 1u) ? c.dot_max[j] : inf;
  Q.dlo = rv(-dm[0], -dm[1], -dm[2], -inf);
  Q.dhi = rv(dm[0], dm[1], dm[2], inf);
  Q.ac0 = rv(c.ac[0][0], c.ac[1][0], c.ac[2][0], z);
  Q.ac1 = rv(c.ac[0][1], c.ac[1][1], c.ac[2][1], z);
  Q.ac2 = rv(c.ac[0][2], c.ac[1][2], c.ac[2][2], z);
  Q.ac3 = rv(c.ac[0][3], c.ac[1][3], c.ac[2][3], z);
  Q.ac4 = rv(c.ac[0][4], c.ac[1][4], c.ac[2][4], z);
  Q.ac5 = rv(c.ac[0][5], c.ac[1][5], c.ac[2][5], z);
  Q.kx = rv(c.gam[1], z, z, z);
  Q.ky = rv(-c.gam[2], c.gam[5], c.gam[7], z);
  Q.kz = rv(z, z, -c.gam[1], z);
  Q.kw = rv(z, -c.gam[6], z, z);
  // rhs_quad's lift / pitch-moment / drag row formula: row 0 lift, row 1 moment (over Jy), row 2 drag, row 3 as row 0
  Q.pa = rv(a.CL0, a.Cm0, a.CL0, a.CL0);
  Q.pb = rv(a.CLa, a.Cma, a.CLa, a.CLa);
  Q.pg = rv(one, one, a.CL0 * a.inv_pi_e_ar, one);
  Q.ph = rv(z, z, a.CLa * a.inv_pi_e_ar, z);
  Q.c0 = rv(z, z, a.CDp, z);
  Q.mu = rv(two, z, z, two);
  Q.mv = rv(z, z, two, z);
  Q.mw = rv(z, a.Cmfp, z, z);
  Q.kq = rv(a.kCLq, a.kCmq, a.kCDq, a.kCLq);
  Q.kde = rv(a.CLde, a.Cmde, z, a.CLde);
  Q.kde2 = rv(z, z, a.CDde, z);
  Q.kb1 = rv(z, z, a.CDb1, z);
  Q.kb2 = rv(z, z, a.CDb2, z);
  const T jm = a.qSc * c.inv_Jy;
  Q.fK = rv(a.qS, jm, a.qS, a.qS);
  // side force Y on row 1, roll / yaw torque rows on rows 0 / 2 (fw_quad.hpp qctx), row 3 zero
  const T g3 = c.gam[3], g4 = c.gam[4], g8 = c.gam[8];
  auto tq = [&](T cl, T cn, T cy) { return rv(g3 * cl + g4 * cn, cy, g4 * cl + g8 * cn, z); };
  Q.tK = rv(a.qSb, a.qS, a.qSb, z);
  Q.t0 = tq(a.Cl0, a.Cn0, a.CY0);
  Q.tb = tq(a.Clb, a.Cnb, a.CYb);
  Q.tp = tq(a.Clp, a.Cnp, a.CYp);
  Q.tr = tq(a.Clr, a.Cnr, a.CYr);
  Q.tda = tq(a.Clda, a.Cnda, a.CYda);
  Q.tpr = rv(-a.kTP2 * g3, z, -a.kTP2 * g4, z);
  Q.kprop = rv(a.prop_k, z, z, z);
  return Q;
}

template <typename T>
__device__ __forceinline__ R<T> clip2(R<T> x, R<T> lo, R<T> hi) {
  R<T> o;
  o.x = clipv(x.x, lo.x, hi.x);
  o.y = clipv(x.y, lo.y, hi.y);
  return o;
}

// PyFly._dynamics (pyfly.py:1450-1482) of the lane's two rows: s = the lane's 6 stage values (kinds: eps / e0,
// omega, pos, vel, actuator, rate), ds = their derivatives.  As rhs_quad: term = the aircraft's first violated
// condition; returns whether any aircraft of the wave violated one (wave-uniform; term only written then).
template <typename T, typename C, typename A>
__device__ __forceinline__ bool rhs_pair(const C& c, const A& a, const PCtx<T>& Q, bool first, const R<T>* s, R<T>* ds,
                                         int& term) {
  using RR = R<T>;
  const bool h0 = Q.h0;
  const int rb = h0 ? 0 : 2;  // the lane's first row
  int key = qd::KEY_NONE;
  RR om = s[1], vel = s[3], av = s[4], ad = s[5];
  T elev = Q.elev0, ail = Q.ail0;
  if (!first) {  // _set_states_from_ode_solution(save=False) + Actuation.set_states (pyfly.py:479-492)
    auto rowcond = [&](RR x, int v0, RR cl, RR ch, RR vl, RR vh, int k0, bool clip) {
      if (c.cmask & (7u << v0)) {  // first violation = the smallest key (groups and rows in rhs()'s order)
        const bool vx = (x.x < cl.x) | (x.x > ch.x), vy = (x.y < cl.y) | (x.y > ch.y);
        key = min(key, vx ? k0 + rb : qd::KEY_NONE);
        key = min(key, vy ? k0 + rb + 1 : qd::KEY_NONE);
      }
      if (clip && (c.clipmask & (7u << v0))) return clip2(x, vl, vh);
      return x;
    };
    om = rowcond(om, FW_V_OMEGA_P, Q.om_cl, Q.om_ch, Q.om_vl, Q.om_vh, 0, true);
    (void)rowcond(s[2], FW_V_POS_N, Q.pos_cl, Q.pos_ch, Q.pos_cl, Q.pos_ch, 3, false);
    vel = rowcond(vel, FW_V_VEL_U, Q.vel_cl, Q.vel_ch, Q.vel_vl, Q.vel_vh, 6, true);
    av = rowcond(av, FW_V_ACT0, Q.act_cl, Q.act_ch, Q.act_vl, Q.act_vh, 9, true);
    if (c.dotmask) ad = clip2(ad, Q.dlo, Q.dhi);
    const T a0 = bc<0>(av), a1 = bc<1>(av);
    if (c.elevon) {
      ail = (-a0 + a1) * T(0.5);
      elev = (a0 + a1) * T(0.5);
      ail = qd::ucond(c, FW_V_AILERON, ail, key, 12);
      elev = qd::ucond(c, FW_V_ELEVATOR, elev, key, 13);
    } else {
      elev = a0;
      ail = a1;
    }
  }
  const T thr = bc<2>(av);
  const RR er = s[0];  // raw attitude (pyfly.py:1464): eps_r, row 3: e0
  const T e0 = bc<3>(er);
  const RR er1 = nx1(er), er2 = nx2(er);

  // ---- _forces (pyfly.py:1484-1643) ----
  const RR omt = om - Q.ta;
  const T p = bc<0>(omt), q = bc<1>(omt), r = bc<2>(omt);
  const RR Rrr = T(-1) + T(2) * (e0 * e0 + er * er);
  const RR Rr1 = T(2) * (er * er1 + er2 * e0);
  const RR Rr2 = T(2) * (er * er2 - er1 * e0);
  const RR var_ = vel - (Rrr * Q.w0 + Rr1 * Q.w1 + Rr2 * Q.w2 + Q.tl);
  const T va0 = bc<0>(var_), va1 = bc<1>(var_), va2 = bc<2>(var_);
  // the scalar front's transcendental chains: lane 1 beta, lane 0 alpha (rhs_quad)
  const T rxz2 = va0 * va0 + va2 * va2;
  const T sq = fsqrt(psel(rxz2, rxz2 + va1 * va1));
  const T rxz = bl<0>(sq), Va_raw = bl<1>(sq);
  const T at = fatan2(psel(va2, va1), psel(va0, rxz));
  T alpha = bl<0>(at), beta = bl<1>(at);
  const T Va = qd::ucond(c, FW_V_VA, Va_raw, key, 14);
  alpha = qd::ucond(c, FW_V_ALPHA, alpha, key, 15);
  beta = qd::ucond(c, FW_V_BETA, beta, key, 16);
  T irxz, iVr, iVa;
  {
    const T rc = frcp(sq);  // 1 / rxz on lane 0, 1 / Va_raw on lane 1
    irxz = bl<0>(rc);
    iVr = bl<1>(rc);
    iVa = ((c.clipmask >> FW_V_VA) & 1u) ? frcp(Va) : iVr;
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
  T sigma;
  if constexpr (sizeof(T) == 4) {  // one reciprocal (rhs_quad FW_QUAD_SIGMA_1RCP)
    const T l2e = T(1.4426950408889634);
    const T ex = __builtin_amdgcn_exp2f(fminf(fmaf(Q.sgn1 * (a.M * l2e), alpha, a.M * a.a0 * l2e), T(120)));
    const T S = T(1) + bl<0>(ex) + bl<1>(ex);
    sigma = S * frcp(S + a.sig_c);
  } else {
    const T ex = fexp(psel(-a.M * (alpha - a.a0), a.M * (alpha + a.a0)));
    sigma = frcp(T(1) + a.sig_c * frcp(T(1) + bl<0>(ex) + bl<1>(ex)));
  }
  const T osig = T(1) - sigma;
  const T ssa = sa * fabs(sa);
  const T qn = q * iVa;
  // lift / moment / drag rows as ONE formula with row constants (rhs_quad), then broadcast
  const RR P = (Q.pa + Q.pb * alpha) * (Q.pg + Q.ph * alpha);
  const RR Cr = Q.c0 + osig * P + (sigma * ssa) * (Q.mu * ca + Q.mv * sa + Q.mw);
  const RR Fr = Q.fK * V2a * (Cr + Q.kq * qn + Q.kde * elev + Q.kde2 * (elev * elev) + Q.kb1 * beta + Q.kb2 * (beta * beta));
  const T flift = bc<0>(Fr), fdrag = bc<2>(Fr);
  const T bp = a.hb * p * iVa, br = a.hb * r * iVa;
  const RR g2 = Q.tK * V2a * (Q.t0 + Q.tb * beta + Q.tp * bp + Q.tr * br + Q.tda * ail) + Q.tpr * (thr * thr);
  const T fy = bc<1>(g2);
  const T U = cb * (-fdrag) + sb * fy;
  RR fa;
  fa.x = psel(ca * U + sa * flift, sa * U - ca * flift);  // rows 0 / 2
  fa.y = sb * fdrag + cb * fy;                             // row 1 (row 3: unused, rowf = 0)
  const RR Dr = er * er + e0 * e0 - er1 * er1 - er2 * er2;
  RR fg;
  fg.x = a.mg * psel(Rr2.x, Dr.x);
  fg.y = a.mg * Rr1.y;
  const T Vd = Va + thr * (a.kmotor - Va);
  const RR fr = Q.kprop * Vd * (Vd - Va) + fg + fa;

  const RR om1 = nx1(om), om2 = nx2(om), vel1 = nx1(vel), vel2 = nx2(vel);
  const RR deps = T(0.5) * (om * e0 + om2 * er1 - om1 * er2);
  const T de0 = T(-0.5) * sum4(om * er);
  RR tw;  // the torque row: row 1 the pitch moment over Jy (Fr), rows 0 / 2 the combined torque rows (g2)
  tw.x = g2.x;
  tw.y = psel(Fr.y, g2.y);
  const RR dw = Q.kx * (om * om1) + Q.ky * (om1 * om2) + Q.kz * (om * om2) + Q.kw * (om2 * om2 - om1 * om1) + tw;
  const RR dp = Dr * vel + T(2) * (er * er1 - er2 * e0) * vel1 + T(2) * (er * er2 + er1 * e0) * vel2;
  const RR dv = om2 * vel1 - om1 * vel2 + fr * (a.inv_mass * Q.rowf);
  const RR da = av * Q.ac0 + Q.sp * Q.ac2 + ad * Q.ac1;
  const RR dd = av * Q.ac3 + Q.sp * Q.ac5 + ad * Q.ac4;
  RR d0 = deps;
  d0.y = psel(deps.y, de0);  // row 3: d e0
  ds[0] = d0;
  ds[1] = dw;
  ds[2] = dp;
  ds[3] = dv;
  ds[4] = da;
  ds[5] = dd;
  if (!any_lane(key != qd::KEY_NONE)) return false;
  key = min2(key);
  term = key == qd::KEY_NONE ? 0 : FW_TERM_VAR(qd::key_var(key));
  return true;
}

// rk45_quad_core on a pair: 6 row-pair values per lane, norms are pair sums; same step control and failure
// semantics (nfev / nacc in Rn).  The accepted state Y, its derivative F and the error sum ER live in this lane's
// LDS slots (sl[p * stride], p = 0..17: Y, F, ER; Y in and out), as the one-lane rk45 keeps y / f / error sum:
// in registers they pushed the instance past the 256 registers of two waves per SIMD (scratch spills)
template <typename T, typename C, typename A>
__device__ __forceinline__ int rk45_pair_core(const C& c, const A& a, const PCtx<T>& Q, R<T>* __restrict__ sl, int stride,
                                              qd::QRun& Rn) {
  using RR = R<T>;
  using namespace dp5;
  constexpr int NQ = 6;
  const T rtol = c.rtol, atol = c.atol;
  const double t_bound = c.t_bound;
  const T inv_sqrt_n = T(0.22941573387056177);  // 1 / sqrt(19)
#define Y(p) sl[(p) * stride]
#define F(p) sl[(NQ + (p)) * stride]
#define ER(p) sl[(2 * NQ + (p)) * stride]
  RR ys[NQ], K[NQ], P2v[NQ], P3[NQ], P4[NQ], P5[NQ], YB[NQ];
  double t = 0.0, h_abs = 0.0, t_new = 0.0, min_step = 0.0;
  T ht = T(0);
  bool rejected = false, active = true, begin_step = false;
  int result = 0, nfev = 0, nacc = 0;
  auto iscale = [&](RR y) {
    RR s;
    s.x = frcp(atol + fabs(y.x) * rtol);
    s.y = frcp(atol + fabs(y.y) * rtol);
    return s;
  };
  auto sq2 = [](RR v) { return v.x * v.x + v.y * v.y; };
  int room = c.max_nfev;
  bool tight = true;
  auto eval = [&](bool first, int k) {
    int term = 0;
    const bool viol = rhs_pair(c, a, Q, first, (const RR*)ys, (RR*)K, term);
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
#pragma unroll
  for (int p = 0; p < NQ; p++) ys[p] = Y(p);
  if (!eval(true, 1)) goto done;
  T d1;
  double h0;
  {  // f0; select_initial_step (common.py:68-110)
    T d0s = T(0), d1s = T(0);
#pragma unroll
    for (int p = 0; p < NQ; p++) {
      F(p) = K[p];
      const RR isc = iscale(Y(p));
      d0s += sq2(Y(p) * isc);
      d1s += sq2(K[p] * isc);
    }
    const T d0 = fsqrt(d0s + swp(d0s)) * inv_sqrt_n;
    d1 = fsqrt(d1s + swp(d1s)) * inv_sqrt_n;
    h0 = (d0 < T(1e-5) || d1 < T(1e-5)) ? 1e-6 : 0.01 * (double)d0 / (double)d1;
    if (h0 > t_bound) h0 = t_bound;
    const T h0t = (T)h0;
#pragma unroll
    for (int p = 0; p < NQ; p++) ys[p] = Y(p) + h0t * F(p);
  }
  if (!eval(false, 2)) goto done;
  if (active) nfev = 2;
  {  // probe; select_initial_step (common.py:111-134)
    T d2s = T(0);
#pragma unroll
    for (int p = 0; p < NQ; p++) d2s += sq2((K[p] - F(p)) * iscale(Y(p)));
    const double d2 = (double)(fsqrt(d2s + swp(d2s)) * inv_sqrt_n) / h0;
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
    {  // one trial step (rk.py:126-137)
      double h = h_abs;
      t_new = t + h;
      if (t_new - t_bound > 0) t_new = t_bound;
      h = t_new - t;
      h_abs = fabs(h);
      ht = (T)h;
#pragma unroll
      for (int p = 0; p < NQ; p++) {
        const RR f = F(p);
        ys[p] = Y(p) + (f * T(A10)) * ht;
        P2v[p] = f * T(A20);
        P3[p] = f * T(A30);
        P4[p] = f * T(A40);
        P5[p] = f * T(A50);
        YB[p] = f * T(B0);
        ER(p) = f * T(E0);
      }
    }
    room = c.max_nfev - nfev;
    tight = any_lane(active && room <= 6);
    if (!eval(false, 1)) break;  // K1
#pragma unroll
    for (int p = 0; p < NQ; p++) {
      ys[p] = Y(p) + (P2v[p] + K[p] * T(A21)) * ht;
      P3[p] += K[p] * T(A31);
      P4[p] += K[p] * T(A41);
      P5[p] += K[p] * T(A51);
    }
    if (!eval(false, 2)) break;  // K2
#pragma unroll
    for (int p = 0; p < NQ; p++) {
      P3[p] += K[p] * T(A32);
      P4[p] += K[p] * T(A42);
      P5[p] += K[p] * T(A52);
      YB[p] += K[p] * T(B2);
      ER(p) += K[p] * T(E2);
      ys[p] = Y(p) + P3[p] * ht;
    }
    if (!eval(false, 3)) break;  // K3
#pragma unroll
    for (int p = 0; p < NQ; p++) {
      P4[p] += K[p] * T(A43);
      P5[p] += K[p] * T(A53);
      YB[p] += K[p] * T(B3);
      ER(p) += K[p] * T(E3);
      ys[p] = Y(p) + P4[p] * ht;
    }
    if (!eval(false, 4)) break;  // K4
#pragma unroll
    for (int p = 0; p < NQ; p++) {
      P5[p] += K[p] * T(A54);
      YB[p] += K[p] * T(B4);
      ER(p) += K[p] * T(E4);
      ys[p] = Y(p) + P5[p] * ht;
    }
    if (!eval(false, 5)) break;  // K5; ys <- y_new
#pragma unroll
    for (int p = 0; p < NQ; p++) {
      YB[p] += K[p] * T(B5);
      ER(p) += K[p] * T(E5);
      ys[p] = Y(p) + ht * YB[p];
    }
    if (!eval(false, 6)) break;  // K = f(t_new, y_new): error norm + step control (rk.py:138-173)
    if (active) nfev += 6;
    T es = T(0);
#pragma unroll
    for (int p = 0; p < NQ; p++) {
      const RR e = (ER(p) + K[p] * T(E6)) * ht;
      const RR y0 = Y(p), y1 = ys[p];
      RR sc;
      sc.x = frcp(atol + fmax_abs(y0.x, y1.x) * rtol);
      sc.y = frcp(atol + fmax_abs(y0.y, y1.y) * rtol);
      es += sq2(e * sc);
    }
    const T en = fsqrt(es + swp(es)) * inv_sqrt_n;
    begin_step = false;
    if (active) {
      if (en < T(1)) {
        double factor = (en == T(0)) ? 10.0 : fmin(10.0, 0.9 * (double)fpow(en, T(-0.2)));
        if (rejected) factor = fmin(1.0, factor);
        h_abs *= factor;
        t = t_new;
#pragma unroll
        for (int p = 0; p < NQ; p++) {
          Y(p) = ys[p];
          F(p) = K[p];
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
  Rn.nfev = nfev;
  Rn.nacc = nacc;
#undef Y
#undef F
#undef ER
  return result;
}

// a fresh integration of y_io (the full 19-element state on both lanes of the pair, in and out); h = lane & 1
// sl: this lane's first LDS slot (18 pairs, stride apart: Y, F, ER)
template <typename T, typename C, typename A>
__device__ __forceinline__ int rk45_pair(const C& c, const A& a, const StepCtx<T>& X, T* y_io, int& nfev, int& nacc,
                                         int h, R<T>* sl, int stride) {
  const PCtx<T> Q = pctx<T>(c, a, X, h);
  // kind k, row r: y[1 + 3 k + r] (r < 3); row 3: e0 in kind 0, zeros otherwise
#pragma unroll
  for (int k = 0; k < 6; k++) {
    R<T> v;
    v.x = h == 0 ? y_io[1 + 3 * k] : y_io[3 + 3 * k];
    v.y = h == 0 ? y_io[2 + 3 * k] : (k == 0 ? y_io[0] : T(0));
    sl[k * stride] = v;
  }
  qd::QRun Rn;
  const int result = rk45_pair_core(c, a, Q, sl, stride, Rn);
  nfev = Rn.nfev;
  nacc = Rn.nacc;
#pragma unroll
  for (int k = 0; k < 6; k++) {  // the accepted state back on both lanes
    const R<T> v = sl[k * stride];
    y_io[1 + 3 * k] = bl<0>(v.x);
    y_io[2 + 3 * k] = bl<0>(v.y);
    y_io[3 + 3 * k] = bl<1>(v.x);
    if (k == 0) y_io[0] = bl<1>(v.y);
  }
  return result;
}

// LDS pairs per lane of the pair integrator (Y, F, ER)
constexpr int LDS_PAIRS = 18;

}  // namespace pr
