/*
 * fw_oracle.c -- CPU ORACLE (test infrastructure only; never shipped, never
 * measured as the product).  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.
 *
 * Plain-C, fp64, one aircraft at a time restatement of the reference hot path:
 *   PyFly.step            magpie/libs/pyfly/pyfly/pyfly.py:1358-1420
 *   scipy solve_ivp RK45  scipy 1.15.3 integrate/_ivp/{rk.py:14-186, common.py:68-134}
 *                         (third-party, not vendored; reference pins scipy==1.6.0 in
 *                          magpie-env.yml:91 -- the container's 1.15.3 is what the
 *                          golden fixtures were generated with)
 *   FixedWingAircraft.step magpie/libs/fixed-wing-gym/gym_fixed_wing/fixed_wing.py:483-628
 *
 * Parity is pinned by the .npz fixtures in tests/golden/, produced by running the reference
 * itself (tests/golden/gen_golden.py).  Reference file:line citations are on
 * every function below (pyfly.py = magpie/libs/pyfly/pyfly/pyfly.py,
 * fixed_wing.py = magpie/libs/fixed-wing-gym/gym_fixed_wing/fixed_wing.py).
 *
 * Build: see oracle/Makefile  ->  oracle/_build/libfworacle.so
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "../include/fwsim.h"

#define NY FW_NY
#define PI_ 3.141592653589793

/* ------------------------------------------------------------------------- */
/* Variable.apply_conditions  pyfly.py:114-133                               */
/* returns 0 ok, else FW_TERM_VAR(v)                                         */
/* ------------------------------------------------------------------------- */
static int cond(const fw_sim_config* c, int v, double* x) {
  const fw_limits* L = &c->lim[v];
  if (*x < L->constraint_min) return FW_TERM_VAR(v);
  if (*x > L->constraint_max) return FW_TERM_VAR(v);
  /* np.clip(value, min, max) (NaN propagates) */
  double val = *x;
  if (val < L->value_min) val = L->value_min;
  if (val > L->value_max) val = L->value_max;
  if (L->wrap && fabs(val) > PI_) {
    double s = (val > 0) - (val < 0);
    val = s * (fmod(fabs(val), PI_) - PI_);
  }
  *x = val;
  return 0;
}

/* clip only (numpy clip semantics) */
static double clipd(double x, double lo, double hi) {
  if (x < lo) x = lo;
  if (x > hi) x = hi;
  return x;
}

static double sgn(double x) { return (double)((x > 0) - (x < 0)); }

/* gammas  pyfly.py:1086-1116 */
static void gammas(const double* P0, double G[9]) {
  double Jx = P0[FW_P_JX], Jy = P0[FW_P_JY], Jz = P0[FW_P_JZ];
  double I02 = -P0[FW_P_JXZ];
  G[0] = Jx * Jz - I02 * I02;
  G[1] = (fabs(I02) * (Jx - Jy + Jz)) / G[0];
  G[2] = (Jz * (Jz - Jy) + I02 * I02) / G[0];
  G[3] = Jz / G[0];
  G[4] = fabs(I02) / G[0];
  G[5] = (Jz - Jx) / Jy;
  G[6] = fabs(I02) / Jy;
  G[7] = ((Jx - Jy) * Jx + I02 * I02) / G[0];
  G[8] = Jx / G[0];
}

/* Actuation._map_elevon_to_elevail  pyfly.py:651-655 */
static void elevon_to_elevail(double er, double el, double* elev, double* ail) {
  *ail = (-er + el) / 2;
  *elev = (er + el) / 2;
}

/* _rot_b_v, quaternion branch  pyfly.py:1780-1800 ; Euler branch :1757-1777 */
static void rot_quat(const double* e, double R[3][3]) {
  double e0 = e[0], e1 = e[1], e2 = e[2], e3 = e[3];
  R[0][0] = -1 + 2 * (e0 * e0 + e1 * e1);
  R[0][1] = 2 * (e1 * e2 + e3 * e0);
  R[0][2] = 2 * (e1 * e3 - e2 * e0);
  R[1][0] = 2 * (e1 * e2 - e3 * e0);
  R[1][1] = -1 + 2 * (e0 * e0 + e2 * e2);
  R[1][2] = 2 * (e2 * e3 + e1 * e0);
  R[2][0] = 2 * (e1 * e3 + e2 * e0);
  R[2][1] = 2 * (e2 * e3 - e1 * e0);
  R[2][2] = -1 + 2 * (e0 * e0 + e3 * e3);
}

static void rot_euler(double phi, double th, double psi, double R[3][3]) {
  R[0][0] = cos(th) * cos(psi);
  R[0][1] = cos(th) * sin(psi);
  R[0][2] = -sin(th);
  R[1][0] = sin(phi) * sin(th) * cos(psi) - cos(phi) * sin(psi);
  R[1][1] = sin(phi) * sin(th) * sin(psi) + cos(phi) * cos(psi);
  R[1][2] = sin(phi) * cos(th);
  R[2][0] = cos(phi) * sin(th) * cos(psi) + sin(phi) * sin(psi);
  R[2][1] = cos(phi) * sin(th) * sin(psi) - sin(phi) * cos(psi);
  R[2][2] = cos(phi) * cos(th);
}

/* _calculate_airspeed_factors  pyfly.py:1830-1850 */
static void airspeed(const double R[3][3], const double* wind, const double* turb_lin, const double* vel,
                     double* Va, double* alpha, double* beta) {
  double va[3];
  for (int i = 0; i < 3; i++) {
    double w = R[i][0] * wind[0] + R[i][1] * wind[1] + R[i][2] * wind[2] + turb_lin[i];
    va[i] = vel[i] - w;
  }
  *Va = sqrt(va[0] * va[0] + va[1] * va[1] + va[2] * va[2]);
  *alpha = atan2(va[2], va[0]);
  *beta = asin(va[1] / *Va);
}

typedef struct ctx {
  const fw_sim_config* c;
  double G[9];
  double sp[3];      /* constrained commands of the dynamics actuators */
  double wind[3];
  double turb[6];    /* vel_lin (3), vel_ang (3) at cur_sim_step (held over the step) */
  double act_elev0, act_ail0; /* stored elevator/aileron values (t == 0 evaluation) */
  int nfev;
  /* parameters PyFly.__init__ froze (inertia I / gammas pyfly.py:1086-1116, aspect ratio ar :1119):
   * with simulator parameter randomisation (fixed_wing.py:748-813) c->param holds the aircraft's
   * sampled values, which _forces reads at every call, while these stay the initial ones */
  const double* P0;
} ctx;

/* PyFly._dynamics  pyfly.py:1450-1482 (with _set_states_from_ode_solution(save=False)
 * :1852-1881, _forces :1484-1643, _f_* :1645-1747, Actuation.rhs :519-543).
 * first != 0 <=> t == 0: the stored (already conditioned) state is used as-is.  */
static int rhs(ctx* X, int first, const double* y, double* dy) {
  const fw_sim_config* c = X->c;
  const double* P = c->param;
  X->nfev++;
  double om[3] = {y[4], y[5], y[6]};
  double vel[3] = {y[10], y[11], y[12]};
  double av[3] = {y[13], y[14], y[15]};
  double ad[3] = {y[16], y[17], y[18]};
  double elev, ail, thr;
  int t;
  if (!first) {
    for (int i = 0; i < 3; i++)
      if ((t = cond(c, FW_V_OMEGA_P + i, &om[i]))) return t;
    double pos[3] = {y[7], y[8], y[9]};
    for (int i = 0; i < 3; i++)
      if ((t = cond(c, FW_V_POS_N + i, &pos[i]))) return t;
    for (int i = 0; i < 3; i++)
      if ((t = cond(c, FW_V_VEL_U + i, &vel[i]))) return t;
    for (int j = 0; j < 3; j++) { /* Actuation.set_states pyfly.py:479-492 */
      if ((t = cond(c, FW_V_ACT0 + j, &av[j]))) return t;
      ad[j] = clipd(ad[j], -c->act[j].dot_max, c->act[j].dot_max);
    }
    if (c->elevon) {
      elevon_to_elevail(av[0], av[1], &elev, &ail);
      if ((t = cond(c, FW_V_AILERON, &ail))) return t;
      if ((t = cond(c, FW_V_ELEVATOR, &elev))) return t;
    } else {
      elev = av[0];
      ail = av[1];
    }
  } else {
    elev = X->act_elev0;
    ail = X->act_ail0;
  }
  thr = av[2];
  const double* q4 = y; /* raw attitude, pyfly.py:1464 */

  /* _forces */
  double p = om[0], q = om[1], r = om[2];
  if (c->turbulence) {
    p -= X->turb[3];
    q -= X->turb[4];
    r -= X->turb[5];
  }
  double R[3][3], Va, alpha, beta;
  rot_quat(q4, R);
  airspeed(R, X->wind, X->turb, vel, &Va, &alpha, &beta);
  if ((t = cond(c, FW_V_VA, &Va))) return t;
  if ((t = cond(c, FW_V_ALPHA, &alpha))) return t;
  if ((t = cond(c, FW_V_BETA, &beta))) return t;

  double rho = c->rho, S = P[FW_P_S_WING], b = P[FW_P_B], cc = P[FW_P_C];
  double pre = 0.5 * rho * Va * Va * S;
  double e0 = q4[0], e1 = q4[1], e2 = q4[2], e3 = q4[3];
  double mg = P[FW_P_MASS] * c->g;
  double fg[3] = {mg * (2 * (e1 * e3 - e2 * e0)), mg * (2 * (e2 * e3 + e1 * e0)),
                  mg * (e3 * e3 + e0 * e0 - e1 * e1 - e2 * e2)};
  double M = P[FW_P_M], a0 = P[FW_P_A0];
  double ar = X->P0[FW_P_B] * X->P0[FW_P_B] / X->P0[FW_P_S_WING]; /* frozen at __init__ (pyfly.py:1119) */
  double ex1 = exp(-M * (alpha - a0)), ex2 = exp(M * (alpha + a0));
  double sigma = (1 + ex1 + ex2) / ((1 + ex1) * (1 + ex2));
  double sa = sin(alpha), ca = cos(alpha);
  double CLlin = P[FW_P_C_L_0] + P[FW_P_C_L_ALPHA] * alpha;
  double CL = (1 - sigma) * CLlin + sigma * (2 * sgn(alpha) * sa * sa * ca);
  double flift = pre * (CL + P[FW_P_C_L_Q] * cc / (2 * Va) * q + P[FW_P_C_L_DELTA_E] * elev);
  double CD = P[FW_P_C_D_P] + (1 - sigma) * (CLlin * CLlin) / (PI_ * P[FW_P_E] * ar) +
              sigma * (2 * sgn(alpha) * pow(sa, 3));
  double CDb = P[FW_P_C_D_BETA1] * beta + P[FW_P_C_D_BETA2] * beta * beta;
  double fdrag = pre * (CD + CDb + P[FW_P_C_D_Q] * cc / (2 * Va) * q + P[FW_P_C_D_DELTA_E] * elev * elev);
  double Cm = (1 - sigma) * (P[FW_P_C_M_0] + P[FW_P_C_M_ALPHA] * alpha) + sigma * (P[FW_P_C_M_FP] * sgn(alpha) * sa * sa);
  double mm = pre * cc * (Cm + P[FW_P_C_M_Q] * b / (2 * Va) * q + P[FW_P_C_M_DELTA_E] * elev);
  double rud = 0.0; /* rudder disabled (pyfly.py:1217-1221) */
  double fy = pre * (P[FW_P_C_Y_0] + P[FW_P_C_Y_BETA] * beta + P[FW_P_C_Y_P] * b / (2 * Va) * p +
                     P[FW_P_C_Y_R] * b / (2 * Va) * r + P[FW_P_C_Y_DELTA_A] * ail + P[FW_P_C_Y_DELTA_R] * rud);
  double ll = pre * b * (P[FW_P_C_L0_ROLL] + P[FW_P_C_L_BETA] * beta + P[FW_P_C_L_P] * b / (2 * Va) * p +
                         P[FW_P_C_L_R] * b / (2 * Va) * r + P[FW_P_C_L_DELTA_A] * ail + P[FW_P_C_L_DELTA_R] * rud);
  double nn = pre * b * (P[FW_P_C_N_0] + P[FW_P_C_N_BETA] * beta + P[FW_P_C_N_P] * b / (2 * Va) * p +
                         P[FW_P_C_N_R] * b / (2 * Va) * r + P[FW_P_C_N_DELTA_A] * ail + P[FW_P_C_N_DELTA_R] * rud);
  double Rw[3][3];
  rot_euler(0.0, alpha, beta, Rw);
  double fa_in[3] = {-fdrag, fy, -flift};
  double fa[3];
  for (int i = 0; i < 3; i++) fa[i] = Rw[i][0] * fa_in[0] + Rw[i][1] * fa_in[1] + Rw[i][2] * fa_in[2];
  double Vd = Va + thr * (P[FW_P_K_MOTOR] - Va);
  double fprop = 0.5 * rho * P[FW_P_S_PROP] * P[FW_P_C_PROP] * Vd * (Vd - Va);
  double kt = P[FW_P_K_OMEGA] * thr;
  double tprop = -P[FW_P_K_T_P] * kt * kt;
  double f[3] = {fprop + fg[0] + fa[0], fg[1] + fa[1], fg[2] + fa[2]};
  double tau[3] = {ll + tprop, mm, nn};

  /* _f_attitude_dot pyfly.py:1645-1657 (omega here is NOT turbulence-corrected) */
  double P0 = om[0], Q0 = om[1], R0 = om[2];
  dy[0] = 0.5 * (-P0 * e1 - Q0 * e2 - R0 * e3);
  dy[1] = 0.5 * (P0 * e0 + R0 * e2 - Q0 * e3);
  dy[2] = 0.5 * (Q0 * e0 - R0 * e1 + P0 * e3);
  dy[3] = 0.5 * (R0 * e0 + Q0 * e1 - P0 * e2);
  /* _f_omega_dot pyfly.py:1659-1683 */
  const double* G = X->G;
  dy[4] = G[1] * P0 * Q0 - G[2] * Q0 * R0 + G[3] * tau[0] + G[4] * tau[2];
  dy[5] = G[5] * P0 * R0 - G[6] * (P0 * P0 - R0 * R0) + tau[1] / X->P0[FW_P_JY]; /* I[1, 1] */
  dy[6] = G[7] * P0 * Q0 - G[1] * Q0 * R0 + G[4] * tau[0] + G[8] * tau[2];
  /* _f_p_dot pyfly.py:1706-1737 */
  double T00 = e1 * e1 + e0 * e0 - e2 * e2 - e3 * e3, T01 = 2 * (e1 * e2 - e3 * e0), T02 = 2 * (e1 * e3 + e2 * e0);
  double T10 = 2 * (e1 * e2 + e3 * e0), T11 = e2 * e2 + e0 * e0 - e1 * e1 - e3 * e3, T12 = 2 * (e2 * e3 - e1 * e0);
  double T20 = 2 * (e1 * e3 - e2 * e0), T21 = 2 * (e2 * e3 + e1 * e0), T22 = e3 * e3 + e0 * e0 - e1 * e1 - e2 * e2;
  dy[7] = T00 * vel[0] + T01 * vel[1] + T02 * vel[2];
  dy[8] = T10 * vel[0] + T11 * vel[1] + T12 * vel[2];
  dy[9] = T20 * vel[0] + T21 * vel[1] + T22 * vel[2];
  /* _f_v_dot pyfly.py:1685-1704 */
  double m = P[FW_P_MASS];
  dy[10] = R0 * vel[1] - Q0 * vel[2] + f[0] / m;
  dy[11] = P0 * vel[2] - R0 * vel[0] + f[1] / m;
  dy[12] = Q0 * vel[0] - P0 * vel[1] + f[2] / m;
  /* Actuation.rhs pyfly.py:519-543 with ControlVariable.coefs :296-304 */
  for (int j = 0; j < 3; j++) {
    const fw_actuator* A = &c->act[j];
    double c00, c01, c02, c10, c11, c12;
    if (A->order == 1) {
      c00 = -1 / A->tau; c01 = 0; c02 = 1 / A->tau; c10 = 0; c11 = 0; c12 = 0;
    } else {
      c00 = 0; c01 = 1; c02 = 0;
      c10 = -(A->omega_0 * A->omega_0); c11 = -2 * A->zeta * A->omega_0; c12 = A->omega_0 * A->omega_0;
    }
    dy[13 + j] = av[j] * c00 + X->sp[j] * c02 + ad[j] * c01;
    dy[16 + j] = av[j] * c10 + X->sp[j] * c12 + ad[j] * c11;
  }
  return 0;
}

/* ------------------------------------------------------------------------- */
/* scipy RK45 (Dormand-Prince 5(4)) with scipy 1.15.3 step control            */
/* ------------------------------------------------------------------------- */
/* stage times C = (0, 1/5, 3/10, 4/5, 8/9, 1): unused, the RHS is autonomous in t except for the t > 0 test */
static const double RK_A[6][5] = {
    {0, 0, 0, 0, 0},
    {1.0 / 5, 0, 0, 0, 0},
    {3.0 / 40, 9.0 / 40, 0, 0, 0},
    {44.0 / 45, -56.0 / 15, 32.0 / 9, 0, 0},
    {19372.0 / 6561, -25360.0 / 2187, 64448.0 / 6561, -212.0 / 729, 0},
    {9017.0 / 3168, -355.0 / 33, 46732.0 / 5247, 49.0 / 176, -5103.0 / 18656}};
static const double RK_B[6] = {35.0 / 384, 0, 500.0 / 1113, 125.0 / 192, -2187.0 / 6784, 11.0 / 84};
static const double RK_E[7] = {-71.0 / 57600, 0, 71.0 / 16695, -71.0 / 1920, 17253.0 / 339200, -22.0 / 525, 1.0 / 40};

/* common.py norm: RMS */
static double rms(const double* x) {
  double s = 0;
  for (int i = 0; i < NY; i++) s += x[i] * x[i];
  return sqrt(s) / sqrt((double)NY);
}

/* Integrate y from 0 to dt (solve_ivp defaults).  Returns termination code
 * (0 = ok, > 0 = constraint, -1 = solver failure).  y_out holds sol.y[:, -1]:
 * the final state, or on a solver failure the last ACCEPTED sub-step (y0 if
 * none) -- solve_ivp appends only accepted steps to sol.y (ivp.py:654-672) and
 * pyfly.py:1393-1396 saves sol.y[:, -1] whatever sol.status is.  Solver
 * failure = TOO_SMALL_STEP (rk.py:128-129; also taken on a NaN step size, where
 * scipy itself would loop for ever) or the max_nfev RHS-evaluation budget
 * (this build's guard; 0 = 6000).  Counts accepted steps.                     */
static int rk45(ctx* X, const double* y0, double* y_out, int* naccept) {
  const fw_sim_config* c = X->c;
  double rtol = c->rtol, atol = c->atol, t_bound = c->dt;
  const int budget = c->max_nfev > 0 ? c->max_nfev : 6000;
  double f[NY], y[NY];
  int t_;
  memcpy(y, y0, sizeof(y));
  *naccept = 0;
#define RHS_(first, yy, ff)                          \
  do {                                               \
    if ((t_ = rhs(X, (first), (yy), (ff)))) return t_; \
    if (X->nfev >= budget) goto solver_failed;       \
  } while (0)
  RHS_(1, y, f); /* RungeKutta.__init__ rk.py:95 */
  /* select_initial_step common.py:68-134 */
  double sc[NY], tmp[NY];
  double interval = fabs(t_bound - 0.0);
  for (int i = 0; i < NY; i++) sc[i] = atol + fabs(y[i]) * rtol;
  for (int i = 0; i < NY; i++) tmp[i] = y[i] / sc[i];
  double d0 = rms(tmp);
  for (int i = 0; i < NY; i++) tmp[i] = f[i] / sc[i];
  double d1 = rms(tmp);
  double h0 = (d0 < 1e-5 || d1 < 1e-5) ? 1e-6 : 0.01 * d0 / d1;
  if (h0 > interval) h0 = interval;
  double y1[NY], f1[NY];
  for (int i = 0; i < NY; i++) y1[i] = y[i] + h0 * f[i];
  RHS_(0, y1, f1);
  for (int i = 0; i < NY; i++) tmp[i] = (f1[i] - f[i]) / sc[i];
  double d2 = rms(tmp) / h0;
  double h1;
  if (d1 <= 1e-15 && d2 <= 1e-15) {
    h1 = 1e-6 > h0 * 1e-3 ? 1e-6 : h0 * 1e-3;
  } else {
    double mx = d1 > d2 ? d1 : d2;
    h1 = pow(0.01 / mx, 1.0 / 5.0);
  }
  double h_abs = 100 * h0;
  if (h1 < h_abs) h_abs = h1;
  if (interval < h_abs) h_abs = interval;

  double t = 0.0;
  double K[7][NY];
  /* solve_ivp loop ivp.py:654-662 + OdeSolver.step base.py:175-206 */
  while (!(t - t_bound >= 0)) {
    /* RungeKutta._step_impl rk.py:111-173 */
    double min_step = 10 * fabs(nextafter(t, INFINITY) - t);
    if (h_abs < min_step) h_abs = min_step;
    int rejected = 0, accepted = 0;
    double t_new = t, ynew[NY];
    while (!accepted) {
      if (!(h_abs >= min_step)) goto solver_failed; /* TOO_SMALL_STEP (rk.py:128-129) */
      double h = h_abs;
      t_new = t + h;
      if (t_new - t_bound > 0) t_new = t_bound;
      h = t_new - t;
      h_abs = fabs(h);
      /* rk_step rk.py:14-64 */
      memcpy(K[0], f, sizeof(f));
      for (int s = 1; s < 6; s++) {
        double ys[NY];
        for (int i = 0; i < NY; i++) {
          double acc = 0;
          for (int j = 0; j < s; j++) acc += K[j][i] * RK_A[s][j];
          ys[i] = y[i] + acc * h;
        }
        RHS_(0, ys, K[s]);
      }
      for (int i = 0; i < NY; i++) {
        double acc = 0;
        for (int j = 0; j < 6; j++) acc += K[j][i] * RK_B[j];
        ynew[i] = y[i] + h * acc;
      }
      RHS_(0, ynew, K[6]);
      double err[NY];
      for (int i = 0; i < NY; i++) {
        double acc = 0;
        for (int j = 0; j < 7; j++) acc += K[j][i] * RK_E[j];
        double s_ = atol + fmax(fabs(y[i]), fabs(ynew[i])) * rtol;
        err[i] = acc * h / s_;
      }
      double en = rms(err);
      if (en < 1) {
        double factor = (en == 0) ? 10.0 : fmin(10.0, 0.9 * pow(en, -1.0 / 5.0));
        if (rejected && factor > 1) factor = 1;
        h_abs *= factor;
        accepted = 1;
      } else {
        h_abs *= fmax(0.2, 0.9 * pow(en, -1.0 / 5.0));
        rejected = 1;
      }
    }
    t = t_new;
    memcpy(y, ynew, sizeof(y));
    memcpy(f, K[6], sizeof(f));
    (*naccept)++;
  }
  memcpy(y_out, y, sizeof(y));
  return 0;
solver_failed:
  memcpy(y_out, y, sizeof(y));
  return -1;
#undef RHS_
}

/* ------------------------------------------------------------------------- */
/* Actuation.set_and_constrain_commands  pyfly.py:545-582                     */
/* cmd (in/out) in input order (elevator, aileron, throttle); sp = dynamics   */
/* setpoints.  Returns a termination code if a command violates a constraint  */
/* (the reference raises outside the try block; we report it).                */
/* ------------------------------------------------------------------------- */
static int constrain_commands(const fw_sim_config* c, double* cmd, double* sp) {
  int t;
  if (c->elevon) {
    double er = -1 * cmd[1] + cmd[0], el = cmd[1] + cmd[0];
    if ((t = cond(c, FW_V_ACT0, &er))) return t;
    if ((t = cond(c, FW_V_ACT1, &el))) return t;
    double thr = cmd[2];
    if ((t = cond(c, FW_V_ACT2, &thr))) return t;
    sp[0] = er; sp[1] = el; sp[2] = thr;
    double elev, ail;
    elevon_to_elevail(er, el, &elev, &ail);
    if ((t = cond(c, FW_V_ELEVATOR, &elev))) return t;
    if ((t = cond(c, FW_V_AILERON, &ail))) return t;
    cmd[0] = elev; cmd[1] = ail; cmd[2] = thr;
  } else {
    for (int j = 0; j < 3; j++) {
      if ((t = cond(c, FW_V_ACT0 + j, &cmd[j]))) return t;
      sp[j] = cmd[j];
    }
  }
  return 0;
}

/* Dryden FIR turbulence at step k (dryden.py:193-261 as wired by pyfly.py:781-783;
 * lsim FOH with vanishing Ad): chunk-local index j = k % L; j == 0 -> 0.
 * noise: [4][len] N(0,1) samples (already NOT scaled; scale sqrt(pi/L) applied). */
/* Chunks too short for the FIR (fw_sim_config.dryden_state): the shaping filters' state-space recurrence
 * (scipy 1.15.3 lsim, first-order hold: x[j] = Ad x[j-1] + Bd0 u[j-1] + Bd1 u[j], y = C x; each chunk c >= 1
 * starts from expm(A c L^2) x_last, _ltisys.py lsim's zero-input step to t[0]), as wired by
 * pyfly.py:781-783 / dryden.py:193-261.  Restated from scratch up to step k (a pure function of k, like
 * the FIR; O(k) per call -- test sizes only). */
static void orc_turbulence_bank(const fw_sim_config* c, const double* noise, int64_t len, int64_t k, double* turb) {
  static const int ord[6] = {1, 2, 2, 1, 3, 3}, chan[6] = {0, 1, 2, 3, 1, 2};
  const int64_t L = c->turb_len;
  const double s = sqrt(PI_ / (double)L);
  int oa = 0, ox = 0;
  for (int f = 0; f < 6; f++) {
    const int n = ord[f];
    const double *Ad = c->dryden_ad + oa, *E1 = c->dryden_e1 + oa;
    double x[3] = {0, 0, 0}, t[3];
    for (int64_t i = 0; i <= k; i++) {
      const int64_t ch = i / L, j = i % L;
      if (j == 0) {
        if (ch > 0) {
          if (ch >= c->dryden_ncut) {
            x[0] = x[1] = x[2] = 0;
          } else {
            for (int64_t p = 0; p < ch; p++) {
              for (int r = 0; r < n; r++) {
                t[r] = 0;
                for (int q = 0; q < n; q++) t[r] += E1[r * n + q] * x[q];
              }
              for (int r = 0; r < n; r++) x[r] = t[r];
            }
          }
        }
      } else {
        const double um1 = len > 0 ? s * noise[chan[f] * len + (i - 1) % len] : 0.0;
        const double u0 = len > 0 ? s * noise[chan[f] * len + i % len] : 0.0;
        for (int r = 0; r < n; r++) {
          t[r] = c->dryden_b0[ox + r] * um1 + c->dryden_b1[ox + r] * u0;
          for (int q = 0; q < n; q++) t[r] += Ad[r * n + q] * x[q];
        }
        for (int r = 0; r < n; r++) x[r] = t[r];
      }
    }
    double y = 0;
    for (int r = 0; r < n; r++) y += c->dryden_c[ox + r] * x[r];
    turb[f] = y;
    oa += n * n;
    ox += n;
  }
}

void orc_turbulence(const fw_sim_config* c, const double* noise, int64_t len, int64_t k, double* turb) {
  for (int i = 0; i < 6; i++) turb[i] = 0;
  if (!c->turbulence) return;
  if (c->dryden_state) {
    orc_turbulence_bank(c, noise, len, k, turb);
    return;
  }
  int64_t L = c->turb_len;
  if (k % L == 0) return;
  if (len < 1) return;
  /* a sequence shorter than the episode wraps: simulate() reads noise[:, (t_span[0] + j) % len] in every
   * branch of dryden.py:209-236 (slice, modulo start, concatenation, np.pad(mode="wrap")) */
  const int64_t km1 = (k - 1) % len, k0 = k % len;
  double s = sqrt(PI_ / (double)L);
  static const int chan[6] = {0, 1, 2, 3, 1, 2}; /* dryden.py:238-252 */
  for (int f = 0; f < 6; f++) {
    double um1 = s * noise[chan[f] * len + km1], u0 = s * noise[chan[f] * len + k0];
    turb[f] = c->dryden_g0[f] * um1 + c->dryden_g1[f] * u0;
  }
}

/* ------------------------------------------------------------------------- */
/* PyFly.step pyfly.py:1358-1420 for one aircraft.                            */
/*   y[19], der[8] (roll pitch yaw Va alpha beta elevator aileron) in/out     */
/*   hist[9]: history[-1] of (roll pitch yaw Va alpha beta p q r) out         */
/* Returns termination code (0 success).                                     */
/* ------------------------------------------------------------------------- */
int orc_sim_step_p(const fw_sim_config* c, const double* P0, double* y, double* der, double* hist,
                   const double* wind, const double* turb, double* cmd, int* nfev, int* naccept) {
  ctx X;
  memset(&X, 0, sizeof(X));
  X.c = c;
  X.P0 = P0 ? P0 : c->param;
  gammas(X.P0, X.G);
  for (int i = 0; i < 3; i++) X.wind[i] = wind[i];
  for (int i = 0; i < 6; i++) X.turb[i] = turb[i];
  X.act_elev0 = der[6];
  X.act_ail0 = der[7];
  double h_prev[9] = {der[0], der[1], der[2], der[3], der[4], der[5], y[4], y[5], y[6]};
  if (hist) memcpy(hist, h_prev, sizeof(h_prev));
  int t = constrain_commands(c, cmd, X.sp);
  *naccept = 0;
  if (t) { *nfev = 0; return t; }
  double y1[NY];
  memcpy(y1, y, sizeof(y1));
  t = rk45(&X, y, y1, naccept);
  *nfev = X.nfev;
  if (t < 0) t = 0; /* solver failure: sol.y[:, -1] (last accepted) is saved as usual (pyfly.py:1393-1396) */
  if (t) return t;

  /* _set_states_from_ode_solution(save=True) pyfly.py:1852-1881 -- commits in
   * order; a constraint raise leaves later variables at their previous value */
  double n = sqrt(y1[0] * y1[0] + y1[1] * y1[1] + y1[2] * y1[2] + y1[3] * y1[3]);
  double e0 = y1[0] / n, e1 = y1[1] / n, e2 = y1[2] / n, e3 = y1[3] / n;
  double ynew[NY];
  memcpy(ynew, y, sizeof(ynew));
  ynew[0] = e0; ynew[1] = e1; ynew[2] = e2; ynew[3] = e3;
  /* AttitudeQuaternion.as_euler_angle pyfly.py:684-708 */
  double eul[3];
  eul[0] = atan2(2 * (e0 * e1 + e2 * e3), e0 * e0 + e3 * e3 - e1 * e1 - e2 * e2);
  eul[1] = asin(2 * (e0 * e2 - e1 * e3));
  eul[2] = atan2(2 * (e0 * e3 + e1 * e2), e0 * e0 + e1 * e1 - e2 * e2 - e3 * e3);
  double nder[8];
  memcpy(nder, der, sizeof(nder));
  double nh[9];
  memcpy(nh, h_prev, sizeof(nh));
#define COMMIT_FAIL(code)                       \
  do {                                          \
    memcpy(y, ynew, sizeof(ynew));              \
    memcpy(der, nder, sizeof(nder));            \
    if (hist) memcpy(hist, nh, sizeof(nh));     \
    return (code);                              \
  } while (0)
  for (int i = 0; i < 3; i++) {
    if ((t = cond(c, FW_V_ROLL + i, &eul[i]))) COMMIT_FAIL(t);
    nder[i] = eul[i];
    nh[i] = eul[i];
  }
  for (int i = 0; i < 9; i++) {
    double v = y1[4 + i];
    if ((t = cond(c, FW_V_OMEGA_P + i, &v))) COMMIT_FAIL(t);
    ynew[4 + i] = v;
    if (i < 3) nh[6 + i] = v;
  }
  for (int j = 0; j < 3; j++) {
    double v = y1[13 + j];
    if ((t = cond(c, FW_V_ACT0 + j, &v))) COMMIT_FAIL(t);
    ynew[13 + j] = v;
    ynew[16 + j] = clipd(y1[16 + j], -c->act[j].dot_max, c->act[j].dot_max);
  }
  if (c->elevon) {
    double elev, ail;
    elevon_to_elevail(ynew[13], ynew[14], &elev, &ail);
    if ((t = cond(c, FW_V_AILERON, &ail))) COMMIT_FAIL(t);
    nder[7] = ail;
    if ((t = cond(c, FW_V_ELEVATOR, &elev))) COMMIT_FAIL(t);
    nder[6] = elev;
  } else {
    nder[6] = ynew[13];
    nder[7] = ynew[14];
  }
  /* post-step airspeed factors, Euler branch pyfly.py:1398-1406 */
  double R[3][3], Va, al, be;
  rot_euler(nder[0], nder[1], nder[2], R);
  airspeed(R, wind, turb, &ynew[10], &Va, &al, &be);
  if ((t = cond(c, FW_V_VA, &Va))) COMMIT_FAIL(t);
  nder[3] = Va; nh[3] = Va;
  if ((t = cond(c, FW_V_ALPHA, &al))) COMMIT_FAIL(t);
  nder[4] = al; nh[4] = al;
  if ((t = cond(c, FW_V_BETA, &be))) COMMIT_FAIL(t);
  nder[5] = be; nh[5] = be;
  memcpy(y, ynew, sizeof(ynew));
  memcpy(der, nder, sizeof(nder));
  if (hist) memcpy(hist, nh, sizeof(nh));
  return 0;
#undef COMMIT_FAIL
}

int orc_sim_step(const fw_sim_config* c, double* y, double* der, double* hist, const double* wind,
                 const double* turb, double* cmd, int* nfev, int* naccept) {
  return orc_sim_step_p(c, NULL, y, der, hist, wind, turb, cmd, nfev, naccept);
}

/* Batched convenience wrapper: arrays are [n][19], [n][8], [n][9], [n][3], [n][6], [n][3]. */
void orc_sim_step_batch(const fw_sim_config* c, int64_t n, double* y, double* der, double* hist,
                        const double* wind, const double* turb, double* cmd, int32_t* term, int32_t* nfev,
                        int32_t* nacc) {
  for (int64_t i = 0; i < n; i++) {
    int nf = 0, na = 0;
    term[i] = orc_sim_step(c, y + i * NY, der + i * 8, hist ? hist + i * 9 : 0, wind + i * 3, turb + i * 6,
                           cmd + i * 3, &nf, &na);
    nfev[i] = nf;
    nacc[i] = na;
  }
}

/* Post-reset airspeed factors / elevator-aileron mapping (pyfly.py:1284-1311). */
void orc_reset_derived(const fw_sim_config* c, const double* y, const double* euler, const double* wind,
                       double* der) {
  double zero[6] = {0, 0, 0, 0, 0, 0};
  double R[3][3];
  rot_euler(euler[0], euler[1], euler[2], R);
  double Va, al, be;
  airspeed(R, wind, zero, &y[10], &Va, &al, &be);
  der[0] = euler[0]; der[1] = euler[1]; der[2] = euler[2];
  cond(c, FW_V_VA, &Va);
  cond(c, FW_V_ALPHA, &al);
  cond(c, FW_V_BETA, &be);
  der[3] = Va; der[4] = al; der[5] = be;
  if (c->elevon) {
    double elev, ail;
    elevon_to_elevail(y[13], y[14], &elev, &ail);
    cond(c, FW_V_ELEVATOR, &elev);
    cond(c, FW_V_AILERON, &ail);
    der[6] = elev; der[7] = ail;
  } else {
    der[6] = y[13]; der[7] = y[14];
  }
  /* ControlVariable.reset of a disabled state ignores the value (pyfly.py:359-363) */
  if (c->disabled_inputs & 1) der[6] = 0.0;
  if (c->disabled_inputs & 2) der[7] = 0.0;
}

/* AttitudeQuaternion._from_euler_angles pyfly.py:714-737 */
void orc_euler_to_quat(const double* eul, double* q) {
  double phi = eul[0], th = eul[1], psi = eul[2];
  q[0] = cos(psi / 2) * cos(th / 2) * cos(phi / 2) + sin(psi / 2) * sin(th / 2) * sin(phi / 2);
  q[1] = cos(psi / 2) * cos(th / 2) * sin(phi / 2) - sin(psi / 2) * sin(th / 2) * cos(phi / 2);
  q[2] = cos(psi / 2) * sin(th / 2) * cos(phi / 2) + sin(psi / 2) * cos(th / 2) * sin(phi / 2);
  q[3] = sin(psi / 2) * cos(th / 2) * cos(phi / 2) - cos(psi / 2) * sin(th / 2) * sin(phi / 2);
}

/* ========================================================================= */
/* Gym env layer: FixedWingAircraft (fixed_wing.py)                           */
/* ========================================================================= */
typedef struct orc_env {
  double y[NY];
  double der[8];        /* .value of roll pitch yaw Va alpha beta elevator aileron */
  double hist[9];       /* history[-1] of roll pitch yaw Va alpha beta p q r */
  double wind[3];
  int32_t steps;        /* steps_count == cur_sim_step */
  int32_t steps_tgt;    /* _steps_for_current_target */
  double target[3];
  double act_hist[FW_MAX_WINDOW][3]; /* raw actions, most recent last */
  int32_t n_act;
  double cmd_hist[FW_MAX_WINDOW][3]; /* constrained commands (input order), most recent last */
  int32_t n_cmd;
  uint8_t goal_all[2048];            /* history["goal"]["all"] */
  int32_t n_goal;
  int32_t goal_achieved;
  double ep_ret;
  /* simulator parameter randomisation: the aircraft's sampled parameters (runtime) and the config's
   * (what PyFly.__init__ froze into I / gammas / ar); has_params = 0: the sim config's for both */
  int32_t has_params;
  double params[FW_NPARAM];
  double params0[FW_NPARAM];
  /* reward.form "potential": self.prev_shaping per function class (fixed_wing.py:296, 470, 1108);
   * has_prev = 0 is the reference's None (set by reset) */
  double prev_shaping[3];
  int32_t has_prev[3];
  /* history["error"] (fixed_wing.py:462-466, 575-579): entry 0 at the reset, one per successful step */
  double err_hist[2048][3];
  int32_t n_err;
} orc_env;

static void push_hist(double h[FW_MAX_WINDOW][3], int32_t* n, const double* v) {
  if (*n == FW_MAX_WINDOW) {
    memmove(&h[0][0], &h[1][0], sizeof(double) * 3 * (FW_MAX_WINDOW - 1));
    (*n)--;
  }
  for (int i = 0; i < 3; i++) h[*n][i] = v[i];
  (*n)++;
}

static double state_value(const orc_env* s, int var) {
  switch (var) {
    case FW_V_ROLL: return s->der[0];
    case FW_V_PITCH: return s->der[1];
    case FW_V_YAW: return s->der[2];
    case FW_V_VA: return s->der[3];
    case FW_V_ALPHA: return s->der[4];
    case FW_V_BETA: return s->der[5];
    case FW_V_ELEVATOR: return s->der[6];
    case FW_V_AILERON: return s->der[7];
    case FW_V_THROTTLE: return s->y[15];
    case FW_V_ACT0: case FW_V_ACT1: case FW_V_ACT2: return s->y[13 + var - FW_V_ACT0];
    default: return s->y[4 + var - FW_V_OMEGA_P];
  }
}

static double state_hist_last(const orc_env* s, int var) {
  switch (var) {
    case FW_V_ROLL: return s->hist[0];
    case FW_V_PITCH: return s->hist[1];
    case FW_V_YAW: return s->hist[2];
    case FW_V_VA: return s->hist[3];
    case FW_V_ALPHA: return s->hist[4];
    case FW_V_BETA: return s->hist[5];
    case FW_V_OMEGA_P: return s->hist[6];
    case FW_V_OMEGA_Q: return s->hist[7];
    case FW_V_OMEGA_R: return s->hist[8];
    default: return state_value(s, var);
  }
}

static const int TGT_VAR[3] = {FW_V_ROLL, FW_V_PITCH, FW_V_VA};

/* _get_angle_dist fixed_wing.py:1332-1344 (numpy float % semantics) */
static double pymod(double a, double b) {
  double r = fmod(a, b);
  if (r != 0 && ((r < 0) != (b < 0))) r += b;
  return r;
}

/* _get_error fixed_wing.py:1318-1330 */
static double get_error(const fw_env_config* e, const orc_env* s, int k) {
  double val = state_value(s, TGT_VAR[k]);
  if (e->target_wrap[k]) {
    double dist = pymod(val - s->target[k] + PI_, 2 * PI_) - PI_;
    if (dist < -PI_) dist += 2 * PI_;
    return dist;
  }
  return s->target[k] - val;
}

/* np.sum(history["error"][k][a:b]) with Python slice bounds already resolved to [a, b) */
static double err_sum(const orc_env* s, int k, int a, int b) {
  double v = 0;
  for (int i = a; i < b; i++) v += s->err_hist[i][k];
  return v;
}
/* Python's list[start:stop] bounds for negative indices on a list of n entries */
static int py_idx(int i, int n) {
  if (i < 0) i += n;
  return i < 0 ? 0 : (i > n ? n : i);
}

/* _get_goal_status fixed_wing.py:1346-1361 ("all" entry) */
static int goal_all(const fw_env_config* e, const orc_env* s) {
  int all = 1;
  for (int k = 0; k < 3; k++) {
    if (isnan(e->target_bound[k])) continue;
    double err = get_error(e, s, k);
    if (!(fabs(err) <= e->target_bound[k])) all = 0;
  }
  return all;
}

/* linear_action_scaling fixed_wing.py:630-652 */
static double scale_fwd(const fw_env_config* e, int i, double a) {
  return (e->act_high[i] - e->act_low[i]) * (a - e->scale_low) / (e->scale_high - e->scale_low) + e->act_low[i];
}
static double scale_bwd(const fw_env_config* e, int i, double a) {
  return (e->scale_high - e->scale_low) * (a - e->act_low[i]) / (e->act_high[i] - e->act_low[i]) + e->scale_low;
}

/* get_observation fixed_wing.py:1113-1262 (length 1, vector, no noise).
 * use_hist: state-type entries read history[-1] (always true in the reference). */
void orc_env_observe(const fw_sim_config* c, const fw_env_config* e, const orc_env* s, double* obs) {
  (void)c;
  for (int o = 0; o < e->n_obs; o++) {
    const fw_obs_entry* E = &e->obs[o];
    double val = 0;
    if (E->kind == FW_OBS_STATE) {
      val = state_hist_last(s, E->var);
    } else if (E->kind == FW_OBS_TARGET_ABS) {
      val = s->target[E->var];
    } else if (E->kind == FW_OBS_TARGET_REL) {
      val = get_error(e, s, E->var);
    } else if (E->kind == FW_OBS_TARGET_INT) {  /* fixed_wing.py:1160-1182, i = 1 */
      const int W = e->integration_window, n = s->n_err;
      val = err_sum(s, E->var, py_idx(-W - 1, n), py_idx(-1, n));
      if (s->steps - 1 < W) val += (double)(W - (s->steps - 1)) * s->err_hist[0][E->var];
    } else { /* action window */
      int ai = E->var;
      if (s->steps - 1 < 0) {
        static const int AVAR[3] = {FW_V_ELEVATOR, FW_V_AILERON, FW_V_THROTTLE};
        val = state_value(s, AVAR[ai]);
        if (e->scale_actions) val = scale_bwd(e, ai, val);
      } else {
        int w = E->window;
        const double(*h)[3] = e->scale_actions ? s->act_hist : s->cmd_hist;
        int n = e->scale_actions ? s->n_act : s->n_cmd;
        int start = n - w < 0 ? 0 : n - w;
        float acc = 0.0f; /* np.sum(..., dtype=np.float32) */
        for (int i = start + 1; i < n; i++) acc += (float)fabs(h[i][ai] - h[i - 1][ai]);
        val = acc;
      }
    }
    if (E->norm) {
      val -= E->mean;
      val /= E->var_;
    }
    obs[o] = val;
  }
}

/* get_reward fixed_wing.py:941-1111 (forms "absolute" and "potential") */
static double get_reward(const fw_env_config* e, orc_env* s, const double* action) {
  double term_val[3] = {0, 0, 0}, term_shape[3] = {0, 0, 0};
  for (int f = 0; f < e->n_rew; f++) {
    const fw_rew_factor* F = &e->rew[f];
    double val = 0;
    if (F->kind == FW_REW_ACTION_VALUE) {
      val = fabs(action[0]) + fabs(action[1]) + fabs(action[2]);
    } else if (F->kind == FW_REW_ACTION_DELTA) {
      if (s->steps > 1) {
        int n = s->n_act, w = F->window;
        int start = n - w < 0 ? 0 : n - w;
        for (int i = start + 1; i < n; i++)
          for (int a = 0; a < 3; a++) val += fabs(s->act_hist[i][a] - s->act_hist[i - 1][a]);
      }
    } else if (F->kind == FW_REW_ACTION_BOUND) {
      for (int a = 0; a < 3; a++) {
        double bmax = e->scale_high * e->bounds_multiplier, bmin = e->scale_low * e->bounds_multiplier;
        double hi = action[a] > bmax ? action[a] - bmax : 0;
        double lo = action[a] < bmin ? action[a] - bmin : 0;
        val += fabs(hi) + fabs(lo);
      }
    } else if (F->kind == FW_REW_STATE_VALUE) {
      val = state_value(s, F->var);
    } else if (F->kind == FW_REW_STATE_INT_ERROR) {  /* fixed_wing.py:1001-1012 */
      const int W = e->integration_window, n = s->n_err;
      val = err_sum(s, F->var, W == 0 ? 0 : py_idx(-W, n), n);  /* [-W:] ([-0:] is the whole list) */
      if (s->steps < W) val += (double)(W - s->steps) * s->err_hist[0][F->var];
    } else { /* state error */
      val = get_error(e, s, F->var);
    }
    if (F->fun == FW_FUN_LINEAR) {
      val = fabs(val) / F->scaling;
      if (val < 0) val = 0;
      if (val > F->max) val = F->max;
    } else {
      val = val * val / F->scaling;
    }
    double sg = sgn(F->sign);
    if (F->shaping) term_shape[F->fun] += val * sg;
    else term_val[F->fun] += val * sg;
  }
  double reward = 0;
  for (int k = 0; k < 3; k++) {
    if (!e->term_present[k]) continue;
    double v;
    if (e->reward_potential) {  /* fixed_wing.py:1080-1104 */
      if (k == FW_FUN_EXPONENTIAL)
        v = s->has_prev[k] ? -1 + exp(term_val[k] + (term_shape[k] - s->prev_shaping[k])) : -1 + exp(term_val[k]);
      else
        v = s->has_prev[k] ? term_val[k] + (term_shape[k] - s->prev_shaping[k]) : term_val[k];
    } else if (k == FW_FUN_EXPONENTIAL) {
      v = -1 + exp(term_val[k] + term_shape[k]);
    } else {
      v = term_val[k] + term_shape[k];
    }
    s->prev_shaping[k] = term_shape[k];  /* :1108, every term of every call */
    s->has_prev[k] = 1;
    reward += e->term_weight[k] * v;
  }
  return reward;
}

/* _get_next_target fixed_wing.py:1363-1471 (constant / compensate) */
static void next_target(const fw_sim_config* c, const fw_env_config* e, const orc_env* s, double* res) {
  for (int k = 0; k < 3; k++) {
    double r = s->target[k];
    if (e->target_class[k] == FW_TGT_COMPENSATE) { /* Va only */
      double pitch_tar = s->target[1];
      if (pitch_tar <= -2.5 * PI_ / 180.0) {
        double va_target = s->target[2];
        double va_end = 28.434 - 40.0841 * pitch_tar;
        double slope;
        if (va_target <= va_end) {
          double a = va_target < va_end * 0.95 ? 1.0 : 1 - va_target / (va_end * 1.5);
          slope = 7 * (a > 0 ? a : 0);
        } else {
          slope = 0;
        }
        r = va_target + (slope * (-s->target[1]) - 0.25) * c->dt;
      } else if (pitch_tar >= 5 * PI_ / 180.0) {
        double va_end = 26.27 - 41.2529 * pitch_tar;
        double va_target = s->target[2];
        if (va_target > va_end) {
          if (s->steps_tgt < 750) r = va_target + (va_end - va_target) * 1 / 150;
          else r = va_end;
        } else {
          r = va_target;
        }
      }
    }
    if (e->target_wrap[k] && fabs(r) > PI_) r = sgn(r) * (fmod(fabs(r), PI_) - PI_);
    res[k] = r;
  }
}

/* FixedWingAircraft.reset with explicit state and target (fixed_wing.py:414-481).
 * init: FW_NINIT values (no NaN allowed here), target[3]. */
int orc_env_reset(const fw_sim_config* c, const fw_env_config* e, orc_env* s, const double* init,
                  const double* target, double* obs) {
  /* FixedWingAircraft.reset computes the observation BEFORE it replaces self.history (fixed_wing.py:452-459):
   * an "integrator" entry then reads the previous episode's error history (None at the first reset) */
  double prev_int[3] = {0, 0, 0};
  const int prev_n = s->n_err, W = e->integration_window;
  for (int k = 0; k < 3 && prev_n > 0; k++)
    prev_int[k] = err_sum(s, k, py_idx(-W - 1, prev_n), py_idx(-1, prev_n)) + (double)(W + 1) * s->err_hist[0][k];
  memset(s, 0, sizeof(*s));
  double eul[3] = {init[FW_I_ROLL], init[FW_I_PITCH], init[FW_I_YAW]};
  int t;
  /* Variable.reset(value) applies conditions pyfly.py:83-104 */
  for (int i = 0; i < 3; i++)
    if ((t = cond(c, FW_V_ROLL + i, &eul[i]))) return t;
  orc_euler_to_quat(eul, s->y);
  for (int i = 0; i < 9; i++) {
    double v = init[FW_I_P + i];
    if ((t = cond(c, FW_V_OMEGA_P + i, &v))) return t;
    s->y[4 + i] = v;
  }
  for (int j = 0; j < 3; j++) {
    double v = init[FW_I_ACT0 + 2 * j];
    if ((t = cond(c, FW_V_ACT0 + j, &v))) return t;
    s->y[13 + j] = v;
    s->y[16 + j] = clipd(init[FW_I_ACT0 + 2 * j + 1], -c->act[j].dot_max, c->act[j].dot_max);
  }
  for (int i = 0; i < 3; i++) s->wind[i] = init[FW_I_WIND_N + i];
  orc_reset_derived(c, s->y, eul, s->wind, s->der);
  s->hist[0] = s->der[0]; s->hist[1] = s->der[1]; s->hist[2] = s->der[2];
  s->hist[3] = s->der[3]; s->hist[4] = s->der[4]; s->hist[5] = s->der[5];
  s->hist[6] = s->y[4]; s->hist[7] = s->y[5]; s->hist[8] = s->y[6];
  for (int k = 0; k < 3; k++) s->target[k] = target[k];
  s->steps = 0;
  s->steps_tgt = 0;
  s->goal_all[0] = (uint8_t)goal_all(e, s);
  s->n_goal = 1;
  for (int k = 0; k < 3; k++) s->err_hist[0][k] = get_error(e, s, k);
  s->n_err = 1;
  if (obs) {
    orc_env_observe(c, e, s, obs);
    for (int o = 0; o < e->n_obs; o++) {
      const fw_obs_entry* E = &e->obs[o];
      if (E->kind != FW_OBS_TARGET_INT) continue;
      double v = prev_n > 0 ? prev_int[E->var] : get_error(e, s, E->var) * (double)W;  /* history None (:1163-1167) */
      if (E->norm) v = (v - E->mean) / E->var_;
      obs[o] = v;
    }
  }
  return 0;
}

/* FixedWingAircraft.step fixed_wing.py:483-628 (no metrics).  noise: [4][len]
 * turbulence samples (may be NULL when turbulence is off).  Returns done.   */
int orc_env_step(const fw_sim_config* c, const fw_env_config* e, orc_env* s, const double* action,
                 const double* noise, int64_t noise_len, double* obs, double* reward, int32_t* term,
                 int32_t* nfev_out) {
  push_hist(s->act_hist, &s->n_act, action);
  double cmd[3];
  for (int i = 0; i < 3; i++) {
    double a = action[i];
    if (e->scale_actions) a = scale_fwd(e, i, clipd(a, e->scale_low, e->scale_high));
    cmd[i] = a;
  }
  double turb[6];
  orc_turbulence(c, noise, noise_len, s->steps, turb);
  int nf = 0, na = 0;
  int t;
  if (s->has_params) {
    fw_sim_config cp = *c;
    memcpy(cp.param, s->params, sizeof(cp.param));
    t = orc_sim_step_p(&cp, s->params0, s->y, s->der, s->hist, s->wind, turb, cmd, &nf, &na);
  } else {
    t = orc_sim_step(c, s->y, s->der, s->hist, s->wind, turb, cmd, &nf, &na);
  }
  if (nfev_out) *nfev_out = nf;
  push_hist(s->cmd_hist, &s->n_cmd, cmd);
  s->steps += 1;
  s->steps_tgt += 1;
  int done = 0;
  *term = FW_TERM_NONE;
  if (s->steps >= e->steps_max && e->steps_max > 0) {
    done = 1;
    *term = FW_TERM_STEPS;
  }
  if (t == 0) {
    int on_step = 0;
    (void)on_step;
    if (e->streak_req > 0) {
      s->goal_all[s->n_goal++] = (uint8_t)goal_all(e, s);
      int req = e->streak_req;
      if (s->steps_tgt >= req) {
        int cnt = 0, n0 = s->n_goal - req < 0 ? 0 : s->n_goal - req;
        for (int i = n0; i < s->n_goal; i++) cnt += s->goal_all[i];
        double mean = (double)cnt / (double)(s->n_goal - n0);
        if (mean >= e->streak_frac) {
          s->goal_achieved = 1;
          if (e->on_success == 1) {
            done = 1;
            *term = FW_TERM_SUCCESS;
          }
        }
      }
    }
    *reward = get_reward(e, s, action);
    double nt[3];
    next_target(c, e, s, nt);
    for (int k = 0; k < 3; k++) s->target[k] = nt[k];
    if (s->n_err < 2048) {  /* history["error"][k].append(self._get_error(k)) (:575-579) */
      for (int k = 0; k < 3; k++) s->err_hist[s->n_err][k] = get_error(e, s, k);
      s->n_err++;
    }
  } else {
    done = 1;
    if (e->step_fail_timesteps) *reward = (double)(s->steps - e->steps_max);
    else *reward = e->step_fail_value;
    *term = t;
  }
  orc_env_observe(c, e, s, obs);
  s->ep_ret += *reward;
  return done;
}

int orc_env_state_size(void) { return (int)sizeof(orc_env); }

/* Teacher forcing (tests only): put an env into a mid-episode state given as the device keeps it -- ODE
 * state, derived values (whose successful-step history[-1] equals them), steady wind, targets, step
 * counters, the last n_act raw actions (oldest first) and the last n_goal "all" goal bits (oldest
 * first).  The next orc_env_step is then the reference's step from exactly that state. */
void orc_env_set_state(void* state, const double* y, const double* der, const double* wind, const double* target,
                       int32_t steps, int32_t steps_tgt, const double* act_hist, int32_t n_act, const uint8_t* goals,
                       int32_t n_goal) {
  orc_env* s = (orc_env*)state;
  for (int i = 0; i < NY; i++) s->y[i] = y[i];
  for (int i = 0; i < 8; i++) s->der[i] = der[i];
  for (int i = 0; i < 6; i++) s->hist[i] = der[i];
  for (int i = 0; i < 3; i++) s->hist[6 + i] = y[4 + i];
  for (int i = 0; i < 3; i++) s->wind[i] = wind[i];
  for (int i = 0; i < 3; i++) s->target[i] = target[i];
  s->steps = steps;
  s->steps_tgt = steps_tgt;
  s->n_act = n_act < FW_MAX_WINDOW ? n_act : FW_MAX_WINDOW;
  for (int k = 0; k < s->n_act; k++)
    for (int i = 0; i < 3; i++) s->act_hist[k][i] = act_hist[3 * k + i];
  s->n_cmd = 0;
  s->n_goal = n_goal < 2048 ? n_goal : 2048;
  for (int k = 0; k < s->n_goal; k++) s->goal_all[k] = goals[k];
}

/* Give the env's aircraft its own parameter values (after orc_env_reset, which clears them). */
void orc_env_set_params(void* state, const fw_sim_config* c, const double* params) {
  orc_env* s = (orc_env*)state;
  s->has_params = 1;
  memcpy(s->params, params, sizeof(s->params));
  memcpy(s->params0, c->param, sizeof(s->params0));
}
int orc_sizeof_sim_config(void) { return (int)sizeof(fw_sim_config); }
int orc_sizeof_env_config(void) { return (int)sizeof(fw_env_config); }
