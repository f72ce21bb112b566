/*
 * fwsim.h -- C ABI of libfwsim.so, the MI355X-native batched fixed-wing stepper.
 *
 * One handle = one GPU = N independent aircraft ("envs"), state kept resident
 * in HBM as structure-of-arrays (SoA, one lane per aircraft).  Every call is
 * asynchronous on the given HIP stream (`void* stream` is a hipStream_t; NULL =
 * the null stream).  All functions return 0 on success and a negative FW_E_*
 * code on error; fw_last_error() returns the message of the last error on the
 * calling thread.  No C++ exception crosses this boundary.
 *
 * Device pointers passed in are plain device addresses (e.g. a torch tensor's
 * data_ptr() on the handle's device).  Element type of every floating-point
 * buffer is the handle's precision: float (FW_F32) or double (FW_F64).
 *
 * Reference interfaces replaced (paths relative to the reference checkout):
 *   fw_create       PyFly.__init__            magpie/libs/pyfly/pyfly/pyfly.py:1054-1249
 *                   FixedWingAircraft.__init__ magpie/libs/fixed-wing-gym/gym_fixed_wing/fixed_wing.py:14-306
 *   fw_seed         PyFly.seed / FixedWingAircraft.seed   pyfly.py:1251-1260, fixed_wing.py:324-332
 *   fw_reset        PyFly.reset               pyfly.py:1262-1311
 *                   FixedWingAircraft.reset   fixed_wing.py:414-481
 *   fw_sim_step     PyFly.step                pyfly.py:1358-1420
 *   fw_env_step     FixedWingAircraft.step    fixed_wing.py:483-628, plus the
 *                   SubprocVecEnv worker's auto-reset + terminal_observation
 *                   (stable_baselines3/common/vec_env/subproc_vec_env.py:25-31)
 *                   and Monitor episode statistics (common/monitor.py:88-115)
 *   fw_get_state /  PyFly.state[name].value reads / writes (pyfly.py:1422-1430)
 *   fw_set_state
 */
#ifndef FWSIM_H
#define FWSIM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FWSIM_ABI_VERSION 12

/* ---- error codes ---------------------------------------------------------- */
#define FW_OK 0
#define FW_E_INVALID (-1)   /* bad argument / config */
#define FW_E_HIP (-2)       /* HIP runtime error */
#define FW_E_UNSUPPORTED (-3)
#define FW_E_NOMEM (-4)

/* ---- precision -------------------------------------------------------------- */
#define FW_F32 0
#define FW_F64 1

/* ---- ODE state vector (pyfly.py:1372-1389 ordering) -------------------------
 * [e0 e1 e2 e3 | p q r | n e d | u v w | act0 act1 act2 | act0' act1' act2']
 * act* are the *dynamics* actuators in config order (elevon_right, elevon_left,
 * throttle for the X8).                                                        */
#define FW_NY 19

/* ---- variable slots with limits / constraints (pyfly.py:114-133, 312-328) --- */
enum fw_var {
  FW_V_ROLL = 0, FW_V_PITCH, FW_V_YAW,
  FW_V_OMEGA_P, FW_V_OMEGA_Q, FW_V_OMEGA_R,
  FW_V_POS_N, FW_V_POS_E, FW_V_POS_D,
  FW_V_VEL_U, FW_V_VEL_V, FW_V_VEL_W,
  FW_V_VA, FW_V_ALPHA, FW_V_BETA,
  FW_V_ACT0, FW_V_ACT1, FW_V_ACT2,       /* dynamics actuators (value limits) */
  FW_V_ELEVATOR, FW_V_AILERON, FW_V_THROTTLE, /* model-input actuator states */
  FW_NVAR
};

/* termination codes: 0 = none, 1 + fw_var = ConstraintException on that variable,
 * FW_TERM_STEPS / FW_TERM_SUCCESS = env terminations (fixed_wing.py:519-559)     */
#define FW_TERM_NONE 0
#define FW_TERM_VAR(v) (1 + (v))
#define FW_TERM_STEPS 100
#define FW_TERM_SUCCESS 101

/* ---- aircraft parameters (x8_param.mat keys) ------------------------------ */
enum fw_param {
  FW_P_MASS = 0, FW_P_JX, FW_P_JY, FW_P_JZ, FW_P_JXZ,
  FW_P_S_WING, FW_P_B, FW_P_C, FW_P_S_PROP, FW_P_C_PROP,
  FW_P_K_MOTOR, FW_P_K_T_P, FW_P_K_OMEGA, FW_P_E, FW_P_M, FW_P_A0,
  FW_P_C_L_0, FW_P_C_L_ALPHA, FW_P_C_L_Q, FW_P_C_L_DELTA_E,
  FW_P_C_D_P, FW_P_C_D_Q, FW_P_C_D_BETA1, FW_P_C_D_BETA2, FW_P_C_D_DELTA_E,
  FW_P_C_M_0, FW_P_C_M_ALPHA, FW_P_C_M_Q, FW_P_C_M_DELTA_E, FW_P_C_M_FP,
  FW_P_C_Y_0, FW_P_C_Y_BETA, FW_P_C_Y_P, FW_P_C_Y_R, FW_P_C_Y_DELTA_A, FW_P_C_Y_DELTA_R,
  FW_P_C_L0_ROLL, FW_P_C_L_BETA, FW_P_C_L_P, FW_P_C_L_R, FW_P_C_L_DELTA_A, FW_P_C_L_DELTA_R,
  FW_P_C_N_0, FW_P_C_N_BETA, FW_P_C_N_P, FW_P_C_N_R, FW_P_C_N_DELTA_A, FW_P_C_N_DELTA_R,
  FW_NPARAM
};

/* Variable limits.  "None" in the reference is +-INFINITY here. */
typedef struct fw_limits {
  double value_min, value_max;           /* clip */
  double constraint_min, constraint_max; /* raise -> termination */
  double init_min, init_max;             /* uniform reset sampling */
  int32_t wrap;                          /* +-pi wrap (pyfly.py:130-131) */
  int32_t pad_;
} fw_limits;

/* Actuator dynamics (ControlVariable, pyfly.py:264-310). */
typedef struct fw_actuator {
  int32_t order;    /* 1 or 2 */
  int32_t pad_;
  double tau;       /* order 1 */
  double omega_0;   /* order 2 */
  double zeta;      /* order 2 */
  double dot_max;   /* +inf = None */
} fw_actuator;

/* Simulator configuration (pyfly_config.json + x8_param.mat after config_kw
 * overrides).  Built by the host from the reference-format JSON files.        */
typedef struct fw_sim_config {
  double dt, rho, g;
  double rtol, atol;                 /* solve_ivp defaults 1e-3 / 1e-6 */
  double param[FW_NPARAM];
  fw_limits lim[FW_NVAR];
  fw_actuator act[3];                /* dynamics actuators, dynamics order */
  int32_t elevon;                    /* 1: dynamics = (elevon_right, elevon_left, throttle) */
  int32_t disabled_inputs;           /* bit0 elevator, bit1 aileron: "disabled" ControlVariables,
                                        whose .value is 0 after reset (pyfly.py:359-363) */
  int32_t wind_random;               /* 1: steady wind magnitude sampled in [mag_min, mag_max] */
  int32_t max_nfev;                  /* RHS-evaluation budget of one step (0 = 65535, the largest count the
                                        stats word reports; 8x the census maximum).  scipy has none;
                                        exhausting it ends the step like solve_ivp's TOO_SMALL_STEP
                                        failure: sol.y[:, -1] (the last accepted sub-step) is committed
                                        and the step counts as a success (pyfly.py:1393-1396).       */
  double wind_mag_min, wind_mag_max;
  double wind_init_min[3], wind_init_max[3]; /* per-component sampling when !wind_random */
  int32_t turbulence;              /* Dryden on/off */
  int32_t turb_len;                  /* chunk length L (turbulence_sim_length) */
  double dryden_g0[6], dryden_g1[6]; /* FIR taps, channels (u v w p q r) */
  /* ABI 9: turbulence chunks too short for the FIR (L below ~45): the shaping filters' discretised state-space
   * form, block-diagonal per filter u v w p q r (orders 1 2 2 1 3 3: 12 states; each block's matrix row-major).
   * Within a chunk x[j] = Ad x[j-1] + Bd0 u[j-1] + Bd1 u[j] and the output is C x[j] (scipy lsim, first-order
   * hold, step L^2 / (L - 1)); chunk c >= 1 starts from E1^c x (lsim's zero-input step to t[0] = c L^2, E1 =
   * e^{A L^2}), which is 0 from chunk dryden_ncut on.                                                        */
  int32_t dryden_state;              /* 0: the FIR above; 1: the filter bank below */
  int32_t dryden_ncut;               /* first chunk whose carried-over state is negligible (E1^c < 1e-30) */
  double dryden_ad[28], dryden_e1[28];
  double dryden_b0[12], dryden_b1[12], dryden_c[12];
} fw_sim_config;

/* ---- gym env configuration (fixed_wing_config.json) ------------------------ */
#define FW_MAX_OBS 32
#define FW_MAX_REW 12   /* ABI 11: 8 -> 12 (the default 5 factors + success / step / goal classes) */
#define FW_MAX_IWIN 256
#define FW_MAX_WINDOW 16
#define FW_MAX_OBS_LEN 16     /* observation.length (history rows) */
#define FW_MAX_OBS_HIST 64    /* past observation rows kept per env: (length - 1) * step + 2 */

/* observation entry kinds (fixed_wing.py:1149-1234) */
#define FW_OBS_STATE 0          /* var = fw_var (roll..beta, omega, pos, vel, act states) */
#define FW_OBS_TARGET_ABS 1     /* var = target index 0..2 (roll, pitch, Va) */
#define FW_OBS_TARGET_REL 2
#define FW_OBS_ACTION_WINDOW 3  /* var = action index 0..2 */
#define FW_OBS_TARGET_INT 4     /* var = target index: "integrator" -- the sum of the error history over
                                 * integration_window entries, the newest excluded, padded with the episode's
                                 * first error (fixed_wing.py:1160-1182); observation length 1 only */

typedef struct fw_obs_entry {
  int32_t kind, var, window, norm;
  double mean, var_;
} fw_obs_entry;

/* reward factor kinds (fixed_wing.py:960-1077) */
#define FW_REW_STATE_ERROR 0    /* var = target index */
#define FW_REW_STATE_VALUE 1    /* var = fw_var */
#define FW_REW_ACTION_DELTA 2
#define FW_REW_ACTION_BOUND 3
#define FW_REW_ACTION_VALUE 4
#define FW_REW_STATE_INT_ERROR 5 /* var = target index: the sum of the last integration_window errors, padded
                                  * with the first (fixed_wing.py:1001-1012) */
/* ABI 11 (fixed_wing.py:1020-1048) */
#define FW_REW_SUCCESS 6        /* the step on which the env reaches its goal streak for the FIRST time in its
                                 * lifetime (goal_achieved is never cleared, :81, 546-547): `value`, or with
                                 * var = 1 ("timesteps") steps_max - steps_count; 0 on every other step */
#define FW_REW_STEP 7           /* `value` on every successful step */
#define FW_REW_GOAL 8           /* var = 0 ("per_state"): value / 3 per bounded target within its bound;
                                 * var = 1 ("all"): value when every bounded target is within its bound */

#define FW_FUN_LINEAR 0
#define FW_FUN_QUADRATIC 1
#define FW_FUN_EXPONENTIAL 2

typedef struct fw_rew_factor {
  int32_t kind, var, window, fun;
  int32_t shaping;
  int32_t randomize;                 /* reward.randomize_scaling with "scaling": [low, high] (fixed_wing.py:473-479):
                                      * each reset draws the factor's scaling from U(scaling, scaling_hi) */
  double scaling, max, sign;         /* max = +inf if absent */
  double scaling_hi;
  double value;                      /* ABI 11: "value" of the success / step / goal classes */
} fw_rew_factor;

/* target classes (fixed_wing.py:1363-1471) */
#define FW_TGT_CONSTANT 0
#define FW_TGT_COMPENSATE 1
/* ABI 11: drawn by sample_target (fixed_wing.py:698-722) at every reset and resample, advanced by
 * _get_next_target (:1433-1448); a target given explicitly at reset flies as "constant" for the episode
 * (fixed_wing.py:444-448)                                                                              */
#define FW_TGT_LINEAR 2         /* target += slope * dt; slope = +-U(slope_low, slope_high) */
#define FW_TGT_SINUSOIDAL 3     /* amplitude sin(2 pi / period (steps_count + phase)) + bias */
/* ABI 12: class "attitude_angular" (fixed_wing.py:671-675, 741-746, 1455-1460, 1558-1642): omega_p / q / r become
 * three further targets (fw_env_config.ang_targets), set at every reset from the roll / pitch errors and
 * low-pass filtered at every step; observation entries (FW_OBS_TARGET_ABS / _REL) and reward factors
 * (FW_REW_STATE_ERROR) address them as target FW_TGT_OMEGA_P + 0 / 1 / 2 (omega_p / q / r)                */
#define FW_TGT_OMEGA_P 3

/* simulator parameter randomisation (FixedWingAircraft.sample_simulator_parameters,
 * fixed_wing.py:748-813: the env config's "simulator": {"model": {...}} block), one entry per
 * randomised parameter, redrawn for an aircraft at each of its resets.                        */
#define FW_DIST_GAUSSIAN 0
#define FW_DIST_UNIFORM 1
typedef struct fw_rand_param {
  int32_t param;    /* fw_param index */
  int32_t dist;     /* FW_DIST_GAUSSIAN: N(original, var), then clipped to original -+ clip;
                       FW_DIST_UNIFORM: U(original - var, original + var)                 */
  double original;  /* the parameter's value before sampling ("original", else the config value) */
  double var;       /* absolute (a "relative" var_type is multiplied by |original| by the host) */
  double clip;      /* absolute, may be negative (relative clip * original, as the reference); NaN = none */
} fw_rand_param;

typedef struct fw_env_config {
  int32_t steps_max;
  int32_t n_obs;
  fw_obs_entry obs[FW_MAX_OBS];
  int32_t scale_actions;              /* action.scale_space */
  int32_t has_bounds;                 /* action.bounds_multiplier present */
  double scale_low, scale_high, bounds_multiplier;
  double act_low[3], act_high[3];     /* actuator state limits (action_scale_to_*) */
  int32_t target_class[3];            /* roll, pitch, Va */
  int32_t target_wrap[3];
  double target_low[3], target_high[3];
  double target_delta[3];             /* NaN = none */
  double target_bound[3];             /* NaN = none */
  int32_t streak_req;                 /* <= 4096 (ABI 11; 128 before); 0 disables goal */
  int32_t on_success;                 /* 0 none, 1 done, 2 new (ABI 11: sample_target on success, :551-552) */
  double streak_frac;
  int32_t n_rew;
  int32_t step_fail_timesteps;        /* reward.step_fail == "timesteps" */
  double step_fail_value;
  double term_weight[3];              /* per function class (linear, quadratic, exponential) */
  int32_t term_present[3];
  int32_t reward_potential;           /* reward.form "potential" (fixed_wing.py:1080-1108): each term's shaping
                                       * enters as its change since the env's previous successful step (the
                                       * first step of an episode: the value alone) */
  fw_rew_factor rew[FW_MAX_REW];
  /* streaming episode metrics (fixed_wing.py:1644-1736), reported per done env through
   * fw_set_metrics_output; 0 = not tracked (no extra state traffic) */
  int32_t metrics;
  int32_t resample_every;             /* target.resample_every (fixed_wing.py:570-574): > 0 draws new targets
                                       * (sample_target, :654-746, from the handle's Philox streams) once the
                                       * current ones have been held that many steps; 0 = never */
  double rise_low, rise_high;         /* rise_time metric "low" / "high" (defaults 0.1, 0.9) */
  /* observation.length / step / noise (get_observation, fixed_wing.py:1113-1262).  The
   * observation of one env is obs_length rows of n_obs entries (row r = lag 1 + r * obs_step),
   * i.e. [obs_length * n_obs] values; "vector" and "matrix" shapes share this memory layout.
   * Rows older than the episode repeat its first row plus a per-row U(-1,1)*dt offset (the
   * reference's init_noise).  obs_noise adds N(obs_noise_mean, obs_noise_std) to every value
   * after normalisation.  Both draws come from the handle's Philox streams.                 */
  int32_t obs_length;                 /* >= 1 (0 is read as 1) */
  int32_t obs_step;                   /* >= 1 (0 is read as 1) */
  int32_t obs_noise;                  /* 1: add observation noise */
  int32_t integration_window;         /* cfg "integration_window" (<= FW_MAX_IWIN; 0 = none) */
  double obs_noise_mean, obs_noise_std;
  /* simulator parameter randomisation: n_rand entries of rand[] (0 = every aircraft flies the sim
   * config's parameters).  Only parameters _forces reads at run time change the dynamics; the
   * inertia gammas, I and the aspect ratio stay the sim config's (computed once by the reference). */
  int32_t n_rand;
  int32_t pad4_;
  fw_rand_param rand[FW_NPARAM];
  /* ABI 11: the linear / sinusoidal target classes' draws (sample_target, fixed_wing.py:698-722), per target
   * (roll, pitch, Va); slope and amplitude are drawn in the config's units and converted with np.radians
   * where target_radians is set (convert_to_radians), the period is not converted                       */
  int32_t target_radians[3];
  int32_t pad11_;
  double target_slope_low[3], target_slope_high[3];
  double target_amp_low[3], target_amp_high[3];
  double target_period_low[3], target_period_high[3];
  /* ABI 12: np_random draws sample_simulator_parameters makes at every reset for "simulator" attributes
   * PyFly never reads (fixed_wing.py:802-813; one each: uniform, or choice with probabilities), which the
   * env-draw tape holds before sample_target's: fw_reset / the auto-reset skip that many tape draws.  They
   * leave the episode unchanged, so nothing else reads them.                                         */
  int32_t tape_skip;
  /* ABI 12: 1 = omega_p / q / r targets of class attitude_angular (all three; no bound, so they stay out of
   * the goal status; no metrics, observation history or observation noise with them), each with its max_vel
   * (rad/s, default pi); they live in rows 12..14 of FW_BLK_TARGET_PROPS */
  int32_t ang_targets;
  double ang_max_vel[3];
} fw_env_config;

/* Episode-metric record written for every done env (SoA [FW_NMETRIC][N] so the stores
 * coalesce; handle precision); NaN where the reference yields NaN.  Per-target entries are (roll, pitch, Va),
 * goal entries (roll, pitch, Va, all).                                                      */
#define FW_M_RISE_TIME 0           /* 3 */
#define FW_M_SETTLING_TIME 3       /* 4 */
#define FW_M_OVERSHOOT 7           /* 3 */
#define FW_M_TOTAL_ERROR 10        /* 3 */
#define FW_M_AVG_ERROR 13          /* 3 */
#define FW_M_CONTROL_VARIATION 16  /* 1 ("all") */
#define FW_M_SUCCESS 17            /* 4 (0 / 1) */
#define FW_M_SUCCESS_TIME_FRAC 21  /* 4 */
#define FW_M_END_ERROR 25          /* 3 */
#define FW_NMETRIC 28
#define FW_M_END_WINDOW 50         /* end_error averages the last 50 errors */

/* explicit reset inputs: SoA [FW_NINIT][N]; NaN = sample like an omitted dict key */
enum fw_init_field {
  FW_I_ROLL = 0, FW_I_PITCH, FW_I_YAW, FW_I_P, FW_I_Q, FW_I_R,
  FW_I_PN, FW_I_PE, FW_I_PD, FW_I_U, FW_I_V, FW_I_W,
  FW_I_ACT0, FW_I_ACT0_DOT, FW_I_ACT1, FW_I_ACT1_DOT, FW_I_ACT2, FW_I_ACT2_DOT,
  FW_I_WIND_N, FW_I_WIND_E, FW_I_WIND_D,
  FW_NINIT
};

/* state blocks for fw_get_state / fw_set_state (all SoA, [rows][N]) */
#define FW_BLK_ODE 0        /* FW_NY rows, T */
#define FW_BLK_DERIVED 1    /* 8 rows, T: roll pitch yaw Va alpha beta elevator aileron */
#define FW_BLK_TARGET 2     /* 3 rows, T */
#define FW_BLK_WIND 3       /* 3 rows, T: steady wind n e d */
#define FW_BLK_STEPS 4      /* 1 row, uint32: steps_count | steps_for_current_target << 16 */
#define FW_BLK_COMMAND 5    /* 3 rows, T: last constrained commands (input order) */
#define FW_BLK_PARAMS 6     /* FW_NPARAM rows, T: per-aircraft parameters (only with env->n_rand > 0) */
#define FW_BLK_ACT_RING 7   /* window*3 rows, T: raw actions, action number k (1-based) in slot (k-1) % window,
                               row slot*3 + component (the action-delta reward / action-window observation).
                               This is the layout fw_get_state / fw_set_state exchange; on the device the ring
                               is indexed by the aircraft's lifetime step count (slots stay aligned across
                               aircraft whose episodes started at different steps, so a wave's ring accesses
                               coalesce) and the two calls translate */
#define FW_BLK_CMD_RING 8   /* window*3 rows, T: constrained commands, same layout (unscaled action windows) */
#define FW_BLK_TARGET_PROPS 10 /* 12 rows, T (ABI 11; linear / sinusoidal target classes only): per target (roll, pitch,
                                * Va) 4 rows: slope (linear) or amplitude, period, phase, bias (sinusoidal); ABI 12:
                                * 15 rows with attitude_angular targets, rows 12..14 = the omega_p / q / r targets */
#define FW_BLK_GOAL 9       /* 4 rows, uint32: the last 128 goal-status bits ("all"), bit 0 of row 0 newest (0 before
                             * the episode's first entry).  Env handles only.  Setting it takes the episode's
                             * history length from FW_BLK_STEPS (steps_count + 1 entries): set FW_BLK_STEPS first */
#define FW_NBLK 10

typedef struct fw_handle fw_handle;

int fw_abi_version(void);
int fw_last_error(char* buf, size_t len);

/* env may be NULL: a PyFly-only handle (fw_env_step then fails).  */
int fw_create(const fw_sim_config* sim, const fw_env_config* env, int64_t n_envs, int32_t precision,
              int32_t device, fw_handle** out);
int fw_destroy(fw_handle* h);
int fw_num_envs(const fw_handle* h, int64_t* n);
int fw_num_obs(const fw_handle* h, int32_t* n);

/* Counter-based RNG key: env i of this handle draws from stream (seed, env_offset + i).  Also restarts
 * every env's episode counter, so a reset after fw_seed repeats the draws of the first reset after
 * fw_create (gym's seed-then-reset reproducibility).  Synchronises the device; a setup call.        */
int fw_seed(fw_handle* h, uint64_t seed, int64_t env_offset);

/* Turbulence noise injection (the turbulence_noise argument of PyFly.reset, pyfly.py:1262, which
 * Wind.reset hands to DrydenGustModel.reset, dryden.py:174-188): N(0,1) samples, SoA [4][len][N],
 * read from index 0 at each reset; step k of an episode reads sample k mod len (dryden.py:209-236
 * wraps a sequence shorter than the episode).  NULL reverts to the on-device Philox generator.  The
 * buffer must stay alive while the handle uses it.  Every call drops the per-env lengths
 * (fw_set_noise_lengths), which describe a buffer: set them again after it.                        */
int fw_set_noise(fw_handle* h, const void* noise_dev, int64_t len);

/* ABI 11: the env's own np_random draws from a caller tape instead of the handle's Philox streams, so a
 * device episode can replay the reference's (FixedWingAircraft.np_random, fixed_wing.py:324-332).  tape_dev:
 * [len][N] (handle precision), aircraft i consumes column i in order; each draw u is used as numpy's
 * uniform(low, high) = low + (high - low) * u.  The draws, in the reference's order: at every reset
 * (fw_reset, the auto-reset of fw_env_step / fw_env_rollout) sample_target per target (roll, pitch, Va):
 * the initial value, then for class linear the slope and its sign (u < 0.5 flips it), for class sinusoidal
 * the amplitude, the period and the phase (fixed_wing.py:654-722) -- also for a target given explicitly,
 * which the reference draws and then overrides (:436-448); then one scaling per randomised reward factor
 * (reward.randomize_scaling, :473-479).  At a resample (target.resample_every, on_success "new",
 * :570-575): sample_target again.  Parameter randomisation (a "model" block) keeps its Philox draws.  Every
 * call restarts the cursors at draw 0; a draw past len is NaN.  NULL: the Philox streams again.  The tape
 * must stay alive while the handle uses it.                                                           */
int fw_set_env_draws(fw_handle* h, const void* tape_dev, int32_t len);

/* Per-env injection (env_method("reset", indices=..., turbulence_noise=...) -> FixedWingAircraft.reset
 * (**sim_reset_kw), fixed_wing.py:414-441): env_len_dev int32[N]; env i with env_len[i] > 0 reads its
 * first env_len[i] samples of the fw_set_noise buffer (column i, wrapped as above; env_len[i] <= the
 * buffer's len), env_len[i] == 0 draws from Philox, env_len[i] < 0 reads the first -env_len[i]
 * samples like a positive length but marks a shared (fw_set_noise-wide) sequence.  The VecEnv
 * auto-reset of fw_env_step / fw_env_rollout zeroes a positive env_len[i] (the SubprocVecEnv worker
 * resets without turbulence_noise, so Dryden.reset(None) draws fresh noise) and keeps a negative one,
 * as an env without per-env lengths keeps the buffer; fw_reset leaves it to the caller.  NULL: every
 * env reads the buffer (fw_set_noise alone).                                                        */
int fw_set_noise_lengths(fw_handle* h, int32_t* env_len_dev);

/* Masked reset.  mask_dev: uint8[N] (NULL = all).  init_dev: [FW_NINIT][N] or
 * NULL (all sampled).  target_dev: [3][N] or NULL.  obs_dev: [N][n_obs] or NULL. */
int fw_reset(fw_handle* h, const uint8_t* mask_dev, const void* init_dev, const void* target_dev,
             void* obs_dev, void* stream);

/* PyFly.step for all envs.  commands_dev: [N][3] in actuation-input order
 * (elevator, aileron, throttle).  Outputs (NULL = skip): commands_out_dev [N][3]
 * constrained commands, success_dev uint8[N], term_dev int32[N] (FW_TERM_*),
 * stats_dev int32[N] = min(nfev, 0xFFFF) | (min(n_accepted, 0x3FFF) << 16);
 * bit 31 set when the RK45 integration failed (TOO_SMALL_STEP, a NaN step or
 * the max_nfev budget) and the last accepted sub-step was committed, as
 * solve_ivp's sol.y[:, -1] is; bit 30 set when that failure was the budget
 * (FW_STATS_BUDGET: a step scipy would have continued).                       */
int fw_sim_step(fw_handle* h, const void* commands_dev, void* commands_out_dev, uint8_t* success_dev,
                int32_t* term_dev, int32_t* stats_dev, void* stream);

/* FixedWingAircraft.step for all envs (+ VecEnv auto-reset when auto_reset != 0).
 * actions_dev [N][3]; obs_dev [N][n_obs]; reward_dev [N]; done_dev uint8[N];
 * term_dev int32[N]; terminal_obs_dev [N][n_obs] (written for done envs only,
 * may be NULL); episode_dev [N][5] = (return, length, final target roll,
 * pitch, Va) written for done envs (may be NULL); stats_dev as in fw_sim_step
 * (may be NULL).                                                             */
int fw_env_step(fw_handle* h, const void* actions_dev, void* obs_dev, void* reward_dev, uint8_t* done_dev,
                int32_t* term_dev, void* terminal_obs_dev, void* episode_dev, int32_t* stats_dev,
                int32_t auto_reset, void* stream);

/* Open-loop rollout: n_steps consecutive fw_env_step calls in ONE launch, for actions known in
 * advance (SAC / TD3 warm-up with uniform actions, off_policy_algorithm.py:354-472 collect_rollouts
 * before learning_starts; scripted command sequences).  Same per-step semantics and results as
 * n_steps fw_env_step launches, bit for bit; each wave advances through the steps on its own instead of
 * every step waiting for the slowest aircraft of the batch.  actions_dev [K][N][3]; per-step outputs
 * stacked: obs_dev [K][N][n_obs], reward_dev [K][N], done_dev uint8[K][N], and (each may be NULL)
 * term_dev int32[K][N], terminal_obs_dev [K][N][n_obs], episode_dev [K][N][5], stats_dev int32[K][N].
 * The metrics record (fw_set_metrics_output) holds each env's last episode that ended in the launch. */
int fw_env_rollout(fw_handle* h, int32_t n_steps, const void* actions_dev, void* obs_dev, void* reward_dev,
                   uint8_t* done_dev, int32_t* term_dev, void* terminal_obs_dev, void* episode_dev, int32_t* stats_dev,
                   int32_t auto_reset, void* stream);

/* Lanes per aircraft of fw_env_step / fw_sim_step (an execution choice, no reference counterpart):
 * 1 = one lane integrates one aircraft; 4 = a lane quad integrates it (the RHS split by rows,
 * DESIGN.md 3.3): lower latency per aircraft, for shards of few aircraft and the RK45 straggler tail;
 * 2 (round 6) = a lane pair (two virtual quad rows per lane), an option the automatic choice never takes.
 * FW_LANES_AUTO (0, the default) picks by N.  The two agree within rounding, not bit for bit; a config
 * with a wrapped ODE-state variable always runs 1 (fw_set_lanes(h, 4) fails).  fw_get_lanes returns the
 * value the next launch uses; fw_env_rollout runs the same, so it still equals fw_env_step launches.   */
#define FW_LANES_AUTO 0
int fw_set_lanes(fw_handle* h, int32_t lanes);
int fw_get_lanes(const fw_handle* h, int32_t* lanes);
/* The automatic rule's threshold: FW_LANES_AUTO runs quads for N <= this (the build's FW_QUAD_AUTO_MAX).
 * A sharded VecEnv applies the same rule to the global batch so every shard runs one integrator. */
int64_t fw_quad_auto_max(void);

/* Observation of the current state (FixedWingAircraft.get_observation). */
int fw_observe(fw_handle* h, void* obs_dev, void* stream);

int fw_get_state(fw_handle* h, int32_t block, void* dst_dev, void* stream);
int fw_set_state(fw_handle* h, int32_t block, const void* src_dev, void* stream);
/* Rows of a state block (its [rows][N] shape) on this handle; element size: uint32 for FW_BLK_STEPS and
 * FW_BLK_GOAL, the handle's precision otherwise.  A block the handle does not hold is FW_E_INVALID. */
int fw_block_rows(const fw_handle* h, int32_t block, int32_t* rows);

/* Curriculum / config update between steps (FixedWingAircraft.set_curriculum_level
 * recomputes ranges on the host and pushes a new env/sim config).            */
int fw_update_config(fw_handle* h, const fw_sim_config* sim, const fw_env_config* env);

/* Register the device buffer [FW_NMETRIC][N] that fw_env_step fills for done envs (the episode
 * metrics of FixedWingAircraft.get_metric, fixed_wing.py:1644-1736, which the reference puts in
 * info on done).  NULL stops the writes.  Requires env->metrics at create time. */
int fw_set_metrics_output(fw_handle* h, void* metrics_dev);

/* The env-side half of VecNormalize.step_wait (stable_baselines3/common/vec_env/vec_normalize.py:106-131),
 * run by fw_env_step's own epilogue while the step's observation is on chip, so a PPO collect step needs
 * no separate statistics pass over the observations (running_mean_std.py:20-24 RunningMeanStd.update's
 * batch moments):
 *   ret      [N] fp64 discounted return: ret = ret * gamma + reward (VecNormalize._update_reward,
 *            vec_normalize.py:126-129), then ret[done] = 0 (vec_normalize.py:130) -- or NULL (no return column)
 *   records  fp64, D = n_obs_values + (ret != NULL): one exact two-pass moment record per launch block
 *            (n_b, mean_b[D], M2_b[D]) of the float32 observation (the VecEnv output: the reset observation
 *            of an auto-reset env) and of ret before its reset -- or NULL.  COLUMN-major: field f of block b
 *            at records[f * R + b], R = fw_collect_records(h)'s n_records (so each field's loads coalesce);
 *            size the buffer (1 + 2D) * max_records.  Merge with fw_moments_merge / fw_vecnorm_merge_update
 *            (fwrollout.h), which read this layout -- or inside the launch (merged).
 *   row_ctrl optional device int32: the launch does row_ctrl[0] += 1 after every block read its inputs
 *            (the rollout row of a captured collect step, fw_collect_policy in fwrollout.h).
 *   merged   (ABI 9; needs records) fp64 [1 + 2D]: the launch itself merges its block records (a tree of
 *            64-record nodes, each merged in block order by the last block to reach it, so the result is
 *            deterministic) into one record (N, mean[D], M2[D]), the layout fw_rms_update reads -- what
 *            fw_moments_merge returns, to rounding (another summation tree).  NULL: merge later.
 *   rms      (ABI 9; needs merged) the fw_rms_update statistics buffer [2d + 4]: the launch also applies
 *            RunningMeanStd.update_from_moments (running_mean_std.py:26-40) with the merged record, the
 *            same arithmetic as fw_rms_update of that one record.  A collect step under one VecNormalize is
 *            then policy + env step, two launches.  NULL: update later (sharded: after the exchange).
 *   defer    (ABI 12; needs merged) 1: the tree stops one level short -- the launch leaves the final node's
 *            records (at most 64, fw_collect_pending) in place and writes neither merged nor rms; the next
 *            fw_collect_policy (fwrollout.h, io->pend) merges them in its prologue and applies the update, or
 *            fw_vecnorm_pending_update does.  Same bits as the in-launch final node (the same sums in the same
 *            order); takes the final node's hand-off chain off the env step's tail.
 * Applies to fw_env_step only (not fw_env_rollout); NULL (or all fields NULL) turns it off. */
typedef struct fw_collect_epilogue {
  double* ret;
  double gamma;
  double* records;
  int32_t* row_ctrl;
  double* merged;
  double* rms;
  int32_t defer;
  int32_t pad;
} fw_collect_epilogue;
int fw_set_collect_epilogue(fw_handle* h, const fw_collect_epilogue* epi);
/* ABI 12: where the deferred final level of the next fw_env_step lives (with the current epilogue and lanes
 * setting): count records of 1 + 2D fp64 fields, field f of record k at records[f * stride + k]; rms_prev =
 * the launch's copy of rms [2d + 4] as it found it, which the merging fw_collect_policy launch reads (its
 * block 0 rewrites rms while other blocks may still be starting). */
typedef struct fw_collect_pend {
  const double* records;
  int64_t stride;
  int32_t count;
  int32_t D;
  const double* rms_prev;
} fw_collect_pend;
int fw_collect_pending(const fw_handle* h, fw_collect_pend* out);
/* Records the next fw_env_step writes (its block count: depends on N and fw_get_lanes) and the most any
 * lanes setting can write (size the buffer with that). */
int fw_collect_records(const fw_handle* h, int64_t* n_records, int64_t* max_records);

#ifdef __cplusplus
}
#endif
#endif /* FWSIM_H */
