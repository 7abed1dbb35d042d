/*
 * satenv.h -- C ABI of the MI355X vectorised satellite pursuit-evasion
 * environment (one HIP lane per env, FP64 SoA state resident in HBM).
 *
 * Drop-in boundary for the reference's environment object
 * (qiaobeibei/PPO-RL-Satellite environment.py):
 *   satenv_create / satenv_set_params  <- satellites.__init__   environment.py:26-62
 *   satenv_reset                       <- satellites.reset      environment.py:66-79
 *   satenv_step                        <- satellites.step       environment.py:81-315 (Flag 0, 1, 2)
 *   satenv_step_autoreset              <- the CPPO_main.py:119-153 inner loop around step/reset
 *   satenv_get_state / satenv_set_state<- attribute access (Pursuer_position, fuel_c, dis, ...)
 *   satenv_default_params / satenv_stm <- ctor defaults + Clohessy_Wiltshire.State_transition_matrix
 *                                          satellite_function.py:753-781
 *
 * Conventions: every pointer argument is a caller-owned DEVICE buffer unless
 * stated otherwise; calls are asynchronous on `stream` (a hipStream_t, NULL =
 * default stream) and capturable into a hipGraph; one handle per stream,
 * not thread-safe.  Return 0 on success or a negative SATENV_ERR_* code
 * (message via satenv_last_error()).  Device-side failures (the reference's
 * crashing 4/5-element orbit branches) are sticky and reported by
 * satenv_check().
 */
#ifndef SATENV_H
#define SATENV_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SATENV_ABI_VERSION 2
#define SATENV_OBS_DIM 18    /* [Pp-Ep, Pv-Ev, Pp, Pv, Ep, Ev]  environment.py:76-77 */
#define SATENV_ACT_DIM 3
#define SATENV_F64_PLANES 15 /* Pp[3] Pv[3] Ep[3] Ev[3] fuel_c fuel_t dis, each [num_envs] */
#define SATENV_I32_PLANES 3  /* dangerous_zone, episode_count, bits (see below) */

enum {
    SATENV_OK = 0,
    SATENV_ERR_ARG = -1,
    SATENV_ERR_HIP = -2,
    SATENV_ERR_ORBIT_CIRCULAR = -4,  /* calculate_orbital_elements e == 0 (satellite_function.py:251) */
    SATENV_ERR_ORBIT_PARABOLIC = -5, /* 2/r - v^2/mu == 0 (satellite_function.py:253) */
    SATENV_ERR_STEP_TOO_SMALL = -6,  /* propagator 2: solve_ivp's RK45 stopped (TOO_SMALL_STEP) */
};

/* numpy scalar type carried by the reference's fuel attributes; bits plane:
 * [1:0] fuel_c type, [3:2] fuel_t type, [4] velocities are int64 (fresh
 * after reset), [6:5] Flag (0 pursuer training, 1 evader training, 2
 * reachable-domain fitting: environment.py:257-315, no danger-zone update,
 * reward 0; its ellipse fit is satenv_rd_orbits + the grid/fit kernels). */
enum { SATENV_NUM_PYINT = 0, SATENV_NUM_I64 = 1, SATENV_NUM_F32 = 2, SATENV_NUM_F64 = 3 };

typedef struct satenv_params {
    double d_capture;          /* environment.py:35; train_* overwrite it (CPPO_main.py:98)  */
    double d_range;            /* environment.py:45 (ctor default 100000)                    */
    double win_reward;         /* environment.py:40                                          */
    double burn_reward;        /* environment.py:39                                          */
    double mu;                 /* 3.986e14                                                    */
    double R_cw[3], V_cw[3];   /* CW reference point, environment.py:338-339                 */
    double stm[36];            /* row-major 6x6 STM, satellite_function.py:766-773, t=100 s  */
    double fuel_c0, fuel_t0;   /* environment.py:42-43 (ctor 320)                             */
    double init_kin[12];       /* ctor Pursuer/Escaper position, vector (environment.py:26-27)*/
    int32_t max_episode_steps; /* args.max_episode_steps, environment.py:46                  */
    int32_t flag;              /* Flag, environment.py:36                                     */
    int32_t fuel_c0_mode;      /* SATENV_NUM_* of fuel_c0 (ctor: python int)                  */
    int32_t fuel_t0_mode;
    /* ABI 2: propagator of the relative states per 100-s step.  0 = the
     * reference's closed-form CW STM (stm[], default); 1 = RK4 on the CW ODE
     * x'' = 2w y' + 3w^2 x, y'' = -2w x', z'' = -w^2 z with rk4_substeps
     * equal steps (optional mode; the reference STM's [1][4] entry is
     * 4s/w - 3*tau, so the two differ by design).
     * 2 = satellite_function.py:783-839 Numerical_calculation_method: the
     * CW orbit_ode with omega from r = 35786 km (9.33e-5 rad/s), scipy
     * solve_ivp RK45 (rtol 1e-3, atol 1e-6, adaptive steps) over the 100-s
     * step, dense output at t (the reference's commented-out alternative,
     * environment.py:124-128; cw_omega/rk4_substeps unused).              */
    double cw_omega;           /* w = sqrt(mu / 42164000**3), satellite_function.py:761 */
    int32_t propagator;
    int32_t rk4_substeps;
} satenv_params;

typedef struct satenv_env satenv_env;   /* opaque */

/* host-only helpers */
int satenv_default_params(satenv_params* p);
int satenv_stm(double t, double* out36);          /* host pointer, row-major */
const char* satenv_last_error(void);
int satenv_abi_version(void);

int satenv_create(satenv_env** out, int64_t num_envs, const satenv_params* p, int device);
int satenv_destroy(satenv_env* h);
int satenv_num_envs(const satenv_env* h, int64_t* n);                /* host int64 */
int satenv_set_params(satenv_env* h, const satenv_params* p);        /* host struct */
/* which step kernel satenv_step / satenv_step_autoreset launch (propagators 0
 * and 1): 2 = the wide kernel (default; one env's chain over the four waves
 * of a workgroup, wide_envs = 64 envs per workgroup, 16 / 32 for A/B), 1 =
 * the four-solve split kernel, 0 = one lane per env.  All three compute
 * every step bit for bit the same (tests/test_env_gpu.py).                 */
int satenv_set_step_kernel(satenv_env* h, int32_t kind, int32_t wide_envs);

/* reset(Flag) for the envs whose env_mask byte is non-zero (NULL = all);
 * writes obs of ALL envs (f32 [N][18] and/or f64 [N][18], either nullable). */
int satenv_reset(satenv_env* h, int32_t flag, const uint8_t* env_mask, float* obs_out, double* obs64_out,
                 void* stream);

/* step(pursuer_action, escaper_action, epsiode_count) for all envs.
 * pa/ea: f32 [N][3]; episode_count: int32 [N] (NULL = use and advance the
 * device-side counters).  Outputs (nullable): obs f32 [N][18], obs f64
 * [N][18], reward f64 [N], done u8 [N].  No automatic reset.              */
int satenv_step(satenv_env* h, const float* pa, const float* ea, const int32_t* episode_count, float* obs_out,
                double* obs64_out, double* reward_out, uint8_t* done_out, void* stream);

/* vectorised training-loop step: episode counters live on the device; a
 * done env is reset (Flag kept) inside the same kernel and obs_out carries
 * the post-reset observation (what the policy sees next).  reward_out f32
 * [N] as stored by ReplayBuffer (replaybuffer.py:34).  stats_out (nullable,
 * f64[4], accumulated with atomics): finished episodes, sum of their
 * returns, sum of rewards, captures.                                       */
int satenv_step_autoreset(satenv_env* h, const float* pa, const float* ea, float* obs_out, float* reward_out,
                          uint8_t* done_out, double* stats_out, void* stream);

/* state transfer (device buffers): f64 [SATENV_F64_PLANES][N], i32 [SATENV_I32_PLANES][N] */
int satenv_get_state(const satenv_env* h, double* f64_planes, int32_t* i32_planes, void* stream);
int satenv_set_state(satenv_env* h, const double* f64_planes, const int32_t* i32_planes, void* stream);

/* Time_window_of_danger_zone(R0_c, V0_c, R0_t, V0_t, Delta_V_c=fuel)
 *   .calculate_number_of_hanger_area()   satellite_function.py:18-99,341-373
 * on n independent absolute states: states f64 [n][12] = R_c V_c R_t V_t,
 * fuel f64 [n], fuel_mode i32 [n] (SATENV_NUM_*), count_out i32 [n] (a
 * negative entry = unsupported orbit branch).                              */
int satenv_danger_zone(int64_t n, const double* states, const double* fuel, const int32_t* fuel_mode,
                       int32_t* count_out, void* stream);

/* Time_window_of_danger_zone.Numerical_iteration_method(Delta_Vm, theta,
 * v_1x, v_1y, h, alpha_guess)  satellite_function.py:558-565 (fsolve) on n
 * independent inputs: in f64 [n][6], alpha_out f64 [n].                    */
int satenv_solve_alpha(int64_t n, const double* in, double* alpha_out, void* stream);

/* Self-test of the env step's f64 sincos (no reference counterpart): the
 * straight-line transcription of OCML's small-argument sincos the fsolve
 * residual uses (use_library = 0), or the library sincos() itself (1), on n
 * arguments x f64 [n] -> s_out, c_out f64 [n].  The two must agree bitwise
 * (tests/test_env_gpu.py), so the hybrd restatement's arithmetic is the
 * library's.                                                              */
int satenv_sincos(int64_t n, const double* x, double* s_out, double* c_out, int32_t use_library, void* stream);
/* Self-test of the env step's f64 acos (no reference counterpart): the
 * straight-line transcription of OCML's acos the orbital elements and the
 * rf theta use (use_library = 0), or the library acos() (1): out f64 [n].
 * The two must agree bitwise (tests/test_env_gpu.py).                     */
int satenv_acos(int64_t n, const double* x, double* out, int32_t use_library, void* stream);

/* synchronises the handle's device; *status = first sticky device error (0 = none) */
int satenv_check(satenv_env* h, int32_t* status);

/* RK4 two-body + J2 propagator of 轨道外推-龙格库塔算法.py (StateEq :15-31,
 * RungeKutta :35-41; mu = 398600 km^3/s^2, Re = 6378.137 km, J2 =
 * 0.00108263), one lane per state: `steps` RK4 steps of size h seconds.
 * rv_in / rv_out: SoA f64 [6][n] (x, y, z, vx, vy, vz planes, km and
 * km/s); in place allowed.                                               */
int satenv_rk4_j2(int64_t n, const double* rv_in, double h, int32_t steps, double* rv_out, void* stream);

/* Reachable domain of a single impulse, single_pluse_model/RD_single_pulse.py
 * Reachable_Domain (:40-148, module params :9-20), for nsets orbits at once.
 * orbits: device array [nsets].  The direction grid is the reference's:
 * impulse dV = -delta_max + 2 delta_max jj/N1 (jj = 1..N1), gama = 2 pi i/N2
 * (i = 0..N2), alpha = -pi/2 + pi j/N3 (j = 0..N3); direction
 * d = ((jj-1)(N2+1) + i)(N3+1) + j, ndir = N1 (N2+1) (N3+1).
 * status u8 [nsets][ndir]: 0 unreachable (:81), 1 reachable, 2 reachable but
 * gama - f outside both theta branches (:87-90; the reference then reuses a
 * stale theta).  rf_max / rf_min f64 [nsets][ndir][3]: the points
 * max/min(|rf_max|, |rf_min|) * P of :123-124 where status == 1; other
 * entries are left untouched.  Compacting status == 1 in d order gives the
 * RF_max / RF_min lists Reachable_Domain passes to Curve_fitting (:140).   */
typedef struct {
    double a;          /* params['a'], semi-major axis [m]          */
    double e0;         /* params['e0'], eccentricity                */
    double f;          /* params['f'], true anomaly of the burn     */
    double delta_max;  /* params['delta_max'], max impulse [m/s]    */
    double mu;         /* params['u'] = 3.986e14                    */
    double dv_f32;     /* non-zero: params['delta_max'] is an np.float32 scalar (a
                        * Flag-2 env's fuel_c after an f32 action), so Delta_V
                        * (:64) and Delta_V ** 2 (:79, :84) are float32 ops   */
} satenv_rd_orbit;
int satenv_reachable_domain(int64_t nsets, const satenv_rd_orbit* orbits, int32_t n1, int32_t n2, int32_t n3,
                            double* rf_max, double* rf_min, uint8_t* status, void* stream);

/* Flag 2 (environment.py:293-296): numerical_method_process(R0_c, V0_c,
 * fuel_c) = RD_single_pulse.Incoming_parameters(calculate_orbital_elements(
 * 3.986e14, R0_c, V0_c), fuel_c) (real_time_data_process.py:11-110,
 * RD_single_pulse.py:22-37) for every env of the handle: orbits_out
 * [N] = (a, e0 = e, f, delta_max = fuel_c, mu = 3.986e14, dv_f32) of the
 * pursuer's absolute state (relative_state_to_absolute_state :334-343),
 * ready for satenv_reachable_domain + satenv_ellipse_fit.  status_out i32
 * [N]: 0, or SATENV_ERR_ORBIT_* where the orbit has no 6-element set (the
 * reference then indexes data[5] of a 4/5-element list and raises).        */
int satenv_rd_orbits(satenv_env* h, satenv_rd_orbit* orbits_out, int32_t* status_out, void* stream);

/* curve_fitting.Curve_fitting(RF_max, RF_min)  single_pluse_model/curve_fitting.py:475-576
 * on the dense grids of satenv_reachable_domain (same rf_max / rf_min /
 * status buffers, ndir directions per set), one workgroup per (set, envelope).
 * ellipse_out f64 [nsets][2][5]: (xc, yc, a, b, theta) of the RF_max
 * (farthest point per angular bin) and RF_min (nearest) ellipse, as the
 * [2][5] array Curve_fitting returns.  info_out i32 [nsets][2]: > 0 the
 * least-squares function evaluations; < 0 no fit (parameters NaN):
 *   -1  a status-2 direction in the set (the reference's stale theta),
 *   -2  more than 8192 distinct reachable points,
 *   -3  fewer than 2 points, or fewer than 5 angular bins (5 parameters).
 * Optional (nullable) intermediates: fit_points_out f64 [nsets][2][128][2]
 * = the points the least squares fits (one per angular bin, the filtered
 * set of :564, NaN-padded), center_out f64 [nsets][2][2] = the
 * EllipticEnvelope location of :547.                                      */
int satenv_ellipse_fit(int64_t nsets, int32_t ndir, const double* rf_max, const double* rf_min, const uint8_t* status,
                       double* ellipse_out, int32_t* info_out, double* fit_points_out, double* center_out,
                       void* stream);

/* config 5: the ImprovedNN surrogate (single_pluse_model/model.py:7-24,
 * 5 -> 256 -> 128 -> 64 -> 10, ReLU, inference: no dropout) in bf16 with f32
 * accumulation, as network_method_process (real_time_data_process.py:112-125)
 * evaluates it on [a, e, i, f, fuel_c] of the pursuer's absolute orbit (the
 * reference's call site environment.py:158 is commented out; the output is
 * the env's ellipse_params and feeds no reward).
 * blob: device buffer of satenv_surrogate_blob_bytes() bytes, filled by
 * satenv_surrogate_pack from the torch Linear parameters (f32 device
 * arrays, weight [out][in] row-major: w1 [256][5], w2 [128][256], w3 [64][128],
 * w4 [10][64]).  satenv_surrogate: out f32 [N][10] from the handle's current
 * state (NaN rows where the orbit has no 6-element set).
 * satenv_surrogate_mlp: the same network on given features x f32 [n][5].   */
int satenv_surrogate_blob_bytes(void);
int satenv_surrogate_pack(const float* w1, const float* b1, const float* w2, const float* b2, const float* w3,
                          const float* b3, const float* w4, const float* b4, void* blob, void* stream);
int satenv_surrogate(satenv_env* h, const void* blob, float* out, void* stream);
int satenv_surrogate_mlp(int64_t n, const float* x, const void* blob, float* out, void* stream);
/* The offline trainer's StandardScalers (single_pulse_fully_connected_model.py:
 * 273-278: input_scaler / output_scaler, fitted on all_input.csv /
 * output_data.csv) into the blob: the kernels standardise the features in f64
 * before the bf16 input layer, (x - in_mean) / in_scale, and map fc4's output
 * back, y * out_scale + out_mean (sklearn's transform / inverse_transform), so
 * a net trained on standardised data emits real ellipse parameters.  Host
 * arrays of 5, 5, 10, 10 doubles (sklearn's mean_ / scale_).  _pack resets
 * them to the identity (the reference's untrained-scaler MLPNet2 path).      */
int satenv_surrogate_set_scalers(void* blob, const double* in_mean, const double* in_scale, const double* out_mean,
                                 const double* out_scale, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SATENV_H */
