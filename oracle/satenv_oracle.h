/*
 * oracle/satenv_oracle.h -- TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline).
 *
 * Plain-C FP64 restatement of the reference environment hot path
 * (environment.py Flag 0/1 step + satellite_function.py CW STM and
 * danger-zone count, incl. a scalar restatement of MINPACK hybrd as called
 * by scipy.optimize.fsolve).  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it.  The product path
 * (ppo-rl-satellite_amd/) never links or calls this.
 *
 * Parity pinning: the fixtures under tests/golden were captured by importing the
 * reference in the build container (tests/golden/capture_golden.py).
 */
#ifndef SATENV_ORACLE_H
#define SATENV_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* numpy scalar type of a reference fuel attribute (environment.py:42-43,106-107):
 * starts as a python int, becomes np.float32 after the first f32 subtraction,
 * np.int64 / np.float64 after an integer [0,0,0] action is subtracted.      */
enum { ORC_PYINT = 0, ORC_I64 = 1, ORC_F32 = 2, ORC_F64 = 3 };

typedef struct {
    double Pp[3], Pv[3], Ep[3], Ev[3];   /* relative (CW frame) pos/vel */
    double fuel_c, fuel_t, dis;          /* persist across reset()        */
    int32_t dz;                          /* self.dangerous_zone           */
    int32_t fuel_c_mode, fuel_t_mode;    /* ORC_* numpy type tags         */
    int32_t vel_int;                     /* velocities are int64 arrays   */
    int32_t flag;                        /* self.Flag                     */
} orc_env;

typedef struct {
    double d_capture, d_range;
    double win_reward, burn_reward;
    int32_t max_episode_steps;
    double mu;            /* 3.986e14 */
    double R_cw[3], V_cw[3];
    double stm[36];       /* row-major 6x6, satellite_function.py:766-773 */
    double cw_omega;      /* mean motion of the STM (satellite_function.py:761) */
    int32_t propagator;   /* 0: closed-form STM (reference), 1: RK4 on the CW ODE, 2: solve_ivp RK45 */
    int32_t rk4_substeps; /* RK4 steps per 100-s env step (propagator 1)         */
} orc_params;

void orc_default_params(orc_params* p, double d_capture, int32_t max_episode_steps);
void orc_stm(double t, double out[36]);
void orc_env_init(orc_env* e);                 /* ctor state, environment.py:26-62 */
void orc_reset(orc_env* e, int32_t flag, double obs[18]);
/* returns 0 ok, <0 unsupported orbit branch (4/5-element) */
int  orc_step(const orc_params* p, orc_env* e, const float pa[3], const float ea[3],
              int32_t episode_count, double obs[18], double* reward, int32_t* done);

/* danger-zone count of environment.py:317-332 on absolute states */
int  orc_danger_zone(const double R0_c[3], const double V0_c[3], const double R0_t[3],
                     const double V0_t[3], double fuel, int32_t fuel_mode, int32_t* count);
int  orc_orbital_elements(double mu, const double R[3], const double V[3], double out[6]);
/* fsolve(P_fai_equation, guess) of satellite_function.py:558-565 */
double orc_solve_alpha(double mu, double dvm, double theta, double v1x, double v1y,
                       double h, double guess, int32_t* nfev);

/* RK4 two-body + J2 propagator of 轨道外推-龙格库塔算法.py (km, km/s):
 * StateEq (:15-31) and one RungeKutta step (:35-41); propagate applies
 * `steps` steps of size h in place.                                       */
void orc_rk4_j2_rhs(const double rv[6], double f[6]);
void orc_rk4_j2_step(const double rv[6], double h, double out[6]);
void orc_rk4_j2_propagate(double rv[6], double h, int32_t steps);
/* RK4 on the Clohessy-Wiltshire ODE x'' = 2w y' + 3w^2 x, y'' = -2w x',
 * z'' = -w^2 z over t seconds in nsub equal steps (propagator 1; the
 * RungeKutta stage combination of the script above)                      */
void orc_cw_rk4(const double x[6], double w, double t, int32_t nsub, double y[6]);
/* satellite_function.py:783-839 Numerical_calculation_method: the CW
 * orbit_ode (omega from r = 35786 km) by scipy solve_ivp RK45 (rtol 1e-3,
 * atol 1e-6) over (0, t), result = the dense output at t (t a multiple of
 * 50, the t_eval spacing).  Returns 0, or -6 (scipy's TOO_SMALL_STEP);
 * *nfev = solve_ivp's function evaluations.                              */
int  orc_cw_rk45(const double x[6], double t, double y[6], int32_t* nfev);

/* reachable-domain direction grid, RD_single_pulse.py:40-148 (params :9-20) */
typedef struct {
    double a, e0, f, delta_max, mu;
    int32_t n1, n2, n3;
    int32_t dv_f32;   /* delta_max is an np.float32 scalar: Delta_V and Delta_V ** 2 in float32 */
} orc_rd_params;
/* fills n1*(n2+1)*(n3+1) directions; returns the number with status 1 */
int64_t orc_reachable_domain(const orc_rd_params* p, double* rf_max, double* rf_min, uint8_t* status);

/* libm-tie probe: non-zero seed = transcendental results moved by one
 * (seed >= 1024: two) ulp, which calls and which way from a hash of seed
 * and call index; 0 = exact glibc (default)                              */
void orc_set_jitter(unsigned long long seed);

/* one step of n envs held as SoA planes (satenv_get_state layout), in place */
int  orc_step_planes(const orc_params* p, int64_t n, double* f64, int32_t* i32, const float* pa,
                     const float* ea, const int32_t* episode_count, double* reward_out, int32_t* done_out,
                     int32_t nthreads);

/* batched replay for the CPU baseline: n envs x steps, actions [steps][n][3] */
int  orc_rollout(const orc_params* p, orc_env* envs, int64_t n, int32_t steps,
                 const float* pa, const float* ea, int32_t* episode_count,
                 double* reward_out, int32_t* done_out, int32_t nthreads);

#ifdef __cplusplus
}
#endif
#endif
