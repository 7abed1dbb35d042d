// satenv_step.h -- one environment step (environment.py:81-255) per lane,
// for both targets: the gfx950 kernels (satenv_kernels.hip) and the host
// build of the same ABI (satenv_cpu.cpp, OpenMP over envs).
//
// Per-handle state layout (num_envs = N):
//   f64 planes [16][N]  Pp0..2 Pv0..2 Ep0..2 Ev0..2 fuel_c fuel_t dis ep_return
//   i32 planes [3][N]   dangerous_zone, episode_count, bits
#pragma once
#include "satenv_device.h"

namespace satenv {

constexpr int kF64Planes = 16;   // 15 public + per-env episode return
constexpr int kI32Planes = 3;
constexpr int kPlaneRet = 15;
constexpr int kPlaneDz = 0, kPlaneCount = 1, kPlaneBits = 2;

struct alignas(8) F32x2 { float x, y; };

struct StepIO {
  const float* pa;
  const float* ea;
  const int32_t* ext_count;   // nullptr -> device counters
  float* obs;
  double* obs64;
  double* rew64;
  float* rew32;
  uint8_t* done;
  double* stats;
  int32_t* err;
};

SATENV_HD void write_obs(float* obs, double* obs64, int64_t i, const double (&k)[12]) {
  // [Pp-Ep, Pv-Ev, Pp, Pv, Ep, Ev]  environment.py:76-77,177-178
  double o[18];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    o[c] = k[c] - k[6 + c];
    o[3 + c] = k[3 + c] - k[9 + c];
    o[6 + c] = k[c];
    o[9 + c] = k[3 + c];
    o[12 + c] = k[6 + c];
    o[15 + c] = k[9 + c];
  }
  if (obs) {
    F32x2* dst = reinterpret_cast<F32x2*>(obs + i * 18);     // 8-B aligned rows
#pragma unroll
    for (int c = 0; c < 9; ++c) dst[c] = F32x2{(float)o[2 * c], (float)o[2 * c + 1]};
  }
  if (obs64) {
#pragma unroll
    for (int c = 0; c < 18; ++c) obs64[i * 18 + c] = o[c];
  }
}

SATENV_HD void reset_kin(const Params& /*p*/, double (&k)[12]) {
  // environment.py:67-71 reset positions/velocities (int64 arrays)
#pragma unroll
  for (int c = 0; c < 12; ++c) k[c] = 0.0;
  k[0] = 200000.0;
  k[6] = 18000.0;
}

// ---------------------------------------------------------------------------
// One environment step (environment.py:81-255), one lane per env, in two
// halves around the danger-zone count: step_begin (actions, fuel, STM,
// terminal tests, the count's set-up) and step_end (count, reward, outputs,
// autoreset, state write-back).
// ---------------------------------------------------------------------------
struct Lane {
  double k[12];
  double fuel_c, fuel_t, dis, dis_prev;
  int dz, count, flag, fcm, ftm;
  bool p_zero;
  float pa[3];
  int err;                // propagator 2: scipy's TOO_SMALL_STEP (-6), else 0
  bool terminal;          // reward/done final, no count: capture or timeout (:139-147 return first), or Flag 2
  double reward;
  bool done;
  double cap;
};

// kRk45: the instantiation that carries propagator 2 (solve_ivp RK45); the
// default kernels leave it out so its registers do not cost the STM path
// occupancy
template <bool kRk45 = false>
SATENV_HD void step_begin(const Params& prm, int64_t n, const double* __restrict__ f64,
                                           const int32_t* __restrict__ i32, const StepIO& io, int64_t i,
                                           bool autoreset, Lane& L) {
  double* k = L.k;
#pragma unroll
  for (int c = 0; c < 12; ++c) k[c] = f64[c * n + i];
  L.fuel_c = f64[12 * n + i];
  L.fuel_t = f64[13 * n + i];
  L.dis = f64[14 * n + i];
  L.dz = i32[kPlaneDz * n + i];
  const int bits = i32[kPlaneBits * n + i];
  if (autoreset || io.ext_count == nullptr) L.count = i32[kPlaneCount * n + i] + 1;
  else L.count = io.ext_count[i];
  L.flag = env_flag(bits);
  const int vi = vel_int(bits);
  L.fcm = fc_mode(bits);
  L.ftm = ft_mode(bits);
  float ea[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    L.pa[c] = clip16(io.pa[i * 3 + c]);                                  // :86-87
    ea[c] = clip16(io.ea[i * 3 + c]);
  }
  L.dis_prev = norm3(k[0] - k[6], k[1] - k[7], k[2] - k[8]);             // :89
  bool p_zero = false, e_zero = false, move_p = true, move_e = true;
  if (L.flag != 1) {                                                      // Flag 0 and Flag 2 (:262-276)
    if (L.dis < prm.d_range && L.dz != 0) { move_p = false; p_zero = true; }   // :91-97
  } else {
    if (L.dz == 0) { move_e = false; e_zero = true; }                         // :194-198
  }
  L.p_zero = p_zero;
#pragma unroll
  for (int c = 0; c < 3; ++c) {                                           // Vector[i] += action[i]
    if (move_p) { const double t = k[3 + c] + (double)L.pa[c]; k[3 + c] = vi ? trunc(t) : t; }
    if (move_e) { const double t = k[9 + c] + (double)ea[c]; k[9 + c] = vi ? trunc(t) : t; }
  }
  fuel_sub(L.fuel_c, L.fcm, p_zero, (fabsf(L.pa[0]) + fabsf(L.pa[1])) + fabsf(L.pa[2]));   // :106
  fuel_sub(L.fuel_t, L.ftm, e_zero, (fabsf(ea[0]) + fabsf(ea[1])) + fabsf(ea[2]));         // :107

  L.err = 0;
  bool propagated = false;
  if constexpr (kRk45) {
    if (prm.propagator == 2) {                                            // optional: solve_ivp RK45 (:783-839)
#pragma unroll 1
      for (int craft = 0; craft < 2; ++craft) {
        double x[6];
#pragma unroll
        for (int c = 0; c < 6; ++c) x[c] = k[6 * craft + c];
        const int rc = cw_rk45(x, 100.0);
        if (rc) L.err = rc;
#pragma unroll
        for (int c = 0; c < 6; ++c) k[6 * craft + c] = x[c];
      }
      propagated = true;
    }
  }
  if (propagated) {
  } else if (prm.propagator == 1) {                                       // optional: RK4 on the CW ODE
#pragma unroll
    for (int craft = 0; craft < 2; ++craft) {
      double x[6];
#pragma unroll
      for (int c = 0; c < 6; ++c) x[c] = k[6 * craft + c];
      cw_rk4(x, prm.cw_omega, 100.0, prm.rk4_substeps);
#pragma unroll
      for (int c = 0; c < 6; ++c) k[6 * craft + c] = x[c];
    }
  } else {
    // Clohessy-Wiltshire STM (satellite_function.py:776-779), OpenBLAS dgemv_t order
    double y[12];
#pragma unroll
    for (int craft = 0; craft < 2; ++craft) {
      const double* x = k + 6 * craft;
#pragma unroll
      for (int r = 0; r < 6; ++r) {
        const double* M = prm.stm + 6 * r;
        const double p0 = M[0] * x[0], p1 = M[1] * x[1], p2 = M[2] * x[2];
        const double p3 = M[3] * x[3], p4 = M[4] * x[4], p5 = M[5] * x[5];
        y[6 * craft + r] = (((p0 + p2) + (p1 + p3)) + p4) + p5;
      }
    }
#pragma unroll
    for (int c = 0; c < 12; ++c) k[c] = y[c];
  }
  L.dis = norm3(k[0] - k[6], k[1] - k[7], k[2] - k[8]);                   // :132
  L.cap = 0.0;
  L.terminal = true;
  L.done = true;
  if (L.dis <= prm.d_capture) {                                           // :139-142, :221-225, :303-306
    L.reward = L.flag == 0 ? prm.win_reward : (L.flag == 1 ? -150.0 : 0.0);
    L.cap = 1.0;
  } else if (L.count >= prm.max_episode_steps) {                         // :144-147, :227-231, :308-311
    L.reward = L.flag == 0 ? prm.burn_reward : (L.flag == 1 ? prm.win_reward : 0.0);
  } else if (L.flag == 2) {                                               // :313-315: reward 0, not done,
    L.reward = 0.0;                                                       // no danger-zone update (the
    L.done = false;                                                       // ellipse fit and the surrogate
  } else {                                                                // training run outside the kernel)
    L.terminal = false;
    L.done = false;
  }
}

// the count-independent reward terms 1*pv1, 0.6*pv2, 0.2*pv3, 2*pv4 (:166-175)
SATENV_HD void reward_terms(const double (&k)[12], const float (&pa)[3], bool p_zero, double (&t)[4]) {
  const double r0 = k[0] - k[6], r1 = k[1] - k[7], r2 = k[2] - k[8];
  const double pv1 = cos_sim(k[0], k[1], k[2], k[6], k[7], k[8]);       // reward_of_action3
  const double pv2 = cos_sim(k[3], k[4], k[5], k[9], k[10], k[11]);     // reward_of_action1
  const double pv3 = cos_sim(r0, r1, r2, k[3], k[4], k[5]);             // reward_of_action2
  double pv4 = 0.0;                                                      // reward_of_action4, :388
  if (!p_zero && pa[0] != 0.0f && pa[1] != 0.0f && pa[2] != 0.0f) {
    const double nr = norm3(r0, r1, r2);
    const float na = norm3f(pa[0], pa[1], pa[2]);
    pv4 = -dot3(r0 / nr, r1 / nr, r2 / nr, (double)(pa[0] / na), (double)(pa[1] / na), (double)(pa[2] / na));
  }
  t[0] = 1 * pv1;
  t[1] = 0.6 * pv2;
  t[2] = 0.2 * pv3;
  t[3] = 2 * pv4;
}

// non-terminal reward with the new danger-zone count (:150, :161-175, :251)
SATENV_HD void step_reward_terms(const Params& prm, Lane& L, int cnt, const double (&t)[4]) {
  L.dz = cnt;
  double r = (L.dis < L.dis_prev) ? 1.0 : -1.0;                          // :161-164
  r += (prm.d_capture <= L.dis && L.dis <= 4 * prm.d_capture) ? -1.0 : -2.0;
  r += (L.dz == 0) ? -1.0 : L.dz * 0.5;
  r += t[0];
  r += t[1];
  r += t[2];
  r += t[3];
  L.reward = L.flag == 0 ? r : -r;                                        // :251
}

SATENV_HD void step_reward(const Params& prm, Lane& L, int cnt) {
  double t[4];
  reward_terms(L.k, L.pa, L.p_zero, t);
  step_reward_terms(prm, L, cnt, t);
}

SATENV_HD void step_end(const Params& prm, int64_t n, double* __restrict__ f64,
                                         int32_t* __restrict__ i32, const StepIO& io, int64_t i, bool autoreset,
                                         Lane& L, double& fin, double& fin_ret, double& rew_acc) {
  if (io.rew64) io.rew64[i] = L.reward;
  if (io.rew32) io.rew32[i] = (float)L.reward;
  if (io.done) io.done[i] = L.done ? 1 : 0;
  double ret = f64[kPlaneRet * n + i] + L.reward;
  rew_acc = L.reward;
  int vi_out = 0;
  if (autoreset && L.done) {                                              // CPPO_main.py:149-153 -> reset(Flag)
    fin = 1.0;
    fin_ret = ret;
    ret = 0.0;
    reset_kin(prm, L.k);
    vi_out = 1;
    L.count = 0;
  }
  write_obs(io.obs, io.obs64, i, L.k);
#pragma unroll
  for (int c = 0; c < 12; ++c) f64[c * n + i] = L.k[c];
  f64[12 * n + i] = L.fuel_c;
  f64[13 * n + i] = L.fuel_t;
  f64[14 * n + i] = L.dis;
  f64[kPlaneRet * n + i] = ret;
  i32[kPlaneDz * n + i] = L.dz;
  i32[kPlaneCount * n + i] = L.count;
  i32[kPlaneBits * n + i] = make_bits(L.fcm, L.ftm, vi_out, L.flag);
}

SATENV_HD int lane_setup(const Params& prm, const Lane& L, DzCtx& z) {
  const double* k = L.k;
  return dz_setup(prm, k[0], k[1], k[2], k[3], k[4], k[5], k[6], k[7], k[8], k[9], k[10], k[11], L.fuel_c, L.fcm,
                  z);
}

}  // namespace satenv
