// satenv_kernels.hip -- gfx950 kernels + C-ABI implementation of include/satenv.h.
//
// Layout in HBM (per handle, num_envs = N):
//   f64 planes [16][N]  Pp0..2 Pv0..2 Ep0..2 Ev0..2 fuel_c fuel_t dis ep_return
//   i32 planes [3][N]   dangerous_zone, episode_count, bits
// One lane per env; every plane access is a unit-stride (coalesced) 8-/4-B
// load/store.  Actions [N][3] f32 and obs [N][18] f32 are row-major as the
// policy GEMMs consume them.  The STM and scalars ride in the kernel's
// argument segment (satenv_params by value -> SGPRs / constant cache).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>

#include "satenv.h"
#include "satenv_device.h"
#include "satenv_step.h"
#include "span_probe.h"
#include "ellipse_device.h"
#include "surrogate_device.h"

using namespace satenv;

namespace {


thread_local std::string g_last_error;

bool params_ok(const satenv_params* p) {
  return p->propagator >= 0 && p->propagator <= 2 && p->rk4_substeps >= 1;
}

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

#define HIP_TRY(expr)                                                                  \
  do {                                                                                 \
    hipError_t e_ = (expr);                                                            \
    if (e_ != hipSuccess) return fail(SATENV_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(e_)); \
  } while (0)

#ifdef SATENV_PHASE_PROBE
// development-only phase stamps of step_kernel_wide (tools/env_phase_probe.py),
// never in the shipped build: [workgroup][stamp][wave][s_memtime]
__device__ unsigned long long g_env_probe[1024][8][4];
#define ENV_PROBE(k)                                                                  \
  do {                                                                                \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 1024)                                 \
      g_env_probe[blockIdx.x][k][threadIdx.x >> 6] = clock64();                       \
  } while (0)
#else
#define ENV_PROBE(k) do {} while (0)
#endif

// wave-level reduction of the per-step stats, one f64 atomic per wave and counter
__device__ __forceinline__ void wave_stats(double* stats, double fin, double fin_ret, double rew, double cap) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    fin += __shfl_xor(fin, off, 64);
    fin_ret += __shfl_xor(fin_ret, off, 64);
    rew += __shfl_xor(rew, off, 64);
    cap += __shfl_xor(cap, off, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    if (fin != 0.0) atomicAdd(stats + 0, fin);
    if (fin_ret != 0.0) atomicAdd(stats + 1, fin_ret);
    atomicAdd(stats + 2, rew);
    if (cap != 0.0) atomicAdd(stats + 3, cap);
  }
}

// one lane per env, the count's four solves one after another (64-lane blocks)
template <bool AUTORESET, bool RK45 = false>
__global__ void __launch_bounds__(64) step_kernel(const Params prm, int64_t n, double* __restrict__ f64,
                                                  int32_t* __restrict__ i32, StepIO io) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  double fin = 0.0, fin_ret = 0.0, rew_acc = 0.0, cap = 0.0;
  if (i < n) {
    Lane L;
    step_begin<RK45>(prm, n, f64, i32, io, i, AUTORESET, L);
    if (L.err) atomicCAS(io.err, 0, L.err);
    cap = L.cap;
    if (!L.terminal) {
      int cnt = 0;
      const int rc = danger_zone(prm, L.k[0], L.k[1], L.k[2], L.k[3], L.k[4], L.k[5], L.k[6], L.k[7], L.k[8],
                                 L.k[9], L.k[10], L.k[11], L.fuel_c, L.fcm, cnt);   // :150, :317-332
      if (rc) atomicCAS(io.err, 0, rc);
      step_reward(prm, L, cnt);
    }
    step_end(prm, n, f64, i32, io, i, AUTORESET, L, fin, fin_ret, rew_acc);
  }
  if (io.stats) wave_stats(io.stats, fin, fin_ret, rew_acc, cap);
}

// 64 envs per 4-wave workgroup: wave 0 runs the env lanes (step_begin, the
// count's set-up, then its finish and step_end), and between two barriers
// wave w solves fsolve problem w of every env of the block (the c-th
// rf_extreme_point's k-th guess, w = 2c + k) -- so the four dependent
// hybrd loops of an env run side by side on four SIMDs instead of one
// after another on one, and a launch has 4x the waves (the step is FP64
// latency bound: 16384 envs are only 256 waves).  Bit-identical to
// step_kernel: every problem runs the same hybrd1.
constexpr int kSplitEnvs = 64;
template <bool AUTORESET, bool RK45 = false>
__global__ void __launch_bounds__(256) step_kernel_split(const Params prm, int64_t n, double* __restrict__ f64,
                                                         int32_t* __restrict__ i32, StepIO io) {
  __shared__ double sA[4][kSplitEnvs], sSt[4][kSplitEnvs], sDvm[4][kSplitEnvs], sX[4][kSplitEnvs];
  __shared__ int sOn[4][kSplitEnvs];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * kSplitEnvs + lane;
  const bool live = w == 0 && i < n;
  Lane L;
  DzCtx z;
  int rc = 0;
  double fin = 0.0, fin_ret = 0.0, rew_acc = 0.0, cap = 0.0;
  if (w == 0) {
    bool on[2] = {false, false};
    if (live) {
      step_begin<RK45>(prm, n, f64, i32, io, i, AUTORESET, L);
      if (L.err) atomicCAS(io.err, 0, L.err);
      cap = L.cap;
      if (!L.terminal) {
        rc = lane_setup(prm, L, z);                                      // :150, :317-332
        if (rc == 0) { on[0] = z.q[0].ok; on[1] = z.q[1].ok; }
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = q >> 1, kk = q & 1;
      sOn[q][lane] = on[c] ? 1 : 0;
      if (on[c]) {
        sA[q][lane] = z.q[c].A[kk];
        sSt[q][lane] = z.q[c].st;
        sDvm[q][lane] = z.q[c].dvm;
        sX[q][lane] = z.q[c].ag[kk];
      }
    }
  }
  __syncthreads();
  if (sOn[w][lane]) sX[w][lane] = hybrd1(sA[w][lane], sSt[w][lane], sDvm[w][lane], sX[w][lane]);
  __syncthreads();
  if (live) {
    if (!L.terminal) {
      int cnt = 0;
      if (rc) {
        atomicCAS(io.err, 0, rc);
      } else {
        double al[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) al[q] = sOn[q][lane] ? sX[q][lane] : z.q[q >> 1].ag[q & 1];
        cnt = dz_finish(z, al);
      }
      step_reward(prm, L, cnt);
    }
    step_end(prm, n, f64, i32, io, i, AUTORESET, L, fin, fin_ret, rew_acc);
  }
  if (w == 0 && io.stats) wave_stats(io.stats, fin, fin_ret, rew_acc, cap);
}

// 64 envs per 4-wave workgroup with the whole per-env chain spread over the
// waves, not only the four solves (step_kernel_split keeps the rest of the
// chain in wave 0).  Between barriers, per env:
//   I   wave 0: step_begin (state, actions, fuel, propagation, terminal tests)
//   II  wave 0: chaser elements | wave 1: target elements | wave 2: the
//       count-independent reward terms (three cosine similarities, pv4)
//   II' wave 0 also: the chaser's set-up (dz_pursuer) for both waves of III
//   III wave 0: latitudinal angles, rf_setup('orbit_c1') | wave 1: the same
//       angles, rf_setup('orbit_c2') | wave 2: the angles, the target radii
//   IV  wave w: fsolve problem w (rf_extreme_point w>>1, guess w&1) and the
//       rf value of its solution
//   V   wave 0: sort, count, reward, outputs, autoreset, state write-back
// Every value is computed by the functions dz_setup / dz_finish /
// step_reward are composed of, in the same order, so the kernel is
// bit-identical to step_kernel_split (and to the host build where the libm
// agrees); only the schedule differs.  Phases II-IV each shorten wave 0's
// dependent FP64 chain (OCML acos/atan/sincos latency) by running next to it.
template <int E>
struct WideSmem {
  double k[12][E];          // state after the propagation
  float pa[3][E];
  int live[E];              // bit 0: count needed (non-terminal), bit 1: pursuer frozen (p_zero)
  double fuel[E];
  int fcm[E];
  double C[6][E], T[6][E];
  int rc[2][E];
  double rt[4][E];          // reward terms
  double P[9][E];                    // the chaser's Pursuer set-up (dz_pursuer), from phase II
  double qA[4][E], qAg[4][E], qSt[2][E], qCt[2][E], qDvm[2][E],
      qVx0[2][E], qVy0[2][E];
  int qOk[2][E];
  double rft[2][E];
  double rf[4][E];
};

template <int E>
__device__ __forceinline__ void put_elements(double (*dst)[E], int lane, const Elements& el) {
  dst[0][lane] = el.a; dst[1][lane] = el.e; dst[2][lane] = el.i;
  dst[3][lane] = el.omega; dst[4][lane] = el.Omega; dst[5][lane] = el.f;
}
template <int E>
__device__ __forceinline__ Elements get_elements(const double (*src)[E], int lane) {
  Elements el;
  el.a = src[0][lane]; el.e = src[1][lane]; el.i = src[2][lane];
  el.omega = src[3][lane]; el.Omega = src[4][lane]; el.f = src[5][lane];
  return el;
}

// ENVS envs per workgroup (lanes >= ENVS of each wave idle): fewer envs per
// wave put more waves, i.e. more independent dependency chains, on each SIMD
// when N is small (the step is latency bound there); 64 at large N
template <bool AUTORESET, int ENVS, bool SPAN = false>
__global__ void __launch_bounds__(256) step_kernel_wide(const Params prm, int64_t n, double* __restrict__ f64,
                                                        int32_t* __restrict__ i32, StepIO io,
                                                        unsigned long long* __restrict__ span) {
  const unsigned long long span_t0 = SPAN ? satrl_span::now() : 0ull;   // (SPAN: span_probe.h)
  __shared__ WideSmem<ENVS> sm;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const bool env_lane = lane < ENVS;
  const int64_t i = (int64_t)blockIdx.x * ENVS + lane;
  const bool in_range = env_lane && i < n;
  Lane L;
  double fin = 0.0, fin_ret = 0.0, rew_acc = 0.0, cap = 0.0;
  ENV_PROBE(0);
  // ---- I -------------------------------------------------------------------
  if (w == 0) {
    int live = 0;
    if (in_range) {
      step_begin(prm, n, f64, i32, io, i, AUTORESET, L);
      if (L.err) atomicCAS(io.err, 0, L.err);
      cap = L.cap;
      live = L.terminal ? 0 : (1 | (L.p_zero ? 2 : 0));
#pragma unroll
      for (int c = 0; c < 12; ++c) sm.k[c][lane] = L.k[c];
#pragma unroll
      for (int c = 0; c < 3; ++c) sm.pa[c][lane] = L.pa[c];
      sm.fuel[lane] = L.fuel_c;
      sm.fcm[lane] = L.fcm;
    }
    if (env_lane) sm.live[lane] = live;
  }
  ENV_PROBE(1);
  __syncthreads();
  const int live = env_lane ? sm.live[lane] : 0;
  // ---- II ------------------------------------------------------------------
  if (live & 1) {
    if (w <= 1) {
      Elements E;
      const int o = 6 * w;                                    // chaser: Pp/Pv, target: Ep/Ev
      const int rc = dz_elements(prm, sm.k[o][lane], sm.k[o + 1][lane], sm.k[o + 2][lane], sm.k[o + 3][lane],
                                 sm.k[o + 4][lane], sm.k[o + 5][lane], E);
      put_elements<ENVS>(w == 0 ? sm.C : sm.T, lane, E);
      sm.rc[w][lane] = rc;
      if (w == 0 && rc == 0) {                                  // the chaser's set-up, off phase III's path
        Pursuer P;
        dz_pursuer(E, sm.fuel[lane], sm.fcm[lane], P);
        sm.P[0][lane] = P.u; sm.P[1][lane] = P.dv2; sm.P[2][lane] = P.e; sm.P[3][lane] = P.f0;
        sm.P[4][lane] = P.p; sm.P[5][lane] = P.r; sm.P[6][lane] = P.sf0; sm.P[7][lane] = P.X;
        sm.P[8][lane] = P.sq;
      }
    } else if (w == 2) {
      double k[12], t[4];
      float pa[3];
#pragma unroll
      for (int c = 0; c < 12; ++c) k[c] = sm.k[c][lane];
#pragma unroll
      for (int c = 0; c < 3; ++c) pa[c] = sm.pa[c][lane];
      reward_terms(k, pa, (live & 2) != 0, t);
#pragma unroll
      for (int c = 0; c < 4; ++c) sm.rt[c][lane] = t[c];
    }
  }
  ENV_PROBE(2);
  __syncthreads();
  // ---- III -----------------------------------------------------------------
  const bool ok_el = (live & 1) && sm.rc[0][lane] == 0 && sm.rc[1][lane] == 0;
  if (ok_el && w <= 2) {
    const Elements C = get_elements<ENVS>(sm.C, lane), T = get_elements<ENVS>(sm.T, lane);
    double u_c1, u_c2, u_t1, u_t2;
    dz_lat(C, T, u_c1, u_c2, u_t1, u_t2);
    if (w <= 1) {
      Pursuer P;
      P.u = sm.P[0][lane]; P.dv2 = sm.P[1][lane]; P.e = sm.P[2][lane]; P.f0 = sm.P[3][lane];
      P.p = sm.P[4][lane]; P.r = sm.P[5][lane]; P.sf0 = sm.P[6][lane]; P.X = sm.P[7][lane];
      P.sq = sm.P[8][lane];
      RfSolve q;
      rf_setup(P, (w == 0 ? u_c1 : u_c2) - C.omega, q);         // rf_extreme_point('orbit_c1' / 'orbit_c2')
      sm.qOk[w][lane] = q.ok ? 1 : 0;
      sm.qA[2 * w][lane] = q.A[0]; sm.qA[2 * w + 1][lane] = q.A[1];
      sm.qAg[2 * w][lane] = q.ag[0]; sm.qAg[2 * w + 1][lane] = q.ag[1];
      sm.qSt[w][lane] = q.st; sm.qCt[w][lane] = q.ct; sm.qDvm[w][lane] = q.dvm;
      sm.qVx0[w][lane] = q.vx0; sm.qVy0[w][lane] = q.vy0;
    } else {
      double r1, r2;
      dz_target_radii(T, u_t1, u_t2, r1, r2);
      sm.rft[0][lane] = r1; sm.rft[1][lane] = r2;
    }
  }
  ENV_PROBE(3);
  __syncthreads();
  // ---- IV: problem w = (rf_extreme_point c = w >> 1, guess k = w & 1) ------
  if (ok_el) {
    const int c = w >> 1;
    if (sm.qOk[c][lane]) {
      RfSolve q;
      q.ok = true;
      q.st = sm.qSt[c][lane]; q.ct = sm.qCt[c][lane]; q.dvm = sm.qDvm[c][lane];
      q.vx0 = sm.qVx0[c][lane]; q.vy0 = sm.qVy0[c][lane];
      const double al = hybrd1(sm.qA[w][lane], q.st, q.dvm, sm.qAg[w][lane]);
      Pursuer P;
      P.u = kDzMu;
      P.r = sm.P[5][lane];
      sm.rf[w][lane] = rf_one(P, q, al);
    }
  }
  ENV_PROBE(4);
  __syncthreads();
  ENV_PROBE(5);
  // ---- V -------------------------------------------------------------------
  if (w == 0 && in_range) {
    if (!L.terminal) {
      int cnt = 0;
      const int rc = sm.rc[0][lane] ? sm.rc[0][lane] : sm.rc[1][lane];
      if (rc) {
        atomicCAS(io.err, 0, rc);
      } else {
        double mx1, mn1, mx2, mn2;
        rf_sort(sm.qOk[0][lane] != 0, sm.rf[0][lane], sm.rf[1][lane], mx1, mn1);
        rf_sort(sm.qOk[1][lane] != 0, sm.rf[2][lane], sm.rf[3][lane], mx2, mn2);
        cnt = dz_count(mx1, mn1, mx2, mn2, sm.rft[0][lane], sm.rft[1][lane]);
      }
      double t[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) t[c] = sm.rt[c][lane];
      step_reward_terms(prm, L, cnt, t);
    }
    step_end(prm, n, f64, i32, io, i, AUTORESET, L, fin, fin_ret, rew_acc);
  }
  if (w == 0 && io.stats) wave_stats(io.stats, fin, fin_ret, rew_acc, cap);
  ENV_PROBE(6);
  if constexpr (SPAN) satrl_span::exit(span, span_t0);
}

__global__ void __launch_bounds__(256) reset_kernel(const Params prm, int64_t n, double* __restrict__ f64,
                                                    int32_t* __restrict__ i32, int32_t flag, const uint8_t* mask,
                                                    float* obs, double* obs64) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double k[12];
  const bool hit = mask == nullptr || mask[i] != 0;
  if (hit) {                                                                // environment.py:66-79
    reset_kin(prm, k);
#pragma unroll
    for (int c = 0; c < 12; ++c) f64[c * n + i] = k[c];
    const int b = i32[kPlaneBits * n + i];
    i32[kPlaneBits * n + i] = make_bits(fc_mode(b), ft_mode(b), 1, flag);
    i32[kPlaneCount * n + i] = 0;
    f64[kPlaneRet * n + i] = 0.0;
  } else {
#pragma unroll
    for (int c = 0; c < 12; ++c) k[c] = f64[c * n + i];
  }
  write_obs(obs, obs64, i, k);
}

__global__ void init_kernel(const Params prm, int64_t n, double* f64, int32_t* i32) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
#pragma unroll
  for (int c = 0; c < 12; ++c) f64[c * n + i] = prm.init_kin[c];           // environment.py:30-33
  f64[12 * n + i] = prm.fuel_c0;                                            // :42-43
  f64[13 * n + i] = prm.fuel_t0;
  f64[14 * n + i] = INFINITY;                                               // :44
  f64[kPlaneRet * n + i] = 0.0;
  i32[kPlaneDz * n + i] = 0;                                                // :41
  i32[kPlaneCount * n + i] = 0;
  i32[kPlaneBits * n + i] = make_bits(prm.fuel_c0_mode, prm.fuel_t0_mode, 1, prm.flag);
}

__global__ void __launch_bounds__(256) danger_zone_kernel(int64_t n, const double* __restrict__ X,
                                                          const double* __restrict__ fuel,
                                                          const int32_t* __restrict__ mode, int32_t* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  satenv_params prm;
  for (int c = 0; c < 3; ++c) { prm.R_cw[c] = 0.0; prm.V_cw[c] = 0.0; }   // states are already absolute
  const double* x = X + i * 12;
  int cnt = 0;
  const int rc = danger_zone(prm, x[0], x[1], x[2], x[3], x[4], x[5], x[6], x[7], x[8], x[9], x[10], x[11],
                             fuel[i], mode[i], cnt);
  out[i] = rc ? rc : cnt;
}

__global__ void __launch_bounds__(256) solve_alpha_kernel(int64_t n, const double* __restrict__ in,
                                                          double* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double* x = in + i * 6;   // Delta_Vm, theta, v_1x, v_1y, h, alpha_guess
  const double u = 3.986e14, dvm = x[0], theta = x[1], v1x = x[2], v1y = x[3], h = x[4];
  const double A = (2.0 * u * (1.0 - cos(theta))) / (h * v1y) - v1x * sin(theta) / v1y;
  out[i] = hybrd1(A, sin(theta), dvm, x[5]);
}

__global__ void __launch_bounds__(256) sincos_kernel(int64_t n, const double* __restrict__ x, double* __restrict__ so,
                                                     double* __restrict__ co, int32_t use_library) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double s, c;
  if (use_library) sincos(x[i], &s, &c);
  else sincos_fast(x[i], s, c);
  so[i] = s;
  co[i] = c;
}

__global__ void __launch_bounds__(256) acos_kernel(int64_t n, const double* __restrict__ x, double* __restrict__ out,
                                                   int32_t use_library) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = use_library ? acos(x[i]) : acos_sl(x[i]);
}

// batched RK4 two-body + J2 propagation (轨道外推-龙格库塔算法.py), SoA [6][n]
__global__ void __launch_bounds__(256) rk4_j2_kernel(int64_t n, const double* __restrict__ in, double h,
                                                     int32_t steps, double* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double s[6];
#pragma unroll
  for (int c = 0; c < 6; ++c) s[c] = in[c * n + i];
  for (int32_t k = 0; k < steps; ++k) {
    double o[6];
    rk4_step(j2_rhs, s, h, o);
#pragma unroll
    for (int c = 0; c < 6; ++c) s[c] = o[c];
  }
#pragma unroll
  for (int c = 0; c < 6; ++c) out[c * n + i] = s[c];
}

// ---------------------------------------------------------------------------
// single_pluse_model/RD_single_pulse.py:40-148 Reachable_Domain, batched over
// orbits.  Direction d = ((jj-1)*(N2+1) + i)*(N3+1) + j.  Only a few percent
// of the directions pass the reachability test (:81), so a workgroup first
// classifies kRdTile directions (cheap: one sin, one tan), compacts the
// reachable ones into an LDS list and then runs the two hybrd solves over
// the list with packed lanes instead of one mostly-idle lane per direction.
// ---------------------------------------------------------------------------
constexpr int kRdBlock = 256, kRdPer = 4, kRdTile = kRdBlock * kRdPer;

struct RdDir { double dV2, gama, alpha, g; };

__device__ __forceinline__ RdDir rd_dir(const satenv_rd_orbit& o, int n1, int n2, int n3, int d) {
  const int per = (n2 + 1) * (n3 + 1);
  const int jj = d / per + 1, rem = d - (jj - 1) * per;
  const int i = rem / (n3 + 1), j = rem - i * (n3 + 1);
  RdDir r;
  if (o.dv_f32 != 0.0) {                                            // np.float32 delta_max: f32 ops
    const float d = (float)o.delta_max;
    const float dV = -d + ((2.0f * d) * (float)jj) / (float)n1;      // :64
    r.dV2 = (double)(dV * dV);                                      // Delta_V ** 2 (float32 square)
  } else {
    const double dV = -o.delta_max + (2.0 * o.delta_max * jj) / n1;   // :64
    r.dV2 = dV * dV;
  }
  r.gama = (kTwoPi * i) / n2;                                       // :66
  r.alpha = -kPi / 2 + (kPi * j) / n3;                              // :68
  r.g = r.gama - o.f;
  return r;
}

__device__ __forceinline__ double rd_X(const satenv_rd_orbit& o) { return 1.0 + o.e0 * cos(o.f); }

// 0 unreachable, 1 reachable, 2 reachable but gama - f outside both theta branches (:87-90)
__device__ __forceinline__ int rd_status(const satenv_rd_orbit& o, double p0, double X, const RdDir& r) {
  const double sg = sin(r.g);
  const double temp1 = (sg * sg) / (o.mu * (X * X) / (p0 * r.dV2) - 1.0);   // :79
  const double ta = tan(r.alpha);
  if (!(0.0 <= ta * ta && ta * ta <= temp1)) return 0;                        // :81
  const double g = r.g;
  if ((-kTwoPi <= g && g < -kPi) || (0.0 <= g && g < kPi)) return 1;
  if ((-kPi <= g && g < 0.0) || (kPi <= g && g < kTwoPi)) return 1;
  return 2;
}

__global__ void __launch_bounds__(kRdBlock) rd_kernel(const satenv_rd_orbit* __restrict__ orbits, int32_t n1,
                                                      int32_t n2, int32_t n3, int32_t ndir, int32_t tiles,
                                                      double* __restrict__ rf_max, double* __restrict__ rf_min,
                                                      uint8_t* __restrict__ status) {
  __shared__ int list[kRdTile];
  __shared__ int cnt;
  const int64_t set = blockIdx.x / tiles;
  const int d0 = (int)(blockIdx.x - set * tiles) * kRdTile;
  const satenv_rd_orbit o = orbits[set];
  const double X = rd_X(o);
  const double p0 = o.a * (1.0 - o.e0 * o.e0);                    // :48
  const double r0 = p0 / X;                                       // :47
  const double sq = sqrt(o.mu / p0);
  const double vx0 = sq * o.e0 * sin(o.f);                        // :95
  const int64_t base = set * (int64_t)ndir;
  if (threadIdx.x == 0) cnt = 0;
  __syncthreads();
#pragma unroll
  for (int q = 0; q < kRdPer; ++q) {
    const int d = d0 + q * kRdBlock + (int)threadIdx.x;
    if (d < ndir) {
      const int st = rd_status(o, p0, X, rd_dir(o, n1, n2, n3, d));
      status[base + d] = (uint8_t)st;
      if (st == 1) list[atomicAdd(&cnt, 1)] = d;
    }
  }
  __syncthreads();
  const int m = cnt;
  for (int k = (int)threadIdx.x; k < m; k += kRdBlock) {
    const int d = list[k];
    const RdDir r = rd_dir(o, n1, n2, n3, d);
    const double sg = sin(r.g);
    const double ta = tan(r.alpha);
    const double beta = atan(ta / sg);                                          // :82
    double sb, cb;
    sincos(beta, &sb, &cb);
    const double dvm = sqrt(r.dV2 - o.mu * (X * X) * (sb * sb) / p0);         // :84
    const double ca = cos(r.alpha);
    const double ac = acos(cos(r.g) * ca);
    const double theta = ((-kTwoPi <= r.g && r.g < -kPi) || (0.0 <= r.g && r.g < kPi)) ? ac : kTwoPi - ac;   // :87-90
    double st, ct;
    sincos(theta, &st, &ct);
    const double vy0 = sq * X * cb;                                             // :96
    double rf[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const double ag = s == 0 ? kPi / 2 : -kPi / 2;                           // :93, :109
      const double sgs = s == 0 ? kSinHalfPi : -kSinHalfPi, cgs = kCosHalfPi;   // sincos(ag)
      const double v1x = vx0 + dvm * cgs, v1y = vy0 + dvm * sgs;
      const double h = r0 * v1y;                                                // :98
      const double A = (2.0 * o.mu * (1.0 - ct)) / (h * v1y) - v1x * st / v1y; // :152
      const double al = hybrd1(A, st, dvm, ag);                                 // :150-157
      double sa, cal;
      sincos(al, &sa, &cal);
      const double vx = vx0 + dvm * cal, vy = vy0 + dvm * sa;                   // :102-104
      const double hm = r0 * vy;
      rf[s] = (hm * hm) / (o.mu * (1.0 - ct) + hm * vy * ct - hm * vx * st);   // :106, :121
    }
    const double a0 = fabs(rf[0]), a1 = fabs(rf[1]);
    const double mx = (a1 > a0) ? a1 : a0;                                      // builtin max, :123
    const double mn = (a1 < a0) ? a1 : a0;                                      // builtin min, :124
    double sgm, cgm;
    sincos(r.gama, &sgm, &cgm);
    const double P[3] = {sgm * ca, cgm * ca, sin(r.alpha)};                     // :71
    double* omx = rf_max + 3 * (base + d);
    double* omn = rf_min + 3 * (base + d);
#pragma unroll
    for (int c = 0; c < 3; ++c) { omx[c] = mx * P[c]; omn[c] = mn * P[c]; }
  }
}

// Flag 2: the Incoming_parameters orbit of every env (include/satenv.h
// satenv_rd_orbits): real_time_data_process.calculate_orbital_elements
// (:11-105, the same element set as satellite_function's, orbital_elements)
// of the pursuer's absolute state, delta_max = fuel_c with its numpy type
__global__ void __launch_bounds__(256) rd_orbits_kernel(const Params prm, int64_t n, const double* __restrict__ f64,
                                                        const int32_t* __restrict__ i32,
                                                        satenv_rd_orbit* __restrict__ out,
                                                        int32_t* __restrict__ status) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Elements E;
  const int rc = orbital_elements(3.986e14, prm.R_cw[0] + f64[0 * n + i], prm.R_cw[1] + f64[1 * n + i],
                                  prm.R_cw[2] + f64[2 * n + i], prm.V_cw[0] + f64[3 * n + i],
                                  prm.V_cw[1] + f64[4 * n + i], prm.V_cw[2] + f64[5 * n + i], E);
  satenv_rd_orbit o;
  o.a = rc ? 0.0 : E.a;                                            // Incoming_parameters :29-33
  o.e0 = rc ? 0.0 : E.e;
  o.f = rc ? 0.0 : E.f;
  o.delta_max = f64[12 * n + i];
  o.mu = 3.986e14;                                                 // RD_single_pulse params['u']
  o.dv_f32 = fc_mode(i32[kPlaneBits * n + i]) == kF32 ? 1.0 : 0.0;
  out[i] = o;
  status[i] = rc;
}

// ---------------------------------------------------------------------------
// config 5: ImprovedNN surrogate (bf16 MFMA) on the pursuer's current orbit,
// network_method_process real_time_data_process.py:112-125.  x == nullptr:
// features from the env state (relative_state_to_absolute_state
// environment.py:334-343 -> calculate_orbital_elements :11-105 -> [a, e, i, f,
// fuel_c] as float32); else x [n][5] f32 directly.  Envs whose orbit has no
// 6-element set (e == 0 / parabolic: the reference builds a 4-feature input
// and crashes) get NaN outputs.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(surrogate::kThreads) surrogate_kernel(const Params prm, int64_t n,
                                                                        const double* __restrict__ f64,
                                                                        const float* __restrict__ x,
                                                                        const uint8_t* __restrict__ blob,
                                                                        float* __restrict__ out) {
  using namespace surrogate;
  __shared__ __align__(16) uint8_t lds[kBlobBytes];
  {
    const uint4* src = reinterpret_cast<const uint4*>(blob);
    uint4* dst = reinterpret_cast<uint4*>(lds);
    for (int i = threadIdx.x; i < kBlobBytes / 16; i += kThreads) dst[i] = src[i];
  }
  __syncthreads();
  const unsigned short* W = reinterpret_cast<const unsigned short*>(lds);
  const float* Bs = reinterpret_cast<const float*>(lds + kBiasOffBytes);
  const Scalers& SC = *reinterpret_cast<const Scalers*>(lds + kScaleOffBytes);
  const int wave = threadIdx.x >> 6, l = threadIdx.x & 63, g = l >> 4, c = l & 15;
  for (int64_t tile = (int64_t)blockIdx.x * 4 + wave; tile * 16 < n; tile += (int64_t)gridDim.x * 4) {
    const int64_t env = tile * 16 + c;
    const bool valid = env < n;
    frag_ab in1[1];
#pragma unroll
    for (int k = 0; k < 8; ++k) in1[0][k] = 0;
    int ok = 0;
    if (g == 0 && valid) {
      double fv[kIn];
      if (x) {
#pragma unroll
        for (int k = 0; k < kIn; ++k) fv[k] = x[env * kIn + k];
        ok = 1;
      } else {
        Elements E;
        const int rc = orbital_elements(3.986e14, prm.R_cw[0] + f64[0 * n + env], prm.R_cw[1] + f64[1 * n + env],
                                        prm.R_cw[2] + f64[2 * n + env], prm.V_cw[0] + f64[3 * n + env],
                                        prm.V_cw[1] + f64[4 * n + env], prm.V_cw[2] + f64[5 * n + env], E);
        ok = rc == 0;
        // the reference's float32 feature tensor (real_time_data_process.py:117)
        fv[0] = (float)E.a; fv[1] = (float)E.e; fv[2] = (float)E.i; fv[3] = (float)E.f;
        fv[4] = (float)f64[12 * n + env];
      }
#pragma unroll
      for (int k = 0; k < kIn; ++k) in1[0][k] = (short)f2bf((float)((fv[k] - SC.in_mean[k]) / SC.in_scale[k]));
    }
    ok = __shfl(ok, c, 64);
    frag_ab h1[8], h2[4], h3[2];
    layer<16, 1, kW1Row>(W + kW1Off, Bs, in1, h1);
    layer<8, 8, kW2Row>(W + kW2Off, Bs + kH1, h1, h2);
    layer<4, 4, kW3Row>(W + kW3Off, Bs + kH1 + kH2, h2, h3);
    frag_cd acc = {0.0f, 0.0f, 0.0f, 0.0f};
    const unsigned short* row = W + kW4Off + c * kW4Row + 8 * g;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(lds_frag(row + 32 * s2), h3[s2], acc, 0, 0, 0);
    if (valid) {
      const float* b4 = Bs + kH1 + kH2 + kH3;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int o = 4 * g + i;
        if (o < kOut)
          out[env * kOut + o] = ok ? (float)((double)(acc[i] + b4[o]) * SC.out_scale[o] + SC.out_mean[o])
                                   : __uint_as_float(0x7fc00000u);
      }
    }
  }
}

int surrogate_grid(int64_t n) {
  const int64_t tiles = (n + 63) / 64;
  return (int)(tiles < 1024 ? tiles : 1024);
}

}  // namespace

struct satenv_env {
  int64_t n = 0;
  int device = 0;
  satenv_params prm{};
  double* f64 = nullptr;
  int32_t* i32 = nullptr;
  int32_t* err = nullptr;
  int split = 2;   // step_kernel_wide (2), step_kernel_split (1) or the one-lane step_kernel (0)
  int wide_envs = 64;
};

namespace {

int grid_for(int64_t n, int block) { return (int)((n + block - 1) / block); }

// envs per workgroup of the wide kernel: 64 (satenv_set_step_kernel: 16 / 32
// for A/B; fewer envs per workgroup measured no faster)
int wide_envs(const satenv_env* h) { return h->wide_envs; }

template <bool AR>
void launch_step(satenv_env* h, const StepIO& io, void* stream) {
  const dim3 grid(grid_for(h->n, kSplitEnvs));
  if (h->prm.propagator == 2)   // the RK45 instantiation (its registers stay out of the STM kernels)
    hipLaunchKernelGGL((step_kernel_split<AR, true>), grid, dim3(256), 0, (hipStream_t)stream, h->prm, h->n, h->f64,
                       h->i32, io);
  else if (h->split == 2) {
    const int envs = wide_envs(h);
    const dim3 gw(grid_for(h->n, envs));
    // the product geometry (64 envs per workgroup) has a SPAN instantiation
    // for the bench's live launch spans (span_probe.h)
    unsigned long long* sp = envs == 64 ? satrl_span::take(satrl_span::kEnvStep, (int64_t)gw.x * 4) : nullptr;
    if (envs == 16)
      hipLaunchKernelGGL((step_kernel_wide<AR, 16>), gw, dim3(256), 0, (hipStream_t)stream, h->prm, h->n, h->f64,
                         h->i32, io, nullptr);
    else if (envs == 32)
      hipLaunchKernelGGL((step_kernel_wide<AR, 32>), gw, dim3(256), 0, (hipStream_t)stream, h->prm, h->n, h->f64,
                         h->i32, io, nullptr);
    else if (sp)
      hipLaunchKernelGGL((step_kernel_wide<AR, 64, true>), gw, dim3(256), 0, (hipStream_t)stream, h->prm, h->n,
                         h->f64, h->i32, io, sp);
    else
      hipLaunchKernelGGL((step_kernel_wide<AR, 64>), gw, dim3(256), 0, (hipStream_t)stream, h->prm, h->n, h->f64,
                         h->i32, io, nullptr);
  }
  else if (h->split == 1)
    hipLaunchKernelGGL(step_kernel_split<AR>, grid, dim3(256), 0, (hipStream_t)stream, h->prm, h->n, h->f64, h->i32,
                       io);
  else
    hipLaunchKernelGGL(step_kernel<AR>, dim3(grid_for(h->n, 64)), dim3(64), 0, (hipStream_t)stream, h->prm, h->n,
                       h->f64, h->i32, io);
}

}  // namespace

extern "C" {

#ifdef SATENV_PHASE_PROBE
int satenv_probe_read(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_env_probe), sizeof(g_env_probe)) == hipSuccess ? 0 : -1;
}
#endif

const char* satenv_last_error(void) { return g_last_error.c_str(); }
int satenv_abi_version(void) { return SATENV_ABI_VERSION; }

int satenv_stm(double t, double* M) {
  if (!M) return fail(SATENV_ERR_ARG, "satenv_stm: null output");
  // satellite_function.py:753-781; r**3 as the correctly rounded python int -> float
  const double R3 = (double)((__int128)42164000 * 42164000 * 42164000);
  const double omega = std::sqrt(3.986e14 / R3);
  const double tau = omega * t, s = std::sin(tau), c = std::cos(tau);
  const double m[36] = {4 - 3 * c, 0, 0, s / omega, 2 * (1 - c) / omega, 0,
                        6 * (s - tau), 1, 0, -2 * (1 - c) / omega, 4 * s / omega - 3 * tau, 0,
                        0, 0, c, 0, 0, s / omega,
                        3 * omega * s, 0, 0, c, 2 * s, 0,
                        6 * omega * (c - 1), 0, 0, -2 * s, 4 * c - 3, 0,
                        0, 0, -omega * s, 0, 0, c};
  std::memcpy(M, m, sizeof(m));
  return SATENV_OK;
}

int satenv_default_params(satenv_params* p) {
  if (!p) return fail(SATENV_ERR_ARG, "satenv_default_params: null");
  std::memset(p, 0, sizeof(*p));
  p->d_capture = 100000;   // environment.py:28 ctor default (train_* overwrite it)
  p->d_range = 100000;
  p->win_reward = 100;
  p->burn_reward = 0;
  p->mu = 3.986e14;
  p->R_cw[0] = 27098000; p->R_cw[1] = 32306000; p->R_cw[2] = 0;
  p->V_cw[0] = -2350; p->V_cw[1] = 1970; p->V_cw[2] = 0;
  satenv_stm(100.0, p->stm);
  p->fuel_c0 = 320; p->fuel_t0 = 320;
  p->fuel_c0_mode = SATENV_NUM_PYINT; p->fuel_t0_mode = SATENV_NUM_PYINT;
  const double kin[12] = {2000, 2000, 1000, 1.71, 1.14, 1.3, 1000, 2000, 0, 1.71, 1.14, 1.3};   // :26-27
  std::memcpy(p->init_kin, kin, sizeof(kin));
  p->max_episode_steps = 1000;   // CPPO_main.py:28
  p->flag = 0;
  // mean motion exactly as State_transition_matrix computes it (satellite_function.py:758-761):
  // r ** 3 is an exact python int, rounded once when it meets the float mu
  p->cw_omega = std::sqrt(3.986e14 / (double)((__int128)42164000 * 42164000 * 42164000));
  p->propagator = 0;
  p->rk4_substeps = 10;
  return SATENV_OK;
}

int satenv_set_step_kernel(satenv_env* h, int32_t kind, int32_t wide_envs) {
  if (!h || kind < 0 || kind > 2 || (wide_envs != 16 && wide_envs != 32 && wide_envs != 64))
    return fail(SATENV_ERR_ARG, "satenv_set_step_kernel: kind 0/1/2, wide_envs 16/32/64");
  h->split = kind;
  h->wide_envs = wide_envs;
  return SATENV_OK;
}

int satenv_create(satenv_env** out, int64_t num_envs, const satenv_params* p, int device) {
  if (!out || !p || num_envs <= 0) return fail(SATENV_ERR_ARG, "satenv_create: bad arguments");
  if (!params_ok(p)) return fail(SATENV_ERR_ARG, "satenv_create: propagator must be 0/1/2, rk4_substeps >= 1");
  HIP_TRY(hipSetDevice(device));
  satenv_env* h = new satenv_env();
  h->n = num_envs;
  h->device = device;
  h->prm = *p;
  hipError_t e = hipMalloc(&h->f64, sizeof(double) * kF64Planes * num_envs);
  if (e == hipSuccess) e = hipMalloc(&h->i32, sizeof(int32_t) * kI32Planes * num_envs);
  if (e == hipSuccess) e = hipMalloc(&h->err, sizeof(int32_t));
  if (e == hipSuccess) e = hipMemset(h->err, 0, sizeof(int32_t));
  if (e != hipSuccess) {
    satenv_destroy(h);
    return fail(SATENV_ERR_HIP, std::string("satenv_create: ") + hipGetErrorString(e));
  }
  hipLaunchKernelGGL(init_kernel, dim3(grid_for(num_envs, 256)), dim3(256), 0, nullptr, h->prm, h->n, h->f64,
                     h->i32);
  e = hipGetLastError();
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    satenv_destroy(h);
    return fail(SATENV_ERR_HIP, std::string("satenv_create init: ") + hipGetErrorString(e));
  }
  *out = h;
  return SATENV_OK;
}

int satenv_destroy(satenv_env* h) {
  if (!h) return SATENV_OK;
  if (h->f64) (void)hipFree(h->f64);
  if (h->i32) (void)hipFree(h->i32);
  if (h->err) (void)hipFree(h->err);
  delete h;
  return SATENV_OK;
}

int satenv_num_envs(const satenv_env* h, int64_t* n) {
  if (!h || !n) return fail(SATENV_ERR_ARG, "satenv_num_envs: null");
  *n = h->n;
  return SATENV_OK;
}

int satenv_set_params(satenv_env* h, const satenv_params* p) {
  if (!h || !p) return fail(SATENV_ERR_ARG, "satenv_set_params: null");
  if (!params_ok(p)) return fail(SATENV_ERR_ARG, "satenv_set_params: propagator must be 0/1/2, rk4_substeps >= 1");
  h->prm = *p;
  return SATENV_OK;
}

int satenv_reset(satenv_env* h, int32_t flag, const uint8_t* env_mask, float* obs_out, double* obs64_out,
                 void* stream) {
  if (!h) return fail(SATENV_ERR_ARG, "satenv_reset: null handle");
  if (flag < 0 || flag > 2) return fail(SATENV_ERR_ARG, "satenv_reset: Flag must be 0, 1 or 2");
  h->prm.flag = flag;
  hipLaunchKernelGGL(reset_kernel, dim3(grid_for(h->n, 256)), dim3(256), 0, (hipStream_t)stream, h->prm, h->n,
                     h->f64, h->i32, flag, env_mask, obs_out, obs64_out);
  HIP_TRY(hipGetLastError());
  return SATENV_OK;
}

int satenv_step(satenv_env* h, const float* pa, const float* ea, const int32_t* episode_count, float* obs_out,
                double* obs64_out, double* reward_out, uint8_t* done_out, void* stream) {
  if (!h || !pa || !ea) return fail(SATENV_ERR_ARG, "satenv_step: null argument");
  StepIO io{pa, ea, episode_count, obs_out, obs64_out, reward_out, nullptr, done_out, nullptr, h->err};
  launch_step<false>(h, io, stream);
  HIP_TRY(hipGetLastError());
  return SATENV_OK;
}

int satenv_step_autoreset(satenv_env* h, const float* pa, const float* ea, float* obs_out, float* reward_out,
                          uint8_t* done_out, double* stats_out, void* stream) {
  if (!h || !pa || !ea) return fail(SATENV_ERR_ARG, "satenv_step_autoreset: null argument");
  StepIO io{pa, ea, nullptr, obs_out, nullptr, nullptr, reward_out, done_out, stats_out, h->err};
  launch_step<true>(h, io, stream);
  HIP_TRY(hipGetLastError());
  return SATENV_OK;
}

int satenv_get_state(const satenv_env* h, double* f64_planes, int32_t* i32_planes, void* stream) {
  if (!h) return fail(SATENV_ERR_ARG, "satenv_get_state: null handle");
  if (f64_planes)
    HIP_TRY(hipMemcpyAsync(f64_planes, h->f64, sizeof(double) * SATENV_F64_PLANES * h->n, hipMemcpyDeviceToDevice,
                           (hipStream_t)stream));
  if (i32_planes)
    HIP_TRY(hipMemcpyAsync(i32_planes, h->i32, sizeof(int32_t) * SATENV_I32_PLANES * h->n,
                           hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return SATENV_OK;
}

int satenv_set_state(satenv_env* h, const double* f64_planes, const int32_t* i32_planes, void* stream) {
  if (!h) return fail(SATENV_ERR_ARG, "satenv_set_state: null handle");
  if (f64_planes)
    HIP_TRY(hipMemcpyAsync(h->f64, f64_planes, sizeof(double) * SATENV_F64_PLANES * h->n, hipMemcpyDeviceToDevice,
                           (hipStream_t)stream));
  if (i32_planes)
    HIP_TRY(hipMemcpyAsync(h->i32, i32_planes, sizeof(int32_t) * SATENV_I32_PLANES * h->n,
                           hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return SATENV_OK;
}

int satenv_danger_zone(int64_t n, const double* states, const double* fuel, const int32_t* fuel_mode,
                       int32_t* count_out, void* stream) {
  if (n <= 0 || !states || !fuel || !fuel_mode || !count_out) return fail(SATENV_ERR_ARG, "satenv_danger_zone: bad args");
  hipLaunchKernelGGL(danger_zone_kernel, dim3(grid_for(n, 64)), dim3(64), 0, (hipStream_t)stream, n, states, fuel,
                     fuel_mode, count_out);
  HIP_TRY(hipGetLastError());
  return SATENV_OK;
}

int satenv_solve_alpha(int64_t n, const double* in, double* alpha_out, void* stream) {
  if (n <= 0 || !in || !alpha_out) return fail(SATENV_ERR_ARG, "satenv_solve_alpha: bad args");
  hipLaunchKernelGGL(solve_alpha_kernel, dim3(grid_for(n, 64)), dim3(64), 0, (hipStream_t)stream, n, in, alpha_out);
  HIP_TRY(hipGetLastError());
  return SATENV_OK;
}

int satenv_sincos(int64_t n, const double* x, double* s_out, double* c_out, int32_t use_library, void* stream) {
  if (n <= 0 || !x || !s_out || !c_out) return fail(SATENV_ERR_ARG, "satenv_sincos: bad args");
  hipLaunchKernelGGL(sincos_kernel, dim3(grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream, n, x, s_out, c_out,
                     use_library);
  HIP_TRY(hipGetLastError());
  return SATENV_OK;
}

int satenv_acos(int64_t n, const double* x, double* out, int32_t use_library, void* stream) {
  if (n <= 0 || !x || !out) return fail(SATENV_ERR_ARG, "satenv_acos: bad args");
  hipLaunchKernelGGL(acos_kernel, dim3(grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream, n, x, out, use_library);
  HIP_TRY(hipGetLastError());
  return SATENV_OK;
}

int satenv_rk4_j2(int64_t n, const double* rv_in, double h, int32_t steps, double* rv_out, void* stream) {
  if (n <= 0 || !rv_in || !rv_out || steps < 0) return fail(SATENV_ERR_ARG, "satenv_rk4_j2: bad args");
  hipLaunchKernelGGL(rk4_j2_kernel, dim3(grid_for(n, 64)), dim3(64), 0, (hipStream_t)stream, n, rv_in, h, steps,
                     rv_out);
  HIP_TRY(hipGetLastError());
  return SATENV_OK;
}

int satenv_reachable_domain(int64_t nsets, const satenv_rd_orbit* orbits, int32_t n1, int32_t n2, int32_t n3,
                            double* rf_max, double* rf_min, uint8_t* status, void* stream) {
  if (nsets <= 0 || !orbits || !rf_max || !rf_min || !status || n1 < 1 || n2 < 1 || n3 < 1)
    return fail(SATENV_ERR_ARG, "satenv_reachable_domain: bad args (N1, N2, N3 >= 1)");
  const int64_t ndir = (int64_t)n1 * (n2 + 1) * (n3 + 1);
  const int64_t tiles = (ndir + kRdTile - 1) / kRdTile;
  if (ndir > INT32_MAX || nsets * tiles > INT32_MAX)
    return fail(SATENV_ERR_ARG, "satenv_reachable_domain: grid too large");
  hipLaunchKernelGGL(rd_kernel, dim3((unsigned)(nsets * tiles)), dim3(kRdBlock), 0, (hipStream_t)stream, orbits, n1,
                     n2, n3, (int32_t)ndir, (int32_t)tiles, rf_max, rf_min, status);
  HIP_TRY(hipGetLastError());
  return SATENV_OK;
}

int satenv_rd_orbits(satenv_env* h, satenv_rd_orbit* orbits_out, int32_t* status_out, void* stream) {
  if (!h || !orbits_out || !status_out) return fail(SATENV_ERR_ARG, "satenv_rd_orbits: null argument");
  hipLaunchKernelGGL(rd_orbits_kernel, dim3(grid_for(h->n, 256)), dim3(256), 0, (hipStream_t)stream, h->prm, h->n,
                     h->f64, h->i32, orbits_out, status_out);
  HIP_TRY(hipGetLastError());
  return SATENV_OK;
}

int satenv_ellipse_fit(int64_t nsets, int32_t ndir, const double* rf_max, const double* rf_min, const uint8_t* status,
                       double* ellipse_out, int32_t* info_out, double* fit_points_out, double* center_out,
                       void* stream) {
  if (nsets <= 0 || ndir <= 0 || !rf_max || !rf_min || !status || !ellipse_out || !info_out)
    return fail(SATENV_ERR_ARG, "satenv_ellipse_fit: bad args");
  if (2 * nsets > INT32_MAX) return fail(SATENV_ERR_ARG, "satenv_ellipse_fit: too many sets");
  hipLaunchKernelGGL(ellipse::ellipse_kernel, dim3((unsigned)(2 * nsets)), dim3(ellipse::kThreads), 0,
                     (hipStream_t)stream, ndir, rf_max, rf_min, status, ellipse_out, info_out, fit_points_out,
                     center_out);
  HIP_TRY(hipGetLastError());
  return SATENV_OK;
}

int satenv_surrogate_blob_bytes(void) { return surrogate::kBlobBytes; }

int satenv_surrogate_pack(const float* w1, const float* b1, const float* w2, const float* b2, const float* w3,
                          const float* b3, const float* w4, const float* b4, void* blob, void* stream) {
  if (!w1 || !b1 || !w2 || !b2 || !w3 || !b3 || !w4 || !b4 || !blob)
    return fail(SATENV_ERR_ARG, "satenv_surrogate_pack: null pointer");
  hipLaunchKernelGGL(surrogate::pack_kernel, dim3(64), dim3(256), 0, (hipStream_t)stream, w1, b1, w2, b2, w3, b3, w4,
                     b4, (uint8_t*)blob);
  HIP_TRY(hipGetLastError());
  return SATENV_OK;
}

int satenv_surrogate_set_scalers(void* blob, const double* in_mean, const double* in_scale, const double* out_mean,
                                 const double* out_scale, void* stream) {
  if (!blob || !in_mean || !in_scale || !out_mean || !out_scale)
    return fail(SATENV_ERR_ARG, "satenv_surrogate_set_scalers: null pointer");
  surrogate::Scalers sc{};
  for (int k = 0; k < 8; ++k) {
    sc.in_mean[k] = k < surrogate::kIn ? in_mean[k] : 0.0;
    sc.in_scale[k] = k < surrogate::kIn ? in_scale[k] : 1.0;
  }
  for (int k = 0; k < surrogate::kOutPad; ++k) {
    sc.out_scale[k] = k < surrogate::kOut ? out_scale[k] : 1.0;
    sc.out_mean[k] = k < surrogate::kOut ? out_mean[k] : 0.0;
  }
  for (int k = 0; k < surrogate::kIn; ++k)
    if (!(sc.in_scale[k] != 0.0)) return fail(SATENV_ERR_ARG, "satenv_surrogate_set_scalers: zero input scale");
  hipLaunchKernelGGL(surrogate::set_scalers_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, sc, (uint8_t*)blob);
  return hipGetLastError() == hipSuccess ? 0 : fail(SATENV_ERR_HIP, "satenv_surrogate_set_scalers: launch");
}

int satenv_surrogate(satenv_env* h, const void* blob, float* out, void* stream) {
  if (!h || !blob || !out) return fail(SATENV_ERR_ARG, "satenv_surrogate: null pointer");
  hipLaunchKernelGGL(surrogate_kernel, dim3(surrogate_grid(h->n)), dim3(surrogate::kThreads), 0, (hipStream_t)stream,
                     h->prm, h->n, h->f64, nullptr, (const uint8_t*)blob, out);
  HIP_TRY(hipGetLastError());
  return SATENV_OK;
}

int satenv_surrogate_mlp(int64_t n, const float* x, const void* blob, float* out, void* stream) {
  if (n <= 0 || !x || !blob || !out) return fail(SATENV_ERR_ARG, "satenv_surrogate_mlp: bad args");
  satenv_params prm;
  std::memset(&prm, 0, sizeof(prm));
  hipLaunchKernelGGL(surrogate_kernel, dim3(surrogate_grid(n)), dim3(surrogate::kThreads), 0, (hipStream_t)stream, prm,
                     n, nullptr, x, (const uint8_t*)blob, out);
  HIP_TRY(hipGetLastError());
  return SATENV_OK;
}

int satenv_check(satenv_env* h, int32_t* status) {
  if (!h || !status) return fail(SATENV_ERR_ARG, "satenv_check: null");
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(status, h->err, sizeof(int32_t), hipMemcpyDeviceToHost));
  return SATENV_OK;
}

}  // extern "C"
