// satenv_cpu.cpp -- host build of the environment ABI (include/satenv_cpu.h).
//
// The env step of the gfx950 kernels, compiled by g++ for host cores: the
// same satenv_device.h / satenv_step.h source, one loop iteration per env
// where the kernel has one lane per env, OpenMP over envs.  Same state
// layout as a device handle (f64 planes [16][N], i32 planes [3][N]), so the
// get/set_state planes are interchangeable between the two builds.
//
// Reference (qiaobeibei/PPO-RL-Satellite): environment.py:26-255 (ctor,
// reset, step Flag 0/1), CPPO_main.py:119-153 (the loop step_autoreset
// stands for), satellite_function.py:18-99,161-255,317-373,462-565 (the
// danger-zone count with fsolve's MINPACK hybrd).
#include <omp.h>

#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "satenv_cpu.h"
#include "satenv_device.h"
#include "satenv_step.h"

using namespace satenv;

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

bool params_ok(const satenv_params* p) {
  return p->propagator >= 0 && p->propagator <= 2 && p->rk4_substeps >= 1;
}

}  // namespace

struct satenv_cpu_env {
  int64_t n = 0;
  int threads = 1;
  satenv_params prm{};
  std::vector<double> f64;
  std::vector<int32_t> i32;
  int32_t err = 0;
};

namespace {

void note_error(satenv_cpu_env* h, int rc) {
#pragma omp critical(satenv_cpu_err)
  if (h->err == 0) h->err = rc;
}

// one env of step_kernel<AUTORESET> (satenv_kernels.hip), host side
void step_env(satenv_cpu_env* h, const StepIO& io, int64_t i, bool autoreset, double* fin_v, double* ret_v,
              double* rew_v, double* cap_v) {
  const Params& prm = h->prm;
  double* f64 = h->f64.data();
  int32_t* i32 = h->i32.data();
  double fin = 0.0, fin_ret = 0.0, rew_acc = 0.0;
  Lane L;
  step_begin<true>(prm, h->n, f64, i32, io, i, autoreset, L);
  if (L.err) note_error(h, L.err);
  if (!L.terminal) {
    int cnt = 0;
    const int rc = danger_zone(prm, L.k[0], L.k[1], L.k[2], L.k[3], L.k[4], L.k[5], L.k[6], L.k[7], L.k[8],
                               L.k[9], L.k[10], L.k[11], L.fuel_c, L.fcm, cnt);   // environment.py:150, :317-332
    if (rc) note_error(h, rc);
    step_reward(prm, L, cnt);
  }
  step_end(prm, h->n, f64, i32, io, i, autoreset, L, fin, fin_ret, rew_acc);
  if (fin_v) {
    fin_v[i] = fin;
    ret_v[i] = fin_ret;
    rew_v[i] = rew_acc;
    cap_v[i] = L.cap;
  }
}

void init_envs(satenv_cpu_env* h) {
  const int64_t n = h->n;
  const satenv_params& p = h->prm;
  for (int64_t i = 0; i < n; ++i) {
    for (int c = 0; c < 12; ++c) h->f64[c * n + i] = p.init_kin[c];          // environment.py:30-33
    h->f64[12 * n + i] = p.fuel_c0;                                          // :42-43
    h->f64[13 * n + i] = p.fuel_t0;
    h->f64[14 * n + i] = INFINITY;                                           // :44
    h->f64[kPlaneRet * n + i] = 0.0;
    h->i32[kPlaneDz * n + i] = 0;                                            // :41
    h->i32[kPlaneCount * n + i] = 0;
    h->i32[kPlaneBits * n + i] = make_bits(p.fuel_c0_mode, p.fuel_t0_mode, 1, p.flag);
  }
}

}  // namespace

extern "C" {

const char* satenv_cpu_last_error(void) { return g_last_error.c_str(); }

int satenv_cpu_create(satenv_cpu_env** out, int64_t num_envs, const satenv_params* p, int device) {
  if (!out || !p || num_envs <= 0 || device < 0) return fail(SATENV_ERR_ARG, "satenv_cpu_create: bad arguments");
  if (!params_ok(p)) return fail(SATENV_ERR_ARG, "satenv_cpu_create: propagator must be 0/1/2, rk4_substeps >= 1");
  satenv_cpu_env* h = new satenv_cpu_env();
  h->n = num_envs;
  h->threads = device > 0 ? device : omp_get_max_threads();
  h->prm = *p;
  h->f64.assign((size_t)kF64Planes * num_envs, 0.0);
  h->i32.assign((size_t)kI32Planes * num_envs, 0);
  init_envs(h);
  *out = h;
  return SATENV_OK;
}

int satenv_cpu_destroy(satenv_cpu_env* h) {
  delete h;
  return SATENV_OK;
}

int satenv_cpu_num_envs(const satenv_cpu_env* h, int64_t* n) {
  if (!h || !n) return fail(SATENV_ERR_ARG, "satenv_cpu_num_envs: null");
  *n = h->n;
  return SATENV_OK;
}

int satenv_cpu_set_params(satenv_cpu_env* h, const satenv_params* p) {
  if (!h || !p) return fail(SATENV_ERR_ARG, "satenv_cpu_set_params: null");
  if (!params_ok(p)) return fail(SATENV_ERR_ARG, "satenv_cpu_set_params: propagator must be 0/1/2, rk4_substeps >= 1");
  const int32_t flag = h->prm.flag;
  h->prm = *p;
  h->prm.flag = flag;
  return SATENV_OK;
}

int satenv_cpu_reset(satenv_cpu_env* h, int32_t flag, const uint8_t* env_mask, float* obs_out, double* obs64_out,
                     void* /*stream*/) {
  if (!h) return fail(SATENV_ERR_ARG, "satenv_cpu_reset: null handle");
  if (flag < 0 || flag > 2) return fail(SATENV_ERR_ARG, "satenv_cpu_reset: Flag must be 0, 1 or 2");
  h->prm.flag = flag;
  const int64_t n = h->n;
  double* f64 = h->f64.data();
  int32_t* i32 = h->i32.data();
#pragma omp parallel for num_threads(h->threads) schedule(static)
  for (int64_t i = 0; i < n; ++i) {                                          // environment.py:66-79
    double k[12];
    if (env_mask == nullptr || env_mask[i] != 0) {
      reset_kin(h->prm, k);
      for (int c = 0; c < 12; ++c) f64[c * n + i] = k[c];
      const int b = i32[kPlaneBits * n + i];
      i32[kPlaneBits * n + i] = make_bits(fc_mode(b), ft_mode(b), 1, flag);
      i32[kPlaneCount * n + i] = 0;
      f64[kPlaneRet * n + i] = 0.0;
    } else {
      for (int c = 0; c < 12; ++c) k[c] = f64[c * n + i];
    }
    write_obs(obs_out, obs64_out, i, k);
  }
  return SATENV_OK;
}

int satenv_cpu_step(satenv_cpu_env* h, const float* pa, const float* ea, const int32_t* episode_count,
                    float* obs_out, double* obs64_out, double* reward_out, uint8_t* done_out, void* /*stream*/) {
  if (!h || !pa || !ea) return fail(SATENV_ERR_ARG, "satenv_cpu_step: null argument");
  const StepIO io{pa, ea, episode_count, obs_out, obs64_out, reward_out, nullptr, done_out, nullptr, nullptr};
#pragma omp parallel for num_threads(h->threads) schedule(dynamic, 64)
  for (int64_t i = 0; i < h->n; ++i) step_env(h, io, i, false, nullptr, nullptr, nullptr, nullptr);
  return SATENV_OK;
}

int satenv_cpu_step_autoreset(satenv_cpu_env* h, const float* pa, const float* ea, float* obs_out,
                              float* reward_out, uint8_t* done_out, double* stats_out, void* /*stream*/) {
  if (!h || !pa || !ea) return fail(SATENV_ERR_ARG, "satenv_cpu_step_autoreset: null argument");
  const StepIO io{pa, ea, nullptr, obs_out, nullptr, nullptr, reward_out, done_out, nullptr, nullptr};
  const int64_t n = h->n;
  std::vector<double> st;
  if (stats_out) st.assign((size_t)4 * n, 0.0);
  double* s = stats_out ? st.data() : nullptr;
#pragma omp parallel for num_threads(h->threads) schedule(dynamic, 64)
  for (int64_t i = 0; i < n; ++i)
    step_env(h, io, i, true, s, s ? s + n : nullptr, s ? s + 2 * n : nullptr, s ? s + 3 * n : nullptr);
  if (stats_out) {            // the kernel's per-wave sums, here in env order (deterministic)
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    for (int k = 0; k < 4; ++k)
      for (int64_t i = 0; i < n; ++i) acc[k] += s[k * n + i];
    for (int k = 0; k < 4; ++k)
      if (k == 2 || acc[k] != 0.0) stats_out[k] += acc[k];
  }
  return SATENV_OK;
}

int satenv_cpu_get_state(const satenv_cpu_env* h, double* f64_planes, int32_t* i32_planes, void* /*stream*/) {
  if (!h) return fail(SATENV_ERR_ARG, "satenv_cpu_get_state: null handle");
  if (f64_planes) std::memcpy(f64_planes, h->f64.data(), sizeof(double) * SATENV_F64_PLANES * h->n);
  if (i32_planes) std::memcpy(i32_planes, h->i32.data(), sizeof(int32_t) * SATENV_I32_PLANES * h->n);
  return SATENV_OK;
}

int satenv_cpu_set_state(satenv_cpu_env* h, const double* f64_planes, const int32_t* i32_planes, void* /*stream*/) {
  if (!h) return fail(SATENV_ERR_ARG, "satenv_cpu_set_state: null handle");
  if (f64_planes) std::memcpy(h->f64.data(), f64_planes, sizeof(double) * SATENV_F64_PLANES * h->n);
  if (i32_planes) std::memcpy(h->i32.data(), i32_planes, sizeof(int32_t) * SATENV_I32_PLANES * h->n);
  return SATENV_OK;
}

int satenv_cpu_danger_zone(int64_t n, const double* states, const double* fuel, const int32_t* fuel_mode,
                           int32_t* count_out, void* /*stream*/) {
  if (n <= 0 || !states || !fuel || !fuel_mode || !count_out)
    return fail(SATENV_ERR_ARG, "satenv_cpu_danger_zone: bad args");
  satenv_params prm;
  std::memset(&prm, 0, sizeof(prm));                      // states are absolute: R_cw = V_cw = 0
#pragma omp parallel for schedule(dynamic, 64)
  for (int64_t i = 0; i < n; ++i) {
    const double* x = states + i * 12;
    int cnt = 0;
    const int rc = danger_zone(prm, x[0], x[1], x[2], x[3], x[4], x[5], x[6], x[7], x[8], x[9], x[10], x[11],
                               fuel[i], fuel_mode[i], cnt);
    count_out[i] = rc ? rc : cnt;
  }
  return SATENV_OK;
}

int satenv_cpu_check(satenv_cpu_env* h, int32_t* status) {
  if (!h || !status) return fail(SATENV_ERR_ARG, "satenv_cpu_check: null");
  *status = h->err;
  return SATENV_OK;
}

}  // extern "C"
