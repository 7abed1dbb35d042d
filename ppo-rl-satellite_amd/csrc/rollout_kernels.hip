// rollout_kernels.hip -- gfx950 kernels behind include/satrl_rollout.h.
#include <hip/hip_runtime.h>

#include <string>

#include "philox_device.h"
#include "satrl_rollout.h"

namespace {

thread_local std::string g_err;

#define HIP_CHECK_LAUNCH()                                                   \
  do {                                                                       \
    hipError_t e_ = hipGetLastError();                                       \
    if (e_ != hipSuccess) { g_err = hipGetErrorString(e_); return -2; }      \
  } while (0)

// ---------------------------------------------------------------------------
// GAE reverse scan (ppo_continuous.py:201-208), one lane per env.  The time
// loop is sequential per env; loads of steps t-1.. are independent of the
// carried gae, so the unrolled loop keeps several rows in flight per lane.
// f32, reference operation order, compiled with -ffp-contract=off.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) gae_kernel(int64_t T, int64_t N, const float* __restrict__ r,
                                                  const uint8_t* __restrict__ done, const float* __restrict__ v,
                                                  float gamma, float c, float* __restrict__ adv,
                                                  float* __restrict__ vt) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  float gae = 0.0f;
  float v_next = v[T * N + i];
#pragma unroll 8
  for (int64_t t = T - 1; t >= 0; --t) {
    const int64_t o = t * N + i;
    const float v_t = v[o];
    const float dw = (float)done[o];
    const float delta = (r[o] + (gamma * (1.0f - dw)) * v_next) - v_t;   // r + g*(1-dw)*vs_ - vs
    gae = delta + (c * gae) * (1.0f - dw);                               // delta + g*l*gae*(1-d)
    adv[o] = gae;
    vt[o] = gae + v_t;                                                    // v_target = adv + vs
    v_next = v_t;
  }
}

// choose_action (ppo_continuous.py:184-188): a = clamp(mean + std*z, +-max);
// log_prob(a) per dim as torch.distributions.Normal.log_prob.  Noise:
// philox_device.h, keyed by (seed, agent, global env id, step).
__global__ void __launch_bounds__(256) gaussian_kernel(int64_t N, const float* __restrict__ mean,
                                                       const float* __restrict__ log_std, float max_action,
                                                       uint32_t k0, uint32_t k1, int64_t env_offset,
                                                       uint64_t step, const uint64_t* __restrict__ step_base,
                                                       float* __restrict__ act,
                                                       float* __restrict__ logp) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  if (step_base) step += *step_base;
  float z[4];
  philox_normal4((uint64_t)(env_offset + i), step, k0, k1, z);
#pragma unroll
  for (int d = 0; d < 3; ++d) gaussian_act(mean[i * 3 + d], log_std[d], z[d], max_action, act[i * 3 + d], logp[i * 3 + d]);
}

__global__ void __launch_bounds__(256) moments_kernel(int64_t n, const float* __restrict__ x,
                                                      double* __restrict__ out) {
  double s = 0.0, s2 = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double v = x[i];
    s += v;
    s2 += v * v;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    s += __shfl_xor(s, off, 64);
    s2 += __shfl_xor(s2, off, 64);
  }
  __shared__ double red[2][4];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { red[0][w] = s; red[1][w] = s2; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0.0, b = 0.0;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) { a += red[0][k]; b += red[1][k]; }
    atomicAdd(out, a);
    atomicAdd(out + 1, b);
  }
}

}  // namespace

extern "C" {

int satrl_gae(int64_t T, int64_t N, const float* r, const uint8_t* done, const float* v, float gamma, float lamda,
              float* adv_out, float* vtarget_out, void* stream) {
  if (T <= 0 || N <= 0 || !r || !done || !v || !adv_out || !vtarget_out) return -1;
  // gamma*lamda is a python float product, rounded to f32 when it meets the
  // np.float32 gae (NEP 50), ppo_continuous.py:205
  const float c = (float)((double)gamma * (double)lamda);
  const int block = 64;   // N = 16384 envs -> 256 single-wave workgroups, one per CU
  hipLaunchKernelGGL(gae_kernel, dim3((unsigned)((N + block - 1) / block)), dim3(block), 0, (hipStream_t)stream, T,
                     N, r, done, v, gamma, c, adv_out, vtarget_out);
  HIP_CHECK_LAUNCH();
  return 0;
}

int satrl_gaussian_sample(int64_t N, const float* mean, const float* log_std, float max_action, uint64_t seed,
                          uint32_t agent, int64_t env_offset, uint64_t step, const uint64_t* step_base,
                          float* act_out, float* logp_out, void* stream) {
  if (N <= 0 || !mean || !log_std || !act_out || !logp_out) return -1;
  uint32_t k0, k1;
  philox_key(seed, agent, k0, k1);
  hipLaunchKernelGGL(gaussian_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, (hipStream_t)stream, N, mean,
                     log_std, max_action, k0, k1, env_offset, step, step_base, act_out, logp_out);
  HIP_CHECK_LAUNCH();
  return 0;
}

int satrl_moments(int64_t n, const float* x, double* out, void* stream) {
  if (n <= 0 || !x || !out) return -1;
  int64_t blocks = (n + 255) / 256;
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(moments_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, n, x, out);
  HIP_CHECK_LAUNCH();
  return 0;
}

const char* satrl_last_error(void) { return g_err.c_str(); }

}  // extern "C"
