// philox_device.h -- counter-based Gaussian draws shared by the sampling
// kernels (rollout_kernels.hip gaussian_kernel, ppo_kernels.hip policy_kernel):
// Philox4x32-10 keyed by (seed, agent), counter (global env id, step), then
// Box-Muller.  The same (seed, agent, env id, step) gives the same draw in
// every kernel and for every sharding of the envs over ranks.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

__device__ __forceinline__ void philox4x32_10(uint32_t (&c)[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int rnd = 0; rnd < 10; ++rnd) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
    const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
    c[0] = n0;
    c[1] = (uint32_t)p1;
    c[2] = n2;
    c[3] = (uint32_t)p0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

__device__ __forceinline__ float philox_u01_open0(uint32_t x) {   // (0, 1]
  return ((float)(x >> 8) + 1.0f) * (1.0f / 16777216.0f);
}
__device__ __forceinline__ float philox_u01(uint32_t x) {         // [0, 1)
  return (float)(x >> 8) * (1.0f / 16777216.0f);
}

// key of (seed, agent)
__host__ __device__ inline void philox_key(uint64_t seed, uint32_t agent, uint32_t& k0, uint32_t& k1) {
  k0 = (uint32_t)seed ^ (agent * 0x85EBCA6Bu);
  k1 = (uint32_t)(seed >> 32) ^ (agent * 0xC2B2AE35u + 0x27D4EB2Fu);
}

// four standard normals for (global env id, step)
__device__ __forceinline__ void philox_normal4(uint64_t gid, uint64_t step, uint32_t k0, uint32_t k1, float (&z)[4]) {
  uint32_t c[4] = {(uint32_t)gid, (uint32_t)(gid >> 32), (uint32_t)step, (uint32_t)(step >> 32)};
  philox4x32_10(c, k0, k1);
  const float r0 = sqrtf(-2.0f * logf(philox_u01_open0(c[0])));
  const float t0 = 6.283185307179586f * philox_u01(c[1]);
  const float r1 = sqrtf(-2.0f * logf(philox_u01_open0(c[2])));
  const float t1 = 6.283185307179586f * philox_u01(c[3]);
  z[0] = r0 * cosf(t0);
  z[1] = r0 * sinf(t0);
  z[2] = r1 * cosf(t1);
  z[3] = r1 * sinf(t1);
}

// choose_action (ppo_continuous.py:184-188) for one dimension:
// a = clamp(mean + std*z, +-max_action); log_prob(a) as Normal.log_prob
__device__ __forceinline__ void gaussian_act(float m, float log_std, float z, float max_action, float& a,
                                             float& logp) {
  const float kLogSqrt2Pi = 0.9189385332046727f;   // math.log(math.sqrt(2 * math.pi))
  const float sd = expf(log_std);                   // std = exp(log_std)
  a = m + sd * z;                                   // Normal.sample()
  a = fminf(fmaxf(a, -max_action), max_action);     // torch.clamp
  const float var = sd * sd;
  const float dv = a - m;
  logp = (-(dv * dv) / (2.0f * var) - logf(sd)) - kLogSqrt2Pi;
}
