/*
 * satrl_rollout.h -- C ABI of the rollout-side HIP kernels of the PPO engine.
 *
 *   satrl_gae               <- ppo_continuous.py:198-210 (deltas, reversed GAE loop,
 *                              v_target = adv + vs), one lane per env, reverse scan
 *                              over the horizon of a time-major [T][N] buffer
 *   satrl_gaussian_sample   <- ppo_continuous.py:176-189 choose_action (Gaussian):
 *                              Normal(mean, exp(log_std)).sample() -> clamp(+-max)
 *                              -> per-dim log_prob; counter-based Philox4x32-10
 *                              keyed by (seed, agent, global env id, step), so a
 *                              rollout is identical for any env sharding
 *   satrl_moments           <- adv.mean() / adv.std() of ppo_continuous.py:210
 *                              (f64 sum and sum of squares, for a global all-reduce)
 *
 * All pointers are device buffers, calls are async on `stream` (hipStream_t,
 * NULL = default) and graph-capturable.  Return 0 or a negative error code.
 */
#ifndef SATRL_ROLLOUT_H
#define SATRL_ROLLOUT_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* r f32 [T][N], done u8 [T][N] (dw == done, CPPO_main.py:136-139 with the
 * env's own timeout), v f32 [T+1][N] = critic(obs[0..T]);  outputs adv and
 * v_target f32 [T][N].  f32 arithmetic in the reference's order, no FMA.   */
int satrl_gae(int64_t T, int64_t N, const float* r, const uint8_t* done, const float* v, float gamma, float lamda,
              float* adv_out, float* vtarget_out, void* stream);

/* mean f32 [N][3], log_std f32 [3]; act/logp f32 [N][3].  The Philox
 * counter's step is `step` plus, if step_base (a device u64) is non-NULL,
 * *step_base -- so a captured hipGraph replays with fresh noise once the
 * caller advances *step_base.                                              */
int satrl_gaussian_sample(int64_t N, const float* mean, const float* log_std, float max_action, uint64_t seed,
                          uint32_t agent, int64_t env_offset, uint64_t step, const uint64_t* step_base,
                          float* act_out, float* logp_out, void* stream);

/* out f64[2] += (sum x, sum x^2) over x f32 [n]  (out must be zeroed first) */
int satrl_moments(int64_t n, const float* x, double* out, void* stream);

const char* satrl_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
