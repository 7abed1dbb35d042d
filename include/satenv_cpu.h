/*
 * satenv_cpu.h -- host build of the environment ABI (include/satenv.h):
 * the same FP64 step code (csrc/satenv_device.h + satenv_step.h) compiled
 * by g++ for x86 host cores, OpenMP over envs, glibc transcendentals.
 *
 * Every satenv_cpu_* entry point has the signature of its satenv_*
 * counterpart, with HOST pointers: the `device` argument of
 * create is the OpenMP thread count (0 = every core this process may run
 * on), and `stream` arguments are accepted and ignored (the calls are
 * synchronous).  It is what the drop-in runs with device="cpu" (BASELINE
 * configs[0]: CPPO_main on CPU, no GPU) and the CPU baseline of bench.py.
 * Replaces, like satenv.h: satellites.__init__ / reset / step
 * (environment.py:26-255), the CPPO_main.py:119-153 loop around them, and
 * Time_window_of_danger_zone (satellite_function.py:18-99,341-373).
 */
#ifndef SATENV_CPU_H
#define SATENV_CPU_H
#include <stdint.h>

#include "satenv.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct satenv_cpu_env satenv_cpu_env;   /* opaque */

const char* satenv_cpu_last_error(void);
int satenv_cpu_create(satenv_cpu_env** out, int64_t num_envs, const satenv_params* p, int device);
int satenv_cpu_destroy(satenv_cpu_env* h);
int satenv_cpu_num_envs(const satenv_cpu_env* h, int64_t* n);
int satenv_cpu_set_params(satenv_cpu_env* h, const satenv_params* p);
int satenv_cpu_reset(satenv_cpu_env* h, int32_t flag, const uint8_t* env_mask, float* obs_out, double* obs64_out,
                     void* stream);
int satenv_cpu_step(satenv_cpu_env* h, const float* pa, const float* ea, const int32_t* episode_count,
                    float* obs_out, double* obs64_out, double* reward_out, uint8_t* done_out, void* stream);
int satenv_cpu_step_autoreset(satenv_cpu_env* h, const float* pa, const float* ea, float* obs_out,
                              float* reward_out, uint8_t* done_out, double* stats_out, void* stream);
int satenv_cpu_get_state(const satenv_cpu_env* h, double* f64_planes, int32_t* i32_planes, void* stream);
int satenv_cpu_set_state(satenv_cpu_env* h, const double* f64_planes, const int32_t* i32_planes, void* stream);
int satenv_cpu_danger_zone(int64_t n, const double* states, const double* fuel, const int32_t* fuel_mode,
                           int32_t* count_out, void* stream);
int satenv_cpu_check(satenv_cpu_env* h, int32_t* status);

#ifdef __cplusplus
}
#endif
#endif /* SATENV_CPU_H */
