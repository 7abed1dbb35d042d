// span_probe.h -- live launch spans of the product kernels (satrl_span_probe,
// include/satrl_ppo.h): the measurement the bench reports as each kernel's
// duration, taken in its own run instead of from a rocprof pass.
//
// Each kernel below has a SPAN instantiation (template flag) that differs
// from the product one only at its exits: lane 0 of every wave stores the
// wave's (first instruction, exit) s_memrealtime pair (100 MHz, the same
// clock on every CU) into a record slot of its own -- one 16-B plain store,
// no atomic, no barrier, nothing another wave waits for.  While a probe
// buffer is set, the launchers take a fresh region of it per launch (graph
// captures included: each captured node keeps its region, so a replay
// rewrites the records of that node) and run the SPAN instantiation; the
// host reads a launch's span as max(exit) - min(start) over its waves.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace satrl_span {

enum Kind { kRowpass = 0, kDw2 = 1, kReduce = 2, kAdam = 3, kPolicyAct = 4, kPolicyValue = 5, kEnvStep = 6 };

// host side (ppo_kernels.hip): the record region of the next launch of `kind`
// with `waves` waves, or nullptr when no probe is set (or it is full)
unsigned long long* take(int kind, int64_t waves);

__device__ __forceinline__ unsigned long long now() { return __builtin_amdgcn_s_memrealtime(); }

// at a wave's exit: lane 0 stores (t0, now) for this wave (call it at every
// point where lane 0 leaves the kernel; a wave whose lane 0 leaves early
// records that point)
__device__ __forceinline__ void exit(unsigned long long* rec, unsigned long long t0) {
  const unsigned long long t1 = now();
  if ((threadIdx.x & 63) == 0) {
    const int64_t wv = (int64_t)blockIdx.x * ((blockDim.x + 63) / 64) + (threadIdx.x >> 6);
    *reinterpret_cast<ulonglong2*>(rec + 2 * wv) = make_ulonglong2(t0, t1);
  }
}

}  // namespace satrl_span
