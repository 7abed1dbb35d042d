// l2_persist.hip -- development microbenchmark (not shipped, not a test): does
// a line one kernel loaded into its XCD's L2 still hit there in the NEXT
// kernel of the stream?  (If so, a kernel could prefetch the next rowpass's
// rows into the L2 of the XCD that will read them.)
// Each of 256 workgroups owns a 16 KB slice of a buffer holding a random
// cyclic permutation of its 128 lines (the first word of each line holds the
// next line's first word index); "touch" loads the whole slice (all lanes);
// "chase" then walks the permutation with one lane, 128 dependent sc1 loads
// (one per line), and records s_memrealtime ticks per load (100 MHz).
// Cases (each after a 1 GiB sweep that evicts everything):
//   cold        chase only
//   same        touch(slice b) by block b, then chase(slice b) by block b
//               (the same XCD under round-robin dealing)
//   shifted     touch(slice b) by block b, then chase(slice b) by block b+1
//               (another XCD)
//   in-kernel   touch and chase inside one kernel (block b, slice b)
//   written     block b rewrites slice b with plain stores (the same words),
//               then chase(slice b) by block b in the next kernel: do lines a
//               kernel WROTE (dirty at its end) still hit on the same XCD?
//   written-shifted   the same, chased by block b+1 (another XCD)
// Output: one JSON object, ns per dependent load (median over blocks).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/l2_persist.hip -o tools/_probe/l2_persist
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <vector>

#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) {                                                                    \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));  \
      std::exit(1);                                                                            \
    }                                                                                          \
  } while (0)

constexpr int kBlocks = 256, kWords = 4096, kLines = kWords / 32, kChase = kLines;

__global__ void __launch_bounds__(256) touch_kernel(const unsigned* __restrict__ buf, unsigned* __restrict__ sink) {
  const unsigned* s = buf + (size_t)blockIdx.x * kWords;
  unsigned acc = 0;
  for (int i = threadIdx.x * 4; i < kWords; i += 256 * 4) {
    const uint4 v = *reinterpret_cast<const uint4*>(s + i);
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0xdeadbeefu) sink[blockIdx.x] = acc;      // (never true: keeps the loads)
}

__device__ __forceinline__ void chase(const unsigned* s, unsigned long long* out, int b) {
  if (threadIdx.x != 0) return;
  unsigned idx = 0;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  // sc1 loads: never an L1 hit, so each dependent load is served by the L2 or
  // beyond; every step a different 128-B line (no reuse inside the chase)
  for (int k = 0; k < kChase; ++k) idx = __hip_atomic_load(&s[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  out[2 * b] = t1 - t0;
  out[2 * b + 1] = idx;
}

// rewrites the slice's words with their own values (plain stores: the lines
// end the kernel dirty in this XCD's L2)
__global__ void __launch_bounds__(256) write_kernel(unsigned* __restrict__ buf, const unsigned* __restrict__ src) {
  unsigned* s = buf + (size_t)blockIdx.x * kWords;
  const unsigned* r = src + (size_t)blockIdx.x * kWords;
  for (int i = threadIdx.x * 4; i < kWords; i += 256 * 4)
    *reinterpret_cast<uint4*>(s + i) = *reinterpret_cast<const uint4*>(r + i);
}

__global__ void __launch_bounds__(256) chase_kernel(const unsigned* __restrict__ buf, int shift,
                                                    unsigned long long* __restrict__ out) {
  const int slice = (blockIdx.x + kBlocks - shift) % kBlocks;   // block b chases slice b - shift
  chase(buf + (size_t)slice * kWords, out, blockIdx.x);
}

__global__ void __launch_bounds__(256) touch_chase_kernel(const unsigned* __restrict__ buf,
                                                          unsigned long long* __restrict__ out) {
  const unsigned* s = buf + (size_t)blockIdx.x * kWords;
  unsigned acc = 0;
  for (int i = threadIdx.x * 4; i < kWords; i += 256 * 4) {
    const uint4 v = *reinterpret_cast<const uint4*>(s + i);
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  __syncthreads();
  if (acc == 0xdeadbeefu) out[0] = acc;
  chase(s, out, blockIdx.x);
}

__global__ void sweep_kernel(const uint4* __restrict__ big, size_t n4, unsigned* __restrict__ sink) {
  unsigned acc = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = big[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0xdeadbeefu) sink[0] = acc;
}

int main() {
  // per slice: a random cyclic permutation of its lines (line l's first word
  // holds the next line's first word index)
  std::vector<unsigned> host((size_t)kBlocks * kWords, 0u);
  std::mt19937 rng(1);
  for (int b = 0; b < kBlocks; ++b) {
    std::vector<unsigned> order(kLines);
    std::iota(order.begin(), order.end(), 0u);
    std::shuffle(order.begin() + 1, order.end(), rng);
    for (int i = 0; i < kLines; ++i) host[(size_t)b * kWords + 32 * order[i]] = 32 * order[(i + 1) % kLines];
  }
  unsigned *buf, *sink, *copy;
  unsigned long long* out;
  CK(hipMalloc(&buf, host.size() * 4));
  CK(hipMemcpy(buf, host.data(), host.size() * 4, hipMemcpyHostToDevice));
  CK(hipMalloc(&copy, host.size() * 4));
  CK(hipMemcpy(copy, host.data(), host.size() * 4, hipMemcpyHostToDevice));
  CK(hipMalloc(&sink, kBlocks * 4));
  CK(hipMalloc(&out, kBlocks * 16));
  const size_t big_bytes = 1ull << 30;
  uint4* big;
  CK(hipMalloc(&big, big_bytes));
  CK(hipMemset(big, 1, big_bytes));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  std::vector<unsigned long long> res(2 * kBlocks);
  auto evict = [&] { hipLaunchKernelGGL(sweep_kernel, dim3(1024), dim3(256), 0, s, big, big_bytes / 16, sink); };
  auto median_ns = [&] {
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(res.data(), out, kBlocks * 16, hipMemcpyDeviceToHost));
    std::vector<double> v;
    for (int b = 0; b < kBlocks; ++b) v.push_back(res[2 * b] * 10.0 / kChase);
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
  };
  std::printf("{\"tool\": \"tools/l2_persist.hip\", \"ns_per_dependent_load\": {");
  const char* names[6] = {"cold", "same", "shifted", "in_kernel", "written", "written_shifted"};
  for (int c = 0; c < 6; ++c) {
    double best = 1e30;
    for (int rep = 0; rep < 5; ++rep) {
      evict();
      if (c == 1 || c == 2) hipLaunchKernelGGL(touch_kernel, dim3(kBlocks), dim3(256), 0, s, buf, sink);
      if (c == 4 || c == 5) hipLaunchKernelGGL(write_kernel, dim3(kBlocks), dim3(256), 0, s, buf, copy);
      if (c == 3)
        hipLaunchKernelGGL(touch_chase_kernel, dim3(kBlocks), dim3(256), 0, s, buf, out);
      else
        hipLaunchKernelGGL(chase_kernel, dim3(kBlocks), dim3(256), 0, s, buf, (c == 2 || c == 5) ? 1 : 0, out);
      best = std::min(best, median_ns());
    }
    std::printf("%s\"%s\": %.1f", c ? ", " : "", names[c], best);
  }
  std::printf("}}\n");
  return 0;
}
