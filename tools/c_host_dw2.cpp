// Development check (not shipped): the H = 256 dW2 entry points from a plain
// C++ host with no torch in the process, so libsatrl.so's libhipblaslt.so.1
// resolves to ROCm 7.2's library.  Prints the solution the plan took, checks
// two runs agree bit for bit and a sample of outputs against fp64 sums, and
// times 200 back-to-back launches.
//   hipcc --offload-arch=gfx950 -O2 -std=c++17 -I include tools/c_host_dw2.cpp \
//     -L ppo-rl-satellite_amd/satrl -lsatrl -Wl,-rpath,$PWD/ppo-rl-satellite_amd/satrl -o tools/_probe/c_host_dw2
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "satrl_ppo.h"

extern "C" const char* satrl_ppo_last_error(void);

int main() {
  const int H = 256, mb = 4096, S = 4;
  const size_t n = 2ull * mb * H;
  std::vector<float> h1(n), dz(n);
  uint32_t x = 99;
  auto rnd = [&]() { x = x * 1664525u + 1013904223u; return (float)((x >> 8) & 0xffff) / 65536.0f - 0.5f; };
  for (auto& v : h1) v = rnd();
  for (auto& v : dz) v = rnd();
  float *dH1, *dZ2, *p2;
  if (hipMalloc(&dH1, n * 4) || hipMalloc(&dZ2, n * 4) || hipMalloc(&p2, 2ull * S * H * H * 4)) return 2;
  (void)hipMemcpy(dH1, h1.data(), n * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(dZ2, dz.data(), n * 4, hipMemcpyHostToDevice);
  int64_t wsb = 0;
  int idx = -1;
  if (satrl_ppo_dw2_lib_workspace(H, mb, -1, S, &wsb, &idx)) {
    std::printf("plan failed: %s\n", satrl_ppo_last_error());
    return 1;
  }
  void* ws = nullptr;
  if (wsb > 0 && hipMalloc(&ws, wsb)) return 2;
  std::printf("solution index %d, workspace %lld B\n", idx, (long long)wsb);
  hipStream_t st;
  (void)hipStreamCreate(&st);
  std::vector<float> o0(2ull * S * H * H), o1(o0.size());
  for (int run = 0; run < 2; ++run) {
    if (satrl_ppo_dw2_lib(H, mb, -1, S, dH1, dZ2, p2, ws, wsb, st)) {
      std::printf("dw2 failed: %s\n", satrl_ppo_last_error());
      return 1;
    }
    (void)hipStreamSynchronize(st);
    (void)hipMemcpy(run ? o1.data() : o0.data(), p2, o0.size() * 4, hipMemcpyDeviceToHost);
  }
  const bool same = std::memcmp(o0.data(), o1.data(), o0.size() * 4) == 0;
  // p2[net][s][i][j] = sum over rows r of split s: dZ2[net][r][i] * H1[net][r][j]
  double worst = 0.0;
  const int K = mb / S;
  for (int t = 0; t < 64; ++t) {
    const int net = t & 1, s = (t >> 1) % S, i = (t * 37) % H, j = (t * 101) % H;
    double ref = 0.0;
    for (int r = s * K; r < (s + 1) * K; ++r)
      ref += (double)dz[((size_t)net * mb + r) * H + i] * (double)h1[((size_t)net * mb + r) * H + j];
    const double got = o0[(((size_t)net * S + s) * H + i) * H + j];
    worst = std::fmax(worst, std::fabs(got - ref));
  }
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, st);
  for (int k = 0; k < 200; ++k) satrl_ppo_dw2_lib(H, mb, -1, S, dH1, dZ2, p2, ws, wsb, st);
  (void)hipEventRecord(e1, st);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  std::printf("bitwise repeat %s, worst |err| vs fp64 %.3g, %.2f us per launch back to back\n",
              same ? "yes" : "NO", worst, ms * 1e3 / 200);
  return same && worst < 1e-3 ? 0 : 1;
}
