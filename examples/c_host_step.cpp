// A C++ host with no Python and no torch in the process driving the hot path
// through the C ABI alone (include/satenv.h, include/satrl_ppo.h): the
// training loop's env steps (satenv_step_autoreset, CPPO_main.py:119-153) and
// PPO minibatch steps at H = 256 (rowpass -> dW2 -> reduce -> Adam,
// ppo_continuous.py:213-239) at mb 4096 and 512.  It writes its inputs and outputs as raw
// little-endian arrays so tests/test_c_host_gpu.py can run the same inputs
// through the Python package and compare.
//
//   c_host_step <out_dir>
//
// Built by `make -C ppo-rl-satellite_amd/csrc c-host` (__graft_entry__.build()).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "satenv.h"
#include "satrl_ppo.h"

namespace {

uint32_t g_x = 20240917u;
float unif(float lo, float hi) {                  // LCG, 24-bit mantissa draw
  g_x = g_x * 1664525u + 1013904223u;
  return lo + (hi - lo) * (float)(g_x >> 8) * (1.0f / 16777216.0f);
}

#define HIP_OK(x)                                                                \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(2);                                                              \
    }                                                                            \
  } while (0)
#define ENV_OK(x)                                                                       \
  do {                                                                                  \
    if ((x) != 0) {                                                                     \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, satenv_last_error());     \
      std::exit(3);                                                                     \
    }                                                                                   \
  } while (0)
#define PPO_OK(x)                                                                       \
  do {                                                                                  \
    if ((x) != 0) {                                                                     \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, satrl_ppo_last_error());  \
      std::exit(4);                                                                     \
    }                                                                                   \
  } while (0)

template <typename T>
T* dev(size_t n) {
  T* p = nullptr;
  HIP_OK(hipMalloc(&p, n * sizeof(T)));
  HIP_OK(hipMemset(p, 0, n * sizeof(T)));
  return p;
}
template <typename T>
T* dev(const std::vector<T>& h) {
  T* p = dev<T>(h.size());
  HIP_OK(hipMemcpy(p, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
  return p;
}
template <typename T>
std::vector<T> host(const T* d, size_t n) {
  std::vector<T> h(n);
  HIP_OK(hipMemcpy(h.data(), d, n * sizeof(T), hipMemcpyDeviceToHost));
  return h;
}
template <typename T>
void save(const std::string& dir, const char* name, const std::vector<T>& v) {
  const std::string path = dir + "/" + name;
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f || std::fwrite(v.data(), sizeof(T), v.size(), f) != v.size()) {
    std::fprintf(stderr, "cannot write %s\n", path.c_str());
    std::exit(5);
  }
  std::fclose(f);
}

// one PPO minibatch step at H = 256 on mb packed rows, the product's kernel
// sequence (rowpass with k-packed bf16 H1 / dZ2 planes -> dW2 on them ->
// reduce -> Adam), plus the f32-row rowpass's H1 / dZ2 for comparison; the
// outputs go to <out>/ppo<mb>_*
void ppo_step(const std::string& out, int mb, hipStream_t st) {
  const int H = 256;
  const std::string tag = "ppo" + std::to_string(mb) + "_";
  int64_t off[SATRL_PPO_NOFF];
  PPO_OK(satrl_ppo_layout(H, off));
  const int64_t total = off[SATRL_PPO_TOTAL];
  std::vector<float> P(total), src((size_t)mb * 32, 0.0f);
  for (auto& v : P) v = unif(-0.06f, 0.06f);
  for (int r = 0; r < mb; ++r) {                  // packed rows: s | a | logp | adv | v_target
    float* row = &src[(size_t)r * 32];
    for (int c = 0; c < 18; ++c) row[c] = unif(-1.0f, 1.0f);
    for (int c = 18; c < 21; ++c) row[c] = unif(-1.6f, 1.6f);
    for (int c = 21; c < 24; ++c) row[c] = -1.0f - unif(0.0f, 1.0f);
    row[24] = unif(-1.0f, 1.0f);
    row[25] = unif(-1.0f, 1.0f);
  }
  // Adam's bias corrections {1 - beta1**k, sqrt(1 - beta2**k)} in double, as
  // torch.optim.Adam computes them in python floats; rows until both are 1.0
  std::vector<double> bct = {0.0, 0.0};
  for (int k = 1;; ++k) {
    const double b1 = 1.0 - std::pow(0.9, k), b2 = std::sqrt(1.0 - std::pow(0.999, k));
    bct.push_back(b1);
    bct.push_back(b2);
    if (b1 == 1.0 && b2 == 1.0) break;
  }
  const std::vector<float> lr = {2e-4f, 2e-4f};
  int64_t nwg = 0, nblk = 0;
  PPO_OK(satrl_ppo_sizes(H, mb, &nwg, &nblk));

  float* d_P = dev(P);
  // the fc2 operand image (the f32 fc2.weight^T), built on the device from P
  const int64_t w2x = satrl_ppo_w2x_floats(H);
  float* d_W2X = dev<float>((size_t)w2x);
  PPO_OK(satrl_ppo_w2x_sync(H, -1, d_P, d_W2X, st));
  float* d_M = dev<float>(total);
  float* d_V = dev<float>(total);
  float* d_G = dev<float>(total);
  float* d_src = dev(src);
  float* d_H1 = dev<float>(2 * (size_t)mb * H);
  float* d_dZ2 = dev<float>(2 * (size_t)mb * H);
  float* d_pt = dev<float>((size_t)nwg * (6 * H + 12));
  float* d_pw = dev<float>((size_t)nwg * 2 * H * 20);
  double* d_nsq = dev<double>(2 * (size_t)nblk);
  double* d_steps = dev<double>(2);
  double* d_bct = dev(bct);
  float* d_lr = dev(lr);

  PPO_OK(satrl_ppo_rowpass(H, mb, -1, d_src, nullptr, d_P, d_W2X, 0.1f, 0.01f, 1.6f, d_H1, d_dZ2, d_pt, d_pw, st));
  HIP_OK(hipStreamSynchronize(st));
  save(out, (tag + "H1.f32").c_str(), host(d_H1, 2 * (size_t)mb * H));
  save(out, (tag + "dZ2.f32").c_str(), host(d_dZ2, 2 * (size_t)mb * H));
  // the product step: the rowpass with k-packed bf16 H1 / dZ2 planes and the
  // split-bf16 dW2 on them (every kernel hand-written, no library tiles)
  const int64_t kxe = satrl_ppo_kx_elems(H, mb);
  uint16_t* d_H1x = dev<uint16_t>((size_t)kxe);
  uint16_t* d_dZ2x = dev<uint16_t>((size_t)kxe);
  const int S = satrl_ppo_dw2_kx_splits(H, mb, -1);
  const int64_t p2n = 2LL * S * H * H;          // every slab call takes these capacities and refuses past them
  float* d_p2 = dev<float>((size_t)p2n);
  PPO_OK(satrl_ppo_rowpass_kx(H, mb, -1, d_src, nullptr, d_P, d_W2X, 0.1f, 0.01f, 1.6f, d_H1x, d_dZ2x, kxe, d_pt,
                              d_pw, st));
  // dW2 with the reduce's W1 / tail regions in the same launch, then the W2 region
  PPO_OK(satrl_ppo_dw2_kx_w1(H, mb, -1, S, d_H1x, d_dZ2x, kxe, d_p2, p2n, 3, d_pw, d_pt, d_G, d_nsq, st));
  PPO_OK(satrl_ppo_reduce(H, mb, -1, S, 3 | 4, d_p2, p2n, nullptr, nullptr, d_G, d_nsq, d_steps, st));
  PPO_OK(satrl_ppo_adam(H, mb, -1, d_nsq, d_steps, d_bct, (int)(bct.size() / 2), d_lr, 0.9f, 0.999f, 1e-5f, 0.5f, 1,
                        d_G, d_P, d_M, d_V, d_W2X, st));
  // up to 1024 rows the rowpass ran the column-split kernel: its in-launch
  // exchange must not have timed out (the call waits for the stream, 60 s at most)
  int xerr = 0;
  PPO_OK(satrl_ppo_rowpass_error(&xerr, 60.0, st));
  if (xerr) {
    std::fprintf(stderr, "c_host_step: the column-split rowpass exchange timed out\n");
    std::exit(1);
  }
  save(out, (tag + "P0.f32").c_str(), P);
  save(out, (tag + "src.f32").c_str(), src);
  save(out, (tag + "bct.f64").c_str(), bct);
  save(out, (tag + "G.f32").c_str(), host(d_G, (size_t)total));
  save(out, (tag + "P.f32").c_str(), host(d_P, (size_t)total));
  save(out, (tag + "M.f32").c_str(), host(d_M, (size_t)total));
  save(out, (tag + "V.f32").c_str(), host(d_V, (size_t)total));
  save(out, (tag + "W2T.f32").c_str(), host(d_W2X, (size_t)w2x));
  save(out, (tag + "steps.f64").c_str(), host(d_steps, 2));
  for (void* q : {(void*)d_P, (void*)d_W2X, (void*)d_M, (void*)d_V, (void*)d_G, (void*)d_src, (void*)d_H1,
                  (void*)d_dZ2, (void*)d_pt, (void*)d_pw, (void*)d_nsq, (void*)d_steps, (void*)d_bct, (void*)d_lr,
                  (void*)d_H1x, (void*)d_dZ2x, (void*)d_p2})
    HIP_OK(hipFree(q));
  std::printf("c_host_step: one minibatch step (H %d, mb %d, dW2 split %d ways)\n", H, mb, S);
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s <out_dir>\n", argv[0]);
    return 1;
  }
  const std::string out = argv[1];
  hipStream_t st;
  HIP_OK(hipStreamCreate(&st));

  // ---- env: N envs, T autoreset steps of uniform actions --------------------------
  const int64_t N = 2048;
  const int T = 40;
  satenv_params p;
  ENV_OK(satenv_default_params(&p));
  p.d_capture = 15000.0;
  p.max_episode_steps = 12;                       // episodes end and reset inside the window
  satenv_env* env = nullptr;
  ENV_OK(satenv_create(&env, N, &p, 0));
  std::vector<float> pa((size_t)T * N * 3), ea((size_t)T * N * 3);
  for (auto& v : pa) v = unif(-1.6f, 1.6f);
  for (auto& v : ea) v = unif(-1.6f, 1.6f);
  float* d_pa = dev(pa);
  float* d_ea = dev(ea);
  float* d_obs = dev<float>((size_t)N * 18);
  float* d_rew = dev<float>((size_t)T * N);
  uint8_t* d_done = dev<uint8_t>((size_t)T * N);
  double* d_stats = dev<double>(4);
  ENV_OK(satenv_reset(env, 0, nullptr, d_obs, nullptr, st));
  for (int t = 0; t < T; ++t)
    ENV_OK(satenv_step_autoreset(env, d_pa + (size_t)t * N * 3, d_ea + (size_t)t * N * 3, d_obs, d_rew + (size_t)t * N,
                                 d_done + (size_t)t * N, d_stats, st));
  HIP_OK(hipStreamSynchronize(st));
  save(out, "env_pa.f32", pa);
  save(out, "env_ea.f32", ea);
  save(out, "env_obs.f32", host(d_obs, (size_t)N * 18));
  save(out, "env_rew.f32", host(d_rew, (size_t)T * N));
  save(out, "env_done.u8", host(d_done, (size_t)T * N));
  save(out, "env_stats.f64", host(d_stats, 4));
  ENV_OK(satenv_destroy(env));

  // ---- one PPO minibatch step, H = 256: the bench's minibatch and configs[3]'s per-rank one
  ppo_step(out, 4096, st);
  ppo_step(out, 512, st);
  std::printf("c_host_step: %lld envs x %d autoreset steps\n", (long long)N, T);
  return 0;
}
