// Development tool (not shipped, not a test): times every hipBLASLt algorithm
// that supports the update's dW2 product at H = 256, mb = 4096, for split-K
// S = 1, 2, 4, 8, 16 (the layout satrl/ppo.py `_dw2` hands to torch.bmm):
//   per net and split s: p2[net][s] (H x H, row-major) = dZ2_s^T H1_s,
//   dZ2_s / H1_s = rows [s*K, (s+1)*K) of the net's [mb][H] row-major block.
// Column-major view: D (H x H) = A * B^T with A = H1_s (H x K, ld H) and
// B = dZ2_s (H x K, ld H), 2S strided batches.  Each algorithm runs twice on
// the same inputs and must reproduce its output bit for bit (split-K
// solutions that fold through atomics would not); the table lists the
// fastest deterministic ones with their solution names.
//
// Built as a shared library and driven by tools/blaslt_search.py after
// `import torch`, so it searches the hipBLASLt that the product actually
// runs on (torch's bundled copy: libsatrl.so's libhipblaslt.so.1 resolves to
// it in-process; /opt/rocm's has other solution indices):
//   hipcc --offload-arch=gfx950 -O2 -std=c++17 -shared -fPIC tools/blaslt_search.cpp \
//         -lhipblaslt -o tools/_probe/libblaslt_search.so
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>
#include <hipblaslt/hipblaslt-ext.hpp>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define HCHECK(x)                                                                   \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                 \
    }                                                                               \
  } while (0)
#define BCHECK(x)                                                                        \
  do {                                                                                   \
    hipblasStatus_t s_ = (x);                                                            \
    if (s_ != HIPBLAS_STATUS_SUCCESS) {                                                  \
      std::fprintf(stderr, "%s:%d hipblaslt status %d\n", __FILE__, __LINE__, (int)s_); \
      std::exit(1);                                                                      \
    }                                                                                    \
  } while (0)

struct Res {
  double us;
  int idx;
  bool det;
  std::string name;
};

extern "C" int blaslt_search(int mb) {
  const int H = 256;
  const int reps = 200;
  const size_t ws_cap = 64ull << 20;
  hipblasLtHandle_t lt;
  BCHECK(hipblasLtCreate(&lt));
  float *H1, *dZ2, *D, *ws;
  HCHECK(hipMalloc(&H1, sizeof(float) * 2 * mb * H));
  HCHECK(hipMalloc(&dZ2, sizeof(float) * 2 * mb * H));
  HCHECK(hipMalloc(&D, sizeof(float) * 2 * 16 * H * H));
  HCHECK(hipMalloc(&ws, ws_cap));
  {
    std::vector<float> h(2 * (size_t)mb * H);
    uint32_t x = 12345;
    for (auto& v : h) { x = x * 1664525u + 1013904223u; v = (float)((x >> 8) & 0xffff) / 65536.0f - 0.5f; }
    HCHECK(hipMemcpy(H1, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    for (auto& v : h) { x = x * 1664525u + 1013904223u; v = ((float)((x >> 8) & 0xffff) / 65536.0f - 0.5f) * 1e-3f; }
    HCHECK(hipMemcpy(dZ2, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  }
  hipStream_t st;
  HCHECK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  HCHECK(hipEventCreate(&e0));
  HCHECK(hipEventCreate(&e1));
  const float alpha = 1.0f, beta = 0.0f;
  std::vector<float> out0(2 * 16 * (size_t)H * H), out1(out0.size());

  std::vector<hipblasLtMatmulHeuristicResult_t> all;
  BCHECK(hipblaslt_ext::getAllAlgos(lt, hipblaslt_ext::GemmType::HIPBLASLT_GEMM, HIPBLAS_OP_N, HIPBLAS_OP_T,
                                    HIP_R_32F, HIP_R_32F, HIP_R_32F, HIP_R_32F, HIPBLAS_COMPUTE_32F, all));
  std::printf("getAllAlgos: %zu algorithms (N, T, f32)\n", all.size());
  std::fflush(stdout);

  for (int S : {1, 2, 4, 8, 16}) {
    const int K = mb / S, B = 2 * S;
    hipblasLtMatmulDesc_t md;
    BCHECK(hipblasLtMatmulDescCreate(&md, HIPBLAS_COMPUTE_32F, HIP_R_32F));
    hipblasOperation_t opA = HIPBLAS_OP_N, opB = HIPBLAS_OP_T;
    BCHECK(hipblasLtMatmulDescSetAttribute(md, HIPBLASLT_MATMUL_DESC_TRANSA, &opA, sizeof(opA)));
    BCHECK(hipblasLtMatmulDescSetAttribute(md, HIPBLASLT_MATMUL_DESC_TRANSB, &opB, sizeof(opB)));
    hipblasLtMatrixLayout_t la, lb, lc;
    BCHECK(hipblasLtMatrixLayoutCreate(&la, HIP_R_32F, H, K, H));
    BCHECK(hipblasLtMatrixLayoutCreate(&lb, HIP_R_32F, H, K, H));
    BCHECK(hipblasLtMatrixLayoutCreate(&lc, HIP_R_32F, H, H, H));
    const int64_t sab = (int64_t)K * H, sc = (int64_t)H * H;
    for (auto l : {la, lb}) {
      BCHECK(hipblasLtMatrixLayoutSetAttribute(l, HIPBLASLT_MATRIX_LAYOUT_BATCH_COUNT, &B, sizeof(B)));
      BCHECK(hipblasLtMatrixLayoutSetAttribute(l, HIPBLASLT_MATRIX_LAYOUT_STRIDED_BATCH_OFFSET, &sab, sizeof(sab)));
    }
    BCHECK(hipblasLtMatrixLayoutSetAttribute(lc, HIPBLASLT_MATRIX_LAYOUT_BATCH_COUNT, &B, sizeof(B)));
    BCHECK(hipblasLtMatrixLayoutSetAttribute(lc, HIPBLASLT_MATRIX_LAYOUT_STRIDED_BATCH_OFFSET, &sc, sizeof(sc)));

    // the heuristic's own first choice (what torch.bmm gets)
    hipblasLtMatmulPreference_t pref;
    BCHECK(hipblasLtMatmulPreferenceCreate(&pref));
    size_t wsz = ws_cap;
    BCHECK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsz, sizeof(wsz)));
    hipblasLtMatmulHeuristicResult_t heur[8];
    int nh = 0;
    hipblasLtMatmulAlgoGetHeuristic(lt, md, la, lb, lc, lc, pref, 8, heur, &nh);
    int heur_idx = nh > 0 ? hipblaslt_ext::getIndexFromAlgo(heur[0].algo) : -1;

    auto run = [&](hipblasLtMatmulAlgo_t* algo, size_t w) {
      return hipblasLtMatmul(lt, md, &alpha, H1, la, dZ2, lb, &beta, D, lc, D, lc, algo, ws, w, st);
    };
    std::vector<Res> res;
    int tried = 0;
    for (auto& r : all) {
      size_t w = 0;
      if (hipblaslt_ext::matmulIsAlgoSupported(lt, md, &alpha, la, lb, &beta, lc, lc, r.algo, w) !=
          HIPBLAS_STATUS_SUCCESS)
        continue;
      if (w > ws_cap) continue;
      ++tried;
      HCHECK(hipMemsetAsync(D, 0, sizeof(float) * B * H * H, st));
      if (run(&r.algo, w) != HIPBLAS_STATUS_SUCCESS) continue;
      HCHECK(hipMemcpyAsync(out0.data(), D, sizeof(float) * B * H * H, hipMemcpyDeviceToHost, st));
      HCHECK(hipMemsetAsync(D, 0xff, sizeof(float) * B * H * H, st));
      for (int i = 0; i < 10; ++i) run(&r.algo, w);
      HCHECK(hipMemcpyAsync(out1.data(), D, sizeof(float) * B * H * H, hipMemcpyDeviceToHost, st));
      HCHECK(hipStreamSynchronize(st));
      const bool det = std::memcmp(out0.data(), out1.data(), sizeof(float) * B * H * H) == 0;
      HCHECK(hipEventRecord(e0, st));
      for (int i = 0; i < reps; ++i) run(&r.algo, w);
      HCHECK(hipEventRecord(e1, st));
      HCHECK(hipEventSynchronize(e1));
      float ms = 0.f;
      HCHECK(hipEventElapsedTime(&ms, e0, e1));
      res.push_back({ms * 1e3 / reps, hipblaslt_ext::getIndexFromAlgo(r.algo), det,
                     hipblaslt_ext::getSolutionNameFromAlgo(lt, r.algo)});
    }
    std::sort(res.begin(), res.end(), [](const Res& a, const Res& b) { return a.us < b.us; });
    double heur_us = -1.0;
    for (auto& r : res)
      if (r.idx == heur_idx) heur_us = r.us;
    std::printf("S=%d (K=%d, batches %d): %d supported; heuristic #1 idx %d at %.2f us\n", S, K, B, tried, heur_idx,
                heur_us);
    int shown = 0;
    for (auto& r : res) {
      if (shown >= 12) break;
      std::printf("  %7.2f us  idx %6d  %s  %s\n", r.us, r.idx, r.det ? "det   " : "NONDET", r.name.c_str());
      ++shown;
    }
    std::fflush(stdout);
    hipblasLtMatmulPreferenceDestroy(pref);
    hipblasLtMatrixLayoutDestroy(la);
    hipblasLtMatrixLayoutDestroy(lb);
    hipblasLtMatrixLayoutDestroy(lc);
    hipblasLtMatmulDescDestroy(md);
  }
  hipblasLtDestroy(lt);
  return 0;
}
