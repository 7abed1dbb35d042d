// Development probe (not shipped): accuracy and issue rate of an f32 product
// computed as three-way bf16 splits on v_mfma_f32_16x16x32_bf16 (six partial
// products hi*hi, hi*mid, mid*hi, mid*mid, hi*lo, lo*hi per 32-wide k chunk)
// against v_mfma_f32_16x16x4_f32 (exact f32 fmaf chain) and an f64 host
// reference, on the rowpass's fc2 shapes (K = 256, activations in (-1, 1),
// weights ~ N(0, 0.06)).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/bf16x3_probe.hip -o tools/_probe/bf16x3_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef short s8 __attribute__((ext_vector_type(8)));

constexpr int K = 256, NT = 4096;   // tiles (one wave each)

static uint16_t bf16_rne(float x) {
  uint32_t u;
  std::memcpy(&u, &x, 4);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
static float bf16_f(uint16_t h) {
  uint32_t u = (uint32_t)h << 16;
  float x;
  std::memcpy(&x, &u, 4);
  return x;
}
// x = hi + mid + lo exactly (each residual is exact in f32; the last has <= 8 bits)
static void split3(float x, uint16_t& h, uint16_t& m, uint16_t& l) {
  h = bf16_rne(x);
  const float r = x - bf16_f(h);
  m = bf16_rne(r);
  const float r2 = r - bf16_f(m);
  l = bf16_rne(r2);
}

// A [NT][16][K] row-major, B [NT][K][16] (k-major): f32
__global__ void k_f32(const float* A, const float* B, float* D, int reps) {
  const int t = blockIdx.x, l = threadIdx.x, i = l & 15, g = l >> 4;
  const float* a = A + (size_t)t * 16 * K + i * K;
  const float* b = B + (size_t)t * K * 16 + i;
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int r = 0; r < reps; ++r)
    for (int c = 0; c < K / 32; ++c)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int k = 32 * c + 8 * g + e;
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[k], b[k * 16], acc, 0, 0, 0);
      }
#pragma unroll
  for (int j = 0; j < 4; ++j) D[(size_t)t * 256 + (4 * g + j) * 16 + i] = acc[j];
}

// planes: A3 [NT][3][16][K], B3 [NT][3][16 cols][K] (col-major so a lane's 8 k are contiguous): bf16 bits
__global__ void k_bf16x3(const uint16_t* A3, const uint16_t* B3, float* D, int reps, int nprod) {
  const int t = blockIdx.x, l = threadIdx.x, i = l & 15, g = l >> 4;
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  const int pa[6] = {0, 0, 1, 1, 0, 2}, pb[6] = {0, 1, 0, 1, 2, 0};
  for (int r = 0; r < reps; ++r)
    for (int c = 0; c < K / 32; ++c) {
      s8 a[3], b[3];
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        a[p] = *reinterpret_cast<const s8*>(A3 + (((size_t)t * 3 + p) * 16 + i) * K + 32 * c + 8 * g);
        b[p] = *reinterpret_cast<const s8*>(B3 + (((size_t)t * 3 + p) * 16 + i) * K + 32 * c + 8 * g);
      }
      // smallest terms first
#pragma unroll
      for (int q = 5; q >= 0; --q)
        if (q < nprod) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[pa[q]], b[pb[q]], acc, 0, 0, 0);
    }
#pragma unroll
  for (int j = 0; j < 4; ++j) D[(size_t)t * 256 + (4 * g + j) * 16 + i] = acc[j];
}

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
      return 1;                                                            \
    }                                                                      \
  } while (0)

int main() {
  std::mt19937 rng(1);
  std::uniform_real_distribution<float> ua(-1.f, 1.f);
  std::normal_distribution<float> nb(0.f, 0.06f);
  std::vector<float> A((size_t)NT * 16 * K), B((size_t)NT * K * 16);
  for (auto& x : A) x = std::tanh(2.f * ua(rng));
  for (auto& x : B) x = nb(rng);
  std::vector<uint16_t> A3((size_t)NT * 3 * 16 * K), B3((size_t)NT * 3 * 16 * K);
  for (int t = 0; t < NT; ++t)
    for (int i = 0; i < 16; ++i)
      for (int k = 0; k < K; ++k) {
        uint16_t h, m, l;
        split3(A[(size_t)t * 16 * K + i * K + k], h, m, l);
        A3[(((size_t)t * 3 + 0) * 16 + i) * K + k] = h;
        A3[(((size_t)t * 3 + 1) * 16 + i) * K + k] = m;
        A3[(((size_t)t * 3 + 2) * 16 + i) * K + k] = l;
        split3(B[(size_t)t * K * 16 + k * 16 + i], h, m, l);
        B3[(((size_t)t * 3 + 0) * 16 + i) * K + k] = h;
        B3[(((size_t)t * 3 + 1) * 16 + i) * K + k] = m;
        B3[(((size_t)t * 3 + 2) * 16 + i) * K + k] = l;
      }
  float *dA, *dB, *dD;
  uint16_t *dA3, *dB3;
  CK(hipMalloc(&dA, A.size() * 4));
  CK(hipMalloc(&dB, B.size() * 4));
  CK(hipMalloc(&dA3, A3.size() * 2));
  CK(hipMalloc(&dB3, B3.size() * 2));
  CK(hipMalloc(&dD, (size_t)NT * 256 * 4));
  CK(hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dA3, A3.data(), A3.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dB3, B3.data(), B3.size() * 2, hipMemcpyHostToDevice));
  std::vector<double> ref((size_t)NT * 256), mag((size_t)NT * 256);
  for (int t = 0; t < NT; ++t)
    for (int i = 0; i < 16; ++i)
      for (int j = 0; j < 16; ++j) {
        double s = 0, m = 0;
        for (int k = 0; k < K; ++k) {
          const double p = (double)A[(size_t)t * 16 * K + i * K + k] * B[(size_t)t * K * 16 + k * 16 + j];
          s += p;
          m += std::fabs(p);
        }
        ref[(size_t)t * 256 + i * 16 + j] = s;
        mag[(size_t)t * 256 + i * 16 + j] = m;
      }
  std::vector<float> D((size_t)NT * 256);
  auto report = [&](const char* name) {
    CK(hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost));
    double mx = 0, sum = 0, mxr = 0;
    for (size_t q = 0; q < D.size(); ++q) {
      const double e = std::fabs(D[q] - ref[q]) / mag[q];
      mx = std::max(mx, e);
      sum += e;
      mxr = std::max(mxr, std::fabs(D[q] - ref[q]) / std::max(std::fabs(ref[q]), 1e-30));
    }
    printf("%-22s err/sum|ab|: max %.3e mean %.3e   max rel %.3e\n", name, mx, sum / D.size(), mxr);
    return 0;
  };
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  k_f32<<<NT, 64>>>(dA, dB, dD, 1);
  CK(hipDeviceSynchronize());
  if (report("f32 16x16x4")) return 1;
  for (int np : {6, 4, 3, 1}) {
    k_bf16x3<<<NT, 64>>>(dA3, dB3, dD, 1, np);
    CK(hipDeviceSynchronize());
    char nm[64];
    snprintf(nm, sizeof nm, "bf16 split, %d products", np);
    if (report(nm)) return 1;
  }
  // issue rate: operands re-read from L1/L2 each chunk; many reps
  const int reps = 200;
  float ms;
  k_f32<<<NT, 64>>>(dA, dB, dD, reps);
  CK(hipEventRecord(e0));
  k_f32<<<NT, 64>>>(dA, dB, dD, reps);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms, e0, e1));
  printf("f32 16x16x4 loop:        %.3f ms (%.1f TF/s effective f32)\n", ms,
         2.0 * NT * 256.0 * K * reps / (ms * 1e-3) / 1e12);
  k_bf16x3<<<NT, 64>>>(dA3, dB3, dD, reps, 6);
  CK(hipEventRecord(e0));
  k_bf16x3<<<NT, 64>>>(dA3, dB3, dD, reps, 6);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms, e0, e1));
  printf("bf16 x6 16x16x32 loop:   %.3f ms (%.1f TF/s effective f32)\n", ms,
         2.0 * NT * 256.0 * K * reps / (ms * 1e-3) / 1e12);
  return 0;
}
