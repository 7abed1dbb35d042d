// surrogate_device.h -- ImprovedNN (single_pluse_model/model.py:7-24,
// 5 -> 256 -> 128 -> 64 -> 10, ReLU) forward in bf16 on gfx950 MFMA, on the
// features network_method_process builds (real_time_data_process.py:112-116):
// [a, e, i, f, fuel_c] of the pursuer's absolute orbit (config 5).
//
// Orientation: every layer computes Y^T = W . X^T with v_mfma_f32_16x16x32_bf16,
// A = the layer's weights (16 output neurons per tile), B = the activations
// (16 envs per wave on the lanes).  The accumulator of a layer (lane = env,
// rows 4g+i = neurons) is, converted pairwise to bf16, directly the next
// layer's B fragment: for K-step s, element j of lane group g carries neuron
// 32s + 16(j>>2) + 4g + (j&3).  The weights are packed once (surrogate_pack)
// with exactly that k permutation, so activations never leave registers and
// every A fragment is one 16-B LDS read.  The whole packed net (91 KB) is
// staged into LDS once per workgroup.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace surrogate {

using frag_ab = __attribute__((ext_vector_type(8))) short;   // 8 bf16
using frag_cd = __attribute__((ext_vector_type(4))) float;

constexpr int kThreads = 256;                 // 4 waves x 16 envs per pass
constexpr int kH1 = 256, kH2 = 128, kH3 = 64, kOut = 10, kOutPad = 16, kIn = 5;
// packed image (bf16 elements), rows padded by 8 elements (16 B) against LDS bank conflicts
constexpr int kW1Row = 8;                     // k 0..7 (features 0..4, zeros)
constexpr int kW2Row = kH1 + 8, kW3Row = kH2 + 8, kW4Row = kH3 + 8;
constexpr int kW1Off = 0;
constexpr int kW2Off = kW1Off + kH1 * kW1Row;
constexpr int kW3Off = kW2Off + kH2 * kW2Row;
constexpr int kW4Off = kW3Off + kH3 * kW3Row;
constexpr int kWElems = kW4Off + kOutPad * kW4Row;
constexpr int kBiasOffBytes = kWElems * 2;                       // f32 b1 | b2 | b3 | b4(16)
constexpr int kBiasElems = kH1 + kH2 + kH3 + kOutPad;
// the trainer's StandardScalers (single_pulse_fully_connected_model.py:273-278),
// f64: x_std = (x - in_mean) / in_scale before the bf16 input, y = y_std *
// out_scale + out_mean after fc4 (sklearn's transform / inverse_transform);
// identity (0 / 1) unless set (satenv_surrogate_set_scalers)
struct Scalers {
  double in_mean[8], in_scale[8], out_scale[kOutPad], out_mean[kOutPad];
};
constexpr int kScaleOffBytes = kBiasOffBytes + kBiasElems * 4;
constexpr int kBlobBytes = kScaleOffBytes + (int)sizeof(Scalers);   // 93 632 B
static_assert(kScaleOffBytes % 16 == 0 && kBlobBytes % 16 == 0, "blob staged as 16-B words");

__device__ __forceinline__ unsigned short f2bf(float f) {        // round to nearest even (torch .to(bfloat16))
  unsigned u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (unsigned short)((u >> 16) | 0x40);   // quiet NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return (unsigned short)(u >> 16);
}
__device__ __forceinline__ float bf2f(unsigned short b) { return __uint_as_float((unsigned)b << 16); }

// position of input neuron kk inside a packed row for layers 2-4 (inverse of
// kk = 32s + 16(j>>2) + 4g + (j&3) -> element 32s + 8g + j)
__host__ __device__ __forceinline__ int packed_pos(int kk) {
  const int s = kk >> 5, r = kk & 31, hi = r >> 4, g = (r >> 2) & 3, lo = r & 3;
  return 32 * s + 8 * g + 4 * hi + lo;
}

// pack torch Linear weights (f32, [out][in] row-major) + biases into the blob
__global__ void pack_kernel(const float* __restrict__ w1, const float* __restrict__ b1, const float* __restrict__ w2,
                            const float* __restrict__ b2, const float* __restrict__ w3, const float* __restrict__ b3,
                            const float* __restrict__ w4, const float* __restrict__ b4, uint8_t* __restrict__ blob) {
  unsigned short* W = reinterpret_cast<unsigned short*>(blob);
  float* B = reinterpret_cast<float*>(blob + kBiasOffBytes);
  const int stride = gridDim.x * blockDim.x;
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < kWElems + kBiasElems; t += stride) {
    if (t >= kWElems) {
      const int b = t - kWElems;
      float v;
      if (b < kH1) v = b1[b];
      else if (b < kH1 + kH2) v = b2[b - kH1];
      else if (b < kH1 + kH2 + kH3) v = b3[b - kH1 - kH2];
      else v = (b - kH1 - kH2 - kH3 < kOut) ? b4[b - kH1 - kH2 - kH3] : 0.0f;
      B[b] = v;
      continue;
    }
    float v = 0.0f;
    if (t < kW2Off) {
      const int n = t / kW1Row, k = t % kW1Row;
      v = k < kIn ? w1[n * kIn + k] : 0.0f;
    } else {
      int base, row, in, outs;
      if (t < kW3Off) { base = kW2Off; row = kW2Row; in = kH1; outs = kH2; }
      else if (t < kW4Off) { base = kW3Off; row = kW3Row; in = kH2; outs = kH3; }
      else { base = kW4Off; row = kW4Row; in = kH3; outs = kOutPad; }
      const int n = (t - base) / row, p = (t - base) % row;
      if (p < in) {
        // find kk with packed_pos(kk) == p
        const int s = p >> 5, r = p & 31, g = r >> 3, j = r & 7;
        const int kk = 32 * s + 16 * (j >> 2) + 4 * g + (j & 3);
        const float* w = (t < kW3Off) ? w2 : (t < kW4Off) ? w3 : w4;
        v = (n < ((t < kW4Off) ? outs : kOut)) ? w[n * in + kk] : 0.0f;
      }
    }
    W[t] = f2bf(v);
  }
  if (blockIdx.x == 0 && threadIdx.x < sizeof(Scalers) / 8) {      // identity scalers
    double* S = reinterpret_cast<double*>(blob + kScaleOffBytes);
    const int k = threadIdx.x;                                     // in_mean 0..7, in_scale 8..15, out_scale 16..31
    S[k] = (k >= 8 && k < 32) ? 1.0 : 0.0;
  }
}

__global__ void set_scalers_kernel(const Scalers sc, uint8_t* __restrict__ blob) {
  *reinterpret_cast<Scalers*>(blob + kScaleOffBytes) = sc;
}

// bias + ReLU of one accumulator tile into half `h` (elements 4h..4h+3) of a bf16 fragment
__device__ __forceinline__ void act_into(const frag_cd& acc, const float* bias, frag_ab& f, int h) {
#pragma unroll
  for (int i = 0; i < 4; ++i) f[4 * h + i] = (short)f2bf(fmaxf(acc[i] + bias[i], 0.0f));
}

__device__ __forceinline__ frag_ab lds_frag(const unsigned short* p) {
  return *reinterpret_cast<const frag_ab*>(p);
}

// One layer Y^T[OUT x 16] = W[OUT x K] X^T[K x 16]: TILES = OUT/16 output
// tiles, STEPS = K/32 k-steps; in[s] is the B fragment of k-step s, out[t/2]
// collects this layer's tiles pairwise as the next layer's fragments.
template <int TILES, int STEPS, int ROW>
__device__ __forceinline__ void layer(const unsigned short* W, const float* bias, const frag_ab (&in)[STEPS],
                                      frag_ab (&out)[TILES / 2]) {
  const int l = threadIdx.x & 63, g = l >> 4, c = l & 15;
#pragma unroll
  for (int t = 0; t < TILES; ++t) {
    frag_cd acc = {0.0f, 0.0f, 0.0f, 0.0f};
    const unsigned short* row = W + (16 * t + c) * ROW + 8 * g;
#pragma unroll
    for (int s = 0; s < STEPS; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(lds_frag(row + 32 * s), in[s], acc, 0, 0, 0);
    act_into(acc, bias + 16 * t + 4 * g, out[t >> 1], t & 1);
    __builtin_amdgcn_sched_barrier(0);   // keep each tile's 16-B LDS reads next to its MFMAs (no 256-VGPR hoist)
  }
}

// features of network_method_process for one env: f32 [a, e, i, f, fuel]
struct Feat { float v[5]; bool ok; };

}  // namespace surrogate
