// ppo_kernels.hip -- fused PPO minibatch-step kernels for gfx950 (include/satrl_ppo.h).
//
// Per minibatch (actor + critic together, same rows):
//   fwd1   gather rows (packed [B][32]) + fc1 + tanh           -> H1, saug, aux
//   [bmm]  Z2  = H1 @ W2^T                                      (hipBLASLt, batch 2)
//   head   fc2 bias+tanh, output layers, losses, d/dZ2, tail partial slabs
//   [bmm]  dH1 = dZ2 @ W2 ; G.W2 = dZ2^T @ H1
//   tanh_bwd dZ1 = dH1 * (1 - H1^2)
//   [bmm]  G.W1 = dZ1^T @ saug      ([dW1 | db1] in one GEMM via the ones column)
//   reduce tail partials -> G, per-block squared norms per net
//   adam   clip coefficient per net + Adam (torch single-tensor formula)
// Every reduction has a fixed order, so a step is bitwise reproducible.
#include <hip/hip_runtime.h>

#include <cmath>
#include <string>

#include "satrl_ppo.h"

namespace {

thread_local std::string g_err;

constexpr int kRows = 16;          // minibatch rows per fwd1/head workgroup
constexpr int kF1Rows = 8;         // rows per fwd1 workgroup
constexpr int kW1Rows = 32;        // rows per dw1 workgroup (split-K chunk of [dW1 | db1])
constexpr float kLogSqrt2Pi = 0.9189385332046727f;   // math.log(math.sqrt(2*math.pi))

struct Layout {
  int64_t W2, W1, b2, W3a, b3a, ls, W3c, b3c, total, tail;
};

__host__ __device__ inline Layout layout(int H) {
  Layout L;
  L.W2 = 0;
  L.W1 = L.W2 + 2LL * H * H;
  L.b2 = L.W1 + 2LL * H * 20;
  L.W3a = L.b2 + 2LL * H;
  L.b3a = L.b2 + 5LL * H;
  L.ls = L.b3a + 4;
  L.W3c = L.ls + 4;
  L.b3c = L.W3c + H;
  L.total = L.b3c + 4;
  L.tail = L.total - L.b2;   // 6H + 12
  return L;
}

// 0 = actor, 1 = critic (pads belong to the net of their segment)
__device__ __forceinline__ int net_of(const Layout& L, int64_t e, int H) {
  if (e < L.W1) return e >= (int64_t)H * H;
  if (e < L.b2) return (e - L.W1) >= (int64_t)H * 20;
  if (e < L.W3a) return (e - L.b2) >= H;
  return e >= L.W3c;
}

// ---------------------------------------------------------------------------
// fwd1: gather + fc1 + tanh.  One workgroup = kRows rows, thread j = hidden unit.
// ---------------------------------------------------------------------------
template <int H>
__global__ void __launch_bounds__(H) fwd1_kernel(int mb, const float* __restrict__ src, const int64_t* __restrict__ idx,
                                                 const float* __restrict__ P, float* __restrict__ H1,
                                                 float* __restrict__ saug, float* __restrict__ aux) {
  const Layout L = layout(H);
  __shared__ float s[kF1Rows][20];
  const int r0 = blockIdx.x * kF1Rows;
  const int t = threadIdx.x;
  // W1 rows of this thread's hidden unit for both nets: 2 x 5 float4 loads
  const float4* wa4 = reinterpret_cast<const float4*>(P + L.W1 + (int64_t)t * 20);
  const float4* wc4 = reinterpret_cast<const float4*>(P + L.W1 + (int64_t)(H + t) * 20);
  float4 qa[5], qc[5];
#pragma unroll
  for (int k = 0; k < 5; ++k) { qa[k] = wa4[k]; qc[k] = wc4[k]; }
  for (int q = t; q < kF1Rows * 26; q += H) {
    const int r = q / 26, c = q % 26, row = r0 + r;
    float v = 0.0f;
    if (row < mb) v = src[idx[row] * 32 + c];
    if (c < 18) s[r][c] = v;
    else if (row < mb) aux[(int64_t)row * 8 + (c - 18)] = v;
  }
  __syncthreads();
  for (int q = t; q < kF1Rows * 20; q += H) {
    const int r = q / 20, c = q % 20, row = r0 + r;
    if (row < mb) saug[(int64_t)row * 20 + c] = c < 18 ? s[r][c] : (c == 18 ? 1.0f : 0.0f);
  }
  const float wa[20] = {qa[0].x, qa[0].y, qa[0].z, qa[0].w, qa[1].x, qa[1].y, qa[1].z, qa[1].w, qa[2].x, qa[2].y,
                        qa[2].z, qa[2].w, qa[3].x, qa[3].y, qa[3].z, qa[3].w, qa[4].x, qa[4].y, qa[4].z, qa[4].w};
  const float wc[20] = {qc[0].x, qc[0].y, qc[0].z, qc[0].w, qc[1].x, qc[1].y, qc[1].z, qc[1].w, qc[2].x, qc[2].y,
                        qc[2].z, qc[2].w, qc[3].x, qc[3].y, qc[3].z, qc[3].w, qc[4].x, qc[4].y, qc[4].z, qc[4].w};
#pragma unroll
  for (int r = 0; r < kF1Rows; ++r) {
    const int row = r0 + r;
    float za = 0.0f, zc = 0.0f;
#pragma unroll
    for (int k = 0; k < 18; ++k) {
      za = fmaf(s[r][k], wa[k], za);
      zc = fmaf(s[r][k], wc[k], zc);
    }
    if (row < mb) {
      H1[(int64_t)row * H + t] = tanhf(za + wa[18]);               // actor fc1 + tanh
      H1[((int64_t)mb + row) * H + t] = tanhf(zc + wc[18]);        // critic fc1 + tanh
    }
  }
}

// ---------------------------------------------------------------------------
// dw1: [dW1 | db1] partials.  dZ1 = dH1 * (1 - H1^2) is formed on the fly
// (layer 1 needs no further backprop), so neither dZ1 nor a K=mb GEMM with
// N=20 is materialised.  One workgroup = kW1Rows rows, thread = hidden unit.
// ---------------------------------------------------------------------------
template <int H>
__global__ void __launch_bounds__(H) dw1_kernel(int mb, const float* __restrict__ dH1, const float* __restrict__ H1,
                                                const float* __restrict__ saug, float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) float s[kW1Rows][20];
  const int r0 = blockIdx.x * kW1Rows;
  const int net = blockIdx.y;                                      // 0 actor, 1 critic
  const int t = threadIdx.x;
  for (int q = t; q < kW1Rows * 20; q += H) {
    const int r = q / 20, c = q % 20, row = r0 + r;
    s[r][c] = row < mb ? saug[(int64_t)row * 20 + c] : 0.0f;
  }
  float g[kW1Rows], y[kW1Rows];
  const int64_t base = (int64_t)net * mb;
#pragma unroll
  for (int r = 0; r < kW1Rows; ++r) {                              // all loads in flight together
    const int row = min(r0 + r, mb - 1);
    g[r] = dH1[(base + row) * H + t];
    y[r] = H1[(base + row) * H + t];
  }
  __syncthreads();
  float acc[20];
#pragma unroll
  for (int k = 0; k < 20; ++k) acc[k] = 0.0f;
#pragma unroll
  for (int r = 0; r < kW1Rows; ++r) {
    const float dz = (r0 + r < mb) ? g[r] * (1.0f - y[r] * y[r]) : 0.0f;   // tanh backward
#pragma unroll
    for (int k4 = 0; k4 < 5; ++k4) {
      const float4 sv = *reinterpret_cast<const float4*>(&s[r][4 * k4]);
      acc[4 * k4 + 0] = fmaf(dz, sv.x, acc[4 * k4 + 0]);
      acc[4 * k4 + 1] = fmaf(dz, sv.y, acc[4 * k4 + 1]);
      acc[4 * k4 + 2] = fmaf(dz, sv.z, acc[4 * k4 + 2]);
      acc[4 * k4 + 3] = fmaf(dz, sv.w, acc[4 * k4 + 3]);
    }
  }
  float4* pp = reinterpret_cast<float4*>(part + (int64_t)blockIdx.x * 2 * H * 20 + (int64_t)(net * H + t) * 20);
#pragma unroll
  for (int k = 0; k < 5; ++k) pp[k] = make_float4(acc[4 * k], acc[4 * k + 1], acc[4 * k + 2], acc[4 * k + 3]);
}

// ---------------------------------------------------------------------------
// head: ppo_continuous.py:216-239 per row, both nets.  Thread j = hidden unit.
// The output layers (3 actor dots + 1 critic dot per row over H) go through
// an LDS transpose: [2][kRows][H] activations, then 4 threads per (row,
// output) each sum H/4 products and finish with two xor-shuffles.
// ---------------------------------------------------------------------------
template <int H>
__global__ void __launch_bounds__(H) head_kernel(int mb, const float* __restrict__ Z2, const float* __restrict__ P,
                                                 const float* __restrict__ aux, float epsilon, float ent_coef,
                                                 float max_action, float* __restrict__ dZ2,
                                                 float* __restrict__ partials, float* __restrict__ row_loss) {
  const Layout L = layout(H);
  static_assert(H >= 64 && H % 64 == 0, "H");
  __shared__ __attribute__((aligned(16))) float hs[2][kRows][H];   // tanh(fc2) activations
  __shared__ __attribute__((aligned(16))) float w3s[4][H];          // W3a rows 0..2, W3c
  __shared__ float sums[kRows][4];
  __shared__ float dz3s[kRows][4];
  __shared__ float lsp[kRows][4];
  const int t = threadIdx.x;
  const int r0 = blockIdx.x * kRows;
  const float b2a = P[L.b2 + t], b2c = P[L.b2 + H + t];
  const float w30 = P[L.W3a + t], w31 = P[L.W3a + H + t], w32 = P[L.W3a + 2 * H + t];
  const float w3c = P[L.W3c + t];
  w3s[0][t] = w30; w3s[1][t] = w31; w3s[2][t] = w32; w3s[3][t] = w3c;
  float ha[kRows], hc[kRows];
#pragma unroll
  for (int r = 0; r < kRows; ++r) {                                  // all loads in flight together
    const int row = min(r0 + r, mb - 1);
    ha[r] = Z2[(int64_t)row * H + t];
    hc[r] = Z2[((int64_t)mb + row) * H + t];
  }
#pragma unroll
  for (int r = 0; r < kRows; ++r) {
    const bool ok = r0 + r < mb;
    ha[r] = ok ? tanhf(ha[r] + b2a) : 0.0f;                        // actor fc2 + tanh
    hc[r] = ok ? tanhf(hc[r] + b2c) : 0.0f;                        // critic fc2 + tanh
    hs[0][r][t] = ha[r];
    hs[1][r][t] = hc[r];
  }
  __syncthreads();
  // 64 (row, output) dots x 4 partial threads; H threads cover 64*4/H rounds
  for (int o4 = t; o4 < kRows * 4 * 4; o4 += H) {
    const int o = o4 >> 2, part = o4 & 3;
    const int r = o >> 2, q = o & 3;
    const float* hrow = &hs[q == 3 ? 1 : 0][r][part * (H / 4)];
    const float* wrow = &w3s[q][part * (H / 4)];
    float acc = 0.0f;
#pragma unroll 8
    for (int k = 0; k < H / 4; k += 4) {
      const float4 x = *reinterpret_cast<const float4*>(hrow + k);
      const float4 y = *reinterpret_cast<const float4*>(wrow + k);
      acc = fmaf(x.x, y.x, acc);
      acc = fmaf(x.y, y.y, acc);
      acc = fmaf(x.z, y.z, acc);
      acc = fmaf(x.w, y.w, acc);
    }
    acc += __shfl_xor(acc, 1, 64);
    acc += __shfl_xor(acc, 2, 64);
    if (part == 0) sums[r][q] = acc;
  }
  __syncthreads();
  if (t < kRows) {
    const int r = t, row = r0 + r;
    float dz[4] = {0.f, 0.f, 0.f, 0.f}, dls[4] = {0.f, 0.f, 0.f, 0.f};
    if (row < mb) {
      const float* ax = aux + (int64_t)row * 8;
      const float inv = 1.0f / (float)mb;
      float th[3], mu[3], dv[3], var[3], logp[3];
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        th[d] = tanhf(sums[r][d] + P[L.b3a + d]);
        mu[d] = max_action * th[d];                                  // 1.6 * tanh(mean_layer)
        const float sd = expf(P[L.ls + d]);
        var[d] = sd * sd;
        dv[d] = ax[d] - mu[d];
        logp[d] = (-(dv[d] * dv[d]) / (2.0f * var[d]) - logf(sd)) - kLogSqrt2Pi;
      }
      const float lsum = (logp[0] + logp[1]) + logp[2];
      const float lold = (ax[3] + ax[4]) + ax[5];
      const float ratio = expf(lsum - lold);
      const float adv = ax[6];
      const float s1 = ratio * adv;
      const float cr = fminf(fmaxf(ratio, 1.0f - epsilon), 1.0f + epsilon);
      const float s2 = cr * adv;
      // torch.min backward splits ties; clamp backward passes inside [lo, hi]
      const float g1 = s1 < s2 ? 1.0f : (s1 == s2 ? 0.5f : 0.0f);
      const float g2 = s2 < s1 ? 1.0f : (s1 == s2 ? 0.5f : 0.0f);
      const float inside = (ratio >= 1.0f - epsilon && ratio <= 1.0f + epsilon) ? 1.0f : 0.0f;
      const float dmin = -inv;
      const float dratio = dmin * g1 * adv + dmin * g2 * adv * inside;
      const float dlsum = dratio * ratio;
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        const float dmu = dlsum * (dv[d] / var[d]);
        dz[d] = (dmu * max_action) * (1.0f - th[d] * th[d]);
        dls[d] = dlsum * (dv[d] * dv[d] / var[d] - 1.0f) - ent_coef * inv;
      }
      const float vc = sums[r][3] + P[L.b3c];
      const float vt = ax[7];
      dz[3] = 2.0f * inv * (vc - vt);                                // d mse / d v
      if (row_loss) {
        float ent = 0.0f;
#pragma unroll
        for (int d = 0; d < 3; ++d) ent += 0.5f + 0.5f * 1.8378770664093453f + logf(expf(P[L.ls + d]));
        row_loss[(int64_t)row * 2 + 0] = -fminf(s1, s2) - ent_coef * ent;
        row_loss[(int64_t)row * 2 + 1] = (vt - vc) * (vt - vc);
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      dz3s[r][q] = dz[q];
      lsp[r][q] = dls[q];
    }
  }
  __syncthreads();
  float db2a = 0.f, db2c = 0.f, g30 = 0.f, g31 = 0.f, g32 = 0.f, g3c = 0.f;
#pragma unroll
  for (int r = 0; r < kRows; ++r) {
    const int row = r0 + r;
    const float d0 = dz3s[r][0], d1 = dz3s[r][1], d2 = dz3s[r][2], dc = dz3s[r][3];   // 0 past mb
    const float dha = (d0 * w30 + d1 * w31) + d2 * w32;            // dZ3 @ W3
    const float dza = dha * (1.0f - ha[r] * ha[r]);                // tanh backward
    const float dzc = (dc * w3c) * (1.0f - hc[r] * hc[r]);
    if (row < mb) {
      dZ2[(int64_t)row * H + t] = dza;
      dZ2[((int64_t)mb + row) * H + t] = dzc;
    }
    db2a += dza;
    db2c += dzc;
    g30 += d0 * ha[r];
    g31 += d1 * ha[r];
    g32 += d2 * ha[r];
    g3c += dc * hc[r];
  }
  float* part = partials + (int64_t)blockIdx.x * L.tail;           // tail-relative layout
  part[t] = db2a;
  part[H + t] = db2c;
  part[2 * H + t] = g30;
  part[3 * H + t] = g31;
  part[4 * H + t] = g32;
  part[5 * H + 8 + t] = g3c;
  if (t < 4) {
    float sb = 0.f, sl = 0.f, sc = 0.f;
    for (int r = 0; r < kRows; ++r) {
      sb += t < 3 ? dz3s[r][t] : 0.0f;
      sl += t < 3 ? lsp[r][t] : 0.0f;
      sc += t == 0 ? dz3s[r][3] : 0.0f;
    }
    part[5 * H + t] = sb;            // b3a
    part[5 * H + 4 + t] = sl;        // log_std
    part[6 * H + 8 + t] = sc;        // b3c
  }
}

__global__ void __launch_bounds__(256) tanh_bwd_kernel(int64_t n4, const float4* __restrict__ dh,
                                                       const float4* __restrict__ h, float4* __restrict__ dz) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const float4 g = dh[i], y = h[i];
    dz[i] = make_float4(g.x * (1.0f - y.x * y.x), g.y * (1.0f - y.y * y.y), g.z * (1.0f - y.z * y.z),
                        g.w * (1.0f - y.w * y.w));
  }
}

// block-level f64 pair sum in fixed order
__device__ __forceinline__ void block_sum2(double& a, double& c, double* sh) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    a += __shfl_xor(a, off, 64);
    c += __shfl_xor(c, off, 64);
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { sh[2 * w] = a; sh[2 * w + 1] = c; }
  __syncthreads();
  if (threadIdx.x == 0) {
    a = 0.0; c = 0.0;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) { a += sh[2 * k]; c += sh[2 * k + 1]; }
  }
  __syncthreads();
  if (threadIdx.x == 0) { sh[0] = a; sh[1] = c; }
  __syncthreads();
}

// ---------------------------------------------------------------------------
// reduce: sums the three partial-slab families into G (fixed order) and/or
// writes per-block squared norms per net.  Block ranges:
//   [0, nb2)          W2 region, 4 elements per thread, S split-K slabs [2][S][H][H]
//   [nb2, nb2+nb1)    W1 region, 64 elements x 4 chunks, nw1 slabs [nw1][2][H][20]
//   [nb2+nb1, ...)    tail, 8 elements x 32 chunks, nwg slabs [nwg][6H+12]
// ---------------------------------------------------------------------------
struct RedGeom { int nb2, nb1, nbt, S, nw1, nwg; };

template <int E, int CH>
__device__ __forceinline__ float chunk_sum(const float* __restrict__ part, int64_t stride, int nparts, int64_t el,
                                           bool valid, float (*sh)[CH + 1]) {
  const int t = threadIdx.x, e = t % E, c = t / E;
  float s = 0.0f;
  if (valid) {
#pragma unroll 8
    for (int w = c; w < nparts; w += CH) s += part[(int64_t)w * stride + el];
  }
  sh[e][c] = s;
  __syncthreads();
  float tot = 0.0f;
  if (c == 0) {
    for (int k = 0; k < CH; ++k) tot += sh[e][k];
  }
  __syncthreads();
  return tot;
}

__global__ void __launch_bounds__(256) reduce_kernel(int H, RedGeom g, int mode, const float* __restrict__ p2,
                                                     const float* __restrict__ p1, const float* __restrict__ pt,
                                                     float* __restrict__ G, double* __restrict__ nsq,
                                                     double* __restrict__ steps) {
  const Layout L = layout(H);
  __shared__ double sh[8];
  __shared__ float red[64][33];
  double sa = 0.0, sc = 0.0;
  const int t = threadIdx.x;
  const int64_t HH = (int64_t)H * H;
  int b = blockIdx.x;
  if (b < g.nb2) {                                                // W2: [2][S] slabs of H*H
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t e = (int64_t)b * 1024 + k * 256 + t;
      if (e < L.W1) {
        const int net = e >= HH;
        float v;
        if (mode & 1) {
          const int64_t i = e - net * HH;
          const float* q = p2 + (int64_t)net * g.S * HH + i;
          v = 0.0f;
          for (int s2 = 0; s2 < g.S; ++s2) v += q[(int64_t)s2 * HH];
          G[e] = v;
        } else {
          v = G[e];
        }
        if (net) sc += (double)v * v; else sa += (double)v * v;
      }
    }
  } else if ((b -= g.nb2) < g.nb1) {                             // W1: [nw1] slabs of 2*H*20
    const int64_t el = (int64_t)b * 64 + (t & 63);
    const bool valid = el < 2LL * H * 20;
    float v = 0.0f;
    if (mode & 1) {
      v = chunk_sum<64, 4>(p1, 2LL * H * 20, g.nw1, el, valid, (float(*)[5])red);
      if ((t >> 6) == 0 && valid) G[L.W1 + el] = v;
    } else if ((t >> 6) == 0 && valid) {
      v = G[L.W1 + el];
    }
    if ((t >> 6) == 0 && valid) {
      if (el >= (int64_t)H * 20) sc += (double)v * v; else sa += (double)v * v;
    }
  } else {                                                        // tail: [nwg] slabs of 6H+12
    b -= g.nb1;
    const int64_t el = (int64_t)b * 8 + (t & 7);
    const bool valid = el < L.tail;
    float v = 0.0f;
    if (mode & 1) {
      v = chunk_sum<8, 32>(pt, L.tail, g.nwg, el, valid, (float(*)[33])red);
      if ((t >> 3) == 0 && valid) G[L.b2 + el] = v;
    } else if ((t >> 3) == 0 && valid) {
      v = G[L.b2 + el];
    }
    if ((t >> 3) == 0 && valid) {
      if (net_of(L, L.b2 + el, H)) sc += (double)v * v; else sa += (double)v * v;
    }
  }
  if (mode & 2) {
    block_sum2(sa, sc, sh);
    if (t == 0) {
      nsq[2 * blockIdx.x] = sa;
      nsq[2 * blockIdx.x + 1] = sc;
      if (blockIdx.x == 0) { steps[0] += 1.0; steps[1] += 1.0; }
    }
  }
}

// ---------------------------------------------------------------------------
// adam: torch.nn.utils.clip_grad_norm_ + torch.optim.Adam (_single_tensor_adam)
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) adam_kernel(int H, int nblk, const double* __restrict__ nsq,
                                                   const double* __restrict__ steps, const double* __restrict__ bct,
                                                   int bct_len, const float* __restrict__ lr, float beta1,
                                                   float beta2, float eps, float max_norm, int use_clip,
                                                   const float* __restrict__ G, float* __restrict__ P,
                                                   float* __restrict__ M, float* __restrict__ V) {
  const Layout L = layout(H);
  __shared__ double sh[8];
  __shared__ float cst[2][3];                                      // coef, step_size, bc2_sqrt per net
  double a = 0.0, c = 0.0;
  for (int k = threadIdx.x; k < nblk; k += blockDim.x) { a += nsq[2 * k]; c += nsq[2 * k + 1]; }
  block_sum2(a, c, sh);
  if (threadIdx.x < 2) {
    const int n = threadIdx.x;
    const double nn = n == 0 ? sh[0] : sh[1];
    const float nrm = (float)sqrt(nn);
    cst[n][0] = use_clip ? fminf(max_norm / (nrm + 1e-6f), 1.0f) : 1.0f;
    // bct[2*step] = 1 - beta1**step, bct[2*step+1] = sqrt(1 - beta2**step) (python float
    // math, as torch.optim.Adam computes them); constant 1.0 past the table
    const int st = (int)steps[n];
    const double bc1 = st < bct_len ? bct[2 * st] : 1.0;
    const double bc2s = st < bct_len ? bct[2 * st + 1] : 1.0;
    cst[n][1] = (float)((double)lr[n] / bc1);
    cst[n][2] = (float)bc2s;
  }
  __syncthreads();
  const float w1 = (float)(1.0 - (double)beta1);                  // lerp weight 1 - beta1
  const float w2 = (float)(1.0 - (double)beta2);
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < L.total; e += (int64_t)gridDim.x * blockDim.x) {
    const int net = net_of(L, e, H);
    float g = G[e];
    if (use_clip) g = g * cst[net][0];                             // grads.mul_(clip_coef_clamped)
    float m = M[e];
    m = m + w1 * (g - m);                                          // exp_avg.lerp_(grad, 1 - beta1)
    float v = V[e];
    v = v * beta2 + w2 * (g * g);                                  // mul_(beta2).addcmul_(g, g, 1 - beta2)
    const float denom = sqrtf(v) / cst[net][2] + eps;
    P[e] = P[e] + (-cst[net][1]) * (m / denom);                    // addcdiv_(m, denom, -step_size)
    M[e] = m;
    V[e] = v;
  }
}

int n_head_wg(int mb) { return (mb + kRows - 1) / kRows; }
int n_w1_wg(int mb) { return (mb + kW1Rows - 1) / kW1Rows; }
RedGeom geom(int H, int mb, int S) {
  const Layout L = layout(H);
  RedGeom g;
  g.nb2 = (int)((L.W1 + 1023) / 1024);
  g.nb1 = (int)((2LL * H * 20 + 63) / 64);
  g.nbt = (int)((L.tail + 7) / 8);
  g.S = S;
  g.nw1 = n_w1_wg(mb);
  g.nwg = n_head_wg(mb);
  return g;
}
int n_blocks(const RedGeom& g) { return g.nb2 + g.nb1 + g.nbt; }

bool valid_h(int H) { return H == 64 || H == 128 || H == 256; }

#define LAUNCH_CHECK()                                                      \
  do {                                                                      \
    hipError_t e_ = hipGetLastError();                                      \
    if (e_ != hipSuccess) { g_err = hipGetErrorString(e_); return -2; }     \
  } while (0)

}  // namespace

extern "C" {

int satrl_ppo_layout(int H, int64_t* off) {
  if (!valid_h(H) || !off) return -1;
  const Layout L = layout(H);
  off[SATRL_PPO_OFF_W2] = L.W2;
  off[SATRL_PPO_OFF_W1] = L.W1;
  off[SATRL_PPO_OFF_B2] = L.b2;
  off[SATRL_PPO_OFF_W3A] = L.W3a;
  off[SATRL_PPO_OFF_B3A] = L.b3a;
  off[SATRL_PPO_OFF_LS] = L.ls;
  off[SATRL_PPO_OFF_W3C] = L.W3c;
  off[SATRL_PPO_OFF_B3C] = L.b3c;
  off[SATRL_PPO_TOTAL] = L.total;
  return 0;
}

int satrl_ppo_sizes(int H, int mb, int64_t* nwg, int64_t* nblk) {
  if (!valid_h(H) || mb <= 0) return -1;
  if (nwg) *nwg = n_head_wg(mb);
  if (nblk) *nblk = n_blocks(geom(H, mb, 1));
  return 0;
}

int satrl_ppo_w1_chunks(int mb) { return mb > 0 ? n_w1_wg(mb) : -1; }

int satrl_ppo_dw1(int H, int mb, const float* dH1, const float* H1, const float* saug, float* part, void* stream) {
  if (!valid_h(H) || mb <= 0 || !dH1 || !H1 || !saug || !part) return -1;
  dim3 gr(n_w1_wg(mb), 2);
  hipStream_t s = (hipStream_t)stream;
  if (H == 64) hipLaunchKernelGGL(dw1_kernel<64>, gr, dim3(64), 0, s, mb, dH1, H1, saug, part);
  else if (H == 128) hipLaunchKernelGGL(dw1_kernel<128>, gr, dim3(128), 0, s, mb, dH1, H1, saug, part);
  else hipLaunchKernelGGL(dw1_kernel<256>, gr, dim3(256), 0, s, mb, dH1, H1, saug, part);
  LAUNCH_CHECK();
  return 0;
}

int satrl_ppo_fwd1(int H, int mb, const float* src, const int64_t* idx, const float* P, float* H1, float* saug,
                   float* aux, void* stream) {
  if (!valid_h(H) || mb <= 0 || !src || !idx || !P || !H1 || !saug || !aux) return -1;
  dim3 g((mb + kF1Rows - 1) / kF1Rows);
  hipStream_t s = (hipStream_t)stream;
  if (H == 64) hipLaunchKernelGGL(fwd1_kernel<64>, g, dim3(64), 0, s, mb, src, idx, P, H1, saug, aux);
  else if (H == 128) hipLaunchKernelGGL(fwd1_kernel<128>, g, dim3(128), 0, s, mb, src, idx, P, H1, saug, aux);
  else hipLaunchKernelGGL(fwd1_kernel<256>, g, dim3(256), 0, s, mb, src, idx, P, H1, saug, aux);
  LAUNCH_CHECK();
  return 0;
}

int satrl_ppo_head(int H, int mb, const float* Z2, const float* P, const float* aux, float epsilon, float ent_coef,
                   float max_action, float* dZ2, float* partials, float* row_loss, void* stream) {
  if (!valid_h(H) || mb <= 0 || !Z2 || !P || !aux || !dZ2 || !partials) return -1;
  dim3 g(n_head_wg(mb));
  hipStream_t s = (hipStream_t)stream;
  if (H == 64)
    hipLaunchKernelGGL(head_kernel<64>, g, dim3(64), 0, s, mb, Z2, P, aux, epsilon, ent_coef, max_action, dZ2,
                       partials, row_loss);
  else if (H == 128)
    hipLaunchKernelGGL(head_kernel<128>, g, dim3(128), 0, s, mb, Z2, P, aux, epsilon, ent_coef, max_action, dZ2,
                       partials, row_loss);
  else
    hipLaunchKernelGGL(head_kernel<256>, g, dim3(256), 0, s, mb, Z2, P, aux, epsilon, ent_coef, max_action, dZ2,
                       partials, row_loss);
  LAUNCH_CHECK();
  return 0;
}

int satrl_ppo_tanh_bwd(int64_t n, const float* dH1, const float* H1, float* dZ1, void* stream) {
  if (n <= 0 || (n & 3) || !dH1 || !H1 || !dZ1) return -1;
  const int64_t n4 = n / 4;
  int64_t blocks = (n4 + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(tanh_bwd_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, n4,
                     (const float4*)dH1, (const float4*)H1, (float4*)dZ1);
  LAUNCH_CHECK();
  return 0;
}

int satrl_ppo_reduce(int H, int mb, int S, int mode, const float* p2, const float* p1, const float* pt, float* G,
                     double* nsq, double* steps, void* stream) {
  if (!valid_h(H) || mb <= 0 || S < 1 || mode < 1 || mode > 3 || !G) return -1;
  if ((mode & 1) && (!p2 || !p1 || !pt)) return -1;
  if ((mode & 2) && (!nsq || !steps)) return -1;
  const RedGeom g = geom(H, mb, S);
  hipLaunchKernelGGL(reduce_kernel, dim3(n_blocks(g)), dim3(256), 0, (hipStream_t)stream, H, g, mode, p2, p1, pt, G,
                     nsq, steps);
  LAUNCH_CHECK();
  return 0;
}

int satrl_ppo_adam(int H, int mb, const double* nsq, const double* steps, const double* bct, int bct_len,
                   const float* lr, float beta1, float beta2, float eps, float max_norm, int use_clip, const float* G,
                   float* P, float* M, float* V, void* stream) {
  if (!valid_h(H) || mb <= 0 || !nsq || !steps || !bct || bct_len < 1 || !lr || !G || !P || !M || !V) return -1;
  const Layout L = layout(H);
  const int nblk = n_blocks(geom(H, mb, 1));
  const int blocks = (int)((L.total + 1023) / 1024);
  hipLaunchKernelGGL(adam_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, H, nblk, nsq, steps, bct, bct_len,
                     lr, beta1, beta2, eps, max_norm, use_clip, G, P, M, V);
  LAUNCH_CHECK();
  return 0;
}

const char* satrl_ppo_last_error(void) { return g_err.c_str(); }

}  // extern "C"
