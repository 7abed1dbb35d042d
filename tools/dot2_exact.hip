// development probe (not shipped): is x - bf16(x) exact through v_dot2c_f32_bf16 with SGPR constants?
// Classes: random magnitudes 2^-30..2^9 (the split's operands), then (round 6)
// signed zeros, f32 denormals, magnitudes 2^100..FLT_MAX (bf16 rounding to
// inf), and inf / NaN in one lane of a pair with a finite neighbour (does the
// neighbour's residual stay finite?).  NaN results compare equal to NaN.
// build: hipcc --offload-arch=gfx950 -O2 -o tools/_probe/dot2_exact tools/dot2_exact.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cmath>
typedef __bf16 bf2v __attribute__((ext_vector_type(2)));
typedef float f2v __attribute__((ext_vector_type(2)));
__global__ void k(const float* in, float* out, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (2 * i + 1 >= n) return;
  f2v x{in[2 * i], in[2 * i + 1]};
  unsigned p = __builtin_bit_cast(unsigned, __builtin_convertvector(x, bf2v));
  const bf2v pv = __builtin_bit_cast(bf2v, p);
  unsigned c0, c1;
  asm("s_mov_b32 %0, %1" : "=s"(c0) : "i"(0x0000bf80u));
  asm("s_mov_b32 %0, %1" : "=s"(c1) : "i"(0xbf800000u));
  out[2 * i] = __builtin_amdgcn_fdot2_f32_bf16(pv, __builtin_bit_cast(bf2v, c0), x.x, false);
  out[2 * i + 1] = __builtin_amdgcn_fdot2_f32_bf16(pv, __builtin_bit_cast(bf2v, c1), x.y, false);
}
static float bf16_rne_host(float x) {
  unsigned u; memcpy(&u, &x, 4);
  unsigned r = u + 0x7fff + ((u >> 16) & 1);
  r &= 0xffff0000u; float y; memcpy(&y, &r, 4); return y;
}
static float from_bits(unsigned u) { float f; memcpy(&f, &u, 4); return f; }
static float rnd_u() { return (rand() + 0.5f) / (RAND_MAX + 1.0f); }
static float sgn() { return rand() & 1 ? -1.f : 1.f; }
int main() {
  const int n = 1 << 22, nc = 5;
  const char* names[nc] = {"random 2^-30..2^9", "signed zeros", "denormals", "2^100..FLT_MAX", "inf/NaN beside finite"};
  float* h = (float*)malloc(n * 4); float* o = (float*)malloc(n * 4);
  srand(1);
  const int per = n / nc & ~1;
  for (int i = 0; i < n; ++i) {
    const int c = i / per < nc ? i / per : nc - 1;
    float x;
    if (c == 0) x = sgn() * rnd_u() * powf(2.f, (float)((rand() % 40) - 30));
    else if (c == 1) x = sgn() * 0.0f;
    else if (c == 2) x = sgn() * from_bits(1u + (unsigned)rand() % 0x7fffffu);
    else if (c == 3) x = sgn() * from_bits((227u << 23) + (unsigned)rand() % ((254u - 227u) << 23 | 0x7fffffu));
    else x = (i & 1) ? sgn() * rnd_u() : (rand() & 1 ? sgn() * INFINITY : NAN);   // even lane special, odd lane finite
    h[i] = x;
  }
  float *di, *dout; hipMalloc(&di, n * 4); hipMalloc(&dout, n * 4);
  hipMemcpy(di, h, n * 4, hipMemcpyHostToDevice);
  k<<<n / 2 / 256, 256>>>(di, dout, n);
  hipMemcpy(o, dout, n * 4, hipMemcpyDeviceToHost);
  int bad[nc] = {0}, cnt[nc] = {0}, shown = 0, nbr_nonfinite = 0;
  for (int i = 0; i < n; ++i) {
    const int c = i / per < nc ? i / per : nc - 1;
    ++cnt[c];
    const float want = h[i] - bf16_rne_host(h[i]);
    const bool eq = (std::isnan(want) && std::isnan(o[i])) || !memcmp(&want, &o[i], 4);
    if (c == 4 && (i & 1) && !std::isfinite(o[i])) ++nbr_nonfinite;
    if (!eq) {
      if (shown++ < 12) printf("[%s] x=%a want=%a got=%a\n", names[c], h[i], want, o[i]);
      ++bad[c];
    }
  }
  for (int c = 0; c < nc; ++c) printf("%-22s mismatches %d of %d\n", names[c], bad[c], cnt[c]);
  printf("finite neighbours of inf/NaN with a non-finite residual: %d of %d\n", nbr_nonfinite, cnt[4] / 2);
  return 0;
}
