// development probe (not shipped): is x - bf16(x) exact through v_dot2c_f32_bf16 with SGPR constants?
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
int main() {
  const int n = 1 << 22;
  float* h = (float*)malloc(n * 4); float* o = (float*)malloc(n * 4);
  srand(1);
  for (int i = 0; i < n; ++i) {
    float u = (rand() + 0.5f) / (RAND_MAX + 1.0f);
    float e = (float)((rand() % 40) - 30);
    h[i] = (rand() & 1 ? -1.f : 1.f) * u * powf(2.f, e);
  }
  float *di, *dout; hipMalloc(&di, n * 4); hipMalloc(&dout, n * 4);
  hipMemcpy(di, h, n * 4, hipMemcpyHostToDevice);
  k<<<n / 2 / 256, 256>>>(di, dout, n);
  hipMemcpy(o, dout, n * 4, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < n; ++i) {
    float want = h[i] - bf16_rne_host(h[i]);
    if (memcmp(&want, &o[i], 4)) {
      if (bad < 12) printf("x=%a want=%a got=%a (rel %.3g)\n", h[i], want, o[i], want ? fabs((o[i] - want) / want) : 0.0);
      ++bad;
    }
  }
  printf("mismatches %d of %d\n", bad, n);
  return 0;
}
