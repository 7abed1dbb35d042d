// ppo_kernels.hip -- fused PPO minibatch-step kernels for gfx950 (include/satrl_ppo.h).
//
// Per minibatch (actor + critic together, same rows), four launches:
//   rowpass  gather, fc1, fc2 (f32 MFMA), output layers, losses, backprop to
//            dZ2 and through fc2 (f32 MFMA) and fc1's tanh; writes H1, dZ2
//            and partial slabs of every small gradient
//   dW2      dZ2^T @ H1 split-K S ways: fused into the rowpass (H <= 128, rowpass_dw2), from the
//            rowpass's k-packed bf16 planes (H = 256, dw2_kx_kernel), or dw2_kernel on f32 rows
//   reduce   partial slabs -> G (fixed order), per-block squared norms per net
//   adam     clip coefficient per net + Adam (torch single-tensor formula),
//            also refreshes fc2.weight^T used by the next rowpass
// Every reduction has a fixed order, so a step is bitwise reproducible.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstring>
#include <cstdlib>
#include <mutex>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "philox_device.h"
#include "span_probe.h"
#include "satrl_ppo.h"
#include "satrl_peer.h"

namespace {

thread_local std::string g_err;

#ifdef SATRL_PHASE_PROBE
// development-only phase stamps (tools/_probe/phase_probe.py), never in the
// shipped build: [workgroup][stamp][wave][s_memrealtime, s_memtime]
__device__ unsigned long long g_probe[512][16][16][2];
#define PHASE_PROBE(k)                                                        \
  do {                                                                        \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 512) {                        \
      g_probe[blockIdx.x][k][threadIdx.x >> 6][0] = wall_clock64();           \
      g_probe[blockIdx.x][k][threadIdx.x >> 6][1] = clock64();                \
    }                                                                         \
  } while (0)
#else
#define PHASE_PROBE(k) do {} while (0)
#endif

constexpr int kRows = 32;     // minibatch rows per rowpass workgroup (and per partial slab)
constexpr int kNW256 = 16;    // waves per rowpass workgroup at H = 256
// short minibatches at H = 256 (configs[3]: 512 rows per rank; ragged tails)
// run 16-row workgroups of the same 16 waves, one 16-row tile each: twice the
// workgroups on the chip, and every row's arithmetic -- the forward's MFMA
// order and output-layer sums included -- is the 32-row kernel's
constexpr int kRowsShort = 16;

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
// rowpass: the whole row-parallel part of a minibatch step in one launch.
// The actor and critic losses are independent given (adv, v_target), so a
// workgroup owns ONE net (blockIdx & 1; with round-robin dispatch the actor
// lands on the even XCDs, the critic on the odd ones) and 32 minibatch rows
// (blockIdx >> 1).  Its NW waves split the hidden columns: wave w owns
// CT = H/16/NW tiles of 16 columns for both 16-row tiles.  Every CU thus
// streams one net's fc2 weights per phase (256 KB at H=256) for 32 rows:
// the two MFMA phases are L2->CU ingest bound.
//   A  gather rows -> S (LDS); Z1 = [S|1] W1aug^T       f32 MFMA 16x16x4
//   B  Z2 = tanh(Z1) W2^T                               f32 MFMA, W2 from L2
//   C  tanh(fc2), output layer(s), the net's loss, dZ2 -> LDS/HBM, tail partials
//   D  dH1 = dZ2 W2 (rows of W2T = fc2.weight^T)        f32 MFMA
//   E  dZ1 = dH1 (1 - H1^2); [dW1|db1] = dZ1^T [S|1]    f32 MFMA, dZ1's
//      accumulator layout is already the A operand
// Accumulator layout of a 16x16x4 tile: acc[rt][ct][j] = D[row 16rt + 4lg + j]
// [col n0 + 16ct + li].  Inside a 32-wide k chunk lane group g takes
// k = 32c + 8g + kk (kk < 8): every B fetch is a 32-B run of a 128-B line and
// A comes as 2 ds_read_b128 per row tile from rows padded by 16 B.
// Partial slabs are per 32-row block: the actor and critic workgroups of a
// block write disjoint parts of the same slab.
// ---------------------------------------------------------------------------
using f4 = __attribute__((ext_vector_type(4))) float;

__device__ __forceinline__ f4 mfma4(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// sum over the 16 lanes of a DPP row (lanes 16k .. 16k+15), result in every
// lane of the row: xor-1 and xor-2 quad permutes, then half-row and row
// mirrors -- VALU DPP, no LDS traffic (ds_bpermute chains were the slowest
// part of the output-layer dot products).  Fixed order, so deterministic.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_f<0xB1>(v);    // quad_perm [1,0,3,2]
  v += dpp_f<0x4E>(v);    // quad_perm [2,3,0,1]
  v += dpp_f<0x141>(v);   // row_half_mirror
  v += dpp_f<0x140>(v);   // row_mirror
  return v;
}
// v + v[lane ^ 16] and v + v[lane ^ 32] by the gfx950 permlane swaps (VALU,
// no ds_bpermute round trip); fp addition commutes, so every lane's bits are
// those of v + __shfl_xor(v, 16 / 32)
__device__ __forceinline__ float xor16_sum(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float xor32_sum(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// row16_sum of NV values stage by stage: NV independent DPP adds between
// dependent ones, so no DPP read-after-write s_nop is needed (value-major
// order left ~90 of them in phase C); every value's ops and order are the
// same as row16_sum's, so the sums are bitwise identical
template <int NV>
__device__ __forceinline__ void row16_sum_n(float (&v)[NV]) {
#pragma unroll
  for (int q = 0; q < NV; ++q) v[q] += dpp_f<0xB1>(v[q]);
#pragma unroll
  for (int q = 0; q < NV; ++q) v[q] += dpp_f<0x4E>(v[q]);
#pragma unroll
  for (int q = 0; q < NV; ++q) v[q] += dpp_f<0x141>(v[q]);
#pragma unroll
  for (int q = 0; q < NV; ++q) v[q] += dpp_f<0x140>(v[q]);
}

// tanh of the MLP activations (fc1, fc2, mean layer).  The split of Cephes
// tanhf: |x| < 0.625 an odd minimax polynomial, else 1 - 2/(e^{2|x|} + 1) on
// the hardware v_exp_f32 / v_rcp_f32; both arms straight-line, then a select.
// Within 2 ulp of the correctly rounded tanh over every f32 (GPU test
// test_tanh_f32_ulp, exhaustive), in ~15 VALU ops where the library tanhf's
// accurate exp and IEEE division take ~3x that.  Every MLP kernel (rollout
// policy/value, update rowpass) calls this one function, so logp_old from the
// rollout still equals the update's recomputation bit for bit.
__device__ __forceinline__ float tanh_f32(float x) {
  const float y = fabsf(x), z = x * x;
  float p = fmaf(-5.70498872745e-3f, z, 2.06390887954e-2f);
  p = fmaf(p, z, -5.37397155531e-2f);
  p = fmaf(p, z, 1.33314422036e-1f);
  p = fmaf(p, z, -3.33332819422e-1f);
  const float small = fmaf(p * z, x, x);
  const float e = __builtin_amdgcn_exp2f(y * 2.8853900817779268f);        // e^{2|x|}; inf -> rcp 0 -> 1
  const float big = fmaf(-2.0f, __builtin_amdgcn_rcpf(e + 1.0f), 1.0f);
  return y < 0.625f ? small : copysignf(big, x);                          // NaN -> big arm -> NaN
}

// The k mapping of a 32-wide chunk (fc2 / dH1 phases): lane group g holds
// k = 8g + 4h + e, each lane's two float4 adjacent, so a wave-instruction
// touches every 128-B row segment at a 32-B stride (k = 16h + 4g + e, 64
// contiguous bytes per float4 instruction, measured no faster: EXPERIMENTS.md
// round 3).  Rollout and update share the mapping, hence the f32 rounding.
constexpr int kGOff = 8;   // floats between lane groups
constexpr int kHOff = 4;   // floats between a lane's two float4

template <int CT, int HOFF = kHOff>
__device__ __forceinline__ void b_chunk(const float* __restrict__ bp, int LDB, float4 (&b)[CT][2]) {
#pragma unroll
  for (int t = 0; t < CT; ++t) {
    b[t][0] = *reinterpret_cast<const float4*>(bp + 16 * t * LDB);
    b[t][1] = *reinterpret_cast<const float4*>(bp + 16 * t * LDB + HOFF);
  }
  __builtin_amdgcn_sched_barrier(0);   // keep the prefetch where it is issued
}

template <int LDA, int RT, int CT, int HOFF = kHOff>
__device__ __forceinline__ void mfma_chunk(const float* __restrict__ ap, const float4 (&b)[CT][2],
                                           f4 (&acc)[RT][CT]) {
  float4 a[RT][2];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    a[rt][0] = *reinterpret_cast<const float4*>(ap + 16 * rt * LDA);
    a[rt][1] = *reinterpret_cast<const float4*>(ap + 16 * rt * LDA + HOFF);
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int t = 0; t < CT; ++t) acc[rt][t] = mfma4(a[rt][h][e], b[t][h][e], acc[rt][t]);
    }
  }
}

// the LDS A operand of one 32-wide k chunk, and the chunk's MFMAs on operands
// already in registers
template <int LDA, int RT>
__device__ __forceinline__ void a_chunk(const float* __restrict__ ap, float4 (&a)[RT][2]) {
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    a[rt][0] = *reinterpret_cast<const float4*>(ap + 16 * rt * LDA);
    a[rt][1] = *reinterpret_cast<const float4*>(ap + 16 * rt * LDA + kHOff);
  }
  __builtin_amdgcn_sched_barrier(0);
}
template <int RT, int CT>
__device__ __forceinline__ void mfma_regs(const float4 (&a)[RT][2], const float4 (&b)[CT][2], f4 (&acc)[RT][CT]) {
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int t = 0; t < CT; ++t) acc[rt][t] = mfma4(a[rt][h][e], b[t][h][e], acc[rt][t]);
}

// acc[rt][t] += A[16rt.. +16][K] (LDS, row stride LDA) x B^T with B[n][k]
// row-major (ld LDB) for columns n0 + 16t, in 32-wide k chunks.  Without
// APRE (the policy kernel): chunk pairs with two register buffers in a rolled
// loop (prefetch distance one chunk), loads unconditional and the last pair
// peeled, so every vmcnt wait is exact.  APRE (the rowpass): the LDS A chunk
// is double-buffered too, so a chunk's MFMAs do not start behind a fresh
// ds_read's latency (34.7 -> 33.6 us), and B runs kBPD chunks ahead.  Its
// registers are what the policy kernel's occupancy does not afford (54 VGPRs
// allow two 16-wave workgroups per CU; APRE: 59 -> 63 us per rollout step, B
// two ahead alone: 64 us).  The MFMA sequence, hence every result bit, is the
// same on every path.
// APRE path: B chunks kBPD ahead (kBPD + 1 register buffers; distance 2
// measured best: 30.7 us per rowpass against 32.5 at 1, 31.0 at 3, 31.7 at 4).
// The first kBPD chunks can be issued early, before the phase's barrier, into
// a WPre (mfma_rows_pre), and handed to mfma_rows<..., PRE = true> (phase D:
// 30.4 -> 29.8 us; the same for phase B measured no gain).
constexpr int kBPD = 2;
template <int CT>
struct WPre {
  float4 bb[kBPD][CT][2];
};
template <int LDB, int CT>
__device__ __forceinline__ void mfma_rows_pre(const float* __restrict__ B, int n0, WPre<CT>& pre) {
  const int l = threadIdx.x & 63, i = l & 15, g = l >> 4;
  const float* bp = B + (int64_t)(n0 + i) * LDB + kGOff * g;
  constexpr int BPD = kBPD < LDB / 32 ? kBPD : LDB / 32;      // (K = LDB here: W2 / W2T rows)
#pragma unroll
  for (int c = 0; c < BPD; ++c) b_chunk<CT>(bp + 32 * c, LDB, pre.bb[c]);
}

template <int K, int LDA, int LDB, int RT, int CT, bool APRE, bool PRE = false>
__device__ __forceinline__ void mfma_rows(const float* __restrict__ A, const float* __restrict__ B, int n0,
                                          f4 (&acc)[RT][CT], const WPre<CT>* pre = nullptr) {
  constexpr int NC = K / 32;
  constexpr int BPD = kBPD < NC ? kBPD : NC;                     // prefetch distance in chunks
  static_assert(NC % 2 == 0, "chunk pairs");
  static_assert(APRE || !PRE, "early-issued chunks feed the APRE path");
  const int l = threadIdx.x & 63, i = l & 15, g = l >> 4;
  const float* ap = A + i * LDA + kGOff * g;
  const float* bp = B + (int64_t)(n0 + i) * LDB + kGOff * g;
  if constexpr (APRE) {
    // fully unrolled so every buffer index is static
    constexpr int NB = BPD + 1;
    float4 bb[NB][CT][2], aa[2][RT][2];
    if constexpr (PRE) {
#pragma unroll
      for (int c = 0; c < BPD; ++c)
#pragma unroll
        for (int t = 0; t < CT; ++t) { bb[c][t][0] = pre->bb[c][t][0]; bb[c][t][1] = pre->bb[c][t][1]; }
    } else {
#pragma unroll
      for (int c = 0; c < BPD; ++c) b_chunk<CT>(bp + 32 * c, LDB, bb[c]);
    }
    a_chunk<LDA, RT>(ap, aa[0]);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      if (c + BPD < NC) b_chunk<CT>(bp + 32 * (c + BPD), LDB, bb[(c + BPD) % NB]);
      if (c + 1 < NC) a_chunk<LDA, RT>(ap + 32 * (c + 1), aa[(c + 1) % 2]);
      mfma_regs<RT, CT>(aa[c % 2], bb[c % NB], acc);
    }
  } else {
    float4 x[CT][2], y[CT][2];
    b_chunk<CT>(bp, LDB, x);
#pragma unroll 1
    for (int c = 0; c < NC - 2; c += 2) {
      b_chunk<CT>(bp + 32 * (c + 1), LDB, y);
      mfma_chunk<LDA, RT, CT>(ap + 32 * c, x, acc);
      b_chunk<CT>(bp + 32 * (c + 2), LDB, x);
      mfma_chunk<LDA, RT, CT>(ap + 32 * (c + 1), y, acc);
    }
    b_chunk<CT>(bp + 32 * (NC - 1), LDB, y);
    mfma_chunk<LDA, RT, CT>(ap + 32 * (NC - 2), x, acc);
    mfma_chunk<LDA, RT, CT>(ap + 32 * (NC - 1), y, acc);
  }
}

// ---------------------------------------------------------------------------
// fc2 products at H = 256 as three-way bf16 splits (kBf3): gfx950 has no
// reduced-precision f32 MFMA, and v_mfma_f32_16x16x4_f32 issues 2048 FLOP per
// 32 cycles where v_mfma_f32_16x16x32_bf16 issues 16384 per 16.  Every f32
// operand x is split x = hi + mid + lo exactly (round-to-nearest bf16 splits:
// each residual is exact in f32 and the last one fits bf16's 8 bits), and a
// product is the six partial products whose magnitude reaches f32's
// rounding (lo*hi, hi*lo, mid*mid, mid*hi, hi*mid, hi*hi, smallest first;
// the dropped mid*lo, lo*mid, lo*lo are below 2^-24 of it), each exact in the
// MFMA's f32 accumulator.  Measured (tools/bf16x3_probe.hip, K = 256): error
// / sum|a*b| max 2.2e-7, mean 1.3e-8 against 2.9e-7 / 1.7e-8 for the f32
// MFMA chain.  The A operand (activations, written once per row block) goes
// to LDS as three bf16 planes; the B operand (fc2.weight / its transpose,
// read once per workgroup from L2) stays f32 and is split in registers, 36
// VALU per 32-wide k chunk beside its 12 MFMAs.  The 16x16x32 operand layout
// (lane l: row / column l & 15, k = 8 (l >> 4) + j) is the f32 path's k
// mapping, and its accumulator layout the 16x16x4's, so nothing else changes.
// ---------------------------------------------------------------------------
template <int H>
inline constexpr bool kBf3 = H == 256;
typedef short s8v __attribute__((ext_vector_type(8)));   // 8 bf16: a 16x16x32 operand (4 VGPRs)

__device__ __forceinline__ unsigned short bf16_rne(float x) { return __builtin_bit_cast(unsigned short, (__bf16)x); }
__device__ __forceinline__ float bf16_up(unsigned short h) { return __uint_as_float((unsigned)h << 16); }
// x = hi + mid + lo exactly
__device__ __forceinline__ void split3(float x, unsigned short& h, unsigned short& m, unsigned short& l) {
  h = bf16_rne(x);
  const float r = x - bf16_up(h);
  m = bf16_rne(r);
  const float q = r - bf16_up(m);
  l = bf16_rne(q);
}
typedef float f2v __attribute__((ext_vector_type(2)));
typedef __bf16 bf2v __attribute__((ext_vector_type(2)));
typedef unsigned u4v __attribute__((ext_vector_type(4)));
// two f32 -> one dword of two bf16 (v_cvt_pk_bf16_f32, round to nearest even), and back
__device__ __forceinline__ unsigned pk_bf16(f2v x) { return __builtin_bit_cast(unsigned, __builtin_convertvector(x, bf2v)); }
__device__ __forceinline__ f2v unpk_bf16(unsigned p) {
  return f2v{__uint_as_float(p << 16), __uint_as_float(p & 0xffff0000u)};
}
// x - (the bf16 pair p, widened), per lane half, as one v_dot2c_f32_bf16 each
// (p . (-1, 0) + x.x and p . (0, -1) + x.y): the difference is exact in f32
// (p is x rounded to bf16), so the dot's single rounding returns it unchanged
// -- two VALU where widening p and a packed subtraction take three
// The (-1, 0) / (0, -1) operands go through SGPRs: the compiler encodes
// (-1, 0) as the inline constant -1.0, which the instruction reads as the f32
// pattern (0, -1) -- the wrong half (tools/dot2_exact.hip).
__device__ __forceinline__ bf2v sgpr_bf16x2(unsigned bits) {
  unsigned r;
  asm("s_mov_b32 %0, %1" : "=s"(r) : "i"(bits));
  return __builtin_bit_cast(bf2v, r);
}
__device__ __forceinline__ f2v resid_bf16(f2v x, unsigned p) {
  const bf2v pv = __builtin_bit_cast(bf2v, p);
  return f2v{__builtin_amdgcn_fdot2_f32_bf16(pv, sgpr_bf16x2(0x0000bf80u), x.x, false),
             __builtin_amdgcn_fdot2_f32_bf16(pv, sgpr_bf16x2(0xbf800000u), x.y, false)};
}
// split3 on a pair, packed: 7 VALU per pair (3 v_cvt_pk_bf16_f32, 4 v_dot2c_f32_bf16)
__device__ __forceinline__ void split3x2(f2v x, unsigned& h, unsigned& m, unsigned& l) {
  h = pk_bf16(x);
  const f2v r = resid_bf16(x, h);
  m = pk_bf16(r);
  const f2v q = resid_bf16(r, m);
  l = pk_bf16(q);
}
__device__ __forceinline__ void split3x8(const float4 (&x)[2], s8v (&o)[3]) {
  unsigned h[4], m[4], l[4];
  split3x2(f2v{x[0].x, x[0].y}, h[0], m[0], l[0]);
  split3x2(f2v{x[0].z, x[0].w}, h[1], m[1], l[1]);
  split3x2(f2v{x[1].x, x[1].y}, h[2], m[2], l[2]);
  split3x2(f2v{x[1].z, x[1].w}, h[3], m[3], l[3]);
  o[0] = __builtin_bit_cast(s8v, u4v{h[0], h[1], h[2], h[3]});
  o[1] = __builtin_bit_cast(s8v, u4v{m[0], m[1], m[2], m[3]});
  o[2] = __builtin_bit_cast(s8v, u4v{l[0], l[1], l[2], l[3]});
}
__device__ __forceinline__ f4 mfma_bf16(s8v a, s8v b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
// the six partial products of one 16x16 tile and 32-wide k chunk, smallest first
__device__ __forceinline__ f4 mfma6(const s8v (&a)[3], const s8v (&bs)[3], f4 c) {
  c = mfma_bf16(a[2], bs[0], c);
  c = mfma_bf16(a[0], bs[2], c);
  c = mfma_bf16(a[1], bs[1], c);
  c = mfma_bf16(a[1], bs[0], c);
  c = mfma_bf16(a[0], bs[1], c);
  return mfma_bf16(a[0], bs[0], c);
}
// one 32-wide k chunk: A planes (registers) x B (f32, split here)
template <int RT, int CT>
__device__ __forceinline__ void mfma3_regs(const s8v (&a)[RT][3], const float4 (&b)[CT][2], f4 (&acc)[RT][CT]) {
#pragma unroll
  for (int t = 0; t < CT; ++t) {
    s8v bs[3];
    split3x8(b[t], bs);
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) acc[rt][t] = mfma6(a[rt], bs, acc[rt][t]);
  }
}
template <int LDP, int PS, int RT>
__device__ __forceinline__ void a3_chunk(const unsigned short* __restrict__ ap, s8v (&a)[RT][3]) {
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int p = 0; p < 3; ++p) a[rt][p] = *reinterpret_cast<const s8v*>(ap + p * PS + 16 * rt * LDP);
  __builtin_amdgcn_sched_barrier(0);
}
// mfma_rows (APRE path) on the split operands: A = three bf16 planes in LDS
// (row stride LDP, plane stride PS elements), B f32 row-major (ld LDB) as
// there, kBPD chunks ahead, its first chunks optionally issued early (pre)
constexpr int kBPD3 = 2;          // B chunks in flight ahead of the MFMAs
constexpr int kADB3 = 1;          // A chunk buffers (2: the next chunk's LDS reads before this one's MFMAs: no faster)
template <int K, int LDP, int PS, int LDB, int RT, int CT, bool PRE = false>
__device__ __forceinline__ void mfma_rows3(const unsigned short* __restrict__ A, const float* __restrict__ B, int n0,
                                           f4 (&acc)[RT][CT], const WPre<CT>* pre = nullptr) {
  constexpr int NC = K / 32;
  constexpr int BPD = kBPD3 < NC ? kBPD3 : NC, NB = BPD + 1;
  static_assert(!PRE || BPD >= kBPD, "early-issued chunks fit the ring");
  const int l = threadIdx.x & 63, i = l & 15, g = l >> 4;
  const unsigned short* ap = A + i * LDP + 8 * g;
  const float* bp = B + (int64_t)(n0 + i) * LDB + kGOff * g;
  float4 bb[NB][CT][2];
  s8v aa[kADB3][RT][3];
  if constexpr (PRE) {
#pragma unroll
    for (int c = 0; c < kBPD; ++c)
#pragma unroll
      for (int t = 0; t < CT; ++t) { bb[c][t][0] = pre->bb[c][t][0]; bb[c][t][1] = pre->bb[c][t][1]; }
#pragma unroll
    for (int c = kBPD; c < BPD; ++c) b_chunk<CT>(bp + 32 * c, LDB, bb[c]);
  } else {
#pragma unroll
    for (int c = 0; c < BPD; ++c) b_chunk<CT>(bp + 32 * c, LDB, bb[c]);
  }
  if constexpr (kADB3 == 2) a3_chunk<LDP, PS, RT>(ap, aa[0]);
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    if (c + BPD < NC) b_chunk<CT>(bp + 32 * (c + BPD), LDB, bb[(c + BPD) % NB]);
    if constexpr (kADB3 == 2) {
      if (c + 1 < NC) a3_chunk<LDP, PS, RT>(ap + 32 * (c + 1), aa[(c + 1) % 2]);
    } else {
      a3_chunk<LDP, PS, RT>(ap + 32 * c, aa[0]);
    }
    mfma3_regs<RT, CT>(aa[kADB3 == 2 ? c % 2 : 0], bb[c % NB], acc);
  }
}

// ---------------------------------------------------------------------------
// The fc2 operand image W2X: the f32 W2^T [2][H][H] of both nets (phases D of
// the rowpass read fc2.weight transposed), written by adam_kernel beside each
// updated 32x32 tile and by satrl_ppo_w2x_sync from P.  A pre-split bf16
// planes image at H = 256 (no split VALU in the rowpass) was built and
// measured slower -- 1.5x the weight bytes from L2 (EXPERIMENTS.md round 4,
// commit e2546b9) -- so every width keeps the f32 image.
// ---------------------------------------------------------------------------
__host__ __device__ constexpr int64_t w2x_floats(int H) { return 2LL * H * H; }
// the three planes of 4 consecutive elements v (at e, plane stride PS) as
// three 8-B stores
__device__ __forceinline__ void put3x4(unsigned short* __restrict__ img, int64_t e, int64_t PS, float4 v) {
  unsigned h0, m0, l0, h1, m1, l1;
  split3x2(f2v{v.x, v.y}, h0, m0, l0);
  split3x2(f2v{v.z, v.w}, h1, m1, l1);
  *reinterpret_cast<uint2*>(img + e) = make_uint2(h0, h1);
  *reinterpret_cast<uint2*>(img + PS + e) = make_uint2(m0, m1);
  *reinterpret_cast<uint2*>(img + 2 * PS + e) = make_uint2(l0, l1);
}

// Row-parallel activations for the split-bf16 dW2 (satrl_ppo_rowpass_kx /
// satrl_ppo_dw2_kx): a [rows][H] f32 tensor of one net as three bf16 planes
// (plane stride PL elements), "k-packed": element (r, n) at ((r / 8) * H + n)
// * 8 + r % 8, so the 8 consecutive rows an MFMA operand lane holds (the
// reduction index of dW2 = dZ2^T H1 is the row) are one 16-B run, and the 16
// columns of a lane group one 256-B run.  A rowpass lane holds rows 4lg..4lg+3
// of a 16-row tile: one 8-B store per plane.
template <int H, int R, int CT>
__device__ __forceinline__ void store_kx(unsigned short* __restrict__ img, int64_t PL, int r0, int n0,
                                         const float (&v)[R / 16][CT][4]) {
  const int l = threadIdx.x & 63, li = l & 15, lg = l >> 4;
#pragma unroll
  for (int rt = 0; rt < R / 16; ++rt)
#pragma unroll
    for (int t = 0; t < CT; ++t) {
      const int r = r0 + 16 * rt + 4 * lg, n = n0 + 16 * t + li;
      put3x4(img, ((int64_t)(r >> 3) * H + n) * 8 + (r & 7), PL,
             make_float4(v[rt][t][0], v[rt][t][1], v[rt][t][2], v[rt][t][3]));
    }
}
// one 8-B store of the k-packed planes; WT: agent-scope write-through
// (global_store_dwordx2 sc0 sc1), so the planes leave L2 during the kernel
// instead of in the release at its end, which the next launch's start waits
// for.  The 16-row (short-minibatch) rowpass writes through: in-graph step at
// mb 512 33.1-33.2 against 34.1 us with plain stores (three alternations on
// two boxes, tools/ab_spans.sh); at mb 4096 the 32-row kernel gets as much
// longer as the boundary gets shorter (rowpass span +2-3 us, step equal), so
// it stores plainly (EXPERIMENTS.md round 6)
template <bool WT>
__device__ __forceinline__ void st_kx(unsigned short* p, uint2 v) {
  if constexpr (WT)
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), ((unsigned long long)v.y << 32) | v.x,
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else
    *reinterpret_cast<uint2*>(p) = v;
}

// store_kx from values already split (split3x2 of rows j, j+1 and j+2, j+3 of
// each lane's four; w[rt][t] = {hi01, hi23, mid01, mid23, lo01, lo23}): the
// same stores, no split VALU
template <int H, int R, int CT, bool WT = false>
__device__ __forceinline__ void store_kx_w(unsigned short* __restrict__ img, int64_t PL, int r0, int n0,
                                           const unsigned (&w)[R / 16][CT][6]) {
  const int l = threadIdx.x & 63, li = l & 15, lg = l >> 4;
#pragma unroll
  for (int rt = 0; rt < R / 16; ++rt)
#pragma unroll
    for (int t = 0; t < CT; ++t) {
      const int r = r0 + 16 * rt + 4 * lg, n = n0 + 16 * t + li;
      const int64_t e = ((int64_t)(r >> 3) * H + n) * 8 + (r & 7);
      st_kx<WT>(img + e, make_uint2(w[rt][t][0], w[rt][t][1]));
      st_kx<WT>(img + PL + e, make_uint2(w[rt][t][2], w[rt][t][3]));
      st_kx<WT>(img + 2 * PL + e, make_uint2(w[rt][t][4], w[rt][t][5]));
    }
}
// four values of one column, rows e, e + LDP, e + 2 LDP, e + 3 LDP of an LDS
// plane image (plane stride PS), split once as pairs (split3x2) into w: each
// bf16 goes out by a 16-bit store of its half of the packed word
// (ds_write_b16 / ds_write_b16_d16_hi), so the planes get the bits put3 gives
// each value, with the split VALU of two pairs instead of four scalars
template <int PS, int LDP>
__device__ __forceinline__ void put3_col4(unsigned short* img, int e, const float (&v)[4], unsigned (&w)[6]) {
  split3x2(f2v{v[0], v[1]}, w[0], w[2], w[4]);
  split3x2(f2v{v[2], v[3]}, w[1], w[3], w[5]);
#pragma unroll
  for (int p = 0; p < 3; ++p) {
    img[p * PS + e] = (unsigned short)w[2 * p];
    img[p * PS + e + LDP] = (unsigned short)(w[2 * p] >> 16);
    img[p * PS + e + 2 * LDP] = (unsigned short)w[2 * p + 1];
    img[p * PS + e + 3 * LDP] = (unsigned short)(w[2 * p + 1] >> 16);
  }
}
// rows of a k-packed tensor: the minibatch padded to whole 32-row chunks
__host__ __device__ constexpr int64_t kx_rows(int mb) { return (mb + 31) / 32 * 32LL; }
// the three planes of x at element e of an LDS plane image (plane stride PS)
template <int PS>
__device__ __forceinline__ void put3(unsigned short* img, int e, float x) {
  unsigned short h, m, l;
  split3(x, h, m, l);
  img[e] = h;
  img[PS + e] = m;
  img[2 * PS + e] = l;
}

// rows r < nvalid of a 32-/16-row block's accumulator-layout values v[rt][t][j]
// (row 16rt + 4lg + j, column n0 + 16t + li) to out[r * ld + column]: a
// uniform branch keeps a full block's stores straight-line (a per-lane test
// made every store its own exec-masked branch)
template <int R, int CT>
__device__ __forceinline__ void store_rows(float* __restrict__ out, int ld, int n0, int nvalid,
                                           const float (&v)[R / 16][CT][4]) {
  const int l = threadIdx.x & 63, li = l & 15, lg = l >> 4;
  if (nvalid >= R) {
#pragma unroll
    for (int rt = 0; rt < R / 16; ++rt)
#pragma unroll
      for (int t = 0; t < CT; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j) out[(int64_t)(16 * rt + 4 * lg + j) * ld + n0 + 16 * t + li] = v[rt][t][j];
  } else {
#pragma unroll
    for (int rt = 0; rt < R / 16; ++rt)
#pragma unroll
      for (int t = 0; t < CT; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int r = 16 * rt + 4 * lg + j;
          if (r < nvalid) out[(int64_t)r * ld + n0 + 16 * t + li] = v[rt][t][j];
        }
  }
}

// Workgroup barrier of the MLP kernels' phases (__syncthreads: LDS-only
// barriers that leave the global stores and early weight chunks in flight
// measured no faster, EXPERIMENTS.md round 3).
__device__ __forceinline__ void rp_barrier() { __syncthreads(); }

// Shared-memory block and forward pass (phases A, B and the output-layer dot
// products of C) common to rowpass_kernel and policy_kernel, so the rollout's
// policy/value forward and the update's forward are the same instructions in
// the same order: logp_old from the rollout equals the update's first
// recomputation bit for bit, and every row's result is independent of N.
template <int H, int NW, int RR = kRows>
struct MlpSmem {
  static constexpr bool BF3 = kBf3<H>;
  static constexpr int R = RR, LDA = H + 4, LDS_S = 36;
  // bf16 planes: rows padded by 32 B, a row stride of 8 banks (mod 64): the
  // 16 lanes of each ds_read_b128 lane group ({0-3,12-15,20-27}, ...) of an
  // MFMA operand read (row i, 16-B column run g) then land on 16 distinct
  // 4-bank slots (8i + 4g mod 64).  A 16-B pad (4 banks) put two lanes of
  // every group on one slot: SQ_LDS_BANK_CONFLICT 1.67 M -> 0.49 M per
  // rowpass (tools/lds_conflict_ab.sh), bitwise the same, no faster
  static constexpr int LDP = H + 16, PS = R * LDP;
  float h1s[BF3 ? 0 : R][LDA] __attribute__((aligned(16)));                // tanh(fc1)
  unsigned short h1p[BF3 ? 3 * PS : 0] __attribute__((aligned(16)));      // (BF3) its three bf16 planes
  float S[R][LDS_S] __attribute__((aligned(16)));     // [s(18) | 1 | 0...] per row
  // per-column-tile output-layer partial sums, [row][output][tile] with the
  // tiles of a (row, output) contiguous (16-B aligned runs, padded to 4k+4
  // floats so the writers' rows 4 apart fall on different bank pairs): the
  // loss head reads each sum's partials as ds_read_b128s instead of one
  // ds_read per tile (the same partials, added in the same tile order)
  static constexpr int OSP = H / 16 + (H == 64 ? 8 : 4);
  float osum[R][3][OSP] __attribute__((aligned(16)));
};

// Rows r < nvalid of the block must be in S[r][0..17] when gather() returns;
// gather(tid, NT) runs while this wave's W1 rows are in flight.  On return
// acc = tanh(fc2) for this wave's columns, h1 = tanh(fc1) (for the fc1
// backward), w3 = this wave's output-layer weights, and osum holds the
// per-wave dot products (after a barrier).  h1out (nullable): row r of
// tanh(fc1) goes to h1out[r * H + n].  PRIO: the caller raised the wave's
// issue priority (s_setprio) for its weight loads; it drops back once phase
// B's are all out (the policy kernel, see there).
template <int H, int NW, int R, bool APRE, bool PRIO = false, class Gather>
__device__ __forceinline__ void mlp_forward(MlpSmem<H, NW, R>& sm, const float* __restrict__ P,
                                            int net, int nvalid,
                                            Gather gather, float* __restrict__ h1out,
                                            f4 (&acc)[R / 16][H / 16 / NW],
                                            float (&h1)[R / 16][H / 16 / NW][4],
                                            float (&w3)[H / 16 / NW][3],
                                            unsigned (&h1w)[R / 16][H / 16 / NW][6]) {
  constexpr int RT = R / 16, LDA = H + 4, CT = H / 16 / NW, LDS_S = 36, NT = NW * 64;
  static_assert(CT >= 1 && H % (16 * NW) == 0, "tile split");
  const Layout L = layout(H);
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, li = l & 15, lg = l >> 4;
  const int n0 = w * (H / NW);

  // ---- A: gather, fc1 on MFMA ------------------------------------------------
  // this wave's W1aug rows [n][20] (k 0..19, zero-padded to 32; lane group g
  // takes k = 8g .. 8g+7), issued first so they overlap the row gather.  The
  // loads are unconditional (in-row offsets clamped) and the zero padding is
  // selected only after the gather's barrier: a load inside a lane-group
  // branch made the wave wait for it before issuing its row loads
  // The fc2 bias and output-layer weights of this wave's columns (used in C)
  // go out with them: __syncthreads drains every outstanding load, so loads
  // issued after the gather would hold up the barrier below
  float4 w1raw[CT][2];
  float b2v[CT], w3raw[CT][3];
  {
    const float* W1 = P + L.W1 + (int64_t)net * H * 20;
    const int o0 = lg < 2 ? 8 * lg : 16, o1 = lg < 2 ? 8 * lg + 4 : 16;
#pragma unroll
    for (int t = 0; t < CT; ++t) {
      const int n = n0 + 16 * t + li;
      const float* bp = W1 + (int64_t)n * 20;
      w1raw[t][0] = *reinterpret_cast<const float4*>(bp + o0);
      w1raw[t][1] = *reinterpret_cast<const float4*>(bp + o1);
      b2v[t] = P[L.b2 + net * H + n];
      w3raw[t][0] = P[(net == 0 ? L.W3a : L.W3c) + n];
      w3raw[t][1] = P[L.W3a + H + n];
      w3raw[t][2] = P[L.W3a + 2 * H + n];
    }
  }
  gather(tid, NT);
  for (int q = tid; q < R * (LDS_S - 18); q += NT) {
    const int r = q / (LDS_S - 18), c = 18 + q % (LDS_S - 18);
    sm.S[r][c] = (c == 18 && r < nvalid) ? 1.0f : 0.0f;           // bias column of W1aug, zero pad
  }
  PHASE_PROBE(8);
  rp_barrier();
  PHASE_PROBE(9);
  // (split-bf16 fc2) phase B's first weight chunks go out now, under fc1 (an
  // LDS-only barrier below, leaving them in flight, measured no faster)
  WPre<CT> preB;
  if constexpr (kBf3<H>) mfma_rows_pre<H, CT>(P + L.W2 + (int64_t)net * H * H, n0, preB);
  float4 bw1[CT][2];
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int t = 0; t < CT; ++t) {
    bw1[t][0] = lg < 3 ? w1raw[t][0] : z4;
    bw1[t][1] = lg < 2 ? w1raw[t][1] : z4;
    w3[t][0] = w3raw[t][0];                                       // actor: mean_layer rows, critic: fc3
    w3[t][1] = net == 0 ? w3raw[t][1] : 0.0f;
    w3[t][2] = net == 0 ? w3raw[t][2] : 0.0f;
  }
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int t = 0; t < CT; ++t) acc[rt][t] = f4{0.f, 0.f, 0.f, 0.f};
  mfma_chunk<LDS_S, RT, CT, 4>(&sm.S[li][8 * lg], bw1, acc);
  PHASE_PROBE(10);
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int t = 0; t < CT; ++t) {
      const int n = n0 + 16 * t + li;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = 16 * rt + 4 * lg + j;
        const float h = tanh_f32(acc[rt][t][j]);                   // fc1 + tanh
        h1[rt][t][j] = h;
        if constexpr (!kBf3<H>) sm.h1s[r][n] = h;
      }
      // (split-bf16) the three planes of the lane's four rows, split once as
      // pairs; the words stay in h1w for the k-packed H1 store (rowpass_kx)
      if constexpr (kBf3<H>)
        put3_col4<MlpSmem<H, NW, R>::PS, MlpSmem<H, NW, R>::LDP>(
            sm.h1p, (16 * rt + 4 * lg) * MlpSmem<H, NW, R>::LDP + n, h1[rt][t], h1w[rt][t]);
      acc[rt][t] = f4{0.f, 0.f, 0.f, 0.f};
    }
  if (h1out != nullptr) store_rows<R, CT>(h1out, H, n0, nvalid, h1);   // straight-line unless ragged
  PHASE_PROBE(11);
  rp_barrier();
  PHASE_PROBE(1);

  // ---- B: Z2 = H1 W2^T -------------------------------------------------------
  if constexpr (kBf3<H>)
    mfma_rows3<H, MlpSmem<H, NW, R>::LDP, MlpSmem<H, NW, R>::PS, H, RT, CT, true>(
        sm.h1p, P + L.W2 + (int64_t)net * H * H, n0, acc, &preB);
  else
    mfma_rows<H, LDA, H, RT, CT, APRE>(&sm.h1s[0][0], P + L.W2 + (int64_t)net * H * H, n0, acc);
  if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
  PHASE_PROBE(2);

  // ---- C (forward part): fc2 tanh, output-layer dot products -----------------
  const int NQ = net == 0 ? 3 : 1;                                  // output columns of this net
  // one partial per 16-column tile (DPP row sums), so the output layer sums
  // the same H/16 partials in the same order whatever the wave count: the
  // 8-wave policy kernel's log-probs are the 16-wave rowpass's bit for bit
  float p[3][CT][RT][4];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int t = 0; t < CT; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float h = tanh_f32(acc[rt][t][j] + b2v[t]);           // fc2 + tanh
        acc[rt][t][j] = h;
#pragma unroll
        for (int q = 0; q < 3; ++q) p[q][t][rt][j] = fmaf(h, w3[t][q], 0.0f);
      }
  // the DPP row sums; NQ is uniform per workgroup (3 actor, 1 critic)
  constexpr int NP = CT * RT * 4;                                   // partials per output column
  float ps[3 * NP];
#pragma unroll
  for (int q = 0; q < 3; ++q)
#pragma unroll
    for (int t = 0; t < CT; ++t)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int j = 0; j < 4; ++j) ps[((q * CT + t) * RT + rt) * 4 + j] = p[q][t][rt][j];
  if (NQ == 3) {
    row16_sum_n<3 * NP>(ps);
  } else {
    float p0[NP];
#pragma unroll
    for (int k = 0; k < NP; ++k) p0[k] = ps[k];
    row16_sum_n<NP>(p0);
#pragma unroll
    for (int k = 0; k < NP; ++k) ps[k] = p0[k];
  }
  if (li == 0) {
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      if (q >= NQ) break;
#pragma unroll
      for (int t = 0; t < CT; ++t)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            sm.osum[16 * rt + 4 * lg + j][q][w * CT + t] = ps[((q * CT + t) * RT + rt) * 4 + j];
    }
  }
  rp_barrier();
  PHASE_PROBE(3);
}

// output-layer pre-activation of row r, column d: the NTL column-tile
// partials in fixed order
template <int NTL, int OSP>
__device__ __forceinline__ float out_sum(const float (*osum)[3][OSP], int r, int d) {
  float od = 0.0f;
#pragma unroll
  for (int k = 0; k < NTL; ++k) od += osum[r][d][k];
  return od;
}

template <int H, int NW, int R = kRows, bool FDW2 = false, bool KX = false, bool SPAN = false>
__global__ void __launch_bounds__(NW * 64, NW * 64 / 256) rowpass_kernel(int mb, const float* __restrict__ src,
                                                      const int64_t* __restrict__ idx, const float* __restrict__ P,
                                                      const void* __restrict__ W2X, float epsilon, float ent_coef,
                                                      float max_action, float* __restrict__ H1g,
                                                      float* __restrict__ dZ2g, float* __restrict__ ptail,
                                                      float* __restrict__ pw1, int net_sel, float* __restrict__ p2,
                                                      int S2, float* __restrict__ ratio_out, float inv_mb,
                                                      unsigned long long* __restrict__ span) {
  const unsigned long long span_t0 = SPAN ? satrl_span::now() : 0ull;   // (SPAN: the measurement instantiation)
  constexpr int RT = R / 16, LDA = H + 4, CT = H / 16 / NW, NT = NW * 64;
  static_assert(!FDW2 || R == 32, "the fused dW2 partial covers one 32-row block (dw2_kernel's chunk)");
  // KX: H1 / dZ2 go out as k-packed bf16 planes (store_kx; H1g / dZ2g point at
  // u16 [2][3][kx_rows(mb)][H]) for satrl_ppo_dw2_kx, whole 32-row chunks (a
  // 16-row kernel's last block zero-fills the chunk's other half)
  static_assert(!KX || ((R == 32 || R == kRowsShort) && kBf3<H> && !FDW2), "k-packed outputs: split-bf16 width");
  const int64_t PLX = kx_rows(mb) * H;                             // (KX) plane elements per net
  const Layout L = layout(H);
  __shared__ MlpSmem<H, NW, R> sm;
  constexpr bool BF3 = kBf3<H>;
  constexpr int LDP = MlpSmem<H, NW, R>::LDP, PS = MlpSmem<H, NW, R>::PS;
  __shared__ __attribute__((aligned(16))) float dzs[BF3 ? 1 : R][BF3 ? 4 : LDA];   // dZ2
  __shared__ __attribute__((aligned(16))) unsigned short dzp[BF3 ? 3 * PS : 8];    // (BF3) its bf16 planes
  __shared__ float ax[R][8];
  __shared__ float dz3s[R][4];
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, li = l & 15, lg = l >> 4;
  // net_sel < 0: both nets, blockIdx = (row block, net); else that net only
  // XCD-matched placement (32-row k-packed kernel, both nets, a row-block
  // count divisible by 8): the row blocks of dW2 split s -- row blocks
  // [s nrb/8, (s+1) nrb/8), both nets -- go to the workgroups b with
  // b % 8 == s, i.e. under round-robin dispatch to the XCD that dw2_kx's
  // split s runs on (its block b takes split b % 8), so the planes dw2_kx
  // reads were written through that XCD's L2 (placement only: every bit is
  // the same; in-graph step at mb 4096 47.5-47.8 against 48.7-49.2 us over
  // three alternations, the rowpass->dw2 boundary 3.6-3.9 against 4.1-4.6
  // us; at mb 512 the 16-row kernel measured 0.2-0.3 us slower with it, so
  // it keeps the (row block, net) = (b / 2, b % 2) order; EXPERIMENTS.md
  // round 6).  Otherwise the actor lands on the even XCDs, the critic on the odd.
  const int nrbk = (mb + R - 1) / R;
  const bool xmap = KX && R == kRows && net_sel < 0 && nrbk % 8 == 0;
  const int bx = (int)blockIdx.x, kx8 = bx >> 3;
  const int net = net_sel < 0 ? (xmap ? (kx8 & 1) : (bx & 1)) : net_sel;
  const int rb = net_sel < 0 ? (xmap ? (bx & 7) * (nrbk >> 3) + (kx8 >> 1) : (bx >> 1)) : bx, n0 = w * (H / NW);
  const int r0 = rb * R;
  auto& S = sm.S;
#ifdef SATRL_PHASE_PROBE
  if (threadIdx.x == 0 && blockIdx.x < 512) {   // placement: XCC_ID and HW_ID (SE/SH/CU) of the workgroup
    g_probe[blockIdx.x][15][0][0] = __builtin_amdgcn_s_getreg((31 << 11) | 20);
    g_probe[blockIdx.x][15][0][1] = __builtin_amdgcn_s_getreg((31 << 11) | 4);
  }
#endif
  PHASE_PROBE(0);
  // The head's scalars (mean_layer bias, log_std, fc3 bias) and its
  // per-dimension constants (var = exp(log_std)^2, log std, 1/var), off the
  // head's dependency chain: lanes 0-3 of the last wave (no row load of its
  // own at H = 256) load them as per-lane vector loads and compute the
  // constants into LDS during the gather (the barriers of the forward pass
  // publish them).  Uniform scalar loads of P here would make the wave's
  // first s_waitcnt lgkmcnt -- the one for the kernel arguments -- wait for
  // them before any row load is issued.
  __shared__ float hcs[3][3];
  __shared__ float hb3s[4];                                        // b3a[0..2], b3c
  const int hd = tid - (NT - 64);                                  // head-scalar lane of the last wave
  float hls_d = 0.0f, hb3_d = 0.0f;
  if (hd >= 0 && hd < 4) {
    hb3_d = P[hd < 3 ? L.b3a + hd : L.b3c];
    hls_d = P[L.ls + (hd < 3 ? hd : 0)];
  }

  f4 acc[RT][CT];
  float h1[RT][CT][4];
  float w3[CT][3];
  unsigned h1w[RT][CT][6];                                         // (split-bf16) the split H1 words
  auto gather = [&](int t0, int nt) {
    auto head_consts = [&] {
      // (opaque to the compiler and ordered after the row loads: otherwise it
      // hoists this arithmetic next to its loads at the top of the kernel,
      // and the whole wave waits for them before issuing any row load)
      asm volatile("" : "+v"(hls_d), "+v"(hb3_d)::"memory");
      if (hd >= 0 && hd < 4) {
        hb3s[hd] = hb3_d;
        if (hd < 3) {
          const float sd = expf(hls_d), var = sd * sd;
          hcs[0][hd] = var;
          hcs[1][hd] = logf(sd);
          hcs[2][hd] = 1.0f / var;
        }
      }
    };
    if (idx == nullptr) {
      // contiguous (staged) rows: one 16-B load per thread covers the block's
      // R x 32 floats, all in flight at once (a loop of dependent scalar
      // loads took four load round trips at H = 64's 256 threads)
      // (branch-free: rows past the minibatch load its last row, zeroed below)
      static_assert(R * 8 <= NT, "one float4 per thread");
      const int r = (t0 >> 3) & (R - 1), c4 = t0 & 7, row = r0 + r;
      const bool in = t0 < R * 8;
      float4 v = reinterpret_cast<const float4*>(src)[(int64_t)(row < mb ? row : mb - 1) * 8 + c4];
      head_consts();
      if (row >= mb) v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (in) {
        const float e4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int c = 4 * c4 + e;                                  // s | a, logp_old, adv, v_target | pad
          if (c < 18) S[r][c] = e4[e];
          else if (c < 26) ax[r][c - 18] = e4[e];
        }
      }
    } else {
      for (int q = t0; q < R * 26; q += nt) {
        const int r = q / 26, c = q % 26, row = r0 + r;
        const float v = row < mb ? src[idx[row] * 32 + c] : 0.0f;
        if (c < 18) S[r][c] = v; else ax[r][c - 18] = v;
      }
      head_consts();
    }
  };
  // the fc2 operand image: the f32 W2^T
  const float* W2T = static_cast<const float*>(W2X);
  // (H = 256: the H1 store after phase B, not between fc1 and B: 8 fewer VGPRs
  // live through B, so the 32-row kernel stays at <= 104)
  // (FDW2, H = 64: at priority 3 until phase B's weight loads are out, as the
  // policy kernel -- in-graph step 18.2 against 18.4 us at configs[1]'s
  // mb 4096, 15.3 against 15.5 at 512; at H = 256 no gain, not set there)
  if constexpr (FDW2) __builtin_amdgcn_s_setprio(3);
  mlp_forward<H, NW, R, true, FDW2>(sm, P, net, mb - r0, gather,
                                   FDW2 || KX || BF3 ? nullptr : H1g + ((int64_t)net * mb + r0) * H, acc, h1, w3,
                                   h1w);
  // (rows past the minibatch: zero inputs, so tanh(fc1) = 0 and dZ2 = 0 there)
  // (KX) the H1 planes: wave 0, which runs the loss head next, stores its
  // share after the head's barrier, off the head's path; the other waves now
  auto h1_kx = [&] {
    store_kx_w<H, R, CT, R == kRowsShort>(reinterpret_cast<unsigned short*>(H1g) + net * 3 * PLX, PLX, r0, n0, h1w);
    if (R < 32 && r0 + R < kx_rows(mb) && r0 + R >= mb) {            // (uniform) the padded chunk's rows past this block
      const float z[R / 16][CT][4] = {};
      store_kx<H, R, CT>(reinterpret_cast<unsigned short*>(H1g) + net * 3 * PLX, PLX, r0 + R, n0, z);
      store_kx<H, R, CT>(reinterpret_cast<unsigned short*>(dZ2g) + net * 3 * PLX, PLX, r0 + R, n0, z);
    }
  };
  if constexpr (KX) {
    if (w != 0) h1_kx();
  }
  else if constexpr (BF3 && !FDW2) store_rows<R, CT>(H1g + ((int64_t)net * mb + r0) * H, H, n0, mb - r0, h1);
  // phase D's first W2T chunks go out now, under the loss head and the tail
  WPre<CT> preD;
  mfma_rows_pre<H, CT>(W2T + (int64_t)net * H * H, n0, preD);

  // ---- C: the net's loss and its gradient, dZ2 ---------------------------------
  if (tid < R) {
    const int r = tid, row = r0 + r;
    float dz[4] = {0.f, 0.f, 0.f, 0.f}, dls[4] = {0.f, 0.f, 0.f, 0.f};
    if (row < mb) {
      const float inv = inv_mb;                                   // 1.0f / (float)mb, IEEE on the host
      if (net == 0) {                                              // actor: clipped surrogate + entropy
        float th[3], mu[3], dv[3], var[3], logp[3];
#pragma unroll
        for (int d = 0; d < 3; ++d) {
          th[d] = tanh_f32(out_sum<H / 16>(sm.osum, r, d) + hb3s[d]);
          mu[d] = max_action * th[d];                              // 1.6 * tanh(mean_layer)
          var[d] = hcs[0][d];
          dv[d] = ax[r][d] - mu[d];
          // (the forward expression of gaussian_act, bit for bit: logp_old)
          logp[d] = (-(dv[d] * dv[d]) / (2.0f * var[d]) - hcs[1][d]) - kLogSqrt2Pi;
        }
        PHASE_PROBE(12);
        const float lsum = (logp[0] + logp[1]) + logp[2];
        const float lold = (ax[r][3] + ax[r][4]) + ax[r][5];
        const float ratio = expf(lsum - lold);
        if (ratio_out != nullptr) ratio_out[row] = ratio;          // (satrl_ppo_rowpass_ratio)
        const float adv = ax[r][6];
        const float s1 = ratio * adv;
        const float cr = fminf(fmaxf(ratio, 1.0f - epsilon), 1.0f + epsilon);
        const float s2 = cr * adv;
        const float g1 = s1 < s2 ? 1.0f : (s1 == s2 ? 0.5f : 0.0f);   // torch.min tie split
        const float g2 = s2 < s1 ? 1.0f : (s1 == s2 ? 0.5f : 0.0f);
        const float inside = (ratio >= 1.0f - epsilon && ratio <= 1.0f + epsilon) ? 1.0f : 0.0f;
        const float dmin = -inv;
        const float dratio = dmin * g1 * adv + dmin * g2 * adv * inside;
        const float dlsum = dratio * ratio;
#pragma unroll
        for (int d = 0; d < 3; ++d) {
          const float dvv = dv[d] * hcs[2][d];                     // (x - mu) / var
          const float dmu = dlsum * dvv;
          dz[d] = (dmu * max_action) * (1.0f - th[d] * th[d]);
          dls[d] = dlsum * (dv[d] * dvv - 1.0f) - ent_coef * inv;
        }
      } else {                                                     // critic: MSE
        const float vc = out_sum<H / 16>(sm.osum, r, 0) + hb3s[3];
        dz[3] = 2.0f * inv * (vc - ax[r][7]);                      // d mse / d v
      }
    }
    PHASE_PROBE(13);
#pragma unroll
    for (int q = 0; q < 4; ++q) dz3s[r][q] = dz[q];
    // the block's b3a / log_std / b3c partials: sums over its R rows, reduced
    // across these R lanes of wave 0 in a fixed order: DPP sums of each
    // 16-lane row, then row 0 + row 1 (readlane), no LDS round trips
    static_assert(R == 16 || R == 32, "row sums cover one or two DPP rows");
    float* tp = ptail + (int64_t)rb * L.tail;
    float red[7] = {dz[0], dz[1], dz[2], dls[0], dls[1], dls[2], dz[3]};
    row16_sum_n<7>(red);
    if (R == 32) {
#pragma unroll
      for (int q = 0; q < 7; ++q)
        red[q] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(red[q]), 0)) +
                 __int_as_float(__builtin_amdgcn_readlane(__float_as_int(red[q]), 16));
    }
    PHASE_PROBE(14);
    if (r == 0) {
      if (net == 0) {
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          tp[5 * H + q] = red[q];          // b3a
          tp[5 * H + 4 + q] = red[3 + q];  // log_std
        }
        tp[5 * H + 3] = 0.0f;
        tp[5 * H + 7] = 0.0f;
      } else {
        tp[6 * H + 8] = red[6];            // b3c
        tp[6 * H + 9] = 0.0f; tp[6 * H + 10] = 0.0f; tp[6 * H + 11] = 0.0f;
      }
    }
  }
  rp_barrier();
  PHASE_PROBE(4);
  // (wave 0's share of the H1 planes after the head's barrier: before it, the
  // barrier's vmcnt(0) waited for those stores' write latency with the other
  // 15 waves idle -- in-graph step 47.73-47.88 against 47.99-48.51 us over
  // four alternations, bitwise the same; EXPERIMENTS.md round 6)
  if constexpr (KX) {
    if (w == 0) h1_kx();
  }
  float* tp = ptail + (int64_t)rb * L.tail;                         // tail-relative slab of this row block
  float d2v[RT][CT][4];
  unsigned d2w[RT][CT][6];                                         // (split-bf16) the split dZ2 words
  // unswitched on the (workgroup-uniform) net: no per-element branches, and
  // the critic skips the actor's three output columns.  (Moving the db2 /
  // dW3 partial sums into phase D's MFMA gaps measured slower: D +2.6 k
  // cycles for 0.5 k saved here, EXPERIMENTS.md round 4.)
  auto tail = [&](auto actor) {
    constexpr bool ACT = decltype(actor)::value;
    constexpr int NC = ACT ? 3 : 1;
#pragma unroll
    for (int t = 0; t < CT; ++t) {
      const int n = n0 + 16 * t + li;
      float cb2 = 0.f, cw[NC];
#pragma unroll
      for (int q = 0; q < NC; ++q) cw[q] = 0.f;
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int r = 16 * rt + 4 * lg + j;
          const float h = acc[rt][t][j];
          float dh;
          if constexpr (ACT) dh = (dz3s[r][0] * w3[t][0] + dz3s[r][1] * w3[t][1]) + dz3s[r][2] * w3[t][2];
          else dh = dz3s[r][3] * w3[t][0];
          const float d2 = dh * (1.0f - h * h);                     // tanh backward
          if constexpr (!BF3) dzs[r][n] = d2;
          d2v[rt][t][j] = d2;
          cb2 += d2;
          if constexpr (ACT) {
            cw[0] = fmaf(dz3s[r][0], h, cw[0]); cw[1] = fmaf(dz3s[r][1], h, cw[1]); cw[2] = fmaf(dz3s[r][2], h, cw[2]);
          } else {
            cw[0] = fmaf(dz3s[r][3], h, cw[0]);
          }
        }
        // (split-bf16) dZ2's LDS planes (phase D's A operand), split once as
        // pairs; the words stay in d2w for the k-packed dZ2 store
        if constexpr (BF3) put3_col4<PS, LDP>(dzp, (16 * rt + 4 * lg) * LDP + n, d2v[rt][t], d2w[rt][t]);
      }
      cb2 = xor32_sum(xor16_sum(cb2));
#pragma unroll
      for (int q = 0; q < NC; ++q) cw[q] = xor32_sum(xor16_sum(cw[q]));
      if (lg == 0) {
        tp[net * H + n] = cb2;                                     // db2
        if constexpr (ACT) {                                       // dW3a
          tp[2 * H + n] = cw[0]; tp[3 * H + n] = cw[1]; tp[4 * H + n] = cw[2];
        } else {
          tp[5 * H + 8 + n] = cw[0];                               // dW3c
        }
      }
    }
  };
  if (net == 0) tail(std::true_type{});
  else tail(std::false_type{});
  if constexpr (KX)
    store_kx_w<H, R, CT, R == kRowsShort>(reinterpret_cast<unsigned short*>(dZ2g) + net * 3 * PLX, PLX, r0, n0, d2w);
  else if constexpr (!FDW2) store_rows<R, CT>(dZ2g + ((int64_t)net * mb + r0) * H, H, n0, mb - r0, d2v);
  rp_barrier();
  PHASE_PROBE(5);

  // ---- D: dH1 = dZ2 W2 -------------------------------------------------------
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int t = 0; t < CT; ++t) acc[rt][t] = f4{0.f, 0.f, 0.f, 0.f};
  if constexpr (BF3)
    mfma_rows3<H, LDP, PS, H, RT, CT, true>(dzp, W2T + (int64_t)net * H * H, n0, acc, &preD);
  else
    mfma_rows<H, LDA, H, RT, CT, true, true>(&dzs[0][0], W2T + (int64_t)net * H * H, n0, acc, &preD);
  PHASE_PROBE(6);

  // ---- E: dZ1 = dH1 (1 - H1^2); [dW1 | db1][n][k'] = sum_r dZ1[r][n] S[r][k'] ----
  // acc[rt][t][j] = dZ1[row 16rt+4lg+j][n0+16t+li] is the A operand A[n][r] of
  // the product (k = row, kk = j); B[r][k'] = S[16rt+4lg+kk][16hb + li] from LDS.
  float* pw = pw1 + (int64_t)rb * 2 * H * 20 + (int64_t)net * H * 20;
#pragma unroll
  for (int t = 0; t < CT; ++t) {
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[rt][t][j] = acc[rt][t][j] * (1.0f - h1[rt][t][j] * h1[rt][t][j]);
#pragma unroll
    for (int hb = 0; hb < 2; ++hb) {
      f4 d = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) d = mfma4(acc[rt][t][kk], S[16 * rt + 4 * lg + kk][16 * hb + li], d);
      // d[j] = dW1aug[n = n0 + 16t + 4lg + j][k' = 16hb + li]
      const int kp = 16 * hb + li;
      if (kp < 20) {
#pragma unroll
        for (int j = 0; j < 4; ++j) pw[(int64_t)(n0 + 16 * t + 4 * lg + j) * 20 + kp] = d[j];
      }
    }
  }
  PHASE_PROBE(7);

  // ---- F (FDW2, H <= 128): this block's dW2 partial = dZ2^T H1 over its rows ---
  // straight from the LDS images (dzs, h1s), written as split-K slab rb of
  // p2 [2][S2][H][H]: the MFMA sequence of dw2_kernel on one 32-row chunk
  // (A[n][k] = dZ2[row][n], B[k][m] = H1[row][m], row = 4ks + lg; rows past
  // the minibatch masked to 0), so the slab is bitwise dw2_kernel's with
  // S = the row-block count -- without the H1 / dZ2 round trip through HBM
  // and the dW2 launch.
  if constexpr (FDW2) {
    constexpr int MT = H / 16;
    const int nvalid = mb - r0;
#pragma unroll
    for (int t = 0; t < CT; ++t) {
      f4 a2[MT];
#pragma unroll
      for (int j = 0; j < MT; ++j) a2[j] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < R / 4; ++ks) {
        const int row = 4 * ks + lg;
        float a = dzs[row][n0 + 16 * t + li];
        if (row >= nvalid) a = 0.0f;
#pragma unroll
        for (int j = 0; j < MT; ++j) a2[j] = mfma4(a, sm.h1s[row][16 * j + li], a2[j]);
      }
      float* out = p2 + ((int64_t)net * S2 + rb) * H * H;
#pragma unroll
      for (int j = 0; j < MT; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          out[(int64_t)(n0 + 16 * t + 4 * lg + q) * H + 16 * j + li] = a2[j][q];
        }
    }
  }
  if constexpr (SPAN) satrl_span::exit(span, span_t0);
}

// ---------------------------------------------------------------------------
// rowpass_cs: the short-minibatch H = 256 k-packed rowpass (16-row blocks)
// with each (row block, net) split by hidden columns over kCsSplit workgroups
// of kCsWaves waves: quarter j owns the 16-column tiles 4j .. 4j+3, its wave w
// the tile 4j + w (columns 64j + 16w ..).  At configs[3]'s 512 rows per rank
// rowpass_kernel<256, 16, 16> puts 64 workgroups of 16 waves on 256 CUs, four
// waves per SIMD issuing phases B and D one after another; here 256
// workgroups of 4 waves, one wave per SIMD.  Every value is computed by the
// instructions of rowpass_kernel<256, 16, kRowsShort, false, true> in the same
// order -- fc1 of all 16 tiles in every quarter (phase B's A operand is all of
// H1), then the same per-tile fc2, output-layer, loss-head, tail, dH1 and dW1
// sequences -- so every output is bitwise that kernel's.
// Two hand-offs inside the launch between the kCsSplit workgroups of a group,
// in the form of row 3 of MI355X_MICROARCH.md's sc1 hand-off table: __device__
// arrays; payload stores sc1 (8 B, every 128-B line by 16 lanes of one store
// instruction); every storing wave's vmcnt(0) wait and a workgroup barrier
// before ONE agent-scope add per workgroup; a global_load_dword sc1 poll; a
// workgroup barrier between the poll and every payload load
// (buffer_load_dwordx4 sc1):
//   X1  each quarter's output-layer tile partials (the loss head sums all 16
//       tiles, in tile order, in every quarter);
//   X2  each quarter's columns of the dZ2 bf16 planes (phase D's k runs over
//       all 256).
// A group's counter only grows, by kCsSplit at each hand-off, so a launch
// finds it at 2 kCsSplit L (L = the group's launches so far) and the value
// an add returns names the launch's targets.  A wait longer than
// kCsTimeoutTicks (a group not co-resident: the launcher checks residency
// first) sets g_cs_err and leaves the kernel, so the grid always drains;
// satrl_ppo_rowpass_error reports it and re-arms the counters.
// ---------------------------------------------------------------------------
constexpr int kCsWaves = 4, kCsSplit = 256 / 16 / kCsWaves;   // waves per workgroup, workgroups per group
// minibatches of up to this many rows (the whole 16-row range: at mb 1024
// 512 workgroups, two per CU; in-graph step 33.2 against 35.5 us, at mb 768
// 32.2 against 34.4, three alternations; EXPERIMENTS.md round 6)
constexpr int kCsMaxMb = 1024;
constexpr int kCsMaxGroups = 2 * (kCsMaxMb / kRowsShort);      // (row block, net) groups
constexpr unsigned long long kCsTimeoutTicks = 50000000ull;     // 0.5 s of s_memrealtime (100 MHz)
__device__ __attribute__((aligned(128))) unsigned g_cs_ctr[kCsMaxGroups][32];   // a 128-B line per counter
__device__ __attribute__((aligned(128))) unsigned g_cs_err[32];
__device__ __attribute__((aligned(128))) float g_cs_x1[kCsMaxGroups][kCsSplit][kRowsShort][3][kCsWaves];
__device__ __attribute__((aligned(128))) unsigned short g_cs_x2[kCsMaxGroups][3][kRowsShort][256];

// one hand-off step (1: X1, 2: X2) of a group: true once every workgroup of
// the group has published it, false (every thread) after a timeout
__device__ __forceinline__ bool cs_handoff(unsigned* ctr, unsigned step, unsigned* ok_lds) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");           // this wave's payload stores are out
  __syncthreads();                                            // ... and every other wave's
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned target = old - old % (2u * kCsSplit) + step * kCsSplit;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    unsigned ok = 1;
    while ((int)(__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - target) < 0) {
      __builtin_amdgcn_s_sleep(1);
      if (__builtin_amdgcn_s_memrealtime() - t0 > kCsTimeoutTicks) {
        __hip_atomic_store(&g_cs_err[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = 0;
        break;
      }
    }
    *ok_lds = ok;
  }
  __syncthreads();
  return *ok_lds != 0;
}
// 16 B of a hand-off payload, from L2 (sc1: never a stale L1 line)
__device__ __forceinline__ float4 cs_load16(const void* base, int bytes, int off) {
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, bytes, 0x00020000);
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 16));
}
__device__ __forceinline__ void cs_store8(void* p, unsigned long long v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <bool SPAN = false>
__global__ void __launch_bounds__(kCsWaves * 64) rowpass_cs_kernel(
    int mb, const float* __restrict__ src, const int64_t* __restrict__ idx, const float* __restrict__ P,
    const float* __restrict__ W2T, float epsilon, float ent_coef, float max_action,
    unsigned short* __restrict__ H1x, unsigned short* __restrict__ dZ2x, float* __restrict__ ptail,
    float* __restrict__ pw1, float* __restrict__ ratio_out, float inv_mb, unsigned long long* __restrict__ span) {
  const unsigned long long span_t0 = SPAN ? satrl_span::now() : 0ull;
  constexpr int H = 256, R = kRowsShort, NT = kCsWaves * 64, LDS_S = 36;
  constexpr int LDP = MlpSmem<H, 16, R>::LDP, PS = MlpSmem<H, 16, R>::PS, OSP = MlpSmem<H, 16, R>::OSP;
  struct Smem {
    unsigned short h1p[3 * PS];                  // tanh(fc1), all 256 columns, three bf16 planes
    unsigned short dzp[3 * PS];                  // dZ2 planes (this quarter's columns, then all)
    float S[R][LDS_S];
    float osum[R][3][OSP];                       // every tile's output-layer partials (after X1)
    float xs[R][3][kCsWaves];                    // this quarter's (X1 staging)
    float ax[R][8];
    float dz3s[R][4];
    float hcs[3][3];
    float hb3s[4];
    unsigned ok;
  };
  __shared__ __attribute__((aligned(16))) Smem sm;
  // group g = (row block, net), quarter j: blocks b, b + 8, b + 16, b + 24 of
  // each 32 form a group (one XCD under round-robin dealing: placement only)
  const int nrbk = (mb + R - 1) / R, ngrp = 2 * nrbk;
  const int bx = (int)blockIdx.x, j = (bx >> 3) & (kCsSplit - 1), grp = (bx & 7) | ((bx >> 5) << 3);
  if (grp >= ngrp) {                                               // (whole groups of the last window)
    if constexpr (SPAN) satrl_span::exit(span, span_t0);
    return;
  }
  const int net = grp & 1, rb = grp >> 1, r0 = rb * R;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, li = l & 15, lg = l >> 4;
  const int n0 = 64 * j + 16 * w;                                  // this wave's tile: 4j + w
  const int64_t PLX = kx_rows(mb) * H;
  const Layout L = layout(H);
  unsigned* ctr = &g_cs_ctr[grp][0];
  PHASE_PROBE(0);

  // head scalars: lanes 0-3 of the last wave (no row load of its own)
  const int hd = tid - (NT - 64);
  float hls_d = 0.0f, hb3_d = 0.0f;
  if (hd >= 0 && hd < 4) {
    hb3_d = P[hd < 3 ? L.b3a + hd : L.b3c];
    hls_d = P[L.ls + (hd < 3 ? hd : 0)];
  }
  // fc1 weights of the wave's four fc1 tiles w, w + 4, w + 8, w + 12 (tile 4j + w
  // among them, t = j), this tile's fc2 bias and output-layer weights
  float4 w1raw[4][2];
  float b2v, w3raw[3];
  {
    const float* W1 = P + L.W1 + (int64_t)net * H * 20;
    const int o0 = lg < 2 ? 8 * lg : 16, o1 = lg < 2 ? 8 * lg + 4 : 16;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const float* bp = W1 + (int64_t)(16 * (w + 4 * t) + li) * 20;
      w1raw[t][0] = *reinterpret_cast<const float4*>(bp + o0);
      w1raw[t][1] = *reinterpret_cast<const float4*>(bp + o1);
    }
    const int n = n0 + li;
    b2v = P[L.b2 + net * H + n];
    w3raw[0] = P[(net == 0 ? L.W3a : L.W3c) + n];
    w3raw[1] = P[L.W3a + H + n];
    w3raw[2] = P[L.W3a + 2 * H + n];
  }
  // ---- A: gather (rowpass_kernel's), fc1 of all 16 tiles ---------------------
  {
    auto head_consts = [&] {
      asm volatile("" : "+v"(hls_d), "+v"(hb3_d)::"memory");
      if (hd >= 0 && hd < 4) {
        sm.hb3s[hd] = hb3_d;
        if (hd < 3) {
          const float sd = expf(hls_d), var = sd * sd;
          sm.hcs[0][hd] = var;
          sm.hcs[1][hd] = logf(sd);
          sm.hcs[2][hd] = 1.0f / var;
        }
      }
    };
    if (idx == nullptr) {
      static_assert(R * 8 <= NT, "one float4 per thread");
      const int r = (tid >> 3) & (R - 1), c4 = tid & 7, row = r0 + r;
      const bool in = tid < R * 8;
      float4 v = reinterpret_cast<const float4*>(src)[(int64_t)(row < mb ? row : mb - 1) * 8 + c4];
      head_consts();
      if (row >= mb) v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (in) {
        const float e4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int c = 4 * c4 + e;
          if (c < 18) sm.S[r][c] = e4[e];
          else if (c < 26) sm.ax[r][c - 18] = e4[e];
        }
      }
    } else {
      for (int q = tid; q < R * 26; q += NT) {
        const int r = q / 26, c = q % 26, row = r0 + r;
        const float v = row < mb ? src[idx[row] * 32 + c] : 0.0f;
        if (c < 18) sm.S[r][c] = v; else sm.ax[r][c - 18] = v;
      }
      head_consts();
    }
  }
  for (int q = tid; q < R * (LDS_S - 18); q += NT) {
    const int r = q / (LDS_S - 18), c = 18 + q % (LDS_S - 18);
    sm.S[r][c] = (c == 18 && r < mb - r0) ? 1.0f : 0.0f;
  }
  PHASE_PROBE(8);
  rp_barrier();
  PHASE_PROBE(9);
  WPre<1> preB;
  mfma_rows_pre<H, 1>(P + L.W2 + (int64_t)net * H * H, n0, preB);
  float w3[3];
  float4 bw1[4][2];
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    bw1[t][0] = lg < 3 ? w1raw[t][0] : z4;
    bw1[t][1] = lg < 2 ? w1raw[t][1] : z4;
  }
  w3[0] = w3raw[0];
  w3[1] = net == 0 ? w3raw[1] : 0.0f;
  w3[2] = net == 0 ? w3raw[2] : 0.0f;
  f4 a1[1][4];
#pragma unroll
  for (int t = 0; t < 4; ++t) a1[0][t] = f4{0.f, 0.f, 0.f, 0.f};
  mfma_chunk<LDS_S, 1, 4, 4>(&sm.S[li][8 * lg], bw1, a1);
  PHASE_PROBE(10);
  float h1[1][1][4];
  unsigned h1w[1][1][6];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    float hv[4];
    unsigned wd[6];
#pragma unroll
    for (int q = 0; q < 4; ++q) hv[q] = tanh_f32(a1[0][t][q]);
    put3_col4<PS, LDP>(sm.h1p, (4 * lg) * LDP + 16 * (w + 4 * t) + li, hv, wd);
    if (t == j) {
#pragma unroll
      for (int q = 0; q < 4; ++q) h1[0][0][q] = hv[q];
#pragma unroll
      for (int q = 0; q < 6; ++q) h1w[0][0][q] = wd[q];
    }
  }
  PHASE_PROBE(11);
  rp_barrier();
  PHASE_PROBE(1);
  // ---- B: this tile of Z2 = H1 W2^T ------------------------------------------
  f4 acc[1][1];
  acc[0][0] = f4{0.f, 0.f, 0.f, 0.f};
  mfma_rows3<H, LDP, PS, H, 1, 1, true>(sm.h1p, P + L.W2 + (int64_t)net * H * H, n0, acc, &preB);
  PHASE_PROBE(2);
  // the H1 k-packed planes of this tile (and the padded chunk's zero rows)
  auto h1_kx = [&] {
    store_kx_w<H, R, 1, true>(H1x + net * 3 * PLX, PLX, r0, n0, h1w);
    if (r0 + R < kx_rows(mb) && r0 + R >= mb) {
      const float z[1][1][4] = {};
      store_kx<H, R, 1>(H1x + net * 3 * PLX, PLX, r0 + R, n0, z);
      store_kx<H, R, 1>(dZ2x + net * 3 * PLX, PLX, r0 + R, n0, z);
    }
  };
  h1_kx();
  WPre<1> preD;
  mfma_rows_pre<H, 1>(W2T + (int64_t)net * H * H, n0, preD);
  // ---- C (forward): tanh(fc2), this tile's output-layer partials -> X1 -------
  const int NQ = net == 0 ? 3 : 1;
  {
    float ps[12];
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4) {
      const float h = tanh_f32(acc[0][0][q4] + b2v);
      acc[0][0][q4] = h;
#pragma unroll
      for (int q = 0; q < 3; ++q) ps[q * 4 + q4] = fmaf(h, w3[q], 0.0f);
    }
    if (NQ == 3) {
      row16_sum_n<12>(ps);
    } else {
      float p0[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) p0[k] = ps[k];
      row16_sum_n<4>(p0);
#pragma unroll
      for (int k = 0; k < 4; ++k) ps[k] = p0[k];
    }
    if (li == 0) {
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        if (q >= NQ) break;
#pragma unroll
        for (int q4 = 0; q4 < 4; ++q4) sm.xs[4 * lg + q4][q][w] = ps[q * 4 + q4];
      }
    }
  }
  PHASE_PROBE(3);
  rp_barrier();
  static_assert(sizeof(sm.xs) == 96 * 8, "X1 staging: 96 8-B stores, six 128-B lines");
  if (tid < 96)
    cs_store8(reinterpret_cast<unsigned long long*>(&g_cs_x1[grp][j][0][0][0]) + tid,
              reinterpret_cast<const unsigned long long*>(&sm.xs[0][0][0])[tid]);
  if (!cs_handoff(ctr, 1u, &sm.ok)) {
    if constexpr (SPAN) satrl_span::exit(span, span_t0);
    return;
  }
  PHASE_PROBE(12);
  if (tid < kCsSplit * R * 3) {                                    // every quarter's partials -> osum[r][q][4jq + w]
    const int jq = tid / (R * 3), rq = tid % (R * 3), r = rq / 3, q = rq % 3;
    *reinterpret_cast<float4*>(&sm.osum[r][q][4 * jq]) =
        cs_load16(&g_cs_x1[grp][0][0][0][0], (int)sizeof(g_cs_x1[0]), ((jq * R + r) * 3 + q) * 16);
  }
  rp_barrier();
  PHASE_PROBE(13);
  // ---- C: the loss head (rowpass_kernel's, in every quarter; quarter 0 stores) --
  float* tp = ptail + (int64_t)rb * L.tail;
  if (tid < R) {
    const int r = tid, row = r0 + r;
    float dz[4] = {0.f, 0.f, 0.f, 0.f}, dls[4] = {0.f, 0.f, 0.f, 0.f};
    if (row < mb) {
      const float inv = inv_mb;
      if (net == 0) {
        float th[3], mu[3], dv[3], var[3], logp[3];
#pragma unroll
        for (int d = 0; d < 3; ++d) {
          th[d] = tanh_f32(out_sum<H / 16>(sm.osum, r, d) + sm.hb3s[d]);
          mu[d] = max_action * th[d];
          var[d] = sm.hcs[0][d];
          dv[d] = sm.ax[r][d] - mu[d];
          logp[d] = (-(dv[d] * dv[d]) / (2.0f * var[d]) - sm.hcs[1][d]) - kLogSqrt2Pi;
        }
        const float lsum = (logp[0] + logp[1]) + logp[2];
        const float lold = (sm.ax[r][3] + sm.ax[r][4]) + sm.ax[r][5];
        const float ratio = expf(lsum - lold);
        if (ratio_out != nullptr && j == 0) ratio_out[row] = ratio;
        const float adv = sm.ax[r][6];
        const float s1 = ratio * adv;
        const float cr = fminf(fmaxf(ratio, 1.0f - epsilon), 1.0f + epsilon);
        const float s2 = cr * adv;
        const float g1 = s1 < s2 ? 1.0f : (s1 == s2 ? 0.5f : 0.0f);
        const float g2 = s2 < s1 ? 1.0f : (s1 == s2 ? 0.5f : 0.0f);
        const float inside = (ratio >= 1.0f - epsilon && ratio <= 1.0f + epsilon) ? 1.0f : 0.0f;
        const float dmin = -inv;
        const float dratio = dmin * g1 * adv + dmin * g2 * adv * inside;
        const float dlsum = dratio * ratio;
#pragma unroll
        for (int d = 0; d < 3; ++d) {
          const float dvv = dv[d] * sm.hcs[2][d];
          const float dmu = dlsum * dvv;
          dz[d] = (dmu * max_action) * (1.0f - th[d] * th[d]);
          dls[d] = dlsum * (dv[d] * dvv - 1.0f) - ent_coef * inv;
        }
      } else {
        const float vc = out_sum<H / 16>(sm.osum, r, 0) + sm.hb3s[3];
        dz[3] = 2.0f * inv * (vc - sm.ax[r][7]);
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) sm.dz3s[r][q] = dz[q];
    float red[7] = {dz[0], dz[1], dz[2], dls[0], dls[1], dls[2], dz[3]};
    row16_sum_n<7>(red);
    if (r == 0 && j == 0) {
      if (net == 0) {
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          tp[5 * H + q] = red[q];
          tp[5 * H + 4 + q] = red[3 + q];
        }
        tp[5 * H + 3] = 0.0f;
        tp[5 * H + 7] = 0.0f;
      } else {
        tp[6 * H + 8] = red[6];
        tp[6 * H + 9] = 0.0f; tp[6 * H + 10] = 0.0f; tp[6 * H + 11] = 0.0f;
      }
    }
  }
  rp_barrier();
  PHASE_PROBE(4);
  // ---- C: tail of this tile (rowpass_kernel's), dZ2 planes -> LDS, k-packed, X2 --
  float d2v[1][1][4];
  unsigned d2w[1][1][6];
  auto tail = [&](auto actor) {
    constexpr bool ACT = decltype(actor)::value;
    constexpr int NC = ACT ? 3 : 1;
    const int n = n0 + li;
    float cb2 = 0.f, cw[NC];
#pragma unroll
    for (int q = 0; q < NC; ++q) cw[q] = 0.f;
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4) {
      const int r = 4 * lg + q4;
      const float h = acc[0][0][q4];
      float dh;
      if constexpr (ACT) dh = (sm.dz3s[r][0] * w3[0] + sm.dz3s[r][1] * w3[1]) + sm.dz3s[r][2] * w3[2];
      else dh = sm.dz3s[r][3] * w3[0];
      const float d2 = dh * (1.0f - h * h);
      d2v[0][0][q4] = d2;
      cb2 += d2;
      if constexpr (ACT) {
        cw[0] = fmaf(sm.dz3s[r][0], h, cw[0]); cw[1] = fmaf(sm.dz3s[r][1], h, cw[1]); cw[2] = fmaf(sm.dz3s[r][2], h, cw[2]);
      } else {
        cw[0] = fmaf(sm.dz3s[r][3], h, cw[0]);
      }
    }
    put3_col4<PS, LDP>(sm.dzp, (4 * lg) * LDP + n, d2v[0][0], d2w[0][0]);
    cb2 = xor32_sum(xor16_sum(cb2));
#pragma unroll
    for (int q = 0; q < NC; ++q) cw[q] = xor32_sum(xor16_sum(cw[q]));
    if (lg == 0) {
      tp[net * H + n] = cb2;
      if constexpr (ACT) {
        tp[2 * H + n] = cw[0]; tp[3 * H + n] = cw[1]; tp[4 * H + n] = cw[2];
      } else {
        tp[5 * H + 8 + n] = cw[0];
      }
    }
  };
  if (net == 0) tail(std::true_type{});
  else tail(std::false_type{});
  store_kx_w<H, R, 1, true>(dZ2x + net * 3 * PLX, PLX, r0, n0, d2w);
  rp_barrier();
  PHASE_PROBE(5);
  // this quarter's 64 columns of the three planes: 48 runs of 128 B, one run
  // per 16 lanes of one 8-B store instruction
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const int u = tid + NT * k, c8 = u & 15, pr = u >> 4, p = pr / R, r = pr % R;
    cs_store8(&g_cs_x2[grp][p][r][64 * j + 4 * c8],
              *reinterpret_cast<const unsigned long long*>(&sm.dzp[p * PS + r * LDP + 64 * j + 4 * c8]));
  }
  if (!cs_handoff(ctr, 2u, &sm.ok)) {
    if constexpr (SPAN) satrl_span::exit(span, span_t0);
    return;
  }
  PHASE_PROBE(14);
  // the other quarters' columns -> dzp (16-B runs)
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    const int u = tid + NT * k, c16 = u & 7, pr = (u >> 3) % (3 * R), jq = u / (8 * 3 * R);
    if (jq != j) {
      const int p = pr / R, r = pr % R, col = 64 * jq + 8 * c16;
      *reinterpret_cast<float4*>(&sm.dzp[p * PS + r * LDP + col]) =
          cs_load16(&g_cs_x2[grp][0][0][0], (int)sizeof(g_cs_x2[0]), ((p * R + r) * 256 + col) * 2);
    }
  }
  rp_barrier();
  // ---- D: this tile of dH1 = dZ2 W2 ------------------------------------------
  acc[0][0] = f4{0.f, 0.f, 0.f, 0.f};
  mfma_rows3<H, LDP, PS, H, 1, 1, true>(sm.dzp, W2T + (int64_t)net * H * H, n0, acc, &preD);
  PHASE_PROBE(6);
  // ---- E: dZ1, [dW1 | db1] rows of this tile (rowpass_kernel's) ---------------
  float* pw = pw1 + (int64_t)rb * 2 * H * 20 + (int64_t)net * H * 20;
#pragma unroll
  for (int q4 = 0; q4 < 4; ++q4) acc[0][0][q4] = acc[0][0][q4] * (1.0f - h1[0][0][q4] * h1[0][0][q4]);
#pragma unroll
  for (int hb = 0; hb < 2; ++hb) {
    f4 d = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) d = mfma4(acc[0][0][kk], sm.S[4 * lg + kk][16 * hb + li], d);
    const int kp = 16 * hb + li;
    if (kp < 20) {
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4) pw[(int64_t)(n0 + 4 * lg + q4) * 20 + kp] = d[q4];
    }
  }
  PHASE_PROBE(7);
  if constexpr (SPAN) satrl_span::exit(span, span_t0);
}

// ---------------------------------------------------------------------------
// policy: the rollout's forward passes on the rowpass's own MLP code
// (mlp_forward), one workgroup per 32-row block and net.
//   MODE 0  actor -> mean = max_action*tanh(.) -> Normal sample -> clamp ->
//           per-dim log-prob (ppo_continuous.py:176-189) for `nagents`
//           parameter sets (blockIdx % nagents = agent: P0 pursuer, P1
//           evader; the actor is net 0 of each flat layout)
//   MODE 1  critic value (net 1 of P0), ppo_continuous.py:200-201
// ---------------------------------------------------------------------------
// rows per policy/value workgroup (64-row tiles measured 62 vs 58.5 us per
// rollout step at 16k envs: fewer, larger workgroups lose more to the tail
// than the halved weight ingest saves)
constexpr int kPolRows = 32;   // rows per policy workgroup
constexpr int kPolNW = 8;      // waves per policy workgroup at H = 256 (16: 61.6 vs 52.3 us per rollout step;
                               // with the wave priority 46.5-47.6 vs 45.1-45.2 us per launch)

template <int H, int NW, int MODE, bool SPAN = false>
__global__ void __launch_bounds__(NW * 64) policy_kernel(int64_t N, const float* __restrict__ obs,
                                                     const float* __restrict__ P0, const float* __restrict__ P1,
                                                     int nagents, float max_action, uint32_t k00, uint32_t k01,
                                                     uint32_t k10, uint32_t k11, int64_t env_offset, uint64_t step,
                                                     const uint64_t* __restrict__ step_base,
                                                     float* __restrict__ act0, float* __restrict__ logp0,
                                                     float* __restrict__ act1, float* __restrict__ logp1,
                                                     float* __restrict__ value, unsigned long long* __restrict__ span) {
  const unsigned long long span_t0 = SPAN ? satrl_span::now() : 0ull;
  constexpr int R = kPolRows, RT = R / 16, CT = H / 16 / NW;
  // Two or more workgroups share a CU, and one finishing its output layer
  // would out-issue (oldest first) one that is still streaming W1 / W2: at
  // priority 3 until phase B's weight loads are out, a starting workgroup's
  // loads go first and overlap the other's tail (46 against 49 us per H 256
  // launch at 16 384 envs; bitwise unchanged)
  __builtin_amdgcn_s_setprio(3);
  const Layout L = layout(H);
  __shared__ MlpSmem<H, NW, R> sm;
  const int agent = MODE == 0 ? (int)(blockIdx.x % nagents) : 0;
  const int64_t r0 = (int64_t)(MODE == 0 ? blockIdx.x / nagents : blockIdx.x) * R;
  const float* P = agent == 0 ? P0 : P1;
  const int nvalid = (int)(N - r0 < R ? N - r0 : R);
  auto gather = [&](int t0, int nt) {
    const float* ob = obs + r0 * 18;
    if (nvalid == R && (reinterpret_cast<uintptr_t>(ob) & 15) == 0) {
      // a full block's R x 18 floats are one contiguous 16-B-aligned span:
      // every float4 in flight at once (R * 18 / 4 <= one per thread)
      static_assert(R * 18 / 4 <= 4 * 64, "one float4 per thread of the smallest workgroup");
      if (t0 < R * 18 / 4) {
        const float4 v = reinterpret_cast<const float4*>(ob)[t0];
        const float e4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int q = 4 * t0 + e;
          sm.S[q / 18][q % 18] = e4[e];
        }
      }
    } else {
      for (int q = t0; q < R * 18; q += nt) {
        const int r = q / 18, c = q % 18;
        sm.S[r][c] = r < nvalid ? obs[(r0 + r) * 18 + c] : 0.0f;
      }
    }
  };
  f4 acc[RT][CT];
  float h1[RT][CT][4];
  float w3[CT][3];
  unsigned h1w[RT][CT][6];
  mlp_forward<H, NW, R, false, true>(sm, P, MODE == 0 ? 0 : 1, nvalid, gather, nullptr, acc, h1, w3, h1w);
  const int r = threadIdx.x;
  if (r >= nvalid) {                                             // no barrier follows
    if constexpr (SPAN) satrl_span::exit(span, span_t0);
    return;
  }
  const int64_t i = r0 + r;
  if (MODE == 1) {
    value[i] = out_sum<H / 16>(sm.osum, r, 0) + P[L.b3c];
    if constexpr (SPAN) satrl_span::exit(span, span_t0);
    return;
  }
  float z[4];
  philox_normal4((uint64_t)(env_offset + i), step + (step_base ? *step_base : 0ull), agent == 0 ? k00 : k10,
                 agent == 0 ? k01 : k11, z);
  float* act = agent == 0 ? act0 : act1;
  float* logp = agent == 0 ? logp0 : logp1;
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    const float mu = max_action * tanh_f32(out_sum<H / 16>(sm.osum, r, d) + P[L.b3a + d]);   // 1.6 * tanh(mean_layer)
    gaussian_act(mu, P[L.ls + d], z[d], max_action, act[i * 3 + d], logp[i * 3 + d]);
  }
  if constexpr (SPAN) satrl_span::exit(span, span_t0);
}

// ---------------------------------------------------------------------------
// dW2 = dZ2^T H1 per net (fc2.weight.grad), split-K over the minibatch rows.
// Workgroup (net, 64x64 output tile, split s) sums rows [s*KR, (s+1)*KR) of
// its tile into slab p2[net][s] with f32 MFMA 16x16x4 (4 waves; wave w owns
// tile rows 16w.., all four 16-column tiles).  32-row chunks of dZ2 and H1
// stream global -> LDS by LDS-DMA (global_load_lds_dwordx4) through a ring of
// kDwD slots with kDwD-1 chunks in flight: counted vmcnt + raw s_barrier, no
// VGPR staging.  The LDS image is XOR-swizzled on the source address (16-float
// groups ^ row&3) so the MFMA operand reads are bank-conflict free.  Block
// b -> split b % S: with S = 8 every split's 16 tiles share one XCD's L2.
// Every sum has a fixed order.
// ---------------------------------------------------------------------------
constexpr int kDwKC = 32, kDwD = 4;   // rows per chunk, ring slots (4/6/8 slots measured alike)
typedef __attribute__((address_space(3))) void lds_void_t;

template <int H>
__global__ void __launch_bounds__(256) dw2_kernel(int mb, int S, int KR, int net_sel, const float* __restrict__ H1g,
                                                  const float* __restrict__ dZ2g, float* __restrict__ p2) {
  constexpr int TT = H / 64;
  __shared__ __attribute__((aligned(16))) float ring[kDwD][2][kDwKC][64];   // [slot][dZ2 | H1][row][64 cols]
  const int t = threadIdx.x, w = t >> 6, l = t & 63, li = l & 15, lg = l >> 4;
  const int b = blockIdx.x, s = b % S, tile = (b / S) % (TT * TT);
  const int net = net_sel < 0 ? b / (S * TT * TT) : net_sel;
  const int n0 = (tile / TT) * 64, m0 = (tile % TT) * 64;
  const int r_begin = s * KR, nvalid = min(mb, r_begin + KR) - r_begin;
  const float* Z = dZ2g + (int64_t)net * mb * H;
  const float* Y = H1g + (int64_t)net * mb * H;
  const int nchunks = KR / kDwKC;
  // wave w stages rows 8w..8w+7 of a chunk: two 1-KB pieces (4 rows x 64 floats) per operand
  auto stage = [&](int c) {
    const int slot = c % kDwD;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int row = 8 * w + 4 * u + (l >> 4), c4 = (l & 15) ^ (4 * (row & 3));   // swizzled source
      const int r = min(r_begin + c * kDwKC + row, mb - 1);                       // rows past the end: masked below
      __builtin_amdgcn_global_load_lds(Z + (int64_t)r * H + n0 + 4 * c4, (lds_void_t*)&ring[slot][0][8 * w + 4 * u][0],
                                       16, 0, 0);
      __builtin_amdgcn_global_load_lds(Y + (int64_t)r * H + m0 + 4 * c4, (lds_void_t*)&ring[slot][1][8 * w + 4 * u][0],
                                       16, 0, 0);
    }
  };
  f4 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < kDwD - 1; ++c) stage(c < nchunks ? c : nchunks - 1);
  for (int c = 0; c < nchunks; ++c) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"((kDwD - 2) * 4) : "memory");   // this wave's part of chunk c landed
    __builtin_amdgcn_s_barrier();                                            // every wave's part; slot c-1 free
    stage(c + kDwD - 1 < nchunks ? c + kDwD - 1 : nchunks - 1);             // (tail: a harmless reload)
    const int slot = c % kDwD, rows = nvalid - c * kDwKC;                    // rows >= `rows` are not ours
    // all of the chunk's operands first (40 ds_reads in flight), then the MFMAs
    float a[kDwKC / 4], bm[kDwKC / 4][4];
#pragma unroll
    for (int ks = 0; ks < kDwKC / 4; ++ks) {
      // A[n][k] = dZ2[row][n 16w+li], B[k][m] = H1[row][m 16j+li], row = 4ks+lg (row & 3 == lg)
      const int row = 4 * ks + lg;
      a[ks] = ring[slot][0][row][16 * (w ^ lg) + li];
      if (row >= rows) a[ks] = 0.0f;
#pragma unroll
      for (int j = 0; j < 4; ++j) bm[ks][j] = ring[slot][1][row][16 * (j ^ lg) + li];
    }
#pragma unroll
    for (int ks = 0; ks < kDwKC / 4; ++ks)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = mfma4(a[ks], bm[ks][j], acc[j]);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // acc[j][q] = dW2[n0 + 16w + 4lg + q][m0 + 16j + li]
  float* out = p2 + ((int64_t)net * S + s) * H * H;
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int q = 0; q < 4; ++q) out[(int64_t)(n0 + 16 * w + 4 * lg + q) * H + m0 + 16 * j + li] = acc[j][q];
}

// ---------------------------------------------------------------------------
// dW2 at H = 256 from k-packed bf16 planes (satrl_ppo_dw2_kx): the rowpass
// wrote H1 and dZ2 already split and laid out so that the reduction index
// (rows) runs along each 16-B run (store_kx), so no transpose, no split and
// no VGPR staging is left here.  Workgroup (net, 64x64 output tile, split s)
// sums rows [s*KR, (s+1)*KR) into slab p2[net][s]; its 4 waves own 32x32
// quarters (2 x 2 v_mfma_f32_16x16x32_bf16 tiles, six partial products
// each, smallest first, as the rowpass).  Each 32-row chunk of the tile's
// operands -- 2 tensors x 3 planes x 4 row groups x 64 columns x 16 B = 24 KB
// -- streams global -> LDS by LDS-DMA (global_load_lds_dwordx4, one 1-KB run
// per instruction, six per wave) through a kKxD-slot ring with counted vmcnt
// and raw s_barrier; the MFMA operands are ds_read_b128 of consecutive 16-B
// (row groups 16 B apart in bank space).  Every sum has a fixed order.
// ---------------------------------------------------------------------------
constexpr int kKxD = 3;        // ring slots (chunks kKxD - 1 ahead; 4 and 5 measured no faster, round 6)
// output tile width TW (64: 16 tiles per net, 8 splits of 512 rows at mb 4096;
// 128: 4 tiles per net, half the plane bytes per workgroup, 32 splits)
constexpr int kKxTW = 64;
template <int TW>
struct KxSmem {
  static constexpr int RUNS = 2 * 3 * 4, KG = TW * 16 + 16;     // runs per chunk (tensor x plane x row group), LDS bytes per run
  unsigned char ring[kKxD][RUNS][KG];
};
// the body of dw2_kx_kernel for workgroup b: the slab tile of (net, tile, split)
template <int TW>
__device__ __forceinline__ void dw2_kx_body(int b, int mb, int S, int KR, int net_sel,
                                            const unsigned short* __restrict__ H1x,
                                            const unsigned short* __restrict__ dZ2x, float* __restrict__ p2,
                                            KxSmem<TW>& sm) {
  constexpr int H = 256, TT = H / TW, RUNS = KxSmem<TW>::RUNS;
  constexpr int PPR = TW / 64;                                   // 1-KB pieces per run
  constexpr int XN = TW / 32, PW = RUNS * PPR / 4;              // 16x16 tiles per wave side, pieces per wave
  auto& ring = sm.ring;
  const int t = threadIdx.x, w = t >> 6, l = t & 63, li = l & 15, lg = l >> 4;
  const int s = b % S, tile = (b / S) % (TT * TT);
  const int net = net_sel < 0 ? b / (S * TT * TT) : net_sel;
  const int o0 = (tile / TT) * TW, n0 = (tile % TT) * TW;
  const int64_t PL = kx_rows(mb) * H;
  const int c_begin = s * (KR / 32), nch = (int)((min((int64_t)(s + 1) * KR, kx_rows(mb)) - (int64_t)s * KR) / 32);
  // piece v = (run u, 64-column half h) of chunk c: 64 columns x 8 rows, 1 KB contiguous in the plane
  auto stage = [&](int c) {
    const int slot = c % kKxD, cg = 4 * (c_begin + c);             // first row group of the chunk
#pragma unroll
    for (int k = 0; k < PW; ++k) {
      const int v = 4 * k + w, u = v / PPR, h = v % PPR;            // wave w: pieces w, w+4, ...
      const int tz = u / 12, p = (u / 4) % 3, q = u % 4;
      const unsigned short* src = (tz == 0 ? dZ2x : H1x) + (int64_t)net * 3 * PL + p * PL +
                                  ((int64_t)(cg + q) * H + (tz == 0 ? o0 : n0) + 64 * h + l) * 8;
      __builtin_amdgcn_global_load_lds(src, (lds_void_t*)&ring[slot][u][1024 * h], 16, 0, 0);
    }
  };
  const int wo = w >> 1, wn = w & 1;
  f4 acc[XN][XN];
#pragma unroll
  for (int x = 0; x < XN; ++x)
#pragma unroll
    for (int y = 0; y < XN; ++y) acc[x][y] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < kKxD - 1; ++c) stage(c < nch ? c : nch - 1);
  for (int c = 0; c < nch; ++c) {
    // this wave's pieces of chunk c landed, and its reads of chunk c-1's slot are done
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"((kKxD - 2) * PW) : "memory");
    __builtin_amdgcn_s_barrier();                                                   // every wave's; slot c-1 free
    stage(c + kKxD - 1 < nch ? c + kKxD - 1 : nch - 1);                             // (tail: a harmless reload)
    const int slot = c % kKxD;
    s8v a[XN][3], bq[XN][3];
#pragma unroll
    for (int x = 0; x < XN; ++x)
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        // A[o][k] = dZ2[row 8lg + k'][o], B[k][n] = H1[row][n]: group lg of plane p
        a[x][p] = *reinterpret_cast<const s8v*>(&ring[slot][0 * 12 + p * 4 + lg][((TW / 2) * wo + 16 * x + li) * 16]);
        bq[x][p] = *reinterpret_cast<const s8v*>(&ring[slot][1 * 12 + p * 4 + lg][((TW / 2) * wn + 16 * x + li) * 16]);
      }
#pragma unroll
    for (int x = 0; x < XN; ++x)
#pragma unroll
      for (int y = 0; y < XN; ++y) acc[x][y] = mfma6(a[x], bq[y], acc[x][y]);
    if (c + kKxD - 1 >= nch) __builtin_amdgcn_s_setprio(0);                         // (the last chunk is staged)
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // acc[x][y][q] = dW2[o0 + (TW/2)wo + 16x + 4lg + q][n0 + (TW/2)wn + 16y + li]
  float* out = p2 + ((int64_t)net * S + s) * H * H;
#pragma unroll
  for (int x = 0; x < XN; ++x)
#pragma unroll
    for (int y = 0; y < XN; ++y)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        out[(int64_t)(o0 + (TW / 2) * wo + 16 * x + 4 * lg + q) * H + n0 + (TW / 2) * wn + 16 * y + li] = acc[x][y][q];
      }
}
template <int TW, bool SPAN = false>
__global__ void __launch_bounds__(256) dw2_kx_kernel(int mb, int S, int KR, int net_sel,
                                                     const unsigned short* __restrict__ H1x,
                                                     const unsigned short* __restrict__ dZ2x, float* __restrict__ p2,
                                                     unsigned long long* __restrict__ span) {
  const unsigned long long span_t0 = SPAN ? satrl_span::now() : 0ull;
  __shared__ __attribute__((aligned(16))) KxSmem<TW> sm;
  // at priority 3 until a wave has staged its last chunk (dw2_kx_body), as
  // the policy kernel: in-graph step 48.8 against 49.1 us at mb 4096 over
  // eight alternations on two boxes, equal (49.4) in three on a third;
  // bitwise the same (EXPERIMENTS.md round 5)
  __builtin_amdgcn_s_setprio(3);
  dw2_kx_body<TW>(blockIdx.x, mb, S, KR, net_sel, H1x, dZ2x, p2, sm);
  if constexpr (SPAN) satrl_span::exit(span, span_t0);
}
// split-K ways of dw2_kx_kernel: about kKxWgs workgroups, whole 32-row chunks,
// no empty split; half as many up to kKxHalfMb rows (mb 512: 4 splits of 128
// rows, in-graph step 28.2-28.8 against 29.2-29.3 us over three
// alternations -- a slower dW2, 3.3 against 2.5 us, but half the slabs for
// the reduce and the boundary before it; at mb 1024 slower, 37.2 against
// 35.6; EXPERIMENTS.md round 6)
constexpr int kKxWgs = 256, kKxHalfMb = 512;
int kx_splits(int mb, int net) {
  const int target = mb <= kKxHalfMb ? kKxWgs / 2 : kKxWgs;
  const int tiles = (net < 0 ? 2 : 1) * (256 / kKxTW) * (256 / kKxTW), nch = (int)(kx_rows(mb) / 32);
  int S = target / tiles;
  if (S > nch) S = nch;
  if (S < 1) S = 1;
  const int cps = (nch + S - 1) / S;                               // chunks per split
  return (nch + cps - 1) / cps;
}

int dw2_splits(int H, int mb, int net) {
  const int tiles = (net < 0 ? 2 : 1) * (H / 64) * (H / 64);
  int S = 256 / tiles;
  const int maxS = (mb + kDwKC - 1) / kDwKC;
  if (S > maxS) S = maxS;
  if (S < 1) S = 1;
  const int KR = ((mb + S - 1) / S + kDwKC - 1) / kDwKC * kDwKC;
  return (mb + KR - 1) / KR;                                     // no empty split
}

// ---------------------------------------------------------------------------
// reduce: sums the three partial-slab families into G (fixed order) and/or
// writes per-block squared norms per net (f64).  Everything moves as float4
// (every region boundary and slab stride is a multiple of 4 floats, and a
// float4 never straddles the actor/critic boundary).  Block ranges:
//   [0, nb2)          W2 region: 64 float4 columns x 4 chunks, S split-K slabs [2][S][H][H]
//   [nb2, nb2+nb1)    W1 region: 32 float4 columns x 8 chunks, nw1 slabs [nw1][2][H][20]
//   [nb2+nb1, ...)    tail: 8 float4 columns x 32 chunks, nwg slabs [nwg][6H+12]
// A chunk sums slabs c, c+CH, ... in that order, every load issued before the
// first add (one latency round), then chunk 0 adds the CH partials in order.
// ---------------------------------------------------------------------------
struct RedGeom { int nb2, nb1, nbt, S, nw1, nwg, net, ch2; };   // net: -1 both, 0 actor, 1 critic
__host__ __device__ inline int n_blocks_dev(const RedGeom& g) { return g.nb2 + g.nb1 + g.nbt; }
// chunks per column: W1, tail, W2 regions; the W2 region at H = 64 takes
// kRedCH2x chunks (its 128 one-block dW2 slabs per minibatch: 8 per thread,
// one load round, 16 float4 columns per block, 4x the blocks)
constexpr int kRedCH1 = 8, kRedCHt = 32, kRedCH2 = 4, kRedCH2x = 16;
__host__ __device__ inline int red_ch2(int H) { return H == 64 ? kRedCH2x : kRedCH2; }

__device__ __forceinline__ float4 f4add(float4 a, float4 b) {
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}
// IEEE division per component, as torch's G.div_(world) after the all-reduce
__device__ __forceinline__ float4 f4div(float4 a, float d) {
  return make_float4(a.x / d, a.y / d, a.z / d, a.w / d);
}
__device__ __forceinline__ double sq4(float4 v) {
  return (double)v.x * v.x + (double)v.y * v.y + (double)v.z * v.z + (double)v.w * v.w;
}

// s += part[w] for w = first, first + step, ... < nparts (at most NL terms), in
// that order: the NL loads go out first (clamped indices, so none is a branch)
// and the terms past nparts are selected to +0, so the sum is the plain loop's
// bit for bit (s starts at +0 and a round-to-nearest sum is never -0, so
// s + 0 == s).  (A runtime-trip loop unrolled by the compiler puts its
// remainder iterations in a prologue of one load, wait, add each: the tail
// region's four slabs per thread were four serial load round trips.)
template <int NL>
__device__ __forceinline__ void sum_strided4(float4& s, const float4* __restrict__ part, int64_t stride4,
                                             int first, int step, int nparts, int64_t col) {
  float4 v[NL];
#pragma unroll
  for (int i = 0; i < NL; ++i) v[i] = part[(int64_t)min(first + i * step, nparts - 1) * stride4 + col];
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int i = 0; i < NL; ++i) s = f4add(s, first + i * step < nparts ? v[i] : z);
}

template <int CH>
__device__ __forceinline__ float4 chunk_sum4(const float4* __restrict__ part, int64_t stride4, int nparts,
                                             int64_t col, bool valid, float4* red) {
  constexpr int EB = 256 / CH;
  const int t = threadIdx.x, e = t % EB, c = t / EB;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (valid && nparts > 0) {                                       // (the clamped index needs a slab)
    const int m = (nparts + CH - 1) / CH;                          // terms of the longest chunk (uniform)
    if (m <= 2) sum_strided4<2>(s, part, stride4, c, CH, nparts, col);
    else if (m <= 4) sum_strided4<4>(s, part, stride4, c, CH, nparts, col);
    else if (m <= 8) sum_strided4<8>(s, part, stride4, c, CH, nparts, col);
    else   // (H = 64's 128 dW2 slabs: two rounds of 16; one round of 32 measured 1.1 us slower)
      for (int w = c; w < nparts; w += 16 * CH) sum_strided4<16>(s, part, stride4, w, CH, nparts, col);
  }
  red[t] = s;
  __syncthreads();
  float4 tot = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c == 0) {
    // the CH partials in order; their LDS reads go out 8 at a time ahead of
    // the adds (one read round trip per 8, not per 2)
    constexpr int KB = CH < 8 ? CH : 8;
#pragma unroll
    for (int k0 = 0; k0 < CH; k0 += KB) {
      float4 part[KB];
#pragma unroll
      for (int k = 0; k < KB; ++k) part[k] = red[(k0 + k) * EB + e];
#pragma unroll
      for (int k = 0; k < KB; ++k) tot = f4add(tot, part[k]);
    }
  }
  return tot;
}

// block-level f64 pair sum in fixed order, result in every thread
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double lane_d(double v, int lane) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), lane),
                          __builtin_amdgcn_readlane(__double2loint(v), lane));
}
// wave sum of (a, c) in a fixed order: DPP sums of each 16-lane row (the
// row16_sum stages), then rows 0..3 by readlane -- no ds_bpermute round trips
__device__ __forceinline__ void wave_sum2(double& a, double& c) {
  a += dpp_d<0xB1>(a); c += dpp_d<0xB1>(c);
  a += dpp_d<0x4E>(a); c += dpp_d<0x4E>(c);
  a += dpp_d<0x141>(a); c += dpp_d<0x141>(c);
  a += dpp_d<0x140>(a); c += dpp_d<0x140>(c);
  a = ((lane_d(a, 0) + lane_d(a, 16)) + lane_d(a, 32)) + lane_d(a, 48);
  c = ((lane_d(c, 0) + lane_d(c, 16)) + lane_d(c, 32)) + lane_d(c, 48);
}
// (256-thread blocks: reduce, adam and the peer all-reduce.  The four wave
// pairs are read at once; a loop over blockDim's wave count was one LDS read
// round trip per wave)
__device__ __forceinline__ void block_sum2(double& a, double& c, double* sh) {
  constexpr int NW = 4;
  wave_sum2(a, c);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { sh[2 * w] = a; sh[2 * w + 1] = c; }
  __syncthreads();
  double v[2 * NW];
#pragma unroll
  for (int k = 0; k < 2 * NW; ++k) v[k] = sh[k];
  a = 0.0; c = 0.0;
#pragma unroll
  for (int k = 0; k < NW; ++k) { a += v[2 * k]; c += v[2 * k + 1]; }
}

// what a reduce thread ends with: the float4 of G it wrote (lead threads
// only: live), its float4 index in the flat layout, and its net
struct RedOut {
  float4 v;
  int64_t e4;
  int net;
  bool live;
};

// the W1 and tail parts of reduce (block b of the W1 region, or of the tail
// after it: b counts from the first W1 block): sums the rowpass slabs into G
// (mode & 1) or rescales G (world > 1), and adds this thread's squares to
// (sa, sc).
__device__ __forceinline__ void reduce_w1_tail(int H, const Layout& L, const RedGeom& g, int b, int mode,
                                               const float* __restrict__ p1, const float* __restrict__ pt,
                                               float4* __restrict__ G4, int world, float4* red, double& sa,
                                               double& sc, RedOut& o) {
  const int t = threadIdx.x;
  if (b < g.nb1) {                                                // W1: [nw1] slabs of 2*H*20
    constexpr int EB = 256 / kRedCH1;
    const int64_t n4 = 2LL * H * 20 / 4, h4 = (int64_t)H * 20 / 4;
    const int64_t col = (g.net > 0 ? h4 : 0) + (int64_t)b * EB + (t % EB);
    const bool valid = col < (g.net == 0 ? h4 : n4), lead = t < EB;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (mode & 1) {
      v = chunk_sum4<kRedCH1>(reinterpret_cast<const float4*>(p1), n4, g.nw1, col, valid, red);
      if (lead && valid) G4[L.W1 / 4 + col] = v;
    } else if (lead && valid) {
      v = G4[L.W1 / 4 + col];
      if (world > 1) { v = f4div(v, (float)world); G4[L.W1 / 4 + col] = v; }
    }
    if (lead && valid) {                                          // (selects, not a pointer to sa / sc)
      const double q = sq4(v);
      const bool crit = col * 4 >= (int64_t)H * 20;
      sa += crit ? 0.0 : q;
      sc += crit ? q : 0.0;
    }
    o = RedOut{v, L.W1 / 4 + col, col * 4 >= (int64_t)H * 20 ? 1 : 0, lead && valid};
  } else {                                                        // tail: [nwg] slabs of 6H+12
    b -= g.nb1;
    constexpr int EB = 256 / kRedCHt;
    const int64_t n4 = L.tail / 4, col = (int64_t)b * EB + (t % EB);
    const bool valid = col < n4 && (g.net < 0 || net_of(L, L.b2 + col * 4, H) == g.net), lead = t < EB;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (mode & 1) {
      v = chunk_sum4<kRedCHt>(reinterpret_cast<const float4*>(pt), n4, g.nwg, col, valid, red);
      if (lead && valid) G4[L.b2 / 4 + col] = v;
    } else if (lead && valid) {
      v = G4[L.b2 / 4 + col];
      if (world > 1) { v = f4div(v, (float)world); G4[L.b2 / 4 + col] = v; }
    }
    const bool crit = valid && net_of(L, L.b2 + col * 4, H);
    if (lead && valid) {
      const double q = sq4(v);
      sa += crit ? 0.0 : q;
      sc += crit ? q : 0.0;
    }
    o = RedOut{v, L.b2 / 4 + col, crit ? 1 : 0, lead && valid};
  }
}

// block b of reduce: the W2 region, else the W1 / tail regions
__device__ __forceinline__ void reduce_block(int H, const Layout& L, const RedGeom& g, int b, int mode,
                                             const float* __restrict__ p2, const float* __restrict__ p1,
                                             const float* __restrict__ pt, float4* __restrict__ G4, int world,
                                             float4* red, double& sa, double& sc, RedOut& o) {
  const int t = threadIdx.x;
  const int64_t HH4 = (int64_t)H * H / 4;
  if (b < g.nb2) {                                                // W2: [2][S] split-K slabs of H*H
    const int EB = 256 / g.ch2;
    const int64_t col = (g.net > 0 ? HH4 : 0) + (int64_t)b * EB + (t % EB);
    const bool valid = col < (g.net < 0 ? 2 : g.net + 1) * HH4, lead = t < EB;
    const int net = col >= HH4;                                   // EB divides HH4: one net per block
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (mode & 1) {
      const float4* p2n = reinterpret_cast<const float4*>(p2) + (int64_t)net * g.S * HH4;
      v = g.ch2 == kRedCH2x ? chunk_sum4<kRedCH2x>(p2n, HH4, g.S, col - net * HH4, valid, red)
                            : chunk_sum4<kRedCH2>(p2n, HH4, g.S, col - net * HH4, valid, red);
      if (lead && valid) G4[col] = v;
    } else if (lead && valid) {
      v = G4[col];
      if (world > 1) { v = f4div(v, (float)world); G4[col] = v; }
    }
    if (lead && valid) {
      if (net) sc += sq4(v); else sa += sq4(v);
    }
    o = RedOut{v, col, net, lead && valid};
  } else {
    reduce_w1_tail(H, L, g, b - g.nb2, mode, p1, pt, G4, world, red, sa, sc, o);
  }
}

template <bool SPAN = false>
__global__ void __launch_bounds__(256) reduce_kernel(int H, RedGeom g, int mode, const float* __restrict__ p2,
                                                     const float* __restrict__ p1, const float* __restrict__ pt,
                                                     float* __restrict__ G, double* __restrict__ nsq,
                                                     double* __restrict__ steps, int world,
                                                     unsigned long long* __restrict__ span) {
  const unsigned long long span_t0 = SPAN ? satrl_span::now() : 0ull;
  const Layout L = layout(H);
  __shared__ double sh[8];
  __shared__ float4 red[256];
  double sa = 0.0, sc = 0.0;
  const int t = threadIdx.x;
  float4* G4 = reinterpret_cast<float4*>(G);
  // the step counters, read before the slab loads (read at the end they were
  // one more load round trip on block 0's path), advanced at the end
  double st0 = 0.0, st1 = 0.0;
  if ((mode & 2) && blockIdx.x == 0 && t == 0) { st0 = steps[0]; st1 = steps[1]; }
  RedOut o;
  reduce_block(H, L, g, blockIdx.x, mode, p2, p1, pt, G4, world, red, sa, sc, o);
  if (mode & 2) {
    block_sum2(sa, sc, sh);
    if (t == 0) {
      nsq[2 * blockIdx.x] = sa;
      nsq[2 * blockIdx.x + 1] = sc;
      if (blockIdx.x == 0) {
        if (g.net != 1) steps[0] = st0 + 1.0;
        if (g.net != 0) steps[1] = st1 + 1.0;
      }
    }
  }
  if constexpr (SPAN) satrl_span::exit(span, span_t0);
}

// dw2_kx and the reduce's W1 / tail regions in one launch
// (satrl_ppo_dw2_kx_w1): blocks [0, ndw) are dw2_kx_kernel's, the rest
// reduce_kernel's W1 / tail blocks.  Their slabs are the rowpass's (ready when
// this launch starts), so they run beside the dW2 stream instead of on the
// reduce's critical path; they write G's W1 / tail regions and (mode & 2)
// their squared-norm pairs at the reduce's own block indices, and
// satrl_ppo_reduce with mode bit 4 then runs the W2 blocks only.  Same code,
// same order: bitwise the two launches' G and norms.
template <int TW, bool SPAN = false>
__global__ void __launch_bounds__(256) dw2_kx_w1_kernel(int mb, int S, int KR, int net_sel,
                                                        const unsigned short* __restrict__ H1x,
                                                        const unsigned short* __restrict__ dZ2x, float* __restrict__ p2,
                                                        int ndw, RedGeom g, int mode, const float* __restrict__ p1,
                                                        const float* __restrict__ pt, float* __restrict__ G,
                                                        double* __restrict__ nsq, unsigned long long* __restrict__ span) {
  const unsigned long long span_t0 = SPAN ? satrl_span::now() : 0ull;
  __shared__ __attribute__((aligned(16))) KxSmem<TW> sm;
  if ((int)blockIdx.x < ndw) {
    __builtin_amdgcn_s_setprio(3);                               // (as dw2_kx_kernel)
    dw2_kx_body<TW>(blockIdx.x, mb, S, KR, net_sel, H1x, dZ2x, p2, sm);
  } else {
    // the reduce block's LDS (its float4 chunk sums, the block's norm pair)
    // inside the ring, which no block of this kind uses
    static_assert(sizeof(KxSmem<TW>) >= 256 * sizeof(float4) + 8 * sizeof(double), "reduce LDS in the ring");
    float4* red = reinterpret_cast<float4*>(&sm.ring[0][0][0]);
    double* sh = reinterpret_cast<double*>(reinterpret_cast<unsigned char*>(&sm.ring[0][0][0]) + 256 * sizeof(float4));
    const int b = (int)blockIdx.x - ndw;
    double sa = 0.0, sc = 0.0;
    RedOut o;
    reduce_w1_tail(256, layout(256), g, b, mode, p1, pt, reinterpret_cast<float4*>(G), 1, red, sa, sc, o);
    if (mode & 2) {
      block_sum2(sa, sc, sh);
      if (threadIdx.x == 0) {
        nsq[2 * (g.nb2 + b)] = sa;
        nsq[2 * (g.nb2 + b) + 1] = sc;
      }
    }
  }
  if constexpr (SPAN) satrl_span::exit(span, span_t0);
}

// ---------------------------------------------------------------------------
// adam: torch.nn.utils.clip_grad_norm_ + torch.optim.Adam (_single_tensor_adam)
// Every block first folds the per-block norms (fixed order, identical in
// every block).  Blocks [0, nbw): one 32x32 tile of a net's fc2.weight each,
// float4 per thread, and the updated tile goes out transposed through LDS
// into W2T (coalesced).  Blocks [nbw, ...): the rest of the layout, float4.
// ---------------------------------------------------------------------------
// The updated 32x32 tile tb of net's fc2.weight (thread t holds row n0 + t/8,
// columns k0 + (t%8)*4 .. +3 in v) into the fc2 operand image, the f32
// transpose (through LDS, so every store is coalesced).  Every thread of the
// block calls it.
__device__ __forceinline__ void w2x_tile(int H, int net, int tb, float4 v, void* __restrict__ W2X,
                                         float (&tile)[32][33]) {
  const int t = threadIdx.x, nl = t >> 3, kl = (t & 7) * 4, ntc = H / 32;
  const int n0 = (tb / ntc) * 32, k0 = (tb % ntc) * 32;
  const int64_t HH = (int64_t)H * H;
  tile[nl][kl] = v.x; tile[nl][kl + 1] = v.y; tile[nl][kl + 2] = v.z; tile[nl][kl + 3] = v.w;
  __syncthreads();
  // W2T[net][k0 + t/8][n0 + (t%8)*4 + q] = W2[net][n0 + (t%8)*4 + q][k0 + t/8]
  const float4 o = make_float4(tile[kl][nl], tile[kl + 1][nl], tile[kl + 2][nl], tile[kl + 3][nl]);
  reinterpret_cast<float4*>(W2X)[((int64_t)net * HH + (int64_t)(k0 + nl) * H + n0 + kl) / 4] = o;
}

// the fc2 operand image of P (satrl_ppo_w2x_sync): adam_kernel's W2 blocks
// without the step
__global__ void __launch_bounds__(256) w2x_sync_kernel(int H, int net_sel, const float* __restrict__ P,
                                                       void* __restrict__ W2X) {
  __shared__ float tile[32][33];
  const int t = threadIdx.x, ntc = H / 32, tb = blockIdx.x % (ntc * ntc);
  const int net = net_sel < 0 ? (int)(blockIdx.x / (ntc * ntc)) : net_sel;
  const int n = (tb / ntc) * 32 + (t >> 3), k = (tb % ntc) * 32 + (t & 7) * 4;
  const float4 v = *reinterpret_cast<const float4*>(P + (int64_t)net * H * H + (int64_t)n * H + k);
  w2x_tile(H, net, tb, v, W2X, tile);
}

__device__ __forceinline__ float adam_elem(float g, float& m, float& v, float p, float coef, float step_size,
                                           float bc2s, float w1, float w2, float beta2, float eps, int use_clip) {
  if (use_clip) g = g * coef;                                      // grads.mul_(clip_coef_clamped)
  m = m + w1 * (g - m);                                            // exp_avg.lerp_(grad, 1 - beta1)
  v = v * beta2 + w2 * (g * g);                                    // mul_(beta2).addcmul_(g, g, 1 - beta2)
  const float denom = sqrtf(v) / bc2s + eps;
  return p + (-step_size) * (m / denom);                           // addcdiv_(m, denom, -step_size)
}

template <bool SPAN = false>
__global__ void __launch_bounds__(256) adam_kernel(int H, int nblk, const double* __restrict__ nsq,
                                                   const double* __restrict__ steps, const double* __restrict__ bct,
                                                   int bct_len, const float* __restrict__ lr, float beta1,
                                                   float beta2, float eps, float max_norm, int use_clip,
                                                   const float* __restrict__ G, float* __restrict__ P,
                                                   float* __restrict__ M, float* __restrict__ V,
                                                   void* __restrict__ W2X, int net_sel,
                                                   unsigned long long* __restrict__ span) {
  const unsigned long long span_t0 = SPAN ? satrl_span::now() : 0ull;
  const Layout L = layout(H);
  __shared__ double sh[8];
  __shared__ float tile[32][33];
  const int t = threadIdx.x;
  const int ntc = H / 32, nbw = (net_sel < 0 ? 2 : 1) * ntc * ntc;
  // this thread's element (float4) and net, and whether it has one
  int64_t e4;
  int net;
  bool live = true;
  if ((int)blockIdx.x < nbw) {
    const int tb = blockIdx.x % (ntc * ntc);
    net = net_sel < 0 ? (int)(blockIdx.x / (ntc * ntc)) : net_sel;
    const int n = (tb / ntc) * 32 + (t >> 3), k = (tb % ntc) * 32 + (t & 7) * 4;
    e4 = ((int64_t)net * H * H + (int64_t)n * H + k) / 4;
  } else {
    e4 = L.W1 / 4 + (int64_t)(blockIdx.x - nbw) * 256 + t;
    live = e4 < L.total / 4;
    net = live ? net_of(L, e4 * 4, H) : 0;
    live = live && (net_sel < 0 || net == net_sel);
  }
  // the norm partials' loads go out first, this thread's G/M/V/P right
  // behind them: the fold below waits only for the partials (vmcnt is in
  // order), so the operand latency overlaps the fold
  // (all loads unconditional on clamped indices, so none becomes a branch)
  const double2* nsq2 = reinterpret_cast<const double2*>(nsq);
  double2 pn2[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) pn2[i] = nsq2[min(t + 256 * i, nblk - 1)];
  const float4* G4 = reinterpret_cast<const float4*>(G);
  float4* P4 = reinterpret_cast<float4*>(P);
  float4* M4 = reinterpret_cast<float4*>(M);
  float4* V4 = reinterpret_cast<float4*>(V);
  const int64_t el = live ? e4 : 0;
  const float4 g = G4[el];
  float4 m = M4[el], v = V4[el];
  const float4 p = P4[el];
  // both nets' step counts, learning rates and bias-correction rows, issued
  // here too: after the fold (a barrier the compiler does not hoist loads
  // over) they were two dependent load round trips on the kernel's path
  const double st_a = steps[0], st_c = steps[1];
  const float lr_a = lr[0], lr_c = lr[1];
  const int ka = (int)st_a, kc = (int)st_c;
  const double2* bct2 = reinterpret_cast<const double2*>(bct);
  const double2 bca = bct2[ka < bct_len ? ka : bct_len - 1], bcc = bct2[kc < bct_len ? kc : bct_len - 1];
  double a = 0.0, c = 0.0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {                                    // k = t, t+256, ... in order, as the loop
    // x * 1.0 == x, x * 0.0 + a == a for these non-negative sums: bitwise the
    // loop's skip, without a branch the compiler would sink the load into
    const double in = t + 256 * i < nblk ? 1.0 : 0.0;
    a += pn2[i].x * in;
    c += pn2[i].y * in;
  }
  if (nblk > 1024) {                                               // (not at the sizes in use)
    for (int k = t + 1024; k < nblk; k += 256) { a += nsq[2 * k]; c += nsq[2 * k + 1]; }
  }
  block_sum2(a, c, sh);
  // every thread folds the same partials in the same order, so each derives
  // its own net's constants (no second barrier)
  float coef, ss, b2s;
  {
    const double nn = net == 0 ? a : c;
    const float nrm = (float)sqrt(nn);
    coef = use_clip ? fminf(max_norm / (nrm + 1e-6f), 1.0f) : 1.0f;
    // bct[2*step] = 1 - beta1**step, bct[2*step+1] = sqrt(1 - beta2**step) (python float
    // math, as torch.optim.Adam computes them); constant 1.0 past the table
    const int st = net == 0 ? ka : kc;
    const double2 bc = net == 0 ? bca : bcc;
    const double bc1 = st < bct_len ? bc.x : 1.0;
    const double bc2s = st < bct_len ? bc.y : 1.0;
    ss = (float)((double)(net == 0 ? lr_a : lr_c) / bc1);
    b2s = (float)bc2s;
  }
  const float w1 = (float)(1.0 - (double)beta1);                  // lerp weight 1 - beta1
  const float w2 = (float)(1.0 - (double)beta2);
  if (!live) {                                                     // (W1.. tail blocks only: no barrier follows)
    if constexpr (SPAN) satrl_span::exit(span, span_t0);
    return;
  }
  float4 pn;
  pn.x = adam_elem(g.x, m.x, v.x, p.x, coef, ss, b2s, w1, w2, beta2, eps, use_clip);
  pn.y = adam_elem(g.y, m.y, v.y, p.y, coef, ss, b2s, w1, w2, beta2, eps, use_clip);
  pn.z = adam_elem(g.z, m.z, v.z, p.z, coef, ss, b2s, w1, w2, beta2, eps, use_clip);
  pn.w = adam_elem(g.w, m.w, v.w, p.w, coef, ss, b2s, w1, w2, beta2, eps, use_clip);
  P4[e4] = pn;
  M4[e4] = m;
  V4[e4] = v;
  if ((int)blockIdx.x < nbw && W2X != nullptr)                     // keep the fc2 operand image current
    w2x_tile(H, net, blockIdx.x % (ntc * ntc), pn, W2X, tile);
  if constexpr (SPAN) satrl_span::exit(span, span_t0);
}

// ---------------------------------------------------------------------------
// stage: the rows of a group of minibatches gathered contiguously, at the
// permutation offset a device counter holds (8 lanes x float4 per 128-B row)
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) stage_kernel(int64_t rows, const float4* __restrict__ src,
                                                    const int64_t* __restrict__ perm,
                                                    const int64_t* __restrict__ group, float4* __restrict__ stage) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, r = t >> 3;
  if (r >= rows) return;
  const int64_t row = perm[group[0] * rows + r];
  stage[t] = src[row * 8 + (t & 7)];
}

__global__ void group_advance_kernel(int64_t* group) { group[0] += 1; }

__global__ void __launch_bounds__(256) tanh_kernel(int64_t n, const float* __restrict__ x, float* __restrict__ y) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) y[i] = tanh_f32(x[i]);
}

// rows per rowpass workgroup for a minibatch of mb rows: kRowsShort at
// H = 256 up to kShortMb rows (twice the workgroups on the chip; measured
// faster up to mb 1024, even at 2048, slower at 4096: DESIGN.md §3.4)
constexpr int kShortMb = 1024;
int short_mb() { return kShortMb; }
int rows_per_wg(int H, int mb) {
  return (H == 256 && kRows == 32 && mb <= short_mb()) ? kRowsShort : kRows;
}
int n_head_wg(int H, int mb) {
  const int R = rows_per_wg(H, mb);
  return (mb + R - 1) / R;
}
int n_w1_wg(int H, int mb) { return n_head_wg(H, mb); }
// slab capacity a minibatch of mb rows needs, and any shorter one (a ragged
// tail of a minibatch above the short threshold can have more row blocks)
int n_head_wg_cap(int H, int mb) {
  const int m = mb < short_mb() ? mb : short_mb();
  const int a = n_head_wg(H, mb), b = m > 0 ? n_head_wg(H, m) : 0;
  return a > b ? a : b;
}
RedGeom geom(int H, int mb, int S, int net = -1) {
  const Layout L = layout(H);
  const int nn = net < 0 ? 2 : 1;                                  // nets covered
  RedGeom g;
  g.ch2 = red_ch2(H);
  g.nb2 = (int)((nn * (int64_t)H * H / 4 + (256 / g.ch2) - 1) / (256 / g.ch2));
  g.nb1 = (int)((nn * (int64_t)H * 20 / 4 + (256 / kRedCH1) - 1) / (256 / kRedCH1));
  g.nbt = (int)((L.tail / 4 + (256 / kRedCHt) - 1) / (256 / kRedCHt));
  g.S = S;
  g.nw1 = n_w1_wg(H, mb);
  g.nwg = n_head_wg(H, mb);
  g.net = net;
  return g;
}
int n_blocks(const RedGeom& g) { return g.nb2 + g.nb1 + g.nbt; }
int n_adam_blocks(int H, int net) {
  const Layout L = layout(H);
  return (net < 0 ? 2 : 1) * (H / 32) * (H / 32) + (int)(((L.total - L.W1) / 4 + 255) / 256);
}

bool valid_h(int H) { return H == 64 || H == 128 || H == 256; }

// Caller-buffer capacity checks of the C-ABI (before any launch).  A one-net
// call (net 1) addresses the second half of a [2][...] buffer, so only net 0
// may pass half the size.
int64_t nets_span(int net) { return net == 0 ? 1 : 2; }
// p2 [2][S][H][H] f32 split-K slabs
bool p2_fits(int H, int net, int S, int64_t p2_floats, const char* who) {
  const int64_t need = nets_span(net) * (int64_t)S * H * H;
  if (p2_floats >= need) return true;
  g_err = std::string(who) + ": p2 holds " + std::to_string(p2_floats) + " floats, " + std::to_string(S) +
          " splits need " + std::to_string(need);
  return false;
}
// the k-packed planes u16 [2][3][kx_rows(mb)][H] (satrl_ppo_kx_elems)
bool kx_fits(int H, int mb, int net, int64_t kx_elems, const char* who) {
  const int64_t need = nets_span(net) * 3 * kx_rows(mb) * H;
  if (kx_elems >= need) return true;
  g_err = std::string(who) + ": the H1x / dZ2x planes hold " + std::to_string(kx_elems) + " elements, mb " +
          std::to_string(mb) + " needs " + std::to_string(need);
  return false;
}

#define LAUNCH_CHECK()                                                      \
  do {                                                                      \
    hipError_t e_ = hipGetLastError();                                      \
    if (e_ != hipSuccess) { g_err = hipGetErrorString(e_); return -2; }     \
  } while (0)

// ---------------------------------------------------------------------------
// peer_allreduce: the data-parallel gradient all-reduce of G over the W ranks
// of one node without RCCL, fused with reduce_dp (G /= W, the per-block
// squared norms, the step counters).  Each rank owns an exchange buffer that
// every peer has mapped (IPC, uncached device memory); a value travels as
// an 8-B granule {tag, f32} written by ONE 8-B system-scope store, so the
// reader polls the granule itself -- no flag, no fence, no barrier
// (MI355X_MICROARCH.md "Valid forms", the granule form).  Two shots:
//   1 reduce-scatter push: every element goes to the rank that owns its
//     slice (slice j = elements [j*sl, (j+1)*sl)), slot [this rank];
//   2 the owner sums slot 0, 1, ... W-1 of each of its elements in rank
//     order, divides by W (IEEE, as reduce_dp) and pushes the result to
//     every rank's gather slot [owner];
//   3 every rank polls its gather slots into G.
// Each slice is summed once, in rank order, then broadcast, so every rank
// gets identical bits (and, at W = 2, the bits of c10d's SUM / 2).  Phase
// 3 hands out G exactly as reduce_kernel's blocks do (a float4 per lead
// thread of each of reduce_dp's blocks), so nsq is bitwise reduce_dp's.
// The grid is at most one workgroup per CU (satrl_ppo_allreduce_peer checks
// that every block is resident): a block takes reduce_dp's blocks
// blockIdx.x, + gridDim.x, ... in turn, so its spinning waves leave every CU
// room for the kernels of other streams or of a rank sharing the device.
// The tag is the call count: block b keeps its own counter in this rank's
// buffer and every call advances every counter once, on every rank (the
// grid size must be the same on every rank).  Waits are bounded (the
// caller's deadline in s_memrealtime ticks): a peer that never pushes sets
// the error word instead of hanging the GPU; satrl_peer_reset re-arms the
// counters and the word once every rank has stopped.
// ---------------------------------------------------------------------------
constexpr int kPeerMaxW = 8, kPeerMaxBlocks = 1024;
constexpr int64_t kPeerHdr = 4 * kPeerMaxBlocks + 256;           // epoch counters, error word
struct PeerBufs {
  unsigned long long* buf[kPeerMaxW];                              // every rank's buffer (this rank's own too)
};
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned int gu32;

__host__ __device__ inline int64_t peer_slice(int64_t n, int world) { return (n + world - 1) / world; }
__host__ __device__ inline int64_t peer_bytes(int64_t n, int world) {
  return kPeerHdr + 2 * (int64_t)world * peer_slice(n, world) * 8;
}

__device__ __forceinline__ void peer_push(unsigned long long* base, int64_t word, unsigned tag, float v) {
  __hip_atomic_store((gu64*)(base) + word, ((unsigned long long)tag << 32) | __float_as_uint(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_SYSTEM);
}
// the sticky error word of a rank's buffer (after the per-block counters)
__device__ __forceinline__ gu64* peer_err_word(unsigned long long* base) {
  return (gu64*)(base) + (4 * kPeerMaxBlocks) / 8;
}
// the value of a granule once its tag is `tag` (bounded wait: once a wait of
// this thread has run out, the rest return at once, the call being invalid).
// Every 16th poll also reads this rank's own error word (`mine`): a peer that
// gave up sets it in every rank's buffer, so the survivors fail fast instead
// of spending their own deadline
__device__ __forceinline__ float peer_pull(const unsigned long long* base, int64_t word, unsigned tag,
                                           unsigned long long* mine, unsigned long long t0,
                                           unsigned long long ticks, bool& ok) {
  const gu64* g = (const gu64*)(base) + word;
  unsigned long long x = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  unsigned polls = 0;
  while (ok && (unsigned)(x >> 32) != tag) {
    if (__builtin_amdgcn_s_memrealtime() - t0 > ticks) { ok = false; break; }   // 100 MHz ticks
    if ((++polls & 15u) == 0 &&
        __hip_atomic_load(peer_err_word(mine), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0ull) {
      ok = false;
      break;
    }
    __builtin_amdgcn_s_sleep(1);
    x = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  return __uint_as_float((unsigned)x);
}

// the float4 of G reduce_dp's block rb hands thread t (its lead threads), or -1
__device__ __forceinline__ int64_t peer_col(const Layout& L, const RedGeom& g, int H, int rb, int t) {
  if (rb < g.nb2) return t < 256 / g.ch2 ? (int64_t)rb * (256 / g.ch2) + t : -1;
  if (rb < g.nb2 + g.nb1) {
    const int64_t c = (int64_t)(rb - g.nb2) * (256 / kRedCH1) + t;
    return t < 256 / kRedCH1 && c < 2LL * H * 20 / 4 ? L.W1 / 4 + c : -1;
  }
  const int64_t c = (int64_t)(rb - g.nb2 - g.nb1) * (256 / kRedCHt) + t;
  return t < 256 / kRedCHt && c < L.tail / 4 ? L.b2 / 4 + c : -1;
}

__global__ void __launch_bounds__(256) peer_allreduce_kernel(int H, RedGeom g, int world, int rank, PeerBufs pb,
                                                             float* __restrict__ G, double* __restrict__ nsq,
                                                             double* __restrict__ steps,
                                                             unsigned long long ticks) {
  const Layout L = layout(H);
  __shared__ double sh[8];
  __shared__ unsigned tag_s;
  const int t = threadIdx.x, b = blockIdx.x, nb = gridDim.x, nred = n_blocks_dev(g);
  const int64_t n = L.total, sl = peer_slice(n, world);
  unsigned long long* mine = pb.buf[rank];
  const int64_t rs = kPeerHdr / 8, ag = rs + (int64_t)world * sl;  // word offsets of the two slot arrays
  __shared__ int failed_s;
  if (t == 0) {                                                    // this call's tag: block b's counter + 1
    // a failed call earlier (this rank's or a peer's: the word is set in every
    // buffer) makes every later call return at once -- the update is invalid
    // until PeerComm.reset, and the calls queued behind the failure (up to a
    // graph group of them) must not each spend the deadline again
    failed_s = __hip_atomic_load(peer_err_word(mine), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0ull;
    gu32* ep = (gu32*)(reinterpret_cast<unsigned*>(mine)) + b;
    const unsigned e = __hip_atomic_load(ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) + 1u;
    __hip_atomic_store(ep, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    tag_s = e;
  }
  __syncthreads();
  if (failed_s) return;                                            // (uniform: no barrier skipped by some threads)
  const unsigned tag = tag_s;
  double st0 = 0.0, st1 = 0.0;                                     // (advanced at the end, as reduce_kernel)
  if (b == 0 && t == 0) { st0 = steps[0]; st1 = steps[1]; }
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  bool ok = true;
  // 1: push this thread's float4 of each of the block's reduce_dp blocks to
  // the owners' reduce-scatter slot [rank]
  for (int rb = b; rb < nred; rb += nb) {
    const int64_t col = peer_col(L, g, H, rb, t);
    if (col >= 0) {
      const float4 v = reinterpret_cast<const float4*>(G)[col];
      const float e4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int64_t e = col * 4 + q, j = e / sl;
        peer_push(pb.buf[j], rs + (int64_t)rank * sl + (e - j * sl), tag, e4[q]);
      }
    }
  }
  // 2: this rank's slice, summed in rank order, / world, to every gather slot [rank]
  const int64_t mylen = min(sl, n - (int64_t)rank * sl);
  for (int64_t k = (int64_t)b * 256 + t; k < mylen; k += (int64_t)nb * 256) {
    float v = peer_pull(mine, rs + k, tag, mine, t0, ticks, ok);
    for (int j = 1; j < world; ++j) v += peer_pull(mine, rs + (int64_t)j * sl + k, tag, mine, t0, ticks, ok);
    v = v / (float)world;                                         // G.div_(world) (reduce_dp's IEEE division)
    // a sum with a missing term is never pushed: a slow peer must not take it
    // for a valid result (it times out, or fails fast on the error word)
    if (ok)
      for (int j = 0; j < world; ++j) peer_push(pb.buf[j], ag + (int64_t)rank * sl + k, tag, v);
  }
  // 3: gather each float4 into G; its squares to that reduce_dp block's norm pair
  for (int rb = b; rb < nred; rb += nb) {
    const int64_t col = peer_col(L, g, H, rb, t);
    double sa = 0.0, sc = 0.0;
    if (col >= 0) {
      float e4[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int64_t e = col * 4 + q, j = e / sl;
        e4[q] = peer_pull(mine, ag + j * sl + (e - j * sl), tag, mine, t0, ticks, ok);
      }
      const float4 v = make_float4(e4[0], e4[1], e4[2], e4[3]);
      reinterpret_cast<float4*>(G)[col] = v;
      const double q = sq4(v);
      const bool crit = net_of(L, col * 4, H);
      sa += crit ? 0.0 : q;
      sc += crit ? q : 0.0;
    }
    block_sum2(sa, sc, sh);
    if (t == 0) {
      nsq[2 * rb] = sa;
      nsq[2 * rb + 1] = sc;
    }
    __syncthreads();                                               // sh is reused by the next block_sum2
  }
  if (!ok) {
    // a peer never pushed (or one gave up): flag it in EVERY rank's buffer, so
    // a peer that is slow but alive fails this call too (its waits poll the
    // word) instead of completing it, and every later call returns at once
    for (int j = 0; j < world; ++j)
      __hip_atomic_store(peer_err_word(pb.buf[j]), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (b == 0 && t == 0) { steps[0] = st0 + 1.0; steps[1] = st1 + 1.0; }
}


struct SpanLaunch { int kind; int64_t off, waves; };
struct SpanState {
  unsigned long long* buf = nullptr;
  int64_t words = 0, used = 0;
  std::vector<SpanLaunch> log;
};
SpanState g_span;

}  // namespace

unsigned long long* satrl_span::take(int kind, int64_t waves) {
  if (!g_span.buf || waves <= 0 || g_span.used + 2 * waves > g_span.words) return nullptr;
  unsigned long long* p = g_span.buf + g_span.used;
  g_span.log.push_back(SpanLaunch{kind, g_span.used, waves});
  g_span.used += 2 * waves;
  return p;
}

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
  if (nwg) *nwg = n_head_wg_cap(H, mb);                         // >= every minibatch of <= mb rows
  if (nblk) *nblk = n_blocks(geom(H, mb, 1, -1));                 // >= the per-net counts
  return 0;
}

// the column-split short rowpass (rowpass_cs_kernel) runs when mb <= kCsMaxMb
// and every workgroup of its grid is resident at once (its groups wait on
// each other inside the launch): the occupancy API's answer, once per process
static bool cs_fits(int mb) {
  if (mb > kCsMaxMb) return false;
  static const int resident = [] {
    int dev = 0, per_cu = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, rowpass_cs_kernel<false>, kCsWaves * 64, 0) !=
            hipSuccess)
      return 0;
    return per_cu * cus;
  }();
  return (2 * ((mb + kRowsShort - 1) / kRowsShort) + 7) / 8 * 32 <= resident;
}

// every rowpass launch: fdw2 (H <= 128) writes the block's dW2 partial to p2
// instead of H1 / dZ2; ratio (nullable) receives the actor's per-row ratio
static int launch_rowpass(int H, int mb, int net, const float* src, const int64_t* idx, const float* P,
                          const void* W2X, float epsilon, float ent_coef, float max_action, float* H1, float* dZ2,
                          float* ptail, float* pw1, float* p2, float* ratio, bool fdw2, void* stream,
                          bool kx = false) {
  const int R = rows_per_wg(H, mb), nrb = n_head_wg(H, mb);
  dim3 g((net < 0 ? 2 : 1) * nrb);   // (row block, net) pairs, or row blocks of one net
  hipStream_t s = (hipStream_t)stream;
  // waves per workgroup: one 16-column tile per wave for both 16-row tiles
  const float inv_mb = 1.0f / (float)mb;
  const int nw = H == 64 ? 4 : H == 128 ? 8 : 16;                  // waves per workgroup
  // (H = 256, k-packed, both nets, mb <= kCsMaxMb: the column-split kernel,
  // groups of kCsSplit workgroups dealt in windows of 32 blocks)
  const bool cs = H == 256 && kx && R == kRowsShort && net < 0 && cs_fits(mb);
  const dim3 gc((unsigned)((2 * nrb + 7) / 8 * 32));
  unsigned long long* sp =
      satrl_span::take(satrl_span::kRowpass, cs ? (int64_t)gc.x * kCsWaves : (int64_t)g.x * nw);
#define RP_ARGS mb, src, idx, P, W2X, epsilon, ent_coef, max_action, H1, dZ2, ptail, pw1, net, p2, nrb, ratio, inv_mb, sp
#define RP_LAUNCH(HH, NWW, RR, F, K)                                                                          \
  do {                                                                                                        \
    if (sp) hipLaunchKernelGGL((rowpass_kernel<HH, NWW, RR, F, K, true>), g, dim3(NWW * 64), 0, s, RP_ARGS);  \
    else hipLaunchKernelGGL((rowpass_kernel<HH, NWW, RR, F, K>), g, dim3(NWW * 64), 0, s, RP_ARGS);           \
  } while (0)
  if (H == 64 && fdw2)
    RP_LAUNCH(64, 4, kRows, true, false);
  else if (H == 64)
    RP_LAUNCH(64, 4, kRows, false, false);
  else if (H == 128 && fdw2)
    RP_LAUNCH(128, 8, kRows, true, false);
  else if (H == 128)
    RP_LAUNCH(128, 8, kRows, false, false);
  else if (cs) {
    if (sp)
      hipLaunchKernelGGL(rowpass_cs_kernel<true>, gc, dim3(kCsWaves * 64), 0, s, mb, src, idx, P,
                         static_cast<const float*>(W2X), epsilon, ent_coef, max_action,
                         reinterpret_cast<unsigned short*>(H1), reinterpret_cast<unsigned short*>(dZ2), ptail, pw1,
                         ratio, inv_mb, sp);
    else
      hipLaunchKernelGGL(rowpass_cs_kernel<false>, gc, dim3(kCsWaves * 64), 0, s, mb, src, idx, P,
                         static_cast<const float*>(W2X), epsilon, ent_coef, max_action,
                         reinterpret_cast<unsigned short*>(H1), reinterpret_cast<unsigned short*>(dZ2), ptail, pw1,
                         ratio, inv_mb, nullptr);
  } else if (kx && R == kRowsShort)
    RP_LAUNCH(256, 16, kRowsShort, false, true);
  else if (kx)
    RP_LAUNCH(256, kNW256, kRows, false, true);
  else if (R == kRowsShort)
    RP_LAUNCH(256, 16, kRowsShort, false, false);
  else
    RP_LAUNCH(256, kNW256, kRows, false, false);
#undef RP_LAUNCH
#undef RP_ARGS
  LAUNCH_CHECK();
  return 0;
}

int satrl_ppo_rowpass(int H, int mb, int net, const float* src, const int64_t* idx, const float* P, const void* W2X,
                      float epsilon, float ent_coef, float max_action, float* H1, float* dZ2, float* ptail,
                      float* pw1, void* stream) {
  if (!valid_h(H) || mb <= 0 || net < -1 || net > 1 || !src || !P || !W2X || !H1 || !dZ2 || !ptail || !pw1)
    return -1;
  return launch_rowpass(H, mb, net, src, idx, P, W2X, epsilon, ent_coef, max_action, H1, dZ2, ptail, pw1, nullptr,
                        nullptr, false, stream);
}

int satrl_ppo_rowpass_ratio(int H, int mb, int net, const float* src, const int64_t* idx, const float* P,
                            const void* W2X, float epsilon, float ent_coef, float max_action, float* H1, float* dZ2,
                            float* ptail, float* pw1, float* ratio, void* stream) {
  if (!valid_h(H) || mb <= 0 || net < -1 || net > 1 || !src || !P || !W2X || !H1 || !dZ2 || !ptail || !pw1 ||
      !ratio)
    return -1;
  return launch_rowpass(H, mb, net, src, idx, P, W2X, epsilon, ent_coef, max_action, H1, dZ2, ptail, pw1, nullptr,
                        ratio, false, stream);
}

int satrl_ppo_row_blocks(int H, int mb) {
  if (!valid_h(H) || mb <= 0) return -1;
  return n_head_wg(H, mb);
}

int satrl_ppo_rowpass_dw2(int H, int mb, int net, const float* src, const int64_t* idx, const float* P,
                          const void* W2X, float epsilon, float ent_coef, float max_action, float* p2,
                          int64_t p2_floats, float* ptail, float* pw1, void* stream) {
  if ((H != 64 && H != 128) || mb <= 0 || net < -1 || net > 1 || !src || !P || !W2X || !p2 || !ptail || !pw1)
    return -1;
  if (!p2_fits(H, net, n_head_wg(H, mb), p2_floats, "satrl_ppo_rowpass_dw2")) return -1;   // one slab per row block
  return launch_rowpass(H, mb, net, src, idx, P, W2X, epsilon, ent_coef, max_action, nullptr, nullptr, ptail, pw1, p2,
                        nullptr, true, stream);
}

int64_t satrl_ppo_kx_elems(int H, int mb) {
  if (H != 256 || mb <= 0) return -1;
  return 2LL * 3 * kx_rows(mb) * H;
}

int satrl_ppo_rowpass_kx(int H, int mb, int net, const float* src, const int64_t* idx, const float* P, const void* W2X,
                         float epsilon, float ent_coef, float max_action, void* H1x, void* dZ2x, int64_t kx_elems,
                         float* ptail, float* pw1, void* stream) {
  if (H != 256 || mb <= 0 || net < -1 || net > 1 || !src || !P || !W2X || !H1x || !dZ2x ||
      !ptail || !pw1)
    return -1;
  if (!kx_fits(H, mb, net, kx_elems, "satrl_ppo_rowpass_kx")) return -1;
  return launch_rowpass(H, mb, net, src, idx, P, W2X, epsilon, ent_coef, max_action, static_cast<float*>(H1x),
                        static_cast<float*>(dZ2x), ptail, pw1, nullptr, nullptr, false, stream, true);
}

int satrl_ppo_rowpass_error(int* err, double timeout_s, void* stream) {
  if (!err || !(timeout_s > 0)) return -1;
  hipStream_t s = (hipStream_t)stream;
  // the error word lands in pinned memory behind an event that is polled
  // against the host deadline: a stream that never drains (e.g. a collective
  // of a dead peer queued before this call) returns -2 instead of hanging.
  // After a timeout the buffer and event stay with the stream (leaked): the
  // next call takes fresh ones.
  static std::mutex mu;
  static unsigned* host = nullptr;
  static hipEvent_t ev = nullptr;
  std::lock_guard<std::mutex> lock(mu);
  void *pe = nullptr, *pc = nullptr;
  if ((!host && hipHostMalloc((void**)&host, 4 * sizeof(unsigned), hipHostMallocDefault) != hipSuccess) ||
      (!ev && hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) ||
      hipGetSymbolAddress(&pe, HIP_SYMBOL(g_cs_err)) != hipSuccess ||
      hipGetSymbolAddress(&pc, HIP_SYMBOL(g_cs_ctr)) != hipSuccess ||
      hipMemcpyAsync(host, pe, sizeof(unsigned), hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipEventRecord(ev, s) != hipSuccess) {
    g_err = "satrl_ppo_rowpass_error: reading the exchange error word failed";
    return -1;
  }
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const hipError_t q = hipEventQuery(ev);
    if (q == hipSuccess) break;
    if (q != hipErrorNotReady) {
      g_err = "satrl_ppo_rowpass_error: waiting for the stream failed";
      return -1;
    }
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s) {
      host = nullptr;
      ev = nullptr;
      g_err = "satrl_ppo_rowpass_error: the stream did not drain within the deadline";
      return -2;
    }
    std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
  const unsigned e = host[0];
  *err = e != 0;
  if (e != 0 && (hipMemsetAsync(pe, 0, sizeof(g_cs_err), s) != hipSuccess ||
                 hipMemsetAsync(pc, 0, sizeof(g_cs_ctr), s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)) {
    g_err = "satrl_ppo_rowpass_error: re-arming the exchange state failed";
    return -1;
  }
  return 0;
}

int satrl_ppo_rowpass_fault_inject(int group, unsigned value, void* stream) {
  if (group < 0 || group >= kCsMaxGroups) return -1;
  hipStream_t s = (hipStream_t)stream;
  void* pc = nullptr;
  if (hipGetSymbolAddress(&pc, HIP_SYMBOL(g_cs_ctr)) != hipSuccess ||
      hipMemcpyAsync(static_cast<unsigned*>(pc) + (size_t)group * 32, &value, sizeof(value), hipMemcpyHostToDevice, s) !=
          hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess) {
    g_err = "satrl_ppo_rowpass_fault_inject: writing the exchange counter failed";
    return -1;
  }
  return 0;
}

int satrl_ppo_dw2_kx_splits(int H, int mb, int net) {
  if (H != 256 || mb <= 0 || net < -1 || net > 1) return -1;
  return kx_splits(mb, net);
}

int satrl_ppo_dw2_kx(int H, int mb, int net, int S, const void* H1x, const void* dZ2x, int64_t kx_elems, float* p2,
                     int64_t p2_floats, void* stream) {
  if (H != 256 || mb <= 0 || net < -1 || net > 1 || S < 1 || !H1x || !dZ2x || !p2) return -1;
  const int nch = (int)(kx_rows(mb) / 32), cps = (nch + S - 1) / S;
  if ((int64_t)cps * (S - 1) >= nch) return -1;                  // an empty split: use satrl_ppo_dw2_kx_splits
  if (!kx_fits(H, mb, net, kx_elems, "satrl_ppo_dw2_kx") || !p2_fits(H, net, S, p2_floats, "satrl_ppo_dw2_kx"))
    return -1;
  const dim3 g((unsigned)((net < 0 ? 2 : 1) * (256 / kKxTW) * (256 / kKxTW) * S));
  unsigned long long* sp = satrl_span::take(satrl_span::kDw2, (int64_t)g.x * 4);
  if (sp)
    hipLaunchKernelGGL((dw2_kx_kernel<kKxTW, true>), g, dim3(256), 0, (hipStream_t)stream, mb, S, cps * 32, net,
                       static_cast<const unsigned short*>(H1x), static_cast<const unsigned short*>(dZ2x), p2, sp);
  else
    hipLaunchKernelGGL((dw2_kx_kernel<kKxTW>), g, dim3(256), 0, (hipStream_t)stream, mb, S, cps * 32, net,
                       static_cast<const unsigned short*>(H1x), static_cast<const unsigned short*>(dZ2x), p2, sp);
  LAUNCH_CHECK();
  return 0;
}

int satrl_ppo_dw2_kx_w1(int H, int mb, int net, int S, const void* H1x, const void* dZ2x, int64_t kx_elems, float* p2,
                        int64_t p2_floats, int mode, const float* p1, const float* pt, float* G, double* nsq,
                        void* stream) {
  if (H != 256 || mb <= 0 || net < -1 || net > 1 || S < 1 || !H1x || !dZ2x || !p2) return -1;
  if (!(mode == 1 || mode == 3) || !p1 || !pt || !G || ((mode & 2) && !nsq)) return -1;
  const int nch = (int)(kx_rows(mb) / 32), cps = (nch + S - 1) / S;
  if ((int64_t)cps * (S - 1) >= nch) return -1;                  // an empty split: use satrl_ppo_dw2_kx_splits
  if (!kx_fits(H, mb, net, kx_elems, "satrl_ppo_dw2_kx_w1") || !p2_fits(H, net, S, p2_floats, "satrl_ppo_dw2_kx_w1"))
    return -1;
  const RedGeom rg = geom(H, mb, S, net);
  const int ndw = (net < 0 ? 2 : 1) * (256 / kKxTW) * (256 / kKxTW) * S;
  const dim3 g((unsigned)(ndw + rg.nb1 + rg.nbt));
  unsigned long long* sp = satrl_span::take(satrl_span::kDw2, (int64_t)g.x * 4);
  const unsigned short *h1 = static_cast<const unsigned short*>(H1x), *dz = static_cast<const unsigned short*>(dZ2x);
  if (sp)
    hipLaunchKernelGGL((dw2_kx_w1_kernel<kKxTW, true>), g, dim3(256), 0, (hipStream_t)stream, mb, S, cps * 32, net, h1,
                       dz, p2, ndw, rg, mode, p1, pt, G, nsq, sp);
  else
    hipLaunchKernelGGL((dw2_kx_w1_kernel<kKxTW>), g, dim3(256), 0, (hipStream_t)stream, mb, S, cps * 32, net, h1, dz,
                       p2, ndw, rg, mode, p1, pt, G, nsq, sp);
  LAUNCH_CHECK();
  return 0;
}

int satrl_ppo_dw2_splits(int H, int mb) {
  if (!valid_h(H) || mb <= 0) return -1;
  return dw2_splits(H, mb, -1);
}

int satrl_ppo_dw2(int H, int mb, int net, int S, const float* H1, const float* dZ2, float* p2, int64_t p2_floats,
                  void* stream) {
  if (!valid_h(H) || mb <= 0 || net < -1 || net > 1 || S < 1 || !H1 || !dZ2 || !p2) return -1;
  const int KR = ((mb + S - 1) / S + kDwKC - 1) / kDwKC * kDwKC;
  if ((int64_t)KR * (S - 1) >= mb) return -1;                    // an empty split: use satrl_ppo_dw2_splits
  if (!p2_fits(H, net, S, p2_floats, "satrl_ppo_dw2")) return -1;
  const dim3 g((unsigned)((net < 0 ? 2 : 1) * (H / 64) * (H / 64) * S));
  hipStream_t st = (hipStream_t)stream;
  if (H == 64)
    hipLaunchKernelGGL(dw2_kernel<64>, g, dim3(256), 0, st, mb, S, KR, net, H1, dZ2, p2);
  else if (H == 128)
    hipLaunchKernelGGL(dw2_kernel<128>, g, dim3(256), 0, st, mb, S, KR, net, H1, dZ2, p2);
  else
    hipLaunchKernelGGL(dw2_kernel<256>, g, dim3(256), 0, st, mb, S, KR, net, H1, dZ2, p2);
  LAUNCH_CHECK();
  return 0;
}

int satrl_ppo_reduce(int H, int mb, int net, int S, int mode, const float* p2, int64_t p2_floats, const float* p1,
                     const float* pt, float* G, double* nsq, double* steps, void* stream) {
  // mode bit 4: the W2 region only (satrl_ppo_dw2_kx_w1 summed the others)
  const bool w2_only = (mode & 4) != 0;
  mode &= 3;
  if (!valid_h(H) || mb <= 0 || net < -1 || net > 1 || S < 1 || mode < 1 || !G || (w2_only && !(mode & 1)))
    return -1;
  if ((mode & 1) && (!p2 || (!w2_only && (!p1 || !pt)))) return -1;
  if ((mode & 1) && !p2_fits(H, net, S, p2_floats, "satrl_ppo_reduce")) return -1;   // the slabs it reads
  if ((mode & 2) && (!nsq || !steps)) return -1;
  const RedGeom g = geom(H, mb, S, net);
  const int nb = w2_only ? g.nb2 : n_blocks(g);
  unsigned long long* sp = satrl_span::take(satrl_span::kReduce, (int64_t)nb * 4);
  if (sp)
    hipLaunchKernelGGL(reduce_kernel<true>, dim3(nb), dim3(256), 0, (hipStream_t)stream, H, g, mode, p2, p1, pt, G,
                       nsq, steps, 1, sp);
  else
    hipLaunchKernelGGL(reduce_kernel<false>, dim3(nb), dim3(256), 0, (hipStream_t)stream, H, g, mode, p2, p1, pt, G,
                       nsq, steps, 1, sp);
  LAUNCH_CHECK();
  return 0;
}

int satrl_ppo_reduce_dp(int H, int mb, int net, int world, float* G, double* nsq, double* steps, void* stream) {
  if (!valid_h(H) || mb <= 0 || net < -1 || net > 1 || world < 1 || !G || !nsq || !steps) return -1;
  const RedGeom g = geom(H, mb, 1, net);
  hipLaunchKernelGGL(reduce_kernel<false>, dim3(n_blocks(g)), dim3(256), 0, (hipStream_t)stream, H, g, 2, nullptr,
                     nullptr, nullptr, G, nsq, steps, world, nullptr);
  LAUNCH_CHECK();
  return 0;
}

int satrl_peer_buffer_bytes(int64_t n, int world, int64_t* bytes) {
  if (n <= 0 || world < 1 || world > kPeerMaxW || !bytes) return -1;
  *bytes = peer_bytes(n, world);
  return 0;
}

int satrl_peer_alloc(int64_t bytes, void** buf, void* ipc_handle) {
  if (bytes <= 0 || !buf || !ipc_handle) return -1;
  void* p = nullptr;
  if (hipExtMallocWithFlags(&p, (size_t)bytes, hipDeviceMallocUncached) != hipSuccess) {
    g_err = "satrl_peer_alloc: hipExtMallocWithFlags(uncached) failed";
    return -2;
  }
  hipIpcMemHandle_t h;
  if (hipMemset(p, 0, (size_t)bytes) != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
      hipIpcGetMemHandle(&h, p) != hipSuccess) {
    (void)hipFree(p);
    g_err = "satrl_peer_alloc: zeroing / hipIpcGetMemHandle failed";
    return -2;
  }
  std::memcpy(ipc_handle, &h, sizeof(h));
  *buf = p;
  return 0;
}

int satrl_peer_open(const void* ipc_handle, void** buf) {
  if (!ipc_handle || !buf) return -1;
  hipIpcMemHandle_t h;
  std::memcpy(&h, ipc_handle, sizeof(h));
  if (hipIpcOpenMemHandle(buf, h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
    g_err = "satrl_peer_open: hipIpcOpenMemHandle failed";
    return -2;
  }
  return 0;
}

int satrl_peer_close(void* buf) { return buf && hipIpcCloseMemHandle(buf) == hipSuccess ? 0 : -2; }
int satrl_peer_free(void* buf) { return buf && hipFree(buf) == hipSuccess ? 0 : -2; }

int satrl_peer_error(const void* buf, uint64_t* err, void* stream) {
  if (!buf || !err) return -1;
  hipStream_t st = (hipStream_t)stream;               // ordered after the calls queued on `stream`
  return hipMemcpyAsync(err, static_cast<const char*>(buf) + 4 * kPeerMaxBlocks, 8, hipMemcpyDeviceToHost, st) ==
                     hipSuccess &&
                 hipStreamSynchronize(st) == hipSuccess
             ? 0
             : -2;
}

int satrl_peer_reset(void* buf, int64_t bytes, void* stream) {
  if (!buf || bytes < kPeerHdr) return -1;
  hipStream_t st = (hipStream_t)stream;
  return hipMemsetAsync(buf, 0, (size_t)bytes, st) == hipSuccess && hipStreamSynchronize(st) == hipSuccess ? 0 : -2;
}

// the peer kernel's grid at width H: reduce_dp's block count, capped at one
// block per CU of the current device and at what can be resident at once
int satrl_peer_blocks(int H, int* blocks) {
  if (!valid_h(H) || !blocks) return -1;
  int dev = 0, cus = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, peer_allreduce_kernel, 256, 0) != hipSuccess) {
    g_err = "satrl_peer_blocks: device query failed";
    return -2;
  }
  const int nb = n_blocks(geom(H, 1, 1, -1));
  *blocks = std::min(nb, std::min(cus, cus * per_cu));
  return *blocks > 0 ? 0 : -2;
}

int satrl_ppo_allreduce_peer(int H, int mb, int world, int rank, void* const* bufs, float* G, double* nsq,
                             double* steps, int blocks, double timeout_s, void* stream) {
  if (!valid_h(H) || mb <= 0 || world < 1 || world > kPeerMaxW || rank < 0 || rank >= world || !bufs || !G || !nsq ||
      !steps || blocks < 1 || blocks > kPeerMaxBlocks || !(timeout_s > 0.0) || timeout_s > 1e7)
    return -1;
  PeerBufs pb{};
  for (int j = 0; j < world; ++j) {
    if (!bufs[j]) return -1;
    pb.buf[j] = static_cast<unsigned long long*>(bufs[j]);
  }
  // every block must be resident at once (a block waits on values other blocks push)
  int dev = 0, cus = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, peer_allreduce_kernel, 256, 0) != hipSuccess) {
    g_err = "satrl_ppo_allreduce_peer: device query failed";
    return -2;
  }
  if (blocks > cus * per_cu) {
    g_err = "satrl_ppo_allreduce_peer: " + std::to_string(blocks) + " blocks cannot all be resident (" +
            std::to_string(cus) + " CUs x " + std::to_string(per_cu) + ")";
    return -1;
  }
  const RedGeom g = geom(H, mb, 1, -1);
  const unsigned long long ticks = (unsigned long long)(timeout_s * 1e8);   // s_memrealtime: 100 MHz
  hipLaunchKernelGGL(peer_allreduce_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, H, g, world, rank, pb, G,
                     nsq, steps, ticks);
  LAUNCH_CHECK();
  return 0;
}

int satrl_ppo_adam(int H, int mb, int net, const double* nsq, const double* steps, const double* bct, int bct_len,
                   const float* lr, float beta1, float beta2, float eps, float max_norm, int use_clip, const float* G,
                   float* P, float* M, float* V, void* W2X, void* stream) {
  if (!valid_h(H) || mb <= 0 || net < -1 || net > 1 || !nsq || !steps || !bct || bct_len < 1 || !lr || !G || !P ||
      !M || !V)
    return -1;
  const int nblk = n_blocks(geom(H, mb, 1, net));
  unsigned long long* sp = satrl_span::take(satrl_span::kAdam, (int64_t)n_adam_blocks(H, net) * 4);
  if (sp)
    hipLaunchKernelGGL(adam_kernel<true>, dim3(n_adam_blocks(H, net)), dim3(256), 0, (hipStream_t)stream, H, nblk,
                       nsq, steps, bct, bct_len, lr, beta1, beta2, eps, max_norm, use_clip, G, P, M, V, W2X, net, sp);
  else
    hipLaunchKernelGGL(adam_kernel<false>, dim3(n_adam_blocks(H, net)), dim3(256), 0, (hipStream_t)stream, H, nblk,
                       nsq, steps, bct, bct_len, lr, beta1, beta2, eps, max_norm, use_clip, G, P, M, V, W2X, net, sp);
  LAUNCH_CHECK();
  return 0;
}

int64_t satrl_ppo_w2x_floats(int H) { return valid_h(H) ? w2x_floats(H) : -1; }

int satrl_ppo_w2x_sync(int H, int net, const float* P, void* W2X, void* stream) {
  if (!valid_h(H) || net < -1 || net > 1 || !P || !W2X) return -1;
  const int ntc = H / 32;
  hipLaunchKernelGGL(w2x_sync_kernel, dim3((net < 0 ? 2 : 1) * ntc * ntc), dim3(256), 0, (hipStream_t)stream, H, net,
                     P, W2X);
  LAUNCH_CHECK();
  return 0;
}

int satrl_ppo_stage(int64_t rows, const float* src, const int64_t* perm, const int64_t* group, float* stage,
                    void* stream) {
  if (rows <= 0 || !src || !perm || !group || !stage) return -1;
  hipLaunchKernelGGL(stage_kernel, dim3((unsigned)((rows * 8 + 255) / 256)), dim3(256), 0, (hipStream_t)stream, rows,
                     reinterpret_cast<const float4*>(src), perm, group, reinterpret_cast<float4*>(stage));
  LAUNCH_CHECK();
  return 0;
}

int satrl_ppo_group_advance(int64_t* group, void* stream) {
  if (!group) return -1;
  hipLaunchKernelGGL(group_advance_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, group);
  LAUNCH_CHECK();
  return 0;
}

int satrl_policy_act(int H, int64_t N, const float* obs, const float* P0, const float* P1, float max_action,
                     uint64_t seed, int64_t env_offset, uint64_t step, const uint64_t* step_base, float* act0,
                     float* logp0, float* act1, float* logp1, void* stream) {
  if (!valid_h(H) || N <= 0 || !obs || !P0 || !act0 || !logp0) return -1;
  if (P1 && (!act1 || !logp1)) return -1;
  const int nag = P1 ? 2 : 1;
  uint32_t k00, k01, k10, k11;
  philox_key(seed, 0, k00, k01);
  philox_key(seed, 1, k10, k11);
  const dim3 g((unsigned)(nag * ((N + kPolRows - 1) / kPolRows)));
  hipStream_t s = (hipStream_t)stream;
  const int nw = H == 64 ? 4 : H == 128 ? 8 : kPolNW;
  unsigned long long* sp = satrl_span::take(satrl_span::kPolicyAct, (int64_t)g.x * nw);
#define POL_ARGS N, obs, P0, P1, nag, max_action, k00, k01, k10, k11, env_offset, step, step_base, act0, logp0, act1, \
                 logp1, nullptr, sp
#define POL_LAUNCH(HH, NWW)                                                                               \
  do {                                                                                                    \
    if (sp) hipLaunchKernelGGL((policy_kernel<HH, NWW, 0, true>), g, dim3(NWW * 64), 0, s, POL_ARGS);     \
    else hipLaunchKernelGGL((policy_kernel<HH, NWW, 0>), g, dim3(NWW * 64), 0, s, POL_ARGS);              \
  } while (0)
  if (H == 64)
    POL_LAUNCH(64, 4);
  else if (H == 128)
    POL_LAUNCH(128, 8);
  else
    POL_LAUNCH(256, kPolNW);
#undef POL_LAUNCH
#undef POL_ARGS
  LAUNCH_CHECK();
  return 0;
}

int satrl_policy_value(int H, int64_t N, const float* obs, const float* P, float* v_out, void* stream) {
  if (!valid_h(H) || N <= 0 || !obs || !P || !v_out) return -1;
  const dim3 g((unsigned)((N + kPolRows - 1) / kPolRows));
  hipStream_t s = (hipStream_t)stream;
  const int nw = H == 64 ? 4 : H == 128 ? 8 : kPolNW;
  unsigned long long* sp = satrl_span::take(satrl_span::kPolicyValue, (int64_t)g.x * nw);
#define VAL_ARGS N, obs, P, nullptr, 1, 0.0f, 0u, 0u, 0u, 0u, (int64_t)0, (uint64_t)0, nullptr, nullptr, nullptr, \
                 nullptr, nullptr, v_out, sp
#define VAL_LAUNCH(HH, NWW)                                                                               \
  do {                                                                                                    \
    if (sp) hipLaunchKernelGGL((policy_kernel<HH, NWW, 1, true>), g, dim3(NWW * 64), 0, s, VAL_ARGS);     \
    else hipLaunchKernelGGL((policy_kernel<HH, NWW, 1>), g, dim3(NWW * 64), 0, s, VAL_ARGS);              \
  } while (0)
  if (H == 64)
    VAL_LAUNCH(64, 4);
  else if (H == 128)
    VAL_LAUNCH(128, 8);
  else
    VAL_LAUNCH(256, kPolNW);
#undef VAL_LAUNCH
#undef VAL_ARGS
  LAUNCH_CHECK();
  return 0;
}

int satrl_ppo_tanh(int64_t n, const float* x, float* y, void* stream) {
  if (n <= 0 || n > (int64_t)256 * 0x7FFFFFFF || !x || !y) return -1;
  hipLaunchKernelGGL(tanh_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, n, x, y);
  LAUNCH_CHECK();
  return 0;
}

// live launch spans (span_probe.h): the probe buffer, its bump pointer and
// the launch log, host state of the library (one probe per process)
int satrl_span_probe(void* buf, int64_t bytes, void* stream) {
  if ((buf == nullptr) != (bytes == 0) || bytes < 0) return -1;
  g_span.buf = static_cast<unsigned long long*>(buf);
  g_span.words = bytes / 8;
  if (!buf) return 0;                                              // stop: the log stays readable
  g_span.used = 0;
  g_span.log.clear();
  if (hipMemsetAsync(buf, 0, (size_t)bytes, (hipStream_t)stream) != hipSuccess) {
    g_span = SpanState{};
    g_err = "satrl_span_probe: hipMemsetAsync failed";
    return -2;
  }
  return 0;
}

int64_t satrl_span_probe_launches(void) { return (int64_t)g_span.log.size(); }

int satrl_span_probe_launch(int64_t i, int* kind, int64_t* word_offset, int64_t* waves) {
  if (i < 0 || i >= (int64_t)g_span.log.size() || !kind || !word_offset || !waves) return -1;
  *kind = g_span.log[(size_t)i].kind;
  *word_offset = g_span.log[(size_t)i].off;
  *waves = g_span.log[(size_t)i].waves;
  return 0;
}

const char* satrl_ppo_last_error(void) { return g_err.c_str(); }

}  // extern "C"


#ifdef SATRL_PHASE_PROBE
extern "C" int satrl_probe_read(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_probe), sizeof(g_probe)) == hipSuccess ? 0 : -1;
}
#endif
