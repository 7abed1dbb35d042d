// satenv_device.h -- FP64 device math of one environment step, one lane per env.
//
// MI355X-native restatement of the reference env hot path:
//   environment.py:81-255  satellites.step (Flag 0 / Flag 1)
//   satellite_function.py:753-781  Clohessy_Wiltshire.State_transition_matrix(100)
//   satellite_function.py:18-99,161-255,317-373,462-565  danger-zone count
//   scipy.optimize.fsolve -> MINPACK hybrd (n = 1, fsolve defaults)
//
// Numerics contract (see DESIGN.md "Parity"): every product/sum the
// reference evaluates through numpy/OpenBLAS is reproduced in the same
// order, incl. the FMA chain of OpenBLAS ddot and the dgemv_t summation
// tree; the file is compiled with -ffp-contract=off so nothing else fuses.
// Transcendentals are OCML (gfx950), which differs from the reference's
// numpy/glibc libm by <= 1-2 ulp; parity is therefore a tolerance on
// continuous outputs and exact on counts/done except libm-sensitive ties.
//
// One source, two targets: hipcc compiles it for gfx950 (the env kernels)
// and g++ compiles the same functions for the host (satenv_cpu.cpp, the
// satenv_cpu_* ABI: SURVEY.md §7 "one FP64 math core").  On the host the
// transcendentals are glibc's, so the host build computes what the
// reference computes with glibc libm; only the fsolve residual's sincos
// differs by target (OCML's transcription on the device, see resid()).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define SATENV_HD __host__ __device__ __forceinline__
#define SATENV_HD_NOINLINE __host__ __device__ __noinline__
#else
#include <cmath>
#include <cstring>
#define SATENV_HD static inline
#define SATENV_HD_NOINLINE static __attribute__((noinline))
static inline long long __double_as_longlong(double x) { long long v; std::memcpy(&v, &x, 8); return v; }
static inline double __longlong_as_double(long long v) { double x; std::memcpy(&x, &v, 8); return x; }
using std::acos; using std::atan; using std::cos; using std::fabs; using std::fma; using std::pow; using std::rint;
using std::sin; using std::sqrt; using std::trunc; using std::nextafter;
#endif

#include "satenv.h"

namespace satenv {

constexpr double kPi = 3.141592653589793;    // np.pi
constexpr double kTwoPi = 6.283185307179586; // 2 * np.pi
constexpr double kEpsMch = 2.220446049250313e-16;

// numpy scalar type of the reference's fuel attributes (environment.py:106-107)
enum : int { kPyInt = 0, kI64 = 1, kF32 = 2, kF64 = 3 };

// per-env int "bits" plane: [1:0] fuel_c mode, [3:2] fuel_t mode, [4] vel_int, [6:5] flag (0/1/2)
SATENV_HD int fc_mode(int b) { return b & 3; }
SATENV_HD int ft_mode(int b) { return (b >> 2) & 3; }
SATENV_HD int vel_int(int b) { return (b >> 4) & 1; }
SATENV_HD int env_flag(int b) { return (b >> 5) & 3; }
SATENV_HD int make_bits(int fc, int ft, int vi, int flag) {
  return (fc & 3) | ((ft & 3) << 2) | ((vi & 1) << 4) | ((flag & 3) << 5);
}

using Params = satenv_params;   // include/satenv.h

// python/numpy scalar `x ** 2` (the reference squares scalars with pow):
// glibc pow(x, 2.0) on the host -- which is not always x*x, it is off by an
// ulp on ~0.05 % of inputs -- and the correctly rounded x*x on gfx950
SATENV_HD double pow2(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return x * x;
#else
  return pow(x, 2.0);
#endif
}
SATENV_HD float pow2f(float x) {            // np.float32 ** 2
#if defined(__HIP_DEVICE_COMPILE__)
  return x * x;
#else
  return powf(x, 2.0f);
#endif
}

// OpenBLAS ddot, n = 3 (numpy np.dot / np.linalg.norm of 3-vectors)
SATENV_HD double dot3(double a0, double a1, double a2, double b0, double b1, double b2) {
  return fma(a2, b2, fma(a1, b1, a0 * b0));
}
SATENV_HD double norm3(double a0, double a1, double a2) {
  return sqrt(dot3(a0, a1, a2, a0, a1, a2));
}

// OCML's __ocml_acos_f64 (ROCm 7.2 ocml.bc) as straight-line code: the
// library branches to its |x| >= 1/2 arm (a sqrt of (1 - |x|)/2 refined in
// double-double and a reciprocal), which keeps a wave's four element acos()
// calls apart; here both arms are computed and selected, operation for
// operation as the bitcode has them, so results are bit-identical to acos()
// (tests/test_env_gpu.py through satenv_acos) while the compiler may
// interleave independent calls.  Device only: the host build is glibc's acos.
SATENV_HD double acos_sl(double x) {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(SATENV_ACOS_LIBRARY)   // (dev A/B: the library call)
  const double ax = fabs(x);
  const bool big = ax >= 0.5;
  const double y = fma(ax, -0.5, 0.5);
  const double u = big ? y : x * x;
  double p = fma(u, 0x1.059859fea6a70p-5, -0x1.0a5a378a05eafp-6);
  p = fma(u, p, 0x1.4052137024d6ap-6);
  p = fma(u, p, 0x1.ab3a098a70509p-8);
  p = fma(u, p, 0x1.8ed60a300c8d2p-7);
  p = fma(u, p, 0x1.c6fa84b77012bp-7);
  p = fma(u, p, 0x1.1c6c111dccb70p-6);
  p = fma(u, p, 0x1.6e89f0a0adacfp-6);
  p = fma(u, p, 0x1.f1c72c668963fp-6);
  p = fma(u, p, 0x1.6db6db41ce4bdp-5);
  p = fma(u, p, 0x1.333333336fd5bp-4);
  p = fma(u, p, 0x1.5555555555380p-3);
  const double r = u * p;
  const double small = fma(0x1.dd9ad336a0500p-1, 0x1.af154eeb562d6p+0, -fma(x, r, x));
  // |x| >= 1/2: s = sqrt(y) by rsq + two refinements, then the double-double remainder
  const double rs = __builtin_amdgcn_rsq(y);
  const double s0 = y * rs, h0 = rs * 0.5;
  const double e0 = fma(-h0, s0, 0.5);
  const double h1 = fma(h0, e0, h0), s1 = fma(s0, e0, s0);
  const double d1 = fma(-s1, s1, y);
  const double s = (y == 0.0) ? y : fma(d1, h1, s1);
  const double ss = s * s, sserr = fma(s, s, -ss);
  const double t1 = y - ss;
  const double rem = t1 + (((y - t1) - ss) - sserr);
  const double s2 = s * 2.0;
  const double q = __builtin_amdgcn_rcp(s2);
  const double q1 = fma(fma(-s2, q, 1.0), q, q);
  const double q2 = fma(fma(-s2, q1, 1.0), q1, q1);
  const double c0 = rem * q2;
  const double corr = (y == 0.0) ? 0.0 : fma(fma(-s2, c0, rem), q2, c0);
  const double hi = s + corr, lo = corr - (hi - s);
  const double neg = fma(0x1.dd9ad336a0500p+0, 0x1.af154eeb562d6p+0, fma(hi, r, hi) * -2.0);
  const double pos = (hi + fma(hi, r, lo)) * 2.0;
  double bigv = x < 0.0 ? neg : pos;
  bigv = x == -1.0 ? 0x1.921fb54442d18p+1 : bigv;
  bigv = x == 1.0 ? 0.0 : bigv;
  return big ? bigv : small;
#else
  return acos(x);
#endif
}

// ---------------------------------------------------------------------------
// satellite_function.py:161-255 calculate_orbital_elements (6-element branch)
// returns 0, or -4 (e == 0: circular branch) / -5 (parabolic branch): the
// reference leaves attributes unset there and crashes later.
// ---------------------------------------------------------------------------
struct Elements { double a, e, i, omega, Omega, f; };

SATENV_HD int orbital_elements(double mu, double R0, double R1, double R2, double V0,
                                                double V1, double V2, Elements& out) {
  const double r_norm = norm3(R0, R1, R2);
  const double v_norm = norm3(V0, V1, V2);
  const double r_dot_v = dot3(R0, R1, R2, V0, V1, V2);
  const double v2 = pow2(v_norm);                          // v_norm ** 2
  const double en = 2.0 / r_norm - v2 / mu;                // :186
  if (en == 0.0) return -5;
  out.a = 1.0 / fabs(en);                                  // :188
  const double c1 = v2 / mu - 1.0 / r_norm, c2 = r_dot_v / mu;
  const double E0 = c1 * R0 - c2 * V0, E1 = c1 * R1 - c2 * V1, E2 = c1 * R2 - c2 * V2;   // :193
  const double e = norm3(E0, E1, E2);
  if (e == 0.0) return -4;
  out.e = e;
  // H = R x V (numpy.cross order), N = Z x H = [-H1, H0, 0]
  const double H0 = R1 * V2 - R2 * V1, H1 = R2 * V0 - R0 * V2, H2 = R0 * V1 - R1 * V0;
  const double h = norm3(H0, H1, H2);
  const double N0 = 0.0 * H2 - 1.0 * H1, N1 = 1.0 * H0 - 0.0 * H2, N2 = 0.0 * H1 - 0.0 * H0;
  const double n = norm3(N0, N1, N2);
  out.i = acos_sl(dot3(0.0, 0.0, 1.0, H0, H1, H2) / h);       // :210
  double omega = (n != 0.0) ? acos_sl(dot3(N0, N1, N2, E0, E1, E2) / n / e) : 0.0;   // :214-217
  if (dot3(0.0, 0.0, 1.0, E0, E1, E2) < 0.0) omega = kTwoPi - omega;               // :221
  double Omega = (n != 0.0) ? acos_sl(dot3(1.0, 0.0, 0.0, N0, N1, N2) / n) : 0.0;      // :230-233
  if (dot3(0.0, 1.0, 0.0, N0, N1, N2) < 0.0) Omega = kTwoPi - Omega;                // :237
  double f = acos_sl(dot3(E0, E1, E2, R0, R1, R2) / e / r_norm);                       // :242
  if (r_dot_v < 0.0) f = kTwoPi - f;                                                // :243
  out.omega = omega;
  out.Omega = Omega;
  out.f = f;
  return 0;
}

// ---------------------------------------------------------------------------
// fsolve(P_fai_equation, guess): MINPACK hybrd specialised to n = 1 with
// scipy's fsolve defaults (xtol 1.49012e-8, maxfev 400, epsfcn = eps,
// factor 100, mode 1).  Residual (satellite_function.py:559-562):
//   g(a) = A * (dvm * cos a) + sin_t * (-dvm * sin a)
// with A = (2u(1-cos t))/(h v1y) - v1x sin t / v1y hoisted (bit-neutral).
// Bounded: every path increments nfev and stops at 400.
// ---------------------------------------------------------------------------
// OCML's __ocml_sincos_f64 for |x| < 2^30 as straight-line code: the
// trigredsmall Cody-Waite reduction by pi/2 and the sincosred2 polynomials,
// transcribed operation for operation from the device library's bitcode
// (ROCm 7.2 ocml.bc), so results are bit-identical to sincos() there.
// Straight-line (no per-call branch on the argument size), several calls
// interleave -- sincos() itself branches to the large-argument reduction,
// which serialises independent calls.  |x| >= 2^30 and inf/NaN go to
// sincos() (see sincos_fast).
SATENV_HD void sincos_small(double x, double& s_out, double& c_out) {
  const double ax = fabs(x);
  // __ocmlpriv_trigredsmall_f64
  const double q = rint(ax * 0x1.45f306dc9c883p-1);                 // 2/pi
  const double r4 = fma(q, -0x1.921fb54442d18p+0, ax);
  const double r5 = fma(q, -0x1.1a62633145c00p-54, r4);
  const double p6 = q * 0x1.1a62633145c00p-54;
  const double r8 = fma(q, 0x1.1a62633145c00p-54, -p6);
  const double r9 = r4 - p6;
  const double r10 = r4 - r9;
  const double r11 = r10 - p6;
  const double r12 = r9 - r5;
  const double r13 = r12 + r11;
  const double r14 = r13 - r8;
  const double r15 = fma(q, -0x1.b839a252049c0p-104, r14);
  const double hi = r5 + r15;
  const double r17 = hi - r5;
  const double lo = r15 - r17;
  const int quad = ((int)q) & 3;
  // __ocmlpriv_sincosred2_f64(hi, lo)
  const double x2 = hi * hi;
  const double h4 = x2 * 0.5;
  const double c5 = 1.0 - h4;
  const double c6 = 1.0 - c5;
  const double c7 = c6 - h4;
  const double x4 = x2 * x2;
  double pc = fma(x2, -0x1.907db46cc5e42p-37, 0x1.1eeb69037ab78p-29);
  pc = fma(x2, pc, -0x1.27e4fa17f65f6p-22);
  pc = fma(x2, pc, 0x1.a01a019f4ec90p-16);
  pc = fma(x2, pc, -0x1.6c16c16c16967p-10);
  pc = fma(x2, pc, 0x1.5555555555555p-5);
  const double c15 = fma(hi, -lo, c7);
  const double c16 = fma(x4, pc, c15);
  const double cr = c5 + c16;
  double ps = fma(x2, 0x1.5e0b2f9a43bb8p-33, -0x1.ae600b42fdfa7p-26);
  ps = fma(x2, ps, 0x1.71de3796cde01p-19);
  ps = fma(x2, ps, -0x1.a01a019e83e5cp-13);
  ps = fma(x2, ps, 0x1.1111111110bb3p-7);
  const double m23 = hi * (-x2);
  const double s25 = fma(m23, ps, lo * 0.5);
  const double s26 = fma(x2, s25, -lo);
  const double s27 = fma(m23, -0x1.5555555555555p-3, s26);
  const double sr = hi - s27;
  // quadrant and sign (__ocml_sincos_f64)
  const unsigned flip = quad > 1 ? 0x80000000u : 0u;
  const bool even = (quad & 1) == 0;
  const double sv = even ? sr : cr;
  const double cv = even ? cr : -sr;
  const unsigned xs = (unsigned)(__double_as_longlong(x) >> 32) & 0x80000000u;
  const long long sb = __double_as_longlong(sv), cb = __double_as_longlong(cv);
  s_out = __longlong_as_double(sb ^ ((long long)(xs ^ flip) << 32));
  c_out = __longlong_as_double(cb ^ ((long long)flip << 32));
}

// sincos() with the straight-line body for |x| < 2^30 (every argument of
// the env step in practice); the rare rest takes the library call
SATENV_HD void sincos_fast(double x, double& s, double& c) {
  sincos_small(x, s, c);
  if (!(fabs(x) < 0x1.0p+30)) sincos(x, &s, &c);
}

SATENV_HD double resid(double A, double st, double dvm, double a) {
  double s, c;
#if defined(__HIP_DEVICE_COMPILE__) && !defined(SATENV_RESID_LIBSINCOS)
  sincos_fast(a, s, c);          // gfx950: OCML's sincos, straight-line
#else
  sincos(a, &s, &c);             // host (glibc) / library check build
#endif
  return A * (dvm * c) + st * (-dvm * s);
}

SATENV_HD_NOINLINE double hybrd1(double A, double st, double dvm, double x) {
  const double xtol = 1.49012e-08, factor = 100.0;
  const double eps = 1.4901161193847656e-08;               // sqrt(max(epsfcn, epsmch))
  double fvec = resid(A, st, dvm, x);
  int nfev = 1;
  double fnorm = fabs(fvec);
  int iter = 1, ncsuc = 0, ncfail = 0, nslow1 = 0, nslow2 = 0;
  double diag = 0.0, delta = 0.0, xnorm = 0.0;
  for (;;) {
    // fdjac1 (forward difference), qrfac, qform for a 1x1 Jacobian
    double hs = eps * fabs(x);
    if (hs == 0.0) hs = eps;
    const double J = (resid(A, st, dvm, x + hs) - fvec) / hs;
    nfev += 1;
    const double acnorm = fabs(J);
    double ajnorm = acnorm, a = J;
    if (ajnorm != 0.0) {
      if (a < 0.0) ajnorm = -ajnorm;
      a = a / ajnorm + 1.0;
    }
    if (iter == 1) {
      diag = (acnorm == 0.0) ? 1.0 : acnorm;
      xnorm = fabs(diag * x);
      delta = factor * xnorm;
      if (delta == 0.0) delta = factor;
    }
    double qtf = fvec, fjac = 1.0;
    if (a != 0.0) {
      const double t = -(0.0 + a * qtf) / a;
      qtf = qtf + a * t;
      fjac = 1.0 - ((0.0 + 1.0 * a) / a) * a;
    }
    double r = -ajnorm;
    diag = (diag > acnorm || acnorm != acnorm) ? diag : acnorm;
    bool jeval = true;
    for (;;) {
      // dogleg
      double tr = r;
      if (tr == 0.0) tr = kEpsMch;                         // epsmch*max|r| == 0 -> epsmch
      const double gn = (qtf - 0.0) / tr;
      const double qnorm = fabs(diag * gn);
      double p;
      if (qnorm <= delta) {
        p = gn;
      } else {
        double w1 = (0.0 + r * qtf) / diag;
        const double gnorm = fabs(w1);
        double sg = 0.0, al = delta / qnorm;
        if (gnorm != 0.0) {
          w1 = (w1 / gnorm) / diag;
          const double tn = fabs(0.0 + r * w1);
          sg = (gnorm / tn) / tn;
          al = 0.0;
          if (sg < delta) {
            const double bn = fabs(qtf), dq = delta / qnorm, sd = sg / delta;
            double t1 = (bn / gnorm) * (bn / qnorm) * sd;
            t1 = t1 - dq * (sd * sd) + sqrt((t1 - dq) * (t1 - dq) + (1.0 - dq * dq) * (1.0 - sd * sd));
            al = (dq * (1.0 - sd * sd)) / t1;
          }
        }
        p = ((1.0 - al) * (sg < delta ? sg : delta)) * w1 + al * gn;
      }
      const double w1 = -p;
      const double w2 = x + w1;
      const double pnorm = fabs(diag * w1);
      if (iter == 1) delta = (delta < pnorm) ? delta : pnorm;
      const double wa4 = resid(A, st, dvm, w2);
      nfev += 1;
      const double fnorm1 = fabs(wa4);
      double actred = -1.0;
      if (fnorm1 < fnorm) actred = 1.0 - (fnorm1 / fnorm) * (fnorm1 / fnorm);
      const double w3 = qtf + (0.0 + r * w1);
      const double tq = fabs(w3);
      double prered = 0.0;
      if (tq < fnorm) prered = 1.0 - (tq / fnorm) * (tq / fnorm);
      const double ratio = (prered > 0.0) ? actred / prered : 0.0;
      if (ratio < 0.1) {
        ncsuc = 0; ncfail += 1; delta = 0.5 * delta;
      } else {
        ncfail = 0; ncsuc += 1;
        if (ratio >= 0.5 || ncsuc > 1) {
          const double t = pnorm / 0.5;
          delta = (delta > t || t != t) ? delta : t;
        }
        if (fabs(ratio - 1.0) <= 0.1) delta = pnorm / 0.5;
      }
      if (ratio >= 1e-4) {
        x = w2;
        xnorm = fabs(diag * x);
        fvec = wa4;
        fnorm = fnorm1;
        iter += 1;
      }
      nslow1 += 1;
      if (actred >= 0.001) nslow1 = 0;
      if (jeval) nslow2 += 1;
      if (ratio >= 0.1) nslow2 = 0;
      if (delta <= xtol * xnorm || fnorm == 0.0) return x;
      const double m1 = 0.1 * delta;
      const double mx = (m1 > pnorm || pnorm != pnorm) ? m1 : pnorm;
      if (nfev >= 400 || 0.1 * mx <= kEpsMch * xnorm || nslow2 == 5 || nslow1 == 10) return x;
      if (ncfail == 2) break;                              // refresh the Jacobian
      const double sum = 0.0 + fjac * wa4;                 // Broyden rank-1 (r1updt, n = 1)
      const double v = (sum - w3) / pnorm;
      const double u = diag * ((diag * w1) / pnorm);
      if (ratio >= 1e-4) qtf = sum;
      r = r + v * u;
      jeval = false;
    }
  }
}

// ---------------------------------------------------------------------------
// satellite_function.py:462-556 rf_extreme_point('orbit_c1'/'orbit_c2'), fai = 0
// ---------------------------------------------------------------------------
struct Pursuer { double u, dv2, e, f0, p, r, sf0, X, sq; };

// the two fsolve problems of one rf_extreme_point call (guesses +pi/2 and
// -pi/2, :516 / :534), set up before any solve so that the danger-zone
// count can advance all four of an env's solves in one hybrdN<4>
struct RfSolve { bool ok; double vx0, vy0, dvm, st, ct; double A[2], ag[2]; };

constexpr double kSinHalfPi = 1.0;                        // sin(np.pi / 2), = -sin(-np.pi / 2)
constexpr double kCosHalfPi = 0x1.1a62633145c07p-54;      // cos(+-np.pi / 2) = 6.123233995736766e-17

SATENV_HD void rf_setup(const Pursuer& P, double f_c, RfSolve& q) {
  const double d = f_c - P.f0;
  const double sd = sin(d);
  const double temp1 = pow2(sd) / (P.u * pow2(P.X) / (P.p * P.dv2) - 1.0);      // :466
  q.ok = (0.0 <= temp1);                                                         // else (0, 0), :477
  q.vx0 = q.vy0 = q.dvm = q.st = q.ct = 0.0;
  q.A[0] = q.A[1] = 0.0;
  q.ag[0] = kPi / 2;
  q.ag[1] = -kPi / 2;
  if (!q.ok) return;
  // beta = atan(0 / sd) (tan(fai) = 0, :469): for a finite non-zero sd the
  // quotient is a signed zero, and atan / sin / cos of +-0 are exact (+-0,
  // +-0, 1) in every IEEE libm, so the three calls drop off the chain
  const double q0 = 0.0 / sd;
  double sb, cb;
  if (q0 == 0.0) { sb = q0; cb = 1.0; }
  else { const double beta = atan(q0); sb = sin(beta); cb = cos(beta); }
  q.dvm = sqrt(P.dv2 - P.u * pow2(P.X) * pow2(sb) / P.p);                        // :470
  double theta = 0.0;
  if ((-kTwoPi <= d && d < -kPi) || (0.0 <= d && d < kPi)) theta = acos_sl(cos(d) * 1.0);          // :473
  else if ((-kPi <= d && d < 0.0) || (kPi <= d && d < kTwoPi)) theta = kTwoPi - acos_sl(cos(d) * 1.0);
  sincos(theta, &q.st, &q.ct);
  q.vx0 = P.sq * P.e * P.sf0;                                                    // :518
  q.vy0 = P.sq * P.X * cb;                                                       // :519
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    // sincos(+-pi/2): the values OCML and glibc both return (the guesses are
    // constants; test_env_gpu / test_oracle_golden check the identity)
    const double sg = k == 0 ? kSinHalfPi : -kSinHalfPi, cg = kCosHalfPi;
    const double v1x = q.vx0 + q.dvm * cg, v1y = q.vy0 + q.dvm * sg;
    const double h = P.r * v1y;
    q.A[k] = (2.0 * P.u * (1.0 - q.ct)) / (h * v1y) - v1x * q.st / v1y;          // :560
  }
}

// rf of one solution alpha (:525-530 / :543-548), before abs and sort
SATENV_HD double rf_one(const Pursuer& P, const RfSolve& q, double al) {
  double sa, ca;
  sincos(al, &sa, &ca);
  const double vx = q.vx0 + q.dvm * ca, vy = q.vy0 + q.dvm * sa;                 // :525-528
  const double hm = P.r * vy;
  return pow2(hm) / (P.u * (1.0 - q.ct) + hm * vy * q.ct - hm * vx * q.st);     // :530
}

// abs and sort of the two rf values (:549-554); (0, 0) when temp1 < 0 (:477)
SATENV_HD void rf_sort(bool ok, double rf0, double rf1, double& rmax, double& rmin) {
  if (!ok) { rmax = 0.0; rmin = 0.0; return; }
  rmax = fabs(rf0);
  rmin = fabs(rf1);
  if (rmax < rmin) { const double t = rmin; rmin = rmax; rmax = t; }
}

// rf from the two solutions, abs and sort (:525-530, :549-556)
SATENV_HD void rf_finish(const Pursuer& P, const RfSolve& q, double al0, double al1, double& rmax,
                                          double& rmin) {
  if (!q.ok) { rmax = 0.0; rmin = 0.0; return; }
  rf_sort(true, rf_one(P, q, al0), rf_one(P, q, al1), rmax, rmin);
}

// self.Delta_V_c ** 2 by numpy scalar type
SATENV_HD double fuel_sq(double fuel, int mode) {
  if (mode == kF32) return (double)pow2f((float)fuel);
  const double exact = fuel * fuel;                        // python int ** 2: exact
  return (mode == kF64) ? pow2(fuel) : exact;              // (one expression on gfx950)
}

// environment.py:317-332 + satellite_function.py:18-99,317-373, cut at its
// fsolve calls: dz_setup computes both element sets, the latitudinal angles,
// the two rf_extreme_point set-ups (up to four fsolve problems, z.q[c].A[k]
// with guess z.q[c].ag[k], live when z.q[c].ok) and the target radii;
// dz_finish takes the four solutions and returns the count.  Returns 0 or
// <0 (a non-6-element orbit branch).  The pieces (dz_elements, dz_pursuer,
// dz_lat, rf_setup, dz_target_radii, rf_one / rf_sort) are what the
// multi-wave env kernel spreads over waves; composed in this order they are
// dz_setup / dz_finish, operation for operation.
struct DzCtx { Pursuer P; RfSolve q[2]; double r_ft1, r_ft2; };

constexpr double kDzMu = 3.986e14;                           // Time_window_of_danger_zone default u

// the chaser's (which = 0) or the target's (1) element set from the relative state
SATENV_HD int dz_elements(const Params& prm, double X0, double X1, double X2, double V0, double V1, double V2,
                          Elements& out) {
  return orbital_elements(kDzMu, prm.R_cw[0] + X0, prm.R_cw[1] + X1, prm.R_cw[2] + X2, prm.V_cw[0] + V0,
                          prm.V_cw[1] + V1, prm.V_cw[2] + V2, out);
}

// Time_window_of_danger_zone attributes of the chaser (:54-58, :82-86)
SATENV_HD void dz_pursuer(const Elements& C, double fuel, int fmode, Pursuer& P) {
  P.u = kDzMu;
  P.dv2 = fuel_sq(fuel, fmode);
  P.e = C.e;
  P.f0 = C.f;
  double sf0, cf0;
  sincos(C.f, &sf0, &cf0);
  P.sf0 = sf0;
  P.X = 1.0 + C.e * cf0;
  P.p = C.a * (1.0 - pow2(C.e));                                                 // :58
  P.r = P.p / P.X;                                                               // :57 (a(1-e^2)/(1+e cos f0))
  P.sq = sqrt(kDzMu / P.p);
}

// :317-339 latitudinal angles u_c1, u_c2 = u_c1 + pi, u_t1, u_t2 = u_t1 + pi
SATENV_HD void dz_lat(const Elements& C, const Elements& T, double& u_c1, double& u_c2, double& u_t1,
                      double& u_t2) {
  double s_it, c_it, s_ic, c_ic, s_d, c_d;
  sincos(T.i, &s_it, &c_it);
  sincos(C.i, &s_ic, &c_ic);
  sincos(C.Omega - T.Omega, &s_d, &c_d);
  const double s_dn = sin(T.Omega - C.Omega), c_dn = cos(T.Omega - C.Omega);
  double temp1 = (s_it * s_d) / (c_it * s_ic - s_it * c_ic * c_d);
  double temp2 = (s_ic * s_dn) / (c_ic * s_it - s_ic * c_it * c_dn);
  if (temp1 != temp1 || temp2 != temp2) { temp1 = 1.0; temp2 = 1.0; }         // :331-332
  u_c1 = atan(temp1);
  u_c2 = kPi + u_c1;
  u_t1 = atan(temp2);
  u_t2 = u_t1 + kPi;
}

// :363-365 target radii, cross-wired as in the reference (r_ft1 from f_t2)
SATENV_HD void dz_target_radii(const Elements& T, double u_t1, double u_t2, double& r_ft1, double& r_ft2) {
  const double pt = T.a * (1.0 - pow2(T.e));
  r_ft1 = pt / (1.0 + T.e * cos(u_t2 - T.omega));                               // :363 (cross-wired f_t2)
  r_ft2 = pt / (1.0 + T.e * cos(u_t1 - T.omega));                               // :365
}

// the count from the two (rmax, rmin) pairs and the target radii (:367-372)
SATENV_HD int dz_count(double mx1, double mn1, double mx2, double mn2, double r_ft1, double r_ft2) {
  const bool in1 = (mn1 <= r_ft1 && r_ft1 <= mx1), in2 = (mn2 <= r_ft2 && r_ft2 <= mx2);
  return (in1 && in2) ? 2 : ((in1 || in2) ? 1 : 0);
}

SATENV_HD int dz_setup(const Params& prm, double Pp0, double Pp1, double Pp2, double Pv0,
                                        double Pv1, double Pv2, double Ep0, double Ep1, double Ep2, double Ev0,
                                        double Ev1, double Ev2, double fuel, int fmode, DzCtx& z) {
  Elements C, T;
  int rc = dz_elements(prm, Pp0, Pp1, Pp2, Pv0, Pv1, Pv2, C);
  if (rc) return rc;
  rc = dz_elements(prm, Ep0, Ep1, Ep2, Ev0, Ev1, Ev2, T);
  if (rc) return rc;
  dz_pursuer(C, fuel, fmode, z.P);
  double u_c1, u_c2, u_t1, u_t2;
  dz_lat(C, T, u_c1, u_c2, u_t1, u_t2);
  rf_setup(z.P, u_c1 - C.omega, z.q[0]);                                         // rf_extreme_point('orbit_c1')
  rf_setup(z.P, u_c2 - C.omega, z.q[1]);                                         // ('orbit_c2')
  dz_target_radii(T, u_t1, u_t2, z.r_ft1, z.r_ft2);
  return 0;
}

// al[2c + k] = the fsolve solution of problem (c, k)
SATENV_HD int dz_finish(const DzCtx& z, const double (&al)[4]) {
  double mx1, mn1, mx2, mn2;
  rf_finish(z.P, z.q[0], al[0], al[1], mx1, mn1);
  rf_finish(z.P, z.q[1], al[2], al[3], mx2, mn2);
  return dz_count(mx1, mn1, mx2, mn2, z.r_ft1, z.r_ft2);
}

// the whole count in one lane (the four solves one after another)
SATENV_HD int danger_zone(const Params& prm, double Pp0, double Pp1, double Pp2, double Pv0,
                                           double Pv1, double Pv2, double Ep0, double Ep1, double Ep2, double Ev0,
                                           double Ev1, double Ev2, double fuel, int fmode, int& count) {
  DzCtx z;
  const int rc = dz_setup(prm, Pp0, Pp1, Pp2, Pv0, Pv1, Pv2, Ep0, Ep1, Ep2, Ev0, Ev1, Ev2, fuel, fmode, z);
  if (rc) return rc;
  double al[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const RfSolve& q = z.q[k >> 1];
    al[k] = q.ok ? hybrd1(q.A[k & 1], q.st, q.dvm, q.ag[k & 1]) : q.ag[k & 1];
  }
  count = dz_finish(z, al);
  return 0;
}

// np.clip(a, -1.6, 1.6) on np.float32
SATENV_HD float clip16(float a) {
  return a < -1.6f ? -1.6f : (a > 1.6f ? 1.6f : a);
}

// fuel -= |a0|+|a1|+|a2| under numpy scalar promotion (environment.py:106-107)
SATENV_HD void fuel_sub(double& fuel, int& mode, bool zero_int_action, float s) {
  if (zero_int_action) {
    mode = (mode == kPyInt) ? kI64 : ((mode == kF32) ? kF64 : mode);
    return;
  }
  if (mode == kPyInt || mode == kF32) { fuel = (double)((float)fuel - s); mode = kF32; }
  else { fuel = fuel - (double)s; mode = kF64; }
}

SATENV_HD double cos_sim(double a0, double a1, double a2, double b0, double b1, double b2) {
  const double na = norm3(a0, a1, a2), nb = norm3(b0, b1, b2);
  return dot3(a0 / na, a1 / na, a2 / na, b0 / nb, b1 / nb, b2 / nb);
}

// float32 np.linalg.norm (OpenBLAS sdot: f32 products summed in double)
SATENV_HD float norm3f(float a0, float a1, float a2) {
  double s = (double)(a0 * a0);
  s += (double)(a1 * a1);
  s += (double)(a2 * a2);
  return sqrtf((float)s);
}

// ---------------------------------------------------------------------------
// RK4 propagators.  rk4_step is the RungeKutta combination of
// 轨道外推-龙格库塔算法.py:35-41 (K2 = f(r0 + h/2 K1), K3 = f(r0 + h/2 K2),
// K4 = f(r0 + h K3), r1 = r0 + h/6 ((K1 + 2K2) + 2K3) + K4), elementwise in
// that order.  The stage weights (h/2, h, h/6 and the 2s) are uniform over a
// launch, so they sit in scalar registers for the whole kernel -- on-chip,
// read at no cost by every lane.  A Butcher table in LDS would hold the same
// doubles (the same rounding) but add an LDS load and its wait per use.
// ---------------------------------------------------------------------------
template <class F>
SATENV_HD void rk4_step(F f, const double (&r0)[6], double h, double (&out)[6]) {
  double k1[6], k2[6], k3[6], k4[6], t[6];
  const double h2 = h / 2.0, h6 = h / 6.0;
  f(r0, k1);
#pragma unroll
  for (int i = 0; i < 6; ++i) t[i] = r0[i] + h2 * k1[i];
  f(t, k2);
#pragma unroll
  for (int i = 0; i < 6; ++i) t[i] = r0[i] + h2 * k2[i];
  f(t, k3);
#pragma unroll
  for (int i = 0; i < 6; ++i) t[i] = r0[i] + h * k3[i];
  f(t, k4);
#pragma unroll
  for (int i = 0; i < 6; ++i) out[i] = r0[i] + h6 * (((k1[i] + 2.0 * k2[i]) + 2.0 * k3[i]) + k4[i]);
}

// StateEq (:15-31), km units; `**` on numpy scalars is pow()
SATENV_HD void j2_rhs(const double (&rv)[6], double (&f)[6]) {
  constexpr double kMu = 398600.0, kRe = 6378.137, kJ2 = 0.00108263;
  const double x = rv[0], y = rv[1], z = rv[2];
  const double r = sqrt((pow(x, 2.0) + pow(y, 2.0)) + pow(z, 2.0));
  const double r3 = pow(r, 3.0), r5 = pow(r, 5.0), zr2 = pow(z / r, 2.0);
  const double c = ((-3.0 / 2.0 * kJ2) * pow(kRe, 2.0)) * kMu;     // -3 / 2 * J2 * Re ** 2 * mu
  f[0] = rv[3]; f[1] = rv[4]; f[2] = rv[5];
  f[3] = (-kMu * x) / r3 + ((c * x) / r5) * (1.0 - 5.0 * zr2);
  f[4] = (-kMu * y) / r3 + ((c * y) / r5) * (1.0 - 5.0 * zr2);
  f[5] = (-kMu * z) / r3 + ((c * z) / r5) * (3.0 - 5.0 * zr2);
}

// RK4 on the CW ODE (propagator 1), t seconds in nsub steps
SATENV_HD void cw_rk4(double (&s)[6], double w, double t, int nsub) {
  const double w2 = w * w, h = t / (double)nsub;
  auto f = [w, w2](const double (&x)[6], double (&o)[6]) {
    o[0] = x[3]; o[1] = x[4]; o[2] = x[5];
    o[3] = (2.0 * w) * x[4] + (3.0 * w2) * x[0];
    o[4] = (-2.0 * w) * x[3];
    o[5] = -w2 * x[2];
  };
  for (int i = 0; i < nsub; ++i) {
    double o[6];
    rk4_step(f, s, h, o);
#pragma unroll
    for (int k = 0; k < 6; ++k) s[k] = o[k];
  }
}

// ---------------------------------------------------------------------------
// Propagator 2: satellite_function.py:783-839 Numerical_calculation_method.
// numerical_calculation(t) integrates orbit_ode (:796-821: the CW equations
// with omega from r = 35786 km, J2 = 0, Tmax = 0) by scipy's solve_ivp RK45
// (rtol 1e-3, atol 1e-6, t_eval = arange(0, t + 50, 50)) and keeps the
// dense output at t.  scipy 1.15.3's select_initial_step, _step_impl,
// rk_step, the RK45 tableau and RkDenseOutput, restated with the
// numpy/OpenBLAS summation orders the reference executes (the oracle's
// orc_cw_rk45 documents the probes; it matches the captured solve_ivp
// outputs bit for bit).  The constants are the reference's python values
// of 2*omega, 3*omega**2, omega**2.  Returns 0, or -6 when scipy would
// stop with TOO_SMALL_STEP.
// ---------------------------------------------------------------------------
constexpr double kCw45W2x = 0x1.8729f82d726ffp-13;   // 2 * omega
constexpr double kCw45W3 = 0x1.c044ec3d320a8p-26;    // 3 * omega ** 2
constexpr double kCw45Wsq = 0x1.2ad89d7e215c5p-27;   // omega ** 2

SATENV_HD void cw45_rhs(const double (&X)[6], double (&f)[6]) {   // orbit_ode :816-820 (+ a_T + pJ2 = +0)
  f[0] = X[3]; f[1] = X[4]; f[2] = X[5];
  f[3] = ((kCw45W2x * X[4]) + (kCw45W3 * X[0])) + 0.0;
  f[4] = ((-kCw45W2x) * X[3]) + 0.0;
  f[5] = ((-kCw45Wsq) * X[2]) + 0.0;
}
SATENV_HD double rms6(const double (&v)[6]) {                      // common.norm (ddot fma chain)
  double t = v[0] * v[0];
#pragma unroll
  for (int j = 1; j < 6; ++j) t = fma(v[j], v[j], t);
  return sqrt(t) / 2.449489742783178;
}
// np.dot(K[:s].T, a[:s])[i] (OpenBLAS dgemv_n, 6 rows: blocks of 4/2/1
// columns for rows 0-3, a fma chain for the tail rows 4-5)
SATENV_HD double rk_gemv(const double (&K)[7][6], const double* a, int s, int i) {
  if (i >= 4) {
    double t = K[0][i] * a[0];
#pragma unroll
    for (int j = 1; j < 7; ++j)
      if (j < s) t = fma(K[j][i], a[j], t);
    return t;
  }
  if (s == 1) return K[0][i] * a[0];
  double t = fma(K[0][i], a[0], K[1][i] * a[1]);
  if (s == 2) return t;
  if (s == 3) return t + K[2][i] * a[2];
  t = fma(K[3][i], a[3], fma(K[2][i], a[2], t));
  int j = 4;
  if (s - j >= 2) { t = t + fma(K[j][i], a[j], K[j + 1][i] * a[j + 1]); j += 2; }
  if (s - j >= 1) t = t + K[j][i] * a[j];
  return t;
}

SATENV_HD int cw_rk45(double (&y)[6], double tb) {
  // RK45 tableau (rk.py:380-404), python int/int divisions = correctly rounded doubles
  constexpr double A[6][5] = {{0, 0, 0, 0, 0},
                              {1.0 / 5, 0, 0, 0, 0},
                              {3.0 / 40, 9.0 / 40, 0, 0, 0},
                              {44.0 / 45, -56.0 / 15, 32.0 / 9, 0, 0},
                              {19372.0 / 6561, -25360.0 / 2187, 64448.0 / 6561, -212.0 / 729, 0},
                              {9017.0 / 3168, -355.0 / 33, 46732.0 / 5247, 49.0 / 176, -5103.0 / 18656}};
  constexpr double B[6] = {35.0 / 384, 0, 500.0 / 1113, 125.0 / 192, -2187.0 / 6784, 11.0 / 84};
  constexpr double E[7] = {-71.0 / 57600, 0, 71.0 / 16695, -71.0 / 1920, 17253.0 / 339200, -22.0 / 525, 1.0 / 40};
  constexpr double P[7][4] = {
      {1, -8048581381.0 / 2820520608, 8663915743.0 / 2820520608, -12715105075.0 / 11282082432},
      {0, 0, 0, 0},
      {0, 131558114200.0 / 32700410799, -68118460800.0 / 10900136933, 87487479700.0 / 32700410799},
      {0, -1754552775.0 / 470086768, 14199869525.0 / 1410260304, -10690763975.0 / 1880347072},
      {0, 127303824393.0 / 49829197408, -318862633887.0 / 49829197408, 701980252875.0 / 199316789632},
      {0, -282668133.0 / 205662961, 2019193451.0 / 616988883, -1453857185.0 / 822651844},
      {0, 40617522.0 / 29380423, -110615467.0 / 29380423, 69997945.0 / 29380423}};
  constexpr double rtol = 1e-3, atol = 1e-6;
  double f[6], K[7][6], sc[6], v[6];
  cw45_rhs(y, f);
  double h_abs;
  {  // select_initial_step (common.py:109-133): t0 = 0, direction 1, order 4
    const double L = fabs(tb - 0.0);
    for (int i = 0; i < 6; ++i) sc[i] = atol + fabs(y[i]) * rtol;
    for (int i = 0; i < 6; ++i) v[i] = y[i] / sc[i];
    const double d0 = rms6(v);
    for (int i = 0; i < 6; ++i) v[i] = f[i] / sc[i];
    const double d1 = rms6(v);
    double h0 = (d0 < 1e-5 || d1 < 1e-5) ? 1e-6 : (0.01 * d0) / d1;
    if (L < h0) h0 = L;
    double y1[6], f1[6];
    for (int i = 0; i < 6; ++i) y1[i] = y[i] + (h0 * 1.0) * f[i];
    cw45_rhs(y1, f1);
    for (int i = 0; i < 6; ++i) v[i] = (f1[i] - f[i]) / sc[i];
    const double d2 = rms6(v) / h0;
    double h1;
    if (d1 <= 1e-15 && d2 <= 1e-15) h1 = (1e-6 < h0 * 1e-3) ? h0 * 1e-3 : 1e-6;
    else h1 = pow(0.01 / ((d2 > d1) ? d2 : d1), 1.0 / 5);
    h_abs = 100 * h0;                                               // min(100*h0, h1, L, max_step)
    if (h1 < h_abs) h_abs = h1;
    if (L < h_abs) h_abs = L;
  }
  double t = 0.0, t_old = 0.0, y_old[6];
  while (!(t - tb >= 0)) {                                          // OdeSolver.step until 'finished'
    const double min_step = 10 * fabs(nextafter(t, (double)INFINITY) - t);
    double hc = h_abs < min_step ? min_step : h_abs;
    bool accepted = false, rejected = false;
    double h = 0.0, t_new = t, yn[6];
    while (!accepted) {                                             // _step_impl (rk.py:111-164)
      if (hc < min_step) return -6;
      t_new = t + hc * 1.0;
      if (1.0 * (t_new - tb) > 0) t_new = tb;
      h = t_new - t;
      hc = fabs(h);
      for (int i = 0; i < 6; ++i) K[0][i] = f[i];                   // rk_step (rk.py:62-73)
#pragma unroll
      for (int s = 1; s < 6; ++s) {
        double ys[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) ys[i] = y[i] + rk_gemv(K, A[s], s, i) * h;
        cw45_rhs(ys, K[s]);
      }
      for (int i = 0; i < 6; ++i) yn[i] = y[i] + h * rk_gemv(K, B, 6, i);
      cw45_rhs(yn, K[6]);
      for (int i = 0; i < 6; ++i) {
        const double ay = fabs(y[i]), an = fabs(yn[i]);
        sc[i] = atol + (ay > an ? ay : an) * rtol;
      }
      for (int i = 0; i < 6; ++i) v[i] = (rk_gemv(K, E, 7, i) * h) / sc[i];
      const double en = rms6(v);
      if (en < 1) {
        double factor = 10;                                         // MAX_FACTOR
        if (en != 0) { factor = 0.9 * pow(en, -0.2); if (!(factor < 10)) factor = 10; }
        if (rejected && !(factor < 1)) factor = 1;
        hc *= factor;
        accepted = true;
      } else {
        double fac = 0.9 * pow(en, -0.2);
        if (!(fac > 0.2)) fac = 0.2;                                // max(MIN_FACTOR, .)
        hc *= fac;
        rejected = true;
      }
    }
    t_old = t;
    for (int i = 0; i < 6; ++i) { y_old[i] = y[i]; y[i] = yn[i]; f[i] = K[6][i]; }
    t = t_new;
    h_abs = hc;
  }
  // RkDenseOutput at t_eval[-1] = t (x = 1): Q = K.T.dot(P) (dgemm: fma
  // chains), y = h * np.dot(Q, p) + y_old, where np.dot is dgemv_t when the
  // last step holds one t_eval point and dgemm when it holds more
  const double hd = t - t_old;
  int m = 0;
  for (double te = 0.0; te <= tb; te += 50.0) m += (te > t_old || t_old == 0.0) ? 1 : 0;
  for (int i = 0; i < 6; ++i) {
    double q[4];
    for (int c = 0; c < 4; ++c) {
      double a = K[0][i] * P[0][c];
      for (int j = 1; j < 7; ++j) a = fma(K[j][i], P[j][c], a);
      q[c] = a;
    }
    const double sum = (m == 1) ? (q[0] + q[2]) + (q[1] + q[3]) : ((q[0] + q[1]) + q[2]) + q[3];
    y[i] = hd * sum + y_old[i];
  }
  return 0;
}

}  // namespace satenv
