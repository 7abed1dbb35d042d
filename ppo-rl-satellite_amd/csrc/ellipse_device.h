// ellipse_device.h -- gfx950 restatement of single_pluse_model/curve_fitting.py
// Curve_fitting (:475-576): the ellipse fitted to each reachable-domain
// envelope, one workgroup per (orbit, envelope), consuming the dense
// direction grid of rd_kernel directly (no host round trip).
//
//   A  gather the reachable xy points (:534-543, NaN rows dropped) into LDS
//   B  bitonic sort (lexicographic, = np.unique(axis=0) order) + duplicate marks
//   C  EllipticEnvelope(support_fraction=1).location_ (:545-547): sample mean /
//      covariance, Mahalanobis distances, median by 8-bit radix select,
//      reweighted mean of the points with corrected distance < chi2(2).isf(.025)
//   D  angular bins around the center (np.digitize on linspace(-pi, pi, 100)),
//      farthest / nearest point per bin, bins in order of first appearance
//   E  scipy least_squares(ellipse_residuals) (:486-492): trf, 2-point Jacobian,
//      exact trust-region solve, ftol = xtol = gtol = 1e-8, max_nfev 500;
//      one wave, rows of J spread over lanes, SVD as Householder QR of [J | f]
//      (wave reductions) + one-sided Jacobi on the 5x5 R (every lane, uniform)
//
// Transcendentals are OCML and the reductions run in a different order than
// numpy/OpenBLAS/LAPACK, so parity with the reference is a tolerance
// (tests/test_rd_gpu.py), like scipy's own cross-platform reproducibility.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ellipse {

constexpr int kThreads = 256;
constexpr int kCap = 8192;                      // unique points per envelope held in LDS (128 KB)
constexpr int kBins = 101;                      // np.digitize indices 0..100
constexpr int kMaxFit = 128;                    // <= 100 filtered points, 2 rows per lane
constexpr double kIsf050 = 1.386294361119891;   // scipy.stats.chi2(2).isf(0.5)
constexpr double kIsf0025 = 7.3777589082278725; // scipy.stats.chi2(2).isf(0.025)
constexpr double kPi = 3.141592653589793;
constexpr double kEps = 2.220446049250313e-16;
constexpr int kMaxNfev = 500;                   // x0.size * 100

// info codes (> 0: least-squares function evaluations)
constexpr int kErrStaleTheta = -1, kErrTooMany = -2, kErrTooFew = -3;

struct Smem {
  double2 pts[kCap];
  double2 fit[kMaxFit];
  unsigned long long best[kBins];
  int first[kBins], pick[kBins];
  int hist[256];
  double red[kThreads / 64][4];
  int cnt, flag, m;
  unsigned long long sel_prefix, sel_mask;
  int sel_k;
};

__device__ __forceinline__ bool lex_less(double2 a, double2 b) { return a.x < b.x || (a.x == b.x && a.y < b.y); }

// order-preserving map of a double to u64
__device__ __forceinline__ unsigned long long okey(double d) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(d);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ double from_okey(unsigned long long k) {
  const unsigned long long b = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
  return __longlong_as_double((long long)b);
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return __shfl(v, 0, 64);   // one lane's rounding, identical in every lane
}

// block-wide sum of up to 4 doubles; result identical in every thread
template <int K>
__device__ __forceinline__ void block_sum(Smem& sm, double (&v)[K]) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    double s = v[k];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if (l == 0) sm.red[w][k] = s;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] = ((sm.red[0][k] + sm.red[1][k]) + sm.red[2][k]) + sm.red[3][k];
  __syncthreads();   // LDS-scalar invariant: every wave has read red[] before the next call rewrites it
}

// Mahalanobis distance of (x, y) to loc under the 2x2 precision P = [[p00, p01], [p01, p11]]
__device__ __forceinline__ double maha(double2 q, double lx, double ly, double p00, double p01, double p11) {
  const double dx = q.x - lx, dy = q.y - ly;
  return (dx * p00 + dy * p01) * dx + (dx * p01 + dy * p11) * dy;   // (np.dot(Xc, prec) * Xc).sum(1)
}

// k-th smallest (0-based) Mahalanobis distance over the n valid points, 8-bit radix select
__device__ double select_kth(Smem& sm, int n, int k, double lx, double ly, double p00, double p01, double p11) {
  if (threadIdx.x == 0) { sm.sel_prefix = 0; sm.sel_mask = 0; sm.sel_k = k; }
  __syncthreads();
  for (int shift = 56; shift >= 0; shift -= 8) {
    for (int b = threadIdx.x; b < 256; b += kThreads) sm.hist[b] = 0;
    __syncthreads();
    // invariant: prefix/mask go to registers here, before the barrier that
    // precedes thread 0's rewrite of them at the end of this pass
    const unsigned long long pre = sm.sel_prefix, msk = sm.sel_mask;
    for (int i = threadIdx.x; i < n; i += kThreads) {
      const double2 q = sm.pts[i];
      if (q.x != q.x) continue;
      const unsigned long long kd = okey(maha(q, lx, ly, p00, p01, p11));
      if ((kd & msk) == pre) atomicAdd(&sm.hist[(kd >> shift) & 255], 1);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      int kk = sm.sel_k, b = 0;
      for (; b < 255; ++b) {
        if (kk < sm.hist[b]) break;
        kk -= sm.hist[b];
      }
      sm.sel_k = kk;
      sm.sel_prefix = pre | ((unsigned long long)b << shift);
      sm.sel_mask = msk | (255ull << shift);
    }
    __syncthreads();
  }
  // every thread reads the result before any thread can start the next call
  // (whose thread 0 resets sel_prefix): without this barrier a late wave
  // could read the reset prefix when the median takes two calls (even count)
  const unsigned long long r = sm.sel_prefix;
  __syncthreads();
  return from_okey(r);
}

// searchsorted(linspace(-pi, pi, 100), a, side='right') = np.digitize(a, bins)
__device__ __forceinline__ int digitize(double a) {
  const double start = -kPi, step = (kPi - start) / 99.0;
  auto edge = [&](int k) { return k == 99 ? kPi : (double)k * step + start; };
  int k = (int)floor((a - start) / step);
  k = k < 0 ? 0 : (k > 99 ? 99 : k);
  while (k < 99 && edge(k + 1) <= a) ++k;
  while (k >= 0 && edge(k) > a) --k;
  return k + 1;
}

// ---- phase E: scipy trf on one wave -----------------------------------------
struct Rows {                 // two residual rows per lane: r = lane, lane + 64
  double x[2], y[2];
  bool ok[2];
};

// curve_fitting.py:478-484 ellipse_residuals
__device__ __forceinline__ double resid1(const double (&p)[5], double ct, double st, double x, double y) {
  const double dx = x - p[0], dy = y - p[1];
  const double xn = ct * dx + st * dy;
  const double yn = -st * dx + ct * dy;
  const double q0 = xn / p[2], q1 = yn / p[3];
  return (q0 * q0 + q1 * q1) - 1.0;
}

__device__ __forceinline__ void resid(const Rows& R, const double (&p)[5], double (&f)[2]) {
  double st, ct;
  sincos(p[4], &st, &ct);
#pragma unroll
  for (int s = 0; s < 2; ++s) f[s] = R.ok[s] ? resid1(p, ct, st, R.x[s], R.y[s]) : 0.0;
}

// _numdiff 2-point dense differences, J[row][col]
__device__ __forceinline__ void jacobian(const Rows& R, const double (&x)[5], const double (&f)[2], double (&J)[2][5]) {
  const double rstep = 1.4901161193847656e-08;   // EPS ** 0.5
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    double x1[5];
#pragma unroll
    for (int c = 0; c < 5; ++c) x1[c] = x[c];
    const double h = rstep * (x[i] >= 0.0 ? 1.0 : -1.0) * fmax(1.0, fabs(x[i]));
    x1[i] += h;
    const double dx = x1[i] - x[i];
    double f1[2];
    resid(R, x1, f1);
#pragma unroll
    for (int s = 0; s < 2; ++s) J[s][i] = R.ok[s] ? (f1[s] - f[s]) / dx : 0.0;
  }
}

__device__ __forceinline__ double dot5(const double (&a)[5], const double (&b)[5]) {
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < 5; ++i) s += a[i] * b[i];
  return s;
}

// thin SVD of J (m x 5, m >= 5): Householder QR of [J | f] over the wave gives
// R (5x5) and Q^T f; one-sided Jacobi on R (uniform in every lane) gives s, V and
// uf = U^T f.  s descending like LAPACK.
__device__ void svd_uf(const double (&J)[2][5], const double (&f)[2], int m, double (&s)[5], double (&V)[5][5],
                       double (&uf)[5]) {
  const int lane = threadIdx.x & 63;
  double a[2][6];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
#pragma unroll
    for (int c = 0; c < 5; ++c) a[r][c] = J[r][c];
    a[r][5] = f[r];
  }
  double Rm[5][6];
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    // rows > k below the diagonal; row k lives in lane k, slot 0
    double part = 0.0;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int row = lane + 64 * r;
      if (row > k && row < m) part += a[r][k] * a[r][k];
    }
    const double xn2 = wave_sum(part);
    const double akk = __shfl(a[0][k], k, 64);
    double beta = akk, tau = 0.0, scal = 0.0;
    if (xn2 > 0.0) {
      beta = -copysign(sqrt(akk * akk + xn2), akk);
      tau = (beta - akk) / beta;
      scal = 1.0 / (akk - beta);
    }
    double v[2];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int row = lane + 64 * r;
      v[r] = (row > k && row < m) ? a[r][k] * scal : 0.0;
    }
#pragma unroll
    for (int j = k + 1; j < 6; ++j) {
      const double w = __shfl(a[0][j], k, 64) + wave_sum(v[0] * a[0][j] + v[1] * a[1][j]);
      const double tw = tau * w;
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        const int row = lane + 64 * r;
        if (row == k) a[r][j] -= tw;
        else if (row > k && row < m) a[r][j] -= tw * v[r];
      }
    }
    if (lane == k) a[0][k] = beta;
  }
#pragma unroll
  for (int k = 0; k < 5; ++k)
#pragma unroll
    for (int j = 0; j < 6; ++j) Rm[k][j] = (j >= k) ? __shfl(a[0][j], k, 64) : 0.0;

  // one-sided Jacobi on the columns of R
  double A[5][5];
#pragma unroll
  for (int i = 0; i < 5; ++i)
#pragma unroll
    for (int j = 0; j < 5; ++j) { A[i][j] = Rm[i][j]; V[i][j] = (i == j) ? 1.0 : 0.0; }
  for (int sweep = 0; sweep < 60; ++sweep) {
    bool rotated = false;
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
      for (int q = p + 1; q < 5; ++q) {
        double al = 0.0, be = 0.0, ga = 0.0;
#pragma unroll
        for (int i = 0; i < 5; ++i) { al += A[i][p] * A[i][p]; be += A[i][q] * A[i][q]; ga += A[i][p] * A[i][q]; }
        if (ga != 0.0 && fabs(ga) > kEps * sqrt(al * be)) {
          rotated = true;
          const double zeta = (be - al) / (2.0 * ga);
          const double t = fabs(zeta) > 1e150 ? 0.5 / zeta
                                              : copysign(1.0, zeta) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
          const double cs = 1.0 / sqrt(1.0 + t * t), sn = cs * t;
#pragma unroll
          for (int i = 0; i < 5; ++i) {
            const double ap = A[i][p], aq = A[i][q];
            A[i][p] = cs * ap - sn * aq;
            A[i][q] = sn * ap + cs * aq;
            const double vp = V[i][p], vq = V[i][q];
            V[i][p] = cs * vp - sn * vq;
            V[i][q] = sn * vp + cs * vq;
          }
        }
      }
    if (!rotated) break;
  }
  int ord[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    double n2 = 0.0, d = 0.0;
#pragma unroll
    for (int i = 0; i < 5; ++i) { n2 += A[i][j] * A[i][j]; d += A[i][j] * Rm[i][5]; }
    s[j] = sqrt(n2);
    uf[j] = s[j] > 0.0 ? d / s[j] : 0.0;
    ord[j] = j;
  }
  // descending order (insertion sort on 5)
  for (int i = 1; i < 5; ++i)
    for (int j = i; j > 0 && s[ord[j]] > s[ord[j - 1]]; --j) { const int t = ord[j]; ord[j] = ord[j - 1]; ord[j - 1] = t; }
  double s2[5], u2[5], V2[5][5];
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    s2[j] = s[ord[j]];
    u2[j] = uf[ord[j]];
#pragma unroll
    for (int i = 0; i < 5; ++i) V2[i][j] = V[i][ord[j]];
  }
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    s[j] = s2[j];
    uf[j] = u2[j];
#pragma unroll
    for (int i = 0; i < 5; ++i) V[i][j] = V2[i][j];
  }
}

__device__ __forceinline__ double norm5(const double (&a)[5]) { return sqrt(dot5(a, a)); }

// scipy.optimize._lsq.common.solve_lsq_trust_region (rtol 0.01, max_iter 10)
__device__ void tr_step(int m, const double (&uf)[5], const double (&s)[5], const double (&V)[5][5], double Delta,
                        double& alpha, double (&p)[5]) {
  double suf[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) suf[i] = s[i] * uf[i];
  const bool full_rank = m >= 5 && s[4] > kEps * m * s[0];
  if (full_rank) {
    double t[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) t[i] = uf[i] / s[i];
#pragma unroll
    for (int i = 0; i < 5; ++i) p[i] = -dot5(V[i], t);
    if (norm5(p) <= Delta) { alpha = 0.0; return; }
  }
  auto phi = [&](double al, double& dphi) {
    double q[5], acc = 0.0;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      const double den = s[i] * s[i] + al;
      q[i] = suf[i] / den;
      acc += suf[i] * suf[i] / (den * den * den);
    }
    const double pn = norm5(q);
    dphi = -acc / pn;
    return pn - Delta;
  };
  double hi = norm5(suf) / Delta, lo = 0.0;
  if (full_rank) {
    double d0;
    const double p0 = phi(0.0, d0);
    lo = -p0 / d0;
  }
  double al = (!full_rank && alpha == 0.0) ? fmax(0.001 * hi, sqrt(lo * hi)) : alpha;
  for (int it = 0; it < 10; ++it) {
    if (al < lo || al > hi) al = fmax(0.001 * hi, sqrt(lo * hi));
    double dph;
    const double ph = phi(al, dph);
    if (ph < 0.0) hi = al;
    const double ratio = ph / dph;
    lo = fmax(lo, al - ratio);
    al -= (ph + Delta) * ratio / Delta;
    if (fabs(ph) < 0.01 * Delta) break;
  }
  double t[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) t[i] = suf[i] / (s[i] * s[i] + al);
#pragma unroll
  for (int i = 0; i < 5; ++i) p[i] = -dot5(V[i], t);
  const double sc = Delta / norm5(p);
#pragma unroll
  for (int i = 0; i < 5; ++i) p[i] *= sc;
  alpha = al;
}

__device__ __forceinline__ void grad(const double (&J)[2][5], const double (&f)[2], double (&g)[5]) {
#pragma unroll
  for (int i = 0; i < 5; ++i) g[i] = wave_sum(J[0][i] * f[0] + J[1][i] * f[1]);
}

// trf_no_bounds (linear loss, x_scale 1, tr_solver 'exact'); returns nfev, *status
__device__ int trf(const Rows& R, int m, double (&x)[5], int& status) {
  const double ftol = 1e-8, xtol = 1e-8, gtol = 1e-8;
  double f[2], J[2][5], g[5];
  resid(R, x, f);
  int nfev = 1;
  jacobian(R, x, f, J);
  double cost = 0.5 * wave_sum(f[0] * f[0] + f[1] * f[1]);
  grad(J, f, g);
  double Delta = norm5(x);
  if (Delta == 0.0) Delta = 1.0;
  double alpha = 0.0;
  status = 0;
  for (;;) {
    double gn = 0.0;
#pragma unroll
    for (int i = 0; i < 5; ++i) gn = fmax(gn, fabs(g[i]));
    if (gn < gtol) status = 1;
    if (status != 0 || nfev == kMaxNfev) break;
    double s[5], V[5][5], uf[5];
    svd_uf(J, f, m, s, V, uf);
    double actual = -1.0, cost_new = 0.0, xn[5], fn[2];
    while (actual <= 0.0 && nfev < kMaxNfev) {
      double step[5];
      tr_step(m, uf, s, V, Delta, alpha, step);
      double js[2];
#pragma unroll
      for (int r = 0; r < 2; ++r) js[r] = dot5(J[r], step);
      const double q = wave_sum(js[0] * js[0] + js[1] * js[1]);
      const double predicted = -(0.5 * q + dot5(step, g));
#pragma unroll
      for (int i = 0; i < 5; ++i) xn[i] = x[i] + step[i];
      resid(R, xn, fn);
      ++nfev;
      const double sn = norm5(step);
      const double fin = wave_sum((isfinite(fn[0]) ? 0.0 : 1.0) + (isfinite(fn[1]) ? 0.0 : 1.0));
      if (fin != 0.0) { Delta = 0.25 * sn; continue; }
      cost_new = 0.5 * wave_sum(fn[0] * fn[0] + fn[1] * fn[1]);
      actual = cost - cost_new;
      double ratio;
      if (predicted > 0.0) ratio = actual / predicted;
      else if (predicted == actual && actual == 0.0) ratio = 1.0;
      else ratio = 0.0;
      double Dn = Delta;
      if (ratio < 0.25) Dn = 0.25 * sn;
      else if (ratio > 0.75 && sn > 0.95 * Delta) Dn = 2.0 * Delta;
      const bool fok = actual < ftol * cost && ratio > 0.25;
      const bool xok = sn < xtol * (xtol + norm5(x));
      status = (fok && xok) ? 4 : fok ? 2 : xok ? 3 : 0;
      if (status != 0) break;
      alpha *= Delta / Dn;
      Delta = Dn;
    }
    if (actual > 0.0) {
#pragma unroll
      for (int i = 0; i < 5; ++i) x[i] = xn[i];
      f[0] = fn[0];
      f[1] = fn[1];
      cost = cost_new;
      jacobian(R, x, f, J);
      grad(J, f, g);
    }
  }
  return nfev;
}

// ---- the kernel ------------------------------------------------------------------
// blockIdx.x = 2 * set + side; side 0 = RF_max (farthest per bin), 1 = RF_min (nearest)
__global__ void __launch_bounds__(kThreads) ellipse_kernel(int32_t ndir, const double* __restrict__ rf_max,
                                                           const double* __restrict__ rf_min,
                                                           const uint8_t* __restrict__ status,
                                                           double* __restrict__ out, int32_t* __restrict__ info,
                                                           double* __restrict__ fit_out, double* __restrict__ center_out) {
  __shared__ Smem sm;
  const int64_t set = blockIdx.x >> 1;
  const int side = blockIdx.x & 1;
  const bool farthest = side == 0;
  const double* rf = (side == 0 ? rf_max : rf_min) + 3 * set * (int64_t)ndir;
  const uint8_t* st = status + set * (int64_t)ndir;
  double* o = out + 5 * blockIdx.x;
  const int tid = threadIdx.x;

  // A: gather (LDS-scalar invariant: cnt / flag are written only here, before
  // the barrier below, and are read-only for the rest of the block)
  if (tid == 0) { sm.cnt = 0; sm.flag = 0; }
  __syncthreads();
  for (int d = tid; d < ndir; d += kThreads) {
    const uint8_t s = st[d];
    if (s == 2) sm.flag = 1;
    if (s != 1) continue;
    const double x = rf[3 * (int64_t)d], y = rf[3 * (int64_t)d + 1];
    if (x != x || y != y) continue;
    const int pos = atomicAdd(&sm.cnt, 1);
    if (pos < kCap) sm.pts[pos] = make_double2(x, y);
  }
  __syncthreads();
  const int n = sm.cnt;
  int err = 0;
  if (sm.flag) err = kErrStaleTheta;
  else if (n > kCap) err = kErrTooMany;
  else if (n < 2) err = kErrTooFew;
  if (err) {
    if (tid < 5) o[tid] = __longlong_as_double(0x7ff8000000000000ll);
    if (tid == 0) info[blockIdx.x] = err;
    return;
  }

  // B: bitonic sort of the padded power of two, then mark duplicates (x := NaN)
  int n2 = 1;
  while (n2 < n) n2 <<= 1;
  for (int i = n + tid; i < n2; i += kThreads) sm.pts[i] = make_double2(INFINITY, INFINITY);
  __syncthreads();
  for (int k = 2; k <= n2; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < n2; i += kThreads) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const double2 a = sm.pts[i], b = sm.pts[ixj];
          const bool up = (i & k) == 0;
          if (lex_less(b, a) == up) { sm.pts[i] = b; sm.pts[ixj] = a; }
        }
      }
      __syncthreads();
    }
  unsigned dupmask = 0;   // up to kCap / kThreads = 32 entries per thread
  for (int r = 0, i = tid; i < n; ++r, i += kThreads)
    if (i > 0 && sm.pts[i].x == sm.pts[i - 1].x && sm.pts[i].y == sm.pts[i - 1].y) dupmask |= 1u << r;
  __syncthreads();
  for (int r = 0, i = tid; i < n; ++r, i += kThreads)
    if (dupmask >> r & 1) sm.pts[i].x = __longlong_as_double(0x7ff8000000000000ll);
  __syncthreads();

  // C: MCD center with support_fraction = 1
  double acc[3] = {0.0, 0.0, 0.0};
  for (int i = tid; i < n; i += kThreads) {
    const double2 q = sm.pts[i];
    if (q.x != q.x) continue;
    acc[0] += q.x; acc[1] += q.y; acc[2] += 1.0;
  }
  block_sum(sm, acc);
  const int nu = (int)acc[2];
  if (nu < 2) {
    if (tid < 5) o[tid] = __longlong_as_double(0x7ff8000000000000ll);
    if (tid == 0) info[blockIdx.x] = kErrTooFew;
    return;
  }
  const double lx = acc[0] / nu, ly = acc[1] / nu;
  double cv[3] = {0.0, 0.0, 0.0};
  for (int i = tid; i < n; i += kThreads) {
    const double2 q = sm.pts[i];
    if (q.x != q.x) continue;
    const double dx = q.x - lx, dy = q.y - ly;
    cv[0] += dx * dx; cv[1] += dx * dy; cv[2] += dy * dy;
  }
  block_sum(sm, cv);
  const double c00 = cv[0] * (1.0 / nu), c01 = cv[1] * (1.0 / nu), c11 = cv[2] * (1.0 / nu);
  const double det = c00 * c11 - c01 * c01;
  const double p00 = c11 / det, p01 = -c01 / det, p11 = c00 / det;
  double med;
  if (nu & 1) {
    med = select_kth(sm, n, nu / 2, lx, ly, p00, p01, p11);
  } else {
    const double lo = select_kth(sm, n, nu / 2 - 1, lx, ly, p00, p01, p11);
    const double hi = select_kth(sm, n, nu / 2, lx, ly, p00, p01, p11);
    med = (lo + hi) / 2.0;
  }
  const double corr = med / kIsf050;
  double rw[3] = {0.0, 0.0, 0.0};
  for (int i = tid; i < n; i += kThreads) {
    const double2 q = sm.pts[i];
    if (q.x != q.x) continue;
    if (maha(q, lx, ly, p00, p01, p11) / corr < kIsf0025) { rw[0] += q.x; rw[1] += q.y; rw[2] += 1.0; }
  }
  block_sum(sm, rw);
  const double cx = rw[0] / rw[2], cy = rw[1] / rw[2];

  // D: one point per angular bin
  for (int b = tid; b < kBins; b += kThreads) {
    sm.best[b] = farthest ? 0ull : ~0ull;
    sm.first[b] = INT32_MAX;
    sm.pick[b] = INT32_MAX;
  }
  __syncthreads();
  for (int i = tid; i < n; i += kThreads) {
    const double2 q = sm.pts[i];
    if (q.x != q.x) continue;
    const double dx = q.x - cx, dy = q.y - cy;
    const int b = digitize(atan2(dy, dx));
    const unsigned long long kd = okey(sqrt(dx * dx + dy * dy));
    atomicMin(&sm.first[b], i);
    if (farthest) atomicMax(&sm.best[b], kd);
    else atomicMin(&sm.best[b], kd);
  }
  __syncthreads();
  for (int i = tid; i < n; i += kThreads) {
    const double2 q = sm.pts[i];
    if (q.x != q.x) continue;
    const double dx = q.x - cx, dy = q.y - cy;
    const int b = digitize(atan2(dy, dx));
    if (okey(sqrt(dx * dx + dy * dy)) == sm.best[b]) atomicMin(&sm.pick[b], i);
  }
  __syncthreads();
  if (tid < kBins) {
    const int fb = sm.first[tid];
    if (fb != INT32_MAX) {
      int rank = 0;
      for (int b = 0; b < kBins; ++b) rank += sm.first[b] < fb;
      sm.fit[rank] = sm.pts[sm.pick[tid]];
    }
  }
  if (tid == 0) {   // (invariant: m is written once, read after the barrier, never rewritten)
    int m = 0;
    for (int b = 0; b < kBins; ++b) m += sm.first[b] != INT32_MAX;
    sm.m = m;
  }
  __syncthreads();
  const int m = sm.m;
  if (center_out && tid < 2) center_out[2 * blockIdx.x + tid] = tid == 0 ? cx : cy;
  if (fit_out)
    for (int i = tid; i < kMaxFit; i += kThreads) {
      const double2 q = i < m ? sm.fit[i] : make_double2(NAN, NAN);
      fit_out[2 * (kMaxFit * (int64_t)blockIdx.x + i)] = q.x;
      fit_out[2 * (kMaxFit * (int64_t)blockIdx.x + i) + 1] = q.y;
    }
  if (tid >= 64) return;   // E runs on wave 0 only (no block barriers below)
  if (m < 5) {
    if (tid < 5) o[tid] = __longlong_as_double(0x7ff8000000000000ll);
    if (tid == 0) info[blockIdx.x] = kErrTooFew;
    return;
  }

  // E: least squares from [mean(x), mean(y), std(x), std(y), 0]
  Rows R;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int row = tid + 64 * s;
    R.ok[s] = row < m;
    R.x[s] = R.ok[s] ? sm.fit[row].x : 0.0;
    R.y[s] = R.ok[s] ? sm.fit[row].y : 0.0;
  }
  const double mx = wave_sum(R.x[0] + R.x[1]) / m, my = wave_sum(R.y[0] + R.y[1]) / m;
  double vx = 0.0, vy = 0.0;
#pragma unroll
  for (int s = 0; s < 2; ++s)
    if (R.ok[s]) {
      const double ax = fabs(R.x[s] - mx), ay = fabs(R.y[s] - my);
      vx += ax * ax;
      vy += ay * ay;
    }
  double x[5] = {mx, my, sqrt(wave_sum(vx) / m), sqrt(wave_sum(vy) / m), 0.0};
  int lsq_status = 0;
  const int nfev = trf(R, m, x, lsq_status);
  if (tid < 5) {
    double v = x[0];
#pragma unroll
    for (int i = 1; i < 5; ++i) v = tid == i ? x[i] : v;
    o[tid] = v;
  }
  if (tid == 0) info[blockIdx.x] = nfev;
}

}  // namespace ellipse
