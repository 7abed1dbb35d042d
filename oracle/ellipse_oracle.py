"""oracle/ellipse_oracle.py -- TEST INFRASTRUCTURE ONLY.

numpy restatement of single_pluse_model/curve_fitting.py:Curve_fitting
(:475-576), the ellipse fit applied to the reachable-domain point lists.
Only tests/ and bench.py's cpu_baseline leg may import it.

Third-party algorithms it depends on, with the versions in this image:
- sklearn 1.7.2 EllipticEnvelope(support_fraction=1.0).fit(points).location_
  (:545-547).  With support_fraction = 1 every FastMCD candidate support is
  the whole sample, so the raw estimate is the sample mean / biased
  covariance; MinCovDet.correct_covariance divides the Mahalanobis distances
  by median(d) / chi2(2).isf(0.5), and reweight_covariance takes the mean of
  the points with corrected d < chi2(2).isf(0.025).  Restated in closed form
  below (`mcd_center`) and checked against sklearn in tests.
- scipy 1.15.3 least_squares(ellipse_residuals, x0) (:491): method 'trf',
  2-point Jacobian, x_scale 1, ftol = xtol = gtol = 1e-8, max_nfev 500.
  `fit_ellipse` calls scipy itself (it is the checker); `trf_restated` is a
  step-by-step restatement of scipy's trf_no_bounds / solve_lsq_trust_region
  with the SVD from numpy, used to pin the HIP kernel's iteration.
"""
from __future__ import annotations

import numpy as np

CHI2_2_ISF_050 = 1.386294361119891     # scipy.stats.chi2(2).isf(0.5)
CHI2_2_ISF_0025 = 7.3777589082278725   # scipy.stats.chi2(2).isf(0.025)
N_BINS = 100                           # curve_fitting.py:554


def unique_points(data):
    """curve_fitting.py:534-543: xy columns, np.unique rows (lexicographic),
    rows with a NaN dropped."""
    xy = np.asarray(data, dtype=np.float64)[:, :2]
    u = np.unique(xy, axis=0)
    return u[~np.isnan(u).any(axis=1)]


def mcd_center(points):
    """EllipticEnvelope(support_fraction=1.0).fit(points).location_ in closed form."""
    loc = points.mean(0)
    xc = points - loc
    cov = xc.T @ xc / len(points)
    prec = np.linalg.pinv(cov, hermitian=True)
    d = ((xc @ prec) * xc).sum(1)
    d = d / (np.median(d) / CHI2_2_ISF_050)
    return points[d < CHI2_2_ISF_0025].mean(0)


def bin_edges():
    return np.linspace(-np.pi, np.pi, N_BINS)


def filter_points(points, center, farthest):
    """curve_fitting.py:550-572: one point per angular bin around the center,
    farthest (flag 1, RF_max) or nearest (flag 0, RF_min); bins in order of
    first appearance, ties keep the first point."""
    ang = np.arctan2(points[:, 1] - center[1], points[:, 0] - center[0])
    dist = np.sqrt(((points - center) ** 2).sum(1))
    idx = np.digitize(ang, bin_edges())
    best = {}
    for k in range(len(points)):
        b = idx[k]
        if b not in best or (dist[k] > best[b][0] if farthest else dist[k] < best[b][0]):
            best[b] = (dist[k], k)
    return points[[k for _, k in best.values()]]


def residuals(p, x, y):
    """curve_fitting.py:478-484 ellipse_residuals."""
    xc, yc, a, b, th = p
    ct, st = np.cos(th), np.sin(th)
    xn = ct * (x - xc) + st * (y - yc)
    yn = -st * (x - xc) + ct * (y - yc)
    return ((xn / a) ** 2 + (yn / b) ** 2) - 1


def initial_guess(fp):
    x, y = fp[:, 0], fp[:, 1]
    return np.array([np.mean(x), np.mean(y), np.std(x), np.std(y), 0.0])   # :489


def fit_ellipse(fp):
    """curve_fitting.py:486-492 with scipy's own least_squares."""
    from scipy.optimize import least_squares
    x, y = fp[:, 0], fp[:, 1]
    return least_squares(residuals, initial_guess(fp), args=(x, y)).x


def trf_restated(fp, ftol=1e-8, xtol=1e-8, gtol=1e-8):
    """scipy.optimize._lsq.trf.trf_no_bounds (tr_solver 'exact', x_scale 1,
    linear loss) + common.solve_lsq_trust_region / update_tr_radius /
    check_termination + _numdiff 2-point dense differences.  Returns
    (x, nfev, status)."""
    x_, y_ = fp[:, 0], fp[:, 1]
    fun = lambda p: residuals(p, x_, y_)
    eps = np.finfo(float).eps
    rstep = eps ** 0.5

    def jac(x0, f0):
        h = rstep * ((x0 >= 0) * 2.0 - 1) * np.maximum(1.0, np.abs(x0))
        J = np.empty((f0.size, x0.size))
        for i in range(x0.size):
            x1 = x0.copy()
            x1[i] += h[i]
            J[:, i] = (fun(x1) - f0) / (x1[i] - x0[i])
        return J

    x = initial_guess(fp)
    n = x.size
    f = fun(x)
    m = f.size
    nfev, max_nfev = 1, 100 * n
    J = jac(x, f)
    cost = 0.5 * f @ f
    g = J.T @ f
    Delta = np.linalg.norm(x) or 1.0
    alpha = 0.0
    status = None
    while True:
        if np.linalg.norm(g, np.inf) < gtol:
            status = 1
        if status is not None or nfev == max_nfev:
            break
        U, s, VT = np.linalg.svd(J, full_matrices=False)
        V = VT.T
        uf = U.T @ f
        actual = -1.0
        while actual <= 0 and nfev < max_nfev:
            step, alpha = _tr_step(n, m, uf, s, V, Delta, alpha)
            Js = J @ step
            predicted = -(0.5 * Js @ Js + step @ g)
            x_new = x + step
            f_new = fun(x_new)
            nfev += 1
            sn = np.linalg.norm(step)
            if not np.all(np.isfinite(f_new)):
                Delta = 0.25 * sn
                continue
            cost_new = 0.5 * f_new @ f_new
            actual = cost - cost_new
            if predicted > 0:
                ratio = actual / predicted
            elif predicted == actual == 0:
                ratio = 1
            else:
                ratio = 0
            Delta_new = Delta
            if ratio < 0.25:
                Delta_new = 0.25 * sn
            elif ratio > 0.75 and sn > 0.95 * Delta:
                Delta_new = 2.0 * Delta
            ftol_ok = actual < ftol * cost and ratio > 0.25
            xtol_ok = sn < xtol * (xtol + np.linalg.norm(x))
            status = 4 if (ftol_ok and xtol_ok) else 2 if ftol_ok else 3 if xtol_ok else None
            if status is not None:
                break
            alpha *= Delta / Delta_new
            Delta = Delta_new
        if actual > 0:
            x, f, cost = x_new, f_new, cost_new
            J = jac(x, f)
            g = J.T @ f
    return x, nfev, status or 0


def _tr_step(n, m, uf, s, V, Delta, alpha0, rtol=0.01, max_iter=10):
    suf = s * uf
    full_rank = m >= n and s[-1] > np.finfo(float).eps * m * s[0]
    if full_rank:
        p = -V @ (uf / s)
        if np.linalg.norm(p) <= Delta:
            return p, 0.0

    def phi(al):
        den = s ** 2 + al
        pn = np.linalg.norm(suf / den)
        return pn - Delta, -np.sum(suf ** 2 / den ** 3) / pn

    hi = np.linalg.norm(suf) / Delta
    if full_rank:
        ph, dph = phi(0.0)
        lo = -ph / dph
    else:
        lo = 0.0
    if not full_rank and alpha0 == 0:
        al = max(0.001 * hi, (lo * hi) ** 0.5)
    else:
        al = alpha0
    for _ in range(max_iter):
        if al < lo or al > hi:
            al = max(0.001 * hi, (lo * hi) ** 0.5)
        ph, dph = phi(al)
        if ph < 0:
            hi = al
        r = ph / dph
        lo = max(lo, al - r)
        al -= (ph + Delta) * r / Delta
        if abs(ph) < rtol * Delta:
            break
    p = -V @ (suf / (s ** 2 + al))
    return p * (Delta / np.linalg.norm(p)), al


def curve_fitting(rf_max, rf_min, solver="scipy"):
    """Curve_fitting(RF_max, RF_min) -> [2][5] (xc, yc, a, b, theta) for the
    farthest (RF_max) and nearest (RF_min) envelopes."""
    out = []
    for data, far in ((rf_max, True), (rf_min, False)):
        pts = unique_points(data)
        fp = filter_points(pts, mcd_center(pts), far)
        out.append(fit_ellipse(fp) if solver == "scipy" else trf_restated(fp)[0])
    return np.array(out)
