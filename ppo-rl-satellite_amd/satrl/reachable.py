"""Reachable domain of a single impulse on the GPU.

Restates single_pluse_model/RD_single_pulse.py:Reachable_Domain (:40-148)
as the satenv_reachable_domain kernel: the N1 x (N2+1) x (N3+1) direction
grid, the reachability test (:79-81), beta / Delta_Vm / theta (:82-90), two
hybrd solves per direction (:93-121, fsolve of :150-157) and the extreme
points max/min(|rf|) * P (:123-124).  Many orbits run in one launch
(`reachable_domain_grid`), which is what a vectorised Flag-2 env needs; the
reference runs one orbit per call at ~0.9 s.

`ellipse_fit` restates curve_fitting.Curve_fitting (:475-576) as the
satenv_ellipse_fit kernel on the same dense grids (no host round trip):
EllipticEnvelope center, angular-bin filtering and scipy's trf least squares.

`params` / `Incoming_parameters` / `Reachable_Domain` mirror the module's
globals-driven API (:9-37, :40-148) and return the [2][5] ellipse array like
the reference; `reachable_points` returns the RF_max / RF_min lists.
"""
import numpy as np
import torch

from . import _lib
from ._lib import check, ptr, stream_ptr

# RD_single_pulse.py:9-20
params = {
    "a": 10 ** 7,
    "i": 0,
    "e0": 0.2,
    "f": np.pi / 2,
    "delta_max": 500,
    "u": 3.986e14,
    "N1": 1,
    "N2": 200,
    "N3": 200,
    "delta_l": 1500,
}

UNREACHABLE, REACHABLE, THETA_UNDEFINED = 0, 1, 2


def orbits_tensor(a, e0, f, delta_max, mu=3.986e14, device="cuda", dv_f32=0.0):
    """[nsets][6] f64 rows (a, e0, f, delta_max, mu, dv_f32) = satenv_rd_orbit;
    scalars broadcast.  dv_f32 != 0: delta_max is an np.float32 scalar."""
    cols = np.broadcast_arrays(*[np.asarray(v, dtype=np.float64) for v in (a, e0, f, delta_max, mu, dv_f32)])
    arr = np.stack([c.reshape(-1) for c in cols], axis=1)
    return torch.tensor(arr, dtype=torch.float64, device=device)


def reachable_domain_grid(orbits, n1=1, n2=200, n3=200, stream=None):
    """Dense grid for every orbit: (rf_max [nsets][ndir][3], rf_min, status
    [nsets][ndir] u8) with ndir = n1*(n2+1)*(n3+1), direction order of the
    reference loops (jj, i, j).  Entries with status != 1 are zero."""
    _lib.require_cuda(orbits, torch.float64, None, "orbits")
    if orbits.dim() != 2 or orbits.shape[1] != 6 or not orbits.is_contiguous():
        raise ValueError("orbits must be a contiguous [nsets][6] f64 tensor (satenv_rd_orbit)")
    nsets = orbits.shape[0]
    ndir = int(n1) * (int(n2) + 1) * (int(n3) + 1)
    dev = orbits.device
    rf_max = torch.zeros((nsets, ndir, 3), dtype=torch.float64, device=dev)
    rf_min = torch.zeros_like(rf_max)
    status = torch.empty((nsets, ndir), dtype=torch.uint8, device=dev)
    check(_lib.lib().satenv_reachable_domain(nsets, ptr(orbits), int(n1), int(n2), int(n3), ptr(rf_max),
                                             ptr(rf_min), ptr(status), stream_ptr(stream)),
          "satenv_reachable_domain")
    return rf_max, rf_min, status


def reachable_domain(a, e0, f, delta_max, n1=1, n2=200, n3=200, mu=3.986e14, device="cuda"):
    """RF_max, RF_min ([m][3] f64, on `device`) of one orbit, in the
    reference's append order (RD_single_pulse.py:123-124, :138-139)."""
    orbits = orbits_tensor(a, e0, f, delta_max, mu, device)
    mx, mn, st = reachable_domain_grid(orbits, n1, n2, n3)
    st = st[0]
    if bool((st == THETA_UNDEFINED).any()):
        raise ValueError("gama - f outside the theta branches of RD_single_pulse.py:87-90 "
                         "(the reference would reuse a stale theta)")
    keep = st == REACHABLE
    return mx[0][keep], mn[0][keep]


ELL_STALE_THETA, ELL_TOO_MANY, ELL_TOO_FEW = -1, -2, -3


def ellipse_fit(rf_max, rf_min, status, stream=None, intermediates=False):
    """curve_fitting.Curve_fitting on dense grids from reachable_domain_grid:
    returns (ellipse [nsets][2][5] f64 = (xc, yc, a, b, theta) of the RF_max
    and RF_min envelopes, info [nsets][2] i32: > 0 least-squares function
    evaluations, < 0 no fit (ELL_*; parameters NaN)).  intermediates=True
    also returns the fitted point sets [nsets][2][128][2] (NaN-padded) and
    the EllipticEnvelope centers [nsets][2][2]."""
    nsets, ndir = status.shape
    _lib.require_cuda(status, torch.uint8, (nsets, ndir), "status")
    _lib.require_cuda(rf_max, torch.float64, (nsets, ndir, 3), "rf_max")
    _lib.require_cuda(rf_min, torch.float64, (nsets, ndir, 3), "rf_min")
    out = torch.empty((nsets, 2, 5), dtype=torch.float64, device=status.device)
    info = torch.empty((nsets, 2), dtype=torch.int32, device=status.device)
    fit = cen = None
    if intermediates:
        fit = torch.empty((nsets, 2, 128, 2), dtype=torch.float64, device=status.device)
        cen = torch.empty((nsets, 2, 2), dtype=torch.float64, device=status.device)
    check(_lib.lib().satenv_ellipse_fit(nsets, ndir, ptr(rf_max), ptr(rf_min), ptr(status), ptr(out), ptr(info),
                                        ptr(fit) if fit is not None else None, ptr(cen) if cen is not None else None,
                                        stream_ptr(stream)), "satenv_ellipse_fit")
    return (out, info, fit, cen) if intermediates else (out, info)


def reachable_ellipses(orbits, n1=1, n2=200, n3=200, stream=None):
    """Grid + fit for every orbit: (ellipse [nsets][2][5], info [nsets][2])."""
    return ellipse_fit(*reachable_domain_grid(orbits, n1, n2, n3, stream), stream=stream)


def reachable_points(device="cuda"):
    """The (RF_max, RF_min) numpy lists Reachable_Domain builds from `params` (:138-139)."""
    p = params
    mx, mn = reachable_domain(p["a"], p["e0"], p["f"], p["delta_max"], p["N1"], p["N2"], p["N3"], p["u"], device)
    return mx.cpu().numpy(), mn.cpu().numpy()


def Reachable_Domain(device="cuda"):
    """RD_single_pulse.Reachable_Domain (:40-148) on the module `params`:
    the [2][5] ellipse array of Curve_fitting (:140)."""
    p = params
    orbits = orbits_tensor(p["a"], p["e0"], p["f"], p["delta_max"], p["u"], device,
                           dv_f32=isinstance(p["delta_max"], np.float32))
    ell, info = reachable_ellipses(orbits, p["N1"], p["N2"], p["N3"])
    info = info.cpu().numpy()
    if (info < 0).any():
        raise ValueError(f"reachable-domain ellipse fit failed (info {info.tolist()}, see satenv_ellipse_fit)")
    return ell[0].cpu().numpy()


def Incoming_parameters(data, delta_max, device="cuda"):
    """RD_single_pulse.py:22-37: orbit elements data = [a, e, i, ., ., f]."""
    params["a"], params["i"], params["e0"], params["f"] = data[0], data[2], data[1], data[5]
    params["delta_max"] = delta_max
    return np.array(Reachable_Domain(device))


def env_orbits(env, stream=None):
    """Flag 2's Incoming_parameters orbit of every env of a VecSatellites
    (environment.py:293-296 -> real_time_data_process.py:107-110):
    ([N][6] f64 satenv_rd_orbit rows, status [N] i32: 0 or the
    SATENV_ERR_ORBIT_* of an orbit without a 6-element set)."""
    n = env.num_envs
    orbits = torch.empty((n, 6), dtype=torch.float64, device=env.device)
    status = torch.empty(n, dtype=torch.int32, device=env.device)
    check(_lib.lib().satenv_rd_orbits(env._h, ptr(orbits), ptr(status), stream_ptr(stream)), "satenv_rd_orbits")
    return orbits, status


def env_ellipse_params(env, chunk=512, n1=None, n2=None, n3=None, stream=None):
    """numerical_method_process for every env (the Flag-2 ellipse_params,
    environment.py:296): [N][2][5] f64 ellipses and info [N][2] i32 (see
    ellipse_fit; rows of envs without a 6-element orbit are NaN with info
    SATENV_ERR_ORBIT_*).  The 201 x 201 direction grids of `chunk` envs at a
    time (2 x 0.97 MB of points per env) go through the grid and fit kernels
    without leaving the GPU."""
    p = params
    n1 = p["N1"] if n1 is None else n1
    n2 = p["N2"] if n2 is None else n2
    n3 = p["N3"] if n3 is None else n3
    orbits, status = env_orbits(env, stream)
    n = env.num_envs
    ell = torch.full((n, 2, 5), float("nan"), dtype=torch.float64, device=env.device)
    info = torch.empty((n, 2), dtype=torch.int32, device=env.device)
    for s0 in range(0, n, chunk):
        s1 = min(n, s0 + chunk)
        e, i = reachable_ellipses(orbits[s0:s1].contiguous(), n1, n2, n3, stream)
        ell[s0:s1] = e
        info[s0:s1] = i
    bad = status != 0
    ell[bad] = float("nan")
    info[bad] = status[bad].unsqueeze(1).expand(-1, 2)
    return ell, info
