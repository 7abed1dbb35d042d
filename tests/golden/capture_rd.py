#!/usr/bin/env python3
"""Capture golden vectors for the reachable-domain grid (build container
ONLY; imports the reference read-only).

single_pluse_model/RD_single_pulse.py:Reachable_Domain (:40-148) sweeps
N1 x (N2+1) x (N3+1) impulse directions, keeps the reachable ones and hands
the rf extreme points to curve_fitting.Curve_fitting.  Here Curve_fitting is
replaced by a recorder, so the fixture holds exactly the RF_max / RF_min
point lists the reference computes (the ellipse fit is host-side sklearn
post-processing, outside the accelerated path).  Each case runs twice: as
is, and with glibc arccos/arctan/tan (numpy's are SVML; see
capture_golden.py), which pins the C oracle bit-exactly.

Fixture rd_grid.npz: for case k, prm_k = [a, e0, f, delta_max, u, N1, N2, N3],
rfmax_k / rfmin_k [m][3] (as is), rfmax_glibc_k / rfmin_glibc_k, and ell_k
[2][5] = the real Curve_fitting(rfmax_k, rfmin_k) (sklearn 1.7.2, scipy 1.15.3).
Plus the reference's own golden pairs (data files, not code):
pairs_in [r][5] = all_input.csv rows (a, e, i, f, fuel), pairs_out [r][10] =
output_data.csv rows, pairs_rows = the row numbers.

Run:  python tests/golden/capture_rd.py     (about a minute)
"""
import contextlib
import math
import os
import sys
import tempfile
import types

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))

CASES = [
    # a, e0, f, delta_max, N1, N2, N3   (u = 3.986e14 as in the reference params)
    (10 ** 7, 0.2, np.pi / 2, 500, 1, 200, 200),          # the module's own params (:9-20)
    (42164000.0, 0.01, 1.0, 300.0, 1, 80, 80),
    (24000000.0, 0.7, 2.5, 800.0, 2, 60, 60),
    (8000000.0, 0.05, 4.0, 150.0, 1, 90, 400),
]


class _GlibcNP(types.ModuleType):
    def __getattr__(self, k):
        return getattr(np, k)


@contextlib.contextmanager
def glibc_libm(mod):
    proxy = _GlibcNP("numpy_glibc")
    proxy.arccos = lambda x: np.float64(math.acos(float(x)))
    proxy.arctan = lambda x: np.float64(math.atan(float(x)))
    proxy.tan = lambda x: np.float64(math.tan(float(x)))
    saved = mod.np
    mod.np = proxy
    try:
        yield
    finally:
        mod.np = saved


def main():
    sys.path.insert(0, REF)
    stub = tempfile.mkdtemp()
    sys.path.insert(0, stub)
    os.environ.setdefault("MPLBACKEND", "Agg")
    import single_pluse_model.RD_single_pulse as rd
    got = {}

    def recorder(RF_max, RF_min):
        got["max"] = np.array(RF_max, dtype=np.float64).reshape(-1, 3)
        got["min"] = np.array(RF_min, dtype=np.float64).reshape(-1, 3)
        return np.zeros((2, 5))

    real_fit = rd.cf.Curve_fitting
    rd.cf.Curve_fitting = recorder
    out = {}
    for k, (a, e0, f, dmax, n1, n2, n3) in enumerate(CASES):
        rd.params.update({"a": a, "e0": e0, "f": f, "delta_max": dmax, "N1": n1, "N2": n2, "N3": n3})
        rd.Reachable_Domain()
        out[f"rfmax_{k}"], out[f"rfmin_{k}"] = got["max"], got["min"]
        with glibc_libm(rd):
            rd.Reachable_Domain()
        out[f"rfmax_glibc_{k}"], out[f"rfmin_glibc_{k}"] = got["max"], got["min"]
        out[f"ell_{k}"] = real_fit(out[f"rfmax_{k}"], out[f"rfmin_{k}"])
        out[f"prm_{k}"] = np.array([a, e0, f, dmax, rd.params["u"], n1, n2, n3], dtype=np.float64)
        print(k, out[f"rfmax_{k}"].shape, out[f"rfmax_glibc_{k}"].shape)
    import csv
    d = os.path.join(REF, "single_pluse_model")
    with open(os.path.join(d, "all_input.csv")) as fi, open(os.path.join(d, "output_data.csv")) as fo:
        rin = [list(map(float, r)) for r in list(csv.reader(fi))[1:]]
        rout = [list(map(float, r)) for r in list(csv.reader(fo))[1:]]
    rows = sorted({0, 1, 100, 400, 800} | set(np.random.default_rng(0).choice(len(rin), 7, replace=False).tolist()))
    out["pairs_rows"] = np.array(rows)
    out["pairs_in"] = np.array([rin[r] for r in rows])
    out["pairs_out"] = np.array([rout[r] for r in rows])
    np.savez_compressed(os.path.join(OUT, "rd_grid.npz"), ncases=np.array(len(CASES)), **out)


if __name__ == "__main__":
    main()
