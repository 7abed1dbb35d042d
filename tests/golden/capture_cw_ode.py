#!/usr/bin/env python3
"""Capture golden vectors for the reference's numerical CW propagator
(build container ONLY; reads /root/reference read-only).

satellite_function.Numerical_calculation_method (satellite_function.py:
783-839): the CW equations of orbit_ode (omega from r = 35786 km, J2 = 0,
Tmax = 0) integrated by scipy's solve_ivp RK45 (rtol 1e-3, atol 1e-6) over
(0, t) with t_eval = arange(0, t + 50, 50); the state after the step is the
dense-output value at t_eval[-1] (solution.y[:, -1]).  environment.py:
124-128 holds the (commented-out) call with t = 600; the env steps 100 s.

Only satellite_function is imported (numpy/scipy/sympy; no gym needed).
Each case runs the reference class itself for the two craft, and
solve_ivp(orbit_ode, ...) once more for the function-evaluation count.

Fixture cw_ode.npz:
  x0    [n][6]     initial states (m, m/s): the reset state, states along
                   the recorded Flag-0/1 trajectories, seeded draws
  t     [m]        propagation intervals (100, 600, 50, 1000)
  out   [m][n][6]  solution.y[:, -1]
  nfev  [m][n]     solve_ivp's function evaluations (2 + 6 per attempted step)

Run:  python tests/golden/capture_cw_ode.py
"""
import os
import sys

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def main():
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    import satellite_function as sf
    from scipy.integrate import solve_ivp

    x0 = [np.array([200000.0, 0, 0, 0, 0, 0]), np.array([18000.0, 0, 0, 0, 0, 0])]
    for name in ("traj_chase_f0", "traj_uniform_f1", "traj_wide_f0"):
        d = np.load(os.path.join(OUT, name + ".npz"))
        for k in range(0, d["b_Pp"].shape[0], 97):
            x0.append(np.concatenate([d["b_Pp"][k], d["b_Pv"][k]]))
            x0.append(np.concatenate([d["b_Ep"][k], d["b_Ev"][k]]))
    rng = np.random.default_rng(783)
    for _ in range(40):
        x0.append(np.concatenate([rng.uniform(-3e5, 3e5, 3), rng.uniform(-30, 30, 3)]))
    x0.append(np.array([1.0, 0, 0, 0, 0, 0]))          # tiny: the d0 < 1e-5 initial-step branch is near
    x0.append(np.zeros(6))                              # all zero: h0 = 1e-6, error 0 -> MAX_FACTOR steps
    x0.append(np.array([0, 0, 5e4, 0, 0, 3.0]))         # out-of-plane only
    x0 = np.array(x0, dtype=np.float64)
    ts = np.array([100.0, 600.0, 50.0, 1000.0])
    n, m = x0.shape[0], ts.shape[0]
    out = np.zeros((m, n, 6))
    nfev = np.zeros((m, n), dtype=np.int64)
    extra = (0, [1, 1])                                  # numerical_calculation's (Tmax, direction)
    for a, t in enumerate(ts):
        tt = float(t) if float(t) != int(t) else int(t)
        for i in range(0, n, 2):
            j = min(i + 1, n - 1)
            nm = sf.Numerical_calculation_method(R0_c=x0[i][:3], V0_c=x0[i][3:], R0_t=x0[j][:3], V0_t=x0[j][3:])
            s_c, s_t = nm.numerical_calculation(tt)
            out[a, i] = s_c
            out[a, j] = s_t
        for i in range(n):
            t_eval = np.arange(0, tt + 50, 50)
            sol = solve_ivp(sf.Numerical_calculation_method.orbit_ode, (0, tt), x0[i], args=extra,
                            method="RK45", t_eval=t_eval)
            assert np.array_equal(sol.y[:, -1], out[a, i]), (t, i)
            nfev[a, i] = sol.nfev
    np.savez_compressed(os.path.join(OUT, "cw_ode.npz"), x0=x0, t=ts, out=out, nfev=nfev)
    print("cw_ode.npz:", n, "states x", m, "intervals; nfev range", nfev.min(), nfev.max())


if __name__ == "__main__":
    main()
