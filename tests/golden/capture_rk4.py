#!/usr/bin/env python3
"""Capture golden vectors for the RK4 two-body + J2 propagator
(build container ONLY; reads /root/reference read-only).

The reference script 轨道外推-龙格库塔算法.py runs a plot pipeline at module
level that needs a CSV which is not in the repository, so only its constants
(mu, Re, J2) and its two functions StateEq / RungeKutta (lines 9-39) are
extracted with `ast` and executed -- nothing else of the module runs.

Fixture rk4_j2.npz:
  rv0      [n][6]  initial states (km, km/s): the script's own RV0
                   (:44) plus seeded LEO/MEO/GEO/inclined draws
  h        [m]     step sizes (s)
  steps    [m]     number of RungeKutta steps per case
  rv       [m][n][6] states after `steps` applications of RungeKutta(t, rv, h)
  f0       [n][6]  StateEq(0, rv0)

Run:  python tests/golden/capture_rk4.py
"""
import ast
import os

import numpy as np

REF = "/root/reference/轨道外推-龙格库塔算法.py"
OUT = os.path.dirname(os.path.abspath(__file__))


def load_functions():
    src = open(REF, encoding="utf-8").read()
    tree = ast.parse(src)
    keep = []
    for node in tree.body:
        if isinstance(node, ast.Assign) and all(isinstance(t, ast.Name) and t.id in ("mu", "Re", "J2")
                                                for t in node.targets):
            keep.append(node)
        elif isinstance(node, ast.FunctionDef) and node.name in ("StateEq", "RungeKutta"):
            keep.append(node)
    mod = ast.Module(body=keep, type_ignores=[])
    ns = {"np": np}
    exec(compile(mod, REF, "exec"), ns)
    assert {"StateEq", "RungeKutta", "mu", "Re", "J2"} <= set(ns), sorted(ns)
    return ns


def main():
    ns = load_functions()
    rng = np.random.default_rng(2024)
    rv0 = [np.array([3971.676026, -2202.172866, -5161.178823, 6.059801, 3.231769, 3.293050])]   # script :44
    for a, inc in ((6878.0, 0.9), (7200.0, 1.7), (26560.0, 0.96), (42164.0, 0.001), (42164.0, 0.3)):
        for _ in range(3):
            u, raan = rng.uniform(0, 2 * np.pi, 2)
            r = np.array([np.cos(u), np.sin(u) * np.cos(inc), np.sin(u) * np.sin(inc)]) * a
            v_dir = np.array([-np.sin(u), np.cos(u) * np.cos(inc), np.cos(u) * np.sin(inc)])
            v = v_dir * np.sqrt(398600 / a) * rng.uniform(0.97, 1.03)
            rot = np.array([[np.cos(raan), -np.sin(raan), 0], [np.sin(raan), np.cos(raan), 0], [0, 0, 1]])
            rv0.append(np.concatenate([rot @ r, rot @ v]))
    rv0 = np.array(rv0)
    f0 = np.array([ns["StateEq"](0, x) for x in rv0])
    hs = [1, 10, 0.5]
    steps = [600, 200, 100]
    out = []
    for h, n in zip(hs, steps):
        res = []
        for x in rv0:
            y = x.copy()
            for i in range(n):
                y = ns["RungeKutta"](i * h, y, h)
            res.append(y)
        out.append(res)
    np.savez_compressed(os.path.join(OUT, "rk4_j2.npz"), rv0=rv0, h=np.array(hs, dtype=np.float64),
                        steps=np.array(steps, dtype=np.int32), rv=np.array(out), f0=f0)
    print("rk4_j2.npz:", rv0.shape, np.array(out).shape)


if __name__ == "__main__":
    main()
