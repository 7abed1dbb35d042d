"""Test configuration: markers, import paths, golden-fixture loader.

`-m "not gpu"` runs on any CPU host (oracle vs golden vectors, host logic,
C-ABI symbol checks, gloo multi-process tests).  `-m gpu` runs the parity
tests proper on an MI355X, through the product's C-ABI library.
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "ppo-rl-satellite_amd")
ORACLE_DIR = os.path.join(ROOT, "oracle")
GOLDEN_DIR = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG_DIR, ORACLE_DIR):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI library)")


def golden(name):
    return np.load(os.path.join(GOLDEN_DIR, name + ".npz"))


@pytest.fixture(scope="session")
def oracle():
    import oracle as O
    O.build()
    return O


TRAJ_NAMES = ["traj_uniform_f0", "traj_wide_f0", "traj_chase_f0", "traj_uniform_f1", "traj_chase_f1"]
STATE_KEYS = ["Pp", "Pv", "Ep", "Ev", "fuel_c", "fuel_t", "dis", "dz", "fuel_c_mode", "fuel_t_mode", "vel_int", "flag"]
