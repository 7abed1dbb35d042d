"""Reachable-domain grid on the MI355X.

satenv_reachable_domain (RD_single_pulse.py:40-148) through the C-ABI vs the
C oracle on the same grids and vs the reference's own point lists
(tests/golden/rd_grid.npz).  The kernel uses OCML transcendentals, so the
reachability test can flip on a direction that sits on the boundary
tan(alpha)^2 == temp1 (none of the cases below has one); reachable points
agree to 1e-9 relative (the hybrd iterate is at an extremum of rf in alpha,
so ulp-level differences in the solve stay second order in rf).
"""
import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu
RTOL = 1e-9


@pytest.fixture(scope="module")
def rd():
    from satrl import reachable
    return reachable


def _compare_grid(got_mx, got_mn, got_st, mx, mn, st, what):
    assert np.array_equal(got_st, st), (what, np.argwhere(got_st != st)[:8])
    keep = st == 1
    for g, r in ((got_mx[keep], mx[keep]), (got_mn[keep], mn[keep])):
        assert np.array_equal(np.isnan(g), np.isnan(r)), what
        ok = ~np.isnan(r)
        np.testing.assert_allclose(g[ok], r[ok], rtol=RTOL, atol=1e-6, err_msg=what)


def test_rd_grid_vs_golden_and_oracle(rd, oracle):
    g = golden("rd_grid")
    for k in range(int(g["ncases"])):
        a, e0, f, dm, u, n1, n2, n3 = g[f"prm_{k}"]
        n1, n2, n3 = int(n1), int(n2), int(n3)
        mx, mn = rd.reachable_domain(a, e0, f, dm, n1, n2, n3, u, device="cuda:0")
        mx, mn = mx.cpu().numpy(), mn.cpu().numpy()
        for name, got in (("max", mx), ("min", mn)):
            ref = g[f"rf{name}_{k}"]
            assert got.shape == ref.shape, (k, name)
            assert np.array_equal(np.isnan(got), np.isnan(ref))
            ok = ~np.isnan(ref)
            np.testing.assert_allclose(got[ok], ref[ok], rtol=RTOL, atol=1e-6, err_msg=f"case {k} {name}")
        orbits = rd.orbits_tensor(a, e0, f, dm, u, device="cuda:0")
        gm, gn, gs = (t[0].cpu().numpy() for t in rd.reachable_domain_grid(orbits, n1, n2, n3))
        _compare_grid(gm, gn, gs, *oracle.reachable_domain_grid(a, e0, f, dm, n1, n2, n3, u), what=f"case {k}")


def test_rd_batch_matches_single_orbits_bitwise(rd):
    rng = np.random.default_rng(7)
    n = 24
    a = rng.uniform(7e6, 5e7, n)
    e0 = rng.uniform(0.0, 0.8, n)
    f = rng.uniform(0.05, 2 * np.pi - 0.05, n)
    dm = rng.uniform(50.0, 1000.0, n)
    orbits = rd.orbits_tensor(a, e0, f, dm, device="cuda:0")
    bm, bn, bs = rd.reachable_domain_grid(orbits, 2, 48, 64)
    for s in (0, 5, 23):
        one = rd.orbits_tensor(a[s], e0[s], f[s], dm[s], device="cuda:0")
        sm, sn, ss = rd.reachable_domain_grid(one, 2, 48, 64)
        assert torch.equal(ss[0], bs[s]) and torch.equal(sm[0], bm[s]) and torch.equal(sn[0], bn[s]), s


def test_rd_random_orbits_vs_oracle(rd, oracle):
    rng = np.random.default_rng(11)
    n = 32
    a = rng.uniform(7e6, 5e7, n)
    e0 = rng.uniform(0.0, 0.8, n)
    f = rng.uniform(0.05, 2 * np.pi - 0.05, n)
    dm = rng.uniform(50.0, 1000.0, n)
    n1, n2, n3 = 2, 60, 80
    orbits = rd.orbits_tensor(a, e0, f, dm, device="cuda:0")
    gm, gn, gs = (t.cpu().numpy() for t in rd.reachable_domain_grid(orbits, n1, n2, n3))
    flips = 0
    for s in range(n):
        mx, mn, st = oracle.reachable_domain_grid(a[s], e0[s], f[s], dm[s], n1, n2, n3)
        flips += int((gs[s] != st).sum())
        both = (gs[s] == 1) & (st == 1)
        np.testing.assert_allclose(gm[s][both], mx[both], rtol=RTOL, atol=1e-6)
        np.testing.assert_allclose(gn[s][both], mn[both], rtol=RTOL, atol=1e-6)
    assert flips <= 2, flips      # libm-boundary directions only


def test_rd_theta_branch_gap_reported(rd, oracle):
    """f = 0: the direction gama = 2 pi, alpha = 0 falls outside both theta
    branches (RD_single_pulse.py:87-90); status 2 like the oracle, and the
    list API refuses instead of reusing a stale theta."""
    orbits = rd.orbits_tensor(1e7, 0.2, 0.0, 500.0, device="cuda:0")
    _, _, st = rd.reachable_domain_grid(orbits, 1, 40, 40)
    _, _, ost = oracle.reachable_domain_grid(1e7, 0.2, 0.0, 500.0, 1, 40, 40)
    assert np.array_equal(st[0].cpu().numpy(), ost)
    with pytest.raises(ValueError):
        rd.reachable_domain(1e7, 0.2, 0.0, 500.0, 1, 40, 40, device="cuda:0")
