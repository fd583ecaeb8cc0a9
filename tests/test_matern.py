"""CPU: the general-smoothness Matern kind (NNGP_COV_MATERN, spNNGP's "matern").

rho(u) = u^nu K_nu(u) / (2^(nu-1) Gamma(nu)), u = phi d.  Three evaluations that share no code:
  * the kernels' (pynngp_amd/csrc/nngp_math.h, host build): Temme's series / the Thompson-Barnett
    continued fraction, scaled so that the small-u limit involves no large exponential;
  * the C oracle's (oracle/nngp_oracle.c): the integral K_nu(u) = int_0^inf e^{-u cosh t} cosh(nu t) dt
    by the trapezoidal rule in long double;
  * the numpy oracle's: scipy.special.kv (AMOS);
all pinned to mpmath (50 digits).  The reference's `cov` is an arbitrary plug-in (nngp.py:6,12);
this kind has no reference output, so its parity is "unpinned by the reference" like every B/F
result, anchored here by mpmath and by the closed forms at nu = 1/2, 3/2, 5/2.
Bounds (absolute, relative to sigma2 = 1 -- the accuracy the factorisation sees):
  kernel <= 2e-15 (measured 1.3e-15 worst over nu in [0.05, 49]); C oracle <= 1e-15 relative;
  scipy <= 2e-13 (AMOS).
"""
import os
import subprocess

import mpmath as mp
import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
NUS = (0.05, 0.2, 0.5, 0.7, 1.0, 1.2, 1.5, 2.0, 2.2, 2.5, 3.7, 5.5, 10.0, 20.3, 49.0)


def _ref(nu, u):
    mp.mp.dps = 50
    if u == 0:
        return mp.mpf(1)
    return mp.mpf(u) ** nu * mp.besselk(nu, u) / (mp.mpf(2) ** (nu - 1) * mp.gamma(nu))


def _grid(seed=3):
    rng = np.random.default_rng(seed)
    pts = []
    for nu in NUS:
        us = list(10 ** rng.uniform(-8, 1.3, 40)) + [1e-150, 1e-30, 1e-3, 1.4999, 1.5, 1.5001, 2.0, 300.0, 700.0]
        pts += [(float(nu), float(u)) for u in us]
    return pts


@pytest.fixture(scope="module")
def kernel_rho(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("matern") / "matern_check")
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-std=c++17", os.path.join(HERE, "host", "matern_check.cpp"),
                    "-o", exe, "-lm"], check=True)

    def run(pairs):
        inp = "\n".join(f"{nu!r} {u!r}" for nu, u in pairs) + "\n"
        out = subprocess.run([exe], input=inp, check=True, capture_output=True, text=True).stdout.split()
        assert len(out) == len(pairs)
        return [float.fromhex(x) for x in out]

    return run


def test_kernel_rho_vs_mpmath(kernel_rho):
    pairs = _grid()
    got = kernel_rho(pairs)
    worst = max(float(abs(g - _ref(nu, u))) for (nu, u), g in zip(pairs, got))
    assert worst <= 2e-15, worst


def test_kernel_rho_closed_forms(kernel_rho):
    """nu = 1/2, 3/2, 5/2 are the exponential, Matern-3/2 and -5/2 kinds: e^-u, (1+u) e^-u,
    (1 + u + u^2/3) e^-u (long double reference)."""
    us = [1e-12, 1e-4, 0.03, 0.4, 1.0, 1.49, 1.51, 3.0, 11.0, 40.0]
    forms = {0.5: lambda u: 1.0, 1.5: lambda u: 1 + u, 2.5: lambda u: 1 + u + u * u / 3}
    for nu, poly in forms.items():
        got = kernel_rho([(nu, u) for u in us])
        for u, g in zip(us, got):
            ul = np.longdouble(u)
            exact = float(poly(ul) * np.exp(-ul))
            assert abs(g - exact) <= 1.5e-15, (nu, u, g, exact)


def test_kernel_rho_limits(kernel_rho):
    """rho(0) = 1 (the limit), rho -> 1 for coincident points (d2 floor 2^-1000), rho = 0 exactly
    past the clamp (far-away padding points decouple), and it decreases in u."""
    got = kernel_rho([(1.7, 0.0), (1.7, 2.0 ** -500), (0.3, 2.0 ** -500), (3.0, 1600.0)])
    assert got[0] == 1.0 and abs(got[1] - 1.0) <= 2e-16 and got[3] == 0.0
    assert abs(got[2] - float(_ref(0.3, 2.0 ** -500))) <= 1e-15
    us = np.linspace(0.001, 30.0, 300).tolist()
    r = kernel_rho([(2.2, u) for u in us])
    assert all(a > b for a, b in zip(r, r[1:]))


@pytest.fixture(scope="module")
def table_rho(tmp_path_factory):
    """The fused pair kernel's Matern-nu path (nngp_matern_tab over the per-launch table), host build."""
    exe = str(tmp_path_factory.mktemp("matern_tab") / "matern_table_check")
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-std=c++17",
                    os.path.join(HERE, "host", "matern_table_check.cpp"), "-o", exe, "-lm"], check=True)

    def run(pairs):
        inp = "\n".join(f"{nu!r} {u!r}" for nu, u in pairs) + "\n"
        out = subprocess.run([exe], input=inp, check=True, capture_output=True, text=True).stdout.split("\n")
        rows = [r.split() for r in out if r.strip()]
        assert len(rows) == len(pairs)
        return [float.fromhex(r[0]) if r[0] != "nan" else float("nan") for r in rows], [int(r[1]) for r in rows]

    return run


TABLE_NUS = tuple(NUS) + (0.45, 1.0000001, 1.97, 2.0, 3.0, 0.05, 0.2, 0.3, 0.44)


def test_table_rho_vs_mpmath(table_rho):
    """Table path (bins of t = u^2: NNGP_MT_K per octave of degree NNGP_MT_NC - 1) against mpmath: the same 2e-15 absolute bound as
    the direct evaluation it is built from, over u from 1e-8 to 20 and at the clamps (u = 0, far)."""
    rng = np.random.default_rng(9)
    worst = 0.0
    for nu in TABLE_NUS:
        us = list(10 ** rng.uniform(-8, 1.3, 60)) + [1e-30, 1e-3, 0.7, 1.0, 1.5, 2.0, 30.0, 300.0]
        got, noct = table_rho([(float(nu), float(u)) for u in us])
        assert all(0 < k <= 160 for k in noct), (nu, noct[0])
        for u, g in zip(us, got):
            worst = max(worst, float(abs(g - _ref(nu, u))))
    assert worst <= 2e-15, worst


def test_table_rho_limits_and_range(table_rho):
    """Coincident points give exactly 1, far points exactly 0 (exact decoupling of padding); nu below the
    table's range (its octaves from 1 - rho < 1e-18 to rho < 1e-18 exceed 160) reports no table (the
    sweep then runs the wavefront kernel); rho decreases along a fine grid."""
    got, noct = table_rho([(1.3, 0.0), (1.3, 1e-200), (1.3, 1e6), (0.7, 0.0), (0.7, 5e3), (0.3, 1.0), (0.05, 1.0),
                           (1.3, 1e160), (0.7, 1e300), (49.0, 1e200)])
    assert got[0] == 1.0 and got[1] == 1.0 and got[2] == 0.0 and got[3] == 1.0 and got[4] == 0.0
    # round 5: small nu has a table too (from t = 2^-64 up; the small-t expansion below it)
    assert 0 < noct[5] <= 160 and 0 < noct[6] <= 160
    assert abs(got[5] - float(_ref(0.3, 1.0))) <= 2e-15 and abs(got[6] - float(_ref(0.05, 1.0))) <= 2e-15
    # u^2 past the double range (a padding point at (m + 1) 1e150 with a large phi): exactly 0, not NaN
    assert got[7] == 0.0 and got[8] == 0.0 and got[9] == 0.0
    us = np.linspace(0.001, 30.0, 400).tolist()
    r, _ = table_rho([(2.2, u) for u in us])
    assert all(a > b for a, b in zip(r, r[1:]))


def test_table_small_nu_below_the_table(table_rho):
    """nu < ~0.45: the table starts at t = 2^-64 and rho = 1 - A t^nu below it (A = Gamma(1 - nu) /
    (4^nu Gamma(1 + nu)); the t and t^(1+nu) terms are under 1e-19 there) -- against mpmath from the
    table's start down to coincident points (u = 0 gives exactly 1)."""
    worst = 0.0
    for nu in (0.02, 0.05, 0.1, 0.2, 0.3, 0.4, 0.44):
        us = [2.0 ** -e for e in (31, 32, 33, 40, 60, 100, 200, 400)] + [2.0 ** -31.9, 1e-12, 1e-100]
        got, noct = table_rho([(nu, u) for u in us] + [(nu, 0.0)])
        assert all(0 < k <= 160 for k in noct)
        # u = 0 (the kernels' floor d^2 = 2^-1000, coincident points): exactly 1 (round 5; 1 - A 2^(-1000 nu)
        # before, 1 - 1e-6 at nu = 0.02)
        assert got[-1] == 1.0
        for u, g in zip(us, got):
            worst = max(worst, float(abs(g - _ref(nu, u))))
    assert worst <= 2e-15, worst


def test_c_oracle_rho_vs_mpmath(c_oracle):
    worst = 0.0
    for nu, u in _grid(5)[::3]:
        ref = _ref(nu, u)
        worst = max(worst, float(abs(c_oracle.c_matern_rho(nu, u) - ref) / max(ref, mp.mpf("1e-280"))))
    assert worst <= 1e-15, worst


def test_scipy_oracle_rho_vs_mpmath(c_oracle):
    for nu in (0.3, 1.0, 1.7, 2.5, 4.2):
        us = np.concatenate([10 ** np.linspace(-9, 1.4, 40), [0.0, 1e-200]])
        r = c_oracle.matern_rho(nu, us)
        for u, g in zip(us, r):
            assert abs(g - float(_ref(nu, u))) <= 2e-13, (nu, u)


@pytest.mark.parametrize("nu,theta", [(0.3, (1.0, 8.0, 0.05)), (1.7, (1.3, 12.0, 0.1)), (4.2, (0.8, 20.0, 0.02))])
def test_c_sweep_vs_numpy_sweep(c_oracle, nu, theta):
    """The two restatements' B / F / log-lik agree (independent K_nu evaluations)."""
    rng = np.random.default_rng(11)
    coords = rng.uniform(0, 1, (400, 2))
    y = rng.standard_normal(400)
    nbr = c_oracle.c_knn_prior(coords, 8)
    th = theta + (nu,)
    Bc, Fc, pc = c_oracle.c_bf_sweep(coords, nbr, "matern", th, y)
    Bn, Fn, pn = c_oracle.bf_sweep(coords, nbr, "matern", th, y)
    assert np.max(np.abs(Fc - Fn) / Fn) <= 1e-9
    assert np.max(np.abs(Bc - Bn)) <= 1e-8
    assert abs(pc[0] - pn[0]) <= 1e-9 * abs(pn[0]) and abs(pc[1] - pn[1]) <= 1e-9 * abs(pn[1])


def test_c_sweep_dense_known_answer(c_oracle):
    """m = N - 1 gives the exact GP log density (numpy dense Cholesky with scipy's K_nu)."""
    rng = np.random.default_rng(4)
    n = 120
    coords = rng.uniform(0, 1, (n, 2))
    y = rng.standard_normal(n)
    th = (1.1, 6.0, 0.2, 1.3)
    nbr = c_oracle.c_knn_prior(coords, n - 1)
    _, _, p = c_oracle.c_bf_sweep(coords, nbr, "matern", th, y)
    ll = c_oracle.loglik_from_partials(p, n)
    assert abs(ll - c_oracle.dense_gp_loglik(coords, "matern", th, y)) <= 1e-9 * abs(ll)


def test_c_sweep_half_integer_nu_equals_closed_kinds(c_oracle):
    rng = np.random.default_rng(9)
    coords = rng.uniform(0, 1, (300, 2))
    y = rng.standard_normal(300)
    nbr = c_oracle.c_knn_prior(coords, 10)
    for nu, kind in ((0.5, "exponential"), (1.5, "matern32"), (2.5, "matern52")):
        th = (1.0, 15.0, 0.1)
        _, F1, p1 = c_oracle.c_bf_sweep(coords, nbr, "matern", th + (nu,), y)
        _, F2, p2 = c_oracle.c_bf_sweep(coords, nbr, kind, th, y)
        assert np.max(np.abs(F1 - F2) / F2) <= 1e-11 and abs(p1[0] - p2[0]) <= 1e-11 * abs(p2[0])


def test_covariance_plugin_matern():
    """pynngp_amd.Covariance("matern", ..., nu) as a plug-in (the reference's cov(a, b)) and its
    argument checks."""
    import torch
    from pynngp_amd import Covariance

    cv = Covariance("matern", 1.5, 4.0, 0.1, nu=1.5)
    a = np.array([[0.0, 0.0], [0.3, 0.1]])
    b = np.array([[0.0, 0.0], [0.2, 0.5], [1.0, 1.0]])
    d = np.sqrt(((a[:, None, :] - b[None, :, :]) ** 2).sum(-1))
    ref = 1.5 * (1 + 4.0 * d) * np.exp(-4.0 * d)
    assert np.allclose(cv(a, b), ref, rtol=1e-13, atol=1e-15)
    assert np.allclose(cv(torch.from_numpy(a), torch.from_numpy(b)).numpy(), ref, rtol=1e-13, atol=1e-15)
    assert cv.nu_arg == 1.5 and Covariance("exponential", 1.0, 2.0).nu_arg is None
    for bad in (None, 0.0, -1.0, 51.0):
        with pytest.raises(ValueError, match="nu"):
            Covariance("matern", 1.0, 2.0, 0.0, nu=bad)
