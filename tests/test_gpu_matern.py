"""GPU parity: the general-smoothness Matern kind (NNGP_COV_MATERN): the pair kernel (m <= 24) and the
four-lane kernel (m = 25..32) evaluating rho from the launch's table for every nu in (0, 50] (below
t = 2^-64 the small-t expansion 1 - A t^nu when nu < 0.9 would need more than 160 octaves), and the
wavefront kernel's direct Bessel evaluation (m > 32, or algo="wave").

Against the C oracle (oracle/nngp_oracle.c: K_nu by a long-double trapezoidal integral, a method
independent of the kernel's Temme series / continued fraction) on the same neighbour sets, with
the tolerances of tests/test_gpu_bf.py (F <= 1e-10 relative, B <= 1e-9 (1 + |B|), log-lik
<= max(1e-12, 1e-15 kappa) relative); the covariance alone (m = 1) against mpmath; nu = 1/2, 3/2,
5/2 against the closed-form kinds' kernels; and the user-facing paths (NNGP.loglik / predict /
fit, ShardedLogLik, SeqNNGP) with a Matern covariance.  Parity unpinned by the reference (its
`cov` is a plug-in; nngp.py:6,12), anchored by mpmath and the closed forms (tests/test_matern.py).
"""
import mpmath as mp
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

RTOL_F = 1e-10
ATOL_B = 1e-9
RTOL_LL = 1e-12


@pytest.fixture(scope="module")
def lib():
    from pynngp_amd import _lib

    return _lib


def _field(n, seed, dim=2):
    rng = np.random.default_rng(seed)
    return rng.uniform(0.0, 1.0, (n, dim)), rng.standard_normal(n)


def _check(dev, lib, O, coords, nbr, theta, nu, y, algo="auto"):
    c = torch.from_numpy(coords).to(dev)
    v = None if y is None else torch.from_numpy(y).to(dev)
    B, F, p = lib.bf_sweep(c, torch.from_numpy(nbr).to(dev), 0, "matern", *theta, values=v, nu=nu, algo=algo)
    Bo, Fo, po = O.c_bf_sweep(coords, nbr, "matern", tuple(theta) + (nu,), y)
    B, F, p = B.cpu().numpy(), F.cpu().numpy(), p.cpu().numpy()
    assert p[2] == -1 and p[3] == -1
    assert np.all(np.abs(F - Fo) <= RTOL_F * Fo), np.max(np.abs(F - Fo) / Fo)
    assert np.all(np.abs(B - Bo) <= ATOL_B * (1 + np.abs(Bo))), np.max(np.abs(B - Bo))
    assert np.all(B[nbr < 0] == 0.0)
    ll, llo = O.loglik_from_partials(p, nbr.shape[0]), O.loglik_from_partials(po, nbr.shape[0])
    kappa = float(np.max((theta[0] + theta[2]) / Fo))
    assert abs(ll - llo) <= max(RTOL_LL, 1e-15 * kappa) * abs(llo), (ll, llo, kappa)


@pytest.mark.parametrize("nu,theta,m,dim", [
    (0.3, (1.0, 20.0, 0.0), 15, 2),
    (0.5, (1.2, 10.0, 0.05), 10, 2),
    (1.0, (1.0, 15.0, 0.1), 15, 2),
    (1.7, (0.9, 12.0, 0.1), 12, 2),
    (2.5, (1.0, 20.0, 0.1), 15, 2),
    (4.2, (1.5, 25.0, 0.2), 8, 2),
    (0.8, (1.0, 6.0, 0.05), 10, 1),
    (1.3, (1.0, 10.0, 0.1), 15, 3),
    (2.2, (1.0, 18.0, 0.1), 40, 2),  # the NR = 64 instantiation
    (11.0, (1.0, 60.0, 0.3), 5, 2),
    (0.45, (1.0, 15.0, 0.05), 15, 2),
    (0.05, (1.0, 10.0, 0.1), 15, 2),  # small nu: the table from 2^-64 (round 5; the wavefront kernel before)
    (0.2, (1.0, 30.0, 0.05), 24, 2),
    (0.3, (1.0, 20.0, 0.1), 28, 2),  # m = 25..32: the four-lane kernel with the table
    (1.7, (1.0, 12.0, 0.1), 32, 3),
    (6.0, (1.0, 40.0, 0.1), 26, 1),
    (35.0, (1.0, 80.0, 0.1), 20, 2),
    (1.0, (1.0, 12.0, 0.1), 24, 3),
    (1.3, (1.0, 10.0, 0.1), 18, 2),  # m = 18: the left-looking Matern kernel (round 6), every dimension
    (0.7, (1.0, 8.0, 0.05), 18, 1),
    (2.9, (1.0, 14.0, 0.05), 18, 3),
    (0.3, (1.0, 20.0, 0.1), 19, 2),  # (m = 19: right-looking again)
])
@pytest.mark.parametrize("algo", ["auto", "wave"])
def test_matern_sweep_vs_oracle(lib, dev, c_oracle, nu, theta, m, dim, algo):
    coords, y = _field(2000, 21 + m, dim)
    nbr = c_oracle.c_knn_prior(coords, m)
    _check(dev, lib, c_oracle, coords, nbr, theta, nu, y, algo)


@pytest.mark.parametrize("m,phi,nu", [(15, 2000.0, 1.3), (24, 2000.0, 2.5), (15, 900.0, 0.6), (24, 5000.0, 10.0)])
def test_matern_large_phi_padding_rows(lib, dev, c_oracle, m, phi, nu):
    """advice r04: a padding point at (a + 1) 1e150 gives d2 ~ (m + 1)^2 1e300, and d2 phi^2 overflowed to
    inf once phi > ~1.3e4 / (m + 1): the table lookup then read out of range and padded rows (the first m
    rows) got NaN.  The argument is clamped past the table: exact zeros, finite B / F, oracle parity."""
    coords, y = _field(1500, 31 + m)
    nbr = c_oracle.c_knn_prior(coords, m)
    assert lib.resolve_algo("auto", m, "matern", 2, nu=nu) == "pairb"
    _check(dev, lib, c_oracle, coords, nbr, (1.0, phi, 0.1), nu, y)


def test_matern_deferred_finalize_wrong_algo(lib, dev, c_oracle):
    """advice r04: a deferred sweep on the wavefront kernel finalised as the pair kernel's records: the fold
    refuses the foreign header (NaN partials), never reads past the workspace; with the algo that ran it is
    the in-line fold's result"""
    coords, y = _field(3000, 77)
    nbr = torch.from_numpy(c_oracle.c_knn_prior(coords, 15)).to(dev)
    c, v = torch.from_numpy(coords).to(dev), torch.from_numpy(y).to(dev)
    ws = lib.bf_workspace(3000, 15, "auto", dev, kind="matern")
    lib.bf_sweep(c, nbr, 0, "matern", 1.0, 20.0, 0.1, values=v, nu=0.3, workspace=ws, defer=True, algo="wave")
    bad = lib.bf_finalize(ws, 3000, 15, "matern", 2, algo="pairb").cpu().numpy()
    assert np.isnan(bad[0]) and np.isnan(bad[1])
    good = lib.bf_finalize(ws, 3000, 15, "matern", 2, algo="wave")
    _, _, ref = lib.bf_sweep(c, nbr, 0, "matern", 1.0, 20.0, 0.1, values=v, nu=0.3, algo="wave")
    assert torch.equal(good, ref)


def test_matern_kernel_choice_and_explicit(lib, dev):
    """auto: the pair kernel with the table for m <= 24, the four-lane kernel with it for 25..32 (every nu),
    the wavefront kernel above; the kernels agree within the parity tolerances; lane is refused."""
    for nu in (0.05, 0.3, 1.2, 49.0):
        assert lib.resolve_algo("auto", 15, "matern", 2, nu=nu) == "pairb"
        assert lib.resolve_algo("auto", 28, "matern", 2, nu=nu) == "quad"
        assert lib.resolve_algo("auto", 40, "matern", 2, nu=nu) == "wave"
    coords, y = _field(5000, 2)
    c = torch.from_numpy(coords).to(dev)
    v = torch.from_numpy(y).to(dev)
    nb = lib.knn_prior(c, 10)
    Bw, Fw, pw = lib.bf_sweep(c, nb, 0, "matern", 1.0, 10.0, 0.1, values=v, nu=1.2, algo="wave")
    Ba, Fa, pa = lib.bf_sweep(c, nb, 0, "matern", 1.0, 10.0, 0.1, values=v, nu=1.2)
    Bp, Fp, pp = lib.bf_sweep(c, nb, 0, "matern", 1.0, 10.0, 0.1, values=v, nu=1.2, algo="pairb")
    assert torch.equal(Ba, Bp) and torch.equal(Fa, Fp) and torch.equal(pa, pp)
    assert torch.all((Fa - Fw).abs() <= RTOL_F * Fw) and torch.all((Ba - Bw).abs() <= ATOL_B * (1 + Bw.abs()))
    assert abs(pa[1].item() - pw[1].item()) <= 1e-11 * abs(pw[1].item())
    with pytest.raises(lib.NNGPExtensionError, match="pair \\(m <= 24\\)"):
        lib.bf_sweep(c, nb, 0, "matern", 1.0, 10.0, 0.1, nu=1.2, algo="lane")
    nb28 = lib.knn_prior(c, 28)
    Bq, Fq, pq = lib.bf_sweep(c, nb28, 0, "matern", 1.0, 10.0, 0.1, values=v, nu=0.3)
    Bw, Fw, pw = lib.bf_sweep(c, nb28, 0, "matern", 1.0, 10.0, 0.1, values=v, nu=0.3, algo="wave")
    assert torch.all((Fq - Fw).abs() <= RTOL_F * Fw) and torch.all((Bq - Bw).abs() <= ATOL_B * (1 + Bw.abs()))
    assert abs(pq[1].item() - pw[1].item()) <= 1e-11 * abs(pw[1].item())
    with pytest.raises(ValueError, match="nu"):
        lib.bf_sweep(c, nb, 0, "matern", 1.0, 10.0, 0.1)


def test_matern_m1_covariance_vs_mpmath(lib, dev, c_oracle):
    """m = 1 isolates the device covariance: B_i = C(d_i) / (sigma2 + tau2) (auto: through the table)."""
    coords, _ = _field(4000, 7)
    nbr = c_oracle.c_knn_prior(coords, 1)
    sigma2, phi, tau2 = 1.3, 9.0, 0.4
    c = torch.from_numpy(coords).to(dev)
    mp.mp.dps = 40
    for nu, algo in ((0.05, "auto"), (0.2, "auto"), (0.4, "auto"), (0.6, "auto"), (1.0, "auto"), (2.3, "auto"),
                     (7.5, "auto"), (42.0, "auto"), (0.2, "wave"), (1.0, "wave"), (7.5, "wave")):
        B, _, p = lib.bf_sweep(c, torch.from_numpy(nbr).to(dev), 0, "matern", sigma2, phi, tau2, nu=nu, algo=algo)
        cov = B.cpu().numpy()[1:, 0] * (sigma2 + tau2)
        j = nbr[1:, 0]
        d2 = (coords[1:, 0] - coords[j, 0]) ** 2 + (coords[1:, 1] - coords[j, 1]) ** 2
        for k in range(0, len(d2), 37):
            u = phi * mp.sqrt(mp.mpf(float(d2[k])))
            ref = sigma2 * u ** nu * mp.besselk(nu, u) / (mp.mpf(2) ** (nu - 1) * mp.gamma(nu))
            assert abs(cov[k] - float(ref)) <= 4e-15 * sigma2, (nu, k, cov[k], float(ref))


@pytest.mark.parametrize("nu", [0.01, 0.05, 0.2, 0.4])
def test_matern_small_nu_near_coincident_points(lib, dev, nu):
    """Small nu below the table: points 1e-30 .. 1e-9 apart (t < 2^-64 with phi = 9) and exact duplicates
    take rho = 1 - A t^nu; the covariance against mpmath (m = 1), the pair and four-lane kernels."""
    rng = np.random.default_rng(40)
    base = rng.uniform(0, 1, (500, 2))
    off = rng.standard_normal((500, 2)) * (10.0 ** rng.uniform(-30, -9, 500))[:, None]
    off[::50] = 0.0  # exact duplicates
    coords = np.empty((1000, 2))
    coords[0::2], coords[1::2] = base, base + off
    nbr = np.full((1000, 1), -1, np.int32)
    nbr[1::2, 0] = np.arange(0, 1000, 2)
    nbr[2::2, 0] = np.arange(1, 999, 2)  # the previous pair's second point (an ordinary distance)
    sigma2, phi, tau2 = 1.0, 9.0, 0.5
    c = torch.from_numpy(coords).to(dev)
    B, _, _ = lib.bf_sweep(c, torch.from_numpy(nbr).to(dev), 0, "matern", sigma2, phi, tau2, nu=nu)
    cov = B.cpu().numpy()[:, 0] * (sigma2 + tau2)
    mp.mp.dps = 50
    for i in range(1, 1000):
        j = nbr[i, 0]
        d = mp.sqrt(mp.mpf(float(coords[i, 0] - coords[j, 0])) ** 2 + mp.mpf(float(coords[i, 1] - coords[j, 1])) ** 2)
        if d == 0:
            ref = mp.mpf(sigma2)
        else:
            u = phi * d
            ref = sigma2 * u ** nu * mp.besselk(nu, u) / (mp.mpf(2) ** (nu - 1) * mp.gamma(nu))
        assert abs(cov[i] - float(ref)) <= 4e-15 * sigma2, (nu, i, cov[i], float(ref))


@pytest.mark.parametrize("nu,kind", [(0.5, "exponential"), (1.5, "matern32"), (2.5, "matern52")])
def test_matern_half_integer_equals_closed_kind(lib, dev, c_oracle, nu, kind):
    """The general kernel at nu = 1/2, 3/2, 5/2 equals the closed-form kinds' fast kernels."""
    coords, y = _field(20000, 3)
    c = torch.from_numpy(coords).to(dev)
    v = torch.from_numpy(y).to(dev)
    nb = lib.knn_prior(c, 15)
    th = (1.0, 20.0, 0.1)
    _, F1, p1 = lib.bf_sweep(c, nb, 0, "matern", *th, values=v, nu=nu)
    _, F2, p2 = lib.bf_sweep(c, nb, 0, kind, *th, values=v)
    F1, F2 = F1.cpu().numpy(), F2.cpu().numpy()
    assert np.max(np.abs(F1 - F2) / F2) <= 1e-10
    ll1, ll2 = c_oracle.loglik_from_partials(p1.cpu().numpy(), 20000), c_oracle.loglik_from_partials(p2.cpu().numpy(), 20000)
    assert abs(ll1 - ll2) <= 1e-11 * abs(ll2)


def test_matern_bit_reproducible(lib, dev):
    coords, y = _field(30000, 5)
    c = torch.from_numpy(coords).to(dev)
    v = torch.from_numpy(y).to(dev)
    nb = lib.knn_prior(c, 15)
    r1 = lib.bf_sweep(c, nb, 0, "matern", 1.0, 25.0, 0.0, values=v, nu=0.9)
    r2 = lib.bf_sweep(c, nb, 0, "matern", 1.0, 25.0, 0.0, values=v, nu=0.9)
    assert all(torch.equal(a, b) for a, b in zip(r1, r2))


def test_matern_nngp_class_paths(dev, c_oracle):
    """NNGP(cov=Covariance("matern", ..., nu)): per-location methods, loglik, predict at t not in
    S (nngp_bf_cross), fit with nu held fixed; ShardedLogLik; a few SeqNNGP iterations."""
    from pynngp_amd import NNGP, Covariance, SeqNNGP
    from pynngp_amd.sweep import ShardedLogLik

    rng = np.random.default_rng(8)
    n = 1500
    t = rng.uniform(0, 1, (n, 2))
    y = rng.standard_normal(n)
    cv = Covariance("matern", 1.0, 9.0, 0.1, nu=1.3)
    g = NNGP(t, y, None, "S=T", 10, cv, device=dev)
    nbr = g.nbr.cpu().numpy()
    th = (1.0, 9.0, 0.1, 1.3)
    _, Fo, po = c_oracle.c_bf_sweep(t, nbr, "matern", th, y)
    assert abs(g.loglik() - c_oracle.loglik_from_partials(po, n)) <= 1e-11 * abs(c_oracle.loglik_from_partials(po, n))
    i = 700
    Bi, Fi = c_oracle.bf_location(t, nbr[i], i, "matern", th)
    assert np.allclose(g._Bsi(i), Bi, rtol=1e-9, atol=1e-12) and abs(g._Fsi(i) - Fi) <= 1e-10 * Fi
    CN, c, Cii = c_oracle.location_blocks(t, nbr[i], i, "matern", th)
    assert np.allclose(g._CNs(i), CN, rtol=1e-12, atol=1e-14) and np.allclose(g._Ccross(i), c, rtol=1e-12, atol=1e-14)

    q = rng.uniform(0, 1, (300, 2))
    mean, F_t = g.predict(values=y, query=q)
    nq = c_oracle.knn_all(q, t, 10).astype(np.int32)
    Bx, Fx, _ = c_oracle.c_bf_cross(t, q, nq, "matern", th, ref_values=y)
    assert np.all(np.abs(F_t - Fx) <= 1e-10 * Fx)
    mean_o = np.einsum("ij,ij->i", Bx, y[nq])
    assert np.allclose(mean, mean_o, rtol=1e-9, atol=1e-11)

    sw = ShardedLogLik(torch.from_numpy(t).to(dev), 10)
    ll_s = sw.loglik(cv, torch.from_numpy(y).to(dev))
    assert abs(ll_s - g.loglik()) <= 1e-12 * abs(ll_s)

    res = g.fit(fix_tau2=0.1, maxiter=60)
    assert g.cov.kind == "matern" and g.cov.nu == 1.3 and np.isfinite(res["loglik"])

    smp = SeqNNGP(t, y, m=10, kind="matern", nu=1.3, sigma2=1.0, tau2=0.1, phi=9.0, seed=1, device=dev)
    for _ in range(5):
        smp.step()
    assert np.isfinite(smp.sigma2) and np.isfinite(smp.tau2) and np.isfinite(smp.phi)
    assert torch.isfinite(smp.w).all()
