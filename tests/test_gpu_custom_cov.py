"""GPU parity: a covariance of the caller's own (IsotropicCovariance; nngp_joint_dist ->
fn -> nngp_bf_sweep_blocks, the bf_pairb kernel reading the joint blocks from memory).

The reference's `cov` is an arbitrary plug-in (pyNNGP/nngp.py:6,12) with no output of its own,
so this is parity "unpinned by the reference", anchored by:
  * the built-in kinds: fn = the kind's formula in torch gives the fused kernels' B / F / log-lik
    (F <= 1e-10 relative, B <= 1e-9 (1 + |B|), log-lik <= 1e-12 relative -- the two paths
    evaluate distance and exp differently, in the last bits);
  * a kind with no fused kernel (powered exponential) against numpy per-location Cholesky
    solves with the same function;
  * the dense GP log density at m = N - 1 and the dense kriging conditional at m = |S|;
  * exact decoupling of slots without a point, the visiting order, bad-index flags.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lib():
    from pynngp_amd import _lib

    return _lib


def _field(n, seed, dim=2):
    rng = np.random.default_rng(seed)
    return rng.uniform(0.0, 1.0, (n, dim)), rng.standard_normal(n)


def _powexp(s2, phi, alpha):
    return lambda d: s2 * torch.exp(-((phi * d) ** alpha))


def _sweep(lib, cov, c, nb, v=None, order=None):
    from pynngp_amd.nngp import _sweep_any

    return _sweep_any(cov, c, nb, 0, values=v, qvalues=v, order=order)


@pytest.mark.parametrize("kind,theta,m", [("exponential", (1.0, 20.0, 0.1), 15), ("matern32", (1.3, 12.0, 0.05), 10),
                                          ("gaussian", (0.9, 8.0, 0.2), 20), ("exponential", (1.0, 30.0, 0.0), 24),
                                          ("spherical", (1.1, 6.0, 0.1), 5), ("matern32", (1.0, 15.0, 0.05), 18),
                                          ("exponential", (1.2, 25.0, 0.1), 21), ("gaussian", (1.0, 6.0, 0.3), 23)])
def test_custom_equals_builtin_kind(lib, dev, c_oracle, kind, theta, m):
    from pynngp_amd import Covariance, IsotropicCovariance

    s2, phi, tau2 = theta
    fns = {"exponential": lambda d: s2 * torch.exp(-phi * d),
           "matern32": lambda d: s2 * (1 + phi * d) * torch.exp(-phi * d),
           "gaussian": lambda d: s2 * torch.exp(-(phi * d) ** 2),
           "spherical": lambda d: torch.where(phi * d < 1, s2 * (1 - 1.5 * phi * d + 0.5 * (phi * d) ** 3),
                                              torch.zeros_like(d))}
    coords, y = _field(20000, 3 + m)
    c = torch.from_numpy(coords).to(dev)
    v = torch.from_numpy(y).to(dev)
    nb = lib.knn_prior(c, m)
    B1, F1, p1 = _sweep(lib, IsotropicCovariance(fns[kind], tau2), c, nb, v)
    B2, F2, p2 = _sweep(lib, Covariance(kind, s2, phi, tau2), c, nb, v)
    B1, F1, B2, F2 = (t.cpu().numpy() for t in (B1, F1, B2, F2))
    p1, p2 = p1.cpu().numpy(), p2.cpu().numpy()
    assert p1[2] == -1 and p1[3] == -1
    assert np.max(np.abs(F1 - F2) / F2) <= 1e-10
    assert np.max(np.abs(B1 - B2) / (1 + np.abs(B2))) <= 1e-9
    assert np.all(B1[nb.cpu().numpy() < 0] == 0.0)
    ll1, ll2 = c_oracle.loglik_from_partials(p1, 20000), c_oracle.loglik_from_partials(p2, 20000)
    kappa = float(np.max((s2 + tau2) / F2))
    assert abs(ll1 - ll2) <= max(1e-12, 1e-15 * kappa) * abs(ll2), (ll1, ll2, kappa)


def _np_location(coords, nbr_row, i, f, tau2):
    idx = nbr_row[nbr_row >= 0].astype(np.int64)
    xs = coords[idx]
    d = np.sqrt(((xs[:, None, :] - xs[None, :, :]) ** 2).sum(-1))
    CN = f(d) + tau2 * np.eye(idx.size)
    c = f(np.sqrt(((coords[i][None, :] - xs) ** 2).sum(-1)))
    Bv = np.linalg.solve(CN, c)
    return Bv, f(np.zeros(1))[0] + tau2 - c @ Bv


@pytest.mark.parametrize("dim", [1, 2, 3])
def test_custom_powered_exponential_vs_numpy(lib, dev, dim):
    """A covariance no fused kernel has: B / F on sampled rows against numpy solves."""
    from pynngp_amd import IsotropicCovariance

    s2, phi, alpha, tau2 = 1.2, 9.0, 1.5, 0.1
    coords, y = _field(5000, 11, dim)
    c = torch.from_numpy(coords).to(dev)
    nb = lib.knn_prior(c, 12)
    B, F, p = _sweep(lib, IsotropicCovariance(_powexp(s2, phi, alpha), tau2), c, nb)
    B, F, nbh = B.cpu().numpy(), F.cpu().numpy(), nb.cpu().numpy()
    f = lambda d: s2 * np.exp(-((phi * d) ** alpha))  # noqa: E731
    for i in list(range(0, 14)) + list(range(100, 5000, 97)):
        Bo, Fo = _np_location(coords, nbh[i], i, f, tau2)
        k = Bo.size
        assert abs(F[i] - Fo) <= 1e-10 * Fo, (i, F[i], Fo)
        assert np.allclose(B[i, :k], Bo, rtol=0, atol=1e-9 * (1 + np.abs(Bo).max(initial=0.0)))
        assert np.all(B[i, k:] == 0.0)


def test_custom_dense_known_answers(lib, dev):
    """m = N - 1: the dense GP log density; prediction at m = |S|: the dense kriging conditional."""
    from pynngp_amd import NNGP, IsotropicCovariance

    rng = np.random.default_rng(5)
    n = 24
    t = rng.uniform(0, 1, (n, 2))
    y = rng.standard_normal(n)
    s2, phi, alpha, tau2 = 1.0, 4.0, 1.2, 0.05
    cov = IsotropicCovariance(_powexp(s2, phi, alpha), tau2)
    g = NNGP(t, y, None, "S=T", n - 1, cov, device=dev)
    f = lambda d: s2 * np.exp(-((phi * d) ** alpha))  # noqa: E731
    D = np.sqrt(((t[:, None, :] - t[None, :, :]) ** 2).sum(-1))
    C = f(D) + tau2 * np.eye(n)
    L = np.linalg.cholesky(C)
    z = np.linalg.solve(L, y)
    ll_dense = -0.5 * (n * np.log(2 * np.pi) + 2 * np.log(np.diag(L)).sum() + z @ z)
    assert abs(g.loglik() - ll_dense) <= 1e-11 * abs(ll_dense)
    q = rng.uniform(0, 1, (40, 2))
    g2 = NNGP(t, y, None, "S=T", n, cov, device=dev)  # predict from all of S
    mean, var = g2.predict(values=y, query=q)
    Cqs = f(np.sqrt(((q[:, None, :] - t[None, :, :]) ** 2).sum(-1)))
    W = np.linalg.solve(C, Cqs.T).T
    assert np.allclose(mean, W @ y, rtol=1e-9, atol=1e-11)
    assert np.allclose(var, s2 + tau2 - np.einsum("ij,ij->i", W, Cqs), rtol=1e-9, atol=1e-12)


def test_custom_order_bad_index_and_limits(lib, dev):
    from pynngp_amd import IsotropicCovariance

    cov = IsotropicCovariance(_powexp(1.0, 15.0, 1.0), 0.1)
    coords, y = _field(30000, 8)
    c = torch.from_numpy(coords).to(dev)
    v = torch.from_numpy(y).to(dev)
    nb = lib.knn_prior(c, 15)
    order, srt = lib.row_order(c, 0, 30000, nb)
    B1, F1, p1 = _sweep(lib, cov, c, nb, v)
    B2, F2, p2 = _sweep(lib, cov, c, srt, v, order=order)
    assert torch.equal(B1, B2) and torch.equal(F1, F2) and torch.allclose(p1[:2], p2[:2], rtol=1e-13, atol=0)
    # bit-reproducible
    B3, F3, p3 = _sweep(lib, cov, c, nb, v)
    assert torch.equal(B1, B3) and torch.equal(F1, F3) and torch.equal(p1, p3)
    # an invalid index in a middle row is flagged
    bad = nb.clone()
    bad[777, 3] = -2
    _, _, pb = _sweep(lib, cov, c, bad, v)
    assert pb[3].item() == 777.0
    # m past the blocks kernels (the two-lane kernel serves 1..24, the four-lane kernel 25..32)
    nb33 = lib.knn_prior(c[:2000], 33)
    with pytest.raises(ValueError, match="m <= 32"):
        _sweep(lib, cov, c[:2000], nb33)
    with pytest.raises(lib.NNGPExtensionError, match="m <= 32"):
        lib.bf_sweep_blocks(torch.zeros((34 * 35 // 2, 2000), dtype=torch.float64, device=dev), nb33, 2000)


def test_matern_elementwise_and_custom_matern(lib, dev, c_oracle):
    """_lib.matern (nngp_matern_eval) against mpmath, and IsotropicCovariance over it against the
    fused Matern-nu kind (the wavefront kernel)."""
    import mpmath as mp

    from pynngp_amd import Covariance, IsotropicCovariance

    mp.mp.dps = 40
    u = torch.tensor([0.0, 1e-9, 1e-3, 0.2, 1.0, 1.4999, 1.5001, 3.0, 40.0, 900.0, float("inf")], dtype=torch.float64,
                     device=dev)
    for nu in (0.3, 1.3, 4.7):
        r = lib.matern(u, nu).cpu().numpy()
        for x, g in zip(u.cpu().tolist(), r):
            ref = 1.0 if x == 0 else (0.0 if x == float("inf") else
                                      float(mp.mpf(x) ** nu * mp.besselk(nu, x) / (mp.mpf(2) ** (nu - 1) * mp.gamma(nu))))
            assert abs(g - ref) <= 2e-15, (nu, x, g, ref)
    coords, y = _field(20000, 4)
    c = torch.from_numpy(coords).to(dev)
    v = torch.from_numpy(y).to(dev)
    nb = lib.knn_prior(c, 15)
    s2, phi, tau2, nu = 1.1, 25.0, 0.1, 1.3
    cust = IsotropicCovariance(lambda d: s2 * lib.matern(phi * d, nu), tau2)
    _, F1, p1 = _sweep(lib, cust, c, nb, v)
    _, F2, p2 = _sweep(lib, Covariance("matern", s2, phi, tau2, nu=nu), c, nb, v)
    F1, F2 = F1.cpu().numpy(), F2.cpu().numpy()
    assert np.max(np.abs(F1 - F2) / F2) <= 1e-10
    ll1, ll2 = c_oracle.loglik_from_partials(p1.cpu().numpy(), 20000), c_oracle.loglik_from_partials(p2.cpu().numpy(), 20000)
    assert abs(ll1 - ll2) <= 1e-12 * abs(ll2)


def test_isotropic_gpu_only_fn_predict_m0_and_onesample(lib, dev):
    """An IsotropicCovariance built on the GPU-only Matern correlation (_lib.matern): C(0) is evaluated on
    the device (the m = 0 prediction variance is C(0) + tau2), and oneSample -- whose phi proposals need a
    fused kind -- refuses it with a TypeError instead of failing inside the sampler."""
    from pynngp_amd import NNGP, IsotropicCovariance

    rng = np.random.default_rng(5)
    t = rng.uniform(size=(300, 2))
    y = rng.standard_normal(300)
    cv = IsotropicCovariance(lambda d: 1.3 * lib.matern(9.0 * d, 1.2), tau2=0.1)
    assert abs(cv.sigma2 - 1.3) <= 1e-15
    g0 = NNGP(t, y, None, "S=T", 0, cv)
    mean, var = g0.predict(values=y, query=rng.uniform(size=(20, 2)))
    assert np.all(mean == 0.0) and np.allclose(var, 1.4, rtol=1e-15, atol=0)
    g = NNGP(t, y, None, "S=T", 8, cv)
    with pytest.raises(TypeError, match="built-in covariance"):
        g.oneSample()
