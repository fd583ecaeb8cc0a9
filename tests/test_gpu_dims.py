"""GPU parity for ordinates of dimension 1 and 3 (and 2 where the same code runs).

The reference's neighbour search is dimension-agnostic (a sklearn KDTree over s[0:i],
pyNNGP/nngp.py:55-61; ('random', nRef, bounds) takes one (lo, hi) per dimension,
nngp.py:26-27,38-40).  Checked here against the reference's own output in 1-D and 3-D
(tests/golden/knn_ref_n1000_m10_d3.npz, knn_ref_n1000_m8_d1.npz, made by
tests/golden/make_golden.py dims) and against the C oracle (sklearn's rdist summed in axis
order, unfused; ties by lower index): neighbour sets bit-exact; B / F / log-lik at the
tolerances of tests/test_gpu_bf.py for every covariance kind; the Z-order visiting order
and the cross-set kernel in 1-D and 3-D; FMA-sensitive near-ties in 3-D.
"""
import numpy as np
import pytest
import torch

from conftest import load_golden

pytestmark = pytest.mark.gpu

RTOL_F = 1e-10
ATOL_B = 1e-9
KINDS = [("exponential", (1.0, 12.0, 0.0)), ("matern32", (1.2, 9.0, 0.1)), ("matern52", (1.0, 8.0, 0.1)),
         ("gaussian", (1.0, 4.0, 0.2)), ("spherical", (0.9, 3.0, 0.05))]


@pytest.fixture(scope="module")
def lib():
    from pynngp_amd import _lib

    return _lib


def _field(n, dim, seed):
    rng = np.random.default_rng(seed)
    return rng.uniform(0.0, 1.0, (n, dim)), rng.standard_normal(n)


def _check_bf(dev, lib, O, coords, nbr, kind, theta, y, algo):
    c = torch.from_numpy(coords).to(dev)
    B, F, p = lib.bf_sweep(c, torch.from_numpy(nbr).to(dev), 0, kind, *theta, values=torch.from_numpy(y).to(dev),
                           algo=algo)
    Bo, Fo, po = O.c_bf_sweep(coords, nbr, kind, theta, y)
    B, F, p = B.cpu().numpy(), F.cpu().numpy(), p.cpu().numpy()
    assert p[2] == -1 and p[3] == -1 and po[2] == -1
    assert np.all(np.abs(F - Fo) <= RTOL_F * Fo), np.max(np.abs(F - Fo) / Fo)
    assert np.all(np.abs(B - Bo) <= ATOL_B * (1 + np.abs(Bo))), np.max(np.abs(B - Bo))
    n = nbr.shape[0]
    ll, llo = O.loglik_from_partials(p, n), O.loglik_from_partials(po, n)
    kappa = float(np.max((theta[0] + theta[2]) / Fo))
    assert abs(ll - llo) <= max(1e-12, 1e-15 * kappa) * abs(llo), (ll, llo)


@pytest.mark.parametrize("name", ["knn_ref_n1000_m10_d3", "knn_ref_n1000_m8_d1"])
def test_knn_matches_reference_fixture_dims(lib, dev, c_oracle, name):
    g = load_golden(name)
    m = int(g["m"])
    got = lib.knn_prior(torch.from_numpy(g["coords"]).to(dev), m).cpu().numpy()
    np.testing.assert_array_equal(got[~g["tie_rows"]], g["Ns"][~g["tie_rows"]])
    np.testing.assert_array_equal(got, c_oracle.c_knn_prior(g["coords"], m))


@pytest.mark.parametrize("dim", [1, 3])
@pytest.mark.parametrize("n,m", [(30000, 15), (5000, 24), (3000, 1), (2000, 40)])
def test_knn_dims_vs_oracle(lib, dev, c_oracle, dim, n, m):
    coords, _ = _field(n, dim, 10 * dim + m)
    coords[100:120] = coords[7]  # exact duplicates: ties by lower index
    got = lib.knn_prior(torch.from_numpy(coords).to(dev), m).cpu().numpy()
    np.testing.assert_array_equal(got, c_oracle.c_knn_prior(coords, m))
    # a row range and a row list of the same sets
    rows = np.random.default_rng(dim).integers(0, n, 500).astype(np.int32)
    c = torch.from_numpy(coords).to(dev)
    q0, q1 = n // 3, n // 2
    np.testing.assert_array_equal(lib.knn_prior(c, m, q0, q1).cpu().numpy(), got[q0:q1])
    np.testing.assert_array_equal(lib.knn_prior_rows(c, m, torch.from_numpy(rows).to(dev)).cpu().numpy(), got[rows])


@pytest.mark.parametrize("dim", [1, 3])
def test_knn_query_dims(lib, dev, c_oracle, dim):
    rng = np.random.default_rng(dim)
    ref, qry = rng.uniform(size=(4000, dim)), rng.uniform(size=(700, dim))
    got = lib.knn_query(torch.from_numpy(ref).to(dev), torch.from_numpy(qry).to(dev), 12).cpu().numpy()
    np.testing.assert_array_equal(got, c_oracle.knn_all(qry, ref, 12))


def test_knn_fma_sensitive_ties_3d(lib, dev, c_oracle):
    from fma_ties import fma_sensitive_clusters

    coords, expect = fma_sensitive_clusters(2000, dim=3, seed=5)
    got = lib.knn_prior(torch.from_numpy(coords).to(dev), 1).cpu().numpy()
    np.testing.assert_array_equal(c_oracle.c_knn_prior(coords, 1)[2::3, 0], expect)
    np.testing.assert_array_equal(got[2::3, 0], expect)


@pytest.mark.parametrize("dim", [1, 3])
@pytest.mark.parametrize("kind,theta", KINDS)
@pytest.mark.parametrize("algo,m", [("auto", 15), ("pairb", 10), ("wave", 15), ("auto", 30)])
def test_bf_dims_vs_oracle(lib, dev, c_oracle, dim, kind, theta, algo, m):
    coords, y = _field(4000, dim, 7 * dim + m)
    nbr = c_oracle.c_knn_prior(coords, m)
    _check_bf(dev, lib, c_oracle, coords, nbr, kind, theta, y, algo)


@pytest.mark.parametrize("dim", [1, 3])
def test_bf_dims_dense_gp_known_answer(lib, dev, c_oracle, dim):
    """m = N-1: the NNGP density is the exact GP density, in 1-D and 3-D."""
    n = 60
    coords, y = _field(n, dim, 90 + dim)
    nbr = c_oracle.c_knn_prior(coords, n - 1)
    for kind, theta in KINDS:
        _, _, p = lib.bf_sweep(torch.from_numpy(coords).to(dev), torch.from_numpy(nbr).to(dev), 0, kind, *theta,
                               values=torch.from_numpy(y).to(dev))
        ll = c_oracle.loglik_from_partials(p.cpu().numpy(), n)
        dense = c_oracle.dense_gp_loglik(coords, kind, theta, y)
        assert abs(ll - dense) <= 1e-9 * abs(dense), (kind, ll, dense)


@pytest.mark.parametrize("dim", [1, 3])
def test_row_order_and_cross_dims(lib, dev, c_oracle, dim):
    coords, y = _field(20000, dim, 50 + dim)
    c = torch.from_numpy(coords).to(dev)
    v = torch.from_numpy(y).to(dev)
    nb = lib.knn_prior(c, 12)
    order, srt = lib.row_order(c, 0, 20000, nb)
    oh = order.cpu().numpy()
    assert np.array_equal(np.sort(oh), np.arange(20000))
    B1, F1, _ = lib.bf_sweep(c, nb, 0, "matern52", 1.0, 9.0, 0.1, values=v)
    B2, F2, _ = lib.bf_sweep(c, srt, 0, "matern52", 1.0, 9.0, 0.1, values=v, order=order)
    assert torch.equal(B1, B2) and torch.equal(F1, F2)
    # Z-order is spatially coherent in any dimension
    step = np.linalg.norm(np.diff(coords[oh], axis=0), axis=1)
    assert np.median(step) < np.median(np.linalg.norm(np.diff(coords, axis=0), axis=1)) / 4
    # cross-set B_t / F_t at off-reference points
    qry = np.random.default_rng(dim).uniform(size=(3000, dim))
    q = torch.from_numpy(qry).to(dev)
    nbq = lib.knn_query(c, q, 12)
    R = torch.empty(3000, dtype=torch.float64, device=dev)
    Bq, Fq, _ = lib.bf_cross(c, q, nbq, "gaussian", 1.0, 4.0, 0.2, ref_values=v, R=R)
    Bo, Fo, _ = c_oracle.c_bf_cross(coords, qry, nbq.cpu().numpy(), "gaussian", (1.0, 4.0, 0.2), y)
    assert np.all(np.abs(Fq.cpu().numpy() - Fo) <= RTOL_F * Fo)
    assert np.all(np.abs(Bq.cpu().numpy() - Bo) <= ATOL_B * (1 + np.abs(Bo)))


def test_nngp_class_3d_and_random_reference_set(dev, c_oracle):
    """The drop-in class with 3-D ordinates, S = T and ('random', nRef, bounds) with three
    (lo, hi) pairs (nngp.py:26-27,38-40: one np.random.uniform column per bound)."""
    from pynngp_amd import NNGP, Covariance

    rng = np.random.default_rng(4)
    t = rng.uniform(0.0, 1.0, (3000, 3))
    y = rng.standard_normal(3000)
    cov = Covariance("exponential", 1.0, 8.0, 0.1)
    model = NNGP(t, y, np.full(3000, 0.1), "S=T", 10, cov)
    np.testing.assert_array_equal(model.nbr.cpu().numpy(), c_oracle.c_knn_prior(t, 10))
    assert model.Ns[0] == [] and np.array_equal(model.Ns[5], c_oracle.c_knn_prior(t, 10, 5, 6)[0, :5])
    ll = model.loglik()
    _, _, po = c_oracle.c_bf_sweep(t, c_oracle.c_knn_prior(t, 10), "exponential", cov.theta, y)
    assert abs(ll - c_oracle.loglik_from_partials(po, 3000)) <= 1e-12 * abs(ll)
    np.random.seed(11)
    model = NNGP(t, y, None, ("random", 800, ((0, 1), (0, 1), (0, 1))), 10, cov)
    np.random.seed(11)
    s = np.vstack([np.random.uniform(lo, hi, 800) for lo, hi in ((0, 1), (0, 1), (0, 1))]).T
    np.testing.assert_array_equal(model.s, s)
    assert model.Nt[0].shape == (10,)
    np.testing.assert_array_equal(np.stack(model.Nt), c_oracle.knn_all(t, s, 10))
    mean, var = model.predict()
    assert mean.shape == (3000,) and np.all(var > 0)
