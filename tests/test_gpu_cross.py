"""GPU parity: B_t / F_t of points outside the reference set (nngp_bf_cross) and the
refType tuple / Nt / predict surface of the drop-in class.

The reference builds ``Nt = KDTree(s).query(t, m)`` (pyNNGP/nngp.py:64-71) but never
evaluates B_t / F_t, and its tuple refTypes crash (``self.typ``, nngp.py:34): parity
is against the oracle restatement (oracle.nngp_oracle.c_bf_cross, pinned to the dense
GP conditional in tests/test_oracle.py), "parity unpinned" w.r.t. the reference.
Tolerances as tests/test_gpu_bf.py: F rel 1e-10, B abs 1e-9 (1 + |B|).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

RTOL_F = 1e-10
ATOL_B = 1e-9


@pytest.fixture(scope="module")
def lib():
    from pynngp_amd import _lib

    return _lib


def _sets(n_ref, n_query, seed, dup=50):
    rng = np.random.default_rng(seed)
    ref = rng.uniform(0, 1, (n_ref, 2))
    query = rng.uniform(-0.05, 1.05, (n_query, 2))
    query[:dup] = ref[rng.integers(0, n_ref, dup)]  # query points that coincide with reference points
    return ref, query, rng.standard_normal(n_ref), rng.standard_normal(n_query)


@pytest.mark.parametrize("m,algo", [(1, "lane"), (5, "lane"), (10, "pairb"), (15, "pairb"), (28, "quad"), (20, "auto"),
                                    (15, "auto"), (20, "pairb"), (24, "wave"), (15, "wave")])
@pytest.mark.parametrize("kind,theta", [("exponential", (1.0, 20.0, 0.1)), ("matern32", (1.4, 12.0, 0.05))])
def test_bf_cross_vs_oracle(lib, dev, c_oracle, m, algo, kind, theta):
    ref, query, vr, vq = _sets(3000, 700, m)
    nbr = c_oracle.knn_all(query, ref, m).astype(np.int32)
    g = lambda a: torch.from_numpy(a).to(dev)  # noqa: E731
    R = torch.empty(len(query), dtype=torch.float64, device=dev)
    B, F, p = lib.bf_cross(g(ref), g(query), g(nbr), kind, *theta, ref_values=g(vr), query_values=g(vq),
                           algo=algo, R=R)
    Bo, Fo, po = c_oracle.c_bf_cross(ref, query, nbr, kind, theta, vr, vq)
    B, F, p, R = B.cpu().numpy(), F.cpu().numpy(), p.cpu().numpy(), R.cpu().numpy()
    assert p[2] == -1 and p[3] == -1
    assert np.all(np.abs(F - Fo) <= RTOL_F * Fo), np.max(np.abs(F - Fo) / Fo)
    assert np.all(np.abs(B - Bo) <= ATOL_B * (1 + np.abs(Bo))), np.max(np.abs(B - Bo))
    wn = vr[nbr]
    np.testing.assert_allclose(R, vq - (Bo * wn).sum(1), rtol=0, atol=1e-9)
    ll, llo = c_oracle.loglik_from_partials(p, len(query)), c_oracle.loglik_from_partials(po, len(query))
    assert abs(ll - llo) <= 1e-11 * abs(llo)


@pytest.mark.parametrize("n_ref,algo", [(20, "pairb"), (16, "lane"), (40, "wave")])
def test_bf_cross_dense_kriging(lib, dev, c_oracle, n_ref, algo):
    """m = |S|: B_t, F_t and the kriging mean equal the exact GP conditional."""
    ref, query, vr, _ = _sets(n_ref, 300, 5, dup=0)
    theta = (1.2, 3.0, 0.02)
    nbr = c_oracle.knn_all(query, ref, n_ref).astype(np.int32)
    g = lambda a: torch.from_numpy(a).to(dev)  # noqa: E731
    R = torch.empty(len(query), dtype=torch.float64, device=dev)
    B, F, _ = lib.bf_cross(g(ref), g(query), g(nbr), "exponential", *theta, ref_values=g(vr), algo=algo, R=R)
    Bd, Fd, mean = c_oracle.dense_kriging(ref, query, "exponential", theta, vr)
    Bk = np.zeros_like(Bd)
    np.put_along_axis(Bk, nbr.astype(np.int64), B.cpu().numpy(), axis=1)
    np.testing.assert_allclose(F.cpu().numpy(), Fd, rtol=1e-9, atol=0)
    np.testing.assert_allclose(Bk, Bd, rtol=0, atol=1e-8)
    np.testing.assert_allclose(-R.cpu().numpy(), mean, rtol=0, atol=1e-8)


def test_bf_cross_row_order_and_ranges(lib, dev, c_oracle):
    ref, query, vr, vq = _sets(5000, 4000, 9)
    m = 15
    nbr = lib.knn_query(torch.from_numpy(ref).to(dev), torch.from_numpy(query).to(dev), m)
    np.testing.assert_array_equal(nbr.cpu().numpy(), c_oracle.knn_all(query, ref, m))
    g = lambda a: torch.from_numpy(a).to(dev)  # noqa: E731
    B1, F1, _ = lib.bf_cross(g(ref), g(query), nbr, "exponential", 1.0, 30.0, 0.1, ref_values=g(vr))
    order, srt = lib.row_order(g(query), 0, len(query), nbr)
    B2, F2, _ = lib.bf_cross(g(ref), g(query), srt, "exponential", 1.0, 30.0, 0.1, ref_values=g(vr), order=order)
    assert torch.equal(B1, B2) and torch.equal(F1, F2)
    B3, F3, _ = lib.bf_cross(g(ref), g(query), nbr[1000:2500], "exponential", 1.0, 30.0, 0.1, q0=1000)
    assert torch.equal(B3, B1[1000:2500]) and torch.equal(F3, F1[1000:2500])
    # zero-variance interpolation is flagged, not silently returned: tau2 = 0 at a coincident point
    _, _, p = lib.bf_cross(g(ref), g(query), nbr, "exponential", 1.0, 30.0, 0.0)
    assert p[2].item() >= 0
    with pytest.raises(Exception):
        lib.bf_cross(g(ref), g(query), nbr[:10], "exponential", 1.0, 30.0, 0.1, q0=len(query) - 5)


def test_nngp_subset_reftype_nt_predict(dev, c_oracle):
    from pynngp_amd import NNGP, Covariance
    from pynngp_amd.nngp import reference_set

    rng = np.random.default_rng(3)
    t = rng.uniform(0, 1, (3000, 2))
    y = np.sin(6 * t[:, 0]) + 0.1 * rng.standard_normal(3000)
    np.random.seed(11)
    s_expected = t[np.random.choice(len(t), size=800)]
    np.random.seed(11)
    cov = Covariance("exponential", 1.0, 10.0, 0.05)
    g = NNGP(t, y, np.full(3000, 0.1), ("subset", 800), 10, cov, device=dev)
    np.testing.assert_array_equal(g.s, s_expected)
    assert g.Ns[0] == [] and len(g.Ns) == 800
    np.testing.assert_array_equal(np.stack(g.Ns[10:]), c_oracle.c_knn_prior(g.s, 10)[10:])
    Nt = g.Nt
    assert len(Nt) == 3000 and Nt is not g.Ns
    np.testing.assert_array_equal(np.stack(Nt), c_oracle.knn_all(t, g.s, 10))
    np.testing.assert_allclose(g.ws, c_oracle.ws_init(t, y, g.s), rtol=0, atol=1e-12)
    mean, var = g.predict()
    Bo, Fo, _ = c_oracle.c_bf_cross(g.s, t, np.stack(Nt).astype(np.int32), "exponential", cov.theta, g.ws)
    np.testing.assert_allclose(var, Fo, rtol=RTOL_F)
    np.testing.assert_allclose(mean, (Bo * g.ws[np.stack(Nt)]).sum(1), rtol=0, atol=1e-9)
    # the same draw the reference's calls make (nngp.py:36-37)
    np.random.seed(11)
    np.testing.assert_array_equal(reference_set(t, ("subset", 800)), s_expected)


def test_nngp_random_reftype(dev, c_oracle):
    from pynngp_amd import NNGP, Covariance

    rng = np.random.default_rng(4)
    t = rng.uniform(0, 1, (1000, 2))
    y = rng.standard_normal(1000)
    np.random.seed(2)
    s_expected = np.vstack([np.random.uniform(lo, hi, 400) for lo, hi in ((0, 1), (0.2, 0.8))]).T
    np.random.seed(2)
    g = NNGP(t, y, None, ("random", 400, ((0, 1), (0.2, 0.8))), 8, Covariance("matern32", 1.0, 8.0, 0.1),
             device=dev)
    np.testing.assert_array_equal(g.s, s_expected)
    np.testing.assert_array_equal(np.stack(g.Nt), c_oracle.knn_all(t, g.s, 8))
    mean, var = g.predict(values=np.zeros(400))
    assert np.all(mean == 0) and np.all((var > 0) & (var <= 1.1 + 1e-12))
    # explicit query points
    q = rng.uniform(0, 1, (50, 2))
    mean_q, var_q = g.predict(values=g.ws, query=q)
    nbr = c_oracle.knn_all(q, g.s, 8).astype(np.int32)
    Bo, Fo, _ = c_oracle.c_bf_cross(g.s, q, nbr, "matern32", (1.0, 8.0, 0.1), g.ws)
    np.testing.assert_allclose(var_q, Fo, rtol=RTOL_F)


def test_bf_cross_op_registered(dev, c_oracle):
    from pynngp_amd import load_ops

    ops = load_ops()

    ref, query, vr, _ = _sets(500, 200, 1)
    g = lambda a: torch.from_numpy(a).to(dev)  # noqa: E731
    nbr = torch.ops.nngp.knn_query(g(ref), g(query), 12)
    B, F, mean = torch.ops.nngp.bf_cross(g(ref), g(query), nbr, ops.kind_code("exponential"), 1.0, 9.0, 0.1,
                                         g(vr), ops.algo_code("auto"))
    Bo, Fo, _ = c_oracle.c_bf_cross(ref, query, nbr.cpu().numpy(), "exponential", (1.0, 9.0, 0.1), vr)
    np.testing.assert_allclose(F.cpu().numpy(), Fo, rtol=RTOL_F)
    np.testing.assert_allclose(mean.cpu().numpy(), (Bo * vr[nbr.cpu().numpy()]).sum(1), rtol=0, atol=1e-9)
