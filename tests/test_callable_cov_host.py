"""CPU tests of the reference-style covariance plug-in ``cov(a, b)`` (pyNNGP/nngp.py:6,12, called
on coordinate rows at :82, :96): the oracle's per-location dense-solve path and the host logic of
``CallableCovariance`` (joint-block gathering, evaluation-mode probing, packing), which is plain
torch and runs on CPU tensors here.  The GPU factorisation of the blocks is tested in
tests/test_gpu_callable_cov.py."""
import numpy as np
import pytest
import torch

from oracle import nngp_oracle as O


def _aniso(s2, A):
    """Anisotropic exponential s2 exp(-sqrt((a-b)^T A (a-b))) -- broadcasting over leading dims."""
    A = np.asarray(A, dtype=np.float64)

    def cov(a, b):
        lib = torch if isinstance(a, torch.Tensor) else np
        t = a[..., :, None, :] - b[..., None, :, :]
        q = A[0, 0] * t[..., 0] ** 2 + 2.0 * A[0, 1] * t[..., 0] * t[..., 1] + A[1, 1] * t[..., 1] ** 2
        return s2 * lib.exp(-lib.sqrt(q))

    return cov


def _loop_only(s2, phi):
    """A plug-in written for 2-D row sets only (no batch dimension), as a reference user would."""
    def cov(a, b):
        a = np.asarray(a).reshape(-1, np.asarray(a).shape[-1])
        b = np.asarray(b).reshape(-1, np.asarray(b).shape[-1])
        d = np.sqrt(((a[:, None, :] - b[None, :, :]) ** 2).sum(-1))
        return s2 * np.exp(-phi * d)

    return cov


def _iso_exp(s2, phi, tau2=0.0):
    def cov(a, b):
        d = np.sqrt(O.rdist(a[:, None, :] - b[None, :, :]))
        c = s2 * np.exp(-phi * d)
        return c + tau2 * (d == 0)

    return cov


def test_oracle_callable_equals_builtin_kind():
    rng = np.random.default_rng(4)
    x = rng.uniform(size=(400, 2))
    y = rng.standard_normal(400)
    nbr = O.knn_prior(x, 8)
    B1, F1, p1 = O.bf_sweep(x, nbr, "exponential", (1.3, 9.0, 0.0), y)
    B2, F2, p2 = O.bf_sweep_callable(x, nbr, _iso_exp(1.3, 9.0), y)
    np.testing.assert_allclose(F2, F1, rtol=1e-12)
    np.testing.assert_allclose(B2, B1, rtol=0, atol=1e-11)
    assert abs(O.loglik_from_partials(p2, 400) - O.loglik_from_partials(p1, 400)) <= 1e-12 * abs(
        O.loglik_from_partials(p1, 400))


def test_oracle_callable_dense_gp_known_answer():
    """m = N - 1: the NNGP density is the exact GP density for any covariance."""
    rng = np.random.default_rng(5)
    n = 60
    x = rng.uniform(size=(n, 2))
    y = rng.standard_normal(n)
    cov = _aniso(1.7, [[30.0, 8.0], [8.0, 6.0]])
    nbr = O.knn_prior(x, n - 1)
    C = cov(x, x) + 0.05 * np.eye(n)  # a nugget keeps the dense matrix well conditioned
    nug = lambda a, b: cov(a, b) + 0.05 * (np.sqrt(O.rdist(a[:, None, :] - b[None, :, :])) == 0)  # noqa: E731
    _, _, p = O.bf_sweep_callable(x, nbr, nug, y)
    L = np.linalg.cholesky(C)
    z = np.linalg.solve(L, y)
    dense = -0.5 * (n * O.LOG_2PI + 2 * np.log(np.diag(L)).sum() + z @ z)
    assert abs(O.loglik_from_partials(p, n) - dense) <= 1e-11 * abs(dense)


def test_joint_points_and_blocks_layout():
    from pynngp_amd.nngp import CallableCovariance, joint_points

    rng = np.random.default_rng(6)
    x = torch.from_numpy(rng.uniform(size=(50, 2)))
    nbr = torch.from_numpy(O.knn_prior(x.numpy(), 5))
    X = joint_points(x, nbr)
    assert X.shape == (50, 6, 2)
    assert torch.equal(X[:, 5], x)
    assert torch.equal(X[10, :5], x[nbr[10].long()])
    assert torch.equal(X[2, 2], x[2]) and torch.equal(X[0, 0], x[0])  # slots without a point repeat the location
    cov = _aniso(1.1, [[20.0, 3.0], [3.0, 9.0]])
    cc = CallableCovariance(cov, tau2=0.25)
    blk = cc.blocks(x, nbr)
    assert cc.mode == "torch"
    assert blk.shape == (21, 50)
    t = 17
    C = cov(X[t].numpy(), X[t].numpy()) + 0.25 * np.eye(6)
    for a in range(6):
        for b in range(a + 1):
            assert blk[a * (a + 1) // 2 + b, t].item() == pytest.approx(C[a, b], rel=1e-14, abs=1e-300)


@pytest.mark.parametrize("which,mode", [("aniso", "torch"), ("loop", "loop")])
def test_mode_probe(which, mode):
    from pynngp_amd.nngp import CallableCovariance, joint_points

    rng = np.random.default_rng(7)
    x = torch.from_numpy(rng.uniform(size=(40, 2)))
    nbr = torch.from_numpy(O.knn_prior(x.numpy(), 4))
    fn = _aniso(1.0, [[9.0, 0.0], [0.0, 4.0]]) if which == "aniso" else _loop_only(1.0, 5.0)
    cc = CallableCovariance(fn)
    blk = cc.blocks(x, nbr)
    assert cc.mode == mode
    X = joint_points(x, nbr).numpy()
    ref = np.stack([np.asarray(fn(X[t], X[t])) for t in range(40)])
    a = np.repeat(np.arange(5), np.arange(1, 6))
    b = np.concatenate([np.arange(k + 1) for k in range(5)])
    np.testing.assert_allclose(blk.numpy(), ref[:, a, b].T, rtol=1e-13, atol=0)


def test_numpy_batched_mode_and_forced_mode():
    from pynngp_amd.nngp import CallableCovariance

    def np_only(a, b):  # numpy-only, but broadcasting over a leading batch dimension
        a, b = np.asarray(a), np.asarray(b)
        d = np.sqrt(((a[..., :, None, :] - b[..., None, :, :]) ** 2).sum(-1))
        return np.exp(-3.0 * d)

    rng = np.random.default_rng(8)
    x = torch.from_numpy(rng.uniform(size=(30, 2)))
    nbr = torch.from_numpy(O.knn_prior(x.numpy(), 3))
    cc = CallableCovariance(np_only)
    b1 = cc.blocks(x, nbr)
    assert cc.mode == "numpy"
    b2 = CallableCovariance(np_only, batch="loop").blocks(x, nbr)
    np.testing.assert_allclose(b1.numpy(), b2.numpy(), rtol=1e-15, atol=0)
    with pytest.raises(ValueError):
        CallableCovariance(np_only, batch="gpu")
    with pytest.raises(TypeError):
        CallableCovariance(3.0)


def test_bad_plugin_raises():
    from pynngp_amd.nngp import CallableCovariance

    x = torch.rand(20, 2, dtype=torch.float64)
    nbr = torch.from_numpy(O.knn_prior(x.numpy(), 3))
    with pytest.raises(TypeError, match="failed"):
        CallableCovariance(lambda a, b: 1 / 0).blocks(x, nbr)
    with pytest.raises(ValueError, match="finite"):
        CallableCovariance(lambda a, b: np.full((np.asarray(a).shape[-2], np.asarray(b).shape[-2]), np.nan)).blocks(
            x, nbr)
