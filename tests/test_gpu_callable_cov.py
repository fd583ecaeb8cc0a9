"""GPU parity: the reference's own covariance plug-in ``cov(a, b)`` (pyNNGP/nngp.py:6,12, called on
coordinate rows at :82, :96) driving B / F / the log-likelihood on the device
(CallableCovariance: joint blocks fn(X, X) -> nngp_bf_sweep_blocks; the two-lane blocked kernel for
m <= 24, the four-lane kernel for 25..32).

Oracle: ``oracle.nngp_oracle.bf_sweep_callable`` -- the same plug-in called as the reference calls
it (C_N = cov(X_N, X_N), c = cov(x_i, X_N), C_ii = cov(x_i, x_i)) and one dense solve per location.
Parity is unpinned by the reference (its _Bsi / _Fsi are stubs); the tolerances are DESIGN.md 2's:
F <= 1e-10 relative, B <= 1e-9 (1 + |B|), log-lik <= 1e-12 relative.
"""
import numpy as np
import pytest
import torch

from oracle import nngp_oracle as O

pytestmark = pytest.mark.gpu


def _aniso(s2, A, tau2=0.0):
    """Anisotropic exponential s2 exp(-sqrt((a-b)^T A (a-b))) (+ tau2 where a == b) -- a covariance
    no built-in kind or isotropic function expresses; broadcasts over leading dimensions in numpy
    and in torch."""
    A = np.asarray(A, dtype=np.float64)

    def cov(a, b):
        lib = torch if isinstance(a, torch.Tensor) else np
        t = a[..., :, None, :] - b[..., None, :, :]
        q = A[0, 0] * t[..., 0] ** 2 + 2.0 * A[0, 1] * t[..., 0] * t[..., 1] + A[1, 1] * t[..., 1] ** 2
        c = s2 * lib.exp(-lib.sqrt(q))
        # (a bool tensor times a Python float is float32 in torch: cast, or the nugget is rounded to fp32 --
        # which the evaluation probe caught, 5e-10 relative against the numpy plug-in, refusing the torch mode)
        z = (q == 0).to(c.dtype) if lib is torch else (q == 0)
        return c + tau2 * z if tau2 else c

    return cov


def _np_only(s2, A, tau2=0.0):
    """The same covariance in numpy only (host evaluation)."""
    f = _aniso(s2, A, tau2)
    return lambda a, b: f(np.asarray(a), np.asarray(b))


def _loop_only(s2, A, tau2=0.0):
    """... and written for 2-D row sets only, as a reference user would (one call per location)."""
    A = np.asarray(A, dtype=np.float64)

    def cov(a, b):
        a, b = np.atleast_2d(np.asarray(a)), np.atleast_2d(np.asarray(b))
        out = np.empty((a.shape[0], b.shape[0]))
        for k in range(a.shape[0]):
            t = b - a[k]
            q = np.einsum("ij,jk,ik->i", t, A, t)
            out[k] = s2 * np.exp(-np.sqrt(q)) + tau2 * (q == 0)
        return out

    return cov


A1 = [[400.0, 150.0], [150.0, 100.0]]


def _check(B, F, p, Bo, Fo, po, n):
    np.testing.assert_allclose(F.cpu().numpy(), Fo, rtol=1e-10, atol=0)
    Bg = B.cpu().numpy()
    assert np.all(np.abs(Bg - Bo) <= 1e-9 * (1 + np.abs(Bo)))
    ll, llo = O.loglik_from_partials(p.cpu().numpy(), n), O.loglik_from_partials(po, n)
    assert abs(ll - llo) <= 1e-12 * abs(llo), (ll, llo)


@pytest.mark.parametrize("form", ["torch", "numpy", "loop"])
@pytest.mark.parametrize("m", [1, 6, 15, 18, 19, 20, 21, 22, 23, 24, 25, 28, 32])  # 18..24: left-looking (round 6)
def test_callable_sweep_vs_oracle(dev, form, m):
    from pynngp_amd import CallableCovariance, _lib
    from pynngp_amd.nngp import _sweep_any

    if form == "loop" and m not in (6, 28):
        pytest.skip("one-call-per-location plug-in: two sizes suffice")
    rng = np.random.default_rng(100 + m)
    n = 1500
    x = rng.uniform(size=(n, 2))
    y = rng.standard_normal(n)
    mk = {"torch": _aniso, "numpy": _np_only, "loop": _loop_only}[form]
    fn = mk(1.4, A1, 0.05)
    cc = CallableCovariance(fn)
    c = torch.from_numpy(x).to(dev)
    v = torch.from_numpy(y).to(dev)
    nb = _lib.knn_prior(c, m)
    B, F, p = _sweep_any(cc, c, nb, 0, values=v, qvalues=v)
    assert cc.mode == form
    assert p[2].item() == -1 and p[3].item() == -1
    Bo, Fo, po = O.bf_sweep_callable(x, nb.cpu().numpy(), _aniso(1.4, A1, 0.05), y)
    _check(B, F, p, Bo, Fo, po, n)


@pytest.mark.parametrize("m", [10, 27])
def test_callable_visiting_order_and_bits(dev, m):
    """Z-order visiting order gives the same bits per row; two runs give the same bits."""
    from pynngp_amd import CallableCovariance, _lib
    from pynngp_amd.nngp import _sweep_any

    rng = np.random.default_rng(7 + m)
    x = rng.uniform(size=(5000, 2))
    y = rng.standard_normal(5000)
    c, v = torch.from_numpy(x).to(dev), torch.from_numpy(y).to(dev)
    nb = _lib.knn_prior(c, m)
    cc = CallableCovariance(_aniso(1.0, [[90.0, -20.0], [-20.0, 30.0]], 0.1))
    B1, F1, p1 = _sweep_any(cc, c, nb, 0, values=v, qvalues=v)
    order, nbs = _lib.row_order(c, nbr=nb)
    B2, F2, p2 = _sweep_any(cc, c, nbs, 0, values=v, qvalues=v, order=order)
    assert torch.equal(F1, F2) and torch.equal(B1, B2)
    B3, F3, p3 = _sweep_any(cc, c, nbs, 0, values=v, qvalues=v, order=order)
    assert torch.equal(p2, p3) and torch.equal(F2, F3)
    np.testing.assert_allclose(p1[:2].cpu().numpy(), p2[:2].cpu().numpy(), rtol=1e-12)


@pytest.mark.parametrize("m", [12, 30])
def test_callable_bad_index_flag(dev, m):
    from pynngp_amd import CallableCovariance, _lib
    from pynngp_amd.nngp import _sweep_any

    rng = np.random.default_rng(3)
    x = torch.from_numpy(rng.uniform(size=(800, 2))).to(dev)
    nb = _lib.knn_prior(x, m)
    nb[400, 3] = 800  # out of range
    _, _, p = _sweep_any(CallableCovariance(_aniso(1.0, A1, 0.1)), x, nb, 0)
    assert p[3].item() == 400


def test_nngp_class_with_reference_style_callable(dev):
    """NNGP(t, y, eps, 'S=T', m, cov) with a plain callable: _CNs / _Ccross / _Cs are the plug-in's
    values, _Bsi / _Fsi / compute_BF / loglik come from the device sweep and match the oracle."""
    from pynngp_amd import NNGP

    rng = np.random.default_rng(11)
    n, m = 1200, 12
    t = rng.uniform(size=(n, 2))
    y = rng.standard_normal(n)
    user_cov = _np_only(2.0, A1, 0.1)
    model = NNGP(t, y, None, "S=T", m, user_cov)
    nbr = model.nbr.cpu().numpy()
    Bo, Fo, po = O.bf_sweep_callable(t, nbr, user_cov, y)
    for i in (0, 1, 5, 600, n - 1):
        k = min(i, m)
        idx = nbr[i, :k]
        np.testing.assert_allclose(model._CNs(i), user_cov(t[idx], t[idx]), rtol=1e-15)
        np.testing.assert_allclose(np.ravel(model._Cs(i))[0], 2.1, rtol=1e-15)
        Bi, Fi = model._Bsi(i), model._Fsi(i)
        assert Bi.shape == (k,)
        np.testing.assert_allclose(Bi, Bo[i, :k], rtol=0, atol=1e-9)
        assert abs(Fi - Fo[i]) <= 1e-10 * Fo[i]
    B, F = model.compute_BF()
    np.testing.assert_allclose(F.cpu().numpy(), Fo, rtol=1e-10)
    assert np.all(np.abs(B.cpu().numpy() - Bo) <= 1e-9 * (1 + np.abs(Bo)))
    ll = model.loglik()
    want = O.loglik_from_partials(po, n)
    assert abs(ll - want) <= 1e-12 * abs(want)
    assert model._blk_cache is None  # a plain callable is evaluated on every sweep (the reference's semantics)
    assert model.loglik() == ll
    y2 = rng.standard_normal(n)
    _, _, p2 = O.bf_sweep_callable(t, nbr, user_cov, y2)
    assert abs(model.loglik(y2) - O.loglik_from_partials(p2, n)) <= 1e-12 * abs(model.loglik(y2))


def test_callable_cache_opt_in_and_mutable_plugin(dev):
    """advice r04: a plug-in whose state changes between sweeps (a closure over a parameter an MLE loop
    moves) must see its current state -- the default re-evaluates; CallableCovariance(fn, cache=True) keeps
    the blocks (keyed on the nugget too) until clear_cache()."""
    from pynngp_amd import NNGP, CallableCovariance

    rng = np.random.default_rng(41)
    n, m = 1000, 10
    t = rng.uniform(size=(n, 2))
    y = rng.standard_normal(n)
    state = {"s2": 1.0}

    def cov(a, b):
        return state["s2"] * _aniso(1.0, A1, 0.1)(a, b)

    model = NNGP(t, y, None, "S=T", m, cov)
    ll1 = model.loglik()
    state["s2"] = 2.0
    ll2 = model.loglik()
    _, _, p2 = O.bf_sweep_callable(t, model.nbr.cpu().numpy(), cov, y)
    assert ll2 != ll1 and abs(ll2 - O.loglik_from_partials(p2, n)) <= 1e-12 * abs(ll2)
    cc = CallableCovariance(cov, cache=True)
    model2 = NNGP(t, y, None, "S=T", m, cc)
    ll_a = model2.loglik()
    assert model2._blk_cache is not None
    state["s2"] = 1.0
    assert model2.loglik() == ll_a  # kept: the caller promised a fixed function
    cc.tau2 = 0.05  # the nugget is part of the key
    assert model2.loglik() != ll_a
    model2.clear_cache()
    cc.tau2 = 0.0
    assert model2.loglik() == ll1


def test_predict_with_callable(dev):
    """Kriging at points outside S with a plug-in (the cross sweep through the blocks kernel) vs the
    oracle with the location rows taken from the query points."""
    from pynngp_amd import NNGP

    rng = np.random.default_rng(12)
    n, m = 900, 10
    t = rng.uniform(size=(n, 2))
    y = rng.standard_normal(n)
    user_cov = _aniso(1.5, A1, 0.02)
    model = NNGP(t, y, None, "S=T", m, user_cov)
    q = rng.uniform(size=(300, 2))
    mean, var = model.predict(values=y, query=q)
    nq = O.knn_all(q, t, m)
    Bo, Fo, _ = O.bf_sweep_callable(t, nq, user_cov, y, qcoords=q, qvalues=np.zeros(300))
    np.testing.assert_allclose(var, Fo, rtol=1e-10)
    np.testing.assert_allclose(mean, (Bo * y[nq]).sum(1), rtol=0, atol=1e-9)
    # the sampler with the plug-in held fixed (round 5; it raised TypeError before): a chain runs, w /
    # tau2 / beta move, sigma2 and phi stay
    smp = model.oneSample(seed=3)
    for _ in range(20):
        smp = model.oneSample()
    assert smp.kind == "custom" and smp.sigma2 == 1.0 and smp.iteration == 21
    assert np.all(np.isfinite(model.ws)) and np.isfinite(smp.tau2) and np.all(np.isfinite(smp.beta))


def test_callable_w_sweep_matches_dense_oracle(dev):
    """The chain's colour sweep with the anisotropic plug-in (B / F from its blocks) equals the dense
    full-conditional sweep of the precision (I - B)^T F^-1 (I - B) + H / tau2 (given normals) -- the check
    tests/test_gpu_gibbs.py::test_w_sweep_matches_dense_oracle makes for the built-in kinds."""
    from oracle import nngp_gibbs_oracle as G
    from pynngp_amd import CallableCovariance, _lib

    rng = np.random.default_rng(5)
    n, m, tau2 = 2000, 10, 0.2
    x = rng.uniform(size=(n, 2))
    c = torch.from_numpy(x).to(dev)
    nbr = _lib.knn_prior(c, m)
    w = torch.from_numpy(rng.standard_normal(n)).to(dev)
    cc = CallableCovariance(_aniso(1.3, A1))
    blk = cc.blocks(c, nbr, 0)
    R = torch.empty(n, dtype=torch.float64, device=dev)
    B, F, p = _lib.bf_sweep_blocks(blk, nbr, n, 0, values=w, qvalues=w, R=R)
    Bo, Fo, _ = O.bf_sweep_callable(x, nbr.cpu().numpy(), _aniso(1.3, A1), w.cpu().numpy())
    np.testing.assert_allclose(F.cpu().numpy(), Fo, rtol=1e-10)
    off, rev_j, rev_k = _lib.reverse_neighbors(nbr)
    colors, nc = _lib.color_moral_graph(nbr.cpu().numpy(), off.cpu().numpy(), rev_j.cpu().numpy())
    members = torch.from_numpy(np.argsort(colors, kind="stable").astype(np.int32)).to(dev)
    color_off = np.concatenate([[0], np.cumsum(np.bincount(colors, minlength=nc))]).astype(np.int32)
    yres = torch.from_numpy(rng.standard_normal(n) * 1.5).to(dev)
    z = torch.from_numpy(rng.standard_normal(n)).to(dev)
    nb_h, B_h, F_h = nbr.cpu().numpy(), B.cpu().numpy(), F.cpu().numpy()
    P = G.precision(nb_h, B_h, F_h) + np.eye(n) / tau2
    w_ref = G.color_sweep(P, yres.cpu().numpy() / tau2, w.cpu().numpy().copy(), colors, z.cpu().numpy())
    prep = _lib.gibbs_prepare(B, F, off, rev_j, rev_k)
    wg, rg = w.clone(), R.clone()
    _lib.gibbs_w_sweep(members, color_off, prep, m, 1.0, tau2, yres, wg, rg, off, rev_j, 123, 0, z=z)
    np.testing.assert_allclose(wg.cpu().numpy(), w_ref, rtol=1e-9, atol=1e-9 * np.abs(w_ref).max())


def test_callable_chain_equals_builtin_with_phi_fixed(dev):
    """An isotropic exponential written as the reference's plug-in runs the same chain as the built-in
    exponential kind with phi and sigma2 held fixed (the same model; B / F differ only by the plug-in's
    torch exp against the kernel's table exp, ~1 ulp, so the chains agree to ~1e-9, not bit for bit)."""
    from pynngp_amd import SeqNNGP

    rng = np.random.default_rng(17)
    n, m, phi = 3000, 10, 12.0
    x = rng.uniform(size=(n, 2))
    y = np.sin(6 * x[:, 0]) + 0.3 * rng.standard_normal(n)

    def cov(a, b):
        lib = torch if isinstance(a, torch.Tensor) else np
        t = a[..., :, None, :] - b[..., None, :, :]
        return lib.exp(-phi * lib.sqrt((t ** 2).sum(-1)))

    kw = dict(m=m, tau2=0.1, seed=9, device=dev)
    ch_c = SeqNNGP(x, y, cov=cov, **kw)
    ch_b = SeqNNGP(x, y, kind="exponential", sigma2=1.0, phi=phi, fix_phi=True, fix_sigma2=True, **kw)
    for _ in range(25):
        ch_c.step()
        ch_b.step()
    assert ch_c.phi == 0.0 and ch_b.phi == phi and ch_c.sigma2 == ch_b.sigma2 == 1.0
    np.testing.assert_allclose(ch_c.tau2, ch_b.tau2, rtol=1e-8)
    np.testing.assert_allclose(ch_c.beta, ch_b.beta, rtol=1e-8, atol=1e-10)
    wc, wb = ch_c.w_t.cpu().numpy(), ch_b.w_t.cpu().numpy()
    np.testing.assert_allclose(wc, wb, rtol=0, atol=1e-8 * np.abs(wb).max())


def test_isotropic_and_callable_agree_at_m28(dev):
    """The four-lane blocks kernel (m = 25..32) with an isotropic function equals the fused
    exponential kernel, as the two-lane blocks kernel does for m <= 24."""
    from pynngp_amd import Covariance, IsotropicCovariance, _lib
    from pynngp_amd.nngp import _sweep_any

    rng = np.random.default_rng(13)
    x = rng.uniform(size=(4000, 2))
    y = rng.standard_normal(4000)
    c, v = torch.from_numpy(x).to(dev), torch.from_numpy(y).to(dev)
    nb = _lib.knn_prior(c, 28)
    B1, F1, p1 = _sweep_any(IsotropicCovariance(lambda d: 1.2 * torch.exp(-20.0 * d), 0.1), c, nb, 0, values=v,
                            qvalues=v)
    B2, F2, p2 = _sweep_any(Covariance("exponential", 1.2, 20.0, 0.1), c, nb, 0, values=v, qvalues=v)
    np.testing.assert_allclose(F1.cpu().numpy(), F2.cpu().numpy(), rtol=1e-10)
    assert torch.all((B1 - B2).abs() <= 1e-9 * (1 + B2.abs()))
    assert abs(p1[1].item() - p2[1].item()) <= 1e-11 * abs(p2[1].item())


@pytest.mark.parametrize("m", [10, 15, 27])
def test_callable_distinct_pairs_equal_blocks(dev, m):
    """Round 5: a broadcasting plug-in is evaluated once per DISTINCT point pair of the sweep's joint blocks
    (the blocks gathered from those values) -- B, F and the partials bit-identical to one evaluation per
    block entry (pairs=False), in index order and in a visiting order; the pair index is cached and rebuilt
    when the neighbour tensor changes in place."""
    from pynngp_amd import CallableCovariance, _lib
    from pynngp_amd.nngp import _sweep_any

    rng = np.random.default_rng(50 + m)
    x = rng.uniform(size=(20_000, 2))
    y = rng.standard_normal(20_000)
    c, v = torch.from_numpy(x).to(dev), torch.from_numpy(y).to(dev)
    nb = _lib.knn_prior(c, m)
    fn = _aniso(1.2, [[90.0, -20.0], [-20.0, 30.0]], 0.05)
    cp, cb = CallableCovariance(fn, pairs=True), CallableCovariance(fn)
    order, nbs = _lib.row_order(c, nbr=nb)
    for kw in (dict(), dict(order=order)):
        nbr = nbs if kw else nb
        rp = _sweep_any(cp, c, nbr, 0, values=v, qvalues=v, **kw)
        rb = _sweep_any(cb, c, nbr, 0, values=v, qvalues=v, **kw)
        assert cp._pairs_ok is True and cp._pidx is not None
        assert all(torch.equal(a, b) for a, b in zip(rp, rb))
        pa = cp._pidx[1][0]
        assert pa.numel() < 0.6 * nbr.shape[0] * (m + 1) * (m + 2) // 2  # shared pairs evaluated once
    nb2 = nb.clone()
    _sweep_any(cp, c, nb2, 0, values=v, qvalues=v)
    nb2[m + 5:m + 500, 0] = -1  # in place: a dropped neighbour (the slot becomes padding)
    rp = _sweep_any(cp, c, nb2, 0, values=v, qvalues=v)
    rb = _sweep_any(cb, c, nb2, 0, values=v, qvalues=v)
    assert all(torch.equal(a, b) for a, b in zip(rp, rb))


def test_callable_pairs_probe_rejects_asymmetric(dev):
    """A plug-in whose fn(a, b) and fn(b, a) differ in the last bits keeps one evaluation per block entry."""
    from pynngp_amd import CallableCovariance, _lib
    from pynngp_amd.nngp import _sweep_any

    base = _aniso(1.0, [[60.0, 0.0], [0.0, 60.0]], 0.1)

    def asym(a, b):  # a - b in a non-commutative form: (a0 - b0) + (a1 - b1) rounds differently from its negation
        t = a[..., :, None, :] - b[..., None, :, :]
        return base(a, b) * (1.0 + 1e-12 * torch.tanh(t[..., 0] * 3.0 + t[..., 1] * 7.0) ** 2 * torch.sign(t[..., 0]))

    rng = np.random.default_rng(3)
    c = torch.from_numpy(rng.uniform(size=(3_000, 2))).to(dev)
    v = torch.from_numpy(rng.standard_normal(3_000)).to(dev)
    nb = _lib.knn_prior(c, 10)
    cp, cb = CallableCovariance(asym, pairs=True), CallableCovariance(asym)
    rp = _sweep_any(cp, c, nb, 0, values=v, qvalues=v)
    rb = _sweep_any(cb, c, nb, 0, values=v, qvalues=v)
    assert cp._pairs_ok is False
    assert all(torch.equal(a, b) for a, b in zip(rp, rb))


@pytest.mark.parametrize("order_kind", ["none", "zorder"])
def test_callable_blocks_chunked_rows(dev, order_kind):
    """Round-5 regression: the per-entry evaluation in several row chunks gives the blocks of one chunk (the
    chunks after the first took the locations i0.. again when the sweep had no visiting order)."""
    from pynngp_amd import CallableCovariance, _lib

    rng = np.random.default_rng(12)
    c = torch.from_numpy(rng.uniform(size=(6_000, 2))).to(dev)
    nb = _lib.knn_prior(c, 12)
    order = None
    if order_kind == "zorder":
        order, nb = _lib.row_order(c, nbr=nb)
    fn = _aniso(1.0, [[50.0, 5.0], [5.0, 40.0]], 0.1)
    one = CallableCovariance(fn, pairs=False).blocks(c, nb, 0, order=order)
    many = CallableCovariance(fn, pairs=False, chunk_bytes=200 * 13 * 13 * 24).blocks(c, nb, 0, order=order)
    pairs = CallableCovariance(fn, pairs=True).blocks(c, nb, 0, order=order)
    valid = torch.cat([nb >= 0, torch.ones(nb.shape[0], 1, dtype=torch.bool, device=dev)], 1)
    a = torch.arange(13, device=dev)
    ta, tb = torch.repeat_interleave(a, a + 1), torch.cat([torch.arange(int(k) + 1, device=dev) for k in range(13)])
    ok = (valid[:, ta] & valid[:, tb]).t()
    assert torch.equal(one, many)
    assert torch.equal(one[ok], pairs[ok])
