"""GPU: the tiled colour sweep of the Gibbs sampler (pynngp_amd/gibbs_tiles.py, gibbs.hip gibbs_tile_phase).

The tiled sweep draws every node's full conditional once, in the plan's (level, phase, colour) order,
with each tile's footprint of the residuals r in LDS.  Parity: one sweep with given normals equals the
dense oracle's colour sweep in that order (oracle/nngp_gibbs_oracle.py, the plan's effective colouring),
the maintained residuals equal the recomputed ones, the Philox-driven tiled sweeps sample the exact
Gaussian posterior, and SeqNNGP(sweep="tiled") recovers the field parameters (S = T and S != T).
Parity unpinned by the reference (its sampler's updates are undefined, nngp.py:98-101)."""
import numpy as np
import pytest
import torch

from oracle import nngp_gibbs_oracle as G

pytestmark = pytest.mark.gpu


def _setup(dev, n, m, phi=6.0, seed=0, tile_nodes=256, coarse="tiles"):
    """A field stored in its tile plan's node order (gibbs_tiles.contiguous_plan), then B / F / r there"""
    from pynngp_amd import _lib
    from pynngp_amd.gibbs_tiles import check_tile_plan, contiguous_plan

    rng = np.random.default_rng(seed)
    c0 = torch.from_numpy(rng.uniform(size=(n, 2))).to(dev)
    nbr0 = _lib.knn_prior(c0, m)
    off0, rev_j0, _ = _lib.reverse_neighbors(nbr0)
    colors0, nc = _lib.color_moral_graph(nbr0.cpu().numpy(), off0.cpu().numpy(), rev_j0.cpu().numpy())
    perm, nbr, off, rev_j, rev_k, tp = contiguous_plan(c0, nbr0, torch.from_numpy(colors0.astype(np.int64)).to(dev),
                                                       nc, nc, tile_nodes=tile_nodes, coarse=coarse)
    check_tile_plan(tp, off, rev_j)
    c = c0[perm].contiguous()
    colors = colors0[perm.cpu().numpy()]
    assert G.coloring_is_valid(nbr.cpu().numpy(), colors) if n <= 5000 else True
    w = torch.from_numpy(rng.standard_normal(n)).to(dev)
    R = torch.empty(n, dtype=torch.float64, device=dev)
    B, F, p = _lib.bf_sweep(c, nbr, 0, "exponential", 1.0, phi, 0.0, values=w, R=R)
    return dict(c=c, nbr=nbr, w=w, R=R, B=B, F=F, off=off, rev_j=rev_j, rev_k=rev_k, colors=colors, tp=tp, rng=rng)


def _residuals(nbr, B, w):
    wn = np.where(nbr >= 0, w[np.maximum(nbr, 0)], 0.0)
    return w - (B * wn).sum(1)


@pytest.mark.parametrize("n,m,sigma2,tau2,weighted,tile_nodes,coarse", [
    (400, 5, 1.3, 0.2, False, 64, "tiles"), (3000, 15, 2.0, 1.0, False, 256, "tiles"),
    (3000, 10, 0.7, 0.05, True, 512, "tiles"), (20000, 15, 1.0, 0.1, False, 2048, "tiles"),
    (400, 5, 1.3, 0.2, False, 64, "colour"), (3000, 15, 2.0, 1.0, True, 256, "colour"),
    (20000, 15, 1.0, 0.1, False, 2048, "colour"),
    (1, 3, 1.0, 0.5, False, 16, "tiles"), (2, 1, 0.8, 0.3, True, 16, "tiles"),  # no / one reverse entry
    (37, 1, 1.1, 0.2, False, 4, "colour")])
def test_tiled_sweep_matches_dense_oracle(dev, n, m, sigma2, tau2, weighted, tile_nodes, coarse):
    """One tiled sweep with given normals equals the dense full-conditional sweep in the plan's order
    (coarse="colour": the nodes above level 0 swept after the tiles, one launch per colour)."""
    from pynngp_amd import _lib

    s = _setup(dev, n, m, seed=n + m, tile_nodes=tile_nodes, coarse=coarse)
    tp = s["tp"]
    assert len(tp.phases) >= (2 if n > 100 else 1)
    if coarse == "colour" and n > 100:
        assert tp.coarse_members is not None and tp.coarse_members.numel() > 0
    rng = s["rng"]
    yres = torch.from_numpy(rng.standard_normal(n) * 1.5).to(dev)
    z = torch.from_numpy(rng.standard_normal(n)).to(dev)
    h = rng.uniform(0.2, 5.0, n) if weighted else np.ones(n)
    nbr, B, F = s["nbr"].cpu().numpy(), s["B"].cpu().numpy(), s["F"].cpu().numpy()
    w0 = s["w"].cpu().numpy().copy()
    w, r = s["w"].clone(), s["R"].clone()
    prep = _lib.gibbs_prepare(s["B"], s["F"], s["off"], s["rev_j"], s["rev_k"])
    _lib.gibbs_w_sweep_tiles(tp, prep, m, sigma2, tau2, yres, w, r, s["off"], z,
                             noise_w=torch.from_numpy(h).to(dev) if weighted else None, rev_j=s["rev_j"])
    wh = w.cpu().numpy()
    if n <= 5000:
        P = G.precision(nbr, B, F * sigma2) + np.diag(h / tau2)
        b = yres.cpu().numpy() * h / tau2
        w_ref = G.color_sweep(P, b, w0, tp.effective_colors, z.cpu().numpy())
        np.testing.assert_allclose(wh, w_ref, rtol=1e-9, atol=1e-9 * np.abs(w_ref).max())
    # maintained residuals equal the recomputed ones
    np.testing.assert_allclose(r.cpu().numpy(), _residuals(nbr, B, wh), rtol=0, atol=1e-10 * (1 + np.abs(wh).max()))


def test_tiled_sweep_equals_colour_sweep_in_the_same_order(dev):
    """The tiled kernel and the per-colour kernel on the plan's effective colouring: the same draws (to the
    children sums' summation order)"""
    from pynngp_amd import _lib

    n, m = 20000, 15
    s = _setup(dev, n, m, seed=5, tile_nodes=1024)
    tp = s["tp"]
    rng = s["rng"]
    yres = torch.from_numpy(rng.standard_normal(n)).to(dev)
    z = torch.from_numpy(rng.standard_normal(n)).to(dev)
    prep = _lib.gibbs_prepare(s["B"], s["F"], s["off"], s["rev_j"], s["rev_k"])
    w1, r1 = s["w"].clone(), s["R"].clone()
    _lib.gibbs_w_sweep_tiles(tp, prep, m, 1.1, 0.3, yres, w1, r1, s["off"], z)
    eff = tp.effective_colors
    members = torch.from_numpy(np.argsort(eff, kind="stable").astype(np.int32)).to(dev)
    color_off = np.concatenate([[0], np.cumsum(np.bincount(eff))]).astype(np.int32)
    w2, r2 = s["w"].clone(), s["R"].clone()
    _lib.gibbs_w_sweep(members, color_off, prep, m, 1.1, 0.3, yres, w2, r2, s["off"], s["rev_j"], 0, 0, z=z)
    np.testing.assert_allclose(w1.cpu().numpy(), w2.cpu().numpy(), rtol=1e-11, atol=1e-11)
    np.testing.assert_allclose(r1.cpu().numpy(), r2.cpu().numpy(), rtol=1e-10, atol=1e-10)


def test_tiled_sweep_stationary_law(dev):
    """Philox-driven tiled sweeps sample N(P^-1 b, P^-1) (exact Gaussian posterior, N=24, 4-node tiles)."""
    from pynngp_amd import _lib

    n, m, sigma2, tau2 = 24, 4, 1.0, 0.5
    s = _setup(dev, n, m, phi=3.0, seed=7, tile_nodes=4)
    rng = s["rng"]
    yres = torch.from_numpy(rng.standard_normal(n)).to(dev)
    nbr, B, F = s["nbr"].cpu().numpy(), s["B"].cpu().numpy(), s["F"].cpu().numpy()
    P = G.precision(nbr, B, F * sigma2) + np.eye(n) / tau2
    mu = np.linalg.solve(P, yres.cpu().numpy() / tau2)
    S = np.linalg.inv(P)
    w, r = s["w"].clone(), s["R"].clone()
    z = torch.empty(n, dtype=torch.float64, device=dev)
    draws = []
    prep = _lib.gibbs_prepare(s["B"], s["F"], s["off"], s["rev_j"], s["rev_k"])
    for t in range(20000):
        _lib.gibbs_normals(z, 99, t)
        _lib.gibbs_w_sweep_tiles(s["tp"], prep, m, sigma2, tau2, yres, w, r, s["off"], z)
        if t >= 100:
            draws.append(w.clone())
    W = torch.stack(draws).cpu().numpy()
    sd = np.sqrt(np.diag(S))
    nb = 50
    bm = W[: len(W) // nb * nb].reshape(nb, -1, n).mean(1)
    se = bm.std(0, ddof=1) / np.sqrt(nb)
    zscore = (W.mean(0) - mu) / np.maximum(se, 1e-3 * sd)
    assert np.abs(zscore).max() < 5.0, zscore
    emp = np.cov(W.T)
    np.testing.assert_allclose(np.sqrt(np.diag(emp)), sd, rtol=0.06)


def test_tiled_sweep_rejects_a_non_contiguous_plan(dev):
    """The kernel reads tile t's nodes as rows [n0, n1): a plan in another node order is refused"""
    import dataclasses

    from pynngp_amd import _lib

    s = _setup(dev, 3000, 10, seed=3, tile_nodes=256)
    prep = _lib.gibbs_prepare(s["B"], s["F"], s["off"], s["rev_j"], s["rev_k"])
    z = torch.zeros(3000, dtype=torch.float64, device=dev)
    with pytest.raises(ValueError, match="contiguous"):
        _lib.gibbs_w_sweep_tiles(dataclasses.replace(s["tp"], contiguous=False), prep, 10, 1.0, 1.0, z,
                                 s["w"].clone(), s["R"].clone(), s["off"], z)


def test_seqnngp_tiled_recovers_parameters(dev):
    from pynngp_amd import Priors, SeqNNGP
    from tests.test_gpu_gibbs import _simulate

    truth = dict(sigma2=1.0, phi=6.0, tau2=0.1)
    beta = np.array([1.0, -0.5])
    c, y, X, w = _simulate(2500, truth["sigma2"], truth["phi"], truth["tau2"], beta, 2)
    pri = Priors(sigma2_ig=(2.0, 1.0), tau2_ig=(2.0, 0.1), phi_unif=(0.5, 60.0))
    s = SeqNNGP(c, y, X, m=10, priors=pri, phi=10.0, tau2=0.5, seed=3, device=dev, phi_tuning=0.1, sweep="tiled")
    assert s._tiles is not None
    res = s.sample(2500, burn=1000, keep_w_mean=True)
    assert 0.1 < res["phi_accept_rate"] < 0.95
    assert abs(res["beta"][:, 1].mean() - beta[1]) < 0.05
    assert 0.5 < res["sigma2"].mean() / truth["sigma2"] < 2.0
    assert 0.5 < res["tau2"].mean() / truth["tau2"] < 2.0
    assert 0.4 < res["phi"].mean() / truth["phi"] < 2.5
    assert np.corrcoef(res["w_mean"], w)[0, 1] > 0.8


def test_seqnngp_tiled_reference_set(dev):
    """S != T: the leaves' colour runs first inside each tile (update_wt before update_ws); one tiled
    sweep with given normals equals the dense DAG sweep in the plan's order"""
    from pynngp_amd import SeqNNGP, _lib

    rng = np.random.default_rng(4)
    t = rng.uniform(size=(1500, 2))
    s_pts = rng.uniform(size=(600, 2))
    y = np.sin(6 * t[:, 0]) + 0.3 * rng.standard_normal(1500)
    g = SeqNNGP(t, y, m=8, ref=s_pts, seed=2, device=dev, sweep="tiled")
    tp = g._tiles
    assert g.n_colors > g.n_colors_ref  # leaves exist
    # effective colours put every leaf of a tile before the tile's reference nodes
    leaf = torch.from_numpy(g.colors == g.n_colors_ref).to(dev)
    z = torch.from_numpy(rng.standard_normal(g.n)).to(dev)
    nbr, B, F = g.nbr.cpu().numpy(), g.B.cpu().numpy(), g.Ft.cpu().numpy()
    h = g.noise_w.cpu().numpy() if g.noise_w is not None else np.ones(g.n)
    P = G.precision(nbr, B, F * g.sigma2) + np.diag(h / g.tau2)
    b = g.yres.cpu().numpy() * h / g.tau2
    w0 = g.w.cpu().numpy().copy()
    w_ref = G.color_sweep(P, b, w0, tp.effective_colors, z.cpu().numpy())
    _lib.gibbs_w_sweep_tiles(tp, g._prep, g.m, g.sigma2, g.tau2, g.yres, g.w, g.r, g.off, z, noise_w=g.noise_w,
                             rev_j=g.rev_j)
    np.testing.assert_allclose(g.w.cpu().numpy(), w_ref, rtol=1e-9, atol=1e-9 * np.abs(w_ref).max())
    assert bool(leaf.any())
    g.sample(50)
    assert np.isfinite(g.w.cpu().numpy()).all()


def test_tile_plan_config5_size(dev):
    """N = 1e6, m = 15 (config 5): the plan's invariants, its launch count and LDS, and 20 tiled iterations"""
    from pynngp_amd import SeqNNGP
    from pynngp_amd.gibbs_tiles import check_tile_plan

    rng = np.random.default_rng(0)
    n = 1_000_000
    c = rng.uniform(size=(n, 2))
    y = 1.0 + np.sin(5 * c[:, 0]) + 0.3 * rng.standard_normal(n)
    g = SeqNNGP(c, y, m=15, seed=1, device=dev, sweep="tiled")
    tp = g._tiles
    check_tile_plan(tp, g.off, g.rev_j)
    assert len(tp.phases) <= 40 and max(tp.phase_lds) <= 144 * 1024
    for _ in range(20):
        g.step()
    assert np.isfinite(g.w.cpu().numpy()).all() and np.isfinite(g.sigma2) and np.isfinite(g.tau2)
