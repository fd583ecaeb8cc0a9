"""The sampler with a reference set S != T (the reference's
oneSample -> update_wt / update_ws / update_y_unobserved, nngp.py:42-47,64-71,98-101).

Checked against the dense oracle of the DAG [S; T_out] (oracle/nngp_gibbs_oracle.py
reference_dag / dag_posterior): the node and neighbour structure, one update_wt +
update_ws pass with given normals against the dense full-conditional sweep, the
stationary law of w and of the predictive draws against the exact Gaussian posterior,
and prediction of held-out responses.  "Parity unpinned" with respect to the reference,
whose sampler methods do not exist."""
import numpy as np
import pytest
import torch

from oracle import nngp_gibbs_oracle as G

pytestmark = pytest.mark.gpu


def _model_order(smp):
    """The sampler's storage-order state mapped back to model (node) order."""
    pos, perm = smp.pos, smp.perm
    nb = smp.nbr[pos].long()
    nbr = torch.where(nb >= 0, perm[nb.clamp(min=0)], -1).cpu().numpy().astype(np.int32)
    h = smp.noise_w[pos].cpu().numpy() if smp.noise_w is not None else np.ones(smp.n)
    return dict(nbr=nbr, B=smp.B[pos].cpu().numpy(), F=smp.Ft[pos].cpu().numpy(), h=h,
                yres=smp.yres[pos].cpu().numpy(), colors=smp.colors[pos.cpu().numpy()],
                z=smp._z[pos].cpu().numpy(), w=smp.w_nodes.cpu().numpy(), r=smp.r[pos].cpu().numpy())


def _data(rng, n_s, n_new, n_in, n_nan):
    s = rng.uniform(size=(n_s, 2))
    t = np.concatenate([rng.uniform(size=(n_new, 2)), s[rng.choice(n_s, n_in, replace=False)]])
    t = t[rng.permutation(len(t))]
    y = np.sin(4 * t[:, 0]) + np.cos(3 * t[:, 1]) + 0.3 * rng.standard_normal(len(t))
    y[rng.choice(len(t), n_nan, replace=False)] = np.nan
    return s, t, y


def test_reference_set_structure_and_sweep_vs_dense(dev, c_oracle):
    from pynngp_amd import SeqNNGP

    rng = np.random.default_rng(21)
    s, t, y = _data(rng, 300, 400, 60, 40)
    smp = SeqNNGP(t, y, m=8, ref=s, sigma2=1.2, tau2=0.3, phi=6.0, seed=3, device=dev)
    assert smp.n == 300 + 400 and smp.n_s == 300 and smp.n_obs == 460 - 40
    node = smp.node_of_t.cpu().numpy()
    hit = node < 300
    assert hit.sum() == 60 and np.array_equal(s[node[hit]], t[hit])
    leaves = np.argsort(node[~hit])
    t_out = t[~hit][leaves]
    coords, nbr_ref = G.reference_dag(s, t_out, 8)
    mo = _model_order(smp)
    np.testing.assert_array_equal(mo["nbr"], nbr_ref)
    assert G.coloring_is_valid(mo["nbr"], mo["colors"]) and np.all(mo["colors"][300:] == smp.n_colors_ref)
    # observation weights: 1 on observed nodes, 0 on the unobserved and on data-free reference points
    h_ref = np.zeros(700)
    h_ref[node[np.isfinite(y)]] = 1.0
    np.testing.assert_array_equal(mo["h"], h_ref)
    # one update_wt + update_ws pass with the sampler's normals = the dense colour sweep
    smp.set_w(ws=rng.standard_normal(300), wt=rng.standard_normal(460))
    from pynngp_amd import _lib

    _lib.gibbs_normals(smp._z, smp.seed, smp.iteration)
    mo = _model_order(smp)
    P, b, _, _ = G.dag_posterior(mo["nbr"], mo["B"], mo["F"], smp.sigma2, smp.tau2, mo["h"], mo["yres"])
    order = np.where(mo["colors"] == smp.n_colors_ref, 0, mo["colors"] + 1)
    expect = G.color_sweep(P, b, mo["w"], order, mo["z"])
    smp.update_wt()
    smp.update_ws()
    got = smp.w_nodes.cpu().numpy()
    np.testing.assert_allclose(got, expect, rtol=1e-9, atol=1e-9 * np.abs(expect).max())
    # maintained residuals r = w - B w_N over the whole DAG
    mo = _model_order(smp)
    wn = np.where(mo["nbr"] >= 0, got[np.maximum(mo["nbr"], 0)], 0.0)
    np.testing.assert_allclose(mo["r"], got - (mo["B"] * wn).sum(1), rtol=0, atol=1e-10 * (1 + np.abs(got).max()))
    # the factors are the oracle's (S rows prior sets, leaf rows cross sets)
    Bo, Fo, _ = c_oracle.c_bf_sweep(coords, nbr_ref, "exponential", (1.0, smp.phi, 0.0))
    np.testing.assert_allclose(mo["F"], Fo, rtol=1e-10)


def test_reference_set_stationary_law(dev):
    """update_wt + update_ws sample the exact posterior of w over [S; T_out], and
    update_y_unobserved the exact predictive of the unobserved responses (N = 12 + 7)."""
    from pynngp_amd import SeqNNGP, _lib

    rng = np.random.default_rng(8)
    s, t, y = _data(rng, 12, 7, 3, 2)
    smp = SeqNNGP(t, y, m=4, ref=s, sigma2=1.0, tau2=0.5, phi=3.0, seed=17, device=dev)
    mo = _model_order(smp)
    _, _, mu, S = G.dag_posterior(mo["nbr"], mo["B"], mo["F"], smp.sigma2, smp.tau2, mo["h"], mo["yres"])
    un_nodes = np.concatenate([smp.node_of_t.cpu().numpy()[smp.unobserved_t], smp.unobserved_ref])
    assert len(smp.unobserved_t) == 2 and len(smp.unobserved_ref) == 12 - 3
    W, Y = [], []
    n_it = 20000
    for k in range(n_it):
        _lib.gibbs_normals(smp._z, smp.seed, smp.iteration)
        smp.update_wt()
        smp.update_ws()
        smp.update_y_unobserved()
        smp.iteration += 1
        if k >= 100:
            W.append(smp.w_nodes.clone())
            Y.append(smp.y_unobserved.clone())
    W, Y = torch.stack(W).cpu().numpy(), torch.stack(Y).cpu().numpy()
    sd = np.sqrt(np.diag(S))
    nb = 50
    for X, m_ex, sd_ex in [(W, mu, sd), (Y, float(smp.beta[0]) + mu[un_nodes],
                                         np.sqrt(np.diag(S)[un_nodes] + smp.tau2))]:
        bm = X[: len(X) // nb * nb].reshape(nb, -1, X.shape[1]).mean(1)
        se = bm.std(0, ddof=1) / np.sqrt(nb)
        zs = (X.mean(0) - m_ex) / np.maximum(se, 1e-3 * sd_ex)
        assert np.abs(zs).max() < 5.0, zs
        np.testing.assert_allclose(X.std(0), sd_ex, rtol=0.06)
    emp = np.cov(W.T)
    corr_emp = emp / np.outer(np.sqrt(np.diag(emp)), np.sqrt(np.diag(emp)))
    assert np.abs(corr_emp - S / np.outer(sd, sd)).max() < 0.08


def test_reference_set_predicts_held_out(dev):
    """A simulated GP field observed at T with 10 % held out; S = 1000 uniform reference
    points: the chain's predictive means track the held-out truth."""
    from pynngp_amd import Priors, SeqNNGP

    rng = np.random.default_rng(31)
    n = 2500
    t = rng.uniform(size=(n, 2))
    d = np.sqrt(((t[:, None, :] - t[None, :, :]) ** 2).sum(-1))
    w = np.linalg.cholesky(np.exp(-6.0 * d) + 1e-10 * np.eye(n)) @ rng.standard_normal(n)
    y_true = 1.0 + w + np.sqrt(0.1) * rng.standard_normal(n)
    hide = rng.choice(n, 250, replace=False)
    y = y_true.copy()
    y[hide] = np.nan
    s = rng.uniform(size=(1000, 2))
    smp = SeqNNGP(t, y, m=10, ref=s, sigma2=1.0, tau2=0.2, phi=5.0, seed=2, device=dev, phi_tuning=0.1,
                  priors=Priors(phi_unif=(1.0, 30.0)))
    res = smp.sample(1500, burn=1000, keep_w_mean=True)  # tau2 and the leaves' w mix slowly
    pred = res["y_unobserved_mean"][: len(hide)]
    assert np.array_equal(smp.unobserved_t, np.sort(hide))
    assert np.corrcoef(pred, y_true[np.sort(hide)])[0, 1] > 0.8
    assert 0.03 < np.mean(res["tau2"]) < 0.3 and abs(np.mean(res["beta"]) - 1.0) < 0.6
    assert res["ws_mean"].shape == (1000,) and res["w_mean"].shape == (n,)


def test_one_sample_random_reference_set(dev):
    """NNGP.oneSample with ('random', nRef, bounds) (nngp.py:38-40): ws lives on S, wt on T,
    y_unobserved holds the predictive draws at S; bit-reproducible."""
    from pynngp_amd import NNGP, Covariance

    rng = np.random.default_rng(6)
    t = rng.uniform(size=(2000, 2))
    y = np.sin(5 * t[:, 0]) + 0.2 * rng.standard_normal(2000)
    runs = []
    for _ in range(2):
        np.random.seed(9)
        g = NNGP(t, y, None, ("random", 600, ((0, 1), (0, 1))), 10, Covariance("exponential", 1.0, 8.0, 0.05),
                 device=dev)
        for _ in range(4):
            smp = g.oneSample(seed=4)
        assert g.ws.shape == (600,) and g.wt.shape == (2000,) and g.y_unobserved.shape == (600,)
        assert smp.n == 2600 and smp.iteration == 4 and np.all(np.isfinite(g.wt))
        runs.append((g.ws, g.wt, g.y_unobserved))
    for a, b in zip(*runs):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("with_ref", [False, True])
def test_checkpoint_resume_bit_identical(dev, tmp_path, with_ref):
    """save() after k iterations + restore() into a fresh sampler continues the chain bit
    for bit (Philox keyed by (seed, location, iteration); host RNG state restored)."""
    from pynngp_amd import SeqNNGP

    rng = np.random.default_rng(4)
    s, t, y = _data(rng, 400, 600, 50, 30)
    kw = dict(m=8, sigma2=1.0, tau2=0.2, phi=5.0, seed=5, device=dev, phi_tuning=0.2, ref=s if with_ref else None)
    if not with_ref:
        y = np.where(np.isfinite(y), y, 0.0)
    a = SeqNNGP(t, y, **kw)
    for _ in range(6):
        a.step()
    a.save(tmp_path / "ck.npz")
    for _ in range(6):
        a.step()
    b = SeqNNGP(t, y, **kw).restore(tmp_path / "ck.npz")
    assert b.iteration == 6
    for _ in range(6):
        b.step()
    assert torch.equal(a.w, b.w) and torch.equal(a.r, b.r) and torch.equal(a.y_unobserved, b.y_unobserved)
    assert (a.phi, a.sigma2, a.tau2, a.n_accept) == (b.phi, b.sigma2, b.tau2, b.n_accept)
    np.testing.assert_array_equal(a.beta, b.beta)
    with pytest.raises(ValueError, match="m="):
        SeqNNGP(t, y, **{**kw, "m": 6}).restore(tmp_path / "ck.npz")
    # same sizes, different data or settings: refused (the running residuals would not match)
    y2 = y.copy()
    y2[np.nonzero(np.isfinite(y2))[0][0]] += 1.0
    with pytest.raises(ValueError, match="different data"):
        SeqNNGP(t, y2, **kw).restore(tmp_path / "ck.npz")
    t2 = t.copy()
    t2[5] += 1e-3
    with pytest.raises(ValueError, match="different data"):
        SeqNNGP(t2, y, **kw).restore(tmp_path / "ck.npz")
    with pytest.raises(ValueError, match="phi_tuning"):
        SeqNNGP(t, y, **{**kw, "phi_tuning": 0.3}).restore(tmp_path / "ck.npz")
    # a checkpoint from before the data fingerprint (pynngp_amd < 0.2) still restores, with a warning
    import json

    with np.load(tmp_path / "ck.npz", allow_pickle=False) as z:
        arrs = {k: z[k] for k in z.files}
    meta = json.loads(str(arrs["meta"]))
    del meta["fingerprint_nodes"]
    arrs["meta"] = np.array(json.dumps(meta))
    np.savez(tmp_path / "ck_old.npz", **arrs)
    with pytest.warns(UserWarning, match="predates the data fingerprint"):
        c = SeqNNGP(t, y, **kw).restore(tmp_path / "ck_old.npz")
    assert c.iteration == 6
    # a 0.2 - 0.3 checkpoint (storage-order fingerprint) restores into the same storage order
    meta["fingerprint"] = a._fingerprint(node_order=False)
    arrs["meta"] = np.array(json.dumps(meta))
    np.savez(tmp_path / "ck_03.npz", **arrs)
    assert SeqNNGP(t, y, **kw).restore(tmp_path / "ck_03.npz").iteration == 6
    # the node-order fingerprint lets a checkpoint move between storage orders: into the tiled sweep's
    # sampler (its rows in the tile plan's order), the same state in node order
    d = SeqNNGP(t, y, **kw, sweep="tiled").restore(tmp_path / "ck.npz")
    assert d.iteration == 6 and not torch.equal(d.perm, a.perm)
    e = SeqNNGP(t, y, **kw).restore(tmp_path / "ck.npz")
    np.testing.assert_array_equal(d.w[d.pos].cpu().numpy(), e.w[e.pos].cpu().numpy())
    np.testing.assert_array_equal(d.r[d.pos].cpu().numpy(), e.r[e.pos].cpu().numpy())
    for _ in range(3):
        d.step()
    assert np.all(np.isfinite(d.w.cpu().numpy()))


def test_reference_set_rejects_repeated_points(dev):
    """A reference set with a repeated point (('subset', nRef) draws with replacement,
    nngp.py:36) makes C_N singular: refused with the offending indices."""
    from pynngp_amd import SeqNNGP

    rng = np.random.default_rng(2)
    t = rng.uniform(size=(500, 2))
    y = rng.standard_normal(500)
    s = t[[3, 10, 3, 40, 77]]  # point 2 repeats point 0
    with pytest.raises(ValueError, match="repeats point 0"):
        SeqNNGP(t, y, m=3, ref=s, device=dev)
    with pytest.raises(ValueError, match="m=0"):
        SeqNNGP(t, y, m=0, device=dev)
