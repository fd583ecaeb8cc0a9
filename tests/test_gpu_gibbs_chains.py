"""GPU: several Gibbs chains per GPU advanced together (SeqNNGPChains, nngp_gibbs_w_sweep_chains).

Config 5's replica mode (BASELINE.json: 1,000 sweeps at N = 1e6 per chain): C independent chains of one
field share the DAG, the colouring and ONE launch per colour.  Each chain's arithmetic is the single-chain
kernel's, operation for operation, so the bar is EXACT: chain k of the batched run equals
``SeqNNGP(..., seed=seeds[k])`` run alone -- w, the residuals r, beta, sigma2, tau2, phi, the MH
counters and the predictive draws, bit for bit -- for S = T, a reference set S != T with unobserved
responses and heteroscedastic noise, and the kernel against one colour sweep per chain.
(The sampler itself is parity-unpinned by the reference, whose oneSample calls methods that do not exist,
nngp.py:98-101; tests/test_gpu_gibbs.py holds the single chain to the dense full conditionals.)"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _field(n, seed, nan_frac=0.0):
    rng = np.random.default_rng(seed)
    x = rng.uniform(size=(n, 2))
    X = np.column_stack([np.ones(n), rng.standard_normal(n)])
    y = X @ np.array([1.0, -0.5]) + np.sin(5 * x[:, 0]) * np.cos(3 * x[:, 1]) + 0.3 * rng.standard_normal(n)
    if nan_frac:
        y[rng.random(n) < nan_frac] = np.nan
    return x, X, y


def _same(a, b):
    assert torch.equal(a.w, b.w) and torch.equal(a.r, b.r)
    assert np.array_equal(a.beta, b.beta)
    assert (a.sigma2, a.tau2, a.phi, a.n_accept, a.iteration) == (b.sigma2, b.tau2, b.phi, b.n_accept, b.iteration)
    assert torch.equal(a.y_unobserved, b.y_unobserved)


@pytest.mark.parametrize("interleave", [True, False])
@pytest.mark.parametrize("C", [1, 2, 3, 4, 8])
def test_chains_equal_single_runs(dev, C, interleave):
    from pynngp_amd import Priors, SeqNNGP, SeqNNGPChains

    x, X, y = _field(12_000, 5)
    kw = dict(m=10, priors=Priors(phi_unif=(2.0, 60.0)), sigma2=1.0, tau2=0.1, phi=12.0, phi_tuning=0.3, device=dev)
    seeds = [11 + 7 * k for k in range(C)]
    multi = SeqNNGPChains(x, y, X, seeds=seeds, interleave=interleave, **kw)
    for _ in range(12):
        multi.step()
    assert sum(c.n_accept for c in multi.chains) > 0  # phi moves (accepted proposals re-prepare B / F)
    for k, s in enumerate(seeds):
        one = SeqNNGP(x, y, X, seed=s, **kw)
        for _ in range(12):
            one.step()
        _same(multi[k], one)


def test_chains_reference_set_nan_and_eps(dev):
    """S != T (the leaves' colour is update_wt's), NaN responses (predictive draws), per-point noise"""
    from pynngp_amd import Priors, SeqNNGP, SeqNNGPChains

    x, X, y = _field(6_000, 9, nan_frac=0.1)
    rng = np.random.default_rng(2)
    ref = rng.uniform(size=(2_500, 2))
    eps = rng.uniform(0.5, 2.0, 6_000)
    kw = dict(m=8, priors=Priors(phi_unif=(2.0, 60.0)), sigma2=1.0, tau2=0.2, phi=10.0, phi_tuning=0.2, device=dev,
              ref=ref, eps=eps)
    seeds = [3, 4, 5]
    multi = SeqNNGPChains(x, y, None, seeds=seeds, **kw)
    assert multi[0].n_colors > multi[0].n_colors_ref  # the leaves' colour exists
    for _ in range(10):
        multi.step()
    for k, s in enumerate(seeds):
        one = SeqNNGP(x, y, None, seed=s, **kw)
        for _ in range(10):
            one.step()
        _same(multi[k], one)


def test_sweep_chains_kernel_equals_per_chain(dev):
    """nngp_gibbs_w_sweep_chains = nngp_gibbs_w_sweep for each chain (own prep, sigma2, tau2, yres, w, r, z)"""
    from pynngp_amd import _lib

    rng = np.random.default_rng(4)
    n, m, C = 20_000, 15, 5
    c = torch.from_numpy(rng.uniform(size=(n, 2))).to(dev)
    nbr = _lib.knn_prior(c, m)
    off, rev_j, rev_k = _lib.reverse_neighbors(nbr)
    colors, nc = _lib.color_moral_graph(nbr.cpu().numpy(), off.cpu().numpy(), rev_j.cpu().numpy())
    members = torch.from_numpy(np.argsort(colors, kind="stable").astype(np.int32)).to(dev)
    color_off = np.concatenate([[0], np.cumsum(np.bincount(colors, minlength=nc))]).astype(np.int32)
    mrows = _lib.gibbs_member_rows(members, off)
    noise = torch.from_numpy(rng.uniform(0.5, 2.0, n)).to(dev)
    st = []
    for k in range(C):
        w = torch.from_numpy(rng.standard_normal(n)).to(dev)
        R = torch.empty(n, dtype=torch.float64, device=dev)
        B, F, _ = _lib.bf_sweep(c, nbr, 0, "exponential", 1.0, 5.0 + 3 * k, 0.0, values=w, R=R)
        prep = _lib.gibbs_prepare(B, F, off, rev_j, rev_k)
        yres = torch.from_numpy(rng.standard_normal(n)).to(dev)
        z = torch.from_numpy(rng.standard_normal(n)).to(dev)
        st.append(dict(prep=prep, w=w, r=R, w0=w.clone(), r0=R.clone(), yres=yres, z=z, s2=0.5 + 0.3 * k,
                       t2=0.1 + 0.05 * k))
    ref = []
    for d in st:
        w, r = d["w"].clone(), d["r"].clone()
        _lib.gibbs_w_sweep(members, color_off, d["prep"], m, d["s2"], d["t2"], d["yres"], w, r, off, rev_j, 0, 0,
                           z=d["z"], noise_w=noise, member_rows=mrows)
        ref.append((w, r))
    # the interleaved entry point: (n, C) copies of w and r, the same results bit for bit
    W = torch.stack([d["w0"] for d in st], dim=1)
    R = torch.stack([d["r0"] for d in st], dim=1)
    _lib.gibbs_w_sweep_chains(mrows, color_off, [d["prep"] for d in st], m, [d["s2"] for d in st],
                              [d["t2"] for d in st], [d["yres"] for d in st], W, R, rev_j, [d["z"] for d in st],
                              noise_w=noise)
    _lib.gibbs_w_sweep_chains(mrows, color_off, [d["prep"] for d in st], m, [d["s2"] for d in st],
                              [d["t2"] for d in st], [d["yres"] for d in st], [d["w"] for d in st],
                              [d["r"] for d in st], rev_j, [d["z"] for d in st], noise_w=noise)
    for k, (d, (w, r)) in enumerate(zip(st, ref)):
        assert torch.equal(d["w"], w) and torch.equal(d["r"], r)
        assert torch.equal(W[:, k], w) and torch.equal(R[:, k], r)
