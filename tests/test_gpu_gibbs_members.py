"""GPU: the one-GPU chain's member records (nngp_gibbs_prepare_members / nngp_gibbs_member_draws /
nngp_gibbs_w_sweep_members).  They hold P_i, 1/F_i, yres_i and z_i in colour-member order so a colour
step reads them with one coalesced load; the values -- and so the chain -- must be bit-identical to
the node-order path (nngp_gibbs_prepare / nngp_gibbs_normals / nngp_gibbs_w_sweep), which the sharded
chain and the dense-oracle tests (test_gpu_gibbs.py) use."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _a256(x):
    return (x + 255) & ~255


def _problem(dev, n, m, seed=0, weighted=False):
    from pynngp_amd import _lib

    rng = np.random.default_rng(seed)
    c = torch.from_numpy(rng.uniform(size=(n, 2))).to(dev)
    nbr = _lib.knn_prior(c, m)
    w = torch.from_numpy(rng.standard_normal(n)).to(dev)
    R = torch.empty(n, dtype=torch.float64, device=dev)
    B, F, _ = _lib.bf_sweep(c, nbr, 0, "exponential", 1.0, 9.0, 0.0, values=w, R=R)
    off, rev_j, rev_k = _lib.reverse_neighbors(nbr)
    colors, nc = _lib.color_moral_graph(nbr.cpu().numpy(), off.cpu().numpy(), rev_j.cpu().numpy())
    members = torch.from_numpy(np.argsort(colors, kind="stable").astype(np.int32)).to(dev)
    color_off = np.concatenate([[0], np.cumsum(np.bincount(colors, minlength=nc))]).astype(np.int32)
    yres = torch.from_numpy(rng.standard_normal(n)).to(dev)
    nw = torch.from_numpy(rng.uniform(0.5, 2.0, n)).to(dev) if weighted else None
    return dict(n=n, m=m, c=c, nbr=nbr, w=w, R=R, B=B, F=F, off=off, rev_j=rev_j, rev_k=rev_k, members=members,
                color_off=color_off, yres=yres, nw=nw)


@pytest.mark.parametrize("n,m", [(1, 3), (700, 1), (5000, 10), (20000, 15)])
def test_member_records_equal_node_arrays(dev, n, m):
    from pynngp_amd import _lib

    s = _problem(dev, n, m, seed=n)
    prep = _lib.gibbs_prepare(s["B"], s["F"], s["off"], s["rev_j"], s["rev_k"])
    mr = _lib.gibbs_member_rows(s["members"], s["off"])
    mrec = torch.full((n, 4), float("nan"), dtype=torch.float64, device=dev)
    prep2 = _lib.gibbs_prepare_members(s["B"], s["F"], s["off"], s["rev_j"], s["rev_k"], mr, mrec)
    # prep layout: Brev, Grev (n m each), P, 1/F (n each), 256-B aligned
    nm = _a256(n * m * 8) // 8
    raw = prep.view(torch.float64) if prep.dtype != torch.float64 else prep
    raw2 = prep2.view(torch.float64) if prep2.dtype != torch.float64 else prep2
    ne = int(s["off"][-1])  # the reverse entries (rows before m have fewer than m parents: a tail is unused)
    assert torch.equal(raw[:ne], raw2[:ne]) and torch.equal(raw[nm:nm + ne], raw2[nm:nm + ne])  # the same pass
    P = raw[2 * nm: 2 * nm + n]
    invF = raw[2 * nm + _a256(n * 8) // 8: 2 * nm + _a256(n * 8) // 8 + n]
    mem = s["members"].long()
    assert torch.equal(mrec[:, 0], P[mem]) and torch.equal(mrec[:, 1], invF[mem])
    z = _lib.gibbs_normals(torch.empty(n, dtype=torch.float64, device=dev), 77, 5)
    _lib.gibbs_member_draws(mr, s["yres"], 77, 5, mrec)
    assert torch.equal(mrec[:, 2], s["yres"][mem]) and torch.equal(mrec[:, 3], z[mem])


@pytest.mark.parametrize("weighted", [False, True])
def test_member_sweep_bit_identical(dev, weighted):
    from pynngp_amd import _lib

    n, m = 30000, 15
    s = _problem(dev, n, m, seed=3, weighted=weighted)
    mr = _lib.gibbs_member_rows(s["members"], s["off"])
    w1, r1 = s["w"].clone(), s["R"].clone()
    w2, r2 = s["w"].clone(), s["R"].clone()
    prep = _lib.gibbs_prepare(s["B"], s["F"], s["off"], s["rev_j"], s["rev_k"])
    mrec = torch.empty((n, 4), dtype=torch.float64, device=dev)
    prep2 = _lib.gibbs_prepare_members(s["B"], s["F"], s["off"], s["rev_j"], s["rev_k"], mr, mrec)
    z = torch.empty(n, dtype=torch.float64, device=dev)
    for it in range(3):
        _lib.gibbs_normals(z, 11, it)
        _lib.gibbs_w_sweep(s["members"], s["color_off"], prep, m, 1.3, 0.2, s["yres"], w1, r1, s["off"], s["rev_j"], 11,
                           it, z=z, noise_w=s["nw"], member_rows=mr)
        _lib.gibbs_member_draws(mr, s["yres"], 11, it, mrec)
        _lib.gibbs_w_sweep_members(mr, s["color_off"], prep2, m, 1.3, 0.2, mrec, w2, r2, s["rev_j"], noise_w=s["nw"])
    assert torch.equal(w1, w2) and torch.equal(r1, r2)
    # ... and the inline-Philox path (no z) draws the same chain
    w3, r3 = s["w"].clone(), s["R"].clone()
    for it in range(3):
        _lib.gibbs_w_sweep(s["members"], s["color_off"], prep, m, 1.3, 0.2, s["yres"], w3, r3, s["off"], s["rev_j"], 11,
                           it, noise_w=s["nw"], member_rows=mr)
    assert torch.equal(w1, w3)


def test_seqnngp_member_records_vs_node_order(dev):
    """Whole iterations (phi MH with accepted proposals re-preparing, sigma2, w, tau2, beta): the chain with
    member records equals the node-order chain bit for bit."""
    from pynngp_amd import SeqNNGP

    class NodeOrder(SeqNNGP):
        _member_records = False

    rng = np.random.default_rng(5)
    n = 6000
    x = rng.uniform(size=(n, 2))
    y = 1.0 + np.sin(6 * x[:, 0]) + 0.3 * rng.standard_normal(n)
    a = SeqNNGP(x, y, m=10, phi=8.0, phi_tuning=0.3, seed=4, device=dev)
    b = NodeOrder(x, y, m=10, phi=8.0, phi_tuning=0.3, seed=4, device=dev)
    assert a._member_records and not b._member_records
    for _ in range(12):
        a.step()
        b.step()
    assert a.n_accept > 0
    assert torch.equal(a.w, b.w) and torch.equal(a.r, b.r)
    assert (a.phi, a.sigma2, a.tau2) == (b.phi, b.sigma2, b.tau2) and np.array_equal(a.beta, b.beta)


def test_member_abi_errors(dev):
    from pynngp_amd import _lib

    s = _problem(dev, 500, 5)
    mr = _lib.gibbs_member_rows(s["members"], s["off"])
    with pytest.raises(ValueError, match="mrec"):
        _lib.gibbs_prepare_members(s["B"], s["F"], s["off"], s["rev_j"], s["rev_k"], mr,
                                   torch.empty((500, 3), dtype=torch.float64, device=dev))
    with pytest.raises(ValueError, match="member_rows"):
        _lib.gibbs_member_draws(mr[:, :3].contiguous(), s["yres"], 0, 0, torch.empty((500, 4), dtype=torch.float64,
                                                                                      device=dev))
    mrec = torch.empty((500, 4), dtype=torch.float64, device=dev)
    prep = _lib.gibbs_prepare_members(s["B"], s["F"], s["off"], s["rev_j"], s["rev_k"], mr, mrec)
    with pytest.raises(Exception, match="tau2"):
        _lib.gibbs_w_sweep_members(mr, s["color_off"], prep, 5, 1.0, 0.0, mrec, s["w"], s["R"], s["rev_j"])
