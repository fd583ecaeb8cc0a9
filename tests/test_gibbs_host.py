"""Host-side Gibbs pieces (no GPU): moral-graph colouring from the C ABI, and the
dense oracle's self-consistency (the colour sweep leaves N(P^-1 b, P^-1) invariant)."""
import numpy as np
import pytest

from oracle import nngp_gibbs_oracle as G


def _reverse(nbr):
    n, m = nbr.shape
    entries = sorted((int(nbr[j, s]), j, s) for j in range(n) for s in range(m) if nbr[j, s] >= 0)
    off = np.zeros(n + 1, np.int64)
    for i, _, _ in entries:
        off[i + 1] += 1
    return np.cumsum(off).astype(np.int32), np.array([e[1] for e in entries], np.int32)


@pytest.mark.parametrize("n,m", [(1, 3), (50, 1), (600, 5), (2000, 15)])
def test_colouring_is_proper(c_oracle, n, m):
    from pynngp_amd import _lib

    rng = np.random.default_rng(n + m)
    nbr = c_oracle.c_knn_prior(rng.uniform(size=(n, 2)), m)
    off, rev_j = _reverse(nbr)
    colors, nc = _lib.color_moral_graph(nbr, off, rev_j)
    assert colors.min() == 0 and colors.max() == nc - 1
    assert G.coloring_is_valid(nbr, colors)
    # greedy in index order: bounded by max moral degree + 1
    assert nc <= m * (m + 1) + 1


def test_colour_sweep_invariant_law():
    """Exact check of the dense oracle: mean and covariance map of one colour sweep."""
    from oracle import nngp_oracle as O

    rng = np.random.default_rng(3)
    n, m = 12, 3
    c = rng.uniform(size=(n, 2))
    nbr = O.knn_prior(c, m)
    B, F = O.bf_sweep(c, nbr, "exponential", (1.0, 5.0, 0.0))[:2]
    P = G.precision(nbr, B, F) + np.eye(n) / 0.3
    b = rng.standard_normal(n)
    off, rev_j = _reverse(nbr)
    colors = np.zeros(n, np.int32)
    for i in range(n):  # simple greedy on the dense moral graph
        used = {colors[j] for j in range(i) if (min(i, j), max(i, j)) in G.moral_edges(nbr)}
        colors[i] = min(set(range(n)) - used)
    assert G.coloring_is_valid(nbr, colors)
    # the sweep is affine in (w, z): w' = A w + C z + d; stationarity of N(mu, S)
    mu = np.linalg.solve(P, b)
    S = np.linalg.inv(P)
    d = G.color_sweep(P, b, np.zeros(n), colors, np.zeros(n))
    A = np.stack([G.color_sweep(P, b, e, colors, np.zeros(n)) - d for e in np.eye(n)], 1)
    C = np.stack([G.color_sweep(P, b, np.zeros(n), colors, e) - d for e in np.eye(n)], 1)
    np.testing.assert_allclose(A @ mu + d, mu, rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(A @ S @ A.T + C @ C.T, S, rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("n,m", [(300, 4), (2000, 10)])
def test_colouring_after_relabelling(c_oracle, n, m):
    """SeqNNGP relabels locations into a spatial storage order, after which a child can
    precede its parents: the greedy colouring must still be proper."""
    from pynngp_amd import _lib

    rng = np.random.default_rng(7 + n)
    nbr0 = c_oracle.c_knn_prior(rng.uniform(size=(n, 2)), m)
    perm = rng.permutation(n)
    pos = np.empty(n, np.int64)
    pos[perm] = np.arange(n)
    nb = nbr0[perm]
    nbr = np.where(nb >= 0, pos[np.maximum(nb, 0)], -1).astype(np.int32)
    off, rev_j = _reverse(nbr)
    colors, nc = _lib.color_moral_graph(nbr, off, rev_j)
    assert G.coloring_is_valid(nbr, colors)


@pytest.mark.parametrize("n_s,n_out,m", [(1, 5, 3), (60, 40, 4), (500, 400, 10)])
def test_reference_dag_colouring(c_oracle, n_s, n_out, m):
    """S != T: the DAG of reference points plus leaf data locations (nngp.py:49-71) is
    coloured properly, with every leaf in the one last colour (update_wt's step)."""
    from pynngp_amd.gibbs import colour_dag

    rng = np.random.default_rng(n_s + n_out)
    _, nbr = G.reference_dag(rng.uniform(size=(n_s, 2)), rng.uniform(size=(n_out, 2)), m)
    off, rev_j = _reverse(nbr)
    colors, nc, nc_ref = colour_dag(nbr, off, rev_j, n_s)
    assert nc == nc_ref + 1 and np.all(colors[n_s:] == nc_ref) and colors[:n_s].max() == nc_ref - 1
    assert G.coloring_is_valid(nbr, colors)


def test_reference_dag_sweep_invariant_law(c_oracle):
    """The colour sweep over the reference-set DAG (leaves first: update_wt, then the
    reference colours: update_ws), with observations on some leaves and on some reference
    points, leaves the exact posterior N(P^-1 b, P^-1) invariant."""
    from pynngp_amd.gibbs import colour_dag

    rng = np.random.default_rng(5)
    n_s, n_out, m = 10, 8, 3
    coords, nbr = G.reference_dag(rng.uniform(size=(n_s, 2)), rng.uniform(size=(n_out, 2)), m)
    n = n_s + n_out
    B, F, _ = c_oracle.c_bf_sweep(coords, nbr, "exponential", (1.0, 4.0, 0.0))
    h = np.zeros(n)
    h[[1, 4, 7]] = 1.0  # three reference points carry data
    h[n_s:] = rng.uniform(0.5, 2.0, n_out)
    h[n_s + 2] = 0.0  # an unobserved data location
    P, b, mu, S = G.dag_posterior(nbr, B, F, 1.3, 0.4, h, rng.standard_normal(n))
    off, rev_j = _reverse(nbr)
    colors, nc, nc_ref = colour_dag(nbr, off, rev_j, n_s)
    order = np.where(colors == nc_ref, 0, colors + 1)  # the leaves' colour step first
    d = G.color_sweep(P, b, np.zeros(n), order, np.zeros(n))
    A = np.stack([G.color_sweep(P, b, e, order, np.zeros(n)) - d for e in np.eye(n)], 1)
    C = np.stack([G.color_sweep(P, b, np.zeros(n), order, e) - d for e in np.eye(n)], 1)
    np.testing.assert_allclose(A @ mu + d, mu, rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(A @ S @ A.T + C @ C.T, S, rtol=1e-9, atol=1e-12)
