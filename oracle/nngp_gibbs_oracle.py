"""Dense-algebra oracle for the NNGP Gibbs sampler (TEST INFRASTRUCTURE ONLY).

The reference's sampler (``NNGP.oneSample``, pyNNGP/nngp.py:98-101) calls methods
that do not exist, so the sampler is "parity unpinned" by the reference.  This
restates the model's full conditionals with dense matrices (N small):

    Q = (I - B)^T F^{-1} (I - B)          NNGP precision of w (B (N,N) from the rows)
    P = Q + I / tau2,  b = (y - X beta) / tau2
    w_i | w_-i ~ N((b_i - sum_{k != i} P_ik w_k) / P_ii, 1 / P_ii)
    posterior w | y, theta ~ N(P^-1 b, P^-1)

and checks colourings of the moral graph.
"""
import numpy as np


def dense_B(nbr, B_rows):
    n, m = nbr.shape
    Bd = np.zeros((n, n))
    for i in range(n):
        for s in range(m):
            j = nbr[i, s]
            if j >= 0:
                Bd[i, j] = B_rows[i, s]
    return Bd


def precision(nbr, B_rows, F):
    n = nbr.shape[0]
    IB = np.eye(n) - dense_B(nbr, B_rows)
    return IB.T @ np.diag(1.0 / F) @ IB


def color_sweep(P, b, w, colors, z):
    """One colour-ordered sweep with given normals z (mirrors nngp_gibbs_w_sweep)."""
    w = w.copy()
    for c in range(int(colors.max()) + 1 if colors.size else 0):
        idx = np.nonzero(colors == c)[0]
        new = {}
        for i in idx:  # members of one colour are conditionally independent
            prec = P[i, i]
            mean = (b[i] - (P[i] @ w - P[i, i] * w[i])) / prec
            new[i] = mean + z[i] / np.sqrt(prec)
        for i, v in new.items():
            w[i] = v
    return w


def moral_edges(nbr):
    n, m = nbr.shape
    E = set()
    for j in range(n):
        par = [int(k) for k in nbr[j] if k >= 0]
        for k in par:
            E.add((min(j, k), max(j, k)))
        for a in par:
            for b in par:
                if a < b:
                    E.add((a, b))
    return E


def coloring_is_valid(nbr, colors):
    return all(colors[a] != colors[b] for a, b in moral_edges(nbr))


# ---------------------------------------------------------------- S != T (reference set)
def reference_dag(s, t_out, m):
    """The DAG of the reference-set model (nngp.py:42-71; TEST INFRASTRUCTURE ONLY): nodes
    [S; T_out]; a reference point's parents are the min(i, m) nearest earlier points of S
    (``_make_s_neighbor_sets``), a data location outside S is a leaf whose parents are its
    m nearest points of S (``_make_t_neighbor_sets``, kdtree.query(t, m) over all of S).
    Returns (coords (n_s + n_out, d), nbr (n_s + n_out, m) int32, -1 padded)."""
    from oracle import nngp_oracle as O

    s = np.asarray(s, dtype=np.float64)
    t_out = np.asarray(t_out, dtype=np.float64)
    nbr_s = O.c_knn_prior(s, m)
    k = min(m, len(s))
    nbr_t = np.full((len(t_out), m), -1, dtype=np.int32)
    if len(t_out):
        nbr_t[:, :k] = O.knn_all(t_out, s, k)
    return np.concatenate([s, t_out]), np.concatenate([nbr_s, nbr_t]).astype(np.int32)


def dag_posterior(nbr, B, F, sigma2, tau2, h, yres):
    """Exact Gaussian full posterior of w over the DAG's nodes: precision
    P = (I - B)^T (sigma2 F)^-1 (I - B) + diag(h / tau2), linear term b = h yres / tau2
    (h = 0 at nodes without an observation).  Returns (P, b, mean, cov)."""
    P = precision(nbr, B, F * sigma2) + np.diag(np.asarray(h) / tau2)
    b = np.asarray(h) * np.asarray(yres) / tau2
    cov = np.linalg.inv(P)
    return P, b, cov @ b, cov
