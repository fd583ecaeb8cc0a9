"""CPU oracle for the NNGP neighbour-set + B/F + log-likelihood path.

TEST INFRASTRUCTURE ONLY.  Nothing in ``pynngp_amd`` imports this module; only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
use it, and only as the checker / the timed CPU baseline -- never as the thing
measured or shipped.

What it restates (reference = ``bwpriest/pyNNGP`` at ``/root/reference``):

* ``knn_prior`` -- ``NNGP._make_s_neighbor_sets`` (``pyNNGP/nngp.py:49-62``): for
  every i the ``min(m, i)`` nearest points among ``s[0:i]``, ascending distance,
  self excluded, ``Ns[0] == []``.  The reference delegates to sklearn 1.7.2
  ``KDTree.query(k, sort_results=True)`` whose ordering key is the fp64 reduced
  distance ``rdist = (0 + t0*t0) + t1*t1`` with ``t = x_query - x_tree`` and no
  FMA (``sklearn/metrics/_dist_metrics.pxd:26-40``).  Exact ties are broken by
  the lower index here (the reference's tie order is arbitrary:
  ``sklearn/utils/_heap.pyx:45-47``); pinned by ``tests/golden/knn_ref_*.npz``.
* ``bf_sweep`` -- the per-location algebra the reference stubs out:
  ``_CNs`` (``nngp.py:78-82``), ``_Ccross`` (``nngp.py:84-86``), ``_Cs``
  (``nngp.py:92-96``), ``_Bsi`` (``nngp.py:73-76``), ``_Fsi`` (``nngp.py:88-90``),
  with the NNGP definitions named by those docstrings (Datta et al. 2016;
  SURVEY.md Appendix A)::

      C_N  = [C(s_a, s_b)]_{a,b in N(i)} + tau2 I
      c    = [C(s_i, s_b)]_{b in N(i)}
      C_ii = sigma2 + tau2
      B_i  = c^T C_N^{-1}          F_i = C_ii - c^T C_N^{-1} c
      log p(v) = -1/2 sum_i [log 2pi + log F_i + (v_i - B_i v_N(i))^2 / F_i]

  B/F/log-lik are "parity unpinned" by the reference (its methods return None);
  this restatement is pinned by known answers instead (``tests/test_oracle.py``):
  m = N-1 equals the dense-GP log density, m = 0 the independent normal, and the
  result is invariant to permuting a neighbour set.

* ``c_bf_cross`` / ``dense_kriging`` -- B_t, F_t of points t outside the reference set
  S against their neighbours in S (the reference builds
  ``Nt = KDTree(s).query(t, m)`` at ``nngp.py:64-71`` but never evaluates B_t/F_t):
  the same algebra with the location row taken from t; parity unpinned by the
  reference, anchored by the dense GP conditional (``dense_kriging``) at m = |S|.

Covariance kinds (the reference's ``cov`` plug-in, ``nngp.py:6,12``; u = phi d, d the
Euclidean distance in fp64 over any number of coordinate columns -- the reference's
KDTree takes ordinates of any dimension, ``nngp.py:55-61``):
``exponential`` sigma2 e^-u; ``matern32`` sigma2 (1 + u) e^-u; ``matern52``
sigma2 (1 + u + u^2/3) e^-u; ``gaussian`` sigma2 e^-u^2; ``spherical``
sigma2 (1 - 3u/2 + u^3/2) for u < 1, else 0 (the spNNGP family); ``matern`` (general
smoothness nu, theta = (sigma2, phi, tau2, nu)) sigma2 u^nu K_nu(u) / (2^(nu-1) Gamma(nu)) through
scipy.special.kv (AMOS) here and a long-double trapezoidal integral in the C restatement.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

KINDS = {"exponential": 0, "matern32": 1, "matern52": 2, "gaussian": 3, "spherical": 4, "matern": 5}
LOG_2PI = float(np.log(2.0 * np.pi))
_HERE = os.path.dirname(os.path.abspath(__file__))


# ----------------------------------------------------------------------------
# neighbour sets (nngp.py:49-62)
# ----------------------------------------------------------------------------
def rdist(t: np.ndarray) -> np.ndarray:
    """sklearn euclidean_rdist64 of difference rows t (..., dim): d = 0; d += t_k * t_k in
    axis order (``_dist_metrics.pxd:26-40``); separate ufuncs, so no FMA contraction."""
    d = np.zeros(t.shape[:-1])
    for k in range(t.shape[-1]):
        d = d + t[..., k] * t[..., k]
    return d


def rdist_to_prior(coords: np.ndarray, i: int) -> np.ndarray:
    """rdist of s_i against s[0:i]."""
    return rdist(coords[i][None, :] - coords[:i])


def knn_prior(coords: np.ndarray, m: int, q0: int = 0, q1: int | None = None) -> np.ndarray:
    """Ordered prior nearest neighbours, int32 (q1-q0, m) padded with -1."""
    coords = np.ascontiguousarray(coords, dtype=np.float64)
    n = coords.shape[0]
    q1 = n if q1 is None else q1
    out = np.full((q1 - q0, m), -1, dtype=np.int32)
    for i in range(q0, q1):
        if i == 0 or m == 0:
            continue
        d = rdist_to_prior(coords, i)
        k = min(m, i)
        if k < i:
            part = np.argpartition(d, k - 1)[:k]
            # include every index tied with the k-th value so (rdist, idx) order is exact
            kth = d[part].max()
            cand = np.nonzero(d <= kth)[0]
        else:
            cand = np.arange(i)
        order = np.lexsort((cand, d[cand]))[:k]
        out[i - q0, :k] = cand[order]
    return out


def knn_all(query: np.ndarray, ref: np.ndarray, k: int) -> np.ndarray:
    """k nearest of every query among all ref points (self included), (rdist, idx) order."""
    out = np.empty((query.shape[0], k), dtype=np.int64)
    for q in range(query.shape[0]):
        d = rdist(query[q][None, :] - ref)
        out[q] = np.lexsort((np.arange(ref.shape[0]), d))[:k]
    return out


def ws_init(t: np.ndarray, y: np.ndarray, s: np.ndarray, k: int = 5) -> np.ndarray:
    """``_init_ws`` (``nngp.py:45-47``): uniform k-NN regression of y on t at s."""
    idx = knn_all(s, t, k)
    return y[idx].mean(axis=1)


# ----------------------------------------------------------------------------
# covariance plug-in and per-location algebra (nngp.py:73-96)
# ----------------------------------------------------------------------------
def _theta(theta):
    """(sigma2, phi, tau2, nu): theta = (sigma2, phi, tau2) or, for the ``matern`` kind, (..., nu)."""
    return float(theta[0]), float(theta[1]), float(theta[2]), (float(theta[3]) if len(theta) > 3 else None)


def matern_rho(nu: float, u: np.ndarray) -> np.ndarray:
    """u^nu K_nu(u) / (2^(nu-1) Gamma(nu)) (1 at u = 0) with scipy's K_nu."""
    from scipy import special
    u = np.asarray(u, dtype=np.float64)
    us = np.where(u > 0, u, 1.0)
    with np.errstate(invalid="ignore", over="ignore", under="ignore", divide="ignore"):
        k = special.kv(nu, us)
        r = np.exp(nu * np.log(us) - (nu - 1.0) * np.log(2.0) - special.gammaln(nu) + np.log(k))
    # K_nu overflows only for u so small (nu > 1/2) that 1 - rho ~ u^2 is far below an ulp
    return np.where((u > 0) & np.isfinite(k), r, 1.0)


def cov_fn(kind: str, d: np.ndarray, sigma2: float, phi: float, nu: float | None = None) -> np.ndarray:
    """The covariance kinds, u = phi d (module docstring)."""
    u = phi * np.asarray(d, dtype=np.float64)
    if kind == "matern":
        return sigma2 * matern_rho(nu, u)
    if kind == "exponential":
        return sigma2 * np.exp(-u)
    if kind == "matern32":
        return sigma2 * (1.0 + u) * np.exp(-u)
    if kind == "matern52":
        return sigma2 * (1.0 + u + u * u / 3.0) * np.exp(-u)
    if kind == "gaussian":
        return sigma2 * np.exp(-u * u)
    if kind == "spherical":
        return np.where(u < 1.0, sigma2 * (1.0 - 1.5 * u + 0.5 * u * u * u), 0.0)
    raise ValueError(f"unknown covariance kind {kind!r}")


def _pair_dist(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    return np.sqrt(rdist(a - b))


def location_blocks(coords, nbr_row, i, kind, theta):
    """(C_N, c, C_ii) for one location: ``_CNs``, ``_Ccross``, ``_Cs``."""
    sigma2, phi, tau2, nu = _theta(theta)
    idx = nbr_row[nbr_row >= 0].astype(np.int64)
    xs = coords[idx]
    CN = cov_fn(kind, _pair_dist(xs[:, None, :], xs[None, :, :]), sigma2, phi, nu)
    CN = CN + tau2 * np.eye(idx.size)
    c = cov_fn(kind, _pair_dist(coords[i][None, :], xs), sigma2, phi, nu)
    return CN, c, sigma2 + tau2


def bf_location(coords, nbr_row, i, kind, theta):
    """(B_i over the valid slots, F_i) by Cholesky, ``_Bsi`` / ``_Fsi``."""
    CN, c, Cii = location_blocks(coords, nbr_row, i, kind, theta)
    if c.size == 0:
        return np.zeros(0), Cii
    L = np.linalg.cholesky(CN)
    v = np.linalg.solve(L, c)
    B = np.linalg.solve(L.T, v)
    return B, Cii - v @ v


def bf_sweep(coords, nbr, kind, theta, values=None, i0=0):
    """Batched fp64 restatement over rows ``i0 .. i0+len(nbr)``.

    Returns ``(B (n, m) padded with 0, F (n,), partials)`` with
    ``partials = [sum log F, sum r^2/F]`` (r = v_i - B_i v_N(i); 0 without values).
    Rows are grouped by their valid-neighbour pattern so numpy's batched
    Cholesky does the work; the math is the per-location ``bf_location``.
    """
    coords = np.ascontiguousarray(coords, dtype=np.float64)
    nbr = np.ascontiguousarray(nbr, dtype=np.int32)
    n, m = nbr.shape
    sigma2, phi, tau2, nu = _theta(theta)
    B = np.zeros((n, m))
    F = np.empty(n)
    valid = nbr >= 0
    k_row = valid.sum(axis=1)
    # rows whose valid slots are not a prefix are handled one by one
    prefix = np.all(valid == (np.arange(m)[None, :] < k_row[:, None]), axis=1)
    rows_i = np.arange(n) + i0
    for k in np.unique(k_row[prefix]):
        sel = np.nonzero(prefix & (k_row == k))[0]
        if k == 0:
            F[sel] = sigma2 + tau2
            continue
        idx = nbr[sel, :k].astype(np.int64)
        xs = coords[idx]  # (b, k, 2)
        CN = cov_fn(kind, _pair_dist(xs[:, :, None, :], xs[:, None, :, :]), sigma2, phi, nu)
        CN = CN + tau2 * np.eye(k)[None]
        c = cov_fn(kind, _pair_dist(coords[rows_i[sel]][:, None, :], xs), sigma2, phi, nu)
        L = np.linalg.cholesky(CN)
        v = np.linalg.solve(L, c[..., None])
        Bk = np.linalg.solve(np.swapaxes(L, 1, 2), v)[..., 0]
        B[sel, :k] = Bk
        F[sel] = (sigma2 + tau2) - np.einsum("bi,bi->b", v[..., 0], v[..., 0])
    for r in np.nonzero(~prefix)[0]:
        Bi, Fi = bf_location(coords, nbr[r], rows_i[r], kind, theta)
        B[r, valid[r]] = Bi
        F[r] = Fi
    logF = np.log(F)
    if values is None:
        quad = np.zeros(n)
    else:
        values = np.asarray(values, dtype=np.float64)
        vn = np.where(valid, values[np.where(valid, nbr, 0)], 0.0)
        resid = values[rows_i] - np.einsum("bi,bi->b", B, vn)
        quad = resid * resid / F
    partials = np.array([logF.sum(), quad.sum()])
    return B, F, partials


def bf_sweep_callable(coords, nbr, cov, values=None, i0=0, qcoords=None, qvalues=None):
    """The same algebra with the reference's plug-in ``cov(a, b)`` as it is called there: on the
    neighbours' coordinate rows, ``C_N = cov(X_N, X_N)`` (``_CNs``, ``nngp.py:78-82``, with rows
    where the reference passes indices), ``c = cov(x_i, X_N)`` (``_Ccross``, ``nngp.py:84-86``) and
    ``C_ii = cov(x_i, x_i)`` (``_Cs``, ``nngp.py:92-96``), then one dense solve per location
    (``np.linalg.solve``, not a Cholesky: an independent route to ``_Bsi`` / ``_Fsi``,
    ``nngp.py:73-76,88-90``): B_i = C_N^{-1} c, F_i = C_ii - c^T B_i, r_i = v_i - B_i v_N(i).
    ``qcoords`` given: the locations are those points (prediction; ``qvalues`` their values).
    Returns ``(B (n, m) padded with 0, F (n,), partials [sum log F, sum r^2/F])``.  Plain
    per-location Python: for the small parity cases only."""
    coords = np.ascontiguousarray(coords, dtype=np.float64)
    nbr = np.asarray(nbr)
    q = coords if qcoords is None else np.ascontiguousarray(qcoords, dtype=np.float64)
    qv = values if qcoords is None else qvalues
    n, m = nbr.shape
    B = np.zeros((n, m))
    F = np.empty(n)
    resid = np.zeros(n)
    for r in range(n):
        i = i0 + r
        ok = (nbr[r] >= 0) & (nbr[r] < coords.shape[0])
        idx = nbr[r][ok].astype(np.int64)
        xi = q[i][None, :]
        Cii = float(np.asarray(cov(xi, xi)).reshape(-1)[0])
        if idx.size == 0:
            F[r] = Cii
            b = np.zeros(0)
        else:
            xs = coords[idx]
            CN = np.asarray(cov(xs, xs), dtype=np.float64).reshape(idx.size, idx.size)
            c = np.asarray(cov(xi, xs), dtype=np.float64).reshape(idx.size)
            b = np.linalg.solve(CN, c)
            B[r, ok] = b
            F[r] = Cii - c @ b
        if values is not None:
            vi = 0.0 if qv is None else float(np.asarray(qv)[i])
            resid[r] = vi - (b @ np.asarray(values)[idx] if idx.size else 0.0)
    partials = np.array([np.log(F).sum(), (resid * resid / F).sum()])
    return B, F, partials


def loglik_from_partials(partials, n):
    return -0.5 * (n * LOG_2PI + partials[0] + partials[1])


def nngp_loglik(coords, nbr, kind, theta, values):
    _, _, p = bf_sweep(coords, nbr, kind, theta, values)
    return loglik_from_partials(p, nbr.shape[0])


def dense_gp_loglik(coords, kind, theta, values):
    """Exact GP log density (known answer for m = N-1)."""
    sigma2, phi, tau2, nu = _theta(theta)
    d = _pair_dist(coords[:, None, :], coords[None, :, :])
    C = cov_fn(kind, d, sigma2, phi, nu) + tau2 * np.eye(coords.shape[0])
    L = np.linalg.cholesky(C)
    z = np.linalg.solve(L, values)
    n = coords.shape[0]
    return -0.5 * (n * LOG_2PI + 2.0 * np.log(np.diag(L)).sum() + z @ z)


# ----------------------------------------------------------------------------
# C restatement (oracle/nngp_oracle.c) through ctypes
# ----------------------------------------------------------------------------
_C = None


def c_oracle_path() -> str:
    return os.path.join(_HERE, "_build", "libnngp_oracle.so")


def build_c_oracle() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return c_oracle_path()


def load_c_oracle():
    global _C
    if _C is not None:
        return _C
    path = c_oracle_path()
    if not os.path.exists(path):
        build_c_oracle()
    lib = ctypes.CDLL(path)
    P = ctypes.c_void_p
    I32, I64 = ctypes.c_int32, ctypes.c_int64
    lib.oracle_knn_prior.argtypes = [P, I64, I32, I32, I64, I64, P]
    lib.oracle_knn_prior.restype = ctypes.c_int
    lib.oracle_knn_prior_rows.argtypes = [P, I64, I32, I32, P, I64, P]
    lib.oracle_knn_prior_rows.restype = ctypes.c_int
    lib.oracle_knn_prior_kdtree_rebuild.argtypes = [P, I64, I32, I32, I64, I64, P]
    lib.oracle_knn_prior_kdtree_rebuild.restype = ctypes.c_int
    lib.oracle_knn_prior_prefix_kdtree.argtypes = [P, I64, I32, I32, I64, I64, P]
    lib.oracle_knn_prior_prefix_kdtree.restype = ctypes.c_int
    lib.oracle_bf_sweep.argtypes = [P, P, I64, I32, I32, I32, P, P, P, P, P, I64, I64]
    lib.oracle_bf_sweep.restype = ctypes.c_int
    lib.oracle_num_threads.restype = ctypes.c_int
    lib.oracle_matern_rho.argtypes = [ctypes.c_double, ctypes.c_double]
    lib.oracle_matern_rho.restype = ctypes.c_double
    lib.oracle_nngp_simulate.argtypes = [P, P, P, ctypes.c_int64, ctypes.c_int32, P, P]
    lib.oracle_nngp_simulate.restype = ctypes.c_int
    _C = lib
    return lib


def _dim(coords):
    if coords.ndim != 2 or coords.shape[1] < 1:
        raise ValueError(f"coordinates must be (n, dim), got {coords.shape}")
    return coords.shape[1]


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


def c_knn_prior(coords, m, q0=0, q1=None):
    lib = load_c_oracle()
    coords = np.ascontiguousarray(coords, dtype=np.float64)
    n = coords.shape[0]
    q1 = n if q1 is None else q1
    out = np.full((q1 - q0, m), -1, dtype=np.int32)
    rc = lib.oracle_knn_prior(_ptr(coords), n, _dim(coords), m, q0, q1, _ptr(out))
    if rc != 0:
        raise RuntimeError(f"oracle_knn_prior failed: {rc}")
    return out


def c_knn_prior_kdtree_rebuild(coords, m, q0=0, q1=None):
    """The reference's algorithm (a fresh kd-tree over s[0:i] per i, nngp.py:55-61),
    single-threaded C: the CPU baseline of the neighbour build.  Same output as c_knn_prior."""
    lib = load_c_oracle()
    coords = np.ascontiguousarray(coords, dtype=np.float64)
    n = coords.shape[0]
    q1 = n if q1 is None else q1
    out = np.full((q1 - q0, m), -1, dtype=np.int32)
    rc = lib.oracle_knn_prior_kdtree_rebuild(_ptr(coords), n, _dim(coords), m, q0, q1, _ptr(out))
    if rc != 0:
        raise RuntimeError(f"oracle_knn_prior_kdtree_rebuild failed: {rc}")
    return out


def c_knn_prior_prefix_kdtree(coords, m, q0=0, q1=None):
    """Exact prior sets through kd-trees over doubling prefixes s[0:2^k] (query i searches the
    smallest prefix holding s[0:i] and skips j >= i), OpenMP over queries: an independent
    check of the GPU grid search that is fast enough for every row at N = 1e7.  Same output
    as c_knn_prior (nngp.py:49-62 key; ties by lower index)."""
    lib = load_c_oracle()
    coords = np.ascontiguousarray(coords, dtype=np.float64)
    n = coords.shape[0]
    q1 = n if q1 is None else q1
    out = np.full((q1 - q0, m), -1, dtype=np.int32)
    rc = lib.oracle_knn_prior_prefix_kdtree(_ptr(coords), n, _dim(coords), m, q0, q1, _ptr(out))
    if rc != 0:
        raise RuntimeError(f"oracle_knn_prior_prefix_kdtree failed: {rc}")
    return out


def c_knn_prior_rows(coords, m, rows):
    """Prior neighbour sets of the locations ``rows`` (any order), one row each, in parallel."""
    lib = load_c_oracle()
    coords = np.ascontiguousarray(coords, dtype=np.float64)
    rows = np.ascontiguousarray(rows, dtype=np.int64)
    out = np.full((rows.size, m), -1, dtype=np.int32)
    rc = lib.oracle_knn_prior_rows(_ptr(coords), coords.shape[0], _dim(coords), m, _ptr(rows), rows.size, _ptr(out))
    if rc != 0:
        raise RuntimeError(f"oracle_knn_prior_rows failed: {rc}")
    return out


def c_bf_sweep(coords, nbr, kind, theta, values=None, i0=0, want_bf=True):
    """C restatement; returns (B, F, partials[3]) with partials[2] = first bad row or -1."""
    lib = load_c_oracle()
    coords = np.ascontiguousarray(coords, dtype=np.float64)
    nbr = np.ascontiguousarray(nbr, dtype=np.int32)
    n, m = nbr.shape
    th = np.ascontiguousarray(theta, dtype=np.float64)
    vals = None if values is None else np.ascontiguousarray(values, dtype=np.float64)
    B = np.zeros((n, m)) if want_bf else None
    F = np.zeros(n) if want_bf else None
    partials = np.zeros(3)
    rc = lib.oracle_bf_sweep(_ptr(coords), _ptr(nbr), coords.shape[0], _dim(coords), m, KINDS[kind], _ptr(th), _ptr(vals),
                             _ptr(B), _ptr(F), _ptr(partials), i0, i0 + n)
    if rc != 0:
        raise RuntimeError(f"oracle_bf_sweep failed: {rc}")
    return B, F, partials


def c_matern_rho(nu: float, u: float) -> float:
    """The C restatement's Matern correlation (long-double trapezoidal integral)."""
    return load_c_oracle().oracle_matern_rho(float(nu), float(u))


def c_nngp_simulate(nbr, B, F, eps):
    """w ~ NNGP by forward substitution (oracle_nngp_simulate): w_i = B_i w_N(i) + sqrt(F_i) eps_i."""
    lib = load_c_oracle()
    nbr = np.ascontiguousarray(nbr, dtype=np.int32)
    n, m = nbr.shape
    B = np.ascontiguousarray(B, dtype=np.float64)
    F = np.ascontiguousarray(F, dtype=np.float64)
    eps = np.ascontiguousarray(eps, dtype=np.float64)
    w = np.zeros(n)
    rc = lib.oracle_nngp_simulate(_ptr(nbr), _ptr(B), _ptr(F), n, m, _ptr(eps), _ptr(w))
    if rc != 0:
        raise RuntimeError(f"oracle_nngp_simulate failed: {rc}")
    return w


def c_bf_cross(ref, query, nbr, kind, theta, ref_values=None, query_values=None, q0=0):
    """B_t, F_t (and partials) of query rows q0 .. q0+len(nbr) against ``ref``: the C sweep
    on the stacked coordinates [ref; query] with location rows n_ref + q (neighbour indices
    already point into ref).  Missing query values are 0 (R = -kriging mean)."""
    ref = np.ascontiguousarray(ref, dtype=np.float64)
    query = np.ascontiguousarray(query, dtype=np.float64)
    both = np.concatenate([ref, query])
    vals = None
    if ref_values is not None:
        qv = np.zeros(len(query)) if query_values is None else np.asarray(query_values, dtype=np.float64)
        vals = np.concatenate([np.asarray(ref_values, dtype=np.float64), qv])
    return c_bf_sweep(both, nbr, kind, theta, vals, i0=len(ref) + q0)


def dense_kriging(ref, query, kind, theta, ref_values=None):
    """Exact GP conditional of the query points given ALL of ref (numpy solve):
    B = C(t, S) (C(S) + tau2 I)^{-1}, F = sigma2 + tau2 - B C(S, t), mean = B v_S."""
    sigma2, phi, tau2, nu = _theta(theta)
    Css = cov_fn(kind, _pair_dist(ref[:, None, :], ref[None, :, :]), sigma2, phi, nu) + tau2 * np.eye(len(ref))
    Cts = cov_fn(kind, _pair_dist(query[:, None, :], ref[None, :, :]), sigma2, phi, nu)
    B = np.linalg.solve(Css, Cts.T).T
    F = sigma2 + tau2 - np.einsum("ij,ij->i", B, Cts)
    mean = None if ref_values is None else B @ np.asarray(ref_values, dtype=np.float64)
    return B, F, mean
