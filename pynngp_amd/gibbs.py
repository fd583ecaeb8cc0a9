"""``SeqNNGP``: Gibbs sampler for the NNGP response model on the GPU.

The reference's sampler entry point is ``NNGP.oneSample`` (pyNNGP/nngp.py:98-101),
which calls ``update_wt`` / ``update_ws`` / ``update_y_unobserved`` -- none of them
exist.  This is the sampler those names describe, for the model of Datta et al.
(2016) that the reference's B/F docstrings (nngp.py:73-96) come from:

    y = X beta + w + e,   e_i ~ N(0, tau2 v_i),   w ~ NNGP(0, sigma2 R(phi))
    beta ~ flat,  sigma2 ~ IG(a_s, b_s),  tau2 ~ IG(a_t, b_t),  phi ~ U(phi_lo, phi_hi)

A covariance of the caller's own (``cov=``, the reference's plug-in ``cov(a, b)``, nngp.py:6,12) is
held fixed: its joint blocks are evaluated once and factored by the covariance-blocks kernel; phi and
sigma2 are then not sampled (the callable carries its own scale), w, tau2 and beta are.

One iteration (``step``):
  1. phi | w, sigma2   -- Metropolis-Hastings, log-normal random walk; the proposal's
                          log density of w is one fused B/F sweep (nngp_bf_sweep at
                          sigma2 = 1, tau2 = 0, values = w), which also returns the
                          proposal's B, F and residuals r = w - B w_N;
  2. sigma2 | w, phi   -- IG(a_s + N/2, b_s + sum r_i^2 / F_i / 2);
  3. w | rest           -- colour-ordered parallel sweep of the full conditionals
                          (nngp_gibbs_w_sweep; moral-graph colouring, Philox normals);
  4. tau2 | ...          -- IG(a_t + N/2, b_t + |y - X beta - w|^2 / 2);
  5. beta | ...          -- N((X'X)^-1 X'(y - w), tau2 (X'X)^-1).
v_i = 1 (homoscedastic) unless ``eps`` is given: then v_i = eps_i^2, the reference's
per-point measurement uncertainties (nngp.py:9, "measurement uncertainties in y",
stored and never used there); with ``fix_tau2=True`` and tau2 = 1 the noise variances
are exactly eps_i^2, otherwise tau2 scales them.  Steps 4-5 then use the weights
h_i = 1/v_i (weighted sums and X' H X).
Scalars (MH decision, conjugate draws) are drawn on the host from a numpy
Generator seeded with ``seed``; every per-location operation runs in
``libnngp_hip.so``.  Parity: the reference has no sampler ("parity unpinned");
``tests/test_gpu_gibbs.py`` checks the w full conditionals against dense linear
algebra, the stationary law of the w sweep against the exact Gaussian posterior,
and recovery of known parameters.
"""
from __future__ import annotations

import dataclasses
import math
from typing import Optional

import numpy as np
import torch

from . import _lib, ops
from .nngp import NNGPNumericalError, _default_device


def _as_points(a, what):
    h = np.ascontiguousarray(a, dtype=np.float64)
    if h.ndim == 1:
        h = h[:, None]
    if h.ndim != 2 or not 1 <= h.shape[1] <= _lib.MAX_DIM or h.shape[0] < 1:
        raise ValueError(f"{what} must be (N >= 1, d) with 1 <= d <= {_lib.MAX_DIM}, got {h.shape}")
    if not np.all(np.isfinite(h)):
        raise ValueError(f"{what} must be finite (NaN / inf would silently decouple locations)")
    return h


def colour_dag(nbr, off, rev_j, n_s):
    """Colour the moral graph of the DAG whose first ``n_s`` nodes are the reference points
    and the rest leaves (in model order: nbr (n, m), reverse CSR off / rev_j -- host numpy arrays
    (the host greedy) or device tensors (nngp_color_moral_graph_dev: the same colours, in parallel
    rounds)).  Greedy over the reference points (leaves come later, so only their co-parent edges
    constrain S); the leaves, never parents and so pairwise non-adjacent, share one last
    colour.  Returns (colors, n_colors, n_colors_ref), colors of the inputs' kind."""
    if isinstance(nbr, torch.Tensor):
        colors, n_colors = _lib.color_moral_graph_dev(nbr, off, rev_j)
        n = colors.shape[0]
        if n > n_s:
            n_colors = int(colors[:n_s].max().item()) + 1 if n_s else 0
            colors[n_s:] = n_colors
            return colors, n_colors + 1, n_colors
        return colors, n_colors, n_colors
    colors, n_colors = _lib.color_moral_graph(nbr, off, rev_j)
    n = colors.shape[0]
    if n > n_s:
        n_colors = int(colors[:n_s].max()) + 1 if n_s else 0
        colors[n_s:] = n_colors
        return colors, n_colors + 1, n_colors
    return colors, n_colors, n_colors


@dataclasses.dataclass
class Priors:
    sigma2_ig: tuple = (2.0, 1.0)  # inverse-gamma (shape, scale)
    tau2_ig: tuple = (2.0, 0.1)
    phi_unif: tuple = (1.0, 100.0)


class SeqNNGP:
    """NNGP response-model Gibbs sampler (see module docstring).

    ``ref=None``: the latent field lives on the data locations (S = T).  With ``ref`` (an
    (n_S, d) reference set S, e.g. the reference's ('random', nRef, bounds) or ('subset',
    nRef) sets) the field lives on S and on the data locations outside S, as the
    reference's ``wt`` / ``ws`` (nngp.py:42-47) linked by ``Nt`` (nngp.py:64-71): the
    DAG's nodes are S (parents: the m nearest earlier points of S) followed by every data
    location not in S as a leaf (parents: its m nearest points of S).  A data location
    that coincides with a point of S carries its observation on that node.  ``y`` may hold
    NaN for unobserved locations: they enter no likelihood term and get posterior-
    predictive draws (``update_y_unobserved``), as do the reference points without data
    when their covariates are known (``X`` None = intercept, or ``X_ref``).  The latent state
    starts at ``w_init`` or, by default, at the reference's initialiser (``_init_ws``,
    nngp.py:45-47: the uniform 5-NN mean of the observed responses at every node).
    """

    # the whole-field phi sweeps through a wave pair plan?  Off: slower than the unplanned kernel
    # (sweep.PLAN_DEFAULT, profiles/r06c); set True on an instance's class to opt in
    _use_plan = False
    # nodes per level-0 tile of the tiled w sweep (sweep="tiled")
    _tile_nodes = 1024
    _tile_max_levels = 8
    _tile_coarse = "colour"  # the nodes above level 0: "colour" (per-colour launches) or "tiles"

    def __init__(self, coords, y, X=None, m: int = 15, kind: str = "exponential", priors: Optional[Priors] = None,
                 sigma2: float = 1.0, tau2: float = 0.1, phi: Optional[float] = None, phi_tuning: float = 0.05,
                 seed: int = 0, device=None, algo: str = "auto", w_init=None, eps=None, fix_tau2: bool = False,
                 ref=None, X_ref=None, nu: Optional[float] = None, cov=None, fix_phi: bool = False,
                 fix_sigma2: bool = False, sweep: str = "colour"):
        if sweep not in ("colour", "tiled"):
            raise ValueError(f"sweep must be 'colour' or 'tiled' (got {sweep!r})")
        self.sweep_mode = sweep
        self.device = _default_device(device)
        dev = self.device
        # a covariance of the caller's own (the reference's plug-in cov(a, b), nngp.py:6,12): the latent
        # covariance is the callable itself, held fixed -- no phi / sigma2 updates (their proposals would
        # re-run the caller's code on every joint block); B / F come from one covariance-blocks sweep
        self._custom = None
        if cov is not None:
            from .nngp import CallableCovariance

            fn = cov.fn if isinstance(cov, CallableCovariance) else cov
            if not callable(fn):
                raise TypeError("cov must be a callable cov(a, b) or a CallableCovariance")
            mode = cov.mode if isinstance(cov, CallableCovariance) else None
            # the latent field's covariance: the callable without a nugget (tau2 is the response model's)
            self._custom = CallableCovariance(fn, 0.0, batch=mode)
            kind, nu, fix_phi, fix_sigma2, sigma2, phi = "custom", None, True, True, 1.0, 0.0
        self.fix_phi, self.fix_sigma2 = bool(fix_phi), bool(fix_sigma2)
        self.kind = kind
        self._nu_arg = -1.0 if self._custom is not None else _lib._check_kind(kind, nu)  # matern's nu; -1 otherwise
        self.nu = nu if kind == "matern" else None
        self.m = int(m)
        if not 1 <= self.m <= _lib.MAX_M:
            raise ValueError(f"m={m} outside [1, {_lib.MAX_M}]")
        self.priors = priors or Priors()
        self.algo = algo
        self.seed = int(seed)
        self.rng = np.random.default_rng(seed)
        to = lambda a: torch.as_tensor(np.ascontiguousarray(a, dtype=np.float64)).to(dev)  # noqa: E731
        t_host = _as_points(coords, "coordinates")
        y_host = np.asarray(y, dtype=np.float64).reshape(-1)
        n_t = t_host.shape[0]
        if y_host.shape != (n_t,):
            raise ValueError(f"y must hold one response per location ({n_t}), got {y_host.shape}")
        if np.any(np.isinf(y_host)):
            raise ValueError("y must be finite or NaN (NaN = unobserved)")
        observed = np.isfinite(y_host)
        X_t = np.ones((n_t, 1)) if X is None else np.asarray(X, dtype=np.float64).reshape(n_t, -1)
        if not np.all(np.isfinite(X_t)):
            raise ValueError("X must be finite")
        self.p = X_t.shape[1]
        self.fix_tau2 = bool(fix_tau2)
        if eps is None:
            h_t = np.ones(n_t)
        else:
            ev = np.asarray(eps, dtype=np.float64).reshape(-1)
            if ev.shape != (n_t,) or not np.all(np.isfinite(ev)) or not np.all(ev > 0):
                raise ValueError(f"eps must hold {n_t} positive finite measurement sigmas")
            h_t = 1.0 / ev ** 2
        self.n_t = n_t

        # ---- the DAG's nodes: S (model rows 0..n_s-1), then the data locations outside S
        t_dev = to(t_host)
        if ref is None:
            s_dev, n_s = t_dev, n_t
            node_of_t = np.arange(n_t)
            nbr0 = _lib.knn_prior(t_dev, self.m)
            coords0 = t_dev
            x_s_known = True
        else:
            s_host = _as_points(ref, "reference set")
            if s_host.shape[1] != t_host.shape[1]:
                raise ValueError(f"reference set has dimension {s_host.shape[1]}, locations {t_host.shape[1]}")
            s_dev, n_s = to(s_host), s_host.shape[0]
            nbr_s = _lib.knn_prior(s_dev, self.m)
            if n_s > 1:  # a repeated reference point makes C_N singular
                j1 = nbr_s[1:, 0].long()
                dup = torch.nonzero((s_dev[1:] == s_dev[j1]).all(dim=1)).flatten()
                if dup.numel() > 0:
                    k = int(dup[0]) + 1
                    raise ValueError(f"reference set point {k} repeats point {int(j1[k - 1])} (C_N would be "
                                     "singular; e.g. ('subset', nRef) draws with replacement)")
            # data locations that coincide with a reference point carry their data on that node
            j0 = _lib.knn_query(s_dev, t_dev, 1)[:, 0].long()
            hit = (t_dev == s_dev[j0]).all(dim=1).cpu().numpy()
            j0h = j0.cpu().numpy()
            if np.unique(j0h[hit]).size != int(hit.sum()):
                raise ValueError("two data locations coincide with the same reference point")
            out_idx = np.nonzero(~hit)[0]
            node_of_t = np.where(hit, j0h, 0)
            node_of_t[out_idx] = n_s + np.arange(out_idx.size)
            k = min(self.m, n_s)
            t_out = t_dev[torch.from_numpy(out_idx).to(dev)]
            nbr_t = _lib.knn_query(s_dev, t_out, k) if out_idx.size else torch.empty((0, k), dtype=torch.int32,
                                                                                       device=dev)
            if k < self.m:
                nbr_t = torch.cat([nbr_t, torch.full((nbr_t.shape[0], self.m - k), -1, dtype=torch.int32,
                                                     device=dev)], dim=1)
            nbr0 = torch.cat([nbr_s, nbr_t]).contiguous()
            coords0 = torch.cat([s_dev, t_out]).contiguous()
            x_s_known = X is None or X_ref is not None
        n = coords0.shape[0]
        self.n, self.n_s = n, n_s
        self.node_of_t = torch.from_numpy(node_of_t.astype(np.int64)).to(dev)

        # per-node data: observation weight h (0 = no observation), y, X
        h_n = np.zeros(n)
        y_n = np.zeros(n)
        X_n = np.zeros((n, self.p))
        h_n[node_of_t[observed]] = h_t[observed]
        y_n[node_of_t[observed]] = y_host[observed]
        X_n[node_of_t] = X_t
        self.n_obs = int(observed.sum())
        if self.n_obs == 0:
            raise ValueError("no observed responses (y is all NaN)")
        # unobserved responses drawn each iteration: data locations with NaN y, then (S != T)
        # the reference points that carry no data, when their covariates are known
        un_t = np.nonzero(~observed)[0]
        un_nodes = node_of_t[un_t]
        un_sd = 1.0 / np.sqrt(h_t[un_t])
        x_un = X_t[un_t]
        self.unobserved_t = un_t  # data-location indices of the first len(un_t) draws
        self.unobserved_ref = np.zeros(0, dtype=np.int64)
        if ref is not None and x_s_known:
            free = np.ones(n_s, dtype=bool)
            free[node_of_t[node_of_t < n_s]] = False
            self.unobserved_ref = np.nonzero(free)[0]
            if X is None:
                x_ref = np.ones((n_s, 1))
            else:
                x_ref = np.asarray(X_ref, dtype=np.float64).reshape(n_s, -1)
                if x_ref.shape[1] != self.p or not np.all(np.isfinite(x_ref)):
                    raise ValueError(f"X_ref must be finite ({n_s}, {self.p})")
                X_n[:n_s][free] = x_ref[free]
            un_nodes = np.concatenate([un_nodes, self.unobserved_ref])
            un_sd = np.concatenate([un_sd, np.ones(self.unobserved_ref.size)])
            x_un = np.concatenate([x_un, x_ref[self.unobserved_ref]])
        XtX = (X_n * h_n[:, None]).T @ X_n
        if np.linalg.matrix_rank(XtX) < self.p:
            raise ValueError("X' H X is singular over the observed locations")
        self._XtX_inv = np.linalg.inv(XtX)
        self._XtX_inv_chol = np.linalg.cholesky(self._XtX_inv)
        homoscedastic = eps is None and self.n_obs == n  # every node observed with weight 1

        # neighbour sets in the model's (node) order; then every per-node array is relabelled
        # into Z-order STORAGE (slot p holds node perm[p]), so that a node's parents and
        # children sit near it in memory: the gathers and scatters of the sweeps share cache
        # lines.  The model is label-invariant (neighbour sets, colouring, conditionals); w is
        # mapped back on output (_relabel).
        # The greedy colouring visits the nodes in MODEL order (S first, spatially scattered for
        # generation-order data: ~2x fewer colours than a scan in the spatial storage order);
        # the moral graph is label-invariant, so the colours carry over.  The leaves (data
        # locations outside S) are never parents, hence pairwise non-adjacent: they form one
        # last colour of their own, swept by update_wt.
        off0, rev_j0, _ = _lib.reverse_neighbors(nbr0)
        # on the device (round 5: the host greedy took ~10 s at N = 1e7; the same colours)
        colors0, self.n_colors, self.n_colors_ref = colour_dag(nbr0, off0, rev_j0, n_s)
        del off0, rev_j0
        perm, _ = _lib.row_order(coords0)
        self._relabel(perm.long(), coords0, y_n, X_n, None if homoscedastic else h_n, nbr0, colors0)
        # (Measured and not kept, round 6, profiles/r06k: colour-major storage -- each colour's members one
        # run of rows, so a colour step reads their operands contiguously: the colour kernel's L2 fetch halved,
        # 44 -> 18 MB per launch, its time unchanged at 15.5 us (latency bound), and the
        # prepare's gathers slowed: 0.797 vs 0.787 ms per iteration.)
        # the tiled w sweep (gibbs_tiles.py): one launch per phase of spatial tiles, r in LDS.  Its kernel
        # wants each tile's nodes (colour-rank order) as one range of storage rows, so the storage order
        # becomes the plan's node order, and the plan is rebuilt on the same tiles in that labelling
        self._tiles = None
        if sweep == "tiled":
            from .gibbs_tiles import build_tile_plan

            tp0 = build_tile_plan(self.coords, self.off, self.rev_j, self._colors_d, self.n_colors, self.n_colors_ref,
                                  tile_nodes=self._tile_nodes, max_levels=self._tile_max_levels,
                                  coarse=self._tile_coarse)
            t0 = tp0.tnodes.long()
            self._relabel(self.perm[t0], coords0, y_n, X_n, None if homoscedastic else h_n, nbr0, colors0)
            self._tiles = build_tile_plan(self.coords, self.off, self.rev_j, self._colors_d, self.n_colors,
                                          self.n_colors_ref, assign=(tp0.node_tile[t0], tp0.tile_level, tp0.coarse_tile))
            assert self._tiles.contiguous
            del tp0, t0
        del self._colors_d
        pos_h = self.pos.cpu().numpy()
        self._un_nodes = torch.from_numpy(pos_h[un_nodes].astype(np.int64)).to(dev)  # storage slots
        self._un_sd = to(un_sd)
        self._un_X = to(x_un.reshape(-1, self.p))
        self.y_unobserved = torch.zeros(len(un_nodes), dtype=torch.float64, device=dev)
        self._zy = torch.empty(len(un_nodes), dtype=torch.float64, device=dev)

        # state
        # (weighted) least squares start over the observed locations
        self.beta = self._XtX_inv @ ((X_n * h_n[:, None]).T @ y_n)
        self.sigma2 = float(sigma2)
        self.tau2 = float(tau2)
        lo, hi = self.priors.phi_unif
        self.phi = float(phi) if phi is not None else math.sqrt(lo * hi)
        self.phi_tuning = float(phi_tuning)
        self.yres = self._residual_y(self.beta)
        if w_init is None:
            # every node starts at the uniform 5-NN mean of the responses less their least-squares
            # mean X beta -- the reference's initialiser of ws (_init_ws, nngp.py:45-47,
            # KNeighborsRegressor(5).fit(t, y).predict(s)) used for all nodes.  (The reference starts
            # wt, the data locations' state, at y itself, _init_wt nngp.py:42-43; here the 5-NN mean
            # of y - X beta, so that w does not carry the mean, which stays with beta.)  A zero start
            # instead lets sigma2 | w = 0 collapse towards 0 and the chain stalls there.
            # NNGP.oneSample passes ws / wt explicitly (SeqNNGP.set_w), the reference's own starts.
            obs_idx = np.nonzero(observed)[0]
            t_obs = t_dev[torch.from_numpy(obs_idx).to(dev)]
            k = min(5, self.n_obs)
            idx = _lib.knn_query(t_obs, coords0, k).long()
            r_obs = y_host[observed] - X_t[observed] @ self.beta
            w0 = to(r_obs)[idx].mean(dim=1).cpu().numpy()
        else:
            w0 = np.asarray(w_init, dtype=np.float64).reshape(-1)
            if w0.shape != (n,):
                raise ValueError(f"w_init must hold one value per node ({n}: reference points, then the data "
                                 "locations outside the reference set)")
        self.w = to(w0)[self.perm].contiguous()  # storage order
        self.iteration = 0
        self.n_accept = 0
        self.n_notpd_reject = 0  # phi proposals rejected because their factor was not positive definite

        # buffers: current and proposal factors of the unit-variance field
        z = lambda *s: torch.empty(s, dtype=torch.float64, device=dev)  # noqa: E731
        self.B, self.Ft, self.r = z(n, self.m), z(n), z(n)
        self._B2, self._Ft2, self._r2 = z(n, self.m), z(n), z(n)
        self._part = z(4)
        self._z = z(n)
        ops.load()  # the sweep goes through torch.ops.nngp.bf_sweep_out (libnngp_torch_ops.so)
        if self._custom is not None:
            if not 1 <= self.m <= _lib.BLOCKS_MAX_M:
                raise ValueError(f"a callable covariance needs 1 <= m <= {_lib.BLOCKS_MAX_M} (m={self.m})")
            # the caller's covariance on every joint block, once (the chain holds it fixed)
            self._cblocks = self._custom.blocks(self.coords, self.nbr, 0)
            self._ws = _lib._workspace(_lib.load().nngp_bf_sweep_blocks_workspace_bytes(n), dev)
            self._kind_code, self._algo_code = -1, ops.algo_code(algo)
        else:
            self._ws = _lib.bf_workspace(n, self.m, algo, dev, kind=kind, dim=self.coords.shape[1])
            self._kind_code, self._algo_code = ops.kind_code(kind), ops.algo_code(algo)
        # wave pair plan for the phi-proposal sweeps (pair_plan.h; the same B / F / r bits, each shared
        # covariance of a wavefront evaluated once): built once, the DAG never changes
        self._plan = (None, None)
        if (self._use_plan and self._custom is None and algo in ("auto", "pairb")
                and _lib.pair_plan_supported(self.m, kind, self.coords.shape[1])):
            self._plan = ops.pair_plan(self.nbr, None, 0, n, self.coords.shape[1])
        self._stats_buf = z(2 + self.p)
        self._sweep_into(self.phi, self.B, self.Ft, self.r)
        self._prep = _lib.gibbs_prepare(self.B, self.Ft, self.off, self.rev_j, self.rev_k)
        ph = self._part.cpu().numpy()
        self._check(ph)
        self.sum_logF, self.quad = float(ph[0]), float(ph[1])

    # ------------------------------------------------------------------ pieces
    def _relabel(self, perm, coords0, y_n, X_n, h_n, nbr0, colors0):
        """Storage order: slot p holds model node perm[p]; every per-node array, the neighbour sets (in
        storage labels), their reverse lists and the colour groups follow it."""
        dev = self.device
        to = lambda a: torch.as_tensor(np.ascontiguousarray(a, dtype=np.float64)).to(dev)  # noqa: E731
        n = coords0.shape[0]
        self.perm = perm
        self.pos = torch.empty_like(self.perm)
        self.pos[self.perm] = torch.arange(n, device=dev)
        self.coords = coords0[self.perm].contiguous()
        self.y = to(y_n)[self.perm].contiguous()
        self.X = to(X_n)[self.perm].contiguous()
        self._Xcols = self.X.t().contiguous()  # (p, n): y - X beta as p contiguous vector ops
        self.noise_w = None if h_n is None else to(h_n)[self.perm].contiguous()  # h_i, storage order
        nb = nbr0[self.perm].long()
        self.nbr = torch.where(nb >= 0, self.pos[nb.clamp(min=0)], -1).to(torch.int32).contiguous()
        self.off, self.rev_j, self.rev_k = _lib.reverse_neighbors(self.nbr)
        colors_d = colors0[self.perm]
        self._colors_d = colors_d
        self.colors = colors_d.cpu().numpy()
        # members grouped by colour, storage order inside a colour
        self.members = torch.sort(colors_d, stable=True)[1].to(torch.int32)
        self.color_off = np.concatenate([[0], np.cumsum(torch.bincount(colors_d, minlength=self.n_colors).cpu().numpy())
                                         ]).astype(np.int32)

    def _residual_y(self, beta):
        """y - X beta as elementwise device ops on contiguous columns (p is small; a tall-skinny
        GEMV is slower, and the strided columns of the row-major X took 18.7 us per op against
        ~4 us contiguous at N = 1e6), into the same buffer every iteration."""
        out = getattr(self, "_yres_buf", None)
        if out is None:
            out = self._yres_buf = torch.empty_like(self.y)
        if self.p == 0:
            return out.copy_(self.y)
        torch.sub(self.y, self._Xcols[0], alpha=float(beta[0]), out=out)
        for c in range(1, self.p):
            out.sub_(self._Xcols[c], alpha=float(beta[c]))
        return out

    def _sweep_into(self, phi, B, Ft, r):
        """Factors of the unit-variance NNGP at phi, and residuals of the current w (a callable
        covariance: the factors of the callable's own covariance, sigma2 = 1)."""
        if self._custom is not None:
            _lib.bf_sweep_blocks(self._cblocks, self.nbr, self.n, 0, values=self.w, qvalues=self.w, R=r, B=B, F=Ft,
                                 partials=self._part, workspace=self._ws)
            return
        torch.ops.nngp.bf_sweep_out(self.coords, self.nbr, None, 0, self._kind_code, 1.0, float(phi), 0.0, self.w, B,
                                    Ft, r, self._part, self._ws, self._algo_code, self._nu_arg, *self._plan)

    @staticmethod
    def _check(p):
        if p[2] >= 0:
            raise NNGPNumericalError(
                f"latent NNGP factor not positive definite at location {int(p[2])} at the initial phi "
                "(duplicate or near-duplicate coordinates make C_N singular; remove duplicates or lower phi)")

    def _ig(self, a, b):
        return 1.0 / self.rng.gamma(a, 1.0 / b)

    def loglik_w(self, sum_logF, quad, sigma2):
        """log p(w | sigma2, phi) from the sweep's partials of the unit-variance field."""
        return -0.5 * (self.n * math.log(2 * math.pi * sigma2) + sum_logF + quad / sigma2)

    def update_phi(self):
        """phi | w, sigma2: log-normal random-walk Metropolis-Hastings; the proposal's log
        density of w is one fused B/F sweep over every node of the DAG."""
        prop = self._phi_draw()
        if prop is not None:
            self._phi_decide(prop, self._propose(prop[0]))

    def _phi_draw(self):
        """The host draws of a phi move: (phi_p, u), or None (phi fixed, or the proposal outside the
        prior's support -- the draws are made either way, as the sampler always did)."""
        if self.fix_phi:
            return None
        phi_p = self.phi * math.exp(self.phi_tuning * self.rng.standard_normal())
        lo, hi = self.priors.phi_unif
        u = self.rng.random()
        if not lo <= phi_p <= hi:
            return None
        return phi_p, u

    def _phi_decide(self, prop, ph):
        """Accept / reject a proposal given its sweep's host partials ``ph``."""
        phi_p, u = prop
        if ph[2] >= 0:
            # the proposal's latent factor is not positive definite (near-duplicate locations
            # with tau2 = 0 and a large phi): zero density there, so the move is rejected
            self.n_notpd_reject += 1
            return
        l_new = self.loglik_w(ph[0], ph[1], self.sigma2)
        l_old = self.loglik_w(self.sum_logF, self.quad, self.sigma2)
        if math.log(u) < l_new - l_old + math.log(phi_p) - math.log(self.phi):
            self.phi = phi_p
            self.B, self._B2 = self._B2, self.B
            self.Ft, self._Ft2 = self._Ft2, self.Ft
            self.r, self._r2 = self._r2, self.r
            self._prepare()
            self.sum_logF, self.quad = float(ph[0]), float(ph[1])
            self.n_accept += 1

    def _propose(self, phi):
        """B / F / residuals of the unit-variance field at the proposal, into the spare buffers;
        returns the host partials (the sharded chain overrides: own rows + halo, folded over ranks)."""
        self._sweep_into(phi, self._B2, self._Ft2, self._r2)
        return self._part.cpu().numpy()

    def _prepare(self):
        """Fold the accepted B / F for the colour steps (the sharded chain: its own rows only)."""
        self._prep = _lib.gibbs_prepare(self.B, self.Ft, self.off, self.rev_j, self.rev_k, prep=self._prep)

    def _stats(self):
        """[sum r^2/F, sum h (yres - w)^2, X'H(y - w)] on the host (the sharded chain: folded over ranks)."""
        return self._stats_dev().cpu().numpy()

    def _stats_dev(self):
        """The same statistics, stream-ordered on the device (no host synchronisation)."""
        return _lib.gibbs_stats(self.r, self.Ft, self.yres, self.y, self.X, self.w, out=self._stats_buf,
                                noise_w=self.noise_w)

    def _member_rows_t(self):
        """The colour-ordered member rows (location, reverse-entry range), built once."""
        if getattr(self, "_member_rows", None) is None and self.members.numel() > 0:
            self._member_rows = _lib.gibbs_member_rows(self.members, self.off)
        return getattr(self, "_member_rows", None)

    def _assemble(self, t):
        """A per-node (storage order) result as every rank sees it (identity on one GPU)."""
        return t

    def _assemble_unobserved(self, t):
        return t

    def _sweep_colours(self, c0, c1):
        if c1 > c0:
            self._member_rows_t()  # (location, reverse-entry range) per member, once
            _lib.gibbs_w_sweep(self.members, self.color_off[c0:c1 + 1], self._prep, self.m, self.sigma2, self.tau2,
                               self.yres, self.w, self.r, self.off, self.rev_j, self.seed, self.iteration, z=self._z,
                               noise_w=self.noise_w, member_rows=self._member_rows)

    def update_wt(self):
        """w_t | w_S, y_t for the data locations outside S (nngp.py:99): the leaves of the DAG,
        conditionally independent given w_S, all drawn in one parallel colour step
        (N(B_t w_N(t), sigma2 F_t) prior times the observation's likelihood).  With S = T
        there are no leaves: w_t is w_s."""
        self._sweep_colours(self.n_colors_ref, self.n_colors)

    def update_ws(self):
        """w_s | rest for the reference points (nngp.py:100): colour-ordered parallel sweep of
        the full conditionals, children on S and leaf children at T included."""
        self._sweep_colours(0, self.n_colors_ref)

    def update_y_unobserved(self):
        """Posterior-predictive draws y* = x beta + w + N(0, tau2 / h) at the unobserved
        locations (nngp.py:101): data locations with NaN y and, for S != T, the reference
        points without data whose covariates are known (``y_unobserved``, in the order
        ``unobserved_t`` then ``unobserved_ref``)."""
        k = self._un_nodes.numel()
        if k == 0:
            return
        # an independent Philox stream: the sweep counter's top bit set
        _lib.gibbs_normals(self._zy, self.seed, self.iteration | (1 << 63))
        xb = self._un_X @ torch.as_tensor(self.beta, dtype=torch.float64, device=self.device)
        torch.addcmul(xb + self.w[self._un_nodes], self._un_sd, self._zy, value=math.sqrt(self.tau2),
                      out=self.y_unobserved)

    def step(self):
        """One iteration: phi; sigma2; update_wt; update_ws; tau2; beta; update_y_unobserved."""
        self.update_phi()
        self._before_w()
        if self._tiles is not None:
            self._sweep_tiles()  # update_wt and update_ws, tile by tile (the plan's order)
        else:
            self.update_wt()
            self.update_ws()
        self._after_w(self._stats())

    def _sweep_tiles(self):
        """One w sweep through the tile plan (nngp_gibbs_w_sweep_tiles): every node's full conditional, in the
        plan's (level, phase, colour) order -- leaves (update_wt) before the reference colours inside a tile."""
        _lib.gibbs_w_sweep_tiles(self._tiles, self._prep, self.m, self.sigma2, self.tau2, self.yres, self.w, self.r,
                                 self.off, self._z, noise_w=self.noise_w, rev_j=self.rev_j)

    def _before_w(self):
        """sigma2 | w, phi (held fixed on request, and with a callable covariance: its own scale), then the
        w sweep's normals in one parallel pass."""
        if not self.fix_sigma2:
            a, b = self.priors.sigma2_ig
            self.sigma2 = self._ig(a + 0.5 * self.n, b + 0.5 * self.quad)
        _lib.gibbs_normals(self._z, self.seed, self.iteration)

    def _after_w(self, st):
        """tau2, beta, y - X beta, the predictive draws, from the host statistics ``st`` of the new w."""
        self.quad = float(st[0])
        # tau2 | y, beta, w (weighted residual sum of squares over the observed; held fixed on request)
        if not self.fix_tau2:
            a, b = self.priors.tau2_ig
            self.tau2 = self._ig(a + 0.5 * self.n_obs, b + 0.5 * float(st[1]))
        # beta | y, w, tau2 (flat prior; weighted least squares)
        mean = self._XtX_inv @ st[2:]
        self.beta = mean + math.sqrt(self.tau2) * (self._XtX_inv_chol @ self.rng.standard_normal(self.p))
        self.yres = self._residual_y(self.beta)
        self.update_y_unobserved()
        self.iteration += 1

    def set_w(self, ws=None, wt=None):
        """Set the latent state: ``ws`` at the reference points (n_S,), ``wt`` at the data
        locations (n_T,; with S != T it sets the leaves only, the locations on S take ``ws``);
        the NNGP residuals are recomputed."""
        to = lambda a: torch.as_tensor(np.asarray(a, dtype=np.float64)).to(self.device)  # noqa: E731
        wn = self.w_nodes.clone()
        if ws is not None:
            wn[: self.n_s] = to(ws).reshape(-1)
        if wt is not None:
            wt = to(wt).reshape(-1)
            if wt.shape != (self.n_t,):
                raise ValueError(f"wt must hold {self.n_t} values")
            leaf = self.node_of_t >= self.n_s
            if self.n_s == self.n_t and self.n == self.n_t and not bool(leaf.any()):
                wn[self.node_of_t] = wt
            else:
                wn[self.node_of_t[leaf]] = wt[leaf]
        if not bool(torch.isfinite(wn).all()):
            raise ValueError("w must be finite")
        self.w = wn[self.perm].contiguous()
        self._sweep_into(self.phi, self.B, self.Ft, self.r)
        ph = self._part.cpu().numpy()
        self.sum_logF, self.quad = float(ph[0]), float(ph[1])

    def clone(self, seed: int) -> "SeqNNGP":
        """A chain on the same field, data and settings started as ``SeqNNGP(..., seed=seed)`` would be:
        the DAG, colouring, reverse lists, plan and covariance blocks are shared (read-only), the state
        and every buffer a step writes are its own.  Cloned before the first step it runs the chain of
        ``seed`` bit for bit (the constructor's state does not depend on the seed)."""
        import copy

        if self.iteration != 0:
            raise ValueError("clone a sampler before its first step")
        c = copy.copy(self)
        c.seed = int(seed)
        c.rng = np.random.default_rng(seed)
        c.beta = np.array(self.beta)
        own = lambda t: None if t is None else t.clone()  # noqa: E731
        c.w, c.r, c.B, c.Ft = own(self.w), own(self.r), own(self.B), own(self.Ft)
        c._B2, c._Ft2, c._r2 = torch.empty_like(self._B2), torch.empty_like(self._Ft2), torch.empty_like(self._r2)
        c._part, c._z, c._stats_buf = own(self._part), torch.empty_like(self._z), own(self._stats_buf)
        c._ws = own(self._ws)
        c._prep = own(self._prep)
        c._yres_buf = own(self._yres_buf)
        c.yres = c._yres_buf
        c.y_unobserved, c._zy = own(self.y_unobserved), torch.empty_like(self._zy)
        return c

    # ------------------------------------------------------------------ checkpoint / resume
    def _settings(self) -> dict:
        return {"algo": self.algo, "phi_tuning": self.phi_tuning, "fix_tau2": self.fix_tau2, "nu": self.nu,
                "fix_phi": self.fix_phi, "fix_sigma2": self.fix_sigma2,
                "priors": {k: list(v) for k, v in dataclasses.asdict(self.priors).items()},
                "n_t": self.n_t, "n_obs": self.n_obs, "n_colors": int(self.n_colors)}

    def _fingerprint(self, node_order: bool = True) -> str:
        """sha256 over the sampler's data (coordinates, responses, covariates, noise weights,
        neighbour sets) and settings: a checkpoint resumes only into a sampler built on the same
        inputs.  node_order: the arrays in the model's node order with node labels (round 6), so a
        checkpoint moves between storage orders (the colour sweep's Z-order, the tiled sweep's plan
        order); False: the storage-order arrays, as checkpoints before round 6 recorded them."""
        import hashlib
        import json

        h = hashlib.sha256()
        arrays = (self.coords, self.y, self.X, self.nbr, self.noise_w, getattr(self, "_cblocks", None))
        if node_order:
            pos, perm = self.pos, self.perm
            nb = self.nbr[pos].long()
            nbr_nodes = torch.where(nb >= 0, perm[nb.clamp(min=0)], -1).to(torch.int32)
            cb = getattr(self, "_cblocks", None)
            arrays = (self.coords[pos], self.y[pos], self.X[pos], nbr_nodes,
                      None if self.noise_w is None else self.noise_w[pos], None if cb is None else cb[:, pos])
        for t in arrays:
            h.update(b"none" if t is None else t.contiguous().cpu().numpy().tobytes())
        h.update(json.dumps(self._settings(), sort_keys=True).encode())
        return h.hexdigest()

    def save(self, path) -> None:
        """Checkpoint the chain: w and the maintained residuals r in node order,
        beta, sigma2, tau2, phi, the partial sums, the iteration counter (the Philox key of
        every later draw) and the host RNG state, to an ``.npz`` (no pickles).  A sampler
        built on the same data and :meth:`restore`-d continues the chain bit for bit."""
        import json

        meta = {"n": self.n, "n_s": self.n_s, "m": self.m, "kind": self.kind, "p": self.p, "seed": self.seed,
                "iteration": self.iteration, "n_accept": self.n_accept, "n_notpd_reject": self.n_notpd_reject,
                "sigma2": self.sigma2, "tau2": self.tau2, "phi": self.phi, "sum_logF": self.sum_logF,
                "quad": self.quad, "rng": self.rng.bit_generator.state, "settings": self._settings(),
                "fingerprint_nodes": self._fingerprint()}
        np.savez(path, w=self.w[self.pos].cpu().numpy(), r=self.r[self.pos].cpu().numpy(), beta=np.asarray(self.beta),
                 y_unobserved=self.y_unobserved.cpu().numpy(), meta=np.array(json.dumps(meta)))

    def restore(self, path) -> "SeqNNGP":
        """Resume from :meth:`save`.  The sampler must be built on the same data and settings:
        sizes, kind and seed are compared one by one, then a fingerprint of the coordinates,
        responses, covariates, noise weights, neighbour sets, algo, phi_tuning, fix_tau2 and
        priors; any mismatch raises ValueError (the running residuals r would otherwise be
        inconsistent with w and B)."""
        import json

        with np.load(path, allow_pickle=False) as z:
            meta = json.loads(str(z["meta"]))
            for k in ("n", "n_s", "m", "kind", "p", "seed"):
                if meta[k] != getattr(self, k):
                    raise ValueError(f"checkpoint {k}={meta[k]!r} does not match this sampler's {getattr(self, k)!r}")
            mine = self._settings()
            for k, v in meta.get("settings", {}).items():
                if mine.get(k) != v:
                    raise ValueError(f"checkpoint setting {k}={v!r} does not match this sampler's {mine.get(k)!r}")
            if "fingerprint_nodes" in meta:
                same = meta["fingerprint_nodes"] == self._fingerprint()
            elif "fingerprint" in meta:  # (pynngp_amd 0.2 - 0.3: storage order)
                same = meta["fingerprint"] == self._fingerprint(node_order=False)
            else:
                import warnings

                warnings.warn("checkpoint predates the data fingerprint (pynngp_amd < 0.2): only sizes, kind, seed "
                              "and settings were compared -- make sure it was written on the same data", stacklevel=2)
                same = True
            if not same:
                raise ValueError("checkpoint was written by a sampler built on different data (coordinates, "
                                 "responses, covariates, noise weights or neighbour sets) or settings")
            to = lambda a: torch.as_tensor(a).to(self.device)  # noqa: E731
            self.w = to(z["w"])[self.perm].contiguous()
            r = to(z["r"])[self.perm].contiguous()
            self.beta = np.array(z["beta"])
            self.y_unobserved.copy_(to(z["y_unobserved"]))
        self.sigma2, self.tau2, self.phi = meta["sigma2"], meta["tau2"], meta["phi"]
        self.iteration, self.n_accept, self.n_notpd_reject = meta["iteration"], meta["n_accept"], meta["n_notpd_reject"]
        self.rng.bit_generator.state = meta["rng"]
        # B, F (and the folded prep) are functions of phi alone; r is the chain's own running value
        self._sweep_into(self.phi, self.B, self.Ft, self.r)
        self._check(self._part.cpu().numpy())
        self.r = r
        self.sum_logF, self.quad = meta["sum_logF"], meta["quad"]
        self._prep = _lib.gibbs_prepare(self.B, self.Ft, self.off, self.rev_j, self.rev_k, prep=self._prep)
        self.yres = self._residual_y(self.beta)
        return self

    @property
    def w_nodes(self) -> torch.Tensor:
        """w in model node order: the reference points, then the data locations outside S."""
        return self.w[self.pos]

    @property
    def w_s(self) -> torch.Tensor:
        """w at the reference points (the reference's ``ws``)."""
        return self.w[self.pos[: self.n_s]]

    @property
    def w_t(self) -> torch.Tensor:
        """w at the data locations (the reference's ``wt``)."""
        return self.w[self.pos[self.node_of_t]]

    @property
    def w_input_order(self) -> torch.Tensor:
        """Current latent field w at the data locations, in the caller's order (the state lives in
        Z-order storage); = :attr:`w_t`."""
        return self.w_t

    def sample(self, n_iter: int, burn: int = 0, thin: int = 1, keep_w_mean: bool = False):
        """Run n_iter iterations; return the thinned post-burn-in draws (numpy)."""
        out = {"beta": [], "sigma2": [], "tau2": [], "phi": []}
        w_sum = torch.zeros_like(self.w) if keep_w_mean else None
        y_sum = torch.zeros_like(self.y_unobserved)
        kept = 0
        for k in range(n_iter):
            self.step()
            if k >= burn and (k - burn) % thin == 0:
                out["beta"].append(self.beta.copy())
                out["sigma2"].append(self.sigma2)
                out["tau2"].append(self.tau2)
                out["phi"].append(self.phi)
                if keep_w_mean:
                    w_sum += self.w
                y_sum += self.y_unobserved
                kept += 1
        res = {k: np.asarray(v) for k, v in out.items()}
        res["phi_accept_rate"] = self.n_accept / max(self.iteration, 1)
        if keep_w_mean:
            wm = self._assemble(w_sum / max(kept, 1))
            res["w_mean"] = wm[self.pos[self.node_of_t]].cpu().numpy()  # data locations, input order
            if self.n > self.n_t or self.n_s != self.n_t:
                res["ws_mean"] = wm[self.pos[: self.n_s]].cpu().numpy()  # reference points
        if self.y_unobserved.numel():
            res["y_unobserved_mean"] = self._assemble_unobserved(y_sum / max(kept, 1)).cpu().numpy()
        return res


class SeqNNGPChains:
    """``C`` independent :class:`SeqNNGP` chains of one field advanced together (BASELINE config 5's
    replica mode, several chains per GPU): chain k is ``SeqNNGP(..., seed=seeds[k])`` bit for bit, but
    the chains share the DAG and colouring, their colour steps run as ONE launch per colour for all
    chains (nngp_gibbs_w_sweep_chains: the launch and member-row round trips paid once, C independent
    gathers in flight per thread), and each iteration synchronises the host twice for all chains
    (the phi proposals' partials, the conjugate statistics) instead of twice per chain.

        chains = SeqNNGPChains(coords, y, seeds=[1, 2, 3, 4], m=15, ...)
        chains.step()                 # one iteration of every chain
        chains[k].beta, chains[k].w   # chain k's state (a SeqNNGP)
    """

    def __init__(self, coords, y, X=None, seeds=(0,), interleave: bool = True, **kw):
        seeds = [int(s) for s in seeds]
        # interleave: the colour steps read the chains' w and r from (n, C) copies (one sector per scattered
        # access for all chains; packed before and unpacked after each iteration's colour sweeps)
        self.interleave = bool(interleave)
        if not 1 <= len(seeds) <= 8:
            raise ValueError("1 to 8 chains per batch")
        if "seed" in kw:
            raise ValueError("give the chains' seeds as seeds=[...]")
        first = SeqNNGP(coords, y, X, seed=seeds[0], **kw)
        self.chains = [first] + [first.clone(s) for s in seeds[1:]]

    def __len__(self):
        return len(self.chains)

    def __getitem__(self, k) -> SeqNNGP:
        return self.chains[k]

    def step(self):
        cs = self.chains
        # phi: every chain's host draws and proposal sweep, then ONE synchronisation for all partials
        props = [c._phi_draw() for c in cs]
        parts = []
        for c, p in zip(cs, props):
            if p is not None:
                c._sweep_into(p[0], c._B2, c._Ft2, c._r2)
                parts.append(c._part.clone())
        ph = torch.stack(parts).cpu().numpy() if parts else None
        k = 0
        for c, p in zip(cs, props):
            if p is not None:
                c._phi_decide(p, ph[k])
                k += 1
        for c in cs:
            c._before_w()
        # w | rest: update_wt (the leaves' colour) then update_ws, one launch per colour for all chains
        c0 = cs[0]
        if c0._member_rows_t() is not None:
            if self.interleave:
                W = torch.stack([c.w for c in cs], dim=1)
                R = torch.stack([c.r for c in cs], dim=1)
            else:
                W, R = [c.w for c in cs], [c.r for c in cs]
            for lo, hi in ((c0.n_colors_ref, c0.n_colors), (0, c0.n_colors_ref)):
                if hi > lo:
                    _lib.gibbs_w_sweep_chains(c0._member_rows, c0.color_off[lo:hi + 1], [c._prep for c in cs], c0.m,
                                              [c.sigma2 for c in cs], [c.tau2 for c in cs], [c.yres for c in cs],
                                              W, R, c0.rev_j, [c._z for c in cs], noise_w=c0.noise_w)
            if self.interleave:
                for k, c in enumerate(cs):
                    c.w.copy_(W[:, k])
                    c.r.copy_(R[:, k])
        # the conjugate statistics of every chain, ONE synchronisation
        st = torch.stack([c._stats_dev() for c in cs]).cpu().numpy()
        for c, s_ in zip(cs, st):
            c._after_w(s_)

    def sample(self, n_iter: int):
        """Run n_iter iterations of every chain; returns per-chain arrays of beta, sigma2, tau2, phi."""
        out = [{"beta": [], "sigma2": [], "tau2": [], "phi": []} for _ in self.chains]
        for _ in range(n_iter):
            self.step()
            for o, c in zip(out, self.chains):
                o["beta"].append(c.beta.copy())
                o["sigma2"].append(c.sigma2)
                o["tau2"].append(c.tau2)
                o["phi"].append(c.phi)
        return [{k: np.asarray(v) for k, v in o.items()} for o in out]
