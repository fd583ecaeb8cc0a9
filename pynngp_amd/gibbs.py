"""``SeqNNGP``: Gibbs sampler for the NNGP response model on the GPU.

The reference's sampler entry point is ``NNGP.oneSample`` (pyNNGP/nngp.py:98-101),
which calls ``update_wt`` / ``update_ws`` / ``update_y_unobserved`` -- none of them
exist.  This is the sampler those names describe, for the model of Datta et al.
(2016) that the reference's B/F docstrings (nngp.py:73-96) come from:

    y = X beta + w + e,   e_i ~ N(0, tau2 v_i),   w ~ NNGP(0, sigma2 R(phi))
    beta ~ flat,  sigma2 ~ IG(a_s, b_s),  tau2 ~ IG(a_t, b_t),  phi ~ U(phi_lo, phi_hi)

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


@dataclasses.dataclass
class Priors:
    sigma2_ig: tuple = (2.0, 1.0)  # inverse-gamma (shape, scale)
    tau2_ig: tuple = (2.0, 0.1)
    phi_unif: tuple = (1.0, 100.0)


class SeqNNGP:
    """NNGP response-model Gibbs sampler (see module docstring)."""

    def __init__(self, coords, y, X=None, m: int = 15, kind: str = "exponential", priors: Optional[Priors] = None,
                 sigma2: float = 1.0, tau2: float = 0.1, phi: Optional[float] = None, phi_tuning: float = 0.05,
                 seed: int = 0, device=None, algo: str = "auto", w_init=None, eps=None, fix_tau2: bool = False):
        self.device = _default_device(device)
        dev = self.device
        self.kind = kind
        self.m = int(m)
        self.priors = priors or Priors()
        self.algo = algo
        self.seed = int(seed)
        self.rng = np.random.default_rng(seed)
        to = lambda a: torch.as_tensor(np.ascontiguousarray(a, dtype=np.float64)).to(dev)  # noqa: E731
        coords0 = to(coords)
        if not bool(torch.isfinite(coords0).all()):
            raise ValueError("coordinates must be finite (NaN / inf would silently decouple locations)")
        y0 = to(y)
        n = y0.shape[0]
        self.n = n
        X0 = to(np.ones((n, 1)) if X is None else np.asarray(X, dtype=np.float64).reshape(n, -1))
        self.p = X0.shape[1]
        Xh = X0.cpu().numpy()
        self.fix_tau2 = bool(fix_tau2)
        if eps is None:
            hh = np.ones(n)
            h0 = None
        else:
            ev = np.asarray(eps, dtype=np.float64).reshape(-1)
            if ev.shape != (n,) or not np.all(np.isfinite(ev)) or not np.all(ev > 0):
                raise ValueError(f"eps must hold {n} positive finite measurement sigmas")
            hh = 1.0 / ev ** 2
            h0 = to(hh)
        self._XtX_inv = np.linalg.inv((Xh * hh[:, None]).T @ Xh)
        self._XtX_inv_chol = np.linalg.cholesky(self._XtX_inv)

        # neighbour sets in the model's (input) order; then every per-location array is
        # relabelled into Z-order STORAGE (slot p holds location perm[p]), so that a
        # location's parents and children sit near it in memory: the gathers and
        # scatters of the sweeps share cache lines.  The model is label-invariant
        # (neighbour sets, colouring, conditionals); w is mapped back on output.
        nbr0 = _lib.knn_prior(coords0, self.m)
        perm, _ = _lib.row_order(coords0)
        self.perm = perm.long()
        self.pos = torch.empty_like(self.perm)
        self.pos[self.perm] = torch.arange(n, device=dev)
        self.coords = coords0[self.perm].contiguous()
        self.y = y0[self.perm].contiguous()
        self.X = X0[self.perm].contiguous()
        self.noise_w = None if h0 is None else h0[self.perm].contiguous()  # h_i = 1 / eps_i^2, storage order
        nb = nbr0[self.perm].long()
        self.nbr = torch.where(nb >= 0, self.pos[nb.clamp(min=0)], -1).to(torch.int32).contiguous()
        self.off, self.rev_j, self.rev_k = _lib.reverse_neighbors(self.nbr)
        # greedy colouring visits the locations in INPUT order (spatially scattered for
        # generation-order data: ~2x fewer colours than a scan in the spatial storage
        # order); the moral graph is label-invariant, so the colours carry over
        off0, rev_j0, _ = _lib.reverse_neighbors(nbr0)
        colors0, self.n_colors = _lib.color_moral_graph(nbr0.cpu().numpy(), off0.cpu().numpy(),
                                                        rev_j0.cpu().numpy())
        colors = colors0[self.perm.cpu().numpy()]
        self.colors = colors
        # members grouped by colour, storage (= Z) order inside a colour
        self.members = torch.from_numpy(np.argsort(colors, kind="stable").astype(np.int32)).to(dev)
        self.color_off = np.concatenate([[0], np.cumsum(np.bincount(colors, minlength=self.n_colors))]).astype(
            np.int32)

        # state
        # (weighted) least squares start; X, y and the weights in the caller's order
        self.beta = self._XtX_inv @ ((Xh * hh[:, None]).T @ y0.cpu().numpy())
        self.sigma2 = float(sigma2)
        self.tau2 = float(tau2)
        lo, hi = self.priors.phi_unif
        self.phi = float(phi) if phi is not None else math.sqrt(lo * hi)
        self.phi_tuning = float(phi_tuning)
        self.yres = self._residual_y(self.beta)
        self.w = to(np.zeros(n) if w_init is None else w_init)[self.perm].contiguous()  # storage order
        self.iteration = 0
        self.n_accept = 0
        self.n_notpd_reject = 0  # phi proposals rejected because their factor was not positive definite

        # buffers: current and proposal factors of the unit-variance field
        z = lambda *s: torch.empty(s, dtype=torch.float64, device=dev)  # noqa: E731
        self.B, self.Ft, self.r = z(n, self.m), z(n), z(n)
        self._B2, self._Ft2, self._r2 = z(n, self.m), z(n), z(n)
        self._part = z(4)
        self._z = z(n)
        self._ws = _lib.bf_workspace(n, self.m, algo, dev, kind=kind, dim=self.coords.shape[1])
        ops.load()  # the sweep goes through torch.ops.nngp.bf_sweep_out (libnngp_torch_ops.so)
        self._kind_code, self._algo_code = ops.kind_code(kind), ops.algo_code(algo)
        self._stats = z(2 + self.p)
        self._sweep_into(self.phi, self.B, self.Ft, self.r)
        self._prep = _lib.gibbs_prepare(self.B, self.Ft, self.off, self.rev_j, self.rev_k)
        ph = self._part.cpu().numpy()
        self._check(ph)
        self.sum_logF, self.quad = float(ph[0]), float(ph[1])

    # ------------------------------------------------------------------ pieces
    def _residual_y(self, beta):
        """y - X beta as elementwise device ops (p is small; a tall-skinny GEMV is slower)."""
        out = self.y.clone()
        for c in range(self.p):
            out.sub_(self.X[:, c], alpha=float(beta[c]))
        return out

    def _sweep_into(self, phi, B, Ft, r):
        """Factors of the unit-variance NNGP at phi, and residuals of the current w."""
        torch.ops.nngp.bf_sweep_out(self.coords, self.nbr, None, 0, self._kind_code, 1.0, float(phi), 0.0, self.w, B,
                                    Ft, r, self._part, self._ws, self._algo_code)

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

    def step(self):
        n = self.n
        # 1. phi | w, sigma2: log-normal random walk MH
        phi_p = self.phi * math.exp(self.phi_tuning * self.rng.standard_normal())
        lo, hi = self.priors.phi_unif
        u = self.rng.random()
        if lo <= phi_p <= hi:
            self._sweep_into(phi_p, self._B2, self._Ft2, self._r2)
            ph = self._part.cpu().numpy()
        if lo <= phi_p <= hi and ph[2] >= 0:
            # the proposal's latent factor is not positive definite (near-duplicate locations
            # with tau2 = 0 and a large phi): zero density there, so the move is rejected
            self.n_notpd_reject += 1
        elif lo <= phi_p <= hi:
            l_new = self.loglik_w(ph[0], ph[1], self.sigma2)
            l_old = self.loglik_w(self.sum_logF, self.quad, self.sigma2)
            if math.log(u) < l_new - l_old + math.log(phi_p) - math.log(self.phi):
                self.phi = phi_p
                self.B, self._B2 = self._B2, self.B
                self.Ft, self._Ft2 = self._Ft2, self.Ft
                self.r, self._r2 = self._r2, self.r
                self._prep = _lib.gibbs_prepare(self.B, self.Ft, self.off, self.rev_j, self.rev_k, prep=self._prep)
                self.sum_logF, self.quad = float(ph[0]), float(ph[1])
                self.n_accept += 1
        # 2. sigma2 | w, phi
        a, b = self.priors.sigma2_ig
        self.sigma2 = self._ig(a + 0.5 * n, b + 0.5 * self.quad)
        # 3. w | rest (colour sweep, in place on w and r)
        _lib.gibbs_normals(self._z, self.seed, self.iteration)  # the sweep's normals, one parallel pass
        _lib.gibbs_w_sweep(self.members, self.color_off, self._prep, self.m, self.sigma2, self.tau2, self.yres, self.w,
                           self.r, self.off, self.rev_j, self.seed, self.iteration, z=self._z, noise_w=self.noise_w)
        st = _lib.gibbs_stats(self.r, self.Ft, self.yres, self.y, self.X, self.w, out=self._stats,
                              noise_w=self.noise_w).cpu().numpy()
        self.quad = float(st[0])
        # 4. tau2 | y, beta, w (weighted residual sum of squares; held fixed on request)
        if not self.fix_tau2:
            a, b = self.priors.tau2_ig
            self.tau2 = self._ig(a + 0.5 * n, b + 0.5 * float(st[1]))
        # 5. beta | y, w, tau2 (flat prior; weighted least squares)
        mean = self._XtX_inv @ st[2:]
        self.beta = mean + math.sqrt(self.tau2) * (self._XtX_inv_chol @ self.rng.standard_normal(self.p))
        self.yres = self._residual_y(self.beta)
        self.iteration += 1

    @property
    def w_input_order(self) -> torch.Tensor:
        """Current latent field w in the caller's location order (the state lives in Z-order storage)."""
        return self.w[self.pos]

    def sample(self, n_iter: int, burn: int = 0, thin: int = 1, keep_w_mean: bool = False):
        """Run n_iter iterations; return the thinned post-burn-in draws (numpy)."""
        out = {"beta": [], "sigma2": [], "tau2": [], "phi": []}
        w_sum = torch.zeros_like(self.w) if keep_w_mean else None
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
                kept += 1
        res = {k: np.asarray(v) for k, v in out.items()}
        res["phi_accept_rate"] = self.n_accept / max(self.iteration, 1)
        if keep_w_mean:
            res["w_mean"] = (w_sum / max(kept, 1))[self.pos].cpu().numpy()  # input order
        return res
