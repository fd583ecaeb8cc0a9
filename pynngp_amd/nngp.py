"""Drop-in ``NNGP`` class (mirrors ``pyNNGP.NNGP``, /root/reference/pyNNGP/nngp.py).

Same constructor ``NNGP(t, y, eps, refType, m, cov)`` (nngp.py:6-18), same
attributes ``t, y, eps, refType, m, cov, s, wt, ws, Ns, Nt`` and the same
per-location methods ``_Bsi, _CNs, _Ccross, _Fsi, _Cs`` (nngp.py:73-96) -- but the
neighbour sets, the B/F algebra and the log-likelihood run on the MI355X through
``libnngp_hip.so``.  Additions: the device-resident ``nbr`` / ``B`` / ``F`` arrays
and ``loglik()``, the sweep the reference's ``oneSample`` (nngp.py:98-101) needs.

Differences from the reference, all deliberate:
* ``cov`` is a :class:`Covariance` (kind + theta: the covariance fused into the kernel, the
  fast path), an :class:`IsotropicCovariance` (a torch function of distance), or -- as in the
  reference -- any Python callable ``cov(a, b)`` on coordinate rows (the reference passes index
  arrays at nngp.py:82, a bug; here the rows).  A callable drives ``_CNs/_Ccross/_Cs`` directly
  and ``_Bsi/_Fsi/compute_BF/loglik/predict`` through :class:`CallableCovariance` (its joint
  blocks evaluated, then factorised on the GPU by the covariance-block kernels, 1 <= m <= 32).
  ``cov=None`` (the reference test) builds neighbour sets only.
* exact distance ties are ordered by lower index (the reference's is arbitrary).
* tuple ``refType`` values work as the reference's comments describe
  (nngp.py:23-27, with the same ``np.random`` calls as nngp.py:36-40, so a seeded
  global RNG gives the S the reference meant to draw); the reference itself raises
  ``AttributeError`` there (``self.typ``, nngp.py:34).  An unknown string raises
  ``ValueError`` (the reference silently leaves ``s`` unset, nngp.py:29-31).
* ``Nt`` for refType != 'S=T' is a list of int64 index arrays into ``s`` (the
  reference appends ``(dist, ind)`` tuples, nngp.py:71, because ``return_distance``
  defaults to True); ``predict()`` evaluates B_t, F_t and the kriging mean at t
  (nngp_bf_cross).
"""
from __future__ import annotations

import dataclasses
import math
from typing import Callable, Optional, Union

import numpy as np
import torch

from . import _lib

LOG_2PI = math.log(2.0 * math.pi)


@dataclasses.dataclass(frozen=True)
class Covariance:
    """Parent-GP covariance plug-in (the reference's ``cov``, nngp.py:6,12), u = phi d:

    ``exponential`` sigma2 e^-u; ``matern32`` sigma2 (1 + u) e^-u; ``matern52``
    sigma2 (1 + u + u^2/3) e^-u; ``gaussian`` sigma2 e^-u^2; ``spherical``
    sigma2 (1 - 3u/2 + u^3/2) for u < 1, else 0 (the spNNGP family, fused in the kernels);
    ``matern`` sigma2 u^nu K_nu(u) / (2^(nu-1) Gamma(nu)) for any smoothness ``nu`` in (0, 50]
    (spNNGP's "matern"; served by the wavefront kernel, nngp.h NNGP_COV_MATERN).
    ``tau2`` is a nugget added to the diagonal (response model; 0 = latent model).
    Called as ``cov(a, b)`` on coordinate rows of any dimension (numpy or torch), it
    returns the cross-covariance matrix without the nugget, like a reference plug-in would.
    """

    kind: str
    sigma2: float
    phi: float
    tau2: float = 0.0
    nu: Optional[float] = None  # smoothness of the ``matern`` kind (None for the others)

    def __post_init__(self):
        if self.kind not in _lib.KIND_CODES:
            raise ValueError(f"unknown covariance kind {self.kind!r}; expected one of {sorted(_lib.KIND_CODES)}")
        if not (self.sigma2 > 0 and self.phi > 0 and self.tau2 >= 0):
            raise ValueError("need sigma2 > 0, phi > 0, tau2 >= 0")
        _lib._check_kind(self.kind, self.nu)

    @property
    def nu_arg(self) -> Optional[float]:
        """``nu`` as the sweeps take it (None unless the kind is ``matern``)."""
        return float(self.nu) if self.kind == "matern" else None

    @property
    def theta(self):
        return (float(self.sigma2), float(self.phi), float(self.tau2))

    def replace(self, **kw) -> "Covariance":
        return dataclasses.replace(self, **kw)

    def __call__(self, a, b):
        lib = torch if isinstance(a, torch.Tensor) else np
        d = a.shape[-1] if a.ndim > 1 else b.shape[-1] if b.ndim > 1 else 1
        a = a.reshape(-1, d)
        b = b.reshape(-1, d)
        t = a[:, None, :] - b[None, :, :]
        u = self.phi * lib.sqrt((t * t).sum(-1))
        if self.kind == "matern":  # K_nu of real order: scipy on the host (torch has only K_0, K_1)
            from scipy import special
            un = u.detach().cpu().numpy() if lib is torch else u
            us = np.where(un > 0, un, 1.0)
            with np.errstate(over="ignore", under="ignore", invalid="ignore", divide="ignore"):
                k = special.kv(self.nu, us)
                r = np.exp(self.nu * np.log(us) - (self.nu - 1.0) * np.log(2.0) - special.gammaln(self.nu) + np.log(k))
            r = self.sigma2 * np.where((un > 0) & np.isfinite(k), r, 1.0)
            return torch.as_tensor(r, dtype=u.dtype, device=u.device) if lib is torch else r
        if self.kind == "gaussian":
            return self.sigma2 * lib.exp(-u * u)
        if self.kind == "spherical":
            return lib.where(u < 1.0, self.sigma2 * (1.0 - 1.5 * u + 0.5 * u * u * u), 0.0 * u)
        e = self.sigma2 * lib.exp(-u)
        if self.kind == "matern32":
            return e * (1.0 + u)
        if self.kind == "matern52":
            return e * (1.0 + u + u * u / 3.0)
        return e


@dataclasses.dataclass(frozen=True)
class IsotropicCovariance:
    """A covariance of the caller's own -- the reference's `cov` plug-in (nngp.py:6,12) as any
    isotropic function of distance -- driving the fused GPU sweep: ``fn`` maps a float64 torch
    tensor of distances (any shape, on the GPU) to covariances elementwise (without the nugget;
    C(0) = ``fn(0)`` is the marginal variance), ``tau2`` is the nugget.  The sweep evaluates
    ``fn`` once over every joint block's distances (``_lib.joint_dist``, +inf for slots without
    a point, whose entries the kernel then ignores) and factorises the blocks in the
    ``bf_pairb`` kernel reading them from memory (nngp_bf_sweep_blocks, 1 <= m <= 24).
    Example: ``IsotropicCovariance(lambda d: 2.0 * torch.exp(-(d / 0.1) ** 1.5), tau2=0.1)``
    (a powered exponential).  Called as ``cov(a, b)`` on coordinate rows it returns the
    cross-covariance matrix, like a reference plug-in."""

    fn: Callable
    tau2: float = 0.0
    name: str = "custom"

    def __post_init__(self):
        if not callable(self.fn):
            raise TypeError("fn must be callable (a torch function of distance)")
        if not self.tau2 >= 0:
            raise ValueError("need tau2 >= 0")

    kind = "custom"

    @property
    def sigma2(self) -> float:
        """C(0) = fn(0), evaluated on the GPU when there is one (``fn`` may be a GPU-only function,
        e.g. one built on ``_lib.matern``)."""
        return self.variance("cuda" if torch.cuda.is_available() else "cpu")

    def variance(self, device) -> float:
        """C(0) = fn(0) evaluated on ``device``."""
        return float(self.fn(torch.zeros(1, dtype=torch.float64, device=device)).item())

    def marginal(self, points: torch.Tensor) -> torch.Tensor:
        """C(x, x) + tau2 at every point (the m = 0 prediction variance)."""
        return torch.full((points.shape[0],), self.variance(points.device) + self.tau2, dtype=torch.float64,
                          device=points.device)

    def blocks(self, dist: torch.Tensor, m: int) -> torch.Tensor:
        """Covariance blocks for :func:`_lib.bf_sweep_blocks`: fn over the distances, tau2 on the
        diagonal entries."""
        c = self.fn(dist)
        if not isinstance(c, torch.Tensor) or c.shape != dist.shape:
            raise ValueError("fn must return a tensor of the distances' shape")
        c = c.to(torch.float64).contiguous()
        if self.tau2 > 0:
            diag = _lib.joint_diagonal(m).to(c.device)
            c[diag] += self.tau2
        return c

    def __call__(self, a, b):
        to_np = not isinstance(a, torch.Tensor)
        ta = torch.as_tensor(np.asarray(a, dtype=np.float64)) if to_np else a
        tb = torch.as_tensor(np.asarray(b, dtype=np.float64)) if to_np else b
        d = ta.shape[-1] if ta.dim() > 1 else tb.shape[-1] if tb.dim() > 1 else 1
        ta, tb = ta.reshape(-1, d), tb.reshape(-1, d)
        t = ta[:, None, :] - tb[None, :, :]
        c = self.fn(torch.sqrt((t * t).sum(-1)))
        return c.cpu().numpy() if to_np else c


class CallableCovariance:
    """The reference's ``cov`` plug-in as it stands (``pyNNGP/nngp.py:6,12``): any callable
    ``fn(a, b)`` that maps two sets of coordinate rows (k_a, d) and (k_b, d) to their
    cross-covariance matrix (k_a, k_b) -- the call ``_CNs`` makes on the neighbours' rows
    (``nngp.py:82``) and ``_Cs`` on a location's row (``nngp.py:96``).  No isotropy or other
    structure is assumed (e.g. an anisotropic exponential exp(-sqrt((a-b)^T A (a-b)))).

    It drives the device sweep through the covariance-block kernels: for every location the joint
    block ``fn(X, X)`` of X = [its neighbours' rows; its own row] is evaluated, packed into
    ``_lib.bf_sweep_blocks``'s layout (lower triangle, entry-major) and factorised on the GPU
    (``nngp_bf_sweep_blocks``: B, F, residuals and the log-likelihood partials; 1 <= m <= 32).
    Evaluation, chosen once per object by probing ``fn`` on a few rows against one call per row:
      * ``"torch"``: ``fn`` broadcasts over a leading batch dimension of torch tensors on the GPU --
        one call per chunk of rows with X of shape (rows, m+1, d), on the device;
      * ``"numpy"``: the same with numpy arrays (host evaluation of the user's function, one call
        per chunk; the blocks then go to the GPU);
      * ``"loop"``: one call per location with the (m+1, d) numpy rows the reference passes.
    ``batch`` forces a mode.  The covariance values are the caller's code; everything after them
    (the factorisation, B, F, the log-likelihood) runs on the GPU, with no CPU path.
    ``tau2`` is an optional nugget added to the diagonal (0: ``fn``'s own values are C)."""

    kind = "custom"
    MODES = ("torch", "numpy", "loop", "loop_torch")

    def __init__(self, fn: Callable, tau2: float = 0.0, batch: Optional[str] = None, chunk_bytes: int = 1 << 28,
                 cache: bool = False, pairs: bool = False):
        if not callable(fn):
            raise TypeError("cov must be callable as cov(a, b) on coordinate rows")
        if not tau2 >= 0:
            raise ValueError("need tau2 >= 0")
        if batch is not None and batch not in self.MODES:
            raise ValueError(f"batch must be one of {self.MODES} or None")
        self.fn, self.tau2, self.batch, self.chunk_bytes = fn, float(tau2), batch, int(chunk_bytes)
        self.mode = batch
        # pairs=True: in "torch" mode, evaluate fn once per DISTINCT point pair of a sweep's joint blocks and
        # gather the blocks from those values (N = 1e6, m = 15: 30.5 M pairs instead of 136 M block entries),
        # when fn on single-row pairs reproduces its joint blocks bit for bit in both argument orders (probed
        # once).  Opt-in: the pair index costs ~42 ms per neighbour set (then cached), and a cheap broadcasting
        # plug-in evaluates (P, 1, 1)-shaped pairs at a lower per-element rate than whole blocks (17.2 against
        # 19.0 ms per sweep's blocks, profiles/r05o) -- it pays for an expensive fn reused over many sweeps
        self.pairs = pairs
        self._pairs_ok = None
        self._pidx = None  # (coords, nbr, order, i0, versions) -> the distinct pairs and the blocks' gather index
        # cache=True: NNGP keeps this covariance's evaluated joint blocks between sweeps (the caller promises
        # fn is a fixed function: no state it reads changes).  Default off, as the reference, which calls cov
        # on every evaluation (nngp.py:82,96): a mutable plug-in (an MLE loop over a closure's parameters)
        # then always sees its current state.
        self.cache = bool(cache)

    def __call__(self, a, b):
        return self.fn(a, b)

    # -- evaluation modes --------------------------------------------------------
    def _eval(self, X: torch.Tensor, mode: str) -> torch.Tensor:
        """fn's joint blocks (r, k, k) on X's device for X (r, k, d)."""
        if mode == "torch":
            C = self.fn(X, X)
            if not isinstance(C, torch.Tensor):
                raise TypeError("not a torch tensor")
            return C.to(device=X.device, dtype=torch.float64)
        Xh = X.detach().cpu().numpy()
        if mode == "numpy":
            C = np.asarray(self.fn(Xh, Xh), dtype=np.float64)
        elif mode == "loop":
            C = np.stack([np.asarray(self.fn(x, x), dtype=np.float64).reshape(x.shape[0], x.shape[0]) for x in Xh]) \
                if Xh.shape[0] else np.zeros((0, X.shape[1], X.shape[1]))
        else:  # loop_torch: one call per location with torch rows on the device
            return torch.stack([torch.as_tensor(self.fn(x, x), dtype=torch.float64, device=X.device).reshape(
                x.shape[0], x.shape[0]) for x in X]) if X.shape[0] else X.new_zeros((0, X.shape[1], X.shape[1]))
        return torch.from_numpy(np.ascontiguousarray(C)).to(X.device)

    def resolve_mode(self, X: torch.Tensor) -> str:
        """Pick (once) the fastest evaluation that reproduces one call per location on sample rows X
        (r, k, d): relative 1e-13 (a batched expression may round in a different order)."""
        if self.mode is not None:
            return self.mode
        ref, ref_mode = None, None
        for lm in ("loop", "loop_torch"):
            try:
                ref = self._eval(X, lm).cpu().numpy()
                ref_mode = lm
                break
            except Exception:  # noqa: BLE001 -- the plug-in decides what it accepts
                continue
        if ref is None:
            raise TypeError("cov(a, b) failed on the joint blocks' coordinate rows (numpy and torch (k, d) inputs)")
        k = X.shape[1]
        if ref.shape != (X.shape[0], k, k) or not np.all(np.isfinite(ref)):
            raise ValueError(f"cov(a, b) must return a finite ({k}, {k}) matrix for two ({k}, d) row sets")
        scale = float(np.max(np.abs(ref))) if ref.size else 1.0
        for bm in ("torch", "numpy"):
            try:
                C = self._eval(X, bm)
            except Exception:  # noqa: BLE001
                continue
            if tuple(C.shape) == ref.shape and np.allclose(C.cpu().numpy(), ref, rtol=1e-13, atol=1e-15 * scale):
                self.mode = bm
                return bm
        self.mode = ref_mode
        return ref_mode

    def _pairs_probe(self, X: torch.Tensor, ta: torch.Tensor, tb: torch.Tensor) -> bool:
        """fn on (P, 1, d) single-row pairs equals its joint blocks' entries bit for bit, in both argument
        orders (the distinct pairs are keyed by (smaller, larger) point index)."""
        if self._pairs_ok is None:
            try:
                C = self._eval(X, "torch")[:, ta, tb].reshape(-1)
                xa, xb = X[:, ta].reshape(-1, 1, X.shape[2]), X[:, tb].reshape(-1, 1, X.shape[2])
                ab = torch.as_tensor(self.fn(xa, xb), dtype=torch.float64, device=X.device).reshape(-1)
                ba = torch.as_tensor(self.fn(xb, xa), dtype=torch.float64, device=X.device).reshape(-1)
                self._pairs_ok = bool(torch.equal(ab, C) and torch.equal(ba, C))
            except Exception:  # noqa: BLE001 -- the plug-in decides what it accepts
                self._pairs_ok = False
        return self._pairs_ok

    def _pair_index(self, coords, nbr, i0, order, ta, tb):
        """The sweep's distinct point pairs (pa, pb: point indices, pa <= pb) and the blocks' gather index
        inv ((m+1)(m+2)/2, rows) into [0, values...] (0: an entry with a slot without a point -- unused by
        the kernels); cached for the same coords / nbr / order tensors (held, and their versions checked)."""
        key = (coords, nbr, order, int(i0), coords._version, nbr._version, None if order is None else order._version)
        c = self._pidx
        if c is not None and all(x is y for x, y in zip(c[0][:3], key[:3])) and c[0][3:] == key[3:]:
            return c[1]
        n = coords.shape[0]
        rows = nbr.shape[0]
        loc = (torch.arange(rows, device=nbr.device) if order is None else order.long()) + int(i0)
        idx = nbr.long()
        g = torch.cat([torch.where((idx >= 0) & (idx < n), idx, torch.full_like(idx, -1)), loc[:, None]], dim=1)
        ga, gb = g[:, ta].t(), g[:, tb].t()  # entry-major (ne, rows)
        keys = torch.where((ga >= 0) & (gb >= 0), torch.minimum(ga, gb) * n + torch.maximum(ga, gb),
                           torch.full_like(ga, -1))
        del g, ga, gb
        uniq, inv = torch.unique(keys, return_inverse=True)
        del keys
        # slot 0 of the values is the unused entries' (a key of -1 sorts first when present)
        if uniq.numel() and int(uniq[0]) < 0:
            uniq = uniq[1:]
        else:
            inv += 1
        res = (uniq // n, uniq % n, inv)
        self._pidx = (key, res)
        return res

    def blocks(self, coords: torch.Tensor, nbr: torch.Tensor, i0: int = 0, qcoords: Optional[torch.Tensor] = None,
               order: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Joint blocks in :func:`_lib.bf_sweep_blocks`'s layout ((m+1)(m+2)/2, rows): fn over
        [neighbour rows; the location's row] for every nbr row (a slot without a point repeats the
        location's row -- the kernel ignores its entries), tau2 on the diagonal entries."""
        m = nbr.shape[1]
        rows = nbr.shape[0]
        dev = nbr.device
        ne = (m + 1) * (m + 2) // 2
        out = torch.empty((ne, rows), dtype=torch.float64, device=dev)
        if rows == 0:
            return out
        a = torch.arange(m + 1, device=dev)
        ta = torch.repeat_interleave(a, a + 1)  # entry e = a (a+1)/2 + b: rows a, then b = 0..a
        tb = torch.cat([torch.arange(int(k) + 1, device=dev) for k in range(m + 1)])
        per_row = (m + 1) * (m + 1) * 8 * 3 + (m + 1) * coords.shape[1] * 8
        chunk = max(1, min(rows, self.chunk_bytes // per_row))
        X4 = joint_points(coords, nbr[:min(rows, 4)], i0, qcoords, None if order is None else order[:min(rows, 4)])
        mode = self.resolve_mode(X4)
        if (self.pairs and mode == "torch" and qcoords is None and dev.type == "cuda" and rows * ne < 2 ** 31
                and coords.shape[0] < 2 ** 31 and self._pairs_probe(X4, ta, tb)):
            pa, pb, inv = self._pair_index(coords, nbr, i0, order, ta, tb)
            vals = torch.empty(pa.numel() + 1, dtype=torch.float64, device=dev)
            vals[0] = 0.0
            # (a pair is a few doubles of fn's temporaries: chunks of millions of pairs keep the launches few)
            pchunk = max(1, 8 * self.chunk_bytes // (8 * (3 + 2 * coords.shape[1])))
            for p0 in range(0, pa.numel(), pchunk):
                p1 = min(pa.numel(), p0 + pchunk)
                C = self.fn(coords[pa[p0:p1]][:, None, :], coords[pb[p0:p1]][:, None, :])
                vals[1 + p0:1 + p1] = torch.as_tensor(C, dtype=torch.float64, device=dev).reshape(-1)
            torch.index_select(vals, 0, inv.reshape(-1), out=out.view(-1))
            if self.tau2 > 0:
                out[_lib.joint_diagonal(m).to(dev)] += self.tau2
            return out
        if mode.startswith("loop"):
            chunk = min(chunk, 4096)
        for r0 in range(0, rows, chunk):
            r1 = min(rows, r0 + chunk)
            # (rows r0.. of a sweep without a visiting order are the locations i0 + r0 ..: round 5 fix -- the
            # chunks after the first took i0 .. again, wrong blocks once rows exceeded one chunk, e.g. m = 27
            # beyond ~14 k rows; found by the distinct-pair evaluation's bit-identity test)
            X = joint_points(coords, nbr[r0:r1], i0 + (r0 if order is None else 0), qcoords,
                             None if order is None else order[r0:r1])
            C = self._eval(X, mode)
            if tuple(C.shape) != (r1 - r0, m + 1, m + 1):
                raise ValueError(f"cov(a, b) returned {tuple(C.shape)} for {r1 - r0} joint blocks of {m + 1} rows")
            out[:, r0:r1] = C[:, ta, tb].t()
        if self.tau2 > 0:
            out[_lib.joint_diagonal(m).to(dev)] += self.tau2
        return out

    def marginal(self, points: torch.Tensor) -> torch.Tensor:
        """C(x, x) + tau2 at every point (the m = 0 prediction variance): fn on each row alone."""
        X = points[:, None, :]
        return self._eval(X, self.resolve_mode(X[:4]))[:, 0, 0] + self.tau2


def joint_points(coords: torch.Tensor, nbr: torch.Tensor, i0: int = 0, qcoords: Optional[torch.Tensor] = None,
                 order: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Coordinates of every joint block, (rows, m+1, d): slots 0..m-1 the neighbours ``coords[nbr]``
    (a slot without a point -- index -1 or out of range -- repeats the location's row), slot m the
    location ``qcoords[i0 + (order[t] if order else t)]`` (``qcoords`` defaults to ``coords``)."""
    q = coords if qcoords is None else qcoords
    rows = nbr.shape[0]
    loc = (torch.arange(rows, device=nbr.device) if order is None else order.long()) + int(i0)
    xi = q[loc]
    idx = nbr.long()
    ok = (idx >= 0) & (idx < coords.shape[0])
    xn = coords[torch.where(ok, idx, torch.zeros_like(idx))]
    xn = torch.where(ok[..., None], xn, xi[:, None, :])
    return torch.cat([xn, xi[:, None, :]], dim=1)


CovLike = Union[Covariance, IsotropicCovariance, CallableCovariance, Callable, None]


def _sweep_any(cv, coords, nbr, i0=0, values=None, want_bf=True, algo="auto", order=None, R=None, qcoords=None,
               qvalues=None, blocks=None):
    """One fused sweep for any covariance form: a built-in kind (nngp_bf_sweep / nngp_bf_cross),
    an :class:`IsotropicCovariance` (joint distances -> fn -> nngp_bf_sweep_blocks) or a
    :class:`CallableCovariance` (fn(a, b) on the joint blocks' rows -> nngp_bf_sweep_blocks;
    ``blocks``: already evaluated blocks of these rows, e.g. cached).  ``qcoords``
    given: the cross sweep of those query points against ``coords`` (prediction); ``qvalues``: the
    values at the locations (S = T sweep: pass ``values``)."""
    if isinstance(cv, (IsotropicCovariance, CallableCovariance)):
        m = nbr.shape[1]
        if not 1 <= m <= _lib.BLOCKS_MAX_M:
            raise ValueError(f"a custom covariance needs 1 <= m <= {_lib.BLOCKS_MAX_M} (the covariance-block kernels)")
        if algo not in ("auto", "pairb", "quad"):
            raise ValueError(f"a custom covariance runs on the covariance-block kernels, not algo {algo!r}")
        if blocks is None and isinstance(cv, CallableCovariance):
            blocks = cv.blocks(coords, nbr, i0, qcoords=qcoords, order=order)
        elif blocks is None:
            dist = _lib.joint_dist(coords, nbr, i0, qcoords=qcoords, order=order)
            blocks = cv.blocks(dist, m)
            del dist
        nq = (coords if qcoords is None else qcoords).shape[0]
        return _lib.bf_sweep_blocks(blocks, nbr, coords.shape[0], i0, values=values, qvalues=qvalues, want_bf=want_bf,
                                    order=order, R=R, n_locs=nq)
    if qcoords is not None:
        return _lib.bf_cross(coords, qcoords, nbr, cv.kind, *cv.theta, ref_values=values, query_values=qvalues,
                             q0=i0, algo=algo, R=R, nu=cv.nu_arg)
    return _lib.bf_sweep(coords, nbr, i0, cv.kind, *cv.theta, values=values, want_bf=want_bf, algo=algo, order=order,
                         R=R, nu=cv.nu_arg)


def _default_device(device):
    if device is not None:
        return torch.device(device)
    if not torch.cuda.is_available():
        raise _lib.NNGPExtensionError("pynngp_amd.NNGP needs a ROCm GPU (torch.cuda.is_available() is False)")
    return torch.device("cuda", torch.cuda.current_device())


class NNGP:
    """Nearest-neighbour GP over ordinates ``t`` (mirrors ``pyNNGP.NNGP``)."""

    def __init__(self, t, y, eps, refType, m, cov: CovLike, device=None):
        self.t = t  # ordinates (held by reference, nngp.py:7)
        self.y = y  # abscissae
        self.eps = eps  # measurement uncertainties in y (stored, unused: SURVEY Appendix A)
        self.refType = refType
        self.m = int(m)
        self.cov = cov
        self.device = _default_device(device)
        if not 0 <= self.m <= _lib.MAX_M:
            raise ValueError(f"m={m} outside [0, {_lib.MAX_M}]")

        self._init_s()
        self._init_wt()
        self._init_ws()
        self._make_s_neighbor_sets()
        self._make_t_neighbor_sets()
        self._B = self._F = None

    # -- construction (nngp.py:21-71) -----------------------------------------
    def _init_s(self):
        """Reference set S (nngp.py:21-40): 'S=T', ('subset', nRef) or ('random', nRef, bounds)."""
        self.s = reference_set(self.t, self.refType)
        t_host = np.ascontiguousarray(self.t, dtype=np.float64)
        if not np.all(np.isfinite(t_host)):  # as sklearn's KDTree / KNeighborsRegressor (nngp.py:46,55)
            raise ValueError("Input contains NaN or infinity (ordinates t)")
        if t_host.ndim == 1:  # a 1-D series given as a vector
            t_host = t_host[:, None]
        self._t_dev = torch.as_tensor(t_host).to(self.device)
        if self._t_dev.dim() != 2 or not 1 <= self._t_dev.shape[1] <= _lib.MAX_DIM:
            raise ValueError(f"ordinates must be (N, d) with 1 <= d <= {_lib.MAX_DIM}, got {tuple(self._t_dev.shape)}")
        if self.s is self.t:
            self._s_dev = self._t_dev
        else:
            s_host = np.ascontiguousarray(self.s, dtype=np.float64)
            if s_host.ndim == 1:
                s_host = s_host[:, None]
            if not np.all(np.isfinite(s_host)):
                raise ValueError("Input contains NaN or infinity (reference set s)")
            self._s_dev = torch.as_tensor(s_host).to(self.device)
            if (self._s_dev.dim() != 2 or self._s_dev.shape[1] != self._t_dev.shape[1]
                    or self._s_dev.shape[0] < 1):
                raise ValueError(f"reference set must be (nRef >= 1, {self._t_dev.shape[1]}), "
                                 f"got {tuple(self._s_dev.shape)}")

    def _init_wt(self):
        self.wt = np.copy(self.y)

    def _init_ws(self, k: int = 5):
        """5-NN uniform regression of y on t at s (nngp.py:45-47) on the GPU."""
        n = self._t_dev.shape[0]
        if n < k:
            raise ValueError(f"Expected n_neighbors <= n_samples_fit, but n_neighbors = {k}, n_samples_fit = {n}")
        idx = _lib.knn_query(self._t_dev, self._s_dev, k).long()
        y = torch.as_tensor(np.asarray(self.y, dtype=np.float64)).to(self.device)
        self.ws = y[idx].mean(dim=1).cpu().numpy()

    def _make_s_neighbor_sets(self):
        self.nbr = _lib.knn_prior(self._s_dev, self.m)  # int32 (N, m) on the device, -1 padded
        # Z-order visiting order + neighbour rows in that order, for the sweeps (speed only)
        self._order, self._nbr_sorted = _lib.row_order(self._s_dev, nbr=self.nbr)
        self._Ns = None

    def set_neighbor_sets(self, nbr: torch.Tensor):
        """Replace the neighbour sets (int32 (N, m) device tensor, -1 padded, prior indices)."""
        if nbr.shape != self.nbr.shape or nbr.dtype != torch.int32:
            raise ValueError(f"nbr must be int32 {tuple(self.nbr.shape)}")
        self.nbr = nbr.to(self.device).contiguous()
        self._order, self._nbr_sorted = _lib.row_order(self._s_dev, nbr=self.nbr)
        self._Ns = None
        self._B = self._F = None
        self._blk_cache = None

    def _make_t_neighbor_sets(self):
        """'S=T': Nt aliases Ns (nngp.py:65-67); otherwise the m nearest points of S to
        every t (nngp.py:68-71), ascending, on the GPU (nngp_knn_query)."""
        self._Nt = None
        if self._same_sets():
            self.nbr_t = None
            return
        k = min(self.m, self._s_dev.shape[0])
        self.nbr_t = _lib.knn_query(self._s_dev, self._t_dev, k) if k > 0 else torch.empty(
            (self._t_dev.shape[0], 0), dtype=torch.int32, device=self.device)

    def _same_sets(self) -> bool:
        return isinstance(self.refType, str) and self.refType == "S=T"

    @property
    def Ns(self):
        """Reference format: list with ``Ns[0] == []`` and int64 arrays of min(i, m) indices."""
        if self._Ns is None:
            a = self.nbr.cpu().numpy().astype(np.int64)
            ns = [[]]
            for i in range(1, a.shape[0]):
                ns.append(a[i, : min(i, self.m)])
            self._Ns = ns
        return self._Ns

    @property
    def Nt(self):
        """'S=T': the same object as ``Ns``; otherwise one int64 index array into ``s`` per t."""
        if self._same_sets():
            return self.Ns
        if self._Nt is None:
            a = self.nbr_t.cpu().numpy().astype(np.int64)
            self._Nt = [row for row in a]
        return self._Nt

    # -- prediction at t ------------------------------
    def predict(self, values=None, cov: Optional[Covariance] = None, query=None, algo: str = "auto"):
        """Kriging of the NNGP at the points ``query`` (default ``t``) from ``values`` on S
        (default ``ws``): returns numpy ``(mean, var)`` with mean_t = B_t v_N(t) and
        var_t = F_t (conditional variance; includes tau2 like C_tt = sigma2 + tau2).
        Neighbours: the m nearest points of S to each query point (for query = t with
        refType != 'S=T' these are ``Nt``)."""
        cv = self._covariance(cov)
        v = self.ws if values is None else values
        v = torch.as_tensor(np.asarray(v, dtype=np.float64) if not isinstance(v, torch.Tensor) else v,
                            dtype=torch.float64).to(self.device)
        if v.shape != (self._s_dev.shape[0],):
            raise ValueError(f"values must have one entry per reference point ({self._s_dev.shape[0]})")
        if query is None and not self._same_sets():
            q, nbr = self._t_dev, self.nbr_t
        else:
            q = self._t_dev if query is None else torch.as_tensor(
                np.ascontiguousarray(query, dtype=np.float64)).to(self.device)
            k = min(self.m, self._s_dev.shape[0])
            nbr = _lib.knn_query(self._s_dev, q, k)
        n = q.shape[0]
        if nbr.shape[1] == 0:  # m = 0: the marginal
            if isinstance(cv, Covariance):
                return np.zeros(n), np.full(n, cv.sigma2 + cv.tau2)
            return np.zeros(n), cv.marginal(q).cpu().numpy()
        R = torch.empty(n, dtype=torch.float64, device=self.device)
        _, F, p = _sweep_any(cv, self._s_dev, nbr, 0, values=v, algo=algo, R=R, qcoords=q)
        _raise_on_bad(p.cpu().numpy())
        return (-R).cpu().numpy(), F.cpu().numpy()

    # -- covariance plumbing ---------------------------------------------------
    def _covariance(self, cov=None):
        """The covariance the device sweeps use: ``cov`` (default ``self.cov``); a plain callable
        ``cov(a, b)`` becomes a :class:`CallableCovariance` (one per callable, so its evaluation mode
        is probed once)."""
        c = self.cov if cov is None else cov
        if isinstance(c, (Covariance, IsotropicCovariance, CallableCovariance)):
            return c
        if c is None or not callable(c):
            raise TypeError("the device B/F sweep needs a covariance: pynngp_amd.Covariance(kind, sigma2, phi, tau2[, "
                            f"nu]), IsotropicCovariance(fn, tau2) or a callable cov(a, b) (got {type(c).__name__})")
        wrapped = getattr(self, "_wrapped_cov", None)
        if wrapped is None or wrapped.fn is not c:
            wrapped = CallableCovariance(c)
            self._wrapped_cov = wrapped
        return wrapped

    def _field_blocks(self, cv):
        """Joint blocks of the whole field (Z-order rows) for a :class:`CallableCovariance` (None for the
        other covariance forms).  Evaluating them is the caller's code and the most expensive step; with
        ``CallableCovariance(fn, cache=True)`` they are kept for the next sweep (8 (m+1)(m+2)/2 bytes per
        location of device memory), keyed on the object, its nugget and the neighbour sets
        (:meth:`clear_cache` drops them); by default every sweep evaluates the plug-in again, as the
        reference calls ``cov`` on every evaluation (advice r04: a mutable plug-in must not see stale
        blocks)."""
        if not isinstance(cv, CallableCovariance):
            return None
        hit = getattr(self, "_blk_cache", None)
        if cv.cache and hit is not None and hit[0] is cv and hit[1] is self._nbr_sorted and hit[2] == cv.tau2:
            return hit[3]
        self._blk_cache = None
        blk = cv.blocks(self._s_dev, self._nbr_sorted, 0, order=self._order)
        if cv.cache:
            self._blk_cache = (cv, self._nbr_sorted, cv.tau2, blk)
        return blk

    def clear_cache(self):
        """Drop kept covariance blocks and factors (a cached plug-in's parameters changed)."""
        self._blk_cache = None
        self._B = self._F = None

    def _nbr_idx(self, i):
        row = self.nbr[i]
        return row[row >= 0].long()

    def _call_cov(self, a, b):
        if self.cov is None:
            raise TypeError("cov is None")
        if isinstance(self.cov, (Covariance, IsotropicCovariance)):
            return self.cov(a, b)
        return self.cov(a.cpu().numpy(), b.cpu().numpy())  # the reference's rows are numpy (nngp.py:7,31)

    # -- per-location algebra (nngp.py:73-96) ----------------------------------
    def _CNs(self, i):
        """C_{N(s_i)} (nngp.py:78-82), with the nugget on the diagonal for a Covariance."""
        x = self._s_dev[self._nbr_idx(i)]
        c = self._call_cov(x, x)
        if isinstance(self.cov, (Covariance, IsotropicCovariance)) and self.cov.tau2 > 0:
            c = c + self.cov.tau2 * torch.eye(x.shape[0], dtype=c.dtype, device=c.device)
        return c.cpu().numpy() if isinstance(c, torch.Tensor) else c

    def _Ccross(self, i):
        """C_{s_i, N(s_i)} (nngp.py:84-86), shape (1, k)."""
        c = self._call_cov(self._s_dev[i][None, :], self._s_dev[self._nbr_idx(i)])
        return c.cpu().numpy() if isinstance(c, torch.Tensor) else c

    def _Cs(self, i):
        """C_{s_i, s_i} (nngp.py:92-96), with the nugget for a Covariance."""
        x = self._s_dev[i][None, :]
        c = self._call_cov(x, x)
        if isinstance(self.cov, (Covariance, IsotropicCovariance)):
            c = c + self.cov.tau2
        return c.cpu().numpy() if isinstance(c, torch.Tensor) else c

    def _row_bf(self, i):
        cv = self._covariance()
        B, F, p = _sweep_any(cv, self._s_dev, self.nbr[i: i + 1], int(i))
        _raise_on_bad(p.cpu().numpy())
        k = min(int(i), self.m)
        return B[0, :k].cpu().numpy(), float(F[0].item())

    def _Bsi(self, i):
        """B_{s_i} = C_{s_i,N} C_N^{-1} (nngp.py:73-76) from the device kernel."""
        return self._row_bf(i)[0]

    def _Fsi(self, i):
        """F_{s_i} = C_ii - B_i C_{N,s_i} (nngp.py:88-90) from the device kernel."""
        return self._row_bf(i)[1]

    # -- whole-field sweep -----------------------------------------------------
    def compute_BF(self, algo: str = "auto"):
        """All B (N, m) and F (N,) as device tensors (one fused sweep)."""
        cv = self._covariance()
        B, F, p = _sweep_any(cv, self._s_dev, self._nbr_sorted, 0, algo=algo, order=self._order,
                             blocks=self._field_blocks(cv))
        _raise_on_bad(p.cpu().numpy())
        self._B, self._F = B, F
        return B, F

    @property
    def B(self):
        return self.compute_BF()[0] if self._B is None else self._B

    @property
    def F(self):
        return self.compute_BF()[1] if self._F is None else self._F

    def loglik(self, values=None, cov: Optional[Covariance] = None, algo: str = "auto") -> float:
        """NNGP log density of ``values`` (default ``y``): -1/2 sum [log 2pi + log F + r^2/F]."""
        cv = self._covariance(cov)
        v = self.y if values is None else values
        v = torch.as_tensor(np.asarray(v, dtype=np.float64) if not isinstance(v, torch.Tensor) else v,
                            dtype=torch.float64).to(self.device)
        if v.dim() != 1 or v.shape[0] != self.nbr.shape[0]:
            raise ValueError(f"loglik needs one value per location ({self.nbr.shape[0]}, 1-D)")
        _, _, p = _sweep_any(cv, self._s_dev, self._nbr_sorted, 0, values=v, qvalues=v, want_bf=False, algo=algo,
                             order=self._order, blocks=self._field_blocks(cv))
        ph = p.cpu().numpy()
        _raise_on_bad(ph)
        n = self.nbr.shape[0]
        return -0.5 * (n * LOG_2PI + ph[0] + ph[1])

    def profile_loglik(self, cov: Covariance, values=None, mean: str = "constant", algo: str = "auto"):
        """NNGP log-likelihood of ``values`` (default y) at ``cov`` with a constant mean
        profiled out by GLS under the NNGP precision (I - B)^T F^-1 (I - B):
        mu = sum(r1 ry / F) / sum(r1^2 / F), r1 = (I - B) 1, ry = (I - B) y (two fused
        sweeps with residual output).  ``mean="zero"`` is :meth:`loglik`.  Returns
        ``(loglik, mu)``."""
        v = self.y if values is None else values
        v = torch.as_tensor(np.asarray(v, dtype=np.float64) if not isinstance(v, torch.Tensor) else v,
                            dtype=torch.float64).to(self.device)
        if mean == "zero":
            return self.loglik(v, cov, algo), 0.0
        if mean != "constant":
            raise ValueError("mean must be 'constant' or 'zero'")
        n = v.shape[0]
        ry = torch.empty(n, dtype=torch.float64, device=self.device)
        r1 = torch.empty_like(ry)
        cov = self._covariance(cov)
        kw = dict(algo=algo, order=self._order, blocks=self._field_blocks(cov))
        _, F, py = _sweep_any(cov, self._s_dev, self._nbr_sorted, 0, values=v, qvalues=v, R=ry, **kw)
        ones = torch.ones_like(v)
        _, _, p1 = _sweep_any(cov, self._s_dev, self._nbr_sorted, 0, values=ones, qvalues=ones, R=r1, **kw)
        s_y1 = torch.sum(ry * r1 / F)
        sums = torch.stack([py[0], py[1], p1[1], s_y1, py[2], py[3]]).cpu().numpy()
        _raise_on_bad(np.array([0.0, 0.0, sums[4], sums[5]]))
        logF, qyy, q11, qy1 = sums[:4]
        mu = qy1 / q11
        quad = qyy - 2.0 * mu * qy1 + mu * mu * q11
        return -0.5 * (n * LOG_2PI + logF + quad), float(mu)

    def fit(self, kind: Optional[str] = None, x0=None, mean: str = "constant", fix_tau2: Optional[float] = None,
            method: str = "Nelder-Mead", maxiter: int = 400, algo: str = "auto", nu: Optional[float] = None):
        """Maximum-likelihood (sigma2, phi, tau2) of the NNGP response model on S = T, each
        objective evaluation one or two fused GPU sweeps (scipy.optimize on log-parameters).
        ``x0`` defaults to ``cov``'s theta; ``fix_tau2`` holds the nugget fixed (e.g. 0 for the
        latent model); ``nu`` the (fixed) smoothness of the ``matern`` kind, default ``cov``'s.
        Sets ``cov`` to the estimate and returns a dict with theta, mu, loglik and the
        optimizer's evaluation count."""
        from scipy.optimize import minimize

        base = self.cov if isinstance(self.cov, Covariance) else None
        kind = kind or (base.kind if base is not None else "exponential")
        if nu is None and base is not None and base.kind == kind:
            nu = base.nu
        th0 = tuple(x0) if x0 is not None else (base.theta if base is not None else (1.0, 10.0, 0.1))
        free_tau = fix_tau2 is None
        z0 = [math.log(th0[0]), math.log(th0[1])] + ([math.log(max(th0[2], 1e-6))] if free_tau else [])

        def theta_of(z):
            return (math.exp(z[0]), math.exp(z[1]), math.exp(z[2]) if free_tau else float(fix_tau2))

        best = {"ll": -math.inf}

        def obj(z):
            th = theta_of(z)
            try:
                ll, mu = self.profile_loglik(Covariance(kind, *th, nu=nu), mean=mean, algo=algo)
            except NNGPNumericalError:
                return 1e300
            if ll > best["ll"]:
                best.update(ll=ll, mu=mu, theta=th)
            return -ll

        res = minimize(obj, np.array(z0), method=method, options={"maxiter": maxiter, "xatol": 1e-6,
                                                                  "fatol": 1e-9} if method == "Nelder-Mead"
                       else {"maxiter": maxiter})
        self.cov = Covariance(kind, *best["theta"], nu=nu)
        self._B = self._F = None
        return {"theta": best["theta"], "mu": best["mu"], "loglik": best["ll"], "n_evals": int(res.nfev),
                "converged": bool(res.success)}

    def oneSample(self, seed: int = 0, X=None, **sampler_kw):
        """One Gibbs iteration of the response model y = X beta + w + eps: the reference's
        ``update_wt`` / ``update_ws`` / ``update_y_unobserved`` (nngp.py:98-101, which do not
        exist there), delegated to :class:`pynngp_amd.SeqNNGP`, created on the first call
        with (sigma2, phi, tau2) from ``cov`` and w initialised from ``ws`` (reference
        points) and ``wt`` (data locations outside S; NaN -> 0).  'S=T': the field lives on
        the data locations; tuple refTypes: on S, with each data location outside S a leaf
        linked to its ``Nt`` (nngp.py:64-71).  ``X`` defaults to an intercept (pass
        ``X_ref`` for the covariates at S to get predictive draws there).  ``eps``
        (nngp.py:9, "measurement uncertainties in y"), when it is one positive sigma per
        location, makes the noise heteroscedastic: variance tau2 eps_i^2 (see SeqNNGP;
        ``fix_tau2=True`` with tau2 = 1 for exactly eps_i^2).  Afterwards ``ws`` / ``wt``
        hold the current w at S / T and ``y_unobserved`` the current predictive draws.
        Returns the sampler (its ``beta, sigma2, tau2, phi`` are the other draws).  With the
        reference's plug-in ``cov(a, b)`` (a callable) the covariance is held fixed: its blocks are
        evaluated once, and w, tau2 and beta are sampled (no phi / sigma2: the callable has no such
        parameters; its nugget ``CallableCovariance(fn, tau2)`` starts tau2)."""
        y = np.asarray(self.y, dtype=np.float64)
        if y.ndim != 1:
            raise ValueError("oneSample needs one response per location (1-D y)")
        if getattr(self, "_sampler", None) is None:
            from .gibbs import SeqNNGP

            cv = self._covariance()
            if isinstance(cv, IsotropicCovariance):
                raise TypeError("the Gibbs sampler takes a built-in covariance kind (pynngp_amd.Covariance) or the "
                                "reference's plug-in cov(a, b) (a callable / CallableCovariance), not an "
                                "IsotropicCovariance: write it as cov(a, b)")
            if "eps" not in sampler_kw and self.eps is not None:
                ev = np.asarray(self.eps, dtype=np.float64)
                if ev.shape == y.shape and np.all(np.isfinite(ev)) and np.all(ev > 0):
                    sampler_kw["eps"] = ev
            ref = None if self._same_sets() else self.s
            if isinstance(cv, CallableCovariance):
                # the plug-in held fixed: w, tau2, beta sampled; no phi / sigma2 (the callable carries its own
                # scale); the nugget, when given, starts tau2
                tau2 = cv.tau2 if cv.tau2 > 0 else 0.1
                smp = SeqNNGP(self.t, y, X=X, m=self.m, cov=cv, tau2=tau2, seed=seed, device=self.device, ref=ref,
                              **sampler_kw)
            else:
                tau2 = cv.tau2 if cv.tau2 > 0 else 0.1 * cv.sigma2
                smp = SeqNNGP(self.t, y, X=X, m=self.m, kind=cv.kind, sigma2=cv.sigma2, tau2=tau2, phi=cv.phi,
                              seed=seed, device=self.device, ref=ref, nu=cv.nu_arg, **sampler_kw)
            ws = np.asarray(self.ws, dtype=np.float64)
            smp.set_w(ws=np.where(np.isfinite(ws), ws, 0.0),
                      wt=None if ref is None else np.where(np.isfinite(self.wt), self.wt, 0.0))
            self._sampler = smp
        self._sampler.step()
        self.ws = self._sampler.w_s.cpu().numpy()
        self.wt = self._sampler.w_t.cpu().numpy()
        self.y_unobserved = self._sampler.y_unobserved.cpu().numpy()
        return self._sampler


def reference_set(t, refType):
    """S for a refType (nngp.py:21-40).  The tuple forms draw from numpy's global RNG with
    the reference's own calls: ('subset', nRef) -> t[np.random.choice(len(t), size=nRef)]
    (with replacement, as nngp.py:36); ('random', nRef, bounds) -> one
    np.random.uniform(lo, hi, nRef) column per (lo, hi) in bounds (nngp.py:39-40)."""
    if isinstance(refType, str):
        if refType != "S=T":
            raise ValueError(f"unknown refType {refType!r} (only 'S=T' is a string option)")
        return t
    if isinstance(refType, tuple) and len(refType) >= 2:
        typ = refType[0]
        if typ == "subset":
            choice = np.random.choice(len(t), size=int(refType[1]))
            return np.asarray(t)[choice]
        if typ == "random":
            if len(refType) < 3:
                raise ValueError("('random', nRef, bounds) needs bounds")
            nRef, bounds = int(refType[1]), refType[2]
            return np.vstack([np.random.uniform(lo, hi, nRef) for lo, hi in bounds]).T
        raise ValueError(f"unknown refType kind {typ!r} (expected 'subset' or 'random')")
    raise TypeError(f"refType must be 'S=T' or a tuple, got {refType!r}")


class NNGPNumericalError(ArithmeticError):
    """A location's neighbour covariance was not positive definite."""


def _raise_on_bad(partials_host) -> None:
    if partials_host[3] >= 0:
        raise IndexError(f"neighbour index out of range at location {int(partials_host[3])}")
    if partials_host[2] >= 0:
        raise NNGPNumericalError(
            f"non-positive Cholesky pivot or F at location {int(partials_host[2])} (add a nugget tau2 or change phi)")
