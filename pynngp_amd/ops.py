"""PyTorch-ROCm operators ``torch.ops.nngp.*`` (native: ``libnngp_torch_ops.so``).

The operators are registered in C++ with ``TORCH_LIBRARY(nngp, ...)``
(``pynngp_amd/csrc/torch_ops.cpp``) and implemented for the CUDA (= HIP on ROCm)
dispatch key only, straight over the C ABI of ``libnngp_hip.so`` on torch's current
stream: CPU tensors raise, there is no fallback.  :func:`load` (called by
``pynngp_amd.load_ops()`` and by the classes that sweep through these ops) loads the
library, loudly failing when it is not built, and registers the fake (meta) kernels used
for tracing.

    torch.ops.nngp.knn_prior(coords, m, q0, q1) -> nbr
    torch.ops.nngp.knn_prior_rows(coords, m, rows) -> nbr
    torch.ops.nngp.knn_query(ref, query, k) -> nbr
    torch.ops.nngp.bf_sweep(coords, nbr, i0, kind, sigma2, phi, tau2, values, want_bf, algo, order=None, nu=-1.0)
        -> (B, F, partials)
    torch.ops.nngp.bf_sweep_out(coords, nbr, order, i0, kind, sigma2, phi, tau2, values, B, F, R, partials,
                                workspace, algo, nu=-1.0, plan=None, plan_info=None) -> ()
                                                                      # the hot path: caller-owned buffers
    torch.ops.nngp.pair_plan(nbr, order, i0, n_points, dim) -> (plan, plan_info)   # wave pair plan (setup)
    torch.ops.nngp.bf_cross(ref, query, nbr, kind, sigma2, phi, tau2, ref_values, algo, nu=-1.0) -> (B, F, mean)
    torch.ops.nngp.row_order(coords, i0, rows, nbr) -> (order, nbr_sorted)
    torch.ops.nngp.combine_partials_out(gathered, out) -> ()

``kind`` / ``algo`` are the integer codes of include/nngp.h (:func:`kind_code`, :func:`algo_code`);
``nu`` is the smoothness of the ``matern`` kind (0 < nu <= 50; ignored by the other kinds).
"""
from __future__ import annotations

import os

import torch

from . import _lib

_KINDS = tuple(_lib.KIND_CODES)  # code order: exponential, matern32, matern52, gaussian, spherical, matern
_ALGOS = dict(_lib.ALGO_CODES)
# always the in-tree build; it binds to whichever libnngp_hip.so _lib loaded first (matched by
# SONAME, so an NNGP_LIB variant build is the one the operators call)
LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_build", "libnngp_torch_ops.so")

_loaded = False


def load() -> None:
    """Load the operator library once (it links libnngp_hip.so); raise if it is not built."""
    global _loaded
    if _loaded:
        return
    if not os.path.exists(LIB_PATH):
        raise _lib.NNGPExtensionError(
            f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(pynngp_amd has no CPU fallback)")
    _lib.load()  # the libnngp_hip.so the op library links (one copy in the process)
    torch.ops.load_library(LIB_PATH)
    _register_fakes()
    _loaded = True


def _register_fakes() -> None:
    def fake(name):
        return torch.library.register_fake(f"nngp::{name}")

    @fake("knn_prior")
    def _(coords, m, q0, q1):
        return coords.new_empty((q1 - q0, m), dtype=torch.int32)

    @fake("knn_prior_rows")
    def _(coords, m, rows):
        return coords.new_empty((rows.shape[0], m), dtype=torch.int32)

    @fake("knn_query")
    def _(ref, query, k):
        return query.new_empty((query.shape[0], k), dtype=torch.int32)

    @fake("bf_sweep")
    def _(coords, nbr, i0, kind, sigma2, phi, tau2, values, want_bf, algo, order=None, nu=-1.0):
        rows, m = nbr.shape
        if want_bf:
            return coords.new_empty((rows, m)), coords.new_empty((rows,)), coords.new_empty((4,))
        return coords.new_empty((0, m)), coords.new_empty((0,)), coords.new_empty((4,))

    @fake("bf_sweep_out")
    def _(coords, nbr, order, i0, kind, sigma2, phi, tau2, values, B, F, R, partials, workspace, algo, nu=-1.0,
          plan=None, plan_info=None):
        return None

    @fake("pair_plan")
    def _(nbr, order, i0, n_points, dim):
        raise RuntimeError("pair_plan is a setup call (it synchronises to read its tile counts): build it eagerly")

    @fake("bf_cross")
    def _(ref, query, nbr, kind, sigma2, phi, tau2, ref_values, algo, nu=-1.0):
        rows, m = nbr.shape
        return query.new_empty((rows, m)), query.new_empty((rows,)), query.new_empty((rows,))

    @fake("row_order")
    def _(coords, i0, rows, nbr):
        srt = torch.empty_like(nbr) if nbr is not None else coords.new_empty((0, 0), dtype=torch.int32)
        return coords.new_empty((rows,), dtype=torch.int32), srt

    @fake("combine_partials_out")
    def _(gathered, out):
        return None


def kind_code(kind: str) -> int:
    try:
        return _KINDS.index(kind)
    except ValueError:
        raise ValueError(f"unknown covariance kind {kind!r}; expected one of {_KINDS}") from None


def algo_code(algo: str) -> int:
    try:
        return _ALGOS[algo]
    except KeyError:
        raise ValueError(f"unknown algo {algo!r}; expected one of {tuple(_ALGOS)}") from None


def bf_sweep_out(coords, nbr, order, i0, kind: str, theta, values, B, F, R, partials, workspace,
                 algo: str = "auto", plan=None) -> None:
    """The fused sweep into caller-owned buffers through ``torch.ops.nngp.bf_sweep_out``
    (stream-ordered on torch's current stream, no host synchronisation).  ``theta`` =
    (sigma2, phi, tau2), or (sigma2, phi, tau2, nu) for the ``matern`` kind.  ``plan``: a
    ``(plan, plan_info)`` pair from :func:`pair_plan` for this nbr / order / i0."""
    load()
    nu = float(theta[3]) if len(theta) > 3 else -1.0
    pbuf, pinfo = plan if plan is not None else (None, None)
    torch.ops.nngp.bf_sweep_out(coords, nbr, order, int(i0), kind_code(kind), float(theta[0]), float(theta[1]),
                                float(theta[2]), values, B, F, R, partials, workspace, algo_code(algo), nu, pbuf,
                                pinfo)


def pair_plan(nbr, order, i0: int, n_points: int, dim: int):
    """The wave pair plan of a sweep over ``nbr`` (``torch.ops.nngp.pair_plan``): ``(plan, plan_info)``.
    A setup call (one host synchronisation); stale once nbr or order change."""
    load()
    return torch.ops.nngp.pair_plan(nbr, order, int(i0), int(n_points), int(dim))


def pair_plan_supported(m: int, kind: str, dim: int) -> bool:
    return _lib.pair_plan_supported(m, kind, dim)

