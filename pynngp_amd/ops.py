"""PyTorch-ROCm custom ops over the C ABI: ``torch.ops.nngp.*``.

Registered with ``torch.library.custom_op`` for the CUDA (= HIP on ROCm)
dispatch key only, so CPU tensors raise instead of silently falling back.
Fake (meta) kernels give shapes for tracing.

    torch.ops.nngp.bf_sweep(coords, nbr, i0, kind, sigma2, phi, tau2, values, want_bf, algo)
        -> (B, F, partials)
    torch.ops.nngp.knn_prior(coords, m, q0, q1) -> nbr
    torch.ops.nngp.knn_query(ref, query, k) -> nbr
    torch.ops.nngp.bf_cross(ref, query, nbr, kind, sigma2, phi, tau2, ref_values, algo) -> (B, F, mean)
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from . import _lib

_KINDS = ("exponential", "matern32")
_ALGOS = ("auto", "lane", "wave", "pair", "quad", "pairb")


@torch.library.custom_op("nngp::bf_sweep", mutates_args=(), device_types="cuda")
def bf_sweep(coords: torch.Tensor, nbr: torch.Tensor, i0: int, kind: int, sigma2: float, phi: float, tau2: float,
             values: Optional[torch.Tensor], want_bf: bool, algo: int) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    B, F, partials = _lib.bf_sweep(coords, nbr, i0, _KINDS[kind], sigma2, phi, tau2, values, want_bf, _ALGOS[algo])
    if not want_bf:
        rows, m = nbr.shape
        B = coords.new_empty((0, m))
        F = coords.new_empty((0,))
    return B, F, partials


@bf_sweep.register_fake
def _(coords, nbr, i0, kind, sigma2, phi, tau2, values, want_bf, algo):
    rows, m = nbr.shape
    if want_bf:
        return coords.new_empty((rows, m)), coords.new_empty((rows,)), coords.new_empty((4,))
    return coords.new_empty((0, m)), coords.new_empty((0,)), coords.new_empty((4,))


@torch.library.custom_op("nngp::knn_prior", mutates_args=(), device_types="cuda")
def knn_prior(coords: torch.Tensor, m: int, q0: int, q1: int) -> torch.Tensor:
    return _lib.knn_prior(coords, m, q0, q1)


@knn_prior.register_fake
def _(coords, m, q0, q1):
    return coords.new_empty((q1 - q0, m), dtype=torch.int32)


@torch.library.custom_op("nngp::knn_query", mutates_args=(), device_types="cuda")
def knn_query(ref: torch.Tensor, query: torch.Tensor, k: int) -> torch.Tensor:
    return _lib.knn_query(ref, query, k)


@knn_query.register_fake
def _(ref, query, k):
    return query.new_empty((query.shape[0], k), dtype=torch.int32)


@torch.library.custom_op("nngp::bf_cross", mutates_args=(), device_types="cuda")
def bf_cross(ref: torch.Tensor, query: torch.Tensor, nbr: torch.Tensor, kind: int, sigma2: float, phi: float,
             tau2: float, ref_values: Optional[torch.Tensor], algo: int) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """B_t, F_t against the reference set and the kriging mean B_t v_N(t) (zeros without ref_values)."""
    rows = nbr.shape[0]
    R = torch.empty((rows,), dtype=torch.float64, device=query.device) if ref_values is not None else None
    B, F, _ = _lib.bf_cross(ref, query, nbr, _KINDS[kind], sigma2, phi, tau2, ref_values=ref_values,
                            algo=_ALGOS[algo], R=R)
    mean = -R if R is not None else torch.zeros((rows,), dtype=torch.float64, device=query.device)
    return B, F, mean


@bf_cross.register_fake
def _(ref, query, nbr, kind, sigma2, phi, tau2, ref_values, algo):
    rows, m = nbr.shape
    return query.new_empty((rows, m)), query.new_empty((rows,)), query.new_empty((rows,))


def kind_code(kind: str) -> int:
    try:
        return _KINDS.index(kind)
    except ValueError:
        raise ValueError(f"unknown covariance kind {kind!r}; expected one of {_KINDS}") from None


def algo_code(algo: str) -> int:
    try:
        return _ALGOS.index(algo)
    except ValueError:
        raise ValueError(f"unknown algo {algo!r}; expected one of {_ALGOS}") from None
