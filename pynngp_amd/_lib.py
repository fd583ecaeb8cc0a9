"""ctypes binding of ``libnngp_hip.so`` (the C ABI in ``include/nngp.h``).

This is the only place that touches the native library.  It loads the in-tree
build (``pynngp_amd/_build/libnngp_hip.so``, made by ``__graft_entry__.build()``
or ``make -C pynngp_amd/csrc``) and fails loudly when it is missing or when a
tensor is not on a ROCm GPU: there is no CPU fallback for the hot path.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Tuple

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# NNGP_LIB overrides the library path (A/B timing of alternative builds only; it must exist)
LIB_PATH = os.environ.get("NNGP_LIB") or os.path.join(_HERE, "_build", "libnngp_hip.so")
SYMBOLS = (
    "nngp_version",
    "nngp_abi_version",
    "nngp_last_error",
    "nngp_knn_workspace_bytes",
    "nngp_knn_prior",
    "nngp_knn_prior_rows",
    "nngp_knn_query",
    "nngp_bf_sweep_workspace_bytes",
    "nngp_bf_sweep",
    "nngp_bf_cross",
    "nngp_bf_finalize",
    "nngp_resolve_algo",
    "nngp_resolve_algo_nu",
    "nngp_loglik_from_partials",
    "nngp_check_partials",
    "nngp_row_order_workspace_bytes",
    "nngp_row_order",
    "nngp_combine_partials",
    "nngp_combine_partials_batch",
    "nngp_matern_eval",
    "nngp_joint_entries",
    "nngp_joint_dist",
    "nngp_bf_sweep_blocks_workspace_bytes",
    "nngp_bf_sweep_blocks",
    "nngp_reverse_workspace_bytes",
    "nngp_reverse_neighbors",
    "nngp_color_moral_graph",
    "nngp_gibbs_prep_bytes",
    "nngp_gibbs_prepare",
    "nngp_gibbs_member_rows",
    "nngp_gibbs_w_sweep",
    "nngp_gibbs_normals",
    "nngp_gibbs_prepare_range",
    "nngp_gibbs_w_color",
    "nngp_gibbs_w_color_dev",
    "nngp_gibbs_w_apply",
    "nngp_gibbs_stats_workspace_bytes",
    "nngp_gibbs_stats",
    "nngp_gibbs_w_sweep_chains",
    "nngp_gibbs_w_sweep_chains_il",
    "nngp_gibbs_w_sweep_tiles",
    "nngp_color_moral_graph_dev",
    "nngp_pair_plan_supported",
    "nngp_pair_plan_bytes",
    "nngp_pair_plan_build",
    "nngp_bf_sweep_plan",
)

KIND_CODES = {"exponential": 0, "matern32": 1, "matern52": 2, "gaussian": 3, "spherical": 4, "matern": 5}
MATERN_NU_MAX = 50.0
ALGO_CODES = {"auto": 0, "lane": 1, "wave": 2, "quad": 4, "pairb": 5}
MAX_M = 63
MAX_DIM = 3
ABI_VERSION = 4  # NNGP_ABI_VERSION of include/nngp.h this binding's signatures follow
PLAN_INFO_LEN = 10  # NNGP_PLAN_INFO_LEN
BLOCKS_MAX_M = 32  # nngp_bf_sweep_blocks: 1 <= m <= 32


class NNGPExtensionError(RuntimeError):
    """The native library is missing, failed to load, or returned an error."""


_lib = None


def load() -> ctypes.CDLL:
    """Load (once) and return the native library; raise if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NNGPExtensionError(
            f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "or `make -C pynngp_amd/csrc` (pynngp_amd has no CPU fallback)"
        )
    lib = ctypes.CDLL(LIB_PATH)
    P, I32, I64, D, SZ = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_double, ctypes.c_size_t
    lib.nngp_version.restype = ctypes.c_char_p
    lib.nngp_abi_version.restype = I32
    if lib.nngp_abi_version() != ABI_VERSION:
        raise NNGPExtensionError(f"{LIB_PATH} has C ABI revision {lib.nngp_abi_version()}, this binding needs "
                                 f"{ABI_VERSION}: rebuild the library")
    lib.nngp_last_error.restype = ctypes.c_char_p
    lib.nngp_knn_workspace_bytes.argtypes = [I64, I32, I32]
    lib.nngp_knn_workspace_bytes.restype = SZ
    lib.nngp_knn_prior.argtypes = [P, I64, I32, I32, I64, I64, P, P, SZ, P]
    lib.nngp_knn_prior.restype = ctypes.c_int
    lib.nngp_knn_prior_rows.argtypes = [P, I64, I32, I32, P, I64, P, P, SZ, P]
    lib.nngp_knn_prior_rows.restype = ctypes.c_int
    lib.nngp_knn_query.argtypes = [P, I64, I32, P, I64, I32, P, P, SZ, P]
    lib.nngp_knn_query.restype = ctypes.c_int
    lib.nngp_bf_sweep_workspace_bytes.argtypes = [I64, I32, I32, I32, I32]
    lib.nngp_bf_sweep_workspace_bytes.restype = SZ
    lib.nngp_bf_sweep.argtypes = [P, I64, I32, P, P, I64, I32, I64, I32, D, D, D, D, P, P, P, P, P, P, SZ, I32, P]
    lib.nngp_bf_cross.argtypes = [P, I64, I32, P, I64, P, P, I64, I32, I64, I32, D, D, D, D, P, P, P, P, P, P, P, SZ,
                                  I32, P]
    lib.nngp_bf_cross.restype = ctypes.c_int
    lib.nngp_row_order_workspace_bytes.argtypes = [I64]
    lib.nngp_row_order_workspace_bytes.restype = SZ
    lib.nngp_row_order.argtypes = [P, I64, I32, P, I32, I64, I64, P, P, P, SZ, P]
    lib.nngp_row_order.restype = ctypes.c_int
    lib.nngp_combine_partials.argtypes = [P, I32, P, P]
    lib.nngp_combine_partials_batch.argtypes = [P, I32, I64, P, P]
    lib.nngp_matern_eval.argtypes = [P, I64, D, P, P]
    lib.nngp_matern_eval.restype = ctypes.c_int
    lib.nngp_joint_entries.argtypes = [I32]
    lib.nngp_joint_entries.restype = I64
    lib.nngp_joint_dist.argtypes = [P, I64, I32, P, I64, P, P, I64, I32, I64, P, P]
    lib.nngp_joint_dist.restype = ctypes.c_int
    lib.nngp_bf_sweep_blocks_workspace_bytes.argtypes = [I64]
    lib.nngp_bf_sweep_blocks_workspace_bytes.restype = SZ
    lib.nngp_bf_sweep_blocks.argtypes = [P, P, P, I64, I64, I32, I64, I64, P, P, P, P, P, P, P, SZ, P]
    lib.nngp_bf_sweep_blocks.restype = ctypes.c_int
    lib.nngp_combine_partials_batch.restype = ctypes.c_int
    lib.nngp_bf_finalize.argtypes = [P, ctypes.c_size_t, I64, I32, I32, I32, I32, P, P]
    lib.nngp_bf_finalize.restype = ctypes.c_int
    lib.nngp_resolve_algo.argtypes = [I32, I32, I32, I32]
    lib.nngp_resolve_algo.restype = I32
    lib.nngp_resolve_algo_nu.argtypes = [I32, I32, I32, I32, D]
    lib.nngp_resolve_algo_nu.restype = I32
    lib.nngp_combine_partials.restype = ctypes.c_int
    U64 = ctypes.c_uint64
    lib.nngp_reverse_workspace_bytes.argtypes = [I64, I32]
    lib.nngp_reverse_workspace_bytes.restype = SZ
    lib.nngp_reverse_neighbors.argtypes = [P, I64, I32, P, P, P, P, SZ, P]
    lib.nngp_reverse_neighbors.restype = ctypes.c_int
    lib.nngp_color_moral_graph.argtypes = [P, P, P, I64, I32, P]
    lib.nngp_color_moral_graph.restype = I64
    lib.nngp_gibbs_prep_bytes.argtypes = [I64, I32]
    lib.nngp_gibbs_prep_bytes.restype = SZ
    lib.nngp_gibbs_prepare.argtypes = [P, P, P, P, P, P, I64, I32, P, SZ, P]
    lib.nngp_gibbs_prepare.restype = ctypes.c_int
    lib.nngp_gibbs_member_rows.argtypes = [P, I64, P, P, P]
    lib.nngp_gibbs_member_rows.restype = ctypes.c_int
    lib.nngp_gibbs_w_sweep.argtypes = [P, P, I32, P, I64, I32, D, D, P, P, P, P, P, P, U64, U64, P]
    lib.nngp_gibbs_w_sweep.restype = ctypes.c_int
    lib.nngp_gibbs_normals.argtypes = [I64, U64, U64, P, P]
    lib.nngp_gibbs_normals.restype = ctypes.c_int
    lib.nngp_gibbs_prepare_range.argtypes = [P, P, P, P, P, I64, I32, I64, I64, P, SZ, P]
    lib.nngp_gibbs_prepare_range.restype = ctypes.c_int
    lib.nngp_gibbs_w_color.argtypes = [P, I64, P, I64, I32, D, D, P, P, P, P, P, P, U64, U64, P, P]
    lib.nngp_gibbs_w_color.restype = ctypes.c_int
    lib.nngp_gibbs_w_color_dev.argtypes = [P, I64, P, I64, I32, P, P, P, P, P, P, P, P, P]
    lib.nngp_gibbs_w_color_dev.restype = ctypes.c_int
    lib.nngp_gibbs_w_apply.argtypes = [P, I64, P, P, I64, I32, P, P, P, P, P]
    lib.nngp_gibbs_w_apply.restype = ctypes.c_int
    lib.nngp_gibbs_stats_workspace_bytes.argtypes = [I64, I32]
    lib.nngp_gibbs_stats_workspace_bytes.restype = SZ
    lib.nngp_gibbs_stats.argtypes = [I64, P, P, P, P, P, I32, P, P, P, P, SZ, P]
    lib.nngp_gibbs_stats.restype = ctypes.c_int
    lib.nngp_bf_sweep.restype = ctypes.c_int
    lib.nngp_color_moral_graph_dev.argtypes = [P, P, P, I64, I32, P, P, SZ, P]
    lib.nngp_color_moral_graph_dev.restype = I64
    lib.nngp_gibbs_w_sweep_tiles.argtypes = [P, P, P, I32, P, P, I32, P, P, P, P, I64, I32, I64, D, D, P, P, P, P,
                                             P, P]
    lib.nngp_gibbs_w_sweep_tiles.restype = ctypes.c_int
    lib.nngp_gibbs_w_sweep_chains.argtypes = [P, P, I32, I32, P, I64, I32, P, P, P, P, P, P, P, P, P]
    lib.nngp_gibbs_w_sweep_chains.restype = ctypes.c_int
    lib.nngp_gibbs_w_sweep_chains_il.argtypes = [P, P, I32, I32, P, I64, I32, P, P, P, P, P, P, P, P, P]
    lib.nngp_gibbs_w_sweep_chains_il.restype = ctypes.c_int
    lib.nngp_pair_plan_supported.argtypes = [I32, I32, I32]
    lib.nngp_pair_plan_supported.restype = ctypes.c_int
    lib.nngp_pair_plan_bytes.argtypes = [I64, I32, I32]
    lib.nngp_pair_plan_bytes.restype = SZ
    lib.nngp_pair_plan_build.argtypes = [P, P, I64, I32, I64, I64, I32, P, SZ, P, P]
    lib.nngp_pair_plan_build.restype = ctypes.c_int
    lib.nngp_bf_sweep_plan.argtypes = [P, I64, I32, P, P, I64, I32, I64, I32, D, D, D, P, P, P, P, P, P, SZ, P, SZ, P,
                                       P]
    lib.nngp_bf_sweep_plan.restype = ctypes.c_int
    lib.nngp_check_partials.argtypes = [P, P, P]
    lib.nngp_check_partials.restype = ctypes.c_int
    lib.nngp_loglik_from_partials.argtypes = [P, I64]
    lib.nngp_loglik_from_partials.restype = D
    _lib = lib
    return lib


def version() -> str:
    return load().nngp_version().decode()


def resolve_algo(algo: str, m: int, kind: str, dim: int, nu: Optional[float] = None) -> str:
    """The kernel ``algo`` ("auto" or explicit) runs as for (m, kind, dim) (nngp_resolve_algo; with ``nu``
    for the ``matern`` kind, whose pair-kernel table covers nu >= ~0.45: nngp_resolve_algo_nu)."""
    if nu is not None:
        code = load().nngp_resolve_algo_nu(ALGO_CODES[algo], int(m), KIND_CODES[kind], int(dim), float(nu))
    else:
        code = load().nngp_resolve_algo(ALGO_CODES[algo], int(m), KIND_CODES[kind], int(dim))
    names = {v: k for k, v in ALGO_CODES.items()}
    return names.get(code, str(code))


def _check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().nngp_last_error().decode()
        raise NNGPExtensionError(f"{what} failed ({rc}): {msg}")


def _require_gpu(*tensors: Optional[torch.Tensor]) -> torch.device:
    dev = None
    for t in tensors:
        if t is None:
            continue
        if t.device.type != "cuda":
            raise NNGPExtensionError(
                f"pynngp_amd needs ROCm GPU tensors (got {t.device}); there is no CPU fallback"
            )
        if dev is None:
            dev = t.device
        elif t.device != dev:
            raise NNGPExtensionError(f"tensors on different devices: {dev} vs {t.device}")
    if dev is None:
        raise NNGPExtensionError("no tensor arguments")
    return dev


def _ptr(t: Optional[torch.Tensor]):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _stream(dev: torch.device):
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def _workspace(nbytes: int, dev: torch.device) -> torch.Tensor:
    # torch's caching allocator returns >= 512-byte aligned blocks; the first 256 bytes (the pair kernel's
    # header: tile count and the fused fold's ticket) start at zero, as include/nngp.h requires
    ws = torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=dev)
    ws[:256].zero_()
    return ws


def _as_coords(coords: torch.Tensor) -> torch.Tensor:
    """float64 (N, dim) ordinates, 1 <= dim <= 3 (nngp.py:55-61 takes any dimension)."""
    if coords.dim() != 2 or not 1 <= coords.shape[1] <= MAX_DIM or coords.dtype != torch.float64:
        raise ValueError(f"coords must be float64 (N, dim), 1 <= dim <= {MAX_DIM}, got {tuple(coords.shape)} "
                         f"{coords.dtype}")
    return coords.contiguous()


def _same_dim(*coords: torch.Tensor) -> int:
    dims = {c.shape[1] for c in coords}
    if len(dims) != 1:
        raise ValueError(f"coordinate arrays of different dimensions: {sorted(dims)}")
    return dims.pop()


def _check_out(t: Optional[torch.Tensor], name: str, shape, dev: torch.device) -> None:
    """Caller-supplied output buffer: float64, the exact shape, contiguous, on dev (the
    kernel writes through the raw pointer, so a wrong buffer would be written out of bounds)."""
    if t is None:
        return
    if t.dtype != torch.float64 or tuple(t.shape) != tuple(shape) or not t.is_contiguous() or t.device != dev:
        raise ValueError(f"{name} must be a contiguous float64 {tuple(shape)} tensor on {dev}, got "
                         f"{t.dtype} {tuple(t.shape)} contiguous={t.is_contiguous()} on {t.device}")


def knn_prior(coords: torch.Tensor, m: int, q0: int = 0, q1: Optional[int] = None,
              out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Ordered prior neighbour sets for rows [q0, q1): int32 (q1-q0, m), -1 padded.

    Replaces ``NNGP._make_s_neighbor_sets`` (pyNNGP/nngp.py:49-62).
    """
    coords = _as_coords(coords)
    dev = _require_gpu(coords)
    n = coords.shape[0]
    q1 = n if q1 is None else int(q1)
    if not 0 <= q0 <= q1 <= n:
        raise ValueError(f"query rows [{q0}, {q1}) outside [0, {n})")
    if out is None:
        out = torch.empty((q1 - q0, m), dtype=torch.int32, device=dev)
    lib = load()
    d = coords.shape[1]
    ws = _workspace(lib.nngp_knn_workspace_bytes(n, d, m), dev)
    _check(lib.nngp_knn_prior(_ptr(coords), n, d, m, q0, q1, _ptr(out), _ptr(ws), ws.numel(), _stream(dev)),
           "nngp_knn_prior")
    return out


def knn_prior_rows(coords: torch.Tensor, m: int, rows: torch.Tensor,
                   out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Prior neighbour sets of the locations ``rows`` (int32 point indices, any order):
    row t of the result is the set of point ``rows[t]`` (nngp_knn_prior_rows)."""
    coords = _as_coords(coords)
    if rows.dtype != torch.int32 or rows.dim() != 1:
        raise ValueError("rows must be int32 (n_rows,)")
    rows = rows.contiguous()
    dev = _require_gpu(coords, rows)
    n = coords.shape[0]
    if out is None:
        out = torch.empty((rows.shape[0], m), dtype=torch.int32, device=dev)
    lib = load()
    d = coords.shape[1]
    ws = _workspace(lib.nngp_knn_workspace_bytes(n, d, m), dev)
    _check(lib.nngp_knn_prior_rows(_ptr(coords), n, d, m, _ptr(rows), rows.shape[0], _ptr(out), _ptr(ws), ws.numel(),
                                   _stream(dev)), "nngp_knn_prior_rows")
    return out


def knn_query(ref: torch.Tensor, query: torch.Tensor, k: int) -> torch.Tensor:
    """k nearest reference points of every query point (no prior restriction).

    int32 (n_query, k) in (rdist, index) order; -1 padded when k > n_ref.  Used for
    ``_init_ws`` (pyNNGP/nngp.py:45-47, sklearn KNeighborsRegressor(5)) and the
    off-reference sets of ``_make_t_neighbor_sets`` (nngp.py:64-71).
    """
    ref = _as_coords(ref)
    query = _as_coords(query)
    d = _same_dim(ref, query)
    dev = _require_gpu(ref, query)
    out = torch.empty((query.shape[0], k), dtype=torch.int32, device=dev)
    lib = load()
    ws = _workspace(lib.nngp_knn_workspace_bytes(ref.shape[0], d, k), dev)
    _check(lib.nngp_knn_query(_ptr(ref), ref.shape[0], d, _ptr(query), query.shape[0], k, _ptr(out), _ptr(ws),
                              ws.numel(), _stream(dev)), "nngp_knn_query")
    return out


def _check_kind(kind: str, nu: Optional[float]) -> float:
    """The kind's code must exist; the ``matern`` kind needs 0 < nu <= 50 (returned as the C argument)."""
    if kind not in KIND_CODES:
        raise ValueError(f"unknown covariance kind {kind!r}; expected one of {sorted(KIND_CODES)}")
    if kind == "matern":
        if nu is None or not 0.0 < float(nu) <= MATERN_NU_MAX:
            raise ValueError(f"the matern kind needs a smoothness 0 < nu <= {MATERN_NU_MAX:g} (got {nu!r})")
        return float(nu)
    return -1.0


class PairPlan:
    """A wave pair plan (``nngp_pair_plan_build``, include/nngp.h): the distinct covariance pairs of
    every sweep wavefront and each lane's map into them, for one (nbr, order, i0, n_points).  Passed to
    :func:`bf_sweep` (``plan=``), it evaluates each shared covariance once per wave; B / F / R and the
    partials are bit-identical to the unplanned pair kernel's.  The plan is stale once nbr or order
    change (rebuild it, as the neighbour sets themselves): :meth:`matches` compares the buffers and
    torch's in-place version counters, the C ABI the buffers, the kernel a per-location checksum."""

    def __init__(self, buf: torch.Tensor, info, nbr: torch.Tensor, order: Optional[torch.Tensor]):
        self.buf = buf
        self.info = (ctypes.c_int64 * PLAN_INFO_LEN)(*info)
        self.n_planned, self.n_direct = int(info[0]), int(info[1])
        self.n_rows, self.m, self.dim, self.i0, self.n_points = (int(v) for v in info[2:7])
        self._nbr_ptr, self._order_ptr = nbr.data_ptr(), (order.data_ptr() if order is not None else 0)
        self._versions = (nbr._version, order._version if order is not None else 0)

    def matches(self, nbr: torch.Tensor, order: Optional[torch.Tensor], i0: int, n_points: int, dim: int) -> bool:
        """True when this plan was built for these nbr / order tensors (same storage, not modified in place
        since) and this geometry."""
        return (nbr.data_ptr() == self._nbr_ptr and (order.data_ptr() if order is not None else 0) == self._order_ptr
                and (nbr._version, order._version if order is not None else 0) == self._versions
                and tuple(nbr.shape) == (self.n_rows, self.m) and i0 == self.i0 and n_points == self.n_points
                and dim == self.dim)


def pair_plan_read_bytes(buf: torch.Tensor, m: int) -> int:
    """Bytes a planned sweep streams from its plan (pair_plan.h: per planned wave the three header words,
    the map chunks, the checksums, the U list and the pair words, in whole rounds) -- the plan's share of
    the sweep's input traffic.  Reads the wave headers back (a setup-time helper: one synchronisation)."""
    hdr = buf[:256].view(torch.int64).cpu()
    nreg, sb = int(hdr[6]), int(hdr[9])
    if nreg == 0:
        return 0
    wsb = sb // 4
    w = buf[256:256 + nreg * sb].view(nreg * 4, wsb)[:, :12].contiguous().view(torch.int32).long().cpu()
    nU, nE, st = w[:, 0], w[:, 1].clamp(min=0), w[:, 2]
    planned = (st.view(nreg, 4) == 0).all(1).repeat_interleave(4)
    np_ = (m + 2) // 2
    che = (np_ * np_ + 7) // 8
    per = 12 + che * 1024 + 256 + 256 * ((nU + 63) // 64) + 1024 * ((nE + 255) // 256)
    return int(per[planned].sum())


def pair_plan_supported(m: int, kind: str, dim: int) -> bool:
    """Whether wave pair plans serve (m, kind, dim) (2 <= m <= 17, kinds exponential .. spherical, dim 1..3)."""
    return kind in KIND_CODES and bool(load().nngp_pair_plan_supported(int(m), KIND_CODES[kind], int(dim)))


def pair_plan(nbr: torch.Tensor, n_points: int, dim: int, i0: int = 0,
              order: Optional[torch.Tensor] = None) -> PairPlan:
    """Build the wave pair plan of a sweep over ``nbr`` (int32 (rows, m) on the GPU; rows are locations
    ``i0 + (order[t] if order else t)`` of an ``n_points``-point field of dimension ``dim``).  A setup
    call: it synchronises torch's current stream once (the plan's tile counts come back to the host)."""
    if nbr.dtype != torch.int32 or nbr.dim() != 2:
        raise ValueError(f"nbr must be int32 (rows, m), got {nbr.dtype} {tuple(nbr.shape)}")
    nbr = nbr.contiguous()
    dev = _require_gpu(nbr, order)
    rows, m = nbr.shape
    if order is not None and (order.dtype != torch.int32 or order.shape != (rows,)):
        raise ValueError("order must be int32 (rows,)")
    lib = load()
    nbytes = lib.nngp_pair_plan_bytes(rows, m, dim)
    if nbytes == 0:
        raise NNGPExtensionError(f"no pair plans for m={m}, dim={dim} (2 <= m <= 17, dim 1..3)")
    buf = _workspace(nbytes, dev)
    info = (ctypes.c_int64 * PLAN_INFO_LEN)()
    _check(lib.nngp_pair_plan_build(_ptr(nbr), _ptr(order), rows, m, int(i0), int(n_points), int(dim), _ptr(buf),
                                    buf.numel(), info, _stream(dev)), "nngp_pair_plan_build")
    return PairPlan(buf, list(info), nbr, order)


def bf_sweep(coords: torch.Tensor, nbr: torch.Tensor, i0: int, kind: str, sigma2: float, phi: float,
             tau2: float = 0.0, values: Optional[torch.Tensor] = None, want_bf: bool = True,
             algo: str = "auto", B: Optional[torch.Tensor] = None, F: Optional[torch.Tensor] = None,
             partials: Optional[torch.Tensor] = None, workspace: Optional[torch.Tensor] = None,
             order: Optional[torch.Tensor] = None,
             R: Optional[torch.Tensor] = None,
             defer: bool = False, nu: Optional[float] = None, plan: Optional[PairPlan] = None
             ) -> Tuple[Optional[torch.Tensor], Optional[torch.Tensor], torch.Tensor]:
    """Fused B/F + log-likelihood sweep over rows ``i0 .. i0 + len(nbr)``.

    ``plan``: a :func:`pair_plan` of this nbr / order / i0 (the pair kernel with every shared
    covariance evaluated once per tile; kinds exponential .. spherical, algo ``auto`` / ``pairb``).

    ``nu``: the smoothness of the ``matern`` kind (0 < nu <= 50; required there, ignored otherwise).

    ``defer=True`` (needs ``workspace``): the final fold is left to :func:`bf_finalize`
    on the same workspace (e.g. on another stream); partials is returned as None.

    Returns ``(B, F, partials)`` (B, F None when ``want_bf`` is False); partials is a
    float64 device tensor ``[sum log F, sum r^2/F, first bad-pivot row, first bad-index row]``.
    Stream-ordered on torch's current stream; no host synchronisation.  With
    ``order`` (int32 (rows,), from :func:`row_order`) row t of ``nbr`` must hold the
    neighbours of location ``i0 + order[t]`` (pass ``nbr_sorted``); only the visiting
    order changes, B and F are written at their natural rows.
    """
    coords = _as_coords(coords)
    if nbr.dtype != torch.int32 or nbr.dim() != 2:
        raise ValueError(f"nbr must be int32 (rows, m), got {nbr.dtype} {tuple(nbr.shape)}")
    nbr = nbr.contiguous()
    if values is not None:
        if values.dtype != torch.float64 or values.shape != (coords.shape[0],):
            raise ValueError("values must be float64 (N,)")
        values = values.contiguous()
    dev = _require_gpu(coords, nbr, values, order)
    rows, m = nbr.shape
    if order is not None and (order.dtype != torch.int32 or order.shape != (rows,)):
        raise ValueError("order must be int32 (rows,)")
    nu = _check_kind(kind, nu)
    lib = load()
    a = ALGO_CODES[algo]
    if want_bf:
        _check_out(B, "B", (rows, m), dev)
        _check_out(F, "F", (rows,), dev)
        B = torch.empty((rows, m), dtype=torch.float64, device=dev) if B is None else B
        F = torch.empty((rows,), dtype=torch.float64, device=dev) if F is None else F
    else:
        B = F = None
    if defer:
        partials = None
    else:
        _check_out(partials, "partials", (4,), dev)
        partials = torch.empty(4, dtype=torch.float64, device=dev) if partials is None else partials
    d = coords.shape[1]
    need = lib.nngp_bf_sweep_workspace_bytes(rows, m, KIND_CODES[kind], d, a)
    if workspace is None or workspace.numel() < need:
        if defer:
            raise ValueError("defer=True needs a workspace of nngp_bf_sweep_workspace_bytes bytes")
        workspace = _workspace(need, dev)
    _check_out(R, "R", (rows,), dev)
    if workspace.device != dev or not workspace.is_contiguous():
        raise ValueError("workspace must be a contiguous tensor on the sweep's device")
    if plan is not None:
        if algo not in ("auto", "pairb"):
            raise ValueError(f"a pair plan runs the pair kernel, not algo {algo!r}")
        if not isinstance(plan, PairPlan) or plan.buf.device != dev:
            raise ValueError("plan must be a PairPlan on the sweep's device")
        if not plan.matches(nbr, order, i0, coords.shape[0], d):
            raise ValueError("stale pair plan: it was built for other nbr / order tensors (or they were modified in "
                             "place since) or another geometry; rebuild it with pair_plan")
        _check(lib.nngp_bf_sweep_plan(_ptr(coords), coords.shape[0], d, _ptr(nbr), _ptr(order), rows, m, i0,
                                      KIND_CODES[kind], float(sigma2), float(phi), float(tau2), _ptr(values), _ptr(B),
                                      _ptr(F), _ptr(R), _ptr(partials), _ptr(workspace), workspace.numel(),
                                      _ptr(plan.buf), plan.buf.numel(), plan.info, _stream(dev)),
               "nngp_bf_sweep_plan")
        return B, F, partials
    _check(lib.nngp_bf_sweep(_ptr(coords), coords.shape[0], d, _ptr(nbr), _ptr(order), rows, m, i0, KIND_CODES[kind],
                             float(sigma2), float(phi), float(tau2), nu, _ptr(values), _ptr(B), _ptr(F), _ptr(R),
                             _ptr(partials), _ptr(workspace), workspace.numel(), a, _stream(dev)),
           "nngp_bf_sweep")
    return B, F, partials


def bf_finalize(workspace: torch.Tensor, rows: int, m: int, kind: str, dim: int, algo: str = "auto",
                out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Fold the block records a ``bf_sweep(..., defer=True)`` left in ``workspace`` into
    ``out`` (float64 (4,)), on torch's current stream (nngp_bf_finalize).  ``rows``, ``m``,
    ``kind``, ``dim`` and ``algo`` must be the sweep's: they select the kernel, hence the record
    layout (the library checks the workspace size against them)."""
    dev = _require_gpu(workspace, out)
    out = torch.empty(4, dtype=torch.float64, device=dev) if out is None else out
    if not workspace.is_contiguous():
        raise ValueError("workspace must be contiguous")
    _check(load().nngp_bf_finalize(_ptr(workspace), workspace.numel() * workspace.element_size(), int(rows), int(m),
                                   KIND_CODES[kind], int(dim), ALGO_CODES[algo], _ptr(out), _stream(dev)),
           "nngp_bf_finalize")
    return out


def bf_cross(ref: torch.Tensor, query: torch.Tensor, nbr: torch.Tensor, kind: str, sigma2: float, phi: float,
             tau2: float = 0.0, ref_values: Optional[torch.Tensor] = None,
             query_values: Optional[torch.Tensor] = None, q0: int = 0, algo: str = "auto",
             B: Optional[torch.Tensor] = None, F: Optional[torch.Tensor] = None,
             partials: Optional[torch.Tensor] = None, workspace: Optional[torch.Tensor] = None,
             order: Optional[torch.Tensor] = None,
             R: Optional[torch.Tensor] = None, nu: Optional[float] = None) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """B_t, F_t of query rows ``q0 .. q0 + len(nbr)`` against the reference set ``ref``
    (nngp_bf_cross; prediction at t not in S).

    ``nbr[r]`` lists indices into ``ref`` (e.g. :func:`knn_query` output).  Returns
    ``(B, F, partials)``; with ``R`` given, ``R = query_values - B_t v_N`` (minus the
    kriging mean when ``query_values`` is None).
    """
    ref, query = _as_coords(ref), _as_coords(query)
    d = _same_dim(ref, query)
    if nbr.dtype != torch.int32 or nbr.dim() != 2:
        raise ValueError(f"nbr must be int32 (rows, m), got {nbr.dtype} {tuple(nbr.shape)}")
    nbr = nbr.contiguous()
    if ref_values is not None:
        if ref_values.dtype != torch.float64 or ref_values.shape != (ref.shape[0],):
            raise ValueError("ref_values must be float64 (n_ref,)")
        ref_values = ref_values.contiguous()
    if query_values is not None:
        if query_values.dtype != torch.float64 or query_values.shape != (query.shape[0],):
            raise ValueError("query_values must be float64 (n_query,)")
        query_values = query_values.contiguous()
    dev = _require_gpu(ref, query, nbr, ref_values, query_values, order)
    rows, m = nbr.shape
    if order is not None and (order.dtype != torch.int32 or order.shape != (rows,)):
        raise ValueError("order must be int32 (rows,)")
    nu = _check_kind(kind, nu)
    lib = load()
    a = ALGO_CODES[algo]
    _check_out(B, "B", (rows, m), dev)
    _check_out(F, "F", (rows,), dev)
    _check_out(partials, "partials", (4,), dev)
    _check_out(R, "R", (rows,), dev)
    B = torch.empty((rows, m), dtype=torch.float64, device=dev) if B is None else B
    F = torch.empty((rows,), dtype=torch.float64, device=dev) if F is None else F
    partials = torch.empty(4, dtype=torch.float64, device=dev) if partials is None else partials
    need = lib.nngp_bf_sweep_workspace_bytes(rows, m, KIND_CODES[kind], d, a)
    if workspace is None or workspace.numel() < need:
        workspace = _workspace(need, dev)
    _check(lib.nngp_bf_cross(_ptr(ref), ref.shape[0], d, _ptr(query), query.shape[0], _ptr(nbr), _ptr(order), rows, m,
                             int(q0), KIND_CODES[kind], float(sigma2), float(phi), float(tau2), nu, _ptr(ref_values),
                             _ptr(query_values), _ptr(B), _ptr(F), _ptr(R), _ptr(partials), _ptr(workspace),
                             workspace.numel(), a, _stream(dev)), "nngp_bf_cross")
    return B, F, partials


def joint_dist(coords: torch.Tensor, nbr: torch.Tensor, i0: int = 0, qcoords: Optional[torch.Tensor] = None,
               order: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Distances of every joint block (nngp_joint_dist): float64 ((m+1)(m+2)/2, rows), entry
    (a, b), b <= a, of nbr row t at ``[a (a+1)/2 + b, t]`` (row m of a block is the location
    ``i0 + (order[t] if order else t)``, taken from ``qcoords``, default ``coords``); 0 on the
    diagonal, +inf for slots without a point.  Map it through a covariance function and pass
    the result to :func:`bf_sweep_blocks`."""
    coords = _as_coords(coords)
    qcoords = coords if qcoords is None else _as_coords(qcoords)
    d = _same_dim(coords, qcoords)
    if nbr.dtype != torch.int32 or nbr.dim() != 2:
        raise ValueError(f"nbr must be int32 (rows, m), got {nbr.dtype} {tuple(nbr.shape)}")
    nbr = nbr.contiguous()
    dev = _require_gpu(coords, qcoords, nbr, order)
    rows, m = nbr.shape
    if order is not None and (order.dtype != torch.int32 or order.shape != (rows,)):
        raise ValueError("order must be int32 (rows,)")
    lib = load()
    ne = int(lib.nngp_joint_entries(m))
    _check_out(out, "out", (ne, rows), dev)
    out = torch.empty((ne, rows), dtype=torch.float64, device=dev) if out is None else out
    _check(lib.nngp_joint_dist(_ptr(coords), coords.shape[0], d, _ptr(qcoords), qcoords.shape[0], _ptr(nbr),
                               _ptr(order), rows, m, int(i0), _ptr(out), _stream(dev)), "nngp_joint_dist")
    return out


def matern(u: torch.Tensor, nu: float) -> torch.Tensor:
    """u^nu K_nu(u) / (2^(nu-1) Gamma(nu)) elementwise on the GPU (nngp_matern_eval; u >= 0, +inf -> 0),
    e.g. ``IsotropicCovariance(lambda d: s2 * matern(phi * d, nu), tau2)``."""
    if u.dtype != torch.float64:
        raise ValueError("u must be float64")
    dev = _require_gpu(u)
    _check_kind("matern", nu)
    u = u.contiguous()
    out = torch.empty_like(u)
    _check(load().nngp_matern_eval(_ptr(u), u.numel(), float(nu), _ptr(out), _stream(dev)), "nngp_matern_eval")
    return out


def joint_diagonal(m: int) -> torch.Tensor:
    """Row indices a (a+1)/2 + a of the diagonal entries of a joint block (for adding a nugget)."""
    a = torch.arange(m + 1)
    return a * (a + 1) // 2 + a


def bf_sweep_blocks(cov: torch.Tensor, nbr: torch.Tensor, n_points: int, i0: int = 0,
                    values: Optional[torch.Tensor] = None, qvalues: Optional[torch.Tensor] = None,
                    want_bf: bool = True, order: Optional[torch.Tensor] = None, R: Optional[torch.Tensor] = None,
                    workspace: Optional[torch.Tensor] = None, n_locs: Optional[int] = None,
                    B: Optional[torch.Tensor] = None, F: Optional[torch.Tensor] = None,
                    partials: Optional[torch.Tensor] = None
                    ) -> Tuple[Optional[torch.Tensor], Optional[torch.Tensor], torch.Tensor]:
    """The fused B/F + log-lik sweep with the joint blocks' covariances given (nngp_bf_sweep_blocks):
    ``cov`` float64 ((m+1)(m+2)/2, rows) in :func:`joint_dist`'s layout (the covariance function
    of the distances, the nugget on the diagonal entries).  ``values`` (n_points,) at the
    neighbours and ``qvalues`` (n_locs,) at the locations (pass ``values`` again for the S = T
    sweep; None: 0, so R = -B v_N, minus the kriging mean).
    Returns ``(B, F, partials)`` as :func:`bf_sweep`.  1 <= m <= 32 (the two-lane kernel up to 24,
    the four-lane kernel above).  The C ABI takes raw pointers, so every length is checked here:
    ``values`` (n_points,), ``qvalues`` (n_locs,), ``order`` int32 (rows,)."""
    if nbr.dtype != torch.int32 or nbr.dim() != 2:
        raise ValueError(f"nbr must be int32 (rows, m), got {nbr.dtype} {tuple(nbr.shape)}")
    nbr = nbr.contiguous()
    rows, m = nbr.shape
    lib = load()
    ne = int(lib.nngp_joint_entries(m))
    if cov.dtype != torch.float64 or tuple(cov.shape) != (ne, rows):
        raise ValueError(f"cov must be float64 ({ne}, {rows}) (joint_dist's layout), got {cov.dtype} {tuple(cov.shape)}")
    cov = cov.contiguous()
    n_locs = int(n_points if n_locs is None else n_locs)
    for name, v, n in (("values", values, n_points), ("qvalues", qvalues, n_locs)):
        if v is not None and (v.dtype != torch.float64 or tuple(v.shape) != (int(n),)):
            raise ValueError(f"{name} must be float64 of shape ({int(n)},), got {v.dtype} {tuple(v.shape)}")
    if order is not None:
        if order.dtype != torch.int32 or tuple(order.shape) != (rows,):
            raise ValueError(f"order must be int32 of shape ({rows},), got {order.dtype} {tuple(order.shape)}")
        order = order.contiguous()
    values = None if values is None else values.contiguous()
    qvalues = None if qvalues is None else qvalues.contiguous()
    dev = _require_gpu(cov, nbr, values, qvalues, order, R)
    if want_bf:
        _check_out(B, "B", (rows, m), dev)
        _check_out(F, "F", (rows,), dev)
        B = torch.empty((rows, m), dtype=torch.float64, device=dev) if B is None else B
        F = torch.empty((rows,), dtype=torch.float64, device=dev) if F is None else F
    else:
        B = F = None
    _check_out(R, "R", (rows,), dev)
    _check_out(partials, "partials", (4,), dev)
    partials = torch.empty(4, dtype=torch.float64, device=dev) if partials is None else partials
    need = lib.nngp_bf_sweep_blocks_workspace_bytes(rows)
    if workspace is None or workspace.numel() < need:
        workspace = _workspace(need, dev)
    _check(lib.nngp_bf_sweep_blocks(_ptr(cov), _ptr(nbr), _ptr(order), int(n_points), rows, m, int(i0), n_locs,
                                    _ptr(values), _ptr(qvalues), _ptr(B), _ptr(F), _ptr(R), _ptr(partials),
                                    _ptr(workspace), workspace.numel(), _stream(dev)), "nngp_bf_sweep_blocks")
    return B, F, partials


def row_order(coords: torch.Tensor, i0: int = 0, rows: Optional[int] = None,
              nbr: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """Z-order visiting order of locations i0 .. i0+rows-1 for :func:`bf_sweep`.

    Returns ``(order, nbr_sorted)``: ``order`` int32 (rows,) and, when ``nbr`` (the
    natural-order neighbour rows of those locations) is given, ``nbr_sorted[t] =
    nbr[order[t]]``.  Sweep with ``bf_sweep(coords, nbr_sorted, i0, ..., order=order)``.
    """
    coords = _as_coords(coords)
    dev = _require_gpu(coords, nbr)
    n = coords.shape[0]
    rows = n - i0 if rows is None else int(rows)
    m = 0 if nbr is None else nbr.shape[1]
    if nbr is not None:
        if nbr.dtype != torch.int32 or nbr.shape[0] != rows:
            raise ValueError("nbr must be int32 (rows, m)")
        nbr = nbr.contiguous()
    out = torch.empty((rows,), dtype=torch.int32, device=dev)
    srt = None if nbr is None else torch.empty_like(nbr)
    lib = load()
    need = lib.nngp_row_order_workspace_bytes(rows)
    if need == 0:
        raise NNGPExtensionError("nngp_row_order_workspace_bytes failed")
    ws = _workspace(need, dev)
    _check(lib.nngp_row_order(_ptr(coords), n, coords.shape[1], _ptr(nbr), m, i0, rows, _ptr(out), _ptr(srt), _ptr(ws),
                              ws.numel(), _stream(dev)), "nngp_row_order")
    return out, srt


def combine_partials(gathered: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Rank-order fold of all-gathered (world, 4) partials into (4,) (one tiny kernel)."""
    if gathered.dtype != torch.float64 or gathered.dim() != 2 or gathered.shape[1] != 4:
        raise ValueError("gathered must be float64 (world, 4)")
    gathered = gathered.contiguous()
    dev = _require_gpu(gathered, out)
    out = torch.empty(4, dtype=torch.float64, device=dev) if out is None else out
    _check(load().nngp_combine_partials(_ptr(gathered), gathered.shape[0], _ptr(out), _stream(dev)),
           "nngp_combine_partials")
    return out


def bf_workspace(rows: int, m: int, algo: str, device, kind: Optional[str] = None, dim: int = 2) -> torch.Tensor:
    """Pre-allocate a sweep workspace (reuse it across calls in a hot loop); ``kind=None``
    sizes it for any covariance kind."""
    kinds = KIND_CODES.values() if kind is None else (KIND_CODES[kind],)
    need = max(load().nngp_bf_sweep_workspace_bytes(rows, m, k, int(dim), ALGO_CODES[algo]) for k in kinds)
    return _workspace(need, torch.device(device))


# ---------------------------------------------------------------------------- Gibbs sampler pieces
def reverse_neighbors(nbr: torch.Tensor):
    """CSR transpose of the neighbour sets: (off (n+1,), rev_j (n*m,), rev_k (n*m,)) int32 on the device."""
    if nbr.dtype != torch.int32 or nbr.dim() != 2:
        raise ValueError("nbr must be int32 (n, m)")
    nbr = nbr.contiguous()
    dev = _require_gpu(nbr)
    n, m = nbr.shape
    off = torch.empty(n + 1, dtype=torch.int32, device=dev)
    rev_j = torch.empty(max(n * m, 1), dtype=torch.int32, device=dev)
    rev_k = torch.empty(max(n * m, 1), dtype=torch.int32, device=dev)
    lib = load()
    need = lib.nngp_reverse_workspace_bytes(n, m)
    if need == 0:
        raise NNGPExtensionError("nngp_reverse_workspace_bytes failed")
    ws = _workspace(need, dev)
    _check(lib.nngp_reverse_neighbors(_ptr(nbr), n, m, _ptr(off), _ptr(rev_j), _ptr(rev_k), _ptr(ws), ws.numel(),
                                      _stream(dev)), "nngp_reverse_neighbors")
    return off, rev_j, rev_k


def color_moral_graph(nbr_host, off_host, rev_j_host):
    """Greedy moral-graph colouring on the host (numpy int32 inputs); returns (colors, n_colors)."""
    import numpy as np

    nbr_host = np.ascontiguousarray(nbr_host, dtype=np.int32)
    off_host = np.ascontiguousarray(off_host, dtype=np.int32)
    rev_j_host = np.ascontiguousarray(rev_j_host, dtype=np.int32)
    n, m = nbr_host.shape
    colors = np.empty(n, dtype=np.int32)
    nc = load().nngp_color_moral_graph(nbr_host.ctypes.data, off_host.ctypes.data, rev_j_host.ctypes.data, n, m,
                                       colors.ctypes.data)
    if nc < 0:
        _check(int(nc), "nngp_color_moral_graph")
    return colors, int(nc)


def color_moral_graph_dev(nbr: torch.Tensor, off: torch.Tensor, rev_j: torch.Tensor):
    """:func:`color_moral_graph` on the device (nngp_color_moral_graph_dev, the same colours bit for bit):
    (colors int32 (n,) device tensor, n_colors).  Falls back to the host greedy past 256 colours."""
    if nbr.dtype != torch.int32 or nbr.dim() != 2:
        raise ValueError("nbr must be int32 (n, m)")
    dev = _require_gpu(nbr, off, rev_j)
    n, m = nbr.shape
    color = torch.empty(n, dtype=torch.int32, device=dev)
    ws = _workspace(256, dev)
    nc = load().nngp_color_moral_graph_dev(_ptr(nbr.contiguous()), _ptr(off), _ptr(rev_j), n, m, _ptr(color), _ptr(ws),
                                           ws.numel(), _stream(dev))
    if nc == -4:  # NNGP_EUNSUP: more than 256 colours
        c, k = color_moral_graph(nbr.cpu().numpy(), off.cpu().numpy(), rev_j.cpu().numpy())
        return torch.from_numpy(c).to(dev), k
    _check(0 if nc >= 0 else int(nc), "nngp_color_moral_graph_dev")
    return color, int(nc)


def gibbs_prepare(B: torch.Tensor, Ft: torch.Tensor, off: torch.Tensor, rev_j: torch.Tensor, rev_k: torch.Tensor,
                  prep: Optional[torch.Tensor] = None, order: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Fold the unit-variance factors (B, Ft) into the reverse-list layout the w sweeps read
    (nngp_gibbs_prepare); returns the device buffer to pass to :func:`gibbs_w_sweep`."""
    dev = _require_gpu(B, Ft, off, rev_j, rev_k, prep, order)
    n, m = B.shape
    if order is not None and (order.dtype != torch.int32 or order.shape != (n,)):
        raise ValueError("order must be int32 (n,)")
    lib = load()
    need = lib.nngp_gibbs_prep_bytes(n, m)
    if prep is None or prep.numel() < need:
        prep = _workspace(need, dev)
    _check(lib.nngp_gibbs_prepare(_ptr(B), _ptr(Ft), _ptr(off), _ptr(rev_j), _ptr(rev_k), _ptr(order), n, m, _ptr(prep),
                                  prep.numel(), _stream(dev)), "nngp_gibbs_prepare")
    return prep


def gibbs_prepare_range(B: torch.Tensor, Ft: torch.Tensor, off: torch.Tensor, rev_j: torch.Tensor,
                        rev_k: torch.Tensor, row0: int, row1: int, prep: Optional[torch.Tensor] = None) -> torch.Tensor:
    """:func:`gibbs_prepare` for the rows [row0, row1) only (nngp_gibbs_prepare_range): a rank's
    own shard of a sharded chain.  ``prep`` keeps the whole-field layout."""
    dev = _require_gpu(B, Ft, off, rev_j, rev_k, prep)
    n, m = B.shape
    lib = load()
    need = lib.nngp_gibbs_prep_bytes(n, m)
    if prep is None or prep.numel() < need:
        prep = _workspace(need, dev)
    _check(lib.nngp_gibbs_prepare_range(_ptr(B), _ptr(Ft), _ptr(off), _ptr(rev_j), _ptr(rev_k), n, m, int(row0),
                                        int(row1), _ptr(prep), prep.numel(), _stream(dev)), "nngp_gibbs_prepare_range")
    return prep


def gibbs_w_color(member_rows: torch.Tensor, prep: torch.Tensor, m: int, sigma2: float, tau2: float,
                  yres: torch.Tensor, w: torch.Tensor, r: torch.Tensor, rev_j: torch.Tensor, seed: int, sweep: int,
                  z: Optional[torch.Tensor] = None, noise_w: Optional[torch.Tensor] = None,
                  w_out: Optional[torch.Tensor] = None) -> None:
    """ONE colour step over ``member_rows`` (rows of :func:`gibbs_member_rows`), in place on w, r;
    ``w_out`` (len(member_rows),) receives the members' new w (nngp_gibbs_w_color)."""
    dev = _require_gpu(member_rows, prep, yres, w, r, rev_j, z, noise_w, w_out)
    _check_noise_w(noise_w, w.shape[0])
    k = member_rows.shape[0]
    if member_rows.dtype != torch.int32 or member_rows.dim() != 2 or member_rows.shape[1] != 4 \
            or not member_rows.is_contiguous():
        raise ValueError("member_rows must be a contiguous int32 (k, 4) tensor")
    _check_out(w_out, "w_out", (k,), dev)
    _check(load().nngp_gibbs_w_color(_ptr(member_rows), k, _ptr(prep), w.shape[0], int(m), float(sigma2), float(tau2),
                                     _ptr(yres), _ptr(noise_w), _ptr(w), _ptr(r), _ptr(rev_j), _ptr(z),
                                     int(seed) & (2 ** 64 - 1), int(sweep), _ptr(w_out), _stream(dev)),
           "nngp_gibbs_w_color")


def gibbs_w_apply(rows: torch.Tensor, w_src: torch.Tensor, B: torch.Tensor, w: torch.Tensor, r: torch.Tensor,
                  rev_j: torch.Tensor, rev_k: torch.Tensor) -> None:
    """Replay other ranks' colour draws (nngp_gibbs_w_apply): rows int32 (k, 4) = (i, off[i],
    off[i + 1], src), w_src[src] the owner's new w_i."""
    dev = _require_gpu(rows, w_src, B, w, r, rev_j, rev_k)
    if rows.dtype != torch.int32 or rows.dim() != 2 or rows.shape[1] != 4 or not rows.is_contiguous():
        raise ValueError("rows must be a contiguous int32 (k, 4) tensor")
    n, m = B.shape
    _check(load().nngp_gibbs_w_apply(_ptr(rows), rows.shape[0], _ptr(w_src), _ptr(B), n, m, _ptr(w), _ptr(r),
                                     _ptr(rev_j), _ptr(rev_k), _stream(dev)), "nngp_gibbs_w_apply")


def _check_noise_w(noise_w: Optional[torch.Tensor], n: int) -> None:
    if noise_w is not None and (noise_w.dtype != torch.float64 or noise_w.shape != (n,)
                                or not noise_w.is_contiguous()):
        raise ValueError(f"noise_w must be a contiguous float64 ({n},) tensor")


def _check_member_rows(rows: torch.Tensor, co, n: int, n_entries: int) -> None:
    """The colour kernels index w / r / the prep with each member row's location and reverse range unchecked:
    verify them once per rows tensor (0 <= location < n, 0 <= first <= end <= n_entries), and the colour
    offsets against the row count on every call."""
    if co.size and int(co[-1]) > rows.shape[0]:  # (negative offsets: refused by the C ABI)
        raise ValueError(f"colour offsets reach past the {rows.shape[0]} member rows")
    key = (n, n_entries, rows.data_ptr())
    if getattr(rows, "_nngp_bounds", None) == key:
        return
    if rows.shape[0]:
        i, e0, e1 = rows[:, 0], rows[:, 1], rows[:, 2]
        if bool(((i < 0) | (i >= n) | (e0 < 0) | (e1 < e0) | (e1 > n_entries)).any()):
            raise ValueError("member_rows hold a location outside [0, n) or a reverse range outside the entries: "
                             "build them with gibbs_member_rows(members, off) for this field")
    rows._nngp_bounds = key


def gibbs_member_rows(members: torch.Tensor, off: torch.Tensor) -> torch.Tensor:
    """int32 (n, 4) rows (location, first / end reverse entry, 0) of the colour-ordered
    ``members`` (nngp_gibbs_member_rows): build once per colouring, pass to :func:`gibbs_w_sweep`."""
    dev = _require_gpu(members, off)
    if members.dtype != torch.int32 or off.dtype != torch.int32 or members.dim() != 1:
        raise ValueError("members and off must be int32, members 1-D")
    members, off = members.contiguous(), off.contiguous()
    rows = torch.empty((members.shape[0], 4), dtype=torch.int32, device=dev)
    _check(load().nngp_gibbs_member_rows(_ptr(members), members.shape[0], _ptr(off), _ptr(rows), _stream(dev)),
           "nngp_gibbs_member_rows")
    return rows


def gibbs_w_sweep(members: torch.Tensor, color_off_host, prep: torch.Tensor, m: int, sigma2: float,
                  tau2: float, yres: torch.Tensor, w: torch.Tensor, r: torch.Tensor, off: torch.Tensor,
                  rev_j: torch.Tensor, seed: int, sweep: int, z: Optional[torch.Tensor] = None,
                  noise_w: Optional[torch.Tensor] = None, member_rows: Optional[torch.Tensor] = None) -> None:
    """One colour-ordered sweep of w_i | rest, in place on w and r (see include/nngp.h);
    ``prep`` from :func:`gibbs_prepare` for the current B / Ft; ``noise_w`` (n,) optional
    weights h_i (noise variance tau2 / h_i); ``member_rows`` from :func:`gibbs_member_rows`
    (built from ``members`` and ``off`` here when not given)."""
    import numpy as np

    dev = _require_gpu(members, prep, yres, w, r, off, rev_j, z, noise_w, member_rows)
    _check_noise_w(noise_w, w.shape[0])
    if member_rows is None:
        member_rows = gibbs_member_rows(members, off)
    elif member_rows.dtype != torch.int32 or tuple(member_rows.shape) != (members.shape[0], 4) \
            or not member_rows.is_contiguous():
        raise ValueError("member_rows must be a contiguous int32 (n, 4) tensor from gibbs_member_rows")
    co = np.ascontiguousarray(color_off_host, dtype=np.int32)
    n = w.shape[0]
    _check_member_rows(member_rows, co, n, 0 if rev_j is None else rev_j.numel())
    _check(load().nngp_gibbs_w_sweep(_ptr(member_rows), co.ctypes.data, len(co) - 1, _ptr(prep), n, int(m),
                                     float(sigma2), float(tau2), _ptr(yres), _ptr(noise_w), _ptr(w), _ptr(r),
                                     _ptr(rev_j),
                                     _ptr(z), int(seed) & (2 ** 64 - 1), int(sweep), _stream(dev)),
           "nngp_gibbs_w_sweep")


def gibbs_w_sweep_tiles(plan, prep: torch.Tensor, m: int, sigma2: float, tau2: float, yres: torch.Tensor,
                        w: torch.Tensor, r: torch.Tensor, off: torch.Tensor, z: torch.Tensor,
                        noise_w: Optional[torch.Tensor] = None, rev_j: Optional[torch.Tensor] = None) -> None:
    """The tiled colour sweep (nngp_gibbs_w_sweep_tiles) over a :class:`pynngp_amd.gibbs_tiles.TilePlan`: one
    launch per phase, each tile's footprint of r in LDS; in place on w and r; ``z`` the normals
    (:func:`gibbs_normals`).  The order is the plan's (level, phase, colour) -- its ``effective_colors`` as a
    colouring.  The plan must be contiguous (its node order is the storage order: ``plan.contiguous``;
    :func:`pynngp_amd.gibbs_tiles.contiguous_plan` / SeqNNGP(sweep="tiled") arrange it).  A plan built with
    coarse="colour" sweeps its coarse nodes after the tiles, one launch per colour (:func:`gibbs_w_sweep`,
    which needs ``rev_j``)."""
    dev = _require_gpu(prep, yres, w, r, off, z, noise_w, plan.tinfo)
    _check_noise_w(noise_w, w.shape[0])
    if not plan.contiguous:
        raise ValueError("the tiled sweep needs a contiguous tile plan (tile t's nodes = storage rows [n0, n1)): "
                         "store the field in plan.tnodes order and rebuild the plan there")
    if plan.tnodes.numel() != w.shape[0]:
        raise ValueError(f"the tile plan covers {plan.tnodes.numel()} nodes, the field has {w.shape[0]}")
    key = (w.shape[0], off.data_ptr())
    if getattr(plan, "_bounds_ok", None) != key:  # what the kernel indexes unchecked, once per plan and field
        from .gibbs_tiles import validate_launch_bounds

        validate_launch_bounds(plan, off, w.shape[0])
        plan._bounds_ok = key
    tiles, poff, plds = plan.launch_arrays()
    _check(load().nngp_gibbs_w_sweep_tiles(_ptr(tiles), poff.ctypes.data, plds.ctypes.data, len(plds),
                                           _ptr(plan.tinfo), _ptr(plan.tstep), int(plan.ecap), _ptr(plan.tfp),
                                           _ptr(off), _ptr(plan.rev_loc), _ptr(prep), w.shape[0], int(m),
                                           int(plan.rev_loc.numel()), float(sigma2), float(tau2), _ptr(yres),
                                           _ptr(noise_w), _ptr(w), _ptr(r), _ptr(z), _stream(dev)),
           "nngp_gibbs_w_sweep_tiles")
    if plan.coarse_members is not None and plan.coarse_members.numel() > 0:
        if rev_j is None:
            raise ValueError("a tile plan with coarse nodes swept per colour needs rev_j")
        if getattr(plan, "_coarse_rows", None) is None:
            plan._coarse_rows = gibbs_member_rows(plan.coarse_members, off)
        gibbs_w_sweep(plan.coarse_members, plan.coarse_color_off, prep, m, sigma2, tau2, yres, w, r, off, rev_j, 0, 0,
                      z=z, noise_w=noise_w, member_rows=plan._coarse_rows)


def gibbs_w_sweep_chains(member_rows: torch.Tensor, color_off_host, preps, m: int, sigma2s, tau2s, yres, w, r,
                         rev_j: torch.Tensor, z, noise_w: Optional[torch.Tensor] = None) -> None:
    """:func:`gibbs_w_sweep` for up to 8 independent chains of one field in ONE launch per colour
    (nngp_gibbs_w_sweep_chains): ``member_rows`` / colours / ``rev_j`` / ``noise_w`` shared, per chain
    lists of ``preps``, ``sigma2s``, ``tau2s``, ``yres`` and given normals ``z``; ``w`` and ``r`` either
    per-chain lists of (n,) vectors or two contiguous (n, C) tensors holding the chains interleaved
    (nngp_gibbs_w_sweep_chains_il: one sector per scattered access for all chains).  Chain c's result is
    bit-identical to :func:`gibbs_w_sweep` on its own arguments with its ``z``."""
    import numpy as np

    C = len(preps)
    il = isinstance(w, torch.Tensor)
    if il != isinstance(r, torch.Tensor):
        raise ValueError("w and r: both per-chain lists or both (n, C) tensors")
    per = (sigma2s, tau2s, yres, z) if il else (sigma2s, tau2s, yres, w, r, z)
    if not 1 <= C <= 8 or not all(len(v) == C for v in per):
        raise ValueError("1..8 chains, one entry per chain in every list")
    n = w.shape[0] if il else w[0].shape[0]
    if il:
        for t in (w, r):
            if t.dtype != torch.float64 or tuple(t.shape) != (n, C) or not t.is_contiguous():
                raise ValueError(f"interleaved w / r must be contiguous float64 ({n}, {C})")
    vecs = list(yres) + list(z) + ([] if il else list(w) + list(r))
    for t in vecs:
        if t.dtype != torch.float64 or tuple(t.shape) != (n,) or not t.is_contiguous():
            raise ValueError(f"per-chain vectors must be contiguous float64 ({n},)")
    if member_rows.dtype != torch.int32 or member_rows.dim() != 2 or member_rows.shape[1] != 4 \
            or not member_rows.is_contiguous():
        raise ValueError("member_rows must be a contiguous int32 (n, 4) tensor from gibbs_member_rows")
    dev = _require_gpu(member_rows, rev_j, noise_w, *preps, *vecs, *((w, r) if il else ()))
    _check_noise_w(noise_w, n)
    co = np.ascontiguousarray(color_off_host, dtype=np.int32)
    _check_member_rows(member_rows, co, n, 0 if rev_j is None else rev_j.numel())
    P = ctypes.c_void_p * C
    D = ctypes.c_double * C
    head = (_ptr(member_rows), co.ctypes.data, len(co) - 1, C, P(*[_ptr(t) for t in preps]), n, int(m),
            D(*map(float, sigma2s)), D(*map(float, tau2s)), P(*[_ptr(t) for t in yres]), _ptr(noise_w))
    tail = (_ptr(rev_j), P(*[_ptr(t) for t in z]), _stream(dev))
    if il:
        _check(load().nngp_gibbs_w_sweep_chains_il(*head, _ptr(w), _ptr(r), *tail), "nngp_gibbs_w_sweep_chains_il")
    else:
        _check(load().nngp_gibbs_w_sweep_chains(*head, P(*[_ptr(t) for t in w]), P(*[_ptr(t) for t in r]), *tail),
               "nngp_gibbs_w_sweep_chains")


def gibbs_normals(z: torch.Tensor, seed: int, sweep: int) -> torch.Tensor:
    """Fill z (float64 (n,)) with the sweep's Philox normals (nngp_gibbs_normals)."""
    dev = _require_gpu(z)
    if z.dtype != torch.float64 or z.dim() != 1:
        raise ValueError("z must be float64 (n,)")
    _check(load().nngp_gibbs_normals(z.shape[0], int(seed) & (2 ** 64 - 1), int(sweep), _ptr(z), _stream(dev)),
           "nngp_gibbs_normals")
    return z


def gibbs_stats(r: torch.Tensor, Ft: torch.Tensor, yres: torch.Tensor, y: torch.Tensor, X: Optional[torch.Tensor],
                w: torch.Tensor, out: Optional[torch.Tensor] = None,
                workspace: Optional[torch.Tensor] = None, noise_w: Optional[torch.Tensor] = None) -> torch.Tensor:
    """[sum r^2/Ft, sum h (yres - w)^2, X^T H (y - w)...] as a float64 device tensor (2 + p,);
    h = ``noise_w`` (n,) or 1."""
    dev = _require_gpu(r, Ft, yres, y, X, w, noise_w)
    _check_noise_w(noise_w, r.shape[0])
    n = r.shape[0]
    p = 0 if X is None else X.shape[1]
    lib = load()
    out = torch.empty(2 + p, dtype=torch.float64, device=dev) if out is None else out
    need = lib.nngp_gibbs_stats_workspace_bytes(n, p)
    if workspace is None or workspace.numel() < need:
        workspace = _workspace(need, dev)
    _check(lib.nngp_gibbs_stats(n, _ptr(r), _ptr(Ft), _ptr(yres), _ptr(y), _ptr(X), p, _ptr(w), _ptr(noise_w), _ptr(out),
                                _ptr(workspace), workspace.numel(), _stream(dev)), "nngp_gibbs_stats")
    return out
