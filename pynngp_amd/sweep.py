"""Device-resident, optionally sharded NNGP log-likelihood sweep.

SURVEY.md 8(e): every location's B_i, F_i and log-lik term is independent given
read-only coordinates and values, so locations shard contiguously -- rank r of
P owns rows [floor(rN/P), floor((r+1)N/P)).  Coordinates and values are
replicated (neighbours j < i may sit in any earlier shard).  Each rank builds the
neighbour sets of its own rows only.  The one exchange per sweep is the summed
log-likelihood: the 4-double partials of every rank are all-gathered (RCCL over
xGMI with the "nccl" backend; gloo in the CPU tests) and summed in rank order,
so the result is bit-identical on every rank and run to run.

The per-shard compute and neighbour build are injectable so the distributed
combination logic is testable on CPU with the oracle (tests/test_distributed.py);
the default compute is the HIP kernel through the native operator
``torch.ops.nngp.bf_sweep_out`` (pynngp_amd/ops.py, libnngp_torch_ops.so).
"""
from __future__ import annotations

import math
import time
from typing import Callable, Optional

import torch
import torch.distributed as dist

from . import _lib, ops
from .nngp import Covariance, LOG_2PI, _raise_on_bad


# ShardedLogLik(plan=None): sweep through a wave pair plan (pair_plan.h)?  Off by default: measured on the
# same box (profiles/r06a, r06c), the planned kernel executes 19.5 % fewer VALU instructions
# at m = 15 but the sweep takes 0.230 against 0.172 ms at N = 1e6 -- the plan's ~420 B per location are a
# dependent HBM stream at every wave's start, and the shared covariances' LDS round trips cost what the saved
# instructions buy (a cache-resident plan: 0.180 ms).  plan=True opts in.
PLAN_DEFAULT = False


def shard_range(n: int, rank: int, world: int):
    """Contiguous shard [lo, hi) of n locations for rank of world."""
    return (n * rank) // world, (n * (rank + 1)) // world


def _collective_default(collective: Optional[bool]) -> bool:
    """Exchange partials through torch.distributed whenever a process group exists (so a
    one-rank RCCL group runs the same all-gather + fold as N ranks), unless told otherwise."""
    if collective is not None:
        return bool(collective)
    return dist.is_available() and dist.is_initialized()


def combine_partials(local: torch.Tensor, world: int, group=None, force: bool = False) -> torch.Tensor:
    """All-gather the (4,) partials and reduce them in rank order.

    [0], [1] are summed; [2], [3] (first bad row or -1) take the smallest non-negative.
    One rank returns ``local`` itself unless ``force`` (then the collective and the fold run
    exactly as with N ranks: the path a one-GPU box can test).
    """
    if world == 1 and not force:
        return local
    gathered = torch.empty((world, 4), dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(gathered, local.reshape(1, 4), group=group)
    if gathered.device.type == "cuda":
        ops.load()  # torch.ops.nngp.combine_partials_out lives in libnngp_torch_ops.so
        out = torch.empty(4, dtype=local.dtype, device=local.device)
        torch.ops.nngp.combine_partials_out(gathered, out)  # one tiny HIP kernel, rank order
        return out
    # CPU (gloo) path: the same fold on the host, for the multi-process tests
    return combine_partials_host(gathered)


class ShardedLogLik:
    """Log-likelihood sweep over this rank's contiguous shard of N locations.

    ``coords`` and ``values`` are the full (replicated) arrays on this rank's device.

    ``layout``:
      * ``"natural"`` -- shard = input rows [lo, hi); rows are visited in Z-order
        (``nngp_row_order``) but B / F are rows of the input order;
      * ``"storage"`` -- every per-location array is relabelled into one global
        Z-order STORAGE order (slot p holds input location ``perm[p]``; all ranks
        compute the same ``perm``), the shard is storage slots [lo, hi) (a spatial
        region), neighbour indices point into storage, and B / F are storage rows.
        A location's neighbours then sit near it in memory (the gathers share cache
        lines, the B / F stores are contiguous): ~8-15 % faster sweeps.
        The log-likelihood is label-invariant (same terms, same visiting order: the
        partials are bit-identical to ``"natural"`` on one rank).  Values are taken in
        input order and gathered per call, or given in storage order
        (``values_layout="storage"``, e.g. an MCMC state kept there).
    """

    def __init__(self, coords: torch.Tensor, m: int, rank: int = 0, world: int = 1, group=None,
                 algo: str = "auto", build_nbr: Optional[Callable] = None, compute: Optional[Callable] = None,
                 spatial_order: bool = True, layout: str = "natural", build_perm: Optional[Callable] = None,
                 api: str = "ops", collective: Optional[bool] = None, plan: Optional[bool] = None):
        if layout not in ("natural", "storage"):
            raise ValueError(f"layout must be 'natural' or 'storage', got {layout!r}")
        if api not in ("ops", "ctypes"):
            raise ValueError(f"api must be 'ops' (torch.ops.nngp) or 'ctypes' (the same C ABI via ctypes), got {api!r}")
        self.api = api
        self.layout = layout
        if not bool(torch.isfinite(coords).all()):
            raise ValueError("coordinates must be finite (NaN / inf would silently decouple locations)")
        self.coords = coords
        self.n = coords.shape[0]
        self.m = int(m)
        self.rank, self.world, self.group = rank, world, group
        # partials go through the all-gather whenever torch.distributed is initialised (also at
        # world 1), or as ``collective`` says
        self.collective = _collective_default(collective)
        self.lo, self.hi = shard_range(self.n, rank, world)
        self.algo = algo
        self._compute = compute
        self._ws = None
        self._partials = None
        self.order = None
        self.perm = self.pos = None
        if layout == "storage":
            # global Z-order storage order (identical on every rank); injectable for the CPU tests
            perm = _lib.row_order(coords)[0] if build_perm is None else build_perm(coords)
            self.perm = perm
            self.pos = torch.empty(self.n, dtype=torch.int32, device=coords.device)
            self.pos[perm.long()] = torch.arange(self.n, dtype=torch.int32, device=coords.device)
            self._coords_sweep = coords[perm.long()].contiguous()
            rows = perm[self.lo:self.hi].contiguous()
            nbr0 = _lib.knn_prior_rows(coords, self.m, rows) if build_nbr is None else build_nbr(coords, self.m, rows)
            nb = nbr0.long()
            self.nbr = torch.where(nb >= 0, self.pos[nb.clamp(min=0)], -1).to(torch.int32).contiguous()
            self._nbr_sweep = self.nbr
            self._vstore = torch.empty(self.n, dtype=torch.float64, device=coords.device)
        else:
            self._coords_sweep = coords
            if build_nbr is None:
                self.nbr = _lib.knn_prior(coords, self.m, self.lo, self.hi)
            else:
                self.nbr = build_nbr(coords, self.m, self.lo, self.hi)
            self._nbr_sweep = self.nbr
            if compute is None and spatial_order and self.hi > self.lo:
                self.order, self._nbr_sweep = _lib.row_order(coords, self.lo, self.hi - self.lo, self.nbr)
        if compute is None:
            ops.load()  # sweeps go through torch.ops.nngp.bf_sweep_out (libnngp_torch_ops.so)
            # the resolved overload: calling it skips the packet's overload resolution per sweep
            # (host issue time is what bounds a sweep of ~10^5 rows)
            self._sweep_op = torch.ops.nngp.bf_sweep_out.default
            self._algo_code = ops.algo_code(algo)
            self._ws = _lib.bf_workspace(self.hi - self.lo, self.m, algo, coords.device, dim=coords.shape[1])
            self._partials = torch.empty(4, dtype=torch.float64, device=coords.device)
            self._B = torch.empty((self.hi - self.lo, self.m), dtype=torch.float64, device=coords.device)
            self._F = torch.empty((self.hi - self.lo,), dtype=torch.float64, device=coords.device)
        # wave pair plan (pair_plan.h): every covariance a wavefront shares evaluated once; built once here
        # (one host synchronisation), used by every sweep of a kind it serves.  plan=None: when supported.
        self._plan = self._plan_ctypes = None
        self.plan_build_s = 0.0
        self.plan_read_bytes = 0  # bytes a planned sweep streams from the plan (_lib.pair_plan_read_bytes)
        want = plan if plan is not None else PLAN_DEFAULT
        d = coords.shape[1]
        if (compute is None and want and self.hi > self.lo and algo in ("auto", "pairb")
                and _lib.pair_plan_supported(self.m, "exponential", d)):
            t0 = time.perf_counter()
            self._plan = ops.pair_plan(self._nbr_sweep, self.order, self.lo, self.n, d)
            self.plan_build_s = time.perf_counter() - t0
            self._plan_ctypes = _lib.PairPlan(self._plan[0], self._plan[1].tolist(), self._nbr_sweep, self.order)
            self.plan_read_bytes = _lib.pair_plan_read_bytes(self._plan[0], self.m)
        elif plan:
            raise ValueError(f"pair plans serve algo auto / pairb, 2 <= m <= 17, dim 1..3 (m={self.m}, dim={d})")

    @property
    def planned(self) -> bool:
        """Whether sweeps of the plan-served kinds (exponential .. spherical) run through a pair plan."""
        return self._plan is not None

    def _plan_for(self, kind: str):
        return self._plan if (self._plan is not None and _lib.KIND_CODES.get(kind, 99) <= 4) else None

    def to_storage(self, values: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Input-order per-location values -> storage order (layout 'storage')."""
        return torch.index_select(values, 0, self.perm, out=out)

    def local_partials(self, cov: Covariance, values: Optional[torch.Tensor], want_bf: bool = True,
                       values_layout: str = "input", out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Stream-ordered partials of this shard (no host sync); into ``out`` (4,) if given."""
        if self.layout == "storage" and values is not None and values_layout == "input":
            values = self.to_storage(values, out=self._vstore)
        if self._compute is not None:
            p = self._compute(self, cov, values, want_bf)
            return p if out is None else out.copy_(p)
        B, F = (self._B, self._F) if want_bf else (None, None)
        p = self._partials if out is None else out
        s2, phi, tau2 = cov.theta
        plan = self._plan_for(cov.kind)
        if self.api == "ctypes":  # the same C-ABI call without the dispatcher (A/B of the op overhead)
            _lib.bf_sweep(self._coords_sweep, self._nbr_sweep, self.lo, cov.kind, s2, phi, tau2, values=values,
                          want_bf=want_bf, algo=self.algo, B=B, F=F, partials=p, workspace=self._ws, order=self.order,
                          nu=cov.nu_arg, plan=self._plan_ctypes if plan is not None else None)
            return p
        pb, pi = plan if plan is not None else (None, None)
        self._sweep_op(self._coords_sweep, self._nbr_sweep, self.order, self.lo, ops.kind_code(cov.kind),
                       float(s2), float(phi), float(tau2), values, B, F, None, p, self._ws, self._algo_code,
                       -1.0 if cov.nu_arg is None else cov.nu_arg, pb, pi)
        return p

    def partials(self, cov: Covariance, values: Optional[torch.Tensor], want_bf: bool = True,
                 values_layout: str = "input") -> torch.Tensor:
        """Global partials (all ranks), stream-ordered."""
        return combine_partials(self.local_partials(cov, values, want_bf, values_layout), self.world, self.group,
                                force=self.collective)

    def loglik(self, cov: Covariance, values: torch.Tensor, want_bf: bool = False,
               values_layout: str = "input") -> float:
        """Global NNGP log-likelihood (synchronises the host)."""
        p = self.partials(cov, values, want_bf, values_layout).cpu().numpy()
        _raise_on_bad(p)
        return -0.5 * (self.n * LOG_2PI + p[0] + p[1])

    def loglik_scan(self, covs, values: torch.Tensor, values_layout: str = "input") -> list:
        """Global log-likelihoods at many covariances (a grid / profile-likelihood scan, a
        batch of MH proposals) with ONE host synchronisation: the sweeps run back to back
        and each sweep's all-gather overlaps the next sweep (:class:`PipelinedCombine`)."""
        covs = list(covs)
        if self.layout == "storage" and values is not None and values_layout == "input":
            values = self.to_storage(values, out=self._vstore)
            values_layout = "storage"
        pipe = PipelinedCombine(self, len(covs))
        for k, cov in enumerate(covs):
            self.local_partials(cov, values, False, values_layout, out=pipe.local[k])
            pipe.exchange(k)
        res = pipe.finish().cpu().numpy()
        out = []
        for p in res:
            _raise_on_bad(p)
            out.append(-0.5 * (self.n * LOG_2PI + p[0] + p[1]))
        return out

    @property
    def rows_input(self) -> torch.Tensor:
        """Input-order location index of each local row of B / F (int64)."""
        if self.layout == "storage":
            return self.perm[self.lo:self.hi].long()
        return torch.arange(self.lo, self.hi, device=self.coords.device)

    @property
    def B(self):
        """(hi - lo, m) rows of this shard (storage rows for layout 'storage'; see rows_input).
        Neighbour slot s of a row refers to ``nbr[row, s]`` (storage indices for 'storage')."""
        return self._B

    @property
    def F(self):
        return self._F


class PipelinedCombine:
    """Throughput mode for independent sweeps (a theta scan, a batch of MH proposals,
    the benchmark): sweep k writes its partials to slot k; every ``batch`` sweeps ONE
    all-gather of the (batch, 4) block of slots runs asynchronously on the RCCL stream and
    the rank-order fold of the whole block on a side stream (nngp_combine_partials_batch),
    so the sweeps go on while the collective is in flight and the per-collective host cost
    is paid once per batch, not per sweep (one collective per sweep measured +15 % per step on
    a one-rank RCCL group: 0.198 vs 0.172 ms).  Every sweep's global partials end up in row k
    of :meth:`finish`, bit-identical to exchanging each sweep alone.

        pipe = PipelinedCombine(sweep, K)
        for k in range(K):
            sweep.local_partials(cov_k, v, out=pipe.local[k])
            pipe.exchange(k)
        res = pipe.finish()      # (K, 4), stream-ordered
    """

    def __init__(self, sweep: "ShardedLogLik", slots: int, batch: int = 16):
        dev = sweep.coords.device
        self.sweep = sweep
        self.world = sweep.world
        self.active = self.world > 1 or getattr(sweep, "collective", False)
        if dev.type == "cuda":
            ops.load()  # torch.ops.nngp.combine_partials_out lives in libnngp_torch_ops.so
        self.batch = max(1, int(batch))
        self.local = torch.empty((slots, 4), dtype=torch.float64, device=dev)
        # the all-gather of slots [b0, b1) lands in gathered[b0 * world * 4 : b1 * world * 4] as (world, b1 - b0, 4)
        self.gathered = torch.empty((slots * self.world * 4,), dtype=torch.float64, device=dev)
        self.results = torch.empty((slots, 4), dtype=torch.float64, device=dev)
        self.side = torch.cuda.Stream(device=dev) if dev.type == "cuda" else None
        self.k = 0
        self.flushed = 0
        self.n_collectives = 0

    def exchange(self, k: int) -> None:
        self.k = max(self.k, k + 1)
        if self.active and self.k - self.flushed >= self.batch:
            self._flush()

    def _flush(self) -> None:
        b0, b1 = self.flushed, self.k
        if b1 <= b0:
            return
        nb = b1 - b0
        out = self.gathered[b0 * self.world * 4: b1 * self.world * 4]
        work = dist.all_gather_into_tensor(out, self.local[b0:b1].reshape(-1), group=self.sweep.group,
                                           async_op=True)
        self.flushed = b1
        self.n_collectives += 1
        g = out.view(self.world, nb, 4)
        if self.side is None:
            work.wait()
            for j in range(nb):
                self.results[b0 + j].copy_(combine_partials_host(g[:, j, :]))
            return
        with torch.cuda.stream(self.side):
            work.wait()  # the side stream waits for the collective, the compute stream does not
            torch.ops.nngp.combine_partials_out(g, self.results[b0:b1])

    def finish(self) -> torch.Tensor:
        if not self.active:
            return self.local[: self.k]
        self._flush()
        if self.side is not None:
            torch.cuda.current_stream(self.side.device).wait_stream(self.side)
        return self.results[: self.k]


def combine_partials_host(g: torch.Tensor) -> torch.Tensor:
    """Rank-order fold of gathered (world, 4) partials on the host (CPU / gloo path)."""
    rows = g.tolist()
    flags = [[r[2] for r in rows if r[2] >= 0], [r[3] for r in rows if r[3] >= 0]]
    out = [0.0, 0.0] + [min(f) if f else -1.0 for f in flags]
    for r in rows:
        out[0] += r[0]
        out[1] += r[1]
    return torch.tensor(out, dtype=g.dtype)


def loglik_from_partials(p, n: int) -> float:
    return -0.5 * (n * LOG_2PI + float(p[0]) + float(p[1]))


__all__ = ["shard_range", "combine_partials", "ShardedLogLik", "PipelinedCombine", "loglik_from_partials", "math"]
