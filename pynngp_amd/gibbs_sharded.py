"""One Gibbs chain sharded over ranks ("for Gibbs (config 5), the w-update adds
per-colour halo exchanges").

``SeqNNGP`` runs one chain per GPU.  ``ShardedSeqNNGP`` runs ONE chain over all ranks of a
``torch.distributed`` group (RCCL over xGMI; gloo in the CPU tests and the one-GPU rehearsal):

* rank r owns the storage rows [lo, hi) of ``shard_range`` -- a spatial region of the Z-order
  storage layout, so a location's parents and children are mostly its own;
* every rank keeps full-length replicas of w and of the residuals r = w - B w_N, exact (bit for
  bit equal to the owner's values) on its own rows, their out-of-shard children (the halo H) and
  the parents of both (the set V); the rest of the replica is never read;
* phi | w: the B/F sweep of the own rows (its partials folded over ranks in rank order) and of
  the halo rows (a second sweep over a gathered table: same kernel, same operands, so the same
  bits as the owner's rows);
* per colour: the own members' colour step (``nngp_gibbs_w_color``) publishes the members' new w
  into a send slot; a halo exchange -- ONE all-gather per colour of only the members some other
  rank keeps a replica of (the boundary: ``exported``; each rank's run of a colour is ordered
  boundary members first, so they are the head of the slot) --; ``nngp_gibbs_w_apply`` replays the
  draws of the other ranks' members in V (dw from this rank's replica = the owner's operands, so
  the owner's bits);
* sigma2, tau2, beta: the stats of the own rows, all-gathered and folded in rank order, so every
  rank draws the same scalars from the same host RNG stream.

The chain is the single-GPU chain: the same Philox normals (keyed by location and sweep), the same
per-location arithmetic; only the summation order of the global sums (the log density of the
proposal, the conjugate statistics) follows the ranks.  With one rank it is ``SeqNNGP``'s chain
bit for bit (tests/test_gpu_gibbs_sharded.py).  Cost per iteration on top of the sharded work:
one all-gather per colour (32 at m = 15) of the boundary members' w (``plan.exchange_bytes`` per
rank and sweep, against ``plan.allgather_bytes`` for every member) and their replay.
"""
from __future__ import annotations

import dataclasses
from typing import Optional

import numpy as np
import torch
import torch.distributed as dist

from . import _lib, ops
from .gibbs import SeqNNGP
from .sweep import combine_partials, shard_range


@dataclasses.dataclass
class GibbsShardPlan:
    """Host-side plan of one rank of a sharded chain (numpy; see :func:`gibbs_shard_plan`)."""
    world: int
    rank: int
    lo: int
    hi: int
    bounds: np.ndarray      # (world + 1,) shard boundaries
    run: np.ndarray         # (n_colors, world + 1): members_x[run[c, r]:run[c, r + 1]] = rank r's members of colour c
    maxc: np.ndarray        # (n_colors,) the largest per-rank run of each colour (the send slot size)
    send_off: np.ndarray    # (n_colors + 1,) colour c's send slot: send[send_off[c]:send_off[c] + maxc[c]]
    recv_off: np.ndarray    # (n_colors + 1,) colour c's gathered block: recv[recv_off[c]:recv_off[c + 1]]
    halo: np.ndarray        # (n_h,) out-of-shard children of the own rows, ascending
    replica: np.ndarray     # (n_v,) V: own rows, halo and the parents of both, ascending
    apply_rows: np.ndarray  # (n_apply, 4) int32 (i, off[i], off[i + 1], src) of the foreign rows of V, by colour
    apply_off: np.ndarray   # (n_colors + 1,)
    members_x: np.ndarray   # (n,) the members by colour; each (colour, rank) run: boundary members first, ascending
    exported: np.ndarray    # (n,) bool: the row is in some other rank's replica set V (the boundary)
    bcount: np.ndarray      # (n_colors, world) boundary members per (colour, rank): the head of each run
    bmax: np.ndarray        # (n_colors,) the largest bcount of each colour: the all-gather size per rank
    exchange_bytes: int     # bytes one rank receives per sweep (sum_c world * bmax[c] * 8)
    allgather_bytes: int    # ... had every member been all-gathered (sum_c world * maxc[c] * 8)


def _tt(a, dev, dtype=torch.int64):
    """an input array as a torch tensor on dev (device tensors stay where they are)"""
    t = a if isinstance(a, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(a))
    return t.to(device=dev, dtype=dtype)


def gibbs_shard_plan(nbr, off, rev_j, colors, members, color_off, world: int, rank: int,
                     exchange: str = "halo", device=None) -> GibbsShardPlan:
    """Plan rank ``rank`` of ``world`` for the DAG in storage order (nbr (n, m), reverse CSR off / rev_j,
    colours, members grouped by colour ascending inside a colour, colour offsets -- numpy arrays or
    torch tensors).  Every rank computes the same runs, slot sizes and sources.  ``exchange="halo"`` moves
    the boundary members only; ``"all"`` every member (round 3's all-gather: the A/B reference, and at
    one rank the only way to put a collective in the colour loop).  The array work runs in torch on
    ``device`` (default: the inputs' device; a sharded chain plans on its GPU -- round 5: 12 s per rank
    at N = 1e7 in host numpy); the plan's fields come back as numpy arrays."""
    if exchange not in ("halo", "all"):
        raise ValueError("exchange must be 'halo' or 'all'")
    dev = torch.device(device) if device is not None else (nbr.device if isinstance(nbr, torch.Tensor)
                                                           else torch.device("cpu"))
    nbr = _tt(nbr, dev, torch.int64)
    off = _tt(off, dev)
    rev_j = _tt(rev_j, dev)
    colors = _tt(colors, dev)
    members = _tt(members, dev)
    color_off = _tt(color_off, dev)
    n = nbr.shape[0]
    n_colors = color_off.numel() - 1
    bounds_l = [shard_range(n, r, world)[0] for r in range(world)] + [n]
    bounds = torch.tensor(bounds_l, dtype=torch.int64, device=dev)
    lo, hi = bounds_l[rank], bounds_l[rank + 1]
    # members ascend inside each colour and the colours are contiguous runs: (colour, member) keys ascend
    # over the whole array, so one searchsorted gives every (colour, rank) run
    key_cm = colors[members] * (n + 1) + members if n_colors else members
    if members.numel() > 1 and not bool((key_cm[1:] > key_cm[:-1]).all()):
        raise ValueError("members must ascend inside each colour (storage order)")
    cidx = torch.arange(n_colors, dtype=torch.int64, device=dev)
    run = torch.searchsorted(key_cm, (cidx[:, None] * (n + 1) + bounds[None, :]).contiguous()) if n_colors else \
        torch.zeros((0, world + 1), dtype=torch.int64, device=dev)
    counts = run[:, 1:] - run[:, :-1]
    maxc = counts.max(dim=1).values if world > 0 and n_colors else torch.zeros(n_colors, dtype=torch.int64, device=dev)
    send_off = torch.cat([torch.zeros(1, dtype=torch.int64, device=dev), torch.cumsum(maxc, 0)])
    exported = gibbs_boundary(nbr, bounds) if exchange == "halo" else torch.ones(n, dtype=torch.bool, device=dev)
    # each (colour, rank) run ordered boundary members first (ascending), then the rest: the colour
    # step's publish slot then starts with exactly the values the other ranks replay.  (Members of a
    # colour are independent and their normals are keyed by location, so the order changes no bit.)
    key = torch.repeat_interleave(torch.arange(n_colors * world, dtype=torch.int64, device=dev), counts.reshape(-1))
    xkey = (key << 33) | ((~exported[members]).to(torch.int64) << 32) | members
    members_x = members[torch.sort(xkey)[1]]
    cs = torch.cat([torch.zeros(1, dtype=torch.int64, device=dev), torch.cumsum(exported[members_x].to(torch.int64), 0)])
    bcount = cs[run[:, 1:]] - cs[run[:, :-1]]
    bmax = bcount.max(dim=1).values if world > 0 and n_colors else torch.zeros(n_colors, dtype=torch.int64, device=dev)
    recv_off = torch.cat([torch.zeros(1, dtype=torch.int64, device=dev), torch.cumsum(bmax * world, 0)])
    # halo: children of the own rows outside the shard; V: own rows, halo, parents of both
    ch = rev_j[int(off[lo]):int(off[hi])]
    halo = torch.unique(ch[(ch < lo) | (ch >= hi)])
    par = torch.cat([nbr[lo:hi].reshape(-1), nbr[halo].reshape(-1)])
    par = par[(par >= 0) & (par < n)]
    replica = torch.unique(torch.cat([torch.arange(lo, hi, dtype=torch.int64, device=dev), halo, par]))
    foreign = replica[(replica < lo) | (replica >= hi)]
    if not bool(exported[foreign].all()):
        raise AssertionError("a foreign replica row is not on its owner's boundary")
    pos = torch.empty(n, dtype=torch.int64, device=dev)
    pos[members_x] = torch.arange(n, dtype=torch.int64, device=dev)
    cf = colors[foreign]
    owner = torch.searchsorted(bounds, foreign, right=True) - 1
    k = pos[foreign] - run[cf, owner]  # rank among the owner's boundary members of the colour
    src = recv_off[cf] + owner * bmax[cf] + k
    order = torch.sort(cf, stable=True)[1]
    apply_rows = torch.stack([foreign, off[foreign], off[foreign + 1], src], dim=1)[order].to(torch.int32)
    apply_off = torch.cat([torch.zeros(1, dtype=torch.int64, device=dev),
                           torch.cumsum(torch.bincount(cf, minlength=n_colors), 0)])
    h = lambda t: t.cpu().numpy()  # noqa: E731
    return GibbsShardPlan(world, rank, lo, hi, h(bounds), h(run), h(maxc), h(send_off), h(recv_off), h(halo),
                          h(replica), np.ascontiguousarray(h(apply_rows)), h(apply_off), h(members_x.to(torch.int32)),
                          h(exported), h(bcount), h(bmax), int(8 * world * int(bmax.sum())),
                          int(8 * world * int(maxc.sum())))


def gibbs_boundary(nbr, bounds):
    """exported[i]: row i is in the replica set V(r) = own(r) + H(r) + parents of both of some rank r
    other than its owner (H(r): the out-of-shard children of own(r)).  i is in V(r), r != owner(i),
    exactly when i has a parent owned by r (i in H(r)), or i is a parent of a row j that r owns or that
    has a parent owned by r (i in parents(own(r) + H(r))).  With T(j) = {owner(j)} + owners of j's
    parents: exported[i] = T(i) != {owner(i)} or T(j) != {owner(i)} for some child j of i -- one pass over
    the parent lists (nbr, -1 padded), identical on every rank.  numpy or torch in, the same kind out."""
    as_np = not isinstance(nbr, torch.Tensor)
    nbr = _tt(nbr, torch.device("cpu") if as_np else nbr.device)
    bounds = _tt(bounds, nbr.device)
    n = nbr.shape[0]
    own = torch.repeat_interleave(torch.arange(bounds.numel() - 1, dtype=torch.int64, device=nbr.device),
                                  bounds[1:] - bounds[:-1])
    valid = (nbr >= 0) & (nbr < n)
    on = torch.where(valid, own[torch.where(valid, nbr, 0)], -1)
    big = torch.iinfo(torch.int64).max
    tmin = torch.minimum(own, torch.where(valid, on, big).min(dim=1).values) if nbr.shape[1] else own
    tmax = torch.maximum(own, on.max(dim=1).values) if nbr.shape[1] else own
    exported = (tmin != own) | (tmax != own)
    jj, ss = torch.nonzero(valid, as_tuple=True)
    pi = nbr[jj, ss]
    hit = (tmin[jj] != own[pi]) | (tmax[jj] != own[pi])
    exported[pi[hit]] = True
    return exported.cpu().numpy() if as_np else exported


class ColourExchange:
    """The per-colour all-gather of a sharded chain: the own members' new w go to
    ``send[send_off[c]:...]`` and arrive at every rank in ``recv[recv_off[c]:recv_off[c + 1]]``
    as (world, maxc[c]) (rank-major).  Device buffers on the chain's device (RCCL), or CPU
    tensors with gloo (the CPU tests)."""

    def __init__(self, plan: GibbsShardPlan, device, group=None, active: bool = True):
        self.plan, self.group, self.active = plan, group, active
        self.send = torch.zeros(int(plan.send_off[-1]) + 1, dtype=torch.float64, device=device)
        self.recv = torch.zeros(int(plan.recv_off[-1]) + 1, dtype=torch.float64, device=device)
        self.n_collectives = 0

    def send_slot(self, c: int) -> torch.Tensor:
        """Colour c's publish slot (maxc[c] values; the head, bmax[c], goes out)."""
        a = int(self.plan.send_off[c])
        return self.send[a:a + int(self.plan.maxc[c])]

    def exchange(self, c: int) -> None:
        """The halo exchange of colour c: every rank's boundary members' new w (the head of its slot,
        bmax[c] values) all-gathered, (world, bmax[c]) rank-major; nothing when no rank has one."""
        p = self.plan
        if not self.active or p.bmax[c] == 0:
            return
        a = int(p.send_off[c])
        dist.all_gather_into_tensor(self.recv[int(p.recv_off[c]):int(p.recv_off[c + 1])],
                                    self.send[a:a + int(p.bmax[c])], group=self.group)
        self.n_collectives += 1


class ShardedSeqNNGP(SeqNNGP):
    """One NNGP Gibbs chain over the ranks of a process group (module docstring).

    Built on every rank with the same arguments as :class:`SeqNNGP` (the same data, seed and
    settings: the DAG, colouring and storage order are computed identically everywhere), plus
    ``rank`` / ``world`` / ``group`` (default: the initialised ``torch.distributed`` group;
    without one, a single rank).  ``collective`` forces the exchanges through the group even at
    one rank (the path a one-GPU box tests).  ``graphs`` (default: on over RCCL) replays the
    colour loop from captured HIP graphs.  Results (``w_nodes`` / ``w_s`` / ``w_t``,
    ``sample``) are gathered over the ranks and identical on every rank.  ``exchange``: "halo" (the
    boundary members per colour, default) or "all" (every member, round 3's all-gather).
    """

    _use_plan = False  # the phi sweeps cover this rank's rows and halo, not the whole field

    def __init__(self, *args, rank: Optional[int] = None, world: Optional[int] = None, group=None,
                 collective: Optional[bool] = None, graphs: Optional[bool] = None, exchange: str = "halo",
                 **kwargs):
        if kwargs.get("cov") is not None:
            raise NotImplementedError("ShardedSeqNNGP runs the built-in covariance kinds; a callable cov(a, b) "
                                      "chain runs on one GPU (SeqNNGP(cov=...))")
        super().__init__(*args, **kwargs)
        inited = dist.is_available() and dist.is_initialized()
        self.rank = int(rank if rank is not None else (dist.get_rank(group) if inited else 0))
        self.world = int(world if world is not None else (dist.get_world_size(group) if inited else 1))
        self.group = group
        self.collective = bool(collective) if collective is not None else inited
        if self.world > 1 and not self.collective:
            raise ValueError("a sharded chain over several ranks needs a torch.distributed process group")
        dev = self.device
        n, m = self.n, self.m
        self.plan = p = gibbs_shard_plan(self.nbr, self.off, self.rev_j, self.colors, self.members, self.color_off,
                                         self.world, self.rank, exchange=exchange, device=dev)
        self.lo, self.hi = p.lo, p.hi
        # the colour runs in the plan's order (boundary members first: the head of each publish slot)
        self._member_rows = _lib.gibbs_member_rows(torch.from_numpy(p.members_x).to(dev), self.off)
        self._apply_rows = torch.from_numpy(p.apply_rows).to(dev)
        self._xchg = ColourExchange(p, dev, group, active=self.collective)
        # halo sweep: the halo rows' own points appended to the coordinate table (row n + t = halo[t]),
        # and w kept in a buffer of n + n_h values whose tail receives w[halo] before each sweep
        self._halo = torch.from_numpy(p.halo).to(dev)
        self._n_h = int(p.halo.size)
        self._coords_ext = torch.cat([self.coords, self.coords[self._halo]]).contiguous()
        self._nbr_h = self.nbr[self._halo].contiguous()
        self._w_ext = torch.empty(n + self._n_h, dtype=torch.float64, device=dev)
        self._w_ext[:n].copy_(self.w)
        self.w = self._w_ext[:n]
        z = lambda *s: torch.empty(s, dtype=torch.float64, device=dev)  # noqa: E731
        self._Bh, self._Fh, self._rh, self._part_h = z(self._n_h, m), z(self._n_h), z(self._n_h), z(4)
        self._ws_own = _lib.bf_workspace(self.hi - self.lo, m, self.algo, dev, kind=self.kind,
                                         dim=self.coords.shape[1])
        self._ws_h = _lib.bf_workspace(max(self._n_h, 1), m, self.algo, dev, kind=self.kind, dim=self.coords.shape[1])
        self._stats_ws = None
        self._L = _lib.load()
        # HIP graphs of the colour loop: over RCCL only (a gloo collective cannot be captured)
        backend = dist.get_backend(group) if self.collective else None
        self._use_graphs = bool(graphs) if graphs is not None else backend == "nccl"
        if self._use_graphs and backend not in (None, "nccl"):
            raise ValueError(f"graphs=True needs the nccl (RCCL) backend or no group, not {backend!r}")
        self._var = torch.empty(2, dtype=torch.float64, device=dev)  # (sigma2, tau2) for the captured steps
        self._graphs, self._graph_seen, self._coll_per_range = {}, set(), {}

    # ------------------------------------------------------------------ sharded pieces
    def _gather_rows(self, t: torch.Tensor) -> torch.Tensor:
        """The full (n,) vector from every rank's own rows (exact: each row comes from its owner)."""
        if not self.collective:
            return t
        b = self.plan.bounds
        size = int(np.max(np.diff(b)))
        send = torch.zeros(size, dtype=t.dtype, device=t.device)
        send[: self.hi - self.lo].copy_(t[self.lo:self.hi])
        recv = torch.empty(size * self.world, dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(recv, send, group=self.group)
        g = recv.view(self.world, size)
        return torch.cat([g[r, : int(b[r + 1] - b[r])] for r in range(self.world)])

    def _fold_rows(self, local: torch.Tensor) -> np.ndarray:
        """All-gather a small per-rank vector and sum it in rank order on the host."""
        if not self.collective:
            return local.cpu().numpy()
        g = torch.empty((self.world,) + tuple(local.shape), dtype=local.dtype, device=local.device)
        dist.all_gather_into_tensor(g, local.reshape((1,) + tuple(local.shape)), group=self.group)
        rows = g.cpu().numpy()
        acc = rows[0].copy()
        for r in range(1, self.world):
            acc += rows[r]
        return acc

    def _propose(self, phi):
        lo, hi, n = self.lo, self.hi, self.n
        torch.ops.nngp.bf_sweep_out(self.coords, self.nbr[lo:hi], None, lo, self._kind_code, 1.0, float(phi), 0.0,
                                    self.w, self._B2[lo:hi], self._Ft2[lo:hi], self._r2[lo:hi], self._part,
                                    self._ws_own, self._algo_code, self._nu_arg)
        if self._n_h:
            torch.index_select(self.w, 0, self._halo, out=self._w_ext[n:])
            torch.ops.nngp.bf_sweep_out(self._coords_ext, self._nbr_h, None, n, self._kind_code, 1.0, float(phi), 0.0,
                                        self._w_ext, self._Bh, self._Fh, self._rh, self._part_h, self._ws_h,
                                        self._algo_code, self._nu_arg)
            self._B2.index_copy_(0, self._halo, self._Bh)
            self._Ft2.index_copy_(0, self._halo, self._Fh)
            self._r2.index_copy_(0, self._halo, self._rh)
        p = combine_partials(self._part, self.world, self.group, force=self.collective)
        return p.cpu().numpy()

    def _prepare(self):
        self._prep = _lib.gibbs_prepare_range(self.B, self.Ft, self.off, self.rev_j, self.rev_k, self.lo, self.hi,
                                              prep=self._prep)

    def _stats(self):
        lo, hi = self.lo, self.hi
        nw = None if self.noise_w is None else self.noise_w[lo:hi]
        if self._stats_ws is None:
            self._stats_ws = _lib._workspace(self._L.nngp_gibbs_stats_workspace_bytes(max(hi - lo, 1), self.p),
                                             self.device)
        st = _lib.gibbs_stats(self.r[lo:hi], self.Ft[lo:hi], self.yres[lo:hi], self.y[lo:hi], self.X[lo:hi],
                              self.w[lo:hi], out=self._stats_buf, workspace=self._stats_ws, noise_w=nw)
        return self._fold_rows(st)

    def _sweep_colours(self, c0, c1):
        """Colour steps c0..c1-1: own members, one all-gather, replay of the foreign replicas.

        Over RCCL the loop is captured once per (colour range, current B / r buffers) into a HIP
        graph and replayed: issuing a colour's three operations from the host costs ~18 us (the
        collective's enqueue dominates), more than the colour's GPU work at N = 1e6 per GPU.  The
        captured launches read sigma2 / tau2 from device memory (nngp_gibbs_w_color_dev), written
        before each replay; the normals come from ``_z`` (filled each iteration)."""
        if c1 <= c0:
            return
        if not self._use_graphs:
            self._colour_loop(c0, c1, graph=False)
            return
        self._var[0].fill_(self.sigma2)
        self._var[1].fill_(self.tau2)
        key = (c0, c1, self.B.data_ptr(), self.r.data_ptr(), self._prep.data_ptr())
        gr = self._graphs.get(key)
        if gr is None:
            if key not in self._graph_seen:  # first use: eager (communicators and buffers settle)
                self._graph_seen.add(key)
                self._colour_loop(c0, c1, graph=True)
                return
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr):
                self._colour_loop(c0, c1, graph=True)
            self._graphs[key] = gr
        gr.replay()
        self._xchg.n_collectives += self._coll_per_range.setdefault((c0, c1), int(
            sum(1 for c in range(c0, c1) if self.plan.bmax[c] > 0)) if self._xchg.active else 0)

    def _colour_loop(self, c0, c1, graph):
        L, p, x = self._L, self.plan, self._xchg
        stream = torch.cuda.current_stream(self.device).cuda_stream
        mr, ap = self._member_rows.data_ptr(), self._apply_rows.data_ptr()
        prep, yres, w, r = self._prep.data_ptr(), self.yres.data_ptr(), self.w.data_ptr(), self.r.data_ptr()
        nw = None if self.noise_w is None else self.noise_w.data_ptr()
        rev_j, rev_k, B, z = self.rev_j.data_ptr(), self.rev_k.data_ptr(), self.B.data_ptr(), self._z.data_ptr()
        send, recv, var = x.send.data_ptr(), x.recv.data_ptr(), self._var.data_ptr()
        seed = self.seed & (2 ** 64 - 1)
        n, m = self.n, self.m
        rk = self.rank
        n0 = x.n_collectives
        for c in range(c0, c1):
            a, b = int(p.run[c, rk]), int(p.run[c, rk + 1])
            out = send + 8 * int(p.send_off[c])
            if graph:
                rc = L.nngp_gibbs_w_color_dev(mr + 16 * a, b - a, prep, n, m, var, yres, nw, w, r, rev_j, z, out,
                                              stream)
            else:
                rc = L.nngp_gibbs_w_color(mr + 16 * a, b - a, prep, n, m, self.sigma2, self.tau2, yres, nw, w, r,
                                          rev_j, z, seed, self.iteration, out, stream)
            if rc != 0:
                _lib._check(rc, "nngp_gibbs_w_color")
            x.exchange(c)
            a2, b2 = int(p.apply_off[c]), int(p.apply_off[c + 1])
            if b2 > a2:
                rc = L.nngp_gibbs_w_apply(ap + 16 * a2, b2 - a2, recv, B, n, m, w, r, rev_j, rev_k, stream)
                if rc != 0:
                    _lib._check(rc, "nngp_gibbs_w_apply")
        if graph and torch.cuda.is_current_stream_capturing():
            x.n_collectives = n0  # counted per replay instead

    # ------------------------------------------------------------------ results (gathered)
    @property
    def w_full(self) -> torch.Tensor:
        """w in storage order, every row from its owner."""
        return self._gather_rows(self.w)

    @property
    def w_nodes(self) -> torch.Tensor:
        return self.w_full[self.pos]

    @property
    def w_s(self) -> torch.Tensor:
        return self.w_full[self.pos[: self.n_s]]

    @property
    def w_t(self) -> torch.Tensor:
        return self.w_full[self.pos[self.node_of_t]]

    def _assemble(self, t):
        return self._gather_rows(t)

    def _assemble_unobserved(self, t):
        """Per-unobserved-node values, each from the rank owning the node (exact: x + 0)."""
        if not self.collective or t.numel() == 0:
            return t
        own = (self._un_nodes >= self.lo) & (self._un_nodes < self.hi)
        t = torch.where(own, t, torch.zeros_like(t))
        dist.all_reduce(t, group=self.group)
        return t

    def y_unobserved_full(self) -> torch.Tensor:
        """The current posterior-predictive draws, each from the rank that owns its node."""
        return self._assemble_unobserved(self.y_unobserved)

    def set_w(self, ws=None, wt=None):
        SeqNNGP.set_w(self, ws, wt)  # gathers w_nodes, rebinds w, reruns the (whole-field) sweep
        self._w_ext[: self.n].copy_(self.w)
        self.w = self._w_ext[: self.n]

    def save(self, path) -> None:
        """Every rank calls it; rank 0 writes the gathered state (a :class:`SeqNNGP` checkpoint)."""
        w_full, r_full = self._gather_rows(self.w), self._gather_rows(self.r)
        y_un = self.y_unobserved_full()
        if self.rank != 0:
            return
        saved = self.w, self.r, self.y_unobserved
        self.w, self.r, self.y_unobserved = w_full, r_full, y_un
        try:
            SeqNNGP.save(self, path)
        finally:
            self.w, self.r, self.y_unobserved = saved

    def restore(self, path) -> "ShardedSeqNNGP":
        SeqNNGP.restore(self, path)  # replicated: w, r, B, F and the prep are exact on every row
        self._w_ext[: self.n].copy_(self.w)
        self.w = self._w_ext[: self.n]
        return self


__all__ = ["ShardedSeqNNGP", "GibbsShardPlan", "gibbs_shard_plan", "gibbs_boundary", "ColourExchange", "ops"]
