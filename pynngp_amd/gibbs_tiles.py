"""Tiled colour sweep of the Gibbs sampler's latent field (SeqNNGP's w update, round 6).

The reference names the update (``update_ws`` / ``update_wt`` in ``oneSample``, pyNNGP/nngp.py:98-101)
but never defines it; SeqNNGP draws every node's full conditional colour by colour (gibbs.hip).  One
launch per colour re-reads the residual vector r from beyond the XCDs' L2s every time (~44 MB per
colour launch at N = 1e6, profiles/r06e): 32 launches move ~1.5 GB per iteration for an 8 MB state.

A tiled sweep keeps r in LDS.  The nodes are cut into spatial tiles (grid cells); a tile's footprint is
the set of r entries its nodes' updates touch (each node and its children: a node's conditional reads
r_i and its children's r_j and writes them and w_i).  Tiles whose footprints are disjoint can be swept
concurrently, each by one workgroup holding its footprint's r (and its nodes' w) in LDS and running
every colour of its nodes in order with a block barrier between colours; a greedy colouring of the
tiles' overlap graph gives the phases (one launch each).  Nodes whose children are far (the first
points of a generation-ordered field, whose prior neighbour sets are sparse) would make the footprints
overlap widely: they go to coarser levels (cells 4x wider each level) swept after the finer ones, or
(coarse="colour", SeqNNGP's default) one launch per colour after the tiles.

Measured (profiles/r06i-r06r): the tiled sweep moves a third of the colour sweep's L2 bytes
and takes the same time -- both are chains of dependent steps (a tile's ~30 steps in series, ~1.45 us each
with their loads removed; a colour launch ~15 us), not byte-bound -- so SeqNNGP keeps the colour sweep by
default and this one is opt-in (``SeqNNGP(sweep="tiled")``).

Any order in which every node is drawn once from its full conditional given the current values, with
no two dependent nodes drawn concurrently, is a valid Gibbs scan: here the order is (level, phase,
colour), and the dense oracle reproduces it as a colouring (``TilePlan.effective_colors``).
"""
from dataclasses import dataclass
from typing import List

import numpy as np
import torch

# LDS the kernel may use per workgroup (gibbs.hip gibbs_tile_phase)
TILE_LDS_BYTES = 144 * 1024
# a step of the kernel: <= 64 members of one colour, whose reverse entries start within STEP_ENTRIES of the
# step's first (so a step holds at most STEP_ENTRIES + the largest child count entries: the plan's ecap)
STEP_MEMBERS = 64
STEP_ENTRIES = 768
MAX_ECAP = 2048  # the kernel's staging registers cover 2 x 1024 entries per step


def tile_lds_bytes(n_footprint, n_nodes, n_steps, ecap):
    """gibbs_tile_phase's LDS for one tile: the footprint's r and the rows' new w (8 B each), two step
    buffers (64 members x 6 doubles, ecap x (B, B / F, local index)), the tile's entry offsets (4 B per row
    + 1) and its step starts (4 B per step + 1), 16-B aligned"""
    ecp = ecap + 1  # (+ a dummy slot)
    b = (8 * n_footprint + 8 * n_nodes + 2 * (8 * (6 * STEP_MEMBERS + 1 + 2 * ecp) + 4 * ecp) + 4 * (n_nodes + 1)
         + 4 * (n_steps + 1))
    return (b + 15) // 16 * 16


@dataclass
class TilePlan:
    tnodes: torch.Tensor      # int32 (n,): nodes grouped by (level, phase, tile), colour rank inside a tile
    tfp: torch.Tensor         # int32: per tile its footprint (its nodes in tnodes order, then the halo)
    tinfo: torch.Tensor       # int32 (n_tiles, 8): node range [n0, n1) in tnodes, footprint range [f0, f1) in
    # tfp, step range [s0, s1) in tstep, 0, 0
    tcoff: torch.Tensor       # int32 (n_tiles, n_ranks + 1): colour-rank offsets inside each tile (from n0)
    rev_loc: torch.Tensor     # int32 (n m,): footprint-local index of reverse entry e's child in its parent's tile
    phases: List[torch.Tensor]  # per launch (level, phase order): int32 tile ids
    phase_lds: List[int]      # dynamic LDS bytes per launch (its largest footprint + tile)
    n_ranks: int
    levels: int
    effective_colors: np.ndarray  # int64 (n,) storage order: the sweep's order as a colouring
    tstep: torch.Tensor = None       # int32: per tile its steps' first members (tile-local), in order
    ecap: int = 0                    # the most reverse entries of one step
    coarse_tile: int = -1            # coarse="colour": the pseudo tile of the nodes above level 0 (not launched)
    coarse_members: torch.Tensor = None  # ... its nodes by colour rank (int32), swept after the tiles
    coarse_color_off: np.ndarray = None  # ... host int32 colour-rank offsets into coarse_members
    node_tile: torch.Tensor = None   # long (n,): each node's tile (storage order)
    tile_level: torch.Tensor = None  # long (n_tiles,)
    contiguous: bool = False  # tnodes is the identity: tile t's nodes are storage rows [n0, n1) (the kernel's
    # requirement: contiguous_plan(); SeqNNGP stores its nodes in the plan's order)

    def launch_arrays(self):
        """(all phases' tile ids on the device, host int32 phase offsets, host int32 LDS bytes per phase)"""
        if getattr(self, "_launch", None) is None:
            tiles = torch.cat(self.phases) if self.phases else torch.zeros(0, dtype=torch.int32,
                                                                          device=self.tnodes.device)
            poff = np.concatenate([[0], np.cumsum([int(p.numel()) for p in self.phases])]).astype(np.int32)
            self._launch = (tiles.contiguous(), poff, np.asarray(self.phase_lds, dtype=np.int32))
        return self._launch


def colour_rank(colors: torch.Tensor, n_colors: int, n_colors_ref: int) -> torch.Tensor:
    """The order of the colours in a sweep: the leaf colour (data locations outside S, ``update_wt``) first,
    then the reference colours 0.. (``update_ws``) -- SeqNNGP.step's order; S = T: the colours as they are."""
    if n_colors > n_colors_ref:
        return torch.where(colors == n_colors_ref, torch.zeros_like(colors), colors + 1)
    return colors.clone()


def _footprints(tile_of, owner, child, n):
    """(tile, node) pairs, unique and sorted: every node of a tile and every child of those nodes"""
    fp_t = torch.cat([tile_of, tile_of[owner]])
    fp_x = torch.cat([torch.arange(n, device=tile_of.device), child])
    fkey = torch.unique(fp_t * n + fp_x)
    return fkey // n, fkey % n


def _tiling(coords, dmax, tile_nodes, max_levels):
    """Grid cells of about tile_nodes nodes; a node whose farthest child lies beyond half a cell goes to
    the next level (cells 4x wider).  Returns (tile of each node, numbered in (level, cell) order; the
    node's level; the number of levels)."""
    dev = coords.device
    n, D = coords.shape
    lo = coords.min(0).values
    span = (coords.max(0).values - lo).clamp(min=1e-300)
    vol = float(span.prod())
    w = (vol * tile_nodes / max(n, 1)) ** (1.0 / D) if vol > 0 else float(span.max())
    w = max(w, float(span.max()) * 1e-6)
    level = torch.full((n,), -1, dtype=torch.long, device=dev)
    cell = torch.zeros(n, dtype=torch.long, device=dev)
    lev = 0
    while True:
        left = level < 0
        if not bool(left.any()):
            break
        last = lev == max_levels - 1 or w >= 2.0 * float(span.max())
        sel = left if last else left & (2.0 * dmax <= w)
        if bool(sel.any()):
            k = torch.floor((coords[sel] - lo) / w).long().clamp(min=0)
            ncell = torch.clamp(torch.floor(span / w).long() + 1, min=1)
            cid = torch.zeros(int(sel.sum()), dtype=torch.long, device=dev)
            for a in range(D):
                cid = cid * int(ncell[a]) + k[:, a]
            cell[sel] = cid
            level[sel] = lev
        lev += 1
        w *= 4.0
    key = level * (int(cell.max()) + 1 if n else 1) + cell
    tile_of = torch.unique(key, return_inverse=True)[1] if n else key
    return tile_of, level, lev


def build_tile_plan(coords: torch.Tensor, off: torch.Tensor, rev_j: torch.Tensor, colors: torch.Tensor,
                    n_colors: int, n_colors_ref: int, tile_nodes: int = 2048, max_levels: int = 8,
                    lds_bytes: int = TILE_LDS_BYTES, assign=None, coarse: str = "tiles") -> TilePlan:
    """Tiles, phases and local indices for the tiled colour sweep (storage-order arrays on the device).

    coords (n, d); off (n + 1,), rev_j: the reverse neighbour lists (children, the first off[n] entries);
    colors (n,) long.  coarse="colour": the nodes above level 0 are not tiled but swept after the tiles, one
    launch per colour (the per-colour kernel; their tiles' serial colour chains cost more than the launches)."""
    if coarse not in ("tiles", "colour"):
        raise ValueError(f"coarse must be 'tiles' or 'colour' (got {coarse!r})")
    dev = coords.device
    n, D = coords.shape
    off = off.long()
    child = rev_j[:int(off[-1])].long()  # (the reverse lists may be allocated for n m entries)
    counts = off[1:] - off[:-1]
    owner = torch.repeat_interleave(torch.arange(n, device=dev), counts)  # reverse entry -> parent
    ne = int(child.numel())
    dist = (coords[owner] - coords[child]).norm(dim=1) if ne else torch.zeros(0, dtype=coords.dtype, device=dev)
    dmax = torch.zeros(n, dtype=coords.dtype, device=dev)
    if ne:
        dmax.scatter_reduce_(0, owner, dist, reduce="amax")
    rank = colour_rank(colors.long(), n_colors, n_colors_ref)
    n_ranks = int(max(n_colors, 1))
    ar = torch.arange(n, device=dev)
    coarse_tile = -1
    maxdeg = int(counts.max()) if n else 0
    ecap_bound = STEP_ENTRIES + maxdeg
    if ecap_bound > MAX_ECAP:
        raise ValueError(f"a node with {maxdeg} children: the tiled sweep takes at most {MAX_ECAP - STEP_ENTRIES}")
    if assign is not None:
        # the tiling of an earlier plan of the same field under another labelling (SeqNNGP relabels its
        # storage into the plan's node order, then rebuilds the plan there: tnodes = identity)
        tile_of, tile_level = assign[0].long(), assign[1].long()
        coarse_tile = int(assign[2]) if len(assign) > 2 else -1
        n_tiles = int(tile_level.numel())
        levels = int(tile_level.max()) + 1 if n_tiles else 0
        fp_t, fp_x = _footprints(tile_of, owner, child, n)
    else:
        tile_of, level, levels = _tiling(coords, dmax, tile_nodes, max_levels)
        cmask = level >= 1 if coarse == "colour" else torch.zeros(n, dtype=torch.bool, device=dev)
        if bool(cmask.any()):  # every coarse node in one pseudo tile (level 1), swept per colour
            tile_of = tile_of.clone()
            tile_of[cmask] = int(tile_of[~cmask].max()) + 1 if bool((~cmask).any()) else 0
            tile_of = torch.unique(tile_of, return_inverse=True)[1]
            level = torch.where(cmask, torch.ones_like(level), level)
            levels = 2
        # A tile whose footprint exceeds the LDS is cut into chunks of its nodes in storage order: the
        # early nodes of a generation-ordered field have ~m ln(n / i) children each, so a coarse cell of a
        # few hundred of them can reach 20k footprint entries (N = 1e6, m = 15).  Any node partition is a
        # valid tiling; the overlap graph decides the phases.
        cap = lds_bytes
        for _ in range(32):
            n_tiles = int(tile_of.max()) + 1 if n else 0
            fp_t, fp_x = _footprints(tile_of, owner, child, n)
            nn_t = torch.bincount(tile_of, minlength=n_tiles)
            need = tile_lds_bytes(torch.bincount(fp_t, minlength=n_tiles), nn_t, nn_t + n_ranks, ecap_bound)
            coarse_tile = int(tile_of[cmask][0]) if bool(cmask.any()) else -1
            if coarse_tile >= 0:
                need[coarse_tile] = 0  # (not run by the tile kernel)
            if n == 0 or int(need.max()) <= cap:
                break
            parts = torch.clamp((need * 5 + 4 * cap - 1) // (4 * cap), min=1)  # ~80% full chunks
            if bool((nn_t[need > cap] == 1).any()):
                raise ValueError(f"a node's children alone need {int(need.max())} B of LDS (> {lds_bytes})")
            srt = torch.argsort(tile_of * n + ar)
            first = torch.zeros(n_tiles, dtype=torch.long, device=dev)
            first.scatter_reduce_(0, tile_of[srt], ar, reduce="amin", include_self=False)
            pos = torch.empty(n, dtype=torch.long, device=dev)
            pos[srt] = ar - first[tile_of[srt]]
            sub = pos * parts[tile_of] // nn_t[tile_of]
            tile_of = torch.unique(tile_of * int(parts.max()) + sub, return_inverse=True)[1]
        else:
            raise ValueError("tile plan: footprints do not fit in LDS after splitting")
        tile_level = torch.zeros(n_tiles, dtype=torch.long, device=dev)
        tile_level[tile_of] = level
    # tile overlap graph: tiles of ONE level sharing a footprint node (levels run one after another)
    order = torch.argsort(fp_x * n_tiles + fp_t)
    xs, ts = fp_x[order], fp_t[order]
    same = (xs[1:] == xs[:-1]) & (tile_level[ts[1:]] == tile_level[ts[:-1]])
    # all pairs within a run of equal x: runs are short (a node lies in a few footprints); expand by offset
    pairs = []
    run_start = torch.ones(xs.numel(), dtype=torch.bool, device=dev)
    run_start[1:] = ~same
    rid = torch.cumsum(run_start.long(), 0) - 1
    rs = torch.nonzero(run_start).flatten()
    pos = torch.arange(xs.numel(), device=dev) - rs[rid]
    maxrun = int(pos.max()) + 1 if xs.numel() else 0
    for dlt in range(1, maxrun):
        ok = torch.nonzero(pos >= dlt).flatten()
        pairs.append(torch.stack([ts[ok - dlt], ts[ok]], 1))
    adj = torch.unique(torch.sort(torch.cat(pairs), 1).values, dim=0).cpu().numpy() if pairs else \
        np.zeros((0, 2), np.int64)
    nbrs = [[] for _ in range(n_tiles)]
    for a, b in adj:
        if a != b:
            nbrs[a].append(b)
            nbrs[b].append(a)
    # greedy colouring per level, tiles in (level, cell) order
    tphase = np.full(n_tiles, -1, dtype=np.int64)
    for t in range(n_tiles):
        used = {tphase[u] for u in nbrs[t] if tphase[u] >= 0}
        c = 0
        while c in used:
            c += 1
        tphase[t] = c

    # node order: (level, phase, tile, colour rank, storage index)
    tph = torch.from_numpy(tphase).to(dev)
    n_ph = int(tphase.max()) + 1 if n_tiles else 0
    launch_of_tile = tile_level * max(n_ph, 1) + tph  # (level, phase) launch key
    nkey = ((launch_of_tile[tile_of] * n_tiles + tile_of) * (n_ranks + 1) + rank) * n + torch.arange(n, device=dev)
    tnodes = torch.argsort(nkey)
    tile_sorted = tile_of[tnodes]
    # node ranges per tile (tiles appear in launch order; record each tile's [n0, n1))
    n0 = torch.full((n_tiles,), n, dtype=torch.long, device=dev)
    n1 = torch.zeros(n_tiles, dtype=torch.long, device=dev)
    idx = torch.arange(n, device=dev)
    n0.scatter_reduce_(0, tile_sorted, idx, reduce="amin")
    n1.scatter_reduce_(0, tile_sorted, idx + 1, reduce="amax")
    pos_in_tile = torch.empty(n, dtype=torch.long, device=dev)
    pos_in_tile[tnodes] = idx - n0[tile_sorted]
    # colour-rank offsets inside each tile
    rk_sorted = rank[tnodes]
    tco = torch.zeros((n_tiles, n_ranks + 1), dtype=torch.long, device=dev)
    cnt = torch.zeros((n_tiles, n_ranks), dtype=torch.long, device=dev)
    cnt.index_put_((tile_sorted, rk_sorted), torch.ones(n, dtype=torch.long, device=dev), accumulate=True)
    tco[:, 1:] = torch.cumsum(cnt, 1)
    # steps: within each (tile, colour rank) run of tnodes, chunks of <= STEP_MEMBERS members whose
    # entries start within STEP_ENTRIES of the chunk's first (both indices only grow along a run)
    deg_s = counts[tnodes]
    run_key = tile_sorted * (n_ranks + 1) + rk_sorted
    run_start = torch.ones(n, dtype=torch.bool, device=dev)
    if n:
        run_start[1:] = run_key[1:] != run_key[:-1]
    rid = torch.cumsum(run_start.long(), 0) - 1
    rs = torch.nonzero(run_start).flatten()
    idx_in_run = idx - rs[rid]
    cum = torch.cumsum(deg_s, 0) - deg_s  # entries before node q (exclusive, over all of tnodes)
    cum_in_run = cum - cum[rs[rid]]
    ca, cb = idx_in_run // STEP_MEMBERS, cum_in_run // STEP_ENTRIES
    sstart = run_start.clone()
    if n:
        sstart[1:] |= (ca[1:] != ca[:-1]) | (cb[1:] != cb[:-1])
    sq = torch.nonzero(sstart).flatten()  # step starts (positions in tnodes), tile by tile in launch order
    st_tile = tile_sorted[sq]
    tstep = sq - n0[st_tile]
    nst = torch.bincount(st_tile, minlength=n_tiles)
    s0 = torch.zeros(n_tiles, dtype=torch.long, device=dev)
    s0[torch.argsort(n0)] = torch.cumsum(nst[torch.argsort(n0)], 0) - nst[torch.argsort(n0)]
    s1 = s0 + nst
    # entries per step (tiles are back to back in tnodes: a tile's last step ends at the next tile's first)
    send = torch.cat([sq[1:], torch.tensor([n], device=dev)]) if n else sq
    step_entries = (cum[send - 1] + deg_s[send - 1] - cum[sq]) if n else sq
    ecap = int(step_entries.max()) if n else 0
    assert ecap <= ecap_bound

    # footprints: the tile's nodes first (tnodes order), then the halo (footprint nodes outside the tile)
    in_tile = tile_of[fp_x] == fp_t
    halo_t, halo_x = fp_t[~in_tile], fp_x[~in_tile]
    nn = n1 - n0
    nh = torch.bincount(halo_t, minlength=n_tiles)
    fsz = nn + nh
    f0 = torch.zeros(n_tiles, dtype=torch.long, device=dev)
    # footprint storage in launch order of the tiles (the same order as their node ranges)
    tord = torch.argsort(n0)
    f0[tord] = torch.cumsum(fsz[tord], 0) - fsz[tord]
    f1 = f0 + fsz
    tfp = torch.empty(int(fsz.sum()), dtype=torch.long, device=dev)
    tfp[f0[tile_sorted] + pos_in_tile[tnodes]] = tnodes
    hord = torch.argsort(halo_t * n + halo_x)
    halo_t, halo_x = halo_t[hord], halo_x[hord]
    hstart = torch.cumsum(nh, 0) - nh
    hpos = torch.arange(halo_t.numel(), device=dev) - hstart[halo_t]
    tfp[f0[halo_t] + nn[halo_t] + hpos] = halo_x
    # rev_loc: the footprint-local index of each reverse entry's child in its parent's tile
    loc_key = fp_t * n + fp_x  # sorted (fkey)
    lpos = torch.empty(fp_t.numel(), dtype=torch.long, device=dev)
    lpos[in_tile] = pos_in_tile[fp_x[in_tile]]
    hk = halo_t * n + halo_x
    hloc = nn[halo_t] + hpos
    lpos[torch.searchsorted(loc_key, hk)] = hloc
    ek = tile_of[owner] * n + child
    rev_loc = lpos[torch.searchsorted(loc_key, ek)] if ne else torch.zeros(0, dtype=torch.long, device=dev)

    # launches: per (level, phase) the tiles, in node-range order
    phases, phase_lds = [], []
    tkey_h = launch_of_tile.cpu().numpy()
    n0_h, fsz_h, nn_h, nst_h = n0.cpu().numpy(), fsz.cpu().numpy(), nn.cpu().numpy(), nst.cpu().numpy()
    coarse_members, coarse_off = None, None
    if coarse_tile >= 0:
        coarse_members = tnodes[int(n0[coarse_tile]):int(n1[coarse_tile])].to(torch.int32).contiguous()
        coarse_off = tco[coarse_tile].cpu().numpy().astype(np.int32)
        tkey_h = tkey_h.copy()
        tkey_h[coarse_tile] = -1
    for lk in np.unique(tkey_h):
        if lk < 0:
            continue
        ts_ = np.nonzero(tkey_h == lk)[0]
        ts_ = ts_[np.argsort(n0_h[ts_])]
        phases.append(torch.from_numpy(ts_.astype(np.int32)).to(dev))
        phase_lds.append(int(tile_lds_bytes(fsz_h[ts_], nn_h[ts_], nst_h[ts_], ecap).max()))
    assert not phase_lds or max(phase_lds) <= lds_bytes
    # the sweep's order as a colouring: (launch, colour rank)
    eff = (launch_of_tile[tile_of] * (n_ranks + 1) + rank).cpu().numpy()
    _, eff = np.unique(eff, return_inverse=True)
    zero = torch.zeros_like(n0)
    tinfo = torch.stack([n0, n1, f0, f1, s0, s1, zero, zero], 1).to(torch.int32).contiguous()
    return TilePlan(tnodes=tnodes.to(torch.int32).contiguous(), tfp=tfp.to(torch.int32).contiguous(), tinfo=tinfo,
                    tcoff=tco.to(torch.int32).contiguous(), rev_loc=rev_loc.to(torch.int32).contiguous(),
                    phases=phases, phase_lds=phase_lds, n_ranks=n_ranks, levels=levels,
                    effective_colors=eff.astype(np.int64), tstep=tstep.to(torch.int32).contiguous(), ecap=ecap,
                    coarse_tile=coarse_tile, coarse_members=coarse_members, coarse_color_off=coarse_off,
                    node_tile=tile_of, tile_level=tile_level,
                    contiguous=bool(torch.equal(tnodes, ar)))


def contiguous_plan(coords: torch.Tensor, nbr: torch.Tensor, colors: torch.Tensor, n_colors: int, n_colors_ref: int,
                    **kw):
    """A field relabelled into its tile plan's node order, and the plan rebuilt there (contiguous: tile t's
    nodes are rows [n0, n1), what nngp_gibbs_w_sweep_tiles wants).  Returns (perm, nbr', off', rev_j',
    rev_k', plan): new row p is old row perm[p]; nbr' in the new labels (a per-node array x moves as
    x[perm])."""
    from . import _lib

    off, rev_j, _ = _lib.reverse_neighbors(nbr)
    tp0 = build_tile_plan(coords, off, rev_j, colors, n_colors, n_colors_ref, **kw)
    perm = tp0.tnodes.long()
    pos = torch.empty_like(perm)
    pos[perm] = torch.arange(perm.numel(), device=perm.device)
    nb = nbr[perm].long()
    nbr2 = torch.where(nb >= 0, pos[nb.clamp(min=0)], -1).to(torch.int32).contiguous()
    off2, rev_j2, rev_k2 = _lib.reverse_neighbors(nbr2)
    kw.pop("assign", None)
    tp = build_tile_plan(coords[perm].contiguous(), off2, rev_j2, colors[perm], n_colors, n_colors_ref,
                         assign=(tp0.node_tile[perm], tp0.tile_level, tp0.coarse_tile), **kw)
    assert tp.contiguous
    return perm, nbr2, off2, rev_j2, rev_k2, tp


def validate_launch_bounds(tp: TilePlan, off: torch.Tensor, n: int) -> None:
    """What gibbs_tile_phase indexes without a check of its own, verified once per plan and field (the C ABI
    checks only sizes; :func:`pynngp_amd._lib.gibbs_w_sweep_tiles` calls this): the launched tiles' row,
    footprint and step ranges inside their arrays, footprint node ids in [0, n) with each footprint starting
    with its tile's rows, step starts increasing from 0 with <= STEP_MEMBERS members and <= ecap reverse
    entries each, every entry's local index inside its tile's footprint, and each launch's LDS bytes covering
    its tiles.  Raises ValueError."""
    def bad(msg):
        raise ValueError(f"tile plan does not fit the tiled sweep kernel: {msg}")

    if tp.tinfo.dtype != torch.int32 or tp.tinfo.dim() != 2 or tp.tinfo.shape[1] != 8:
        bad("tinfo must be int32 (n_tiles, 8)")
    if not 0 <= int(tp.ecap) <= MAX_ECAP:
        bad(f"ecap={tp.ecap} outside [0, {MAX_ECAP}]")
    tiles, poff, plds = tp.launch_arrays()
    if tiles.numel() == 0:
        return
    dev = tp.tinfo.device
    ar = lambda k: torch.arange(k, device=dev)  # noqa: E731
    tl = tiles.long().to(dev)
    if int(tl.min()) < 0 or int(tl.max()) >= tp.tinfo.shape[0]:
        bad("tile ids outside the plan")
    n0, n1, f0, f1, s0, s1 = tp.tinfo.long()[tl].unbind(1)[:6]
    nn, nf, S = n1 - n0, f1 - f0, s1 - s0
    if bool(((n0 < 0) | (nn < 0) | (n1 > n)).any()):
        bad("tile rows outside [0, n)")
    if bool(((f0 < 0) | (nf < nn) | (f1 > tp.tfp.numel())).any()):
        bad("footprint ranges")
    if bool(((s0 < 0) | (S < (nn > 0).long()) | (s1 > tp.tstep.numel())).any()):
        bad("step ranges")
    offl = off.long().to(dev)
    if offl.numel() != n + 1 or tp.rev_loc.numel() < int(offl[-1]):
        bad("off / rev_loc do not cover the field's reverse entries")
    fpv = tp.tfp.long()
    if fpv.numel() and bool(((fpv < 0) | (fpv >= n)).any()):
        bad("footprint node ids outside [0, n)")
    seg = lambda cnt: torch.repeat_interleave(ar(cnt.numel()), cnt)  # noqa: E731
    within = lambda cnt: ar(int(cnt.sum())) - torch.repeat_interleave(torch.cumsum(cnt, 0) - cnt, cnt)  # noqa: E731
    rt, k = seg(nn), within(nn)  # the launched rows: tile, tile-local index
    rows = n0[rt] + k
    if not torch.equal(fpv[f0[rt] + k], rows):
        bad("a footprint must start with its tile's rows")
    qt = seg(S)
    qi = s0[qt] + within(S)
    st = tp.tstep.long()
    a = st[qi]
    b = torch.where(qi == s1[qt] - 1, nn[qt], st[(qi + 1).clamp(max=max(st.numel() - 1, 0))])
    if bool(((a < 0) | (b <= a) | (b > nn[qt]) | ((qi == s0[qt]) & (a != 0))).any()):
        bad("step starts must increase from 0 inside their tile")
    if bool(((b - a) > STEP_MEMBERS).any()):
        bad(f"a step of more than {STEP_MEMBERS} members")
    if bool(((offl[n0[qt] + b] - offl[n0[qt] + a]) > int(tp.ecap)).any()):
        bad(f"a step of more than ecap={tp.ecap} reverse entries")
    cnt = offl[rows + 1] - offl[rows]
    et = torch.repeat_interleave(rt, cnt)
    loc = tp.rev_loc.long()[torch.repeat_interleave(offl[rows], cnt) + within(cnt)]
    if bool(((loc < 0) | (loc >= nf[et])).any()):
        bad("a reverse entry's local index outside its tile's footprint")
    phase = torch.repeat_interleave(ar(len(plds)), torch.as_tensor(np.diff(poff), device=dev).long())
    need = tile_lds_bytes(nf, nn, S, int(tp.ecap))
    if bool((torch.as_tensor(plds, device=dev).long()[phase] < need).any()) or int(plds.max()) > 160 * 1024:
        bad("a launch's LDS bytes do not cover its tiles (or exceed 160 KB)")


def check_tile_plan(tp: TilePlan, off: torch.Tensor, rev_j: torch.Tensor) -> None:
    """The plan's invariants (setup check): every node in exactly one tile; within a launch the tiles'
    footprints are disjoint; each reverse entry's local index names its child in its parent's footprint."""
    n = tp.tnodes.numel()
    assert torch.equal(torch.sort(tp.tnodes.long()).values, torch.arange(n, device=tp.tnodes.device))
    ti = tp.tinfo.long()
    for ph in tp.phases:
        p = ph.long()
        seg = [tp.tfp[int(ti[t, 2]):int(ti[t, 3])].long() for t in p.tolist()]
        allf = torch.cat(seg) if seg else torch.zeros(0, dtype=torch.long)
        assert allf.numel() == torch.unique(allf).numel(), "overlapping footprints in one launch"
    # entry e of parent i (tile t): tfp[f0[t] + rev_loc[e]] == rev_j[e]
    counts = (off[1:] - off[:-1]).long()
    owner = torch.repeat_interleave(torch.arange(n, device=off.device), counts)
    tile_of = torch.empty(n, dtype=torch.long, device=off.device)
    for t in range(ti.shape[0]):
        tile_of[tp.tnodes[int(ti[t, 0]):int(ti[t, 1])].long()] = t
    f0 = ti[:, 2][tile_of[owner]]
    assert torch.equal(tp.tfp.long()[f0 + tp.rev_loc.long()], rev_j[:owner.numel()].long())
