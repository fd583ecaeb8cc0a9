"""The tiled Gibbs sweep's plan on the host (pynngp_amd/gibbs_tiles.py, CPU tensors, no GPU).

The plan is a valid Gibbs scan when every node lies in one tile, the tiles of one launch have disjoint
footprints (each node and its children), every reverse entry's local index names its child, and the
sweep order (level, phase, colour rank) is a proper colouring of the moral graph."""
import numpy as np
import pytest
import torch

from oracle import nngp_gibbs_oracle as G
from tests.test_gibbs_host import _reverse


def off_of(nbr):
    return _reverse(nbr)[0]


def _plan(c_oracle, n, m, tile_nodes, seed, storage_perm=True, **kw):
    from pynngp_amd import _lib
    from pynngp_amd.gibbs_tiles import build_tile_plan, check_tile_plan

    rng = np.random.default_rng(seed)
    c = rng.uniform(size=(n, 2))
    nbr0 = c_oracle.c_knn_prior(c, m)
    if storage_perm:  # a spatial-ish relabelling, as SeqNNGP stores nodes (children may precede parents)
        perm = np.lexsort((c[:, 1], np.floor(c[:, 0] * 8)))
        pos = np.empty(n, np.int64)
        pos[perm] = np.arange(n)
        nbr = np.where(nbr0[perm] >= 0, pos[np.maximum(nbr0[perm], 0)], -1).astype(np.int32)
        c = c[perm]
    else:
        nbr = nbr0
    off, rev_j = _reverse(nbr)
    colors, nc = _lib.color_moral_graph(nbr, off, rev_j)
    rev_j = np.concatenate([rev_j, np.zeros(n * m - rev_j.size, np.int32)])  # allocated for n m, as on the device
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a))  # noqa: E731
    tp = build_tile_plan(t(c), t(off.astype(np.int64)), t(rev_j.astype(np.int64)), t(colors.astype(np.int64)), nc, nc,
                         tile_nodes=tile_nodes, **kw)
    check_tile_plan(tp, t(off.astype(np.int64)), t(rev_j.astype(np.int64)))
    return nbr, colors, nc, tp


@pytest.mark.parametrize("n,m,tile_nodes", [(1, 3, 16), (50, 1, 8), (600, 5, 32), (3000, 15, 256), (3000, 10, 4096)])
def test_tile_plan_invariants(c_oracle, n, m, tile_nodes):
    nbr, colors, nc, tp = _plan(c_oracle, n, m, tile_nodes, n + m)
    assert G.coloring_is_valid(nbr, tp.effective_colors)
    assert tp.effective_colors.min() == 0
    ti = tp.tinfo.numpy()
    assert (ti[:, 1] >= ti[:, 0]).all() and (ti[:, 3] - ti[:, 2] >= ti[:, 1] - ti[:, 0]).all()
    # each footprint starts with its tile's nodes, in tnodes order
    for a in range(ti.shape[0]):
        np.testing.assert_array_equal(tp.tfp[ti[a, 2]:ti[a, 2] + ti[a, 1] - ti[a, 0]].numpy(),
                                      tp.tnodes[ti[a, 0]:ti[a, 1]].numpy())
    # colour-rank offsets cover each tile's nodes, and the nodes of rank k sit in [tcoff[k], tcoff[k+1])
    tc = tp.tcoff.numpy()
    np.testing.assert_array_equal(tc[:, -1], ti[:, 1] - ti[:, 0])
    for a in range(ti.shape[0]):
        nodes = tp.tnodes[ti[a, 0]:ti[a, 1]].numpy()
        for k in range(tp.n_ranks):
            assert (colors[nodes[tc[a, k]:tc[a, k + 1]]] == k).all()
    assert sum(int(p.numel()) for p in tp.phases) == ti.shape[0]
    assert max(tp.phase_lds) <= 144 * 1024
    # steps: each inside one colour run of its tile, <= 64 members, <= ecap entries, covering the tile
    deg = np.diff(off_of(nbr))
    st = tp.tstep.numpy()
    for a in range(ti.shape[0]):
        ks = list(st[ti[a, 4]:ti[a, 5]]) + [ti[a, 1] - ti[a, 0]]
        assert ks[0] == 0 and all(x < y for x, y in zip(ks, ks[1:]))
        nodes = tp.tnodes[ti[a, 0]:ti[a, 1]].numpy()
        for x, y in zip(ks, ks[1:]):
            assert y - x <= 64 and len(set(colors[nodes[x:y]])) == 1
            assert deg[nodes[x:y]].sum() <= tp.ecap
        # colour boundaries are step boundaries
        for k in range(tp.n_ranks + 1):
            assert tc[a, k] in ks


def test_tile_plan_cuts_into_several_launches(c_oracle):
    _, _, nc, tp = _plan(c_oracle, 3000, 15, 256, 1)
    assert tp.tinfo.shape[0] >= 8
    # far fewer launches than tiles x colours; the phases of level 0 cover most nodes
    assert len(tp.phases) < 4 * 9
    ti = tp.tinfo.numpy()
    lev0 = sum(int(ti[t, 1] - ti[t, 0]) for p in tp.phases[:1] for t in p.tolist())
    assert lev0 > 0


def test_tile_plan_reference_leaves_first(c_oracle):
    """S != T: the leaf colour (update_wt) runs first inside each tile, then the reference colours."""
    from pynngp_amd.gibbs import colour_dag
    from pynngp_amd.gibbs_tiles import build_tile_plan, check_tile_plan

    rng = np.random.default_rng(5)
    s_pts, t_pts = rng.uniform(size=(400, 2)), rng.uniform(size=(900, 2))
    coords, nbr = G.reference_dag(s_pts, t_pts, 6)
    off, rev_j = _reverse(nbr)
    colors, nc, nc_ref = colour_dag(nbr, off, rev_j, 400)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a))  # noqa: E731
    tp = build_tile_plan(t(np.asarray(coords, np.float64)), t(off.astype(np.int64)), t(rev_j.astype(np.int64)),
                         t(np.asarray(colors, np.int64)), nc, nc_ref, tile_nodes=128)
    check_tile_plan(tp, t(off.astype(np.int64)), t(rev_j.astype(np.int64)))
    assert G.coloring_is_valid(nbr, tp.effective_colors)
    ti, tc = tp.tinfo.numpy(), tp.tcoff.numpy()
    for a in range(ti.shape[0]):
        nodes = tp.tnodes[ti[a, 0]:ti[a, 1]].numpy()
        assert (np.asarray(colors)[nodes[:tc[a, 1]]] == nc_ref).all()  # rank 0 = the leaves
        assert (np.asarray(colors)[nodes[tc[a, 1]:]] < nc_ref).all()


def test_tile_plan_splits_tiles_over_the_lds(c_oracle):
    """A tile whose footprint exceeds the LDS budget is cut into chunks of its nodes; the plan stays valid."""
    nbr, colors, nc, tp0 = _plan(c_oracle, 3000, 15, 4096, 9)
    lim = 64 * 1024  # (the step buffers take a fixed ~40 KB, a 3000-node tile ~48 KB more)
    assert max(tp0.phase_lds) > lim
    _, _, _, tp = _plan(c_oracle, 3000, 15, 4096, 9, lds_bytes=lim)
    assert max(tp.phase_lds) <= lim and tp.tinfo.shape[0] > tp0.tinfo.shape[0]
    assert G.coloring_is_valid(nbr, tp.effective_colors)
    with pytest.raises(ValueError, match="children alone"):
        _plan(c_oracle, 3000, 15, 1024, 9, lds_bytes=64)


def test_tile_plan_coarse_colour(c_oracle):
    """coarse="colour": the nodes above level 0 leave the tiles for one pseudo tile swept per colour, last"""
    nbr, colors, nc, tp = _plan(c_oracle, 3000, 15, 64, 11, coarse="colour")
    assert tp.coarse_tile >= 0 and tp.coarse_members is not None
    cm = tp.coarse_members.numpy()
    co = tp.coarse_color_off
    assert co[0] == 0 and co[-1] == cm.size and (np.diff(co) >= 0).all()
    for k in range(len(co) - 1):
        assert (colors[cm[co[k]:co[k + 1]]] == k).all()
    launched = np.concatenate([p.numpy() for p in tp.phases])
    assert tp.coarse_tile not in launched
    assert G.coloring_is_valid(nbr, tp.effective_colors)
    # the coarse nodes come last in the sweep order
    eff = tp.effective_colors
    rest = np.setdiff1d(np.arange(3000), cm)
    assert eff[cm].min() > eff[rest].max()


def _contiguous(c_oracle, n, m, tile_nodes, seed, **kw):
    """A plan rebuilt in its own node order (what the kernel wants: tile t's nodes are rows [n0, n1))."""
    from pynngp_amd.gibbs_tiles import build_tile_plan

    nbr0, colors0, nc, tp0 = _plan(c_oracle, n, m, tile_nodes, seed, storage_perm=False, **kw)
    c0 = np.random.default_rng(seed).uniform(size=(n, 2))
    perm = tp0.tnodes.numpy().astype(np.int64)
    pos = np.empty(n, np.int64)
    pos[perm] = np.arange(n)
    nbr = np.where(nbr0[perm] >= 0, pos[np.maximum(nbr0[perm], 0)], -1).astype(np.int32)
    off, rev_j = _reverse(nbr)
    rev_j = np.concatenate([rev_j, np.zeros(n * m - rev_j.size, np.int32)])
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a))  # noqa: E731
    tp = build_tile_plan(t(c0[perm]), t(off.astype(np.int64)), t(rev_j.astype(np.int64)),
                         t(np.asarray(colors0)[perm].astype(np.int64)), nc, nc,
                         assign=(tp0.node_tile[t(perm)], tp0.tile_level, tp0.coarse_tile), **kw)
    assert tp.contiguous
    return t(off.astype(np.int64)), tp


@pytest.mark.parametrize("coarse", ["tiles", "colour"])
def test_launch_bounds_accepts_built_plans_and_rejects_corrupt_ones(c_oracle, coarse):
    """validate_launch_bounds (run by gibbs_w_sweep_tiles once per plan) passes what build_tile_plan makes and
    refuses plans the kernel would index out of range."""
    import copy

    from pynngp_amd.gibbs_tiles import validate_launch_bounds

    n = 3000
    off, tp = _contiguous(c_oracle, n, 15, 256, 3, coarse=coarse)
    validate_launch_bounds(tp, off, n)
    with pytest.raises(ValueError, match="rows outside|do not cover"):
        validate_launch_bounds(tp, off, n - 1)

    def corrupt(fn, match):
        bad = copy.copy(tp)
        bad._launch = None
        fn(bad)
        with pytest.raises(ValueError, match=match):
            validate_launch_bounds(bad, off, n)

    t0 = int(tp.phases[0][0])

    def tfp_out(p):
        p.tfp = p.tfp.clone()
        p.tfp[int(p.tinfo[t0, 3]) - 1] = n

    corrupt(tfp_out, "footprint node ids")

    def loc_out(p):
        p.rev_loc = p.rev_loc.clone()
        r = int(p.tinfo[t0, 0])
        while int(off[r + 1]) == int(off[r]):
            r += 1
        p.rev_loc[int(off[r])] = int(p.tinfo[t0, 3] - p.tinfo[t0, 2])

    corrupt(loc_out, "local index")

    def ecap_small(p):
        p.ecap = 1

    corrupt(ecap_small, "ecap")

    def step_big(p):  # merge every step of the first tile into one
        p.tstep = p.tstep.clone()
        p.tinfo = p.tinfo.clone()
        s0 = int(p.tinfo[t0, 4])
        p.tinfo[t0, 5] = s0 + 1

    corrupt(step_big, "members|entries")

    def lds_small(p):
        p.phase_lds = [x // 2 for x in p.phase_lds]

    corrupt(lds_small, "LDS")
