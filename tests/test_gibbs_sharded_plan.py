"""CPU: the sharded single-chain Gibbs plan (pynngp_amd.gibbs_sharded).

A numpy restatement of the colour step (nngp_gibbs_w_color's arithmetic, per member in a fixed
order) and of the replay (nngp_gibbs_w_apply) runs the plan of every rank: each rank keeps its own
replicas of w and r, updates its own members, exchanges the new w per colour and replays the other
ranks' members it holds.  After a sweep every rank's replica must equal the one-process sweep BIT
FOR BIT on its replica set V (own rows, halo, parents of both) -- the property the GPU chain relies
on.  In-process for worlds 1..5, and over a real gloo group (world 2, ColourExchange's all-gather).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from pynngp_amd.gibbs_sharded import ColourExchange, gibbs_shard_plan


def _problem(n=700, m=6, seed=0, storage="sorted"):
    from oracle import nngp_oracle as O
    from pynngp_amd import _lib

    rng = np.random.default_rng(seed)
    coords = rng.uniform(0, 1, (n, 2))
    nbr0 = O.c_knn_prior(coords, m)
    # storage relabelling: sorted by x (spatial shards) or a random permutation (worst-case halos)
    perm = np.argsort(coords[:, 0], kind="stable") if storage == "sorted" else rng.permutation(n)
    pos = np.empty(n, dtype=np.int64)
    pos[perm] = np.arange(n)
    nb = nbr0[perm]
    nbr = np.where(nb >= 0, pos[np.maximum(nb, 0)], -1).astype(np.int32)
    # reverse CSR (ascending child), host
    e = np.nonzero(nbr.ravel() >= 0)[0]
    par = nbr.ravel()[e]
    o = np.lexsort((e // m, par))
    rev_j = (e[o] // m).astype(np.int32)
    rev_k = (e[o] % m).astype(np.int32)
    off = np.concatenate([[0], np.cumsum(np.bincount(par, minlength=n))]).astype(np.int32)
    colors, n_colors = _lib.color_moral_graph(nbr, off, rev_j)
    members = np.argsort(colors, kind="stable").astype(np.int32)
    color_off = np.concatenate([[0], np.cumsum(np.bincount(colors, minlength=n_colors))]).astype(np.int32)
    B = np.where(nbr >= 0, rng.normal(0, 0.3, (n, m)), 0.0)
    F = rng.uniform(0.2, 1.0, n)
    w = rng.standard_normal(n)
    r = w - np.array([sum(B[i, s] * w[nbr[i, s]] for s in range(m) if nbr[i, s] >= 0) for i in range(n)])
    yres = rng.standard_normal(n)
    z = rng.standard_normal(n)
    return dict(n=n, m=m, nbr=nbr, off=off, rev_j=rev_j, rev_k=rev_k, colors=colors, members=members,
                color_off=color_off, B=B, F=F, w=w, r=r, yres=yres, z=z, sigma2=1.3, tau2=0.4)


def _colour_member(P, i, w, r):
    """nngp_gibbs_w_color for one member (the kernel's formulas; children in reverse-list order)."""
    it2, is2 = 1.0 / P["tau2"], 1.0 / P["sigma2"]
    acc = 0.0
    Pi = 0.0
    for e in range(P["off"][i], P["off"][i + 1]):
        j = P["rev_j"][e]
        b = P["B"][j, P["rev_k"][e]]
        acc += (b / P["F"][j]) * r[j]
        Pi += b * (b / P["F"][j])
    iF = 1.0 / P["F"][i]
    prec = (iF + Pi) * is2 + it2
    lin = P["yres"][i] * it2 + is2 * ((w[i] - r[i]) * iF + (w[i] * Pi + acc))
    wn = P["z"][i] / np.sqrt(prec) + lin / prec
    dw = wn - w[i]
    w[i] = wn
    r[i] = r[i] + dw
    for e in range(P["off"][i], P["off"][i + 1]):
        j = P["rev_j"][e]
        r[j] = r[j] - P["B"][j, P["rev_k"][e]] * dw
    return wn


def _apply_member(P, i, wn, w, r):
    """nngp_gibbs_w_apply for one row."""
    dw = wn - w[i]
    for e in range(P["off"][i], P["off"][i + 1]):
        j = P["rev_j"][e]
        r[j] = r[j] - P["B"][j, P["rev_k"][e]] * dw
    r[i] = r[i] + dw
    w[i] = wn


def _single_sweep(P):
    w, r = P["w"].copy(), P["r"].copy()
    for c in range(len(P["color_off"]) - 1):
        for g in range(P["color_off"][c], P["color_off"][c + 1]):
            _colour_member(P, P["members"][g], w, r)
    return w, r


def _rank_colour(P, plan, c, w, r, send):
    a, b = plan.run[c, plan.rank], plan.run[c, plan.rank + 1]
    so = plan.send_off[c]
    for k, g in enumerate(range(a, b)):  # the plan's run order: boundary members first
        send[so + k] = _colour_member(P, plan.members_x[g], w, r)


def _rank_apply(P, plan, c, w, r, recv):
    for row in plan.apply_rows[plan.apply_off[c]:plan.apply_off[c + 1]]:
        _apply_member(P, int(row[0]), recv[int(row[3])], w, r)


@pytest.mark.parametrize("world,storage", [(1, "sorted"), (2, "sorted"), (3, "sorted"), (5, "sorted"),
                                           (3, "random")])
def test_sharded_sweep_equals_single_bitwise(world, storage):
    P = _problem(storage=storage, seed=world)
    w_ref, r_ref = _single_sweep(P)
    plans = [gibbs_shard_plan(P["nbr"], P["off"], P["rev_j"], P["colors"], P["members"], P["color_off"], world, k)
             for k in range(world)]
    for p in plans[1:]:  # every rank computes the same runs and slots
        assert np.array_equal(p.run, plans[0].run) and np.array_equal(p.maxc, plans[0].maxc)
    W = [P["w"].copy() for _ in range(world)]
    R = [P["r"].copy() for _ in range(world)]
    sends = [np.zeros(plans[0].send_off[-1] + 1) for _ in range(world)]
    recv = np.zeros(plans[0].recv_off[-1] + 1)
    for c in range(len(P["color_off"]) - 1):
        for k in range(world):
            _rank_colour(P, plans[k], c, W[k], R[k], sends[k])
        mc, ro = plans[0].bmax[c], plans[0].recv_off[c]
        for k in range(world):  # the halo all-gather: the head (bmax[c]) of each rank's slot, rank-major
            recv[ro + k * mc: ro + (k + 1) * mc] = sends[k][plans[0].send_off[c]: plans[0].send_off[c] + mc]
        for k in range(world):
            _rank_apply(P, plans[k], c, W[k], R[k], recv)
    covered = np.zeros(P["n"], dtype=int)
    for k, p in enumerate(plans):
        V = p.replica
        assert np.array_equal(W[k][V], w_ref[V]), k
        # r is exact where the chain reads it: own rows and the halo
        OH = np.concatenate([np.arange(p.lo, p.hi), p.halo]).astype(np.int64)
        assert np.array_equal(R[k][OH], r_ref[OH]), k
        covered[p.lo:p.hi] += 1
    assert np.all(covered == 1)
    if world > 1:
        assert sum(p.apply_rows.shape[0] for p in plans) > 0
        if storage == "sorted":  # spatial shards: the halo is a small part of the shard
            assert all(p.halo.size < p.hi - p.lo for p in plans)
            # the halo exchange moves the boundary only
            assert plans[0].exchange_bytes < plans[0].allgather_bytes
    # every rank's plan agrees on the boundary and the runs' order; the boundary is exactly the union of
    # the foreign parts of the replica sets
    union = np.zeros(P["n"], dtype=bool)
    for p in plans:
        assert np.array_equal(p.exported, plans[0].exported) and np.array_equal(p.members_x, plans[0].members_x)
        f = p.replica[(p.replica < p.lo) | (p.replica >= p.hi)]
        union[f] = True
    assert np.array_equal(union, plans[0].exported)
    assert np.array_equal(np.sort(plans[0].members_x), np.sort(P["members"]))


def test_plan_sources_point_at_owners():
    P = _problem(n=400, m=5, seed=7)
    world = 3
    plans = [gibbs_shard_plan(P["nbr"], P["off"], P["rev_j"], P["colors"], P["members"], P["color_off"], world, k)
             for k in range(world)]
    pos = np.empty(P["n"], dtype=np.int64)
    p0 = plans[0]
    pos[p0.members_x] = np.arange(P["n"])
    for p in plans:
        for c in range(len(P["color_off"]) - 1):
            rows = p.apply_rows[p.apply_off[c]:p.apply_off[c + 1]]
            for i, e0, e1, src in rows:
                assert P["colors"][i] == c and not (p.lo <= i < p.hi)
                assert (e0, e1) == (P["off"][i], P["off"][i + 1])
                blk = src - p0.recv_off[c]
                owner, k = divmod(int(blk), int(p0.bmax[c]))
                assert plans[owner].lo <= i < plans[owner].hi
                assert pos[i] == p0.run[c, owner] + k and k < p0.bcount[c, owner]
                assert p0.exported[i]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _gloo_worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    P = _problem(n=500, m=6, seed=3)
    plan = gibbs_shard_plan(P["nbr"], P["off"], P["rev_j"], P["colors"], P["members"], P["color_off"], world, rank)
    x = ColourExchange(plan, torch.device("cpu"))
    w, r = P["w"].copy(), P["r"].copy()
    for c in range(len(P["color_off"]) - 1):
        send = x.send.numpy()
        _rank_colour(P, plan, c, w, r, send)
        x.exchange(c)
        _rank_apply(P, plan, c, w, r, x.recv.numpy())
    w_ref, r_ref = _single_sweep(P)
    V = plan.replica
    out[rank] = (bool(np.array_equal(w[V], w_ref[V])), int(x.n_collectives), int(plan.hi - plan.lo))
    dist.destroy_process_group()


def test_gloo_colour_exchange_world2():
    """The real per-colour all-gather (gloo) carries the plan's slots between two processes."""
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_gloo_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    n_col = None
    for k in range(world):
        ok, ncoll, rows = out[k]
        assert ok, k
        n_col = ncoll if n_col is None else n_col
        assert ncoll == n_col > 0
    assert out[0][2] + out[1][2] == 500


def test_plan_exchange_all_is_every_member():
    """exchange="all" (round 3's all-gather, the A/B reference): every row is exported, the gathered
    block is the whole slot, and the runs keep the colour order."""
    P = _problem(n=300, m=5, seed=9)
    p = gibbs_shard_plan(P["nbr"], P["off"], P["rev_j"], P["colors"], P["members"], P["color_off"], 3, 1,
                         exchange="all")
    assert p.exported.all() and np.array_equal(p.bmax, p.maxc) and p.exchange_bytes == p.allgather_bytes
    assert np.array_equal(p.members_x, P["members"])
    with pytest.raises(ValueError):
        gibbs_shard_plan(P["nbr"], P["off"], P["rev_j"], P["colors"], P["members"], P["color_off"], 3, 1,
                         exchange="some")
