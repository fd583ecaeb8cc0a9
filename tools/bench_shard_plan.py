"""Host setup cost of the sharded single-chain plan (gibbs_shard_plan, pynngp_amd/gibbs_sharded.py) at
config 4's size: N = 1e7 uniform points, m = 15, the Z-order storage layout, one rank's plan of a
world of 8 (every rank computes the same global boundary, then its own replica set and sources).

    python tools/bench_shard_plan.py [--n 10000000] [--m 15] [--world 8] [--out profiles/<tag>/shard_plan.json]

Runs on the CPU (the plan is host numpy, identical on every rank): the neighbour sets come from the C
oracle's exact prefix kd-tree search, the colouring from the library's host colouring
(nngp_color_moral_graph), as ShardedSeqNNGP would build them on the GPU.  Reports the plan's wall time
per rank and the exchange volume per sweep (halo exchange vs an all-gather of every member).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def morton(coords, bits=16):
    q = np.minimum((coords * (1 << bits)).astype(np.uint64), (1 << bits) - 1)
    code = np.zeros(coords.shape[0], dtype=np.uint64)
    for b in range(bits):
        code |= ((q[:, 0] >> np.uint64(b)) & np.uint64(1)) << np.uint64(2 * b)
        code |= ((q[:, 1] >> np.uint64(b)) & np.uint64(1)) << np.uint64(2 * b + 1)
    return code


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--m", type=int, default=15)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--out", default=None)
    ap.add_argument("--gpu", action="store_true",
                    help="the round-5 device path: SeqNNGP's whole setup (kNN, Z-order, reverse lists, the device "
                         "colouring, the pair plan) and the shard plan on the GPU, timed")
    a = ap.parse_args()
    if a.gpu:
        return main_gpu(a)
    from oracle import nngp_oracle as O
    from pynngp_amd import _lib
    from pynngp_amd.gibbs_sharded import gibbs_shard_plan

    t = {}
    rng = np.random.default_rng(2)
    coords = rng.uniform(0, 1, (a.n, 2))
    t0 = time.perf_counter()
    nbr0 = O.c_knn_prior_prefix_kdtree(coords, a.m)
    t["knn_cpu_s"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    perm = np.argsort(morton(coords), kind="stable")  # storage slot p holds input location perm[p]
    pos = np.empty(a.n, dtype=np.int64)
    pos[perm] = np.arange(a.n)
    # the colouring runs in input order (as SeqNNGP colours it: 32 colours at m = 15, where a scan in
    # storage order needs ~75), then moves with the rows into storage order
    e_in = np.flatnonzero(nbr0.ravel() >= 0)
    par_in = nbr0.ravel()[e_in]
    o_in = np.lexsort((e_in // a.m, par_in))
    off_in = np.concatenate([[0], np.cumsum(np.bincount(par_in, minlength=a.n))]).astype(np.int32)
    colors_in, n_colors = _lib.color_moral_graph(nbr0, off_in, (e_in[o_in] // a.m).astype(np.int32))
    del e_in, par_in, o_in, off_in
    nb = nbr0[perm]
    del nbr0
    nbr = np.where(nb >= 0, pos[np.maximum(nb, 0)], -1).astype(np.int32)
    del nb
    e = np.flatnonzero(nbr.ravel() >= 0)
    par = nbr.ravel()[e]
    o = np.lexsort((e // a.m, par))
    rev_j = (e[o] // a.m).astype(np.int32)
    off = np.concatenate([[0], np.cumsum(np.bincount(par, minlength=a.n))]).astype(np.int32)
    del e, par, o
    colors = colors_in[perm]
    members = np.argsort(colors, kind="stable").astype(np.int32)
    color_off = np.concatenate([[0], np.cumsum(np.bincount(colors, minlength=n_colors))]).astype(np.int32)
    t["dag_and_colouring_s"] = time.perf_counter() - t0
    res = {"n": a.n, "m": a.m, "world": a.world, "n_colors": int(n_colors), "ranks": []}
    for rank in (0, a.world // 2, a.world - 1):
        t0 = time.perf_counter()
        p = gibbs_shard_plan(nbr, off, rev_j, colors, members, color_off, a.world, rank)
        el = time.perf_counter() - t0
        res["ranks"].append({"rank": rank, "plan_s": el, "own_rows": p.hi - p.lo, "halo": int(p.halo.size),
                             "replica": int(p.replica.size), "apply_rows": int(p.apply_rows.shape[0]),
                             "exchange_bytes_per_sweep": p.exchange_bytes,
                             "allgather_bytes_per_sweep": p.allgather_bytes,
                             "boundary_rows_all_ranks": int(p.exported.sum())})
        print(json.dumps(res["ranks"][-1]), flush=True)
    res.update(t)
    res["host"] = {"cpus": os.cpu_count()}
    print(json.dumps(res))
    if a.out:
        os.makedirs(os.path.dirname(a.out), exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


def main_gpu(a):
    import torch

    from pynngp_amd import SeqNNGP
    from pynngp_amd.gibbs_sharded import gibbs_shard_plan

    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(2)
    coords = rng.uniform(0, 1, (a.n, 2))
    y = np.sin(6 * coords[:, 0]) + 0.3 * rng.standard_normal(a.n)
    torch.ones(1, device=dev).sum().item()  # context
    res = {"n": a.n, "m": a.m, "world": a.world, "device": torch.cuda.get_device_name(0), "ranks": []}
    for rep in range(2):  # the first pays one-time library / allocator warm-up
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        s = SeqNNGP(coords, y, m=a.m, sigma2=1.0, tau2=0.1, phi=30.0, device=dev)
        torch.cuda.synchronize()
        res[f"seqnngp_setup_s_{rep}"] = time.perf_counter() - t0
        res["n_colors"] = int(s.n_colors)
        if rep == 0:
            del s
    for rank in (0, a.world // 2, a.world - 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        p = gibbs_shard_plan(s.nbr, s.off, s.rev_j, s.colors, s.members, s.color_off, a.world, rank, device=dev)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        res["ranks"].append({"rank": rank, "plan_s": el, "own_rows": p.hi - p.lo, "halo": int(p.halo.size),
                             "replica": int(p.replica.size), "exchange_bytes_per_sweep": p.exchange_bytes,
                             "allgather_bytes_per_sweep": p.allgather_bytes})
        print(json.dumps(res["ranks"][-1]), flush=True)
    print(json.dumps(res))
    if a.out:
        os.makedirs(os.path.dirname(a.out), exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
