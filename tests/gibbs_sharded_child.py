"""Child process of tests/test_gpu_gibbs_sharded.py: one rank of a sharded Gibbs chain
(pynngp_amd.ShardedSeqNNGP) on cuda:0.  RANK / WORLD_SIZE / MASTER_* from the environment;
argv: backend ("nccl" for a one-rank RCCL group, "gloo" to rehearse several ranks on one GPU),
output path (.npz, written by rank 0), iterations, exchange ("halo", default, or "all")."""
import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pynngp_amd import ShardedSeqNNGP, _lib  # noqa: E402


def problem(n=20000, seed=5):
    rng = np.random.default_rng(seed)
    t = rng.uniform(0, 1, (n, 2))
    X = np.column_stack([np.ones(n), rng.standard_normal(n)])
    y = X @ np.array([1.0, -0.5]) + rng.standard_normal(n) * 0.7
    y[rng.choice(n, 50, replace=False)] = np.nan  # some unobserved responses
    return t, y, X


KW = dict(m=10, kind="exponential", sigma2=1.0, tau2=0.2, phi=8.0, seed=17)


def main():
    backend, out, iters = sys.argv[1], sys.argv[2], int(sys.argv[3])
    exchange = sys.argv[4] if len(sys.argv) > 4 else "halo"
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=dev)
    else:
        dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    t, y, X = problem()
    g = ShardedSeqNNGP(t, y, X, device=dev, exchange=exchange, **KW)
    assert g.collective and g.world == world and g.rank == rank
    # one w sweep at the initial hyperparameters (Philox normals of sweep 0)
    _lib.gibbs_normals(g._z, g.seed, 0)
    g.update_wt()
    g.update_ws()
    w_sweep = g.w_nodes.cpu().numpy()
    res = g.sample(iters)
    w_final = g.w_nodes.cpu().numpy()
    y_un = g.y_unobserved_full().cpu().numpy()
    torch.cuda.synchronize()
    if rank == 0:
        np.savez(out, w_sweep=w_sweep, w_final=w_final, y_un=y_un, beta=res["beta"], sigma2=res["sigma2"],
                 tau2=res["tau2"], phi=res["phi"],
                 meta=np.array(json.dumps({"world": world, "n_collectives": g._xchg.n_collectives,
                                           "exchange_bytes": g.plan.exchange_bytes,
                                           "allgather_bytes": g.plan.allgather_bytes,
                                           "halo": int(g._n_h), "apply": int(g._apply_rows.shape[0]),
                                           "rows": [g.lo, g.hi], "n_accept": g.n_accept,
                                           "graphs": len(g._graphs), "iterations": g.iteration})))
    dist.barrier()
    dist.destroy_process_group()
    print("GIBBS_SHARDED_OK", rank)


if __name__ == "__main__":
    main()
