"""CPU, world_size 2 (gloo): the sharded sweep's host logic.

Contiguous shards, per-rank neighbour build for its own rows
only, and the rank-order combination of the 4-double partials must reproduce the
single-process log-likelihood.  The per-shard compute here is the C oracle
(injected; the GPU path runs the HIP kernel through the same ShardedLogLik).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from pynngp_amd.sweep import ShardedLogLik, combine_partials, shard_range


def test_shard_range_covers():
    for n in [0, 1, 7, 1000, 10_000_001]:
        for world in [1, 2, 3, 8]:
            bounds = [shard_range(n, r, world) for r in range(world)]
            assert bounds[0][0] == 0 and bounds[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(bounds[:-1], bounds[1:]))
            sizes = [hi - lo for lo, hi in bounds]
            assert max(sizes) - min(sizes) <= 1


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _oracle_build(coords, m, lo, hi):
    from oracle import nngp_oracle as O

    return torch.from_numpy(O.c_knn_prior(coords.numpy(), m, lo, hi))


def _oracle_compute(sweep, cov, values, want_bf):
    from oracle import nngp_oracle as O

    _, _, p = O.c_bf_sweep(sweep.coords.numpy(), sweep.nbr.numpy(), cov.kind, cov.theta,
                           None if values is None else values.numpy(), i0=sweep.lo)
    return torch.tensor([p[0], p[1], p[2], -1.0], dtype=torch.float64)


def _oracle_build_rows(coords, m, rows):
    from oracle import nngp_oracle as O

    full = O.c_knn_prior(coords.numpy(), m)
    return torch.from_numpy(full[rows.numpy()])


def _random_perm(coords):
    return torch.from_numpy(np.random.default_rng(99).permutation(coords.shape[0]).astype(np.int32))


def _oracle_compute_storage(sweep, cov, values, want_bf):
    """The C oracle on the relabelled (storage-order) arrays the device kernel would see."""
    from oracle import nngp_oracle as O

    _, _, p = O.c_bf_sweep(sweep._coords_sweep.numpy(), sweep._nbr_sweep.numpy(), cov.kind, cov.theta,
                           None if values is None else values.numpy(), i0=sweep.lo)
    return torch.tensor([p[0], p[1], p[2], -1.0], dtype=torch.float64)


def _worker_storage(rank, world, port, n, m, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from pynngp_amd import Covariance

    rng = np.random.default_rng(0)
    coords = torch.from_numpy(rng.uniform(size=(n, 2)))
    values = torch.from_numpy(rng.standard_normal(n))
    sweep = ShardedLogLik(coords, m, rank, world, layout="storage", build_perm=_random_perm,
                          build_nbr=_oracle_build_rows, compute=_oracle_compute_storage)
    cov = Covariance("exponential", 1.3, 9.0, 0.05)
    # pipelined exchange (throughput mode): three independent sweeps, each fully combined
    from pynngp_amd.sweep import PipelinedCombine

    assert sweep.collective  # a process group exists: even one rank exchanges through it
    pipe = PipelinedCombine(sweep, 3)
    assert pipe.active
    for k, c in enumerate([cov, cov.replace(phi=4.0), cov]):
        sweep.local_partials(c, values, out=pipe.local[k])
        pipe.exchange(k)
    res = pipe.finish()
    assert torch.equal(res[0], res[2]) and not torch.equal(res[0], res[1])
    # batched exchanges (2 sweeps per all-gather, a partial last batch): the same rows
    covs5 = [cov, cov.replace(phi=4.0), cov, cov.replace(tau2=0.2), cov.replace(phi=4.0)]
    pipe2 = PipelinedCombine(sweep, 5, batch=2)
    for k, c in enumerate(covs5):
        sweep.local_partials(c, values, out=pipe2.local[k])
        pipe2.exchange(k)
    res2 = pipe2.finish()
    assert pipe2.n_collectives == 3
    for k, c in enumerate(covs5):
        assert torch.equal(res2[k], sweep.partials(c, values)), k
    out[rank] = (sweep.loglik(cov, values), sweep.rows_input.tolist(), res[0].tolist())
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2, 3])
def test_gloo_storage_layout_matches_single(world):
    """Relabelled storage shards (any global permutation, identical on every rank) give
    the input-order log-likelihood, and the shards' rows cover every location once."""
    from oracle import nngp_oracle as O

    n, m = 2500, 8
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker_storage, args=(world, _free_port(), n, m, out), nprocs=world, join=True)
    rng = np.random.default_rng(0)
    coords = rng.uniform(size=(n, 2))
    values = rng.standard_normal(n)
    _, _, p = O.c_bf_sweep(coords, O.c_knn_prior(coords, m), "exponential", (1.3, 9.0, 0.05), values)
    want = O.loglik_from_partials(p, n)
    lls = [out[r][0] for r in range(world)]
    assert all(v == lls[0] for v in lls)
    assert abs(lls[0] - want) <= 1e-11 * abs(want)
    assert sorted(sum((out[r][1] for r in range(world)), [])) == list(range(n))
    assert abs(O.loglik_from_partials(out[0][2], n) - lls[0]) <= 1e-12 * abs(lls[0])


def _worker(rank, world, port, n, m, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from pynngp_amd import Covariance

    rng = np.random.default_rng(0)
    coords = torch.from_numpy(rng.uniform(size=(n, 2)))
    values = torch.from_numpy(rng.standard_normal(n))
    sweep = ShardedLogLik(coords, m, rank, world, build_nbr=_oracle_build, compute=_oracle_compute)
    cov = Covariance("matern32", 1.0, 12.0, 0.1)
    ll = sweep.loglik(cov, values)
    # flags: smallest non-negative over ranks, -1 if none
    f = torch.tensor([0.0, 0.0, -1.0 if rank == 0 else 5.0 + rank, 9.0 if rank == 0 else -1.0], dtype=torch.float64)
    comb = combine_partials(f, world).tolist()
    out[rank] = (ll, sweep.lo, sweep.hi, comb)
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_gloo_sharded_loglik_matches_single(world):
    from oracle import nngp_oracle as O

    n, m = 3001, 10
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), n, m, out), nprocs=world, join=True)
    rng = np.random.default_rng(0)
    coords = rng.uniform(size=(n, 2))
    values = rng.standard_normal(n)
    nbr = O.c_knn_prior(coords, m)
    _, _, p = O.c_bf_sweep(coords, nbr, "matern32", (1.0, 12.0, 0.1), values)
    want = O.loglik_from_partials(p, n)
    lls = [out[r][0] for r in range(world)]
    assert lls[0] == lls[1]  # every rank sees the same (rank-order) sum
    assert abs(lls[0] - want) <= 1e-12 * abs(want)
    assert [(out[r][1], out[r][2]) for r in range(world)] == [shard_range(n, r, world) for r in range(world)]
    assert out[0][3] == [0.0, 0.0, 6.0, 9.0]


def test_no_group_no_collective():
    """Without a process group a one-rank sweep skips the exchange (the plain bench path)."""
    assert not dist.is_initialized()
    coords = torch.from_numpy(np.random.default_rng(1).uniform(size=(300, 2)))
    sw = ShardedLogLik(coords, 5, 0, 1, build_nbr=_oracle_build, compute=_oracle_compute)
    assert not sw.collective
    p = torch.tensor([1.0, 2.0, -1.0, -1.0], dtype=torch.float64)
    assert combine_partials(p, 1) is p
