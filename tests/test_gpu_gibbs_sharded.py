"""GPU: one Gibbs chain sharded over ranks (pynngp_amd.ShardedSeqNNGP).

Fresh child processes (tests/gibbs_sharded_child.py) run the sharded chain; the parent runs
the single-GPU ``SeqNNGP`` chain on the same data and seed:
  * one rank over an RCCL ("nccl") group -- every exchange goes through the collective and the
    colour loop replays from captured HIP graphs (sigma2 / tau2 read from device memory): the
    chain is SeqNNGP's bit for bit (w after a sweep and after 25 iterations, every scalar draw);
  * 2 and 3 ranks on the one GPU over gloo (the rehearsal of the N-GPU flow): one w sweep at
    fixed hyperparameters is bit-identical (each location's draw is its owner's arithmetic on
    replicas the exchange keeps exact); the 25-iteration chain agrees to rounding (the global
    sums fold in rank order: relative 1e-9 on w and the scalars).
Parity against the exact full conditionals is tests/test_gpu_gibbs.py's (the same kernels).
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ITERS = 25


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(world, backend, out, exchange="halo"):
    port = _port()
    procs = []
    for rank in range(world):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), LOCAL_RANK="0",
                   WORLD_SIZE=str(world))
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "gibbs_sharded_child.py"), backend,
                                       out, str(ITERS), exchange], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                      text=True))
    outs = []
    for p in procs:
        try:
            so, se = p.communicate(timeout=300)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append((p.returncode, so, se))
    for rc, so, se in outs:
        assert rc == 0 and "GIBBS_SHARDED_OK" in so, (rc, so[-2000:], se[-4000:])
    with np.load(out, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="module")
def single(dev):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import gibbs_sharded_child as C
    from pynngp_amd import SeqNNGP, _lib

    t, y, X = C.problem()
    g = SeqNNGP(t, y, X, device=dev, **C.KW)
    _lib.gibbs_normals(g._z, g.seed, 0)
    g.update_wt()
    g.update_ws()
    w_sweep = g.w_nodes.cpu().numpy()
    res = g.sample(ITERS)
    return dict(w_sweep=w_sweep, w_final=g.w_nodes.cpu().numpy(), y_un=g.y_unobserved.cpu().numpy(), **res)


@pytest.mark.parametrize("exchange", ["all", "halo"])
def test_one_rank_rccl_equals_single_chain(single, tmp_path, exchange):
    """One rank over RCCL: with exchange="all" every colour's all-gather runs (captured in the HIP graphs
    of the colour loop); with the halo exchange a single rank has no boundary, so no colour collective."""
    got = _run(1, "nccl", str(tmp_path / "r1.npz"), exchange)
    meta = json.loads(str(got["meta"]))
    assert meta["world"] == 1
    if exchange == "all":
        assert meta["n_collectives"] > 0 and meta["exchange_bytes"] == meta["allgather_bytes"] > 0
    else:
        assert meta["n_collectives"] == 0 and meta["exchange_bytes"] == 0
    assert meta["graphs"] >= 1  # the colour loop replayed from captured HIP graphs
    assert np.array_equal(got["w_sweep"], single["w_sweep"])
    for k in ("beta", "sigma2", "tau2", "phi"):
        assert np.array_equal(got[k], single[k]), k
    assert np.array_equal(got["w_final"], single["w_final"])
    assert np.array_equal(got["y_un"], single["y_un"])


@pytest.mark.parametrize("world,exchange", [(2, "halo"), (3, "halo"), (2, "all")])
def test_ranks_on_one_gpu_gloo(single, tmp_path, world, exchange):
    got = _run(world, "gloo", str(tmp_path / f"r{world}.npz"), exchange)
    meta = json.loads(str(got["meta"]))
    assert meta["world"] == world and meta["halo"] > 0 and meta["apply"] > 0
    if exchange == "halo":  # the boundary only
        assert 0 < meta["exchange_bytes"] < meta["allgather_bytes"]
    assert np.array_equal(got["w_sweep"], single["w_sweep"])  # one sweep: bit for bit
    for k in ("sigma2", "tau2", "phi"):
        np.testing.assert_allclose(got[k], single[k], rtol=1e-9, atol=0)
    np.testing.assert_allclose(got["beta"], single["beta"], rtol=1e-9, atol=1e-12)
    wf = single["w_final"]
    np.testing.assert_allclose(got["w_final"], wf, rtol=0, atol=1e-9 * np.abs(wf).max())
    np.testing.assert_allclose(got["y_un"], single["y_un"], rtol=0, atol=1e-9 * np.abs(single["y_un"]).max())
