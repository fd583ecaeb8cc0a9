"""The native operator library (torch.ops.nngp.*, libnngp_torch_ops.so) is the path the
drop-in classes sweep through (ShardedLogLik, SeqNNGP): its results are bit-identical to the
same C-ABI call made through ctypes (pynngp_amd._lib), for every operator."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ops():
    from pynngp_amd import load_ops

    return load_ops()


def _field(n, dim, seed):
    rng = np.random.default_rng(seed)
    return rng.uniform(0.0, 1.0, (n, dim)), rng.standard_normal(n)


@pytest.mark.parametrize("dim,kind,algo,m", [(2, "exponential", "auto", 15), (2, "matern32", "pairb", 10),
                                             (3, "gaussian", "auto", 12), (1, "matern52", "wave", 20),
                                             (2, "spherical", "auto", 30)])
def test_bf_sweep_out_bit_identical_to_ctypes(ops, dev, dim, kind, algo, m):
    from pynngp_amd import _lib

    coords, y = _field(20000, dim, m)
    c, v = torch.from_numpy(coords).to(dev), torch.from_numpy(y).to(dev)
    theta = (1.3, 9.0, 0.2)
    nb = _lib.knn_prior(c, m)
    order, srt = _lib.row_order(c, 0, 20000, nb)
    B1, F1, p1 = _lib.bf_sweep(c, srt, 0, kind, *theta, values=v, algo=algo, order=order,
                               R=(R1 := torch.empty(20000, dtype=torch.float64, device=dev)))
    ws = _lib.bf_workspace(20000, m, algo, dev, kind=kind, dim=dim)
    B2, F2, R2 = (torch.full_like(B1, np.nan), torch.full_like(F1, np.nan), torch.full_like(R1, np.nan))
    p2 = torch.full((4,), np.nan, dtype=torch.float64, device=dev)
    torch.ops.nngp.bf_sweep_out(c, srt, order, 0, ops.kind_code(kind), *theta, v, B2, F2, R2, p2, ws,
                                ops.algo_code(algo))
    assert torch.equal(B1, B2) and torch.equal(F1, F2) and torch.equal(R1, R2) and torch.equal(p1, p2)
    # the allocating variant and the no-values / no-B path
    B3, F3, p3 = torch.ops.nngp.bf_sweep(c, srt, 0, ops.kind_code(kind), *theta, v, True, ops.algo_code(algo), order)
    assert torch.equal(B1, B3) and torch.equal(F1, F3) and torch.equal(p1, p3)
    _, _, p4 = _lib.bf_sweep(c, nb, 0, kind, *theta, want_bf=False, algo=algo)
    B5, F5, p5 = torch.ops.nngp.bf_sweep(c, nb, 0, ops.kind_code(kind), *theta, None, False, ops.algo_code(algo))
    assert B5.numel() == 0 and F5.numel() == 0 and torch.equal(p4, p5)


def test_knn_row_order_cross_combine_ops_bit_identical(ops, dev):
    from pynngp_amd import _lib

    coords, y = _field(30000, 2, 3)
    c, v = torch.from_numpy(coords).to(dev), torch.from_numpy(y).to(dev)
    assert torch.equal(torch.ops.nngp.knn_prior(c, 15, 100, 9000), _lib.knn_prior(c, 15, 100, 9000))
    rows = torch.randperm(30000, device=dev)[:5000].to(torch.int32)
    assert torch.equal(torch.ops.nngp.knn_prior_rows(c, 15, rows), _lib.knn_prior_rows(c, 15, rows))
    q = torch.rand((4000, 2), dtype=torch.float64, device=dev)
    nq = torch.ops.nngp.knn_query(c, q, 10)
    assert torch.equal(nq, _lib.knn_query(c, q, 10))
    nb = _lib.knn_prior(c, 15)
    o1, s1 = torch.ops.nngp.row_order(c, 0, 30000, nb)
    o2, s2 = _lib.row_order(c, 0, 30000, nb)
    assert torch.equal(o1, o2) and torch.equal(s1, s2)
    Bq, Fq, mean = torch.ops.nngp.bf_cross(c, q, nq, ops.kind_code("matern32"), 1.0, 7.0, 0.1, v, ops.algo_code("auto"))
    R = torch.empty(4000, dtype=torch.float64, device=dev)
    Bq2, Fq2, _ = _lib.bf_cross(c, q, nq, "matern32", 1.0, 7.0, 0.1, ref_values=v, R=R)
    assert torch.equal(Bq, Bq2) and torch.equal(Fq, Fq2) and torch.equal(mean, -R)
    g = torch.randn((5, 4), dtype=torch.float64, device=dev)
    out = torch.empty(4, dtype=torch.float64, device=dev)
    torch.ops.nngp.combine_partials_out(g, out)
    assert torch.equal(out, _lib.combine_partials(g))


@pytest.mark.parametrize("layout", ["natural", "storage"])
def test_sharded_loglik_goes_through_the_op(ops, dev, c_oracle, layout):
    """ShardedLogLik sweeps through torch.ops.nngp.bf_sweep_out; its partials equal the
    ctypes call on the same buffers bit for bit, and the C oracle to 1e-12."""
    from pynngp_amd import Covariance, ShardedLogLik, _lib

    coords, y = _field(50000, 2, 8)
    c, v = torch.from_numpy(coords).to(dev), torch.from_numpy(y).to(dev)
    sw = ShardedLogLik(c, 15, layout=layout)
    cov = Covariance("exponential", 1.0, 20.0, 0.1)
    p_op = sw.local_partials(cov, v).clone()
    vs = sw.to_storage(v) if layout == "storage" else v
    _, _, p_ct = _lib.bf_sweep(sw._coords_sweep, sw._nbr_sweep, sw.lo, cov.kind, *cov.theta, values=vs,
                               order=sw.order, algo=sw.algo)
    assert torch.equal(p_op, p_ct)
    ll = sw.loglik(cov, v)
    _, _, po = c_oracle.c_bf_sweep(coords, c_oracle.c_knn_prior(coords, 15), "exponential", cov.theta, y)
    assert abs(ll - c_oracle.loglik_from_partials(po, 50000)) <= 1e-12 * abs(ll)


def test_ops_reject_cpu_and_bad_buffers(ops, dev):
    c = torch.rand((100, 2), dtype=torch.float64, device=dev)
    nb = torch.ops.nngp.knn_prior(c, 5, 0, 100)
    ws = torch.empty(1 << 20, dtype=torch.uint8, device=dev)
    p = torch.empty(4, dtype=torch.float64, device=dev)
    with pytest.raises(Exception):
        torch.ops.nngp.knn_prior(c.cpu(), 5, 0, 100)
    with pytest.raises(RuntimeError, match="B"):
        torch.ops.nngp.bf_sweep_out(c, nb, None, 0, 0, 1.0, 5.0, 0.1, None, torch.empty((100, 4), dtype=torch.float64,
                                    device=dev), None, None, p, ws, 0)
    with pytest.raises(RuntimeError, match="partials"):
        torch.ops.nngp.bf_sweep_out(c, nb, None, 0, 0, 1.0, 5.0, 0.1, None, None, None, None,
                                    torch.empty(3, dtype=torch.float64, device=dev), ws, 0)


def test_bf_sweep_out_graph_replay_bit_identical(ops, dev):
    """The bench's launch-bound mode (bench.py --graph): the sweep and its record fold captured
    once in a hipGraph (torch.cuda.CUDAGraph) and replayed give the direct call's bits."""
    from pynngp_amd.sweep import Covariance, ShardedLogLik

    coords, y = _field(100_000, 2, 11)
    c, v = torch.from_numpy(coords).to(dev), torch.from_numpy(y).to(dev)
    sweep = ShardedLogLik(c, 15, 0, 1, layout="storage")
    cov = Covariance("matern32", 1.0, 17.320508075688772, 0.1)
    direct = sweep.local_partials(cov, v, True, "storage").clone()
    B0, F0 = sweep.B.clone(), sweep.F.clone()
    out = torch.empty(4, dtype=torch.float64, device=dev)
    side = torch.cuda.Stream(device=dev)
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        sweep.local_partials(cov, v, True, "storage", out=out)
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        sweep.local_partials(cov, v, True, "storage", out=out)
    sweep.B.fill_(np.nan)
    sweep.F.fill_(np.nan)
    out.fill_(np.nan)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, direct) and torch.equal(sweep.B, B0) and torch.equal(sweep.F, F0)
