"""GPU parity at the BASELINE.json configurations' full sizes, every row.

Configs (BASELINE.json "configs", SURVEY.md 8(d) inputs):
  2: N = 1e5, m = 15, Matern-3/2 (phi = sqrt(3)/0.1), tau2 = 0.1, seed 2
  3: N = 1e6, m = 15, exponential (phi = 30), tau2 = 0, seed 0   (the headline)
  4: N = 1e7, m = 20, exponential (phi = 30), tau2 = 0, seed 1   (8 shards at N = 1e7)
For each: the GPU neighbour sets against the C oracle's brute force
(oracle/nngp_oracle.c: nngp.py:49-62 restated, sklearn's unfused rdist, ties by
lower index) -- every row at configs 2 and 3; at config 4 EVERY row against the
independent doubling-prefix kd-tree search (oracle_knn_prior_prefix_kdtree: trees over
s[0:2^k], pinned to the brute force in tests/test_oracle.py; ~6 s on 16 threads where the
brute force would take ~1 h) plus 12,000 rows against the brute force itself -- then B and
F of EVERY row and the whole-field log-likelihood against the
C oracle's sweep on the GPU's neighbour sets.  Config 3 also runs through the
benchmark's own path (ShardedLogLik, Z-order storage layout) and config 4 through its
8-shard decomposition.  Tolerances as tests/test_gpu_bf.py:
  F: |dF| / F <= 1e-10;  B: |dB| <= 1e-9 (1 + |B|);
  log-lik: |dl| / |l| <= max(1e-12, 1e-15 kappa), kappa = max_i (sigma2 + tau2) / F_i.
Also: the HIP sweep on the committed golden vectors (tests/golden/bf_golden_*.npz,
made on reference-produced neighbour sets) against their frozen B / F / log-lik.
"""
import numpy as np
import pytest
import torch

from conftest import load_golden

pytestmark = pytest.mark.gpu

RTOL_F = 1e-10
ATOL_B = 1e-9
RTOL_LL = 1e-12

CONFIGS = {
    2: dict(n=100_000, m=15, kind="matern32", theta=(1.0, float(np.sqrt(3.0) / 0.1), 0.1), seed=2),
    3: dict(n=1_000_000, m=15, kind="exponential", theta=(1.0, 30.0, 0.0), seed=0),
    4: dict(n=10_000_000, m=20, kind="exponential", theta=(1.0, 30.0, 0.0), seed=1),
}


@pytest.fixture(scope="module")
def lib():
    from pynngp_amd import _lib

    return _lib


def _field(cfg):
    rng = np.random.default_rng(cfg["seed"])
    coords = rng.uniform(0.0, 1.0, (cfg["n"], 2))
    return coords, rng.standard_normal(cfg["n"])


def _ll_tol(theta, Fo):
    kappa = float(np.max((theta[0] + theta[2]) / Fo))
    return max(RTOL_LL, 1e-15 * kappa)


def _compare_bf(B, F, ll, Bo, Fo, llo, theta, nbr):
    dF = np.abs(F - Fo) / Fo
    assert np.all(dF <= RTOL_F), (float(dF.max()), int(np.argmax(dF)))
    dB = np.abs(B - Bo) / (1.0 + np.abs(Bo))
    assert np.all(dB <= ATOL_B), (float(dB.max()), np.unravel_index(int(np.argmax(dB)), dB.shape))
    assert np.all(B[nbr < 0] == 0.0)
    assert abs(ll - llo) <= _ll_tol(theta, Fo) * abs(llo), (ll, llo)


def _knn_all_rows(lib, dev, c_oracle, coords, m):
    got = lib.knn_prior(torch.from_numpy(coords).to(dev), m).cpu().numpy()
    np.testing.assert_array_equal(got, c_oracle.c_knn_prior(coords, m))
    return got


@pytest.mark.parametrize("config", [2, 3])
def test_config_all_rows(lib, dev, c_oracle, config):
    """Neighbour sets bit-exact on every row; B / F on every row and the log-likelihood."""
    cfg = CONFIGS[config]
    coords, y = _field(cfg)
    n, m, kind, theta = cfg["n"], cfg["m"], cfg["kind"], cfg["theta"]
    nbr = _knn_all_rows(lib, dev, c_oracle, coords, m)
    c = torch.from_numpy(coords).to(dev)
    v = torch.from_numpy(y).to(dev)
    B, F, p = lib.bf_sweep(c, torch.from_numpy(nbr).to(dev), 0, kind, *theta, values=v)
    Bo, Fo, po = c_oracle.c_bf_sweep(coords, nbr, kind, theta, y)
    p = p.cpu().numpy()
    assert p[2] == -1 and p[3] == -1 and po[2] == -1
    _compare_bf(B.cpu().numpy(), F.cpu().numpy(), c_oracle.loglik_from_partials(p, n), Bo, Fo,
                c_oracle.loglik_from_partials(po, n), theta, nbr)


def test_config3_bench_path_all_rows(lib, dev, c_oracle):
    """The benchmark's own path at config 3 (ShardedLogLik, Z-order storage layout, the
    auto kernel): every storage row's B / F is bit-identical to the input-order sweep's
    row and within tolerance of the oracle; the log-likelihood matches the oracle's."""
    from pynngp_amd import Covariance, ShardedLogLik

    cfg = CONFIGS[3]
    coords, y = _field(cfg)
    n, m, kind, theta = cfg["n"], cfg["m"], cfg["kind"], cfg["theta"]
    c = torch.from_numpy(coords).to(dev)
    v = torch.from_numpy(y).to(dev)
    sw = ShardedLogLik(c, m, 0, 1, layout="storage")
    ll = sw.loglik(Covariance(kind, *theta), v, want_bf=True)
    perm = sw.perm.long().cpu().numpy()
    # storage neighbour indices -> input indices: the input-order sets, row by row
    ns = sw.nbr.cpu().numpy()
    nbr_in = np.full((n, m), -1, dtype=np.int32)
    nbr_in[perm] = np.where(ns >= 0, perm[np.maximum(ns, 0)], -1)
    Bs, Fs = sw.B.cpu().numpy(), sw.F.cpu().numpy()
    B = np.empty_like(Bs)
    F = np.empty_like(Fs)
    B[perm], F[perm] = Bs, Fs
    Bn, Fn, _ = lib.bf_sweep(c, torch.from_numpy(nbr_in).to(dev), 0, kind, *theta, values=v)
    assert np.array_equal(B, Bn.cpu().numpy()) and np.array_equal(F, Fn.cpu().numpy())
    Bo, Fo, po = c_oracle.c_bf_sweep(coords, nbr_in, kind, theta, y)
    _compare_bf(B, F, ll, Bo, Fo, c_oracle.loglik_from_partials(po, n), theta, nbr_in)


def test_config4_rows_and_shards(lib, dev, c_oracle):
    """N = 1e7, m = 20: every neighbour row bit-exact vs the prefix kd-tree search and 12,000
    rows vs the brute force; B / F of every row and the log-likelihood vs the oracle; the 8-shard storage decomposition's
    rank-order sum equals the oracle's log-likelihood too."""
    from pynngp_amd import Covariance, ShardedLogLik

    cfg = CONFIGS[4]
    coords, y = _field(cfg)
    n, m, kind, theta = cfg["n"], cfg["m"], cfg["kind"], cfg["theta"]
    c = torch.from_numpy(coords).to(dev)
    v = torch.from_numpy(y).to(dev)
    nb = lib.knn_prior(c, m)
    nbr = nb.cpu().numpy()
    rng = np.random.default_rng(44)
    rows = np.unique(np.concatenate([np.arange(1000), n - 1000 + np.arange(1000), rng.integers(0, n, 10_000)]))
    np.testing.assert_array_equal(nbr[rows], c_oracle.c_knn_prior_rows(coords, m, rows))
    kd = c_oracle.c_knn_prior_prefix_kdtree(coords, m)
    np.testing.assert_array_equal(nbr, kd)  # all 1e7 rows
    del kd
    B, F, p = lib.bf_sweep(c, nb, 0, kind, *theta, values=v)
    Bo, Fo, po = c_oracle.c_bf_sweep(coords, nbr, kind, theta, y)
    llo = c_oracle.loglik_from_partials(po, n)
    _compare_bf(B.cpu().numpy(), F.cpu().numpy(), c_oracle.loglik_from_partials(p.cpu().numpy(), n), Bo, Fo, llo,
                theta, nbr)
    del B, F
    cov = Covariance(kind, *theta)
    tot = np.zeros(2)
    for r in range(8):
        sh = ShardedLogLik(c, m, r, 8, layout="storage")
        pr = sh.local_partials(cov, v).cpu().numpy()
        assert pr[2] == -1 and pr[3] == -1
        tot += pr[:2]
    ll8 = -0.5 * (n * c_oracle.LOG_2PI + tot[0] + tot[1])
    assert abs(ll8 - llo) <= _ll_tol(theta, Fo) * abs(llo), (ll8, llo)


@pytest.mark.parametrize("name", ["bf_golden_n1000_m10_exp", "bf_golden_n2000_m15_matern32"])
@pytest.mark.parametrize("algo", ["auto", "lane", "pairb", "wave"])
def test_hip_sweep_on_golden_vectors(lib, dev, name, algo):
    """The HIP sweep on the committed golden vectors (reference-produced neighbour sets,
    frozen oracle B / F / log-lik): the same tolerances."""
    g = load_golden(name)
    coords, nbr, y, theta = g["coords"], g["Ns"], g["y"], tuple(g["theta"])
    kind = str(g["kind"])
    if algo == "lane" and nbr.shape[1] > 16:
        pytest.skip("lane kernel serves m <= 16")
    B, F, p = lib.bf_sweep(torch.from_numpy(coords).to(dev), torch.from_numpy(nbr).to(dev), 0, kind, *theta,
                           values=torch.from_numpy(y).to(dev), algo=algo)
    p = p.cpu().numpy()
    ll = -0.5 * (nbr.shape[0] * np.log(2 * np.pi) + p[0] + p[1])
    _compare_bf(B.cpu().numpy(), F.cpu().numpy(), ll, g["B"], g["F"], float(g["loglik"]), theta, nbr)
