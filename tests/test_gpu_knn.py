"""GPU parity: neighbour sets (nngp_knn_prior / nngp_knn_query) vs the reference.

Bar: bit-exact indices.  Golden fixtures come from the reference itself
(tests/golden/make_golden.py imports pyNNGP and runs _make_s_neighbor_sets,
pyNNGP/nngp.py:49-62); larger cases compare with the C oracle's brute force
(oracle/nngp_oracle.c, same (rdist, index) order).  Rows with an exact distance
tie are excluded from the reference comparison: its tie order is arbitrary
(sklearn/utils/_heap.pyx:45-47) and ours is lower-index-first (checked against
the oracle instead).
"""
import numpy as np
import pytest
import torch

from conftest import load_golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lib():
    from pynngp_amd import _lib

    return _lib


@pytest.mark.parametrize("name", ["knn_ref_n200_m3", "knn_ref_n1000_m10", "knn_ref_n5000_m15", "knn_ref_lattice6_m4"])
def test_knn_matches_reference_fixture(lib, dev, c_oracle, name):
    g = load_golden(name)
    m = int(g["m"])
    got = lib.knn_prior(torch.from_numpy(g["coords"]).to(dev), m).cpu().numpy()
    ok = ~g["tie_rows"]
    np.testing.assert_array_equal(got[ok], g["Ns"][ok])
    # every row (ties included) equals the lower-index-first oracle
    np.testing.assert_array_equal(got, c_oracle.c_knn_prior(g["coords"], m))
    # reference test assertion (tests/test_init.py:22-23): no self-neighbour, j < i
    for i in range(got.shape[0]):
        row = got[i][got[i] >= 0]
        assert i not in row and np.all(row < i) and row.size == min(i, m)


@pytest.mark.parametrize("n,m,seed", [(20000, 15, 0), (20000, 10, 1), (8000, 20, 2), (3000, 1, 3), (5000, 32, 4),
                                      (4000, 64, 5)])
def test_knn_random_vs_oracle(lib, dev, c_oracle, n, m, seed):
    rng = np.random.default_rng(seed)
    coords = rng.uniform(0.0, 1.0, (n, 2))
    got = lib.knn_prior(torch.from_numpy(coords).to(dev), m).cpu().numpy()
    np.testing.assert_array_equal(got, c_oracle.c_knn_prior(coords, m))


def test_knn_clustered_anisotropic_duplicates(lib, dev, c_oracle):
    rng = np.random.default_rng(11)
    n = 6000
    a = rng.normal(0.0, 1e-3, (n // 2, 2)) + np.array([5.0, -3.0])
    b = rng.uniform(0.0, 1.0, (n // 2, 2)) * np.array([1000.0, 0.01])
    coords = np.concatenate([a, b])[rng.permutation(n)]
    coords[100:140] = coords[50]  # exact duplicates: ties broken by index
    got = lib.knn_prior(torch.from_numpy(coords).to(dev), 12).cpu().numpy()
    np.testing.assert_array_equal(got, c_oracle.c_knn_prior(coords, 12))


def test_knn_lattice_ties_and_degenerate_axis(lib, dev, c_oracle):
    g = np.arange(40, dtype=np.float64)
    coords = np.stack(np.meshgrid(g, g, indexing="ij"), -1).reshape(-1, 2)
    coords = coords[np.random.default_rng(0).permutation(coords.shape[0])].copy()
    got = lib.knn_prior(torch.from_numpy(coords).to(dev), 8).cpu().numpy()
    np.testing.assert_array_equal(got, c_oracle.c_knn_prior(coords, 8))
    line = np.stack([np.linspace(0, 1, 3000), np.zeros(3000)], 1)[np.random.default_rng(1).permutation(3000)].copy()
    got = lib.knn_prior(torch.from_numpy(line).to(dev), 6).cpu().numpy()
    np.testing.assert_array_equal(got, c_oracle.c_knn_prior(line, 6))


def test_knn_edge_sizes_and_ranges(lib, dev, c_oracle):
    one = torch.zeros((1, 2), dtype=torch.float64, device=dev)
    assert lib.knn_prior(one, 5).cpu().numpy().tolist() == [[-1] * 5]
    rng = np.random.default_rng(5)
    coords = rng.uniform(size=(10, 2))
    np.testing.assert_array_equal(lib.knn_prior(torch.from_numpy(coords).to(dev), 15).cpu().numpy(),
                                  c_oracle.c_knn_prior(coords, 15))
    assert lib.knn_prior(torch.from_numpy(coords).to(dev), 0).shape == (10, 0)
    coords = rng.uniform(size=(30000, 2))
    full = c_oracle.c_knn_prior(coords, 15)
    c = torch.from_numpy(coords).to(dev)
    for q0, q1 in [(0, 1), (0, 1000), (12345, 23456), (29999, 30000), (7, 7)]:
        np.testing.assert_array_equal(lib.knn_prior(c, 15, q0, q1).cpu().numpy(), full[q0:q1])


@pytest.mark.parametrize("n_ref,n_q,k", [(5000, 5000, 5), (3000, 700, 15), (4, 10, 5)])
def test_knn_query_vs_oracle(lib, dev, c_oracle, n_ref, n_q, k):
    rng = np.random.default_rng(n_ref + k)
    ref = rng.uniform(size=(n_ref, 2))
    qry = ref if n_q == n_ref else rng.uniform(size=(n_q, 2))
    got = lib.knn_query(torch.from_numpy(ref).to(dev), torch.from_numpy(qry).to(dev), k).cpu().numpy()
    kk = min(k, n_ref)
    np.testing.assert_array_equal(got[:, :kk], c_oracle.knn_all(qry, ref, kk))
    assert np.all(got[:, kk:] == -1)


def test_knn_fma_sensitive_ties(lib, dev, c_oracle):
    """Near-ties whose order flips if rdist is contracted into an FMA (either direction;
    tests/fma_ties.py): every q must pick p1, as sklearn's unfused rdist and the oracle do,
    through the brute-force prefix (i < 1024), the grid path and the unrestricted query."""
    from fma_ties import fma_sensitive_clusters

    coords, expect = fma_sensitive_clusters(3000, dim=2, seed=7)
    got = lib.knn_prior(torch.from_numpy(coords).to(dev), 1).cpu().numpy()
    np.testing.assert_array_equal(c_oracle.c_knn_prior(coords, 1)[2::3, 0], expect)
    np.testing.assert_array_equal(got[2::3, 0], expect)
    ref = np.delete(coords, np.s_[2::3], axis=0)  # p1, p2 of every cluster: rows 2c, 2c + 1
    qry = coords[2::3].copy()
    got = lib.knn_query(torch.from_numpy(ref).to(dev), torch.from_numpy(qry).to(dev), 1).cpu().numpy()
    np.testing.assert_array_equal(got[:, 0], np.arange(len(qry)) * 2)


def test_knn_ops_registered(dev):
    from pynngp_amd import load_ops

    ops = load_ops()

    coords = torch.rand((500, 2), dtype=torch.float64, device=dev)
    a = torch.ops.nngp.knn_prior(coords, 7, 0, 500)
    from pynngp_amd import _lib

    b = _lib.knn_prior(coords, 7, 0, 500)
    assert torch.equal(a, b) and a.dtype == torch.int32
    with pytest.raises(Exception):
        torch.ops.nngp.knn_prior(coords.cpu(), 7, 0, 500)
