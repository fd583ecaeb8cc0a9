"""GPU: the largest field one MI355X takes comfortably -- N = 1.5e8 locations, m = 15 -- where the
(N, m) neighbour and B arrays hold 2.25e9 entries, past 2^31: every (row, slot) offset in the kNN and
sweep kernels must be 64-bit (an int32 product would wrap from row 143,165,577 on).

Checked against the oracle: the neighbour sets of rows on both sides of that boundary
by the exact brute-force prior search, their B / F by the per-location restatement, and the whole
field's log-likelihood against the C restatement (OpenMP) -- the same tolerances as configs 2-4
(tests/test_gpu_fullsize.py).  ~40 GB of HBM, ~25 GB of host memory."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

N, M = 150_000_000, 15
THETA = (1.0, 30.0, 0.0)


def test_sweep_past_2_31_entries(dev, c_oracle):
    from pynngp_amd import _lib

    O = c_oracle
    free, _ = torch.cuda.mem_get_info(dev)
    if free < 80 * 2 ** 30:
        pytest.skip(f"needs ~40 GB of free HBM with headroom ({free / 2 ** 30:.0f} GB free)")
    rng = np.random.default_rng(31)
    x = rng.uniform(size=(N, 2))
    y = rng.standard_normal(N)
    c = torch.from_numpy(x).to(dev)
    v = torch.from_numpy(y).to(dev)
    nb = _lib.knn_prior(c, M)
    assert nb.shape == (N, M) and nb.numel() > 2 ** 31
    B, F, p = _lib.bf_sweep(c, nb, 0, "exponential", *THETA, values=v)
    assert p[2].item() == -1 and p[3].item() == -1
    edge = (2 ** 31 - 1) // M  # the first row whose int32 offset row * m would wrap
    rows = [3, 1_000_000, edge - 1, edge, edge + 1, 149_999_998, N - 1]
    nbh = nb[rows].cpu().numpy()
    Bh, Fh = B[rows].cpu().numpy(), F[rows].cpu().numpy()
    for k, r in enumerate(rows):
        np.testing.assert_array_equal(nbh[k], O.knn_prior(x, M, r, r + 1)[0], err_msg=f"row {r}")
        Bo, Fo, _ = O.bf_sweep(x, nbh[k:k + 1], "exponential", THETA, y, i0=r)
        assert abs(Fh[k] - Fo[0]) <= 1e-10 * Fo[0], r
        assert np.all(np.abs(Bh[k] - Bo[0]) <= 1e-9 * (1 + np.abs(Bo[0]))), r
    del B, F
    nb_h = nb.cpu().numpy()
    del nb, c, v
    torch.cuda.empty_cache()
    _, _, po = O.c_bf_sweep(x, nb_h, "exponential", THETA, y, want_bf=False)
    ll, llo = O.loglik_from_partials(p.cpu().numpy(), N), O.loglik_from_partials(po, N)
    assert abs(ll - llo) <= 1e-12 * abs(llo), (ll, llo)
