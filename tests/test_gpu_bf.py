"""GPU parity: fused B/F + log-likelihood sweep (nngp_bf_sweep) vs the oracle.

Oracle: oracle/nngp_oracle.c (fp64, libm exp/sqrt, row-oriented Cholesky) on the
same neighbour sets.  Tolerances (fp64; the kernel uses its own ~1 ulp exp/sqrt
and a right-looking factorisation, so results differ in the last bits):
  F:        |dF| / F          <= 1e-10
  B:        |dB|              <= 1e-9 * (1 + |B|)
  loglik:   |dl| / |l|        <= max(1e-12, 1e-15 * kappa),  kappa = max_i (sigma2 + tau2) / F_i
The log-lik bound scales with kappa because F_i = C_ii - c^T C_N^{-1} c is a
difference of nearly equal numbers when the field is smooth relative to the
neighbour spacing (Matern-3/2 with tau2 = 0 reaches kappa ~ 3e5 below): its
relative rounding error, and that of r_i^2 / F_i, is ~ eps * kappa in any fp64
evaluation order (the oracle's included).
Bit-reproducibility run to run is exact.  Known answer on the GPU: m = N-1 gives
the dense-GP log density.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

RTOL_F = 1e-10
ATOL_B = 1e-9
RTOL_LL = 1e-12


@pytest.fixture(scope="module")
def lib():
    from pynngp_amd import _lib

    return _lib


def _field(n, seed):
    rng = np.random.default_rng(seed)
    return rng.uniform(0.0, 1.0, (n, 2)), rng.standard_normal(n)


def _check(dev, lib, O, coords, nbr, kind, theta, y, algo, i0=0):
    rows = nbr.shape[0]
    c = torch.from_numpy(coords).to(dev)
    v = None if y is None else torch.from_numpy(y).to(dev)
    B, F, p = lib.bf_sweep(c, torch.from_numpy(nbr).to(dev), i0, kind, *theta, values=v, algo=algo)
    Bo, Fo, po = O.c_bf_sweep(coords, nbr, kind, theta, y, i0=i0)
    B, F, p = B.cpu().numpy(), F.cpu().numpy(), p.cpu().numpy()
    assert p[2] == -1 and p[3] == -1
    assert np.all(np.abs(F - Fo) <= RTOL_F * Fo), np.max(np.abs(F - Fo) / Fo)
    assert np.all(np.abs(B - Bo) <= ATOL_B * (1 + np.abs(Bo))), np.max(np.abs(B - Bo))
    assert np.all(B[nbr < 0] == 0.0)
    ll = O.loglik_from_partials(p, rows)
    llo = O.loglik_from_partials(po, rows)
    kappa = float(np.max((theta[0] + theta[2]) / Fo))
    assert abs(ll - llo) <= max(RTOL_LL, 1e-15 * kappa) * abs(llo), (ll, llo, kappa)
    return p


CASES = [
    ("exponential", (1.0, 30.0, 0.0), 15),
    ("exponential", (1.3, 4.0, 0.1), 10),
    ("matern32", (1.0, 17.320508075688772, 0.1), 15),
    ("matern32", (2.0, 40.0, 0.0), 8),
    ("exponential", (0.7, 12.0, 0.05), 1),
    ("exponential", (1.0, 30.0, 0.0), 16),
    ("matern52", (1.0, 20.0, 0.1), 15),
    ("matern52", (1.5, 35.0, 0.02), 10),
    ("gaussian", (1.0, 10.0, 0.1), 15),
    ("gaussian", (0.8, 25.0, 0.2), 12),
    ("spherical", (1.0, 10.0, 0.05), 15),
    ("spherical", (1.2, 25.0, 0.0), 20),
]
CLASSIC = ("exponential", "matern32")  # the kinds the lane / quad kernels serve
ALL_KINDS = ("exponential", "matern32", "matern52", "gaussian", "spherical")


QUAD_M = tuple(range(25, 33))  # instantiated for the 4-lane kernel
PAIRB_M = tuple(range(1, 33))  # and for the 2x2-blocked 2-lane kernel (m = 25..32: left-looking, kinds 0..4)


@pytest.mark.parametrize("algo", ["lane", "wave", "pairb"])
@pytest.mark.parametrize("kind,theta,m", CASES)
def test_bf_vs_oracle(lib, dev, c_oracle, kind, theta, m, algo):
    if (algo == "lane" and m > 16) or (algo == "lane" and kind not in CLASSIC):
        pytest.skip("not instantiated")
    coords, y = _field(6000, m)
    nbr = c_oracle.c_knn_prior(coords, m)
    _check(dev, lib, c_oracle, coords, nbr, kind, theta, y, algo)


@pytest.mark.parametrize("m", [20, 24, 31, 40, 63])
def test_bf_large_m(lib, dev, c_oracle, m):
    coords, y = _field(3000, 100 + m)
    nbr = c_oracle.c_knn_prior(coords, m)
    _check(dev, lib, c_oracle, coords, nbr, "exponential", (1.0, 8.0, 0.05), y, "auto")
    _check(dev, lib, c_oracle, coords, nbr, "matern32", (1.0, 10.0, 0.1), y, "wave")
    for algo, ms in (("quad", QUAD_M), ("pairb", PAIRB_M)):
        if m in ms:
            _check(dev, lib, c_oracle, coords, nbr, "matern32", (1.0, 10.0, 0.1), y, algo)
            _check(dev, lib, c_oracle, coords, nbr, "exponential", (1.0, 30.0, 0.0), y, algo)


@pytest.mark.parametrize("m", list(range(25, 33)))
def test_bf_quad_all_m(lib, dev, c_oracle, m):
    """4-lane kernel at every m it is instantiated for (25..32), duplicates included."""
    coords, y = _field(2500, 400 + m)
    coords[1000:1010] = coords[500]
    nbr = c_oracle.c_knn_prior(coords, m)
    _check(dev, lib, c_oracle, coords, nbr, "exponential", (1.0, 20.0, 0.3), y, "quad")
    _check(dev, lib, c_oracle, coords, nbr, "matern32", (1.3, 15.0, 0.2), y, "quad")
    _check(dev, lib, c_oracle, coords, nbr, "exponential", (0.8, 30.0, 0.01), None, "auto")


@pytest.mark.parametrize("m", list(range(25, 33)))
@pytest.mark.parametrize("kind,theta", [("exponential", (1.0, 20.0, 0.3)), ("matern32", (1.3, 15.0, 0.2)),
                                        ("matern52", (1.0, 12.0, 0.1)), ("gaussian", (1.0, 6.0, 0.2)),
                                        ("spherical", (1.0, 8.0, 0.05))])
@pytest.mark.parametrize("dim", [1, 2, 3])
def test_bf_quad_generic_m25_32(lib, dev, c_oracle, m, kind, theta, dim):
    """m = 25..32 on the four-lane kernel (2-D exponential / Matern-3/2 instantiations, one
    runtime-kind, runtime-dimension instantiation per m for the rest), every kind and dimension; and
    the same sweep under algo "auto" (the pair kernel except at m = 31, never the wavefront kernel)."""
    rng = np.random.default_rng(500 + m + 7 * dim)
    coords = rng.uniform(0.0, 1.0, (1500, dim))
    coords[700:705] = coords[300]
    y = rng.standard_normal(1500)
    nbr = c_oracle.c_knn_prior(coords, m)
    _check(dev, lib, c_oracle, coords, nbr, kind, theta, y, "quad")
    _check(dev, lib, c_oracle, coords, nbr, kind, theta, y, "auto")


@pytest.mark.parametrize("m", list(range(25, 33)))
@pytest.mark.parametrize("kind,theta", [("exponential", (1.0, 20.0, 0.3)), ("matern32", (1.3, 15.0, 0.2)),
                                        ("matern52", (1.0, 12.0, 0.1)), ("gaussian", (1.0, 6.0, 0.2)),
                                        ("spherical", (1.0, 8.0, 0.05))])
@pytest.mark.parametrize("dim", [1, 2, 3])
def test_bf_pairb_m25_32_kinds_dims(lib, dev, c_oracle, m, kind, theta, dim):
    """The left-looking pair kernel at m = 25..32 (one wave per SIMD, 7 factor rows in LDS), every
    fused kind and dimension, duplicates included."""
    rng = np.random.default_rng(900 + m + 7 * dim)
    coords = rng.uniform(0.0, 1.0, (1500, dim))
    coords[700:705] = coords[300]
    y = rng.standard_normal(1500)
    nbr = c_oracle.c_knn_prior(coords, m)
    _check(dev, lib, c_oracle, coords, nbr, kind, theta, y, "pairb")


def test_auto_never_wave_below_33(lib):
    for m in range(1, 33):
        for kind in ALL_KINDS:
            for dim in (1, 2, 3):
                assert lib.resolve_algo("auto", m, kind, dim) == ("quad" if m == 31 else "pairb"), (m, kind, dim)
    assert lib.resolve_algo("auto", 33, "exponential", 2) == "wave"


@pytest.mark.parametrize("m", list(PAIRB_M))
def test_bf_pairb_all_m(lib, dev, c_oracle, m):
    """Blocked pair kernel, every instantiated m (odd m ends on a (neighbour, location) pair,
    even m on (location, padding)); duplicated points exercise coincident coordinates."""
    coords, y = _field(2500, 300 + m)
    coords[1000:1010] = coords[500]  # exact duplicates (d2 = 0 -> the 2^-1000 floor)
    nbr = c_oracle.c_knn_prior(coords, m)
    _check(dev, lib, c_oracle, coords, nbr, "exponential", (1.0, 20.0, 0.3), y, "pairb")
    _check(dev, lib, c_oracle, coords, nbr, "matern32", (1.3, 15.0, 0.2), y, "pairb")
    _check(dev, lib, c_oracle, coords, nbr, "exponential", (0.8, 30.0, 0.01), None, "pairb")


def test_bf_m0_and_no_values(lib, dev, c_oracle):
    coords, y = _field(500, 9)
    nbr = np.zeros((500, 0), dtype=np.int32)
    p = _check(dev, lib, c_oracle, coords, nbr, "exponential", (1.5, 3.0, 0.2), y, "auto")
    # m = 0: independent N(0, sigma2 + tau2)
    ll = c_oracle.loglik_from_partials(p, 500)
    s = 1.7
    assert abs(ll - (-0.5 * (500 * np.log(2 * np.pi * s) + (y * y).sum() / s))) < 1e-9
    nbr = c_oracle.c_knn_prior(coords, 12)
    p = _check(dev, lib, c_oracle, coords, nbr, "exponential", (1.0, 10.0, 0.0), None, "lane")
    assert p[1] == 0.0


def test_bf_dense_gp_known_answer(lib, dev, c_oracle):
    """m = N-1: the NNGP density is the exact GP density (Vecchia with full conditioning)."""
    n = 60
    coords, y = _field(n, 21)
    nbr = c_oracle.c_knn_prior(coords, n - 1)
    for kind, theta in [("exponential", (1.3, 4.0, 0.1)), ("matern32", (1.0, 3.0, 0.05))]:
        c = torch.from_numpy(coords).to(dev)
        _, _, p = lib.bf_sweep(c, torch.from_numpy(nbr).to(dev), 0, kind, *theta,
                               values=torch.from_numpy(y).to(dev))
        ll = c_oracle.loglik_from_partials(p.cpu().numpy(), n)
        dense = c_oracle.dense_gp_loglik(coords, kind, theta, y)
        assert abs(ll - dense) <= 1e-10 * abs(dense), (ll, dense)


def test_bf_shards_sum_and_reproducible(lib, dev, c_oracle):
    coords, y = _field(20000, 3)
    m = 15
    nbr = c_oracle.c_knn_prior(coords, m)
    c = torch.from_numpy(coords).to(dev)
    v = torch.from_numpy(y).to(dev)
    nb = torch.from_numpy(nbr).to(dev)
    theta = (1.0, 30.0, 0.0)
    B, F, p = lib.bf_sweep(c, nb, 0, "exponential", *theta, values=v)
    B2, F2, p2 = lib.bf_sweep(c, nb, 0, "exponential", *theta, values=v)
    assert torch.equal(B, B2) and torch.equal(F, F2) and torch.equal(p, p2)
    cuts = [0, 1, 777, 5000, 13333, 20000]
    tot = torch.zeros(2, dtype=torch.float64, device=dev)
    for a, b in zip(cuts[:-1], cuts[1:]):
        Bs, Fs, ps = lib.bf_sweep(c, nb[a:b], a, "exponential", *theta, values=v)
        assert torch.equal(Bs, B[a:b]) and torch.equal(Fs, F[a:b])
        tot += ps[:2]
    assert torch.allclose(tot, p[:2], rtol=1e-13, atol=0)
    _, _, pe = lib.bf_sweep(c, nb[:0], 0, "exponential", *theta, values=v)
    assert pe.cpu().tolist() == [0.0, 0.0, -1.0, -1.0]


def test_bf_flags_bad_rows(lib, dev, c_oracle):
    coords, y = _field(2000, 4)
    nbr = c_oracle.c_knn_prior(coords, 10)
    c = torch.from_numpy(coords).to(dev)
    sing = nbr.copy()
    sing[1234, 1] = sing[1234, 0]  # repeated neighbour: C_N singular, second pivot exactly 0 (sigma2 = 1)
    sing[1500, 1] = sing[1500, 0]
    for algo in ["lane", "wave", "pairb"]:
        B, F, p = lib.bf_sweep(c, torch.from_numpy(sing).to(dev), 0, "exponential", 1.0, 5.0, 0.0, algo=algo)
        _, _, po = c_oracle.c_bf_sweep(coords, sing, "exponential", (1.0, 5.0, 0.0), None)
        assert p[2].item() == 1234 == po[2]
        Fh = F.cpu().numpy()
        assert np.isnan(Fh[1234]) and np.isnan(Fh[1500]) and np.all(np.isfinite(np.delete(Fh, [1234, 1500])))
        assert np.all(np.isnan(B.cpu().numpy()[1234]))
    bad = nbr.copy()
    bad[1234, 3] = 2000  # out-of-range neighbour index
    _, _, p = lib.bf_sweep(c, torch.from_numpy(bad).to(dev), 0, "exponential", 1.0, 5.0, 0.1)
    assert p[3].item() == 1234


@pytest.mark.parametrize("algo,m", [("lane", 10), ("wave", 10), ("pairb", 10), ("pairb", 15), ("pairb", 19),
                                    ("pairb", 20), ("pairb", 22), ("quad", 26), ("quad", 31)])
@pytest.mark.parametrize("bad_value", [-2, -7, -2147483648, 2000, 2147483647])
def test_bf_flags_every_invalid_index(lib, dev, c_oracle, algo, m, bad_value):
    """Any neighbour index < -1 or >= n_points sets partials[3] to the first such row, for every
    kernel (-1 is the only padding value); the C oracle marks the same row bad."""
    coords, _ = _field(2000, 5)
    nbr = c_oracle.c_knn_prior(coords, m)
    bad = nbr.copy()
    bad[1234, m // 2] = bad_value  # a middle row, a middle slot
    bad[1500, 0] = bad_value
    c = torch.from_numpy(coords).to(dev)
    _, _, p = lib.bf_sweep(c, torch.from_numpy(bad).to(dev), 0, "exponential", 1.0, 5.0, 0.1, algo=algo)
    assert p[3].item() == 1234
    _, Fo, po = c_oracle.c_bf_sweep(coords, bad, "exponential", (1.0, 5.0, 0.1), None)
    assert po[2] == 1234 and np.isnan(Fo[1234]) and np.isnan(Fo[1500])
    # -1 padding alone is never flagged
    _, _, p = lib.bf_sweep(c, torch.from_numpy(nbr).to(dev), 0, "exponential", 1.0, 5.0, 0.1, algo=algo)
    assert p[3].item() == -1


def test_bf_full_size_properties(lib, dev, c_oracle):
    """Config 3 size (N=1e6, m=15): lane == wave, sampled rows vs oracle, F in (0, sigma2]."""
    n, m = 1_000_000, 15
    coords, y = _field(n, 0)
    c = torch.from_numpy(coords).to(dev)
    v = torch.from_numpy(y).to(dev)
    nb = lib.knn_prior(c, m)
    theta = (1.0, 30.0, 0.0)
    B, F, p = lib.bf_sweep(c, nb, 0, "exponential", *theta, values=v, algo="lane")
    ll = c_oracle.loglik_from_partials(p.cpu().numpy(), n)
    for algo in ("wave", "pairb"):
        Bw, Fw, pw = lib.bf_sweep(c, nb, 0, "exponential", *theta, values=v, algo=algo)
        assert torch.allclose(F, Fw, rtol=1e-12, atol=0)
        assert torch.allclose(B, Bw, rtol=0, atol=1e-10)
        llw = c_oracle.loglik_from_partials(pw.cpu().numpy(), n)
        assert abs(ll - llw) <= 1e-12 * abs(ll)
    Fh = F.cpu().numpy()
    assert np.all(Fh > 0) and np.all(Fh <= 1.0 + 1e-12)
    rows = np.random.default_rng(1).integers(0, n, 4000)
    rows = np.unique(np.concatenate([rows, np.arange(20)]))
    nbr_h = nb.cpu().numpy()
    for r0 in rows[::400]:
        r1 = min(n, r0 + 400)
        Bo, Fo, _ = c_oracle.c_bf_sweep(coords, nbr_h[r0:r1], "exponential", theta, y, i0=int(r0))
        assert np.all(np.abs(Fh[r0:r1] - Fo) <= RTOL_F * Fo)
        assert np.all(np.abs(B[r0:r1].cpu().numpy() - Bo) <= ATOL_B * (1 + np.abs(Bo)))


def test_bf_op_registered(dev, c_oracle):
    from pynngp_amd import load_ops

    ops = load_ops()

    coords, y = _field(1000, 8)
    c = torch.from_numpy(coords).to(dev)
    nb = torch.ops.nngp.knn_prior(c, 10, 0, 1000)
    B, F, p = torch.ops.nngp.bf_sweep(c, nb, 0, ops.kind_code("matern32"), 1.0, 5.0, 0.1,
                                      torch.from_numpy(y).to(dev), True, ops.algo_code("auto"))
    Bo, Fo, po = c_oracle.c_bf_sweep(coords, nb.cpu().numpy(), "matern32", (1.0, 5.0, 0.1), y)
    assert np.allclose(F.cpu().numpy(), Fo, rtol=RTOL_F, atol=0)
    _, _, p2 = torch.ops.nngp.bf_sweep(c, nb, 0, 1, 1.0, 5.0, 0.1, None, False, 0)
    assert abs(p2[0].item() - po[0]) <= 1e-12 * abs(po[0])


@pytest.mark.parametrize("algo", ["lane", "wave", "pairb"])
def test_bf_row_order_bit_identical(lib, dev, c_oracle, algo):
    """Visiting rows in Z-order (nngp_row_order) changes nothing per row."""
    coords, y = _field(30000, 12)
    c = torch.from_numpy(coords).to(dev)
    v = torch.from_numpy(y).to(dev)
    nb = lib.knn_prior(c, 15)
    for i0, rows in [(0, 30000), (777, 10000), (29990, 10)]:
        order, srt = lib.row_order(c, i0, rows, nb[i0:i0 + rows])
        oh = order.cpu().numpy()
        assert np.array_equal(np.sort(oh), np.arange(rows))
        assert torch.equal(srt, nb[i0:i0 + rows][order.long()])
        B1, F1, p1 = lib.bf_sweep(c, nb[i0:i0 + rows], i0, "exponential", 1.0, 30.0, 0.0, values=v, algo=algo)
        B2, F2, p2 = lib.bf_sweep(c, srt, i0, "exponential", 1.0, 30.0, 0.0, values=v, algo=algo, order=order)
        assert torch.equal(B1, B2) and torch.equal(F1, F2)
        assert torch.allclose(p1[:2], p2[:2], rtol=1e-13, atol=0) and torch.equal(p1[2:], p2[2:])
    # Z-order really is spatially coherent: consecutive rows are close
    order = lib.row_order(c)[0].cpu().numpy()
    step = np.linalg.norm(np.diff(coords[order], axis=0), axis=1)
    assert np.median(step) < 0.01


def test_combine_partials_rank_order(lib, dev):
    g = torch.tensor([[1.5, 2.0, -1.0, 7.0], [0.25, 3.0, 5.0, -1.0], [1e-17, 1.0, 9.0, 2.0]],
                     dtype=torch.float64, device=dev)
    out = lib.combine_partials(g).cpu().tolist()
    assert out == [(1.5 + 0.25) + 1e-17, (2.0 + 3.0) + 1.0, 5.0, 2.0]
    out = lib.combine_partials(g[:1, :]).cpu().tolist()
    assert out == [1.5, 2.0, -1.0, 7.0]


@pytest.mark.parametrize("algo", ["lane", "pairb", "wave"])
@pytest.mark.parametrize("kind", ["exponential", "matern32", "matern52", "gaussian", "spherical"])
def test_bf_m1_covariance_ulp(lib, dev, c_oracle, kind, algo):
    """m = 1 isolates the device covariance: B_i = C(d_i) / (sigma2 + tau2) with d_i the
    nearest-prior distance.  Checked against 80-bit long double at 2e-15 relative, i.e.
    a few ulp (v_rsq_f64 alone is only good to ~2^-24; one plain Newton step for sqrt
    would leave ~1e-14 relative error here)."""
    if algo == "lane" and kind not in CLASSIC:
        pytest.skip("lane kernel: exponential / Matern-3/2")
    coords, _ = _field(20000, 77)
    nbr = c_oracle.c_knn_prior(coords, 1)
    sigma2, phi, tau2 = 1.3, 9.0, 0.4
    c = torch.from_numpy(coords).to(dev)
    B, F, p = lib.bf_sweep(c, torch.from_numpy(nbr).to(dev), 0, kind, sigma2, phi, tau2, algo=algo)
    j = nbr[1:, 0]
    dx = coords[1:, 0].astype(np.longdouble) - coords[j, 0]
    dy = coords[1:, 1].astype(np.longdouble) - coords[j, 1]
    u = np.longdouble(phi) * np.sqrt(dx * dx + dy * dy)
    cov = sigma2 * {"exponential": np.exp(-u), "matern32": (1 + u) * np.exp(-u),
                    "matern52": (1 + u + u * u / 3) * np.exp(-u), "gaussian": np.exp(-u * u),
                    "spherical": np.where(u < 1, 1 - 1.5 * u + 0.5 * u ** 3, 0)}[kind]
    Bx = cov / np.longdouble(sigma2 + tau2)
    Bg = B.cpu().numpy()[1:, 0].astype(np.longdouble)
    if kind == "spherical":
        # 1 - 3u/2 + u^3/2 cancels towards the range (it reaches exactly 0 at u = 1): a few ulp
        # of sigma2 absolute, as the oracle's own evaluation
        err = np.abs(Bg - Bx) / (sigma2 / (sigma2 + tau2))
        assert float(err.max()) <= 1e-15, float(err.max())
        return
    rel = np.abs(Bg - Bx) / Bx
    bound = 4e-15 if kind == "matern52" else 2e-15
    assert float(rel.max()) <= bound, float(rel.max())


@pytest.mark.parametrize("algo", ["lane", "pairb", "wave"])
def test_bf_extreme_inputs(lib, dev, c_oracle, algo):
    """UTM-like coordinates (offset 1e6, spread ~1e3), tiny and huge phi, exact duplicates:
    the kernel's clamps (d2 floor, exp underflow bound) and far-point padding hold."""
    rng = np.random.default_rng(8)
    n, m = 4000, 12
    coords = 1e6 + rng.uniform(0, 1000.0, (n, 2))
    coords[2000:2010] = coords[100]
    y = rng.standard_normal(n)
    nbr = c_oracle.c_knn_prior(coords, m)
    for kind, theta in [("exponential", (2.0, 1e-2, 0.3)), ("matern32", (1.0, 3e-3, 0.2)),
                        ("exponential", (1.0, 50.0, 0.1)), ("exponential", (1e6, 0.5, 1e5))]:
        _check(dev, lib, c_oracle, coords, nbr, kind, theta, y, algo if m <= 16 or algo != "lane" else "auto")


def test_bf_tiny_fields(lib, dev, c_oracle):
    """N <= m (every row padded), N = 1 and N = 2."""
    for n, m in [(1, 4), (2, 4), (5, 15), (16, 15), (3, 20)]:
        coords, y = _field(n, 40 + n)
        nbr = c_oracle.c_knn_prior(coords, m)
        for algo in ("auto", "wave", "pairb"):
            _check(dev, lib, c_oracle, coords, nbr, "exponential", (1.0, 5.0, 0.1), y, algo)


@pytest.mark.parametrize("algo", ["auto", "lane", "wave", "quad"])
def test_deferred_finalize_same_bits(lib, dev, c_oracle, algo):
    """nngp_bf_sweep with partials = NULL + nngp_bf_finalize (the pipelined benchmark's
    path) gives exactly the in-line partials, for every record layout."""
    m = {"auto": 15, "lane": 10, "wave": 15, "quad": 26}[algo]
    coords, y = _field(20000, 77)
    nbr = torch.from_numpy(c_oracle.c_knn_prior(coords, m)).to(dev)
    c, v = torch.from_numpy(coords).to(dev), torch.from_numpy(y).to(dev)
    _, _, p = lib.bf_sweep(c, nbr, 0, "exponential", 1.0, 20.0, 0.1, values=v, algo=algo)
    ws = lib.bf_workspace(nbr.shape[0], m, algo, dev)
    _, _, none = lib.bf_sweep(c, nbr, 0, "exponential", 1.0, 20.0, 0.1, values=v, algo=algo, workspace=ws, defer=True)
    assert none is None
    q = lib.bf_finalize(ws, nbr.shape[0], m, "exponential", 2, algo)
    assert torch.equal(p, q)
    # a finalize whose (m, kind, dim, algo) do not match the sweep's record layout is refused
    if algo == "wave":
        with pytest.raises(lib.NNGPExtensionError):
            lib.bf_finalize(ws[:256], nbr.shape[0], 15, "exponential", 2, "pairb")
