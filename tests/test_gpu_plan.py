"""GPU parity: wave pair plans (nngp_pair_plan_build / nngp_bf_sweep_plan, pair_plan.h).

A planned sweep evaluates every covariance a wavefront's locations share once, into the wave's LDS
slice, and factors each location's joint block from there.  Covariances are symmetric bit for bit ((a - b)^2 == (b - a)^2
in IEEE arithmetic) and everything after them is the unplanned pair kernel's code, so the bar is
EXACT equality with the unplanned sweep (NNGP_ALGO_PAIRB) on the same arguments: B, F, the residuals
R and the four partials, for every kind the plans serve, m = 2..17, dimensions 1..3, with and without
a visiting order, shards (i0 > 0), padded first rows, invalid neighbour indices, and tiles that
exceed the LDS budget (swept by the unplanned kernel into the same records), and stale plans.  The unplanned kernel
itself is held to the C oracle by tests/test_gpu_bf.py and tests/test_gpu_fullsize.py; one case here
also checks the planned sweep against the oracle directly.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

KINDS = ["exponential", "matern32", "matern52", "gaussian", "spherical"]
THETA = {"exponential": (1.0, 30.0, 0.0), "matern32": (1.0, 17.320508075688772, 0.1),
         "matern52": (1.2, 12.0, 0.05), "gaussian": (0.8, 9.0, 0.2), "spherical": (1.0, 8.0, 0.1)}


@pytest.fixture(scope="module")
def lib():
    from pynngp_amd import _lib

    return _lib


def _field(dev, n, dim, seed):
    rng = np.random.default_rng(seed)
    c = torch.from_numpy(rng.uniform(0.0, 1.0, (n, dim))).to(dev)
    v = torch.from_numpy(rng.standard_normal(n)).to(dev)
    return c, v


def _both(lib, c, nbr, kind, theta, v, i0=0, order=None, plan=None):
    """unplanned and planned sweeps of the same rows: (B, F, R, partials) each"""
    rows, m = nbr.shape
    if plan is None:
        plan = lib.pair_plan(nbr, c.shape[0], c.shape[1], i0=i0, order=order)
    out = []
    for p in (None, plan):
        R = torch.empty(rows, dtype=torch.float64, device=c.device) if v is not None else None
        B, F, part = lib.bf_sweep(c, nbr, i0, kind, *theta, values=v, algo="pairb", order=order, R=R, plan=p)
        out.append((B, F, R, part))
    return out, plan


def _assert_same(a, b):
    for x, y, name in zip(a, b, ("B", "F", "R", "partials")):
        if x is None:
            assert y is None
            continue
        assert torch.equal(x, y), (name, float((x - y).abs().max()))


@pytest.mark.parametrize("kind", KINDS)
def test_plan_equals_unplanned_every_kind(dev, lib, kind):
    c, v = _field(dev, 30_000, 2, 1)
    nbr = lib.knn_prior(c, 15)
    order, nbr_s = lib.row_order(c, 0, c.shape[0], nbr)
    (a, b), plan = _both(lib, c, nbr_s, kind, THETA[kind], v, order=order)
    assert plan.n_planned > 0 and plan.n_planned + plan.n_direct == (c.shape[0] + 127) // 128
    _assert_same(a, b)
    assert float(a[3][2]) == -1.0 and float(a[3][3]) == -1.0


@pytest.mark.parametrize("m", list(range(2, 18)))
def test_plan_equals_unplanned_every_m(dev, lib, m):
    c, v = _field(dev, 9_000, 2, m)
    nbr = lib.knn_prior(c, m)
    order, nbr_s = lib.row_order(c, 0, c.shape[0], nbr)
    for kind in ("exponential", "matern32"):
        (a, b), plan = _both(lib, c, nbr_s, kind, THETA[kind], v, order=order)
        assert plan.n_planned > 0
        _assert_same(a, b)


@pytest.mark.parametrize("dim", [1, 3])
@pytest.mark.parametrize("m", [5, 10, 15, 17])
def test_plan_equals_unplanned_dims(dev, lib, dim, m):
    c, v = _field(dev, 12_000, dim, 10 * dim + m)
    nbr = lib.knn_prior(c, m)
    order, nbr_s = lib.row_order(c, 0, c.shape[0], nbr)
    for kind in ("exponential", "gaussian"):
        (a, b), plan = _both(lib, c, nbr_s, kind, THETA[kind], v, order=order)
        # (3-D points take 32 bytes of LDS each and a sparse 3-D field shares fewer pairs: at m >= 15 the
        # waves of this 12,000-point field overflow their slices and every tile is direct -- still exact)
        assert plan.n_planned > 0 or (dim == 3 and m >= 15)
        _assert_same(a, b)


def test_plan_storage_layout_sharded(dev, lib):
    """ShardedLogLik's storage layout (the bench's path): planned = unplanned, whole field and a shard"""
    from pynngp_amd import Covariance
    from pynngp_amd.sweep import ShardedLogLik

    c, v = _field(dev, 50_000, 2, 7)
    cov = Covariance("exponential", 1.0, 30.0, 0.0)
    for rank, world in ((0, 1), (1, 3), (2, 3)):
        s_pl = ShardedLogLik(c, 15, rank, world, layout="storage", plan=True)
        s_un = ShardedLogLik(c, 15, rank, world, layout="storage", plan=False)
        assert s_pl.planned and not s_un.planned
        p_pl = s_pl.local_partials(cov, v, True).clone()
        p_un = s_un.local_partials(cov, v, True).clone()
        assert torch.equal(p_pl, p_un)
        assert torch.equal(s_pl.B, s_un.B) and torch.equal(s_pl.F, s_un.F)
        # the ctypes path through the same plan
        s_ct = ShardedLogLik(c, 15, rank, world, layout="storage", plan=True, api="ctypes")
        assert torch.equal(s_ct.local_partials(cov, v, True), p_un)


def test_plan_shard_rows_i0(dev, lib):
    """a shard of rows [i0, i0 + n) (the natural layout with its own visiting order)"""
    c, v = _field(dev, 20_000, 2, 3)
    i0, n = 6_000, 7_777
    nbr = lib.knn_prior(c, 15, i0, i0 + n)
    order, nbr_s = lib.row_order(c, i0, n, nbr)
    (a, b), plan = _both(lib, c, nbr_s, "matern32", THETA["matern32"], v, i0=i0, order=order)
    _assert_same(a, b)
    # no visiting order: the rows in index order
    (a, b), _ = _both(lib, c, nbr, "matern32", THETA["matern32"], v, i0=i0)
    _assert_same(a, b)


def test_plan_padding_rows_small_fields(dev, lib):
    """rows i < m (padded slots, exact zeros), fields smaller than one tile, one row"""
    for n, m in ((1, 5), (2, 5), (17, 15), (127, 15), (128, 15), (129, 15), (300, 17)):
        c, v = _field(dev, n, 2, n)
        nbr = lib.knn_prior(c, m)
        (a, b), plan = _both(lib, c, nbr, "exponential", THETA["exponential"], v)
        _assert_same(a, b)
        assert torch.all(a[0][nbr < 0] == 0.0)


def test_plan_empty_sweep(dev, lib):
    c, v = _field(dev, 100, 2, 5)
    nbr = torch.empty((0, 15), dtype=torch.int32, device=dev)
    plan = lib.pair_plan(nbr, c.shape[0], 2)
    assert plan.n_planned == 0 and plan.n_direct == 0
    _, _, p = lib.bf_sweep(c, nbr, 0, "exponential", 1.0, 30.0, 0.0, values=v, plan=plan)
    assert p.cpu().tolist() == [0.0, 0.0, -1.0, -1.0]


def test_plan_without_values(dev, lib):
    c, _ = _field(dev, 10_000, 2, 9)
    nbr = lib.knn_prior(c, 15)
    (a, b), _ = _both(lib, c, nbr, "exponential", THETA["exponential"], None)
    _assert_same(a, b)


def test_plan_direct_tiles(dev, lib):
    """tiles past the LDS budget (non-spatial neighbour sets: ~2,000 distinct points per tile) go to the
    unplanned kernel, in the same records: a mixed sweep and an all-direct sweep stay bit-identical"""
    c, v = _field(dev, 40_000, 2, 11)
    nbr = lib.knn_prior(c, 15)
    order, nbr_s = lib.row_order(c, 0, c.shape[0], nbr)
    g = torch.Generator(device="cpu").manual_seed(0)
    rnd = nbr_s.clone()
    rows = torch.arange(10_000, 14_000)
    lim = (order[rows].long().cpu()).clamp(min=1)
    rnd[rows] = (torch.rand((len(rows), 15), generator=g) * lim[:, None].double()).long().to(torch.int32).to(dev)
    # (random sets may repeat a point: the nugget keeps C_N + tau2 I positive definite)
    (a, b), plan = _both(lib, c, rnd, "matern32", THETA["matern32"], v, order=order)
    assert plan.n_direct >= 25 and plan.n_planned > 0, (plan.n_planned, plan.n_direct)
    _assert_same(a, b)
    allrnd = (torch.rand((c.shape[0], 15), generator=g) * torch.arange(c.shape[0]).clamp(min=1)[:, None].double()
              ).long().to(torch.int32).to(dev)
    (a, b), plan = _both(lib, c, allrnd, "matern32", THETA["matern32"], v)
    # (the first tile's rows draw from a few hundred earlier points: it fits)
    assert plan.n_planned <= 2 and plan.n_direct >= (c.shape[0] + 127) // 128 - 2, (plan.n_planned, plan.n_direct)
    _assert_same(a, b)


def test_plan_invalid_indices_flagged(dev, lib):
    c, v = _field(dev, 20_000, 2, 13)
    nbr = lib.knn_prior(c, 15)
    for bad in (-2, -7, -(2 ** 31), 20_000, 2 ** 31 - 1):
        nb = nbr.clone()
        nb[12_345, 4] = bad
        nb[15_000, 0] = bad
        (a, b), _ = _both(lib, c, nb, "exponential", THETA["exponential"], v)
        _assert_same(a, b)
        assert float(b[3][3]) == 12_345.0


def test_plan_geometry_mismatch_rejected(dev, lib):
    c, v = _field(dev, 5_000, 2, 17)
    nbr = lib.knn_prior(c, 10, 1_000, 3_000)
    plan = lib.pair_plan(nbr, c.shape[0], 2, i0=1_000)
    # (PairPlan.matches refuses these in Python; the C ABI checks the same geometry)
    with pytest.raises((ValueError, lib.NNGPExtensionError)):
        lib.bf_sweep(c, nbr, 0, "exponential", 1.0, 30.0, 0.0, values=v, plan=plan)  # i0 differs
    with pytest.raises((ValueError, lib.NNGPExtensionError)):
        lib.bf_sweep(c, nbr[:1_500], 1_000, "exponential", 1.0, 30.0, 0.0, values=v, plan=plan)  # rows differ
    with pytest.raises(lib.NNGPExtensionError):
        lib.bf_sweep(c, nbr, 1_000, "matern", 1.0, 30.0, 0.0, values=v, plan=plan, nu=1.3)  # kind not served


def test_plan_stale_rejected_or_flagged(dev, lib):
    """a plan of other neighbour sets: another buffer is refused (Python and the C ABI); the same buffer
    changed in place is refused by PairPlan.matches (torch's version counter) and, reached through the C
    ABI anyway, flagged by the kernel's per-location checksum with NaN B / F"""
    import ctypes

    c, v = _field(dev, 20_000, 2, 19)
    order, nbr = lib.row_order(c, 0, c.shape[0], lib.knn_prior(c, 15))  # (Z-order: planned waves)
    plan = lib.pair_plan(nbr, c.shape[0], 2, order=order)
    assert plan.n_planned > 0.8 * (plan.n_planned + plan.n_direct)
    other = nbr.clone()
    with pytest.raises(ValueError, match="stale"):
        lib.bf_sweep(c, other, 0, "exponential", 1.0, 30.0, 0.0, values=v, plan=plan, order=order)
    rows_changed = list(range(500, 20_000, 500))
    for t in rows_changed:  # swap two neighbours in place
        nbr[t, 3], nbr[t, 4] = int(nbr[t, 4]), int(nbr[t, 3])
    with pytest.raises(ValueError, match="stale"):
        lib.bf_sweep(c, nbr, 0, "exponential", 1.0, 30.0, 0.0, values=v, plan=plan, order=order)
    # the C ABI directly (its pointer check passes: same buffer): the kernel flags the changed location
    L = lib.load()
    rows, m = nbr.shape
    B = torch.empty((rows, m), dtype=torch.float64, device=dev)
    F = torch.empty(rows, dtype=torch.float64, device=dev)
    p = torch.empty(4, dtype=torch.float64, device=dev)
    ws = lib.bf_workspace(rows, m, "pairb", dev)
    P = ctypes.c_void_p
    rc = L.nngp_bf_sweep_plan(P(c.data_ptr()), c.shape[0], 2, P(nbr.data_ptr()), P(order.data_ptr()), rows, m, 0, 0,
                              1.0, 30.0, 0.0,
                              P(v.data_ptr()), P(B.data_ptr()), P(F.data_ptr()), None, P(p.data_ptr()),
                              P(ws.data_ptr()), ws.numel(), P(plan.buf.data_ptr()), plan.buf.numel(), plan.info,
                              P(torch.cuda.current_stream(dev).cuda_stream))
    assert rc == 0
    torch.cuda.synchronize(dev)
    # (B / F are written at their natural rows; a changed row in a direct tile -- swept by the unplanned
    # kernel from nbr itself -- is simply right)
    changed = {int(order[t]) for t in rows_changed}
    nan_at = set(torch.nonzero(torch.isnan(F)).flatten().tolist())
    assert nan_at and nan_at <= changed, (len(nan_at), sorted(nan_at - changed)[:5])
    assert float(p[3]) == float(min(nan_at))
    assert all(torch.isnan(B[i]).all() for i in nan_at)


def test_plan_vs_oracle(dev, lib, c_oracle):
    """the planned sweep against the C oracle directly (config-2-like field, Matern-3/2 with a nugget)"""
    O = c_oracle
    c, v = _field(dev, 20_000, 2, 21)
    nbr = lib.knn_prior(c, 15)
    plan = lib.pair_plan(nbr, c.shape[0], 2)
    theta = THETA["matern32"]
    B, F, p = lib.bf_sweep(c, nbr, 0, "matern32", *theta, values=v, plan=plan)
    cn, nn, vn = c.cpu().numpy(), nbr.cpu().numpy(), v.cpu().numpy()
    Bo, Fo, po = O.c_bf_sweep(cn, nn, "matern32", theta, vn)
    F, B, p = F.cpu().numpy(), B.cpu().numpy(), p.cpu().numpy()
    assert np.all(np.abs(F - Fo) <= 1e-10 * Fo)
    assert np.all(np.abs(B - Bo) <= 1e-9 * (1 + np.abs(Bo)))
    ll, llo = O.loglik_from_partials(p, len(F)), O.loglik_from_partials(po, len(F))
    kappa = float(np.max((theta[0] + theta[2]) / Fo))
    assert abs(ll - llo) <= max(1e-12, 1e-15 * kappa) * abs(llo)


def test_plan_op_matches_ctypes(dev, lib):
    """torch.ops.nngp.pair_plan + bf_sweep_out(plan=...) = the ctypes path, bit for bit"""
    from pynngp_amd import ops

    c, v = _field(dev, 15_000, 2, 23)
    nbr = lib.knn_prior(c, 15)
    pb, pi = ops.pair_plan(nbr, None, 0, c.shape[0], 2)
    assert pi.device.type == "cpu" and pi.dtype == torch.int64
    B = torch.empty((15_000, 15), dtype=torch.float64, device=dev)
    F = torch.empty(15_000, dtype=torch.float64, device=dev)
    p = torch.empty(4, dtype=torch.float64, device=dev)
    ws = lib.bf_workspace(15_000, 15, "auto", dev)
    ops.bf_sweep_out(c, nbr, None, 0, "exponential", (1.0, 30.0, 0.0), v, B, F, None, p, ws, plan=(pb, pi))
    B2, F2, p2 = lib.bf_sweep(c, nbr, 0, "exponential", 1.0, 30.0, 0.0, values=v, algo="pairb")
    assert torch.equal(B, B2) and torch.equal(F, F2) and torch.equal(p, p2)
