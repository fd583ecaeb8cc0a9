"""CPU: the C-ABI library loads, exports every symbol include/nngp.h declares, and
rejects bad arguments before touching the GPU (no compute calls here)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "nngp.h")


def header_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(nngp_[a-z_0-9]+)\s*\(", text)))


@pytest.fixture(scope="module")
def lib():
    from pynngp_amd import _lib

    if not os.path.exists(_lib.LIB_PATH):
        pytest.fail(f"{_lib.LIB_PATH} missing: run __graft_entry__.build()")
    return _lib.load()


def test_header_symbols_exported(lib):
    syms = header_symbols()
    assert len(syms) >= 8
    for s in syms:
        assert hasattr(lib, s), s
    from pynngp_amd import _lib

    assert sorted(_lib.SYMBOLS) == syms


def test_version_and_loglik_helper(lib):
    from pynngp_amd import _lib

    assert _lib.version().startswith("pynngp_amd") and "gfx950" in _lib.version()
    p = (ctypes.c_double * 2)(3.0, 4.0)
    got = lib.nngp_loglik_from_partials(ctypes.cast(p, ctypes.c_void_p), 10)
    assert abs(got - (-0.5 * (10 * 1.8378770664093453 + 7.0))) < 1e-12


def test_workspace_sizes(lib):
    # (n_rows, m, kind, dim, algo): the blocked pair kernel keeps one 32-B record and one 4-B exponent
    # per 128-location tile, the lane kernel a record per 256 rows
    # (a 256-B header with the tile count; records for the most tiles a balanced tiling uses: the plain
    # 128-row tiles plus up to one round of 3 x 256 block slots, at more than 96 rows per tile)
    al = lambda b: (b + 255) // 256 * 256  # noqa: E731
    tiles = (1_000_000 + 127) // 128
    bound = max(tiles, min(tiles + 767, 1_000_000 // 97))
    assert lib.nngp_bf_sweep_workspace_bytes(1_000_000, 15, 0, 2, 0) == 256 + al(32 * bound) + al(4 * bound)
    assert lib.nngp_bf_sweep_workspace_bytes(1_000_000, 8, 0, 2, 0) >= 4 * 8 * (1_000_000 // 256)
    assert lib.nngp_bf_sweep_workspace_bytes(1_000_000, 8, 3, 2, 0) == 256 + al(32 * bound) + al(4 * bound)
    small = lib.nngp_bf_sweep_workspace_bytes(1000, 15, 0, 2, 0)  # bound max(8, min(8 + 767, 1000 // 97))
    assert small == 256 + al(32 * 10) + al(4 * 10)
    assert lib.nngp_bf_sweep_workspace_bytes(-1, 15, 0, 2, 0) == 0
    assert lib.nngp_bf_sweep_workspace_bytes(0, 15, 0, 2, 0) == 0
    assert lib.nngp_bf_sweep_workspace_bytes(10, 40, 0, 3, 0) > 0


def _sweep(lib, **kw):
    a = dict(coords=1, n_points=10, dim=2, nbr=1, n_rows=10, m=15, i0=0, kind=0, sigma2=1.0, phi=1.0, tau2=0.0,
             nu=-1.0, values=None, B=None, F=None, partials=1, workspace=256, workspace_bytes=1 << 20, algo=0, stream=None)
    a.update(kw)
    P = lambda v: None if v is None else ctypes.c_void_p(v)  # noqa: E731
    return lib.nngp_bf_sweep(P(a["coords"]), a["n_points"], a["dim"], P(a["nbr"]), None, a["n_rows"], a["m"], a["i0"],
                             a["kind"],
                             a["sigma2"], a["phi"], a["tau2"], a["nu"], P(a["values"]), P(a["B"]), P(a["F"]), P(a.get("R")),
                             P(a["partials"]), P(a["workspace"]), a["workspace_bytes"], a["algo"], P(a["stream"]))


@pytest.mark.parametrize("kw,code,msg", [
    (dict(coords=None), -1, "non-null"),
    (dict(m=64), -4, "m=64"),
    (dict(m=-1), -4, "m=-1"),
    (dict(n_rows=11), -1, "outside"),
    (dict(i0=5), -1, "outside"),
    (dict(kind=7), -1, "unknown kind"),
    (dict(kind=-1), -1, "unknown kind"),
    (dict(dim=0), -4, "dim=0"),
    (dict(dim=4), -4, "dim=4"),
    (dict(algo=1, m=8, kind=2), -4, "2-D exponential and Matern-3/2 only"),
    (dict(algo=1, m=10, dim=3), -4, "2-D exponential and Matern-3/2 only"),
    (dict(algo=4, m=20), -4, "4-lane kernel"),
    (dict(algo=3, m=15), -1, "unknown algo"),  # the removed comparison kernels
    (dict(algo=7, m=15), -1, "unknown algo"),
    (dict(algo=5, m=33), -4, "blocked pair kernel"),
    (dict(sigma2=0.0), -1, "theta"),
    (dict(phi=float("nan")), -1, "theta"),
    (dict(tau2=-1.0), -1, "theta"),
    (dict(B=256), -1, "B given without F"),
    (dict(F=256), -1, "F given without B"),
    (dict(workspace=257), -1, "aligned"),
    (dict(algo=1, m=17), -4, "lane kernel"),
    (dict(algo=9), -1, "unknown algo"),
    (dict(workspace_bytes=16), -1, "workspace too small"),
    (dict(R=256), -1, "R (residuals) needs values"),
    (dict(kind=5, nu=0.0), -1, "nu"),  # general-smoothness Matern: 0 < nu <= 50
    (dict(kind=5, nu=50.5), -1, "nu"),
    (dict(kind=5, nu=float("nan")), -1, "nu"),
    (dict(kind=5, nu=1.2, algo=1, m=8), -4, "pair (m <= 24), four-lane (25..32) or wavefront kernel"),
    (dict(kind=5, nu=0.3, algo=1, m=8), -4, "pair (m <= 24), four-lane (25..32) or wavefront kernel"),
    (dict(kind=5, nu=1.5, algo=5, m=25), -4, "matern kind runs on the pair kernel for m <= 24"),  # (advice r05)
    (dict(kind=5, nu=1.5, algo=5, m=32), -4, "matern kind runs on the pair kernel for m <= 24"),
])
def test_bf_sweep_rejects(lib, kw, code, msg):
    assert _sweep(lib, **kw) == code
    assert msg in lib.nngp_last_error().decode()


def test_row_order_rejects(lib):
    P = ctypes.c_void_p
    assert lib.nngp_row_order(None, 10, 2, None, 0, 0, 10, P(1), None, P(256), 1 << 20, None) == -1
    assert lib.nngp_row_order(P(1), 10, 2, None, 0, 5, 6, P(1), None, P(256), 1 << 20, None) == -1
    assert lib.nngp_row_order(P(1), 10, 2, None, 0, 0, 10, None, None, P(256), 1 << 20, None) == -1
    assert lib.nngp_row_order(P(1), 10, 2, None, 5, 0, 10, P(1), P(1), P(256), 1 << 20, None) == -1
    assert lib.nngp_row_order(P(1), 10, 2, P(1), 70, 0, 10, P(1), P(1), P(256), 1 << 20, None) == -4
    assert lib.nngp_row_order(P(1), 10, 4, None, 0, 0, 10, P(1), None, P(256), 1 << 20, None) == -4


def test_knn_rejects(lib):
    P = ctypes.c_void_p
    assert lib.nngp_knn_prior(None, 10, 2, 5, 0, 10, P(1), P(256), 1 << 20, None) == -1
    assert lib.nngp_knn_prior(P(1), 10, 2, 65, 0, 10, P(1), P(256), 1 << 20, None) == -4
    assert lib.nngp_knn_prior(P(1), 10, 2, 5, 3, 2, P(1), P(256), 1 << 20, None) == -1
    assert lib.nngp_knn_prior(P(1), 0, 2, 5, 0, 0, P(1), P(256), 1 << 20, None) == -1
    assert lib.nngp_knn_prior(P(1), 10, 0, 5, 0, 10, P(1), P(256), 1 << 20, None) == -4
    assert lib.nngp_knn_prior(P(1), 10, 4, 5, 0, 10, P(1), P(256), 1 << 20, None) == -4
    assert lib.nngp_knn_query(P(1), 10, 2, None, 5, 3, P(1), P(256), 1 << 20, None) == -1
    assert lib.nngp_knn_query(P(1), 10, 2, P(1), 5, 99, P(1), P(256), 1 << 20, None) == -4
    assert lib.nngp_knn_workspace_bytes(1000, 3, 15) > lib.nngp_knn_workspace_bytes(1000, 1, 15) > 0
    assert lib.nngp_knn_workspace_bytes(1000, 4, 15) == 0


def test_no_cpu_fallback():
    import torch

    from pynngp_amd import _lib

    c = torch.zeros((4, 2), dtype=torch.float64)
    with pytest.raises(_lib.NNGPExtensionError, match="no CPU fallback"):
        _lib.knn_prior(c, 3)
    with pytest.raises(_lib.NNGPExtensionError, match="no CPU fallback"):
        _lib.bf_sweep(c, torch.zeros((4, 3), dtype=torch.int32), 0, "exponential", 1.0, 1.0)


def test_check_partials_codes(lib):
    """-2 for a non-positive pivot with the first bad location reported."""
    import ctypes

    import numpy as np

    def run(p):
        a = np.asarray(p, dtype=np.float64)
        r, i = ctypes.c_int64(7), ctypes.c_int64(7)
        rc = lib.nngp_check_partials(a.ctypes.data_as(ctypes.c_void_p), ctypes.byref(r), ctypes.byref(i))
        return rc, r.value, i.value

    assert run([1.0, 2.0, -1.0, -1.0]) == (0, -1, -1)
    assert run([1.0, 2.0, 1234.0, -1.0]) == (-2, 1234, -1)
    assert b"1234" in lib.nngp_last_error()
    assert run([1.0, 2.0, 5.0, 99.0]) == (-1, 5, 99)


def test_resolve_algo_table(lib):
    """auto: the blocked pair kernel for 1 <= m <= 32 except m = 31 (the four-lane kernel) at kinds
    0..4 and every dimension, the wavefront kernel above; the general-smoothness Matern kind (5): the pair
    kernel for m <= 24 and the four-lane kernel for 25..32, for every nu in (0, 50] (since round 5 the
    launch's table serves small nu too: below t = 2^-64 the small-t expansion 1 - A t^nu); explicit codes
    pass through."""
    for m in (1, 15, 20, 24, 25, 28, 30, 31, 32):
        for kind in range(6):
            for dim in (1, 2, 3):
                want = (5 if m <= 24 else 4) if kind == 5 else (4 if m == 31 else 5)
                assert lib.nngp_resolve_algo(0, m, kind, dim) == want, (m, kind, dim)
    assert lib.nngp_resolve_algo(0, 33, 0, 2) == 2
    assert lib.nngp_resolve_algo(0, 63, 4, 3) == 2
    assert lib.nngp_resolve_algo(1, 15, 0, 2) == 1
    for m in (1, 15, 24, 25, 32, 33, 40):
        for nu in (0.01, 0.05, 0.3, 0.44, 0.45, 0.5, 1.0, 2.5, 49.0, 50.0):
            assert lib.nngp_resolve_algo_nu(0, m, 5, 2, nu) == (5 if m <= 24 else 4 if m <= 32 else 2), (m, nu)
    assert lib.nngp_resolve_algo_nu(2, 15, 5, 2, 1.5) == 2 and lib.nngp_resolve_algo_nu(0, 15, 0, 2, 1.5) == 5


def test_finalize_checks_workspace(lib):
    P = ctypes.c_void_p
    need = lib.nngp_bf_sweep_workspace_bytes(100_000, 15, 0, 2, 0)
    assert lib.nngp_bf_finalize(P(256), need - 256, 100_000, 15, 0, 2, 0, P(512), None) == -1
    assert "smaller" in lib.nngp_last_error().decode()
    assert lib.nngp_bf_finalize(P(256), need, 100_000, 15, 9, 2, 0, P(512), None) == -1
    assert lib.nngp_bf_finalize(P(256), need, 100_000, 15, 0, 2, 3, P(512), None) == -1
    assert lib.nngp_bf_finalize(None, need, 100_000, 15, 0, 2, 0, P(512), None) == -1
    # a matern sweep's records depend on nu (pair kernel with its table, or the wavefront kernel): AUTO is refused
    need5 = lib.nngp_bf_sweep_workspace_bytes(100_000, 15, 5, 2, 0)
    assert need5 >= lib.nngp_bf_sweep_workspace_bytes(100_000, 15, 5, 2, 2)
    assert need5 >= lib.nngp_bf_sweep_workspace_bytes(100_000, 15, 5, 2, 5) > need
    assert lib.nngp_bf_finalize(P(256), need5, 100_000, 15, 5, 2, 0, P(512), None) == -1
    assert "resolved algo" in lib.nngp_last_error().decode()


def test_blocks_entry_points_reject(lib):
    """Covariance-block sweeps (a caller's own covariance): argument checks without a GPU."""
    P = ctypes.c_void_p
    assert lib.nngp_joint_entries(15) == 136 and lib.nngp_joint_entries(0) == 1
    # enough for the two-lane kernel's tile records (m <= 24) and the four-lane kernel's block records (25..32)
    need = lib.nngp_bf_sweep_blocks_workspace_bytes(1_000_000)
    assert need == max(lib.nngp_bf_sweep_workspace_bytes(1_000_000, 15, 0, 2, 5),
                       lib.nngp_bf_sweep_workspace_bytes(1_000_000, 28, 0, 2, 4))
    args = lambda **kw: [kw.get("cov", P(256)), P(256), None, 10, 10, kw.get("m", 15), 0, 10, None, None, None, None,  # noqa: E731
                         None, P(256), P(256), 1 << 20, None]
    assert lib.nngp_bf_sweep_blocks(*args(m=33)) == -4
    assert "m <= 32" in lib.nngp_last_error().decode()
    assert lib.nngp_bf_sweep_blocks(*args(m=0)) == -4
    assert lib.nngp_abi_version() == 4 and b"0.4.0" in lib.nngp_version()
    assert lib.nngp_bf_sweep_blocks(*args(cov=None)) == -1
    assert lib.nngp_joint_dist(P(256), 10, 4, P(256), 10, P(256), None, 10, 5, 0, P(256), None) == -4
    assert lib.nngp_joint_dist(P(256), 10, 2, P(256), 10, P(256), None, 11, 5, 0, P(256), None) == -1



def test_sharded_gibbs_entries_reject(lib):
    """The sharded-chain entries validate before any device call (no GPU here)."""
    P = ctypes.c_void_p
    prep = P(256)
    # prepare_range: rows outside [0, n), null pointers, a short prep buffer
    assert lib.nngp_gibbs_prepare_range(P(8), P(8), P(8), P(8), P(8), 10, 3, 5, 11, prep, 1 << 20, None) == -1
    assert lib.nngp_gibbs_prepare_range(P(8), P(8), P(8), P(8), P(8), 10, 3, 6, 5, prep, 1 << 20, None) == -1
    assert lib.nngp_gibbs_prepare_range(P(8), None, P(8), P(8), P(8), 10, 3, 0, 10, prep, 1 << 20, None) == -1
    assert lib.nngp_gibbs_prepare_range(P(8), P(8), P(8), P(8), P(8), 10, 3, 0, 10, prep, 8, None) == -1
    assert b"prep too small" in lib.nngp_last_error()
    # one colour step: bad sizes, nulls, non-positive variances; zero members is a no-op
    args = (P(16), 4, prep, 10, 3, 1.0, 0.5, P(8), None, P(8), P(8), P(8), None, 0, 0, None, None)
    assert lib.nngp_gibbs_w_color(*args[:1], 11, *args[2:]) == -1
    assert lib.nngp_gibbs_w_color(*args[:5], 0.0, *args[6:]) == -1
    assert lib.nngp_gibbs_w_color(None, *args[1:]) == -1
    assert lib.nngp_gibbs_w_color(*args[:1], 0, *args[2:]) == 0
    # the device-scalar variant needs var and z
    assert lib.nngp_gibbs_w_color_dev(P(16), 4, prep, 10, 3, None, P(8), None, P(8), P(8), P(8), P(8), None,
                                      None) == -1
    assert lib.nngp_gibbs_w_color_dev(P(16), 4, prep, 10, 3, P(8), P(8), None, P(8), P(8), P(8), None, None,
                                      None) == -1
    # replay: misaligned rows, nulls; zero rows is a no-op
    assert lib.nngp_gibbs_w_apply(P(4), 3, P(8), P(8), 10, 3, P(8), P(8), P(8), P(8), None) == -1
    assert lib.nngp_gibbs_w_apply(P(16), 3, None, P(8), 10, 3, P(8), P(8), P(8), P(8), None) == -1
    assert lib.nngp_gibbs_w_apply(P(16), 0, None, None, 10, 3, None, None, None, None, None) == 0


def test_gibbs_chains_entry_points_reject(lib):
    """nngp_gibbs_w_sweep_chains / _il argument checks without a GPU: chain count, null and misaligned pointers."""
    import ctypes

    P = ctypes.c_void_p
    C = 2
    arr = (P * C)(P(256), P(512))
    dbl = (ctypes.c_double * C)(1.0, 1.0)
    off = (ctypes.c_int32 * 2)(0, 10)
    args = lambda chains, w, r: (P(256), off, 1, chains, arr, 10, 5, dbl, dbl, arr, None, w, r, P(256), arr, None)
    assert lib.nngp_gibbs_w_sweep_chains_il(*args(9, P(1024), P(2048))) == -1
    assert "chains" in lib.nngp_last_error().decode()
    assert lib.nngp_gibbs_w_sweep_chains_il(*args(C, None, P(2048))) == -1
    assert lib.nngp_gibbs_w_sweep_chains_il(*args(C, P(1032), P(2048))) == -1
    assert "16-byte" in lib.nngp_last_error().decode()
    assert lib.nngp_gibbs_w_sweep_chains(*args(0, arr, arr)) == -1


def test_gibbs_tiles_entry_point_rejects(lib):
    """nngp_gibbs_w_sweep_tiles validates before any device call: nulls, sizes, the step-entry cap, tinfo
    alignment, phase offsets and LDS, the variances."""
    P = ctypes.c_void_p
    I32 = ctypes.c_int32
    poff = (I32 * 3)(0, 2, 3)
    plds = (I32 * 2)(4096, 8192)

    def call(tiles=P(256), po=poff, pl=plds, n_phases=2, tinfo=P(256), ecap=768, n=10, m=3, n_entries=20,
             sigma2=1.0, tau2=0.5, rev_loc=P(256), w=P(256)):
        return lib.nngp_gibbs_w_sweep_tiles(tiles, po, pl, n_phases, tinfo, P(256), ecap, P(256), P(256), rev_loc,
                                            P(256), n, m, n_entries, sigma2, tau2, P(256), None, w, P(256), P(256),
                                            None)

    assert call(tiles=None) == -1 and "null" in lib.nngp_last_error().decode()
    assert call(w=None) == -1
    assert call(rev_loc=None) == -1  # entries need their local slots
    assert call(n_entries=31) == -1 and "n_entries" in lib.nngp_last_error().decode()  # > n * m
    assert call(m=64) == -1
    assert call(ecap=2049) == -1 and "ecap" in lib.nngp_last_error().decode()
    assert call(tinfo=P(264)) == -1 and "16-byte" in lib.nngp_last_error().decode()
    assert call(po=(I32 * 3)(0, 2, 1)) == -1 and "decrease" in lib.nngp_last_error().decode()
    assert call(pl=(I32 * 2)(4096, 160 * 1024 + 16)) == -1 and "LDS" in lib.nngp_last_error().decode()
    assert call(tau2=0.0) == -1 and "tau2" in lib.nngp_last_error().decode()
    assert call(sigma2=float("inf")) == -1


def test_gibbs_sweep_rejects_negative_colour_offsets(lib):
    """A negative colour offset would index before the member rows: refused before any device call."""
    P = ctypes.c_void_p
    co = (ctypes.c_int32 * 3)(-4, 2, 10)
    assert lib.nngp_gibbs_w_sweep(P(256), co, 2, P(256), 10, 3, 1.0, 0.5, P(256), None, P(256), P(256), P(256),
                                  P(256), 0, 0, None) == -1
    assert "negative colour offset" in lib.nngp_last_error().decode()
