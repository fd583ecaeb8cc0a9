"""GPU: the drop-in NNGP class (mirrors pyNNGP.NNGP, /root/reference/pyNNGP/nngp.py).

Attributes against the reference's own output (tests/golden/knn_ref_*.npz):
Ns (list format, Ns[0] == []), Nt aliasing Ns, s aliasing t, wt a copy of y, ws
the 5-NN uniform regression; per-location _CNs/_Ccross/_Cs/_Bsi/_Fsi and the
whole-field loglik against the oracle.
"""
import numpy as np
import pytest
import torch

from conftest import load_golden

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["knn_ref_n200_m3", "knn_ref_n1000_m10", "knn_ref_n5000_m15"])
def test_constructor_matches_reference(dev, name):
    from pynngp_amd import NNGP

    g = load_golden(name)
    m = int(g["m"])
    model = NNGP(g["coords"], g["y"], np.full_like(g["y"], 1e-3), "S=T", m, None)
    assert model.s is model.t and model.Nt is model.Ns
    np.testing.assert_array_equal(model.wt, g["y"])
    assert model.wt is not model.y
    assert model.Ns[0] == []
    for i in range(1, len(model.Ns)):
        assert model.Ns[i].dtype == np.int64
        np.testing.assert_array_equal(model.Ns[i], g["Ns"][i, : min(i, m)])
    np.testing.assert_allclose(model.ws, g["ws"], rtol=0, atol=1e-15)


def test_reference_test_init_shape(dev):
    """tests/test_init.py: 2-column y and eps, m=3, cov=None; self never a neighbour."""
    from pynngp_amd import NNGP

    rng = np.random.default_rng(0)
    t = rng.uniform(size=(200, 2))
    model = NNGP(t, np.zeros_like(t), np.ones_like(t) * 0.001, "S=T", 3, None)
    for i in range(200):
        assert i not in model.Ns[i]
    assert model.ws.shape == (200, 2)


def test_per_location_methods_vs_oracle(dev, c_oracle):
    from pynngp_amd import NNGP, Covariance

    rng = np.random.default_rng(1)
    t = rng.uniform(size=(800, 2))
    y = rng.standard_normal(800)
    cov = Covariance("matern32", 1.2, 9.0, 0.05)
    model = NNGP(t, y, None, "S=T", 12, cov)
    nbr = model.nbr.cpu().numpy()
    np.testing.assert_array_equal(nbr, c_oracle.c_knn_prior(t, 12))
    for i in [0, 1, 5, 12, 13, 400, 799]:
        CN, c, Cii = c_oracle.location_blocks(t, nbr[i], i, "matern32", cov.theta)
        np.testing.assert_allclose(model._CNs(i), CN, rtol=1e-13, atol=1e-15)
        np.testing.assert_allclose(model._Ccross(i)[0], c, rtol=1e-13, atol=1e-15)
        assert abs(float(np.asarray(model._Cs(i)).ravel()[0]) - Cii) < 1e-14
        Bo, Fo = c_oracle.bf_location(t, nbr[i], i, "matern32", cov.theta)
        np.testing.assert_allclose(model._Bsi(i), Bo, rtol=0, atol=1e-10)
        assert abs(model._Fsi(i) - Fo) <= 1e-10 * Fo
    B, F = model.compute_BF()
    Bo, Fo, po = c_oracle.c_bf_sweep(t, nbr, "matern32", cov.theta, y)
    np.testing.assert_allclose(F.cpu().numpy(), Fo, rtol=1e-10)
    ll = model.loglik()
    want = c_oracle.loglik_from_partials(po, 800)
    assert abs(ll - want) <= 1e-12 * abs(want)
    ll2 = model.loglik(cov=cov.replace(phi=4.0))
    _, _, p2 = c_oracle.c_bf_sweep(t, nbr, "matern32", (1.2, 4.0, 0.05), y)
    assert abs(ll2 - c_oracle.loglik_from_partials(p2, 800)) <= 1e-12 * abs(ll2)


def test_callable_cov_and_errors(dev):
    from pynngp_amd import NNGP, Covariance, NNGPNumericalError

    rng = np.random.default_rng(2)
    t = rng.uniform(size=(100, 2))
    y = rng.standard_normal(100)

    def user_cov(a, b):
        d = np.sqrt(((a[:, None, :] - b[None, :, :]) ** 2).sum(-1))
        return 2.0 * np.exp(-3.0 * d)

    model = NNGP(t, y, None, "S=T", 4, user_cov)
    assert model._CNs(10).shape == (4, 4)
    # the plug-in drives the device sweep (CallableCovariance -> nngp_bf_sweep_blocks)
    from oracle import nngp_oracle as O

    Bo, Fo, po = O.bf_sweep_callable(t, model.nbr.cpu().numpy(), user_cov, y)
    np.testing.assert_allclose(model._Bsi(10), Bo[10], rtol=0, atol=1e-10)
    assert abs(model._Fsi(10) - Fo[10]) <= 1e-10 * Fo[10]
    assert abs(model.loglik() - O.loglik_from_partials(po, 100)) <= 1e-12 * abs(O.loglik_from_partials(po, 100))
    smp = model.oneSample(seed=1)  # the sampler with the plug-in held fixed (w, tau2, beta; round 5)
    assert smp.kind == "custom" and np.all(np.isfinite(model.ws))
    with pytest.raises(TypeError, match="needs a covariance"):
        NNGP(t, y, None, "S=T", 4, None).loglik()
    with pytest.raises(ValueError):
        NNGP(t, y, None, ("grid", 10), 4, None)
    with pytest.raises(ValueError):
        NNGP(t, y, None, "S=X", 4, None)
    bad = t.copy()
    bad[7, 1] = np.nan  # sklearn's KDTree raises on non-finite input too
    with pytest.raises(ValueError, match="NaN or infinity"):
        NNGP(bad, y, None, "S=T", 4, None)
    dup = t.copy()
    model = NNGP(dup, y, None, "S=T", 4, Covariance("exponential", 1.0, 3.0, 0.0))
    nb = model.nbr.clone()
    nb[50, 1] = nb[50, 0]
    model.set_neighbor_sets(nb)
    with pytest.raises(NNGPNumericalError, match="location 50"):
        model.loglik()


def test_knn_prior_rows_matches_ranges(dev):
    from pynngp_amd import _lib

    rng = np.random.default_rng(31)
    c = torch.from_numpy(rng.uniform(size=(20000, 2))).to(dev)
    full = _lib.knn_prior(c, 15)
    rows = torch.from_numpy(np.concatenate([np.arange(20), rng.permutation(20000)[:3000]]).astype(np.int32)).to(dev)
    got = _lib.knn_prior_rows(c, 15, rows)
    assert torch.equal(got, full[rows.long()])


@pytest.mark.parametrize("kind,theta", [("exponential", (1.0, 30.0, 0.0)), ("matern32", (1.0, 17.3, 0.1))])
def test_sharded_storage_layout_equals_natural(dev, kind, theta):
    """Relabelling into Z-order storage changes nothing but the row labels: per-row B / F
    bit-identical, the one-rank partials bit-identical (same visiting order), and the
    shards of a 3-way split sum to the whole."""
    from pynngp_amd import Covariance, ShardedLogLik
    from pynngp_amd.sweep import combine_partials  # noqa: F401

    rng = np.random.default_rng(5)
    n = 60000
    c = torch.from_numpy(rng.uniform(size=(n, 2))).to(dev)
    v = torch.from_numpy(rng.standard_normal(n)).to(dev)
    cov = Covariance(kind, *theta)
    nat = ShardedLogLik(c, 15, layout="natural")
    sto = ShardedLogLik(c, 15, layout="storage")
    pn = nat.partials(cov, v).clone()
    ps = sto.partials(cov, v).clone()
    assert torch.equal(pn, ps)
    rows = sto.rows_input
    assert torch.equal(sto.F, nat.F[rows]) and torch.equal(sto.B, nat.B[rows])
    # storage-order values give the same result
    ps2 = sto.partials(cov, sto.to_storage(v), values_layout="storage")
    assert torch.equal(ps2, ps)
    tot = torch.zeros(2, dtype=torch.float64, device=dev)
    seen = []
    for r in range(3):
        sh = ShardedLogLik(c, 15, rank=r, world=3, layout="storage")
        tot += sh.local_partials(cov, v)[:2]
        seen.append(sh.rows_input)
        assert torch.equal(sh.F, nat.F[sh.rows_input])
    assert torch.equal(torch.sort(torch.cat(seen)).values, torch.arange(n, device=dev))
    assert torch.allclose(tot, pn[:2], rtol=1e-12, atol=0)


def test_one_sample_drop_in(dev):
    """NNGP.oneSample (nngp.py:98-101) runs the Gibbs iteration and updates ws / wt."""
    from pynngp_amd import NNGP, Covariance

    rng = np.random.default_rng(12)
    t = rng.uniform(size=(3000, 2))
    y = np.sin(5 * t[:, 0]) + 0.2 * rng.standard_normal(3000)
    runs = []
    for _ in range(2):
        g = NNGP(t, y, None, "S=T", 10, Covariance("exponential", 1.0, 8.0, 0.05), device=dev)
        ws0 = g.ws.copy()
        for _ in range(5):
            s = g.oneSample(seed=4)
        assert g.ws.shape == (3000,) and np.array_equal(g.wt, g.ws) and not np.array_equal(g.ws, ws0)
        assert s.iteration == 5 and np.isfinite(s.sigma2) and np.isfinite(s.tau2)
        runs.append(g.ws)
    np.testing.assert_array_equal(runs[0], runs[1])  # bit-reproducible chain
    assert np.corrcoef(runs[0], y)[0, 1] > 0.5


def test_profile_loglik_and_fit(dev, c_oracle):
    """profile_loglik equals the oracle's log density of y - mu at the GLS mu (found by
    brute force over mu); fit() recovers the parameters of a simulated field."""
    from pynngp_amd import NNGP, Covariance

    rng = np.random.default_rng(17)
    n = 1500
    t = rng.uniform(size=(n, 2))
    d = np.sqrt(((t[:, None, :] - t[None, :, :]) ** 2).sum(-1))
    sigma2, phi, tau2, mu = 1.5, 8.0, 0.2, 3.0
    L = np.linalg.cholesky(sigma2 * np.exp(-phi * d) + tau2 * np.eye(n))
    y = mu + L @ rng.standard_normal(n)
    cov = Covariance("exponential", 1.0, 5.0, 0.1)
    g = NNGP(t, y, None, "S=T", 15, cov, device=dev)
    ll, mu_hat = g.profile_loglik(cov)
    nbr = g.nbr.cpu().numpy()
    _, _, p = c_oracle.c_bf_sweep(t, nbr, "exponential", cov.theta, y - mu_hat)
    assert abs(ll - c_oracle.loglik_from_partials(p, n)) <= 1e-10 * abs(ll)
    for dm in (-1e-3, 1e-3):  # mu_hat maximises the log-likelihood
        _, _, p2 = c_oracle.c_bf_sweep(t, nbr, "exponential", cov.theta, y - mu_hat - dm)
        assert c_oracle.loglik_from_partials(p2, n) < ll
    res = g.fit()
    s2, ph, t2 = res["theta"]
    assert res["loglik"] >= ll
    assert abs(res["mu"] - mu) < 1.0 and 0.5 < s2 / sigma2 < 2.0 and 0.4 < ph / phi < 2.5 and 0.3 < t2 / tau2 < 3.0
    assert g.cov.theta == res["theta"]


def _splitmix_uniforms(seed, count):
    """The SplitMix64 stream of examples/capi_demo.c as numpy uniforms in [0, 1)."""
    with np.errstate(over="ignore"):
        k = np.arange(1, count + 1, dtype=np.uint64)
        z = np.uint64(seed) + k * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z ^= z >> np.uint64(31)
    return (z >> np.uint64(11)).astype(np.float64) * 2.0 ** -53


def test_capi_demo_plain_c_caller(dev, c_oracle):
    """A plain C program (examples/capi_demo.c, built by build()) drives the C ABI with
    hipMalloc'd buffers -- no Python, no torch -- and gets the oracle's log-likelihood."""
    import os
    import subprocess

    from pynngp_amd import _lib

    exe = os.path.join(os.path.dirname(_lib.LIB_PATH), "capi_demo")
    assert os.path.exists(exe), "capi_demo not built (make -C pynngp_amd/csrc)"
    n, m, seed = 20000, 15, 5
    out = subprocess.run([exe, str(n), str(m), str(seed)], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr
    f = out.stdout.split()
    ll, first_bad, F_last = float(f[1]), int(f[3]), float(f[5])
    u = _splitmix_uniforms(seed, 2 * n + 2 * n)
    coords = u[: 2 * n].reshape(n, 2)
    u1, u2 = u[2 * n::2] + 2.0 ** -54, u[2 * n + 1::2]
    v = np.sqrt(-2.0 * np.log(u1)) * np.cos(6.283185307179586 * u2)
    nbr = c_oracle.c_knn_prior(coords, m)
    _, Fo, po = c_oracle.c_bf_sweep(coords, nbr, "exponential", (1.0, 30.0, 0.1), v)
    llo = c_oracle.loglik_from_partials(po, n)
    assert first_bad == -1
    assert abs(F_last - Fo[-1]) <= 1e-10 * Fo[-1]
    assert abs(ll - llo) <= 1e-9 * abs(llo), (ll, llo)


def test_loglik_scan_matches_single_calls(dev):
    """ShardedLogLik.loglik_scan (pipelined sweeps, one host sync) equals one loglik call per theta."""
    from pynngp_amd import Covariance, ShardedLogLik

    rng = np.random.default_rng(23)
    n = 50000
    c = torch.from_numpy(rng.uniform(size=(n, 2))).to(dev)
    v = torch.from_numpy(rng.standard_normal(n)).to(dev)
    for layout in ("natural", "storage"):
        sh = ShardedLogLik(c, 15, layout=layout)
        covs = [Covariance("exponential", 1.0, phi, 0.1) for phi in (5.0, 10.0, 20.0, 40.0)]
        scan = sh.loglik_scan(covs, v)
        single = [sh.loglik(cv, v) for cv in covs]
        assert scan == single
