"""The native operator library loads without a GPU and registers every torch.ops.nngp
operator with its schema; CPU tensors are refused (there is no CPU implementation)."""
import pytest
import torch

OPS = ["knn_prior", "knn_prior_rows", "knn_query", "bf_sweep", "bf_sweep_out", "bf_cross", "row_order",
       "combine_partials_out", "pair_plan"]


def test_op_library_registers_all_ops():
    from pynngp_amd import load_ops

    ops = load_ops()
    for name in OPS:
        assert hasattr(torch.ops.nngp, name), name
    schema = str(torch.ops.nngp.bf_sweep_out.default._schema)
    assert "Tensor(a!)? B" in schema and "Tensor(d!) partials" in schema and "Tensor? plan=None" in schema
    assert ops.kind_code("gaussian") == 3 and ops.algo_code("pairb") >= 0
    with pytest.raises(ValueError):
        ops.kind_code("cauchy")


def test_ops_refuse_cpu_tensors():
    from pynngp_amd import load_ops

    load_ops()
    c = torch.rand((50, 2), dtype=torch.float64)
    with pytest.raises(NotImplementedError):
        torch.ops.nngp.knn_prior(c, 4, 0, 50)
    with pytest.raises(NotImplementedError):
        torch.ops.nngp.bf_sweep(c, torch.zeros((50, 4), dtype=torch.int32), 0, 0, 1.0, 5.0, 0.0, None, False, 0)
    with pytest.raises(NotImplementedError):
        torch.ops.nngp.pair_plan(torch.zeros((50, 4), dtype=torch.int32), None, 0, 50, 2)


def test_config1_needs_the_gpu():
    """BASELINE config 1 (N = 10^3, the reference's CPU-sized case) runs on the GPU like every
    other config -- the product has no CPU path (a CPU result would come from code the GPU tests do not
    exercise); without a GPU the drop-in class raises instead of computing."""
    import numpy as np

    from pynngp_amd import NNGP, _lib

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    t = np.random.default_rng(0).uniform(size=(1000, 2))
    with pytest.raises(_lib.NNGPExtensionError, match="needs a ROCm GPU"):
        NNGP(t, np.zeros(1000), None, "S=T", 10, None)


def test_fake_kernels_trace_shapes():
    from torch._subclasses.fake_tensor import FakeTensorMode

    from pynngp_amd import load_ops

    load_ops()
    with FakeTensorMode():
        c = torch.empty((64, 3), dtype=torch.float64)
        nb = torch.ops.nngp.knn_prior(c, 6, 0, 64)
        B, F, p = torch.ops.nngp.bf_sweep(c, nb, 0, 1, 1.0, 5.0, 0.0, None, True, 0)
        o, s = torch.ops.nngp.row_order(c, 0, 64, nb)
    assert tuple(nb.shape) == (64, 6) and nb.dtype == torch.int32
    assert tuple(B.shape) == (64, 6) and tuple(F.shape) == (64,) and tuple(p.shape) == (4,)
    assert tuple(o.shape) == (64,) and tuple(s.shape) == (64, 6)


def test_bf_sweep_blocks_checks_lengths_before_any_device_call():
    """nngp_bf_sweep_blocks takes raw pointers: the binding checks every length first (values (n_points,),
    qvalues (n_locs,), order int32 (rows,)), so a short array can never reach the kernel."""
    import pytest as _pytest
    import torch as _torch

    from pynngp_amd import _lib

    m, rows, n = 4, 10, 12
    cov = _torch.zeros((m + 1) * (m + 2) // 2, rows, dtype=_torch.float64)
    nbr = _torch.zeros(rows, m, dtype=_torch.int32)
    bad = [dict(values=_torch.zeros(n - 1, dtype=_torch.float64)),
           dict(qvalues=_torch.zeros(n + 1, dtype=_torch.float64)),
           dict(order=_torch.zeros(rows, dtype=_torch.int64)),
           dict(order=_torch.zeros(rows - 1, dtype=_torch.int32))]
    for kw in bad:
        with _pytest.raises(ValueError):
            _lib.bf_sweep_blocks(cov, nbr, n, **kw)
    with _pytest.raises(ValueError):
        _lib.bf_sweep_blocks(cov[:-1], nbr, n)
    # well-formed CPU tensors reach the device check (no CPU path)
    with _pytest.raises(_lib.NNGPExtensionError):
        _lib.bf_sweep_blocks(cov, nbr, n, values=_torch.zeros(n, dtype=_torch.float64))
