"""Generate the reference-pinned golden fixtures for the neighbour-set path.

Runs ONLY in the build container (it needs ``/root/reference``, which does not
exist on the GPU box).  It imports the reference package ``pyNNGP`` and runs its
constructor ``NNGP(t, y, eps, 'S=T', m, cov)`` (``pyNNGP/nngp.py:6-18``) on seeded
inputs, then stores what the constructor produced:

* ``Ns``  -- ``_make_s_neighbor_sets`` (``nngp.py:49-62``), padded to int32 (N, m)
  with -1 (row i holds ``min(i, m)`` indices, ascending distance);
* ``ws``  -- ``_init_ws`` (``nngp.py:45-47``), 5-NN uniform regression of y at s;
* ``wt``  -- ``_init_wt`` (``nngp.py:42-43``), a copy of y.

Import shim (recorded in DESIGN.md): ``nngp.py:2`` does
``from past.builtins import basestring``; the ``future`` package is not installed
here, which raises an ordinary ``ModuleNotFoundError``.  The shim registers a
module ``past.builtins`` whose ``basestring`` is ``str`` -- the Python-3 meaning
of ``future``'s alias -- and nothing else.  Bytecode writing is disabled so
nothing is written under the read-only reference tree.

Usage::

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py        # the 2-D fixtures
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py dims   # 1-D and 3-D ordinates
"""
import os
import sys
import types

sys.dont_write_bytecode = True

import numpy as np  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


def _import_reference():
    past = types.ModuleType("past")
    builtins = types.ModuleType("past.builtins")
    builtins.basestring = str
    past.builtins = builtins
    sys.modules.setdefault("past", past)
    sys.modules.setdefault("past.builtins", builtins)
    sys.path.insert(0, REF)
    import pyNNGP  # noqa: WPS433

    return pyNNGP


def _pad(Ns, m):
    n = len(Ns)
    out = np.full((n, m), -1, dtype=np.int32)
    for i, row in enumerate(Ns):
        row = np.asarray(row, dtype=np.int64)
        out[i, : row.size] = row
    return out


def _tie_rows(coords, m):
    """Rows whose (rdist) order has an exact tie that straddles or sits inside the set.

    On such rows the reference order is not a contract (sklearn's heap keeps the
    first-visited point, ``sklearn/utils/_heap.pyx:45-47``; its sort is unstable).
    """
    n = coords.shape[0]
    ties = np.zeros(n, dtype=bool)
    for i in range(1, n):
        t = coords[i][None, :] - coords[:i]
        d = np.zeros(i)
        for k in range(coords.shape[1]):  # sklearn's rdist order, any dimension
            d = d + t[:, k] * t[:, k]
        k = min(m, i)
        srt = np.sort(d)
        # any tie among the first k, or between the k-th and the (k+1)-th
        if np.any(srt[1:k] == srt[: k - 1]) or (k < i and srt[k - 1] == srt[k]):
            ties[i] = True
    return ties


def make_case(pyNNGP, name, coords, y, m):
    eps = np.full_like(y, 1e-3)
    model = pyNNGP.NNGP(coords, y, eps, "S=T", m, None)
    Ns = _pad(model.Ns, m)
    assert model.Nt is model.Ns
    assert model.s is coords
    np.testing.assert_array_equal(model.wt, y)
    out = dict(
        coords=coords,
        y=y,
        m=np.int32(m),
        Ns=Ns,
        ws=np.asarray(model.ws, dtype=np.float64),
        tie_rows=_tie_rows(coords, m),
    )
    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path}: N={coords.shape[0]} m={m} tie_rows={int(out['tie_rows'].sum())}")


def main(only=None):
    pyNNGP = _import_reference()
    if only == "dims":
        # ordinates of dimension 1 and 3 (the reference's KDTree takes any d, nngp.py:55-61)
        rng = np.random.default_rng(43)
        c = rng.uniform(0.0, 1.0, (1000, 3))
        make_case(pyNNGP, "knn_ref_n1000_m10_d3", c, rng.standard_normal(1000), 10)
        rng = np.random.default_rng(44)
        c = rng.uniform(0.0, 1.0, (1000, 1))
        make_case(pyNNGP, "knn_ref_n1000_m8_d1", c, rng.standard_normal(1000), 8)
        return
    # reference test shape (tests/test_init.py:7-17), seeded, scalar y
    rng = np.random.default_rng(7)
    c = rng.uniform(size=(200, 2))
    make_case(pyNNGP, "knn_ref_n200_m3", c, rng.standard_normal(200), 3)
    # BASELINE config 1 (N=1000, m=10) and a m=15 case
    rng = np.random.default_rng(42)
    c = rng.uniform(0.0, 1.0, (1000, 2))
    make_case(pyNNGP, "knn_ref_n1000_m10", c, rng.standard_normal(1000), 10)
    rng = np.random.default_rng(42)
    c = rng.uniform(0.0, 1.0, (5000, 2))
    make_case(pyNNGP, "knn_ref_n5000_m15", c, rng.standard_normal(5000), 15)
    # 6x6 lattice: exact distance ties (reference order on ties is not a contract)
    g = np.arange(6, dtype=np.float64) / 5.0
    c = np.stack(np.meshgrid(g, g, indexing="ij"), -1).reshape(-1, 2).copy()
    make_case(pyNNGP, "knn_ref_lattice6_m4", c, np.linspace(-1.0, 1.0, 36), 4)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else None)
