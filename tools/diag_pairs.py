"""Diagnose pairs-mode vs per-entry blocks of a callable covariance (which entries differ)."""
import numpy as np
import torch

from pynngp_amd import CallableCovariance, _lib
from pynngp_amd.nngp import _sweep_any
import sys
sys.path.insert(0, "tests")
from test_gpu_callable_cov import _aniso  # noqa: E402

dev = torch.device("cuda:0")
for m in (15, 27):
    rng = np.random.default_rng(50 + m)
    x = rng.uniform(size=(20_000, 2))
    y = rng.standard_normal(20_000)
    c, v = torch.from_numpy(x).to(dev), torch.from_numpy(y).to(dev)
    nb = _lib.knn_prior(c, m)
    fn = _aniso(1.2, [[90.0, -20.0], [-20.0, 30.0]], 0.05)
    cp, cb = CallableCovariance(fn), CallableCovariance(fn, pairs=False)
    bp, bb = cp.blocks(c, nb, 0), cb.blocks(c, nb, 0)
    a = torch.arange(m + 1)
    ta = torch.repeat_interleave(a, a + 1)
    tb = torch.cat([torch.arange(int(k) + 1) for k in range(m + 1)])
    idx = nb.long().cpu()
    valid = torch.cat([(idx >= 0), torch.ones(idx.shape[0], 1, dtype=torch.bool)], 1)  # (rows, m+1)
    ent_ok = (valid[:, ta] & valid[:, tb]).t().to(dev)  # (ne, rows)
    diff = (bp != bb) & ent_ok
    print("m", m, "pairs_ok", cp._pairs_ok, "differing valid entries", int(diff.sum()), "of", int(ent_ok.sum()))
    if diff.any():
        e, r = torch.nonzero(diff)[0].tolist()
        print("  first: entry", e, "(rows", int(ta[e]), int(tb[e]), ") row", r, "vals", bp[e, r].item(), bb[e, r].item())
    rp = _sweep_any(cp, c, nb, 0, values=v, qvalues=v)
    rb = _sweep_any(cb, c, nb, 0, values=v, qvalues=v)
    print("  results equal:", [torch.equal(p, q) for p, q in zip(rp, rb)])
    if not torch.equal(rp[1], rb[1]):
        d = torch.nonzero(rp[1] != rb[1]).flatten()[:5].tolist()
        print("  F differs at", d, rp[1][d].tolist(), rb[1][d].tolist())
