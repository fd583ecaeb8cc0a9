"""Time the caller-covariance path (IsotropicCovariance: nngp_joint_dist -> fn -> nngp_bf_sweep_blocks)
against the fused kernels at N = 1e6, m = 15 (Z-order visiting order), HIP events; one JSON line."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pynngp_amd import Covariance, IsotropicCovariance, _lib  # noqa: E402

dev = torch.device("cuda", 0)
rng = np.random.default_rng(0)
n, m = 1_000_000, 15
c = torch.from_numpy(rng.uniform(0, 1, (n, 2))).to(dev)
v = torch.from_numpy(rng.standard_normal(n)).to(dev)
nb = _lib.knn_prior(c, m)
order, srt = _lib.row_order(c, 0, n, nb)
out = {}


def timed(fn, reps=20):
    for _ in range(5):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev]))


cov = IsotropicCovariance(lambda d: torch.exp(-30.0 * d), 0.0)
dist = _lib.joint_dist(c, srt, 0, order=order)
blocks = cov.blocks(dist, m)
out["joint_dist_ms"] = timed(lambda: _lib.joint_dist(c, srt, 0, order=order, out=dist))
out["fn_ms"] = timed(lambda: cov.blocks(dist, m))
out["blocks_sweep_ms"] = timed(lambda: _lib.bf_sweep_blocks(blocks, srt, n, 0, values=v, qvalues=v, order=order))
out["fused_exponential_ms"] = timed(lambda: _lib.bf_sweep(c, srt, 0, "exponential", 1.0, 30.0, 0.0, values=v,
                                                          order=order))
mat = Covariance("matern", 1.0, 30.0, 0.0, nu=1.3)
out["fused_matern_nu_ms"] = timed(lambda: _lib.bf_sweep(c, srt, 0, "matern", 1.0, 30.0, 0.0, values=v, order=order,
                                                        nu=1.3), reps=5)
matc = IsotropicCovariance(lambda d: _lib.matern(30.0 * d, 1.3), 0.0)


def custom_matern():
    d = _lib.joint_dist(c, srt, 0, order=order, out=dist)
    return _lib.bf_sweep_blocks(matc.blocks(d, m), srt, n, 0, values=v, qvalues=v, order=order)


out["custom_matern_total_ms"] = timed(custom_matern, reps=5)
out["matern_eval_ms"] = timed(lambda: _lib.matern(dist, 1.3), reps=5)
_, _, p1 = _lib.bf_sweep_blocks(blocks, srt, n, 0, values=v, qvalues=v, order=order)
_, _, p2 = _lib.bf_sweep(c, srt, 0, "exponential", 1.0, 30.0, 0.0, values=v, order=order)
out["loglik_blocks"] = float(-0.5 * (n * np.log(2 * np.pi) + p1[0].item() + p1[1].item()))
out["loglik_fused"] = float(-0.5 * (n * np.log(2 * np.pi) + p2[0].item() + p2[1].item()))
print(json.dumps(out))
