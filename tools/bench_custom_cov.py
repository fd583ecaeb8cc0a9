"""Time the caller-covariance paths against the fused kernels at N = 1e6, m = 15 (Z-order visiting order),
HIP events; one JSON line: IsotropicCovariance (nngp_joint_dist -> fn -> nngp_bf_sweep_blocks) and, round 4,
CallableCovariance (a reference-style cov(a, b) -- here an anisotropic exponential in torch, batched on the
GPU -- on every joint block's coordinate rows -> nngp_bf_sweep_blocks), the fused Matern-nu kind (the pair
kernel's table) and the m = 28 blocks path (four-lane kernel)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pynngp_amd import CallableCovariance, Covariance, IsotropicCovariance, _lib  # noqa: E402

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
A = (400.0, 150.0, 100.0)


def aniso(a, b):  # a reference-style plug-in: cross-covariance of two row sets, broadcasting over leading dims
    t = a[..., :, None, :] - b[..., None, :, :]
    q = A[0] * t[..., 0] ** 2 + 2.0 * A[1] * t[..., 0] * t[..., 1] + A[2] * t[..., 1] ** 2
    return 1.4 * torch.exp(-torch.sqrt(q))


cc = CallableCovariance(aniso, tau2=0.05, pairs=True)
cblk = cc.blocks(c, srt, 0, order=order)
out["callable_mode"] = cc.mode
out["callable_blocks_ms"] = timed(lambda: cc.blocks(c, srt, 0, order=order), reps=5)
out["callable_distinct_pairs"] = int(cc._pidx[1][0].numel()) if cc._pidx is not None else None
out["callable_block_entries"] = int(srt.shape[0] * (srt.shape[1] + 1) * (srt.shape[1] + 2) // 2)
cc_blocks = CallableCovariance(aniso, tau2=0.05, pairs=False)
out["callable_blocks_per_entry_ms"] = timed(lambda: cc_blocks.blocks(c, srt, 0, order=order), reps=5)
cc_fresh = CallableCovariance(aniso, tau2=0.05, pairs=True)
import time as _t  # noqa: E402
_ph = {}
_x = c[cc._pidx[1][0][:1]] if cc._pidx is not None else None
torch.cuda.synchronize()
_t0 = _t.perf_counter()
for _ in range(3):
    pa_, pb_, inv_ = cc._pidx[1]
    _v = aniso(c[pa_][:, None, :], c[pb_][:, None, :])
torch.cuda.synchronize()
out["callable_pairs_fn_ms"] = (_t.perf_counter() - _t0) / 3 * 1e3
_vals = torch.zeros(pa_.numel() + 1, dtype=torch.float64, device=c.device)
torch.cuda.synchronize()
_t0 = _t.perf_counter()
for _ in range(3):
    _o = _vals[inv_.reshape(-1)]
torch.cuda.synchronize()
out["callable_pairs_gather_ms"] = (_t.perf_counter() - _t0) / 3 * 1e3
del _o, _v, _vals
out["callable_pair_index_build_ms"] = timed(lambda: (setattr(cc_fresh, "_pidx", None),
                                                     cc_fresh.blocks(c, srt, 0, order=order)), reps=3)
out["callable_sweep_ms"] = timed(lambda: _lib.bf_sweep_blocks(cblk, srt, n, 0, values=v, qvalues=v, order=order))
del cblk
nb28 = _lib.knn_prior(c, 28)
o28, s28 = _lib.row_order(c, 0, n, nb28)
d28 = _lib.joint_dist(c, s28, 0, order=o28)
b28 = cov.blocks(d28, 28)
del d28
out["blocks_sweep_m28_ms"] = timed(lambda: _lib.bf_sweep_blocks(b28, s28, n, 0, values=v, qvalues=v, order=o28), reps=5)
out["fused_exponential_m28_ms"] = timed(lambda: _lib.bf_sweep(c, s28, 0, "exponential", 1.0, 30.0, 0.0, values=v,
                                                              order=o28), reps=5)
del b28
_, _, p1 = _lib.bf_sweep_blocks(blocks, srt, n, 0, values=v, qvalues=v, order=order)
_, _, p2 = _lib.bf_sweep(c, srt, 0, "exponential", 1.0, 30.0, 0.0, values=v, order=order)
out["loglik_blocks"] = float(-0.5 * (n * np.log(2 * np.pi) + p1[0].item() + p1[1].item()))
out["loglik_fused"] = float(-0.5 * (n * np.log(2 * np.pi) + p2[0].item() + p2[1].item()))
print(json.dumps(out))
