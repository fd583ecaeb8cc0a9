"""Time the covariance-blocks sweep (nngp_bf_sweep_blocks: an isotropic exponential evaluated by the caller
over nngp_joint_dist's distances) at N = 1e6 for several m (Z-order visiting order), HIP events; one JSON line
with the median ms per sweep and the log-likelihood per m.   python tools/bench_blocks_m.py [m ...]"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pynngp_amd import IsotropicCovariance, _lib  # noqa: E402

dev = torch.device("cuda", 0)
rng = np.random.default_rng(0)
n = 1_000_000
c = torch.from_numpy(rng.uniform(0, 1, (n, 2))).to(dev)
v = torch.from_numpy(rng.standard_normal(n)).to(dev)
cov = IsotropicCovariance(lambda d: torch.exp(-30.0 * d), 0.05)
out = {"lib": os.path.relpath(_lib.LIB_PATH)}
for m in [int(a) for a in sys.argv[1:]] or [18, 20, 22, 24]:
    nb = _lib.knn_prior(c, m)
    order, srt = _lib.row_order(c, 0, n, nb)
    blocks = cov.blocks(_lib.joint_dist(c, srt, 0, order=order), m)
    run = lambda: _lib.bf_sweep_blocks(blocks, srt, n, 0, values=v, qvalues=v, order=order)  # noqa: E731
    for _ in range(5):
        run()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
    for a, b in ev:
        a.record()
        run()
        b.record()
    torch.cuda.synchronize()
    _, _, p = run()
    out[f"m{m}_ms"] = float(np.median([a.elapsed_time(b) for a, b in ev]))
    out[f"m{m}_loglik"] = float(-0.5 * (n * np.log(2 * np.pi) + p[0].item() + p[1].item()))
    del blocks
print(json.dumps(out))
