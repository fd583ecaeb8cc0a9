"""Time nngp_gibbs_prepare (the per-accepted-phi fold of B / Ft into reverse-list order) at N = 1e6,
m = 15 with HIP events; prints one JSON line.  (A/B of prepare variants via NNGP_LIB.)"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pynngp_amd import _lib  # noqa: E402

dev = torch.device("cuda", 0)
rng = np.random.default_rng(0)
n, m = 1_000_000, 15
c = torch.from_numpy(rng.uniform(0, 1, (n, 2))).to(dev)
order, _ = _lib.row_order(c)
c = c[order.long()].contiguous()
nbr = _lib.knn_prior(c, m)
B, F, _ = _lib.bf_sweep(c, nbr, 0, "exponential", 1.0, 30.0, 0.0)
off, rev_j, rev_k = _lib.reverse_neighbors(nbr)
prep = _lib.gibbs_prepare(B, F, off, rev_j, rev_k)
ref = prep.clone()
for _ in range(20):
    _lib.gibbs_prepare(B, F, off, rev_j, rev_k, prep=prep)
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(50)]
for a, b in ev:
    a.record()
    _lib.gibbs_prepare(B, F, off, rev_j, rev_k, prep=prep)
    b.record()
torch.cuda.synchronize()
print(json.dumps({"prepare_ms": float(np.median([a.elapsed_time(b) for a, b in ev])),
                  "bit_identical_to_first": bool(torch.equal(prep, ref)), "lib": _lib.LIB_PATH}))
