"""Neighbour-set build timing (row A1: nngp_knn_prior) at N points, m neighbours, one GPU.

Prints one JSON line: mean ms over `reps` calls (HIP events; first call excluded: code
object load and workspace allocation).
    python tools/bench_knn.py [--n 1000000 --m 15 --reps 5 --dim 2]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pynngp_amd import _lib  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=1_000_000)
ap.add_argument("--m", type=int, default=15)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--dim", type=int, default=2, choices=[1, 2, 3])
args = ap.parse_args()
dev = torch.device("cuda", 0)
c = torch.from_numpy(np.random.default_rng(0).uniform(0, 1, (args.n, args.dim))).to(dev)
nb = _lib.knn_prior(c, args.m)
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ts = []
for _ in range(args.reps):
    a.record()
    nb2 = _lib.knn_prior(c, args.m)
    b.record()
    torch.cuda.synchronize()
    ts.append(a.elapsed_time(b))
print(json.dumps({"n": args.n, "m": args.m, "dim": args.dim, "ms": float(np.mean(ts)), "min_ms": float(np.min(ts)),
                  "identical_across_calls": bool(torch.equal(nb, nb2))}))
