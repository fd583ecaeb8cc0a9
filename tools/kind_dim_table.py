"""Sweep time for every covariance kind and ordinate dimension (N = 1e6, m = 15, Z-order).

One JSON line per (kind, dim): mean time of the fused B/F + log-lik sweep from HIP events
after a clock-settling run, plus the neighbour-build time.  DESIGN.md 6.
    python tools/kind_dim_table.py [--n 1000000] [--m 15]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pynngp_amd import _lib  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=1_000_000)
ap.add_argument("--m", type=int, default=15)
ap.add_argument("--reps", type=int, default=50)
args = ap.parse_args()
dev = torch.device("cuda", 0)
THETA = {"exponential": (1.0, 30.0, 0.0), "matern32": (1.0, 17.320508075688772, 0.1),
         "matern52": (1.0, 15.0, 0.1), "gaussian": (1.0, 10.0, 0.1), "spherical": (1.0, 8.0, 0.1)}
for dim in (1, 2, 3):
    rng = np.random.default_rng(dim)
    c = torch.from_numpy(rng.uniform(0, 1, (args.n, dim))).to(dev)
    v = torch.from_numpy(rng.standard_normal(args.n)).to(dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    nb = _lib.knn_prior(c, args.m)
    torch.cuda.synchronize()
    knn_ms = (time.perf_counter() - t0) * 1e3
    order, srt = _lib.row_order(c, 0, args.n, nb)
    B = torch.empty((args.n, args.m), dtype=torch.float64, device=dev)
    F = torch.empty((args.n,), dtype=torch.float64, device=dev)
    for kind, theta in THETA.items():
        ws = _lib.bf_workspace(args.n, args.m, "auto", dev, kind=kind, dim=dim)

        def run():
            _lib.bf_sweep(c, srt, 0, kind, *theta, values=v, B=B, F=F, workspace=ws, order=order)

        t_end = time.perf_counter() + 0.08  # clock settling
        while time.perf_counter() < t_end:
            for _ in range(10):
                run()
            torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            run()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.reps
        print(json.dumps({"dim": dim, "kind": kind, "m": args.m, "n": args.n, "sweep_ms": round(ms, 5),
                          "gloc_s": round(args.n / ms / 1e6, 4), "knn_ms": round(knn_ms, 2)}), flush=True)
