"""Time every sweep kernel variant for m = 1..20 (N = 1e6, exponential, Z-order) in one process.

Prints one JSON line per (m, algo) with the mean kernel time from HIP events; used
to choose the NNGP_ALGO_AUTO table in pynngp_amd/csrc/capi.hip.
    python tools/algo_table.py [--n 1000000] [--ms 1-20] [--kind exponential]
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
ap.add_argument("--ms", default="1-20")
ap.add_argument("--kind", default="exponential")
ap.add_argument("--reps", type=int, default=10)
args = ap.parse_args()
lo, hi = (int(x) for x in args.ms.split("-"))
dev = torch.device("cuda", 0)
rng = np.random.default_rng(0)
c = torch.from_numpy(rng.uniform(0, 1, (args.n, 2))).to(dev)
v = torch.from_numpy(rng.standard_normal(args.n)).to(dev)
theta = (1.0, 30.0, 0.0) if args.kind == "exponential" else (1.0, 17.320508075688772, 0.1)
for m in range(lo, hi + 1):
    nb = _lib.knn_prior(c, m)
    order, srt = _lib.row_order(c, 0, args.n, nb)
    B = torch.empty((args.n, m), dtype=torch.float64, device=dev)
    F = torch.empty((args.n,), dtype=torch.float64, device=dev)
    algos = ["lane"] if m <= 16 else []
    algos += ["pair"] if 10 <= m <= 20 else []
    algos += ["quad"] if m in (15, 16, 20) else []
    algos += ["pairb"] if 2 <= m <= 20 else []
    algos += ["wave"]
    ref = None
    for algo in algos:
        ws = _lib.bf_workspace(args.n, m, algo, dev)
        for _ in range(2):
            _, _, p = _lib.bf_sweep(c, srt, 0, args.kind, *theta, values=v, algo=algo, B=B, F=F, workspace=ws,
                                    order=order)
        reps = 2 if algo == "wave" else args.reps
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
        for a, b in ev:
            a.record()
            _lib.bf_sweep(c, srt, 0, args.kind, *theta, values=v, algo=algo, B=B, F=F, workspace=ws, order=order)
            b.record()
        torch.cuda.synchronize()
        ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
        Fh = F.cpu().numpy()
        if ref is None:
            ref = Fh
        print(json.dumps({"m": m, "algo": algo, "kernel_ms": round(ms, 5), "gloc_s": round(args.n / ms / 1e6, 4),
                          "max_rel_dF_vs_first": float(np.max(np.abs(Fh - ref) / ref))}), flush=True)
