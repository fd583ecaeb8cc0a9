"""Time every sweep kernel variant for m in a range (N = 1e6, exponential, Z-order) in one process.

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
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--algos", default=None, help="comma-separated subset of kernels to time (default: every one)")
ap.add_argument("--rounds", type=int, default=6)
ap.add_argument("--settle-ms", type=float, default=80.0,
                help="back-to-back sweeps before each m's timing (the GPU clock settles over ~50 ms)")
args = ap.parse_args()
lo, hi = (int(x) for x in args.ms.split("-"))
dev = torch.device("cuda", 0)
rng = np.random.default_rng(0)
c = torch.from_numpy(rng.uniform(0, 1, (args.n, 2))).to(dev)
v = torch.from_numpy(rng.standard_normal(args.n)).to(dev)
theta = (1.0, 30.0, 0.0) if args.kind == "exponential" else (1.0, 17.320508075688772, 0.1)
ap2 = None
for m in range(lo, hi + 1):
    nb = _lib.knn_prior(c, m)
    order, srt = _lib.row_order(c, 0, args.n, nb)
    B = torch.empty((args.n, m), dtype=torch.float64, device=dev)
    F = torch.empty((args.n,), dtype=torch.float64, device=dev)
    algos = ["lane"] if m <= 16 else []
    algos += ["quad"] if 25 <= m <= 32 else []
    algos += ["pairb"] if 1 <= m <= 32 else []
    algos += ["wave"]
    if args.algos:
        algos = [a for a in algos if a in args.algos.split(",")]
    wss = {a: _lib.bf_workspace(args.n, m, a, dev) for a in algos}

    def run(algo):
        _lib.bf_sweep(c, srt, 0, args.kind, *theta, values=v, algo=algo, B=B, F=F, workspace=wss[algo], order=order)

    for a in algos:
        for _ in range(2):
            run(a)
    import time
    t_end = time.perf_counter() + args.settle_ms * 1e-3
    while time.perf_counter() < t_end:
        for _ in range(10):
            run(algos[0])
        torch.cuda.synchronize()
    times = {a: [] for a in algos}
    # interleaved rounds (clock / thermal drift hits every algo alike); median per algo
    for rnd in range(args.rounds):
        for a in algos:
            reps = 1 if a == "wave" else args.reps
            if a == "wave" and rnd > 0:
                continue
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                run(a)
            e1.record()
            torch.cuda.synchronize()
            times[a].append(e0.elapsed_time(e1) / reps)
    ref = None
    for a in algos:
        run(a)
        torch.cuda.synchronize()
        Fh = F.cpu().numpy()
        ref = Fh if ref is None else ref
        ms = float(np.median(times[a]))
        print(json.dumps({"m": m, "algo": a, "kernel_ms": round(ms, 5), "gloc_s": round(args.n / ms / 1e6, 4),
                          "rounds_ms": [round(t, 5) for t in times[a]],
                          "max_rel_dF_vs_first": float(np.max(np.abs(Fh - ref) / ref))}), flush=True)
