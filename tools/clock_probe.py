"""Is the slow start of a bench run the GPU clock or the memory system?  (diagnostic, not a bench)

    python tools/clock_probe.py [--preheat-ms 0] [--sweeps 300]

Times every one of the first --sweeps config-3 sweeps (N = 1e6, m = 15, exponential, storage
layout) with HIP events on the sweep's stream and prints the per-sweep kernel times in groups.
With --preheat-ms T the GPU first runs T ms of fp64 GEMMs on data the sweep never touches: if the
early sweeps then run at the settled speed, the slow start is the clock ramping under load (DVFS),
not cold caches / TLBs of the sweep's own working set.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pynngp_amd import Covariance  # noqa: E402
from pynngp_amd.sweep import ShardedLogLik  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--preheat-ms", type=float, default=0.0)
ap.add_argument("--sweeps", type=int, default=300)
args = ap.parse_args()
dev = torch.device("cuda", 0)
rng = np.random.default_rng(0)
n = 1_000_000
coords = torch.from_numpy(rng.uniform(0, 1, (n, 2))).to(dev)
values = torch.from_numpy(rng.standard_normal(n)).to(dev)
sw = ShardedLogLik(coords, 15, layout="storage")
cov = Covariance("exponential", 1.0, 30.0, 0.0)
vs = sw.to_storage(values)
torch.cuda.synchronize()
time.sleep(1.0)  # let the clock fall back after the setup work
if args.preheat_ms > 0:
    a = torch.randn(4096, 4096, dtype=torch.float64, device=dev)
    b = torch.randn(4096, 4096, dtype=torch.float64, device=dev)
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < args.preheat_ms:
        c = a @ b
        torch.cuda.synchronize()
    del a, b, c
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.sweeps)]
for k in range(args.sweeps):
    ev[k][0].record()
    sw.local_partials(cov, vs, want_bf=True, values_layout="storage")
    ev[k][1].record()
torch.cuda.synchronize()
ms = np.array([s.elapsed_time(e) for s, e in ev])
groups = [(0, 5), (5, 25), (25, 50), (50, 100), (100, 200), (200, args.sweeps)]
print(json.dumps({"preheat_ms": args.preheat_ms,
                  "mean_ms_by_sweep_range": {f"{a}-{b}": float(ms[a:b].mean()) for a, b in groups if b <= args.sweeps},
                  "first10": [round(float(x), 4) for x in ms[:10]]}))
