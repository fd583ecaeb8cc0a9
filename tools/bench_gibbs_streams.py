"""Several independent Gibbs chains on ONE GPU, each on its own HIP stream and host thread
(BASELINE config 5's replica mode, more chains per GPU): does a second chain fill the colour
steps' launch floors and the host synchronisations of the first?

    python tools/bench_gibbs_streams.py [--n 1000000 --m 15 --iters 300 --warmup 100 --chains 1 2 3]

For each C: C SeqNNGP chains (seeds 1..C) on C torch streams, one Python thread per chain (the
GIL is released while a thread waits on its stream and inside the ctypes / operator calls);
prints one JSON line per C with chain-iterations/s.
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pynngp_amd import SeqNNGP  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=1_000_000)
ap.add_argument("--m", type=int, default=15)
ap.add_argument("--iters", type=int, default=300)
ap.add_argument("--warmup", type=int, default=100)
ap.add_argument("--chains", type=int, nargs="+", default=[1, 2, 3])
args = ap.parse_args()
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
rng = np.random.default_rng(2)
coords = rng.uniform(0, 1, (args.n, 2))
y = 1.0 + rng.standard_normal(args.n) * 0.5 + 0.3 * rng.standard_normal(args.n)

for C in args.chains:
    streams = [torch.cuda.Stream(dev) for _ in range(C)]
    chains = []
    for k in range(C):
        with torch.cuda.stream(streams[k]):
            chains.append(SeqNNGP(coords, y, m=args.m, sigma2=1.0, tau2=0.1, phi=30.0, seed=1 + k, device=dev))
    torch.cuda.synchronize()

    def run(k, iters):
        with torch.cuda.stream(streams[k]):
            for _ in range(iters):
                chains[k].step()
        streams[k].synchronize()

    def all_chains(iters):
        th = [threading.Thread(target=run, args=(k, iters)) for k in range(C)]
        for t in th:
            t.start()
        for t in th:
            t.join()

    all_chains(args.warmup)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    all_chains(args.iters)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print(json.dumps({"chains": C, "n": args.n, "m": args.m, "iters": args.iters,
                      "chain_iters_per_s": C * args.iters / el, "ms_per_iter_per_chain": 1e3 * el / args.iters,
                      "accept": [c.n_accept / max(1, c.iteration) for c in chains]}), flush=True)
    del chains
    torch.cuda.empty_cache()
