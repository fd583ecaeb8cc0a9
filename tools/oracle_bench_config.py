"""The bench's own sweep at one rank against the C oracle (for the N-rank rehearsals):

    python tools/oracle_bench_config.py --config 4      (N = 1e7, m = 20, exponential, storage layout)

Builds exactly bench.py's workload (synth(seed 0), ShardedLogLik world 1, storage layout), runs one GPU sweep
and oracle/nngp_oracle.c's c_bf_sweep on the same coordinates / neighbour rows / values (storage order), and
prints one JSON line with both log-likelihoods and their relative difference -- the reference value an N-rank
rehearsal's log-likelihood (bench.py --rehearse-on-one-gpu) is compared with."""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=4, choices=[2, 3, 4])
    a = ap.parse_args()
    import bench
    from oracle import nngp_oracle as O
    from pynngp_amd import Covariance, ShardedLogLik

    n, m, kind, theta = {2: (100_000, 15, "matern32", (1.0, 17.320508075688772, 0.1)),
                         3: (1_000_000, 15, "exponential", (1.0, 30.0, 0.0)),
                         4: (10_000_000, 20, "exponential", (1.0, 30.0, 0.0))}[a.config]
    dev = torch.device("cuda", 0)
    coords, values = bench.synth(n, seed=0)
    c = torch.from_numpy(coords).to(dev)
    v = torch.from_numpy(values).to(dev)
    sw = ShardedLogLik(c, m, 0, 1, layout="storage")
    p = sw.partials(Covariance(kind, *theta), v, True, "storage").cpu().numpy()
    ll = -0.5 * (n * np.log(2 * np.pi) + p[0] + p[1])
    _, _, po = O.c_bf_sweep(sw._coords_sweep.cpu().numpy(), sw.nbr.cpu().numpy(), kind, theta, values, want_bf=False)
    llo = O.loglik_from_partials(po, n)
    print(json.dumps({"config": a.config, "n": n, "m": m, "loglik_gpu": float(ll), "loglik_oracle": float(llo),
                      "rel_diff": float(abs(ll - llo) / abs(llo))}))


if __name__ == "__main__":
    main()
