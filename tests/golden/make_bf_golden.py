"""B/F/log-lik golden vectors.

The reference's B/F methods are stubs (pyNNGP/nngp.py:73-90), so these vectors
come from the numpy oracle (oracle/nngp_oracle.py, pinned by the known-answer
tests in tests/test_oracle.py) evaluated on the REFERENCE-produced neighbour
sets of tests/golden/knn_ref_*.npz.  They freeze the oracle's output so later
rounds can detect drift without rerunning anything.

    python tests/golden/make_bf_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import nngp_oracle as O  # noqa: E402


def make(src, name, kind, theta, n):
    with np.load(os.path.join(HERE, src + ".npz"), allow_pickle=False) as z:
        coords, Ns, y = z["coords"][:n], z["Ns"][:n], z["y"][:n]
    B, F, p = O.bf_sweep(coords, Ns, kind, theta, y)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), coords=coords, Ns=Ns, y=y, kind=np.str_(kind),
                        theta=np.array(theta), B=B, F=F, loglik=np.float64(O.loglik_from_partials(p, n)))
    print(name, O.loglik_from_partials(p, n))


if __name__ == "__main__":
    make("knn_ref_n1000_m10", "bf_golden_n1000_m10_exp", "exponential", (1.0, 30.0, 0.0), 1000)
    make("knn_ref_n5000_m15", "bf_golden_n2000_m15_matern32", "matern32", (1.0, 17.320508075688772, 0.1), 2000)
