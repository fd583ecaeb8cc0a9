"""Inputs whose neighbour order depends on FMA contraction of the squared distance.

sklearn orders neighbours by rdist = (0 + t0*t0) + t1*t1 (+ t2*t2 ...) computed with
separate multiplies and adds (sklearn/metrics/_dist_metrics.pxd:26-40, no FMA in the
x86-64 wheel).  A compiler that contracts the sum into fused multiply-adds rounds
differently, and on near-ties that reorders two candidates.

Construction: a cluster is (p1, p2, q) in index order with q - p1 = a e_u + b e_v and
q - p2 = b e_u + a e_v (axes u < v, every other component 0; q and the offsets are
multiples of the largest coordinate's ulp, so q - p is exact).  Unfused, both rdists are fl(fl(a^2) + fl(b^2)):
an exact tie, so q's nearest prior point is p1 (lower index).  Fused, the two sums
round differently; (a, b) are drawn so that fl(a^2 + fl(b^2)) > fl(b^2 + fl(a^2)).
Clusters of type A (p1 gets (a, b)) then flip when the u-term is the fused one, type B
(the roles swapped) when it is the v-term: a kernel that contracts either way picks
p2 on half of the clusters.  Exact fused results use rational arithmetic
(float(Fraction) rounds correctly).
"""
from fractions import Fraction

import numpy as np

def _fused(x, y):
    """fl(x^2 + fl(y^2)): y^2 rounded, x^2 fused."""
    return float(Fraction(x) * Fraction(x) + Fraction(y * y))


def fma_sensitive_clusters(n_clusters, dim=2, seed=0, spacing=8.0):
    """(coords (3 n_clusters, dim), expected m=1 nearest prior of every q: its p1).

    Cluster c occupies rows 3c, 3c+1, 3c+2 = (p1, p2, q); clusters sit `spacing` apart,
    so q's candidates are p1 and p2, tied under the unfused rdist."""
    if dim < 2:
        raise ValueError("a one-term rdist has no addition to contract (dim >= 2)")
    rng = np.random.default_rng(seed)
    side = int(np.ceil(n_clusters ** (1.0 / dim)))
    axes = [(u, v) for u in range(dim) for v in range(u + 1, dim)]
    # quantum: the ulp of the largest coordinate, so q - t and q - p are exact
    top = 4.0 + side * spacing + 1.0
    quantum = 2.0 ** (int(np.ceil(np.log2(top))) - 52)
    pts = []
    c = 0
    while c < n_clusters:
        a = np.floor(rng.uniform(0.3, 1.0) / quantum) * quantum
        b = np.floor(rng.uniform(0.3, 1.0) / quantum) * quantum
        if not _fused(a, b) > _fused(b, a):
            continue
        assert (0.0 + a * a) + b * b == (0.0 + b * b) + a * a
        u, v = axes[c % len(axes)]
        cell = np.array([(c // side ** k) % side for k in range(dim)], dtype=np.float64)
        q = 4.0 + cell * spacing + np.floor(rng.uniform(0.0, 1.0, dim) / quantum) * quantum
        t1 = np.zeros(dim)
        t2 = np.zeros(dim)
        if (c // len(axes)) % 2 == 0:  # type A
            t1[u], t1[v], t2[u], t2[v] = a, b, b, a
        else:  # type B
            t1[u], t1[v], t2[u], t2[v] = b, a, a, b
        p1, p2 = q - t1, q - t2
        assert np.array_equal(q - p1, t1) and np.array_equal(q - p2, t2)
        pts += [p1, p2, q]
        c += 1
    return np.array(pts), np.arange(n_clusters, dtype=np.int32) * 3
