"""Covariance-pair reuse inside the sweep's tiles (CPU analysis, no GPU).

    python tools/reuse_stats.py [--n 1000000] [--m 15] [--tile 128]

For a uniform field in generation order (the bench's synthetic input), exact prior kNN (the C
oracle's doubling-prefix kd-tree), relabelled into Z-order storage order as the bench's storage
layout does, and tiles of `tile` consecutive storage rows: per tile, the number of distinct joint
points U (each row's neighbours and itself) and of distinct off-diagonal joint-block pairs, against
the per-row count m(m+1)/2.  Rows with fewer than m neighbours are skipped (their padding pairs are
exact zeros, not evaluations).
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from oracle import nngp_oracle as orc  # noqa: E402  (analysis tool: the oracle's exact kNN)


def morton2(c, bits=16):
    lo, hi = c.min(0), c.max(0)
    q = ((c - lo) / (hi - lo) * ((1 << bits) - 1)).astype(np.uint64)

    def spread(x):
        x = x & np.uint64(0xFFFF)
        x = (x | (x << np.uint64(8))) & np.uint64(0x00FF00FF)
        x = (x | (x << np.uint64(4))) & np.uint64(0x0F0F0F0F)
        x = (x | (x << np.uint64(2))) & np.uint64(0x33333333)
        x = (x | (x << np.uint64(1))) & np.uint64(0x55555555)
        return x

    return spread(q[:, 0]) | (spread(q[:, 1]) << np.uint64(1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--m", type=int, default=15)
    ap.add_argument("--tile", type=int, default=128)
    ap.add_argument("--tiles", type=int, default=2000, help="tiles sampled")
    a = ap.parse_args()
    rng = np.random.default_rng(0)
    c = rng.uniform(0, 1, (a.n, 2))
    nbr = orc.c_knn_prior_prefix_kdtree(c, a.m)
    perm = np.argsort(morton2(c), kind="stable")
    pos = np.empty(a.n, np.int64)
    pos[perm] = np.arange(a.n)
    snbr = np.where(nbr[perm] >= 0, pos[np.maximum(nbr[perm], 0)], -1)
    self_ = np.arange(a.n)
    T = a.n // a.tile
    pick = np.random.default_rng(1).choice(T, min(a.tiles, T), replace=False)
    iu = np.triu_indices(a.m + 1, 1)
    fr, us, full = [], [], []
    for t in pick:
        rows = np.arange(t * a.tile, (t + 1) * a.tile)
        jp = np.concatenate([snbr[rows], self_[rows, None]], 1)  # (tile, m+1)
        ok = (jp >= 0).all(1)
        jp = jp[ok]
        if len(jp) == 0:
            continue
        A = jp[:, iu[0]]
        B = jp[:, iu[1]]
        key = np.minimum(A, B).astype(np.int64) * a.n + np.maximum(A, B)
        d = len(np.unique(key))
        fr.append(d / key.size)
        full.append(d)
        us.append(len(np.unique(jp)))
    fr, us, full = np.array(fr), np.array(us), np.array(full)
    print(f"N={a.n} m={a.m} tile={a.tile}: distinct pair fraction mean {fr.mean():.3f} "
          f"(p10 {np.percentile(fr, 10):.3f}, p90 {np.percentile(fr, 90):.3f}, max {fr.max():.3f}); "
          f"distinct pairs per tile mean {full.mean():.0f} max {full.max()}; |U| mean {us.mean():.0f} max {us.max()}")


if __name__ == "__main__":
    main()
