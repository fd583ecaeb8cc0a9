"""Diagnose a planned sweep that differs from the unplanned one: which regions differ, planned or direct.

python tools/diag_plan.py --m 13 --seed 13 --n 9000
"""
import argparse

import numpy as np
import torch

from pynngp_amd import _lib

ap = argparse.ArgumentParser()
ap.add_argument("--m", type=int, nargs="+", default=[12, 13])
ap.add_argument("--n", type=int, default=9000)
ap.add_argument("--seed", type=int, default=None)
args = ap.parse_args()
dev = torch.device("cuda:0")
THETA = {"exponential": (1.0, 30.0, 0.0), "matern32": (1.0, 17.320508075688772, 0.1)}
for m in args.m:
    rng = np.random.default_rng(m if args.seed is None else args.seed)
    c = torch.from_numpy(rng.uniform(0.0, 1.0, (args.n, 2))).to(dev)
    v = torch.from_numpy(rng.standard_normal(args.n)).to(dev)
    nbr = _lib.knn_prior(c, m)
    order, nbr_s = _lib.row_order(c, 0, c.shape[0], nbr)
    plan = _lib.pair_plan(nbr_s, c.shape[0], 2, i0=0, order=order)
    info = list(plan.info)
    buf = plan.buf.cpu().numpy()
    nreg = (args.n + 127) // 128
    hdr = buf[:256].view(np.int64)
    sb = int(hdr[9])
    st = []
    for r in range(nreg):
        h = buf[256 + r * sb: 256 + r * sb + 16].view(np.int32)
        st.append((int(h[0]), int(h[1]), int(h[2])))
    print(f"m={m} info={info} slot_bytes={sb} planned={plan.n_planned} direct={plan.n_direct}")
    print("  regions (nU, nE, status):", st[:8], "...", "max nU", max(s[0] for s in st), "max nE", max(s[1] for s in st))
    T = nreg
    q, rem = args.n // T, args.n % T
    for kind in THETA:
        outs = []
        for p in (None, plan):
            R = torch.empty(args.n, dtype=torch.float64, device=dev)
            B, F, part = _lib.bf_sweep(c, nbr_s, 0, kind, *THETA[kind], values=v, algo="pairb", order=order, R=R, plan=p)
            outs.append((B.cpu().numpy(), F.cpu().numpy(), R.cpu().numpy(), part.cpu().numpy()))
        (B0, F0, R0, p0), (B1, F1, R1, p1) = outs
        bad = np.nonzero(np.any(B0 != B1, axis=1) | (F0 != F1) | (R0 != R1))[0]
        regs = sorted(set(int(np.searchsorted(np.array([t * q + min(t, rem) for t in range(T + 1)]), r, side="right") - 1)
                          for r in bad))
        print(f"  {kind}: {len(bad)} rows differ; partials {p0} vs {p1}")
        if len(bad):
            print("   regions:", regs[:20], "statuses:", [st[r][2] for r in regs[:20]])
            r = int(bad[0])
            print("   first row", r, "B0", B0[r][:6], "B1", B1[r][:6], "F", F0[r], F1[r])
