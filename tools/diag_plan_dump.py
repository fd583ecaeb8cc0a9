"""Dump a plan (first regions), its inputs and both sweeps' B / F for offline decoding (diagnosis)."""
import argparse

import numpy as np
import torch

from pynngp_amd import _lib

ap = argparse.ArgumentParser()
ap.add_argument("--m", type=int, default=13)
ap.add_argument("--n", type=int, default=9000)
ap.add_argument("--regions", type=int, default=3)
ap.add_argument("--out", default="gpurun_out/plan_dump.npz")
args = ap.parse_args()
dev = torch.device("cuda:0")
m = args.m
rng = np.random.default_rng(m)
c = torch.from_numpy(rng.uniform(0.0, 1.0, (args.n, 2))).to(dev)
v = torch.from_numpy(rng.standard_normal(args.n)).to(dev)
nbr = _lib.knn_prior(c, m)
order, nbr_s = _lib.row_order(c, 0, c.shape[0], nbr)
plan = _lib.pair_plan(nbr_s, c.shape[0], 2, i0=0, order=order)
buf = plan.buf.cpu().numpy()
sb = int(buf[:256].view(np.int64)[9])
outs = {}
for name, p in (("un", None), ("pl", plan)):
    B, F, part = _lib.bf_sweep(c, nbr_s, 0, "exponential", 1.0, 30.0, 0.0, values=v, algo="pairb", order=order, plan=p)
    outs["B_" + name], outs["F_" + name] = B.cpu().numpy(), F.cpu().numpy()
nreg = (args.n + 127) // 128
hdrs = np.stack([buf[256 + r * sb: 256 + r * sb + 16].view(np.int32) for r in range(nreg)])
badrow = np.nonzero(np.any(outs["B_un"] != outs["B_pl"], axis=1))[0]
inv = np.argsort(order.cpu().numpy())
T = nreg
q, rem = args.n // T, args.n % T
starts = np.array([t * q + min(t, rem) for t in range(T + 1)])
badreg = sorted(set((np.searchsorted(starts, inv[badrow], side="right") - 1).tolist()))
print("bad regions", badreg, "headers", [tuple(hdrs[r][:3]) for r in badreg])
print("info", list(plan.info), "ecap-ish max planned nE", int(hdrs[hdrs[:, 2] == 0, 1].max()))
r0 = badreg[0] if badreg else 0
np.savez_compressed(args.out, plan=buf[:256 + args.regions * sb], sb=sb, hdrs=hdrs, badreg=np.array(badreg),
                    slot_bad=buf[256 + r0 * sb: 256 + (r0 + 1) * sb], nbr=nbr_s.cpu().numpy(),
                    order=order.cpu().numpy(), coords=c.cpu().numpy(), **outs)
print("dumped", args.out, "slot bytes", sb, "rows differing", int(np.sum(np.any(outs["B_un"] != outs["B_pl"], axis=1))))
