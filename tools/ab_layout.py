import sys, os, time, json
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import numpy as np, torch
from pynngp_amd import _lib
dev = torch.device("cuda", 0)
rng = np.random.default_rng(0)
n, m = 1_000_000, 15
coords = rng.uniform(0, 1, (n, 2)); vals = rng.standard_normal(n)
c = torch.from_numpy(coords).to(dev); v = torch.from_numpy(vals).to(dev)
nbr = _lib.knn_prior(c, m)
order, srt = _lib.row_order(c, nbr=nbr)
perm = order.long(); pos = torch.empty_like(perm); pos[perm] = torch.arange(n, device=dev)
cz = c[perm].contiguous(); nb = nbr[perm].long()
nz = torch.where(nb >= 0, pos[nb.clamp(min=0)], -1).to(torch.int32).contiguous()
B = torch.empty((n, m), dtype=torch.float64, device=dev); F = torch.empty(n, dtype=torch.float64, device=dev)
ws = _lib.bf_workspace(n, m, "auto", dev); P = torch.empty(4, dtype=torch.float64, device=dev)
vz = torch.empty_like(v)
def t(fn, reps=30):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record(); fn(); b.record()
    torch.cuda.synchronize()
    return float(np.mean([a.elapsed_time(b) for a, b in ev]))
nat = lambda: _lib.bf_sweep(c, srt, 0, "exponential", 1.0, 30.0, 0.0, values=v, B=B, F=F, partials=P, workspace=ws, order=order)
sto = lambda: _lib.bf_sweep(cz, nz, 0, "exponential", 1.0, 30.0, 0.0, values=vz, B=B, F=F, partials=P, workspace=ws)
def sto_perm():
    torch.index_select(v, 0, perm, out=vz)
    sto()
for rep in range(2):
    print(json.dumps({"natural_ms": t(nat), "storage_ms": t(sto), "storage_with_value_gather_ms": t(sto_perm)}))
nat(); p1 = P.clone(); torch.index_select(v, 0, perm, out=vz); sto(); p2 = P.clone()
print("partials natural", p1.tolist(), "storage", p2.tolist())
