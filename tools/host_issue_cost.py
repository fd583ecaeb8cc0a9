"""Host issue cost of one sweep through ShardedLogLik.local_partials at N = 10^5, m = 15 (config 2):
the resolved torch.ops overload (the default) against the overload packet.  Run on the GPU box.
    python tools/host_issue_cost.py
"""
import time, torch, numpy as np, sys, json
sys.path.insert(0, '.')
from pynngp_amd.sweep import ShardedLogLik, Covariance
dev = torch.device('cuda', 0)
rng = np.random.default_rng(0)
c = torch.from_numpy(rng.uniform(0, 1, (100000, 2))).to(dev)
v = torch.from_numpy(rng.standard_normal(100000)).to(dev)
sw = ShardedLogLik(c, 15, 0, 1, layout="storage")
cov = Covariance("matern32", 1.0, 17.320508075688772, 0.1)
out = torch.empty(4, dtype=torch.float64, device=dev)
for _ in range(2000): sw.local_partials(cov, v, True, "storage", out=out)
torch.cuda.synchronize()
res = {}
for mode in ("op", "packet"):
    if mode == "packet":
        sw._sweep_op = torch.ops.nngp.bf_sweep_out
    t0 = time.perf_counter()
    for _ in range(2000): sw.local_partials(cov, v, True, "storage", out=out)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    res[mode] = {"host_us_per_call": (t1 - t0) / 2000 * 1e6, "wall_us_per_sweep": (t2 - t0) / 2000 * 1e6}
print(json.dumps(res))
