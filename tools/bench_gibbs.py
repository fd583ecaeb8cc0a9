"""Gibbs sampler timing (BASELINE.json configs[4]: 1,000 sweeps at N=1M, m=15; here one GPU).

One iteration = SeqNNGP.step(): MH proposal for phi (one fused B/F sweep + residuals),
conjugate sigma2, the colour-ordered w sweep, tau2 and beta draws (host scalars).
Synthetic response data y = 1 + w + eps from the seed; prints one JSON line.
    python tools/bench_gibbs.py [--n 1000000 --m 15 --iters 300 --warmup 100]
    --single-chain: ONE chain sharded over the ranks (ShardedSeqNNGP); with --force-group on one
    GPU a one-rank "nccl" group, so every per-colour exchange runs through RCCL
(100 warm-up iterations: the GPU clock settles over the first ~50 ms of sustained load)
"""
import argparse
import json
import os
import sys
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
ap.add_argument("--single-chain", action="store_true")
ap.add_argument("--force-group", action="store_true")
ap.add_argument("--backend", default="nccl")
ap.add_argument("--graphs", type=int, default=None, help="single chain: 1/0 forces the HIP-graph colour loop on/off")
ap.add_argument("--sweep", default="colour", choices=["colour", "tiled"],
                help="the w sweep: one launch per colour, or the tiled sweep (gibbs_tiles.py, one launch per phase)")
ap.add_argument("--graph-probe", action="store_true", help="also time the w sweep replayed from a captured HIP "
                "graph (timing probe: sigma2 / tau2 frozen at capture)")
ap.add_argument("--sweep-only", action="store_true", help="time only the w sweep (no iterations: timing probes "
                                                             "whose values are wrong)")
ap.add_argument("--tile-nodes", type=int, default=None, help="--sweep tiled: nodes per level-0 tile")
ap.add_argument("--tile-levels", type=int, default=None, help="--sweep tiled: at most this many tile levels")
args = ap.parse_args()
if args.tile_nodes:
    SeqNNGP._tile_nodes = args.tile_nodes
if args.tile_levels:
    SeqNNGP._tile_max_levels = args.tile_levels
# several GPUs (torchrun): independent chains, one per GPU ("replicas only")
world = int(os.environ.get("WORLD_SIZE", "1"))
rank = int(os.environ.get("RANK", "0"))
dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
torch.cuda.set_device(dev)
grouped = world > 1 or args.force_group
if grouped:
    import torch.distributed as dist

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29513")
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    if args.backend == "nccl":
        dist.init_process_group("nccl", device_id=dev)
    else:
        dist.init_process_group(args.backend)
rng = np.random.default_rng(2)
coords = rng.uniform(0, 1, (args.n, 2))
y = 1.0 + rng.standard_normal(args.n) * 0.5 + 0.3 * rng.standard_normal(args.n)
torch.cuda.synchronize()
t0 = time.perf_counter()
if args.single_chain:
    from pynngp_amd import ShardedSeqNNGP

    g = ShardedSeqNNGP(coords, y, m=args.m, sigma2=1.0, tau2=0.1, phi=30.0, seed=1, device=dev,
                       graphs=None if args.graphs is None else bool(args.graphs))
else:
    g = SeqNNGP(coords, y, m=args.m, sigma2=1.0, tau2=0.1, phi=30.0, seed=1 + rank, device=dev, sweep=args.sweep)
torch.cuda.synchronize()
setup_s = time.perf_counter() - t0
for _ in range(0 if args.sweep_only else args.warmup):
    g.step()
torch.cuda.synchronize()
if grouped:
    dist.barrier()
t0 = time.perf_counter()
for _ in range(0 if args.sweep_only else args.iters):
    g.step()
torch.cuda.synchronize()
if grouped:
    dist.barrier()
el = time.perf_counter() - t0
if grouped:
    t = torch.tensor([el], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el = float(t.item())
# the w sweep alone (normals drawn once; the same work as inside step())
w_sweep_ms = None
if not args.single_chain:
    w_sweep = g._sweep_tiles if g._tiles is not None else (lambda: (g.update_wt(), g.update_ws()))
    for _ in range(10):
        w_sweep()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(100):
        w_sweep()
    e1.record()
    torch.cuda.synchronize()
    w_sweep_ms = e0.elapsed_time(e1) / 100
    if args.graph_probe:
        gr = torch.cuda.CUDAGraph()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            w_sweep()
        torch.cuda.current_stream().wait_stream(side)
        with torch.cuda.graph(gr):
            w_sweep()
        for _ in range(10):
            gr.replay()
        e0.record()
        for _ in range(100):
            gr.replay()
        e1.record()
        torch.cuda.synchronize()
        w_sweep_graph_ms = e0.elapsed_time(e1) / 100
if rank == 0:
    extra = {"sweep": args.sweep, "w_sweep_ms": w_sweep_ms}
    if args.graph_probe:
        extra["w_sweep_graph_ms"] = w_sweep_graph_ms
    if getattr(g, "_tiles", None) is not None:
        tp = g._tiles
        extra.update(tiles=int(tp.tinfo.shape[0]), tile_launches=len(tp.phases), tile_levels=tp.levels,
                     tiles_per_launch=[int(p.numel()) for p in tp.phases], steps=int(tp.tstep.numel()), ecap=tp.ecap,
                     halo_fraction=float(tp.tfp.numel()) / args.n - 1.0)
    if args.single_chain:
        extra.update({"halo_rows": int(g._n_h), "replayed_rows": int(g._apply_rows.shape[0]),
                 "collectives_per_iter": g._xchg.n_collectives / max(1, g.iteration), "group": grouped,
                 "backend": args.backend if grouped else None, "graphs": len(g._graphs)})
    chains = 1 if args.single_chain else world
    what = "ONE chain sharded over the GPUs" if args.single_chain else "one chain per GPU"
    print(json.dumps({"workload": f"SeqNNGP Gibbs, N={args.n}, m={args.m}, exponential, {what}", **extra,
                      "chains": chains, "chain_iters_per_s": chains * args.iters / max(el, 1e-9), "iters": args.iters, "ms_per_iter": 1e3 * el / max(args.iters, 1), "iters_per_s": args.iters / max(el, 1e-9),
                  "locations_per_s": args.n * args.iters / max(el, 1e-9), "setup_s": setup_s, "n_colors": int(g.n_colors),
                  "phi": g.phi, "sigma2": g.sigma2, "tau2": g.tau2, "accept": g.n_accept / max(1, g.iteration)}))
if grouped:
    dist.destroy_process_group()
