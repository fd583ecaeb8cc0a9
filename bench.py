"""NNGP fused B/F + log-likelihood sweep benchmark (BASELINE.json headline).

One step = one sweep over this rank's shard of locations: the gfx950 kernel
builds every location's (m+1)x(m+1) joint covariance block, factors it, writes
B (rows, m) and F (rows,), and reduces the log-likelihood partials; with more
than one rank the partials are all-gathered over RCCL and summed in rank order.

Workload (BASELINE.json configs[2], the headline): N = 1,000,000 locations per
GPU (weak scaling: N_total = 1e6 x world), m = 15, exponential covariance
(sigma2 = 1, phi = 30, tau2 = 0), synthetic uniform [0,1]^2 coordinates and
N(0,1) values from numpy default_rng(0).  Inputs and neighbour
sets are resident in HBM before timing; the one-off neighbour build is timed
separately (``neighbor_build_s``).

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...
    python bench.py --config {2,4,5}              # the other BASELINE presets (5: the Gibbs sampler;
                                                   # --chains-per-gpu C, --single-chain)
"""
import argparse
import json
import os
import platform
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from pynngp_amd import Covariance, ShardedLogLik, _lib  # noqa: E402
from pynngp_amd.sweep import PipelinedCombine  # noqa: E402

HBM_PEAK = 8.0e12  # B/s, MI355X spec (MI355X_MICROARCH.md chip table)
FP64_PEAK = 78.6e12  # FLOP/s, MI355X fp64 vector spec
METRIC = "NNGP log-lik sweeps/sec (N=1M, m=15) at 1/2/4/8 MI355X; % HBM roofline"


def bytes_per_location(m):
    # 4m idx + 16 own coord + 16m nbr coords + 8 own value + 8m nbr values + (8m + 8) B, F writes
    return 36 * m + 32


def flops_per_location(m):
    # Cholesky m^3/3 + solves 2m^2 + covariance fill 4.5 m(m+1) + 4m
    return m ** 3 / 3 + 2 * m ** 2 + 4.5 * m * (m + 1) + 4 * m


def synth(n_total, seed=0):
    rng = np.random.default_rng(seed)
    coords = rng.uniform(0.0, 1.0, (n_total, 2))
    values = rng.standard_normal(n_total)
    return coords, values


def knn_cpu_baseline(coords, m, n_full, n_sample=10_000):
    """Neighbour-set build on the host, the reference's own algorithm: a KD-tree over
    s[0:i] rebuilt for every i, queried for min(i, m) neighbours (pyNNGP/nngp.py:49-62;
    restated single-threaded in C, oracle_knn_prior_kdtree_rebuild, leaf size 40 as
    sklearn's default).  Timed on the first ``n_sample`` locations and extrapolated to
    ``n_full`` as N^2 log N (the rebuild of an i-point tree costs i log i; summed over i)."""
    from oracle import nngp_oracle as O

    n = min(n_sample, coords.shape[0])
    t = time.perf_counter()
    O.c_knn_prior_kdtree_rebuild(coords[:n], m)
    el = time.perf_counter() - t
    scale = (n_full / n) ** 2 * np.log(n_full) / np.log(n)
    return {"seconds_measured": el, "n_measured": n, "seconds_extrapolated": el * scale,
            "n_extrapolated": n_full, "cores": 1,
            "kind": "port (per-i KD-tree rebuild as pyNNGP/nngp.py:55-61, C restatement; extrapolated as N^2 log N)"}


def committed_profile(args, want_bf):
    """The committed rocprofv3 --pmc measurement (profiles/traffic.json) of this exact kernel
    config, or None."""
    try:
        with open(os.path.join(ROOT, "profiles", "traffic.json")) as f:
            entries = json.load(f)["entries"]
    except (OSError, ValueError, KeyError):
        return None
    for e in entries:
        if e.get("preset") is not None or e.get("role", "sweep") != "sweep":
            continue  # the Gibbs preset's kernels (gibbs_profile)
        if (e["n_per_gpu"] == args.n and e["m"] == args.m and e["kind"] == args.kind and e["layout"] == args.layout
                and e["write_BF"] == want_bf and args.algo == "auto"):
            return e
    return None


def gibbs_profile(args, role):
    """The committed rocprofv3 entry of config 5's kernel `role` ("sweep": the phi proposal's fused
    B/F sweep, "colour": the w sweep's colour step) at this N and m, or None."""
    try:
        with open(os.path.join(ROOT, "profiles", "traffic.json")) as f:
            entries = json.load(f)["entries"]
    except (OSError, ValueError, KeyError):
        return None
    for e in entries:
        if e.get("preset") == 5 and e.get("role") == role and e["n_per_gpu"] == args.n and e["m"] == args.m:
            return e
    return None


def committed_traffic(args, want_bf):
    """HBM bytes per launch measured for this exact kernel config by a committed rocprofv3
    --pmc pass (profiles/traffic.json), or (None, None)."""
    e = committed_profile(args, want_bf)
    if e is None:
        return None, None
    return e["bytes_per_launch"], f'{e["source"]} (rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE, {e["kernel"]})'


# VALU issue peak: 256 CUs x 4 SIMDs x 16 fp64 FMA lanes per clock x 2.4 GHz -- one wave64 fp64
# instruction every 4 cycles per SIMD, the 78.6 TFLOP/s fp64 vector rate.  Measured on gfx950
# (tools/ubench/valu_mix.hip, profiles/r03d): at two waves per SIMD a wave-instruction occupies the
# SIMD for ~5.1 cycles (fp64 FMA / MUL), ~4.8-4.9 (DPP moves, VOP3 32-bit such as v_lshl_add_u32,
# v_bfi_b32), ~2.9 only for VOP2 32-bit (v_and, v_mov), ~16.8 (v_rsq_f64 / v_rcp_f64) and ~4.3 for a
# 3:1 fp64 / DPP mix, so 32-bit work is not cheaper than 4 cycles here; the sweep measures 4.37
# VALU-active cycles per instruction (SQ_ACTIVE_INST_VALU), see valu_roofline.
VALU_LANE_OPS_PEAK = 256 * 4 * 16 * 2.4e9


def valu_roofline(prof, rows, kern_ms):
    """Vector-issue roofline: lane-operations per second (VALU instructions per wave from the
    committed PMC profile x 64 lanes / locations per wave x locations/s) vs the fp64 issue peak,
    plus the committed profile's measured VALU-active cycles per instruction and SIMD VALU-busy
    share (tools/valu_busy.py): the direct measure of how close the sweep is to its issue limit."""
    if prof is None or "valu_per_wave" not in prof:
        return None
    per_loc = prof["valu_per_wave"] * 64 / prof["locations_per_wave"]
    achieved = per_loc * rows / (kern_ms * 1e-3)
    out = {"achieved": achieved / 1e12, "peak": VALU_LANE_OPS_PEAK / 1e12, "unit": "T lane-ops/s",
           "frac": achieved / VALU_LANE_OPS_PEAK, "valu_lane_ops_per_location": per_loc,
           "source": prof["source"] + " (SQ_INSTS_VALU / SQ_WAVES)"}
    for k in ("valu_active_cycles_per_instr", "simd_valu_busy", "valu_source"):
        if k in prof:
            out[k] = prof[k]
    return out


def colour_roofline(prof):
    """The w sweep's colour step (config 5's largest kernel-time share) from its committed rocprofv3
    passes: average launch time, HBM bytes per launch (FETCH_SIZE x2 + WRITE_SIZE) and VALU issue.
    Its members' children are gathered at random, so it is latency bound, not HBM bound: the
    fraction is reported against 8 TB/s for scale only."""
    if prof is None or "bytes_per_launch" not in prof:
        return None
    bw = prof["bytes_per_launch"] / (prof["avg_ns"] * 1e-9)
    out = {"kernel": prof["kernel"], "avg_us": prof["avg_ns"] / 1e3, "traffic": prof["bytes_per_launch"],
           "hbm_GBps": bw / 1e9, "hbm_frac": bw / HBM_PEAK, "source": prof["source"],
           "traffic_note": "FETCH_SIZE x2 is MI355X_MICROARCH.md's calibration for 16-B-per-lane streaming reads; "
                           "this kernel's reads are 8-B gathers (uncalibrated), so the figure is an upper bound"}
    for k in ("valu_per_wave", "valu_active_cycles_per_instr", "simd_valu_busy"):
        if k in prof:
            out[k] = prof[k]
    return out


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def cpu_baseline(coords, values, nbr_host, kind, theta, budget_s, F_gpu):
    """C oracle (oracle/nngp_oracle.c, OpenMP) on a bounded sample of the same workload."""
    from oracle import nngp_oracle as O

    threads = O.load_c_oracle().oracle_num_threads()
    rows_done, t_cpu = 0, 0.0
    chunk = 50_000
    max_dF = 0.0
    r0 = 0
    n = nbr_host.shape[0]
    while t_cpu < budget_s:
        if r0 >= n:  # whole field done: another pass over it
            r0 = 0
        r1 = min(n, r0 + chunk)
        t = time.perf_counter()
        _, Fo, _ = O.c_bf_sweep(coords, nbr_host[r0:r1], kind, theta, values, i0=r0)
        t_cpu += time.perf_counter() - t
        max_dF = max(max_dF, float(np.max(np.abs(F_gpu[r0:r1] - Fo) / Fo)))
        rows_done += r1 - r0
        r0 = r1
        chunk = min(400_000, chunk * 2)
    return {
        "value": rows_done / t_cpu,
        "unit": "locations/s",
        "cores": int(threads),
        "kind": "port",
        "sample": f"{rows_done} location-sweeps ({rows_done / n:.2f} passes over the same field, fused B/F + "
                  f"log-lik), C oracle (OpenMP, {threads} threads, {cpu_model()}) in {t_cpu:.2f} s",
        "parity_max_rel_dF": max_dF,
    }


def synth_gibbs_field(n, seed, sigma2, phi, tau2, beta, dev, features=2048):
    """Synthetic response data for the Gibbs preset: y = X beta + w + e on uniform [0,1]^2
    coordinates, w a stationary exponential-covariance GP field (sigma2, phi) drawn with random
    Fourier features (2-D exponential spectral density: omega = phi z / |g|, z ~ N(0, I_2),
    g ~ N(0, 1)), e ~ N(0, tau2), X = [1, N(0,1)].  Generated on the GPU in chunks; a
    spatially structured field keeps the chain in the regime config 5 describes."""
    rng = np.random.default_rng(seed)
    coords = rng.uniform(0.0, 1.0, (n, 2))
    omega = phi * rng.standard_normal((2, features)) / np.abs(rng.standard_normal(features))
    bias = rng.uniform(0.0, 2 * np.pi, features)
    x1 = rng.standard_normal(n)
    noise = rng.standard_normal(n)
    c = torch.from_numpy(coords).to(dev)
    om, b = torch.from_numpy(omega).to(dev), torch.from_numpy(bias).to(dev)
    w = torch.empty(n, dtype=torch.float64, device=dev)
    for a in range(0, n, 65536):
        w[a:a + 65536] = torch.cos(c[a:a + 65536] @ om + b).sum(dim=1)
    w *= np.sqrt(2.0 * sigma2 / features)
    wh = w.cpu().numpy()
    X = np.column_stack([np.ones(n), x1])
    y = X @ np.asarray(beta) + wh + np.sqrt(tau2) * noise
    return coords, X, y, wh


def run_gibbs(args, dev, rank, world, distributed, json_fd):
    """BASELINE config 5: the Gibbs sampler (SeqNNGP) at N = 1e6, m = 15 -- one chain per GPU
    ("replicas only": the w sweep's per-colour halo exchange would cost more than the sweep at this
    N); a step = one full iteration (phi MH with its fused B/F sweep, sigma2, the
    colour-ordered w sweep, tau2, beta)."""
    from pynngp_amd import Priors, SeqNNGP, SeqNNGPChains, ShardedSeqNNGP

    single = args.single_chain
    n = args.n * world if single else args.n  # single chain: n locations per GPU, one field over all
    m = args.m
    sigma2, phi, tau2, beta = 1.0, 30.0, 0.1, (1.0, -0.5)
    coords, X, y, _ = synth_gibbs_field(n, 5, sigma2, phi, tau2, beta, dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    # --chains-per-gpu C > 1 (replica mode only): C independent chains per GPU, each on its own HIP
    # stream driven by its own host thread -- one chain leaves the GPU idle in its colour steps' launch
    # floors and its host synchronisations (tools/bench_gibbs_streams.py)
    cpg = 1 if single else max(1, args.chains_per_gpu)
    batched = cpg > 1 and args.chain_mode in ("batched", "batched-percopy")
    # batched-streams: two batches of C / 2 chains, each on its own stream and host thread, so one batch's
    # colour steps (memory-latency bound) overlap the other's phi-proposal sweeps (VALU bound)
    groups = min(args.chain_groups, cpg) if cpg > 1 and args.chain_mode == "batched-streams" else 0
    if groups and cpg % groups:
        raise SystemExit("--chain-mode batched-streams needs --chains-per-gpu divisible by --chain-groups")
    streams = ([torch.cuda.current_stream(dev)] if cpg == 1 or batched
               else [torch.cuda.Stream(dev) for _ in range(groups or cpg)])
    chains = []
    kw = dict(m=m, priors=Priors(), sigma2=sigma2, tau2=tau2, phi=phi, phi_tuning=0.01, device=dev)
    # the w sweep of a single chain per GPU: one launch per colour, or the tiled sweep (gibbs_tiles.py)
    tiled = args.gibbs_sweep == "tiled" and not single and cpg == 1
    if single:
        chains.append(ShardedSeqNNGP(coords, y, X, seed=1, collective=distributed, **kw))
    elif batched:
        # C chains advanced together: one launch per colour for all, two host synchronisations per iteration
        multi = SeqNNGPChains(coords, y, X, seeds=[1 + rank * cpg + k for k in range(cpg)],
                              interleave=args.chain_mode == "batched", **kw)
        chains = list(multi.chains)
    elif groups:
        per = cpg // groups
        batches = []
        for k in range(groups):
            with torch.cuda.stream(streams[k]):
                batches.append(SeqNNGPChains(coords, y, X, seeds=[1 + rank * cpg + k * per + j for j in range(per)],
                                             **kw))
        chains = [c for b in batches for c in b.chains]
    else:
        for k in range(cpg):
            with torch.cuda.stream(streams[k]):
                chains.append(SeqNNGP(coords, y, X, seed=1 + rank * cpg + k, sweep="tiled" if tiled else "colour",
                                      **kw))
    g = chains[0]
    torch.cuda.synchronize()
    setup_s = time.perf_counter() - t0

    def run_chains(iters):
        if batched:
            for _ in range(iters):
                multi.step()
            return
        if cpg == 1:
            for _ in range(iters):
                g.step()
            return
        import threading

        errors = []

        units = batches if groups else chains

        def one(k):
            try:
                with torch.cuda.stream(streams[k]):
                    for _ in range(iters):
                        units[k].step()
            except BaseException as e:  # re-raised below: a failed chain must fail the run
                errors.append(e)

        th = [threading.Thread(target=one, args=(k,)) for k in range(len(units))]
        for t in th:
            t.start()
        for t in th:
            t.join()
        if errors:
            raise errors[0]

    run_chains(args.warmup)
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    t0 = time.perf_counter()
    run_chains(args.steps)
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if distributed:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # the fused B/F sweep of one phi proposal, timed on its own (HIP events on the launch stream),
    # and the colour-ordered w sweep: their shares of an iteration
    stream = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 50
    e0.record(stream)
    for _ in range(reps):
        if single:  # own rows + halo rows, partials folded over the ranks
            g._propose(g.phi)
        else:
            g._sweep_into(g.phi, g._B2, g._Ft2, g._r2)
    e1.record(stream)
    torch.cuda.synchronize()
    sweep_ms = e0.elapsed_time(e1) / reps
    w_save, r_save = g.w.clone(), g.r.clone()
    e0.record(stream)
    for _ in range(reps):
        if tiled:
            g._sweep_tiles()
        else:
            g.update_wt()
            g.update_ws()
    e1.record(stream)
    torch.cuda.synchronize()
    wsweep_ms = e0.elapsed_time(e1) / reps
    g.w.copy_(w_save)
    g.r.copy_(r_save)
    ms_iter = 1e3 * elapsed / args.steps
    if rank == 0:
        sweep_prof = gibbs_profile(args, "sweep") if not single else None
        colour_prof = gibbs_profile(args, "colour") if not single else None
        bpl = bytes_per_location(m) + 8  # + the residual r written for the sampler
        rows = g.hi - g.lo if single else n
        achieved = bpl * rows / (sweep_ms * 1e-3)
        n_chains = 1 if single else world * cpg
        out = {
            "metric": "NNGP Gibbs sampler iterations/sec (BASELINE config 5: N=1M, m=15, 1,000 sweeps; " + (
                "ONE chain sharded over the GPUs)" if single else "one chain per GPU)"),
            "value": n_chains * args.steps / elapsed,
            "unit": "chain-iterations/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_iter,
            "iterations_per_s_per_chain": args.steps / elapsed,
            "locations_per_s": n_chains * n * args.steps / elapsed,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: uniform [0,1]^2 coords, y = X beta + w + e, w an exponential GP field (sigma2=1, "
                    "phi=30; random Fourier features), tau2=0.1, beta=(1, -0.5)",
            "config": {
                "workload": f"BASELINE config 5: {'ShardedSeqNNGP' if single else 'SeqNNGP'} Gibbs sampler, "
                            f"N={n} per chain, m={m}, exponential, "
                            f"{args.steps} timed iterations after {args.warmup} warm-up",
                "n_per_gpu": args.n, "m": m, "kind": "exponential", "chains": n_chains, "chains_per_gpu": cpg,
                "parallelism": (f"one chain over {world} GPU(s): storage-row shards, one halo all-gather (the "
                                "boundary members) per colour"
                                if single else f"replicas x{world * cpg} ({cpg} independent chain(s) per GPU"
                                + ("" if cpg == 1 else (", advanced together: one launch per colour for all"
                                                        if batched else ", each on its own stream")) + ")"),
                "chain_mode": args.chain_mode if (batched or groups) else ("streams" if cpg > 1 else "single"),
                "chain_groups": groups or None,
                "w_sweep": "tiled" if tiled else "colour",
            },
            "breakdown": {
                "bf_sweep_ms": sweep_ms, "bf_sweep_share": sweep_ms / ms_iter,
                "w_sweep_ms": wsweep_ms, "w_sweep_share": wsweep_ms / ms_iter, "n_colors": int(g.n_colors),
                "w_sweep": ("tiled: one launch per phase of spatial tiles, r in LDS (%d tiles, %d launches)"
                            % (g._tiles.tinfo.shape[0], len(g._tiles.phases))) if tiled else "one launch per colour",
                "phi_accept_rate": g.n_accept / max(1, g.iteration), "setup_s": setup_s,
            },
            "roofline": {
                "bound": "hbm", "kernel": "fused B/F + residual sweep of a phi proposal",
                "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s", "frac": achieved / HBM_PEAK,
                "traffic": sweep_prof.get("bytes_per_launch") if sweep_prof else None,
                "traffic_source": (f'{sweep_prof["source"]} (rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE, '
                                   f'{sweep_prof["kernel"]})') if sweep_prof else None,
                "algorithmic_bytes_per_location": bpl, "kernel_ms": sweep_ms, "kernel_rows": rows,
            },
            "roofline_valu": valu_roofline(sweep_prof, rows, sweep_ms) if sweep_prof else None,
            "roofline_colour": colour_roofline(colour_prof),
            "state": {"phi": g.phi, "sigma2": g.sigma2, "tau2": g.tau2, "beta": list(map(float, g.beta))},
            "lib": os.path.relpath(_lib.LIB_PATH, ROOT),
        }
        if world == 1 and args.cpu_seconds > 0:
            F_gpu = g.Ft.cpu().numpy()
            out["cpu_baseline"] = cpu_baseline(g.coords.cpu().numpy(), g.w.cpu().numpy(), g.nbr.cpu().numpy(),
                                               "exponential", (1.0, g.phi, 0.0), args.cpu_seconds, F_gpu)
            out["cpu_baseline"]["sample"] += " -- the B/F + log-lik sweep of one phi proposal (no CPU Gibbs sampler)"
        sys.stdout.flush()
        os.write(json_fd, (json.dumps(out) + "\n").encode())


def main():
    # The result must be the only line on stdout: libraries (RCCL prints a version
    # banner at communicator creation) write to fd 1 too, so point fd 1 at stderr
    # for the whole run and keep a private handle for the JSON line.
    json_fd = os.dup(1)
    os.dup2(2, 1)
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--gibbs-sweep", default="colour", choices=["colour", "tiled"],
                    help="config 5, one chain per GPU: the w sweep as one launch per colour, or tiled (one launch "
                         "per phase of spatial tiles holding r in LDS, pynngp_amd/gibbs_tiles.py)")
    ap.add_argument("--config", type=int, choices=[2, 3, 4, 5], default=None,
                    help="BASELINE.json config preset: 2 = N=1e5, m=15, Matern-3/2 (tau2=0.1); 3 = the headline "
                         "(default flags); 4 = N=1e7 / world per GPU, m=20, exponential; 5 = the Gibbs sampler "
                         "(SeqNNGP, N=1e6, m=15, 1,000 iterations after 100 warm-up, one chain per GPU)")
    # defaults: the GPU clock settles over the first ~50 ms of sustained load (the sweep
    # kernel goes from ~218 to ~187 us over its first ~200 launches), so the
    # default warm-up is 200 sweeps; both still finish in well under a second
    ap.add_argument("--steps", type=int, default=None, help="timed steps (default 200; config 5: 1,000 iterations)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed steps (default 200; config 5: 100)")
    ap.add_argument("--n", "--n-per-gpu", dest="n", type=int, default=1_000_000, help="locations per GPU")
    ap.add_argument("--m", type=int, default=15)
    ap.add_argument("--kind", default="exponential", choices=list(_lib.KIND_CODES))
    ap.add_argument("--theta", default="1.0,30.0,0.0", help="sigma2,phi,tau2")
    ap.add_argument("--nu", type=float, default=None, help="smoothness of --kind matern")
    ap.add_argument("--algo", default="auto", choices=["auto", "lane", "wave", "quad", "pairb"])
    ap.add_argument("--loglik-only", action="store_true", help="skip the B/F writes (log-lik partials only)")
    ap.add_argument("--no-order", action="store_true", help="visit rows in index order (no Z-order; natural layout)")
    ap.add_argument("--layout", default="storage", choices=["storage", "natural"],
                    help="storage: per-location arrays relabelled into Z-order storage (default); natural: input rows")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline budget in seconds of CPU work (a bounded sample; 0 = skip)")
    ap.add_argument("--rehearse-on-one-gpu", action="store_true",
                    help="testing only: every rank on cuda:0 with gloo collectives (the N-rank flow on one GPU)")
    ap.add_argument("--sweep-api", default="ops", choices=["ops", "ctypes"],
                    help="ops: torch.ops.nngp.bf_sweep_out (default); ctypes: the same C ABI via ctypes (A/B)")
    ap.add_argument("--event-stride", type=int, default=None,
                    help="bracket every S-th timed sweep with HIP events for kernel_ms (1 = every sweep; default "
                         "min(10, steps // 5): at least 5 samples from 5 steps on)")
    ap.add_argument("--exchange-batch", type=int, default=16,
                    help="sweeps whose (4,) partials share one all-gather (PipelinedCombine batch)")
    ap.add_argument("--force-collective", action="store_true",
                    help="exchange the partials through torch.distributed even on one rank (a one-rank RCCL group "
                         "when not launched by torchrun): the N-rank all-gather + fold path on a one-GPU box")
    ap.add_argument("--chains-per-gpu", type=int, default=1,
                    help="config 5 replica mode: independent chains per GPU, one stream and host thread each")
    ap.add_argument("--chain-mode", default="batched-streams",
                    choices=["batched", "batched-percopy", "batched-streams", "streams"],
                    help="--chains-per-gpu C > 1: advance the C chains together (SeqNNGPChains: one launch per colour "
                         "for all, w / r interleaved; batched-percopy: per-chain w / r; batched-streams: two such "
                         "batches on their own streams and host threads) or each on its own stream and host thread")
    ap.add_argument("--chain-groups", type=int, default=2,
                    help="--chain-mode batched-streams: the number of batches (streams / host threads)")
    ap.add_argument("--single-chain", action="store_true",
                    help="config 5: ONE chain sharded over the GPUs (ShardedSeqNNGP, n locations per GPU) instead "
                         "of one chain per GPU")
    ap.add_argument("--plan", default="auto", choices=["auto", "on", "off"],
                    help="wave pair plans (shared covariances evaluated once per wavefront; built with the neighbour "
                         "sets, outside the timed region): auto = sweep.PLAN_DEFAULT (off: measured slower, DESIGN.md 4.1b)")
    ap.add_argument("--pmc-traffic", type=float, default=None,
                    help="HBM bytes per launch from a separate rocprofv3 --pmc pass (fills roofline.traffic)")
    args = ap.parse_args()
    if args.steps is None:
        args.steps = 1000 if args.config == 5 else 200
    if args.warmup is None:
        args.warmup = 100 if args.config == 5 else 200
    if args.config == 2:
        args.n, args.m, args.kind, args.theta = 100_000, 15, "matern32", "1.0,17.320508075688772,0.1"
    elif args.config == 4:
        args.n, args.m = 10_000_000 // int(os.environ.get("WORLD_SIZE", "1")), 20

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if args.rehearse_on_one_gpu:
        local_rank = 0  # rehearsal of the N-rank flow on a one-GPU box (gloo collectives)
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    distributed = "RANK" in os.environ and "MASTER_ADDR" in os.environ  # launched by torch.distributed.run
    if not distributed and args.force_collective:
        # a one-rank RCCL group of our own (127.0.0.1, a free port): the collective path on one GPU
        import socket

        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
        distributed = True
    if distributed:
        if args.rehearse_on_one_gpu:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    if args.config == 5:
        run_gibbs(args, dev, rank, world, distributed, json_fd)
        if distributed:
            dist.destroy_process_group()
        return

    sigma2, phi, tau2 = (float(x) for x in args.theta.split(","))
    cov = Covariance(args.kind, sigma2, phi, tau2, nu=args.nu)
    n_total = args.n * world
    coords, values = synth(n_total, seed=0)
    c = torch.from_numpy(coords).to(dev)
    v = torch.from_numpy(values).to(dev)

    torch.cuda.synchronize()
    t0 = time.perf_counter()
    sweep = ShardedLogLik(c, args.m, rank, world, algo=args.algo, spatial_order=not args.no_order,
                          layout=args.layout, api=args.sweep_api, collective=distributed,
                          plan={"auto": None, "on": True, "off": False}[args.plan])
    if args.layout == "storage":
        # the synthetic field lives in the engine's storage order (an MCMC state would);
        # same iid N(0,1) values, assigned to locations in storage order
        v_sweep, v_layout = v, "storage"
    else:
        v_sweep, v_layout = v, "input"
    torch.cuda.synchronize()
    knn_s = time.perf_counter() - t0
    want_bf = not args.loglik_only
    rows = sweep.hi - sweep.lo

    for _ in range(args.warmup):
        sweep.partials(cov, v_sweep, want_bf, v_layout)
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    stream = torch.cuda.current_stream(dev)
    # HIP events around the sweep op of every --event-stride-th step: a timing event pair makes the
    # queue drain around the op it brackets (~6-8 us of idle GPU per bracketed sweep, measured:
    # config 2 runs 29.0 us per sweep without events and 36.8 us with a pair around every sweep,
    # profiles/r02am), so only a sample of the steps is bracketed; kernel_ms is their mean.
    # With few steps (the driver's 20) the stride shrinks so that >= 5 sweeps are sampled; one more event
    # pair around the whole timed loop gives the GPU time per step over every step (kernel_ms_loop).
    stride = max(1, args.event_stride if args.event_stride is not None else min(10, args.steps // 5))
    ev = {k: (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for k in range(min(stride // 2, args.steps - 1), args.steps, stride)}  # the middle step of each window
    ev_loop = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    # independent sweeps: the all-gather of sweep k overlaps sweep k+1 (RCCL stream + side
    # stream for the fold); every sweep's global partials are complete when the clock stops.
    # (Deferring the block-record fold to the side stream as well, nngp_bf_finalize, issued
    # 9x the host work per step and measured 0.35 vs 0.25 ms per step: the in-line fold stays.)
    pipe = PipelinedCombine(sweep, args.steps, batch=args.exchange_batch)
    t0 = time.perf_counter()
    ev_loop[0].record(stream)
    for k in range(args.steps):
        if k in ev:
            ev[k][0].record(stream)
        sweep.local_partials(cov, v_sweep, want_bf, v_layout, out=pipe.local[k])
        if k in ev:
            ev[k][1].record(stream)
        pipe.exchange(k)
    ev_loop[1].record(stream)
    per_sweep = pipe.finish()
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if distributed:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev.values()]))
    loop_ms = ev_loop[0].elapsed_time(ev_loop[1]) / args.steps
    p = per_sweep[-1].cpu().numpy()
    assert all(np.array_equal(q, p, equal_nan=True) for q in per_sweep.cpu().numpy()), \
        "sweeps of the same field must give identical partials"
    ll = -0.5 * (n_total * np.log(2 * np.pi) + p[0] + p[1])

    if rank == 0:
        bpl = bytes_per_location(args.m) if want_bf else bytes_per_location(args.m) - 8 * args.m - 8
        # a planned sweep also streams its wave pair plan: those bytes count as the sweep's input
        plan_bpl = (sweep.plan_read_bytes / rows if sweep._plan_for(args.kind) is not None and rows > 0 else 0.0)
        achieved = (bpl + plan_bpl) * rows / (kern_ms * 1e-3)
        fpl = flops_per_location(args.m)
        traffic, traffic_src = args.pmc_traffic, "--pmc-traffic" if args.pmc_traffic is not None else None
        if traffic is None:
            traffic, traffic_src = committed_traffic(args, want_bf)
        out = {
            "metric": METRIC,
            "value": n_total * args.steps / elapsed,
            "unit": "locations/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / args.steps,
            "sweeps_per_s": args.steps / elapsed,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: uniform [0,1]^2 coords + N(0,1) values, numpy default_rng(0)" + (
                "; values resident in the engine's Z-order storage layout" if args.layout == "storage" else ""),
            "config": {
                "workload": "BASELINE config 3: fused B/F + log-lik sweep, N=1,000,000 locations per GPU, m=15, "
                            "exponential covariance" if (args.n == 1_000_000 and args.m == 15
                                                         and args.kind == "exponential") else
                            (f"BASELINE config {args.config}: " if args.config else "")
                            + f"fused B/F + log-lik sweep, N={args.n} per GPU, m={args.m}, {args.kind}",
                "n_per_gpu": args.n,
                "n_total": n_total,
                "m": args.m,
                "kind": args.kind,
                "theta": [sigma2, phi, tau2] + ([args.nu] if args.kind == "matern" else []),
                "algo": args.algo,
                "row_order": "index" if args.no_order else "z-order",
                "layout": args.layout,
                "write_BF": want_bf,
                "pair_plan": ({"tiles_planned": sweep._plan_ctypes.n_planned,
                               "tiles_direct": sweep._plan_ctypes.n_direct, "build_s": sweep.plan_build_s,
                               "bytes": int(sweep._plan[0].numel())}
                              if sweep._plan_for(args.kind) is not None else None),
                "sweep_api": "torch.ops.nngp.bf_sweep_out" if args.sweep_api == "ops" else "ctypes",
                "global_batch": n_total,
                "parallelism": f"dp{world} (contiguous Z-order location shards; the (4,) partials of every "
                               f"{args.exchange_batch} sweeps in one RCCL all-gather, overlapped with the next sweeps, "
                               "then a rank-order fold)",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved / 1e9,
                "peak": HBM_PEAK / 1e9,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK,
                "traffic": traffic,
                "traffic_source": traffic_src,
                "algorithmic_bytes_per_location": bpl + plan_bpl,
                "plan_bytes_per_location": plan_bpl,
                "frac_without_plan_bytes": bpl * rows / (kern_ms * 1e-3) / HBM_PEAK,
                "kernel_ms": kern_ms,
                "kernel_ms_samples": len(ev),
                "event_stride": stride,
                "kernel_ms_loop": loop_ms,
                "kernel_ms_loop_samples": args.steps,
                "kernel_rows": rows,
            },
            "roofline_valu": valu_roofline(committed_profile(args, want_bf), rows, kern_ms),
            "roofline_fp64": {
                "achieved": fpl * rows / (kern_ms * 1e-3) / 1e12,
                "peak": FP64_PEAK / 1e12,
                "unit": "TFLOP/s",
                "frac": fpl * rows / (kern_ms * 1e-3) / FP64_PEAK,
                "algorithmic_flops_per_location": fpl,
            },
            "neighbor_build_s": knn_s,
            "loglik": ll,
            "bad_rows": [int(p[2]), int(p[3])],
            "collective": "torch.distributed all_gather_into_tensor (" + dist.get_backend() + ") + rank-order fold"
                          if distributed else "none (one rank)",
            "lib": os.path.relpath(_lib.LIB_PATH, ROOT),
        }
        if world == 1 and args.cpu_seconds > 0:
            F_gpu = sweep.F.cpu().numpy() if want_bf else None
            c_sw = sweep._coords_sweep  # storage- or input-order coordinates the rows / nbr refer to
            if F_gpu is None:
                _, F_t, _ = _lib.bf_sweep(c_sw, sweep.nbr, 0, cov.kind, *cov.theta, nu=cov.nu_arg)
                F_gpu = F_t.cpu().numpy()
            out["neighbor_build_cpu"] = knn_cpu_baseline(coords, args.m, n_total)
            out["cpu_baseline"] = cpu_baseline(c_sw.cpu().numpy(), values, sweep.nbr.cpu().numpy(), args.kind,
                                               (sigma2, phi, tau2) + ((args.nu,) if args.kind == "matern" else ()),
                                               args.cpu_seconds, F_gpu)
        sys.stdout.flush()
        os.write(json_fd, (json.dumps(out) + "\n").encode())
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
