#!/bin/bash
# round 6: the tile plan's launch-bound validation (gibbs_w_sweep_tiles) on the GPU tests and at N = 1e6
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
o=gpurun_out/r06ad
mkdir -p $o
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gibbs_tiles.py tests/test_gpu_gibbs_ref.py > $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
tail -2 $o/tests.txt
timeout -k 10 300 python3 - > $o/validate.txt 2>&1 <<'PY' || { cat $o/validate.txt; exit 1; }
import time, numpy as np, torch
from pynngp_amd import SeqNNGP
from pynngp_amd.gibbs_tiles import validate_launch_bounds
rng = np.random.default_rng(2)
n = 1_000_000
c = rng.uniform(0, 1, (n, 2)); y = 1.0 + rng.standard_normal(n) * 0.5
g = SeqNNGP(c, y, m=15, phi=30.0, seed=1, device="cuda", sweep="tiled")
torch.cuda.synchronize(); t0 = time.perf_counter()
validate_launch_bounds(g._tiles, g.off, n)
torch.cuda.synchronize(); print("validate_launch_bounds at N=1e6:", round(1e3 * (time.perf_counter() - t0), 1), "ms")
g.sample(5); print("sampled ok", g.iteration)
PY
cat $o/validate.txt
