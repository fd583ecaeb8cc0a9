#!/bin/bash
# round 6: colour-major rows + fixed reverse-entry slots (nngp_gibbs_w_sweep_cm): parity, then the A/B
set -o pipefail
O=gpurun_out/r06x
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gibbs_cm.py \
    tests/test_gpu_gibbs.py tests/test_gpu_gibbs_ref.py tests/test_gpu_gibbs_chains.py tests/test_gpu_gibbs_sharded.py \
    tests/test_gpu_gibbs_tiles.py > $O/tests.log 2>&1 && \
for L in z colour z colour; do
  timeout -k 10 300 python -u tools/bench_gibbs.py --iters 300 --warmup 100 --layout $L >> $O/ab.jsonl 2>>$O/err.log || exit 1
done
