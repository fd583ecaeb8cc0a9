#!/bin/bash
# Round 5: the left-looking pair kernel at m = 25..32 -- parity (every kind / dimension, vs the C oracle),
# then the kernel table against the four-lane kernel at N = 1e6
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r05z3
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf.py -k "pairb_all_m or pairb_m25_32 or large_m" \
  -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r05z3/pytest.txt 2>&1 || { tail -30 gpurun_out/r05z3/pytest.txt; exit 1; }
tail -1 gpurun_out/r05z3/pytest.txt
for kind in exponential matern32 gaussian; do
  timeout -k 10 400 python tools/algo_table.py --ms 25-32 --algos pairb,quad --kind $kind --rounds 4 > gpurun_out/r05z3/algo_$kind.jsonl || exit 1
done
