#!/bin/bash
# Round 4: the maximum-size parity test (N = 1.5e8, past 2^31 entries), then a same-box A/B of the
# first-round stagger probe (NNGP_PAIRB_STAGGER) at configs 3 and 4.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/r04k
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -v -s --durations=5 --timeout 550 --timeout-method thread tests/test_gpu_maxsize.py > $o/pytest_maxsize.txt 2>&1 || exit 1
VARIANTS="base:ab/base/libnngp_hip.so:auto s5:ab/stag5/libnngp_hip.so:auto s10:ab/stag10/libnngp_hip.so:auto" REPS=3 STEPS=300 WARMUP=300 \
  bash tools/gpu_ab.sh > $o/ab_c3.txt 2>&1 || exit 1
mkdir -p $o/c3 && mv gpurun_out/ab/*.json $o/c3/
VARIANTS="base:ab/base/libnngp_hip.so:auto s5:ab/stag5/libnngp_hip.so:auto s10:ab/stag10/libnngp_hip.so:auto" REPS=3 STEPS=30 WARMUP=30 \
  bash tools/gpu_ab.sh --config 4 > $o/ab_c4.txt 2>&1 || exit 1
