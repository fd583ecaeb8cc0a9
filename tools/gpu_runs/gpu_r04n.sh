#!/bin/bash
# Round 4 probe: the four-lane kernel (bf_group<15, KIND, 4>) against the pair kernel at config 2's small
# field (N = 1e5: 1.5 rounds of two-wave slots for the pair kernel) and at config 3.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/r04n
mkdir -p $o
VARIANTS="pair:ab/base/libnngp_hip.so:auto quad:ab/quad15/libnngp_hip.so:quad" REPS=3 STEPS=2000 WARMUP=3000 \
  bash tools/gpu_ab.sh --config 2 > $o/ab_c2.txt 2>&1 || exit 1
mkdir -p $o/c2 && mv gpurun_out/ab/*.json $o/c2/
VARIANTS="pair:ab/base/libnngp_hip.so:auto quad:ab/quad15/libnngp_hip.so:quad" REPS=2 STEPS=300 WARMUP=300 \
  bash tools/gpu_ab.sh > $o/ab_c3.txt 2>&1 || exit 1
