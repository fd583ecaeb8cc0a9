#!/bin/bash
# Round 4 timing probe: the exp table read from LDS replaced by register arithmetic (NNGP_PROBE_NO_TABLE, wrong values) -- what the LDS latency of the covariance phase costs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/r04s
mkdir -p $o
VARIANTS="base:ab/base/libnngp_hip.so:auto notab:ab/notab/libnngp_hip.so:auto" REPS=3 STEPS=400 WARMUP=400 \
  bash tools/gpu_ab.sh > $o/ab_c3.txt 2>&1 || exit 1
