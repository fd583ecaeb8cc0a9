#!/bin/bash
# Round 4: the table exp with its polynomial before the table value is used (NNGP_EXP_POLY_FIRST; with a
# scheduling barrier after it: NNGP_EXP_POLY_BARRIER) -- the same arithmetic (same bits), the LDS read of
# the exp table further from its first use.  Same-box A/B at config 3.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/r04u
mkdir -p $o
VARIANTS="base:ab/base/libnngp_hip.so:auto pf:ab/pf/libnngp_hip.so:auto pfb:ab/pfb/libnngp_hip.so:auto" REPS=4 STEPS=400 WARMUP=400 \
  bash tools/gpu_ab.sh > $o/ab_c3.txt 2>&1 || exit 1
