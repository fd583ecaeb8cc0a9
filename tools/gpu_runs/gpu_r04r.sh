#!/bin/bash
# Round 4 timing probe: how much of the m = 15 sweep is the tile-start gather chain?  NNGP_PAIRB_PROBE_LOCAL
# replaces the neighbour-index load by the preceding storage rows (no index round trip; cache-resident
# coordinates) -- the same instruction stream; an upper bound on what a prefetching schedule could save.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/r04r
mkdir -p $o
VARIANTS="base:ab/base/libnngp_hip.so:auto local:ab/plocal/libnngp_hip.so:auto" REPS=3 STEPS=400 WARMUP=400 \
  bash tools/gpu_ab.sh > $o/ab_c3.txt 2>&1 || exit 1
