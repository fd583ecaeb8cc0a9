#!/bin/bash
# Round 4: the colour kernel without the inline-Philox code in the z-given instantiation (70 -> 46 VGPRs,
# 7 -> 8 waves per SIMD): same-box A/B on the Gibbs iteration at N = 1e6.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r04l
VARIANTS="base:pynngp_amd/_build/libnngp_hip.so split:ab/gsplit/libnngp_hip.so" REPS=4 \
  bash tools/gpu_ab_gibbs.sh --iters 300 --warmup 100 > gpurun_out/r04l/ab_gibbs.txt 2>&1 || exit 1
cp -r gpurun_out/abg gpurun_out/r04l/abg
