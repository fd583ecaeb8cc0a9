#!/bin/bash
# Round 4: the record fold with the tile count from the launch and 16 records in flight per thread --
# same-box A/B at configs 2 and 3 (kernel_ms covers sweep + fold), plus kernel traces of both builds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/r04m
mkdir -p $o
VARIANTS="base:ab/base/libnngp_hip.so:auto fold16:ab/fold16/libnngp_hip.so:auto" REPS=3 STEPS=2000 WARMUP=3000 \
  bash tools/gpu_ab.sh --config 2 > $o/ab_c2.txt 2>&1 || exit 1
mkdir -p $o/c2 && mv gpurun_out/ab/*.json $o/c2/
VARIANTS="base:ab/base/libnngp_hip.so:auto fold16:ab/fold16/libnngp_hip.so:auto" REPS=3 STEPS=300 WARMUP=300 \
  bash tools/gpu_ab.sh > $o/ab_c3.txt 2>&1 || exit 1
mkdir -p $o/c3 && mv gpurun_out/ab/*.json $o/c3/
for v in base fold16; do
  NNGP_LIB=ab/$v/libnngp_hip.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $o/trace_$v -o run -- \
    python3 bench.py --config 2 --steps 500 --warmup 500 --cpu-seconds 0 > $o/trace_$v.json 2> $o/trace_$v.err || exit 1
done
