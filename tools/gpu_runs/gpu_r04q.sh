#!/bin/bash
# Round 4 probe: the separate record fold with 512 / 1,024 threads (fewer load rounds per thread at config 3's
# 7,813 records) against 256 -- same-box A/B at configs 3 and 2 (kernel_ms = sweep + fold).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/r04q
mkdir -p $o
V="base:ab/base/libnngp_hip.so:auto f512:ab/f512/libnngp_hip.so:auto f1024:ab/f1024/libnngp_hip.so:auto"
VARIANTS="$V" REPS=3 STEPS=400 WARMUP=400 bash tools/gpu_ab.sh > $o/ab_c3.txt 2>&1 || exit 1
mkdir -p $o/c3 && mv gpurun_out/ab/*.json $o/c3/
VARIANTS="$V" REPS=3 STEPS=2000 WARMUP=3000 bash tools/gpu_ab.sh --config 2 > $o/ab_c2.txt 2>&1 || exit 1
for v in base f1024; do
  NNGP_LIB=ab/$v/libnngp_hip.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $o/trace_$v -o run -- \
    python3 bench.py --steps 300 --warmup 300 --cpu-seconds 0 > $o/trace_$v.json 2> $o/trace_$v.err || exit 1
done
