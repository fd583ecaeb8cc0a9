#!/bin/bash
# Round 5: left-looking pair kernel at m = 21 / 23 / 24 (variants ab/left2w, ab/left1w7) vs the
# right-looking default -- parity on the variants, then interleaved kernel timings at N = 1e6
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r05z
for v in left2w left1w7; do
  NNGP_LIB=ab/$v/libnngp_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_bf.py -k "pairb_all_m and (21 or 23 or 24)" \
    -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r05z/pytest_$v.txt 2>&1 || { tail -20 gpurun_out/r05z/pytest_$v.txt; exit 1; }
  tail -1 gpurun_out/r05z/pytest_$v.txt
done
for rep in 1 2; do
  for v in base left2w left1w7; do
    lib=pynngp_amd/_build/libnngp_hip.so; [ $v != base ] && lib=ab/$v/libnngp_hip.so
    NNGP_LIB=$lib timeout -k 10 300 python tools/algo_table.py --ms 21-24 --algos pairb > gpurun_out/r05z/algo_${v}_$rep.jsonl || exit 1
  done
done
