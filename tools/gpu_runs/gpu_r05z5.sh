#!/bin/bash
# Round 5: left-looking pair kernel at m = 16..18 (variant ab/left16) vs the right-looking default
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r05z5
NNGP_LIB=ab/left16/libnngp_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_bf.py -k "pairb_all_m and (16 or 17 or 18)" \
  -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r05z5/pytest_left16.txt 2>&1 || { tail -20 gpurun_out/r05z5/pytest_left16.txt; exit 1; }
tail -1 gpurun_out/r05z5/pytest_left16.txt
for kind in exponential matern32; do
  for rep in 1 2; do
    for v in right left16; do
      lib=pynngp_amd/_build/libnngp_hip.so; [ $v != right ] && lib=ab/$v/libnngp_hip.so
      NNGP_LIB=$lib timeout -k 10 300 python tools/algo_table.py --ms 16-18 --algos pairb --kind $kind > gpurun_out/r05z5/algo_${kind}_${v}_$rep.jsonl || exit 1
    done
  done
done
