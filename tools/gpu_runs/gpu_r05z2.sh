#!/bin/bash
# Round 5: left-looking pair kernel at m = 19..24 (new default) -- parity suites that cover m = 21..24,
# then interleaved kernel timings against the previous mask (ab/r04mask) for two kinds
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r05z2
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf.py tests/test_gpu_dims.py tests/test_gpu_cross.py tests/test_gpu_api.py tests/test_gpu_maxsize.py \
  -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r05z2/pytest.txt 2>&1 || { tail -30 gpurun_out/r05z2/pytest.txt; exit 1; }
tail -1 gpurun_out/r05z2/pytest.txt
for kind in exponential matern32; do
  for rep in 1 2; do
    for v in new old; do
      lib=pynngp_amd/_build/libnngp_hip.so; [ $v = old ] && lib=ab/r04mask/libnngp_hip.so
      NNGP_LIB=$lib timeout -k 10 300 python tools/algo_table.py --ms 19-24 --algos pairb --kind $kind > gpurun_out/r05z2/algo_${kind}_${v}_$rep.jsonl || exit 1
    done
  done
done
