#!/bin/bash
# Round 6: the covariance-blocks kind left-looking at m = 18..24 in the product build -- the callable /
# custom-covariance and pair-kernel GPU tests, then the blocks sweep times at N = 10^6
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/r06q
mkdir -p $o
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_callable_cov.py tests/test_gpu_custom_cov.py tests/test_gpu_matern.py tests/test_gpu_bf.py -p no:cacheprovider > $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
timeout -k 10 300 python tools/bench_blocks_m.py 18 19 20 21 22 23 24 > $o/blocks.json 2>> $o/err.log || exit 1
cat $o/blocks.json
