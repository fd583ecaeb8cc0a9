#!/bin/bash
# Round 5: diagnose the planned/unplanned mismatch at m = 13, then the other new GPU test files.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/r05c
mkdir -p $o
timeout -k 10 300 env PYTHONPATH=. python -u tools/diag_plan.py --m 11 12 13 14 15 > $o/diag.txt 2>&1 || { tail -30 $o/diag.txt; exit 1; }
cat $o/diag.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf.py tests/test_gpu_fullsize.py -k "pairb or auto or 19 or 20 or 22" -x -q --timeout 120 --timeout-method thread > $o/pytest_bf.txt 2>&1 || { tail -40 $o/pytest_bf.txt; exit 1; }
tail -2 $o/pytest_bf.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_gibbs_chains.py tests/test_gpu_callable_cov.py \
  tests/test_gpu_matern.py tests/test_gpu_api.py tests/test_gpu_gibbs.py tests/test_gpu_gibbs_sharded.py -v --timeout 120 --timeout-method thread \
  > $o/pytest_rest.txt 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR" $o/pytest_rest.txt | grep -v PASSED | head -40
tail -3 $o/pytest_rest.txt
exit $rc
