#!/bin/bash
# Round 5: the callable plug-in evaluated once per distinct point pair -- GPU tests and the block times
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/r05o
mkdir -p $o
timeout -k 10 900 python -u -m pytest tests/test_gpu_callable_cov.py tests/test_gpu_api.py -q --timeout 120 --timeout-method thread -p no:cacheprovider > $o/pytest.txt 2>&1; rc=$?
grep -E "^(FAILED|ERROR)" $o/pytest.txt | head; tail -1 $o/pytest.txt
case $rc in 0) ;; *) tail -40 $o/pytest.txt; exit $rc;; esac
timeout -k 10 600 env PYTHONPATH=. python -u tools/bench_custom_cov.py > $o/custom.json 2> $o/custom.err || { tail -20 $o/custom.err; exit 1; }
cat $o/custom.json
