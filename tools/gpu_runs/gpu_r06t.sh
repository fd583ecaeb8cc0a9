#!/bin/bash
# Round 6: the node-order checkpoint fingerprint -- the Gibbs GPU tests (checkpoint / resume across storage
# orders, sharded chain, chains, colour sweep)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/r06t
mkdir -p $o
timeout -k 10 800 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gibbs_ref.py \
  tests/test_gpu_gibbs_sharded.py tests/test_gpu_gibbs_chains.py tests/test_gpu_gibbs.py -p no:cacheprovider > $o/tests.txt 2>&1 \
  || { tail -30 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
