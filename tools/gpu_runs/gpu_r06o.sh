#!/bin/bash
# Round 6: the Matern kind left-looking at m = 18 in the product build -- its oracle tests, the pair-kernel
# tests, and its time at N = 10^6 (nu = 1.3) beside m = 19
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/r06o
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_matern.py tests/test_gpu_bf.py -p no:cacheprovider > $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
for m in 18 19; do for r in 1 2; do
  timeout -k 10 120 python bench.py --steps 30 --warmup 30 --cpu-seconds 0 --kind matern --nu 1.3 --m $m --n 1000000 > $o/m$m.$r.json 2>> $o/err.log || exit 1
  python3 -c "import json; d=json.load(open('$o/m$m.$r.json')); print('m=$m', round(d['roofline']['kernel_ms'],4), 'ms', d['config'].get('algo'))"
done; done
