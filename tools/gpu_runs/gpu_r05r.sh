#!/bin/bash
# Round 5: Matern sweeps after the coincident-point fix of the small-nu branch (the four-lane kernel at m = 28)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/r05r
mkdir -p $o
run() {
  timeout -k 10 300 python bench.py --cpu-seconds 0 --steps 30 --warmup 30 $2 > $o/$1.json 2> $o/$1.err || { tail -5 $o/$1.err; exit 1; }
  python -c "import json; d=json.load(open('$o/$1.json')); print('$1', round(d['ms_per_step'], 4), d['bad_rows'])"
}
T="--theta 1.0,30.0,0.1"
run m15_matern32 "--kind matern32 $T"
for nu in 0.01 0.05 0.5 1.7; do run m15_nu$nu "--kind matern --nu $nu $T"; done
run m28_matern32 "--kind matern32 --m 28 $T"
for nu in 0.01 0.3 1.7; do run m28_nu$nu "--kind matern --nu $nu --m 28 $T"; done
timeout -k 10 600 python -u -m pytest tests/test_gpu_matern.py -q --timeout 120 --timeout-method thread -p no:cacheprovider > $o/pytest.txt 2>&1; rc=$?
grep -E "^(FAILED|ERROR)" $o/pytest.txt | head; tail -1 $o/pytest.txt
exit $rc
