#!/bin/bash
# Round 5: Matern table with 8 bins per octave of degree 9 (was 4 of degree 13) -- GPU tests and sweep times
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/r05m
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_matern.py -q --timeout 120 --timeout-method thread -p no:cacheprovider > $o/pytest.txt 2>&1; rc=$?
grep -E "^(FAILED|ERROR)" $o/pytest.txt | head; tail -1 $o/pytest.txt
case $rc in 124|134|137|139) exit $rc;; esac
run() {
  timeout -k 10 300 python bench.py --cpu-seconds 0 --steps 30 --warmup 30 $2 > $o/$1.json 2> $o/$1.err || { tail -5 $o/$1.err; exit 1; }
  python -c "import json; d=json.load(open('$o/$1.json')); print('$1', round(d['ms_per_step'], 4), round(d['roofline']['kernel_ms'], 4), d['bad_rows'])"
}
T="--theta 1.0,30.0,0.1"
run m15_matern32 "--kind matern32 $T"
for nu in 0.05 0.5 1.7 10; do run m15_nu$nu "--kind matern --nu $nu $T"; done
for nu in 0.3 1.7; do run m28_nu$nu "--kind matern --nu $nu --m 28 $T"; done
