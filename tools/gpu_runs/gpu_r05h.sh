#!/bin/bash
# Round 5: general-smoothness Matern on the table kernels -- sweep time per nu at N = 1e6 (m = 15 and the
# four-lane m = 28) against Matern-3/2 and the wavefront kernel (tau2 = 0.1: smooth nu are singular without)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/r05h
mkdir -p $o
run() {  # name, args
  timeout -k 10 300 python bench.py --cpu-seconds 0 --steps 30 --warmup 30 $2 > $o/$1.json 2> $o/$1.err || { tail -5 $o/$1.err; exit 1; }
  python -c "import json; d=json.load(open('$o/$1.json')); print('$1', round(d['ms_per_step'], 4), round(d['roofline']['kernel_ms'], 4), d['config'].get('algo'), d['bad_rows'])"
}
T="--theta 1.0,30.0,0.1"
run n_m15_matern32 "--kind matern32 $T"
for nu in 0.05 0.5 10 49; do run n_m15_nu$nu "--kind matern --nu $nu $T"; done
run m15_nu0.5_wave "--kind matern --nu 0.5 --algo wave"
run m15_nu0.5_pairb "--kind matern --nu 0.5"
run m28_matern32 "--kind matern32 --m 28 $T"
for nu in 0.3 1.7 10; do run m28_nu$nu "--kind matern --nu $nu --m 28 $T"; done
run m28_nu0.3_wave "--kind matern --nu 0.3 --m 28 --algo wave $T"
