#!/bin/bash
# Round 5: Matern-nu table in LDS (default) vs read in place from global memory (ab/mtglobal), same box
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/r05s
mkdir -p $o
run() {  # name, env, args
  timeout -k 10 300 env $2 python bench.py --cpu-seconds 0 --steps 30 --warmup 30 $3 > $o/$1.json 2> $o/$1.err || { tail -5 $o/$1.err; exit 1; }
  python -c "import json; d=json.load(open('$o/$1.json')); print('$1', round(d['ms_per_step'], 4), d['bad_rows'], d['loglik'])"
}
T="--theta 1.0,30.0,0.1"
for r in 1 2; do
  for nu in 0.5 1.7; do
    run lds_nu${nu}_$r "" "--kind matern --nu $nu $T"
    run glob_nu${nu}_$r "NNGP_LIB=ab/mtglobal/libnngp_hip.so" "--kind matern --nu $nu $T"
  done
done
