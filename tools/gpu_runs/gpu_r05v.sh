#!/bin/bash
# Round 5: config 2 with the record fold fused into the sweep (the outputs stored after the ticket) vs the
# separate fold launch, same box; config 3 default for reference
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/r05v
mkdir -p $o
run() {
  timeout -k 10 300 env $2 python bench.py --cpu-seconds 0 $3 > $o/$1.json 2> $o/$1.err || { tail -5 $o/$1.err; exit 1; }
  python -c "import json; d=json.load(open('$o/$1.json')); print('$1', round(d['ms_per_step'], 5), d['loglik'], d['bad_rows'])"
}
for r in 1 2 3; do
  run c2_sep_$r "" "--config 2 --steps 3000 --warmup 3000"
  run c2_fused_$r "NNGP_LIB=ab/fusedfold/libnngp_hip.so" "--config 2 --steps 3000 --warmup 3000"
done
run c3_default "" ""
