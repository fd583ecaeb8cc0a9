#!/bin/bash
# round 6: the colour kernel's workgroup size (128 / 256 / 512 / 1024 threads), interleaved, same box
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
o=gpurun_out/r06ac
mkdir -p $o
for rep in 1 2; do
  for v in base bs128 bs512 bs1024; do
    if [ $v = base ]; then lib=""; else lib=$PWD/ab/colour_$v/libnngp_hip.so; fi
    NNGP_LIB=$lib timeout -k 10 300 python3 tools/bench_gibbs.py --iters 300 --warmup 100 > $o/$v.$rep.json 2>> $o/err.log || exit 1
    python3 -c "import json; d=json.load(open('$o/$v.$rep.json')); print('$v', round(d['ms_per_iter'],4), round(d['w_sweep_ms'],4))"
  done
done
