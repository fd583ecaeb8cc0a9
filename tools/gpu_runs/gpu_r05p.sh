#!/bin/bash
# Round 5: config 2 (N = 1e5, m = 15, Matern-3/2) on each kernel: the one-lane kernel fills the GPU in one round
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/r05p
mkdir -p $o
for a in pairb lane quad wave; do
  timeout -k 10 300 python bench.py --config 2 --algo $a --cpu-seconds 0 --steps 2000 --warmup 2000 > $o/c2_$a.json 2> $o/c2_$a.err || { tail -3 $o/c2_$a.err; continue; }
  python -c "import json; d=json.load(open('$o/c2_$a.json')); print('c2 $a', round(d['ms_per_step'], 5), round(d['roofline']['kernel_ms'], 5))"
done
for n in 50000 200000 400000; do
  for a in pairb lane; do
    timeout -k 10 300 python bench.py --config 2 --n $n --algo $a --cpu-seconds 0 --steps 1000 --warmup 1000 > $o/c2_${n}_$a.json 2> $o/c2_${n}_$a.err || { tail -3 $o/c2_${n}_$a.err; continue; }
    python -c "import json; d=json.load(open('$o/c2_${n}_$a.json')); print('n $n $a', round(d['ms_per_step'], 5))"
  done
done
