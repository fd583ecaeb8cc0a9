#!/bin/bash
# Round 5: timing probe -- the batched colour kernel without its per-chain scalar loads (wrong draws; an upper
# bound for interleaving them), same box
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/r05x
mkdir -p $o
A="--config 5 --chains-per-gpu 4 --chain-mode batched --cpu-seconds 0 --steps 200 --warmup 30"
for r in 1 2; do
  timeout -k 10 300 python bench.py $A > $o/base_$r.json 2> $o/base_$r.err || exit 1
  python -c "import json; d=json.load(open('$o/base_$r.json')); print('base', round(d['value'], 1))"
  timeout -k 10 300 env NNGP_LIB=ab/noscalars/libnngp_hip.so python bench.py $A > $o/probe_$r.json 2> $o/probe_$r.err || exit 1
  python -c "import json; d=json.load(open('$o/probe_$r.json')); print('probe', round(d['value'], 1))"
done
