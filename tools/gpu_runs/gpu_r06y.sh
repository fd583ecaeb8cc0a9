#!/bin/bash
# round 6: the colour loop's launch floor -- w sweep eager vs replayed from a HIP graph (timing probe)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/r06y
mkdir -p $o
for k in 1 2; do
timeout -k 10 300 python3 tools/bench_gibbs.py --iters 300 --warmup 100 --graph-probe >> $o/probe.jsonl 2>> $o/err.log || exit 1
done
python3 -c "
import json
for l in open('$o/probe.jsonl'):
    d=json.loads(l); print(round(d['ms_per_iter'],4), 'eager', round(d['w_sweep_ms'],4), 'graph', round(d['w_sweep_graph_ms'],4))"
