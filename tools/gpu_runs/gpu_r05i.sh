#!/bin/bash
# Round 5: interleaved chains (vector w / r accesses) -- GPU tests, then config 5 with 1 / 2 / 4 / 8 chains,
# interleaved and per-chain layouts on the same box, and a kernel trace at 4 chains
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/r05i
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_gibbs_chains.py -q --timeout 120 --timeout-method thread -p no:cacheprovider > $o/pytest.txt 2>&1; rc=$?
grep -E "^(FAILED|ERROR)" $o/pytest.txt | head; tail -1 $o/pytest.txt
case $rc in 0) ;; *) exit $rc;; esac
b() {  # name, args
  timeout -k 10 400 python bench.py --config 5 --cpu-seconds 0 --steps 300 --warmup 50 $2 > $o/$1.json 2> $o/$1.err || { tail -5 $o/$1.err; exit 1; }
  python -c "import json; d=json.load(open('$o/$1.json')); print('$1', round(d['value'], 1), round(d['ms_per_step'], 4), d['config'].get('chain_mode'))"
}
b c5_1 ""
for c in 2 4 8; do b c5_$c "--chains-per-gpu $c"; b c5_${c}_percopy "--chains-per-gpu $c --chain-mode batched-percopy"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/c5x4_trace -o run -- \
  python3 bench.py --config 5 --chains-per-gpu 4 --cpu-seconds 0 --steps 50 --warmup 10 > $o/c5x4_prof.json 2> $o/c5x4_prof.err || exit 1
f=$(find $o/c5x4_trace -name "*kernel_stats.csv" | head -1)
python3 -c "
import csv
rows=list(csv.DictReader(open('$f')))
tot=sum(float(r['TotalDurationNs']) for r in rows)
for r in rows[:10]: print('c5x4', r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,2), 'us', round(float(r['TotalDurationNs'])/tot,3))
"
