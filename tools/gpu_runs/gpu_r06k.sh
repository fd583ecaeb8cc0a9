#!/bin/bash
# Round 6: colour-major storage for the colour sweep -- the Gibbs GPU tests, then colour vs z layout (same box,
# alternating), then the colour kernel's trace and L2 fetch in the colour layout
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/r06k
mkdir -p $o
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gibbs.py \
  tests/test_gpu_gibbs_chains.py tests/test_gpu_gibbs_ref.py tests/test_gpu_gibbs_sharded.py tests/test_gpu_gibbs_tiles.py \
  > $o/tests.log 2>&1 || { tail -40 $o/tests.log; exit 1; }
tail -2 $o/tests.log
for lay in colour z colour z; do
  timeout -k 10 300 python tools/bench_gibbs.py --iters 300 --warmup 100 --layout $lay >> $o/ab.jsonl 2>> $o/ab.err || exit 1
done
cat $o/ab.jsonl
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $o/trace -o run -- \
  python3 tools/bench_gibbs.py --iters 50 --warmup 20 > $o/trace.json 2> $o/trace.err || exit 1
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $o/fetch -o run -- \
  python3 tools/bench_gibbs.py --iters 30 --warmup 10 > $o/fetch.json 2> $o/fetch.err || exit 1
python3 - $o <<'PY'
import csv, glob, sys, collections
o = sys.argv[1]
for r in csv.DictReader(open(glob.glob(f'{o}/trace/**/*kernel_stats.csv', recursive=True)[0])):
    if 'gibbs' in r['Name'] or 'bf_pairb' in r['Name']:
        print(r['Name'][:40], r['Calls'], round(float(r['AverageNs']) / 1e3, 2), 'us avg')
agg = collections.defaultdict(list)
for f in glob.glob(f'{o}/fetch/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'gibbs_w_color' in r['Kernel_Name']:
            agg[r['Counter_Name']].append(float(r['Counter_Value']))
for c, v in agg.items():
    print('gibbs_w_color', c, 'launches', len(v), 'avg per launch', round(sum(v) / len(v) / 1e3, 2), 'MB (kB units)')
PY
