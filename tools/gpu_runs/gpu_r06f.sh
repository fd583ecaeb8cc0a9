#!/bin/bash
# Round 6: the tiled Gibbs sweep -- its parity tests, then colour vs tiled iteration and w-sweep times
# (same box), then the tiled kernel's trace and L2 fetch / write bytes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/r06f
mkdir -p $o
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_gibbs_tiles.py \
  > $o/tests.log 2>&1 || { tail -40 $o/tests.log; exit 1; }
tail -3 $o/tests.log
for sw in colour tiled colour tiled; do
  timeout -k 10 300 python tools/bench_gibbs.py --iters 200 --warmup 100 --sweep $sw >> $o/ab.jsonl 2>> $o/ab.err || exit 1
done
cat $o/ab.jsonl
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $o/tiled_trace -o run -- \
  python3 tools/bench_gibbs.py --iters 50 --warmup 20 --sweep tiled > $o/tiled_trace.json 2> $o/tiled_trace.err || exit 1
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $o/tiled_fetch -o run -- \
  python3 tools/bench_gibbs.py --iters 30 --warmup 10 --sweep tiled > $o/tiled_fetch.json 2> $o/tiled_fetch.err || exit 1
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $o/tiled_write -o run -- \
  python3 tools/bench_gibbs.py --iters 30 --warmup 10 --sweep tiled > $o/tiled_write.json 2> $o/tiled_write.err || exit 1
python3 - $o <<'PY'
import csv, glob, sys, collections
o = sys.argv[1]
for r in csv.DictReader(open(glob.glob(f'{o}/tiled_trace/**/*kernel_stats.csv', recursive=True)[0])):
    if 'gibbs' in r['Name'] or 'bf_pairb' in r['Name']:
        print(r['Name'][:40], r['Calls'], round(float(r['AverageNs']) / 1e3, 2), 'us avg', round(float(r['TotalDurationNs']) / 1e6 / 70, 4), 'ms/iter (70 it + 100 w sweeps)')
for k in ('fetch', 'write'):
    agg = collections.defaultdict(list)
    for f in glob.glob(f'{o}/tiled_{k}/**/*counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            if 'gibbs_tile_phase' in r['Kernel_Name']:
                agg[r['Counter_Name']].append(float(r['Counter_Value']))
    for c, v in agg.items():
        print('gibbs_tile_phase', c, 'launches', len(v), 'sum per launch avg', round(sum(v) / len(v) / 1e3, 3), 'MB (kB units)')
PY
