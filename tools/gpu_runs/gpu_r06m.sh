#!/bin/bash
# Round 6: config 2 with and without wave plans (same box, alternating), config 2's kernel counters, and the
# tiled Gibbs sweep's L2 fetch / write per launch (final tiled configuration)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/r06m
mkdir -p $o
for r in 1 2; do for p in off on; do
  timeout -k 10 300 python bench.py --config 2 --steps 500 --warmup 3000 --cpu-seconds 0 --plan $p > $o/c2_$p.$r.json 2> $o/c2_$p.$r.err || exit 1
done; done
for f in $o/c2_*.json; do python3 -c "import json,sys; d=json.load(open('$f')); print('$f', round(d['ms_per_step']*1e3,2), 'us/step', 'kernel', round(d['roofline']['kernel_ms']*1e3,2))"; done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $o/c2_trace -o run -- python3 bench.py --config 2 --steps 500 --warmup 3000 --cpu-seconds 0 > $o/c2_trace.json 2> $o/c2_trace.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES --output-format csv -d $o/c2_sq -o run -- python3 bench.py --config 2 --steps 200 --warmup 200 --cpu-seconds 0 > $o/c2_sq.json 2> $o/c2_sq.err || exit 1
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $o/tile_fetch -o run -- python3 tools/bench_gibbs.py --iters 30 --warmup 10 --sweep tiled > $o/tile_fetch.json 2> $o/tile_fetch.err || exit 1
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $o/tile_write -o run -- python3 tools/bench_gibbs.py --iters 30 --warmup 10 --sweep tiled > $o/tile_write.json 2> $o/tile_write.err || exit 1
python3 - $o <<'PY'
import csv, glob, sys, collections
o = sys.argv[1]
for r in csv.DictReader(open(glob.glob(f'{o}/c2_trace/**/*kernel_stats.csv', recursive=True)[0])):
    print('c2', r['Name'][:44], r['Calls'], round(float(r['AverageNs']) / 1e3, 2), 'us avg')
agg = collections.defaultdict(list)
for f in glob.glob(f'{o}/c2_sq/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'bf_pairb' in r['Kernel_Name']:
            agg[r['Counter_Name']].append(float(r['Counter_Value']))
a = {k: sum(v) / len(v) for k, v in agg.items()}
w = a.get('SQ_WAVES', 1)
print('c2 per wave', {k: round(v / w, 1) for k, v in sorted(a.items()) if k not in ('SQ_WAVES', 'SQ_BUSY_CYCLES')}, 'waves', w, 'busy', a.get('SQ_BUSY_CYCLES'))
for k in ('fetch', 'write'):
    t = collections.defaultdict(list)
    for f in glob.glob(f'{o}/tile_{k}/**/*counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            if 'gibbs' in r['Kernel_Name']:
                t[(r['Kernel_Name'][:30], r['Counter_Name'])].append(float(r['Counter_Value']))
    for (kn, c), v in sorted(t.items()):
        print('tiled', kn, c, 'launches', len(v), 'avg per launch kB', round(sum(v) / len(v), 1), 'sum per launch-set', round(sum(v), 1))
PY
