#!/bin/bash
# Round 6: tiled Gibbs sweep v2 (contiguous plan, prefetched steps) -- parity tests, colour vs tiled
# (tile sizes 1024 / 2048 / 4096), then the tiled kernel's trace per launch size
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/r06g
mkdir -p $o
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_gibbs_tiles.py \
  > $o/tests.log 2>&1 || { tail -40 $o/tests.log; exit 1; }
tail -3 $o/tests.log
timeout -k 10 300 python tools/bench_gibbs.py --iters 200 --warmup 100 --sweep colour >> $o/ab.jsonl 2>> $o/ab.err || exit 1
for tn in 2048 1024 4096; do
  timeout -k 10 300 python tools/bench_gibbs.py --iters 200 --warmup 100 --sweep tiled --tile-nodes $tn >> $o/ab.jsonl 2>> $o/ab.err || exit 1
done
cat $o/ab.jsonl
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $o/tiled_trace -o run -- \
  python3 tools/bench_gibbs.py --iters 50 --warmup 20 --sweep tiled > $o/tiled_trace.json 2> $o/tiled_trace.err || exit 1
python3 - $o <<'PY'
import csv, glob, sys, collections
o = sys.argv[1]
d = collections.defaultdict(list)
for r in csv.DictReader(open(glob.glob(f'{o}/tiled_trace/**/*kernel_trace.csv', recursive=True)[0])):
    if 'gibbs_tile_phase' in r['Kernel_Name']:
        d[int(r['Grid_Size_X']) // 1024].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
for k, v in sorted(d.items()):
    print('tiles', k, 'launches', len(v), 'avg us', round(sum(v) / len(v), 1))
PY
