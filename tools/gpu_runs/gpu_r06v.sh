#!/bin/bash
# Round 6: the padded colour sweep (nngp_gibbs_w_sweep_pad) -- the Gibbs GPU tests (bit identity with the CSR
# sweep, chains, sharded, checkpoint), then padded vs CSR iteration and w-sweep times (same box, alternating)
# and the colour kernels' durations
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/r06v
mkdir -p $o
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gibbs.py \
  tests/test_gpu_gibbs_chains.py tests/test_gpu_gibbs_sharded.py tests/test_gpu_gibbs_ref.py tests/test_gpu_gibbs_tiles.py \
  -p no:cacheprovider > $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
for r in 1 2 3; do for v in pad csr; do
  timeout -k 10 200 python tools/bench_gibbs.py --iters 300 --warmup 100 $([ $v = csr ] && echo --csr) > $o/$v.$r.json 2>> $o/err.log || exit 1
  python3 -c "import json; d=json.load(open('$o/$v.$r.json')); print('$v', round(d['w_sweep_ms'],4), 'ms per w sweep', round(d['ms_per_iter'],4), 'ms/iter', d['padded'])"
done; done
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $o/trace -o run -- \
  python3 tools/bench_gibbs.py --iters 50 --warmup 20 > $o/trace.json 2> $o/trace.err || exit 1
python3 - $o <<'PY'
import csv, glob, sys
o = sys.argv[1]
for r in csv.DictReader(open(glob.glob(f'{o}/trace/**/*kernel_stats.csv', recursive=True)[0])):
    if 'gibbs' in r['Name'] or 'bf_pairb' in r['Name']:
        print(r['Name'][:40], r['Calls'], round(float(r['AverageNs']) / 1e3, 2), 'us avg')
PY
