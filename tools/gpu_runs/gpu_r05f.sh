#!/bin/bash
# Round 5: same-box A/B of the planned pair kernel (configs 3 and 2: duration, VALU, occupancy, clock),
# then kernel traces of config 5 with one chain and with four batched chains.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
bash tools/ab_clock.sh r05f "c3_off||--plan off" "c3_on||--plan on" "c2_off||--config 2 --plan off" "c2_on||--config 2 --plan on" || exit 1
for c in 1 4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05f/c5x${c}_trace -o run -- \
    python3 bench.py --config 5 --chains-per-gpu $c --cpu-seconds 0 --steps 50 --warmup 10 > gpurun_out/r05f/c5x${c}.json 2> gpurun_out/r05f/c5x${c}.err || exit 1
  f=$(find gpurun_out/r05f/c5x${c}_trace -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
tot=sum(float(r['TotalDurationNs']) for r in rows)
for r in rows[:12]: print('c5x$c', r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3,2), 'us', round(float(r['TotalDurationNs'])/tot,3))
"
done
