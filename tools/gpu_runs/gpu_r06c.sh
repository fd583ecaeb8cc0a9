#!/bin/bash
# Round 6: wave plans after the capacity fix (words of group g parked in group g - 2's slots, the last group's
# unused lanes storing over spent points) and the header-free U-list loads: A/B on / off and the
# cache-resident-plan probe (4), same box; then the plan parity tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/${TAG:-r06c}
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_plan.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > $o/pytest.txt 2>&1 || { tail -30 $o/pytest.txt; exit 1; }
tail -1 $o/pytest.txt
for rep in 1 2; do
  for v in off:pynngp_amd/_build/libnngp_hip.so on:pynngp_amd/_build/libnngp_hip.so p4:ab/probe4/libnngp_hip.so; do
    label=${v%%:*}; lib=${v#*:}; plan=on; [ $label = off ] && plan=off
    NNGP_LIB=$(pwd)/$lib timeout -k 10 120 python bench.py --steps 200 --warmup 200 --cpu-seconds 0 --plan $plan \
      > $o/$label.$rep.json 2>> $o/err.log || exit 1
    python3 -c "import json; d=json.load(open('$o/$label.$rep.json')); print('$label', $rep, round(d['roofline']['kernel_ms'],4), 'ms', round(d['value']/1e9,3), 'Gloc/s', d['config']['pair_plan'])"
  done
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $o/on_trace -o run -- \
  python3 bench.py --cpu-seconds 0 --steps 100 --warmup 100 --plan on > $o/on_trace.json 2> $o/on_trace.err || exit 1
python3 -c "
import csv,glob
for r in csv.DictReader(open(glob.glob('$o/on_trace/**/*kernel_stats.csv', recursive=True)[0])):
    if 'bf_' in r['Name']: print(r['Name'][:48], r['Calls'], round(float(r['AverageNs'])/1e3, 2), 'us')
"
