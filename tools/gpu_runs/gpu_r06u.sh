#!/bin/bash
# Round 6: timing probe -- the colour kernel without its member-row load (tools/variants/gibbs_no_member_row.patch:
# the member's location and reverse range synthesised, wrong values) against the product kernel: the colour
# sweep's time (bench_gibbs w_sweep_ms) and the colour kernel's average duration
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
o=gpurun_out/r06u
mkdir -p $o
for r in 1 2; do for v in cur:pynngp_amd/_build/libnngp_hip.so nomr:ab/gibbs_nomr/libnngp_hip.so; do
  label=${v%%:*}; lib=$(pwd)/${v#*:}
  NNGP_LIB=$lib timeout -k 10 200 python tools/bench_gibbs.py --iters 100 --warmup 50 $([ $label = nomr ] && echo --sweep-only) > $o/$label.$r.json 2>> $o/err.log || exit 1
  python3 -c "import json; d=json.load(open('$o/$label.$r.json')); print('$label', round(d['w_sweep_ms'],4), 'ms per w sweep', round(d['ms_per_iter'],4), 'ms/iter')"
done; done
for v in cur:pynngp_amd/_build/libnngp_hip.so nomr:ab/gibbs_nomr/libnngp_hip.so; do
  label=${v%%:*}; lib=$(pwd)/${v#*:}
  NNGP_LIB=$lib timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $o/${label}_trace -o run -- \
    python3 tools/bench_gibbs.py --iters 30 --warmup 10 --sweep-only > $o/${label}_trace.json 2> $o/${label}_trace.err || exit 1
  python3 - $o $label <<'PY'
import csv, glob, sys
o, label = sys.argv[1], sys.argv[2]
for r in csv.DictReader(open(glob.glob(f'{o}/{label}_trace/**/*kernel_stats.csv', recursive=True)[0])):
    if 'gibbs_w_color' in r['Name']:
        print(label, r['Name'][:32], r['Calls'], round(float(r['AverageNs']) / 1e3, 2), 'us avg')
PY
done
