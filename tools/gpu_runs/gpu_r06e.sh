#!/bin/bash
# Round 6: non-temporal streams in the Gibbs colour step (NNGP_GIBBS_NT) -- same-box A/B of the iteration
# time, then the colour kernel's duration and L2 fetch bytes for both builds
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/r06e
mkdir -p $o
VARIANTS="nt1:$(pwd)/pynngp_amd/_build/libnngp_hip.so nt0:$(pwd)/ab/nt0/libnngp_hip.so" REPS=3 bash tools/gpu_ab_gibbs.sh --iters 200 --warmup 100 || exit 1
for v in nt1:pynngp_amd/_build/libnngp_hip.so nt0:ab/nt0/libnngp_hip.so; do
  label=${v%%:*}; lib=$(pwd)/${v#*:}
  NNGP_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $o/${label}_trace -o run -- \
    python3 tools/bench_gibbs.py --iters 50 --warmup 20 > $o/${label}_trace.json 2> $o/${label}_trace.err || exit 1
  NNGP_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $o/${label}_fetch -o run -- \
    python3 tools/bench_gibbs.py --iters 50 --warmup 20 > $o/${label}_fetch.json 2> $o/${label}_fetch.err || exit 1
  NNGP_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $o/${label}_write -o run -- \
    python3 tools/bench_gibbs.py --iters 50 --warmup 20 > $o/${label}_write.json 2> $o/${label}_write.err || exit 1
  python3 - $o $label <<'PY'
import csv, glob, sys, collections
o, label = sys.argv[1], sys.argv[2]
for r in csv.DictReader(open(glob.glob(f'{o}/{label}_trace/**/*kernel_stats.csv', recursive=True)[0])):
    if 'gibbs' in r['Name'] or 'bf_pairb' in r['Name']:
        print(label, r['Name'][:40], r['Calls'], round(float(r['AverageNs']) / 1e3, 2), 'us', round(float(r['TotalDurationNs']) / 1e6 / 70, 4), 'ms/iter')
for k in ('fetch', 'write'):
    agg = collections.defaultdict(list)
    for f in glob.glob(f'{o}/{label}_{k}/**/*counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            if 'gibbs_w_color' in r['Kernel_Name']:
                agg[r['Counter_Name']].append(float(r['Counter_Value']))
    for c, v in agg.items():
        print(label, 'gibbs_w_color', c, round(sum(v) / len(v) / 1e3, 2), 'MB per launch (kB units / 1e3)')
PY
done
