#!/bin/bash
# Round 5: the whole GPU suite, then the benches of the new paths (plans on/off, config 2, chains),
# a kernel trace and the device shard plan at N = 1e7.  Stops at a fault / timeout (not at a test failure).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1 PYTHONPATH=.
o=gpurun_out/r05e
mkdir -p $o
stop() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > $o/pytest_gpu.txt 2>&1; rc=$?; stop $rc pytest
grep -E "^(FAILED|ERROR)" $o/pytest_gpu.txt | head -30; tail -1 $o/pytest_gpu.txt
for r in 1 2; do
  for p in off on; do
    timeout -k 10 300 python bench.py --plan $p --cpu-seconds 0 > $o/bench_c3_${p}_$r.json 2> $o/bench_c3_${p}_$r.err; rc=$?; stop $rc bench
    python -c "import json; d=json.load(open('$o/bench_c3_${p}_$r.json')); print('c3 $p', d['ms_per_step'], d['roofline']['kernel_ms'], d['config'].get('pair_plan'))" || true
  done
done
for p in off on; do
  timeout -k 10 300 python bench.py --config 2 --plan $p --cpu-seconds 0 --steps 3000 --warmup 3000 > $o/bench_c2_$p.json 2> $o/bench_c2_$p.err; rc=$?; stop $rc bench2
  python -c "import json; d=json.load(open('$o/bench_c2_$p.json')); print('c2 $p', d['ms_per_step'], d['roofline']['kernel_ms'], d['config'].get('pair_plan'))" || true
done
timeout -k 10 300 python bench.py --config 4 --cpu-seconds 0 > $o/bench_c4.json 2> $o/bench_c4.err; rc=$?; stop $rc bench4
python -c "import json; d=json.load(open('$o/bench_c4.json')); print('c4', d['ms_per_step'], d['roofline']['kernel_ms'])" || true
timeout -k 10 300 python bench.py --config 5 --cpu-seconds 0 --steps 300 --warmup 50 > $o/bench_c5_1.json 2> $o/bench_c5_1.err; rc=$?; stop $rc bench5
python -c "import json; d=json.load(open('$o/bench_c5_1.json')); print('c5 x1', d['value'], d['ms_per_step'])" || true
for c in 2 4 8; do
  timeout -k 10 400 python bench.py --config 5 --chains-per-gpu $c --cpu-seconds 0 --steps 300 --warmup 50 > $o/bench_c5_$c.json 2> $o/bench_c5_$c.err; rc=$?; stop $rc bench5c
  python -c "import json; d=json.load(open('$o/bench_c5_$c.json')); print('c5 x$c', d['value'], d['ms_per_step'])" || true
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof -o run -- python3 bench.py --plan on --cpu-seconds 0 > $o/prof.log 2>&1; rc=$?; stop $rc rocprof
find $o/prof -name "*kernel_stats.csv" -exec cp {} $o/kernel_stats_plan.csv \;
head -6 $o/kernel_stats_plan.csv
timeout -k 10 300 python tools/bench_shard_plan.py --gpu --n 10000000 --out $o/shard_plan_gpu.json > $o/shard_plan.log 2>&1; rc=$?; stop $rc shard
tail -2 $o/shard_plan.log
