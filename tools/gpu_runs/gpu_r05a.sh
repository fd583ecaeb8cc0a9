#!/bin/bash
# Round 5, first pass: tile pair plans -- the plan tests (planned = unplanned bit for bit), then the
# config-3 / config-2 benches with and without the plan on the same box, and a kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/r05a
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_plan.py -x -v --timeout 120 --timeout-method thread \
  > $o/pytest_plan.txt 2>&1 || { tail -40 $o/pytest_plan.txt; exit 1; }
tail -3 $o/pytest_plan.txt
for r in 1 2; do
  for p in off on; do
    timeout -k 10 300 python bench.py --plan $p --cpu-seconds 0 > $o/bench_c3_${p}_$r.json 2> $o/bench_c3_${p}_$r.err || exit 1
    python -c "import json,sys; d=json.load(open('$o/bench_c3_${p}_$r.json')); print('c3 $p', d['ms_per_step'], d['roofline']['kernel_ms'], d['config']['pair_plan'])"
  done
done
for p in off on; do
  timeout -k 10 300 python bench.py --config 2 --plan $p --cpu-seconds 0 --steps 3000 --warmup 3000 > $o/bench_c2_$p.json 2> $o/bench_c2_$p.err || exit 1
  python -c "import json,sys; d=json.load(open('$o/bench_c2_$p.json')); print('c2 $p', d['ms_per_step'], d['roofline']['kernel_ms'], d['config']['pair_plan'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof -o run -- python3 bench.py --plan on --cpu-seconds 0 \
  > $o/prof.log 2>&1 || exit 1
find $o/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $o/kernel_stats_plan.csv
head -8 $o/kernel_stats_plan.csv
