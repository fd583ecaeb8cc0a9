#!/bin/bash
# Round 5: the GPU tests of this round's new paths (plans, chains, callable sampler, Matern clamp), then the
# config-3 / config-2 / config-5 benches with and without the new paths on the same box, and a kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/r05b
mkdir -p $o
timeout -k 10 900 python -u -m pytest tests/test_gpu_plan.py tests/test_gpu_gibbs_chains.py tests/test_gpu_callable_cov.py \
  tests/test_gpu_matern.py tests/test_gpu_api.py tests/test_gpu_gibbs.py tests/test_gpu_gibbs_sharded.py -x -v --timeout 120 --timeout-method thread \
  > $o/pytest_new.txt 2>&1 || { tail -60 $o/pytest_new.txt; exit 1; }
tail -3 $o/pytest_new.txt
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
timeout -k 10 300 python bench.py --config 5 --cpu-seconds 0 --steps 300 --warmup 50 > $o/bench_c5_1.json 2> $o/bench_c5_1.err || exit 1
python -c "import json; d=json.load(open('$o/bench_c5_1.json')); print('c5 x1', d['value'], d['ms_per_step'], d['breakdown'])"
for c in 2 4 8; do
  timeout -k 10 400 python bench.py --config 5 --chains-per-gpu $c --cpu-seconds 0 --steps 300 --warmup 50 > $o/bench_c5_$c.json 2> $o/bench_c5_$c.err || exit 1
  python -c "import json; d=json.load(open('$o/bench_c5_$c.json')); print('c5 x$c', d['value'], d['ms_per_step'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof -o run -- python3 bench.py --plan on --cpu-seconds 0 \
  > $o/prof.log 2>&1 || exit 1
find $o/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $o/kernel_stats_plan.csv
head -8 $o/kernel_stats_plan.csv
timeout -k 10 300 python tools/bench_shard_plan.py --gpu --n 10000000 --out $o/shard_plan_gpu.json > $o/shard_plan.log 2>&1 || { tail -20 $o/shard_plan.log; exit 1; }
tail -1 $o/shard_plan.log
