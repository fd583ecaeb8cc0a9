#!/bin/bash
# Round 4 final tree: the whole GPU suite, smoke, driver-flag and default benches, configs 2, 4, 5,
# the caller-covariance costs (pairwise plug-in evaluation), and a rocprofv3 kernel-trace summary.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/r04j
mkdir -p $o
timeout -k 10 900 python -u -m pytest -x -v --durations=25 --timeout 300 --timeout-method thread -m gpu tests > $o/tests.txt 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.txt 2>&1 || exit 1
for r in 1 2; do timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $o/bench_driver_$r.json 2> $o/bench_driver_$r.err || exit 1; done
timeout -k 10 300 python bench.py > $o/bench_default.json 2> $o/bench_default.err || exit 1
timeout -k 10 300 python bench.py --config 2 --steps 500 --warmup 3000 --cpu-seconds 0 > $o/bench_config2.json 2> $o/bench_config2.err || exit 1
timeout -k 10 300 python bench.py --config 4 --steps 50 --warmup 50 --cpu-seconds 0 > $o/bench_config4.json 2> $o/bench_config4.err || exit 1
timeout -k 10 300 python bench.py --config 5 --steps 100 --warmup 20 --cpu-seconds 0 > $o/bench_config5.json 2> $o/bench_config5.err || exit 1
timeout -k 10 400 python tools/bench_custom_cov.py > $o/bench_custom_cov.json 2> $o/bench_custom_cov.err || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$o/prof" -o run -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --steps 200 --warmup 200 --cpu-seconds 0 > "$GRAFT_REPO_ROOT/$o/prof_bench.json" 2> "$GRAFT_REPO_ROOT/$o/prof_bench.err"
