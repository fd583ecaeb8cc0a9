# One GPU-box session (run via gpurun): GPU test suite, the bench with the driver's flags and
# with its defaults, the per-m pairb table and the rocprofv3 evidence of the default bench.
#   bash tools/gpu_batch.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-b}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $out/tests.txt 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $out/bench_driver_$r.json 2> $out/bench_driver_$r.err || exit 1
done
timeout -k 10 300 python bench.py > $out/bench_default.json 2> $out/bench_default.err || exit 1
timeout -k 10 300 python tools/algo_table.py --ms 10-24 --algos pairb > $out/algo_pairb_m10_24.jsonl 2> $out/algo.err || exit 1
bash tools/profile.sh $tag --steps 200 --warmup 200 || exit 1
