# round-4 first GPU session: callable-covariance parity tests, then the bench and the provenance passes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r04a
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_callable_cov.py tests/test_gpu_custom_cov.py tests/test_gpu_api.py > gpurun_out/r04a/pytest_callable.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r04a/bench_driver.json 2> gpurun_out/r04a/bench_driver.err || exit 1
timeout -k 10 300 python bench.py --cpu-seconds 0 > gpurun_out/r04a/bench_default.json 2> gpurun_out/r04a/bench_default.err || exit 1
TAG=r04a bash tools/gpu_provenance.sh
