# round-4 session e: driver-flag and default benches of the final kernels, then the roofline provenance of
# every preset (tools/gpu_provenance.sh -> tools/make_traffic.py on the host)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r04e
mkdir -p $out
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $out/bench_driver.json 2> $out/bench_driver.err || exit 1
timeout -k 10 300 python bench.py --cpu-seconds 0 > $out/bench_default.json 2> $out/bench_default.err || exit 1
TAG=r04e bash tools/gpu_provenance.sh || exit 1
