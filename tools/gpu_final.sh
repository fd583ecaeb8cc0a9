# Final-build GPU check (run via gpurun): the GPU suite, smoke, the bench with the driver's
# flags (twice) and its defaults, configs 2 and 4, and the rocprofv3 evidence of the default
# bench (tools/profile.sh -> profiles/<TAG>).   TAG=<tag> bash tools/gpu_final.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/${TAG:-r02ah}
timeout -k 10 900 python -u -m pytest -x -v --durations=25 --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/${TAG:-r02ah}/tests.txt 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG:-r02ah}/smoke.txt 2>&1 || exit 1
for r in 1 2; do timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG:-r02ah}/bench_driver_$r.json 2> gpurun_out/${TAG:-r02ah}/bench_driver_$r.err || exit 1; done
timeout -k 10 300 python bench.py > gpurun_out/${TAG:-r02ah}/bench_default.json 2> gpurun_out/${TAG:-r02ah}/bench_default.err || exit 1
timeout -k 10 300 python bench.py --config 2 --steps 500 --warmup 3000 --cpu-seconds 0 > gpurun_out/${TAG:-r02ah}/bench_config2.json 2> gpurun_out/${TAG:-r02ah}/bench_config2.err || exit 1
timeout -k 10 300 python bench.py --config 4 --steps 50 --warmup 50 --cpu-seconds 0 > gpurun_out/${TAG:-r02ah}/bench_config4.json 2> gpurun_out/${TAG:-r02ah}/bench_config4.err || exit 1
bash tools/profile.sh ${TAG:-r02ah} --steps 200 --warmup 200 || exit 1
