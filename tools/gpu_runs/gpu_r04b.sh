# round-4 session b: fp64 torch diagnostic, callable / Matern-table parity, Matern-table bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r04b
timeout -k 10 120 python tools/diag_torch_fp64.py > gpurun_out/r04b/diag_torch_fp64.txt 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_callable_cov.py tests/test_gpu_matern.py tests/test_gpu_custom_cov.py tests/test_gpu_api.py > gpurun_out/r04b/pytest.txt 2>&1
for nu in 0.5 1.3 2.5 10.0; do timeout -k 10 120 python bench.py --kind matern --nu $nu --theta 1.0,17.320508075688772,0.1 --steps 200 --warmup 200 --cpu-seconds 0 > gpurun_out/r04b/bench_matern_nu$nu.json 2>> gpurun_out/r04b/bench.err || exit 1; done
timeout -k 10 120 python bench.py --kind matern32 --theta 1.0,17.320508075688772,0.1 --steps 200 --warmup 200 --cpu-seconds 0 > gpurun_out/r04b/bench_matern32.json 2>> gpurun_out/r04b/bench.err || exit 1
timeout -k 10 120 python bench.py --kind matern --nu 1.3 --algo wave --theta 1.0,17.320508075688772,0.1 --steps 20 --warmup 5 --cpu-seconds 0 > gpurun_out/r04b/bench_matern_wave.json 2>> gpurun_out/r04b/bench.err || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04b/prof_matern -o run -- python3 bench.py --kind matern --nu 1.3 --theta 1.0,17.320508075688772,0.1 --steps 50 --warmup 50 --cpu-seconds 0 > gpurun_out/r04b/prof_matern.json 2> gpurun_out/r04b/prof_matern.err || exit 1
# three waves per SIMD at m = 15: forced-occupancy builds of the right-looking kernel
# (168 VGPRs; w3: 64 spilled dwords, w3z: values in LDS, 49) against the shipped kernel, same box
timeout -k 10 600 bash tools/ab_clock.sh r04b_w3 "base||" "w3|NNGP_LIB=ab/w3/libnngp_hip.so|" "w3z|NNGP_LIB=ab/w3z/libnngp_hip.so|" > gpurun_out/r04b/ab_w3.txt 2>&1 || exit 1
