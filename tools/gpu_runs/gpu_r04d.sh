# round-4 session d: the whole GPU suite, smoke, the driver-flag bench; same-box A/B of the tile
# balancing (nobal: plain 128-row tiles) and the fused record fold (ff) at configs 2 and 3
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r04d
mkdir -p $out
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_gibbs_sharded.py > $out/pytest_sharded.txt 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $out/bench_driver.json 2> $out/bench_driver.err || exit 1
timeout -k 10 600 bash tools/ab_clock.sh r04d_c3 "base||" "nobal|NNGP_LIB=ab/nobal/libnngp_hip.so|" "ff|NNGP_LIB=ab/ff/libnngp_hip.so|" > $out/ab_c3.txt 2>&1 || exit 1
timeout -k 10 600 bash tools/ab_clock.sh r04d_c2 "base||--config 2" "nobal|NNGP_LIB=ab/nobal/libnngp_hip.so|--config 2" "ff|NNGP_LIB=ab/ff/libnngp_hip.so|--config 2" > $out/ab_c2.txt 2>&1 || exit 1
for v in base nobal ff; do
  lib=pynngp_amd/_build/libnngp_hip.so; [ $v != base ] && lib=ab/$v/libnngp_hip.so
  NNGP_LIB=$lib timeout -k 10 120 python bench.py --config 2 --steps 500 --warmup 3000 --cpu-seconds 0 > $out/bench_c2_$v.json 2>> $out/bench_c2.err || exit 1
done
