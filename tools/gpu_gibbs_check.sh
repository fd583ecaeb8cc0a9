# Gibbs check (via gpurun): the Gibbs GPU tests on the in-tree build, then an interleaved A/B of
# library variants on the Gibbs iteration (tools/gpu_ab_gibbs.sh) -> gpurun_out/${TAG:-r03q}
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/${TAG:-r03q}
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_gibbs.py tests/test_gpu_gibbs_ref.py tests/test_gpu_gibbs_sharded.py > gpurun_out/${TAG:-r03q}/pytest_gibbs.txt 2>&1 || exit 1
VARIANTS="g32x1:ab/g32x1/libnngp_hip.so g16x2:pynngp_amd/_build/libnngp_hip.so g8x4:ab/g8x4/libnngp_hip.so g32x2:ab/g32x2/libnngp_hip.so" REPS=3 timeout -k 10 500 bash tools/gpu_ab_gibbs.sh --iters 300 --warmup 100 > gpurun_out/${TAG:-r03q}/ab_gibbs.txt 2>&1 || exit 1
