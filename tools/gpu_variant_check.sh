# Parity suite and same-box A/B of one variant library (run via gpurun):
#   VARIANT=ab/<name>/libnngp_hip.so TAG=<tag> bash tools/gpu_variant_check.sh [bench args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
NNGP_LIB=$VARIANT timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/$TAG/tests.txt 2>&1 || exit 1
VARIANTS="cur:pynngp_amd/_build/libnngp_hip.so:auto var:$VARIANT:auto" REPS=${REPS:-4} STEPS=200 WARMUP=200 bash tools/gpu_ab.sh "$@" > gpurun_out/$TAG/ab.txt 2>&1 || exit 1
