# Per-m pairb timings (m = 17..20) of variant libraries on one box, plus the GPU suite on the
# last one (run via gpurun):  VARIANTS="name:lib ..." bash tools/gpu_occ_ab.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/occ
last=
for v in $VARIANTS; do
  n=${v%%:*}; lib=${v#*:}; last=$lib
  NNGP_LIB=$lib timeout -k 10 300 python tools/algo_table.py --ms 17-20 --algos pairb > gpurun_out/occ/$n.jsonl 2> gpurun_out/occ/$n.err || exit 1
done
NNGP_LIB=$last timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/occ/tests.txt 2>&1 || exit 1
