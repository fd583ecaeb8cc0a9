# compare the sweep kernels (lane / pair / quad / wave) and the visiting order on the GPU box
#   SPECS="15 pair,15 lane" bash tools/gpu_algos.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/algos
IFS=',' read -ra specs <<< "${SPECS:-15 lane,15 pair,15 quad,10 lane,10 pair,16 lane,16 quad,20 pair,20 quad}"
for spec in "${specs[@]}"; do
  set -- $spec
  for ord in "" "--no-order"; do
    steps=20; [ "$2" = wave ] && steps=3
    tag=m$1_$2${ord:+_idx}
    timeout -k 10 120 python bench.py --steps $steps --warmup 2 --cpu-seconds 0 --m $1 --algo $2 $ord ${BENCH_ARGS:-} > gpurun_out/algos/$tag.json 2>>gpurun_out/algos/err.log || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/algos/$tag.json')); print('$tag', round(d['value']/1e9,3), 'Gloc/s', round(d['roofline']['kernel_ms'],4), 'ms')"
  done
done
