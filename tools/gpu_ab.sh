# A/B timing of library builds / algos on ONE GPU box (run via gpurun).
#   VARIANTS="label:libpath:algo ..." REPS=3 bash tools/gpu_ab.sh [bench args...]
# Each variant runs the bench (no CPU baseline) REPS times, interleaved, so clock / box
# differences cancel; prints kernel ms per run and the median per variant.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for rep in $(seq 1 ${REPS:-2}); do
  for v in $VARIANTS; do
    label=${v%%:*}; rest=${v#*:}; lib=${rest%%:*}; algo=${rest#*:}
    NNGP_LIB=$lib timeout -k 10 120 python bench.py --steps ${STEPS:-30} --warmup ${WARMUP:-5} --cpu-seconds 0 --algo $algo "$@" \
      > gpurun_out/ab/$label.$rep.json 2>> gpurun_out/ab/err.log || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/ab/$label.$rep.json')); print('$label', $rep, round(d['roofline']['kernel_ms'],4), 'ms', round(d['value']/1e9,3), 'Gloc/s')"
  done
done
python3 - <<'PY'
import glob, json, collections, statistics
t = collections.defaultdict(list)
for f in glob.glob('gpurun_out/ab/*.json'):
    t[f.split('/')[-1].rsplit('.', 2)[0]].append(json.load(open(f))['roofline']['kernel_ms'])
for k, v in sorted(t.items()):
    print('median', k, round(statistics.median(v), 4), 'ms over', len(v))
PY
